cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_torch_mode.py tests/test_gpu_parity.py tests/test_gpu_segments.py -q -x -k "torch or mt19937 or split or randk or segments or reducer" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r03j.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r03j.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/time_torch_mode.py > gpurun_out/torch_mode_r03j.log 2>&1 || exit $?
cat gpurun_out/torch_mode_r03j.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r03j.log 2>&1 || exit $?
tail -c 600 gpurun_out/bench_r03j.log
