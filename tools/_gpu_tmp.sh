cd "${GRAFT_REPO_ROOT:-/root/repo}"
PYTEST_K="greedy4 or qsgdbp or packer or bytepack or torch_mode or randk or reducers or golden_big" bash tools/gpu.sh r04d tests || exit $?
(cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r04d -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_packers.py > $GRAFT_REPO_ROOT/gpurun_out/prof_r04d.log 2>&1) || exit $?
bash tools/gpu.sh r04d cmd -- python tools/time_torch_mode.py 0,128,192,256 1,2,3 || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --legs config4,torch,packers --cpu-seconds 0 > gpurun_out/bench_legs_r04d.log 2>&1
