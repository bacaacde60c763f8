cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_torch_mode.py tests/test_mt_jump.py tests/test_gpu_golden_big.py tests/test_gpu_parity.py -q -x -k "torch or mt19937 or split or golden or digest" --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_seq_r03zc.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_seq_r03zc.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 300 python tools/time_torch_mode.py > gpurun_out/torch_mode_r03zc_$i.log 2>&1 || exit $?
grep -E "J = 261456|383 generators|speculate=True, wait next jumps=False" gpurun_out/torch_mode_r03zc_$i.log
done
