cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_rccl_r03q.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_rccl_r03q.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python tools/ms_size_sweep.py > gpurun_out/ms_sweep_r03q.log 2>&1 || exit $?
cat gpurun_out/ms_sweep_r03q.log
