cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r03o.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r03o.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/time_ms_kernels.py > gpurun_out/ms_kernels_r03o.log 2>&1 || exit $?
cat gpurun_out/ms_kernels_r03o.log
timeout -k 10 900 bash tools/profile_r02.sh r03o
