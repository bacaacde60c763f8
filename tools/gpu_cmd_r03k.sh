cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r03k.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_r03k.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash tools/profile_r02.sh r03k
