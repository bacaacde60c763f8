set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 tools/lab_ms > gpurun_out/lab_ms_r03d.log 2>&1
rc=$?; echo "lab rc=$rc"; tail -45 gpurun_out/lab_ms_r03d.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider -k "ms_ or twoscale or multiscale or wide_levels or golden_big or hook" > gpurun_out/pytest_r03d.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r03d.log; exit $rc
