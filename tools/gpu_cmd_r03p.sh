cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03p.log 2>&1 || exit $?
tail -2 gpurun_out/smoke_r03p.log
timeout -k 10 60 python tools/rccl_probe.py 1 > gpurun_out/rccl1_r03p.log 2>&1; echo "rccl1 rc=$?"; tail -3 gpurun_out/rccl1_r03p.log
timeout -k 10 90 python tools/rccl_probe.py 2 > gpurun_out/rccl2_r03p.log 2>&1; rc=$?; echo "rccl2 rc=$rc"; tail -5 gpurun_out/rccl2_r03p.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r03p.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_r03p.log; exit $rc
