cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide_levels.py tests/test_gpu_golden_big.py -q -x -k "ms or two_scale or multi or wide" --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r03m.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r03m.log; [ $rc -ne 0 ] && exit $rc
for t in 1 2 3; do
  GC_MS_FUSED_TILES=$t timeout -k 10 200 python tools/time_ms_kernels.py >> gpurun_out/ms_tiles_r03m.log 2>&1 || exit $?
done
cat gpurun_out/ms_tiles_r03m.log | grep tiles=
