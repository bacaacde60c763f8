cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r03k.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_r03k.log; [ $rc -ne 0 ] && exit $rc
for t in 1 2 3 4; do
  GC_MS_FUSED_TILES=$t timeout -k 10 200 tools/lab_ms > gpurun_out/lab_ms_r03k_t$t.log 2>&1 || exit $?
  echo "tiles=$t"; grep -E "one-pass|cached|mask \+ cache|select from cache" gpurun_out/lab_ms_r03k_t$t.log | grep -v "==" | head -8
done
timeout -k 10 900 bash tools/profile_r02.sh r03k
