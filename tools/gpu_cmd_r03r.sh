cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
GC_MS_FUSED_SPLIT=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "encode_w1 or ms_one_pass or fused" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_split_r03r.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_split_r03r.log; [ $rc -ne 0 ] && exit $rc
for s in 1 2 1 2; do
GC_MS_FUSED_SPLIT=$s timeout -k 10 300 python tools/ms_size_sweep.py > gpurun_out/ms_sweep_r03r_s$s.log 2>&1 || exit $?
echo "split=$s"; cut -c1-75 gpurun_out/ms_sweep_r03r_s$s.log | grep n=
done
