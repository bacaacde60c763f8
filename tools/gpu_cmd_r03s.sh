cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for u in 2 3; do
GC_MS_FUSED_U=$u timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "encode_w1 or ms_one_pass or fused" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_u${u}_r03s.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_u${u}_r03s.log; [ $rc -ne 0 ] && exit $rc
done
for u in 1 2 3 1 2 3; do
GC_MS_FUSED_U=$u timeout -k 10 300 python tools/ms_size_sweep.py > gpurun_out/ms_sweep_r03s_u$u.log 2>&1 || exit $?
echo "U=$u"; cut -c1-75 gpurun_out/ms_sweep_r03s_u$u.log | grep -E "rounds=(1.000|1.246|2.000|3.000)"
done
