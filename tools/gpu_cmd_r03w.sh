cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
GC_MS_SKEY=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide_levels.py -q -x -k "cache or encode_w1 or ms_one_pass or fused" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_skey_r03w.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_skey_r03w.log; [ $rc -ne 0 ] && exit $rc
for b in 0 1 0 1; do
GC_MS_SKEY=$b timeout -k 10 300 python tools/ms_size_sweep.py > gpurun_out/ms_sweep_r03w_k$b.log 2>&1 || exit $?
echo "skey=$b"; grep -E "rounds=(1.000|1.246|2.000|3.000)" gpurun_out/ms_sweep_r03w_k$b.log | cut -c25-120
done
