cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
GC_MS_MASK_PF=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide_levels.py -q -x -k "cache" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pf_r03zg.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_pf_r03zg.log; [ $rc -ne 0 ] && exit $rc
for b in 0 1 0 1; do
GC_MS_MASK_PF=$b timeout -k 10 300 python tools/ms_size_sweep.py > gpurun_out/ms_sweep_r03zg_p$b.log 2>&1 || exit $?
echo "pf=$b"; grep -E "rounds=(1.000|1.246|3.000)" gpurun_out/ms_sweep_r03zg_p$b.log | cut -c60-100
done
