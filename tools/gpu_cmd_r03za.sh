cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for w in 2 1; do
GC_MT_GEN_TW=$w timeout -k 10 400 python -u -m pytest tests/test_gpu_torch_mode.py tests/test_mt_jump.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_tw_${w}_r03za.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_tw_${w}_r03za.log; [ $rc -ne 0 ] && exit $rc
done
for w in 4 2 1 4 2 1; do
GC_MT_GEN_TW=$w timeout -k 10 300 python tools/time_torch_mode.py > gpurun_out/torch_mode_r03za_tw$w.log 2>&1 || exit $?
echo "TW=$w"; grep -E "J = 261456|383 generators|speculate=True, wait next jumps=False" gpurun_out/torch_mode_r03za_tw$w.log
done
