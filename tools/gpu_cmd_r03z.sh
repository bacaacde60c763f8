cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for w in 3 2; do
GC_MT_JUMP_W4=$w timeout -k 10 400 python -u -m pytest tests/test_gpu_torch_mode.py tests/test_mt_jump.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_w4_${w}_r03z.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_w4_${w}_r03z.log; [ $rc -ne 0 ] && exit $rc
done
for w in 1 3 2 1 3; do
GC_MT_JUMP_W4=$w timeout -k 10 300 python tools/time_torch_mode.py > gpurun_out/torch_mode_r03z_w$w.log 2>&1 || exit $?
echo "W4=$w"; grep -E "J = 261456|383 generators|speculate=True, wait next jumps=False" gpurun_out/torch_mode_r03z_w$w.log
done
