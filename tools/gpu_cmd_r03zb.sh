cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for g in 0 256 512 1024 2048 4096 0 512 1024; do
GC_ENC_STREAM_GRID=$g timeout -k 10 300 python tools/time_torch_mode.py > gpurun_out/torch_mode_r03zb_g$g.log 2>&1 || exit $?
echo "grid cap=$g"; grep -E "speculate=True, wait next jumps=False" gpurun_out/torch_mode_r03zb_g$g.log
done
