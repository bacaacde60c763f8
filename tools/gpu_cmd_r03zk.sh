cd "${GRAFT_REPO_ROOT:-/root/repo}"
for g in 0 8192 16384 24576 6144 0 16384 24576; do
if [ $g = 0 ]; then unset GC_ENC_GRID; else export GC_ENC_GRID=$g; fi
timeout -k 10 200 python tools/enc_grid_sweep.py 2>&1 | grep "grid cap" || exit 1
done
