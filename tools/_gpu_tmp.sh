cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PYTEST_K="greedy4 or qsgdbp or packer" bash tools/gpu.sh r04z tests || exit $?
for L in 1 0 1 0; do
  GC_G4_LOOP=$L timeout -k 10 300 python bench.py --steps 5 --warmup 2 --legs packers --cpu-seconds 0 > gpurun_out/packers_loop${L}_r04z.log 2>&1 || exit $?
  grep -o '"greedy4_pack_[a-z]*": {"us": [0-9.]*' gpurun_out/packers_loop${L}_r04z.log | sed "s/^/loop=$L /" >> gpurun_out/packers_ab_r04z.log
done
