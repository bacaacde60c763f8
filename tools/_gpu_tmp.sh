cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for q in 4 8 16; do
  echo "== GPU_MAX_HW_QUEUES=$q" >> gpurun_out/torch_hwq_r04r.log
  GPU_MAX_HW_QUEUES=$q timeout -k 10 250 python tools/time_torch_mode.py 128,256 2,3 >> gpurun_out/torch_hwq_r04r.log 2>&1 || exit $?
done
