cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PYTEST_K="greedy4 or qsgdbp or packer" bash tools/gpu.sh r04ze tests || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --legs packers --cpu-seconds 0 > gpurun_out/packers_r04ze.log 2>&1
