cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PYTEST_K="greedy4 or qsgdbp or packer or torch_mode" bash tools/gpu.sh r04q tests || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --legs packers,torch --cpu-seconds 0 > gpurun_out/bench_legs_r04q.log 2>&1
