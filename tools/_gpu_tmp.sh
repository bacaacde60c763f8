cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PYTEST_K="randk or grandk or segments or multirank or golden or reducer" bash tools/gpu.sh r04zh tests || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --legs config4 --cpu-seconds 0 > gpurun_out/bench_c4_r04zh.log 2>&1
