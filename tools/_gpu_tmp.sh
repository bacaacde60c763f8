cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
AB=1 timeout -k 10 300 python tools/time_torch_mode.py > gpurun_out/torch_ab_r04p.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --legs config3,torch --cpu-seconds 0 > gpurun_out/bench_legs_r04p.log 2>&1
