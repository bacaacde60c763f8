cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PYTEST_K="quantize or qsgdbp or facade or two_scale or ts_ or golden" bash tools/gpu.sh r04zg tests || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --legs packers --cpu-seconds 0 > gpurun_out/packers_r04zg.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r04zg -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_packers.py > $GRAFT_REPO_ROOT/gpurun_out/prof_r04zg.log 2>&1
