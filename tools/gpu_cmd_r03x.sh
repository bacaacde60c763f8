cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/prof_r03x_tm" -o run -- python3 "$ROOT/tools/trace_torch_mode.py" > "$ROOT/gpurun_out/trace_tm_r03x.log" 2>&1 || exit $?
cd "$ROOT"
python tools/overlap.py gpurun_out/prof_r03x_tm > gpurun_out/overlap_r03x.txt
tail -45 gpurun_out/overlap_r03x.txt
