# quick GPU check: MS lab, torch-mode timing, torch-mode + MS tests
set -u
export GRAFT_REPO_ROOT="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-q}
timeout -k 10 200 tools/lab_ms > gpurun_out/lab_ms_$T.log 2>&1
rc=$?; echo "lab rc=$rc"; grep -E "one-pass|mask encode|select|==" gpurun_out/lab_ms_$T.log | tail -30
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python tools/time_torch_mode.py > gpurun_out/torch_mode_$T.log 2>&1
rc=$?; echo "torch-mode timing rc=$rc"; cat gpurun_out/torch_mode_$T.log | tail -20
[ $rc -ge 124 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/trace_torch_$T" -o run -- python3 "$GRAFT_REPO_ROOT/tools/trace_torch_mode.py" > "$GRAFT_REPO_ROOT/gpurun_out/trace_torch_$T.log" 2>&1
rc=$?; echo "torch trace rc=$rc"; cd "$GRAFT_REPO_ROOT"
[ $rc -ge 124 ] && exit $rc
python tools/overlap.py gpurun_out/trace_torch_$T | tail -25
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider -k "torch or mt19937 or golden or ms_encode_w1" > gpurun_out/pytest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$T.log; exit $rc
