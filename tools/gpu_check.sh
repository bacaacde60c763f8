#!/bin/bash
# One gpurun call: smoke -> GPU tests -> bench -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; a fault / abort / segfault / timeout
# (exit >= 124 or a signal) ends the script; plain test failures (exit 1) do not.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-r01}
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -5 $OUT/$name.log
  if [ $rc -ge 124 ] || [ $rc -ge 128 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
rocm-smi --showproductname > $OUT/gpu_info.log 2>&1 || true
run smoke 400 python -c "import __graft_entry__ as g; g.smoke()" || { [ $? -eq 1 ] || exit 1; }
run pytest_gpu 900 python -m pytest tests -m gpu -q --maxfail=20 -p no:cacheprovider
run bench 600 python bench.py --steps 20 --warmup 5
export TMPDIR=/tmp
run rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-extras
echo ALL DONE
