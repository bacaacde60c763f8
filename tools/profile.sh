#!/bin/bash
# rocprofv3 evidence for one round (run on the GPU box via gpurun):
#   1. --kernel-trace --stats of the bench command (per-kernel durations)
#   2. separate --pmc passes for FETCH_SIZE and WRITE_SIZE (never combined
#      with other tracing; MI355X_MICROARCH.md: FETCH_SIZE is x0.5 on gfx950
#      for wide streaming reads -> doubled by tools/pmc_traffic.py)
# Output: gpurun_out/prof_<tag>/...  then  python tools/pmc_traffic.py <tag>
set -u
TAG=${1:-r01}
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-extras"
KREGEX='k_qsgd_encode|k_absmax|k_qsgd_decode'
step() {
  local name=$1; shift
  echo "== $name" | tee -a "$OUT/steps.log"
  timeout -k 10 300 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  [ $rc -ge 124 ] && { echo "STOP (rc=$rc)"; exit $rc; }
  return 0
}
step trace rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH
step fetch rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KREGEX" --output-format csv -d "$OUT/fetch" -o run -- python3 $BENCH
step write rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KREGEX" --output-format csv -d "$OUT/write" -o run -- python3 $BENCH
echo PROFILE DONE
