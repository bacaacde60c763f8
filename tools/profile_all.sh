#!/bin/bash
# rocprofv3 --kernel-trace --stats of the full bench (every config leg), for
# per-kernel times of the non-headline kernels (multi-scale, GRandK, pipeline)
set -u
TAG=${1:-all}
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/profall_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --cpu-seconds 0 > "$OUT/bench.log" 2>&1
rc=$?
echo "rc=$rc"
f=$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cut -c1-220 "$f" | head -40
exit $rc
