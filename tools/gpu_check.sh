#!/bin/bash
# One gpurun call: lab -> smoke -> GPU tests -> bench -> rocprofv3 (trace + PMC).
# Every GPU step has its own time limit; a fault / abort / segfault / timeout
# (exit >= 124 or a signal) ends the script; plain test failures (exit 1) do not.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-r01}
MODE=${2:-all}
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 $OUT/$name.log
  if [ $rc -ge 124 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
[ -x tools/lab2 ] && run lab_$TAG 200 tools/lab2
[ -x tools/lab_ms ] && run labms_$TAG 200 tools/lab_ms
[ "$MODE" = "lab" ] && exit 0
run smoke_$TAG 400 python -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu_$TAG 900 python -m pytest tests -m gpu -q --maxfail=20 -p no:cacheprovider
run bench_$TAG 600 python bench.py
run gloo2_$TAG 300 env GC_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 3 --cpu-seconds 0
run profile_$TAG 1000 bash tools/profile.sh $TAG
echo ALL DONE
