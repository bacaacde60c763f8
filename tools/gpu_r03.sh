#!/bin/bash
# Round-3 GPU evidence in one gpurun call.  Every GPU step has its own time
# limit; a timeout, signal or fault (exit >= 124) ends the script, and so does a
# failing smoke.  MODE: all | tests | bench | prof | lab, or a comma list
# (e.g. lab,tests,bench)
#   smoke -> pytest -m gpu -> bench (the driver's exact command) -> rocprofv3
#   --kernel-trace --stats of that same command -> N=2 gloo rehearsal ->
#   FETCH/WRITE PMC passes over the bench -> steady-state kernel workload
#   (tools/prof_kernels.py: trace, PMC, SQ)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
TAG=${1:-r03}
MODE=${2:-all}
DRIVER="bench.py --gpus 1 --steps 20 --warmup 5"
has() { [ "$MODE" = all ] || [[ ",$MODE," == *",$1,"* ]]; }
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps_$TAG.log"
  timeout -k 10 "$t" "$@" > "$OUT/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps_$TAG.log"
  tail -3 "$OUT/${name}_$TAG.log" | cut -c1-600
  if [ $rc -ge 124 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
if has lab; then
  [ -x tools/lab_ms ] && { run lab_ms 200 tools/lab_ms || true; }
  [ -x tools/lab2 ] && { run lab2 200 tools/lab2 || true; }
fi
if has tests; then
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
  run pytest_gpu 1500 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 240 --timeout-method thread -p no:cacheprovider
fi
if has bench; then
  run bench 400 python3 $DRIVER
  run torch_mode 300 python tools/time_torch_mode.py
  cd /tmp && export TMPDIR=/tmp
  run rocprof_driver 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG/driver" -o run -- python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5
  cd "$ROOT"
  run gloo2 300 env GC_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 3 --cpu-seconds 0
fi
if has prof; then
  cd /tmp && export TMPDIR=/tmp
  B="$ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-extras"
  KREGEX='k_qsgd_encode|k_absmax|k_qsgd_decode'
  run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KREGEX" --output-format csv -d "$OUT/prof_$TAG/fetch" -o run -- python3 $B
  run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KREGEX" --output-format csv -d "$OUT/prof_$TAG/write" -o run -- python3 $B
  cd "$ROOT"
  timeout -k 10 900 bash tools/profile_r02.sh "$TAG"
fi
echo ALL DONE
