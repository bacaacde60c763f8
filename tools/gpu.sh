#!/bin/bash
# The one GPU-box launcher (run through gpurun):
#
#   gpurun --timeout 1200 -- bash tools/gpu.sh TAG STEPS [-- extra command]
#
# STEPS is a comma list, run in this order:
#   lab       tools/lab_ms, tools/lab2 (if built)
#   smoke     __graft_entry__.smoke()
#   tests     pytest -m gpu (whole suite; PYTEST_K=expr narrows it)
#   bench     the driver's exact command (bench.py --gpus 1 --steps 20 --warmup 5)
#   benchfull bench.py with its defaults
#   torch     tools/time_torch_mode.py
#   driver    rocprofv3 --kernel-trace --stats of the driver's command
#   scale     plain `bench.py --gpus 2` and `--gpus 4` over gloo (the SCALE form; ranks share cuda:0)
#   pmc       FETCH_SIZE / WRITE_SIZE passes over the headline kernels
#   kprof     tools/prof_kernels.py: trace, FETCH, WRITE, SQ, LDS passes
#   g4prof    the same five passes over tools/prof_packers.py (the drop-in packers)
#   cmd       the command after "--" (e.g. a lab sweep), with a 600 s limit
#
# Every GPU step has its own time limit.  A timeout, signal, abort or fault
# (exit >= 124) ends the script; so does a failing smoke.  Logs go to
# gpurun_out/<step>_<TAG>.log and the step list to gpurun_out/steps_<TAG>.log.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
TAG=${1:-t}
STEPS=${2:-smoke,tests,bench}
shift 2 2>/dev/null || shift $#
EXTRA=()
if [ "${1:-}" = "--" ]; then shift; EXTRA=("$@"); fi
DRIVER="bench.py --gpus 1 --steps 20 --warmup 5"
has() { [[ ",$STEPS," == *",$1,"* ]]; }
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
prof() {  # name, timeout, rocprofv3 args... (from /tmp, the profiler's working directory)
  local name=$1 t=$2; shift 2
  (cd /tmp && TMPDIR=/tmp run "$name" "$t" rocprofv3 "$@") || { local rc=$?; [ $rc -ge 124 ] && exit $rc; return $rc; }
}
if has lab; then
  [ -x tools/lab_ms ] && { run lab_ms 200 tools/lab_ms || true; }
  [ -x tools/lab2 ] && { run lab2 200 tools/lab2 || true; }
fi
if has smoke; then
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
if has tests; then
  run pytest_gpu 1500 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 240 --timeout-method thread \
    -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"}
fi
if has bench; then
  run bench 400 python3 $DRIVER
fi
if has benchfull; then
  run benchfull 900 python3 bench.py
fi
if has torch; then
  run torch_mode 300 python tools/time_torch_mode.py
fi
if has driver; then
  prof rocprof_driver 500 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG/driver" -o run -- \
    python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5
fi
if has scale; then
  for n in 2 4; do
    run scale$n 300 env GC_BENCH_BACKEND=gloo python3 bench.py --gpus $n --steps 20 --warmup 3 --cpu-seconds 0 \
      --legs reduce,config5 --n5 100000000
  done
fi
if has pmc; then
  B="$ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-extras"
  KREGEX='k_qsgd_encode|k_absmax|k_qsgd_decode'
  prof pmc_fetch 300 --pmc FETCH_SIZE --kernel-include-regex "$KREGEX" --output-format csv \
    -d "$OUT/prof_$TAG/fetch" -o run -- python3 $B
  prof pmc_write 300 --pmc WRITE_SIZE --kernel-include-regex "$KREGEX" --output-format csv \
    -d "$OUT/prof_$TAG/write" -o run -- python3 $B
fi
if has kprof; then
  K="$ROOT/tools/prof_kernels.py"
  D="$OUT/prof_${TAG}_k"
  prof k_trace 240 --kernel-trace --stats --output-format csv -d "$D/trace" -o run -- python3 $K || exit $?
  prof k_fetch 240 --pmc FETCH_SIZE --output-format csv -d "$D/fetch" -o run -- python3 $K || exit $?
  prof k_write 240 --pmc WRITE_SIZE --output-format csv -d "$D/write" -o run -- python3 $K || exit $?
  prof k_sq 240 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d "$D/sq" -o run -- python3 $K || exit $?
  prof k_lds 240 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES \
    SQ_WAVES --output-format csv -d "$D/lds" -o run -- python3 $K || exit $?
fi
if has g4prof; then
  K="$ROOT/tools/prof_packers.py"
  D="$OUT/prof_${TAG}_g4"
  export PACK_SRC=xi
  prof g4_trace 240 --kernel-trace --stats --output-format csv -d "$D/trace" -o run -- python3 $K || exit $?
  prof g4_fetch 240 --pmc FETCH_SIZE --output-format csv -d "$D/fetch" -o run -- python3 $K || exit $?
  prof g4_write 240 --pmc WRITE_SIZE --output-format csv -d "$D/write" -o run -- python3 $K || exit $?
  prof g4_sq 240 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d "$D/sq" -o run -- python3 $K || exit $?
  prof g4_lds 240 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES \
    SQ_WAVES --output-format csv -d "$D/lds" -o run -- python3 $K || exit $?
fi
if has cmd && [ ${#EXTRA[@]} -gt 0 ]; then
  run cmd 600 "${EXTRA[@]}"
fi
echo ALL DONE
