#!/bin/bash
# rocprofv3 passes over tools/prof_kernels.py (run on the GPU box via gpurun):
#   trace: --kernel-trace --stats; then one --pmc pass per counter group
#   (never combined with tracing; MI355X_MICROARCH.md: FETCH_SIZE x2 on gfx950).
set -u
TAG=${1:-r02}
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/prof_${TAG}_k"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
W="$ROOT/tools/prof_kernels.py"
step() {
  local name=$1; shift
  echo "== $name" | tee -a "$OUT/steps.log"
  timeout -k 10 240 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  [ $rc -ge 124 ] && { echo "STOP (rc=$rc)"; exit $rc; }
  [ $rc -ne 0 ] && { tail -5 "$OUT/$name.log"; exit $rc; }
  return 0
}
step trace rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $W
[ "${2:-}" = "trace" ] && { echo PROFILE DONE; exit 0; }
step fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 $W
step write rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 $W
step sq rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d "$OUT/sq" -o run -- python3 $W
step lds rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d "$OUT/lds" -o run -- python3 $W
echo PROFILE DONE
