#!/bin/bash
# VALU-issue counters for the encode kernel (separate pass; no tracing combined)
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/pmc_valu"
mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_INT64 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
  --kernel-include-regex "k_qsgd_encode|k_absmax" --output-format csv -d "$OUT" -o run -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 2 --cpu-seconds 0 --no-extras > "$OUT/log.txt" 2>&1
echo "pmc rc=$?"
