#!/bin/bash
# one gpurun call: lab2 (ENC_INT A/B + MALL reuse) and the VALU rate table
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-lab2}
timeout -k 10 240 tools/lab2 > gpurun_out/${TAG}.log 2>&1 || { echo "lab2 rc=$?"; tail -5 gpurun_out/${TAG}.log; exit 1; }
tail -60 gpurun_out/${TAG}.log
if [ -x tools/valu_rates ]; then timeout -k 10 60 tools/valu_rates > gpurun_out/${TAG}_valu.log 2>&1; cat gpurun_out/${TAG}_valu.log; fi
