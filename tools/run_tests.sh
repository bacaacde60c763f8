#!/bin/bash
# one gpurun call: GPU test suite (+ optional bench)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-t}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
if [ "${2:-}" = "bench" ]; then
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 > gpurun_out/bench_$TAG.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_$TAG.log | cut -c1-400
fi
