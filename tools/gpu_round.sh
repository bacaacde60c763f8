#!/bin/bash
# one gpurun call: full GPU test suite, then the default bench (every step has
# its own time limit; a timeout / signal / fault ends the script)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-t}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
if [ "${2:-}" = "bench" ]; then
  timeout -k 10 600 python bench.py --steps 50 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1 || exit $?
  tail -c 300 gpurun_out/bench_$TAG.log
fi
