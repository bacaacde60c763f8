#!/bin/bash
# One gpurun call for a round's closing evidence: smoke, GPU tests, bench,
# the N=2 gloo rehearsal of the bench, rocprofv3 over the bench (trace + PMC)
# and over tools/prof_kernels.py (trace + PMC + SQ).  Every step has its own
# time limit; a timeout, signal or fault (exit >= 124) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-final}
bash tools/gpu_check.sh "$TAG" || exit $?
grep -q "STOP after" gpurun_out/steps.log && exit 1
timeout -k 10 900 bash tools/profile_r02.sh "$TAG"
