cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PYTEST_K="ms or scale or wide or segments" bash tools/gpu.sh r04y tests || exit $?
timeout -k 10 300 tools/lab_ms > gpurun_out/lab_ms_r04y.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
K=$GRAFT_REPO_ROOT/tools/prof_kernels.py
D=$GRAFT_REPO_ROOT/gpurun_out/prof_r04y_k
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 $K > $GRAFT_REPO_ROOT/gpurun_out/k_trace_r04y.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $D/sq -o run -- python3 $K > $GRAFT_REPO_ROOT/gpurun_out/k_sq_r04y.log 2>&1
