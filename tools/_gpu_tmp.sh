cd "${GRAFT_REPO_ROOT:-/root/repo}"
PYTEST_K="greedy4 or qsgdbp or packer or torch_mode" bash tools/gpu.sh r04k tests || exit $?
(cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r04k -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_packers.py > $GRAFT_REPO_ROOT/gpurun_out/prof_r04k.log 2>&1) || exit $?
cd /tmp && export TMPDIR=/tmp
REPS=5 timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex "k_g4" --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_r04k -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_packers.py > $GRAFT_REPO_ROOT/gpurun_out/pmc_r04k.log 2>&1
