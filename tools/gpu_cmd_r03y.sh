cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python tools/torch_mode_sched.py > gpurun_out/torch_sched_r03y.log 2>&1; rc=$?; cat gpurun_out/torch_sched_r03y.log; exit $rc
