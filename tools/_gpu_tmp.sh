cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PYTEST_K="torch_mode or ms or scale or wide or segments or golden or multirank or parity" bash tools/gpu.sh r04o tests || exit $?
timeout -k 10 300 tools/lab_ms > gpurun_out/lab_ms_r04o.log 2>&1 || exit $?
timeout -k 10 300 python tools/time_torch_mode.py 0,192,256 2,3 > gpurun_out/torch_mode_r04o.log 2>&1 || exit $?
PACKED24=0 timeout -k 10 300 python tools/time_torch_mode.py 0 2 > gpurun_out/torch_mode32_r04o.log 2>&1
