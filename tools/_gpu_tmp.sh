cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/ms_host_profile.py > gpurun_out/ms_host_r04zd.log 2>&1
