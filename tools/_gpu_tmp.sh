cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for b in lab_ms lab_ms_wpe6 lab_ms_wpe7 lab_ms; do
  echo "== $b" >> gpurun_out/lab_ms_wpe_r04zb.log
  timeout -k 10 200 tools/$b 2>&1 | grep "^product one\|^lab one-pass octet PREFETCH\|^lab mask + cache octet ROLL\|^lab select octet ROLL\|^product mask + cache\|^product select encode" >> gpurun_out/lab_ms_wpe_r04zb.log || exit $?
done
