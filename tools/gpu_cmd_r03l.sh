cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for b in lab_ms lab_ms_w8; do
  timeout -k 10 200 tools/$b > gpurun_out/${b}_r03l.log 2>&1 || exit $?
  echo "== $b"; grep -E "us |==|differ|MISMATCH" gpurun_out/${b}_r03l.log | grep -iE "one-pass|cache|differ|mismatch|product math" | cut -c1-90
done
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r03l.log 2>&1 || exit $?
tail -c 300 gpurun_out/bench_r03l.log
