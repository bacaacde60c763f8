cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
GCODEC_LIB=$(pwd)/gradient-compression_amd/lib_w7/libgcodec.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "encode_w1 or ms_one_pass or fused" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_w7_r03zf.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_w7_r03zf.log; [ $rc -ne 0 ] && exit $rc
for v in base w7 base w7; do
if [ $v = w7 ]; then export GCODEC_LIB=$(pwd)/gradient-compression_amd/lib_w7/libgcodec.so; else unset GCODEC_LIB; fi
timeout -k 10 300 python tools/ms_size_sweep.py > gpurun_out/ms_sweep_r03zf_$v.log 2>&1 || exit $?
echo "$v"; grep -E "rounds=(1.000|1.246|3.000)" gpurun_out/ms_sweep_r03zf_$v.log | cut -c25-60
done
