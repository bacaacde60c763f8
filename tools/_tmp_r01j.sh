set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_r01j.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r01j.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 tools/encode_lab > gpurun_out/lab_r01j.log 2>&1 || exit $?
echo done
