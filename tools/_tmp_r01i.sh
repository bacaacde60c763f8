set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_r01i.log 2>&1 || exit $?
tail -1 gpurun_out/bench_r01i.log | cut -c1-600
GC_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/bench_r01i_w2gloo.log 2>&1 || exit $?
tail -1 gpurun_out/bench_r01i_w2gloo.log | cut -c1-400
echo done
