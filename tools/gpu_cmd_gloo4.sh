# N = 4 rehearsal of the bench's multi-rank control flow on one GPU (gloo, 4
# ranks sharing the card): exercises the world >= 4 legs (the 2x-node
# NodeTopology reduce path) before a driver SCALE run.  Not a perf number.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rm -f gpurun_out/gloo4.rc
( env GC_BENCH_BACKEND=gloo timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 3 --warmup 1 --cpu-seconds 0 \
    > gpurun_out/gloo4_r03zj.log 2>&1; echo $? > gpurun_out/gloo4.rc ) &
while [ ! -f gpurun_out/gloo4.rc ]; do sleep 30; echo "tick $(date +%T)"; done
rc=$(cat gpurun_out/gloo4.rc); echo "rc=$rc"; tail -c 1500 gpurun_out/gloo4_r03zj.log; exit $rc
