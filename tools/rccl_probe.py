"""Probe: can RCCL run W ranks on ONE GPU (the pool's boxes have one card)?

Spawns W processes, all on cuda:0, each initialising an "nccl" (= RCCL)
process group, then runs the path's collectives once: all_reduce(MAX) of a
float32 norm and all_reduce(SUM) of int32 packed words.  Prints one line per
rank and exits non-zero on any failure.  Run under `timeout -k`.
usage: python tools/rccl_probe.py [W]
"""
import os
import sys
import tempfile

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, init_file):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"file://{init_file}", rank=rank, world_size=world, device_id=dev)
    nrm = torch.tensor([float(rank + 1)], device=dev)
    dist.all_reduce(nrm, op=dist.ReduceOp.MAX)
    w = torch.full((1 << 20,), rank + 1, dtype=torch.int32, device=dev)
    dist.all_reduce(w)
    torch.cuda.synchronize()
    ok = nrm.item() == world and int(w[0].item()) == world * (world + 1) // 2 and bool((w == w[0]).all())
    print(f"rank {rank}: backend {dist.get_backend()} world {dist.get_world_size()} "
          f"rccl {torch.cuda.nccl.version()} max {nrm.item()} sum {int(w[0].item())} ok {ok}", flush=True)
    dist.barrier()
    dist.destroy_process_group()
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(worker, args=(world, os.path.join(td, "init")), nprocs=world, join=True)
    print("RCCL probe OK", flush=True)
