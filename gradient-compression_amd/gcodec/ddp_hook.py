"""DDP communication hook: the packed QSGD-MaxNorm codec on torch DDP's
gradient buckets (bucketed backward/communication overlap).

The reference reduces ONE monolithic bucket after the whole backward pass
(trainer.py:183-196 -> reducer.reduce, reducer.py:498-554).  torch's
DistributedDataParallel instead hands every gradient bucket (bucket_cap_mb,
default 25 MB) to a communication hook as soon as autograd has produced it,
so the encode -> all-reduce -> decode of bucket k runs while the backward
pass is still computing the gradients of the layers in front of it.  Per
bucket the hook runs the same algorithm as QSGDMaxNormReducer:

    local max-norm (HIP) -> all_reduce MAX (4 B) -> quantize + stochastic
    round + pack (HIP, carry-free lanes sized for W) -> async all_reduce SUM
    of the packed words -> decode + 1/W into the bucket (HIP) when the
    collective's future completes

    model = torch.nn.parallel.DistributedDataParallel(model)
    model.register_comm_hook(QSGDHookState(bits=4), qsgd_hook)

With the "nccl" backend (RCCL on ROCm) the collectives run on RCCL's stream
and the decode is enqueued behind the SUM without blocking the host.  The
draws come from a per-rank Generator (the reference seeds every rank with
seed + rank, trainer.py:158); each bucket reserves n draws, so a bucket's
words are reproducible from (seed, offset) like every other codec call.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import codec as _hip_codec
from .rng import Generator


class QSGDHookState:
    """State of qsgd_hook: quantization bits, process group, RNG, codec."""

    def __init__(self, bits: int = 4, process_group=None, generator: Generator | None = None, codec=None,
                 seed: int = 42, topology=None):
        self.bits = int(bits)
        self.group = process_group
        self.topology = topology  # NodeTopology (multi-node): two-level collectives, lanes sized for the world
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        rank = dist.get_rank(process_group) if dist.is_initialized() else 0
        self.gen = generator or Generator(seed + rank, "philox")
        self.codec = codec or _hip_codec
        self.buckets = 0    # buckets reduced
        self.bits_sent = 0  # norm + packed words, per rank (reducer.py n_bits convention)


def qsgd_hook(state: QSGDHookState, bucket) -> torch.futures.Future:
    """DDP comm hook (register_comm_hook): reduce one gradient bucket with the
    packed QSGD-MaxNorm codec; the future's value is the averaged bucket."""
    x = bucket.buffer()
    n = x.numel()
    codec, W = state.codec, state.world
    norm = codec.absmax(x)
    topo = state.topology
    if W > 1:
        if topo is not None:
            topo.all_reduce(norm, dist.ReduceOp.MAX)
        else:
            dist.all_reduce(norm, op=dist.ReduceOp.MAX, group=state.group)
    rng = state.gen.reserve(n, 1, device=x.device, backend=codec)
    words = codec.qsgd_encode(x, norm, state.bits, rng, W)
    state.buckets += 1
    state.bits_sent += 32 + 32 * words.numel()
    if W > 1 and topo is None:
        fut = dist.all_reduce(words, group=state.group, async_op=True).get_future()
    elif W > 1:  # reduce-scatter / inter-node all-reduce / all-gather, enqueued in order
        topo.all_reduce(words)
        fut = torch.futures.Future()
        fut.set_result([words])
    else:
        fut = torch.futures.Future()
        fut.set_result([words])

    def _decode(f):
        summed = f.value()[0]
        return codec.qsgd_decode(summed, n, norm, state.bits, W, 1.0 / W, out=x)

    return fut.then(_decode)
