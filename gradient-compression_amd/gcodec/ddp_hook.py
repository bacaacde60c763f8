"""DDP communication hook: the packed QSGD-MaxNorm codecs on torch DDP's
gradient buckets (bucketed backward/communication overlap).

The reference reduces ONE monolithic bucket after the whole backward pass
(trainer.py:183-196 -> reducer.reduce, reducer.py:498-554, 1454-1531,
1636-1715).  torch's DistributedDataParallel instead hands every gradient
bucket (bucket_cap_mb, default 25 MB) to a communication hook as soon as
autograd has produced it, so the encode -> all-reduce -> decode of bucket k
runs while the backward pass is still computing the gradients of the layers
in front of it.  Per bucket the hook runs the same algorithm as the reducers:

    QSGD-MaxNorm (levels=None; QSGDMaxNormReducer):
        local max-norm (HIP) -> all_reduce MAX (4 B) -> quantize + stochastic
        round + pack (HIP, carry-free lanes sized for W) -> async all_reduce
        SUM of the packed words -> decode + 1/W into the bucket (HIP) when the
        collective's future completes

    two-scale / multi-scale (levels=[lo, hi, ...]; QSGDMaxNormTwoScaleReducer,
    QSGDMaxNormMultiScaleReducer):
        max-norm -> MAX -> mask encode (thermometer lanes) -> SUM of the mask
        lanes (the reference's PRODUCT / MIN, reducer.py:1494-1499, 1680-1685)
        -> select encode at the common levels -> async SUM of the packed words
        -> decode (order 1 two-scale, order 0 multi-scale) + 1/W into the
        bucket when the future completes

    model = torch.nn.parallel.DistributedDataParallel(model)
    model.register_comm_hook(QSGDHookState(bits=4), qsgd_hook)
    model.register_comm_hook(QSGDHookState(levels=[2, 4], two_scale=True), qsgd_hook)

With the "nccl" backend (RCCL on ROCm) the collectives run on RCCL's stream
and every kernel is enqueued behind them without blocking the host.  The
draws come from a per-rank Generator (the reference seeds every rank with
seed + rank, trainer.py:158); each bucket reserves n (x levels) draws, so a
bucket's words are reproducible from (seed, offset) like every other codec call.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import codec as _hip_codec
from .rng import Generator


class QSGDHookState:
    """State of qsgd_hook: quantization bits (or multi-scale levels), process
    group, RNG, codec."""

    def __init__(self, bits: int = 4, process_group=None, generator: Generator | None = None, codec=None,
                 seed: int = 42, topology=None, levels=None, two_scale: bool = False):
        self.bits = int(bits)
        self.levels = sorted(int(b) for b in levels) if levels else None
        if self.levels is not None and len(self.levels) < 2:
            raise ValueError("levels: at least two quantization levels (or levels=None for QSGD-MaxNorm)")
        if two_scale and (self.levels is None or len(self.levels) != 2):
            raise ValueError("two_scale needs exactly two levels")
        # decode op order: two-scale RN(RN(norm/s)*q) (compressors.py:668-680),
        # multi-scale RN(RN(q*norm)/s) (819-826)
        self.order = 1 if two_scale else 0
        self.group = process_group
        self.topology = topology  # NodeTopology (multi-node): two-level collectives, lanes sized for the world
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        rank = dist.get_rank(process_group) if dist.is_initialized() else 0
        self.gen = generator or Generator(seed + rank, "philox")
        self.codec = codec or _hip_codec
        self.buckets = 0    # buckets reduced
        self.bits_sent = 0  # norm + mask + packed words, per rank (reducer.py n_bits convention)


def _sum_future(state: QSGDHookState, t: torch.Tensor) -> torch.futures.Future:
    """SUM all-reduce of t as a future (RCCL async; the topology's three
    collectives are enqueued in order; a completed future at W = 1)."""
    if state.world > 1 and state.topology is None:
        return dist.all_reduce(t, group=state.group, async_op=True).get_future()
    if state.world > 1:
        state.topology.all_reduce(t)
    fut = torch.futures.Future()
    fut.set_result([t])
    return fut


def _keep(t: torch.Tensor):
    """The callbacks run on a stream from torch's pool, and torch records only
    the future's value storages there: a tensor allocated on the hook's stream
    (the norm) must be recorded on the callback's stream before a kernel there
    reads it, or the caching allocator may hand its block to the backward pass
    first."""
    if t.is_cuda:
        t.record_stream(torch.cuda.current_stream(t.device))


def qsgd_hook(state: QSGDHookState, bucket) -> torch.futures.Future:
    """DDP comm hook (register_comm_hook): reduce one gradient bucket with the
    packed QSGD-MaxNorm codec (or its two-/multi-scale form when state.levels
    is set); the future's value is the averaged bucket."""
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
    state.buckets += 1
    if state.levels is not None:
        return _multiscale(state, x, n, norm)
    rng = state.gen.reserve(n, 1, device=x.device, backend=codec)
    words = codec.qsgd_encode(x, norm, state.bits, rng, W)
    state.bits_sent += 32 + 32 * words.numel()

    def _decode(f):
        summed = f.value()[0]
        _keep(norm)
        return codec.qsgd_decode(summed, n, norm, state.bits, W, 1.0 / W, out=x)

    return _sum_future(state, words).then(_decode)


def _multiscale(state: QSGDHookState, x, n, norm) -> torch.futures.Future:
    codec, W, levels = state.codec, state.world, state.levels
    rng = state.gen.reserve(n, len(levels), device=x.device, backend=codec)
    w1_ok = getattr(codec, "ms_w1_ok", None)
    if W == 1 and w1_ok is not None and w1_ok(x, levels):
        # one pass over x (the MIN over one rank is the identity): the same
        # words as the mask + select passes below
        mask, words = codec.ms_encode_w1(x, norm, levels, rng)
    else:
        # W > 1: the mask pass also writes the packed q cache when the backend
        # has one for these levels, and the select reads it instead of x and
        # the draws (no Philox in the select; _MultiScalePacked's q_cache)
        cbytes = getattr(codec, "ms_cache_bytes", None)
        nb = cbytes(n, levels) if W > 1 and cbytes is not None and x.data_ptr() % 16 == 0 else 0
        ck = {"cache": torch.empty(n * nb, dtype=torch.uint8, device=x.device)} if nb else {}
        mask = codec.ms_mask_encode(x, norm, levels, rng, W, **ck)
        # the mask SUM is enqueued in line (with RCCL the stream waits on it, the
        # host does not): the select pass needs the common levels before it runs
        if W > 1:
            if state.topology is not None:
                state.topology.all_reduce(mask)
            else:
                dist.all_reduce(mask, group=state.group)
        words = codec.ms_select_encode(x, norm, levels, rng, mask, W, **ck)
    state.bits_sent += 32 + 32 * mask.numel() + 32 * words.numel()

    def _decode(f):
        summed = f.value()[0]
        _keep(norm)
        _keep(mask)
        return codec.ms_decode(summed, mask, n, norm, levels, W, state.order, 1.0 / W, out=x)

    return _sum_future(state, words).then(_decode)
