"""Data-parallel reducers with the reference's names and phase structure
(reducer.py), on the packed carry-free codec and RCCL.

    reference (reducer.py)                              here
    Reducer / TensorBuffer                 26-68        Reducer / TensorBuffer
    QSGDMaxNormReducer                     498-554      QSGDMaxNormReducer
    GlobalRandKMaxNormReducer              697-766      GlobalRandKMaxNormReducer
    QSGDMaxNormTwoScaleReducer             1454-1531    QSGDMaxNormTwoScaleReducer
    GlobalRandKMaxNormTwoScaleReducer      1534-1633    GlobalRandKMaxNormTwoScaleReducer
    QSGDMaxNormMultiScaleReducer           1636-1715    QSGDMaxNormMultiScaleReducer

Per step: flatten -> local max-norm (HIP) -> all_reduce MAX (4 B) ->
[multi-scale: mask encode -> all_reduce SUM of thermometer lanes] -> encode
(quantize + pack, HIP) -> ONE all_reduce SUM of the packed uint32 words ->
decode (+ 1/W, HIP) -> setgrad.  The reference all-gathers the norm and
all-reduces int8/int32 q (which overflows int8 once W*(2^b-1) > 127); the
packed lanes are sized for W so the SUM never carries (SURVEY §7 hard part 4).
Outputs equal the reference's (torch-mode RNG) for every W where the
reference does not overflow.
"""
from __future__ import annotations

import collections
import contextlib
import random

import numpy as np
import torch
import torch.distributed as dist

from . import codec as _hip_codec
from . import compressors as C
from .rng import default_generator


class _NullTimer:
    def __call__(self, label, epoch=-1.0, verbosity=1):
        return contextlib.nullcontext()


def set_seed(seed: int, generator=None):
    """seed.py:6-11 plus the codec's own generator."""
    np.random.seed(seed)
    random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    (generator or default_generator).manual_seed(seed)


class Reducer:
    """reducer.py:26-43."""

    SEG_CACHE = 8  # gc_segments tables kept (grad_in + grad_out lists of a few recent steps)

    def __init__(self, device, timer=None, codec=None, generator=None, group=None, fused=True, topology=None):
        if dist.is_available() and dist.is_initialized():
            self.n_workers = dist.get_world_size(group)
            self.rank = dist.get_rank(group)
        else:
            self.n_workers = 1
            self.rank = 0
        self._device = device
        self._timer = timer or _NullTimer()
        self._codec = codec or _hip_codec
        self._gen = generator or default_generator
        self._group = group
        self._topology = topology  # NodeTopology: two-level (xGMI / network) collectives
        if topology is not None and group is not None:
            raise ValueError("topology spans the default process group; pass one or the other")
        self._fused = fused
        self._seg_cache = collections.OrderedDict()  # LRU of gc_segments tables by tensor-list key

    def reduce(self, grad_in, grad_out):
        raise NotImplementedError()

    # -- collectives (RCCL over xGMI when the group is "nccl") -------------
    def _all_reduce(self, t, op=dist.ReduceOp.SUM):
        if self.n_workers > 1:
            if self._topology is not None:  # multi-node: reduce-scatter / all-reduce / all-gather
                return self._topology.all_reduce(t, op)
            dist.all_reduce(t, op=op, group=self._group)
        return t

    def _compressor(self, cls, *args):
        c = cls(self._device, *args, generator=self._gen)
        c.backend = self._codec
        return c

    @staticmethod
    def n_bits(tensor):
        return 8 * tensor.nelement() * tensor.element_size()

    def _setgrad(self, flat, grad_out):
        """reducer.py:543-549 (the 1/W is already folded into `flat`)."""
        for grad, out in zip(flat, grad_out):
            out.copy_(grad)

    def _setgrad_scaled(self, flat, grad_out, alpha):
        """reducer.py:755-761: out[:] = 0; out.add_(grad, alpha) — RN(alpha*g) + 0."""
        segs = self._segments(grad_out)
        if segs is not None:
            self._codec.segments_scatter(flat.buffer, segs, alpha)
            return
        for grad, out in zip(flat, grad_out):
            out.zero_()
            out.add_(grad, alpha=alpha)

    # -- fused TensorBuffer (gc_segments) ----------------------------------
    def _segments(self, tensors):
        """The codec's device table for a parameter list (cached per list), or
        None when the codec has none or a tensor is not contiguous fp32 on the
        GPU — then the reducer takes the TensorBuffer path."""
        make = getattr(self._codec, "Segments", None)
        if not self._fused or make is None:
            return None
        if not isinstance(tensors, (list, tuple)):
            tensors = list(tensors)
        if not tensors:
            return None
        # keyed by the tensors' data pointers and sizes (what the table holds): a
        # table stays valid while the list it describes lives at the same
        # addresses (the caching allocator usually hands a re-created p.grad the
        # same block every step); LRU, so the stable send-buffer entry survives
        # reallocated grad lists.  fp32 / one GPU / contiguous is checked when a
        # table is built (Segments.eligible_list), not on every hit.
        key = make.key_of(tensors)
        segs = self._seg_cache.get(key)
        if segs is None:
            if not make.eligible_list(tensors):
                return None
            if len(self._seg_cache) >= self.SEG_CACHE:
                self._seg_cache.popitem(last=False)
            segs = self._seg_cache[key] = make(tensors)
        else:
            self._seg_cache.move_to_end(key)
        return segs

    def _flat_pack(self, grad_in):
        """reducer.py:512-516: TensorBuffer(grad_in) (+ the local max-norm).
        Fused: one pass over the tensors writes the flat bucket and the norm.
        -> (flat TensorBuffer, local norm or None)"""
        segs = self._segments(grad_in)
        if segs is None:
            with self._timer("reduce.flat_pack"):
                flat = TensorBuffer(grad_in)
            return flat, None
        with self._timer("reduce.flat_pack"):
            buf, norm = self._codec.segments_flatten_absmax(segs)
        return TensorBuffer.of_flat(grad_in, buf), norm

    def _max_norm(self, flat, local=None, idx=None):
        with self._timer("reduce.norm", verbosity=2):
            if local is None or idx is not None:
                local = self._codec.absmax(flat.buffer, idx=idx)
            return self._all_reduce(local, dist.ReduceOp.MAX)


class TensorBuffer:
    """reducer.py:46-68: flatten a list of tensors into one fp32 bucket."""

    def __init__(self, tensors):
        indices = [0]
        for tensor in tensors:
            indices.append(indices[-1] + tensor.nelement())
        self._start_idx = indices[:-1]
        self._end_idx = indices[1:]
        self._len_tensors = len(tensors)
        self._tensor_shapes = [tensor.size() for tensor in tensors]
        self.buffer = torch.cat([tensor.reshape(-1) for tensor in tensors])

    def __getitem__(self, index):
        return self.buffer[self._start_idx[index]:self._end_idx[index]].view(self._tensor_shapes[index])

    def __len__(self):
        return self._len_tensors

    @classmethod
    def of_flat(cls, tensors, buffer):
        """A TensorBuffer over an already-flattened bucket (no torch.cat)."""
        self = cls.__new__(cls)
        indices = [0]
        for tensor in tensors:
            indices.append(indices[-1] + tensor.nelement())
        self._start_idx = indices[:-1]
        self._end_idx = indices[1:]
        self._len_tensors = len(tensors)
        self._tensor_shapes = [tensor.size() for tensor in tensors]
        self.buffer = buffer
        return self

    def with_buffer(self, buffer):
        self.buffer = buffer
        return self


class QSGDMaxNormReducer(Reducer):
    """reducer.py:498-554."""

    def __init__(self, device, timer=None, quantization_level=8, **kw):
        super().__init__(device, timer, **kw)
        self._quantization_level = quantization_level

    def reduce(self, grad_in, grad_out):
        W = self.n_workers
        comp = self._compressor(C.QSGDMaxNormCompressor, self._quantization_level)
        flat, local = self._flat_pack(grad_in)
        n = flat.buffer.numel()
        norm = self._max_norm(flat, local)
        with self._timer("reduce.compress", verbosity=2):
            words = comp.encode(norm, flat.buffer, world=W)
        with self._timer("reduce.reduce.vector", verbosity=2):
            self._all_reduce(words)
        bits = self.n_bits(norm) + self.n_bits(words)
        out_segs = self._segments(grad_out)
        with self._timer("reduce.decompress", verbosity=2):
            if out_segs is not None:  # decode + 1/W straight into grad_out (setgrad fused)
                comp.decode_segments(norm, words, out_segs, world=W, alpha=1.0 / W)
            else:
                flat.buffer = comp.decode(norm, words, n, world=W, alpha=1.0 / W)
        with self._timer("reduce.setgrad", verbosity=2):
            if out_segs is None:
                self._setgrad(flat, grad_out)
        return bits


class GlobalRandKMaxNormReducer(Reducer):
    """reducer.py:697-766: K coordinates per step from a seeded permutation,
    popped from the end; unselected coordinates keep the local gradient."""

    def __init__(self, device, timer=None, seed=42, K=10000, quantization_level=8, **kw):
        super().__init__(device, timer, **kw)
        self._quantization_level = quantization_level
        self._seed = seed
        self._K = K
        self._indices_queue = []
        self._bufs = {}

    def _next_indices(self, n, device):
        """reducer.py:717-722: on refill set_seed, torch.randperm(n) (CPU
        generator, the reference's permutation) split into K-chunks, popped
        from the end.  The permutation goes to the device ONCE per refill (one
        8n-byte copy every ceil(n/K) steps: 118 MB per 1,473 steps for VGG16)
        and the queue holds device slices, so a step does no host->device
        index copy (the reference copies its numpy chunk every step, 722-723)."""
        if not self._indices_queue:
            set_seed(self._seed, self._gen)
            perm = torch.randperm(n)
            if perm.device != device:
                perm = perm.pin_memory().to(device, non_blocking=True) if device.type == "cuda" else perm.to(device)
            self._indices_queue = list(perm.split(self._K))
        return self._indices_queue.pop()

    def _step_buffers(self, k, device, world):
        """(gathered subset, norm, packed words) for a K-subset, allocated once
        per (K, device, W) and reused every step: the kernels that read the
        previous step's buffers are queued ahead on the same stream, and the
        collectives are waited for in stream order (a fresh torch.empty of each
        cost host time every step; the refill's last chunk has its own K)."""
        key = (k, device, world)
        b = self._bufs.get(key)
        if b is None:
            lanes = self._codec.qsgd_layout(k, self._quantization_level, world)
            if len(self._bufs) >= 4:
                self._bufs.clear()
            b = self._bufs[key] = (torch.empty(k, dtype=torch.float32, device=device),
                                   torch.empty(1, dtype=torch.float32, device=device),
                                   torch.empty(lanes.plane_words, dtype=torch.int32, device=device))
        return b

    def _randk_compressor(self):
        return self._compressor(C.GlobalRandKMaxNormCompressor, self._quantization_level)

    def _reduce_segments(self, comp, in_segs, out_segs):
        """The step with grad_in / grad_out addressed in place (no flat bucket):
        gather + norm (+ encode at W = 1) read each index from its tensor, the
        setgrad copies every coordinate tensor to tensor (x 1/W) and the
        decode-scatter overwrites the K selected ones (reducer.py:754-761: the
        same values, written once instead of via the bucket)."""
        W = self.n_workers
        idx = self._next_indices(in_segs.n, in_segs.device)
        k = idx.numel()
        codec = self._codec
        xk, norm, words = self._step_buffers(k, in_segs.device, W)
        if codec.randk_fused_ok(k, self._quantization_level, W):
            with self._timer("reduce.compress", verbosity=2):
                words, norm = comp.encode_w1_segments(in_segs, idx, out=words, xk=xk, norm=norm)
        else:
            with self._timer("reduce.norm", verbosity=2):
                xk, local = codec.randk_gather_absmax_segments(in_segs, idx, xk=xk, norm=norm)
                norm = self._all_reduce(local, dist.ReduceOp.MAX)
            with self._timer("reduce.compress", verbosity=2):
                words = comp.encode(norm, xk, world=W, out=words)
        with self._timer("reduce.reduce.vector", verbosity=2):
            self._all_reduce(words)
        bits = self.n_bits(norm) + self.n_bits(words)
        with self._timer("reduce.setgrad", verbosity=2):
            codec.segments_copy(in_segs, out_segs, 1.0 / W)
        with self._timer("reduce.decompress", verbosity=2):
            comp.decode_scatter_segments(norm, words, idx, out_segs, world=W, alpha=1.0 / W)
        return bits

    def _segment_pair(self, grad_in, grad_out):
        """(in, out) tables when both lists are fused-addressable with equal
        tensor sizes and the subset fits the gather kernel, else None."""
        codec = self._codec
        if not hasattr(codec, "randk_gather_absmax_segments"):
            return None
        in_segs = self._segments(grad_in)
        out_segs = self._segments(grad_out) if in_segs is not None else None
        if out_segs is None or in_segs.key[1] != out_segs.key[1] or min(self._K, in_segs.n) > codec.RANDK_GATHER_MAX:
            return None
        return in_segs, out_segs

    def reduce(self, grad_in, grad_out):
        W = self.n_workers
        comp = self._randk_compressor()
        pair = self._segment_pair(grad_in, grad_out)
        if pair is not None:
            return self._reduce_segments(comp, *pair)
        flat, _ = self._flat_pack(grad_in)
        n = flat.buffer.numel()
        idx = self._next_indices(n, flat.buffer.device)
        k = idx.numel()
        codec = self._codec
        if hasattr(codec, "randk_fused_ok") and codec.randk_fused_ok(k, self._quantization_level, W):
            # gather + max-norm + encode in one launch (the MAX over one rank is the identity)
            with self._timer("reduce.compress", verbosity=2):
                words, norm = comp.encode_w1(flat.buffer, idx)
        elif hasattr(codec, "randk_gather_absmax") and k <= codec.RANDK_GATHER_MAX:
            # the subset gathered once (with its local norm); the encode reads it densely
            with self._timer("reduce.norm", verbosity=2):
                xk, local = codec.randk_gather_absmax(flat.buffer, idx)
                norm = self._all_reduce(local, dist.ReduceOp.MAX)
            with self._timer("reduce.compress", verbosity=2):
                words = comp.encode(norm, xk, world=W)
        else:
            norm = self._max_norm(flat, idx=idx)
            with self._timer("reduce.compress", verbosity=2):
                words = comp.encode(norm, flat.buffer, world=W, idx=idx)
        with self._timer("reduce.reduce.vector", verbosity=2):
            self._all_reduce(words)
        bits = self.n_bits(norm) + self.n_bits(words)
        with self._timer("reduce.decompress", verbosity=2):
            comp.decode(norm, words, k, world=W, alpha=1.0, idx=idx, out=flat.buffer)
        with self._timer("reduce.setgrad", verbosity=2):
            self._setgrad_scaled(flat, grad_out, 1.0 / W)
        return bits


class QSGDMaxNormTwoScaleReducer(Reducer):
    """reducer.py:1454-1531: common high-resolution mask (AND over ranks),
    blended two-scale integers, one integer all-reduce."""

    _cls = C.QSGDMaxNormTwoScaleCompressor

    def __init__(self, device, timer=None, lower_quantization_level=6, higher_quantization_level=10, **kw):
        super().__init__(device, timer, **kw)
        self._lower_quantization_level = lower_quantization_level
        self._higher_quantization_level = higher_quantization_level

    def _make(self):
        return self._compressor(self._cls, self._lower_quantization_level, self._higher_quantization_level)

    def _reduce_scales(self, comp, flat, idx, n, local=None):
        W = self.n_workers
        codec = self._codec
        x = flat.buffer
        if idx is not None and hasattr(codec, "randk_gather_absmax") and idx.numel() <= codec.RANDK_GATHER_MAX:
            # GlobalRandK: gather the subset once (with its local norm); both
            # multi-scale passes then read it densely
            with self._timer("reduce.norm", verbosity=2):
                x, local = codec.randk_gather_absmax(flat.buffer, idx)
                norm = self._all_reduce(local, dist.ReduceOp.MAX)
            idx = None
        else:
            norm = self._max_norm(flat, local, idx)
        with self._timer("reduce.compress", verbosity=2):
            both = comp.encode_w1(norm, x) if W == 1 and idx is None else None
            if both is not None:  # one pass: the mask MIN over one rank is the identity
                mask, words = both
            else:
                mask = comp.encode_mask(norm, x, world=W, idx=idx)
                self._all_reduce(mask)
                words = comp.encode(norm, x, mask, world=W, idx=idx)
        with self._timer("reduce.reduce.vector", verbosity=2):
            self._all_reduce(words)
        bits = self.n_bits(norm) + self.n_bits(mask) + self.n_bits(words)
        return norm, mask, words, bits

    def reduce(self, grad_in, grad_out):
        W = self.n_workers
        comp = self._make()
        flat, local = self._flat_pack(grad_in)
        n = flat.buffer.numel()
        norm, mask, words, bits = self._reduce_scales(comp, flat, None, n, local)
        out_segs = self._segments(grad_out)
        with self._timer("reduce.decompress", verbosity=2):
            if out_segs is not None:  # decode + 1/W straight into grad_out (setgrad fused)
                comp.decode_segments(norm, words, mask, out_segs, world=W, alpha=1.0 / W)
            else:
                flat.buffer = comp.decode(norm, words, mask, n, world=W, alpha=1.0 / W)
        with self._timer("reduce.setgrad", verbosity=2):
            if out_segs is None:
                self._setgrad(flat, grad_out)
        return bits


class GlobalRandKMaxNormTwoScaleReducer(QSGDMaxNormTwoScaleReducer):
    """reducer.py:1534-1633."""

    _cls = C.GlobalRandKMaxNormTwoScaleCompressor

    def __init__(self, device, timer=None, seed=42, K=10000, lower_quantization_level=6,
                 higher_quantization_level=10, **kw):
        super().__init__(device, timer, lower_quantization_level, higher_quantization_level, **kw)
        self._seed = seed
        self._K = K
        self._indices_queue = []

    _next_indices = GlobalRandKMaxNormReducer._next_indices
    _segment_pair = GlobalRandKMaxNormReducer._segment_pair

    def _reduce_segments(self, comp, in_segs, out_segs):
        """The step without a flat bucket (as GlobalRandKMaxNormReducer's):
        the subset gathered from the tensors, the two-scale passes on it, the
        setgrad tensor to tensor and the decode-scatter into grad_out
        (reducer.py:1568-1628)."""
        W = self.n_workers
        codec = self._codec
        idx = self._next_indices(in_segs.n, in_segs.device)
        with self._timer("reduce.norm", verbosity=2):
            xk, local = codec.randk_gather_absmax_segments(in_segs, idx)
            norm = self._all_reduce(local, dist.ReduceOp.MAX)
        with self._timer("reduce.compress", verbosity=2):
            both = comp.encode_w1(norm, xk) if W == 1 else None
            if both is not None:
                mask, words = both
            else:
                mask = comp.encode_mask(norm, xk, world=W)
                self._all_reduce(mask)
                words = comp.encode(norm, xk, mask, world=W)
        with self._timer("reduce.reduce.vector", verbosity=2):
            self._all_reduce(words)
        bits = self.n_bits(norm) + self.n_bits(mask) + self.n_bits(words)
        with self._timer("reduce.setgrad", verbosity=2):
            codec.segments_copy(in_segs, out_segs, 1.0 / W)
        with self._timer("reduce.decompress", verbosity=2):
            comp.decode_scatter_segments(norm, words, mask, idx, out_segs, world=W, alpha=1.0 / W)
        return bits

    def reduce(self, grad_in, grad_out):
        W = self.n_workers
        comp = self._make()
        pair = self._segment_pair(grad_in, grad_out)
        if pair is not None and hasattr(comp, "decode_scatter_segments"):
            return self._reduce_segments(comp, *pair)
        flat, _ = self._flat_pack(grad_in)
        n = flat.buffer.numel()
        idx = self._next_indices(n, flat.buffer.device)
        k = idx.numel()
        norm, mask, words, bits = self._reduce_scales(comp, flat, idx, k)
        with self._timer("reduce.decompress", verbosity=2):
            comp.decode(norm, words, mask, k, world=W, alpha=1.0, idx=idx, out=flat.buffer)
        with self._timer("reduce.setgrad", verbosity=2):
            self._setgrad_scaled(flat, grad_out, 1.0 / W)
        return bits


class QSGDMaxNormMultiScaleReducer(QSGDMaxNormTwoScaleReducer):
    """reducer.py:1636-1715: resolution mask MIN over ranks (thermometer lanes
    + SUM), selected-level integers, one integer all-reduce."""

    def __init__(self, device, timer=None, quantization_levels=None, **kw):
        Reducer.__init__(self, device, timer, **kw)
        if not quantization_levels:
            quantization_levels = [6, 10]
        self._quantization_levels = sorted(quantization_levels)

    def _make(self):
        return self._compressor(C.QSGDMaxNormMultiScaleCompressor, list(self._quantization_levels))
