"""Tensor-level API over libgcodec (the HIP backend).

Every function takes/returns torch tensors on a gfx950 device, enqueues on
the current HIP stream and never synchronises (except the torch-mode RNG
hand-off).  Packed streams are int32 tensors (torch/RCCL have no uint32
SUM); the bits are the uint32 lane words of include/gcodec.h.
"""
from __future__ import annotations

import collections
import ctypes as C
import operator
import functools

import numpy as np
import torch

from . import _lib
from ._lib import check

DTYPE_CODE = {torch.int8: _lib.GC_I8, torch.int32: _lib.GC_I32, torch.int64: _lib.GC_I64}


def _dev(t: torch.Tensor) -> torch.device:
    if not t.is_cuda:
        raise _lib.GCodecError(_lib.GC_ENODEV, "gcodec runs on the GPU only: tensor is on "
                               f"{t.device}; there is no CPU fallback")
    _lib.require_device(t.device.index if t.device.index is not None else torch.cuda.current_device())
    return t.device


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream(device) -> C.c_void_p:
    """The current HIP stream of `device` as a raw pointer.  The raw accessor
    skips the Stream object torch.cuda.current_stream builds (~4 us per call,
    tools/host_overhead.py)."""
    if _raw_stream is not None:
        return C.c_void_p(_raw_stream(device.index if device.index is not None else torch.cuda.current_device()))
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _p(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _f32(x: torch.Tensor, what: str) -> torch.Tensor:
    if x.dtype != torch.float32:
        raise _lib.GCodecError(_lib.GC_EINVAL, f"{what}: expected float32, got {x.dtype}")
    if not x.is_contiguous():
        x = x.contiguous()
    return x.view(-1)


def _idx(idx, device):
    if idx is None:
        return None
    if not isinstance(idx, torch.Tensor):
        idx = torch.as_tensor(np.asarray(idx), dtype=torch.int64)
    if idx.dtype != torch.int64:
        idx = idx.to(torch.int64)
    if idx.device != device:
        idx = idx.to(device, non_blocking=True)
    return idx.contiguous().view(-1)


def norm_tensor(norm, device) -> torch.Tensor:
    """The max-norm as a device float32 scalar tensor (no host sync)."""
    if isinstance(norm, torch.Tensor):
        if norm.dtype == torch.float32 and norm.device == device:
            return norm  # the kernels read element 0 through the data pointer
        t = norm.detach()
        if t.dtype != torch.float32:
            t = t.float()
        if t.device != device:
            t = t.to(device)
        return t.reshape(1) if t.dim() == 0 else t.view(-1)[:1]
    return torch.tensor([float(norm)], dtype=torch.float32, device=device)


# ---------------------------------------------------------------------------
# layouts
# ---------------------------------------------------------------------------
@functools.lru_cache(maxsize=512)
def qsgd_layout(n: int, bits: int, world: int = 1) -> _lib.gc_lanes:
    """Lane layout (cached: a per-call ctypes round trip on every encode;
    callers treat the struct as read-only)."""
    ln = _lib.gc_lanes()
    check(_lib.load().gc_qsgd_layout(n, bits, world, C.byref(ln)), "gc_qsgd_layout")
    return ln


def lane_layout(n: int, value_range: int, world: int = 1, offset: int = 0) -> _lib.gc_lanes:
    ln = _lib.gc_lanes()
    check(_lib.load().gc_lane_layout(n, value_range, world, offset, C.byref(ln)), "gc_lane_layout")
    return ln


def _levels_key(levels) -> tuple:
    return tuple(sorted(int(b) for b in levels))


@functools.lru_cache(maxsize=256)
def _levels_struct(lv: tuple) -> _lib.gc_levels:
    if not 1 <= len(lv) <= _lib.GC_MAX_LEVELS:
        raise _lib.GCodecError(_lib.GC_EINVAL, f"1..{_lib.GC_MAX_LEVELS} levels supported")
    s = _lib.gc_levels()
    s.count = len(lv)
    for i, b in enumerate(lv):
        s.bits[i] = b
    return s


def levels_struct(levels) -> _lib.gc_levels:
    """The sorted level list as a gc_levels (cached; callers treat it as read-only)."""
    return _levels_struct(_levels_key(levels))


@functools.lru_cache(maxsize=512)
def _ms_layouts(n: int, lv: tuple, world: int):
    s = _levels_struct(lv)
    ql, ml = _lib.gc_lanes(), _lib.gc_lanes()
    check(_lib.load().gc_ms_layout(n, C.byref(s), world, C.byref(ql)), "gc_ms_layout")
    check(_lib.load().gc_ms_mask_layout(n, C.byref(s), world, C.byref(ml)), "gc_ms_mask_layout")
    return ql, ml


def ms_layouts(n: int, levels, world: int = 1):
    """(q lanes, mask lanes) of a multi-scale bucket (cached like qsgd_layout:
    two ctypes round trips per call otherwise; read-only)."""
    return _ms_layouts(int(n), _levels_key(levels), int(world))


def mask_words_total(ml: _lib.gc_lanes, levels) -> int:
    return (len(levels) - 1) * ml.plane_words


# ---------------------------------------------------------------------------
# max-norm
# ---------------------------------------------------------------------------
_WS = {}


_WS_POOL = {}  # device index -> [zeroed pool tensor, slots handed out]
_WS_POOL_SLOTS = 64


def _absmax_ws(dev, stream) -> torch.Tensor:
    """Self-resetting last-block workspace, one per (device, stream).  Slots
    are cut from a pool zeroed once per device, so a stream's first call
    launches no fill: under HIP-graph capture (a capture stream is a new
    stream) a fill would be captured and re-run at every replay (VERDICT r04
    item 6: the GRandK replay carried a FillFunctor node per step).

    A pool is never made under capture: its zero fill would only
    be a graph node, so eager streams taking slots from it later would find
    unzeroed tickets, and every replay would reset the slots of streams in
    use.  A capture that needs a slot when no pool has one left raises; one
    eager call on the device beforehand makes the pool (64 slots, a new pool
    when they run out; a slot is 256 bytes and stays with its stream)."""
    key = (dev.index, stream.value)
    ws = _WS.get(key)
    if ws is None:
        size = -(-int(_lib.load().gc_absmax_workspace_size()) // 256) * 256
        pool = _WS_POOL.get(dev.index)
        if pool is None or pool[1] == _WS_POOL_SLOTS:
            if torch.cuda.is_current_stream_capturing():
                raise _lib.GCodecError(_lib.GC_EINVAL, "absmax: no zeroed workspace slot for a stream first seen "
                                       "under HIP-graph capture; run one eager absmax on this device first")
            pool = _WS_POOL[dev.index] = [torch.zeros(size * _WS_POOL_SLOTS, dtype=torch.uint8, device=dev), 0]
            # other streams take slots later: the zero fill must be done
            torch.cuda.current_stream(dev).synchronize()
        ws = _WS[key] = pool[0][pool[1] * size:(pool[1] + 1) * size]
        pool[1] += 1
    return ws


def absmax(x: torch.Tensor, idx=None, out: torch.Tensor | None = None) -> torch.Tensor:
    dev = _dev(x)
    x = _f32(x, "absmax")
    idx = _idx(idx, dev)
    n = idx.numel() if idx is not None else x.numel()
    if out is None:
        out = torch.empty(1, dtype=torch.float32, device=dev)
    st = _stream(dev)
    check(_lib.load().gc_absmax_f32(_p(x), _p(idx), n, _p(out), _p(_absmax_ws(dev, st)), st), "gc_absmax_f32")
    return out


# ---------------------------------------------------------------------------
# QSGD-MaxNorm packed
# ---------------------------------------------------------------------------
def qsgd_encode(x, norm, bits, rng, world=1, idx=None, out=None, lanes=None) -> torch.Tensor:
    dev = _dev(x)
    x = _f32(x, "qsgd_encode")
    idx = _idx(idx, dev)
    n = idx.numel() if idx is not None else x.numel()
    lanes = lanes or qsgd_layout(n, bits, world)
    nt = norm_tensor(norm, dev)
    if out is None:
        out = torch.empty(lanes.plane_words, dtype=torch.int32, device=dev)
    r = rng.struct()
    check(_lib.load().gc_qsgd_encode(_p(x), _p(idx), n, _p(nt), bits, C.byref(lanes), C.byref(r), _p(out),
                                     _stream(dev)), "gc_qsgd_encode")
    return out


def qsgd_decode(words, n, norm, bits, world=1, alpha=1.0, idx=None, out=None, lanes=None) -> torch.Tensor:
    dev = _dev(words)
    idx = _idx(idx, dev)
    lanes = lanes or qsgd_layout(n, bits, world)
    nt = norm_tensor(norm, dev)
    if out is None:
        out = torch.empty(n, dtype=torch.float32, device=dev)
    check(_lib.load().gc_qsgd_decode(_p(words), _p(idx), n, _p(nt), bits, C.byref(lanes), float(alpha), _p(out),
                                     _stream(dev)), "gc_qsgd_decode")
    return out


# ---------------------------------------------------------------------------
# small-K GlobalRandK (reducer.py:717-754)
# ---------------------------------------------------------------------------
RANDK_FUSED_MAX = 16384      # K of the one-launch W = 1 encode (gc_randk_encode_w1)
RANDK_FUSED_MAX_BITS = 15    # its lanes are staged as uint16 in LDS (values up to 2 (2^b - 1))


def randk_fused_ok(k: int, bits: int, world: int = 1) -> bool:
    """Whether gc_randk_encode_w1 takes this step (W = 1, K and b within its LDS staging)."""
    return world == 1 and k <= RANDK_FUSED_MAX and bits <= RANDK_FUSED_MAX_BITS
RANDK_GATHER_MAX = 256 * 1024  # K of gc_randk_gather_absmax


def randk_gather_absmax(x, idx, xk=None, norm=None):
    """(xk, norm): the subset x[idx] stored contiguously and its max-norm, in one
    launch (reducer.py:722-726).  At W > 1 the encode then reads xk densely after
    the MAX all-reduce, so the subset is gathered once."""
    dev = _dev(x)
    x = _f32(x, "randk_gather_absmax")
    idx = _idx(idx, dev)
    k = idx.numel()
    if xk is None:
        xk = torch.empty(k, dtype=torch.float32, device=dev)
    if norm is None:
        norm = torch.empty(1, dtype=torch.float32, device=dev)
    st = _stream(dev)
    check(_lib.load().gc_randk_gather_absmax(_p(x), _p(idx), k, _p(xk), _p(norm), _p(_absmax_ws(dev, st)), st),
          "gc_randk_gather_absmax")
    return xk, norm


def randk_encode_w1(x, idx, bits, rng, xk=None, norm=None, out=None, lanes=None):
    """(words, norm) of the W = 1 GlobalRandK step: gather + max-norm + quantize
    + pack in one launch (the MAX over one rank is the identity); words equal
    qsgd_encode(x, max|x[idx]|, bits, rng, 1, idx=idx)."""
    dev = _dev(x)
    x = _f32(x, "randk_encode_w1")
    idx = _idx(idx, dev)
    k = idx.numel()
    lanes = lanes or qsgd_layout(k, bits, 1)
    if xk is None:
        xk = torch.empty(k, dtype=torch.float32, device=dev)
    if norm is None:
        norm = torch.empty(1, dtype=torch.float32, device=dev)
    if out is None:
        out = torch.empty(lanes.plane_words, dtype=torch.int32, device=dev)
    r = rng.struct()
    st = _stream(dev)
    check(_lib.load().gc_randk_encode_w1(_p(x), _p(idx), k, _p(xk), _p(norm), bits, C.byref(lanes), C.byref(r),
                                         _p(out), _p(_absmax_ws(dev, st)), st), "gc_randk_encode_w1")
    return out, norm


def randk_gather_absmax_segments(segs, idx, xk=None, norm=None):
    """randk_gather_absmax with x given as the per-parameter tensors of segs:
    each index is read from its tensor, so no flat bucket is built."""
    dev = segs.device
    idx = _idx(idx, dev)
    k = idx.numel()
    if xk is None:
        xk = torch.empty(k, dtype=torch.float32, device=dev)
    if norm is None:
        norm = torch.empty(1, dtype=torch.float32, device=dev)
    st = _stream(dev)
    check(_lib.load().gc_randk_gather_absmax_segments(C.byref(segs.struct), _p(idx), k, _p(xk), _p(norm),
                                                      _p(_absmax_ws(dev, st)), st),
          "gc_randk_gather_absmax_segments")
    return xk, norm


def randk_encode_w1_segments(segs, idx, bits, rng, xk=None, norm=None, out=None, lanes=None):
    """randk_encode_w1 reading the K indices from the tensors of segs."""
    dev = segs.device
    idx = _idx(idx, dev)
    k = idx.numel()
    lanes = lanes or qsgd_layout(k, bits, 1)
    if xk is None:
        xk = torch.empty(k, dtype=torch.float32, device=dev)
    if norm is None:
        norm = torch.empty(1, dtype=torch.float32, device=dev)
    if out is None:
        out = torch.empty(lanes.plane_words, dtype=torch.int32, device=dev)
    r = rng.struct()
    st = _stream(dev)
    check(_lib.load().gc_randk_encode_w1_segments(C.byref(segs.struct), _p(idx), k, _p(xk), _p(norm), bits,
                                                  C.byref(lanes), C.byref(r), _p(out), _p(_absmax_ws(dev, st)), st),
          "gc_randk_encode_w1_segments")
    return out, norm


def qsgd_decode_scatter_segments(words, idx, norm, bits, segs, world=1, alpha=1.0, lanes=None):
    """element idx[i] of the tensors of segs = RN(decode_i * alpha) + 0 (the
    GlobalRandK decode-scatter, reducer.py:754, with the setgrad's 1/W)."""
    dev = _dev(words)
    idx = _idx(idx, dev)
    k = idx.numel()
    lanes = lanes or qsgd_layout(k, bits, world)
    nt = norm_tensor(norm, dev)
    check(_lib.load().gc_qsgd_decode_scatter_segments(_p(words), _p(idx), k, _p(nt), bits, C.byref(lanes),
                                                      float(alpha), C.byref(segs.struct), _stream(dev)),
          "gc_qsgd_decode_scatter_segments")


class RandKStep:
    """A pre-resolved GlobalRandK encode / decode for a fixed bucket, K and lane
    layout (BASELINE config 4: K = 10,000 of a 14.7M bucket).  At this size the
    kernels take a few microseconds and an eager step is bound by the host work
    of each call (argument checks, layout and workspace lookups, ctypes struct
    building: 7-10 us per call, profiles/r01s_host_overhead.log); here every
    pointer and struct is built once and a call is one ctypes call.  Philox
    draws only (torch mode draws come from the host generator every call:
    use the codec functions).

        step = RandKStep(x, k, bits, generator, world)
        words, norm = step.encode(idx)          # W = 1: one launch
        xk, local = step.gather(idx)            # W > 1: gather + local norm,
        step.encode_gathered()                  #   MAX all-reduce, dense encode
        step.decode(words, idx, out, alpha)     # decode + scatter
    """

    def __init__(self, x, k: int, bits: int, generator, world: int = 1):
        dev = _dev(x)
        if generator.mode != "philox":
            raise _lib.GCodecError(_lib.GC_EINVAL, "RandKStep: Philox generators only")
        self.x = _f32(x, "RandKStep")
        self.k, self.bits, self.world, self.gen, self.device = int(k), int(bits), int(world), generator, dev
        self.lanes = qsgd_layout(self.k, self.bits, self.world)
        self.words = torch.empty(self.lanes.plane_words, dtype=torch.int32, device=dev)
        self.norm = torch.empty(1, dtype=torch.float32, device=dev)
        self.xk = torch.empty(self.k, dtype=torch.float32, device=dev)
        self.fused = randk_fused_ok(self.k, self.bits, self.world)
        self._rng = _lib.gc_rng(_lib.GC_RNG_PHILOX, 0, 0, 0, None)
        self._ws = {}
        lib = _lib.load()
        self._enc1, self._gather, self._enc, self._dec = (lib.gc_randk_encode_w1, lib.gc_randk_gather_absmax,
                                                          lib.gc_qsgd_encode, lib.gc_qsgd_decode)
        self._xp, self._xkp, self._np, self._wp = (self.x.data_ptr(), self.xk.data_ptr(), self.norm.data_ptr(),
                                                   self.words.data_ptr())
        self._lanes_ref = C.byref(self.lanes)
        self._rng_ref = C.byref(self._rng)
        self._idx = None
        self._idxp = None

    def _ws_for(self, st):
        ws = self._ws.get(st.value)
        if ws is None:
            ws = self._ws[st.value] = _absmax_ws(self.device, st).data_ptr()
        return ws

    def _set_idx(self, idx):
        if idx is not self._idx:
            if idx.numel() != self.k or idx.dtype != torch.int64 or idx.device != self.device or not idx.is_contiguous():
                raise _lib.GCodecError(_lib.GC_EINVAL, f"RandKStep: idx must be {self.k} contiguous int64 on "
                                       f"{self.device}")
            self._idx, self._idxp = idx, idx.data_ptr()

    def _draws(self):
        self._rng.seed = self.gen.reserve_key() & (2 ** 64 - 1)
        self._rng.offset = self.gen.offset
        self.gen.offset += self.k

    def encode(self, idx):
        """W = 1: gather + max-norm + encode in one launch -> (words, norm)."""
        if not self.fused:
            raise _lib.GCodecError(_lib.GC_EINVAL, "RandKStep.encode: the one-launch step needs W = 1 and "
                                   f"K <= {RANDK_FUSED_MAX}; use gather() + encode_gathered()")
        self._set_idx(idx)
        self._draws()
        st = _stream(self.device)
        check(self._enc1(self._xp, self._idxp, self.k, self._xkp, self._np, self.bits, self._lanes_ref,
                         self._rng_ref, self._wp, self._ws_for(st), st), "gc_randk_encode_w1")
        return self.words, self.norm

    def gather(self, idx):
        """xk = x[idx] and its local max-norm (before the MAX all-reduce)."""
        self._set_idx(idx)
        st = _stream(self.device)
        check(self._gather(self._xp, self._idxp, self.k, self._xkp, self._np, self._ws_for(st), st),
              "gc_randk_gather_absmax")
        return self.xk, self.norm

    def encode_gathered(self):
        """encode of the gathered subset with the (global) norm in self.norm."""
        self._draws()
        st = _stream(self.device)
        check(self._enc(self._xkp, None, self.k, self._np, self.bits, self._lanes_ref, self._rng_ref, self._wp, st),
              "gc_qsgd_encode")
        return self.words

    def decode(self, words, idx, out, alpha: float):
        """out[idx] = decode(words) * alpha (the scatter of reducer.py:754)."""
        self._set_idx(idx)
        check(self._dec(words.data_ptr(), self._idxp, self.k, self._np, self.bits, self._lanes_ref, float(alpha),
                        out.data_ptr(), _stream(self.device)), "gc_qsgd_decode")
        return out


# ---------------------------------------------------------------------------
# per-parameter tensors (reducer.py:46-68 TensorBuffer, 543-549 setgrad)
# ---------------------------------------------------------------------------
_dtype_of = operator.attrgetter("dtype")


class Segments:
    """gc_segments for a list of contiguous fp32 tensors on one device: the
    reference's TensorBuffer (reducer.py:46-68) as a device table, so flatten,
    max-norm, decode and setgrad address the tensors in place.  Built once per
    parameter list (one small H2D copy) and reused.  It holds NO reference to
    the tensors: a table is valid for any list whose key_of (data pointers and
    sizes: exactly what the table records) equals self.key, which callers
    check on every use — so a cached table never pins freed gradients in
    device memory.  dtype, device and contiguity are validated when a table is
    built (eligible_list); a list that reuses a table's pointers and sizes is
    taken to be the same fp32 tensors (in-place metadata changes of a gradient,
    e.g. t_() or set_() keeping the storage, are not supported)."""

    CHUNK_SHIFT = 12

    def __init__(self, tensors, chunk_shift: int = CHUNK_SHIFT):
        tensors = list(tensors)
        if not tensors:
            raise _lib.GCodecError(_lib.GC_EINVAL, "Segments: empty tensor list")
        dev = _dev(tensors[0])
        for t in tensors:
            if t.device != dev or t.dtype != torch.float32 or not t.is_contiguous():
                raise _lib.GCodecError(_lib.GC_EINVAL, "Segments: tensors must be contiguous float32 on "
                                       f"{dev} (got {t.dtype} on {t.device}, contiguous={t.is_contiguous()})")
        lib = _lib.load()
        count = len(tensors)
        sizes = np.array([t.numel() for t in tensors], dtype=np.uint64)
        ptrs = (C.c_void_p * count)(*[t.data_ptr() or None for t in tensors])
        n = int(sizes.sum())
        chunks = int(lib.gc_segments_chunks(n, chunk_shift))
        seg_host = np.zeros((count, 4), dtype=np.uint64)
        chunk_host = np.zeros(max(chunks, 1), dtype=np.uint32)
        n_out = C.c_uint64(0)
        check(lib.gc_segments_plan(sizes.ctypes.data_as(C.c_void_p), ptrs, count, chunk_shift,
                                   seg_host.ctypes.data_as(C.c_void_p), chunk_host.ctypes.data_as(C.c_void_p),
                                   chunks, C.byref(n_out)), "gc_segments_plan")
        self.device = dev
        self.n = n
        self.count = count
        self.key = Segments.key_of(tensors)
        self._seg = torch.from_numpy(seg_host.view(np.int64)).to(dev)
        self._chunk = torch.from_numpy(chunk_host.view(np.int32)).to(dev)
        self.sizes_hash = int(lib.gc_segments_sizes_hash(sizes.ctypes.data_as(C.c_void_p), count))
        self.struct = _lib.gc_segments(count, n, self._seg.data_ptr(), self._chunk.data_ptr(), chunk_shift,
                                       self.sizes_hash)

    @staticmethod
    def key_of(tensors):
        """(data pointers, sizes, element sizes, contiguity) of a tensor list:
        what the table records plus what makes it valid for the list.  A list
        at recycled addresses with the same sizes but another dtype (a model
        cast to fp16 / bf16) or a non-contiguous view of the same storage gets
        another key, so it never hits an fp32 table.  Device and
        the fp32 dtype itself are checked when a table is built
        (eligible_list); four attribute maps, no per-tensor Python loop."""
        return (tuple(map(torch.Tensor.data_ptr, tensors)), tuple(map(torch.Tensor.numel, tensors)),
                tuple(map(torch.Tensor.element_size, tensors)), tuple(map(torch.Tensor.is_contiguous, tensors)))

    @staticmethod
    def eligible_list(tensors) -> bool:
        """Contiguous fp32 tensors on one GPU (checked once per new table)."""
        return (all(map(torch.Tensor.is_contiguous, tensors)) and frozenset(map(_dtype_of, tensors)) == _F32_SET
                and len(devs := frozenset(map(torch.Tensor.get_device, tensors))) == 1 and min(devs) >= 0)


_F32_SET = frozenset((torch.float32,))


def segments_flatten_absmax(segs: Segments, flat: torch.Tensor | None = None, norm: torch.Tensor | None = None,
                            store: bool = True):
    """flat = cat(tensors) (if store) and norm = max |x| in one pass.  -> (flat | None, norm)"""
    dev = segs.device
    if store and flat is None:
        flat = torch.empty(segs.n, dtype=torch.float32, device=dev)
    if norm is None:
        norm = torch.empty(1, dtype=torch.float32, device=dev)
    st = _stream(dev)
    check(_lib.load().gc_segments_flatten_absmax(C.byref(segs.struct), _p(flat) if store else None, _p(norm),
                                                 _p(_absmax_ws(dev, st)), st), "gc_segments_flatten_absmax")
    return (flat if store else None), norm


def segments_scatter(flat: torch.Tensor, segs: Segments, alpha: float = 1.0):
    """tensor[s][:] = RN(flat[start:end] * alpha) — the reference's setgrad loop."""
    _dev(flat)
    flat = _f32(flat, "segments_scatter")
    check(_lib.load().gc_segments_scatter(_p(flat), float(alpha), C.byref(segs.struct), _stream(segs.device)),
          "gc_segments_scatter")


def segments_copy(src: Segments, dst: Segments, alpha: float = 1.0):
    """dst tensor element = RN(src tensor element * alpha) + 0 for two lists of
    the same tensor sizes (the GlobalRandK setgrad, reducer.py:759-761)."""
    if src.key[1] != dst.key[1] or src.device != dst.device:
        raise _lib.GCodecError(_lib.GC_EINVAL, "segments_copy: the two lists differ in tensor sizes or device")
    check(_lib.load().gc_segments_copy(C.byref(src.struct), C.byref(dst.struct), float(alpha), _stream(src.device)),
          "gc_segments_copy")


def qsgd_decode_segments(words, norm, bits, segs: Segments, world=1, alpha=1.0, lanes=None):
    """qsgd_decode straight into the tensors (decode + 1/W + setgrad)."""
    dev = _dev(words)
    lanes = lanes or qsgd_layout(segs.n, bits, world)
    nt = norm_tensor(norm, dev)
    check(_lib.load().gc_qsgd_decode_segments(_p(words), segs.n, _p(nt), bits, C.byref(lanes), float(alpha),
                                              C.byref(segs.struct), _stream(dev)), "gc_qsgd_decode_segments")


def ms_decode_scatter_segments(words, mask_words, idx, norm, levels, segs: Segments, world=1, order=0, alpha=1.0):
    """ms_decode(..., idx=idx) writing element idx[i] straight into its tensor,
    RN(decode_i * alpha) + 0 (the GlobalRandK two-scale setgrad)."""
    dev = _dev(words)
    idx = _idx(idx, dev)
    k = idx.numel()
    ql, ml = ms_layouts(k, levels, world)
    lv = levels_struct(levels)
    nt = norm_tensor(norm, dev)
    check(_lib.load().gc_ms_decode_scatter_segments(_p(words), _p(mask_words), _p(idx), k, _p(nt), C.byref(lv),
                                                    C.byref(ml), C.byref(ql), int(order), float(alpha),
                                                    C.byref(segs.struct), _stream(dev)),
          "gc_ms_decode_scatter_segments")


def ms_decode_segments(words, mask_words, norm, levels, segs: Segments, world=1, order=0, alpha=1.0):
    dev = _dev(words)
    ql, ml = ms_layouts(segs.n, levels, world)
    lv = levels_struct(levels)
    nt = norm_tensor(norm, dev)
    check(_lib.load().gc_ms_decode_segments(_p(words), _p(mask_words), segs.n, _p(nt), C.byref(lv), C.byref(ml),
                                            C.byref(ql), int(order), float(alpha), C.byref(segs.struct),
                                            _stream(dev)), "gc_ms_decode_segments")


# ---------------------------------------------------------------------------
# QSGD-MaxNorm unpacked (compressors.py compress/decompress semantics)
# ---------------------------------------------------------------------------
def qsgd_quantize(x, norm, bits, rng, level=0, dtype=torch.int8, le_bits=None):
    dev = _dev(x)
    x = _f32(x, "qsgd_quantize")
    nt = norm_tensor(norm, dev)
    q = torch.empty(x.numel(), dtype=dtype, device=dev)
    le = torch.empty(x.numel(), dtype=torch.int8, device=dev) if le_bits else None
    r = rng.struct()
    check(_lib.load().gc_qsgd_quantize_le(_p(x), x.numel(), _p(nt), bits, C.byref(r), level, _p(q),
                                          DTYPE_CODE[dtype], _p(le), int(le_bits or 0), _stream(dev)),
          "gc_qsgd_quantize")
    return (q, le) if le_bits else q


def qsgd_quantize_split(x, norm, bits, rng):
    """(xi, sign): int32 magnitudes and 1-iff-negative sign bits (the QSGDBP
    call site, compressors.py:344-353)."""
    dev = _dev(x)
    x = _f32(x, "qsgd_quantize_split")
    nt = norm_tensor(norm, dev)
    xi = torch.empty(x.numel(), dtype=torch.int32, device=dev)
    sg = torch.empty(x.numel(), dtype=torch.int32, device=dev)
    r = rng.struct()
    check(_lib.load().gc_qsgd_quantize_split(_p(x), x.numel(), _p(nt), bits, C.byref(r), _p(xi), _p(sg),
                                             _stream(dev)), "gc_qsgd_quantize_split")
    return xi, sg


def qsgd_dequantize(q, norm, bits, alpha=1.0, out=None):
    dev = _dev(q)
    q = q.contiguous().view(-1)
    if q.dtype not in (torch.int8, torch.int32):
        q = q.to(torch.int32)
    nt = norm_tensor(norm, dev)
    if out is None:
        out = torch.empty(q.numel(), dtype=torch.float32, device=dev)
    check(_lib.load().gc_qsgd_dequantize(_p(q), DTYPE_CODE[q.dtype], q.numel(), _p(nt), bits, float(alpha),
                                         _p(out), _stream(dev)), "gc_qsgd_dequantize")
    return out


def lane_pack(q, lanes, out=None):
    dev = _dev(q)
    q = q.contiguous().view(-1)
    if q.dtype not in (torch.int8, torch.int32):
        q = q.to(torch.int32)
    if out is None:
        out = torch.empty(lanes.plane_words, dtype=torch.int32, device=dev)
    check(_lib.load().gc_lane_pack(_p(q), DTYPE_CODE[q.dtype], C.byref(lanes), _p(out), _stream(dev)),
          "gc_lane_pack")
    return out


def lane_unpack(words, lanes, out=None):
    dev = _dev(words)
    if out is None:
        out = torch.empty(lanes.n, dtype=torch.int32, device=dev)
    check(_lib.load().gc_lane_unpack(_p(words), C.byref(lanes), _p(out), _stream(dev)), "gc_lane_unpack")
    return out


# ---------------------------------------------------------------------------
# multi-scale packed
# ---------------------------------------------------------------------------
def ms_cache_bytes(n: int, levels) -> int:
    """Bytes per element of the packed q cache for these levels (0: none)."""
    lv = levels_struct(levels)
    b = C.c_uint32(0)
    check(_lib.load().gc_ms_cache_bytes(n, C.byref(lv), C.byref(b)), "gc_ms_cache_bytes")
    return int(b.value)


def ms_mask_encode(x, norm, levels, rng, world=1, idx=None, out=None, cache=None):
    """Thermometer mask lanes; with `cache` (uint8, n * ms_cache_bytes) also the
    packed q cache that ms_select_encode(..., cache=cache) reads instead of x."""
    dev = _dev(x)
    x = _f32(x, "ms_mask_encode")
    idx = _idx(idx, dev)
    n = idx.numel() if idx is not None else x.numel()
    _, ml = ms_layouts(n, levels, world)
    lv = levels_struct(levels)
    nt = norm_tensor(norm, dev)
    if out is None:
        out = torch.empty(mask_words_total(ml, levels), dtype=torch.int32, device=dev)
    r = rng.struct()
    if cache is not None:
        if idx is not None:
            raise _lib.GCodecError(_lib.GC_EINVAL, "ms_mask_encode: the q cache needs a dense x (no idx)")
        check(_lib.load().gc_ms_mask_encode_cached(_p(x), n, _p(nt), C.byref(lv), C.byref(r), C.byref(ml), _p(out),
                                                   _p(cache), _stream(dev)), "gc_ms_mask_encode_cached")
        return out
    check(_lib.load().gc_ms_mask_encode(_p(x), _p(idx), n, _p(nt), C.byref(lv), C.byref(r), C.byref(ml), _p(out),
                                        _stream(dev)), "gc_ms_mask_encode")
    return out


MS_FUSED_MAX_R = 8  # ms_fast.h kMsFusedMaxR: q words per mask word of the coupled W = 1 layout


def ms_w1_ok(x, levels) -> bool:
    """Whether gc_ms_encode_w1 (the one-pass W = 1 multi-scale encode) takes
    this bucket — exactly the C entry point's preconditions: dense 16-byte
    aligned fp32 x, n < 2^32, 2 or 3 levels of <= 24 bits, and a q lane of at
    most 8 bits (r = 32 / lanes-per-word <= 8 q words per mask word: two levels
    with a lower level of <= 7 bits, three with <= 6).  Otherwise callers run
    the mask + select passes."""
    lv = sorted(int(b) for b in levels)
    if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and x.data_ptr() % 16 == 0
            and x.numel() < 2 ** 32 and len(lv) in (2, 3) and lv[-1] <= 24):
        return False
    ql, _ = ms_layouts(x.numel(), lv, 1)
    return 32 // ql.per_word <= MS_FUSED_MAX_R


def ms_encode_w1(x, norm, levels, rng, mask_out=None, out=None):
    """(mask_words, words) of the W = 1 multi-scale encode in ONE pass over x:
    the same streams as ms_mask_encode + ms_select_encode (the MIN over one rank
    is the identity).  See ms_w1_ok for the buckets it takes."""
    dev = _dev(x)
    x = _f32(x, "ms_encode_w1")
    n = x.numel()
    ql, ml = ms_layouts(n, levels, 1)
    lv = levels_struct(levels)
    nt = norm_tensor(norm, dev)
    if mask_out is None:
        mask_out = torch.empty(mask_words_total(ml, levels), dtype=torch.int32, device=dev)
    if out is None:
        out = torch.empty(ql.plane_words, dtype=torch.int32, device=dev)
    r = rng.struct()
    check(_lib.load().gc_ms_encode_w1(_p(x), n, _p(nt), C.byref(lv), C.byref(r), C.byref(ml), C.byref(ql),
                                      _p(mask_out), _p(out), _stream(dev)), "gc_ms_encode_w1")
    return mask_out, out


def ms_select_encode(x, norm, levels, rng, mask_words, world=1, idx=None, out=None, cache=None):
    """Packed q at the common levels of the W-summed mask; with `cache` (written
    by ms_mask_encode for this x, norm and rng) from the cache cells."""
    dev = _dev(x)
    x = _f32(x, "ms_select_encode")
    idx = _idx(idx, dev)
    n = idx.numel() if idx is not None else x.numel()
    ql, ml = ms_layouts(n, levels, world)
    lv = levels_struct(levels)
    if out is None:
        out = torch.empty(ql.plane_words, dtype=torch.int32, device=dev)
    if cache is not None:
        if idx is not None:
            raise _lib.GCodecError(_lib.GC_EINVAL, "ms_select_encode: the q cache needs a dense x (no idx)")
        check(_lib.load().gc_ms_select_cached(_p(cache), n, C.byref(lv), _p(mask_words), C.byref(ml), C.byref(ql),
                                              _p(out), _stream(dev)), "gc_ms_select_cached")
        return out
    nt = norm_tensor(norm, dev)
    r = rng.struct()
    check(_lib.load().gc_ms_select_encode(_p(x), _p(idx), n, _p(nt), C.byref(lv), C.byref(r), _p(mask_words),
                                          C.byref(ml), C.byref(ql), _p(out), _stream(dev)), "gc_ms_select_encode")
    return out


def ms_decode(words, mask_words, n, norm, levels, world=1, order=0, alpha=1.0, idx=None, out=None):
    dev = _dev(words)
    idx = _idx(idx, dev)
    ql, ml = ms_layouts(n, levels, world)
    lv = levels_struct(levels)
    nt = norm_tensor(norm, dev)
    if out is None:
        out = torch.empty(n, dtype=torch.float32, device=dev)
    check(_lib.load().gc_ms_decode(_p(words), _p(mask_words), _p(idx), n, _p(nt), C.byref(lv), C.byref(ml),
                                   C.byref(ql), int(order), float(alpha), _p(out), _stream(dev)), "gc_ms_decode")
    return out


def ms_mask_unpack(mask_words, n, levels, world=1):
    dev = _dev(mask_words)
    _, ml = ms_layouts(n, levels, world)
    out = torch.empty(n, dtype=torch.int8, device=dev)
    check(_lib.load().gc_ms_mask_unpack(_p(mask_words), C.byref(ml), len(levels), _p(out), _stream(dev)),
          "gc_ms_mask_unpack")
    return out


# ---------------------------------------------------------------------------
# multi-scale unpacked
# ---------------------------------------------------------------------------
def ms_quantize_mask(x, norm, levels, rng):
    dev = _dev(x)
    x = _f32(x, "ms_quantize_mask")
    lv = levels_struct(levels)
    nt = norm_tensor(norm, dev)
    mask = torch.empty(x.numel(), dtype=torch.int8, device=dev)
    r = rng.struct()
    check(_lib.load().gc_ms_quantize_mask(_p(x), x.numel(), _p(nt), C.byref(lv), C.byref(r), _p(mask),
                                          _stream(dev)), "gc_ms_quantize_mask")
    return mask


def ms_select_quantize(x, norm, levels, rng, mask, dtype=torch.int8):
    dev = _dev(x)
    x = _f32(x, "ms_select_quantize")
    lv = levels_struct(levels)
    nt = norm_tensor(norm, dev)
    mask = mask.to(torch.int8).contiguous().view(-1)
    q = torch.empty(x.numel(), dtype=dtype, device=dev)
    r = rng.struct()
    check(_lib.load().gc_ms_select_quantize(_p(x), x.numel(), _p(nt), C.byref(lv), C.byref(r), _p(mask), _p(q),
                                            DTYPE_CODE[dtype], _stream(dev)), "gc_ms_select_quantize")
    return q


def ms_dequantize(q, mask, norm, levels, order=0, alpha=1.0):
    dev = _dev(q)
    q = q.contiguous().view(-1)
    if q.dtype not in (torch.int8, torch.int32):
        q = q.to(torch.int32)
    mask = mask.to(torch.int8).contiguous().view(-1)
    lv = levels_struct(levels)
    nt = norm_tensor(norm, dev)
    out = torch.empty(q.numel(), dtype=torch.float32, device=dev)
    check(_lib.load().gc_ms_dequantize(_p(q), DTYPE_CODE[q.dtype], _p(mask), q.numel(), _p(nt), C.byref(lv),
                                       int(order), float(alpha), _p(out), _stream(dev)), "gc_ms_dequantize")
    return out


# ---------------------------------------------------------------------------
# torch-generator stream on the GPU
# ---------------------------------------------------------------------------
def mt19937_seed_state(seed: int) -> np.ndarray:
    st = np.empty(625, dtype=np.uint32)
    check(_lib.load().gc_mt19937_seed(seed, st.ctypes.data_as(C.c_void_p)), "gc_mt19937_seed")
    return st


_MT_TABLE = {}  # (device index, J) -> (int32 tensor [gens * 624], gens, ready event): jump coefficients of generators 1..gens
_MT_WS = {}     # (device index, stream) -> workspace tensor
MT_MAX_GENERATORS = 1024


def mt_generator_draws(count: int) -> int:
    """Draws per parallel generator J for `count` draws.  The jump costs about
    0.37 us of chip time per generator and a generator about 0.34 us per
    624-draw block (latency-bound: measured with 382 and 256 generators), so
    G = sqrt(count * 0.34 / (624 * 0.37)) generators balance the two kernels
    (DESIGN_HISTORY §7); J is a multiple of 624.  1e8 draws: G = 383, J = 261,456."""
    g = int(min(MT_MAX_GENERATORS, max(1, round((count * 1.47e-3) ** 0.5))))
    return 624 * max(1, -(-count // (624 * g)))


def _mt_jump_table(dev, gens: int, J: int = _lib.GC_MT_JUMP_DRAWS, stream=None):
    """Device jump table covering generators 1..gens for generators of J draws
    (host-computed once per process and J, grown geometrically; it depends
    only on J and the generator index, not on the seed) -> (table, gens).

    The table is (re)built on the caller's current stream (the upload is
    synchronous, the growth's torch.cat is a kernel); `stream` (default: the
    current stream) is made to wait for that build, so a table grown on one
    stream is never read unwritten by kernels on another."""
    key = (dev.index, J)
    cur = _MT_TABLE.get(key)
    have = cur[1] if cur is not None else 0
    if have < gens:
        total = max(gens, 2 * have, 16)
        host = np.empty((total - have) * 624, dtype=np.uint32)
        check(_lib.load().gc_mt19937_jump_table_j(J, have + 1, total - have, host.ctypes.data_as(C.c_void_p)),
              "gc_mt19937_jump_table")
        part = torch.from_numpy(host.view(np.int32)).to(dev)
        table = part if cur is None else torch.cat([cur[0], part])
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(dev))
        cur = _MT_TABLE[key] = (table, total, ready)
    (stream or torch.cuda.current_stream(dev)).wait_event(cur[2])
    return cur[0], cur[1]


def mt19937_generate(state_dev: torch.Tensor, count: int, out=None, parallel: bool = True,
                     J: int | None = None) -> torch.Tensor:
    """The next `count` draws of the MT19937 state on the device (625 words:
    state + read index), which advances.  parallel: the jumped multi-generator
    kernels (gc_mt19937_generate_jumped_j) with generators of J draws (default:
    mt_generator_draws(count)); else one workgroup walks the stream."""
    dev = _dev(state_dev)
    if out is None:
        out = torch.empty(count, dtype=torch.int32, device=dev)
    st = _stream(dev)
    lib = _lib.load()
    if not parallel:
        check(lib.gc_mt19937_generate(_p(state_dev), _p(out), count, st), "gc_mt19937_generate")
        return out
    if count == 0:
        return out
    J = J or mt_generator_draws(count)
    gens = -(-count // J)
    table, tgens = _mt_jump_table(dev, gens - 1, J) if gens > 1 else (None, 0)
    ws = _mt_ws(dev, st, count, J)
    check(lib.gc_mt19937_generate_jumped_j(_p(state_dev), _p(table), tgens, J, _p(out), count, _p(ws), st),
          "gc_mt19937_generate_jumped")
    return out


def _mt_ws(dev, st, count: int, J: int) -> torch.Tensor:
    need = int(_lib.load().gc_mt19937_workspace_size_j(count, J))
    key = (dev.index, st.value)
    ws = _MT_WS.get(key)
    if ws is None or ws.numel() < need:
        ws = _MT_WS[key] = torch.empty(need, dtype=torch.uint8, device=dev)
    return ws


_MT_PIN = {}  # device index -> {path: (pinned state in, pinned states out, device state)}: 625 int32 each


def _mt_bufs(device, path: str = "draws", stream=None):
    """Per device and path ("draws": mt19937_draws, two out slots for its
    speculative runs; "fused": the generator-quantize path): separate buffers,
    so a run still queued on one path never writes what the other reads.  The
    device state is allocated on `stream`, the stream that writes it (the
    caching allocator then never hands it a block whose last user is still
    queued on another stream)."""
    d = _MT_PIN.setdefault(device.index, {})
    b = d.get(path)
    if b is None:
        with torch.cuda.stream(stream or torch.cuda.current_stream(device)):
            b = d[path] = (torch.empty(625, dtype=torch.int32).pin_memory(),
                           [torch.empty(625, dtype=torch.int32).pin_memory() for _ in range(MT_MAX_SLOTS)],
                           torch.empty(625, dtype=torch.int32, device=device))
    return b


def _torch_state_to(device) -> torch.Tensor:
    """torch's CPU-generator state (624 words + read index) on `device`, copied
    asynchronously from a pinned buffer: the host does not wait for the work
    already queued on the stream (a pageable copy would)."""
    from .rng import torch_mt_state

    words, idx = torch_mt_state()
    hin, _, dst = _mt_bufs(device, "fused")
    h = hin.numpy().view(np.uint32)  # free: the previous call synchronised after its copy
    h[:624] = words
    h[624] = idx
    dst.copy_(hin, non_blocking=True)
    return dst


def _torch_state_back(state_dev: torch.Tensor):
    """Advance torch's CPU generator to the device state (synchronises: the
    draws' consumers may be queued behind the copy but the state must reach
    the host before torch's generator is used again)."""
    from .rng import set_torch_mt_state

    hout = _mt_bufs(state_dev.device, "fused")[1][0]
    hout.copy_(state_dev, non_blocking=True)
    torch.cuda.current_stream(state_dev.device).synchronize()
    new = hout.numpy().view(np.uint32)
    set_torch_mt_state(new[:624].copy(), int(new[624]))


def _quantize_mt(x, norm_t, bits, q, state_dev):
    dev = _dev(x)
    n = x.numel()
    st = _stream(dev)
    J = mt_generator_draws(max(n, 1))
    gens = -(-n // J) if n else 1
    table, tgens = _mt_jump_table(dev, gens - 1, J) if gens > 1 else (None, 0)
    check(_lib.load().gc_qsgd_quantize_mt19937(_p(x), n, _p(norm_t), bits, _p(state_dev), _p(table), tgens, J, _p(q),
                                               DTYPE_CODE[q.dtype], _p(_mt_ws(dev, st, n, J)), st),
          "gc_qsgd_quantize_mt19937")


def qsgd_quantize_torch(x, norm, bits, dtype=None, out=None) -> torch.Tensor:
    """compressors.py:299-316 under torch's CPU generator (torch mode): the
    MT19937 draws are generated on the GPU and consumed in the same kernel (no
    4n draw buffer); torch's generator state advances by x.numel() draws."""
    dev = _dev(x)
    x = _f32(x, "qsgd_quantize_torch")
    dtype = dtype or (torch.int8 if bits < 8 else torch.int32)
    q = out if out is not None else torch.empty(x.numel(), dtype=dtype, device=dev)
    state_dev = _torch_state_to(dev)
    _quantize_mt(x, norm_tensor(norm, dev), bits, q, state_dev)
    _torch_state_back(state_dev)
    return q


def qsgd_encode_torch(x, norm, bits, world=1, out=None, lanes=None) -> torch.Tensor:
    """Packed words of the torch-mode encode (the same words as qsgd_encode with
    a torch-mode reservation): the fused MT19937 quantize into int8 / int32 q,
    then the planar lane pack."""
    dev = _dev(x)
    x = _f32(x, "qsgd_encode_torch")
    n = x.numel()
    lanes = lanes or qsgd_layout(n, bits, world)
    q = torch.empty(n, dtype=torch.int8 if bits < 8 else torch.int32, device=dev)
    if out is None:
        out = torch.empty(lanes.plane_words, dtype=torch.int32, device=dev)
    state_dev = _torch_state_to(dev)
    _quantize_mt(x, norm_tensor(norm, dev), bits, q, state_dev)
    lane_pack(q, lanes, out)
    _torch_state_back(state_dev)
    return out


_MT_SIDE = {}  # device index -> (jump stream, [generator stream per slot]) the torch-mode draws are made on
_MT_LAST = {}  # device index -> (624 words, read index) last written back to torch
_MT_SPEC = {}  # device index -> the speculative runs of the next same-size calls (oldest first)
_MT_SLOT = {}  # device index -> runs enqueued so far (a run's slot = that count mod the slots in use)
_MT_END = {}   # (device index, end block B) -> device coefficients of x^(624 B - 1) mod P
_MT_WSS = {}   # (device index, slot) -> workspace of the runs in that slot
_MT_BUSY = {}  # (device index, slot) -> event after the last generators that read the slot's workspace
_MT_PREV = {}  # device index -> the count of the last mt19937_draws call
_MT_NSLOT = {}  # device index -> the slot rotation the queued runs were enqueued with
MT_SPECULATE = True  # generate the draws of the next same-size torch-mode calls ahead (mt19937_draws)
# how many calls ahead: each speculative run holds its calls' draws (mt_format_bytes each) + one
# generator workspace on the device until its call; runs start only after two calls in a row of the
# same count, and never above MT_SPECULATE_MAX_DRAWS
MT_SPECULATE_DEPTH = 16  # calls' draws kept enqueued ahead of the current one (at most)
MT_SPECULATE_MAX_DRAWS = 1 << 30  # per run (a run of MT_MULTI_CALLS calls holds that many times count)
# device bytes the draws of the runs in flight (the current run's and those queued ahead) may hold
# (bounded, visible through mt_reserved_bytes): the calls per run and the depth shrink to
# fit it (_mt_plan); None = min(MT_SPECULATE_DEFAULT_BYTES, two runs of MT_MULTI_CALLS calls).
# Measured at 1e8 per call: 1 GiB leaves one call ahead and doubles the call
# time; 4 GiB costs ~5 % against an unbounded queue
MT_SPECULATE_BUDGET = None
MT_SPECULATE_DEFAULT_BYTES = 4 << 30
MT_MAX_SLOTS = 8  # workspace / pinned-state slots of the runs in flight
# calls per run once a count repeats: one set of generators (and of generator
# jumps, the LDS-bound part) makes the draws of this many consecutive calls,
# each call taking its slice and its own end state (gc_mt19937_generate_multi_j)
MT_MULTI_CALLS = 8
# generators per pipelined run (mt19937_draws): None = mt_pipe_generators(count).  With the runs
# made calls ahead, a generator's latency no longer bounds the call; fewer generators cut the
# jump work, which shares the chip with the encodes (DESIGN_HISTORY section 7)
MT_PIPE_GENERATORS = None
MT_WAIT_NEXT_JUMPS = False  # consumers also wait for the speculative run's jumps (mt19937_draws)
# side-stream priorities ("high" or "normal") of the jumps and of the generators
MT_SIDE_PRIORITY = ("high", "high")


def mt_pipe_generators(count: int, multi: bool = False) -> int:
    """Generators of one pipelined torch-mode run of `count` draws.  A
    single-call run: about one per 781k draws (128 for 1e8 draws; swept at
    1e8 per call, profiles/r05i_torch_mode_sweep.log: 0.291 ms per encode back
    to back against 0.314 ms at 256 and 0.349 ms at 64).  A multi-call run
    (MT_MULTI_CALLS calls, gc_mt19937_generate_multi_j): one per 1.56M draws
    (512 for 8 calls of 1e8; profiles/r05j/r05k/r05m_torch_mode_*.log: 512 and
    1024 within noise, 16 calls per run over the speculation budget)."""
    if MT_PIPE_GENERATORS:
        return int(MT_PIPE_GENERATORS)
    return max(1, min(MT_MAX_GENERATORS, -(-count // (1_562_500 if multi else 781_250))))


def mt_pipe_generator_draws(count: int, multi: bool = False) -> int:
    """Draws per generator J (a multiple of 624) of a pipelined run."""
    g = mt_pipe_generators(count, multi)
    return 624 * max(1, -(-count // (624 * g)))


def _mt_side(device):
    """High-priority streams: one for the jumps (LDS-bound; they also produce
    the end state, so run c+1's jumps follow run c's) and one per slot for the
    generators (latency-bound), so the generators of the runs in flight run
    side by side instead of one after another.  The encodes the draws feed
    fill the CUs they leave idle."""
    s = _MT_SIDE.get(device.index)
    if s is None:
        lo, hi = torch.cuda.Stream.priority_range()
        pj, pg = (min(lo, hi) if p == "high" else max(lo, hi) for p in MT_SIDE_PRIORITY)
        s = _MT_SIDE[device.index] = (torch.cuda.Stream(device, priority=pj),
                                      [torch.cuda.Stream(device, priority=pg) for _ in range(MT_MAX_SLOTS)])
    return s


def _mt_upload_side(dev, host: np.ndarray) -> torch.Tensor:
    """host (uint32) on the device, copied on the jump stream: every reader
    of the end coefficients runs on that stream or after its phase-1 event.
    A pinned, non-blocking copy: a pageable .to(dev) on the caller's stream
    blocked the host until that stream drained (the GEMMs of a backward), and
    the call's encode then started only after the host caught up
    (profiles/r06t_host_torch_mode.log: 2.7-3.8 ms host stalls at the calls
    that enqueue a speculative run with new end blocks)."""
    js = _mt_side(dev)[0]
    src = torch.from_numpy(np.ascontiguousarray(host).view(np.int32)).pin_memory()
    with torch.cuda.stream(js):
        t = torch.empty(src.shape, dtype=torch.int32, device=dev)
        t.copy_(src, non_blocking=True)
    return t


def _mt_end_coef(dev, block: int):
    """Coefficients of the jump to raw block `block` (x^(624 block - 1) mod P)
    on the device (uploaded on the jump stream), cached: a bucket size takes
    at most two end blocks."""
    if block == 0:
        return None
    key = (dev.index, block)
    t = _MT_END.get(key)
    if t is None:
        host = np.empty(624, dtype=np.uint32)
        check(_lib.load().gc_mt19937_jump_table_j(624 * block, 1, 1, host.ctypes.data_as(C.c_void_p)),
              "gc_mt19937_jump_table_j")
        if len(_MT_END) >= 64:
            _MT_END.clear()
        t = _MT_END[key] = _mt_upload_side(dev, host)
    return t


def _mt_ws_slot(dev, slot: int, count: int, J: int, js) -> torch.Tensor:
    """The workspace of a slot's runs, allocated on the jump stream js that
    writes it (its generators on the other side stream read it after js's
    phase-1 event, and record_stream keeps it alive for them)."""
    need = int(_lib.load().gc_mt19937_workspace_size_j(count, J))
    key = (dev.index, slot)
    ws = _MT_WSS.get(key)
    if ws is None or ws.numel() < need:
        busy = _MT_BUSY.get(key)
        if busy is not None:
            busy.synchronize()  # the old buffer may still be read by queued generators
        _MT_WSS.pop(key, None)
        with torch.cuda.stream(js):
            ws = _MT_WSS[key] = torch.empty(need, dtype=torch.uint8, device=dev)
        ws.record_stream(_mt_side(dev)[1][slot])
    return ws


class _MtRun:
    """One enqueued generation of `calls` calls' draws: its draws, the read
    index after it, the pinned slot its end states go to, the next call's
    slice (k), and events after its jumps (p1), after the end states' copy to
    the host (state_ready) and after its generators (done)."""

    __slots__ = ("count", "packed", "out", "slot", "idx_end", "p1", "state_ready", "done", "calls", "k", "ends")


def _mt_enqueue(dev, st_dev, count: int, idx: int, hout, slot: int, fmt: str = "plain") -> _MtRun:
    """Phase 1 on the jump stream: sequence + jumps + the end state (written
    over st_dev, gc_mt19937_generate_split_j) and its copy into hout[slot];
    phase 2 on the generator stream, after phase 1: the draws (packed: their
    low 24 bits, 3 bytes each, gc_mt19937_generate_split24_j)."""
    packed = fmt == "packed24"
    J = mt_pipe_generator_draws(count)
    gens = -(-count // J)
    js, gss = _mt_side(dev)
    gs = gss[slot]
    table, tgens = _mt_jump_table(dev, gens - 1, J, stream=js) if gens > 1 else (None, 0)
    block = (idx + count - 1) // 624
    end = _mt_end_coef(dev, block)
    ws = _mt_ws_slot(dev, slot, count, J, js)
    busy = _MT_BUSY.get((dev.index, slot))
    lib = _lib.load()
    run = _MtRun()
    run.count, run.packed, run.slot, run.idx_end = count, "packed24" if packed else "plain", slot, \
        idx + count - 624 * block
    run.calls, run.k, run.ends = 1, 0, None
    with torch.cuda.stream(js):
        if busy is not None:
            js.wait_event(busy)  # that slot's previous generators have read the workspace
        check(lib.gc_mt19937_generate_split_j(_p(st_dev), _p(table), tgens, J, _p(end), block, None, count, _p(ws),
                                              1, _stream(dev)), "gc_mt19937_generate_split_j")
        run.p1 = torch.cuda.Event()
        run.p1.record()
        hout[slot].copy_(st_dev, non_blocking=True)
        run.state_ready = torch.cuda.Event()
        run.state_ready.record()
    # the jump table and the end coefficients live on the caller's stream and
    # may be replaced (table growth, cache eviction) while these runs are queued
    for t in (table, end):
        if t is not None:
            t.record_stream(js)
            t.record_stream(gs)
    with torch.cuda.stream(gs):
        gs.wait_event(run.p1)
        if packed:
            run.out = torch.empty(count // 4 * 3, dtype=torch.int32, device=dev)
            check(lib.gc_mt19937_generate_split24_j(_p(st_dev), _p(table), tgens, J, _p(end), block, _p(run.out),
                                                    count, idx, _p(ws), 2, _stream(dev)),
                  "gc_mt19937_generate_split24_j")
        else:
            run.out = torch.empty(count, dtype=torch.int32, device=dev)
            check(lib.gc_mt19937_generate_split_j(_p(st_dev), _p(table), tgens, J, _p(end), block, _p(run.out),
                                                  count, _p(ws), 2, _stream(dev)), "gc_mt19937_generate_split_j")
        run.done = torch.cuda.Event()
        run.done.record()
    _MT_BUSY[(dev.index, slot)] = run.done
    return run


_MT_ENDS = {}   # (device index, slot) -> pinned (MT_MULTI_MAX, 626) int32 end states of that slot's run
_MT_ENDCAT = {}  # (device index, end blocks) -> device (len, 624) coefficient tables of a multi-call run
MT_MULTI_MAX = 64


_MT_END_HOST = {}  # end block -> host coefficients of x^(624 block - 1) mod P (624 uint32)


def _mt_end_coefs(dev, blocks: tuple) -> torch.Tensor:
    """The end coefficient tables of a multi-call run, one per end block,
    contiguous on the device (cached: a bucket size takes a few tuples).
    Built on the host and uploaded on the jump stream (_mt_upload_side), so
    the side streams never wait for the caller's stream (a device-side stack
    would run on the caller's stream: the table growth test holds that stream
    busy)."""
    key = (dev.index, blocks)
    t = _MT_ENDCAT.get(key)
    if t is None:
        if len(_MT_ENDCAT) >= 256:
            _MT_ENDCAT.clear()
        host = np.empty((len(blocks), 624), dtype=np.uint32)
        for i, b in enumerate(blocks):
            h = _MT_END_HOST.get(b)
            if h is None:
                if len(_MT_END_HOST) >= 4096:
                    _MT_END_HOST.clear()
                h = _MT_END_HOST[b] = np.empty(624, dtype=np.uint32)
                check(_lib.load().gc_mt19937_jump_table_j(624 * b, 1, 1, h.ctypes.data_as(C.c_void_p)),
                      "gc_mt19937_jump_table_j")
            host[i] = h
        t = _MT_ENDCAT[key] = _mt_upload_side(dev, host)
    return t


_MT_WARNED = set()  # (count, format) the budget turned speculation off for (warned once)


def _mt_plan(count: int, fmt: str, multi: bool):
    """(calls per run, calls kept ahead) for repeated calls of `count` draws in
    format fmt under the speculation budget: the draws of the current run and
    of the runs ahead, mt_format_bytes(count, fmt) per call, fit in
    MT_SPECULATE_BUDGET bytes (default: the smaller of
    MT_SPECULATE_DEFAULT_BYTES and two runs of MT_MULTI_CALLS calls).  A run takes at most half of what fits, the rest is
    depth (at most MT_SPECULATE_DEPTH).  When not even one call fits ahead the
    speculation is off for this count (warned once: the calls then wait for
    their draws)."""
    calls_max = max(1, min(int(MT_MULTI_CALLS), MT_MULTI_MAX)) if multi else 1
    bpc = max(1, mt_format_bytes(count, fmt))
    budget = MT_SPECULATE_BUDGET
    if budget is None:
        budget = min(int(MT_SPECULATE_DEFAULT_BYTES), 2 * calls_max * bpc)
    hold = int(budget) // bpc
    calls = max(1, min(calls_max, hold // 2))
    depth = max(0, min(int(MT_SPECULATE_DEPTH), hold - calls))
    if depth == 0 and MT_SPECULATE and int(MT_SPECULATE_DEPTH) > 0 and (count, fmt) not in _MT_WARNED:
        import warnings
        _MT_WARNED.add((count, fmt))
        warnings.warn(f"gcodec torch mode: {count} draws per call ({bpc} bytes as {fmt}) leave no room ahead in "
                      f"the speculation budget of {int(budget)} bytes (codec.MT_SPECULATE_BUDGET): each call "
                      "waits for its own draws", RuntimeWarning, stacklevel=3)
    return calls, depth


def mt_format_bytes(count: int, fmt: str) -> int:
    """Device bytes of one call's `count` draws in format fmt ("plain": 4 per
    draw, "packed24": 3, "split8" / "split16": the two planes of
    gc_rng_split_bytes, 16-byte padded)."""
    if fmt == "plain":
        return 4 * count
    if fmt == "packed24":
        return 3 * count
    return int(_lib.load().gc_rng_split_bytes(count, _SPLIT_BITS[fmt]))


_SPLIT_BITS = {"split8": 8, "split16": 16}
_FMT_KIND = {"plain": _lib.GC_RNG_STREAM, "packed24": _lib.GC_RNG_STREAM24, "split8": _lib.GC_RNG_SPLIT8,
             "split16": _lib.GC_RNG_SPLIT16}


def _mt_enqueue_multi(dev, st_dev, count: int, calls: int, idx: int, slot: int, fmt: str = "plain") -> _MtRun:
    """Like _mt_enqueue for `calls` consecutive calls of `count` draws: one
    generation of calls * count draws, the end state after each call's slice
    (gc_mt19937_generate_multi_j; "packed24": the 24-bit draws of
    gc_mt19937_generate_multi24_j; "split8" / "split16": the split-plane
    regions of gc_mt19937_generate_multi_split_j, one per call; both need
    count and idx multiples of 4).  count >= 624."""
    packed = fmt == "packed24"
    total = count * calls
    J = mt_pipe_generator_draws(total, True)
    gens = -(-total // J)
    js, gss = _mt_side(dev)
    gs = gss[slot]
    table, tgens = _mt_jump_table(dev, gens - 1, J, stream=js) if gens > 1 else (None, 0)
    blocks = tuple((idx + (k + 1) * count - 1) // 624 for k in range(calls))
    ends = _mt_end_coefs(dev, blocks)
    lib = _lib.load()
    need = int(lib.gc_mt19937_workspace_size_multi_j(total, J, calls))
    key = (dev.index, slot)
    ws = _MT_WSS.get(key)
    busy = _MT_BUSY.get(key)
    if ws is None or ws.numel() < need:
        if busy is not None:
            busy.synchronize()  # the old buffer may still be read by queued generators
        _MT_WSS.pop(key, None)
        with torch.cuda.stream(js):
            ws = _MT_WSS[key] = torch.empty(need, dtype=torch.uint8, device=dev)
        ws.record_stream(gs)
    pin = _MT_ENDS.get(key)
    if pin is None:
        pin = _MT_ENDS[key] = torch.empty((MT_MULTI_MAX, 626), dtype=torch.int32).pin_memory()
    dev_ends = _MT_ENDS.get(("dev",) + key)
    if dev_ends is None:
        with torch.cuda.stream(js):
            dev_ends = _MT_ENDS[("dev",) + key] = torch.empty((MT_MULTI_MAX, 626), dtype=torch.int32, device=dev)
    run = _MtRun()
    run.count, run.packed, run.slot, run.calls, run.k = count, fmt, slot, calls, 0
    run.idx_end = idx + total - 624 * blocks[-1]

    def gen(out, phase):
        if fmt in _SPLIT_BITS:
            check(lib.gc_mt19937_generate_multi_split_j(_p(st_dev), _p(table), tgens, J, _p(ends), calls, count, idx,
                                                        _SPLIT_BITS[fmt], _p(dev_ends), out, 0, 0, 0,
                                                        0xFFFFFFFFFFFFFFFF, _p(ws), phase, _stream(dev)),
                  "gc_mt19937_generate_multi_split_j")
        elif packed:
            check(lib.gc_mt19937_generate_multi24_j(_p(st_dev), _p(table), tgens, J, _p(ends), calls, count, idx,
                                                    _p(dev_ends), out, _p(ws), phase, _stream(dev)),
                  "gc_mt19937_generate_multi24_j")
        else:
            check(lib.gc_mt19937_generate_multi_j(_p(st_dev), _p(table), tgens, J, _p(ends), calls, count,
                                                  _p(dev_ends), out, _p(ws), phase, _stream(dev)),
                  "gc_mt19937_generate_multi_j")

    with torch.cuda.stream(js):
        if busy is not None:
            js.wait_event(busy)  # that slot's previous generators have read the workspace
        gen(None, 1)
        run.p1 = torch.cuda.Event()
        run.p1.record()
        pin[:calls].copy_(dev_ends[:calls], non_blocking=True)
        run.state_ready = torch.cuda.Event()
        run.state_ready.record()
    run.ends = pin
    for t in (table, ends):
        if t is not None:
            t.record_stream(js)
            t.record_stream(gs)
    with torch.cuda.stream(gs):
        gs.wait_event(run.p1)
        if fmt in _SPLIT_BITS:
            run.out = torch.empty(calls * mt_format_bytes(count, fmt), dtype=torch.uint8, device=dev)
        else:
            run.out = torch.empty(total // 4 * 3 if packed else total, dtype=torch.int32, device=dev)
        gen(_p(run.out), 2)
        run.done = torch.cuda.Event()
        run.done.record()
    _MT_BUSY[key] = run.done
    return run


def mt19937_packable(count: int, idx: int) -> bool:
    """Whether a run of `count` draws from read index `idx` can be packed to
    24 bits (whole quads of draws: count and idx multiples of 4)."""
    return count > 0 and count % 4 == 0 and idx % 4 == 0


def mt19937_draws(count: int, device, packed24: bool = False) -> torch.Tensor:
    """`count` draws of torch's CPU generator on `device` (see mt19937_reserve):
    the plain 32-bit draws, or with packed24 where mt19937_packable their low
    24 bits, 3 bytes each (GC_RNG_STREAM24; the caller tells the two apart by
    numel)."""
    return mt19937_reserve(count, device, "packed24" if packed24 else "plain")[0]


def mt19937_reserve(count: int, device, fmt: str = "plain"):
    """`count` draws of torch's CPU generator, produced on `device`; torch's
    generator state advances exactly as torch.bernoulli would advance it
    (synchronously: the new state is in torch's generator when this returns).
    Returns (draws tensor, gc_rng kind).

    fmt: "plain" = the 32-bit draws (int32, GC_RNG_STREAM).  Where
    mt19937_packable (count and torch's read index multiples of 4) the draws
    can be cut to the 24 bits torch's rounding reads (compressors.py:301 via
    torch.rand), so the encode is bit-identical and moves fewer draw bytes:
    "packed24" = 3 bytes per draw (GC_RNG_STREAM24).  For count >= 624 (any
    read index) "split8" / "split16" = one HI plane of the top 8 / 16 of those
    bits and one LO plane of the rest (uint8 region of mt_format_bytes bytes,
    GC_RNG_SPLIT8 / SPLIT16): the encode reads the LO plane only where the HI
    bits tie (about 1 draw in 2^8 / 2^16).  A request the run cannot honour
    gets plain draws.

    The draws are generated on two high-priority side streams
    (gc_mt19937_generate_split_j): phase 1 (jump stream) = the state's
    sequence, the LDS-bound jumps and one more jump straight to the END state;
    phase 2 (generator stream) = the latency-bound generators.  The host waits
    only for the end state (phase 1 and a 2.5 KB copy), never for the draws or
    the caller's queued work; the caller's stream waits for the draws.  With
    MT_SPECULATE the runs of the next MT_SPECULATE_DEPTH same-size calls are
    kept enqueued behind this one (each from the previous run's end state), so
    a call's draws are made while the calls before it encode; a speculative
    run is used only if torch's generator is exactly where the previous call
    left it and the count matches, else every queued run is dropped and the
    state is sent to the device again."""
    from .rng import set_torch_mt_state, torch_mt_state

    device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    d = device.index
    words, idx = torch_mt_state()
    js, _ = _mt_side(device)
    hin, hout, dst = _mt_bufs(device, "draws", stream=js)
    cur = torch.cuda.current_stream(device)
    repeat = _MT_PREV.get(d) == count
    _MT_PREV[d] = count
    last = _MT_LAST.get(d)
    untouched = last is not None and last[1] == idx and np.array_equal(last[0], words)

    multi = count >= 624  # multi-call runs (gc_mt19937_generate_multi_j / _multi24_j / _multi_split_j)
    if fmt not in _FMT_KIND:
        raise ValueError(f"mt19937_reserve: unknown draw format {fmt!r}")
    if fmt == "packed24" and not (count > 0 and mt19937_packable(count, int(idx))):
        fmt = "plain"
    if fmt in _SPLIT_BITS and not multi:  # the split planes come from multi-call runs (count >= 624)
        fmt = "plain"
    calls, depth = _mt_plan(count, fmt, multi) if count > 0 else (1, 0)
    # slots in rotation: the runs in flight (the current one, those holding the
    # next `depth` calls: ceil(depth / calls) runs, one more while the current
    # run still has calls left) + one; a change of the rotation drops the queue
    # (its runs' slots were counted for the old rotation).  Each
    # run's state / ends slot must outlive the enqueue of the runs behind it:
    # the state is read after them
    nslot = min(MT_MAX_SLOTS, -(-depth // calls) + 3)
    queue = _MT_SPEC.pop(d, [])
    dropped = False  # queued runs dropped here: they moved dst past torch's state
    if _MT_NSLOT.get(d) != nslot:
        for r in queue:
            r.done.synchronize()
        dropped = bool(queue)
        queue = []
        _MT_NSLOT[d] = nslot

    def next_slot():
        k = _MT_SLOT.get(d, 0)
        _MT_SLOT[d] = k + 1
        return k % nslot

    if count == 0:
        if queue or dropped:  # dropped runs still moved dst on: send the state next time
            _MT_LAST.pop(d, None)
        return torch.empty(0, dtype=torch.int32, device=device), _lib.GC_RNG_STREAM

    def enqueue(st_idx, ncalls):
        f = fmt if fmt != "packed24" or mt19937_packable(count, st_idx) else "plain"
        if multi:
            return _mt_enqueue_multi(device, dst, count, ncalls, st_idx, next_slot(), f)
        return _mt_enqueue(device, dst, count, st_idx, hout, next_slot(), f)

    if queue and untouched and queue[0].count == count and queue[0].packed == fmt:
        run = queue[0]
        _MT_STATS["queued"] += 1
    else:
        _MT_STATS["fresh"] += 1
        _MT_STATS["fresh_" + ("dropped" if dropped else "touched" if not untouched and last is not None else
                              "mismatch" if queue else "empty" if last is not None else "first")] += 1
        if queue or dropped or not untouched:  # dst is not torch's state: send it
            with torch.cuda.stream(js):
                h = hin.numpy().view(np.uint32)  # free: earlier copies from it were waited for
                h[:624] = words
                h[624] = idx
                dst.copy_(hin, non_blocking=True)
        queue = [enqueue(int(idx), 1)]
        run = queue[0]
    k = run.k if run.calls > 1 or multi else 0
    run.k = k + 1
    if run.k >= run.calls:
        queue.pop(0)
    if MT_SPECULATE and repeat and depth > 0 and count * calls <= MT_SPECULATE_MAX_DRAWS:
        ahead = sum(r.calls - r.k for r in queue)
        behind = sum(1 for r in queue if r is not run)  # runs enqueued after this one
        # calls' draws enqueued behind this one, chained from the last run's end;
        # never a full rotation behind it (this run's state slot is read below)
        while ahead < depth and behind < nslot - 1:
            tail_idx = queue[-1].idx_end if queue else run.idx_end
            queue.append(enqueue(tail_idx, calls))
            _MT_STATS["speculative_runs"] += 1
            ahead += queue[-1].calls
            behind += 1
    elif run.k >= run.calls:
        queue = []  # (none were kept: a queue exists only after a repeat)
    cur.wait_event(run.done)
    if queue and MT_WAIT_NEXT_JUMPS:
        cur.wait_event(queue[0].p1)
    per = {"plain": count, "packed24": count // 4 * 3}.get(run.packed) or mt_format_bytes(count, run.packed)
    out = run.out[k * per:(k + 1) * per] if run.calls > 1 else run.out
    run.out.record_stream(cur)
    if queue:
        _MT_SPEC[d] = queue
    run.state_ready.synchronize()
    if multi:
        new = run.ends[k].numpy().view(np.uint32)
    else:
        new = hout[run.slot].numpy().view(np.uint32)
    w2, i2 = new[:624].copy(), int(new[624])
    set_torch_mt_state(w2, i2)
    _MT_LAST[d] = (w2, i2)
    return out, _FMT_KIND[run.packed]


_MT_STATS = collections.Counter()


def mt_stats(reset: bool = False) -> dict:
    """Counters of mt19937_reserve since the last reset: calls served from
    the speculative queue ("queued") or from a run made on demand ("fresh",
    split by why: "fresh_first" / "fresh_empty" (no run queued) /
    "fresh_touched" (torch's generator moved since the last call) /
    "fresh_mismatch" (a queued run of another count or format) /
    "fresh_dropped" (the slot rotation changed)), and the speculative runs
    enqueued."""
    out = dict(_MT_STATS)
    if reset:
        _MT_STATS.clear()
    return out


def mt_reserved_bytes(device=None) -> int:
    """Device bytes the torch-mode machinery holds on `device` (all devices if
    None) between calls, invisible to the caller: the queued speculative runs'
    draws, the generator workspaces, the jump and end-coefficient tables and
    the per-slot end-state buffers.  mt_release() frees them."""
    if device is not None:
        device = torch.device(device)
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
    want = (lambda d: True) if device is None else (lambda d: d == device.index)

    def nb(t):
        return t.numel() * t.element_size()

    total = 0
    for d, runs in _MT_SPEC.items():
        if want(d):
            total += sum(nb(r.out) for r in runs if getattr(r, "out", None) is not None)
    total += sum(nb(t) for k, t in _MT_WSS.items() if want(k[0]))
    total += sum(nb(v[0]) for k, v in _MT_TABLE.items() if want(k[0]))
    total += sum(nb(t) for k, t in _MT_ENDCAT.items() if want(k[0]))
    total += sum(nb(t) for k, t in _MT_END.items() if want(k[0]))
    total += sum(nb(t) for k, t in _MT_ENDS.items() if k[0] == "dev" and want(k[1]))
    return int(total)


def mt_release(device=None):
    """Drop the torch-mode state kept between calls on `device` (all devices
    if None): the speculative runs (4 * count bytes of draws each), the
    generator workspaces and the device state buffers.  Called when a
    generator leaves torch mode; the next torch-mode call starts from torch's
    state again."""
    if device is not None:
        device = torch.device(device)
        if device.index is None:  # 'cuda' means the current device (was a silent no-op)
            device = torch.device("cuda", torch.cuda.current_device())
    keys = [device.index] if device is not None else sorted({k for k in _MT_SPEC} | {k[0] for k in _MT_WSS}
                                                               | set(_MT_PIN) | set(_MT_LAST))
    for d in keys:
        for k in [k for k in _MT_BUSY if k[0] == d]:
            _MT_BUSY.pop(k).synchronize()  # queued generators may still read the workspaces
        for run in _MT_SPEC.pop(d, []):
            run.done.synchronize()
        for k in [k for k in _MT_WSS if k[0] == d]:
            del _MT_WSS[k]
        _MT_PIN.pop(d, None)
        _MT_LAST.pop(d, None)
        _MT_PREV.pop(d, None)
        _MT_NSLOT.pop(d, None)
        for k in [k for k in _MT_ENDS if k[-2] == d]:
            del _MT_ENDS[k]


# ---------------------------------------------------------------------------
# reference-compatible packers
# ---------------------------------------------------------------------------
def bytepack8(src: torch.Tensor) -> torch.Tensor:
    dev = _dev(src)
    src = src.contiguous().view(-1)
    if src.dtype not in DTYPE_CODE:
        src = src.to(torch.int64)
    out = torch.empty((src.numel() + 7) // 8, dtype=torch.int64, device=dev)
    check(_lib.load().gc_bytepack8(_p(src), DTYPE_CODE[src.dtype], src.numel(), _p(out), _stream(dev)),
          "gc_bytepack8")
    return out


def byteunpack8(words: torch.Tensor) -> torch.Tensor:
    dev = _dev(words)
    words = words.contiguous().view(-1).to(torch.int64)
    out = torch.empty(8 * words.numel(), dtype=torch.int8, device=dev)
    check(_lib.load().gc_byteunpack8(_p(words), words.numel(), _p(out), _stream(dev)), "gc_byteunpack8")
    return out


def qsgdbp_decode(sign: torch.Tensor, xi: torch.Tensor, c: torch.Tensor, n: int) -> torch.Tensor:
    """QSGDBPCompressor.decompress's combine (compressors.py:375-376) in one
    kernel: (c * (+-1)) * float(xi) over the first n unpacked values."""
    dev = _dev(xi)
    sign = sign.contiguous().view(-1).to(torch.int32)
    xi = xi.contiguous().view(-1).to(torch.int32)
    if sign.numel() < n or xi.numel() < n:
        raise _lib.GCodecError(_lib.GC_EINVAL, "qsgdbp_decode: fewer unpacked values than n")
    ct = c.reshape(1).to(device=dev, dtype=torch.float32)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    check(_lib.load().gc_qsgdbp_decode(_p(sign), _p(xi), n, _p(ct), _p(out), _stream(dev)), "gc_qsgdbp_decode")
    return out


def _g4_result(res: torch.Tensor, what: str) -> int:
    """(count, status) written by the device packer: one 16-byte D2H read."""
    count, status = (int(v) for v in res.cpu().tolist())
    return _g4_check(count, status, what)


def _g4_check(count: int, status: int, what: str) -> int:
    if status & 1:
        raise _lib.GCodecError(_lib.GC_ERANGE, f"{what}: a value outside [0, 255] (the greedy format's domain)")
    if status & 2:
        raise _lib.GCodecError(_lib.GC_ENOSPC, f"{what}: output capacity too small")
    if status & 4:
        raise _lib.GCodecError(_lib.GC_EHIP, f"{what}: a block of the persistent pack waited too long "
                                             "(the workspace must be zeroed again before its next use)")
    return count


class Greedy4Device:
    """Device greedy-4 packing of buckets of one size with the buffers
    allocated once: pack() / unpack() only enqueue (no allocation, no host
    sync); result() / unpack_result() read the (count, status) pair back (one
    16-byte D2H each).  Pack and unpack keep separate result pairs and
    workspaces, so a pack's word count survives an unpack enqueued before it
    is read.  The pack workspace starts zeroed; every pack leaves it so."""

    def __init__(self, n: int, device, unpack_words: int | None = None):
        lib = _lib.load()
        self.device = torch.device(device)
        self.n = int(n)
        self.cap = self.n // 3 + 2
        self.words = torch.empty(self.cap, dtype=torch.int32, device=self.device)
        nw = self.cap if unpack_words is None else int(unpack_words)
        self.ucap = max(15 * nw, 1)
        self.values = torch.empty(self.ucap, dtype=torch.int32, device=self.device)
        self.ws = torch.zeros(int(lib.gc_greedy4_workspace_size(self.n)), dtype=torch.uint8, device=self.device)
        self.uws = torch.empty(int(lib.gc_greedy4_unpack_workspace_size(nw)), dtype=torch.uint8, device=self.device)
        self.res = torch.zeros(2, dtype=torch.int64, device=self.device)
        self.ures = torch.zeros(2, dtype=torch.int64, device=self.device)

    def pack(self, a: torch.Tensor):
        """a: int32 [n] on the device -> self.words (count via result())."""
        assert a.dtype == torch.int32 and a.numel() == self.n and a.is_contiguous()
        with _g4_one_pack(self.device):
            check(_lib.load().gc_greedy4_pack_device(_p(a), self.n, _p(self.words), self.cap, _p(self.res),
                                                     C.c_void_p(self.res.data_ptr() + 8), _p(self.ws),
                                                     _stream(self.device)), "gc_greedy4_pack_device")

    def unpack(self, w: torch.Tensor):
        """w: int32 words on the device -> self.values (count via unpack_result())."""
        assert w.dtype == torch.int32 and w.is_contiguous() and 15 * w.numel() <= self.ucap
        check(_lib.load().gc_greedy4_unpack_device(_p(w), w.numel(), _p(self.values), self.ucap, _p(self.ures),
                                                   C.c_void_p(self.ures.data_ptr() + 8), _p(self.uws),
                                                   _stream(self.device)), "gc_greedy4_unpack_device")

    def result(self, what: str = "greedy4_pack") -> int:
        """The last pack's word count.  After a timed-out pack (status 4) the
        workspace is zeroed again before raising (blocks that start
        late tag their granules with the next launch's tags, which the next
        pack would otherwise compose as valid)."""
        count, status = (int(v) for v in self.res.cpu().tolist())
        if status & 4:
            self.ws.zero_()
        return _g4_check(count, status, what)

    def unpack_result(self, what: str = "greedy4_unpack") -> int:
        """The last unpack's value count."""
        return _g4_result(self.ures, what)


def greedy4_pack(src: torch.Tensor) -> torch.Tensor:
    """The reference's greedy 4-mode format (extensions/Extension CPU/bitpacking.cpp:5-124).
    Device tensors: HIP segment-table scan packer (gc_greedy4_pack_device); host
    tensors: the host packer, like the reference's CPU extension."""
    lib = _lib.load()
    if src.is_cuda:
        a = src.detach().contiguous().view(-1)
        if a.dtype != torch.int32:
            a = a.to(torch.int32)
        pk = Greedy4Device(a.numel(), _dev(a), unpack_words=0)
        pk.pack(a)
        return pk.words[:pk.result("greedy4_pack")]
    a = np.ascontiguousarray(src.detach().numpy().astype(np.int32, copy=False)).reshape(-1)
    out = np.empty(a.size + 1, dtype=np.int32)
    nw = check(lib.gc_greedy4_pack(a.ctypes.data_as(C.c_void_p), a.size, out.ctypes.data_as(C.c_void_p),
                                   out.size), "gc_greedy4_pack")
    return torch.from_numpy(out[:nw].copy())


_G4_WS = {}  # device index -> the pack workspace, zeroed once (every pack leaves it so)
_G4_LAST = {}  # device index -> (event after the last pack enqueued on the device, its stream)


class _g4_one_pack:
    """One persistent pack in flight per device (gcodec.h): a pack
    enqueued on a stream other than the previous pack's waits for that pack's
    event, then records its own."""

    def __init__(self, dev):
        self.dev = dev

    def __enter__(self):
        cur = torch.cuda.current_stream(self.dev)
        last = _G4_LAST.get(self.dev.index)
        if last is not None and last[1] != cur:
            cur.wait_event(last[0])
        self.cur = cur
        return self

    def __exit__(self, *exc):
        ev = torch.cuda.Event()
        ev.record(self.cur)
        _G4_LAST[self.dev.index] = (ev, self.cur)
        return False


def _g4_pack_ws(dev) -> torch.Tensor:
    """The device's one pack workspace (one pack in flight per device)."""
    ws = _G4_WS.get(dev.index)
    if ws is None:
        ws = _G4_WS[dev.index] = torch.zeros(int(_lib.load().gc_greedy4_workspace_size(0)), dtype=torch.uint8,
                                             device=dev)
    return ws


def greedy4_pack_many(*srcs: torch.Tensor) -> list:
    """greedy4_pack of several arrays with one host synchronisation: on the
    device every pack is enqueued on the caller's stream (one workspace per
    stream, zeroed once), then the word counts of all of them come back in one
    D2H read.  QSGDBPCompressor.compress packs the sign bits and the
    magnitudes this way (compressors.py:357-358 packs them one after the other
    on the host).  Host tensors: greedy4_pack each."""
    if not srcs or not all(t.is_cuda for t in srcs):
        return [greedy4_pack(t) for t in srcs]
    dev = _dev(srcs[0])
    if any(_dev(t) != dev for t in srcs):
        raise ValueError("greedy4_pack_many: arrays on different devices")
    lib = _lib.load()
    st = _stream(dev)
    ws = _g4_pack_ws(dev)
    res = torch.zeros(2 * len(srcs), dtype=torch.int64, device=dev)  # (count, status) per pack, written by each
    outs, keep = [], []
    with _g4_one_pack(dev):
        for i, src in enumerate(srcs):
            a = src.detach().contiguous().view(-1)
            if a.dtype != torch.int32:
                a = a.to(torch.int32)
            keep.append(a)  # alive until the launches are enqueued (the stream orders their use)
            cap = a.numel() // 3 + 2
            words = torch.empty(cap, dtype=torch.int32, device=dev)
            check(lib.gc_greedy4_pack_device(_p(a), a.numel(), _p(words), cap, C.c_void_p(res.data_ptr() + 16 * i),
                                             C.c_void_p(res.data_ptr() + 16 * i + 8), _p(ws), st),
                  "gc_greedy4_pack_device")
            outs.append(words)
    pairs = res.cpu().view(-1, 2).tolist()
    if any(int(stt) & 4 for _, stt in pairs):
        ws.zero_()  # a timed-out pack: zero the workspace again (the stream orders it after the packs)
    return [w[:_g4_check(int(c), int(stt), "greedy4_pack")] for w, (c, stt) in zip(outs, pairs)]


def greedy4_unpack_many(*words: torch.Tensor) -> list:
    """greedy4_unpack of several word arrays with one host synchronisation
    (every unpack enqueued, then all value counts in one D2H read); host
    tensors: greedy4_unpack each."""
    if not words or not all(t.is_cuda for t in words):
        return [greedy4_unpack(t) for t in words]
    dev = _dev(words[0])
    if any(_dev(t) != dev for t in words):
        raise ValueError("greedy4_unpack_many: arrays on different devices")
    lib = _lib.load()
    st = _stream(dev)
    res = torch.empty(2 * len(words), dtype=torch.int64, device=dev)
    outs, keep = [], []
    for i, w in enumerate(words):
        a = w.detach().contiguous().view(-1)
        if a.dtype != torch.int32:
            a = a.to(torch.int32)
        nw = a.numel()
        cap = 15 * nw
        out = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
        ws = torch.empty(int(lib.gc_greedy4_unpack_workspace_size(nw)), dtype=torch.uint8, device=dev)
        keep += [a, ws]  # alive until enqueued: the stream orders their reuse by the allocator
        check(lib.gc_greedy4_unpack_device(_p(a), nw, _p(out), cap, C.c_void_p(res.data_ptr() + 16 * i),
                                           C.c_void_p(res.data_ptr() + 16 * i + 8), _p(ws), st),
              "gc_greedy4_unpack_device")
        outs.append(out)
    pairs = res.cpu().view(-1, 2).tolist()
    return [o[:_g4_check(int(c), int(stt), "greedy4_unpack")] for o, (c, stt) in zip(outs, pairs)]


def greedy4_unpack(words: torch.Tensor) -> torch.Tensor:
    """Inverse of greedy4_pack; emits whole words (callers truncate, compressors.py:371)."""
    lib = _lib.load()
    if words.is_cuda:
        dev = _dev(words)
        a = words.detach().contiguous().view(-1)
        if a.dtype != torch.int32:
            a = a.to(torch.int32)
        nw = a.numel()
        cap = 15 * nw
        out = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
        ws = torch.empty(int(lib.gc_greedy4_unpack_workspace_size(nw)), dtype=torch.uint8, device=dev)
        res = torch.zeros(2, dtype=torch.int64, device=dev)
        check(lib.gc_greedy4_unpack_device(_p(a), nw, _p(out), cap, _p(res), C.c_void_p(res.data_ptr() + 8), _p(ws),
                                           _stream(dev)), "gc_greedy4_unpack_device")
        return out[:_g4_result(res, "greedy4_unpack")]
    a = np.ascontiguousarray(words.detach().numpy().astype(np.int32, copy=False)).reshape(-1)
    out = np.empty(15 * a.size + 1, dtype=np.int32)
    cnt = check(lib.gc_greedy4_unpack(a.ctypes.data_as(C.c_void_p), a.size, out.ctypes.data_as(C.c_void_p),
                                      out.size), "gc_greedy4_unpack")
    return torch.from_numpy(out[:cnt].copy())
