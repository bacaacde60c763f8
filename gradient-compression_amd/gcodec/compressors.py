"""Drop-in compressor classes with the reference's names, constructor
arguments and method signatures (compressors.py), backed by the gfx950 HIP
kernels of libgcodec.

    reference (compressors.py)                       here
    QSGDMaxNormCompressor            283-321         QSGDMaxNormCompressor
    GlobalRandKMaxNormCompressor     419-456         GlobalRandKMaxNormCompressor
    QSGDMaxNormTwoScaleCompressor    612-680         QSGDMaxNormTwoScaleCompressor
    GlobalRandKMaxNormTwoScaleCompressor 683-751     GlobalRandKMaxNormTwoScaleCompressor
    QSGDMaxNormMultiScaleCompressor  754-826         QSGDMaxNormMultiScaleCompressor
    QSGDBPCompressor (commented)     324-378         QSGDBPCompressor (greedy 4-mode packing on the GPU)

compress()/decompress() return exactly what the reference returns (int8 for
b < 8 else int32; float32), on the same device.  With the generator in
"torch" mode (gcodec.manual_seed(seed, mode="torch") or
gcodec.set_rng_mode("torch")) the draws are torch's CPU-generator stream, so
`torch.manual_seed(s); c.compress(norm, x)` is bit-identical to the
reference.  Each class also offers the packed, all-reduce-compatible
encode()/decode() the reducers use.

Divergences (documented in DESIGN.md): a zero / non-finite max-norm gives
q = 0 where torch.bernoulli raises; the multi-scale constructor copies and
sorts the caller's level list instead of sorting it in place (768).
"""
from __future__ import annotations

import numpy as np
import torch

from . import codec as _codec
from .rng import default_generator


def _qdtype(bits: int) -> torch.dtype:
    # compressors.py:294-297
    return torch.int8 if bits < 8 else torch.int32


# torch mode: the draw format the packed QSGD encode asks for
# (rng.Generator.reserve fmt; codec.mt19937_reserve): "plain" 32-bit draws,
# "packed24" (3 bytes per draw), or the split planes "split8" / "split16"
# (the encode reads 1 / 2 bytes per draw and the rest only where the rounding
# is undecided).  Formats the run cannot take fall back to plain draws.
# Plain: the split16 encode is faster alone (122 against 145 us per 1e8), but
# its generator takes 1.2-1.4 against 0.81 ms per 64-walker run and the
# pipelined call came out equal back to back and slower in a training cadence
# (profiles/r06*_torch_*.log)
TORCH_DRAW_FORMAT = "plain"


class _Base:
    backend = _codec

    def __init__(self, device, generator=None):
        self._device = device
        self._gen = generator or default_generator

    def _reserve(self, n: int, levels: int, device, fmt: str | None = None):
        if fmt and fmt != "plain":  # torch mode: cut draws where the run allows (rng.Generator.reserve)
            return self._gen.reserve(n, levels, device=device, backend=self.backend, fmt=fmt)
        return self._gen.reserve(n, levels, device=device, backend=self.backend)


class QSGDMaxNormCompressor(_Base):
    """compressors.py:283-321.  Code: sign array * xi array."""

    def __init__(self, device, quantization_level=8, generator=None):
        super().__init__(device, generator)
        self._quantization_level = quantization_level
        self._dtype = _qdtype(quantization_level)

    def compress(self, norm, tensor):
        # torch mode: the draws are generated on the GPU into a buffer, then
        # quantized by the full-chip kernel.  (codec.qsgd_quantize_torch, the
        # generator kernel consuming its own draws, gives the same q but runs
        # slower on MI355X: DESIGN_HISTORY §7.)
        rng = self._reserve(tensor.numel(), 1, tensor.device)
        return self.backend.qsgd_quantize(tensor, norm, self._quantization_level, rng, 0, self._dtype)

    def decompress(self, norm, sign_xi_array):
        return self.backend.qsgd_dequantize(sign_xi_array, norm, self._quantization_level)

    # packed, SUM-all-reduce-compatible stream (carry-free lanes for `world`)
    def encode(self, norm, tensor, world=1, idx=None, out=None):
        n = idx.numel() if idx is not None else tensor.numel()
        rng = self._reserve(n, 1, tensor.device, fmt=TORCH_DRAW_FORMAT)
        return self.backend.qsgd_encode(tensor, norm, self._quantization_level, rng, world, idx, out)

    def decode(self, norm, words, n, world=1, alpha=1.0, idx=None, out=None):
        return self.backend.qsgd_decode(words, n, norm, self._quantization_level, world, alpha, idx, out)

    def decode_segments(self, norm, words, segs, world=1, alpha=1.0):
        return self.backend.qsgd_decode_segments(words, norm, self._quantization_level, segs, world, alpha)


class GlobalRandKMaxNormCompressor(QSGDMaxNormCompressor):
    """compressors.py:419-456 — the same arithmetic applied to the K-subset."""

    def encode_w1(self, tensor, idx, out=None):
        """W = 1: gather + max-norm + encode of tensor[idx] in one launch ->
        (words, norm); the same words as encode(max|tensor[idx]|, tensor, idx=idx)."""
        rng = self._reserve(idx.numel(), 1, tensor.device)
        return self.backend.randk_encode_w1(tensor, idx, self._quantization_level, rng, out=out)

    def encode_w1_segments(self, segs, idx, out=None, xk=None, norm=None):
        """encode_w1 with the tensor given as the per-parameter tensors of segs
        (out / xk / norm: preallocated words, gathered subset and norm)."""
        rng = self._reserve(idx.numel(), 1, segs.device)
        return self.backend.randk_encode_w1_segments(segs, idx, self._quantization_level, rng, xk=xk, norm=norm,
                                                     out=out)

    def decode_scatter_segments(self, norm, words, idx, segs, world=1, alpha=1.0):
        """decode(..., idx=idx) writing element idx[i] straight into its tensor."""
        return self.backend.qsgd_decode_scatter_segments(words, idx, norm, self._quantization_level, segs, world,
                                                         alpha)


class QSGDBPCompressor(_Base):
    """compressors.py:324-378 (kept commented out in the reference because it
    needs the custom extension): QSGD with the bucket's own max-norm, the sign
    bits and the magnitudes packed separately in the greedy 4-mode format of
    extensions/Extension CPU/bitpacking.cpp.  Code: (norm / s, sign_packed,
    xi_packed, xi_size).  Here the quantize (gc_qsgd_quantize_split) and both
    packers (gc_greedy4_pack_device / _unpack_device) run on the GPU — the
    reference moves each array to the host, packs it there and copies it back
    (compressors.py:357-358, 370-372).  Defined for b <= 8 (the format's
    domain is [0, 255])."""

    def __init__(self, device, quantization_level=8, generator=None):
        super().__init__(device, generator)
        if not 1 <= quantization_level <= 8:
            raise ValueError("QSGDBPCompressor: the greedy 4-mode format holds values in [0, 255] (b <= 8)")
        self._quantization_level = quantization_level

    def compress(self, tensor):
        s = (1 << self._quantization_level) - 1
        norm = self.backend.absmax(tensor)  # compressors.py:341 (the bucket's own max)
        rng = self._reserve(tensor.numel(), 1, tensor.device)
        xi, sign = self.backend.qsgd_quantize_split(tensor, norm, self._quantization_level, rng)
        many = getattr(self.backend, "greedy4_pack_many", None)
        if many is not None:  # both packs enqueued, one host sync for the two word counts
            sign_packed, xi_packed = many(sign, xi)
        else:
            sign_packed = self.backend.greedy4_pack(sign)
            xi_packed = self.backend.greedy4_pack(xi)
        xi_size = torch.tensor(xi_packed.size(), device=tensor.device)
        # norm / s, correctly rounded (numpy float32 division; the packers above already synchronised)
        c = torch.tensor(np.float32(norm.item()) / np.float32(s), dtype=torch.float32, device=tensor.device)
        return c, sign_packed, xi_packed, xi_size

    def decompress(self, norm, sign_packed, xi_packed, tensor_size):
        n = int(tensor_size)
        many = getattr(self.backend, "greedy4_unpack_many", None)
        if many is not None:  # both unpacks enqueued, one host sync for the two value counts
            sign, xi = many(sign_packed, xi_packed)
        else:
            sign = self.backend.greedy4_unpack(sign_packed)
            xi = self.backend.greedy4_unpack(xi_packed)
        fused = getattr(self.backend, "qsgdbp_decode", None)
        if fused is not None and xi.is_cuda:
            return fused(sign, xi, norm, n)  # one kernel (gc_qsgdbp_decode)
        sign, xi = sign[:n], xi[:n]
        # norm * sign * xi in the reference's order, fp32: (c * (+-1)) is exact, then one
        # rounding; a negative x that rounded to 0 decodes to -0.0 as in the reference
        sgn = torch.where(sign == 1, -1.0, 1.0).to(torch.float32)
        return (norm * sgn) * xi.to(torch.float32)


class _MultiScalePacked(_Base):
    """Packed mask + select of the two-scale and multi-scale classes.

    The reference splits the work as compress_cache (every level's sign*xi
    into an L x n float32 cache) -> compress_mask -> MIN all-reduce ->
    compress(mask), which reads the cache (compressors.py:778-817).  Here
    encode_mask writes the thermometer mask lanes and, when the backend has a
    packed form of the cache for these levels (codec.ms_cache_bytes > 0: dense
    x, 2-3 levels of <= 24 bits), the cache as one 1-2 byte cell per element;
    encode then reads the cells at the common level instead of x and the
    draws.  Without a cache encode recomputes the chosen level from the same
    reserved draws.  Either way the words are identical.  q_cache=None (the
    default) picks by world size: at W = 1 the reducers run the one-pass
    encode (encode_w1, no cache needed); at W > 1 the cache pays, because the
    select then runs no Philox at all (ResNet50 bucket, MI355X r02y: mask 41.2
    + select 15.3 us with the cache against 25.7 + 38.5 us without; both
    kernels are VALU-issue bound).  True / False force
    it on / off."""

    def __init__(self, device, generator=None, q_cache=None):
        super().__init__(device, generator)
        self.q_cache = q_cache
        self._rng = None
        self._cache = None
        self._cache_key = None

    def _packed_levels(self):
        raise NotImplementedError

    def _cache_buffer(self, tensor, n, idx, levels, world):
        nbytes = getattr(self.backend, "ms_cache_bytes", None)
        use = self.q_cache if self.q_cache is not None else world > 1
        if not use or nbytes is None or idx is not None or tensor.data_ptr() % 16:
            return None
        nb = nbytes(n, levels)
        if not nb:
            return None
        if self._cache is None or self._cache.numel() < n * nb or self._cache.device != tensor.device:
            self._cache = torch.empty(n * nb, dtype=torch.uint8, device=tensor.device)
        return self._cache

    def encode_mask(self, norm, tensor, world=1, idx=None):
        levels = self._packed_levels()
        n = idx.numel() if idx is not None else tensor.numel()
        self._rng = self._reserve(n, len(levels), tensor.device)
        self._cache_key = None
        cache = self._cache_buffer(tensor, n, idx, levels, world)
        if cache is None:
            return self.backend.ms_mask_encode(tensor, norm, levels, self._rng, world, idx)
        self._cache_key = (tensor.data_ptr(), n)
        return self.backend.ms_mask_encode(tensor, norm, levels, self._rng, world, cache=cache)

    def encode_w1(self, norm, tensor):
        """W = 1: (mask_words, words) in one pass over x (the MIN all-reduce of
        the mask over one rank is the identity), the same streams as
        encode_mask + encode; None when the backend has no one-pass form for
        this bucket (the caller then runs the two passes)."""
        levels = self._packed_levels()
        ok = getattr(self.backend, "ms_w1_ok", None)
        if ok is None or not ok(tensor, levels):
            return None
        self._rng = self._reserve(tensor.numel(), len(levels), tensor.device)
        self._cache_key = None
        return self.backend.ms_encode_w1(tensor, norm, levels, self._rng)

    def encode(self, norm, tensor, mask_words, world=1, idx=None):
        levels = self._packed_levels()
        n = idx.numel() if idx is not None else tensor.numel()
        if idx is None and self._cache_key == (tensor.data_ptr(), n):
            return self.backend.ms_select_encode(tensor, norm, levels, self._rng, mask_words, world,
                                                 cache=self._cache)
        return self.backend.ms_select_encode(tensor, norm, levels, self._rng, mask_words, world, idx)


class QSGDMaxNormTwoScaleCompressor(_MultiScalePacked):
    """compressors.py:612-680.  compress_lower consumes draws [0, n) and
    compress_higher [n, 2n) of one reservation (level 0 / level 1)."""

    def __init__(self, device, lower_quantization_level=6, higher_quantization_level=10, generator=None,
                 q_cache=None):
        super().__init__(device, generator, q_cache)
        self._lower_quantization_level = lower_quantization_level
        self._higher_quantization_level = higher_quantization_level
        self._dtype = _qdtype(lower_quantization_level)

    @property
    def levels(self):
        return [self._lower_quantization_level, self._higher_quantization_level]

    def _packed_levels(self):
        return self.levels

    def compress_lower(self, norm, tensor):
        self._rng = self._reserve(tensor.numel(), 2, tensor.device)
        return self.backend.qsgd_quantize(tensor, norm, self._lower_quantization_level, self._rng, 0, self._dtype)

    def compress_higher(self, norm, tensor):
        if self._rng is None or self._rng.n != tensor.numel():
            self._rng = self._reserve(tensor.numel(), 2, tensor.device)
        q, h = self.backend.qsgd_quantize(tensor, norm, self._higher_quantization_level, self._rng, 1, self._dtype,
                                          le_bits=self._lower_quantization_level)
        self._rng = None
        return q, h

    def decompress(self, norm, sign_xi_array, higher_resolution_mask):
        return self.backend.ms_dequantize(sign_xi_array, higher_resolution_mask, norm, self.levels, order=1)

    # packed: encode_mask / encode (_MultiScalePacked) over the two levels
    def decode(self, norm, words, mask_words, n, world=1, alpha=1.0, idx=None, out=None):
        return self.backend.ms_decode(words, mask_words, n, norm, self.levels, world, 1, alpha, idx, out)

    def decode_segments(self, norm, words, mask_words, segs, world=1, alpha=1.0):
        return self.backend.ms_decode_segments(words, mask_words, norm, self.levels, segs, world, 1, alpha)


class GlobalRandKMaxNormTwoScaleCompressor(QSGDMaxNormTwoScaleCompressor):
    """compressors.py:683-751 — identical arithmetic on the K-subset."""

    def decode_scatter_segments(self, norm, words, mask_words, idx, segs, world=1, alpha=1.0):
        """decode(..., idx=idx) writing element idx[i] straight into its tensor."""
        return self.backend.ms_decode_scatter_segments(words, mask_words, idx, norm, self.levels, segs, world, 1,
                                                       alpha)


class QSGDMaxNormMultiScaleCompressor(_MultiScalePacked):
    """compressors.py:754-826.  Unpacked forms: no L x n float cache, the
    select pass recomputes the chosen level from the same reserved draws.
    Packed forms: optionally the cache as 1-2 byte cells where the levels
    allow it (_MultiScalePacked, q_cache=True)."""

    def __init__(self, device, quantization_levels=None, generator=None, q_cache=None):
        super().__init__(device, generator, q_cache)
        if not quantization_levels:
            quantization_levels = [6, 10]
        self._quantization_levels = sorted(quantization_levels)
        self._dtype = _qdtype(self._quantization_levels[0])
        self._x = None
        self._norm = None

    def _packed_levels(self):
        return self._quantization_levels

    def compress_cache(self, norm, tensor):
        self._rng = self._reserve(tensor.numel(), len(self._quantization_levels), tensor.device)
        self._x, self._norm = tensor, norm

    def compress_mask(self, norm, tensor):
        self.compress_cache(norm, tensor)
        return self.backend.ms_quantize_mask(tensor, norm, self._quantization_levels, self._rng)

    def compress(self, resolution_mask):
        return self.backend.ms_select_quantize(self._x, self._norm, self._quantization_levels, self._rng,
                                               resolution_mask, self._dtype)

    def decompress(self, norm, sign_xi_array, resolution_mask):
        return self.backend.ms_dequantize(sign_xi_array, resolution_mask, norm, self._quantization_levels, order=0)

    # packed: encode_mask / encode (_MultiScalePacked)
    def decode(self, norm, words, mask_words, n, world=1, alpha=1.0, idx=None, out=None):
        return self.backend.ms_decode(words, mask_words, n, norm, self._quantization_levels, world, 0, alpha, idx,
                                      out)

    def decode_segments(self, norm, words, mask_words, segs, world=1, alpha=1.0):
        return self.backend.ms_decode_segments(words, mask_words, norm, self._quantization_levels, segs, world, 0,
                                               alpha)
