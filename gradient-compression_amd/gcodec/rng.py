"""Random streams for the stochastic rounding (compressors.py:310 torch.bernoulli).

Two modes, one descriptor (include/gcodec.h `gc_rng`):

* ``"philox"`` — the performance mode.  Philox4x32-10 keyed by ``seed``;
  element i of scale level l in a call that starts at draw ``offset`` uses
  word ``i & 3`` of the block at counter ``(i >> 2, l, offset)``.  Counter
  based, so the draws do not depend on the launch configuration and any
  element can be recomputed (the multi-scale select pass re-reads its draw
  instead of caching L x n values).  The reference's own GPU runs draw with
  torch.cuda's Philox too; those draws are not reproducible off-device, so
  this stream's oracle is oracle/gcodec_oracle.c.

* ``"torch"`` — the reference-parity mode.  Draws come from torch's global CPU
  generator (MT19937, seeded by torch.manual_seed, seed.py:6-11) exactly as
  torch.bernoulli on CPU consumes them: one 32-bit draw per element, in
  order.  The state is read from torch.get_rng_state(), the draws are
  generated on the GPU (gc_mt19937_generate) and the advanced state is
  written back, so a caller's torch RNG stays where compressors.py would
  have left it.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

MT_N = 624
_STATE_BYTES = 5056  # sizeof(at::CPUGeneratorImplState) on torch 2.x
_OFF_LEFT, _OFF_NEXT, _OFF_STATE = 8, 16, 24


def torch_mt_state():
    """(624 uint32 words, next index) of torch's CPU generator."""
    raw = torch.get_rng_state().numpy()
    if raw.size != _STATE_BYTES:
        raise _lib.GCodecError(_lib.GC_EINVAL, f"unexpected torch RNG state size {raw.size}")
    left = int(raw[_OFF_LEFT:_OFF_LEFT + 4].view(np.int32)[0])
    nxt = int(raw[_OFF_NEXT:_OFF_NEXT + 8].view(np.uint64)[0])
    words = raw[_OFF_STATE:_OFF_STATE + 8 * MT_N].view(np.uint64).astype(np.uint32)
    idx = MT_N if left <= 1 else nxt
    return words, idx


def set_torch_mt_state(words: np.ndarray, idx: int):
    raw = torch.get_rng_state().numpy().copy()
    raw[_OFF_STATE:_OFF_STATE + 8 * MT_N] = words.astype(np.uint64).view(np.uint8)
    raw[_OFF_LEFT:_OFF_LEFT + 4] = np.array([MT_N + 1 - idx if idx >= 1 else 1], np.int32).view(np.uint8)
    raw[_OFF_NEXT:_OFF_NEXT + 8] = np.array([idx if idx >= 1 else 0], np.uint64).view(np.uint8)
    torch.set_rng_state(torch.from_numpy(raw))


class Reservation:
    """Draws reserved for one compress call: ``levels`` blocks of ``n``."""

    def __init__(self, kind: int, seed: int = 0, offset: int = 0, stream: torch.Tensor | None = None, n: int = 0,
                 levels: int = 1):
        self.kind, self.seed, self.offset, self.stream, self.n, self.levels = kind, seed, offset, stream, n, levels

    def struct(self) -> _lib.gc_rng:
        ptr = self.stream.data_ptr() if self.stream is not None else None
        return _lib.gc_rng(self.kind, 0, self.seed & (2 ** 64 - 1), self.offset, ptr)

    def draws(self) -> np.ndarray | None:
        return None if self.stream is None else self.stream.cpu().numpy().view(np.uint32)


def _process_rank() -> int:
    import torch.distributed as dist

    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


class Generator:
    """Draw allocator of one codec stream.

    per_rank=True keys the Philox stream by seed + the process's global rank
    (read at every reservation), so ranks that share one Generator object by
    default still draw independent uniforms — the reference seeds every rank's
    torch generator with seed + rank (model_dispatcher.py:59, trainer.py:158).
    Identical draws on every rank would correlate the ranks' rounding errors
    instead of averaging them down with W.

    A caller that already follows the reference's seeding (seed + rank per
    rank, trainer.py:158) passes the BASE seed to a per_rank generator, or
    uses per_rank=False with its own seed + rank; passing seed + rank to a
    per_rank generator keys the stream with seed + 2 rank.  The process-wide
    default_generator is per_rank; gcodec.manual_seed(seed, per_rank=False)
    switches it to the caller's key."""

    def __init__(self, seed: int = 42, mode: str = "philox", per_rank: bool = False):
        self.per_rank = per_rank
        self.set_mode(mode)
        self.manual_seed(seed)

    def set_mode(self, mode: str):
        if mode not in ("philox", "torch"):
            raise ValueError("rng mode must be 'philox' or 'torch'")
        if getattr(self, "mode", None) == "torch" and mode != "torch":
            from . import codec

            codec.mt_release()  # the speculative draws and workspaces torch mode kept on the device
        self.mode = mode

    def manual_seed(self, seed: int):
        self.seed = int(seed)
        self.offset = 0
        return self

    def reserve_key(self) -> int:
        """The Philox key the next reservation uses (seed, + rank if per_rank)."""
        return self.seed + (_process_rank() if self.per_rank else 0)

    def reserve(self, n: int, levels: int = 1, device=None, backend=None, packed24: bool = False,
                fmt: str | None = None) -> Reservation:
        """Reserve n*levels draws (advances the stream like torch's generator).
        Torch mode, one level: fmt "packed24" (or packed24=True) / "split8" /
        "split16" cuts the draws to the 24 bits the rounding reads where the
        run allows it (codec.mt19937_reserve), else the plain 32-bit draws are
        returned; only the QSGD encode (gc_qsgd_encode) takes such a
        reservation."""
        count = n * levels
        if self.mode == "philox":
            r = Reservation(_lib.GC_RNG_PHILOX, self.reserve_key(), self.offset, None, n, levels)
            self.offset += count
            return r
        if backend is None:
            from . import codec as backend
        fmt = fmt or ("packed24" if packed24 else "plain")
        if fmt != "plain" and levels == 1 and hasattr(backend, "mt19937_reserve"):
            stream, kind = backend.mt19937_reserve(count, device, fmt)
            return Reservation(kind, 0, 0, stream, n, levels)
        if fmt == "packed24" and levels == 1:
            stream = backend.mt19937_draws(count, device, packed24=True)
            kind = _lib.GC_RNG_STREAM24 if count and stream.numel() != count else _lib.GC_RNG_STREAM
            return Reservation(kind, 0, 0, stream, n, levels)
        stream = backend.mt19937_draws(count, device)
        return Reservation(_lib.GC_RNG_STREAM, 0, 0, stream, n, levels)


# The mode of the stream every compressor / reducer / pipeline uses when none
# is passed: "torch", so the reference-named classes give the reference's
# integers with no mode call (torch.manual_seed(s) then compress, exactly as
# compressors.py:299-316 under seed.py:6-11).  "philox" is the fast,
# non-identical stream: gcodec.manual_seed(seed, mode="philox"),
# gcodec.set_rng_mode("philox") or an explicit gcodec.Generator(seed, "philox").
DEFAULT_MODE = "torch"

# one object per process; in philox mode keyed per rank (see Generator)
default_generator = Generator(per_rank=True, mode=DEFAULT_MODE)


def manual_seed(seed: int, mode: str | None = None, per_rank: bool | None = None) -> Generator:
    """Seed the default generator.  per_rank (kept when None) adds the process
    rank to the Philox key: pass the base seed with per_rank=True, or the
    caller's own seed + rank with per_rank=False (see Generator)."""
    if mode is not None:
        default_generator.set_mode(mode)
    if per_rank is not None:
        default_generator.per_rank = bool(per_rank)
    return default_generator.manual_seed(seed)


def set_mode(mode: str):
    default_generator.set_mode(mode)
