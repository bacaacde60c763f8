"""A CPU stand-in for gcodec.codec built on the oracle — TEST ONLY.

It exposes the functions gcodec.reducer calls, computed by
oracle/gcodec_oracle.c on CPU tensors, so the reducers' host logic (norm
collective, lane sizing for W, thermometer mask reduction, GRandK queue,
setgrad) can run under a gloo process group on CPU and be compared with the
reference reducers' golden outputs.  The product never imports this.
"""
from __future__ import annotations

import numpy as np
import torch

from oracle import oracle as O


def _np(t):
    return np.ascontiguousarray(t.detach().cpu().numpy())


def _norm(norm) -> np.float32:
    if isinstance(norm, torch.Tensor):
        return np.float32(norm.reshape(-1)[0].item())
    return np.float32(norm)


def _rng(r):
    if r.kind == 0:
        return O.philox_rng(r.seed, r.offset)
    return O.stream_rng(r.stream.numpy().view(np.uint32))


def _gather(x, idx):
    xa = _np(x).reshape(-1)
    return xa if idx is None else xa[_np(idx).astype(np.int64)]


def _qmax_ms(levels):
    lv = sorted(levels)
    return (1 << lv[0]) - 1 + (1 if len(lv) >= 3 else 0)


def absmax(x, idx=None, out=None):
    v = torch.tensor([O.absmax(_gather(x, idx))], dtype=torch.float32)
    if out is not None:
        out.copy_(v)
        return out
    return v


RANDK_FUSED_MAX = 16384
RANDK_GATHER_MAX = 256 * 1024


def randk_gather_absmax(x, idx, xk=None, norm=None):
    xs = _gather(x, idx)
    return torch.from_numpy(xs.copy()), torch.tensor([O.absmax(xs)], dtype=torch.float32)


def randk_encode_w1(x, idx, bits, rng, xk=None, norm=None, out=None, lanes=None):
    xs = _gather(x, idx)
    nk = O.absmax(xs)
    words = O.qsgd_encode(xs, nk, bits, 1, _rng(rng))
    return torch.from_numpy(words.view(np.int32).copy()), torch.tensor([nk], dtype=torch.float32)


def qsgd_encode(x, norm, bits, rng, world=1, idx=None, out=None, lanes=None):
    words = O.qsgd_encode(_gather(x, idx), _norm(norm), bits, world, _rng(rng))
    return torch.from_numpy(words.view(np.int32).copy())


def qsgd_decode(words, n, norm, bits, world=1, alpha=1.0, idx=None, out=None, lanes=None):
    dec = O.qsgd_decode(_np(words).view(np.uint32), n, _norm(norm), bits, world, np.float32(alpha))
    return _place(dec, idx, out)


def _place(vals, idx, out):
    if idx is None:
        t = torch.from_numpy(vals)
        if out is not None:
            out.copy_(t)
            return out
        return t
    out[torch.as_tensor(_np(idx).astype(np.int64))] = torch.from_numpy(vals)
    return out


def ms_mask_encode(x, norm, levels, rng, world=1, idx=None, out=None):
    xa = _gather(x, idx)
    n = xa.size
    m = O.ms_mask(xa, _norm(norm), levels, _rng(rng)).astype(np.int32)
    w, L, M = O.lane_layout(n, 1, world)
    fields = [O.lane_pack((m > f).astype(np.int32), 0, w, L, M) for f in range(len(levels) - 1)]
    return torch.from_numpy(np.concatenate(fields).view(np.int32).copy())


def _mask_from_sum(mask_words, n, levels, world):
    w, L, M = O.lane_layout(n, 1, world)
    mw = _np(mask_words).view(np.uint32)
    m = np.zeros(n, np.int32)
    for f in range(len(levels) - 1):
        m += O.lane_unpack(mw[f * M:(f + 1) * M], n, 0, world, w, L, M) == world
    return m.astype(np.uint8)


def ms_select_encode(x, norm, levels, rng, mask_words, world=1, idx=None, out=None):
    xa = _gather(x, idx)
    n = xa.size
    m = _mask_from_sum(mask_words, n, levels, world)
    q = O.ms_select(xa, _norm(norm), levels, _rng(rng), m)
    qmax = _qmax_ms(levels)
    w, L, M = O.lane_layout(n, 2 * qmax, world)
    return torch.from_numpy(O.lane_pack(q, qmax, w, L, M).view(np.int32).copy())


def ms_w1_ok(x, levels):
    return len(levels) in (2, 3) and x.dim() == 1


def ms_encode_w1(x, norm, levels, rng, mask_out=None, out=None):
    m = ms_mask_encode(x, norm, levels, rng, 1)
    return m, ms_select_encode(x, norm, levels, rng, m, 1)


def ms_decode(words, mask_words, n, norm, levels, world=1, order=0, alpha=1.0, idx=None, out=None):
    m = _mask_from_sum(mask_words, n, levels, world)
    qmax = _qmax_ms(levels)
    w, L, M = O.lane_layout(n, 2 * qmax, world)
    q = O.lane_unpack(_np(words).view(np.uint32), n, qmax, world, w, L, M)
    dec = O.ms_dequantize(q, _norm(norm), levels, m, order, np.float32(alpha))
    return _place(dec, idx, out)


def mt19937_draws(count, device=None, packed24=False):
    """torch CPU-generator draws via the oracle MT; advances torch's state
    (always the plain 32-bit draws: packed24 is a device-side layout)."""
    from gcodec.rng import set_torch_mt_state, torch_mt_state

    words, idx = torch_mt_state()
    st = O.MT19937(0)
    st._st.s[:] = [int(v) for v in words]
    st._st.idx = idx
    d = st.draws(count)
    s2, i2 = st.state()
    set_torch_mt_state(s2, i2)
    return torch.from_numpy(d.view(np.int32).copy())
