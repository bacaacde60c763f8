"""ctypes/numpy wrapper around liboracle.so — the CPU restatement of the
reference QSGD-MaxNorm codec (see gcodec_oracle.c for file:line citations).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by the product package (`gcodec`).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

RNG_PHILOX = 0
RNG_STREAM = 1


class _Rng(C.Structure):
    _fields_ = [
        ("kind", C.c_uint32),
        ("reserved", C.c_uint32),
        ("seed", C.c_uint64),
        ("offset", C.c_uint64),
        ("stream", C.c_void_p),
    ]


class _MT(C.Structure):
    _fields_ = [("s", C.c_uint32 * 624), ("idx", C.c_uint32)]


def build() -> str:
    import fcntl

    with open(os.path.join(HERE, ".build.lock"), "w") as lk:  # concurrent test workers
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(
            os.path.join(HERE, "gcodec_oracle.c")
        ):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        u64, u32, i32, f32 = C.c_uint64, C.c_uint32, C.c_int32, C.c_float
        sig = {
            "or_mt_seed": (None, [P, u64]),
            "or_mt_fill": (None, [P, P, u64]),
            "or_philox_draw": (u32, [u64, u64, u32, u64]),
            "or_ms2_draw": (u32, [u64, u64, u32, u64]),
            "or_absmax": (f32, [P, u64]),
            "or_absmax_par": (f32, [P, u64, u32]),
            "or_qsgd_encode_par": (None, [P, u64, f32, u32, u32, P, P, u32]),
            "or_qsgd_quantize": (None, [P, u64, f32, u32, P, u32, P]),
            "or_qsgd_dequantize": (None, [P, u64, f32, u32, f32, P]),
            "or_lane_layout": (C.c_int, [u64, u64, u32, P, P, P]),
            "or_lane_pack": (None, [P, u64, i32, u32, u32, u64, P]),
            "or_lane_unpack": (None, [P, u64, i32, u32, u32, u32, u64, P]),
            "or_qsgd_encode": (None, [P, u64, f32, u32, u32, P, P]),
            "or_qsgd_decode": (None, [P, u64, f32, u32, u32, f32, P]),
            "or_ms_mask": (None, [P, u64, f32, P, u32, P, P]),
            "or_ms_select": (None, [P, u64, f32, P, u32, P, P, P]),
            "or_ms_dequantize": (None, [P, u64, f32, P, P, C.c_int, f32, P]),
            "or_greedy4_pack": (C.c_int64, [P, u64, P, u64]),
            "or_greedy4_unpack": (C.c_int64, [P, u64, P, u64]),
            "or_bytepack8": (None, [P, u64, P]),
            "or_byteunpack8": (None, [P, u64, P]),
            "or_gen_input": (None, [P, u64, u64, C.c_int, f32]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.c_void_p)


# --------------------------------------------------------------------------
# RNG
# --------------------------------------------------------------------------
class MT19937:
    """torch CPU generator (at::mt19937) restated; torch.manual_seed(seed)."""

    def __init__(self, seed: int):
        self._st = _MT()
        lib().or_mt_seed(C.byref(self._st), seed)

    def draws(self, count: int) -> np.ndarray:
        out = np.empty(max(count, 1), dtype=np.uint32)
        lib().or_mt_fill(C.byref(self._st), _p(out), count)
        return out[:count]

    def state(self):
        return np.frombuffer(bytes(self._st.s), dtype=np.uint32).copy(), int(self._st.idx)


def philox_rng(seed: int, offset: int = 0):
    r = _Rng(RNG_PHILOX, 0, seed, offset, None)
    return r, None


def stream_rng(draws: np.ndarray):
    d = np.ascontiguousarray(draws, dtype=np.uint32)
    r = _Rng(RNG_STREAM, 0, 0, 0, d.ctypes.data)
    return r, d  # keep d alive


def philox_draw(seed: int, offset: int, level: int, i: int) -> int:
    return int(lib().or_philox_draw(seed, offset, level, i))


def ms2_draw(seed: int, offset: int, level: int, i: int) -> int:
    """The dense two-level stream of the 2-level multi-scale codecs (24 bits)."""
    return int(lib().or_ms2_draw(seed, offset, level, i))


# --------------------------------------------------------------------------
# Codec
# --------------------------------------------------------------------------
def absmax(x: np.ndarray) -> np.float32:
    x = np.ascontiguousarray(x, dtype=np.float32)
    return np.float32(lib().or_absmax(_p(x), x.size))


def qsgd_quantize(x, norm, bits, rng, level=0) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    q = np.empty(max(x.size, 1), dtype=np.int32)
    lib().or_qsgd_quantize(_p(x), x.size, float(norm), bits, C.byref(rng[0]), level, _p(q))
    return q[: x.size]


def qsgd_dequantize(q, norm, bits, alpha=1.0) -> np.ndarray:
    q = np.ascontiguousarray(q, dtype=np.int32)
    out = np.empty(max(q.size, 1), dtype=np.float32)
    lib().or_qsgd_dequantize(_p(q), q.size, float(norm), bits, float(alpha), _p(out))
    return out[: q.size]


def lane_layout(n: int, value_range: int, world: int):
    w, L, M = C.c_uint32(), C.c_uint32(), C.c_uint64()
    rc = lib().or_lane_layout(n, value_range, world, C.byref(w), C.byref(L), C.byref(M))
    if rc != 0:
        raise ValueError(f"lane layout rc={rc}")
    return w.value, L.value, M.value


def lane_pack(q, qoff, w, L, M) -> np.ndarray:
    q = np.ascontiguousarray(q, dtype=np.int32)
    out = np.empty(max(M, 1), dtype=np.uint32)
    lib().or_lane_pack(_p(q), q.size, qoff, w, L, M, _p(out))
    return out[:M]


def lane_unpack(words, n, qoff, world, w, L, M) -> np.ndarray:
    words = np.ascontiguousarray(words, dtype=np.uint32)
    out = np.empty(max(n, 1), dtype=np.int32)
    lib().or_lane_unpack(_p(words), n, qoff, world, w, L, M, _p(out))
    return out[:n]


def qsgd_encode(x, norm, bits, world, rng) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    s = (1 << bits) - 1
    _, _, M = lane_layout(x.size, 2 * s, world)
    out = np.empty(max(M, 1), dtype=np.uint32)
    lib().or_qsgd_encode(_p(x), x.size, float(norm), bits, world, C.byref(rng[0]), _p(out))
    return out[:M]


def absmax_par(x: np.ndarray, threads: int) -> np.float32:
    x = np.ascontiguousarray(x, dtype=np.float32)
    return np.float32(lib().or_absmax_par(_p(x), x.size, threads))


def qsgd_encode_par(x, norm, bits, world, rng, threads: int) -> np.ndarray:
    """qsgd_encode split over word ranges on `threads` host threads (CPU baseline)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    s = (1 << bits) - 1
    _, _, M = lane_layout(x.size, 2 * s, world)
    out = np.empty(max(M, 1), dtype=np.uint32)
    lib().or_qsgd_encode_par(_p(x), x.size, float(norm), bits, world, C.byref(rng[0]), _p(out), threads)
    return out[:M]


def qsgd_decode(words, n, norm, bits, world, alpha=1.0) -> np.ndarray:
    words = np.ascontiguousarray(words, dtype=np.uint32)
    out = np.empty(max(n, 1), dtype=np.float32)
    lib().or_qsgd_decode(_p(words), n, float(norm), bits, world, float(alpha), _p(out))
    return out[:n]


def ms_mask(x, norm, levels, rng) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    lv = np.ascontiguousarray(sorted(levels), dtype=np.uint32)
    m = np.empty(max(x.size, 1), dtype=np.uint8)
    lib().or_ms_mask(_p(x), x.size, float(norm), _p(lv), lv.size, C.byref(rng[0]), _p(m))
    return m[: x.size]


def ms_select(x, norm, levels, rng, mask) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    lv = np.ascontiguousarray(sorted(levels), dtype=np.uint32)
    mask = np.ascontiguousarray(mask, dtype=np.uint8)
    q = np.empty(max(x.size, 1), dtype=np.int32)
    lib().or_ms_select(_p(x), x.size, float(norm), _p(lv), lv.size, C.byref(rng[0]), _p(mask), _p(q))
    return q[: x.size]


def ms_dequantize(q, norm, levels, mask, order=0, alpha=1.0) -> np.ndarray:
    q = np.ascontiguousarray(q, dtype=np.int32)
    lv = np.ascontiguousarray(sorted(levels), dtype=np.uint32)
    mask = np.ascontiguousarray(mask, dtype=np.uint8)
    out = np.empty(max(q.size, 1), dtype=np.float32)
    lib().or_ms_dequantize(_p(q), q.size, float(norm), _p(lv), _p(mask), order, float(alpha), _p(out))
    return out[: q.size]


def greedy4_pack(src) -> np.ndarray:
    src = np.ascontiguousarray(src, dtype=np.int32)
    cap = src.size + 1
    out = np.empty(cap, dtype=np.int32)
    nw = lib().or_greedy4_pack(_p(src), src.size, _p(out), cap)
    if nw < 0:
        raise ValueError(f"greedy4_pack rc={nw}")
    return out[:nw]


def greedy4_unpack(words) -> np.ndarray:
    words = np.ascontiguousarray(words, dtype=np.int32)
    cap = 15 * words.size + 1
    out = np.empty(cap, dtype=np.int32)
    cnt = lib().or_greedy4_unpack(_p(words), words.size, _p(out), cap)
    if cnt < 0:
        raise ValueError(f"greedy4_unpack rc={cnt}")
    return out[:cnt]


def bytepack8(src) -> np.ndarray:
    src = np.ascontiguousarray(src, dtype=np.int64)
    nw = (src.size + 7) // 8
    out = np.empty(max(nw, 1), dtype=np.int64)
    lib().or_bytepack8(_p(src), src.size, _p(out))
    return out[:nw]


def byteunpack8(words) -> np.ndarray:
    words = np.ascontiguousarray(words, dtype=np.int64)
    out = np.empty(max(8 * words.size, 1), dtype=np.int8)
    lib().or_byteunpack8(_p(words), words.size, _p(out))
    return out[: 8 * words.size]


def gen_input(n: int, seed: int = 42, kind: int = 0, scale: float = 1e-2) -> np.ndarray:
    out = np.empty(max(n, 1), dtype=np.float32)
    lib().or_gen_input(_p(out), n, seed, kind, scale)
    return out[:n]
