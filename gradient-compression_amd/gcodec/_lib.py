"""ctypes binding of libgcodec.so (include/gcodec.h).

The product path has exactly one implementation: the HIP kernels in
gradient-compression_amd/csrc.  If the library is missing or no gfx950 device
is visible, every codec call raises GCodecError — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("GCODEC_LIB", os.path.join(PKG_ROOT, "lib", "libgcodec.so"))

GC_OK = 0
GC_EINVAL = -1
GC_EHIP = -2
GC_ERANGE = -3
GC_ENOSPC = -4
GC_ENODEV = -5

GC_I8, GC_I32, GC_I64 = 1, 4, 8
GC_RNG_PHILOX, GC_RNG_STREAM, GC_RNG_STREAM24 = 0, 1, 2
GC_RNG_SPLIT8, GC_RNG_SPLIT16 = 3, 4  # split-plane draws (include/gcodec.h)
GC_MAX_LEVELS = 8
GC_MT_JUMP_DRAWS = 262080  # include/gcodec.h: draws per generator of the parallel MT19937 stream


class GCodecError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"gcodec error {code}: {msg}")
        self.code = code


class gc_rng(C.Structure):
    _fields_ = [
        ("kind", C.c_uint32),
        ("reserved", C.c_uint32),
        ("seed", C.c_uint64),
        ("offset", C.c_uint64),
        ("stream", C.c_void_p),
    ]


class gc_lanes(C.Structure):
    _fields_ = [
        ("n", C.c_uint64),
        ("plane_words", C.c_uint64),
        ("bits", C.c_uint32),
        ("per_word", C.c_uint32),
        ("offset", C.c_uint32),
        ("world", C.c_uint32),
        ("range", C.c_uint64),
    ]

    def __repr__(self):
        return (f"gc_lanes(n={self.n}, M={self.plane_words}, w={self.bits}, L={self.per_word}, "
                f"offset={self.offset}, world={self.world}, range={self.range})")


class gc_levels(C.Structure):
    _fields_ = [("count", C.c_uint32), ("bits", C.c_uint32 * GC_MAX_LEVELS)]


class gc_seg(C.Structure):
    _fields_ = [("start", C.c_uint64), ("end", C.c_uint64), ("ptr", C.c_void_p), ("reserved", C.c_uint64)]


class gc_segments(C.Structure):
    _fields_ = [
        ("count", C.c_uint64),
        ("n", C.c_uint64),
        ("seg", C.c_void_p),
        ("chunk_seg", C.c_void_p),
        ("chunk_shift", C.c_uint32),
        ("sizes_hash", C.c_uint32),
    ]


P = C.c_void_p
u64, u32, i32, f32, i64 = C.c_uint64, C.c_uint32, C.c_int32, C.c_float, C.c_int64
RNGP, LANESP, LEVP = C.POINTER(gc_rng), C.POINTER(gc_lanes), C.POINTER(gc_levels)
SEGSP = C.POINTER(gc_segments)

# name -> (restype, argtypes); must match include/gcodec.h exactly
SIGNATURES = {
    "gc_version": (C.c_char_p, []),
    "gc_last_error": (C.c_char_p, []),
    "gc_abi_version": (C.c_int, []),
    "gc_device_check": (C.c_int, [C.c_int]),
    "gc_lane_layout": (C.c_int, [u64, u64, u32, u32, LANESP]),
    "gc_qsgd_layout": (C.c_int, [u64, u32, u32, LANESP]),
    "gc_ms_layout": (C.c_int, [u64, LEVP, u32, LANESP]),
    "gc_ms_mask_layout": (C.c_int, [u64, LEVP, u32, LANESP]),
    "gc_absmax_workspace_size": (C.c_size_t, []),
    "gc_absmax_f32": (C.c_int, [P, P, u64, P, P, P]),
    "gc_qsgd_encode": (C.c_int, [P, P, u64, P, u32, LANESP, RNGP, P, P]),
    "gc_qsgd_decode": (C.c_int, [P, P, u64, P, u32, LANESP, f32, P, P]),
    "gc_qsgd_quantize": (C.c_int, [P, u64, P, u32, RNGP, u32, P, u32, P]),
    "gc_qsgd_quantize_le": (C.c_int, [P, u64, P, u32, RNGP, u32, P, u32, P, u32, P]),
    "gc_qsgd_dequantize": (C.c_int, [P, u32, u64, P, u32, f32, P, P]),
    "gc_qsgd_quantize_split": (C.c_int, [P, u64, P, u32, RNGP, P, P, P]),
    "gc_lane_pack": (C.c_int, [P, u32, LANESP, P, P]),
    "gc_lane_unpack": (C.c_int, [P, LANESP, P, P]),
    "gc_segments_chunks": (u64, [u64, u32]),
    "gc_segments_sizes_hash": (u32, [P, u64]),
    "gc_segments_plan": (C.c_int, [P, P, u64, u32, P, P, u64, P]),
    "gc_segments_flatten_absmax": (C.c_int, [SEGSP, P, P, P, P]),
    "gc_segments_scatter": (C.c_int, [P, f32, SEGSP, P]),
    "gc_segments_copy": (C.c_int, [SEGSP, SEGSP, f32, P]),
    "gc_qsgd_decode_scatter_segments": (C.c_int, [P, P, u64, P, u32, LANESP, f32, SEGSP, P]),
    "gc_qsgd_decode_segments": (C.c_int, [P, u64, P, u32, LANESP, f32, SEGSP, P]),
    "gc_ms_mask_encode": (C.c_int, [P, P, u64, P, LEVP, RNGP, LANESP, P, P]),
    "gc_ms_select_encode": (C.c_int, [P, P, u64, P, LEVP, RNGP, P, LANESP, LANESP, P, P]),
    "gc_ms_encode_w1": (C.c_int, [P, u64, P, LEVP, RNGP, LANESP, LANESP, P, P, P]),
    "gc_ms_cache_bytes": (C.c_int, [u64, LEVP, P]),
    "gc_ms_mask_encode_cached": (C.c_int, [P, u64, P, LEVP, RNGP, LANESP, P, P, P]),
    "gc_ms_select_cached": (C.c_int, [P, u64, LEVP, P, LANESP, LANESP, P, P]),
    "gc_ms_decode": (C.c_int, [P, P, P, u64, P, LEVP, LANESP, LANESP, C.c_int, f32, P, P]),
    "gc_ms_decode_segments": (C.c_int, [P, P, u64, P, LEVP, LANESP, LANESP, C.c_int, f32, SEGSP, P]),
    "gc_ms_decode_scatter_segments": (C.c_int, [P, P, P, u64, P, LEVP, LANESP, LANESP, C.c_int, f32, SEGSP, P]),
    "gc_ms_mask_unpack": (C.c_int, [P, LANESP, u32, P, P]),
    "gc_ms_quantize_mask": (C.c_int, [P, u64, P, LEVP, RNGP, P, P]),
    "gc_ms_select_quantize": (C.c_int, [P, u64, P, LEVP, RNGP, P, P, u32, P]),
    "gc_ms_dequantize": (C.c_int, [P, u32, P, u64, P, LEVP, C.c_int, f32, P, P]),
    "gc_mt19937_seed": (C.c_int, [u64, P]),
    "gc_mt19937_generate": (C.c_int, [P, P, u64, P]),
    "gc_mt19937_jump_table": (C.c_int, [u64, u64, P]),
    "gc_mt19937_workspace_size": (C.c_size_t, [u64]),
    "gc_mt19937_generate_jumped": (C.c_int, [P, P, u64, P, u64, P, P]),
    "gc_qsgd_quantize_mt19937": (C.c_int, [P, u64, P, u32, P, P, u64, u64, P, u32, P, P]),
    "gc_mt19937_jump_table_j": (C.c_int, [u64, u64, u64, P]),
    "gc_mt19937_workspace_size_j": (C.c_size_t, [u64, u64]),
    "gc_mt19937_generate_jumped_j": (C.c_int, [P, P, u64, u64, P, u64, P, P]),
    "gc_mt19937_generate_phase_j": (C.c_int, [P, P, u64, u64, P, u64, P, C.c_int, P]),
    "gc_mt19937_generate_split_j": (C.c_int, [P, P, u64, u64, P, u64, P, u64, P, C.c_int, P]),
    "gc_mt19937_generate_split24_j": (C.c_int, [P, P, u64, u64, P, u64, P, u64, u64, P, C.c_int, P]),
    "gc_mt19937_workspace_size_multi_j": (C.c_size_t, [u64, u64, u32]),
    "gc_mt19937_generate_multi_j": (C.c_int, [P, P, u64, u64, P, u32, u64, P, P, P, C.c_int, P]),
    "gc_mt19937_generate_multi24_j": (C.c_int, [P, P, u64, u64, P, u32, u64, u64, P, P, P, C.c_int, P]),
    "gc_rng_split_bytes": (u64, [u64, u32]),
    "gc_mt19937_generate_multi_split_j": (C.c_int, [P, P, u64, u64, P, u32, u64, u64, u32, P, P, u32, u32, u64, u64,
                                                    P, C.c_int, P]),
    "gc_qsgdbp_decode": (C.c_int, [P, P, u64, P, P, P]),
    "gc_randk_workspace_size": (C.c_size_t, []),
    "gc_randk_gather_absmax": (C.c_int, [P, P, u64, P, P, P, P]),
    "gc_randk_encode_w1": (C.c_int, [P, P, u64, P, P, u32, LANESP, RNGP, P, P, P]),
    "gc_randk_gather_absmax_segments": (C.c_int, [SEGSP, P, u64, P, P, P, P]),
    "gc_randk_encode_w1_segments": (C.c_int, [SEGSP, P, u64, P, P, u32, LANESP, RNGP, P, P, P]),
    "gc_greedy4_pack": (i64, [P, u64, P, u64]),
    "gc_greedy4_unpack": (i64, [P, u64, P, u64]),
    "gc_greedy4_workspace_size": (C.c_size_t, [u64]),
    "gc_greedy4_pack_device": (C.c_int, [P, u64, P, u64, P, P, P, P]),
    "gc_greedy4_unpack_workspace_size": (C.c_size_t, [u64]),
    "gc_greedy4_unpack_device": (C.c_int, [P, u64, P, u64, P, P, P, P]),
    "gc_bytepack8": (C.c_int, [P, u32, u64, P, P]),
    "gc_byteunpack8": (C.c_int, [P, u64, P, P]),
    "gc_bytepack8_host": (C.c_int, [P, u64, P]),
    "gc_byteunpack8_host": (C.c_int, [P, u64, P]),
}

_lock = threading.Lock()
_lib = None
_device_ok = {}


def load():
    """Load libgcodec.so (raises GCodecError if it is absent)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise GCodecError(GC_ENODEV, f"libgcodec.so not built ({LIB_PATH}); run "
                                      "`python -c 'import __graft_entry__ as g; g.build()'`")
                lib = C.CDLL(LIB_PATH)
                for name, (res, args) in SIGNATURES.items():
                    fn = getattr(lib, name)
                    fn.restype = res
                    fn.argtypes = args
                _lib = lib
    return _lib


def last_error() -> str:
    return load().gc_last_error().decode()


def check(rc: int, what: str = ""):
    if rc < 0:
        raise GCodecError(rc, f"{what}: {last_error()}")
    return rc


def require_device(device_index: int):
    """The HIP path is the only path: refuse to run without a gfx950 GPU."""
    ok = _device_ok.get(device_index)
    if ok is None:
        rc = load().gc_device_check(device_index)
        ok = rc == GC_OK
        _device_ok[device_index] = ok
        if not ok:
            raise GCodecError(rc, last_error())
    return ok
