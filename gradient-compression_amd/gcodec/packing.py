"""Drop-ins for the reference's three packing extensions
(extensions/*/setup.py:10-14 build modules `bitpacking`, `gpu_bitpacking`,
`bytepacking`, each exporting packing(Tensor) -> Tensor and
unpacking(Tensor) -> Tensor; pybind11 defs at bitpacking.cpp:127-131,
gpu_bitpacking.cpp:128-132, bytepacking.cpp:67-71).

    from gcodec.packing import bitpacking, gpu_bitpacking, bytepacking

Same formats and outputs on [0, 255] (greedy 4-mode) / any ints (bytes).
Where the reference loops forever (a value >= 256) or silently corrupts the
mode tag (negatives), these raise GCodecError(GC_ERANGE).
"""
from __future__ import annotations

import ctypes as C
import types

import numpy as np
import torch

from . import _lib
from . import codec as _codec
from ._lib import check


def _np(t: torch.Tensor, dtype) -> np.ndarray:
    return np.ascontiguousarray(t.detach().cpu().numpy().astype(dtype, copy=False)).reshape(-1)


def _bp_pack(src: torch.Tensor) -> torch.Tensor:
    if src.is_cuda:
        return _codec.bytepack8(src)
    a = _np(src, np.int64)
    out = np.empty(max((a.size + 7) // 8, 1), dtype=np.int64)
    check(_lib.load().gc_bytepack8_host(a.ctypes.data_as(C.c_void_p), a.size, out.ctypes.data_as(C.c_void_p)),
          "gc_bytepack8_host")
    return torch.from_numpy(out[:(a.size + 7) // 8].copy())


def _bp_unpack(src: torch.Tensor) -> torch.Tensor:
    if src.is_cuda:
        return _codec.byteunpack8(src)
    a = _np(src, np.int64)
    out = np.empty(max(8 * a.size, 1), dtype=np.int8)
    check(_lib.load().gc_byteunpack8_host(a.ctypes.data_as(C.c_void_p), a.size, out.ctypes.data_as(C.c_void_p)),
          "gc_byteunpack8_host")
    return torch.from_numpy(out[:8 * a.size].copy())


bitpacking = types.SimpleNamespace(packing=_codec.greedy4_pack, unpacking=_codec.greedy4_unpack)
gpu_bitpacking = types.SimpleNamespace(packing=_codec.greedy4_pack, unpacking=_codec.greedy4_unpack)
bytepacking = types.SimpleNamespace(packing=_bp_pack, unpacking=_bp_unpack)
