"""Occupancy-round sweep of the multi-scale kernels: the one-pass W = 1 encode
and the cached mask (W = 2 lanes) for levels [2, 4] at bucket sizes that fill
a fraction f of one round of resident blocks (f = 1: 2304 three-wave blocks =
9 per CU at 7 waves per SIMD), plus the ResNet50 bucket (1.25 rounds).  A
kernel whose time per element rises between f = 1 and f = 1.25 and falls
back at f = 2 loses time to the partial last round (the tail).

    python tools/ms_size_sweep.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402

dev = torch.device("cuda", 0)
ROUND = 2304 * 64 * 4 * 32  # elements that fill one round of one-pass blocks: 18,874,368
sizes = [int(ROUND * f) for f in (0.5, 0.75, 1.0, 1.125, 1.25, 1.5, 1.75, 2.0, 3.0)] + [23_520_842]
xall = torch.randn(max(sizes), device=dev, generator=torch.Generator(device=dev).manual_seed(3)).mul_(0.01)
levels = [2, 4]

from time_ms_kernels_core import timed  # noqa: E402

for n in sizes:
    x = xall[:n]
    norm = codec.absmax(x)
    gen = gcodec.Generator(5, "philox")
    r = gen.reserve(n, len(levels))
    mw, w = codec.ms_encode_w1(x, norm, levels, r)
    t1 = timed(lambda: codec.ms_encode_w1(x, norm, levels, r, mask_out=mw, out=w))
    m = codec.ms_mask_encode(x, norm, levels, r, 2)
    cache = torch.empty(n * codec.ms_cache_bytes(n, levels), dtype=torch.uint8, device=dev)
    t2 = timed(lambda: codec.ms_mask_encode(x, norm, levels, r, 2, out=m, cache=cache))
    tn = timed(lambda: codec.absmax(x, out=norm))
    print(f"n={n:>11,d} rounds={n / ROUND:5.3f} one_pass={t1:7.1f}us ({t1 * 1e3 / n:.3f} ns/el) "
          f"mask_cache_w2={t2:7.1f}us ({t2 * 1e3 / n:.3f} ns/el) absmax={tn:6.1f}us ({tn * 1e3 / n:.3f} ns/el)",
          flush=True)
