"""Multi-scale encode kernels through the product entry points on the ResNet50
bucket (23,520,842 fp32, randn * 0.01), W = 1 and W = 2 lane layouts, for the
level sets of the reference's runs: per kernel the mean of REPS launches
queued behind a GPU hold (so the host's issue rate does not show).  One line
per (levels, kernel).  GC_MS_FUSED_TILES (read once per process by the
library) selects the tiles per block: run the script once per value.

    GC_MS_FUSED_TILES=2 python tools/time_ms_kernels.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))
import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402

REPS = 50
dev = torch.device("cuda", 0)
n = 23_520_842
x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(3)).mul_(0.01)
norm = codec.absmax(x)
torch.cuda.synchronize()


def hold(ms):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    torch.cuda._sleep(1_000_000)
    e.record()
    e.synchronize()
    torch.cuda._sleep(int(ms / max(s.elapsed_time(e), 1e-3) * 1e6))


def timed(fn):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        fn()
    issue_ms = (time.perf_counter() - t0) / 3 * 1e3
    torch.cuda.synchronize()
    hold(1.5 * issue_ms * REPS + 0.5)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(REPS):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / REPS * 1e3


tiles = os.environ.get("GC_MS_FUSED_TILES", "1")
for levels in ([2, 4], [4, 8], [2, 4, 6], [6, 10]):
    gen = gcodec.Generator(5, "philox")
    r = gen.reserve(n, len(levels))
    res = {}
    if codec.ms_w1_ok(x, levels):
        mw, w = codec.ms_encode_w1(x, norm, levels, r)
        res["one_pass_w1"] = timed(lambda: codec.ms_encode_w1(x, norm, levels, r, mask_out=mw, out=w))
    for world in (1, 2):
        m = codec.ms_mask_encode(x, norm, levels, r, world)
        res[f"mask_w{world}"] = timed(lambda: codec.ms_mask_encode(x, norm, levels, r, world, out=m))
        res[f"select_w{world}"] = timed(lambda: codec.ms_select_encode(x, norm, levels, r, m, world))
        cb = codec.ms_cache_bytes(n, levels)
        if cb:
            cache = torch.empty(n * cb, dtype=torch.uint8, device=dev)
            res[f"mask_cache_w{world}"] = timed(lambda: codec.ms_mask_encode(x, norm, levels, r, world, out=m,
                                                                            cache=cache))
            res[f"select_cache_w{world}"] = timed(lambda: codec.ms_select_encode(x, norm, levels, r, m, world,
                                                                                cache=cache))
    print(f"tiles={tiles} levels={levels} " + " ".join(f"{k}={v:.1f}us" for k, v in res.items()), flush=True)
