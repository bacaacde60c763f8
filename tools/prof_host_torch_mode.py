"""Host-side profile (cProfile) of back-to-back torch-mode calls (1e8 fp32,
4-bit, W = 1, product defaults): where a call's host time goes, in
particular the calls that enqueue the next speculative run.

    python tools/prof_host_torch_mode.py
"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))
import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402

dev = torch.device("cuda", 0)
n = 100_000_000
x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(1)).mul_(0.01)
nm = codec.absmax(x)
lanes = codec.qsgd_layout(n, 4, 1)
words = torch.empty(lanes.plane_words, dtype=torch.int32, device=dev)
gen = gcodec.Generator(0, "torch")
fmt = os.environ.get("FMT", "plain")
torch.manual_seed(42)


def step():
    codec.absmax(x, out=nm)
    codec.qsgd_encode(x, nm, 4, gen.reserve(n, fmt=fmt), 1, out=words, lanes=lanes)


for _ in range(24):
    step()
torch.cuda.synchronize()
times = []
pr = cProfile.Profile()
for i in range(int(os.environ.get("REPS", "40"))):
    t0 = time.perf_counter()
    pr.enable()
    step()
    pr.disable()
    times.append((time.perf_counter() - t0) * 1e3)
torch.cuda.synchronize()
print("host ms per call:", " ".join(f"{t:.2f}" for t in times))
pstats.Stats(pr).sort_stats("cumulative").print_stats(30)
