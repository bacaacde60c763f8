"""Host (Python + ctypes) time of the config-3 q-cache step's calls: each
call's issue time over many steps (the GPU falls behind; the host time is
what bench.py's synchronised step loop adds when it is host-bound), then a
cProfile of the same loop.

    python tools/ms_host_profile.py
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
n = 23_520_842
x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(3)).mul_(0.01)
nrm = torch.empty(1, device=dev)
ms = gcodec.QSGDMaxNormTwoScaleCompressor(dev, 2, 4, generator=gcodec.Generator(5, "philox"), q_cache=True)
out = torch.empty(n, device=dev)


def step():
    codec.absmax(x, out=nrm)
    m = ms.encode_mask(nrm, x, 1)
    w = ms.encode(nrm, x, m, 1)
    ms.decode(nrm, w, m, n, 1, 1.0, out=out)


for _ in range(20):
    step()
torch.cuda.synchronize()
parts = {"absmax": lambda: codec.absmax(x, out=nrm)}
m = ms.encode_mask(nrm, x, 1)
w = ms.encode(nrm, x, m, 1)
parts["encode_mask"] = lambda: ms.encode_mask(nrm, x, 1)
parts["encode"] = lambda: ms.encode(nrm, x, m, 1)
parts["decode"] = lambda: ms.decode(nrm, w, m, n, 1, 1.0, out=out)
parts["step"] = step
for k, f in parts.items():
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        f()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"{k}: host {(t1 - t0) / 200 * 1e6:.1f} us per call (issue only)", flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(300):
    step()
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
