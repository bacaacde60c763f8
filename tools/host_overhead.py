"""Host-side cost of the Python -> C-ABI calls (GPU box): wall time per call
of the config-4 (GRandK, K = 10,000) codec calls with the GPU far ahead of
the host, plus a cProfile of the same loop.

    python tools/host_overhead.py
"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "gradient-compression_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402


def main(reps=2000):
    dev = torch.device("cuda", 0)
    n, K = 14_728_266, 10_000
    x = torch.randn(n, device=dev).mul_(0.01)
    idx = torch.randperm(n, generator=torch.Generator().manual_seed(42))[:K].to(dev)
    comp = gcodec.GlobalRandKMaxNormCompressor(dev, 4, generator=gcodec.Generator(7, "philox"))
    nrm = torch.empty(1, device=dev)
    w = comp.encode(nrm, x, 1, idx=idx)
    calls = {
        "absmax(idx)": lambda: codec.absmax(x, idx=idx, out=nrm),
        "encode(idx)": lambda: comp.encode(nrm, x, 1, idx=idx),
        "decode(idx)": lambda: comp.decode(nrm, w, K, 1, 1.0, idx=idx, out=x),
        "torch add_ (reference point)": lambda: nrm.add_(0.0),
    }
    for name, f in calls.items():
        for _ in range(50):
            f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            f()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{name:32s} host {1e6 * (t1 - t0) / reps:7.2f} us/call   host+drain {1e6 * (t2 - t0) / reps:7.2f} us/call")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(500):
        codec.absmax(x, idx=idx, out=nrm)
        comp.encode(nrm, x, 1, idx=idx)
        comp.decode(nrm, w, K, 1, 1.0, idx=idx, out=x)
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
