"""Config 4 (GlobalRandK K=10000 of a 14.7M bucket, 4-bit, W=1) step loop for
rocprofv3 --kernel-trace --stats: the kernels' own durations, separate from
the host issue time that bench.py's back-to-back event timing includes.

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rk -o run -- python3 tools/prof_grandk.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "gradient-compression_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402


def main(steps=500):
    dev = torch.device("cuda", 0)
    n, K = 14_728_266, 10_000
    x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(12)).mul_(0.01)
    idx = torch.randperm(n, generator=torch.Generator().manual_seed(42))[:K].to(dev)
    comp = gcodec.GlobalRandKMaxNormCompressor(dev, 4, generator=gcodec.Generator(7, "philox"))
    nrm = torch.empty(1, device=dev)
    for _ in range(steps):
        codec.absmax(x, idx=idx, out=nrm)
        w = comp.encode(nrm, x, 1, idx=idx)
        comp.decode(nrm, w, K, 1, 1.0, idx=idx, out=x)
    torch.cuda.synchronize()
    print("done", steps)


if __name__ == "__main__":
    main()
