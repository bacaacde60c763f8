"""Workload for rocprofv3 counter passes over the round-2 kernels: the config-3
multi-scale kernels on the ResNet50 bucket (one-pass W = 1 encode, the two W > 1
passes, decode; the q-cache mask and cache select at W = 2 lanes), the parallel MT19937 (1e8 draws), the small-K GlobalRandK step,
the headline absmax + encode (1e8, 4-bit) and its torch-parity form
(MT19937 draws consumed by the generator kernel, then the lane pack).  Each runs `REPS` times.

Steady state: a clock settle first (SETTLE seconds of config-3 steps, as
bench.py's --settle), and every kernel name is launched at ONE size only, so a
kernel's rocprof average / spread describes one workload (k_absmax: the
ResNet50 bucket; the 1e8 headline kernels are profiled over bench.py itself,
tools/gpu.sh pmc)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402

import time  # noqa: E402

REPS = int(os.environ.get("REPS", "20"))
SETTLE = float(os.environ.get("SETTLE", "0.5"))
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(11)
n3 = 23_520_842
x3 = torch.randn(n3, device=dev, generator=g).mul_(0.01)
gen = gcodec.Generator(5, "philox")
LV = [int(v) for v in os.environ.get("LEVELS", "2,4").split(",")]  # the two-scale levels (the reference's runs: 4,8)
ms = gcodec.QSGDMaxNormTwoScaleCompressor(dev, LV[0], LV[1], generator=gen)
nrm = codec.absmax(x3)
t0 = time.perf_counter()
while time.perf_counter() - t0 < SETTLE:  # clocks ramp over ~0.1-0.3 s of sustained load
    for _ in range(20):
        codec.absmax(x3, out=nrm)
        ms.encode_w1(nrm, x3)
    torch.cuda.synchronize()
dout = torch.empty(n3, device=dev)  # the decode writes one preallocated buffer, as in bench.py
for _ in range(REPS):
    codec.absmax(x3, out=nrm)
    m, w = ms.encode_w1(nrm, x3)
    m2 = ms.encode_mask(nrm, x3, 1)
    w2 = ms.encode(nrm, x3, m2, 1)
    ms.decode(nrm, w2, m2, n3, 1, 1.0, out=dout)
# the W > 1 default (q_cache): mask pass + q cache cells, then the select from
# the cache, at W = 2 lane sizing (one rank's mask: timing only)
msc = gcodec.QSGDMaxNormTwoScaleCompressor(dev, LV[0], LV[1], generator=gen, q_cache=True)
for _ in range(REPS):
    m3 = msc.encode_mask(nrm, x3, 2)
    w3 = msc.encode(nrm, x3, m3, 2)
torch.cuda.synchronize()
del x3
if os.environ.get("MS_ONLY") == "1":  # the config-3 kernels only
    sys.exit(0)
st = torch.from_numpy(codec.mt19937_seed_state(42).view(np.int32)).to(dev)
d = torch.empty(100_000_000, dtype=torch.int32, device=dev)
for _ in range(REPS):
    codec.mt19937_generate(st, d.numel(), out=d)
torch.cuda.synchronize()
del d
n4, K4 = 14_728_266, 10_000
x4 = torch.randn(n4, device=dev, generator=g).mul_(0.01)
idx = torch.randperm(n4, generator=torch.Generator().manual_seed(42))[:K4].to(dev)
rk = codec.RandKStep(x4, K4, 4, gen, 1)
for _ in range(REPS):
    w4, nk = rk.encode(idx)
    rk.decode(w4, idx, x4, 1.0)
torch.cuda.synchronize()
del x4
n = 100_000_000
x = torch.randn(n, device=dev, generator=g).mul_(0.01)
words = torch.empty(codec.qsgd_layout(n, 4, 1).plane_words, dtype=torch.int32, device=dev)
nrm = x.abs().max().reshape(1)  # torch's reduction: k_absmax stays at one size in this profile
torch.cuda.synchronize()
torch.manual_seed(42)  # torch-parity mode: draws -> encode from the draws; and the fused form
tgen = gcodec.Generator(0, "torch")
for _ in range(REPS):
    codec.qsgd_encode(x, nrm, 4, tgen.reserve(n), 1, out=words)
for _ in range(REPS):
    codec.qsgd_encode_torch(x, nrm, 4, 1, out=words)
torch.cuda.synchronize()
print("prof workload done")
