"""Workload for rocprofv3 over the drop-in packers on the ResNet50 bucket
(23,520,842 elements, the QSGDBP call site's 4-bit magnitudes and sign bits):
device greedy 4-mode pack / unpack and byte pack / unpack, REPS launches each
after a short clock settle (tools/gpu.sh cmd: rocprofv3 --kernel-trace --stats)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))

import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402

REPS = int(os.environ.get("REPS", "20"))
SRCS = os.environ.get("PACK_SRC", "both")  # xi | sign | both
dev = torch.device("cuda", 0)
n = 23_520_842
g = torch.Generator(device=dev).manual_seed(21)
x = torch.randn(n, device=dev, generator=g).mul_(0.01)
nm = codec.absmax(x)
gen = gcodec.Generator(7, "philox")
xi, sg = codec.qsgd_quantize_split(x, nm, 4, gen.reserve(n))
q8 = codec.qsgd_quantize(x, nm, 4, gen.reserve(n))
pk = codec.Greedy4Device(n, dev)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:  # clock settle
    pk.pack(xi)
    torch.cuda.synchronize()
for src in {"xi": (xi,), "sign": (sg,)}.get(SRCS, (xi, sg)):
    pk.pack(src)
    w = pk.words[:pk.result()].clone()
    print("words", w.numel())
    for _ in range(REPS):
        pk.pack(src)
    for _ in range(REPS):
        pk.unpack(w)
    torch.cuda.synchronize()
bw = codec.bytepack8(q8)
for _ in range(REPS):
    codec.bytepack8(q8)
    codec.byteunpack8(bw)
torch.cuda.synchronize()
print("done")
