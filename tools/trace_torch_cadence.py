"""Torch-mode (MT19937, reference parity) in a training cadence, for a
rocprofv3 kernel trace: CALLS iterations of (a stand-in backward: 3 bf16 GEMMs
of 8192^2, then absmax + the torch-mode encode of a 1e8 bucket), the same
loop as bench.py's torch_parity_mode.training_cadence leg.  With TIME=1 (no
profiler) it prints the added time per call against the backward alone.
tools/cadence_timeline.py turns the trace into the timeline of
profiles/<tag>_torch_cadence_timeline.txt."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))
import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402

CALLS = int(os.environ.get("CALLS", "8"))
FMT = os.environ.get("FMT", "plain")  # draw format: plain / packed24 / split8 / split16
dev = torch.device("cuda", 0)
n = 100_000_000
x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(1)).mul_(0.01)
nm = codec.absmax(x)
lanes = codec.qsgd_layout(n, 4, 1)
words = torch.empty(lanes.plane_words, dtype=torch.int32, device=dev)
gen = gcodec.Generator(0, "torch")
torch.manual_seed(42)
a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
c = torch.empty_like(a)


def backward():
    for _ in range(3):
        torch.mm(a, a, out=c)


def step():
    codec.absmax(x, out=nm)
    codec.qsgd_encode(x, nm, 4, gen.reserve(n, fmt=FMT), 1, out=words, lanes=lanes)


for _ in range(4):  # warm: jump tables, end coefficients, the speculation started
    backward()
    step()
torch.cuda.synchronize()
if os.environ.get("TIME") == "1":
    def per(fn, reps=10):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    bw = min(per(backward) for _ in range(3))
    both = min(per(lambda: (backward(), step())) for _ in range(3))
    print(f"backward {bw:.3f} ms, backward + step {both:.3f} ms, added {both - bw:.3f} ms per call; "
          f"reserve paths {codec.mt_stats()}")
else:
    codec.mt_stats(reset=True)
    paths = []
    for _ in range(CALLS):
        backward()
        step()
        st = codec.mt_stats(reset=True)
        paths.append("+".join(sorted(k for k in st if k != "fresh")) or "-")
    torch.cuda.synchronize()
    print("per call:", " | ".join(paths))
print("done")
