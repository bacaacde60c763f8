"""Config 3's TS (2,4) steps on the ResNet50 bucket as bench.py times them
(absmax -> one-pass encode -> decode at W = 1; absmax -> mask + q cache ->
select from the cache -> decode for the q-cache form), STEPS of each in a
row, for a rocprofv3 kernel trace: per kernel its duration inside the step
sequence, and the gaps between consecutive kernels (tools/ms_step_gaps.py).
With TIME=1 (no profiler) it prints each form's per-step time and host issue
time."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))
import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402

STEPS = int(os.environ.get("STEPS", "100"))
dev = torch.device("cuda", 0)
n = 23_520_842
x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(11)).mul_(0.01)
nrm = torch.empty(1, device=dev)
gen = gcodec.Generator(5, "philox")
one = gcodec.QSGDMaxNormTwoScaleCompressor(dev, 2, 4, generator=gen)
qc = gcodec.QSGDMaxNormTwoScaleCompressor(dev, 2, 4, generator=gen, q_cache=True)
out = torch.empty(n, device=dev)
mark = torch.zeros(1, device=dev)


def step_one():
    codec.absmax(x, out=nrm)
    m, w = one.encode_w1(nrm, x)
    one.decode(nrm, w, m, n, 1, 1.0, out=out)


def step_qc():
    codec.absmax(x, out=nrm)
    m = qc.encode_mask(nrm, x, 1)
    w = qc.encode(nrm, x, m, 1)
    qc.decode(nrm, w, m, n, 1, 1.0, out=out)


for _ in range(10):
    step_one()
    step_qc()
torch.cuda.synchronize()
if os.environ.get("TIME") == "1":
    for name, fn in (("one-pass", step_one), ("q cache", step_qc)):
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(STEPS):
                fn()
            host = (time.perf_counter() - t0) / STEPS * 1e6
            torch.cuda.synchronize()
            el = (time.perf_counter() - t0) / STEPS * 1e6
            print(f"{name}: {el:.1f} us per step, host issue {host:.1f} us", flush=True)
else:
    mark.neg_()
    for _ in range(STEPS):
        step_one()
    mark.neg_()
    for _ in range(STEPS):
        step_qc()
    mark.neg_()
    torch.cuda.synchronize()
print("done")
