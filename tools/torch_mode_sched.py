"""Torch-mode (reference-bit-exact MT19937) encode at 1e8: per-call time of
back-to-back calls under different stream priorities for the two side
streams (jumps, generators) and the caller's stream.  Measurement only: the
product keeps both side streams at the highest priority unless this shows a
better choice.

    python tools/torch_mode_sched.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))
import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402

REPS = 30
dev = torch.device("cuda", 0)
n = 100_000_000
x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(1)).mul_(0.01)
nm = codec.absmax(x)
lanes = codec.qsgd_layout(n, 4, 1)
words = torch.empty(lanes.plane_words, dtype=torch.int32, device=dev)
gen = gcodec.Generator(0, "torch")
torch.manual_seed(42)
lo, hi = torch.cuda.Stream.priority_range()
HIGH, NORM = min(lo, hi), max(lo, hi)


def per_call(caller=None):
    call = lambda: codec.qsgd_encode(x, nm, 4, gen.reserve(n), 1, out=words, lanes=lanes)  # noqa: E731
    ctx = torch.cuda.stream(caller) if caller is not None else torch.cuda.stream(torch.cuda.current_stream(dev))
    with ctx:
        for _ in range(3):
            call()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(REPS):
            call()
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / REPS * 1e3


for js_p, gs_p, cs_p in ((HIGH, HIGH, None), (HIGH, NORM, None), (NORM, HIGH, None), (NORM, NORM, None),
                         (HIGH, HIGH, HIGH), (NORM, HIGH, HIGH), (HIGH, NORM, HIGH)):
    torch.cuda.synchronize()
    codec._MT_SIDE[dev.index] = (torch.cuda.Stream(dev, priority=js_p),
                                 [torch.cuda.Stream(dev, priority=gs_p) for _ in range(codec.MT_MAX_SLOTS)])
    codec._MT_SPEC.pop(dev.index, None)
    codec._MT_LAST.pop(dev.index, None)  # the dropped run moved the device state: send torch's again
    caller = torch.cuda.Stream(dev, priority=cs_p) if cs_p is not None else None
    name = lambda p: "high" if p == HIGH else "normal"  # noqa: E731
    print(f"jumps {name(js_p)}, generators {name(gs_p)}, caller {name(cs_p) if cs_p is not None else 'default'}: "
          f"{per_call(caller):.3f} ms per call", flush=True)
