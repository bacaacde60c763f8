"""The torch-mode encode kernel alone, per draw format (draws made once, then
the encode timed from them with HIP events): plain 32-bit draws, packed24, and
the split planes (split8 / split16), 1e8 fp32, 4-bit, W = 1, against the
Philox encode.  Kernel-level view of what the draw bytes cost.

    python tools/time_split_encode.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))
import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402

dev = torch.device("cuda", 0)
n = int(float(os.environ.get("N", "1e8")))
bits = int(os.environ.get("BITS", "4"))
x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(1)).mul_(0.01)
nm = codec.absmax(x)
lanes = codec.qsgd_layout(n, bits, 1)
words = torch.empty(lanes.plane_words, dtype=torch.int32, device=dev)
gen = gcodec.Generator(0, "torch")
torch.manual_seed(42)
codec.MT_SPECULATE = False
ref = None
for fmt in ("plain", "packed24", "split8", "split16", "philox"):
    torch.manual_seed(42)  # the same draws for every format: the words must agree
    r = gcodec.Generator(3, "philox").reserve(n) if fmt == "philox" else gen.reserve(n, fmt=fmt)
    for _ in range(3):
        codec.qsgd_encode(x, nm, bits, r, 1, out=words, lanes=lanes)
    torch.cuda.synchronize()
    if fmt == "plain":
        ref = words.clone()
    same = fmt == "philox" or torch.equal(words, ref)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 30
    e0.record()
    for _ in range(reps):
        codec.qsgd_encode(x, nm, bits, r, 1, out=words, lanes=lanes)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    draw_bytes = 0 if fmt == "philox" else codec.mt_format_bytes(n, fmt)
    print(f"{fmt:8s} encode {us:7.1f} us  draw bytes {draw_bytes / 1e6:6.0f} MB  words equal plain: {same}",
          flush=True)
