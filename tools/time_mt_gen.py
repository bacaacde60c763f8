"""The torch-mode generator kernels alone, per draw format: REPS reservations
of 1e8 draws each with the speculation off (each call makes its own draws),
for a rocprofv3 kernel trace (k_mt_gen<0> plain, <3> packed24, <4>/<5> split
planes; k_mt_jump, k_mt_seq).

    rocprofv3 --kernel-trace --stats -- python tools/time_mt_gen.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))
import torch  # noqa: E402

from gcodec import codec  # noqa: E402

dev = torch.device("cuda", 0)
n = int(float(os.environ.get("N", "1e8")))
reps = int(os.environ.get("REPS", "8"))
codec.MT_SPECULATE = False
torch.manual_seed(1)
for fmt in os.environ.get("FMTS", "plain,packed24,split8,split16").split(","):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    codec.mt19937_reserve(n, dev, fmt)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        codec.mt19937_reserve(n, dev, fmt)
    e1.record()
    torch.cuda.synchronize()
    print(f"{fmt:8s} {e0.elapsed_time(e1) / reps:.3f} ms per 1e8-draw call (speculation off)", flush=True)
