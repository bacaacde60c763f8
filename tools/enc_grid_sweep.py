"""The headline step (absmax -> QSGD-MN 4-bit encode, 100M fp32), timed as
queued loops.  For the r03zk sweep (profiles/r03zk_enc_grid_sweep.log) the
library temporarily read a GC_ENC_GRID grid cap; the product keeps its fixed
12288-block grid, so this now times the product step.
    python tools/enc_grid_sweep.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402
from time_ms_kernels_core import timed  # noqa: E402

dev = torch.device("cuda", 0)
n = 100_000_000
x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(1)).mul_(0.01)
lanes = codec.qsgd_layout(n, 4, 1)
words = torch.empty(lanes.plane_words, dtype=torch.int32, device=dev)
norm = torch.empty(1, device=dev)
gen = gcodec.Generator(42, "philox")
r = gen.reserve(n)


def step():
    codec.absmax(x, out=norm)
    codec.qsgd_encode(x, norm, 4, r, 1, out=words, lanes=lanes)


for _ in range(200):
    step()
torch.cuda.synchronize()
s = timed(step)
a = timed(lambda: codec.absmax(x, out=norm))
print(f"grid cap {os.environ.get('GC_ENC_GRID', 'default')}: step {s:.1f} us, absmax {a:.1f} us, "
      f"encode in step {s - a:.1f} us", flush=True)
