"""Short torch-mode workload for a rocprofv3 kernel trace: 8 back-to-back
draw-buffer encodes at 1e8 (the generation on the side stream, the encode on
the caller's stream); tools/overlap.py reads the timeline."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))
import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402

dev = torch.device("cuda", 0)
n = 100_000_000
x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(1)).mul_(0.01)
nm = codec.absmax(x)
lanes = codec.qsgd_layout(n, 4, 1)
words = torch.empty(lanes.plane_words, dtype=torch.int32, device=dev)
gen = gcodec.Generator(0, "torch")
torch.manual_seed(42)
for _ in range(8):
    codec.qsgd_encode(x, nm, 4, gen.reserve(n), 1, out=words, lanes=lanes)
torch.cuda.synchronize()
print("done")
