"""Workload for a rocprofv3 kernel trace of BASELINE config 5's pipeline
(ChunkedQSGDAllReduce: 1e9 fp32, 8-bit, 8 chunks, W = 1) and of the parallel
MT19937 generator at 1e8 draws:

    rocprofv3 --kernel-trace --stats --output-format csv -d DIR -o run -- python3 tools/trace_pipeline.py

then  python tools/pipeline_overlap.py DIR  reads the trace."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402

dev = torch.device("cuda", 0)
n = 1_000_000_000
x = torch.empty(n, device=dev).normal_(0, 0.01)
out = torch.empty_like(x)
pipe = gcodec.ChunkedQSGDAllReduce(n, 8, dev, chunks=8, generator=gcodec.Generator(1, "philox"))
for _ in range(4):
    pipe(x, out)
torch.cuda.synchronize()
del x, out
st = torch.from_numpy(codec.mt19937_seed_state(42).view(np.int32)).to(dev)
d = torch.empty(100_000_000, dtype=torch.int32, device=dev)
for _ in range(5):
    codec.mt19937_generate(st, d.numel(), out=d)
torch.cuda.synchronize()
print("trace workload done")
