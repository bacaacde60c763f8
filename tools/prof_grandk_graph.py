"""Config 4's GRandK step (K = 10,000 of the VGG16 bucket, 4-bit, W = 1:
gather + max-norm + encode in one launch, then the decode-scatter) eager and
as a captured HIP graph, for a rocprofv3 kernel trace (VERDICT r04 item 6:
why a replay took 21.3 us against 11.7 us eager).  STEPS eager steps, then
STEPS replays, each phase bracketed by a marker kernel (a 1-element neg_) so
tools/graph_gaps.py can split the trace.  Without the profiler (TIME=1) it
also prints the per-step host issue time of both forms, and the
event-timed rate of each."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))
import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402

STEPS = int(os.environ.get("STEPS", "200"))
dev = torch.device("cuda", 0)
n4, K4 = 14_728_266, 10_000
x4 = torch.randn(n4, device=dev, generator=torch.Generator(device=dev).manual_seed(12)).mul_(0.01)
idx = torch.randperm(n4, generator=torch.Generator().manual_seed(42))[:K4].to(dev)
rk = codec.RandKStep(x4, K4, 4, gcodec.Generator(5, "philox"), 1)
mark = torch.zeros(1, device=dev)


def rk_step():
    w, _ = rk.encode(idx)
    rk.decode(w, idx, x4, 1.0)


graph = torch.cuda.CUDAGraph()
side = torch.cuda.Stream(dev)
side.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(side):
    rk_step()
torch.cuda.current_stream(dev).wait_stream(side)
with torch.cuda.graph(graph):
    rk_step()
for _ in range(20):
    rk_step()
    graph.replay()
torch.cuda.synchronize()


def timed(fn, label):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    for _ in range(STEPS):
        fn()
    e1.record()
    host = (time.perf_counter() - t0) / STEPS * 1e6
    torch.cuda.synchronize()
    print(f"{label}: {e0.elapsed_time(e1) / STEPS * 1e3:.2f} us per step on the stream, host issue "
          f"{host:.2f} us per step", flush=True)


mark.neg_()
if os.environ.get("TIME") == "1":
    timed(rk_step, "eager")
    timed(graph.replay, "graph replay")
else:
    for _ in range(STEPS):
        rk_step()
    mark.neg_()
    for _ in range(STEPS):
        graph.replay()
    mark.neg_()
torch.cuda.synchronize()
print("done")
