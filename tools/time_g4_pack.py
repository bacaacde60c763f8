"""Event-timed device greedy4 pack on the ResNet50 bucket's 4-bit magnitudes
and sign bits (the QSGDBP call site, 23,520,842 elements), for A/B runs of a
build switch read from the environment (e.g. GC_G4_PRIO=0 / 1 in separate
processes): per source the mean µs per pack over LOOPS loops of REPS
back-to-back launches (best loop), and a digest of the words so the forms can
be compared.
    GC_G4_PRIO=1 python tools/time_g4_pack.py"""
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))

import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402

REPS = int(os.environ.get("REPS", "100"))
LOOPS = int(os.environ.get("LOOPS", "5"))
dev = torch.device("cuda", 0)
n = 23_520_842
g = torch.Generator(device=dev).manual_seed(21)
x = torch.randn(n, device=dev, generator=g).mul_(0.01)
nm = codec.absmax(x)
gen = gcodec.Generator(7, "philox")
xi, sg = codec.qsgd_quantize_split(x, nm, 4, gen.reserve(n))
pk = codec.Greedy4Device(n, dev)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:  # clock settle
    pk.pack(xi)
    torch.cuda.synchronize()
env = {k: v for k, v in os.environ.items() if k.startswith("GC_G4")}
for name, src in (("xi", xi), ("sign", sg)):
    pk.pack(src)
    nw = pk.result()
    dig = hashlib.sha1(pk.words[:nw].cpu().numpy().tobytes()).hexdigest()[:16]
    best = []
    for _ in range(LOOPS):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(REPS):
            pk.pack(src)
        e1.record()
        torch.cuda.synchronize()
        best.append(e0.elapsed_time(e1) / REPS * 1e3)
    print(f"{env} {name}: words {nw} sha1 {dig}  us/pack best {min(best):.2f} all "
          f"{' '.join(f'{v:.2f}' for v in best)}", flush=True)
    w = pk.words[:nw].clone()
    pk.unpack(w)
    nv = pk.unpack_result()
    same = bool(nv >= n and torch.equal(pk.values[:n].to(src.dtype), src))
    best = []
    for _ in range(LOOPS):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(REPS):
            pk.unpack(w)
        e1.record()
        torch.cuda.synchronize()
        best.append(e0.elapsed_time(e1) / REPS * 1e3)
    print(f"{env} {name}: unpack round trip exact {same}  us/unpack best {min(best):.2f} all "
          f"{' '.join(f'{v:.2f}' for v in best)}", flush=True)
