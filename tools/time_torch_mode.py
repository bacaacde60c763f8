"""Per-call time of the torch-parity (MT19937) encode at 1e8, 4-bit, W = 1:
the draw-buffer path (compressor / reducer default) and the fused generator
quantize, each over REPS back-to-back calls (includes the torch state hand-off)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402

REPS = 20
dev = torch.device("cuda", 0)
n = 100_000_000
x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(1)).mul_(0.01)
nm = codec.absmax(x)
lanes = codec.qsgd_layout(n, 4, 1)
words = torch.empty(lanes.plane_words, dtype=torch.int32, device=dev)
gen = gcodec.Generator(0, "torch")
torch.manual_seed(42)
for f in ("buffer", "fused", "buffer", "fused"):
    call = ((lambda: codec.qsgd_encode(x, nm, 4, gen.reserve(n), 1, out=words, lanes=lanes)) if f == "buffer"
            else (lambda: codec.qsgd_encode_torch(x, nm, 4, 1, out=words, lanes=lanes)))
    call()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(REPS):
        call()
    torch.cuda.synchronize()
    print(f"{f}: {(time.perf_counter() - t0) / REPS * 1e3:.3f} ms per call")

# generator length: the package's per-count J against the fixed default
st = torch.from_numpy(codec.mt19937_seed_state(7).view(np.int32)).to(dev)
for cnt in (10_000_000, 23_520_842 * 2, 100_000_000):
    out = torch.empty(cnt, dtype=torch.int32, device=dev)
    for J in (gcodec._lib.GC_MT_JUMP_DRAWS, codec.mt_generator_draws(cnt)):
        codec.mt19937_generate(st, cnt, out=out, J=J)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(REPS):
            codec.mt19937_generate(st, cnt, out=out, J=J)
        torch.cuda.synchronize()
        print(f"mt19937 {cnt} draws, J = {J} ({-(-cnt // J)} generators): "
              f"{(time.perf_counter() - t0) / REPS * 1e3:.3f} ms")

# the draw-buffer path with the generators on the side stream: the encode of
# call i runs under the generation of call i + 1, so the balance of jump and
# generator time moves; per-call time for a few generator counts
orig = codec.mt_generator_draws
for G in (256, 320, 383, 448, 512, 640):
    codec.mt_generator_draws = lambda c, G=G: 624 * max(1, -(-c // (624 * G)))
    call = lambda: codec.qsgd_encode(x, nm, 4, gen.reserve(n), 1, out=words, lanes=lanes)  # noqa: E731
    call()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(REPS):
        call()
    torch.cuda.synchronize()
    print(f"buffer path, {G} generators: {(time.perf_counter() - t0) / REPS * 1e3:.3f} ms per call")
codec.mt_generator_draws = orig

# speculation on / off, and what the consumer waits for (the next run's jumps
# or just this run's draws)
for spec, wj in ((True, True), (True, False), (False, False)):
    codec.MT_SPECULATE, codec.MT_WAIT_NEXT_JUMPS = spec, wj
    call = lambda: codec.qsgd_encode(x, nm, 4, gen.reserve(n), 1, out=words, lanes=lanes)  # noqa: E731
    call()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(REPS):
        call()
    torch.cuda.synchronize()
    print(f"buffer path, speculate={spec}, wait next jumps={wj}: {(time.perf_counter() - t0) / REPS * 1e3:.3f} ms per call")
codec.MT_SPECULATE, codec.MT_WAIT_NEXT_JUMPS = True, False
