"""Per-call time of the torch-parity (MT19937) encode at 1e8, 4-bit, W = 1,
back to back (REPS calls, the fastest of RUNS loops; includes the torch state
hand-off), swept over the pipelined run's generator count and the
speculation depth (codec.MT_PIPE_GENERATORS / MT_SPECULATE_DEPTH), encode
only and absmax + encode; then the Philox step in the same harness, and the
fused generator-quantize path for contrast.

    python tools/time_torch_mode.py [G,G,...] [D,D,...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))
import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402

REPS, RUNS = 20, 3
dev = torch.device("cuda", 0)
n = 100_000_000
x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(1)).mul_(0.01)
nm = codec.absmax(x)
lanes = codec.qsgd_layout(n, 4, 1)
words = torch.empty(lanes.plane_words, dtype=torch.int32, device=dev)
gen = gcodec.Generator(0, "torch")
px = gcodec.Generator(5, "philox")
torch.manual_seed(42)
GS = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 96, 128, 192, 256, 383]
DS = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 3]


CADENCE = os.environ.get("CADENCE", "0") == "1"  # each call behind ~2.4 ms of bf16 GEMMs (a backward)
if CADENCE:
    _a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    _c = torch.empty_like(_a)


def backward():
    for _ in range(3):
        torch.mm(_a, _a, out=_c)


def per_call(fn):
    if CADENCE:  # the time a call adds to a backward
        return _per_call(lambda: (backward(), fn())) - _per_call(backward)
    return _per_call(fn)


def _per_call(fn):
    for _ in range(6):
        fn()
    torch.cuda.synchronize()
    best = []
    for _ in range(RUNS):
        t0 = time.perf_counter()
        for _ in range(REPS):
            fn()
        torch.cuda.synchronize()
        best.append((time.perf_counter() - t0) / REPS * 1e3)
    return min(best)


FMT = os.environ.get("FMT", "plain")  # draw format: plain / packed24 / split8 / split16
if os.environ.get("BUDGET"):  # speculation budget in bytes (codec.MT_SPECULATE_BUDGET)
    codec.MT_SPECULATE_BUDGET = int(float(os.environ["BUDGET"]))
PACKED = FMT == "packed24"


def enc():
    codec.qsgd_encode(x, nm, 4, gen.reserve(n, fmt=FMT), 1, out=words, lanes=lanes)


def step():
    codec.absmax(x, out=nm)
    enc()


if os.environ.get("AB_FMTS"):  # interleaved A/B of draw formats, e.g. AB_FMTS=plain,split8,split16
    for rep in range(int(os.environ.get("AB_REPS", "3"))):
        for f in os.environ["AB_FMTS"].split(","):
            FMT = f
            codec.mt_release()
            e, s_ = per_call(enc), per_call(step)
            held = codec.mt_reserved_bytes(dev) if hasattr(codec, "mt_reserved_bytes") else -1
            plan = codec._mt_plan(n, f, True) if hasattr(codec, "_mt_plan") else None
            print(f"AB rep {rep} fmt={f}{' cadence' if CADENCE else ''} budget {codec.MT_SPECULATE_BUDGET} "
                  f"(calls/run, depth) {plan}: encode {e:.3f} ms, absmax + encode "
                  f"{s_:.3f} ms per call, held {held / 1e9:.2f} GB", flush=True)
    sys.exit(0)

if os.environ.get("AB") == "1":  # interleaved A/B of the packed and plain draws, the product's G and depth
    codec.mt_release()
    for rep in range(4):
        for packed in (True, False):
            FMT = "packed24" if packed else "plain"
            codec.mt_release()
            print(f"AB rep {rep} packed24={packed}: encode {per_call(enc):.3f} ms, absmax + encode "
                  f"{per_call(step):.3f} ms per call", flush=True)
    sys.exit(0)

MS = [int(v) for v in os.environ.get("MULTI", str(codec.MT_MULTI_CALLS)).split(",")]
if os.environ.get("PRIO"):  # side-stream priorities, e.g. PRIO=high,normal (jumps, generators)
    codec.MT_SIDE_PRIORITY = tuple(os.environ["PRIO"].split(","))
for G in GS:
    for D in DS:
        for M in MS:
            codec.MT_PIPE_GENERATORS = G or None
            codec.MT_SPECULATE_DEPTH = D
            codec.MT_MULTI_CALLS = M
            codec.mt_release()
            e, s = per_call(enc), per_call(step)
            print(f"generators {G or codec.mt_pipe_generators(n * M, M > 1)} depth {D} calls/run {M}"
                  f"{' cadence' if CADENCE else ''}{' packed24' if PACKED else ''}"
                  f"{' prio ' + ','.join(codec.MT_SIDE_PRIORITY) if os.environ.get('PRIO') else ''}: encode {e:.3f} ms, "
                  f"absmax + encode {s:.3f} ms per call", flush=True)
if os.environ.get("SWEEP_ONLY") == "1":
    sys.exit(0)
codec.MT_PIPE_GENERATORS, codec.MT_SPECULATE_DEPTH = None, 2
codec.mt_release()
pe = per_call(lambda: codec.qsgd_encode(x, nm, 4, px.reserve(n), 1, out=words, lanes=lanes))


def pstep():
    codec.absmax(x, out=nm)
    codec.qsgd_encode(x, nm, 4, px.reserve(n), 1, out=words, lanes=lanes)


print(f"philox: encode {pe:.3f} ms, absmax + encode {per_call(pstep):.3f} ms per call", flush=True)
print(f"fused generator-quantize: {per_call(lambda: codec.qsgd_encode_torch(x, nm, 4, 1, out=words, lanes=lanes)):.3f}"
      " ms per call", flush=True)
