"""SHA-256 digests of the REFERENCE's outputs at the BASELINE.json config sizes.

Run in the build container only (needs /root/reference; the GPU box has none):

    python tests/golden/make_golden_big.py      -> tests/golden/golden_big.json

make_golden.py pins the codec at <= 3e6 elements.  This script runs the
reference's compressors.py / reducer.py (torch 2.10 CPU, torch.manual_seed(42)
before each compress, as make_golden.py does) on formula inputs of the full
config sizes and records digests only (the arrays are 0.1-1 GB each):

  config 2  QSGD-MN 4-bit, n = 1e8                  compressors.py:299-321
  config 5  QSGD-MN 8-bit, n = 1e8 (int32 q)        compressors.py:294-321
  config 3  TwoScale (2,4) and (4,8), MultiScale [2,4], n = 23,520,842
                                                     compressors.py:630-680, 778-826
  config 4  GlobalRandK K = 10,000 on the VGG16 bucket (n = 14,728,266): the
            reducer's flow at W = 1 (set_seed -> randperm(n).split(K) -> pop
            from the end -> gather -> norm -> compress -> decompress) for the
            first two pops (8,266 then 10,000 indices; the draws continue),
            and the reference GlobalRandKMaxNormReducer itself under a gloo
            group on the VGG16 tensor list for the same two steps, at W = 1
            and (round 4) W = 2, 4, 8 (rank r's gradient: gen_input seed
            42 + r, so rank 0 holds the W = 1 input)
                                                     reducer.py:697-766

    python tests/golden/make_golden_big.py --only randk_reducer_k10000_vgg16_w4,...
regenerates the named digests only and keeps the others.

Inputs are oracle.gen_input (libm-free integer formula): numpy, C and HIP
regenerate the identical x, so only digests are committed.
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REF)
sys.path.insert(0, ROOT)

import compressors  # noqa: E402  (reference)

from oracle import oracle  # noqa: E402  (only for the formula input generator)

CPU = torch.device("cpu")
SEED = 42


def sha(a) -> str:
    if isinstance(a, torch.Tensor):
        a = a.numpy()
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def vgg16_sizes():
    spec = importlib.util.spec_from_file_location("gshapes", os.path.join(ROOT, "gradient-compression_amd", "gcodec",
                                                                          "shapes.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.vgg16_sizes()


def qsgd_digest(n, kind, bits):
    x = oracle.gen_input(n, seed=SEED, kind=kind)
    t = torch.from_numpy(x)
    norm = t.abs().max()
    comp = compressors.QSGDMaxNormCompressor(CPU, bits)
    torch.manual_seed(SEED)
    q = comp.compress(norm, t)
    dec = comp.decompress(norm, q)
    return dict(n=n, kind=kind, bits=bits, norm=float(norm.item()), x=sha(x), q=sha(q), dec=sha(dec),
                q_dtype=str(q.dtype))


def ts_digest(n, lo, hi):
    x = oracle.gen_input(n, seed=SEED, kind=0)
    t = torch.from_numpy(x)
    norm = t.abs().max()
    comp = compressors.QSGDMaxNormTwoScaleCompressor(CPU, lo, hi)
    torch.manual_seed(SEED)
    q_lo = comp.compress_lower(norm, t)
    q_hi, h = comp.compress_higher(norm, t)
    q = h * q_hi + (1 - h) * q_lo  # reducer.py:1503-1505 at W = 1
    dec = comp.decompress(norm, q, h)
    return dict(n=n, kind=0, levels=[lo, hi], norm=float(norm.item()), x=sha(x), h=sha(h), q=sha(q), dec=sha(dec))


def ms_digest(n, levels):
    x = oracle.gen_input(n, seed=SEED, kind=0)
    t = torch.from_numpy(x)
    norm = t.abs().max()
    comp = compressors.QSGDMaxNormMultiScaleCompressor(CPU, list(levels))
    torch.manual_seed(SEED)
    mask = comp.compress_mask(norm, t)
    q = comp.compress(mask)
    dec = comp.decompress(norm, q, mask)
    return dict(n=n, kind=0, levels=list(levels), norm=float(norm.item()), x=sha(x), mask=sha(mask), q=sha(q),
                dec=sha(dec))


def randk_digest(n, K, bits, pops=2):
    """reducer.py:717-751 at W = 1: one set_seed, then `pops` steps."""
    x = oracle.gen_input(n, seed=SEED, kind=0)
    buf = torch.from_numpy(x)
    torch.manual_seed(SEED)
    chunks = list(torch.randperm(n).split(K))
    out = []
    for _ in range(pops):
        idx = chunks.pop()
        xk = buf[idx.numpy()]
        norm = xk.abs().max()
        comp = compressors.GlobalRandKMaxNormCompressor(CPU, bits)
        q = comp.compress(norm, xk)
        dec = comp.decompress(norm, q)
        out.append(dict(k=int(idx.numel()), idx=sha(idx.to(torch.int64)), norm=float(norm.item()), q=sha(q),
                        dec=sha(dec)))
    return dict(n=n, kind=0, K=K, bits=bits, x=sha(x), pops=out)


class _NoTimer:
    def __call__(self, *a, **k):
        import contextlib

        return contextlib.nullcontext()


def _randk_reducer_worker(rank, world, init_file, out_file, K, bits, steps):
    import torch.distributed as dist

    sys.path.insert(0, REF)
    import reducer as reducer_mod

    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    sizes = vgg16_sizes()
    n = sum(sizes)
    x = torch.from_numpy(oracle.gen_input(n, seed=SEED + rank, kind=0))
    gin = list(torch.split(x, sizes))
    red = reducer_mod.GlobalRandKMaxNormReducer(CPU, _NoTimer(), SEED, K=K, quantization_level=bits)
    res = []
    for _ in range(steps):
        gout = [torch.empty_like(g) for g in gin]
        bits_sent = red.reduce(gin, gout)
        res.append(dict(out=sha(torch.cat(gout)), bits=int(bits_sent)))
    with open(f"{out_file}.{rank}", "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


def randk_reducer_digest(K, bits, steps=2, world=1):
    import torch.multiprocessing as mp

    torch.set_num_threads(max(1, 8 // world))
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "r.json")
        mp.spawn(_randk_reducer_worker, args=(world, os.path.join(td, "init"), out, K, bits, steps), nprocs=world,
                 join=True)
        ranks = []
        for r in range(world):
            with open(f"{out}.{r}") as f:
                ranks.append(json.load(f))
    torch.set_num_threads(8)
    sizes = vgg16_sizes()
    d = dict(n=sum(sizes), tensors=len(sizes), kind=0, K=K, bits=bits, world=world, steps=ranks[0])
    if world > 1:
        d["input_seeds"] = [SEED + r for r in range(world)]
        d["ranks"] = ranks
    return d


def main():
    torch.set_num_threads(8)
    meta = {"torch": torch.__version__, "seed": SEED, "generator": "tests/golden/make_golden_big.py", "digests": {}}
    d = meta["digests"]
    jobs = [
        ("qsgd_b4_1e8_k0", lambda: qsgd_digest(100_000_000, 0, 4)),
        ("qsgd_b8_1e8_k1", lambda: qsgd_digest(100_000_000, 1, 8)),
        ("ts_2_4_resnet50", lambda: ts_digest(23_520_842, 2, 4)),
        ("ts_4_8_resnet50", lambda: ts_digest(23_520_842, 4, 8)),
        ("ms_2_4_resnet50", lambda: ms_digest(23_520_842, (2, 4))),
        ("randk_k10000_vgg16", lambda: randk_digest(14_728_266, 10_000, 4)),
        ("randk_reducer_k10000_vgg16", lambda: randk_reducer_digest(10_000, 4)),
        ("randk_reducer_k10000_vgg16_w2", lambda: randk_reducer_digest(10_000, 4, world=2)),
        ("randk_reducer_k10000_vgg16_w4", lambda: randk_reducer_digest(10_000, 4, world=4)),
        ("randk_reducer_k10000_vgg16_w8", lambda: randk_reducer_digest(10_000, 4, world=8)),
    ]
    only = None
    if "--only" in sys.argv:
        only = set(sys.argv[sys.argv.index("--only") + 1].split(","))
        with open(os.path.join(HERE, "golden_big.json")) as f:
            old = json.load(f)
        d.update(old["digests"])
    for name, fn in jobs:
        if only is not None and name not in only:
            continue
        t0 = time.time()
        d[name] = fn()
        print(f"{name}: {time.time() - t0:.1f} s", flush=True)
    with open(os.path.join(HERE, "golden_big.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("written", os.path.join(HERE, "golden_big.json"))


if __name__ == "__main__":
    main()
