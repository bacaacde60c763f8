"""Generate the committed golden fixtures by running the REFERENCE itself.

Run in the build container only (needs /root/reference, which does not exist
on the GPU box):  python tests/golden/make_golden.py
                  python tests/golden/make_golden.py --reducer-worlds 4,8
(the second form writes only reducers_w4.npz / reducers_w8.npz: the six
hot-path reducers under gloo at W = 4 and 8)

It imports the reference's compressors.py / reducer.py on CPU (torch 2.10 CPU,
the reference pins 1.7.1) and records inputs and outputs.  The fixtures are
data only (npz without pickles + a JSON of digests); no reference source is
copied.  The greedy-4 / byte-pack vectors come from the reference's own C++
extensions compiled from their sources by oracle/build_ref.py into
oracle/_ref/ (skipped when that build is unavailable).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import tempfile

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


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def edge_input(n: int, seed: int) -> np.ndarray:
    """Gaussian-ish values plus the edge values the reference's arithmetic
    hits: zeros, -0.0, +/-max, exact level boundaries, subnormals."""
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(n, generator=g) * 1e-2).numpy().astype(np.float32)
    norm = np.float32(np.abs(x).max())
    specials = [0.0, -0.0, norm, -norm, norm / 2, -norm / 3, 1e-40, -1e-42, 1e-30, norm * 0.999999]
    for b in (2, 4, 8):
        s = (1 << b) - 1
        specials += [norm * k / s for k in (1, 2, s - 1)]
    sp = np.array(specials, dtype=np.float32)
    if n >= sp.size:
        x[np.linspace(0, n - 1, sp.size).astype(np.int64)] = sp
    elif n > 1:
        x[-1] = -0.0  # keep a nonzero max so the reference does not raise
    return x


def qsgd_case(x: np.ndarray, bits: int, cls=compressors.QSGDMaxNormCompressor):
    t = torch.from_numpy(x.copy())
    norm = t.abs().max()
    comp = cls(CPU, bits)
    torch.manual_seed(SEED)
    q = comp.compress(norm, t)
    dec = comp.decompress(norm, q)
    return dict(
        x=x,
        norm=np.float32(norm.item()),
        q=q.numpy(),
        dec=dec.numpy().astype(np.float32),
        bits=np.int32(bits),
        seed=np.int64(SEED),
    )


def ts_case(x: np.ndarray, lo: int, hi: int):
    t = torch.from_numpy(x.copy())
    norm = t.abs().max()
    comp = compressors.QSGDMaxNormTwoScaleCompressor(CPU, lo, hi)
    torch.manual_seed(SEED)
    q_lo = comp.compress_lower(norm, t)
    q_hi, h = comp.compress_higher(norm, t)
    # reducer.py:1503-1505 at W=1 (no mask all-reduce)
    q = h * q_hi + (1 - h) * q_lo
    dec = comp.decompress(norm, q, h)
    return dict(
        x=x, norm=np.float32(norm.item()), q_lo=q_lo.numpy(), q_hi=q_hi.numpy(), h=h.numpy(),
        q=q.numpy(), dec=dec.numpy().astype(np.float32), levels=np.array([lo, hi], np.int32),
        seed=np.int64(SEED),
    )


def ms_case(x: np.ndarray, levels):
    t = torch.from_numpy(x.copy())
    norm = t.abs().max()
    comp = compressors.QSGDMaxNormMultiScaleCompressor(CPU, list(levels))
    torch.manual_seed(SEED)
    mask = comp.compress_mask(norm, t)
    q = comp.compress(mask)
    dec = comp.decompress(norm, q, mask)
    return dict(
        x=x, norm=np.float32(norm.item()), mask=mask.numpy(), q=q.numpy(),
        dec=dec.numpy().astype(np.float32), levels=np.array(sorted(levels), np.int32),
        seed=np.int64(SEED),
    )


def randk_case(n: int, K: int, bits: int, data_seed: int):
    """Follows GlobalRandKMaxNormReducer.reduce (reducer.py:710-751) at W=1
    for the first popped chunk: set_seed -> randperm(n).split(K) -> pop()
    -> gather -> norm -> compress (draws continue after randperm's)."""
    g = torch.Generator().manual_seed(data_seed)
    buf = torch.randn(n, generator=g) * 1e-2
    torch.manual_seed(SEED)
    chunks = list(torch.randperm(n).split(K))
    idx = chunks.pop().numpy()
    xk = buf[idx]
    norm = xk.abs().max()
    comp = compressors.GlobalRandKMaxNormCompressor(CPU, bits)
    q = comp.compress(norm, xk)
    dec = comp.decompress(norm, q)
    perm_head = torch.cat(chunks[:2]).numpy() if len(chunks) >= 2 else np.zeros(0, np.int64)
    return dict(
        buf=buf.numpy(), idx=idx.astype(np.int64), norm=np.float32(norm.item()), q=q.numpy(),
        dec=dec.numpy().astype(np.float32), bits=np.int32(bits), K=np.int64(K), seed=np.int64(SEED),
        perm_head=perm_head.astype(np.int64), draws_before=np.int64(n - 1),
    )


# --------------------------------------------------------------------------
# Reducers under gloo (W = 1, 2), reducer.py:498-554, 697-766, 1454-1715
# --------------------------------------------------------------------------
SHAPES = [(16, 3, 3, 3), (16,), (10, 16), (10,), (7, 5)]


class _NoTimer:
    def __call__(self, *a, **k):
        import contextlib

        return contextlib.nullcontext()


def _make_reducer(name, reducer_mod):
    t = _NoTimer()
    if name == "qsgd":
        return reducer_mod.QSGDMaxNormReducer(CPU, t, quantization_level=4)
    if name == "ts":
        return reducer_mod.QSGDMaxNormTwoScaleReducer(CPU, t, 2, 4)
    if name == "ms":
        return reducer_mod.QSGDMaxNormMultiScaleReducer(CPU, t, [2, 4])
    if name == "ms3":
        return reducer_mod.QSGDMaxNormMultiScaleReducer(CPU, t, [2, 4, 6])
    if name == "randk":
        return reducer_mod.GlobalRandKMaxNormReducer(CPU, t, SEED, K=100, quantization_level=4)
    if name == "randk_ts":
        return reducer_mod.GlobalRandKMaxNormTwoScaleReducer(CPU, t, SEED, K=100,
                                                             lower_quantization_level=2,
                                                             higher_quantization_level=4)
    raise KeyError(name)


REDUCERS = ["qsgd", "ts", "ms", "ms3", "randk", "randk_ts"]
STEPS = 2


def _grads(rank: int, step: int):
    g = torch.Generator().manual_seed(1000 * step + 17 * rank + 5)
    return [torch.randn(s, generator=g) * (0.01 * (1 + rank)) for s in SHAPES]


def _reducer_worker(rank, world, init_file, out_dir):
    import torch.distributed as dist

    sys.path.insert(0, REF)
    import reducer as reducer_mod

    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    res = {}
    for name in REDUCERS:
        red = _make_reducer(name, reducer_mod)
        torch.manual_seed(SEED + rank)  # model_dispatcher.py:59 per-rank stream
        for step in range(STEPS):
            gin = _grads(rank, step)
            gout = [torch.empty_like(g) for g in gin]
            bits = red.reduce(gin, gout)
            for i, g in enumerate(gin):
                res[f"{name}/s{step}/in{i}"] = g.numpy()
            for i, g in enumerate(gout):
                res[f"{name}/s{step}/out{i}"] = g.numpy()
            res[f"{name}/s{step}/bits"] = np.int64(bits)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


def reducer_fixtures(world: int):
    import torch.multiprocessing as mp

    with tempfile.TemporaryDirectory() as td:
        init_file = os.path.join(td, "init")
        mp.spawn(_reducer_worker, args=(world, init_file, td), nprocs=world, join=True)
        out = {}
        for r in range(world):
            with np.load(os.path.join(td, f"r{r}.npz")) as z:
                for k in z.files:
                    out[f"r{r}/{k}"] = z[k]
    out["world"] = np.int64(world)
    out["shapes"] = np.array([len(s) for s in SHAPES])
    return out


def packer_fixtures():
    try:
        from oracle import build_ref

        bitpacking, bytepacking = build_ref.load()
    except Exception as e:  # unbuildable here -> skip, recorded in digests.json
        print("reference extensions unavailable:", e)
        return None
    rng = np.random.default_rng(7)
    cases = {}
    srcs = {
        "small": rng.integers(0, 4, 64),
        "mixed": np.concatenate([rng.integers(0, 4, 40), rng.integers(0, 16, 30), rng.integers(0, 128, 21),
                                 rng.integers(0, 256, 17), rng.integers(0, 4, 5)]),
        "demo": np.abs((10 * rng.standard_normal(1000))).astype(np.int32),
        "full": rng.integers(0, 256, 999),
        "ragged1": np.array([3]),
        "ragged2": np.array([200, 1]),
        "tail": rng.integers(0, 16, 23),
    }
    for name, s in srcs.items():
        t = torch.from_numpy(np.ascontiguousarray(s, dtype=np.int32))
        packed = bitpacking.packing(t)
        unpacked = bitpacking.unpacking(packed)
        cases[f"g4/{name}/src"] = t.numpy()
        cases[f"g4/{name}/packed"] = packed.numpy()
        cases[f"g4/{name}/unpacked"] = unpacked.numpy()
    bsrcs = {
        "q8": rng.integers(-15, 16, 37),
        "wide": rng.integers(-300, 300, 64),
        "one": np.array([-1]),
    }
    for name, s in bsrcs.items():
        t = torch.from_numpy(np.ascontiguousarray(s, dtype=np.int32))
        packed = bytepacking.packing(t)
        unpacked = bytepacking.unpacking(packed)
        cases[f"bp/{name}/src"] = t.numpy()
        cases[f"bp/{name}/packed"] = packed.numpy()
        cases[f"bp/{name}/unpacked"] = unpacked.numpy()
    return cases


def main():
    if "--reducer-worlds" in sys.argv:  # round 4: only the reducer fixtures at these world sizes
        for w in (int(v) for v in sys.argv[sys.argv.index("--reducer-worlds") + 1].split(",")):
            torch.set_num_threads(max(1, 8 // w))
            np.savez_compressed(os.path.join(HERE, f"reducers_w{w}.npz"), **reducer_fixtures(w))
            print("written", f"reducers_w{w}.npz", flush=True)
        return
    torch.set_num_threads(8)
    meta = {"torch": torch.__version__, "seed": SEED, "generator": "tests/golden/make_golden.py"}

    # 1) QSGD-MN (compressors.py:283-321) incl. edge values and ragged sizes
    cases = {}
    x = edge_input(4099, 1)
    for b in (2, 4, 8):
        for k, v in qsgd_case(x, b).items():
            cases[f"b{b}/{k}"] = v
    for n in (1, 2, 3, 5, 63, 64, 65, 1000):
        for k, v in qsgd_case(edge_input(n, 100 + n), 4).items():
            cases[f"n{n}/{k}"] = v
    # GlobalRandK compressor on a dense vector (identical code path, 435-456)
    for k, v in qsgd_case(x, 4, compressors.GlobalRandKMaxNormCompressor).items():
        cases[f"grk_b4/{k}"] = v
    np.savez_compressed(os.path.join(HERE, "qsgd.npz"), **cases)

    # 2) Two-scale and multi-scale
    cases = {}
    for lo, hi in ((2, 4), (4, 8), (2, 6), (6, 10)):
        for k, v in ts_case(x, lo, hi).items():
            cases[f"ts{lo}_{hi}/{k}"] = v
    for lv in ((2, 4), (4, 8), (2, 4, 6), (3, 5, 7, 9), (6, 10)):
        for k, v in ms_case(x, lv).items():
            cases[f"ms{'_'.join(map(str, lv))}/{k}"] = v
    np.savez_compressed(os.path.join(HERE, "multiscale.npz"), **cases)

    # 3) GlobalRandK selection + compress (reducer.py:710-751)
    cases = {}
    for n, K in ((20011, 1000), (5000, 5000), (3001, 1000)):
        for k, v in randk_case(n, K, 4, 3).items():
            cases[f"n{n}_k{K}/{k}"] = v
    np.savez_compressed(os.path.join(HERE, "randk.npz"), **cases)

    # 4) Reducers under gloo, W = 1 and 2 (4 and 8: --reducer-worlds 4,8)
    for w in (1, 2):
        np.savez_compressed(os.path.join(HERE, f"reducers_w{w}.npz"), **reducer_fixtures(w))

    # 5) Digests at sizes too large to commit, formula inputs (oracle.gen_input
    #    is libm-free, so numpy/C/HIP regenerate the identical x)
    digests = {}
    big = [
        ("qsgd_b4_1e6_k0", 1_000_000, 0, 4),
        ("qsgd_b8_1e6_k1", 1_000_000, 1, 8),
        ("qsgd_b2_3e6_k0", 3_000_000, 0, 2),
    ]
    for name, n, kind, b in big:
        xb = oracle.gen_input(n, seed=SEED, kind=kind)
        r = qsgd_case(xb, b)
        digests[name] = dict(n=n, kind=kind, bits=b, norm=float(r["norm"]), q=sha(r["q"]), dec=sha(r["dec"]),
                             x=sha(xb))
    for name, n, lv in (("ms_2_4_1e6", 1_000_000, (2, 4)), ("ms_4_8_1e6", 1_000_000, (4, 8))):
        xb = oracle.gen_input(n, seed=SEED, kind=0)
        r = ms_case(xb, lv)
        digests[name] = dict(n=n, kind=0, levels=list(lv), norm=float(r["norm"]), mask=sha(r["mask"]),
                             q=sha(r["q"]), dec=sha(r["dec"]), x=sha(xb))
    meta["digests"] = digests

    # 6) Reference C++ packers (built from their sources into oracle/_ref)
    pk = packer_fixtures()
    meta["packers"] = "oracle/_ref" if pk is not None else "unavailable"
    if pk is not None:
        np.savez_compressed(os.path.join(HERE, "packers.npz"), **pk)

    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
