"""Worker bodies for the multi-process (gloo, CPU) reducer tests."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "gradient-compression_amd"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

SEED = 42
REDUCERS = ["qsgd", "ts", "ms", "ms3", "randk", "randk_ts"]


def make_reducer(name, **kw):
    from gcodec import reducer as R

    dev = torch.device("cpu")
    if name == "qsgd":
        return R.QSGDMaxNormReducer(dev, None, quantization_level=4, **kw)
    if name == "ts":
        return R.QSGDMaxNormTwoScaleReducer(dev, None, 2, 4, **kw)
    if name == "ms":
        return R.QSGDMaxNormMultiScaleReducer(dev, None, [2, 4], **kw)
    if name == "ms3":
        return R.QSGDMaxNormMultiScaleReducer(dev, None, [2, 4, 6], **kw)
    if name == "randk":
        return R.GlobalRandKMaxNormReducer(dev, None, SEED, K=100, quantization_level=4, **kw)
    if name == "randk_ts":
        return R.GlobalRandKMaxNormTwoScaleReducer(dev, None, SEED, K=100, lower_quantization_level=2,
                                                   higher_quantization_level=4, **kw)
    raise KeyError(name)


def reducer_vs_reference(rank, world, init_file, fixture, out_dir, local_size=None):
    """Run our reducers (oracle codec, torch-mode RNG) on the golden grads
    (local_size: through gcodec.NodeTopology's two-level collectives)."""
    import gcodec
    import oracle_codec

    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    z = np.load(fixture, allow_pickle=False)
    gen = gcodec.Generator(0, "torch")
    res = {}
    topo = None
    if local_size is not None:
        from gcodec.topology import NodeTopology

        topo = NodeTopology(local_size)
    for name in REDUCERS:
        red = make_reducer(name, codec=oracle_codec, generator=gen, topology=topo)
        torch.manual_seed(SEED + rank)
        for step in range(2):
            gin = []
            i = 0
            while f"r{rank}/{name}/s{step}/in{i}" in z.files:
                gin.append(torch.from_numpy(z[f"r{rank}/{name}/s{step}/in{i}"].copy()))
                i += 1
            gout = [torch.empty_like(g) for g in gin]
            bits = red.reduce(gin, gout)
            for i, g in enumerate(gout):
                res[f"{name}/s{step}/out{i}"] = g.numpy()
            res[f"{name}/s{step}/bits"] = np.int64(bits)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


def hip_reducer_vs_reference(rank, world, init_file, fixture, out_dir, local_size=None):
    """Our reducers on the GPU (HIP codec, torch-mode RNG), gloo over CUDA
    tensors; local_size: every collective through gcodec.NodeTopology (the
    multi-node two-level path, nodes of local_size ranks)."""
    import gcodec

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    z = np.load(fixture, allow_pickle=False)
    gen = gcodec.Generator(0, "torch")
    res = {}
    topo = None
    if local_size is not None:
        from gcodec.topology import NodeTopology

        topo = NodeTopology(local_size)

    for name in REDUCERS:
        red = make_reducer(name, generator=gen, topology=topo)
        red._device = dev
        torch.manual_seed(SEED + rank)
        for step in range(2):
            gin = []
            i = 0
            while f"r{rank}/{name}/s{step}/in{i}" in z.files:
                gin.append(torch.from_numpy(z[f"r{rank}/{name}/s{step}/in{i}"].copy()).to(dev))
                i += 1
            gout = [torch.empty_like(g) for g in gin]
            bits = red.reduce(gin, gout)
            torch.cuda.synchronize()
            for i, g in enumerate(gout):
                res[f"{name}/s{step}/out{i}"] = g.cpu().numpy()
            res[f"{name}/s{step}/bits"] = np.int64(bits)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


def hip_pipeline_world(rank, world, init_file, out_dir, n, bits, chunks):
    """ChunkedQSGDAllReduce on the GPU with a gloo group (CUDA tensors)."""
    import gcodec
    from oracle import oracle as O

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    x = O.gen_input(n, seed=100 + rank, kind=rank % 2)
    gen = gcodec.Generator(7 + rank, "philox")
    pipe = gcodec.ChunkedQSGDAllReduce(n, bits, dev, chunks=chunks, generator=gen)
    out = pipe(torch.from_numpy(x).to(dev))
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"p{rank}.npz"), out=out.cpu().numpy(),
             bounds=np.array(pipe.bounds, dtype=np.int64))
    dist.barrier()
    dist.destroy_process_group()


def ddp_hook_world(rank, world, init_file, out_dir, use_gpu, levels=None, two_scale=False):
    """torch DDP with gcodec.ddp_hook.qsgd_hook on a small MLP, several buckets,
    three steps; records every hook call's input bucket, RNG offset and result
    (levels: the two-/multi-scale form of the hook)."""
    import gcodec
    from gcodec.ddp_hook import QSGDHookState, qsgd_hook
    from torch.nn.parallel import DistributedDataParallel as DDP

    if use_gpu:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        codec = None
    else:
        import oracle_codec as codec

        dev = torch.device("cpu")
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    torch.manual_seed(0)  # same initial weights on every rank
    model = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.Tanh(), torch.nn.Linear(64, 64), torch.nn.Tanh(),
                                torch.nn.Linear(64, 8)).to(dev)
    ddp = DDP(model, bucket_cap_mb=0.008)  # ~2k floats per bucket -> several buckets per step
    state = QSGDHookState(bits=4, generator=gcodec.Generator(100 + rank, "philox"), codec=codec, levels=levels,
                          two_scale=two_scale)
    rec = []

    def hook(st, bucket):
        x_in = bucket.buffer().detach().cpu().numpy().copy()
        off = st.gen.offset
        slot = len(rec)  # the call order (bucket order), not the order the futures complete in
        rec.append(None)
        fut = qsgd_hook(st, bucket)

        def keep(f):
            out = f.value()
            rec[slot] = (x_in, off, out.detach().cpu().numpy().copy())
            return out

        return fut.then(keep)

    ddp.register_comm_hook(state, hook)
    g = torch.Generator().manual_seed(1000 + rank)
    for _ in range(3):
        inp = torch.randn(16, 32, generator=g).to(dev)
        ddp.zero_grad()
        ddp(inp).square().sum().backward()
    if use_gpu:
        torch.cuda.synchronize()
    res = {"calls": np.int64(len(rec))}
    for i, (x_in, off, out) in enumerate(rec):
        res[f"c{i}/x"] = x_in
        res[f"c{i}/off"] = np.int64(off)
        res[f"c{i}/out"] = out
    res["grad0"] = model[0].weight.grad.detach().cpu().numpy()
    np.savez(os.path.join(out_dir, f"h{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


def topology_world(rank, world, init_file, out_dir, local_size):
    """NodeTopology (world = nodes x local_size) against flat all-reduces:
    int32 word sums (wrapping past 2^31, ragged lengths), MAX, and every
    reducer with the oracle codec, hierarchical vs flat, step by step."""
    import gcodec
    import oracle_codec
    from gcodec.topology import NodeTopology

    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    topo = NodeTopology(local_size)
    res = {}
    g = torch.Generator().manual_seed(100 + rank)
    for n in (1, 3, 7, 64, 1001, 4099):
        w = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, generator=g)
        flat = w.clone()
        dist.all_reduce(flat)
        hier = topo.all_reduce(w.clone())
        res[f"sum{n}"] = np.int64((hier == flat).all().item())
        m = torch.rand(n, generator=g)
        mf = m.clone()
        dist.all_reduce(mf, op=dist.ReduceOp.MAX)
        res[f"max{n}"] = np.int64((topo.all_reduce(m.clone(), dist.ReduceOp.MAX) == mf).all().item())
    for name in REDUCERS:
        outs = []
        for use_topo in (False, True):
            gen = gcodec.Generator(0, "torch")
            red = make_reducer(name, codec=oracle_codec, generator=gen, topology=topo if use_topo else None)
            torch.manual_seed(SEED + rank)
            gen.manual_seed(SEED + rank)
            got = []
            for step in range(2):
                gin = [torch.randn(s, generator=torch.Generator().manual_seed(1000 * step + 10 * rank + i))
                       for i, s in enumerate((37, 500, 1999))]
                gout = [torch.empty_like(t) for t in gin]
                red.reduce(gin, gout)
                got += [t.numpy().copy() for t in gout]
            outs.append(got)
        res[f"red_{name}"] = np.int64(all(a.tobytes() == b.tobytes() for a, b in zip(*outs)))
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()



def default_generator_world(rank, world, init_file, out_dir):
    """QSGDMaxNormCompressor.encode with NO generator argument on identical
    inputs on every rank (oracle codec on CPU), the default generator in its
    philox mode (the per-rank key; the default mode is torch)."""
    import gcodec
    import oracle_codec
    from oracle import oracle as O

    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    gcodec.set_rng_mode("philox")
    x = O.gen_input(10_001, seed=3)
    comp = gcodec.QSGDMaxNormCompressor(torch.device("cpu"), 4)
    comp.backend = oracle_codec
    r = gcodec.rng.default_generator.reserve(0)  # the key this rank's default stream uses
    off = gcodec.rng.default_generator.offset
    words = comp.encode(torch.tensor([O.absmax(x)]), torch.from_numpy(x), world=world)
    ref = O.qsgd_encode(x, O.absmax(x), 4, world, O.philox_rng(r.seed, off))
    np.savez(os.path.join(out_dir, f"g{rank}.npz"), words=words.numpy(), key=np.int64(r.seed),
             oracle=ref.view(np.int32))
    dist.barrier()
    dist.destroy_process_group()


HOOK_CASES = {"qsgd": dict(bits=4), "ts": dict(levels=[2, 4], two_scale=True), "ms": dict(levels=[2, 4]),
              "ms3": dict(levels=[2, 4, 6])}


class _Bucket:
    def __init__(self, t):
        self._t = t

    def buffer(self):
        return self._t


def hook_vs_reference(rank, world, init_file, fixture, out_dir, use_gpu):
    """gcodec.ddp_hook.qsgd_hook on ONE bucket holding the whole gradient in
    TensorBuffer order (what DDP hands the hook when bucket_cap_mb covers the
    model and the bucket order is the reference's), torch-mode RNG, on the
    reducers' golden grads: the result must equal the reference reducers'
    grad_out (reducer.py:498-554, 1454-1531, 1636-1715)."""
    import gcodec
    from gcodec.ddp_hook import QSGDHookState, qsgd_hook

    if use_gpu:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        codec = None
    else:
        import oracle_codec as codec

        dev = torch.device("cpu")
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    z = np.load(fixture, allow_pickle=False)
    res = {}
    for name, kw in HOOK_CASES.items():
        state = QSGDHookState(generator=gcodec.Generator(0, "torch"), codec=codec, **kw)
        torch.manual_seed(SEED + rank)
        for step in range(2):
            gin = []
            i = 0
            while f"r{rank}/{name}/s{step}/in{i}" in z.files:
                gin.append(torch.from_numpy(z[f"r{rank}/{name}/s{step}/in{i}"].copy()))
                i += 1
            flat = torch.cat([g.reshape(-1) for g in gin]).to(dev)
            out = qsgd_hook(state, _Bucket(flat)).wait()
            if use_gpu:
                torch.cuda.synchronize()
            out = out.cpu()
            pos = 0
            for i, g in enumerate(gin):
                res[f"{name}/s{step}/out{i}"] = out[pos:pos + g.numel()].reshape(g.shape).numpy()
                pos += g.numel()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


def rccl_path_world(rank, world, init_file, out_dir):
    """The QSGD-MN and multi-scale DP paths with every collective on RCCL
    ("nccl"): absmax -> all_reduce(MAX) -> encode -> all_reduce(SUM words)
    -> decode; mask lanes -> all_reduce(SUM) -> select -> all_reduce(SUM) ->
    decode (reducer.py:516-554, 1636-1715).  Saves what the test checks."""
    import gcodec
    from gcodec import codec
    from oracle import oracle as O

    dev = torch.device("cuda", rank)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"file://{init_file}", rank=rank, world_size=world, device_id=dev)
    n, bits, levels = 1_000_003, 4, [2, 4]
    x = torch.from_numpy(O.gen_input(n, seed=11, kind=1)).to(dev)
    gen = gcodec.Generator(9, "philox", per_rank=False)
    norm = codec.absmax(x)
    dist.all_reduce(norm, op=dist.ReduceOp.MAX)
    off_q = gen.offset
    words = codec.qsgd_encode(x, norm, bits, gen.reserve(n), world)
    dist.all_reduce(words)
    dec = codec.qsgd_decode(words, n, norm, bits, world, 1.0 / world)
    off_ms = gen.offset
    r = gen.reserve(n, len(levels))
    mw = codec.ms_mask_encode(x, norm, levels, r, world)
    dist.all_reduce(mw)
    mwords = codec.ms_select_encode(x, norm, levels, r, mw, world)
    dist.all_reduce(mwords)
    mdec = codec.ms_decode(mwords, mw, n, norm, levels, world, 0, 1.0 / world)
    mask = codec.ms_mask_unpack(mw, n, levels, world)
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"rccl{rank}.npz"), n=n, bits=bits, levels=np.array(levels), key=gen.seed,
             off_q=off_q, off_ms=off_ms, backend=np.array(dist.get_backend()), world=dist.get_world_size(),
             norm=norm.cpu().numpy(), words=words.cpu().numpy(), dec=dec.cpu().numpy(),
             ms_mask=mask.cpu().numpy().astype(np.uint8), ms_dec=mdec.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def hip_randk_vgg16_world(rank, world, init_file, out_dir, K, bits, steps):
    """GlobalRandKMaxNormReducer (HIP codec, torch-mode RNG) on the VGG16 tensor
    list, rank r's gradient = gen_input(seed 42 + r), gloo over CUDA tensors on
    cuda:0: the SHA-256 of every step's grad_out (tests/golden/make_golden_big.py
    ran the REFERENCE reducer the same way)."""
    import hashlib
    import json

    import gcodec
    from gcodec import shapes
    from oracle import oracle as O

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    sizes = shapes.vgg16_sizes()
    x = torch.from_numpy(O.gen_input(sum(sizes), seed=SEED + rank, kind=0)).to(dev)
    gin = list(torch.split(x, sizes))
    red = gcodec.GlobalRandKMaxNormReducer(dev, seed=SEED, K=K, quantization_level=bits,
                                           generator=gcodec.Generator(0, "torch"))
    res = []
    for _ in range(steps):
        gout = [torch.empty_like(g) for g in gin]
        nbits = red.reduce(gin, gout)
        torch.cuda.synchronize()
        out = torch.cat(gout).cpu().numpy()
        res.append({"out": hashlib.sha256(out.tobytes()).hexdigest(), "bits": int(nbits)})
    with open(os.path.join(out_dir, f"v{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()
