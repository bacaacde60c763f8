"""The HIP reducers at W = 1, 2, 4 and 8 on the GPU box (W processes on
cuda:0, gloo over CUDA tensors), bit-compared with the REFERENCE reducers'
outputs (tests/golden/reducers_w*.npz; golden_big.json for the VGG16
GlobalRandK reducer at W = 2 / 4 / 8).  RCCL needs one GPU per rank, so the
collective here is gloo; the codec calls, stream handling and lane sizing
for W are the product path."""
import os
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import torch.multiprocessing as mp  # noqa: E402

import _gloo_workers as W  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _check_vs_reference(world, td):
    ref = np.load(os.path.join(GOLD, f"reducers_w{world}.npz"), allow_pickle=False)
    for r in range(world):
        got = np.load(os.path.join(td, f"r{r}.npz"), allow_pickle=False)
        for name in W.REDUCERS:
            for step in range(2):
                i = 0
                while f"{name}/s{step}/out{i}" in got.files:
                    a = got[f"{name}/s{step}/out{i}"]
                    b = ref[f"r{r}/{name}/s{step}/out{i}"]
                    assert a.tobytes() == b.tobytes(), f"rank {r} {name} step {step} tensor {i}"
                    i += 1
                assert i > 0


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_hip_reducers_match_reference(world):
    fixture = os.path.join(GOLD, f"reducers_w{world}.npz")
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(W.hip_reducer_vs_reference, args=(world, os.path.join(td, "init"), fixture, td), nprocs=world,
                 join=True)
        _check_vs_reference(world, td)


@pytest.mark.parametrize("world,chunks", [(2, 3), (3, 1)])
def test_chunked_pipeline_multirank(world, chunks):
    """Every rank's result = oracle: per chunk, sum the ranks' packed words and decode."""
    from oracle import oracle as O

    n, bits = 300_007, 4
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(W.hip_pipeline_world, args=(world, os.path.join(td, "init"), td, n, bits, chunks), nprocs=world,
                 join=True)
        outs = [np.load(os.path.join(td, f"p{r}.npz"), allow_pickle=False) for r in range(world)]
    xs = [O.gen_input(n, seed=100 + r, kind=r % 2) for r in range(world)]
    norm = max(O.absmax(x) for x in xs)
    bounds = outs[0]["bounds"]
    exp = np.empty(n, np.float32)
    off = 0
    for s, e in bounds:
        tot = None
        for r in range(world):
            w = O.qsgd_encode(xs[r][s:e], norm, bits, world, O.philox_rng(7 + r, off)).astype(np.uint64)
            tot = w if tot is None else tot + w
        exp[s:e] = O.qsgd_decode(tot.astype(np.uint32), e - s, norm, bits, world, np.float32(1.0 / world))
        off += e - s
    for r in range(world):
        assert outs[r]["out"].tobytes() == exp.tobytes(), f"rank {r}"


@pytest.mark.parametrize("world", [1, 2])
def test_ddp_qsgd_hook_on_gpu(world):
    """gcodec.ddp_hook on cuda:0 (HIP codec), DDP over gloo with CUDA tensors:
    every bucket's result equals the oracle's reduction of the ranks' inputs."""
    from test_ddp_hook_gloo import check_hook_records

    with tempfile.TemporaryDirectory() as td:
        mp.spawn(W.ddp_hook_world, args=(world, os.path.join(td, "init"), td, True), nprocs=world, join=True)
        recs = [np.load(os.path.join(td, f"h{r}.npz"), allow_pickle=False) for r in range(world)]
        check_hook_records(recs, world)


@pytest.mark.parametrize("levels,two_scale", [((2, 4), True), ((2, 4, 6), False)])
@pytest.mark.parametrize("world", [1, 2])
def test_ddp_multiscale_hook_on_gpu(world, levels, two_scale):
    """The two-/multi-scale DDP hook on cuda:0: W = 1 runs the one-pass encode
    (gc_ms_encode_w1), W = 2 the mask pass with the q cache, the mask SUM and
    the select from the cache; every bucket equals the oracle's reduction."""
    from test_ddp_hook_gloo import check_hook_records

    with tempfile.TemporaryDirectory() as td:
        mp.spawn(W.ddp_hook_world, args=(world, os.path.join(td, "init"), td, True, list(levels), two_scale),
                 nprocs=world, join=True)
        recs = [np.load(os.path.join(td, f"h{r}.npz"), allow_pickle=False) for r in range(world)]
        check_hook_records(recs, world, levels=list(levels), order=1 if two_scale else 0)


@pytest.mark.parametrize("local_size", [1, 2])
def test_hip_reducers_through_node_topology(local_size):
    """gcodec.NodeTopology (two-level collectives: intra-node reduce-scatter,
    inter-node all-reduce of the shard, intra-node all-gather) with the HIP
    codec, W = 2 as 2 nodes x 1 or 1 node x 2: every reducer's gradients equal
    the REFERENCE reducers' outputs (tests/golden/reducers_w2.npz) bit for bit."""
    world = 2
    fixture = os.path.join(GOLD, f"reducers_w{world}.npz")
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(W.hip_reducer_vs_reference, args=(world, os.path.join(td, "init"), fixture, td, local_size),
                 nprocs=world, join=True)
        _check_vs_reference(world, td)


@pytest.mark.parametrize("world", [1, 2])
def test_single_bucket_hook_matches_reference_reducers_gpu(world):
    """gcodec.ddp_hook.qsgd_hook with the HIP codec on one bucket holding the
    whole gradient (TensorBuffer order), torch-mode RNG: == the REFERENCE
    reducers' grad_out (reducers_w{1,2}.npz) for QSGD-MN, two-scale and
    multi-scale [2,4] / [2,4,6] (W = 1: one-pass encode; W = 2: q cache)."""
    from test_ddp_hook_gloo import check_hook_vs_reference

    fixture = os.path.join(GOLD, f"reducers_w{world}.npz")
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(W.hook_vs_reference, args=(world, os.path.join(td, "init"), fixture, td, True), nprocs=world,
                 join=True)
        check_hook_vs_reference(world, td)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_randk_reducer_vgg16_multirank_vs_reference(world):
    """Config 4 at its world sizes: GlobalRandKMaxNormReducer, K = 10,000,
    4-bit, the VGG16 tensor list, W ranks with different gradients, two steps:
    every rank's grad_out equals the REFERENCE reducer's (SHA-256 from
    make_golden_big.py, the reference run under gloo at the same W)."""
    import json

    big = json.load(open(os.path.join(GOLD, "golden_big.json")))["digests"]
    meta = big[f"randk_reducer_k10000_vgg16_w{world}"]
    assert meta["world"] == world
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(W.hip_randk_vgg16_world, args=(world, os.path.join(td, "init"), td, meta["K"], meta["bits"],
                                                len(meta["steps"])), nprocs=world, join=True)
        for r in range(world):
            got = json.load(open(os.path.join(td, f"v{r}.json")))
            for s, (g, ref) in enumerate(zip(got, meta["ranks"][r])):
                assert g["out"] == ref["out"], f"rank {r} step {s}"
                # W >= 4: 7-8 bit carry-free lanes, the int8 vector's size + the plane alignment
                assert 0 < g["bits"] <= ref["bits"] + (0 if world <= 2 else 128)
