"""gcodec.ddp_hook (bucketed backward/communication
overlap) under torch DDP with gloo on CPU, W = 1 and 2, the oracle standing
in for the HIP codec.  Every hook call's result must equal the oracle's
reduction of the ranks' bucket inputs: MAX norm, per-rank encode with the
rank's Philox stream at the recorded offset, SUM of the packed words,
decode with alpha = 1/W."""
import os
import tempfile

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402

import _gloo_workers as W  # noqa: E402


def _expected_bucket(O, xs, offs, world, bits, levels, order):
    n = xs[0].size
    norm = max(O.absmax(x) for x in xs)
    alpha = np.float32(1.0 / world)
    if levels is None:
        tot = None
        for rk in range(world):
            w = O.qsgd_encode(xs[rk], norm, bits, world, O.philox_rng(100 + rk, offs[rk]))
            tot = w.astype(np.uint64) if tot is None else tot + w
        return O.qsgd_decode(tot.astype(np.uint32), n, norm, bits, world, alpha)
    # common resolution level = MIN over ranks (reducer.py:1680-1685; the AND of
    # two-scale, 1494-1499), every rank's q at it, summed, decoded
    masks = [O.ms_mask(xs[rk], norm, levels, O.philox_rng(100 + rk, offs[rk])) for rk in range(world)]
    common = np.minimum.reduce(masks)
    qsum = sum(O.ms_select(xs[rk], norm, levels, O.philox_rng(100 + rk, offs[rk]), common).astype(np.int64)
               for rk in range(world)).astype(np.int32)
    return O.ms_dequantize(qsum, norm, levels, common, order, alpha)


def check_hook_records(recs, world, bits=4, levels=None, order=0):
    from oracle import oracle as O

    calls = int(recs[0]["calls"])
    assert calls >= 4, "expected several buckets over three steps"
    assert all(int(r["calls"]) == calls for r in recs)
    for c in range(calls):
        xs = [r[f"c{c}/x"] for r in recs]
        offs = [int(r[f"c{c}/off"]) for r in recs]
        exp = _expected_bucket(O, xs, offs, world, bits, levels, order)
        for rk in range(world):
            assert recs[rk][f"c{c}/out"].tobytes() == exp.tobytes(), f"call {c} rank {rk}"
    # every rank ends with the same averaged gradients
    for rk in range(1, world):
        assert recs[rk]["grad0"].tobytes() == recs[0]["grad0"].tobytes()


@pytest.mark.parametrize("world", [1, 2])
def test_ddp_qsgd_hook_matches_oracle(world):
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(W.ddp_hook_world, args=(world, os.path.join(td, "init"), td, False), nprocs=world, join=True)
        recs = [np.load(os.path.join(td, f"h{r}.npz"), allow_pickle=False) for r in range(world)]
        check_hook_records(recs, world)


@pytest.mark.parametrize("levels,two_scale", [((2, 4), True), ((2, 4, 6), False)])
@pytest.mark.parametrize("world", [1, 2])
def test_ddp_multiscale_hook_matches_oracle(world, levels, two_scale):
    """The two-/multi-scale hook: mask lanes SUM (= MIN of the levels) in one
    future, select + words SUM + decode in its callback, vs the oracle."""
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(W.ddp_hook_world, args=(world, os.path.join(td, "init"), td, False, list(levels), two_scale),
                 nprocs=world, join=True)
        recs = [np.load(os.path.join(td, f"h{r}.npz"), allow_pickle=False) for r in range(world)]
        check_hook_records(recs, world, levels=list(levels), order=1 if two_scale else 0)


def check_hook_vs_reference(world, td):
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"reducers_w{world}.npz")
    ref = np.load(gold, allow_pickle=False)
    for r in range(world):
        got = np.load(os.path.join(td, f"r{r}.npz"), allow_pickle=False)
        for name in W.HOOK_CASES:
            for step in range(2):
                i = 0
                while f"{name}/s{step}/out{i}" in got.files:
                    a, b = got[f"{name}/s{step}/out{i}"], ref[f"r{r}/{name}/s{step}/out{i}"]
                    assert a.tobytes() == b.tobytes(), f"rank {r} {name} step {step} tensor {i}"
                    i += 1
                assert i > 0


@pytest.mark.parametrize("world", [1, 2])
def test_single_bucket_hook_matches_reference_reducers(world):
    """The hook on one bucket = the whole gradient in TensorBuffer order equals
    the REFERENCE reducers (reducers_w{1,2}.npz) bit for bit (oracle codec on
    CPU, torch-mode RNG).  With several buckets the hook scales each bucket by
    its own max-norm, which the reference (one monolithic bucket) never does:
    DESIGN §6 / INTEGRATION §5."""
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"reducers_w{world}.npz")
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(W.hook_vs_reference, args=(world, os.path.join(td, "init"), gold, td, False), nprocs=world,
                 join=True)
        check_hook_vs_reference(world, td)
