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


def check_hook_records(recs, world, bits=4):
    from oracle import oracle as O

    calls = int(recs[0]["calls"])
    assert calls >= 4, "expected several buckets over three steps"
    assert all(int(r["calls"]) == calls for r in recs)
    for c in range(calls):
        xs = [r[f"c{c}/x"] for r in recs]
        n = xs[0].size
        norm = max(O.absmax(x) for x in xs)
        tot = None
        for rk in range(world):
            w = O.qsgd_encode(xs[rk], norm, bits, world, O.philox_rng(100 + rk, int(recs[rk][f"c{c}/off"])))
            tot = w.astype(np.uint64) if tot is None else tot + w
        exp = O.qsgd_decode(tot.astype(np.uint32), n, norm, bits, world, np.float32(1.0 / world))
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
