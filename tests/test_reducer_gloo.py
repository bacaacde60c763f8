"""Multi-rank host logic of gcodec.reducer under gloo on CPU (W = 1, 2),
with the oracle standing in for the HIP codec, against the outputs of the
REFERENCE reducers on the same per-rank gradients and RNG streams
(tests/golden/reducers_w*.npz, made by running reducer.py under gloo)."""
import os
import tempfile

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402

import _gloo_workers as W  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("world", [1, 2])
def test_reducers_match_reference(world):
    fixture = os.path.join(GOLD, f"reducers_w{world}.npz")
    ref = np.load(fixture, allow_pickle=False)
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(W.reducer_vs_reference, args=(world, os.path.join(td, "init"), fixture, td), nprocs=world,
                 join=True)
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
                    # packed lanes never send more than the reference's int8 vector
                    assert got[f"{name}/s{step}/bits"] <= ref[f"r{r}/{name}/s{step}/bits"] + 32
