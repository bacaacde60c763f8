"""The HIP reducers at W = 1 and 2 on the GPU box (two processes on cuda:0,
gloo over CUDA tensors), bit-compared with the REFERENCE reducers' outputs
(tests/golden/reducers_w*.npz).  RCCL needs one GPU per rank, so the
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


@pytest.mark.parametrize("world", [1, 2])
def test_hip_reducers_match_reference(world):
    fixture = os.path.join(GOLD, f"reducers_w{world}.npz")
    ref = np.load(fixture, allow_pickle=False)
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(W.hip_reducer_vs_reference, args=(world, os.path.join(td, "init"), fixture, td), nprocs=world,
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
