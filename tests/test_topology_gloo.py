"""Two-level (intra-node / inter-node) collectives of gcodec.topology under
gloo on CPU: 4 ranks as 2 nodes x 2 and 1 node x 4, 3 ranks as 3 nodes x 1.
The hierarchical SUM of packed words and MAX of norms equal the flat
all-reduce bit for bit, and every reducer gives the same gradients either way
(SURVEY §8(f) row 4)."""
import os
import tempfile

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402

import _gloo_workers as W  # noqa: E402


@pytest.mark.parametrize("world,local_size", [(4, 2), (4, 4), (3, 1)])
def test_hierarchical_equals_flat(world, local_size):
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(W.topology_world, args=(world, os.path.join(td, "init"), td, local_size), nprocs=world, join=True)
        for r in range(world):
            got = np.load(os.path.join(td, f"r{r}.npz"), allow_pickle=False)
            bad = [k for k in got.files if int(got[k]) != 1]
            assert not bad, (r, bad)
            assert any(k.startswith("red_") for k in got.files)
