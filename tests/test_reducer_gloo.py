"""Multi-rank host logic of gcodec.reducer under gloo on CPU (W = 1, 2, 4, 8),
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


def _check(world, td, bits_bound=True):
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
                if bits_bound:
                    # W <= 2: packed lanes never send more than the reference's int8 vector.  W >= 4:
                    # the carry-free lanes are 7-8 bits (4-bit: bit_length(2 W 15)), the int8 vector's
                    # size, plus plane padding on these tiny tensors (where the reference's int8 SUM
                    # would overflow beyond W (2^b - 1) > 127, ours does not)
                    rb = int(ref[f"r{r}/{name}/s{step}/bits"])
                    assert got[f"{name}/s{step}/bits"] <= (rb + 32 if world <= 2 else rb * 5 // 4 + 128)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_reducers_match_reference(world):
    fixture = os.path.join(GOLD, f"reducers_w{world}.npz")
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(W.reducer_vs_reference, args=(world, os.path.join(td, "init"), fixture, td), nprocs=world,
                 join=True)
        _check(world, td)


@pytest.mark.parametrize("local_size", [1, 2])
def test_reducers_through_node_topology_match_reference(local_size):
    """the reducers with every collective split into
    intra-node / inter-node steps (gcodec.NodeTopology; W = 2 as 2 nodes x 1
    or 1 node x 2) still give the REFERENCE reducers' gradients bit for bit."""
    world = 2
    fixture = os.path.join(GOLD, f"reducers_w{world}.npz")
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(W.reducer_vs_reference, args=(world, os.path.join(td, "init"), fixture, td, local_size),
                 nprocs=world, join=True)
        _check(world, td, bits_bound=False)


def test_reducers_w8_as_two_nodes_of_four_match_reference():
    """W = 8 as 2 nodes x 4 ranks through NodeTopology == the reference at W = 8."""
    world = 8
    fixture = os.path.join(GOLD, f"reducers_w{world}.npz")
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(W.reducer_vs_reference, args=(world, os.path.join(td, "init"), fixture, td, 4),
                 nprocs=world, join=True)
        _check(world, td, bits_bound=False)


def test_default_generator_is_keyed_per_rank():
    """Without an explicit generator every rank draws its own uniforms (the
    default Philox stream is keyed by seed + rank, like the reference's
    per-rank torch seeds): identical inputs give different packed words on
    the two ranks, and each rank's words equal the oracle at key 42 + rank."""
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(W.default_generator_world, args=(2, os.path.join(td, "init"), td), nprocs=2, join=True)
        got = [np.load(os.path.join(td, f"g{r}.npz"), allow_pickle=False) for r in range(2)]
    assert got[0]["words"].tobytes() != got[1]["words"].tobytes()
    for r in range(2):
        assert int(got[r]["key"]) == 42 + r
        assert got[r]["words"].tobytes() == got[r]["oracle"].tobytes()
