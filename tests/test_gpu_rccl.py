"""The encode -> all-reduce -> decode path with its collectives on RCCL (the
"nccl" backend of torch.distributed on ROCm) on the GPU box.

The pool's boxes have one GPU, and RCCL refuses two ranks on one device
("Duplicate GPU detected", profiles/r03p_rccl2.log), so this runs ONE rank:
every collective of the path still executes as an RCCL kernel on the
caller's stream, between the codec's kernels, with the product's dtypes
(float32 MAX of the norm, int32 SUM of the mask lanes and of the packed
words).  The result must equal the oracle bit for bit; W > 1 sums are covered
by the gloo tests (test_gpu_multirank.py) and the driver's multi-GPU bench.
Reference: reducer.py:516-554 (QSGD-MN), 1636-1715 (multi-scale).
"""
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


def test_rccl_one_rank_path_matches_oracle():
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(W.rccl_path_world, args=(1, os.path.join(td, "init"), td), nprocs=1, join=True)
        got = np.load(os.path.join(td, "rccl0.npz"), allow_pickle=False)
    from oracle import oracle as O

    n, bits, levels = int(got["n"]), int(got["bits"]), [int(v) for v in got["levels"]]
    assert str(got["backend"]) == "nccl" and int(got["world"]) == 1
    x = O.gen_input(n, seed=11, kind=1)
    norm = O.absmax(x)
    assert got["norm"].view(np.uint32)[0] == np.float32(norm).view(np.uint32)
    w_ref = O.qsgd_encode(x, norm, bits, 1, O.philox_rng(int(got["key"]), int(got["off_q"])))
    assert got["words"].view(np.uint32).tobytes() == w_ref.view(np.uint32).tobytes()
    d_ref = O.qsgd_decode(w_ref, n, norm, bits, 1, 1.0)
    assert got["dec"].view(np.uint32).tobytes() == d_ref.view(np.uint32).tobytes()
    rng = O.philox_rng(int(got["key"]), int(got["off_ms"]))
    m_ref = O.ms_mask(x, norm, levels, rng)
    q_ref = O.ms_select(x, norm, levels, rng, m_ref)
    assert got["ms_mask"].tobytes() == m_ref.tobytes()
    md_ref = O.ms_dequantize(q_ref, norm, levels, m_ref, 0, np.float32(1.0))
    assert got["ms_dec"].view(np.uint32).tobytes() == md_ref.view(np.uint32).tobytes()
