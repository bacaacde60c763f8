"""Reference-pinned parity at the BASELINE.json config sizes (VERDICT r02
missing #2): the HIP codec in torch-RNG mode (the reference's MT19937 stream,
generated on the GPU) against SHA-256 digests of the reference's OWN outputs,
made by tests/golden/make_golden_big.py from compressors.py / reducer.py on the
same formula inputs:

  config 2  QSGD-MN 4-bit, 1e8            compress / decompress and the packed words
  config 5  QSGD-MN 8-bit, 1e8            int32 q
  config 3  TwoScale (2,4), (4,8), MultiScale [2,4] on 23,520,842
  config 4  GlobalRandK K = 10,000 on 14,728,266: the first two pops, and the
            GlobalRandKMaxNormReducer step itself on the VGG16 tensor list

Integers and floats must match bit for bit (the digest of every array)."""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # collected on CPU, skipped there
    pytest.skip("no GPU", allow_module_level=True)

import gcodec  # noqa: E402
from gcodec import codec, shapes  # noqa: E402
from oracle import oracle as O  # noqa: E402

DEV = torch.device("cuda", 0)
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BIG = json.load(open(os.path.join(GOLD, "golden_big.json")))["digests"]


def sha(t) -> str:
    a = t.detach().contiguous().cpu().numpy() if isinstance(t, torch.Tensor) else t
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture
def torch_mode():
    gcodec.set_rng_mode("torch")
    try:
        yield
    finally:
        gcodec.set_rng_mode(gcodec.rng.DEFAULT_MODE)


def _x(meta):
    x = O.gen_input(meta["n"], seed=42, kind=meta["kind"])
    assert "x" not in meta or sha(x) == meta["x"]
    return torch.from_numpy(x).to(DEV)


@pytest.mark.parametrize("name", ["qsgd_b4_1e8_k0", "qsgd_b8_1e8_k1"])
def test_qsgd_full_size_vs_reference(name, torch_mode):
    meta = BIG[name]
    bits = meta["bits"]
    xd = _x(meta)
    norm = codec.absmax(xd)
    assert norm.item() == meta["norm"]
    c = gcodec.QSGDMaxNormCompressor(DEV, bits)
    torch.manual_seed(42)
    q = c.compress(norm, xd)
    assert str(q.dtype) == meta["q_dtype"] and sha(q) == meta["q"]
    assert sha(c.decompress(norm, q)) == meta["dec"]
    del q
    # the packed, all-reduce-compatible stream carries the same integers
    torch.manual_seed(42)
    words = c.encode(norm, xd)
    ln = codec.qsgd_layout(meta["n"], bits, 1)
    qu = codec.lane_unpack(words, ln).to(torch.int8 if bits < 8 else torch.int32)
    assert sha(qu) == meta["q"]
    assert sha(c.decode(norm, words, meta["n"])) == meta["dec"]


@pytest.mark.parametrize("name", ["ts_2_4_resnet50", "ts_4_8_resnet50"])
def test_twoscale_resnet50_vs_reference(name, torch_mode):
    meta = BIG[name]
    lo, hi = meta["levels"]
    xd = _x(meta)
    norm = codec.absmax(xd)
    assert norm.item() == meta["norm"]
    c = gcodec.QSGDMaxNormTwoScaleCompressor(DEV, lo, hi)
    torch.manual_seed(42)
    q_lo = c.compress_lower(norm, xd)
    q_hi, h = c.compress_higher(norm, xd)
    q = h * q_hi + (1 - h) * q_lo  # reducer.py:1503-1505 at W = 1
    assert sha(h) == meta["h"] and sha(q) == meta["q"]
    assert sha(c.decompress(norm, q, h)) == meta["dec"]
    del q_lo, q_hi, q, h
    # packed W = 1 path (the one-pass encode where it applies, else the two passes)
    torch.manual_seed(42)
    both = c.encode_w1(norm, xd)
    if both is None:
        mw = c.encode_mask(norm, xd, 1)
        words = c.encode(norm, xd, mw, 1)
    else:
        mw, words = both
    m = codec.ms_mask_unpack(mw, meta["n"], [lo, hi])
    assert sha(m) == meta["h"]
    ql, _ = codec.ms_layouts(meta["n"], [lo, hi], 1)
    assert sha(codec.lane_unpack(words, ql).to(torch.int8 if lo < 8 else torch.int32)) == meta["q"]
    assert sha(c.decode(norm, words, mw, meta["n"])) == meta["dec"]


def test_multiscale_resnet50_vs_reference(torch_mode):
    meta = BIG["ms_2_4_resnet50"]
    lv = meta["levels"]
    xd = _x(meta)
    norm = codec.absmax(xd)
    c = gcodec.QSGDMaxNormMultiScaleCompressor(DEV, list(lv))
    torch.manual_seed(42)
    mask = c.compress_mask(norm, xd)
    q = c.compress(mask)
    assert sha(mask) == meta["mask"] and sha(q) == meta["q"]
    assert sha(c.decompress(norm, q, mask)) == meta["dec"]
    torch.manual_seed(42)
    mw, words = c.encode_w1(norm, xd)
    assert sha(codec.ms_mask_unpack(mw, meta["n"], lv)) == meta["mask"]
    ql, _ = codec.ms_layouts(meta["n"], lv, 1)
    assert sha(codec.lane_unpack(words, ql).to(torch.int8)) == meta["q"]
    assert sha(c.decode(norm, words, mw, meta["n"])) == meta["dec"]


def test_randk_vgg16_pops_vs_reference(torch_mode):
    """reducer.py:717-751 at W = 1: set_seed -> randperm -> pop (8,266 then
    10,000 indices) -> gather -> norm -> compress; the one-launch packed encode
    (gather + max-norm + encode) reproduces the same integers."""
    meta = BIG["randk_k10000_vgg16"]
    n, K, bits = meta["n"], meta["K"], meta["bits"]
    xd = _x(meta)
    for packed in (False, True):
        torch.manual_seed(42)
        chunks = list(torch.randperm(n).split(K))
        for p in meta["pops"]:
            idx = chunks.pop()
            assert idx.numel() == p["k"] and sha(idx.to(torch.int64)) == p["idx"]
            idd = idx.to(DEV)
            c = gcodec.GlobalRandKMaxNormCompressor(DEV, bits)
            if not packed:
                xk = xd[idd]
                norm = codec.absmax(xk)
                assert norm.item() == p["norm"]
                q = c.compress(norm, xk)
                assert sha(q) == p["q"] and sha(c.decompress(norm, q)) == p["dec"]
            else:
                words, norm = c.encode_w1(xd, idd)
                assert norm.item() == p["norm"]
                ln = codec.qsgd_layout(idx.numel(), bits, 1)
                assert sha(codec.lane_unpack(words, ln).to(torch.int8)) == p["q"]
                assert sha(c.decode(norm, words, idx.numel())) == p["dec"]


def test_randk_reducer_vgg16_vs_reference(torch_mode):
    """GlobalRandKMaxNormReducer.reduce on the VGG16 list (54 tensors) at
    W = 1, two steps, torch mode == the reference reducer's grad_out."""
    meta = BIG["randk_reducer_k10000_vgg16"]
    sizes = shapes.vgg16_sizes()
    assert sum(sizes) == meta["n"] and len(sizes) == meta["tensors"]
    xd = _x(meta)
    gin = list(torch.split(xd, sizes))
    red = gcodec.GlobalRandKMaxNormReducer(DEV, seed=42, K=meta["K"], quantization_level=meta["bits"],
                                           generator=gcodec.Generator(0, "torch"))
    for st in meta["steps"]:
        gout = [torch.empty_like(g) for g in gin]
        bits = red.reduce(gin, gout)
        assert sha(torch.cat(gout)) == st["out"]
        assert 0 < int(bits) <= st["bits"]  # 5-bit lanes in packed words: fewer bits than the reference's int8
