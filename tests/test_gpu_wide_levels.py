"""Wide levels at W = 1: the one-pass multi-scale encode and the one-launch
GlobalRandK encode have narrower domains than the codecs they speed up
(coupled layouts of <= 8 q words per mask word; 16-bit LDS lanes).  Buckets
outside them must take the general kernels — through the compressors, the
reducers and the DDP hook — and still match the oracle bit for bit
(compressors.py:625 allows any lower/higher pair; reducer.py:697-766 any b)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # collected on CPU, skipped there
    pytest.skip("no GPU", allow_module_level=True)

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402
from gcodec._lib import GCodecError  # noqa: E402
from oracle import oracle as O  # noqa: E402

DEV = torch.device("cuda", 0)


def u32(t):
    return t.detach().contiguous().cpu().numpy().view(np.uint32)


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


# levels whose q lane is 9+ bits at W = 1 (r = 32 / lanes-per-word >= 10): no one-pass form
WIDE = [(8, 16), (7, 10, 12), (8, 12), (9, 11)]
NARROW = [(7, 8), (6, 9, 12), (2, 4), (4, 8)]


@pytest.mark.parametrize("levels", WIDE + NARROW)
def test_ms_w1_ok_matches_the_c_entry_point(levels):
    """ms_w1_ok is True exactly when gc_ms_encode_w1 accepts the bucket."""
    n = 10_007
    x = dev(O.gen_input(n, seed=3, kind=1))
    ok = codec.ms_w1_ok(x, levels)
    assert ok == (tuple(levels) in NARROW)
    r = gcodec.rng.Reservation(0, 5, 0, None, n, len(levels))
    if ok:
        codec.ms_encode_w1(x, 0.5, levels, r)
    else:
        with pytest.raises(GCodecError):
            codec.ms_encode_w1(x, 0.5, levels, r)


def _oracle_ms(flat, levels, seed, order, alpha=np.float32(1.0)):
    nrm = O.absmax(flat)
    m = O.ms_mask(flat, nrm, list(levels), O.philox_rng(seed, 0))
    q = O.ms_select(flat, nrm, list(levels), O.philox_rng(seed, 0), m)
    return O.ms_dequantize(q, nrm, list(levels), m, order, alpha)


@pytest.mark.parametrize("levels", WIDE)
def test_reducers_w1_wide_levels_vs_oracle(levels):
    """TwoScale (two levels) and MultiScale reducers at W = 1 with wide levels:
    the one-pass encode declines, the two passes run, == the oracle."""
    sizes = [1000, 37, 65_536, 4099, 3]
    ts = [dev(O.gen_input(s, seed=7 + i, kind=1)) for i, s in enumerate(sizes)]
    flat = np.concatenate([t.cpu().numpy() for t in ts])
    seed = 31
    reds = [(gcodec.QSGDMaxNormMultiScaleReducer(DEV, quantization_levels=list(levels),
                                                 generator=gcodec.Generator(seed, "philox")), 0)]
    if len(levels) == 2:
        reds.append((gcodec.QSGDMaxNormTwoScaleReducer(DEV, lower_quantization_level=levels[0],
                                                       higher_quantization_level=levels[1],
                                                       generator=gcodec.Generator(seed, "philox")), 1))
    for red, order in reds:
        out = [torch.empty_like(t) for t in ts]
        red.reduce(ts, out)
        got = torch.cat(out).cpu().numpy()
        exp = _oracle_ms(flat, levels, seed, order)
        assert got.view(np.uint32).tobytes() == exp.view(np.uint32).tobytes(), (type(red).__name__, levels)


@pytest.mark.parametrize("levels", [(8, 16), (7, 10, 12)])
def test_ddp_hook_w1_wide_levels_vs_oracle(levels):
    """the multi-scale DDP hook at W = 1 with wide levels (two passes) == oracle"""
    from gcodec.ddp_hook import QSGDHookState, qsgd_hook

    class _Bucket:
        def __init__(self, t):
            self._t = t

        def buffer(self):
            return self._t

    n = 100_003
    x = O.gen_input(n, seed=9, kind=1)
    st = QSGDHookState(levels=list(levels), generator=gcodec.Generator(13, "philox"))
    xd = dev(x)
    got = qsgd_hook(st, _Bucket(xd)).wait()
    torch.cuda.synchronize()
    exp = _oracle_ms(x, levels, 13, 0)
    assert u32(got).tobytes() == exp.view(np.uint32).tobytes()


@pytest.mark.parametrize("bits", [16, 20, 24])
def test_randk_fused_rejects_wide_lanes(bits):
    """gc_randk_encode_w1 stages lanes as uint16: b >= 16 is refused, not truncated"""
    n, K = 50_000, 1000
    x = dev(O.gen_input(n, seed=bits))
    idx = dev(np.random.default_rng(bits).permutation(n)[:K].astype(np.int64))
    assert not codec.randk_fused_ok(K, bits, 1)
    with pytest.raises(GCodecError):
        codec.randk_encode_w1(x, idx, bits, gcodec.rng.Reservation(0, 1, 0, None, K, 1))
    assert codec.randk_fused_ok(K, 15, 1)


@pytest.mark.parametrize("bits", [15, 16, 24])
def test_randk_reducer_w1_wide_bits_vs_oracle(bits):
    """GlobalRandKMaxNormReducer at W = 1 and b in {15, 16, 24}: the one-launch
    path only up to 15 bits, the gather + dense encode above; == the oracle of
    reducer.py:717-761 (first pop of the seeded permutation)."""
    sizes = [30_000, 17, 20_011]
    ts = [dev(O.gen_input(s, seed=40 + i, kind=1)) for i, s in enumerate(sizes)]
    flat = np.concatenate([t.cpu().numpy() for t in ts])
    n, K, seed = flat.size, 2000, 42
    gen = gcodec.Generator(77, "philox")
    red = gcodec.GlobalRandKMaxNormReducer(DEV, seed=seed, K=K, quantization_level=bits, generator=gen)
    out = [torch.empty_like(t) for t in ts]
    red.reduce(ts, out)
    torch.manual_seed(seed)
    idx = list(torch.randperm(n).split(K))[-1].numpy()
    xs = flat[idx]
    nk = O.absmax(xs)
    words = O.qsgd_encode(xs, nk, bits, 1, O.philox_rng(seed, 0))  # set_seed re-keys the generator
    exp = flat.copy()
    exp[idx] = O.qsgd_decode(words, idx.size, nk, bits, 1, np.float32(1.0))
    exp = np.float32(0.0) + exp * np.float32(1.0)  # setgrad: out.zero_(); out.add_(g, alpha=1/W)
    got = torch.cat(out).cpu().numpy()
    assert got.view(np.uint32).tobytes() == exp.view(np.uint32).tobytes()
