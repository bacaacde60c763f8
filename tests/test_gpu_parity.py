"""HIP kernels (through the C ABI) vs the CPU oracle and the reference's
golden vectors.  Integers and packed words: bit-exact.  Floats: bit-exact
(the kernels use the reference's operation order; the north-star tolerance
is 1 ULP, the tests demand 0)."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # collected on CPU, skipped there
    pytest.skip("no GPU", allow_module_level=True)

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402
from oracle import oracle as O  # noqa: E402

DEV = torch.device("cuda", 0)
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def gz(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def u32(t):
    return t.detach().cpu().numpy().view(np.uint32)


def bits_eq(a, b):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    return a.shape == b.shape and a.tobytes() == b.tobytes()


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


SIZES = [1, 3, 4, 5, 63, 64, 65, 127, 1000, 4099, 65536 + 3, 1_000_003]


# --------------------------------------------------------------------------- absmax
@pytest.mark.parametrize("n", SIZES + [10_000_019])
def test_absmax(n):
    x = O.gen_input(n, seed=n, kind=1)
    assert codec.absmax(dev(x)).item() == float(O.absmax(x))


def test_absmax_unaligned_gather_nan():
    x = O.gen_input(100_001, seed=3)
    xd = dev(x)
    assert codec.absmax(xd[1:]).item() == float(O.absmax(x[1:]))  # scalar path
    idx = np.random.default_rng(0).choice(x.size, 997, replace=False).astype(np.int64)
    assert codec.absmax(xd, idx=dev(idx)).item() == float(O.absmax(x[idx]))
    x2 = x.copy()
    x2[5000] = np.nan
    assert np.isnan(codec.absmax(dev(x2)).item())
    assert codec.absmax(dev(np.zeros(10, np.float32))).item() == 0.0


# --------------------------------------------------------------------------- QSGD packed, Philox
@pytest.mark.parametrize("bits", [2, 4, 8])
@pytest.mark.parametrize("world", [1, 2, 8])
@pytest.mark.parametrize("n", [1, 5, 64, 65, 4099, 1_000_003])
def test_encode_decode_philox_vs_oracle(bits, world, n):
    x = O.gen_input(n, seed=7 * n + bits, kind=n % 2)
    norm = O.absmax(x)
    seed, off = 1234 + bits, 77 * n
    r = gcodec.rng.Reservation(gcodec._lib.GC_RNG_PHILOX, seed, off, None, n, 1)
    words = codec.qsgd_encode(dev(x), float(norm), bits, r, world)
    ref = O.qsgd_encode(x, norm, bits, world, O.philox_rng(seed, off))
    assert bits_eq(u32(words), ref)
    alpha = np.float32(1.0 / world)
    dec = codec.qsgd_decode(words, n, float(norm), bits, world, float(alpha))
    assert bits_eq(u32(dec), O.qsgd_decode(ref, n, norm, bits, world, alpha).view(np.uint32))


def test_encode_unaligned_and_gather():
    n, bits = 50_001, 4
    x = O.gen_input(n + 1, seed=9)
    xd = dev(x)
    norm = O.absmax(x[1:])
    r = gcodec.rng.Reservation(0, 5, 0, None, n, 1)
    words = codec.qsgd_encode(xd[1:], float(norm), bits, r, 1)  # misaligned x -> scalar path
    assert bits_eq(u32(words), O.qsgd_encode(x[1:], norm, bits, 1, O.philox_rng(5, 0)))
    idx = np.random.default_rng(1).permutation(n + 1)[:10_000].astype(np.int64)
    normk = O.absmax(x[idx])
    rk = gcodec.rng.Reservation(0, 5, 3, None, idx.size, 1)
    wk = codec.qsgd_encode(xd, float(normk), bits, rk, 2, idx=dev(idx))
    refk = O.qsgd_encode(x[idx], normk, bits, 2, O.philox_rng(5, 3))
    assert bits_eq(u32(wk), refk)
    out = torch.zeros(n + 1, dtype=torch.float32, device=DEV)
    codec.qsgd_decode(wk, idx.size, float(normk), bits, 2, 1.0, idx=dev(idx), out=out)
    exp = np.zeros(n + 1, np.float32)
    exp[idx] = O.qsgd_decode(refk, idx.size, normk, bits, 2, 1.0)
    assert bits_eq(u32(out), exp.view(np.uint32))


@pytest.mark.parametrize("bits,world", [(1, 1), (2, 8), (4, 2), (8, 1), (8, 8)])
@pytest.mark.parametrize("K", [1, 7, 10_000, 100_003])
def test_grandk_batched_gather_scatter(bits, world, K):
    """GRandK gather encode / scatter decode (gather_planes, gather_idx: index
    loads batched per chunk of <= 8 planes).  1-bit lanes at W=1 give 16 planes
    per word (two chunks); ragged K leaves partial last planes; K=1 a single
    element.  Non-selected elements keep their value (reducer.py:754)."""
    n = 200_003
    x = O.gen_input(n, seed=K + bits, kind=1)
    idx = np.random.default_rng(K + world).permutation(n)[:K].astype(np.int64)
    xd, idd = dev(x), dev(idx)
    normk = O.absmax(x[idx])
    assert codec.absmax(xd, idx=idd).item() == float(normk)
    r = gcodec.rng.Reservation(0, 11, K, None, K, 1)
    wk = codec.qsgd_encode(xd, float(normk), bits, r, world, idx=idd)
    refk = O.qsgd_encode(x[idx], normk, bits, world, O.philox_rng(11, K))
    assert bits_eq(u32(wk), refk)
    alpha = np.float32(1.0 / world)
    out = dev(x)
    codec.qsgd_decode(wk, K, float(normk), bits, world, float(alpha), idx=idd, out=out)
    exp = x.copy()
    exp[idx] = O.qsgd_decode(refk, K, normk, bits, world, alpha)
    assert bits_eq(u32(out), exp.view(np.uint32))


@pytest.mark.parametrize("levels", [(2, 4), (1, 2, 3, 4, 5, 6, 7, 8)])
@pytest.mark.parametrize("K", [3, 10_001])
def test_ms_grandk_gather_scatter(levels, K):
    """multi-scale mask / select / decode through idx (GRandK two-scale,
    reducer.py:1568-1621): batched gathers vs the oracle on x[idx]."""
    n, world = 50_021, 2
    x = O.gen_input(n, seed=K, kind=1)
    idx = np.random.default_rng(K).permutation(n)[:K].astype(np.int64)
    xk = x[idx]
    norm = O.absmax(xk)
    L = len(levels)
    r = gcodec.rng.Reservation(0, 5, 1, None, K, L)
    xd, idd = dev(x), dev(idx)
    mw = codec.ms_mask_encode(xd, float(norm), levels, r, world, idx=idd)
    assert bits_eq(u32(mw), u32(codec.ms_mask_encode(dev(xk), float(norm), levels, r, world)))
    mw_sum = (mw.to(torch.int64) * world).to(torch.int32)
    m_ref = O.ms_mask(xk, norm, levels, O.philox_rng(5, 1))
    words = codec.ms_select_encode(xd, float(norm), levels, r, mw_sum, world, idx=idd)
    q_ref = O.ms_select(xk, norm, levels, O.philox_rng(5, 1), m_ref)
    ql, _ = codec.ms_layouts(K, levels, world)
    assert bits_eq(u32(words), O.lane_pack(q_ref, ql.offset, ql.bits, ql.per_word, ql.plane_words))
    wsum = (words.to(torch.int64) * world).to(torch.int32)
    out = dev(x)
    codec.ms_decode(wsum, mw_sum, K, float(norm), levels, world, 0, 0.5, idx=idd, out=out)
    exp = x.copy()
    exp[idx] = O.ms_dequantize(q_ref * world, norm, levels, m_ref, 0, np.float32(0.5))
    assert bits_eq(u32(out), exp.view(np.uint32))


@pytest.mark.parametrize("world", [1, 4])
def test_encode_non_finite_and_tiny_inputs(world):
    """NaN -> 0, +/-inf and |x| > norm saturate at +/-s, subnormal and
    below-2^-100 magnitudes take the exact-division branch — all vs the oracle."""
    n, bits = 4 * 6 * 997, 4
    x = O.gen_input(n, seed=5)
    x[::97] = np.nan
    x[5::101] = np.inf
    x[7::103] = -np.inf
    x[11::89] = np.float32(3e-41)      # subnormal
    x[13::83] = np.float32(-1e-35)     # normal, below 2^-100 * norm? (norm ~1e-2)
    x[17::79] = np.float32(7e-31)
    x[19::73] = 0.25                   # |x| > norm
    x[23::71] = -0.0
    norm = np.float32(np.nanmax(np.abs(x[np.isfinite(x)])) / 8)  # finite, smaller than some |x|
    r = gcodec.rng.Reservation(0, 77, 1, None, n, 1)
    words = codec.qsgd_encode(dev(x), float(norm), bits, r, world)
    assert bits_eq(u32(words), O.qsgd_encode(x, norm, bits, world, O.philox_rng(77, 1)))
    # tiny norms take the generic exact-division path for every element
    for tiny in (np.float32(1e-38), np.float32(2e-45), np.float32(3e33)):
        words = codec.qsgd_encode(dev(x), float(tiny), bits, r, world)
        assert bits_eq(u32(words), O.qsgd_encode(x, tiny, bits, world, O.philox_rng(77, 1))), tiny


def _int_path_input(n, norm, s, seed):
    """Values that stress the integer stochastic rounding of full tiles:
    exact level boundaries k*norm/s and their float neighbours (p = 0 and p
    just above 0 / just below 1), +-norm, +-0, l < 1/2 with a non-integer
    l*2^24, and a few subnormals (their tiles take the IEEE branch)."""
    rng = np.random.default_rng(seed)
    x = O.gen_input(n, seed=seed, kind=seed % 2) * np.float32(norm / 0.05)
    k = rng.integers(-s, s + 1, n).astype(np.float32)
    lvl = (k * np.float32(norm)) / np.float32(s)
    pick = rng.random(n)
    x = np.where(pick < 0.15, lvl, x)
    x = np.where((pick >= 0.15) & (pick < 0.25), np.nextafter(lvl, np.float32(np.inf)), x)
    x = np.where((pick >= 0.25) & (pick < 0.35), np.nextafter(lvl, np.float32(-np.inf)), x)
    tiny = (rng.random(n).astype(np.float32) * np.float32(norm) * np.float32(2.0**-28))
    x = np.where((pick >= 0.35) & (pick < 0.40), tiny, x)
    x = np.clip(x, -norm, norm).astype(np.float32)
    x[::4099] = norm
    x[7::4111] = -norm
    x[3::1009] = 0.0
    x[5::1013] = -0.0
    x[11::50021] = np.float32(1e-40)  # subnormal: that tile takes the IEEE branch
    return x


@pytest.mark.parametrize("bits", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("world", [1, 2, 8])
def test_encode_integer_rounding_path_edges(bits, world):
    """The dense full-tile body rounds in integers (qsgd_encode.h ENC_INT:
    v_cvt_flr of -|Ls| + 24-bit add for b <= 7, ceil(|Ls|) + (~r & 0xFFFFFF)
    for b = 8): it must equal the oracle's float arithmetic on adversarial
    values, and so must the IEEE branch that tiny norms and subnormal tiles take."""
    s = (1 << bits) - 1
    n = 6 * 4 * 4096 + 13
    for norm in (np.float32(0.05), np.float32(3.0), np.float32(2.0**-60)):
        x = _int_path_input(n, norm, s, seed=bits * 31 + world)
        nh = O.absmax(x)
        r = gcodec.rng.Reservation(0, 4242 + bits, 5, None, n, 1)
        words = codec.qsgd_encode(dev(x), float(nh), bits, r, world)
        ref = O.qsgd_encode(x, nh, bits, world, O.philox_rng(4242 + bits, 5))
        assert bits_eq(u32(words), ref), (bits, world, float(norm))


def test_zero_bucket_gives_zero():
    n, bits = 1000, 4
    x = np.zeros(n, np.float32)
    r = gcodec.rng.Reservation(0, 1, 0, None, n, 1)
    words = codec.qsgd_encode(dev(x), 0.0, bits, r, 1)
    dec = codec.qsgd_decode(words, n, 0.0, bits, 1)
    assert bits_eq(u32(words), O.qsgd_encode(x, np.float32(0), bits, 1, O.philox_rng(1, 0)))
    assert torch.all(dec == 0)


# --------------------------------------------------------------------------- torch-mode = reference
@pytest.mark.parametrize("case", ["b2", "b4", "b8", "n1", "n3", "n65", "n1000"])
def test_facade_compress_matches_reference(case):
    z = gz("qsgd.npz")
    x, norm, q, dec, bits = (z[f"{case}/{k}"] for k in ("x", "norm", "q", "dec", "bits"))
    gcodec.set_rng_mode("torch")
    try:
        torch.manual_seed(int(z[f"{case}/seed"]))
        c = gcodec.QSGDMaxNormCompressor(DEV, int(bits))
        qg = c.compress(torch.tensor(norm, device=DEV), dev(x))
        assert qg.dtype == torch.from_numpy(q).dtype
        assert bits_eq(qg.cpu().numpy(), q)
        dg = c.decompress(torch.tensor(norm, device=DEV), qg)
        assert bits_eq(u32(dg), dec.view(np.uint32))
        # the packed stream in torch mode is the reference's q, lane-packed
        torch.manual_seed(int(z[f"{case}/seed"]))
        words = c.encode(torch.tensor(norm, device=DEV), dev(x))
        s = (1 << int(bits)) - 1
        w, L, M = O.lane_layout(x.size, 2 * s, 1)
        assert bits_eq(u32(words), O.lane_pack(q.astype(np.int32), s, w, L, M))
    finally:
        gcodec.set_rng_mode(gcodec.rng.DEFAULT_MODE)


def test_default_mode_is_reference_identical():
    """with NO mode call, the reference-named class gives
    the reference's integers (golden.json:qsgd_b4_1e6_k0, made by importing
    compressors.py) after torch.manual_seed, and its packed encode the same q
    lane-packed; philox stays an explicit opt-in."""
    import hashlib

    assert gcodec.rng.default_generator.mode == "torch"
    meta = json.load(open(os.path.join(GOLD, "golden.json")))["digests"]["qsgd_b4_1e6_k0"]
    x = O.gen_input(meta["n"], seed=42, kind=meta["kind"])
    xd = dev(x)
    norm = codec.absmax(xd)
    torch.manual_seed(42)
    q = gcodec.QSGDMaxNormCompressor(DEV, meta["bits"]).compress(norm, xd)
    assert hashlib.sha256(q.cpu().numpy().tobytes()).hexdigest() == meta["q"]
    torch.manual_seed(42)
    words = gcodec.QSGDMaxNormCompressor(DEV, meta["bits"]).encode(norm, xd)
    s = (1 << meta["bits"]) - 1
    w, L, M = O.lane_layout(x.size, 2 * s, 1)
    assert bits_eq(u32(words), O.lane_pack(q.cpu().numpy().astype(np.int32), s, w, L, M))


def test_torch_generator_state_advances_like_reference():
    gcodec.set_rng_mode("torch")
    try:
        torch.manual_seed(5)
        x = dev(O.gen_input(3001, seed=1))
        gcodec.QSGDMaxNormCompressor(DEV, 4).compress(codec.absmax(x), x)
        after = torch.rand(5)
        torch.manual_seed(5)
        torch.bernoulli(torch.full((3001,), 0.5))
        assert torch.equal(after, torch.rand(5))
    finally:
        gcodec.set_rng_mode(gcodec.rng.DEFAULT_MODE)


def test_mt19937_kernel_matches_oracle():
    st = codec.mt19937_seed_state(42)
    sd = torch.from_numpy(st.view(np.int32)).to(DEV)
    a = codec.mt19937_generate(sd, 1000)
    b = codec.mt19937_generate(sd, 123_457)
    mt = O.MT19937(42)
    assert bits_eq(u32(a), mt.draws(1000))
    assert bits_eq(u32(b), mt.draws(123_457))


MTJ = gcodec._lib.GC_MT_JUMP_DRAWS


@pytest.mark.parametrize("J", [MTJ, 1872])
@pytest.mark.parametrize("mult", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("pre", [0, 1, 300])
def test_mt19937_jumped_matches_serial(J, mult, pre):
    """The parallel (jump-ahead) MT19937 stream == the serial one: every draw
    and the advanced state (state array + read index) bit for bit, from read
    indices 624 (fresh seed), 1 and 300; generator boundaries at J - 1, J,
    J + 1 for the default generator length and a short one (J = 3 x 624)."""
    count = [1, 1000, J - 1, J, J + 1, 3 * J + 5][mult]
    st = codec.mt19937_seed_state(42)
    sd = torch.from_numpy(st.view(np.int32)).to(DEV)
    if pre:
        codec.mt19937_generate(sd, pre, parallel=False)
    s2 = sd.clone()
    a = codec.mt19937_generate(sd, count, J=J)
    b = codec.mt19937_generate(s2, count, parallel=False)
    assert torch.equal(a, b)
    assert torch.equal(sd, s2)
    if count <= 3 * J + 5:
        mt = O.MT19937(42)
        mt.draws(pre)
        assert bits_eq(u32(a), mt.draws(count))


@pytest.mark.parametrize("bits", [2, 4, 8])
@pytest.mark.parametrize("n", [1, 1000, MTJ - 3, MTJ + 1, 2 * MTJ + 7])
@pytest.mark.parametrize("pre", [0, 5])
def test_torch_mode_fused_quantize_matches_draw_path(bits, n, pre):
    """Torch mode with the MT19937 draws consumed inside the generator kernel
    (gc_qsgd_quantize_mt19937, no draw buffer) == the oracle fed with torch's
    stream, == the draw-buffer path (torch-mode reservation + gc_qsgd_quantize),
    and torch's CPU generator ends in the same state; the packed form
    (qsgd_encode_torch) == qsgd_encode from the draws, at W = 1 and 8."""
    x = torch.from_numpy(O.gen_input(n, seed=n + bits)).to(DEV)
    x[::97] = 0.0
    x[1::211] = -0.0
    x[3::1009] = 1e-39   # subnormal / tiny |x|: the exact-division branch
    x[5::2003] = -3e-42
    norm = codec.absmax(x)
    dtype = torch.int8 if bits < 8 else torch.int32

    def fresh():
        torch.manual_seed(7)
        torch.bernoulli(torch.zeros(pre))  # consumes `pre` draws: the read index moves off the block start

    fresh()
    q1 = codec.qsgd_quantize_torch(x, norm, bits)
    s1 = torch.get_rng_state()
    fresh()
    q2 = codec.qsgd_quantize(x, norm, bits, gcodec.Generator(0, "torch").reserve(n, 1, DEV), 0, dtype)
    assert torch.equal(q1, q2)
    assert torch.equal(s1, torch.get_rng_state())
    mt = O.MT19937(7)
    mt.draws(pre)
    exp = O.qsgd_quantize(x.cpu().numpy(), np.float32(norm.item()), bits, O.stream_rng(mt.draws(n)))
    assert np.array_equal(q1.cpu().numpy().astype(np.int32), exp.astype(np.int32))
    for world in (1, 8):
        fresh()
        w1 = codec.qsgd_encode_torch(x, norm, bits, world)
        fresh()
        w2 = codec.qsgd_encode(x, norm, bits, gcodec.Generator(0, "torch").reserve(n, 1, DEV), world)
        assert torch.equal(w1, w2)


def test_mt19937_jumped_1e8_vs_oracle():
    """1e8 draws (382 generators) of the parallel stream == the oracle's
    serial MT19937, and the final state == the serial GPU kernel's."""
    n = 100_000_000
    st = codec.mt19937_seed_state(1234)
    sd = torch.from_numpy(st.view(np.int32)).to(DEV)
    s2 = sd.clone()
    a = codec.mt19937_generate(sd, n)
    assert bits_eq(u32(a), O.MT19937(1234).draws(n))
    del a
    codec.mt19937_generate(s2, n, parallel=False)
    assert torch.equal(sd, s2)


@pytest.mark.parametrize("name", ["qsgd_b4_1e6_k0", "qsgd_b8_1e6_k1"])
def test_large_digest_torch_mode(name):
    import hashlib

    meta = json.load(open(os.path.join(GOLD, "golden.json")))["digests"][name]
    x = O.gen_input(meta["n"], seed=42, kind=meta["kind"])
    gcodec.set_rng_mode("torch")
    try:
        torch.manual_seed(42)
        xd = dev(x)
        norm = codec.absmax(xd)
        c = gcodec.QSGDMaxNormCompressor(DEV, meta["bits"])
        q = c.compress(norm, xd)
        assert hashlib.sha256(q.cpu().numpy().tobytes()).hexdigest() == meta["q"]
        d = c.decompress(norm, q)
        assert hashlib.sha256(d.cpu().numpy().tobytes()).hexdigest() == meta["dec"]
    finally:
        gcodec.set_rng_mode(gcodec.rng.DEFAULT_MODE)


# --------------------------------------------------------------------------- two-/multi-scale
@pytest.mark.parametrize("lohi", [(2, 4), (4, 8), (2, 6), (6, 10)])
def test_two_scale_facade_matches_reference(lohi):
    lo, hi = lohi
    z = gz("multiscale.npz")
    c = f"ts{lo}_{hi}"
    x, norm = z[f"{c}/x"], z[f"{c}/norm"]
    gcodec.set_rng_mode("torch")
    try:
        torch.manual_seed(int(z[f"{c}/seed"]))
        comp = gcodec.QSGDMaxNormTwoScaleCompressor(DEV, lo, hi)
        nt = torch.tensor(norm, device=DEV)
        q_lo = comp.compress_lower(nt, dev(x))
        q_hi, h = comp.compress_higher(nt, dev(x))
        assert bits_eq(q_lo.cpu().numpy(), z[f"{c}/q_lo"])
        assert bits_eq(q_hi.cpu().numpy(), z[f"{c}/q_hi"])
        assert bits_eq(h.cpu().numpy(), z[f"{c}/h"])
        q = h * q_hi + (1 - h) * q_lo
        assert bits_eq(q.cpu().numpy(), z[f"{c}/q"])
        d = comp.decompress(nt, q, h)
        assert bits_eq(u32(d), z[f"{c}/dec"].view(np.uint32))
    finally:
        gcodec.set_rng_mode(gcodec.rng.DEFAULT_MODE)


@pytest.mark.parametrize("levels", [(2, 4), (4, 8), (2, 4, 6), (3, 5, 7, 9), (6, 10)])
def test_multi_scale_facade_matches_reference(levels):
    z = gz("multiscale.npz")
    c = "ms" + "_".join(map(str, levels))
    x, norm = z[f"{c}/x"], z[f"{c}/norm"]
    gcodec.set_rng_mode("torch")
    try:
        torch.manual_seed(int(z[f"{c}/seed"]))
        comp = gcodec.QSGDMaxNormMultiScaleCompressor(DEV, list(levels))
        nt = torch.tensor(norm, device=DEV)
        mask = comp.compress_mask(nt, dev(x))
        assert bits_eq(mask.cpu().numpy(), z[f"{c}/mask"])
        q = comp.compress(mask)
        assert bits_eq(q.cpu().numpy(), z[f"{c}/q"])
        d = comp.decompress(nt, q, mask)
        assert bits_eq(u32(d), z[f"{c}/dec"].view(np.uint32))
    finally:
        gcodec.set_rng_mode(gcodec.rng.DEFAULT_MODE)


@pytest.mark.parametrize("levels", [(2, 4), (4, 8), (2, 4, 6), (3, 5, 7, 9)])
@pytest.mark.parametrize("world", [1, 3, 8])
@pytest.mark.parametrize("n", [5, 4099, 300_001])
def test_ms_packed_vs_oracle(levels, world, n):
    """mask thermometer lanes + select + decode, Philox, vs the oracle."""
    x = O.gen_input(n, seed=n + world, kind=1)
    norm = O.absmax(x)
    L = len(levels)
    r = gcodec.rng.Reservation(0, 99, 11, None, n, L)
    xd = dev(x)
    mw = codec.ms_mask_encode(xd, float(norm), levels, r, world)
    m_ref = O.ms_mask(x, norm, levels, O.philox_rng(99, 11))
    # W identical ranks: the summed thermometer lanes decode to the same mask
    mw_sum = (mw.to(torch.int64) * world).to(torch.int32)
    got_mask = codec.ms_mask_unpack(mw_sum, n, levels, world)
    assert bits_eq(got_mask.cpu().numpy().astype(np.uint8), m_ref)
    words = codec.ms_select_encode(xd, float(norm), levels, r, mw_sum, world)
    q_ref = O.ms_select(x, norm, levels, O.philox_rng(99, 11), m_ref)
    ql, _ = codec.ms_layouts(n, levels, world)
    assert bits_eq(u32(words), O.lane_pack(q_ref, ql.offset, ql.bits, ql.per_word, ql.plane_words))
    wsum = (words.to(torch.int64) * world).to(torch.int32)
    for order in (0, 1):
        d = codec.ms_decode(wsum, mw_sum, n, float(norm), levels, world, order, 1.0)
        ref = O.ms_dequantize(q_ref * world, norm, levels, m_ref, order)
        assert bits_eq(u32(d), ref.view(np.uint32))


@pytest.mark.parametrize("levels", [(2, 4), (1, 3), (3, 7), (2, 4, 6), (1, 2, 3, 4, 5, 6, 7), (4, 8), (3, 10, 16)])
@pytest.mark.parametrize("world", [1, 2, 8])
def test_ms_fast_path_edges_vs_oracle(levels, world):
    """ms_fast.h (dense, levels <= 7 bits): integer rounding per level,
    multiply-high mask positions, Markstein order-0 decode — on adversarial
    values (level boundaries of every level, +-norm, +-0, subnormal tiles)
    and norms inside and outside the Markstein range, vs the oracle."""
    n = 7 * 4 * 4096 + 9
    L = len(levels)
    for norm0 in (np.float32(0.05), np.float32(3.0), np.float32(2.0**-110)):
        s = (1 << levels[-1]) - 1
        x = _int_path_input(n, norm0, s, seed=world * 7 + L)
        if len(levels) > 1:  # boundaries of the lowest level too
            s0 = (1 << levels[0]) - 1
            k = np.random.default_rng(L).integers(-s0, s0 + 1, n // 3).astype(np.float32)
            x[: n // 3] = np.clip((k * np.float32(norm0)) / np.float32(s0), -norm0, norm0)
        norm = O.absmax(x)
        r = gcodec.rng.Reservation(0, 313 + L, 2, None, n, L)
        xd = dev(x)
        mw = codec.ms_mask_encode(xd, float(norm), levels, r, world)
        m_ref = O.ms_mask(x, norm, levels, O.philox_rng(313 + L, 2))
        mw_sum = (mw.to(torch.int64) * world).to(torch.int32)
        assert bits_eq(codec.ms_mask_unpack(mw_sum, n, levels, world).cpu().numpy().astype(np.uint8), m_ref)
        words = codec.ms_select_encode(xd, float(norm), levels, r, mw_sum, world)
        q_ref = O.ms_select(x, norm, levels, O.philox_rng(313 + L, 2), m_ref)
        ql, _ = codec.ms_layouts(n, levels, world)
        assert bits_eq(u32(words), O.lane_pack(q_ref, ql.offset, ql.bits, ql.per_word, ql.plane_words))
        wsum = (words.to(torch.int64) * world).to(torch.int32)
        alpha = np.float32(1.0 / world)
        for order in (0, 1):
            d = codec.ms_decode(wsum, mw_sum, n, float(norm), levels, world, order, float(alpha))
            ref = O.ms_dequantize(q_ref * world, norm, levels, m_ref, order, alpha)
            assert bits_eq(u32(d), ref.view(np.uint32)), (order, float(norm))


@pytest.mark.parametrize("levels,cell", [((2, 4), 1), ((1, 3), 1), ((3, 7), 1), ((1, 2, 3), 2), ((2, 4, 6), 2),
                                         ((4, 7), 2), ((3, 4, 5), 2), ((5, 6, 7), 0), ((2, 8), 1), ((4, 8), 2),
                                         ((3, 9, 12), 2), ((2, 16), 1), ((6, 10), 2), ((9, 10), 0)])
@pytest.mark.parametrize("world", [1, 2, 8])
def test_ms_q_cache_vs_oracle(levels, cell, world):
    """q cache (compress_cache kept as packed cells): the cached mask kernel
    writes the same mask words, and the select from the cells equals the oracle
    at a COMMON mask below this rank's own levels (other ranks' inputs force
    lower levels), on level-boundary values, +-norm, zeros and subnormal tiles,
    inside and outside the Markstein range."""
    n = 3 * 4 * 4096 + 7
    assert codec.ms_cache_bytes(n, levels) == cell
    if not cell:
        return
    L = len(levels)
    for norm0 in (np.float32(0.05), np.float32(3.0), np.float32(2.0**-110)):
        s = (1 << levels[-1]) - 1
        x = _int_path_input(n, norm0, s, seed=world + 5 * L)
        s0 = (1 << levels[0]) - 1
        k = np.random.default_rng(L).integers(-s0, s0 + 1, n // 3).astype(np.float32)
        x[: n // 3] = np.clip((k * np.float32(norm0)) / np.float32(s0), -norm0, norm0)
        other = np.random.default_rng(world).permutation(x)  # another rank's bucket
        norm = max(O.absmax(x), O.absmax(other))
        r = gcodec.rng.Reservation(0, 71 + L, 4, None, n, L)
        r2 = gcodec.rng.Reservation(0, 72 + L, 4, None, n, L)
        xd = dev(x)
        cache = torch.empty(n * cell, dtype=torch.uint8, device=DEV)
        mw = codec.ms_mask_encode(xd, float(norm), levels, r, world, cache=cache)
        assert bits_eq(u32(mw), u32(codec.ms_mask_encode(xd, float(norm), levels, r, world)))
        mw_other = codec.ms_mask_encode(dev(other), float(norm), levels, r2, world)
        mw_sum = (mw.to(torch.int64) + mw_other.to(torch.int64) * (world - 1)).to(torch.int32)
        m_common = codec.ms_mask_unpack(mw_sum, n, levels, world).cpu().numpy().astype(np.uint8)
        m_own = O.ms_mask(x, norm, levels, O.philox_rng(71 + L, 4))
        assert np.all(m_common <= m_own)
        if world > 1:
            assert np.any(m_common < m_own)
        words = codec.ms_select_encode(xd, float(norm), levels, r, mw_sum, world, cache=cache)
        q_ref = O.ms_select(x, norm, levels, O.philox_rng(71 + L, 4), m_common)
        ql, _ = codec.ms_layouts(n, levels, world)
        assert bits_eq(u32(words), O.lane_pack(q_ref, ql.offset, ql.bits, ql.per_word, ql.plane_words))
        assert bits_eq(u32(words), u32(codec.ms_select_encode(xd, float(norm), levels, r, mw_sum, world)))


def test_ms_compressor_uses_q_cache():
    """the packed compressors take the cache path for cacheable levels and
    give the same words as with q_cache=False."""
    n = 100_003
    x = dev(O.gen_input(n, seed=3, kind=1))
    for cls, kw in ((gcodec.QSGDMaxNormTwoScaleCompressor, dict(lower_quantization_level=2,
                                                                 higher_quantization_level=4)),
                    (gcodec.QSGDMaxNormMultiScaleCompressor, dict(quantization_levels=[4, 2]))):
        out = []
        for qc in (True, False):
            c = cls(DEV, generator=gcodec.Generator(9, "philox"), q_cache=qc, **kw)
            norm = codec.absmax(x)
            m = c.encode_mask(norm, x, 2)
            assert (c._cache_key is not None) == qc
            out.append((u32(m), u32(c.encode(norm, x, (m.to(torch.int64) * 2).to(torch.int32), 2))))
        assert bits_eq(out[0][0], out[1][0]) and bits_eq(out[0][1], out[1][1])


# --------------------------------------------------------------------------- GRandK
@pytest.mark.parametrize("case",["n20011_k1000", "n5000_k5000", "n3001_k1000"])
def test_grandk_torch_mode_matches_reference(case):
    z = gz("randk.npz")
    buf, idx, norm, q = (z[f"{case}/{k}"] for k in ("buf", "idx", "norm", "q"))
    gcodec.set_rng_mode("torch")
    try:
        torch.manual_seed(int(z[f"{case}/seed"]))
        perm = torch.randperm(buf.size)  # consumes n-1 draws, like the reducer
        assert np.array_equal(list(perm.split(int(z[f"{case}/K"])))[-1].numpy(), idx)
        bd = dev(buf)
        nk = codec.absmax(bd, idx=dev(idx))
        assert nk.item() == float(norm)
        c = gcodec.GlobalRandKMaxNormCompressor(DEV, int(z[f"{case}/bits"]))
        qk = c.compress(nk, bd[dev(idx)])
        assert bits_eq(qk.cpu().numpy(), q)
    finally:
        gcodec.set_rng_mode(gcodec.rng.DEFAULT_MODE)


# --------------------------------------------------------------------------- packers
@pytest.mark.parametrize("n", [70_001, 96, 95, 400_003])
def test_lane_pack_unpack_kernels(n):
    """int8 / int32 q -> planar words (k_lane_pack4; k_lane_pack16 when the
    planes are 16-word aligned: n = 96 and 400,003 at W = 1) and back."""
    rng = np.random.default_rng(3)
    for world in (1, 2, 8):
        s = 15
        q = rng.integers(-s, s + 1, n).astype(np.int32)
        ln = codec.qsgd_layout(n, 4, world)
        for dt in (torch.int8, torch.int32):
            words = codec.lane_pack(dev(q).to(dt), ln)
            assert bits_eq(u32(words), O.lane_pack(q, s, ln.bits, ln.per_word, ln.plane_words))
        back = codec.lane_unpack((words.to(torch.int64) * world).to(torch.int32), ln)
        assert np.array_equal(back.cpu().numpy(), q * world)


@pytest.mark.parametrize("shift", [1, 2, 3])
def test_lane_pack_misaligned_q(shift):
    """q slices at every misalignment of the vector loads (int8 4 B, int32 16 B)
    take the scalar-load kernel; misaligned words are refused (GC_EINVAL)."""
    n, s = 70_001, 15
    q = np.random.default_rng(shift).integers(-s, s + 1, n + shift).astype(np.int32)
    ln = codec.qsgd_layout(n, 4, 1)
    exp = O.lane_pack(q[shift:], s, ln.bits, ln.per_word, ln.plane_words)
    for dt in (torch.int8, torch.int32):
        qd = dev(q).to(dt)[shift:]
        assert qd.data_ptr() % (4 if dt == torch.int8 else 16)
        assert bits_eq(u32(codec.lane_pack(qd, ln)), exp)
    wbuf = torch.empty(ln.plane_words + 4, dtype=torch.int32, device=DEV)
    with pytest.raises(gcodec.GCodecError):
        codec.lane_pack(dev(q[:n]).to(torch.int8), ln, out=wbuf[shift:])


def test_bytepack_kernels_match_reference_vectors():
    p = os.path.join(GOLD, "packers.npz")
    if not os.path.exists(p):
        pytest.skip("no packer fixtures")
    z = gz("packers.npz")
    for nm in sorted({k.split("/")[1] for k in z.files if k.startswith("bp/")}):
        src = z[f"bp/{nm}/src"]
        w = codec.bytepack8(dev(src))
        assert bits_eq(w.cpu().numpy(), z[f"bp/{nm}/packed"])
        assert bits_eq(codec.byteunpack8(w).cpu().numpy(), z[f"bp/{nm}/unpacked"])


@pytest.mark.parametrize("dt", [torch.int8, torch.int32, torch.int64])
@pytest.mark.parametrize("n,shift", [(16, 0), (17, 0), (33, 0), (1_000_003, 0), (23_520_842, 0), (1001, 1), (4099, 3)])
def test_bytepack_vector_and_scalar_paths_match_host(dt, n, shift):
    """The 16-byte vector kernels (aligned src / out) and the scalar kernels
    (shifted src) against the host byte packer (Extension CPU BP/bytepacking.cpp:6-64
    restated, pinned by the reference vectors in test_capi), for int8 / int32 /
    int64 sources, ragged n, and the ResNet50 bucket size."""
    from gcodec.packing import bytepacking
    rng = np.random.default_rng(n + shift)
    a = rng.integers(-300, 300, n + shift).astype(np.int64)
    src = torch.from_numpy(a).to(dt)
    d = src.to(DEV)[shift:]
    host = bytepacking.packing(src[shift:].to(torch.int64))
    w = codec.bytepack8(d)
    assert torch.equal(w.cpu(), host)
    u = codec.byteunpack8(w)
    assert torch.equal(u.cpu(), bytepacking.unpacking(host))
    if shift == 0:  # unpack into a shifted (8-byte aligned) output: the scalar path
        out = torch.empty(8 * w.numel() + 8, dtype=torch.int8, device=DEV)[8:]
        from gcodec import _lib
        import ctypes as C
        assert _lib.load().gc_byteunpack8(C.c_void_p(w.data_ptr()), w.numel(), C.c_void_p(out.data_ptr()),
                                          codec._stream(DEV)) == 0
        assert torch.equal(out.cpu(), u.cpu())


# --------------------------------------------------------------------------- full-size properties
def test_full_size_properties_100m():
    """BASELINE config 2 size: no oracle run at 1e8; size-independent checks —
    |decode - x| <= norm/s, lanes within range, unbiasedness, determinism."""
    n, bits = 100_000_000, 4
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(n, device=DEV, generator=g).mul_(0.01)
    norm = codec.absmax(x)
    assert norm.item() == x.abs().max().item()
    r = gcodec.rng.Reservation(0, 42, 0, None, n, 1)
    w1 = codec.qsgd_encode(x, norm, bits, r, 1)
    w2 = codec.qsgd_encode(x, norm, bits, r, 1)
    assert torch.equal(w1, w2)  # launch-invariant counter RNG
    d = codec.qsgd_decode(w1, n, norm, bits, 1)
    step = norm.item() / 15
    err = (d - x).abs().max().item()
    assert err <= step * (1 + 1e-6)
    bias = (d - x).double().mean().item()
    assert abs(bias) < 5 * step / np.sqrt(n)
    lanes = codec.lane_unpack(w1, codec.qsgd_layout(n, bits, 1))
    assert lanes.min().item() >= -15 and lanes.max().item() <= 15
    # chunk of the full bucket against the oracle (same counters)
    k0 = 64 * 1000
    xs = x[:k0].cpu().numpy()
    q_ref = O.qsgd_quantize(xs, np.float32(norm.item()), bits, O.philox_rng(42, 0))
    assert np.array_equal(lanes[:k0].cpu().numpy(), q_ref)


# --------------------------------------------------------------------------- chunked pipeline
@pytest.mark.parametrize("chunks", [1, 3, 7])
def test_chunked_pipeline_world1(chunks):
    """torch mode: chunked == unchunked bit for bit; Philox mode: every chunk
    equals the oracle's encode/decode of that chunk."""
    n, bits = 1_000_003, 4
    x = O.gen_input(n, seed=21, kind=1)
    xd = dev(x)
    gcodec.set_rng_mode("torch")
    try:
        torch.manual_seed(3)
        c = gcodec.QSGDMaxNormCompressor(DEV, bits)
        norm = codec.absmax(xd)
        ref = c.decode(norm, c.encode(norm, xd), n)
        torch.manual_seed(3)
        pipe = gcodec.ChunkedQSGDAllReduce(n, bits, DEV, chunks=chunks)
        got = pipe(xd)
        torch.cuda.synchronize()
        assert bits_eq(u32(got), u32(ref))
    finally:
        gcodec.set_rng_mode(gcodec.rng.DEFAULT_MODE)
    gen = gcodec.Generator(99, "philox")
    pipe = gcodec.ChunkedQSGDAllReduce(n, bits, DEV, chunks=chunks, generator=gen)
    got = pipe(xd).cpu().numpy()
    nh = O.absmax(x)
    off = 0
    for s, e in pipe.bounds:
        w = O.qsgd_encode(x[s:e], nh, bits, 1, O.philox_rng(99, off))
        assert bits_eq(got[s:e], O.qsgd_decode(w, e - s, nh, bits, 1))
        off += e - s


# --------------------------------------------------------------------------- config 5: 8-bit chunked, full size
class _IdenticalRanks(gcodec.ChunkedQSGDAllReduce):
    """W identical ranks on one GPU: the SUM of W equal packed streams is W
    times the stream (the lanes are sized for W, so nothing carries), and the
    MAX of W equal norms is the norm.  Exercises the W-dependent lane layout
    (8-bit at W = 8: 12-bit lanes, 2 per word) through the product pipeline."""

    def _max(self, norm):
        pass

    def _reduce(self, words):
        words.mul_(self.world)
        return None


def _unchunked_reduce(x, bits, world, rng):
    """encode the whole bucket, SUM of `world` identical ranks, decode * 1/W"""
    n = x.numel()
    norm = codec.absmax(x)
    w = codec.qsgd_encode(x, norm, bits, rng, world)
    w.mul_(world)
    return codec.qsgd_decode(w, n, norm, bits, world, 1.0 / world)


def _check_chunk_heads(pipe, x, out, bits, world, seed, k=1 << 16):
    """Philox mode: chunk c draws at offset = its start; the head of every
    chunk equals the oracle's quantize -> W-sum -> dequantize bit for bit."""
    s_ = (1 << bits) - 1
    norm = np.float32(codec.absmax(x).item())
    alpha = np.float32(1.0 / world)
    for s, e in pipe.bounds:
        m = min(k, e - s)
        xs = x[s:s + m].cpu().numpy()
        q = O.qsgd_quantize(xs, norm, bits, O.philox_rng(seed, s))
        assert np.all(np.abs(q) <= s_)
        exp = O.qsgd_dequantize(q * world, norm, bits, alpha)
        assert bits_eq(u32(out[s:s + m]), exp.view(np.uint32)), (s, e)


@pytest.mark.parametrize("world", [1, 8])
def test_config5_chunked_8bit_1e8(world):
    """BASELINE config 5's pipeline (8-bit, 8 chunks) at n = 1e8 + 3 with the
    lane layouts of W = 1 (9-bit lanes x3) and W = 8 (12-bit lanes x2):
    torch mode: chunked == unchunked bit for bit (draws consumed in element
    order); Philox mode: every chunk's head == the oracle."""
    n, bits, chunks = 100_000_003, 8, 8
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(n, device=DEV, generator=g).mul_(0.01)
    gcodec.set_rng_mode("torch")
    try:
        torch.manual_seed(17)
        ref = _unchunked_reduce(x, bits, world, gcodec.rng.default_generator.reserve(n, 1, device=DEV))
        torch.manual_seed(17)
        pipe = _IdenticalRanks(n, bits, DEV, chunks=chunks, world=world)
        assert pipe.lanes[0].bits == (9 if world == 1 else 12)
        got = pipe(x)
        torch.cuda.synchronize()
        assert torch.equal(got.view(torch.int32), ref.view(torch.int32))
    finally:
        gcodec.set_rng_mode(gcodec.rng.DEFAULT_MODE)
    pipe = _IdenticalRanks(n, bits, DEV, chunks=chunks, world=world, generator=gcodec.Generator(99, "philox"))
    out = pipe(x)
    torch.cuda.synchronize()
    _check_chunk_heads(pipe, x, out, bits, world, 99)


def test_config5_chunked_8bit_1e9_properties():
    """config 5 at its full size, 1e9 fp32, 8-bit, W = 8 lanes, 8 chunks:
    size-independent properties (|dec - x| <= norm/s, unbiased, launch
    invariant) plus every chunk's head vs the oracle."""
    n, bits, world = 1_000_000_000, 8, 8
    g = torch.Generator(device=DEV).manual_seed(9)
    x = torch.randn(n, device=DEV, generator=g).mul_(0.01)
    pipe = _IdenticalRanks(n, bits, DEV, chunks=8, world=world, generator=gcodec.Generator(7, "philox"))
    out = pipe(x)
    pipe2 = _IdenticalRanks(n, bits, DEV, chunks=8, world=world, generator=gcodec.Generator(7, "philox"))
    assert torch.equal(pipe2(x), out)
    del pipe2
    torch.cuda.synchronize()
    step = codec.absmax(x).item() / 255
    d = out - x
    assert d.abs().max().item() <= step * (1 + 1e-6)
    assert abs(d.double().mean().item()) < 5 * step / np.sqrt(n)
    del d
    _check_chunk_heads(pipe, x, out, bits, world, 7, k=1 << 14)


# --------------------------------------------------------------------------- multi-scale large-plane layout
@pytest.mark.parametrize("name", ["ms_2_4_1e6", "ms_4_8_1e6"])
def test_ms_large_digest_torch_mode(name):
    """The reference's 1e6-element multi-scale digests (q planes of >= 65536
    words: the 64-word plane alignment) through the unpacked facade AND the
    packed mask -> select -> decode path, torch-mode draws."""
    import hashlib

    def sha(a):
        return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()

    meta = json.load(open(os.path.join(GOLD, "golden.json")))["digests"][name]
    lv = meta["levels"]
    x = O.gen_input(meta["n"], seed=42, kind=meta["kind"])
    xd = dev(x)
    qdt = np.int8 if lv[0] < 8 else np.int32
    gcodec.set_rng_mode("torch")
    try:
        torch.manual_seed(42)
        norm = codec.absmax(xd)
        assert norm.item() == meta["norm"]
        c = gcodec.QSGDMaxNormMultiScaleCompressor(DEV, list(lv))
        mask = c.compress_mask(norm, xd)
        assert sha(mask.cpu().numpy()) == meta["mask"]
        q = c.compress(mask)
        assert sha(q.cpu().numpy()) == meta["q"]
        assert sha(c.decompress(norm, q, mask).cpu().numpy()) == meta["dec"]
        # packed: thermometer mask lanes, planar q lanes, fused decode
        torch.manual_seed(42)
        cp = gcodec.QSGDMaxNormMultiScaleCompressor(DEV, list(lv))
        mw = cp.encode_mask(norm, xd)
        ql, ml = codec.ms_layouts(x.size, lv, 1)
        assert ql.plane_words % 64 == 0 and -(-x.size // ql.per_word) >= 65536
        assert sha(codec.ms_mask_unpack(mw, x.size, lv).cpu().numpy()) == meta["mask"]
        words = cp.encode(norm, xd, mw)
        qp = codec.lane_unpack(words, ql).cpu().numpy().astype(qdt)
        assert sha(qp) == meta["q"]
        assert sha(cp.decode(norm, words, mw, x.size).cpu().numpy()) == meta["dec"]
    finally:
        gcodec.set_rng_mode(gcodec.rng.DEFAULT_MODE)


@pytest.mark.parametrize("levels", [(2, 4), (4, 8)])
@pytest.mark.parametrize("world", [1, 2])
def test_ms_resnet50_bucket_vs_oracle(levels, world):
    """BASELINE config 3's bucket (n = 23,520,842, planes of 64-word
    alignment, mask planes > 65536 words) with Philox draws: mask, select at
    the common levels of two ranks (W = 2), and both decode orders (two-scale
    order 1, multi-scale order 0) vs the oracle, bit for bit."""
    n = 23_520_842
    L = len(levels)
    x = O.gen_input(n, seed=L + world, kind=1)
    xs = [x] + [np.random.default_rng(world).permutation(x) for _ in range(world - 1)]
    norm = max(O.absmax(v) for v in xs)
    rngs = [gcodec.rng.Reservation(0, 31 + r, 3, None, n, L) for r in range(world)]
    ql, ml = codec.ms_layouts(n, levels, world)
    assert ql.plane_words % 64 == 0
    mws = [codec.ms_mask_encode(dev(v), float(norm), levels, rngs[r], world) for r, v in enumerate(xs)]
    masks = [O.ms_mask(v, norm, levels, O.philox_rng(31 + r, 3)) for r, v in enumerate(xs)]
    for r in range(world):  # each rank's own levels (its lanes times W: W identical ranks)
        own = codec.ms_mask_unpack((mws[r].to(torch.int64) * world).to(torch.int32), n, levels, world)
        assert bits_eq(own.cpu().numpy().astype(np.uint8), masks[r])
    mw_sum = sum(m.to(torch.int64) for m in mws).to(torch.int32)
    common = np.minimum.reduce(masks)
    assert bits_eq(codec.ms_mask_unpack(mw_sum, n, levels, world).cpu().numpy().astype(np.uint8), common)
    words = [codec.ms_select_encode(dev(v), float(norm), levels, rngs[r], mw_sum, world) for r, v in enumerate(xs)]
    qs = [O.ms_select(v, norm, levels, O.philox_rng(31 + r, 3), common) for r, v in enumerate(xs)]
    assert bits_eq(u32(words[0]), O.lane_pack(qs[0], ql.offset, ql.bits, ql.per_word, ql.plane_words))
    wsum = sum(w.to(torch.int64) for w in words).to(torch.int32)
    qsum = sum(q.astype(np.int64) for q in qs).astype(np.int32)
    alpha = np.float32(1.0 / world)
    for order in (0, 1):
        d = codec.ms_decode(wsum, mw_sum, n, float(norm), levels, world, order, float(alpha))
        assert bits_eq(u32(d), O.ms_dequantize(qsum, norm, levels, common, order, alpha).view(np.uint32)), order


@pytest.mark.parametrize("n", [1, 1000, 65_536, 69_633, 300_007, 1_000_003, 4_000_037, 26_000_011])
def test_absmax_workspace_reuse_many_grids(n):
    """The last-block hand-off of k_absmax (sc1 partials + two levels of
    agent-scope tickets, include/gcodec.h) over grids of 1, 16, 17, 74, 245
    and 512 blocks (groups of one block, full groups, a ragged last group),
    the self-resetting workspace reused 50 times on one stream, every result
    vs the oracle."""
    x = O.gen_input(n, seed=n, kind=1)
    x[(n * 7) // 11] = np.float32(-0.75)  # a unique maximum somewhere inside
    xd = dev(x)
    out = torch.empty(50, dtype=torch.float32, device=DEV)
    for i in range(50):
        codec.absmax(xd, out=out[i:i + 1])
    assert np.all(out.cpu().numpy() == O.absmax(x))


# --------------------------------------------------------------------------- small-K GlobalRandK (config 4)
@pytest.mark.parametrize("bits", [1, 2, 4, 8])
@pytest.mark.parametrize("K", [1, 3, 1000, 10_000, 16_384])
def test_randk_fused_w1_vs_oracle(bits, K):
    """gc_randk_encode_w1: gather + max-norm + encode in one launch (W = 1) ==
    the oracle's encode of x[idx] with max |x[idx]|; the subset and the norm
    are written too."""
    n = 300_007
    x = O.gen_input(n, seed=K + 17 * bits, kind=K % 2)
    idx = np.random.default_rng(K).permutation(n)[:K].astype(np.int64)
    r = gcodec.rng.Reservation(0, 23 + bits, 7 * K, None, K, 1)
    xk = torch.empty(K, dtype=torch.float32, device=DEV)
    words, norm = codec.randk_encode_w1(dev(x), dev(idx), bits, r, xk=xk)
    nk = O.absmax(x[idx])
    assert norm.item() == float(nk)
    assert bits_eq(u32(xk), x[idx].view(np.uint32))
    assert bits_eq(u32(words), O.qsgd_encode(x[idx], nk, bits, 1, O.philox_rng(23 + bits, 7 * K)))


def test_randk_fused_w1_torch_stream_and_edges():
    """the fused kernel with caller draws (torch-mode stream), NaN / +-inf /
    zero subsets vs the oracle, and the ticket re-armed across many calls"""
    n, K, bits = 50_021, 10_000, 4
    x = O.gen_input(n, seed=5, kind=1)
    idx = np.random.default_rng(2).permutation(n)[:K].astype(np.int64)
    draws = O.MT19937(9).draws(K)
    rs = gcodec.rng.Reservation(1, 0, 0, dev(draws.view(np.int32)), K, 1)
    words, norm = codec.randk_encode_w1(dev(x), dev(idx), bits, rs)
    nk = O.absmax(x[idx])
    assert bits_eq(u32(words), O.qsgd_encode(x[idx], nk, bits, 1, O.stream_rng(draws)))
    xz = np.zeros(n, np.float32)
    w0, n0 = codec.randk_encode_w1(dev(xz), dev(idx), bits, gcodec.rng.Reservation(0, 1, 0, None, K, 1))
    assert n0.item() == 0.0
    assert bits_eq(u32(w0), O.qsgd_encode(xz[idx], np.float32(0), bits, 1, O.philox_rng(1, 0)))
    x2 = x.copy()
    x2[idx[17]] = np.inf
    x2[idx[9000]] = np.nan
    for i in range(30):  # many launches on one workspace (self-resetting ticket)
        w2, n2 = codec.randk_encode_w1(dev(x2), dev(idx), bits, gcodec.rng.Reservation(0, 3, i, None, K, 1))
    assert np.isnan(n2.item())
    assert bits_eq(u32(w2), O.qsgd_encode(x2[idx], np.float32(np.nan), bits, 1, O.philox_rng(3, 29)))


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("K", [7, 10_000, 262_144])
def test_randk_gather_then_dense_encode(world, K):
    """W > 1 path: gc_randk_gather_absmax (subset + local norm, one launch),
    then the dense encode of the subset == the gather encode through idx ==
    the oracle; and the one-element-per-thread decode-scatter."""
    n = 1_000_003
    x = O.gen_input(n, seed=K + world, kind=1)
    idx = np.random.default_rng(K + 1).permutation(n)[:K].astype(np.int64)
    xd, idd = dev(x), dev(idx)
    xk, nk = codec.randk_gather_absmax(xd, idd)
    assert bits_eq(u32(xk), x[idx].view(np.uint32))
    assert nk.item() == float(O.absmax(x[idx]))
    r = gcodec.rng.Reservation(0, 4, 11, None, K, 1)
    wd = codec.qsgd_encode(xk, nk, 4, r, world)
    assert torch.equal(wd, codec.qsgd_encode(xd, nk, 4, r, world, idx=idd))
    ref = O.qsgd_encode(x[idx], O.absmax(x[idx]), 4, world, O.philox_rng(4, 11))
    assert bits_eq(u32(wd), ref)
    wsum = (wd.to(torch.int64) * world).to(torch.int32)
    out = dev(x)
    codec.qsgd_decode(wsum, K, nk, 4, world, 1.0 / world, idx=idd, out=out)
    exp = x.copy()
    refsum = (ref.astype(np.uint64) * world).astype(np.uint32)
    exp[idx] = O.qsgd_decode(refsum, K, O.absmax(x[idx]), 4, world, np.float32(1.0 / world))
    assert bits_eq(u32(out), exp.view(np.uint32))


def test_randk_step_matches_codec_calls():
    """codec.RandKStep (pre-resolved pointers, one ctypes call per launch) ==
    the plain codec calls, step after step (draw offsets advance by K)."""
    n, K, bits = 14_728_266, 10_000, 4
    g = torch.Generator(device=DEV).manual_seed(12)
    x = torch.randn(n, device=DEV, generator=g).mul_(0.01)
    idx = torch.randperm(n, generator=torch.Generator().manual_seed(42))[:K].to(DEV)
    ga, gb = gcodec.Generator(5, "philox"), gcodec.Generator(5, "philox")
    step = codec.RandKStep(x, K, bits, ga)
    out_a, out_b = x.clone(), x.clone()
    for _ in range(3):
        wa, na = step.encode(idx)
        wb, nb = codec.randk_encode_w1(x, idx, bits, gb.reserve(K))
        assert torch.equal(wa, wb) and torch.equal(na, nb)
        step.decode(wa, idx, out_a, 1.0)
        codec.qsgd_decode(wb, K, nb, bits, 1, 1.0, idx=idx, out=out_b)
        assert torch.equal(out_a, out_b)
    assert ga.offset == gb.offset == 3 * K
    xk, nk = step.gather(idx)
    w2 = step.encode_gathered()
    assert torch.equal(w2, codec.qsgd_encode(x, nk, bits, gcodec.rng.Reservation(0, 5, 3 * K, None, K, 1), 1,
                                             idx=idx))


# --------------------------------------------------------------------------- QSGDBP call site (a14)
def test_qsgdbp_compressor_matches_reference_vectors():
    """gcodec.QSGDBPCompressor (compressors.py:324-378): device quantize into
    sign bits + magnitudes, device greedy 4-mode packing, unpack + truncate +
    sign map — against vectors made with the reference's quantizer and its own
    compiled bitpacking extension (tests/golden/make_golden_bp.py), torch mode."""
    z = gz("qsgdbp.npz")
    cases = sorted({k.split("/")[0] for k in z.files})
    gcodec.set_rng_mode("torch")
    try:
        for c in cases:
            x, bits = z[f"{c}/x"], int(z[f"{c}/bits"])
            torch.manual_seed(int(z[f"{c}/seed"]))
            comp = gcodec.QSGDBPCompressor(DEV, bits)
            norm_s, sp, xp, size = comp.compress(dev(x))
            assert norm_s.item() == float(z[f"{c}/norm_over_s"]), c
            assert bits_eq(sp.cpu().numpy(), z[f"{c}/sign_packed"]), c
            assert bits_eq(xp.cpu().numpy(), z[f"{c}/xi_packed"]), c
            assert int(size.item()) == int(z[f"{c}/xi_size"])
            d = comp.decompress(norm_s, sp, xp, x.size)
            assert bits_eq(u32(d), z[f"{c}/dec"].view(np.uint32)), c
    finally:
        gcodec.set_rng_mode(gcodec.rng.DEFAULT_MODE)


# --------------------------------------------------------------------------- one-pass W = 1 multi-scale
@pytest.mark.parametrize("levels", [(2, 4), (1, 3), (3, 7), (2, 4, 6), (1, 2, 3), (4, 7), (4, 8), (2, 8), (6, 10),
                                    (3, 10, 16)])
@pytest.mark.parametrize("n", [5, 4099, 7 * 4 * 4096 + 9, 300_001])
def test_ms_encode_w1_matches_two_pass_and_oracle(levels, n):
    """gc_ms_encode_w1 (mask + select in one pass, coupled W = 1 layouts) ==
    gc_ms_mask_encode + gc_ms_select_encode bit for bit, == the oracle, on
    level-boundary values, +-norm, zeros and subnormal tiles, with norms inside
    and outside the Markstein range (the generic per-element branch)."""
    L = len(levels)
    for norm0 in (np.float32(0.05), np.float32(2.0**-110)):
        s = (1 << levels[-1]) - 1
        x = _int_path_input(n, norm0, s, seed=n % 1000 + 7 * L)
        if n > 3:
            s0 = (1 << levels[0]) - 1
            k = np.random.default_rng(L).integers(-s0, s0 + 1, n // 3).astype(np.float32)
            x[: n // 3] = np.clip((k * np.float32(norm0)) / np.float32(s0), -norm0, norm0)
        norm = O.absmax(x)
        r = gcodec.rng.Reservation(0, 17 + L, 9, None, n, L)
        xd = dev(x)
        assert codec.ms_w1_ok(xd, levels)
        mw, words = codec.ms_encode_w1(xd, float(norm), levels, r)
        mw2 = codec.ms_mask_encode(xd, float(norm), levels, r, 1)
        assert torch.equal(mw, mw2), (levels, n, float(norm))
        assert torch.equal(words, codec.ms_select_encode(xd, float(norm), levels, r, mw2, 1))
        m_ref = O.ms_mask(x, norm, levels, O.philox_rng(17 + L, 9))
        assert bits_eq(codec.ms_mask_unpack(mw, n, levels, 1).cpu().numpy().astype(np.uint8), m_ref)
        q_ref = O.ms_select(x, norm, levels, O.philox_rng(17 + L, 9), m_ref)
        ql, ml = codec.ms_layouts(n, levels, 1)
        assert ql.plane_words == (32 // ql.per_word) * ml.plane_words  # the coupled layouts
        assert bits_eq(u32(words), O.lane_pack(q_ref, ql.offset, ql.bits, ql.per_word, ql.plane_words))


@pytest.mark.parametrize("levels", [(2, 4), (4, 8), (2, 4, 6)])
def test_ms_encode_w1_non_finite_given_norm(levels):
    """the one-pass encode with a caller's finite norm below max |x| and NaN,
    +-inf, |x| > norm, subnormal, tiny and -0 inputs scattered over the bucket
    (v_cvt_flr_i32_f32 turns a NaN into INT_MIN, so a NaN must take the
    generic branch: the range check catches it) == the two-pass kernels ==
    the oracle."""
    n = 7 * 4 * 4096 + 9
    L = len(levels)
    x = O.gen_input(n, seed=21)
    x[::997] = np.nan
    x[5::1001] = np.inf
    x[7::1003] = -np.inf
    x[11::889] = np.float32(3e-41)
    x[13::883] = np.float32(-1e-35)
    x[19::773] = 0.25
    x[23::71] = -0.0
    norm = np.float32(np.nanmax(np.abs(x[np.isfinite(x)])) / 4)
    r = gcodec.rng.Reservation(0, 5 + L, 3, None, n, L)
    xd = dev(x)
    mw, words = codec.ms_encode_w1(xd, float(norm), levels, r)
    mw2 = codec.ms_mask_encode(xd, float(norm), levels, r, 1)
    assert torch.equal(mw, mw2)
    assert torch.equal(words, codec.ms_select_encode(xd, float(norm), levels, r, mw2, 1))
    m_ref = O.ms_mask(x, norm, levels, O.philox_rng(5 + L, 3))
    assert bits_eq(codec.ms_mask_unpack(mw, n, levels, 1).cpu().numpy().astype(np.uint8), m_ref)
    q_ref = O.ms_select(x, norm, levels, O.philox_rng(5 + L, 3), m_ref)
    ql, _ = codec.ms_layouts(n, levels, 1)
    # |x| > norm: the lanes saturate at +-qmax (DESIGN §2 divergences; the
    # reference's unpacked q would hold the unclamped value)
    q_ref = np.clip(q_ref, -int(ql.offset), int(ql.offset))
    assert bits_eq(u32(words), O.lane_pack(q_ref, ql.offset, ql.bits, ql.per_word, ql.plane_words))


@pytest.mark.parametrize("name", ["ms_2_4_1e6", "ms_4_8_1e6"])
def test_ms_encode_w1_torch_mode_digests(name):
    """the one-pass W = 1 encode with torch-mode draws (caller stream, KIND 1)
    reproduces the reference's 1e6-element multi-scale digests"""
    import hashlib

    meta = json.load(open(os.path.join(GOLD, "golden.json")))["digests"][name]
    lv = meta["levels"]
    x = O.gen_input(meta["n"], seed=42, kind=meta["kind"])
    xd = dev(x)
    gcodec.set_rng_mode("torch")
    try:
        torch.manual_seed(42)
        norm = codec.absmax(xd)
        c = gcodec.QSGDMaxNormMultiScaleCompressor(DEV, list(lv))
        mw, words = c.encode_w1(norm, xd)
        m = codec.ms_mask_unpack(mw, x.size, lv).cpu().numpy()
        assert hashlib.sha256(m.tobytes()).hexdigest() == meta["mask"]
        ql, _ = codec.ms_layouts(x.size, lv, 1)
        q = codec.lane_unpack(words, ql).cpu().numpy().astype(np.int8 if lv[0] < 8 else np.int32)
        assert hashlib.sha256(q.tobytes()).hexdigest() == meta["q"]
        d = c.decode(norm, words, mw, x.size)
        assert hashlib.sha256(d.cpu().numpy().tobytes()).hexdigest() == meta["dec"]
    finally:
        gcodec.set_rng_mode(gcodec.rng.DEFAULT_MODE)
