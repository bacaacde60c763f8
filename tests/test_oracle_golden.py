"""The CPU oracle (oracle/gcodec_oracle.c) against the golden vectors the
REFERENCE itself produced (tests/golden/make_golden.py imports
compressors.py / reducer.py and the reference's C++ packers).  This pins the
oracle before any HIP result is compared with it."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def _cases(z):
    return sorted({k.split("/")[0] for k in z.files})


def _bits_eq(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    return a.shape == b.shape and a.tobytes() == b.tobytes()


def test_mt19937_matches_numpy_legacy_seeding():
    mt = np.random.MT19937(0)
    mt._legacy_seeding(42)
    assert np.array_equal(O.MT19937(42).draws(3000), mt.random_raw(3000).astype(np.uint32))


def test_mt19937_matches_torch_generator():
    torch = pytest.importorskip("torch")
    torch.manual_seed(1234)
    # torch.randint over [0, 2^32) is not a raw draw; use random_ on int64 with
    # the documented 32-bit path: bernoulli(0.5) consumes one draw/element.
    p = torch.full((5000,), 0.5)
    b = torch.bernoulli(p).numpy()
    u = (O.MT19937(1234).draws(5000) & 0xFFFFFF).astype(np.float32) * np.float32(2.0 ** -24)
    assert np.array_equal(b.astype(bool), u < np.float32(0.5))


@pytest.mark.parametrize("case", ["b2", "b4", "b8", "grk_b4", "n1", "n2", "n3", "n5", "n63", "n64", "n65", "n1000"])
def test_qsgd_quantize_dequantize(case):
    z = _load("qsgd.npz")
    x, norm, q, dec, bits = (z[f"{case}/{k}"] for k in ("x", "norm", "q", "dec", "bits"))
    bits = int(bits)
    rng = O.stream_rng(O.MT19937(int(z[f"{case}/seed"])).draws(x.size))
    qo = O.qsgd_quantize(x, norm, bits, rng)
    assert _bits_eq(qo.astype(q.dtype), q)  # int8 for b<8, int32 for b>=8 (compressors.py:294-297)
    deco = O.qsgd_dequantize(q.astype(np.int32), norm, bits)
    assert _bits_eq(deco, dec)


@pytest.mark.parametrize("lohi", [(2, 4), (4, 8), (2, 6), (6, 10)])
def test_two_scale(lohi):
    lo, hi = lohi
    z = _load("multiscale.npz")
    c = f"ts{lo}_{hi}"
    x, norm = z[f"{c}/x"], z[f"{c}/norm"]
    n = x.size
    draws = O.MT19937(int(z[f"{c}/seed"])).draws(2 * n)
    rng = O.stream_rng(draws)
    q_lo = O.qsgd_quantize(x, norm, lo, rng, level=0)
    q_hi = O.qsgd_quantize(x, norm, hi, rng, level=1)
    h = (np.abs(q_hi) <= (1 << lo) - 1).astype(np.int8)
    assert _bits_eq(q_lo.astype(z[f"{c}/q_lo"].dtype), z[f"{c}/q_lo"])
    assert _bits_eq(q_hi.astype(z[f"{c}/q_hi"].dtype), z[f"{c}/q_hi"])
    assert _bits_eq(h, z[f"{c}/h"])
    # multi-scale kernels with two levels give the same mask and integers
    mask = O.ms_mask(x, norm, [lo, hi], rng)
    assert np.array_equal(mask, h.astype(np.uint8))
    q = O.ms_select(x, norm, [lo, hi], rng, mask)
    assert _bits_eq(q.astype(z[f"{c}/q"].dtype), z[f"{c}/q"])
    dec = O.ms_dequantize(q, norm, [lo, hi], mask, order=1)
    assert _bits_eq(dec, z[f"{c}/dec"])


@pytest.mark.parametrize("levels", [(2, 4), (4, 8), (2, 4, 6), (3, 5, 7, 9), (6, 10)])
def test_multi_scale(levels):
    z = _load("multiscale.npz")
    c = "ms" + "_".join(map(str, levels))
    x, norm = z[f"{c}/x"], z[f"{c}/norm"]
    rng = O.stream_rng(O.MT19937(int(z[f"{c}/seed"])).draws(len(levels) * x.size))
    mask = O.ms_mask(x, norm, levels, rng)
    assert _bits_eq(mask.astype(np.int8), z[f"{c}/mask"])
    q = O.ms_select(x, norm, levels, rng, mask)
    assert _bits_eq(q.astype(z[f"{c}/q"].dtype), z[f"{c}/q"])
    dec = O.ms_dequantize(q, norm, levels, mask, order=0)
    assert _bits_eq(dec, z[f"{c}/dec"])


@pytest.mark.parametrize("case", ["n20011_k1000", "n5000_k5000", "n3001_k1000"])
def test_grandk(case):
    z = _load("randk.npz")
    buf, idx, norm, q, dec = (z[f"{case}/{k}"] for k in ("buf", "idx", "norm", "q", "dec"))
    n = buf.size
    mt = O.MT19937(int(z[f"{case}/seed"]))
    mt.draws(int(z[f"{case}/draws_before"]))  # torch.randperm(n): n-1 draws
    xk = buf[idx]
    assert O.absmax(xk) == norm
    qo = O.qsgd_quantize(xk, norm, int(z[f"{case}/bits"]), O.stream_rng(mt.draws(idx.size)))
    assert _bits_eq(qo.astype(q.dtype), q)
    assert _bits_eq(O.qsgd_dequantize(q.astype(np.int32), norm, int(z[f"{case}/bits"])), dec)


def test_randperm_is_fisher_yates_on_mt19937():
    """torch.randperm(n) (CPU, n < 2^32/20): swap i <-> i + r % (n - i)."""
    z = _load("randk.npz")
    case = "n3001_k1000"
    n = z[f"{case}/buf"].size
    r = O.MT19937(42).draws(n - 1).astype(np.int64)
    perm = np.arange(n, dtype=np.int64)
    for i in range(n - 1):
        j = i + int(r[i] % (n - i))
        perm[i], perm[j] = perm[j], perm[i]
    K = int(z[f"{case}/K"])
    chunks = [perm[i:i + K] for i in range(0, n, K)]
    assert np.array_equal(chunks[-1], z[f"{case}/idx"])
    assert np.array_equal(np.concatenate(chunks[:2]), z[f"{case}/perm_head"])


def test_absmax_golden():
    z = _load("qsgd.npz")
    for c in ("b4", "n1", "n65", "n1000"):
        assert O.absmax(z[f"{c}/x"]) == z[f"{c}/norm"]


@pytest.mark.parametrize("name", ["qsgd_b4_1e6_k0", "qsgd_b8_1e6_k1", "qsgd_b2_3e6_k0"])
def test_large_digests(name):
    meta = json.load(open(os.path.join(GOLD, "golden.json")))["digests"][name]
    x = O.gen_input(meta["n"], seed=42, kind=meta["kind"])
    assert hashlib.sha256(x.tobytes()).hexdigest() == meta["x"]
    norm = O.absmax(x)
    assert float(norm) == meta["norm"]
    q = O.qsgd_quantize(x, norm, meta["bits"], O.stream_rng(O.MT19937(42).draws(x.size)))
    qd = q.astype(np.int8 if meta["bits"] < 8 else np.int32)
    assert hashlib.sha256(qd.tobytes()).hexdigest() == meta["q"]
    dec = O.qsgd_dequantize(q, norm, meta["bits"])
    assert hashlib.sha256(dec.tobytes()).hexdigest() == meta["dec"]


@pytest.mark.parametrize("name", ["ms_2_4_1e6", "ms_4_8_1e6"])
def test_large_ms_digests(name):
    meta = json.load(open(os.path.join(GOLD, "golden.json")))["digests"][name]
    x = O.gen_input(meta["n"], seed=42, kind=meta["kind"])
    lv = meta["levels"]
    norm = O.absmax(x)
    rng = O.stream_rng(O.MT19937(42).draws(len(lv) * x.size))
    mask = O.ms_mask(x, norm, lv, rng)
    assert hashlib.sha256(mask.astype(np.int8).tobytes()).hexdigest() == meta["mask"]
    q = O.ms_select(x, norm, lv, rng, mask)
    assert hashlib.sha256(q.astype(np.int8 if lv[0] < 8 else np.int32).tobytes()).hexdigest() == meta["q"]
    dec = O.ms_dequantize(q, norm, lv, mask, order=0)
    assert hashlib.sha256(dec.tobytes()).hexdigest() == meta["dec"]


def _packer_cases(prefix):
    p = os.path.join(GOLD, "packers.npz")
    if not os.path.exists(p):
        pytest.skip("reference packers were unbuildable when fixtures were made")
    z = _load("packers.npz")
    return z, sorted({k.split("/")[1] for k in z.files if k.startswith(prefix + "/")})


def test_greedy4_known_answers():
    z, names = _packer_cases("g4")
    for nm in names:
        src = z[f"g4/{nm}/src"]
        assert _bits_eq(O.greedy4_pack(src), z[f"g4/{nm}/packed"]), nm
        assert _bits_eq(O.greedy4_unpack(z[f"g4/{nm}/packed"]), z[f"g4/{nm}/unpacked"]), nm


def test_bytepack_known_answers():
    z, names = _packer_cases("bp")
    for nm in names:
        src = z[f"bp/{nm}/src"]
        assert _bits_eq(O.bytepack8(src), z[f"bp/{nm}/packed"]), nm
        assert _bits_eq(O.byteunpack8(z[f"bp/{nm}/packed"]), z[f"bp/{nm}/unpacked"]), nm


def test_greedy4_rejects_out_of_domain():
    with pytest.raises(ValueError):
        O.greedy4_pack(np.array([1, 256], np.int32))
    with pytest.raises(ValueError):
        O.greedy4_pack(np.array([-1, 2], np.int32))


def test_lane_layout_examples():
    # 4-bit W=1 -> w=5, L=6; W=8 -> w=8; 8-bit W=8 -> w=12
    assert O.lane_layout(100, 30, 1)[:2] == (5, 6)
    assert O.lane_layout(100, 30, 8)[:2] == (8, 4)
    assert O.lane_layout(100, 510, 8)[:2] == (12, 2)


def test_lane_pack_roundtrip_and_sum_compat():
    rng = np.random.default_rng(0)
    for W in (1, 2, 3, 8):
        n, s = 1001, 15
        w, L, M = O.lane_layout(n, 2 * s, W)
        qs = [rng.integers(-s, s + 1, n).astype(np.int32) for _ in range(W)]
        words = [O.lane_pack(q, s, w, L, M) for q in qs]
        tot = np.zeros(M, np.uint64)
        for wd in words:
            tot += wd
        assert tot.max() < 2 ** 32
        got = O.lane_unpack(tot.astype(np.uint32), n, s, W, w, L, M)
        assert np.array_equal(got, np.sum(qs, axis=0))


def _bp_cases():
    z = _load("qsgdbp.npz")
    return z, sorted({k.split("/")[0] for k in z.files})


def test_qsgdbp_golden_vs_oracle():
    """The QSGDBP call site fixture (tests/golden/make_golden_bp.py: the
    reference's quantizer + its compiled greedy packer) restated by the
    oracle: MT19937 draws -> quantize -> sign bits / magnitudes -> greedy4."""
    z, cases = _bp_cases()
    assert cases
    for c in cases:
        x, bits = z[f"{c}/x"], int(z[f"{c}/bits"])
        norm = O.absmax(x)
        q = O.qsgd_quantize(x, norm, bits, O.stream_rng(O.MT19937(int(z[f"{c}/seed"])).draws(x.size)))
        sign = (x < 0).astype(np.int32)
        assert np.array_equal(O.greedy4_pack(sign), z[f"{c}/sign_packed"]), c
        assert np.array_equal(O.greedy4_pack(np.abs(q)), z[f"{c}/xi_packed"]), c
        assert int(z[f"{c}/xi_size"]) == z[f"{c}/xi_packed"].size
        s = (1 << bits) - 1
        assert np.float32(norm) / np.float32(s) == z[f"{c}/norm_over_s"]
        # (norm / s) * sign * xi with sign in {-1, +1}: a negative x that rounds to 0 gives -0.0
        sgn = np.where(sign == 1, np.float32(-1), np.float32(1))
        dec = (np.float32(norm) / np.float32(s) * sgn).astype(np.float32) * np.abs(q).astype(np.float32)
        assert dec.astype(np.float32).tobytes() == z[f"{c}/dec"].tobytes(), c


# ---------------------------------------------------------------------------
# Philox4x32-10: the published known-answer vectors (Salmon et al., SC'11;
# Random123 kat_vectors) and the two draw layouts built on it
# ---------------------------------------------------------------------------
def _philox_py(ctr, key):
    c, (k0, k1) = list(ctr), key
    M = 0xFFFFFFFF
    for _ in range(10):
        p0, p1 = 0xD2511F53 * c[0], 0xCD9E8D57 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k0) & M, p1 & M, ((p0 >> 32) ^ c[3] ^ k1) & M, p0 & M]
        k0, k1 = (k0 + 0x9E3779B9) & M, (k1 + 0xBB67AE85) & M
    return c


@pytest.mark.parametrize("ctr,key,out", [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
])
def test_philox_known_answers(ctr, key, out):
    assert tuple(_philox_py(ctr, key)) == out
    if ctr[1] == 0:  # the per-quad draw counter: (i >> 2, level << 16, offset), key = seed
        seed, off = key[0] | key[1] << 32, ctr[2] | ctr[3] << 32
        assert tuple(O.philox_draw(seed, off, 0, 4 * ctr[0] + e) for e in range(4)) == out


def test_ms2_dense_draws_layout():
    """Elements 8g..8g+7 at levels 0/1: 24-bit fields d = 8 level + e of the
    3 blocks (g, b << 16, offset), b = 0..2 (gc_device.h ms2_*)."""
    seed, off = 0x1234_5678_9ABC_DEF0, 0x0000_0003_0000_0007
    for g in (0, 1, 77, 2**32 - 1, 2**32 + 5):
        w = []
        for b in range(3):
            w += _philox_py((g & 0xFFFFFFFF, ((g >> 32) & 0xFFFF) | b << 16, off & 0xFFFFFFFF, off >> 32),
                            (seed & 0xFFFFFFFF, seed >> 32))
        bits = sum(v << (32 * k) for k, v in enumerate(w))
        for lvl in (0, 1):
            for e in range(8):
                want = (bits >> (24 * (8 * lvl + e))) & 0xFFFFFF
                assert O.ms2_draw(seed, off, lvl, 8 * g + e) == want
