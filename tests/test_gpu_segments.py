"""gc_segments (the reference's TensorBuffer, reducer.py:46-68, and the setgrad
loop, reducer.py:543-549) on the GPU: fused flatten + max-norm, decode straight
into per-parameter tensors, scaled scatter.  Bit-exact against the oracle /
the unfused kernels, on ragged tensor lists (empty tensors, odd sizes, every
4-byte misalignment, boundaries inside a vector group) and on the reference's
own model shapes (ResNet50: 161 tensors, 23,520,842 elements)."""
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

RAGGED = [0, 1, 3, 4, 5, 17, 1000, 0, 4099, 70_001, 2, 250_000, 7, 0, 64, 65]


def u32(t):
    return t.detach().contiguous().cpu().numpy().view(np.uint32)


def carve(sizes, seed, misalign=True, dtype=torch.float32):
    """Contiguous tensors cut out of one storage at random 4-byte offsets, so
    tensor pointers have every alignment mod 16 B; values from the oracle's
    input generator (heavy-tailed) -> returns (tensors, concatenation as numpy)."""
    rng = np.random.default_rng(seed)
    gaps = rng.integers(0, 4, len(sizes)) if misalign else np.zeros(len(sizes), dtype=np.int64)
    total = int(sum(sizes) + gaps.sum() + 8)
    base = torch.from_numpy(O.gen_input(total, seed=seed, kind=1)).to(DEV)
    out, pos = [], 0
    for sz, g in zip(sizes, gaps):
        pos += int(g)
        out.append(base[pos:pos + sz])
        pos += sz
    flat = np.concatenate([t.cpu().numpy() for t in out]) if out else np.zeros(0, np.float32)
    return out, flat


@pytest.mark.parametrize("shift", [4, 12])
@pytest.mark.parametrize("misalign", [False, True])
def test_flatten_absmax(shift, misalign):
    ts, ref = carve(RAGGED, seed=11 + shift, misalign=misalign)
    segs = codec.Segments(ts, chunk_shift=shift)
    assert segs.n == ref.size
    flat, norm = codec.segments_flatten_absmax(segs)
    assert u32(flat).tobytes() == ref.view(np.uint32).tobytes()
    assert norm.item() == float(O.absmax(ref))
    none, norm2 = codec.segments_flatten_absmax(segs, store=False)
    assert none is None and norm2.item() == float(O.absmax(ref))


def test_flatten_absmax_nonfinite():
    ts, ref = carve([5, 1000, 33], seed=5)
    ts[1][17] = float("inf")
    segs = codec.Segments(ts)
    assert codec.segments_flatten_absmax(segs)[1].item() == float("inf")
    ts[2][3] = float("nan")  # NaN wins, like torch.max
    assert np.isnan(codec.segments_flatten_absmax(segs)[1].item())


def test_flatten_absmax_resnet50_shapes():
    ts, ref = carve(shapes.resnet50_sizes(), seed=50)
    segs = codec.Segments(ts)
    assert segs.count == 161 and segs.n == 23_520_842
    flat, norm = codec.segments_flatten_absmax(segs)
    assert torch.equal(flat.view(torch.int32), torch.cat(ts).view(torch.int32))
    assert norm.item() == float(O.absmax(ref))


@pytest.mark.parametrize("alpha", [1.0, 1.0 / 3.0, 0.125])
def test_scatter_scaled(alpha):
    ts, _ = carve(RAGGED, seed=21)
    segs = codec.Segments(ts, chunk_shift=5)
    src = O.gen_input(segs.n, seed=9, kind=1)
    src[::97] = -0.0  # the reference's 0 + alpha*g maps -0 to +0
    codec.segments_scatter(torch.from_numpy(src).to(DEV), segs, alpha)
    want = src * np.float32(alpha) + np.float32(0.0)
    got = np.concatenate([t.cpu().numpy() for t in ts])
    assert got.view(np.uint32).tobytes() == want.view(np.uint32).tobytes()


@pytest.mark.parametrize("bits,world", [(2, 1), (4, 1), (4, 3), (8, 2)])
def test_qsgd_decode_segments(bits, world):
    ts, ref = carve(RAGGED, seed=31 + bits)
    segs = codec.Segments(ts, chunk_shift=6)
    n = segs.n
    x = torch.from_numpy(ref).to(DEV)
    norm = codec.absmax(x)
    gen = gcodec.Generator(7, "philox")
    words = codec.qsgd_encode(x, norm, bits, gen.reserve(n), world)
    words = words * world if world > 1 else words  # W identical ranks
    dense = codec.qsgd_decode(words, n, norm, bits, world, 1.0 / world)
    codec.qsgd_decode_segments(words, norm, bits, segs, world, 1.0 / world)
    got = torch.cat(ts)
    assert torch.equal(got.view(torch.int32), dense.view(torch.int32))
    want = O.qsgd_decode(u32(words), n, np.float32(norm.item()), bits, world, np.float32(1.0 / world))
    assert u32(got).tobytes() == want.view(np.uint32).tobytes()


@pytest.mark.parametrize("levels,order", [([2, 4], 1), ([2, 4], 0), ([3, 5, 7], 0)])
def test_ms_decode_segments(levels, order):
    ts, ref = carve(RAGGED, seed=41 + order)
    segs = codec.Segments(ts, chunk_shift=4)
    n = segs.n
    x = torch.from_numpy(ref).to(DEV)
    norm = codec.absmax(x)
    gen = gcodec.Generator(3, "philox")
    rng = gen.reserve(n, len(levels))
    mask = codec.ms_mask_encode(x, norm, levels, rng)
    words = codec.ms_select_encode(x, norm, levels, rng, mask)
    dense = codec.ms_decode(words, mask, n, norm, levels, 1, order, 0.5)
    codec.ms_decode_segments(words, mask, norm, levels, segs, 1, order, 0.5)
    assert torch.equal(torch.cat(ts).view(torch.int32), dense.view(torch.int32))


def test_segments_reject_bad_input():
    with pytest.raises(gcodec.GCodecError):
        codec.Segments([torch.zeros(4, device=DEV, dtype=torch.float64)])
    with pytest.raises(gcodec.GCodecError):
        codec.Segments([torch.zeros(4, 4, device=DEV).t()])  # not contiguous
    segs = codec.Segments([torch.zeros(10, device=DEV)])
    words = torch.zeros(codec.qsgd_layout(11, 4).plane_words, dtype=torch.int32, device=DEV)
    lanes = codec.qsgd_layout(11, 4)
    with pytest.raises(gcodec.GCodecError):  # bucket size != segments
        codec.qsgd_decode_segments(words, torch.ones(1, device=DEV), 4, segs, lanes=lanes)


@pytest.mark.parametrize("k", [1, 1000, 16_384, 20_000])
def test_randk_segments_equal_flat(k):
    """The GlobalRandK kernels addressing the tensors in place (gather from
    segments, encode at W = 1, decode-scatter into segments, tensor-to-tensor
    setgrad) give the bits of the flat-bucket kernels."""
    ts, ref = carve(RAGGED, seed=61)
    segs = codec.Segments(ts, chunk_shift=5)
    x = torch.from_numpy(ref).to(DEV)
    x[::31] = -0.0
    for t, (a, b) in zip(ts, zip(np.cumsum([0] + RAGGED[:-1]), np.cumsum(RAGGED))):
        t.copy_(x[a:b])
    g = torch.Generator().manual_seed(k)
    idx = torch.randperm(segs.n, generator=g)[:k].to(DEV)
    xk, nk = codec.randk_gather_absmax(x, idx)
    xs, ns = codec.randk_gather_absmax_segments(segs, idx)
    assert torch.equal(xk.view(torch.int32), xs.view(torch.int32)) and torch.equal(nk, ns)
    bits = 4
    if k <= codec.RANDK_FUSED_MAX:
        w1, n1 = codec.randk_encode_w1(x, idx, bits, gcodec.Generator(3, "philox").reserve(k))
        w2, n2 = codec.randk_encode_w1_segments(segs, idx, bits, gcodec.Generator(3, "philox").reserve(k))
        assert torch.equal(w1, w2) and torch.equal(n1, n2)
    else:
        w1 = codec.qsgd_encode(xk, nk, bits, gcodec.Generator(3, "philox").reserve(k), 2)
        w1 = w1 * 2
    world = 1 if k <= codec.RANDK_FUSED_MAX else 2
    # flat: scatter into the bucket, then setgrad x 1/W; segments: copy + decode-scatter
    flat = x.clone()
    codec.qsgd_decode(w1, k, nk, bits, world, 1.0, idx=idx, out=flat)
    want = flat * np.float32(1.0 / world) + 0.0
    outs = [torch.full_like(t, 7.0) for t in ts]
    osegs = codec.Segments(outs, chunk_shift=7)
    codec.segments_copy(segs, osegs, 1.0 / world)
    codec.qsgd_decode_scatter_segments(w1, idx, nk, bits, osegs, world, 1.0 / world)
    assert u32(torch.cat(outs)).tobytes() == u32(want).tobytes()
    with pytest.raises(gcodec.GCodecError):  # different tensor sizes
        codec.segments_copy(segs, codec.Segments(outs[:-1]))


@pytest.mark.parametrize("levels,world", [([2, 4], 1), ([2, 4], 2), ([4, 8], 3)])
def test_ms_decode_scatter_segments_equal_flat(levels, world):
    """gc_ms_decode_scatter_segments (the GlobalRandK two-scale decode-scatter
    into the tensors, x 1/W, + 0) == ms_decode with idx into a flat bucket
    followed by the setgrad 0 + RN(g / W)."""
    ts, ref = carve(RAGGED, seed=71)
    segs = codec.Segments(ts, chunk_shift=6)
    k = 20_000
    idx = torch.randperm(segs.n, generator=torch.Generator().manual_seed(k))[:k].to(DEV)
    xk = torch.from_numpy(ref).to(DEV)[idx]
    norm = codec.absmax(xk)
    r = gcodec.Generator(9, "philox").reserve(k, len(levels))
    m = codec.ms_mask_encode(xk, norm, levels, r, world)
    w = codec.ms_select_encode(xk, norm, levels, r, m, world)
    flat = torch.from_numpy(ref).to(DEV)
    codec.ms_decode(w, m, k, norm, levels, world, 1, 1.0, idx=idx, out=flat)
    want = flat * np.float32(1.0 / world) + 0.0
    outs = [torch.full_like(t, 5.0) for t in ts]
    osegs = codec.Segments(outs, chunk_shift=9)
    codec.segments_copy(segs, osegs, 1.0 / world)
    codec.ms_decode_scatter_segments(w, m, idx, norm, levels, osegs, world, 1, 1.0 / world)
    assert u32(torch.cat(outs)).tobytes() == u32(want).tobytes()


REDUCERS = [
    ("QSGDMaxNormReducer", dict(quantization_level=4)),
    ("QSGDMaxNormTwoScaleReducer", dict(lower_quantization_level=2, higher_quantization_level=4)),
    ("QSGDMaxNormMultiScaleReducer", dict(quantization_levels=[2, 4, 6])),
    ("GlobalRandKMaxNormReducer", dict(K=1000, quantization_level=4)),
    ("GlobalRandKMaxNormReducer", dict(K=20_000, quantization_level=4)),  # gather + encode (K > fused max)
    ("GlobalRandKMaxNormReducer", dict(K=1000, quantization_level=16)),   # b above the fused lanes
    ("GlobalRandKMaxNormTwoScaleReducer", dict(K=1000, lower_quantization_level=2, higher_quantization_level=4)),
    ("GlobalRandKMaxNormTwoScaleReducer", dict(K=30_000, lower_quantization_level=4, higher_quantization_level=8)),
]


@pytest.mark.parametrize("name,kw", REDUCERS)
@pytest.mark.parametrize("inplace", [False, True])
def test_reducer_fused_equals_unfused(name, kw, inplace):
    """The fused reducer (gc_segments flatten+norm, decode into grad_out) gives
    the same bits as the TensorBuffer path, including grad_out is grad_in."""
    cls = getattr(gcodec, name)
    sizes = [27, 64, 0, 1000, 3, 4099, 10, 70_001]
    results = []
    for fused in (False, True):
        ts, _ = carve(sizes, seed=77)
        ts[3][::5] = -0.0
        outs = ts if inplace else [torch.full_like(t, 9.0) for t in ts]
        r = cls(DEV, generator=gcodec.Generator(5, "philox"), fused=fused, **kw)
        for _ in range(2):
            bits = r.reduce(ts, outs)
        results.append((bits, [u32(o) for o in outs]))
    (b0, o0), (b1, o1) = results
    assert b0 == b1
    for a, b in zip(o0, o1):
        assert a.tobytes() == b.tobytes()


def test_reducer_fresh_grad_out_every_step_pins_nothing():
    """The reference trainer hands fresh p.grad tensors to the reducer every
    step (zero_grad sets them to None).  The fused reducer must give the same
    bits as with stable tensors, keep at most SEG_CACHE tables, and hold no
    reference to any step's gradients (the table cache must not pin
    old gradient generations in device memory)."""
    import gc
    import weakref

    sizes = [27, 64, 1000, 3, 4099, 70_001]
    ts, _ = carve(sizes, seed=91)
    stable = [torch.empty_like(t) for t in ts]
    ref = gcodec.QSGDMaxNormReducer(DEV, generator=gcodec.Generator(3, "philox"), quantization_level=4)
    r = gcodec.QSGDMaxNormReducer(DEV, generator=gcodec.Generator(3, "philox"), quantization_level=4)
    dead = []
    for step in range(12):
        ref.reduce(ts, stable)
        fresh = [torch.full_like(t, float(step)) for t in ts]  # new allocations every step
        r.reduce(ts, fresh)
        for a, b in zip(stable, fresh):
            assert u32(a).tobytes() == u32(b).tobytes()
        dead += [weakref.ref(t) for t in fresh]
        del fresh, a, b
        assert len(r._seg_cache) <= r.SEG_CACHE
    gc.collect()
    alive = [i for i, w in enumerate(dead) if w() is not None]
    assert not alive, f"{len(alive)} of {len(dead)} gradient tensors still referenced: {alive[:12]}"


def test_segment_cache_rejects_recycled_addresses_of_another_dtype_or_layout():
    """a cached fp32 segment table keyed by (pointers, sizes) alone
    would be hit by a half-precision list living at the same addresses with
    the same element counts (a model cast after the first step), or by a
    non-contiguous view of the same storage: the kernels would then read and
    write 4-byte elements through 2-byte tensors.  Such lists must miss the
    cache and take the TensorBuffer path (no table)."""
    sizes = [1000, 24, 4096, 7]
    starts = np.concatenate([[0], np.cumsum(sizes)[:-1]]).tolist()
    store = torch.zeros(sum(sizes) + 64, dtype=torch.float32, device=DEV)
    f32 = [store[s:s + z] for s, z in zip(starts, sizes)]
    st = store.untyped_storage()
    f16 = [torch.empty(0, dtype=torch.float16, device=DEV).set_(st, 2 * s, (z,)) for s, z in zip(starts, sizes)]
    assert [t.data_ptr() for t in f16] == [t.data_ptr() for t in f32]
    sq = store[:64 * 64].view(64, 64)
    nc = [sq.t(), store[4096:4096 + 10]]  # the transpose shares the first tensor's pointer and size
    red = gcodec.QSGDMaxNormReducer(DEV, quantization_level=4, generator=gcodec.Generator(1, "philox"))
    assert red._segments(f32) is not None
    assert codec.Segments.key_of(f16) != codec.Segments.key_of(f32)
    assert red._segments(f16) is None
    assert red._segments([sq.reshape(-1)[:4096].view(64, 64), store[4096:4106]]) is not None
    assert red._segments(nc) is None
    assert red._segments(f32) is not None  # the fp32 table is still served
