"""Device greedy 4-mode packer (gc_greedy4_*_device) — the reference's
bitpacking format (extensions/Extension CPU/bitpacking.cpp:5-124), produced
by a scan over segment tables.  Bit-exact against the reference extension's
own known-answer vectors (tests/golden/packers.npz) and against the oracle /
host packer on inputs that stress the boundaries (32-position segments,
8192-position tiles, 128-tile groups, the top walk past 64 groups):
all-mode-0 runs, all-mode-3 runs, mixes, ragged ends, and the QSGDBP call
site's ResNet50 bucket (23,520,842 sign bits and 4-bit magnitudes)."""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # collected on CPU, skipped there
    pytest.skip("no GPU", allow_module_level=True)

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402
from gcodec.packing import gpu_bitpacking  # noqa: E402
from oracle import oracle as O  # noqa: E402

DEV = torch.device("cuda", 0)
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_device_packer_matches_reference_vectors():
    z = np.load(os.path.join(GOLD, "packers.npz"), allow_pickle=False)
    names = sorted({k.split("/")[1] for k in z.files if k.startswith("g4/")})
    assert names
    for nm in names:
        src = z[f"g4/{nm}/src"]
        w = codec.greedy4_pack(torch.from_numpy(src.astype(np.int32)).to(DEV))
        assert w.is_cuda
        assert np.array_equal(w.cpu().numpy(), z[f"g4/{nm}/packed"].astype(np.int32)), nm
        u = codec.greedy4_unpack(w)
        assert np.array_equal(u.cpu().numpy(), z[f"g4/{nm}/unpacked"].astype(np.int32)), nm


def _inputs():
    rng = np.random.default_rng(4)
    yield "empty", np.zeros(0, np.int32)
    yield "one", np.array([200], np.int32)
    for n in (2047, 2048, 2049, 2048 * 256 - 1, 2048 * 256 + 5, 1_000_003):
        yield f"mix{n}", rng.choice([0, 1, 3, 9, 15, 100, 255], n, p=[.3, .2, .15, .15, .1, .05, .05]).astype(np.int32)
    yield "zeros", np.zeros(2048 * 300 + 17, np.int32)
    yield "max", np.full(2048 * 3 + 1, 255, np.int32)
    # runs that flip modes right at chunk boundaries
    a = np.zeros(2048 * 8, np.int32)
    for c in range(1, 8):
        a[2048 * c - 7:2048 * c + 3] = 200
    yield "edges", a
    yield "qsgd4", np.abs(rng.normal(0, 4, 3_000_000)).clip(0, 15).astype(np.int32)
    # runs that flip modes right at segment / tile boundaries, unaligned starts
    b = np.zeros(8192 * 5 + 9, np.int32)
    for c in range(1, 5):
        b[8192 * c - 16:8192 * c + 1] = 130
        b[4096 * c + 7:4096 * c + 8] = 17
    b[::16] = 5
    yield "tile_edges", b
    yield "mode3_all", rng.integers(128, 256, 8192 * 3 + 31).astype(np.int32)
    # more groups than the emit walks itself (> 64): k_g4p_top, over two 128-group chunks (> 128 x 128 x 8192)
    yield "chunks2", rng.choice([0, 1, 2, 3, 7, 15], 140_000_000, p=[.4, .2, .15, .15, .05, .05]).astype(np.int32)


@pytest.mark.parametrize("name,src", list(_inputs()), ids=lambda v: v if isinstance(v, str) else "")
def test_device_packer_matches_host(name, src):
    want = O.greedy4_pack(src) if src.size <= 200_000 else None
    host = codec.greedy4_pack(torch.from_numpy(src))  # host packer (pinned to the oracle in test_capi)
    if want is not None:
        assert np.array_equal(host.numpy(), want)
    w = gpu_bitpacking.packing(torch.from_numpy(src).to(DEV))
    assert np.array_equal(w.cpu().numpy(), host.numpy()), name
    u = gpu_bitpacking.unpacking(w)
    assert np.array_equal(u.cpu().numpy()[:src.size], src)
    assert np.array_equal(u.cpu().numpy(), codec.greedy4_unpack(host).numpy())


def test_device_packer_rejects_out_of_domain():
    for bad in ([1, 2, 256], [-1, 3]):
        with pytest.raises(gcodec.GCodecError):
            codec.greedy4_pack(torch.tensor(bad, dtype=torch.int32, device=DEV))


@pytest.mark.parametrize("bits", [4, 8])
def test_qsgdbp_resnet50_bucket_packs_exactly(bits):
    """The QSGDBP call site at the ResNet50 bucket size (23,520,842): the sign
    bits and the magnitudes packed on the device equal the host packer's words
    (the reference format), and unpack returns the values."""
    n = 23_520_842
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn(n, device=DEV, generator=g).mul_(0.01)
    norm = codec.absmax(x)
    xi, sg = codec.qsgd_quantize_split(x, norm, bits, gcodec.Generator(9, "philox").reserve(n))
    for src in (xi, sg):
        host_words = codec.greedy4_pack(src.cpu())
        dev_words = codec.greedy4_pack(src)
        assert np.array_equal(dev_words.cpu().numpy(), host_words.numpy())
        u = codec.greedy4_unpack(dev_words)
        assert torch.equal(u[:n], src)


def test_pack_many_equals_one_by_one():
    """greedy4_pack_many (one host sync for all word counts, the per-stream
    workspace reused across calls) gives each array the words greedy4_pack
    gives it: sizes from 1 to a multi-round 3 M, an unaligned slice, an empty
    array, repeated calls, and a side stream of its own."""
    rng = np.random.default_rng(12)
    arrs = [rng.choice([0, 1, 3, 9, 15, 100, 255], m, p=[.3, .2, .15, .15, .1, .05, .05]).astype(np.int32)
            for m in (1, 15, 4097, 300_001, 3_000_000)]
    d = [torch.from_numpy(a).to(DEV) for a in arrs]
    srcs = d + [d[3][1:], torch.empty(0, dtype=torch.int32, device=DEV)]
    want = [codec.greedy4_pack(t.cpu()).numpy() for t in srcs]
    for _ in range(3):
        got = codec.greedy4_pack_many(*srcs)
        assert len(got) == len(srcs)
        for g, w in zip(got, want):
            assert g.is_cuda and np.array_equal(g.cpu().numpy(), w)
    side = torch.cuda.Stream(DEV)
    side.wait_stream(torch.cuda.current_stream(DEV))
    with torch.cuda.stream(side):
        got = codec.greedy4_pack_many(d[4], d[2])
    assert np.array_equal(got[0].cpu().numpy(), want[4]) and np.array_equal(got[1].cpu().numpy(), want[2])
    host = codec.greedy4_pack_many(srcs[2].cpu(), srcs[3].cpu())  # host tensors: the host packer
    assert not host[0].is_cuda and np.array_equal(host[1].numpy(), want[3])
    vals = codec.greedy4_unpack_many(*got, *codec.greedy4_pack_many(*srcs))
    want_u = [codec.greedy4_unpack(torch.from_numpy(w)).numpy() for w in (want[4], want[2], *want)]
    assert len(vals) == len(want_u)
    for v, w in zip(vals, want_u):
        assert v.is_cuda and np.array_equal(v.cpu().numpy(), w)


def test_pack_many_rejects_out_of_domain():
    ok = torch.tensor([1, 2, 3], dtype=torch.int32, device=DEV)
    with pytest.raises(gcodec.GCodecError):
        codec.greedy4_pack_many(ok, torch.tensor([1, 256], dtype=torch.int32, device=DEV))
    assert np.array_equal(codec.greedy4_pack_many(ok)[0].cpu().numpy(), codec.greedy4_pack(ok.cpu()).numpy())


def test_device_packer_unaligned_source():
    """src not 16-byte aligned (a slice at +1 element): the scalar-load path."""
    rng = np.random.default_rng(8)
    a = rng.choice([0, 1, 3, 9, 15, 100, 255], 300_001, p=[.3, .2, .15, .15, .1, .05, .05]).astype(np.int32)
    d = torch.from_numpy(a).to(DEV)[1:]
    assert d.data_ptr() % 16 != 0
    host = codec.greedy4_pack(torch.from_numpy(a[1:].copy()))
    assert np.array_equal(codec.greedy4_pack(d).cpu().numpy(), host.numpy())


@pytest.mark.parametrize("n", [1, 7, 4099, 23_520_842])
def test_qsgdbp_fused_decode_equals_reference_ops(n):
    """gc_qsgdbp_decode == the reference's fp32 ops (c * sgn) * float(xi)
    (compressors.py:375-376) bit for bit, -0.0 for a negative x rounded to 0,
    any n % 4 tail, on oversized unpack buffers (whole words)."""
    g = torch.Generator(device=DEV).manual_seed(n)
    m = n + 13
    sign = torch.randint(0, 2, (m,), device=DEV, generator=g, dtype=torch.int32)
    xi = torch.randint(0, 16, (m,), device=DEV, generator=g, dtype=torch.int32)
    c = torch.tensor([0.0123], device=DEV)
    got = codec.qsgdbp_decode(sign, xi, c, n)
    sgn = torch.where(sign[:n] == 1, -1.0, 1.0).to(torch.float32)
    ref = (c * sgn) * xi[:n].to(torch.float32)
    assert got.shape == (n,)
    assert np.array_equal(got.cpu().numpy().view(np.uint32), ref.cpu().numpy().view(np.uint32))


@pytest.mark.parametrize("nwords", [1, 1000, 5000, 5_000_000])
def test_device_unpack_capacity_writes_nothing(nwords):
    """gc_greedy4_unpack_device with too small a cap: status 2, the count is
    still reported, and not one output element is written (both the
    two-launch form, where every block checks the total itself, and the scan
    form above 4 M words); with enough cap the values come back."""
    from gcodec import _lib

    lib = _lib.load()
    rng = np.random.default_rng(nwords)
    vals = rng.integers(128, 256, 3 * nwords).astype(np.int32)  # 3 values per word (mode 3)
    vals[rng.integers(0, vals.size, vals.size // 50)] = 1      # and some shorter runs
    w = codec.greedy4_pack(torch.from_numpy(vals).to(DEV))
    nw = w.numel()
    need = int(codec.greedy4_unpack(w).numel())
    ws = torch.empty(int(lib.gc_greedy4_unpack_workspace_size(nw)), dtype=torch.uint8, device=DEV)
    for cap, ok in ((need - 1, False), (need, True)):
        out = torch.full((need + 8,), -7, dtype=torch.int32, device=DEV)
        res = torch.full((2,), 123, dtype=torch.int64, device=DEV)
        assert lib.gc_greedy4_unpack_device(C.c_void_p(w.data_ptr()), nw, C.c_void_p(out.data_ptr()), cap,
                                            C.c_void_p(res.data_ptr()), C.c_void_p(res.data_ptr() + 8),
                                            C.c_void_p(ws.data_ptr()), None) == 0
        torch.cuda.synchronize()
        count, status = int(res[0].item()), int(res[1].item()) & 0xFFFFFFFF
        assert count == need
        if ok:
            assert status == 0
            assert torch.equal(out[:need], codec.greedy4_unpack(w))
        else:
            assert status == 2 and bool((out == -7).all())


def test_late_block_timeout_is_reported_and_workspace_rearmed():
    """a pack whose block 0 starts ~1.5 s late (the
    header's test_delay field; 0 in every product workspace).  Every other
    block times out waiting for block 0's round-0 granules and writes none of
    its words; block 0 then sees every granule and, alone, would have
    reported status 0.  Every block's timeout is collected now: the status is
    4 and result() raises.  It also zeroes the workspace again before raising
    (late blocks tag granules with the next launch's tags), so the
    next pack on the same object is exact."""
    rng = np.random.default_rng(5)
    src = rng.choice([0, 1, 3, 9, 15, 100, 255], 3_000_000).astype(np.int32)
    a = torch.from_numpy(src).to(DEV)
    want = codec.greedy4_pack(a.cpu()).numpy()
    pk = codec.Greedy4Device(a.numel(), DEV, unpack_words=0)
    pk.pack(a)
    assert np.array_equal(pk.words[:pk.result()].cpu().numpy(), want)
    # G1Hdr: seq u64 @0, done u32 @8, tmo u32 @12, test_delay u64 @16 (100 MHz ticks)
    pk.ws[16:24] = torch.tensor([150_000_000], dtype=torch.int64).view(torch.uint8).to(DEV)
    pk.pack(a)
    with pytest.raises(gcodec.GCodecError):
        pk.result()
    assert int(pk.ws.count_nonzero()) == 0
    pk.pack(a)
    assert np.array_equal(pk.words[:pk.result()].cpu().numpy(), want)


def test_packs_on_two_streams_run_one_at_a_time():
    """one persistent pack in flight per device — a pack enqueued
    on a second stream waits for the first stream's pack (event), so the two
    never hold each other's CUs; both results are exact."""
    rng = np.random.default_rng(6)
    srcs = [torch.from_numpy(rng.choice([0, 3, 15, 200], 2_000_000).astype(np.int32)).to(DEV) for _ in range(2)]
    want = [codec.greedy4_pack(s.cpu()).numpy() for s in srcs]
    s1, s2 = torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)
    for s in (s1, s2):
        s.wait_stream(torch.cuda.current_stream(DEV))
    pks = [codec.Greedy4Device(s.numel(), DEV, unpack_words=0) for s in srcs]
    with torch.cuda.stream(s1):
        torch.cuda._sleep(20_000_000)  # the first pack starts late: the second must wait for it
        pks[0].pack(srcs[0])
    with torch.cuda.stream(s2):
        pks[1].pack(srcs[1])
    torch.cuda.synchronize()
    for pk, w in zip(pks, want):
        assert np.array_equal(pk.words[:pk.result()].cpu().numpy(), w)
