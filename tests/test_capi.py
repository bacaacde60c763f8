"""CPU-side checks of the C ABI: the library loads, exports every symbol
include/gcodec.h declares, and its pure host functions (layouts, error
reporting, greedy-4 / byte packers) behave — no device calls."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gcodec.h")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(gc_\w+)\s*\(", src, re.M)))


def test_header_declares_the_entry_points():
    syms = declared_symbols()
    for s in ("gc_absmax_f32", "gc_qsgd_encode", "gc_qsgd_decode", "gc_ms_mask_encode", "gc_ms_select_encode",
              "gc_ms_decode", "gc_mt19937_generate", "gc_greedy4_pack", "gc_bytepack8", "gc_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from gcodec import _lib

    lib = _lib.load()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    # the ctypes table covers the header exactly
    assert set(_lib.SIGNATURES) == set(declared_symbols())


def test_strict_library_exports_every_declared_symbol():
    """lib/libgcodec_strict.so (GC_STRICT_HANDOFF=1, built by build() beside
    the product library) exports the same ABI: a stale strict build fails
    here on the CPU instead of in tests/test_gpu_strict_handoff.py."""
    path = os.path.join(ROOT, "gradient-compression_amd", "lib", "libgcodec_strict.so")
    if not os.path.exists(path):
        pytest.skip("strict library not built")
    lib = C.CDLL(path)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_version_and_abi():
    from gcodec import _lib

    assert _lib.load().gc_abi_version() == 1
    assert b"gfx950" in _lib.load().gc_version()


def test_layouts_match_oracle():
    from gcodec import codec
    from oracle import oracle as O

    for n in (0, 1, 5, 64, 1000, 23_520_842, 100_000_000):
        for bits in (1, 2, 4, 8, 12):
            for world in (1, 2, 3, 8):
                ln = codec.qsgd_layout(n, bits, world)
                s = (1 << bits) - 1
                assert (ln.bits, ln.per_word, ln.plane_words) == O.lane_layout(n, 2 * s, world)
                assert ln.per_word * ln.plane_words >= n and ln.plane_words % 4 == 0
                assert world * 2 * s < (1 << ln.bits)


def test_ms_layouts():
    from gcodec import codec

    ql, ml = codec.ms_layouts(23_520_842, [4, 2], 1)
    assert (ql.offset, ql.bits, ql.per_word) == (3, 3, 10)
    assert (ml.bits, ml.per_word) == (1, 32)
    ql3, _ = codec.ms_layouts(1000, [2, 4, 6], 1)
    assert ql3.offset == 4  # |q| <= s0 + 1 with >= 3 levels
    ql8, ml8 = codec.ms_layouts(1000, [2, 4], 8)
    assert ml8.bits == 4 and ql8.bits == 6


def test_errors_are_reported_not_raised():
    from gcodec import _lib, codec

    with pytest.raises(_lib.GCodecError) as e:
        codec.qsgd_layout(10, 0, 1)
    assert e.value.code == _lib.GC_EINVAL and "bits" in str(e.value)
    with pytest.raises(_lib.GCodecError):
        codec.lane_layout(10, 1 << 31, 4)


def test_device_calls_refuse_cpu_tensors():
    torch = pytest.importorskip("torch")
    from gcodec import _lib, codec

    with pytest.raises(_lib.GCodecError) as e:
        codec.absmax(torch.zeros(10))
    assert "no CPU fallback" in str(e.value)


def test_greedy4_host_matches_reference_vectors():
    torch = pytest.importorskip("torch")
    from gcodec.packing import bitpacking

    p = os.path.join(ROOT, "tests", "golden", "packers.npz")
    if not os.path.exists(p):
        pytest.skip("no packer fixtures")
    z = np.load(p, allow_pickle=False)
    for nm in sorted({k.split("/")[1] for k in z.files if k.startswith("g4/")}):
        src = torch.from_numpy(z[f"g4/{nm}/src"])
        packed = bitpacking.packing(src)
        assert np.array_equal(packed.numpy(), z[f"g4/{nm}/packed"]), nm
        assert np.array_equal(bitpacking.unpacking(packed).numpy(), z[f"g4/{nm}/unpacked"]), nm


def test_greedy4_rejects_out_of_domain():
    torch = pytest.importorskip("torch")
    from gcodec import _lib
    from gcodec.packing import bitpacking

    for bad in ([0, 256], [3, -1]):
        with pytest.raises(_lib.GCodecError) as e:
            bitpacking.packing(torch.tensor(bad, dtype=torch.int32))
        assert e.value.code == _lib.GC_ERANGE


def test_bytepack_host_matches_reference_vectors():
    torch = pytest.importorskip("torch")
    from gcodec.packing import bytepacking

    p = os.path.join(ROOT, "tests", "golden", "packers.npz")
    if not os.path.exists(p):
        pytest.skip("no packer fixtures")
    z = np.load(p, allow_pickle=False)
    for nm in sorted({k.split("/")[1] for k in z.files if k.startswith("bp/")}):
        src = torch.from_numpy(z[f"bp/{nm}/src"])
        packed = bytepacking.packing(src)
        assert np.array_equal(packed.numpy(), z[f"bp/{nm}/packed"])
        assert np.array_equal(bytepacking.unpacking(packed).numpy(), z[f"bp/{nm}/unpacked"])


def test_reference_extension_oracle_agrees_with_host_packers():
    """oracle/_ref (the reference's own C++ built from its sources) vs ours on fresh inputs."""
    torch = pytest.importorskip("torch")
    from oracle import build_ref

    if not build_ref.available():
        pytest.skip("oracle/_ref not built")
    from gcodec.packing import bitpacking, bytepacking

    ref_bit, ref_byte = build_ref.load()
    rng = np.random.default_rng(11)
    for _ in range(20):
        n = int(rng.integers(1, 400))
        hi = int(rng.choice([4, 16, 128, 256]))
        src = torch.from_numpy(rng.integers(0, hi, n).astype(np.int32))
        assert torch.equal(bitpacking.packing(src), ref_bit.packing(src))
        b = torch.from_numpy(rng.integers(-500, 500, n).astype(np.int32))
        assert torch.equal(bytepacking.packing(b), ref_byte.packing(b))


@pytest.mark.parametrize("shift", [4, 7, 12])
def test_segments_plan(shift):
    """gc_segments_plan (host): records are the TensorBuffer offsets
    (reducer.py:51-58) and chunk_seg[c] is the segment holding element c<<shift."""
    from gcodec import _lib
    from gcodec.shapes import resnet50_sizes

    lib = _lib.load()
    for sizes in ([0, 1, 3, 0, 0, 17, 1000, 4, 0], resnet50_sizes(), [5]):
        count = len(sizes)
        sz = np.array(sizes, dtype=np.uint64)
        ptrs = (C.c_void_p * count)(*[0x1000 * (i + 1) for i in range(count)])
        n = int(sz.sum())
        chunks = int(lib.gc_segments_chunks(n, shift))
        assert chunks == (n + (1 << shift) - 1) >> shift
        seg = np.zeros((count, 4), dtype=np.uint64)
        cs = np.zeros(max(chunks, 1), dtype=np.uint32)
        n_out = C.c_uint64(0)
        rc = lib.gc_segments_plan(sz.ctypes.data_as(C.c_void_p), ptrs, count, shift,
                                  seg.ctypes.data_as(C.c_void_p), cs.ctypes.data_as(C.c_void_p), chunks,
                                  C.byref(n_out))
        assert rc == 0 and n_out.value == n
        starts = np.concatenate([[0], np.cumsum(sz)]).astype(np.uint64)
        assert (seg[:, 0] == starts[:-1]).all() and (seg[:, 1] == starts[1:]).all()
        assert (seg[:, 2] == np.array([0x1000 * (i + 1) for i in range(count)], dtype=np.uint64)).all()
        first = np.arange(chunks, dtype=np.uint64) << np.uint64(shift)
        want = np.searchsorted(starts[1:], first, side="right")  # first segment with end > e
        assert (cs[:chunks] == want).all()
        # too small a chunk table / bad shift are errors, not crashes
        if chunks > 1:
            assert lib.gc_segments_plan(sz.ctypes.data_as(C.c_void_p), ptrs, count, shift,
                                        seg.ctypes.data_as(C.c_void_p), cs.ctypes.data_as(C.c_void_p),
                                        chunks - 1, None) == _lib.GC_EINVAL
    assert lib.gc_segments_chunks(10, 3) == 0


def test_segments_copy_refuses_different_sizes():
    """two tables with the same count and n but different
    per-tensor sizes are refused on the host (sizes_hash), before any launch."""
    from gcodec import _lib

    lib = _lib.load()

    def h(sizes):
        a = np.array(sizes, dtype=np.uint64)
        return int(lib.gc_segments_sizes_hash(a.ctypes.data_as(C.c_void_p), len(sizes)))

    assert h([3, 5]) != h([5, 3]) and h([3, 5]) == h([3, 5]) and h([]) != 0
    fake = C.c_void_p(0x1000)
    a = _lib.gc_segments(2, 8, fake, fake, 12, h([3, 5]))
    b = _lib.gc_segments(2, 8, fake, fake, 12, h([5, 3]))
    assert lib.gc_segments_copy(C.byref(a), C.byref(b), 1.0, None) == _lib.GC_EINVAL
    assert b"different sizes" in lib.gc_last_error()


def test_ms_cache_bytes():
    """q cache cells (gc_ms_cache_bytes, host only): count * bit_length(2 qmax)
    bits in 1 or 2 bytes on the dense wave-split kernels (2-3 levels of <= 24 bits)."""
    from gcodec import codec

    n = 23_520_842
    for levels, cell in (((2, 4), 1), ((1, 3), 1), ((3, 7), 1), ((4, 7), 2), ((6, 7), 2), ((1, 2, 3), 2),
                         ((2, 4, 6), 2), ((3, 4, 5), 2), ((5, 6, 7), 0), ((2, 8), 1), ((6, 10), 2),
                         ((4, 8), 2), ((2, 24), 1), ((9, 10), 0), ((1, 2, 3, 4), 0), ((4,), 0)):
        assert codec.ms_cache_bytes(n, levels) == cell, levels
    assert codec.ms_cache_bytes(1 << 32, (2, 4)) == 0  # beyond the fast path's 32-bit indices
    assert codec.ms_cache_bytes(0, (2, 4)) == 1


def test_product_package_never_reaches_the_oracle():
    """The shipped package (gcodec/ + csrc/) must not import, load or link
    anything under oracle/: the oracle is the test checker only."""
    import re

    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "gradient-compression_amd")
    pat = re.compile(r"(import\s+oracle|from\s+oracle|liboracle|oracle/_ref)")
    offenders = []
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")) or f == "Makefile":
                p = os.path.join(dirpath, f)
                with open(p, encoding="utf-8", errors="replace") as fh:
                    for i, line in enumerate(fh, 1):
                        if pat.search(line):
                            offenders.append(f"{p}:{i}: {line.strip()}")
    assert not offenders, "\n".join(offenders)


def test_ms_layouts_cached_and_exact():
    """codec.ms_layouts / levels_struct are cached per (n, sorted levels, W):
    the cached structs equal a fresh gc_ms_layout / gc_ms_mask_layout call,
    and the key distinguishes world sizes and level order-insensitively."""
    import ctypes as C

    from gcodec import _lib, codec

    lib = _lib.load()
    for n, levels, world in ((23_520_842, (2, 4), 1), (23_520_842, (4, 2), 8), (1000, (2, 4, 6), 2)):
        ql, ml = codec.ms_layouts(n, levels, world)
        assert codec.ms_layouts(n, list(levels), world)[0] is ql  # cache hit, list or tuple
        lv = _lib.gc_levels()
        lv.count = len(levels)
        for i, b in enumerate(sorted(levels)):
            lv.bits[i] = b
        q2, m2 = _lib.gc_lanes(), _lib.gc_lanes()
        assert lib.gc_ms_layout(n, C.byref(lv), world, C.byref(q2)) == 0
        assert lib.gc_ms_mask_layout(n, C.byref(lv), world, C.byref(m2)) == 0
        for a, b in ((ql, q2), (ml, m2)):
            assert bytes(a) == bytes(b)
    assert codec.ms_layouts(1000, (2, 4), 1)[0] is not codec.ms_layouts(1000, (2, 4), 2)[0]


def test_stream24_contract_checked_on_host():
    """The 24-bit packed draw layout (GC_RNG_STREAM24) is refused on the host
    where it cannot hold: counts / read indices not multiples of 4 in the
    generator, misaligned draws in the encode, any kind the multi-scale codecs
    do not take.  Every refusal happens before a launch."""
    from gcodec import _lib

    lib = _lib.load()
    fake = C.c_void_p(0x1000)
    for count, idx in ((6, 0), (8, 2), (0, 0), (8, 625)):
        assert lib.gc_mt19937_generate_split24_j(fake, fake, 1, 262_080, fake, 1, fake, count, idx, fake, 3,
                                                 None) == _lib.GC_EINVAL
        assert b"multiples of 4" in lib.gc_last_error()
    lanes = _lib.gc_lanes()
    assert lib.gc_qsgd_layout(1000, 4, 1, C.byref(lanes)) == _lib.GC_OK
    rng = _lib.gc_rng(_lib.GC_RNG_STREAM24, 0, 0, 0, C.c_void_p(0x1002))
    w = C.c_void_p(0x2000)
    assert lib.gc_qsgd_encode(fake, None, 1000, fake, 4, C.byref(lanes), C.byref(rng), w, None) == _lib.GC_EINVAL
    assert b"4-byte aligned" in lib.gc_last_error()
