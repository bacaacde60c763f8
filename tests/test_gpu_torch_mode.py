"""Torch-mode draws (the reference's MT19937 stream, compressors.py:310 under
seed.py:6-11) generated on the GPU side stream with the next same-size call
generated speculatively (codec.mt19937_draws, MT_SPECULATE): every call must
return exactly torch's next `count` draws and leave torch's CPU generator
where torch.bernoulli would — across repeated sizes (speculation used),
changed sizes (speculation dropped), torch's generator used or reseeded in
between (speculation invalid), and with speculation off.  The oracle is the
serial MT19937 of oracle/gcodec_oracle.c continued from torch's state."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # collected on CPU, skipped there
    pytest.skip("no GPU", allow_module_level=True)

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402
from gcodec.rng import torch_mt_state  # noqa: E402
from oracle import oracle as O  # noqa: E402

DEV = torch.device("cuda", 0)


def _oracle_next(count):
    """(draws, state words, read index) of torch's generator after `count` more draws"""
    words, idx = torch_mt_state()
    st = O.MT19937(0)
    st._st.s[:] = [int(v) for v in words]
    st._st.idx = idx
    d = st.draws(count)
    w2, i2 = st.state()
    return d, np.asarray(w2, dtype=np.uint32), int(i2)


@pytest.mark.parametrize("speculate", [True, False])
def test_draw_sequences_vs_serial_stream(speculate):
    old = codec.MT_SPECULATE
    codec.MT_SPECULATE = speculate
    try:
        torch.manual_seed(123)
        seq = [300_007, 300_007, 300_007, 5_000, 5_000, 624, 1, 300_007, 300_007, 2 * 300_007]
        for i, cnt in enumerate(seq):
            ref, w2, i2 = _oracle_next(cnt)
            got = codec.mt19937_draws(cnt, DEV)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy().view(np.uint32), ref), (i, cnt)
            words, idx = torch_mt_state()
            assert idx == i2 and np.array_equal(words, w2), (i, cnt)
            if i == 4:
                torch.rand(7)  # torch's generator used between two calls
            if i == 6:
                torch.manual_seed(99)  # and reseeded
    finally:
        codec.MT_SPECULATE = old


@pytest.mark.parametrize("depth", [2, 4, 8])
@pytest.mark.parametrize("count", [1, 100, 623, 4_000])
def test_repeated_calls_every_depth_vs_serial_stream(depth, count):
    """Repeated same-size calls (the speculation runs enqueued ahead, each in
    its slot of the rotation) for single-call runs (count < 624) and
    multi-call runs, at every speculation depth: each call's draws and torch's
    state after it are the serial stream's.  (A rotation sized for multi-call
    runs once gave single-call runs' speculation the slot of the run whose
    state was still to be read: torch's state came back wrong.)"""
    old = codec.MT_SPECULATE_DEPTH
    codec.MT_SPECULATE_DEPTH = depth
    codec.mt_release()
    try:
        torch.manual_seed(depth * 1000 + count)
        for i in range(3 * depth + 5):
            ref, w2, i2 = _oracle_next(count)
            got = codec.mt19937_draws(count, DEV)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy().view(np.uint32), ref), i
            words, idx = torch_mt_state()
            assert idx == i2 and np.array_equal(words, w2), i
    finally:
        codec.MT_SPECULATE_DEPTH = old
        codec.mt_release()


def test_switching_run_forms_without_reseeding_vs_serial_stream():
    """Multi-call runs (plain draws, count >= 624), then packed single-call
    runs, then plain again, with torch's generator never touched in between:
    the switch changes the slot rotation and drops the queued runs, which had
    already moved the device state past torch's, so the state must be sent
    again (bench r05n: a packed call after the multi-call runs returned a
    read index of -160).  Every call's draws and torch's state after it are
    the serial stream's."""
    torch.manual_seed(4321)
    count = 20_000
    seq = [False] * 5 + [True] * 4 + [False] * 4 + [True] * 2
    for i, packed in enumerate(seq):
        ref, w2, i2 = _oracle_next(count)
        got = codec.mt19937_draws(count, DEV, packed24=packed)
        torch.cuda.synchronize()
        if packed:
            b = got.cpu().numpy().view(np.uint8).reshape(-1, 3).astype(np.uint32)
            assert np.array_equal(b[:, 0] | b[:, 1] << 8 | b[:, 2] << 16, ref & 0xFFFFFF), i
        else:
            assert np.array_equal(got.cpu().numpy().view(np.uint32), ref), i
        words, idx = torch_mt_state()
        assert idx == i2 and np.array_equal(words, w2), i
    codec.mt_release()


def test_torch_mode_compressor_back_to_back_vs_oracle():
    """QSGDMaxNormCompressor.compress in torch mode, five back-to-back calls on
    the same bucket (the speculative draws used four times), then the fused
    generator-quantize path in between (its own state buffers): q == the
    oracle's quantize of the serial stream every time."""
    n, bits = 1_000_003, 4
    x = O.gen_input(n, seed=3)
    xd = torch.from_numpy(x).to(DEV)
    norm = O.absmax(x)
    gcodec.set_rng_mode("torch")
    try:
        torch.manual_seed(5)
        c = gcodec.QSGDMaxNormCompressor(DEV, bits)
        for i in range(6):
            ref_draws, _, _ = _oracle_next(n)
            if i == 3:
                q = codec.qsgd_quantize_torch(xd, float(norm), bits)
            else:
                q = c.compress(torch.tensor([norm], device=DEV), xd)
            exp = O.qsgd_quantize(x, norm, bits, O.stream_rng(ref_draws))
            assert np.array_equal(q.cpu().numpy().astype(np.int32), np.asarray(exp, dtype=np.int32)), i
    finally:
        gcodec.set_rng_mode(gcodec.rng.DEFAULT_MODE)


@pytest.mark.parametrize("idx,count", [(0, 1), (623, 1), (624, 1), (5, 619), (5, 620), (0, 624), (624, 624),
                                       (3, 1248), (100, 2 * 262_080 + 17), (624, 3_000_001), (17, 10_000_000)])
def test_split_end_state_vs_serial_stream(idx, count):
    """gc_mt19937_generate_split_j: the end state jumped to directly in phase 1
    (written over the device state before any draw exists) equals the serial
    generator's state after `count` draws, including the read index, for read
    indices 0 / mid / 624 and counts inside block 0, ending exactly on a block
    boundary, and spanning many generators; the draws of phase 2 equal the
    serial stream's."""
    import ctypes as C
    from gcodec import _lib

    st = O.MT19937(1234)
    st.draws(1000)
    st._st.idx = idx
    w0, i0 = st.state()
    ref = st.draws(count)
    w1, i1 = st.state()
    state = torch.from_numpy(np.append(np.asarray(w0, np.uint32), np.uint32(i0)).view(np.int32)).to(DEV)
    J = codec.mt_generator_draws(count)
    gens = -(-count // J)
    table, tgens = codec._mt_jump_table(DEV, gens - 1, J) if gens > 1 else (None, 0)
    block = (idx + count - 1) // 624
    end = codec._mt_end_coef(DEV, block)
    ws = torch.empty(int(_lib.load().gc_mt19937_workspace_size_j(count, J)), dtype=torch.uint8, device=DEV)
    out = torch.empty(count, dtype=torch.int32, device=DEV)
    lib = _lib.load()
    p = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
    s = codec._stream(DEV)
    assert lib.gc_mt19937_generate_split_j(p(state), p(table), tgens, J, p(end), block, None, count, p(ws), 1, s) == 0
    torch.cuda.synchronize()
    got = state.cpu().numpy().view(np.uint32)
    assert int(got[624]) == i1 and np.array_equal(got[:624], np.asarray(w1, np.uint32))
    assert lib.gc_mt19937_generate_split_j(p(state), p(table), tgens, J, p(end), block, p(out), count, p(ws), 2, s) == 0
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), np.asarray(ref, np.uint32))
    # the state is left alone by phase 2
    assert np.array_equal(state.cpu().numpy().view(np.uint32), got)


def test_table_growth_while_caller_stream_busy():
    """the jump table grows (torch.cat) on the caller's stream while
    the draws run on the side streams.  With the caller's stream held busy by a
    sleep kernel, the side streams must still wait for the grown table: the
    draws equal the serial stream's."""
    codec.mt_release()
    codec._MT_TABLE.clear()
    torch.manual_seed(7)
    for cnt, hold in ((1_000_003, 0), (30_000_001, 50_000_000), (30_000_001, 0), (60_000_017, 50_000_000)):
        ref, w2, i2 = _oracle_next(cnt)
        if hold:
            torch.cuda._sleep(hold)  # the caller's stream stays busy while the table grows
        got = codec.mt19937_draws(cnt, DEV)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy().view(np.uint32), ref), cnt
        words, idx = torch_mt_state()
        assert idx == i2 and np.array_equal(words, w2), cnt


def test_release_drops_speculation_and_stays_exact():
    """mt_release (called when a generator leaves torch mode) drops the
    speculative run and workspaces; the next calls start from torch's state."""
    torch.manual_seed(11)
    for i in range(5):
        if i == 3:
            codec.mt_release(DEV)
            assert DEV.index not in codec._MT_SPEC
        ref, _, _ = _oracle_next(200_003)
        got = codec.mt19937_draws(200_003, DEV)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy().view(np.uint32), ref), i


@pytest.mark.parametrize("count", [4, 624, 1_000_000, 2 * 262_080 + 8])
def test_packed24_draws_are_the_low_bytes(count):
    """gc_mt19937_generate_split24_j: 3 bytes per draw, little-endian, the
    low 24 bits of exactly the draws the plain generator makes, and the same
    state afterwards."""
    torch.manual_seed(77)
    ref, w2, i2 = _oracle_next(count)
    got = codec.mt19937_draws(count, DEV, packed24=True)
    torch.cuda.synchronize()
    assert got.numel() == count // 4 * 3
    b = got.cpu().numpy().view(np.uint8).reshape(-1, 3).astype(np.uint32)
    assert np.array_equal(b[:, 0] | b[:, 1] << 8 | b[:, 2] << 16, ref & 0xFFFFFF)
    words, idx = torch_mt_state()
    assert idx == i2 and np.array_equal(words, w2)


def test_packed24_encode_back_to_back_matches_plain_and_falls_back():
    """The torch-mode encode with packed draws (the product's form, speculation
    used on repeats) gives the same words as the plain draws, call after call;
    a read index that is not a multiple of 4 (torch.rand(1) in between) falls
    back to the plain draws, and the stream stays exact."""
    n, bits = 1_000_000, 4
    x = torch.from_numpy(O.gen_input(n, seed=8)).to(DEV)
    nm = codec.absmax(x)
    lanes = codec.qsgd_layout(n, bits, 1)
    gen = gcodec.Generator(0, "torch")
    from gcodec import _lib

    def run(packed, steps):
        torch.manual_seed(1234)
        outs, kinds = [], []
        for i in range(steps):
            if i == 3:
                torch.rand(1)  # read index now 1 mod 4
            if i == 5:
                torch.rand(3)  # and back to a multiple of 4
            r = gen.reserve(n, packed24=packed)
            kinds.append(r.kind)
            outs.append(codec.qsgd_encode(x, nm, bits, r, 1, lanes=lanes).cpu().numpy())
        return outs, kinds, torch_mt_state()

    a, ka, sa = run(True, 8)
    b, kb, sb = run(False, 8)
    assert ka[:3] == [_lib.GC_RNG_STREAM24] * 3 and ka[3] == _lib.GC_RNG_STREAM and ka[5] == _lib.GC_RNG_STREAM24
    assert set(kb) == {_lib.GC_RNG_STREAM}
    for i, (u, v) in enumerate(zip(a, b)):
        assert np.array_equal(u, v), i
    assert sa[1] == sb[1] and np.array_equal(sa[0], sb[0])


def _split_planes(got, count, hb):
    """(hi, lo) integer arrays of one call's split-plane region"""
    b = got.cpu().numpy().view(np.uint8)
    hpad = (count * (hb // 8) + 15) // 16 * 16
    if hb == 8:
        hi = b[:count].astype(np.uint32)
        lo = b[hpad:hpad + 2 * count].view(np.uint16).astype(np.uint32)
    else:
        hi = b[:2 * count].view(np.uint16).astype(np.uint32)
        lo = b[hpad:hpad + count].astype(np.uint32)
    return hi, lo


@pytest.mark.parametrize("fmt,hb", [("split8", 8), ("split16", 16)])
@pytest.mark.parametrize("count", [624, 100_000, 2 * 262_080 + 8])
def test_split_draws_are_the_planes_of_the_low_24_bits(fmt, hb, count):
    """gc_mt19937_generate_multi_split_j through mt19937_reserve: every call's
    region holds the top hb of each draw's low 24 bits in the HI plane and the
    rest in the LO plane, for the serial stream's draws, call after call (the
    speculative multi-call runs: one region per call), and torch's state after
    each call is the serial generator's."""
    from gcodec import _lib
    codec.mt_release()
    torch.manual_seed(hb * 100 + count % 97)
    kind = _lib.GC_RNG_SPLIT8 if hb == 8 else _lib.GC_RNG_SPLIT16
    for i in range(11):
        ref, w2, i2 = _oracle_next(count)
        got, k = codec.mt19937_reserve(count, DEV, fmt)
        torch.cuda.synchronize()
        assert k == kind and got.numel() == codec.mt_format_bytes(count, fmt), i
        hi, lo = _split_planes(got, count, hb)
        r24 = np.asarray(ref, np.uint32) & 0xFFFFFF
        assert np.array_equal(hi, r24 >> (24 - hb)), i
        assert np.array_equal(lo, r24 & ((1 << (24 - hb)) - 1)), i
        words, idx = torch_mt_state()
        assert idx == i2 and np.array_equal(words, w2), i
    codec.mt_release()


@pytest.mark.parametrize("bits", [1, 2, 4, 8])
@pytest.mark.parametrize("fmt", ["split8", "split16"])
def test_split_encode_back_to_back_matches_plain_and_falls_back(fmt, bits):
    """The torch-mode QSGD encode from split-plane draws (the HI plane decides
    unless the rounding ties, then the LO plane is read) gives the words of
    the plain 32-bit draws call after call, across the narrow (b <= 7) and wide
    (b = 8) integer paths, L = 16 / 10 / 6 / 4 lanes per word, and read indices
    that are not multiples of 4 (torch.rand(1) in between).  The inputs hit the
    tie path: the test counts, on the host, elements whose HI bits equal those
    of ceil(p 2^24) - 1."""
    from gcodec import _lib
    n = 1_000_003  # odd: every call's region starts mid-quad of the stream
    x = torch.from_numpy(O.gen_input(n, seed=bits)).to(DEV)
    x[:4096] = 0.0  # zeros and exact multiples: F = 0 and tiny-F quads
    nm = codec.absmax(x)
    lanes = codec.qsgd_layout(n, bits, 1)
    gen = gcodec.Generator(0, "torch")
    kind = _lib.GC_RNG_SPLIT8 if fmt == "split8" else _lib.GC_RNG_SPLIT16

    def run(f, steps):
        torch.manual_seed(4321 + bits)
        outs, kinds = [], []
        for i in range(steps):
            if i == 3:
                torch.rand(1)  # read index now 1 mod 4
            if i == 5:
                torch.rand(3)  # and back to a multiple of 4
            r = gen.reserve(n, fmt=f)
            kinds.append(r.kind)
            outs.append(codec.qsgd_encode(x, nm, bits, r, 1, lanes=lanes).cpu().numpy())
        return outs, kinds, torch_mt_state()

    codec.mt_release()
    a, ka, sa = run(fmt, 9)
    codec.mt_release()
    b, kb, sb = run("plain", 9)
    assert set(ka) == {kind}  # any read index (torch.rand(1) leaves it odd)
    assert set(kb) == {_lib.GC_RNG_STREAM}
    for i, (u, v) in enumerate(zip(a, b)):
        assert np.array_equal(u, v), i
    assert sa[1] == sb[1] and np.array_equal(sa[0], sb[0])
    # the words above equal the oracle's too (first call, plain stream = torch's)
    torch.manual_seed(4321 + bits)
    ref, _, _ = _oracle_next(n)
    xs = x.cpu().numpy()
    exp = O.qsgd_encode(xs, float(nm.item()), bits, 1, O.stream_rng(ref))
    assert np.array_equal(a[0].view(np.uint32), np.asarray(exp, np.uint32))
    # and the first call went through the tie path: F = ceil(frac(l) 2^24)
    hb = 8 if fmt == "split8" else 16
    lv = (np.abs(xs) / np.float32(nm.item())).astype(np.float32) * np.float32((1 << bits) - 1)
    F = np.ceil((lv - np.floor(lv)).astype(np.float64) * 2.0 ** 24).astype(np.int64)
    r24 = np.asarray(ref, np.int64) & 0xFFFFFF
    ties = int(np.count_nonzero((F >= 1) & (((F - 1) >> (24 - hb)) == (r24 >> (24 - hb)))))
    assert ties >= 1
    codec.mt_release()


def test_mt_reserved_bytes_counts_the_queue_and_release_frees_it():
    """mt_reserved_bytes reports the draws queued ahead (plus workspaces and
    tables) and mt_release drops them."""
    codec.mt_release()
    torch.manual_seed(3)
    for _ in range(4):
        codec.mt19937_reserve(1_000_000, DEV, "split16")
    held = codec.mt_reserved_bytes(DEV)
    assert held >= codec.mt_format_bytes(1_000_000, "split16")
    codec.mt_release(DEV)
    assert codec.mt_reserved_bytes(DEV) < held
    assert DEV.index not in codec._MT_SPEC


def test_repeated_calls_are_served_from_the_queue_without_host_stalls():
    """Once a size repeats, every call takes its draws from the speculative
    queue (codec.mt_stats: no run made on demand), and a call that enqueues
    the next run does not block the host on the caller's stream: the end
    coefficients go up on the jump stream (_mt_upload_side).  The caller's
    stream is held busy meanwhile, so a synchronous upload on it would take
    the host as long as that work."""
    codec.mt_release()
    torch.manual_seed(11)
    count = 1_000_003
    for _ in range(3):
        codec.mt19937_reserve(count, DEV, "plain")
    codec._MT_ENDCAT.clear()  # new end blocks: every enqueue uploads again
    codec._MT_END_HOST.clear()
    codec.mt_stats(reset=True)
    a = torch.randn(4096, 4096, device=DEV)
    import time
    worst = 0.0
    for _ in range(12):
        for _ in range(4):
            a = a @ a
            a /= a.abs().max()  # keeps the caller's stream busy for milliseconds
        t0 = time.perf_counter()
        codec.mt19937_reserve(count, DEV, "plain")
        worst = max(worst, time.perf_counter() - t0)
    torch.cuda.synchronize()
    st = codec.mt_stats()
    assert st.get("queued", 0) == 12 and st.get("fresh", 0) == 0, st
    assert st.get("speculative_runs", 0) >= 1, st
    # the queued runs' host work is milliseconds at most; the busy stream holds ~4 x 4 GEMMs of 4096^3
    assert worst < 0.02, worst


def _as_draws24(got, kind, count):
    """The low 24 bits of each draw from a reservation of any format"""
    from gcodec import _lib
    if kind == _lib.GC_RNG_STREAM:
        return got.cpu().numpy().view(np.uint32) & 0xFFFFFF
    if kind == _lib.GC_RNG_STREAM24:
        b = got.cpu().numpy().view(np.uint8).reshape(-1, 3).astype(np.uint32)
        return b[:, 0] | b[:, 1] << 8 | b[:, 2] << 16
    hb = 8 if kind == _lib.GC_RNG_SPLIT8 else 16
    hi, lo = _split_planes(got, count, hb)
    return hi << (24 - hb) | lo


def test_randomised_schedule_vs_serial_stream():
    """200 torch-mode calls on a seeded random schedule,
    each call's draws (plain: all 32 bits; cut formats: the 24 the rounding
    reads) and torch's generator state after it compared with the serial
    MT19937 oracle.  The schedule mixes counts below / at / above 624 and
    multiples / non-multiples of 4 (repeated often, so the speculation and the
    multi-call runs are used), all four draw formats, changes of depth,
    calls per run and budget, interleaved torch.rand and torch.manual_seed,
    mt_release, and calls made on a side stream."""
    import random
    from gcodec import _lib
    rnd = random.Random(20261018)
    counts = [1, 3, 4, 100, 623, 624, 625, 1248, 4000, 4001, 20_000, 100_003, 262_084]
    fmts = ["plain", "packed24", "split8", "split16"]
    side = torch.cuda.Stream(DEV)
    saved = (codec.MT_SPECULATE_DEPTH, codec.MT_MULTI_CALLS, codec.MT_SPECULATE_BUDGET)
    codec.mt_release()
    torch.manual_seed(1)
    count, fmt = 624, "plain"
    try:
        for i in range(200):
            op = rnd.random()
            if op < 0.05:
                torch.rand(rnd.randint(1, 9))
            elif op < 0.08:
                torch.manual_seed(rnd.randint(0, 2 ** 31))
            elif op < 0.10:
                codec.mt_release()
            elif op < 0.13:
                codec.MT_SPECULATE_DEPTH = rnd.choice([0, 1, 2, 4, 8, 16])
            elif op < 0.16:
                codec.MT_MULTI_CALLS = rnd.choice([1, 2, 3, 8])
            elif op < 0.18:
                codec.MT_SPECULATE_BUDGET = rnd.choice([None, 4_000, 100_000, 1 << 30])
            if rnd.random() > 0.65:
                count = rnd.choice(counts)
            if rnd.random() > 0.75:
                fmt = rnd.choice(fmts)
            on_side = rnd.random() < 0.15
            ref, w2, i2 = _oracle_next(count)
            with torch.cuda.stream(side if on_side else torch.cuda.current_stream(DEV)):
                got, kind = codec.mt19937_reserve(count, DEV, fmt)
            torch.cuda.synchronize()
            tag = (i, count, fmt, kind, on_side)
            if kind == _lib.GC_RNG_STREAM:
                assert np.array_equal(got.cpu().numpy().view(np.uint32), ref), tag
            else:
                assert np.array_equal(_as_draws24(got, kind, count), np.asarray(ref, np.uint32) & 0xFFFFFF), tag
            words, idx = torch_mt_state()
            assert idx == i2 and np.array_equal(words, w2), tag
    finally:
        codec.MT_SPECULATE_DEPTH, codec.MT_MULTI_CALLS, codec.MT_SPECULATE_BUDGET = saved
        codec.mt_release()
