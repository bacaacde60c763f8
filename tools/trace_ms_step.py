"""Config 3's TS (2,4) steps on the ResNet50 bucket as bench.py times them
(absmax -> one-pass encode -> decode at W = 1; absmax -> mask + q cache ->
select from the cache -> decode for the q-cache form), STEPS of each in a
row, for a rocprofv3 kernel trace: per kernel its duration inside the step
sequence, and the gaps between consecutive kernels (tools/ms_step_gaps.py).
With TIME=1 (no profiler) it prints each form's per-step time and host issue
time."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))
import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402

STEPS = int(os.environ.get("STEPS", "100"))
dev = torch.device("cuda", 0)
n = 23_520_842
x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(11)).mul_(0.01)
nrm = torch.empty(1, device=dev)
gen = gcodec.Generator(5, "philox")
one = gcodec.QSGDMaxNormTwoScaleCompressor(dev, 2, 4, generator=gen)
qc = gcodec.QSGDMaxNormTwoScaleCompressor(dev, 2, 4, generator=gen, q_cache=True)
out = torch.empty(n, device=dev)
mark = torch.zeros(1, device=dev)


def step_one():
    codec.absmax(x, out=nrm)
    m, w = one.encode_w1(nrm, x)
    one.decode(nrm, w, m, n, 1, 1.0, out=out)


def step_qc():
    codec.absmax(x, out=nrm)
    m = qc.encode_mask(nrm, x, 1)
    w = qc.encode(nrm, x, m, 1)
    qc.decode(nrm, w, m, n, 1, 1.0, out=out)


# the one-pass step as bare C-ABI calls with every argument built once (no
# codec / compressor Python per call): separates host-side from GPU-side cost
from gcodec import _lib  # noqa: E402
import ctypes as C  # noqa: E402

lib = _lib.load()
lvls = one._packed_levels()
ql, ml = codec.ms_layouts(n, lvls, 1)
lvs = codec.levels_struct(lvls)
mw_raw = torch.empty(codec.mask_words_total(ml, lvls), dtype=torch.int32, device=dev)
w_raw = torch.empty(ql.plane_words, dtype=torch.int32, device=dev)
rs = gen.reserve(n, len(lvls), dev).struct()
st = codec._stream(dev)
ws_raw = codec._absmax_ws(dev, st)
P = (x.data_ptr(), nrm.data_ptr(), ws_raw.data_ptr(), mw_raw.data_ptr(), w_raw.data_ptr(), out.data_ptr())
refs = (C.byref(lvs), C.byref(rs), C.byref(ml), C.byref(ql))


def step_raw():
    lib.gc_absmax_f32(P[0], None, n, P[1], P[2], st)
    lib.gc_ms_encode_w1(P[0], n, P[1], refs[0], refs[1], refs[2], refs[3], P[3], P[4], st)
    lib.gc_ms_decode(P[4], P[3], None, n, P[1], refs[0], refs[2], refs[3], 1, 1.0, P[5], st)


for _ in range(10):
    step_one()
    step_qc()
    step_raw()
torch.cuda.synchronize()
if os.environ.get("ALIGN") == "1":  # x's base address: the one-pass kernel alone and the bare step
    big = torch.empty(n + (1 << 21), device=dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for off_bytes in (4096,):
        xs = big[off_bytes // 4:off_bytes // 4 + n]
        xs.copy_(x)
        Px = (xs.data_ptr(),) + P[1:]
        def enc():
            lib.gc_ms_encode_w1(Px[0], n, Px[1], refs[0], refs[1], refs[2], refs[3], Px[3], Px[4], st)
        def stp():
            lib.gc_absmax_f32(Px[0], None, n, Px[1], Px[2], st)
            enc()
            lib.gc_ms_decode(Px[4], Px[3], None, n, Px[1], refs[0], refs[2], refs[3], 1, 1.0, Px[5], st)
        def stp0():  # decode order 0
            lib.gc_absmax_f32(Px[0], None, n, Px[1], Px[2], st)
            enc()
            lib.gc_ms_decode(Px[4], Px[3], None, n, Px[1], refs[0], refs[2], refs[3], 0, 1.0, Px[5], st)
        def am_enc():
            lib.gc_absmax_f32(Px[0], None, n, Px[1], Px[2], st)
            enc()
        def enc_dec():
            enc()
            lib.gc_ms_decode(Px[4], Px[3], None, n, Px[1], refs[0], refs[2], refs[3], 1, 1.0, Px[5], st)
        mw_alt, w_alt = mw_raw.clone(), w_raw.clone()

        def enc_dec_other():  # the decode reads words / mask the encode did not just write
            enc()
            lib.gc_ms_decode(w_alt.data_ptr(), mw_alt.data_ptr(), None, n, Px[1], refs[0], refs[2], refs[3], 1, 1.0,
                             Px[5], st)

        def enc_enc():
            enc()
            enc()

        def dec1():
            lib.gc_ms_decode(Px[4], Px[3], None, n, Px[1], refs[0], refs[2], refs[3], 1, 1.0, Px[5], st)
        def dec0():
            lib.gc_ms_decode(Px[4], Px[3], None, n, Px[1], refs[0], refs[2], refs[3], 0, 1.0, Px[5], st)
        def am():
            lib.gc_absmax_f32(Px[0], None, n, Px[1], Px[2], st)
        for name, fn in (("one-pass alone", enc), ("bare step", stp), ("bare step, decode order 0", stp0),
                         ("absmax + one-pass", am_enc), ("one-pass + decode", enc_dec),
                         ("one-pass + decode of other words", enc_dec_other), ("one-pass x2", enc_enc), ("decode order 1 alone", dec1),
                         ("decode order 0 alone", dec0), ("absmax alone", am)):
            for _ in range(5):
                fn()
            ev0.record()
            for _ in range(STEPS):
                fn()
            ev1.record()
            torch.cuda.synchronize()
            print(f"x at base + {off_bytes:8d} B (addr % 2 MiB = {Px[0] % (1 << 21):8d}): {name} "
                  f"{ev0.elapsed_time(ev1) / STEPS * 1e3:.1f} us", flush=True)
    sys.exit(0)
if os.environ.get("TIME") == "1":
    for name, fn in (("one-pass", step_one), ("one-pass, bare C-ABI calls", step_raw), ("q cache", step_qc)):
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(STEPS):
                fn()
            host = (time.perf_counter() - t0) / STEPS * 1e6
            torch.cuda.synchronize()
            el = (time.perf_counter() - t0) / STEPS * 1e6
            print(f"{name}: {el:.1f} us per step, host issue {host:.1f} us", flush=True)
else:
    mark.neg_()
    for _ in range(STEPS):
        step_one()
    mark.neg_()
    for _ in range(STEPS):
        step_qc()
    mark.neg_()
    torch.cuda.synchronize()
print("done")
