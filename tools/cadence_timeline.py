"""Timeline of tools/trace_torch_cadence.py's rocprofv3 kernel trace: every
kernel's start / end (us from the first GEMM of the traced calls) and queue,
then per call (one per absmax launch) where its GEMMs, the jumps and
generators of the runs in flight and its encode ran, and how long the GPU was
busy beyond the GEMMs.
    python tools/cadence_timeline.py <trace dir> > profiles/<tag>_torch_cadence_timeline.txt"""
import csv
import glob
import sys


def short(name):
    for k in ("Cijk", "gemm", "k_mt_seq", "k_mt_jump", "k_mt_end", "k_mt_gen", "k_qsgd_encode", "k_absmax"):
        if k in name:
            return "gemm" if k in ("Cijk", "gemm") else k
    return name.split("(")[0][:40]


rows = []
for p in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(p)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]) for r in rows]
ab = [i for i, k in enumerate(ks) if k[0] == "k_absmax"]
calls = ab[-8:] if len(ab) >= 8 else ab
first = calls[0]
g0 = max(i for i in range(first) if ks[i][0] == "gemm") - 2  # the 3 GEMMs before the first traced call
t0 = ks[g0][1]
print("kernel                start_us     end_us    dur_us  queue")
for k in ks[g0:]:
    print(f"{k[0]:18s} {(k[1] - t0) / 1e3:10.1f} {(k[2] - t0) / 1e3:10.1f} {(k[2] - k[1]) / 1e3:9.1f}  q{k[3]}")
print()
print("per call: GEMM span, side-stream (jump/gen) kernels overlapping the GEMMs, the call's absmax+encode,")
print("and the time from the last GEMM's end to the encode's end (what the call adds to a backward)")
for j, ia in enumerate(calls):
    gems = [k for k in ks[:ia] if k[0] == "gemm"][-3:]
    gs, ge = gems[0][1], gems[-1][2]
    enc = next(k for k in ks[ia:] if k[0] == "k_qsgd_encode")
    side = [k for k in ks if k[0] in ("k_mt_jump", "k_mt_gen", "k_mt_seq", "k_mt_end") and k[1] < ge and k[2] > gs]
    busy = sum(min(k[2], ge) - max(k[1], gs) for k in side)
    print(f"call {j}: gemms {(gs - t0) / 1e3:9.1f}-{(ge - t0) / 1e3:9.1f}  side kernels inside: {len(side):3d} "
          f"({busy / 1e3:7.1f} us summed)  absmax {(ks[ia][1] - t0) / 1e3:9.1f}  encode "
          f"{(enc[1] - t0) / 1e3:9.1f}-{(enc[2] - t0) / 1e3:9.1f}  added {(enc[2] - ge) / 1e3:7.1f} us")
