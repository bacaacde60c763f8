"""Split tools/trace_ms_step.py's kernel trace at its marker kernels (neg_)
into the one-pass and the q-cache step sequences: per kernel its mean
duration in the sequence, and the mean gap before it (end of the previous
kernel to its start).
    python tools/ms_step_gaps.py <trace dir>"""
import csv
import glob
import statistics
import sys

rows = []
for p in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(p)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "neg" in r["Kernel_Name"].lower()][-3:]


def short(nm):
    return nm.split("(")[0].replace("void ", "")[:52]


for label, a, b in (("one-pass step", marks[0], marks[1]), ("q-cache step", marks[1], marks[2])):
    ks = rows[a + 1:b]
    d, g = {}, {}
    for prev, r in zip(rows[a:b], ks):
        k = short(r["Kernel_Name"])
        d.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        g.setdefault(k, []).append((int(r["Start_Timestamp"]) - int(prev["End_Timestamp"])) / 1e3)
    span = (int(ks[-1]["End_Timestamp"]) - int(ks[0]["Start_Timestamp"])) / 1e3
    steps = len(d[short(ks[0]["Kernel_Name"])])
    print(f"== {label}: {len(ks)} kernels, {span / steps:.1f} us per step")
    for k in d:
        print(f"   {k:52s} x{len(d[k]):4d} mean {statistics.mean(d[k]):6.2f} us, gap before it: mean "
              f"{statistics.mean(g[k]):5.2f} median {statistics.median(g[k]):5.2f} us")
