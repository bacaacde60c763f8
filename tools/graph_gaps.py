"""Split tools/prof_grandk_graph.py's rocprofv3 kernel trace at its marker
fills into the eager and the graph-replay phase; per phase the kernels per
step, their mean durations, and the mean gap between consecutive kernels
(end of one to the start of the next), split by the kind of boundary (inside
a step: encode -> decode-scatter; between steps: decode-scatter -> next
encode).
    python tools/graph_gaps.py <trace dir>"""
import csv
import glob
import statistics
import sys

rows = []
for p in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(p)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "neg" in r["Kernel_Name"].lower()]  # the marker neg_ kernels
marks = marks[-3:]
phases = {"eager": rows[marks[0] + 1:marks[1]], "graph replay": rows[marks[1] + 1:marks[2]]}


def short(n):
    return n.split("(")[0].replace("void ", "")[:48]


for name, ks in phases.items():
    names = sorted({short(r["Kernel_Name"]) for r in ks})
    print(f"== {name}: {len(ks)} kernels, queues {sorted({r['Queue_Id'] for r in ks})}")
    for nm in names:
        d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ks if short(r["Kernel_Name"]) == nm]
        print(f"   {nm:48s} x{len(d):4d} mean {statistics.mean(d) / 1e3:7.2f} us")
    gi, gb = [], []
    for a, b in zip(ks, ks[1:]):
        gap = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
        (gb if "encode" in b["Kernel_Name"] or "gather" in b["Kernel_Name"] else gi).append(gap)
    span = (int(ks[-1]["End_Timestamp"]) - int(ks[0]["Start_Timestamp"])) / 1e3
    steps = sum(1 for r in ks if "scatter" in r["Kernel_Name"])
    print(f"   gap inside a step  mean {statistics.mean(gi):7.2f} us, median {statistics.median(gi):7.2f}")
    if gb:
        print(f"   gap between steps  mean {statistics.mean(gb):7.2f} us, median {statistics.median(gb):7.2f}")
    print(f"   span {span:.1f} us over {steps} steps = {span / max(steps, 1):.2f} us per step")
