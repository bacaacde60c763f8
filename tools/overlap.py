"""Timeline of a rocprofv3 kernel trace: per kernel start/end relative to the
first, with the stream (queue) id; shows which kernels ran concurrently.
    python tools/overlap.py <trace dir> [name filter]"""
import csv
import glob
import sys

rows = []
for p in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(p)))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
rows = [r for r in rows if flt in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"]) if rows else 0
for r in rows[-60:]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"q{r['Queue_Id']:>3} {s / 1e3:10.1f} {e / 1e3:10.1f} {(e - s) / 1e3:8.1f}  {r['Kernel_Name'][:60]}")
