"""Per-(kernel, launch shape) duration statistics from a rocprofv3 kernel trace.

rocprofv3 --stats averages a kernel over every launch of that name; the bench
launches k_qsgd_encode at several bucket sizes (the 100M headline, the 4M
pipelined self-check, the GRandK subsets, ...), so its average mixes them.
This splits the trace by (kernel template, grid, workgroup) and writes

    name, grid, workgroup, calls, mean_ns, median_ns, min_ns, max_ns, std_ns, std_pct

    python tools/kstats.py <trace dir> <out.csv> [min_calls]
"""
import collections
import csv
import glob
import statistics
import sys


def main(src, dst, min_calls=1):
    groups = collections.defaultdict(list)
    for p in glob.glob(f"{src}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            key = (name, int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))
            groups[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    rows = []
    for (name, grid, wg), d in groups.items():
        if len(d) < min_calls:
            continue
        mean = statistics.mean(d)
        sd = statistics.pstdev(d)
        rows.append([name, grid, wg, len(d), round(mean), round(statistics.median(d)), min(d), max(d), round(sd),
                     round(100.0 * sd / mean, 2) if mean else 0.0])
    rows.sort(key=lambda r: -r[3] * r[4])
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["name", "grid", "workgroup", "calls", "mean_ns", "median_ns", "min_ns", "max_ns", "std_ns",
                    "std_pct"])
        w.writerows(rows)
    for r in rows[:25]:
        print(f"{r[0][:70]:70s} grid {r[1]:>9} wg {r[2]:>4} x{r[3]:<5} mean {r[4] / 1e3:8.1f} us  "
              f"median {r[5] / 1e3:8.1f}  std {r[9]:5.1f}%")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 1)
