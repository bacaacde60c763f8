"""Read a rocprofv3 kernel trace of tools/trace_pipeline.py: per pipeline call,
when each chunk's encode / decode ran, and whether decode(0) starts before the
last encode ends (the encode | all-reduce | decode overlap of SURVEY §8(e)).
Also the MT19937 kernels' average durations."""
import csv
import glob
import json
import statistics
import sys


def main(d):
    rows = []
    for p in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        with open(p) as f:
            rows += list(csv.DictReader(f))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ev = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    calls, cur = [], None
    for name, s, e in ev:
        if "k_absmax" in name and (cur is None or cur["enc"]):
            cur = {"absmax": (s, e), "enc": [], "dec": []}
            calls.append(cur)
        elif cur is not None and "k_qsgd_encode" in name:
            cur["enc"].append((s, e))
        elif cur is not None and "k_qsgd_decode" in name:
            cur["dec"].append((s, e))
    out = {"pipeline_calls": []}
    for c in calls:
        if len(c["enc"]) != 8 or len(c["dec"]) != 8:
            continue
        t0 = c["absmax"][0]
        out["pipeline_calls"].append({
            "us_total": (max(e for _, e in c["dec"]) - t0) / 1e3,
            "encode_us": [[round((s - t0) / 1e3, 1), round((e - t0) / 1e3, 1)] for s, e in c["enc"]],
            "decode_us": [[round((s - t0) / 1e3, 1), round((e - t0) / 1e3, 1)] for s, e in c["dec"]],
            "decode0_starts_before_last_encode_ends": c["dec"][0][0] < c["enc"][-1][1],
        })
    mt = {}
    for name, s, e in ev:
        for k in ("k_mt_seq", "k_mt_jump", "k_mt_gen"):
            if k in name:
                mt.setdefault(k, []).append((e - s) / 1e3)
    out["mt19937_us"] = {k: {"launches": len(v), "avg_us": statistics.mean(v)} for k, v in mt.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
