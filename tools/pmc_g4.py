"""Summarise tools/gpu.sh g4prof (rocprofv3 passes over tools/prof_packers.py,
the ResNet50 bucket: 23,520,842 4-bit magnitudes and sign bits) into
profiles/<tag>_g4_pmc.json: per packer kernel the mean duration, HBM bytes per
launch (2 * FETCH_SIZE + WRITE_SIZE, KiB; the gfx950 correction of
MI355X_MICROARCH.md 'HBM'), the SQ wait / issue fractions and LDS bank
conflicts per LDS instruction.  The traffic ratio is against the pack's
algorithmic bytes (4n read + 4 * words written) of the magnitudes' pack."""
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _short(name):
    name = name.split("(", 1)[0]
    return name.replace("void ", "").strip()[:80]


def _counters(d):
    vals = {}
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                k = _short(r.get("Kernel_Name", ""))
                vals.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return vals


def main(tag, n=23_520_842, words_xi=None):
    base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_g4")
    durs = {}
    for p in glob.glob(os.path.join(base, "trace", "**", "*kernel_trace.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                k = _short(r["Kernel_Name"])
                durs.setdefault(k, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    cnt = {}
    for which in ("fetch", "write", "sq", "lds"):
        for k, cs in _counters(os.path.join(base, which)).items():
            for c, v in cs.items():
                cnt.setdefault(k, {})[c] = v
    out = {"tag": tag, "workload": "tools/prof_packers.py (ResNet50 bucket, 4-bit xi then sign bits)", "n": n,
           "kernels": {}}
    for k in sorted(set(durs) | set(cnt)):
        if not (k.startswith("gc::k_g4") or k.startswith("k_g4") or "bytepack" in k or "byteunpack" in k):
            continue
        e = {}
        if k in durs:
            d = durs[k]
            e["launches"] = len(d)
            e["mean_us"] = statistics.mean(d) / 1e3
            e["median_us"] = statistics.median(d) / 1e3
        m = {c: statistics.median(v) for c, v in cnt.get(k, {}).items()}
        e.update(m)
        if "FETCH_SIZE" in m or "WRITE_SIZE" in m:
            e["hbm_bytes_per_launch"] = (2 * m.get("FETCH_SIZE", 0.0) + m.get("WRITE_SIZE", 0.0)) * 1024
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if c in m:
                    e[c.replace("SQ_", "frac_")] = m[c] / wc
        if m.get("SQ_INSTS_LDS"):
            e["lds_conflict_per_lds_inst"] = m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_INSTS_LDS"]
        out["kernels"][k] = e
    if words_xi:
        out["pack_algorithmic_bytes_xi"] = 4 * n + 4 * int(words_xi)
    path = os.path.join(ROOT, "profiles", f"{tag}_g4_pmc.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], words_xi=int(sys.argv[2]) if len(sys.argv) > 2 else None)
