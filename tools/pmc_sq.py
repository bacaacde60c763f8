"""Summarise the SQ / LDS counter passes of tools/gpu.sh kprof (prof_<tag>_k)
into profiles/<tag>_k_sq.json: per kernel, the median per launch of every
counter, and the wait / issue fractions of SQ_WAVE_CYCLES."""
import csv
import glob
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import ROOT, _short  # noqa: E402


def main(tag):
    vals = {}
    for which in ("sq", "lds"):
        for p in glob.glob(os.path.join(ROOT, "gpurun_out", f"prof_{tag}_k", which, "**", "*counter_collection.csv"),
                           recursive=True):
            with open(p) as f:
                for r in csv.DictReader(f):
                    k = _short(r.get("Kernel_Name", ""))
                    if not k.startswith("k_"):
                        continue
                    vals.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    out = {"tag": tag, "workload": "tools/prof_kernels.py", "kernels": {}}
    for k, cs in sorted(vals.items()):
        m = {c: statistics.median(v) for c, v in cs.items()}
        wc = m.get("SQ_WAVE_CYCLES") or 0.0
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if c in m:
                    m[c.replace("SQ_", "frac_")] = m[c] / wc
        out["kernels"][k] = m
    for name in (f"{tag}_k_sq.json", "pmc_sq.json"):  # pmc_sq.json: the latest, read by bench.py
        with open(os.path.join(ROOT, "profiles", name), "w") as fh:
            json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r02q")
