"""Summarise a tools/gpu.sh driver / pmc run into profiles/:
  profiles/<tag>_kernel_stats.csv   (rocprofv3 --stats, copied)
  profiles/<tag>_pmc.json           (per-kernel HBM bytes per launch)
  profiles/pmc_traffic.json         (latest, read by bench.py for roofline.traffic)
HBM bytes per launch = 2 * FETCH_SIZE (gfx950 reports half of a wide streaming
read, MI355X_MICROARCH.md 'HBM') + WRITE_SIZE, both in KiB from rocprofv3."""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rows(pattern):
    for p in glob.glob(pattern, recursive=True):
        with open(p) as f:
            yield from csv.DictReader(f)


KERNELS = ("k_qsgd_encode", "k_absmax", "k_qsgd_decode", "k_ms_fused_w1", "k_ms_mask_fast", "k_ms_select_fast",
           "k_ms_select_cache",
           "k_ms_decode_fast", "k_mt_seq", "k_mt_jump", "k_mt_gen", "k_randk_gather", "k_decode_scatter1")


def _short(name):
    for k in KERNELS:
        if k in name:
            if k == "k_ms_mask_fast":  # <LM, KIND, NL, VAR, CBY>: CBY > 0 also writes the q cache
                targs = name.split("<", 1)[1].split(">", 1)[0].split(",") if "<" in name else []
                # the octet kernel k_ms_mask_fast_o2<LM, VAR, CBY>
                cby = targs[2] if "k_ms_mask_fast_o2" in name and len(targs) >= 3 else (
                    targs[4] if len(targs) >= 5 else "0")
                if cby.strip() != "0":
                    return k + "_cache"
            return k
    return name[:60]


def counter(tag, which, cname):
    vals = {}
    for r in _rows(os.path.join(ROOT, "gpurun_out", f"prof_{tag}", which, "**", "*counter_collection.csv")):
        if r.get("Counter_Name") != cname:
            continue
        vals.setdefault(_short(r.get("Kernel_Name", "")), []).append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in vals.items()}


def main(tag, n=100_000_000, bits=4):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    if stats:
        shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    fetch = counter(tag, "fetch", "FETCH_SIZE")
    write = counter(tag, "write", "WRITE_SIZE")
    out = {"tag": tag, "n": n, "bits": bits, "units": "bytes per launch",
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; hbm = (2*FETCH_SIZE + WRITE_SIZE)*1024",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k), write.get(k)
        out["kernels"][k] = {"fetch_size_kib_raw": f, "write_size_kib": w,
                             "hbm_bytes_per_launch": None if f is None or w is None else (2 * f + w) * 1024}
    # the per-kernel workload of tools/prof_kernels.py (tools/gpu.sh kprof -> prof_<tag>_k)
    if os.path.isdir(os.path.join(ROOT, "gpurun_out", f"prof_{tag}_k")):
        kf, kw = counter(f"{tag}_k", "fetch", "FETCH_SIZE"), counter(f"{tag}_k", "write", "WRITE_SIZE")
        kstats = glob.glob(os.path.join(ROOT, "gpurun_out", f"prof_{tag}_k", "trace", "**", "*kernel_stats.csv"),
                           recursive=True)
        if kstats:
            shutil.copy(kstats[0], os.path.join(ROOT, "profiles", f"{tag}_k_kernel_stats.csv"))
        out["prof_kernels"] = {"workload": "tools/prof_kernels.py (see its docstring)", "kernels": {
            k: {"fetch_size_kib_raw": kf.get(k), "write_size_kib": kw.get(k),
                "hbm_bytes_per_launch": None if kf.get(k) is None or kw.get(k) is None else (2 * kf[k] + kw[k]) * 1024}
            for k in sorted(set(kf) | set(kw))}}
    else:  # keep the last per-kernel workload passes in the latest summary (tagged)
        try:
            with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as fh:
                prev = json.load(fh)
            if "prof_kernels" in prev:
                out["prof_kernels"] = dict(prev["prof_kernels"], tag=prev["prof_kernels"].get("tag", prev.get("tag")))
        except (OSError, ValueError):
            pass
    for name in (f"{tag}_pmc.json", "pmc_traffic.json"):
        with open(os.path.join(ROOT, "profiles", name), "w") as fh:
            json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
