"""Where a back-to-back torch-mode call's time goes (1e8 fp32, 4-bit, W = 1,
product defaults): the host's enqueue time per call (no sync inside the
loop) beside the wall time, for a rocprofv3 kernel trace of the same loop.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python tools/trace_torch_mode.py
    python tools/trace_torch_mode.py --analyse OUT/run_kernel_trace.csv

The analysis splits the traced loop (the calls after the warmup) into the
main stream's absmax / encode busy time, the generator walkers' busy time and
the main stream's idle gaps.
"""
import csv
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def analyse(path):
    rows = list(csv.DictReader(open(path)))
    ks = []
    for r in rows:
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", ""),
                   r.get("Stream_Id", "")))
    ks.sort()
    ab = [k for k in ks if "k_absmax" in k[2]]
    nc = int(os.environ.get("CALLS", "39"))  # whole calls analysed: the timed loop's but its last
    if len(ab) < nc + 2:
        print("too few absmax launches", len(ab))
        return
    t0, t1 = ab[-nc - 1][0], ab[-1][0]
    win = [k for k in ks if k[0] < t1 and k[1] > t0]

    def busy(sel):
        iv = sorted((max(s, t0), min(e, t1)) for s, e, n, *_ in win if sel(n))
        tot, cur_s, cur_e = 0, None, None
        for s, e in iv:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    tot += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            tot += cur_e - cur_s
        return tot / nc / 1e3

    span = (t1 - t0) / nc / 1e3
    names = sorted({n.split("(")[0] for _, _, n, *_ in win})
    print(f"per call over {nc} calls: {span:.1f} us")
    for nm in names:
        c = sum(1 for k in win if k[2].split("(")[0] == nm)
        print(f"  {nm[:70]:70s} launches {c / nc:5.2f}/call  busy {busy(lambda n, nm=nm: n.split('(')[0] == nm):7.1f} us/call")
    main = busy(lambda n: "k_absmax" in n or "k_qsgd_encode" in n)
    gen = busy(lambda n: "k_mt_" in n)
    anyk = busy(lambda n: True)
    print(f"  main-stream (absmax + encode) busy {main:.1f} us/call, MT kernels busy {gen:.1f}, any kernel {anyk:.1f}")


def run():
    sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))
    import torch

    import gcodec
    from gcodec import codec

    dev = torch.device("cuda", 0)
    n = 100_000_000
    x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(1)).mul_(0.01)
    nm = codec.absmax(x)
    lanes = codec.qsgd_layout(n, 4, 1)
    words = torch.empty(lanes.plane_words, dtype=torch.int32, device=dev)
    gen = gcodec.Generator(0, "torch")
    fmt = os.environ.get("FMT", "plain")
    torch.manual_seed(42)

    def step():
        codec.absmax(x, out=nm)
        codec.qsgd_encode(x, nm, 4, gen.reserve(n, fmt=fmt), 1, out=words, lanes=lanes)

    for _ in range(int(os.environ.get("WARM", "24"))):
        step()
    torch.cuda.synchronize()
    codec.mt_stats(reset=True)
    reps = int(os.environ.get("REPS", "40"))
    t0 = time.perf_counter()
    host = []
    for _ in range(reps):
        h0 = time.perf_counter()
        step()
        host.append(time.perf_counter() - h0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("reserve paths in the timed loop:", codec.mt_stats(), flush=True)
    host.sort()
    print(f"fmt {fmt}: wall {(t2 - t0) / reps * 1e3:.3f} ms per call, host enqueue {(t1 - t0) / reps * 1e3:.3f} ms "
          f"per call (median {host[reps // 2] * 1e3:.3f}, max {host[-1] * 1e3:.3f})", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyse":
        analyse(sys.argv[2])
    else:
        run()
