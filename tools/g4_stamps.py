"""Lab: the persistent greedy4 pack's phase times per block (round 0), from a
build with GC_G4_STAMPS=1 (make -C gradient-compression_amd/csrc stamps; run
with GCODEC_LIB=<repo>/gradient-compression_amd/lib/libgcodec_stamps.so).
Prints, over the blocks, the median / min / max of each phase's duration and
of each boundary's time from the earliest block start (s_memrealtime, 10 ns)."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gradient-compression_amd"))

import torch  # noqa: E402

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402

PH = ["load", "classes+dp", "trees+publish", "granule wait", "compose+walk", "lists+pack"]


def main():
    dev = torch.device("cuda", 0)
    n = int(os.environ.get("N", "23520842"))
    g = torch.Generator(device=dev).manual_seed(21)
    x = torch.randn(n, device=dev, generator=g).mul_(0.01)
    nm = codec.absmax(x)
    xi, sg = codec.qsgd_quantize_split(x, nm, 4, gcodec.Generator(7, "philox").reserve(n))
    pk = codec.Greedy4Device(n, dev)
    for src_name, src in (("xi", xi), ("sign", sg)):
        for _ in range(50):
            pk.pack(src)
        torch.cuda.synchronize()
        ws = pk.ws.view(torch.int64)
        off = (256 + 2 * 256 * 16 * 8) // 8
        st = ws[off:off + 256 * 8].view(256, 8).cpu()
        nb = int((st[:, 0] != 0).sum())
        st = st[:nb, :len(PH) + 1].double() * 10e-3  # us
        t0 = float(st[:, 0].min())
        print(f"== {src_name}: {nb} blocks, words {pk.result()}")
        print("  starts spread: %.2f us" % (float(st[:, 0].max()) - t0))
        for i, nm_ in enumerate(PH):
            d = (st[:, i + 1] - st[:, i]).tolist()
            e = (st[:, i + 1] - t0).tolist()
            print("  %-26s dur med %6.2f min %6.2f max %6.2f | ends at med %6.2f max %6.2f" %
                  (nm_, statistics.median(d), min(d), max(d), statistics.median(e), max(e)))


if __name__ == "__main__":
    main()
