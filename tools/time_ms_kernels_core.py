"""hold() + timed(): a kernel's mean time over REPS launches queued behind a
GPU hold, so the host's issue rate does not show (shared by the MS timing
scripts)."""
import time

import torch

REPS = 50


def hold(ms):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    torch.cuda._sleep(1_000_000)
    e.record()
    e.synchronize()
    torch.cuda._sleep(int(ms / max(s.elapsed_time(e), 1e-3) * 1e6))


def timed(fn):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        fn()
    issue_ms = (time.perf_counter() - t0) / 3 * 1e3
    torch.cuda.synchronize()
    hold(1.5 * issue_ms * REPS + 0.5)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(REPS):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / REPS * 1e3
