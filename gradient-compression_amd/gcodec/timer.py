"""Phase timer with the reference's interface and labels (timer.py:10-163),
timed with HIP events on the rank's own current stream instead of
host wall clock + torch.cuda.synchronize() of device 0 (timer.py:146-149 never
sets the device, so rank != 0 synchronised the wrong GPU)."""
from __future__ import annotations

import json
from contextlib import contextmanager

import torch


class Timer:
    def __init__(self, verbosity_level=1, skip_first=True, on_cuda=True):
        self.verbosity_level = verbosity_level
        self.skip_first = skip_first
        self.on_cuda = on_cuda and torch.cuda.is_available()
        self.reset()

    def reset(self):
        self._events = {}  # label -> list of (start, end) events
        self.call_counts = {}

    @contextmanager
    def __call__(self, label, epoch=-1.0, verbosity=1):
        if verbosity > self.verbosity_level or not self.on_cuda:
            yield
            return
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        yield
        e.record()
        cnt = self.call_counts.get(label, 0) + 1
        self.call_counts[label] = cnt
        if not (self.skip_first and cnt == 1):
            self._events.setdefault(label, []).append((s, e))

    def totals(self):
        torch.cuda.synchronize()
        return {k: sum(s.elapsed_time(e) for s, e in v) / 1e3 for k, v in self._events.items()}

    def summary(self):
        tot = self.totals()
        return {k: {"label": k, "average_duration": tot[k] / len(self._events[k]), "n_events": len(self._events[k]),
                    "total_time": tot[k]} for k in tot}

    def save_summary(self, path):
        with open(path, "w") as f:
            json.dump(self.summary(), f, indent=1)
