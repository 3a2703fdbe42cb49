"""Per-phase wall-clock timers (the reference has none) — device-synchronising on demand so
phase times are real GPU times, plus a roctx-style range helper for rocprofv3 timelines."""
from __future__ import annotations

import contextlib
import time
from collections import defaultdict

import torch


class PhaseTimer:
    def __init__(self, sync=False):
        self.sync = sync
        self.total = defaultdict(float)
        self.count = defaultdict(int)

    @contextlib.contextmanager
    def phase(self, name):
        if self.sync and torch.cuda.is_available():
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        try:
            with range_push(name):
                yield
        finally:
            if self.sync and torch.cuda.is_available():
                torch.cuda.synchronize()
            self.total[name] += time.perf_counter() - t0
            self.count[name] += 1

    def summary(self):
        return {k: {"s": round(v, 4), "n": self.count[k]} for k, v in self.total.items()}


@contextlib.contextmanager
def range_push(name):
    """Annotate a range for rocprofv3 --marker-trace (no-op without a GPU)."""
    pushed = False
    try:
        if torch.cuda.is_available():
            torch.cuda.nvtx.range_push(name)
            pushed = True
    except Exception:  # noqa: BLE001 - markers are best effort
        pushed = False
    try:
        yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()
