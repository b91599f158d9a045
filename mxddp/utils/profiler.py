"""Device-side phase timers (hipEvent-based) and roctx ranges.

``PhaseTimer`` brackets named phases (fwd / bwd / comm / opt) with GPU events on the current
stream and reports per-phase milliseconds without a host sync per step (events are resolved
lazily at ``summary()``).  ``range`` emits roctx markers that rocprofv3 --marker-trace picks up.
"""
from __future__ import annotations

import contextlib
from collections import defaultdict

import torch


class PhaseTimer:
    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self._pending = []
        self.totals = defaultdict(float)
        self.counts = defaultdict(int)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        try:
            yield
        finally:
            e.record()
            self._pending.append((name, s, e))

    def summary(self) -> dict:
        for name, s, e in self._pending:
            e.synchronize()
            self.totals[name] += s.elapsed_time(e)
            self.counts[name] += 1
        self._pending.clear()
        return {k: self.totals[k] / max(self.counts[k], 1) for k in self.totals}


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    pushed = False
    if torch.cuda.is_available():
        try:
            torch.cuda.nvtx.range_push(name)  # maps to roctx on ROCm builds
            pushed = True
        except Exception:
            pushed = False
    try:
        yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()
