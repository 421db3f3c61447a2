"""Tracing / profiling helpers.

* ``prof_range(name)`` -- a ``torch.profiler.record_function`` range (shows up in torch.profiler traces
  and as a roctx-style marker) when ``DALLE_AMD_PROFILE=1``; a no-op otherwise.
* ``StepTimer`` -- wall-clock per phase (fwd / bwd / averaging / optimizer) with device sync, for the
  samples/s accounting that the reference reports through its performance EMA.
* Kernel-level evidence comes from ``rocprofv3 --kernel-trace --stats`` (see scripts/ and profiles/).
"""
from __future__ import annotations

import contextlib
import os
import time
from collections import defaultdict

import torch

_ENABLED = os.environ.get("DALLE_AMD_PROFILE") == "1"


@contextlib.contextmanager
def prof_range(name: str):
    if not _ENABLED:
        yield
        return
    with torch.profiler.record_function(name):
        yield


class StepTimer:
    def __init__(self, sync: bool = True):
        self.sync = sync and torch.cuda.is_available()
        self.totals = defaultdict(float)
        self.counts = defaultdict(int)

    @contextlib.contextmanager
    def __call__(self, name: str):
        if self.sync:
            torch.cuda.synchronize()
        t = time.perf_counter()
        with prof_range(name):
            yield
        if self.sync:
            torch.cuda.synchronize()
        self.totals[name] += time.perf_counter() - t
        self.counts[name] += 1

    def summary(self) -> dict:
        return {k: round(self.totals[k] / max(1, self.counts[k]) * 1e3, 3) for k in self.totals}
