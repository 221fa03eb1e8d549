"""Timeline markers and per-stage timers for the serving path.

The reference only has offline cProfile (prof.py:3-8). Here every serving phase can
be seen on the rocprofv3 timeline next to the HIP kernels it launches:

    SHELLAC_TRACE=1 rocprofv3 --marker-trace --kernel-trace -d out -- python3 bench.py

``trace_range("name")`` pushes an ROCTX range (a no-op branch unless tracing is on;
the native HbmCache / HbmBackend entry points carry their own ranges), and
``StageTimer`` accumulates host wall time per stage for the stats endpoint / logs.
"""
from __future__ import annotations

import contextlib
import time
from collections import defaultdict

from .._native import core


def enable(on: bool = True) -> None:
    core().trace_enable(bool(on))


def enabled() -> bool:
    return bool(core().trace_on())


@contextlib.contextmanager
def trace_range(name: str):
    c = core()
    if not c.trace_on():
        yield
        return
    c.trace_push(name)
    try:
        yield
    finally:
        c.trace_pop()


def mark(name: str) -> None:
    core().trace_mark(name)


class StageTimer:
    """Accumulated host wall time per named stage (cheap: two perf_counter calls)."""

    def __init__(self):
        self.total = defaultdict(float)
        self.count = defaultdict(int)

    @contextlib.contextmanager
    def stage(self, name: str):
        t0 = time.perf_counter()
        with trace_range(name):
            yield
        self.total[name] += time.perf_counter() - t0
        self.count[name] += 1

    def summary(self) -> dict:
        return {k: {"calls": self.count[k], "ms_total": round(self.total[k] * 1e3, 3),
                    "us_mean": round(self.total[k] * 1e6 / max(self.count[k], 1), 2)}
                for k in sorted(self.total)}
