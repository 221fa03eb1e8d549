"""Profiling helpers.

* ``shellac-prof out.prof`` prints the top 20 cumulative entries of a cProfile dump
  (reference: src/python/shellac/server/prof.py:1-9).
* ``shellac-prof --rocprof DIR`` summarises a ``rocprofv3 --kernel-trace --stats``
  output directory (per-kernel calls / total / average / share).
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import pstats
import sys
from typing import Optional, Sequence


def cprofile_top(path: str, n: int = 20) -> None:
    pstats.Stats(path).strip_dirs().sort_stats("cumulative").print_stats(n)


def rocprof_summary(directory: str, n: int = 25) -> list:
    files = glob.glob(os.path.join(directory, "**", "*kernel_stats.csv"), recursive=True)
    if not files:
        raise FileNotFoundError(f"no *kernel_stats.csv under {directory}")
    rows = []
    for f in files:
        rows.extend(csv.DictReader(open(f)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    out = []
    for r in rows[:n]:
        out.append((r["Name"][:90], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6,
                    float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    return out


def main(argv: Optional[Sequence[str]] = None) -> int:
    p = argparse.ArgumentParser(prog="shellac-prof")
    p.add_argument("path", help="cProfile dump, or rocprofv3 output dir with --rocprof")
    p.add_argument("--rocprof", action="store_true")
    p.add_argument("-n", type=int, default=20)
    a = p.parse_args(argv)
    if a.rocprof:
        print(f"{'kernel':90s} {'calls':>7s} {'total_ms':>10s} {'avg_us':>10s} {'pct':>6s}")
        for name, calls, tot, avg, pct in rocprof_summary(a.path, a.n):
            print(f"{name:90s} {calls:7d} {tot:10.3f} {avg:10.2f} {pct:6.2f}")
    else:
        cprofile_top(a.path, a.n)
    return 0


if __name__ == "__main__":
    sys.exit(main())
