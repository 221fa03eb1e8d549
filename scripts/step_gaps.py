#!/usr/bin/env python3
"""Raw kernel timeline of consecutive bench steps from a rocprofv3 kernel trace: start,
end, duration and queue of every kernel between two step markers, so GPU idle time
between steps (host-bound gaps) is visible.

usage: step_gaps.py TRACE.csv [--marker k_coalesce] [--steps 2]
"""
from __future__ import annotations

import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="k_coalesce")
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(idx) < a.steps + 2:
        raise SystemExit("not enough steps in the trace")
    lo, hi = idx[-a.steps - 2], idx[-2]
    t0 = int(rows[lo]["Start_Timestamp"])
    busy_end = t0
    idle = 0
    for r in rows[lo:hi + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s > busy_end:
            idle += s - busy_end
        busy_end = max(busy_end, e)
        q = r.get("Queue_Id") or r.get("Stream_Id") or ""
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q:<3} "
              f"{r['Kernel_Name'][:48]}")
    span = int(rows[hi]["Start_Timestamp"]) - t0
    print(f"# {a.steps} steps: {span / 1e3 / a.steps:.1f} us/step, GPU idle "
          f"{idle / 1e3 / a.steps:.1f} us/step")


if __name__ == "__main__":
    main()
