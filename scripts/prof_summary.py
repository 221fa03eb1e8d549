#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of bench.py into markdown.

Two views: (1) per-kernel totals over the timed steps only (everything after the
(steps)-th-from-last k_probe launch, so the populate phase is excluded), and (2) a
timeline of the last step (start offset, duration and gap per kernel).

usage: prof_summary.py TRACE.csv --steps K [--title T] > out.md
"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = re.sub(r"^void ", "", n)
    m = re.match(r"([\w:]+(<[^()]*?>)?)", n)
    base = m.group(1) if m else n
    if base.startswith("at::native::") or base.startswith("rocprim"):
        base = base.split("<")[0]
    return base.replace("shellac::", "")[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--marker", default="k_probe", help="kernel that opens each step")
    ap.add_argument("--title", default="bench.py kernel trace")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if a.marker in r[2]]
    if len(marks) < a.steps:
        raise SystemExit(f"only {len(marks)} '{a.marker}' launches")
    first = marks[-a.steps]
    timed = rows[first:]
    span_ns = timed[-1][1] - timed[0][0]
    tot = defaultdict(lambda: [0, 0])
    for s, e, n in timed:
        tot[short(n)][0] += 1
        tot[short(n)][1] += e - s
    busy = sum(v[1] for v in tot.values())
    print(f"# {a.title}\n")
    print(f"Last {a.steps} steps: wall {span_ns / 1e3 / a.steps:.1f} us/step (first kernel start to "
          f"last kernel end), GPU busy {busy / 1e3 / a.steps:.1f} us/step "
          f"({100.0 * busy / span_ns:.0f}%).\n")
    print("| kernel | calls/step | us/step | avg us | % busy |\n|---|---:|---:|---:|---:|")
    for k, (c, d) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"| `{k}` | {c / a.steps:.1f} | {d / 1e3 / a.steps:.1f} | {d / 1e3 / c:.1f} | "
              f"{100.0 * d / busy:.1f} |")
    last = rows[marks[-1]:]
    t0 = last[0][0]
    print("\n## Timeline of the last step\n")
    print("| start us | dur us | gap before us | kernel |\n|---:|---:|---:|---|")
    prev_end = t0
    for s, e, n in last:
        print(f"| {(s - t0) / 1e3:.1f} | {(e - s) / 1e3:.1f} | {(s - prev_end) / 1e3:.1f} | `{short(n)}` |")
        prev_end = max(prev_end, e)


if __name__ == "__main__":
    main()
