#!/usr/bin/env python3
"""Per-step kernel statistics of a rocprofv3 --kernel-trace CSV of bench.py: the last
`--steps` steps, delimited by the launches of a marker kernel (default: the step's first
kernel, k_coalesce), as markdown: per-kernel time per step, then the last step's timeline
(queue, start, duration).

usage: step_kernel_stats.py TRACE.csv [--steps 8] [--marker k_coalesce] [--title T]
"""
import argparse
import csv
import re
from collections import defaultdict


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n).replace("shellac::", "")
    m = re.match(r"([\w:]+(<[^()]*?>)?)", n)
    b = m.group(1) if m else n
    return b.split("<")[0] if b.startswith(("at::", "rocprim", "ncclDevKernel")) else b[:48]


ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--steps", type=int, default=8)
ap.add_argument("--marker", default="k_coalesce")
ap.add_argument("--title", default="bench.py kernel trace")
a = ap.parse_args()
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
               r.get("Queue_Id", "")) for r in csv.DictReader(open(a.trace)))
marks = [s for s, _, n, _ in rows if n.startswith(a.marker)]
# the same marker kernel can run on two queues per step (e.g. routed: replica + owner):
# take one per step, the first after a gap
starts = []
for s in marks:
    if not starts or s - starts[-1] > 20_000:
        starts.append(s)
st = starts[-a.steps - 1:]
t0, t1 = st[0], st[-1]
k = len(st) - 1
tot = defaultdict(lambda: [0, 0])
for s, e, n, _ in rows:
    if t0 <= s < t1:
        tot[n][0] += 1
        tot[n][1] += e - s
busy = sum(v[1] for v in tot.values())
print(f"# {a.title}\n")
print(f"Last {k} steps: wall {(t1 - t0) / 1e3 / k:.1f} µs/step (step start to step start), "
      f"kernel time {busy / 1e3 / k:.1f} µs/step (kernels on two streams overlap).\n")
print("| kernel | calls/step | µs/step | µs/call |\n|---|---:|---:|---:|")
for n, (c, d) in sorted(tot.items(), key=lambda x: -x[1][1]):
    print(f"| `{n}` | {c / k:.1f} | {d / 1e3 / k:.1f} | {d / 1e3 / c:.1f} |")
a0, a1 = st[-2], st[-1]
print("\n## Timeline of the last step\n\n| queue | start µs | end µs | µs | kernel |\n|---|---:|---:|---:|---|")
for s, e, n, q in rows:
    if a0 <= s < a1:
        print(f"| {q} | {(s - a0) / 1e3:.1f} | {(e - a0) / 1e3:.1f} | {(e - s) / 1e3:.1f} | `{n}` |")
