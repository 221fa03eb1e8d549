#!/usr/bin/env python3
"""Response-time plot from ab-style -g TSVs (reference: benchmarks/requests.p plots
column 9 = ttime for baseline/shellac/varnish) and a memory plot from a CSV of
`name,used_MB` rows (reference: benchmarks/memory.p over dstat output)."""
import csv
import os

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402

here = os.path.dirname(os.path.abspath(__file__))
series = []
for name in ("baseline", "shellac", "varnish"):
    f = os.path.join(here, f"{name}.dat")
    if os.path.exists(f):
        rows = list(csv.reader(open(f), delimiter="\t"))[1:]
        ttime = sorted(int(r[4]) for r in rows)
        series.append((name, ttime))
if series:
    plt.figure(figsize=(8, 5))
    for name, t in series:
        plt.plot(range(len(t)), t, label=name)
    plt.xlabel("requests (sorted)")
    plt.ylabel("response time (ms)")
    plt.legend()
    plt.savefig(os.path.join(here, "requests.png"), dpi=120)
mem = os.path.join(here, "memory.csv")
if os.path.exists(mem):
    rows = list(csv.reader(open(mem)))
    plt.figure(figsize=(6, 4))
    plt.bar([r[0] for r in rows], [float(r[1]) for r in rows])
    plt.ylabel("peak memory (MB)")
    plt.savefig(os.path.join(here, "memory.png"), dpi=120)
print("graphs written to", here)
