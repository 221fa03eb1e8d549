#!/usr/bin/env python3
"""Join PMC byte counters with kernel durations: achieved HBM bandwidth per kernel.

usage: pmc_summary.py DIR  (fetch_/write_counter_collection.csv, time_kernel_trace.csv)"""
import csv
import os
import re
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n)
    return re.match(r"([\w:]+(<[^()]*?>)?)", n).group(1).replace("shellac::", "")


def main():
    d = sys.argv[1]
    cnt = defaultdict(lambda: defaultdict(list))
    for part in ("fetch", "write"):
        with open(os.path.join(d, f"{part}_counter_collection.csv")) as f:
            for r in csv.DictReader(f):
                cnt[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = defaultdict(list)
    with open(os.path.join(d, "time_kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    occ = defaultdict(lambda: defaultdict(list))
    p = os.path.join(d, "occ_counter_collection.csv")
    if os.path.exists(p):
        with open(p) as f:
            for r in csv.DictReader(f):
                occ[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("| kernel | calls | median us | HBM read MiB | HBM write MiB | achieved GB/s | waves |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for k in sorted(cnt):
        fs = sorted(cnt[k]["FETCH_SIZE"])
        ws = sorted(cnt[k]["WRITE_SIZE"])
        ds = sorted(dur.get(k, [0]))
        if not fs or not ds:
            continue
        rd, wr, us = fs[len(fs) // 2] / 1024, ws[len(ws) // 2] / 1024, ds[len(ds) // 2] / 1e3
        gbs = (rd + wr) * 1.048576 / us * 1e3 if us else 0  # MB/us -> GB/s
        wv = occ[k]["SQ_WAVES"]
        print(f"| `{k}` | {len(fs)} | {us:.1f} | {rd:.1f} | {wr:.1f} | {gbs:.0f} | "
              f"{int(sorted(wv)[len(wv)//2]) if wv else ''} |")


if __name__ == "__main__":
    main()
