#!/usr/bin/env python3
"""Per-kernel roofline table from scripts/pmc_roofline.sh output: median duration per
dispatch (kernel-trace pass), HBM bytes per dispatch (FETCH_SIZE / WRITE_SIZE passes,
KiB), achieved GB/s and the share of the measured 6.29 TB/s copy bandwidth
(MI355X_MICROARCH.md). Only dispatches of the timed steps' kernels matter; the medians
hide the warm-up and populate launches."""
import csv
import glob
import os
import re
import statistics
import sys

PEAK = 6290.0  # GB/s, measured float4 copy (8 TB/s spec)


def short(name: str) -> str:
    m = re.search(r"\b(k_\w+(?:<[^()]*?>)?)", name)
    return m.group(1) if m else name.replace("void ", "").split("(")[0][:48]


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main(d, last=6):
    """last: dispatches per kernel kept (the timed steps run last; earlier ones are the
    populate and warm-up launches)."""
    dur = {}
    for r in rows(os.path.join(d, "trace", "**", "*kernel_trace.csv")):
        k = short(r["Kernel_Name"])
        dur.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    ctr = {}
    for sub in ("fetch", "write", "sq"):
        for r in rows(os.path.join(d, sub, "**", "*counter_collection.csv")):
            k = short(r["Kernel_Name"])
            ctr.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    dur = {k: v[-last:] for k, v in dur.items()}
    ctr = {k: {c: vals[-last:] for c, vals in cs.items()} for k, cs in ctr.items()}
    print("| kernel | calls/step | median us | fetch MiB | write MiB | GB/s | % of 6.29 TB/s | VALU instr/wave | VMEM instr/wave | wait cycles/wave |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    items = sorted(dur.items(), key=lambda kv: -statistics.median(kv[1]) * len(kv[1]))
    for k, v in items:
        if not k.startswith("k_"):
            continue
        med = statistics.median(v)
        c = ctr.get(k, {})
        fe = statistics.median(c["FETCH_SIZE"]) if "FETCH_SIZE" in c else float("nan")  # KiB
        wr = statistics.median(c["WRITE_SIZE"]) if "WRITE_SIZE" in c else float("nan")
        gbps = (fe + wr) * 1024 / (med * 1e3) if med else 0.0
        waves = statistics.median(c["SQ_WAVES"]) if "SQ_WAVES" in c else 0
        valu = statistics.median(c["SQ_INSTS_VALU"]) / waves if waves else float("nan")
        vmem = ((statistics.median(c.get("SQ_INSTS_VMEM_RD", [0])) +
                 statistics.median(c.get("SQ_INSTS_VMEM_WR", [0]))) / waves) if waves else float("nan")
        wait = statistics.median(c.get("SQ_WAIT_INST_ANY", [0])) / waves if waves else float("nan")
        print(f"| `{k}` | {len(v) / last:.0f} | {med:.1f} | {fe / 1024:.1f} | {wr / 1024:.1f} | {gbps:.0f} | "
              f"{100 * gbps / PEAK:.0f}% | {valu:.0f} | {vmem:.0f} | {wait:.0f} |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 6)
