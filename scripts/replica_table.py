#!/usr/bin/env python3
"""Per-N hot-replica table from a scripts/replica_sweep.sh run: for each simulated world
size N and replica size R, the simulated owner's measured step (compute: every kernel of
rank 0's step, the collectives mirrored on-device), the bytes each xGMI link carries per
step (fixed slot capacities, each direction: request slot, reply slot, SET slot; from
the bench JSON's routed_diag), that traffic's time at a per-link rate, and two step
models: overlapped (max of compute and link) and serial (their sum). Prints markdown.

usage: replica_table.py SWEEP_DIR [LINK_GBPS]"""
import glob
import json
import os
import re
import sys


def main():
    d = sys.argv[1]
    gbps = float(sys.argv[2]) if len(sys.argv) > 2 else 55.0
    rows = []
    for f in glob.glob(os.path.join(d, "sim*_rep*.json")):
        m = re.search(r"sim(\d+)_rep(\d+)\.json$", f)
        if not m:
            continue
        j = json.load(open(f))
        rd = j.get("routed_diag") or {}
        per_peer = rd.get("link_bytes_per_peer_per_step")
        if per_peer is None:
            continue
        rows.append((int(m.group(1)), int(m.group(2)), j["ms_per_step"],
                     j.get("replica_hit_fraction", 0.0), per_peer))
    rows.sort()
    print(f"| N | replicated objects | sim compute ms/step | replica hit fraction | "
          f"MB per link per step | link ms at {gbps:.0f} GB/s | model max(compute, link) | "
          f"model compute + link |")
    print("|---:|---:|---:|---:|---:|---:|---:|---:|")
    best = {}
    for n, r, ms, hit, b in rows:
        link = b / (gbps * 1e9) * 1e3
        mx, sm = max(ms, link), ms + link
        best.setdefault(n, (mx, r))
        if mx < best[n][0]:
            best[n] = (mx, r)
        print(f"| {n} | {r:,} | {ms:.3f} | {hit:.3f} | {b / 1e6:.1f} | {link:.3f} | "
              f"{mx:.3f} | {sm:.3f} |")
    for n, (mx, r) in sorted(best.items()):
        print(f"\nN={n}: lowest overlapped model {mx:.3f} ms/step at {r:,} replicated objects")


if __name__ == "__main__":
    main()
