#!/usr/bin/env python3
"""Is a step host-bound? From a rocprofv3 --hip-trace --kernel-trace --marker-trace run
(scripts/trace_bench.sh with HIP_TRACE=1): for every kernel of the last STEPS steps, when
the host called the launch and when the kernel started on the GPU (joined on the
correlation id). A kernel that starts within a few microseconds of its launch call waited
for the host; one that starts long after it waited for the GPU. Prints the per-step
timeline of the last two steps and, per kernel name, the median launch-to-start delay.

usage: launch_lag.py TRACE_DIR [STEPS] [STEP_MARKER] [PREFIX]"""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n)
    m = re.match(r"([\w:]+(<[^()]*?>)?)", n)
    b = m.group(1) if m else n
    return b.replace("shellac::", "")[:44]


def main():
    d = sys.argv[1]
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    marker = sys.argv[3] if len(sys.argv) > 3 else "hbm.lookup_coalesced"
    prefix = sys.argv[4] if len(sys.argv) > 4 else "bench"
    mk = list(csv.DictReader(open(f"{d}/{prefix}_marker_api_trace.csv")))
    api = list(csv.DictReader(open(f"{d}/{prefix}_hip_api_trace.csv")))
    kt = list(csv.DictReader(open(f"{d}/{prefix}_kernel_trace.csv")))
    launch = {}
    for r in api:
        if "Launch" in r["Function"]:
            launch[r["Correlation_Id"]] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    starts = sorted(int(r["Start_Timestamp"]) for r in mk if r["Function"] == marker)
    st = starts[-nsteps - 1:]
    t0, t1 = st[0], st[-1]
    rows = []
    for r in kt:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        lc = launch.get(r["Correlation_Id"])
        if lc and t0 <= lc[0] < t1 + 2_000_000:
            rows.append((lc[0], s, e, short(r["Kernel_Name"]), r.get("Queue_Id", "")))
    rows.sort(key=lambda x: x[1])
    lag = defaultdict(list)
    for lc, s, e, n, q in rows:
        if t0 <= s < t1:
            lag[n].append((s - lc) / 1e3)
    print(f"{len(st) - 1} steps; wall/step {(t1 - t0) / 1e3 / (len(st) - 1):.1f} us")
    print("median launch-call -> GPU start (us), per kernel:")
    for n, v in sorted(lag.items(), key=lambda x: sorted(x[1])[len(x[1]) // 2]):
        v = sorted(v)
        print(f"  {v[len(v) // 2]:9.1f}  (min {v[0]:8.1f})  {n}")
    a = st[-3] if len(st) >= 3 else st[0]
    print("--- last two steps: host launch call, GPU start, GPU end (us from the first marker)")
    for lc, s, e, n, q in rows:
        if a <= s < t1:
            print(f"  call {(lc - a) / 1e3:8.1f}  start {(s - a) / 1e3:8.1f}  end {(e - a) / 1e3:8.1f}"
                  f"  q{q:>3}  {n}")


if __name__ == "__main__":
    main()
