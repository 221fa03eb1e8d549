#!/usr/bin/env python3
"""Host-wait audit of the bench step from a rocprofv3 --hip-trace --marker-trace
--kernel-trace run (scripts/trace_bench.sh with --hip-trace): for each of the last STEPS
steps (between consecutive STEP_MARKER ranges), every HIP runtime call that can make the
host wait for the GPU — stream / event / device synchronisation, synchronous copies and
memsets, frees — with its count and the time the host spent inside it, plus the GPU's
busy time against the wall time.

A host-sync-free step shows no such call, or only event synchronisations on events that
had already completed (microseconds: the routed step's pinned-ring harvest of the matrix
published two steps earlier).

usage: host_wait_audit.py TRACE_DIR [STEPS] [STEP_MARKER] [PREFIX]"""
import csv
import re
import sys
from collections import defaultdict

BLOCKING = re.compile(r"^hip(StreamSynchronize|EventSynchronize|DeviceSynchronize|Memcpy|"
                      r"MemcpyDtoH|MemcpyHtoD|MemcpyDtoD|Memset|MemcpyWithStream|Free|"
                      r"FreeHost|HostFree|StreamWaitValue)")
ASYNC = re.compile(r"Async$")


def main():
    d = sys.argv[1]
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    marker = sys.argv[3] if len(sys.argv) > 3 else "serve.plan"
    prefix = sys.argv[4] if len(sys.argv) > 4 else "bench"
    mk = list(csv.DictReader(open(f"{d}/{prefix}_marker_api_trace.csv")))
    api = list(csv.DictReader(open(f"{d}/{prefix}_hip_api_trace.csv")))
    kt = list(csv.DictReader(open(f"{d}/{prefix}_kernel_trace.csv")))
    starts = sorted(int(r["Start_Timestamp"]) for r in mk if r["Function"] == marker)
    st = starts[-nsteps - 1:]
    print(f"{len(starts)} '{marker}' markers; auditing the last {len(st) - 1} steps")
    t0, t1 = st[0], st[-1]
    per_call = defaultdict(lambda: [0, 0, 0])  # count, total ns, max ns
    per_step = [0] * (len(st) - 1)
    api_ns = 0
    for r in api:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if not (t0 <= s < t1):
            continue
        api_ns += e - s
        f = r["Function"]
        if BLOCKING.match(f) and not ASYNC.search(f):
            c = per_call[f]
            c[0] += 1
            c[1] += e - s
            c[2] = max(c[2], e - s)
            for i in range(len(st) - 1):
                if st[i] <= s < st[i + 1]:
                    per_step[i] += e - s
    busy = 0
    for r in kt:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= s < t1:
            busy += e - s
    n = len(st) - 1
    print(f"wall/step {(t1 - t0) / 1e3 / n:.1f} us; kernel busy/step {busy / 1e3 / n:.1f} us "
          f"(summed over streams); HIP API time/step {api_ns / 1e3 / n:.1f} us")
    if not per_call:
        print("calls that can wait for the GPU: none")
    else:
        print("calls that can wait for the GPU (count/step, us/step, max us):")
        for f, (c, tot, mx) in sorted(per_call.items(), key=lambda x: -x[1][1]):
            print(f"  {f:28s} {c / n:6.2f}  {tot / 1e3 / n:8.2f}  {mx / 1e3:8.2f}")
    print("host time inside them, per step (us):",
          " ".join(f"{v / 1e3:.1f}" for v in per_step))


if __name__ == "__main__":
    main()
