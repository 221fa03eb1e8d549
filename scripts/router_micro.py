#!/usr/bin/env python3
"""Host router throughput (csrc/host_router.cc) on this machine's cores: one global Zipf(0.99)
GET stream of N x 1M requests over N x 4M keys, ketama with 1024 points per GPU, with and
with hot sets of the given sizes (designated ranks; default "0,1024,65536"), 1 and T
threads, the 8-lane AVX-512 path and the scalar rule. CPU only; run from a source tree's
root (`python scripts/router_micro.py [N] [T] [HOT,HOT,...]`)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.getcwd())
from shellac_amd.bench.workload import Workload  # noqa: E402
from shellac_amd.parallel.hotspread import HotSpread  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
T = int(sys.argv[2]) if len(sys.argv) > 2 else 16
wl = Workload(W << 22, torch.device("cpu"))
sp = HotSpread(W, torch.device("cpu"), points_per_shard=1024)
kh = wl.digests.index_select(0, wl.sample_ids(W << 20, 1000)).contiguous()
buf = torch.empty(kh.shape[0], dtype=torch.int32)
for hot in [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "0,1024,65536").split(",")]:
    if hot:
        sp.plan(wl.digests.index_select(0, wl.sample_ids(1 << 22, 8800)), hot)
    else:
        sp.set_hot(None)
    for lanes in (False, True):
        sp.router.lanes = lanes
        for th in (1, T):
            best = 1e9
            for _ in range(3):
                t0 = time.perf_counter()
                sp.host_route_gets(kh, seq0=0, threads=th, out=buf)
                best = min(best, time.perf_counter() - t0)
            print(f"N={W} hot={hot} lanes={sp.router.lanes} threads={th}: "
                  f"{kh.shape[0] / best / 1e6:.0f} M req/s", flush=True)
