#!/usr/bin/env python3
"""Is the N=1 serving step host-bound? Runs the bench step (1M Zipf GETs + 64K SETs,
same shard and workload as bench.py) and splits each step's host time into the spin on
the lookup total (waiting for the GPU) and everything else (Python, bindings, launches).
If the non-spin host time after the spin exceeds the gather it overlaps, the GPU idles
between steps.

usage: python scripts/host_time_n1.py [--steps 200]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shellac_amd.bench.workload import Workload  # noqa: E402
from shellac_amd.models.sharded_cache import ShardedCache  # noqa: E402
from shellac_amd.ops.cache import CacheShard  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--batch", type=int, default=1 << 20)
ap.add_argument("--sets", type=int, default=1 << 16)
a = ap.parse_args()
dev = torch.device("cuda", 0)
keys = 4 << 20
wl = Workload(keys, dev)
shard = CacheShard(16 << 30, keys, max_item=1 << 20, device=dev)
sc = ShardedCache(shard)
for s in range(0, keys, 1 << 18):
    sc.set(wl.set_batch(torch.arange(s, min(s + (1 << 18), keys), device=dev)))
P = 16
gets = [wl.digests.index_select(0, wl.sample_ids(a.batch, 1000 + i)).contiguous() for i in range(P)]
sets = [wl.set_batch(wl.uniform_ids(a.sets, 5000 + i)) for i in range(P)]
shard.reserve(max(a.sets * 2, 1 << 18))

spin = [0.0]
orig = shard.host_total


def timed_total(slot, timeout_ms=10000):
    t = time.perf_counter()
    r = orig(slot, timeout_ms)
    spin[0] += time.perf_counter() - t
    spin_end.append(time.perf_counter())
    return r


spin_end = []
shard.host_total = timed_total
for i in range(10):
    sc.serve(gets[i % P], sets[i % P])
torch.cuda.synchronize()
spin[0] = 0.0
spin_end.clear()
starts = []
t0 = time.perf_counter()
for i in range(a.steps):
    starts.append(time.perf_counter())
    sc.serve(gets[i % P], sets[i % P])
torch.cuda.synchronize()
el = time.perf_counter() - t0
# host time from the end of step i's spin to the end of step i+1's launches up to its
# spin start is what must hide under step i's gather
after = [starts[i + 1] - spin_end[i] for i in range(a.steps - 1)]
after.sort()
print(f"wall {el / a.steps * 1e6:.1f} us/step; spin {spin[0] / a.steps * 1e6:.1f} us/step; "
      f"non-spin host {(el - spin[0]) / a.steps * 1e6:.1f} us/step")
print(f"host from spin end to next step start: median {after[len(after) // 2] * 1e6:.1f} us, "
      f"p90 {after[int(len(after) * 0.9)] * 1e6:.1f} us")
pre = [spin_end[i] - starts[i] for i in range(a.steps)]
pre.sort()
print(f"step start to spin end (launch + spin): median {pre[len(pre) // 2] * 1e6:.1f} us")
