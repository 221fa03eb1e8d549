#!/usr/bin/env python3
"""Host-side timeline of the N=1 serve step (bench.py's default config): wraps the
shard calls ShardedCache.serve makes and reports, per step, how long the host spends
before the lookup launch, in each launch call, spinning on the lookup total, and from
the end of that spin to the next step's lookup launch (the part that can starve the GPU
when it exceeds the gather)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import shellac_amd.models.sharded_cache as scm  # noqa: E402
from shellac_amd.bench.workload import Workload  # noqa: E402
from shellac_amd.models.sharded_cache import ShardedCache  # noqa: E402
from shellac_amd.ops.cache import CacheShard, reserve_step_streams  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    reserve_step_streams(dev)
    keys = 4 << 20
    wl = Workload(keys, dev, min_val=64, max_val=4096)
    shard = CacheShard(16 << 30, keys, max_item=1 << 20, device=dev)
    sc = ShardedCache(shard)
    for s in range(0, keys, 1 << 18):
        sc.set(wl.set_batch(torch.arange(s, min(s + (1 << 18), keys), device=dev)))
    gets = [wl.digests.index_select(0, wl.sample_ids(1 << 20, 1000 + i)).contiguous() for i in range(16)]
    sets = [wl.set_batch(wl.uniform_ids(1 << 16, 5000 + i)) for i in range(16)]
    shard.reserve(1 << 18)
    torch.cuda.synchronize()
    marks = []

    def wrap(obj, name, tag):
        f = getattr(obj, name)

        def g(*a, **k):
            marks.append((tag + "<", time.perf_counter()))
            r = f(*a, **k)
            marks.append((tag + ">", time.perf_counter()))
            return r
        setattr(obj, name, g)

    for nm in ("lookup_coalesced", "store", "gather", "host_total"):
        wrap(shard, nm, nm)
    wrap(scm, "expand_out", "expand_out")
    ready = torch.cuda.Event()
    ready.record()
    for i in range(30):
        sc.serve(gets[i % 16], sets[i % 16], inputs_ready=ready)
    torch.cuda.synchronize()
    marks.clear()
    steps = 60
    t0 = time.perf_counter()
    for i in range(steps):
        marks.append(("serve<", time.perf_counter()))
        sc.serve(gets[i % 16], sets[i % 16], inputs_ready=ready)
        marks.append(("serve>", time.perf_counter()))
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    per = {}
    cur = {}
    last_spin_end = None
    spin_to_next = []
    for tag, t in marks:
        if tag == "serve<":
            cur = {"serve<": t}
        cur[tag] = t
        if tag == "lookup_coalesced>" and last_spin_end is not None:
            spin_to_next.append(t - last_spin_end)
        if tag == "host_total>":
            last_spin_end = t
        if tag == "serve>":
            for a, b in (("serve<", "lookup_coalesced<"), ("lookup_coalesced<", "lookup_coalesced>"),
                         ("store<", "store>"), ("expand_out<", "expand_out>"),
                         ("gather<", "gather>"), ("host_total<", "host_total>"),
                         ("host_total>", "serve>"), ("serve<", "serve>")):
                if a in cur and b in cur:
                    per.setdefault(f"{a[:-1]}..{b[:-1]}", []).append(cur[b] - cur[a])
    print(f"wall per step {wall * 1e3:.4f} ms")
    for k, v in per.items():
        print(f"  {k:40s} median {np.median(v) * 1e6:8.1f} us")
    print(f"  spin end -> next lookup launched      median {np.median(spin_to_next) * 1e6:8.1f} us")


if __name__ == "__main__":
    main()
