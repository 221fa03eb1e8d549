#!/usr/bin/env python3
"""A/B of the event fence that orders the N=1 step's main and side streams
(ShardedCache.event_fence: "device" = release to device, "none" = no system fence;
"nostart" = "device" without the side stream's per-step wait for the main stream, an
upper bound of what dropping that marker packet could save — results unchecked),
alternating rounds on one cache (bench.py's default workload on a 64 GiB log, which no round wraps; wall time per step)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from shellac_amd.bench.workload import Workload  # noqa: E402
from shellac_amd.models.sharded_cache import ShardedCache  # noqa: E402
from shellac_amd.ops.cache import CacheShard, reserve_step_streams  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    reserve_step_streams(dev)
    keys = 4 << 20
    wl = Workload(keys, dev)
    shard = CacheShard(64 << 30, keys, max_item=1 << 20, device=dev)
    sc = ShardedCache(shard)
    for s in range(0, keys, 1 << 18):
        sc.set(wl.set_batch(torch.arange(s, min(s + (1 << 18), keys), device=dev)))
    gets = [wl.digests.index_select(0, wl.sample_ids(1 << 20, 1000 + i)).contiguous() for i in range(16)]
    sets = [wl.set_batch(wl.uniform_ids(1 << 16, 5000 + i)) for i in range(16)]
    shard.reserve(1 << 18)
    torch.cuda.synchronize()
    k = 0
    for rnd in range(3):
        for fence in sys.argv[1:] or ("device", "none"):
            sc.event_fence = "device" if fence == "nostart" else fence
            sc._events = {}
            if fence == "nostart":
                orig = ShardedCache._xwait
                sc._xwait = (lambda w, s_, name, _o=orig, _sc=sc:
                             None if name == "start" else _o(_sc, w, s_, name))
            else:
                sc.__dict__.pop("_xwait", None)
            for _ in range(10):
                sc.serve(gets[k % 16], sets[k % 16])
                k += 1
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(100):
                sc.serve(gets[k % 16], sets[k % 16])
                k += 1
            torch.cuda.synchronize()
            print(f"round {rnd} fence={fence}: {(time.perf_counter() - t0) * 10:.4f} ms/step",
                  flush=True)


if __name__ == "__main__":
    main()
