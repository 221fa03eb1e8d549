#!/usr/bin/env python3
"""Diagnostics for the N=1 serve step's ground-truth test
(tests/test_hbm_gpu.py::test_serve_steps_return_ground_truth_records): repeat it with
fresh caches; per run report keys missing from the index after the fill, and for every
request a serve step missed whether a plain (uncoalesced) lookup finds the key right
after the step — an index loss or a lookup-side miss — plus the SET counters."""
import sys

import torch

sys.path.insert(0, ".")
from shellac_amd.bench.workload import Workload  # noqa: E402
from shellac_amd.models.sharded_cache import ShardedCache  # noqa: E402
from shellac_amd.ops.cache import CacheShard  # noqa: E402


def one(dev, overlap, coalesce):
    wl = Workload(40000, dev)
    shard = CacheShard(256 << 20, 1 << 15, 1 << 16, dev)
    sc = ShardedCache(shard)
    sc.overlap_store = overlap
    sc.coalesce = coalesce
    for s0 in range(0, 40000, 10000):
        sc.set(wl.set_batch(torch.arange(s0, s0 + 10000, device=dev)))
    torch.cuda.synchronize()
    lk = shard.lookup(wl.digests)
    torch.cuda.synchronize()
    fill_miss = int((lk.size[:40000] == 0).sum())
    notes = []
    for step in range(4):
        ids = wl.sample_ids(100000, 11 + step)
        keys = wl.digests.index_select(0, ids).contiguous()
        r = sc.serve(keys, wl.set_batch(wl.uniform_ids(4096, 21 + step)))
        torch.cuda.synchronize()
        miss = (r.size == 0).nonzero().flatten()
        if miss.numel():
            mk = keys.index_select(0, miss)
            lk2 = shard.lookup(mk)
            torch.cuda.synchronize()
            found = (lk2.size[: mk.shape[0]] > 0).tolist()
            mids = ids.index_select(0, miss).tolist()
            dup = [int((ids == i).sum()) for i in mids[:4]]
            notes.append((step, miss.numel(), list(zip(mids[:4], found[:4], dup))))
    c = shard.counters()
    return fill_miss, notes, {k: c[k] for k in ("set_evicted", "set_dropped")}


def main():
    dev = torch.device("cuda", 0)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    for overlap, coalesce in ((True, True), (False, True), (False, False)):
        bad = 0
        for r in range(reps):
            fill_miss, notes, c = one(dev, overlap, coalesce)
            if fill_miss or notes:
                bad += 1
                print(f"  run {r}: fill misses {fill_miss}, {c}, step misses "
                      f"(step, n, [(id, found after, requests)]): {notes}", flush=True)
        print(f"overlap={overlap} coalesce={coalesce}: {bad} of {reps} runs wrong", flush=True)


if __name__ == "__main__":
    main()
