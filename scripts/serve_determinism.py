#!/usr/bin/env python3
"""Diagnostic: run the same serve() sequence on fresh shards several times and report, per
run and step, how many requests differ from the workload's ground truth (wrong value) and
how many missed (the cache holds every key). A correct step is deterministic."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shellac_amd.bench.workload import Workload  # noqa: E402
from shellac_amd.models.sharded_cache import ShardedCache  # noqa: E402
from shellac_amd.ops.cache import CacheShard, unpack_records  # noqa: E402

dev = torch.device("cuda", 0)
wl = Workload(40000, dev)


def run():
    shard = CacheShard(256 << 20, 1 << 15, 1 << 16, dev)
    sc = ShardedCache(shard)
    for s0 in range(0, 40000, 10000):
        sc.set(wl.set_batch(torch.arange(s0, s0 + 10000, device=dev)))
    out = []
    for step in range(4):
        ids = wl.sample_ids(100000, 11 + step)
        keys = wl.digests.index_select(0, ids).contiguous()
        r = sc.serve(keys, wl.set_batch(wl.uniform_ids(4096, 21 + step)))
        torch.cuda.synchronize()
        recs = unpack_records(r.data, r.off, r.size)
        wrong = sum(1 for i, x in zip(ids.tolist(), recs) if x is not None and x[0] != wl.expected_value(i))
        miss = sum(1 for x in recs if x is None)
        out.append((wrong, miss))
    return out


for rep in range(8):
    print(f"rep {rep}: (wrong, misses) per step {run()}", flush=True)
