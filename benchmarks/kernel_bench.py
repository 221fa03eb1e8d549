#!/usr/bin/env python3
"""Per-kernel timing of the HBM cache pipeline against speed-of-light references.

For a realistic GET batch (Zipf keys over a populated shard, 64 B..4 KiB values):
  * lookup  (k_probe + hipcub scan) vs. a raw random 2x128 B read bound
  * gather  (k_segcopy<0>) vs. a D2D copy of the same byte count (HBM floor)
  * store   (dedupe + scan + k_segcopy<1> + k_set_index) for the SET batch
Times with HIP events, median of --iters. Prints JSON.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from shellac_amd.bench.workload import Workload  # noqa: E402
from shellac_amd.ops.cache import CacheShard  # noqa: E402


def timeit(fn, iters):
    ts = []
    for _ in range(iters):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=4 << 20)
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--sets", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    wl = Workload(a.keys, dev)
    nb = 1
    while nb * 2 < a.keys:
        nb *= 2
    shard = CacheShard(16 << 30, nb, 1 << 20, dev)
    for s in range(0, a.keys, 1 << 18):
        ids = torch.arange(s, min(s + (1 << 18), a.keys), device=dev)
        b = wl.set_batch(ids)
        shard.store(b.keys, b.values, b.val_off, b.vlen, b.flags, b.expire)
    keys = wl.digests.index_select(0, wl.sample_ids(a.batch, 7)).contiguous()
    sb = wl.set_batch(wl.uniform_ids(a.sets, 9))
    shard.reserve(1 << 18)
    lk = shard.lookup(keys)
    total = int(lk.off[-1])
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    res = {"batch": a.batch, "gather_bytes": total}
    res["lookup_us"] = timeit(lambda: shard.lookup(keys), a.iters)
    res["gather_us"] = timeit(lambda: shard.gather(lk, out), a.iters)
    src = torch.empty(total, dtype=torch.uint8, device=dev)
    res["d2d_copy_us"] = timeit(lambda: out.copy_(src), a.iters)
    res["gather_GBps"] = 2 * total / res["gather_us"] / 1e3
    res["d2d_GBps"] = 2 * total / res["d2d_copy_us"] / 1e3
    res["gather_vs_copy"] = res["d2d_copy_us"] / res["gather_us"]
    res["store_us"] = timeit(lambda: shard.store(sb.keys, sb.values, sb.val_off, sb.vlen, sb.flags,
                                                 sb.expire), a.iters)
    # random 2 x 128 B line reads (the probe's memory bound): index_select of 128-B rows
    idx_rows = torch.randint(0, nb, (2 * a.batch,), device=dev)
    table = torch.empty((nb, 32), dtype=torch.int32, device=dev)
    res["random_lines_us"] = timeit(lambda: table.index_select(0, idx_rows), a.iters)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
