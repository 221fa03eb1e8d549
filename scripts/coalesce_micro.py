#!/usr/bin/env python3
"""Micro-benchmark of the GET coalescing kernels on one GPU (HIP events, 20 reps).

Decomposes the coalescing lookup of a 1M-request batch over a populated 4M-object shard:
  coalesce   : k_coalesce<false> (LDS collapse + global claim table, no probe)
  lookup_co  : k_coalesce<true>  (the same + the index probe of every claimer) + k_offsets
  probe_all  : k_probe of every request + k_offsets (the uncoalesced lookup)
  probe_first: k_probe skipping duplicates (given `first`) + k_offsets
for Zipf(0.99) requests (~30 % distinct) and uniform requests (~all distinct).

usage: python scripts/coalesce_micro.py [--n 1048576] [--keys 4194304]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from shellac_amd.bench.workload import Workload  # noqa: E402
from shellac_amd.ops.cache import CacheShard, coalesce  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--keys", type=int, default=4 << 20)
    ap.add_argument("--dist", choices=["zipf", "uniform", "both"], default="both",
                    help="one distribution only (for rocprofv3 --stats per-kernel averages: "
                         "the event timings include host launch overhead)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    wl = Workload(a.keys, dev)
    nb = 1
    while nb < a.keys:
        nb *= 2
    shard = CacheShard(16 << 30, nb, 1 << 20, dev)
    for s in range(0, a.keys, 1 << 18):
        b = wl.set_batch(torch.arange(s, min(s + (1 << 18), a.keys), device=dev))
        shard.store(b.keys, b.values, b.val_off, b.vlen, b.flags, b.expire)
    torch.cuda.synchronize()
    out = {}
    for dist in (("zipf", "uniform") if a.dist == "both" else (a.dist,)):
        ids = wl.sample_ids(a.n, 1) if dist == "zipf" else wl.uniform_ids(a.n, 1)
        keys = wl.digests.index_select(0, ids).contiguous()
        first = coalesce(keys)
        nuniq = int((first.long() == torch.arange(a.n, device=dev)).sum())
        r = {"distinct_fraction": round(nuniq / a.n, 4)}
        r["coalesce_us"] = round(timed(lambda: coalesce(keys)), 1)
        r["lookup_co_us"] = round(timed(lambda: shard.lookup_coalesced(keys)), 1)
        r["probe_all_us"] = round(timed(lambda: shard.lookup(keys)), 1)
        r["probe_first_us"] = round(timed(lambda: shard.lookup(keys, first=first)), 1)
        out[dist] = r
        print(f"[micro] {dist}: {r}", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
