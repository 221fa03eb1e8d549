"""Hit ratio under capacity pressure: the cache's eviction policy against an exact-LRU
oracle on a Zipf request trace (cache-aside, as the proxy fills it).

The reference stores its objects in memcached (src/python/shellac/server/Server.py:81-83,
get :335, set on miss :432), whose segmented LRU keeps recently read objects. The HBM
log here is a circular FIFO; with ``evict="clock"`` the eviction hand re-appends objects
read since it last passed (hbm_cache.h, HostCache::reclaim_locked). This script drives
one shard — DRAM (``--device cpu``) or HBM (``cuda``) — with the same trace and reports
its hit ratio next to a byte-capacity LRU of the same size and the FIFO log.

Trace: ``--requests`` GETs, Zipf(``--zipf``) over ``--objects`` keys whose sizes are
log-uniform in [min_val, max_val]; every batch of ``--batch`` GETs is looked up, then
its distinct misses are SET (one batch), like the proxy's micro-batches.

Usage: python -m shellac_amd.bench.evict_sim --device cpu --ratio 3
"""
from __future__ import annotations

import argparse
import json
from collections import OrderedDict

import numpy as np
import torch


def item_bytes(v: int) -> int:
    return 32 + ((v + 15) & ~15)


def make_trace(objects: int, requests: int, zipf: float, min_val: int, max_val: int,
               seed: int = 7):
    rng = np.random.default_rng(seed)
    u = rng.random(objects)
    sizes = np.floor(min_val * (max_val / min_val) ** u).astype(np.int64)
    ranks = np.arange(1, objects + 1, dtype=np.float64)
    w = ranks ** (-zipf)
    cdf = np.cumsum(w) / w.sum()
    perm = rng.permutation(objects)
    reqs = perm[np.minimum(np.searchsorted(cdf, rng.random(requests)), objects - 1)]
    return sizes, reqs


def lru_hit_ratio(sizes, reqs, capacity: int, batch: int, warm: int) -> float:
    """Exact byte-capacity LRU with the cache's batch semantics (lookups of a batch see
    the state before the batch's fills; a hit refreshes recency)."""
    lru: OrderedDict = OrderedDict()
    used = 0
    hits = total = 0
    for s in range(0, len(reqs), batch):
        b = reqs[s:s + batch]
        miss = []
        for k in b:
            k = int(k)
            if k in lru:
                lru.move_to_end(k)
                if s >= warm:
                    hits += 1
            else:
                miss.append(k)
            if s >= warm:
                total += 1
        for k in dict.fromkeys(miss):
            if k in lru:
                continue
            sz = item_bytes(int(sizes[k]))
            lru[k] = sz
            used += sz
            while used > capacity:
                _, v = lru.popitem(last=False)
                used -= v
    return hits / max(total, 1)


def cache_hit_ratio(sizes, reqs, log_bytes: int, batch: int, warm: int, device: str,
                    evict: str, nbuckets: int | None = None) -> dict:
    from ..ops.cache import CacheShard

    n_obj = len(sizes)
    if nbuckets is None:  # index large enough that the log, not the index, bounds capacity
        nbuckets = 1024
        while nbuckets * 4 < 4 * n_obj:
            nbuckets *= 2
    dev = torch.device(device)
    sh = CacheShard(log_bytes, nbuckets, max_item=1 << 16, device=dev, evict=evict)
    # digests: two random 64-bit words per object id (fixed)
    g = np.random.default_rng(99)
    dig = torch.from_numpy(g.integers(-(1 << 62), 1 << 62, size=(n_obj, 2), dtype=np.int64))
    dig_d = dig.to(dev)
    maxv = int(sizes.max())
    pool = torch.randint(0, 256, (maxv + 32,), dtype=torch.uint8).to(dev)
    sizes_t = torch.from_numpy(sizes.astype(np.int32))
    hits = total = 0
    for s in range(0, len(reqs), batch):
        ids = torch.from_numpy(reqs[s:s + batch].astype(np.int64))
        lk = sh.lookup(dig_d.index_select(0, ids.to(dev)).contiguous(), now=1)
        hit = (lk.size[: ids.numel()] > 0).cpu()
        if s >= warm:
            hits += int(hit.sum())
            total += ids.numel()
        miss = torch.unique(ids[~hit])
        if miss.numel():
            k = dig_d.index_select(0, miss.to(dev)).contiguous()
            vl = sizes_t.index_select(0, miss).to(dev).contiguous()
            vo = torch.zeros(miss.numel(), dtype=torch.int64, device=dev)
            sh.store(k, pool, vo, vl, now=1,
                     bytes_bound=int(sum(item_bytes(int(x)) for x in sizes[miss.numpy()])))
    c = sh.counters()
    return {"hit_ratio": hits / max(total, 1), "reinserted": int(c["reinserted"]),
            "evicted_index": int(c["set_evicted"])}


def run(objects=20000, requests=400000, zipf=0.99, min_val=64, max_val=4096, ratio=3.0,
        batch=256, device="cpu", warm_frac=0.25) -> dict:
    sizes, reqs = make_trace(objects, requests, zipf, min_val, max_val)
    ws = int(sum(item_bytes(int(v)) for v in sizes))
    log_bytes = max(1 << 20, int(ws / ratio)) // 16 * 16
    warm = int(requests * warm_frac) // batch * batch
    out = {"objects": objects, "requests": requests, "zipf": zipf, "working_set_bytes": ws,
           "capacity_bytes": log_bytes, "ratio": ratio, "batch": batch, "device": device}
    out["lru"] = lru_hit_ratio(sizes, reqs, log_bytes, batch, warm)
    for ev in ("fifo", "clock"):
        r = cache_hit_ratio(sizes, reqs, log_bytes, batch, warm, device, ev)
        out[ev] = r["hit_ratio"]
        out[ev + "_reinserted"] = r["reinserted"]
        out[ev + "_index_evictions"] = r["evicted_index"]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--objects", type=int, default=20000)
    ap.add_argument("--requests", type=int, default=400000)
    ap.add_argument("--zipf", type=float, default=0.99)
    ap.add_argument("--ratio", type=float, nargs="+", default=[2.0, 3.0, 4.0])
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    for r in a.ratio:
        print(json.dumps(run(a.objects, a.requests, a.zipf, ratio=r, batch=a.batch,
                             device=a.device)), flush=True)


if __name__ == "__main__":
    main()
