#!/usr/bin/env python3
"""Index consistency under heavy eviction: 3000 keys SET in micro-batches into a 1024-slot
shard; every digest that export_keys reports live must hit in lookup, and vice versa."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from shellac_amd.ops.cache import CacheShard, digest_strings, pack_values  # noqa: E402


def run(dev, bs):
    sh = CacheShard(64 << 20, 256, 1 << 16, dev)
    keys = [b"/pf/%d" % i for i in range(3000)]
    for s in range(0, 3000, bs):
        d = digest_strings(keys[s:s + bs]).to(dev)
        v, vo, vl = pack_values([b"v%d" % i for i in range(s, min(s + bs, 3000))], dev)
        sh.store(d, v, vo, vl)
    dall = digest_strings(keys).to(dev)
    lk = sh.lookup(dall)
    hit = (lk.size[:3000] > 0).cpu()
    if dev.type == "cuda":
        out = torch.empty((4096, 2), dtype=torch.int64, device=dev)
        nlive = sh._impl.export_keys(out.data_ptr(), 4096, sh.now(), torch.cuda.current_stream().cuda_stream)
        live = {tuple(r) for r in out[:nlive].cpu().tolist()}
    else:
        live = None
    hitset = {tuple(r) for r, h in zip(dall.cpu().tolist(), hit.tolist()) if h}
    return int(hit.sum()), live, hitset


for bs in (1, 7, 64, 500):
    h, live, hs = run(torch.device("cuda", 0), bs)
    hc, _, hsc = run(torch.device("cpu"), bs)
    extra = len(live - hs) if live is not None else -1
    print(f"[idx] batch {bs}: gpu hits {h} live {len(live)} live-not-hit {extra} "
          f"hit-not-live {len(hs - live)} | host hits {hc} same-set {hs == hsc}", flush=True)
