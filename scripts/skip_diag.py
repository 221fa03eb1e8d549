#!/usr/bin/env python3
"""Do SET skip rows (vlen = kSkipVlen, the HBM backend's size-class padding) ever land in
the index? SET 3000 keys in micro-batches padded to 64 rows with {0,0} skip rows, then
export the live digests and look for {0,0}."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from shellac_amd.ops.cache import CacheShard, digest_strings, pack_values, unpack_records  # noqa: E402

dev = torch.device("cuda", 0)
for bs, pad in ((300, 512), (1500, 2048), (3000, 4096), (3000, 3000)):
    sh = CacheShard(64 << 20, 256, 1 << 16, dev)
    keys = [b"/pf/%d" % i for i in range(3000)]
    for s in range(0, 3000, bs):
        kk = keys[s:s + bs]
        d = torch.zeros((pad, 2), dtype=torch.int64)
        d[: len(kk)] = digest_strings(kk)
        v, vo, vl = pack_values([b"v%d" % i for i in range(s, s + len(kk))] + [b""] * (pad - len(kk)))
        vl[len(kk):] = -1  # kSkipVlen
        vo[len(kk):] = 0
        sh.store(d.to(dev), v.to(dev), vo.to(dev), vl.to(dev))
    out = torch.empty((4096, 2), dtype=torch.int64, device=dev)
    nlive = sh._impl.export_keys(out.data_ptr(), 4096, sh.now(), torch.cuda.current_stream().cuda_stream)
    live = out[:nlive].cpu()
    zeros = int(((live[:, 0] == 0) & (live[:, 1] == 0)).sum())
    lk = sh.lookup(digest_strings(keys).to(dev))
    hits = int((lk.size[:3000] > 0).sum())
    data = sh.gather(lk)
    try:
        recs = unpack_records(data, lk.off[:3000], lk.size[:3000])
        right = sum(1 for i, r in enumerate(recs) if r is not None and r[0] == b"v%d" % i)
        err = ""
    except RuntimeError as e:
        right, err = -1, str(e)
    # the header's digest must be the key's
    hdr_ok = 0
    o = data.cpu().numpy()
    dk = digest_strings(keys).numpy()
    for i in range(3000):
        if int(lk.size[i]) > 0:
            b = int(lk.off[i])
            h = o[b:b + 32].view("<i8")
            hdr_ok += int(h[0] == dk[i][0] and h[1] == dk[i][1])
    print(f"[skip] batch {bs} pad {pad}: live {nlive} zero-digest entries {zeros} key hits {hits} "
          f"right values {right} header digest ok {hdr_ok} {err}", flush=True)
