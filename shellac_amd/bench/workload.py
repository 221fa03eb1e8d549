"""Synthetic web-cache workload generated on the device.

Key i is the URL ``/static/obj/<i:010d>.html`` (26 bytes); its digest is
computed by the HIP ``k_digest`` kernel from key bytes built on the GPU. Object
sizes are log-uniform in [min_val, max_val] per key (web objects: fragments,
JSON, small assets). Requests follow a Zipf(s) popularity law over the whole
key space, with popularity ranks scattered over key ids by a fixed random
permutation so hot keys land on every shard. Every rank derives the same key
space (fixed seeds) and its own request stream (rank-dependent seeds).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from ..ops.cache import digest_packed

KEY_PREFIX = b"/static/obj/"
KEY_SUFFIX = b".html"
KEY_DIGITS = 10
KEY_LEN = len(KEY_PREFIX) + KEY_DIGITS + len(KEY_SUFFIX)


def key_bytes(ids: torch.Tensor) -> torch.Tensor:
    """[n] int64 ids -> [n, KEY_LEN] uint8 URL bytes (on ids.device)."""
    n = ids.numel()
    out = torch.empty((n, KEY_LEN), dtype=torch.uint8, device=ids.device)
    out[:, : len(KEY_PREFIX)] = torch.tensor(list(KEY_PREFIX), dtype=torch.uint8, device=ids.device)
    p = len(KEY_PREFIX)
    v = ids.clone()
    for d in range(KEY_DIGITS - 1, -1, -1):
        out[:, p + d] = (v % 10 + 48).to(torch.uint8)
        v = torch.div(v, 10, rounding_mode="floor")
    out[:, p + KEY_DIGITS :] = torch.tensor(list(KEY_SUFFIX), dtype=torch.uint8, device=ids.device)
    return out


def key_string(i: int) -> bytes:
    return KEY_PREFIX + str(i).zfill(KEY_DIGITS).encode() + KEY_SUFFIX


def digests_for_ids(ids: torch.Tensor, chunk: int = 1 << 22) -> torch.Tensor:
    outs = []
    for s in range(0, ids.numel(), chunk):
        part = ids[s : s + chunk]
        kb = key_bytes(part).reshape(-1).contiguous()
        offs = torch.arange(0, part.numel() + 1, dtype=torch.int64, device=ids.device) * KEY_LEN
        outs.append(digest_packed(kb, offs))
    return torch.cat(outs) if outs else torch.empty((0, 2), dtype=torch.int64, device=ids.device)


@dataclass
class Workload:
    total_keys: int
    device: torch.device
    zipf_s: float = 0.99
    min_val: int = 64
    max_val: int = 4096
    pool_bytes: int = 64 << 20
    seed: int = 1234

    def __post_init__(self):
        dev = self.device
        g = torch.Generator(device="cpu").manual_seed(self.seed)
        u = torch.rand(self.total_keys, generator=g, dtype=torch.float64)
        lo, hi = float(self.min_val), float(self.max_val)
        self.vlen = (lo * (hi / lo) ** u).floor().to(torch.int32).to(dev)
        self.rank_to_id = torch.randperm(self.total_keys, generator=g).to(dev)
        ranks = torch.arange(1, self.total_keys + 1, dtype=torch.float64)
        w = ranks.pow(-self.zipf_s)
        self.cdf = (torch.cumsum(w, 0) / w.sum()).to(dev)
        self.digests = digests_for_ids(torch.arange(self.total_keys, device=dev))
        pool = torch.randint(0, 256, (self.pool_bytes + 16,), generator=g, dtype=torch.uint8)
        self.pool = pool.to(dev)
        # payload of key i = pool[val_off[i] : + vlen[i]] (16-B aligned)
        span = self.pool_bytes - self.max_val - 16
        self.val_off = ((torch.arange(self.total_keys, dtype=torch.int64) * 2654435761) % span
                        & ~15).to(dev)

    def sample_ids(self, n: int, seed: int, rank_to_id: torch.Tensor = None) -> torch.Tensor:
        """Zipf(s)-popular object ids (GET traffic); ``rank_to_id``: another popularity
        order (a drifted hot set, see ``drifted``)."""
        g = torch.Generator(device=self.device).manual_seed(seed)
        r = torch.rand(n, generator=g, dtype=torch.float64, device=self.device)
        idx = torch.searchsorted(self.cdf, r).clamp_(max=self.total_keys - 1)
        return (self.rank_to_id if rank_to_id is None else rank_to_id).index_select(0, idx)

    def drifted(self, rank_to_id: torch.Tensor, top: int, m: int, seed: int) -> torch.Tensor:
        """A drifted popularity order: `m` objects of the top `top` ranks (at random ranks)
        trade places with `m` objects of the tail — content going cold while new content
        becomes popular, the rest of the order unchanged."""
        g = torch.Generator(device="cpu").manual_seed(seed)
        top = min(top, self.total_keys // 2)
        a = torch.randperm(top, generator=g)[:m].to(self.device)
        b = (top + torch.randperm(self.total_keys - top, generator=g)[:m]).to(self.device)
        out = rank_to_id.clone()
        out[a], out[b] = rank_to_id[b], rank_to_id[a]
        return out

    def uniform_ids(self, n: int, seed: int) -> torch.Tensor:
        """Uniform object ids (cache-fill / refresh SET traffic: in a TTL cache every
        requested object is refetched about once per TTL, independent of popularity)."""
        g = torch.Generator(device=self.device).manual_seed(seed)
        return torch.randint(0, self.total_keys, (n,), generator=g, device=self.device)

    def _offsets(self, ids: torch.Tensor, version: int) -> torch.Tensor:
        off = self.val_off.index_select(0, ids)
        if version:
            # another payload of the same size (an updated object): shifted in the pool
            span = self.pool_bytes - self.max_val - 16
            off = torch.remainder(off + version * 1048573 * 16, span) & ~15
        return off

    def set_batch(self, ids: torch.Tensor, ttl_expire: int = 0, version: int = 0):
        """SETs of objects `ids`; `version` > 0 gives them other payload bytes (updates)."""
        from ..models.sharded_cache import SetBatch

        n = ids.numel()
        return SetBatch(
            keys=self.digests.index_select(0, ids).contiguous(),
            values=self.pool,
            val_off=self._offsets(ids, version).contiguous(),
            vlen=self.vlen.index_select(0, ids).contiguous(),
            flags=(ids % 65536).to(torch.int32).contiguous(),
            expire=torch.full((n,), ttl_expire, dtype=torch.int32, device=self.device),
        )

    def expected_value(self, i: int, version: int = 0) -> bytes:
        o = int(self._offsets(torch.tensor([i], device=self.device), version)[0])
        return self.pool[o : o + int(self.vlen[i])].cpu().numpy().tobytes()
