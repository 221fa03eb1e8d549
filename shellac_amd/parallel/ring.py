"""Consistent-hash rings that map object digests to cache shards.

The reference spreads keys over memcached nodes with libmemcached's ketama
(src/python/shellac/server/Server.py:81-83, behaviors={'ketama': True}): losing
a node remaps only that node's keys. ``ShardRing`` is the same idea for GPU
shards: every shard owns ``points_per_shard`` pseudo-random points on a 32-bit
ring (weights scale the count), and a digest belongs to the first point at or
after ``ring_position(digest)`` (the top 32 bits of digest.hi). The sorted point
array + owner array is what the HIP ``k_route`` kernel binary-searches.

The libmemcached-compatible (MD5) ketama ring for talking to real memcached
nodes lives in the native core (``csrc/ketama.cc``, ``KetamaRing``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np
import torch

from .._native import core


@dataclass
class ShardRing:
    shards: list  # shard ids (e.g. global ranks, or "host:gpu" strings)
    points_per_shard: int = 160
    weights: Optional[Sequence[float]] = None
    pts: np.ndarray = field(init=False)
    owner: np.ndarray = field(init=False)

    def __post_init__(self):
        c = core()
        pts, own = [], []
        w = list(self.weights) if self.weights is not None else [1.0] * len(self.shards)
        for idx, (sid, wi) in enumerate(zip(self.shards, w)):
            npts = max(1, int(round(self.points_per_shard * wi)))
            for j in range(npts):
                _, hi = c.digest(f"shellac-shard-{sid}-{j}".encode())
                pts.append((hi >> 32) & 0xFFFFFFFF)
                own.append(idx)
        order = np.argsort(np.array(pts, dtype=np.uint64), kind="stable")
        self.pts = np.array(pts, dtype=np.uint64)[order].astype(np.uint32)
        self.owner = np.array(own, dtype=np.int32)[order]

    @property
    def nshards(self) -> int:
        return len(self.shards)

    def owner_of_position(self, pos: int) -> int:
        i = int(np.searchsorted(self.pts, np.uint32(pos), side="left"))
        return int(self.owner[0 if i == len(self.pts) else i])

    def owner_of_digest(self, lo: int, hi: int) -> int:
        return self.owner_of_position((hi >> 32) & 0xFFFFFFFF)

    def owner_of_key(self, key: bytes) -> int:
        lo, hi = core().digest(key)
        return self.owner_of_digest(lo, hi)

    def tensors(self, device) -> tuple[torch.Tensor, torch.Tensor]:
        """(points as an int32 bit pattern, owner ids int32) for ``ops.routing.route``.
        Owner ids are the shard ids when shards are ints (ranks), else ring indices."""
        pts = torch.from_numpy(self.pts.view(np.int32).copy()).to(device)
        if all(isinstance(x, (int, np.integer)) for x in self.shards):
            ids = np.asarray(self.shards, dtype=np.int32)[self.owner]
        else:
            ids = self.owner
        own = torch.from_numpy(np.ascontiguousarray(ids, dtype=np.int32)).to(device)
        return pts, own

    def without(self, shard) -> "ShardRing":
        """Ring after removing a failed shard (only its keys move)."""
        keep = [s for s in self.shards if s != shard]
        w = None
        if self.weights is not None:
            w = [wi for s, wi in zip(self.shards, self.weights) if s != shard]
        return ShardRing(keep, self.points_per_shard, w)

    def moved_fraction(self, other: "ShardRing", samples: int = 20000, seed: int = 0) -> float:
        """Fraction of random positions whose owner id differs between two rings."""
        rng = np.random.default_rng(seed)
        pos = rng.integers(0, 2**32, size=samples, dtype=np.uint64)
        a = [self.shards[self.owner_of_position(int(p))] for p in pos]
        b = [other.shards[other.owner_of_position(int(p))] for p in pos]
        return float(np.mean([x != y for x, y in zip(a, b)]))
