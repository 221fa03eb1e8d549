"""Hot-object spreading for the host-routed multi-GPU topology.

Reference: the cache client sends every request to the memcached node that owns its key
by ketama (src/python/shellac/server/Server.py:81-83), so a node takes its keys' true
share of the traffic — a Zipf hot key loads one node (README.md:30 sells ketama for node
loss, not for load). SURVEY.md §5.8 asks for hot-object replication over xGMI: here the
hottest objects live on every GPU, a GET of one goes to a GPU chosen to even out the load
and a SET of one is written through to every GPU.

Routing decisions are a pure function of (digest, stream position), implemented twice
with identical results (tests check it): ``route_gets`` / ``route_sets`` below in tensor
ops (the bench prepares its request batches with them on the GPU) and the native
``HostRouter`` (csrc/host_router.cc, the host proxy's router, whose throughput the bench
measures):

* ``owner(d)``: the first ``ShardRing`` point at or after ``ring_position(d)``.
* a GET of a hot object goes to its *designated* rank (every rank holds a replica; the
  designation is made when the hot set is picked, to even out the load), or — for the
  few objects too hot for one rank — to the rank a Weyl sequence picks at its stream
  position j with the spray weights: u = top 53 bits of (j * 0x9E3779B97F4A7C15 mod
  2^64) / 2^53, rank = #{cumulative weight <= u}; every other GET to its owner.
* a SET of a hot object goes to every rank (dest -1), every other SET to its owner.

Why designate instead of spraying every hot object: the serving step collapses duplicate
requests (GET coalescing), so a rank's work is mostly per *distinct* key (probe, record
copy) and little per request. Spraying 64K hot objects over 8 GPUs made every GPU probe
and copy each of them every step — the most loaded simulated rank got slower (0.363 vs
0.341 ms) although its requests fell from 1.43x to 1.01x the mean (profiles/r5c_hostsim).
Designation (greedy: hottest first, each to the least loaded rank, starting from the
ranks' non-hot owner loads) evens out requests without copying any key's work; objects
above 1/(4N) of the traffic are sprayed, their duplicated work is a handful of keys. The
per-rank *distinct-key* balance is the ring's key-space balance: more ring points per
shard (the bench uses 1024: 1.045x, against 1.118x at 160, for 8 shards) even it out.

``water_fill`` (the spray weights' level) is kept for ``policy="spray"``, which sprays
every hot object.

Replicas are ordinary objects of each rank's shard (one lookup, one gather per step; the
CLOCK hand keeps them, they are the most read objects). ``replicate_hot`` fills them from
their owners with one all-gather of records (RCCL over xGMI on GPUs, gloo on the CPU).
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch
import torch.distributed as dist

from .._native import core
from ..ops import routing as R
from .ring import ShardRing

PHI = 0x9E3779B97F4A7C15 - (1 << 64)   # the Weyl constant as an int64 bit pattern
_M53 = (1 << 53) - 1


def cumulative(weights: Sequence[float]) -> list:
    """Normalised cumulative weights, computed exactly as HostRouter::set_hot does."""
    tot = 0.0
    for w in weights:
        if w < 0:
            raise ValueError("spray weights must be non-negative")
        tot += float(w)
    if tot <= 0:
        raise ValueError("spray weights sum to zero")
    out, acc = [], 0.0
    for w in weights:
        acc += float(w)
        out.append(acc / tot)
    out[-1] = 1.0
    return out


def spray_ranks(pos: torch.Tensor, cw: torch.Tensor) -> torch.Tensor:
    """Rank of each stream position (int64) under cumulative weights ``cw`` (float64)."""
    h = pos * PHI                                   # wraps mod 2^64 (two's complement)
    u = ((h >> 11) & _M53).to(torch.float64) * (1.0 / (1 << 53))
    r = torch.searchsorted(cw, u, right=True)
    return r.clamp_(max=cw.numel() - 1).to(torch.int32)


def water_fill(owner_share: Sequence[float], hot_share: float) -> list:
    """Spray weights that bring every rank's share as close to 1/N as ``hot_share`` allows:
    w_r proportional to max(0, T - L_r), sum = hot_share."""
    n = len(owner_share)
    if hot_share <= 0:
        return [1.0] * n
    order = sorted(range(n), key=lambda r: owner_share[r])
    level = 0.0
    for k in range(1, n + 1):
        # raise the k lowest ranks to the (k+1)-th lowest share or until H is spent
        lo = [owner_share[order[i]] for i in range(k)]
        nxt = owner_share[order[k]] if k < n else float("inf")
        need = sum(nxt - x for x in lo)
        if need >= hot_share or k == n:
            level = (hot_share + sum(lo)) / k
            break
    w = [max(0.0, level - owner_share[r]) for r in range(n)]
    return w if sum(w) > 0 else [1.0] * n


def member(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Rows of ``a`` that are rows of ``b`` (digests [n, 2]; ``b`` sorted by lo)."""
    if a.shape[0] == 0 or b is None or b.shape[0] == 0:
        return torch.zeros(a.shape[0], dtype=torch.bool, device=a.device)
    at = torch.searchsorted(b[:, 0].contiguous(), a[:, 0].contiguous())
    at = torch.clamp(at, max=b.shape[0] - 1)
    return (b.index_select(0, at) == a).all(dim=1)


class HotSpread:
    """The host-routed topology's routing state: the ketama ring over ``world`` GPUs, the
    replicated hot set and its spray weights, as tensors (device routing) and as the
    native ``HostRouter`` (host routing)."""

    def __init__(self, world: int, device, points_per_shard: int = 160):
        self.world = world
        self.device = torch.device(device)
        self.ring = ShardRing(list(range(world)), points_per_shard)
        self.pts, self.own = self.ring.tensors(self.device)
        self.router = core().HostRouter(world, points_per_shard)
        self.hot: Optional[torch.Tensor] = None     # [h, 2] sorted by lo
        self.hot_rank: Optional[torch.Tensor] = None  # int32 [h]: designated rank, -1 spray
        self.weights = [1.0] * world
        self.cw = torch.tensor(cumulative(self.weights), dtype=torch.float64, device=self.device)

    # -- decisions -----------------------------------------------------------------
    def owners(self, keys: torch.Tensor) -> torch.Tensor:
        return R.route(keys.contiguous(), self.pts, self.own, self.world)[0]

    def is_hot(self, keys: torch.Tensor) -> torch.Tensor:
        return member(keys, self.hot)

    def route_gets(self, keys: torch.Tensor, seq0: int = 0) -> torch.Tensor:
        """dest int32 [n] for a GET stream starting at stream position ``seq0``."""
        dest = self.owners(keys)
        if self.hot is None:
            return dest
        h = self.hot
        at = torch.clamp(torch.searchsorted(h[:, 0].contiguous(), keys[:, 0].contiguous()),
                         max=h.shape[0] - 1)
        hot = (h.index_select(0, at) == keys).all(dim=1)
        hr = self.hot_rank.to(keys.device).index_select(0, at)
        pos = torch.arange(keys.shape[0], dtype=torch.int64, device=keys.device) + int(seq0)
        sprayed = torch.where(hr >= 0, hr, spray_ranks(pos, self.cw.to(keys.device)))
        return torch.where(hot, sprayed, dest)

    def route_sets(self, keys: torch.Tensor) -> torch.Tensor:
        """dest int32 [n]: the owner, or -1 (a hot object: every rank stores it)."""
        dest = self.owners(keys)
        if self.hot is None:
            return dest
        return torch.where(self.is_hot(keys), torch.full_like(dest, -1), dest)

    # -- the hot set -----------------------------------------------------------------
    @staticmethod
    def top_keys(sample: torch.Tensor, k: int) -> torch.Tensor:
        """The k digests requested most often in ``sample`` (ties by digest order), sorted
        by lo: identical on every rank that sees the same sample."""
        if k <= 0 or sample.shape[0] == 0:
            return sample[:0]
        ulo, inv, cnt = torch.unique(sample[:, 0].contiguous(), return_inverse=True,
                                     return_counts=True)
        uniq = torch.empty((ulo.numel(), 2), dtype=torch.int64, device=sample.device)
        uniq[inv] = sample
        order = torch.sort(-cnt, stable=True).indices[:k]
        top = uniq.index_select(0, order)
        return top.index_select(0, torch.argsort(top[:, 0])).contiguous()

    def plan(self, sample: torch.Tensor, k: int, policy: str = "designate",
             spray_above: Optional[float] = None) -> dict:
        """Pick the hot set (top ``k`` of an observed GET sample) and how its GETs are
        spread, from the same sample, and install it. ``policy="designate"``: greedy
        designation (hottest first, each to the rank with the least load so far, starting
        from the non-hot owner loads); objects above ``spray_above`` of the traffic (default
        1/(4N)) are sprayed evenly. ``policy="spray"``: every hot object sprayed, water-filled
        weights. Returns the sample's shares and the planned per-rank load."""
        hot, ranks, w, info = self.design(sample, k, policy, spray_above)
        self.set_hot(hot, ranks, w)
        return info

    def design(self, sample: torch.Tensor, k: int, policy: str = "designate",
               spray_above: Optional[float] = None):
        """``plan`` without installing: (hot digests hottest first or None, designated ranks
        (None: all sprayed), spray weights, info)."""
        n = max(sample.shape[0], 1)
        if k <= 0 or sample.shape[0] == 0:
            return None, None, None, {"hot_share": 0.0}
        ulo, inv, cnt = torch.unique(sample[:, 0].contiguous(), return_inverse=True,
                                     return_counts=True)
        uniq = torch.empty((ulo.numel(), 2), dtype=torch.int64, device=sample.device)
        uniq[inv] = sample
        order = torch.sort(-cnt, stable=True).indices[:k]
        hot, hcnt = uniq.index_select(0, order), cnt.index_select(0, order)
        hmask = member(sample, hot.index_select(0, torch.argsort(hot[:, 0])))
        own = self.owners(sample).long()
        owner_load = torch.bincount(own[~hmask], minlength=self.world).double()
        hshare = float(hmask.float().mean())
        if policy == "spray":
            w = water_fill((owner_load / n).tolist(), hshare)
            return hot, None, w, {"hot_share": hshare, "owner_share": (owner_load / n).tolist(),
                                  "weights": w}
        if policy != "designate":
            raise ValueError(f"unknown spreading policy {policy!r}")
        thr = (spray_above if spray_above is not None else 1.0 / (4 * self.world)) * n
        load = owner_load.tolist()
        ranks = []
        import heapq

        cl = hcnt.tolist()
        sprayed = sum(c for c in cl if c > thr)
        for r in range(self.world):
            load[r] += sprayed / self.world
        heap = [(load[r], r) for r in range(self.world)]
        heapq.heapify(heap)
        for c in cl:
            if c > thr:
                ranks.append(-1)
                continue
            lr, r = heapq.heappop(heap)
            ranks.append(r)
            heapq.heappush(heap, (lr + c, r))
        for lr, r in heap:
            load[r] = lr
        return hot, torch.tensor(ranks, dtype=torch.int32), [1.0] * self.world, {
            "hot_share": hshare, "owner_share": (owner_load / n).tolist(),
            "sprayed_objects": sum(1 for r in ranks if r < 0),
            "planned_load": [x / n for x in load]}

    def set_hot(self, hot: Optional[torch.Tensor], ranks: Optional[torch.Tensor] = None,
                weights: Optional[Sequence[float]] = None):
        """Install a hot set: digests ``hot`` [h, 2], each one's designated rank (``ranks``
        int32 [h], -1 = sprayed; None = all sprayed) and the spray weights."""
        if hot is None or hot.shape[0] == 0:
            self.hot, self.hot_rank, self.weights = None, None, [1.0] * self.world
            self.router.set_hot(0, 0, 0, self.weights)
        else:
            order = torch.argsort(hot[:, 0])
            self.hot = hot.index_select(0, order).contiguous().to(self.device)
            r = (torch.full((hot.shape[0],), -1, dtype=torch.int32) if ranks is None
                 else ranks.to(torch.int32).cpu().index_select(0, order.cpu()))
            self.hot_rank = r.contiguous().to(self.device)
            self.weights = list(weights) if weights is not None else [1.0] * self.world
            # the native router in the given order (plan's: hottest first, so the objects
            # that carry most requests get their home slots)
            h = hot.cpu().contiguous()
            rh = (torch.full((hot.shape[0],), -1, dtype=torch.int32) if ranks is None
                  else ranks.to(torch.int32).cpu().contiguous())
            self.router.set_hot(h.data_ptr(), h.shape[0], rh.data_ptr(), self.weights)
        self.cw = torch.tensor(cumulative(self.weights), dtype=torch.float64, device=self.device)

    # -- the native router ---------------------------------------------------------------
    def host_route_gets(self, keys_host: torch.Tensor, seq0: int = 0, threads: int = 1,
                        out: Optional[torch.Tensor] = None):
        """The native router on host digests: (dest int32 [n], counts int64 [world]).
        ``out``: a reused int32 destination buffer (a proxy routes into buffers it keeps;
        fresh pages would add first-touch faults to the routing time)."""
        keys_host = keys_host.contiguous()
        dest = out if out is not None else torch.empty(keys_host.shape[0], dtype=torch.int32)
        counts = torch.zeros(self.world, dtype=torch.int64)
        self.router.route_gets(keys_host.data_ptr(), keys_host.shape[0], int(seq0),
                               dest.data_ptr(), counts.data_ptr(), int(threads))
        return dest, counts

    def host_route_sets(self, keys_host: torch.Tensor, threads: int = 1):
        keys_host = keys_host.contiguous()
        dest = torch.empty(keys_host.shape[0], dtype=torch.int32)
        counts = torch.zeros(self.world, dtype=torch.int64)
        self.router.route_sets(keys_host.data_ptr(), keys_host.shape[0], dest.data_ptr(),
                               counts.data_ptr(), int(threads))
        return dest, counts


def replicate_hot(cache, hot: torch.Tensor, owner: torch.Tensor, rank: int, world: int,
                  group=None, now: Optional[int] = None, if_absent: bool = False) -> int:
    """Collective: every rank stores, as ordinary objects of its shard, the hot objects it
    does not own, fetched from their owners — each owner looks its hot objects up and
    gathers their records, one all-gather moves them (RCCL over xGMI between GPUs, gloo
    between CPU ranks). ``cache`` is the rank's local (unrouted) ShardedCache, ``owner``
    the owner rank of each hot digest. ``if_absent``: a rank keeps a copy it already holds
    (a write-through SET that landed after the router began writing the object through is
    newer than the owner's copy read here). Returns the objects this rank stored (fetched)."""
    from ..models.sharded_cache import GetResult, records_to_set_batch

    dev = hot.device
    # gloo moves host tensors (a rehearsal of GPU ranks over gloo stages through the host)
    cdev = (torch.device("cpu") if dist.get_backend(group) == "gloo" else dev)
    mine = hot[owner.to(dev) == rank].contiguous()
    sh = cache.shard
    cache.sync_sets()
    lk = sh.lookup(mine, now)
    n = mine.shape[0]
    data = sh.gather(lk)
    nbytes = int(lk.off[n])
    meta = torch.tensor([n, nbytes], dtype=torch.int64, device=cdev)
    metas = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    m = torch.stack(metas).cpu()
    maxn, maxb = int(m[:, 0].max()), int(m[:, 1].max())
    # fixed-size blocks per rank: [keys | off | size] rows and the record bytes
    rows = torch.zeros((max(maxn, 1), 4), dtype=torch.int64, device=cdev)
    rows[:n, :2] = mine
    rows[:n, 2] = lk.off[:n]
    rows[:n, 3] = lk.size[:n]
    recs = torch.zeros(max(maxb, 16), dtype=torch.uint8, device=cdev)
    recs[:nbytes] = data[:nbytes]
    all_rows = [torch.empty_like(rows) for _ in range(world)]
    all_recs = [torch.empty_like(recs) for _ in range(world)]
    dist.all_gather(all_rows, rows, group=group)
    dist.all_gather(all_recs, recs, group=group)
    stored = 0
    for p in range(world):
        cnt = int(m[p, 0])
        if p == rank or cnt == 0:
            continue
        r = all_rows[p][:cnt].to(dev)
        res = GetResult(all_recs[p].to(dev), r[:, 2].contiguous(), r[:, 3].contiguous())
        sb = records_to_set_batch(r[:, :2].contiguous(), res)
        cache.set(sb, now, if_absent=if_absent)
        stored += int((r[:, 3] > 0).sum())
    cache.sync_sets()
    return stored


def refresh_hot(cache, spread: HotSpread, sample: torch.Tensor, k: int, rank: int, world: int,
                group=None, budget_bytes: Optional[int] = None, now: Optional[int] = None,
                policy: str = "designate", fetch=None, sizes=None) -> dict:
    """Collective (every rank, the same ``sample`` of the GET stream): move the replicated
    hot set to the top ``k`` of ``sample`` incrementally — only objects that became hot are
    fetched, at most ``budget_bytes`` of their records (hottest first; the rest wait for a
    later refresh), and the replicas of objects that cooled are dropped. Order, so that no GET
    is ever answered by a stale copy:

    1. the router writes the newly hot objects' SETs through to every rank, their GETs still
       going to their owners (they are hot, designated to the owner);
    2. their records are fetched from the owners into the other ranks, insert-if-absent (a
       SET written through since step 1 is newer than the owner's copy read here);
    3. the router installs the new hot set and designations (GETs of new objects may now go
       to any replica; objects that cooled go back to their owners, GETs and SETs);
    4. replicas of the cooled objects are deleted on the non-owner ranks (no SET reaches them
       any more: a later promotion must fetch a fresh copy, which insert-if-absent would
       otherwise refuse).

    ``cache``: this rank's local (unrouted) ShardedCache. ``fetch(digests, owners)`` and
    ``sizes(digests)`` replace the collectives (a simulated rank, bench.py --simulate-world:
    its peers' records come from the workload). Returns counts."""
    dev = spread.device
    old = spread.hot if spread.hot is not None else torch.zeros((0, 2), dtype=torch.int64,
                                                                  device=dev)
    old_rank = (spread.hot_rank if spread.hot_rank is not None
                else torch.zeros(0, dtype=torch.int32, device=dev))
    new, new_rank, new_w, info = spread.design(sample.to(dev), k, policy)
    if new is None:
        new = torch.zeros((0, 2), dtype=torch.int64, device=dev)
        new_rank = torch.zeros(0, dtype=torch.int32, device=dev)
    if new_rank is None:
        new_rank = torch.full((new.shape[0],), -1, dtype=torch.int32, device=dev)
    new_rank = new_rank.to(dev)
    old_sorted = old  # (sorted by lo)
    is_added = ~member(new, old_sorted)
    added, added_rank = new[is_added], new_rank[is_added]
    new_sorted = new.index_select(0, torch.argsort(new[:, 0])) if new.shape[0] else new
    removed = old[~member(old, new_sorted)]
    owner_added = spread.owners(added).long() if added.shape[0] else torch.zeros(
        0, dtype=torch.long, device=dev)
    # the budget, hottest first: record sizes from the owners (an all-reduce of each rank's
    # sizes of the objects it owns)
    deferred = 0
    if budget_bytes is not None and added.shape[0]:
        if sizes is not None:
            szc = sizes(added).to(torch.int64)
        else:
            sh = cache.shard
            cache.sync_sets()
            sz = torch.zeros(added.shape[0], dtype=torch.int64, device=dev)
            mine = owner_added == rank
            if bool(mine.any()):
                lk = sh.lookup(added[mine].contiguous(), now)
                sz[mine] = lk.size[: int(mine.sum())].to(torch.int64)
            cdev = torch.device("cpu") if dist.get_backend(group) == "gloo" else dev
            szc = sz.to(cdev)
            dist.all_reduce(szc, group=group)
        # every non-owner rank stores a copy: (world - 1) x the record per object
        keep = torch.cumsum(szc.to(dev) * (world - 1), 0) <= int(budget_bytes)
        deferred = int((~keep).sum())
        added, added_rank, owner_added = added[keep], added_rank[keep], owner_added[keep]
    kept = new[~is_added]
    kept_rank = new_rank[~is_added]
    # 1. write-through for the newly hot objects, their GETs still to their owners
    spread.set_hot(torch.cat([old, added]),
                   torch.cat([old_rank.to(dev), owner_added.to(torch.int32)]), spread.weights)
    # 2. fetch them into the other ranks, insert-if-absent
    fetched = (fetch(added, owner_added) if fetch is not None else
               replicate_hot(cache, added, owner_added, rank, world, group, now, if_absent=True))
    # 3. the new hot set (objects past the budget stay cold until a later refresh)
    final = torch.cat([kept, added])
    final_rank = torch.cat([kept_rank, added_rank])
    if final.shape[0]:
        spread.set_hot(final, final_rank, new_w if new_w is not None else spread.weights)
    else:
        spread.set_hot(None)
    # 4. drop the cooled objects' replicas (not on their owners)
    dropped = 0
    if removed.shape[0]:
        gone = removed[spread.owners(removed).long() != rank].contiguous()
        if gone.shape[0]:
            dropped = int(cache.delete(gone, now).sum())
    cache.sync_sets()
    return {"added": int(added.shape[0]), "deferred": deferred, "removed": int(removed.shape[0]),
            "replicas_dropped": dropped, "fetched": fetched, "hot": int(final.shape[0]),
            "hot_share": info.get("hot_share", 0.0)}
