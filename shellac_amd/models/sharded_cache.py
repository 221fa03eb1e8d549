"""ShardedCache: the flagship "model" — one logical cache over every GPU of a job.

Reference capability: "a single logical cache out of extra memory across the
entire cluster" (README.md:12, :30) built from ketama-sharded memcached nodes
(src/python/shellac/server/Server.py:79-83). Here each rank owns one
``CacheShard`` (its GPU's HBM), a ``ShardRing`` assigns digests to ranks, and a
serving step moves whole request batches with RCCL all-to-alls:

  GET:  route (k_route) -> group by owner (k_scatter + k_permute) -> a2a digests
        -> owner probe + scan (k_probe, hipcub) -> a2a sizes -> owner gather
        (k_segcopy, straight into the a2a send buffer) -> a2a values.
  SET:  route -> group -> pack payloads by owner (k_segcopy) -> a2a digests,
        metadata, payloads -> owner store (dedupe, scan-allocate, log write,
        CAS insert).

Two host syncs per phase (the split sizes all_to_all_single needs) and no
per-request host work. With one rank every step is purely local.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from ..ops.cache import CacheShard, Lookup
from ..ops import routing as R
from ..parallel.exchange import all_to_all_rows, dist_info, exchange_counts, segment_sums
from ..parallel.ring import ShardRing


@dataclass
class GetResult:
    """Values for a GET batch, in the caller's request order.

    ``data`` holds [ItemHeader|value|pad] records; request i's record is
    data[off[i] : off[i] + size[i]] (size 0 = miss)."""

    data: torch.Tensor
    off: torch.Tensor
    size: torch.Tensor

    def hit_mask(self) -> torch.Tensor:
        return self.size > 0


@dataclass
class SetBatch:
    keys: torch.Tensor      # int64 [n, 2]
    values: torch.Tensor    # uint8 payload buffer (16-B aligned values, +16 slack)
    val_off: torch.Tensor   # int64 [n]
    vlen: torch.Tensor      # int32 [n]
    flags: Optional[torch.Tensor] = None   # int32 [n]
    expire: Optional[torch.Tensor] = None  # int32 [n]


class ShardedCache:
    def __init__(self, shard: CacheShard, group=None, points_per_shard: int = 160):
        self.shard = shard
        self.group = group
        self.rank, self.world = dist_info(group)
        self.device = shard.device
        self.ring = ShardRing(list(range(self.world)), points_per_shard)
        self.ring_pts, self.ring_own = self.ring.tensors(self.device)
        self.stats = {"get_requests": 0, "set_requests": 0, "remote_gets": 0}

    # ------------------------------------------------------------------------------
    def _group_by_owner(self, keys: torch.Tensor):
        dest, counts = R.route(keys, self.ring_pts, self.ring_own, self.world)
        perm = R.scatter_positions(dest, counts)
        return dest, counts, perm

    def get(self, keys: torch.Tensor, now: Optional[int] = None) -> GetResult:
        n = keys.shape[0]
        self.stats["get_requests"] += n
        if self.world == 1:
            lk = self.shard.lookup(keys, now)
            data = self.shard.gather(lk)
            return GetResult(data, lk.off[:n], lk.size[:n])

        _, counts, perm = self._group_by_owner(keys)
        send_keys = R.permute(keys, perm)
        recv_counts = exchange_counts(counts, self.group)
        both = torch.cat([counts, recv_counts]).cpu()          # sync 1
        send_rows = both[: self.world].tolist()
        recv_rows = both[self.world :].tolist()
        req = all_to_all_rows(send_keys, send_rows, recv_rows, self.group)

        # owner side: probe my shard for everything I received
        lk = self.shard.lookup(req, now)
        m = req.shape[0]
        rc = torch.tensor(recv_rows, dtype=torch.int64, device=self.device)
        reply_bytes = segment_sums(lk.off, rc)                  # bytes I send back per source
        got_bytes = exchange_counts(reply_bytes, self.group)    # bytes I receive per owner
        nbytes = torch.cat([reply_bytes, got_bytes]).cpu()      # sync 2
        send_b = nbytes[: self.world].tolist()
        recv_b = nbytes[self.world :].tolist()
        out = torch.empty(max(int(sum(send_b)), 16), dtype=torch.uint8, device=self.device)
        self.shard.gather(lk, out)
        sizes_back = all_to_all_rows(lk.size[:m], recv_rows, send_rows, self.group)
        data = all_to_all_rows(out[: int(sum(send_b))], send_b, recv_b, self.group)

        # requester side: sizes_back/data are in grouped (perm) order
        goff = R.exclusive_scan(sizes_back)
        size = sizes_back.index_select(0, perm)
        off = goff.index_select(0, perm)
        self.stats["remote_gets"] += n - int(send_rows[self.rank])
        return GetResult(data, off, size)

    def set(self, batch: SetBatch, now: Optional[int] = None) -> None:
        n = batch.keys.shape[0]
        self.stats["set_requests"] += n
        if self.world == 1:
            self.shard.store(batch.keys, batch.values, batch.val_off, batch.vlen, batch.flags,
                             batch.expire, now)
            return
        dev = self.device
        _, counts, perm = self._group_by_owner(batch.keys)
        # metadata records [vlen, flags, expire, 0] as int32x4 (16 B)
        meta = torch.zeros((n, 4), dtype=torch.int32, device=dev)
        meta[:, 0] = batch.vlen
        if batch.flags is not None:
            meta[:, 1] = batch.flags
        if batch.expire is not None:
            meta[:, 2] = batch.expire
        send_keys = R.permute(batch.keys, perm)
        send_meta = R.permute(meta, perm)
        # pack payloads contiguously in owner order
        padded = (send_meta[:, 0].to(torch.int64) + 15) & ~15
        dst_off = R.exclusive_scan(padded)
        src_off = R.permute(batch.val_off.view(-1, 1), perm).view(-1)
        seg_bytes = segment_sums(dst_off, counts)
        recv_counts = exchange_counts(counts, self.group)
        recv_bytes = exchange_counts(seg_bytes, self.group)
        host = torch.cat([counts, recv_counts, seg_bytes, recv_bytes]).cpu()  # sync 1
        w = self.world
        send_rows, recv_rows = host[:w].tolist(), host[w : 2 * w].tolist()
        send_b, recv_b = host[2 * w : 3 * w].tolist(), host[3 * w :].tolist()
        payload = torch.empty(int(sum(send_b)) + 16, dtype=torch.uint8, device=dev)
        R.segcopy(batch.values, src_off, dst_off, payload)
        rkeys = all_to_all_rows(send_keys, send_rows, recv_rows, self.group)
        rmeta = all_to_all_rows(send_meta, send_rows, recv_rows, self.group)
        rvals = torch.empty(int(sum(recv_b)) + 16, dtype=torch.uint8, device=dev)
        dist_out = rvals[: int(sum(recv_b))]
        torch.distributed.all_to_all_single(dist_out, payload[: int(sum(send_b))],
                                            output_split_sizes=recv_b, input_split_sizes=send_b,
                                            group=self.group)
        rvlen = rmeta[:, 0].contiguous()
        roff = R.exclusive_scan((rvlen.to(torch.int64) + 15) & ~15)[:-1].contiguous()
        self.shard.store(rkeys, rvals, roff, rvlen, rmeta[:, 1].contiguous(),
                         rmeta[:, 2].contiguous(), now)

    def delete(self, keys: torch.Tensor, now: Optional[int] = None) -> torch.Tensor:
        n = keys.shape[0]
        if self.world == 1:
            return self.shard.remove(keys, now)
        _, counts, perm = self._group_by_owner(keys)
        send_keys = R.permute(keys, perm)
        recv_counts = exchange_counts(counts, self.group)
        both = torch.cat([counts, recv_counts]).cpu()
        send_rows, recv_rows = both[: self.world].tolist(), both[self.world :].tolist()
        req = all_to_all_rows(send_keys, send_rows, recv_rows, self.group)
        found = self.shard.remove(req, now).to(torch.int32)
        back = all_to_all_rows(found, recv_rows, send_rows, self.group)
        return back.index_select(0, perm).bool()

    def counters(self) -> dict:
        from ..parallel.exchange import allreduce_stats

        return allreduce_stats(self.shard.counters(), self.device, self.group)
