"""Collective primitives of the sharded cache (one process per GPU, RCCL over xGMI).

The reference has no collectives: each proxy makes a blocking TCP round trip to
the memcached node that ketama picks (src/python/shellac/server/Server.py:335,
:432). With one process per MI355X the equivalent is *batched*: every rank
routes a whole batch of digests on the device, and one ``all_to_all_single``
moves each rank's requests to their owner shards (and one more moves the
values back) — the same dispatch/combine shape as expert parallelism. On the
CPU (tests) the same code runs over gloo.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch
import torch.distributed as dist


def dist_info(group=None) -> tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def all_to_all_rows(x: torch.Tensor, send_rows: Sequence[int], recv_rows: Sequence[int],
                    group=None) -> torch.Tensor:
    """all_to_all_single over the first dim with explicit row splits."""
    out = torch.empty((int(sum(recv_rows)),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_to_all_single(out, x.contiguous(), output_split_sizes=list(map(int, recv_rows)),
                           input_split_sizes=list(map(int, send_rows)), group=group)
    return out


def exchange_counts(counts: torch.Tensor, group=None) -> torch.Tensor:
    """counts[r] = rows I send to r  ->  rows r sends to me (same device)."""
    out = torch.empty_like(counts)
    dist.all_to_all_single(out, counts.contiguous(), group=group)
    return out


def allreduce_stats(stats: dict, device, group=None) -> dict:
    """Sum integer counters over all shards with one tiny all-reduce."""
    keys = sorted(stats)
    t = torch.tensor([int(stats[k]) for k in keys], dtype=torch.int64, device=device)
    if dist_info(group)[1] > 1:
        dist.all_reduce(t, group=group)
    return {k: int(v) for k, v in zip(keys, t.tolist())}


def segment_sums(off: torch.Tensor, counts: torch.Tensor) -> torch.Tensor:
    """Given an exclusive scan ``off`` ([n+1]) of per-row sizes and row counts per
    segment, return the byte total of each segment (device op, no sync)."""
    ends = torch.cumsum(counts, 0)
    starts = ends - counts
    return off.index_select(0, ends) - off.index_select(0, starts)
