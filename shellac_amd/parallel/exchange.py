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


class MirrorComm:
    """Single-process stand-in for an N-rank group whose traffic is symmetric: every
    peer sends me exactly what I send it, so an all-to-all returns its input.

    Profiling tool only (``bench.py --simulate-world N``): it runs the complete routed
    serving step of rank 0 of an N-rank job on one GPU — routing, packing, owner
    lookups, gathers, stores, host syncs, Python overhead — with the interconnect
    transfers replaced by local copies. It never produces a scaling number."""

    def __init__(self, world: int, rank: int = 0):
        self.world, self.rank = int(world), int(rank)


class BounceComm:
    """Device tensors exchanged through a host (gloo) process group: every collective
    copies to the CPU, runs over gloo, and copies back (synchronously).

    Test tool: it runs the real multi-process routed step — asymmetric traffic, every
    rank its own shard — when the ranks share one GPU and RCCL cannot be used (RCCL
    refuses two ranks on one device). Never a performance path."""

    def __init__(self, pg=None):
        self.pg = pg
        self.rank, self.world = dist.get_rank(pg), dist.get_world_size(pg)


class LocalComm:
    """The group of a rank that serves only the keys it owns: a host-routed process of an
    N-GPU job (ketama runs on the host proxies), or any process that has a
    default process group for other work. World 1, every collective an identity; without
    it ``group=None`` would mean the default (world) group once torch.distributed is up,
    and the cache would route its batches over it."""

    rank, world = 0, 1


class _Done:
    def wait(self):
        return True


def dist_info(group=None) -> tuple[int, int]:
    if isinstance(group, (MirrorComm, BounceComm, LocalComm)):
        return group.rank, group.world
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def all_to_all_single(out: torch.Tensor, inp: torch.Tensor, output_split_sizes=None,
                      input_split_sizes=None, group=None, async_op: bool = False):
    """torch.distributed.all_to_all_single (RCCL on ROCm) or the mirror stand-in."""
    if isinstance(group, (MirrorComm, LocalComm)):
        if out.numel() != inp.numel():
            raise ValueError("mirror all_to_all needs symmetric splits")
        out.copy_(inp.view(out.shape) if out.shape != inp.shape else inp)
        return _Done() if async_op else None
    if isinstance(group, BounceComm):
        host_out = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(host_out, inp.cpu(), output_split_sizes=output_split_sizes,
                               input_split_sizes=input_split_sizes, group=group.pg)
        out.copy_(host_out)
        return _Done() if async_op else None
    # Straight to the process group's C++ collective: torch.distributed's Python wrapper
    # spends ~36 us per call on argument checks and group bookkeeping (cProfile of the
    # routed step, profiles/archive/r2_routed_host_profile.txt), and a step issues 5 of them.
    pg = group if group is not None else _default_group()
    opts = dist.AllToAllOptions()
    work = pg.alltoall_base(out, inp, list(output_split_sizes or []),
                            list(input_split_sizes or []), opts)
    if async_op:
        return work
    work.wait()  # stream-ordered: the current stream waits for the collective
    return None


def _default_group():
    from torch.distributed import distributed_c10d

    return distributed_c10d._get_default_group()


_MIRROR_IDX: dict = {}


def _mirror_index(k: int, world: int, me: int, peer_blocks: int, device) -> torch.Tensor:
    """Gather index of every rank's row under MirrorComm's symmetric traffic: what rank q
    sends to x is what I send to x with the roles of me and q exchanged (q -> me equals
    me -> q); one index_select builds the whole matrix."""
    key = (k, world, me, peer_blocks, str(device))
    idx = _MIRROR_IDX.get(key)
    if idx is None:
        rows = []
        for q in range(world):
            r = list(range(k))
            if q != me:
                for b in range(peer_blocks):
                    r[b * world + me], r[b * world + q] = r[b * world + q], r[b * world + me]
            rows += r
        idx = _MIRROR_IDX[key] = torch.tensor(rows, dtype=torch.int64, device=device)
    return idx


def all_gather_rows(out: torch.Tensor, row: torch.Tensor, group=None, peer_blocks: int = 0) -> None:
    """out[q * K : (q + 1) * K] = rank q's ``row`` (K words) for every rank q, stream-ordered
    (the current stream waits for it). ``peer_blocks``: the row starts with that many
    blocks of one entry per peer (used only to mirror rows under ``MirrorComm``)."""
    rank, world = dist_info(group)
    if isinstance(group, LocalComm):
        out.copy_(row)
        return
    if isinstance(group, MirrorComm):
        torch.index_select(row, 0, _mirror_index(row.numel(), world, rank, peer_blocks,
                                                 row.device), out=out)
        return
    if isinstance(group, BounceComm):
        host = [torch.empty(row.shape, dtype=row.dtype) for _ in range(world)]
        dist.all_gather(host, row.cpu(), group=group.pg)
        out.copy_(torch.cat(host))
        return
    pg = group if group is not None else _default_group()
    if hasattr(pg, "_allgather_base"):
        pg._allgather_base(out, row).wait()  # the C++ collective (no Python-wrapper overhead)
    else:
        dist.all_gather_into_tensor(out, row, group=group)


def all_gather(tensors: list, t: torch.Tensor, group=None) -> None:
    if isinstance(group, (MirrorComm, LocalComm)):
        for x in tensors:
            x.copy_(t)
        return
    if isinstance(group, BounceComm):
        host = [torch.empty(x.shape, dtype=x.dtype) for x in tensors]
        dist.all_gather(host, t.cpu(), group=group.pg)
        for x, h in zip(tensors, host):
            x.copy_(h)
        return
    dist.all_gather(tensors, t, group=group)


def all_reduce(t: torch.Tensor, op=None, group=None) -> None:
    op = dist.ReduceOp.SUM if op is None else op
    if isinstance(group, LocalComm):
        return
    if isinstance(group, MirrorComm):
        if op == dist.ReduceOp.SUM:
            t.mul_(group.world)
        return
    if isinstance(group, BounceComm):
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group.pg)
        t.copy_(h)
        return
    dist.all_reduce(t, op=op, group=group)


def barrier(group=None) -> None:
    if isinstance(group, BounceComm):
        dist.barrier(group=group.pg)
    elif not isinstance(group, (MirrorComm, LocalComm)):
        dist.barrier(group=group)


def all_to_all_rows(x: torch.Tensor, send_rows: Sequence[int], recv_rows: Sequence[int],
                    group=None) -> torch.Tensor:
    """all_to_all_single over the first dim with explicit row splits."""
    out = torch.empty((int(sum(recv_rows)),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    all_to_all_single(out, x.contiguous(), output_split_sizes=list(map(int, recv_rows)),
                      input_split_sizes=list(map(int, send_rows)), group=group)
    return out


def exchange_counts(counts: torch.Tensor, group=None) -> torch.Tensor:
    """counts[r] = rows I send to r  ->  rows r sends to me (same device)."""
    out = torch.empty_like(counts)
    all_to_all_single(out, counts.contiguous(), group=group)
    return out


def allreduce_stats(stats: dict, device, group=None) -> dict:
    """Sum integer counters over all shards with one tiny all-reduce."""
    keys = sorted(stats)
    t = torch.tensor([int(stats[k]) for k in keys], dtype=torch.int64, device=device)
    if dist_info(group)[1] > 1:
        all_reduce(t, group=group)
    return {k: int(v) for k, v in zip(keys, t.tolist())}


def segment_sums(off: torch.Tensor, counts: torch.Tensor) -> torch.Tensor:
    """Given an exclusive scan ``off`` ([n+1]) of per-row sizes and row counts per
    segment, return the byte total of each segment (device op, no sync)."""
    ends = torch.cumsum(counts, 0)
    starts = ends - counts
    return off.index_select(0, ends) - off.index_select(0, starts)


# ---- communicators of the native routed step (csrc/step_comm.h) ----------------------------
_RCCL_COMMS: dict = {}
_RCCL_SEQ = [0]


class _BounceNative:
    """``BounceComm`` for the native executor: the step's collectives call back into
    Python with raw device pointers; bytes are staged through host memory and exchanged
    over gloo (tests only: several ranks sharing one GPU)."""

    def __init__(self, comm: BounceComm):
        self.comm = comm

    def native_all_gather(self, out: int, inp: int, words: int, peer_blocks: int,
                          stream: int) -> None:
        from .._native import core

        c = core()
        row = torch.frombuffer(bytearray(c.stream_copy_to_host(inp, 8 * words, stream)),
                               dtype=torch.int64)
        host = [torch.empty(words, dtype=torch.int64) for _ in range(self.comm.world)]
        dist.all_gather(host, row, group=self.comm.pg)
        c.stream_copy_from_host(out, torch.cat(host).numpy().tobytes(), stream)

    def native_all_to_all(self, rbuf: int, roff, rbytes, sbuf: int, soff, sbytes,
                          stream: int) -> None:
        from .._native import core

        c = core()
        me, w = self.comm.rank, self.comm.world
        sb = [0 if p == me else int(sbytes[p]) for p in range(w)]
        rb = [0 if q == me else int(rbytes[q]) for q in range(w)]
        blob = b"".join(c.stream_copy_to_host(sbuf + int(soff[p]), sb[p], stream)
                        for p in range(w) if sb[p])
        send = (torch.frombuffer(bytearray(blob), dtype=torch.uint8) if blob
                else torch.empty(0, dtype=torch.uint8))
        recv = torch.empty(sum(rb), dtype=torch.uint8)
        dist.all_to_all_single(recv, send, output_split_sizes=rb, input_split_sizes=sb,
                               group=self.comm.pg)
        pos = 0
        for q in range(w):
            if rb[q]:
                c.stream_copy_from_host(rbuf + int(roff[q]), recv[pos:pos + rb[q]].numpy().tobytes(),
                                        stream)
                pos += rb[q]


def _rccl_comm(world: int, rank: int, device: int):
    """RCCL communicators of our own (one per channel of the routed step), shared by every
    executor of this process. Collective on first use: rank 0 makes the unique ids and
    publishes them in the torch.distributed store, every rank joins."""
    from .._native import core

    key = (world, rank, device)
    comm = _RCCL_COMMS.get(key)
    if comm is None:
        c = core()
        store = _default_store()
        name = f"shellac_amd/rccl_ids/{_RCCL_SEQ[0]}"
        _RCCL_SEQ[0] += 1
        nch = 3
        if rank == 0:
            ids = [c.rccl_unique_id() for _ in range(nch)]
            store.set(name, b"".join(ids))
        blob = bytes(store.get(name))
        ids = [blob[i * 128:(i + 1) * 128] for i in range(nch)]
        comm = _RCCL_COMMS[key] = c.make_rccl_comm(world, rank, device, ids)
    return comm


def _default_store():
    from torch.distributed import distributed_c10d

    return distributed_c10d._get_default_store()


def step_comm(group, device: torch.device):
    """The communicator the native routed step (``RoutedStep.step``) issues its collectives
    on, or None when only the multi-call path can serve this group (a custom torch group,
    a non-RCCL backend, a CPU shard)."""
    from .._native import core

    if device.type != "cuda" or isinstance(group, LocalComm):
        return None
    c = core()
    if isinstance(group, MirrorComm):
        return c.make_mirror_comm(group.world, group.rank)
    if isinstance(group, BounceComm):
        return c.make_python_comm(_BounceNative(group), group.world, group.rank)
    if not (dist.is_available() and dist.is_initialized()):
        return None
    if group is not None and group is not _default_group():
        return None
    if dist.get_backend() != "nccl":
        return None
    return _rccl_comm(dist.get_world_size(), dist.get_rank(), device.index)
