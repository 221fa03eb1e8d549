"""ShardedCache: the flagship "model" — one logical cache over every GPU of a job.

Reference capability: "a single logical cache out of extra memory across the
entire cluster" (README.md:12, :30) built from ketama-sharded memcached nodes
(src/python/shellac/server/Server.py:79-83). Here each rank owns one
``CacheShard`` (its GPU's HBM), a ``ShardRing`` assigns digests to ranks, and a
serving step moves whole request batches with RCCL all-to-alls:

  GET:  [replica probe] -> route (k_route) -> group by owner (k_scatter,
        k_permute) -> a2a digests -> owner probe + scan (k_probe, hipcub) ->
        a2a sizes -> owner gather (k_segcopy, straight into the a2a send
        buffer) -> a2a values into the caller's response buffer.
  SET:  route (+ fan-out of replicated keys to every rank) -> group -> pack
        payloads (k_segcopy) -> a2a digests, metadata, payloads -> owner store
        (dedupe, scan-allocate, log write, CAS insert) / replica store.

Hot-object replication (SURVEY.md §5.8 "hot-key broadcast"): Zipf-popular
objects are copied into a small per-rank *replica* shard so their GETs never
leave the GPU. ``refresh_replica`` picks the global top-k keys from recent
request samples (one all_gather of candidates + one routed GET). Consistency is
write-through with no extra collective: a SET for a replicated key is fanned out
by the same all-to-all to its owner (main shard) and to every other rank
(replica shard), so a GET issued after a SET step never sees the old value.

Two host syncs per phase (the split sizes all_to_all_single needs) and no
per-request host work. With one rank every step is purely local.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import routing as R
from ..ops.cache import CacheShard, StreamEvent, coalesce, expand, expand_out
from ..parallel.exchange import (MirrorComm, all_gather, all_gather_rows, all_reduce, all_to_all_rows,
                                 all_to_all_single, allreduce_stats, dist_info, exchange_counts,
                                 segment_sums, step_comm)
from ..parallel.ring import ShardRing
from .._native import core as _core

SKIP_VLEN = -1  # int32 view of the kSkipVlen sentinel (row not for this tier)
HDR_WORDS = 8   # ItemHeader = 8 x u32: d0 lo/hi, d1 lo/hi, vlen, flags, expire, magic


@dataclass
class GetResult:
    """Values for a GET batch, in the caller's request order.

    ``data`` holds [ItemHeader|value|pad] records; request i's record is
    data[off[i] : off[i] + size[i]] (size 0 = miss)."""

    data: torch.Tensor
    off: torch.Tensor
    size: torch.Tensor
    _pending: Optional[object] = None  # value all-to-all still in flight (routed serve)

    def wait(self) -> "GetResult":
        """Order the current stream after the reply transfer. A routed ``serve`` returns
        while its reply all-to-all (and the per-request assembly that reads its in-band
        headers) is still running, so the next step's routing overlaps it; a host-edge
        ``serve`` returns while the DMA copy of its response into host memory runs (then
        this blocks the host until it is done); call this before reading ``data``, ``off``
        or ``size``."""
        if self._pending is not None:
            self._pending.wait()
            self._pending = None
        return self

    def hit_mask(self) -> torch.Tensor:
        return self.size > 0


class _HostCopy:
    """A response still being copied to host memory (host edge): wait() blocks the host
    until the copy is done."""

    def __init__(self, event):
        self.event = event

    def wait(self):
        self.event.synchronize()


@dataclass
class SetBatch:
    keys: torch.Tensor      # int64 [n, 2]
    values: torch.Tensor    # uint8 payload buffer (16-B aligned values, +16 slack)
    val_off: torch.Tensor   # int64 [n]
    vlen: torch.Tensor      # int32 [n]
    flags: Optional[torch.Tensor] = None   # int32 [n]
    expire: Optional[torch.Tensor] = None  # int32 [n]
    # simulated world only (bench.py --simulate-world): the digests the owner stores
    probe_keys: Optional[torch.Tensor] = None  # int64 [n, 2]


class _StreamDone:
    """A routed step's reply transfer + assembly, finished on a side stream: wait() makes
    the current stream wait for it (no host synchronisation)."""

    def __init__(self, event):
        self.event = event

    def wait(self):
        torch.cuda.current_stream(self.event.device).wait_event(self.event)
        return True


def records_to_set_batch(keys: torch.Tensor, res: GetResult) -> SetBatch:
    """Turn GET records back into a SET batch (replica fill, shard migration).
    Misses become skip rows."""
    words = res.data[: res.data.numel() // 4 * 4].view(torch.int32)
    hit = res.size > 0
    base = torch.where(hit, torch.div(res.off, 4, rounding_mode="floor"), torch.zeros_like(res.off))
    v = words.index_select(0, base + 4)
    vlen = torch.where(hit, v, torch.full_like(v, SKIP_VLEN))
    flags = words.index_select(0, base + 5)
    expire = words.index_select(0, base + 6)
    val_off = torch.where(hit, res.off + 32, torch.zeros_like(res.off))
    return SetBatch(keys=keys.contiguous(), values=res.data, val_off=val_off.contiguous(),
                    vlen=vlen.contiguous(), flags=flags.contiguous(), expire=expire.contiguous())


def _hot_directory(hot: torch.Tensor) -> torch.Tensor:
    """dir[b] = first row of ``hot`` (sorted by signed lo) whose order-preserving unsigned
    image of lo has top-16 bits >= b; b in [0, 65536]. Lets the device membership test
    binary-search ~len(hot)/65536 rows instead of all of them."""
    b = torch.arange(65537, dtype=torch.int64, device=hot.device)
    bounds = (b - 32768) << 48            # signed value whose unsigned image is b << 48
    bounds[-1] = torch.iinfo(torch.int64).max
    d = torch.searchsorted(hot[:, 0].contiguous(), bounds, side="left")
    d[-1] = hot.shape[0]
    return d.contiguous()


class _Phases:
    """Consecutive ROCTX ranges for the phases of one serving step (no-op when
    tracing is off; see shellac_amd.utils.trace)."""

    def __init__(self, prefix: str):
        self.c = _core()
        self.on = self.c.trace_on()
        self.prefix = prefix
        self.open = False

    def next(self, name: str) -> None:
        if not self.on:
            return
        if self.open:
            self.c.trace_pop()
        self.c.trace_push(self.prefix + name)
        self.open = True

    def end(self) -> None:
        if self.on and self.open:
            self.c.trace_pop()
            self.open = False


def _event_handle(ev) -> int:
    """hipEvent_t of a recorded torch.cuda.Event / StreamEvent (0: none)."""
    if ev is None:
        return 0
    if isinstance(ev, StreamEvent):
        return int(ev.handle)
    return int(ev.cuda_event)


class ShardedCache:
    HANDS = ("early", "inline")

    def __init__(self, shard: CacheShard, group=None, points_per_shard: int = 160,
                 replica: Optional[CacheShard] = None, sample_rows: int = 65536,
                 sample_batches: int = 8, data_group=None, routed: Optional[bool] = None,
                 comm_mode: str = "channels", hand: str = "early"):
        self.shard = shard
        self.group = group
        # native routed step: "single" = every collective of a step on one communicator and
        # one stream in a fixed order (cannot deadlock); "channels" (the default) = one
        # communicator per channel (control, reply, SET) on the stream producing its data
        if comm_mode not in ("single", "channels"):
            raise ValueError(f"comm_mode must be 'single' or 'channels', not {comm_mode!r}")
        self.comm_mode = comm_mode
        # Optional second communicator for the value all-to-all: its stream runs the
        # previous step's value transfer while this step's small exchanges proceed.
        self.data_group = data_group if data_group is not None else group
        self.rank, self.world = dist_info(group)
        # routed: batches go through the collectives (routing, all-to-alls, replica tier).
        # Default: with more than one rank. routed=True at world 1 runs the same path over
        # a one-rank group — a real RCCL communicator on one GPU (the test and rehearsal of
        # the multi-GPU step's collective calls that a one-GPU box can run)
        self.routed = self.world > 1 if routed is None else bool(routed)
        self.device = shard.device
        self.ring = ShardRing(list(range(self.world)), points_per_shard)
        self.ring_pts, self.ring_own = self.ring.tensors(self.device)
        self.replica = replica if self.routed else None
        self.sample_rows = sample_rows
        self.sample_batches = sample_batches
        self._samples: List[torch.Tensor] = []
        self._hot: Optional[torch.Tensor] = None   # sorted hot digests [h, 2] (same on all ranks)
        # GPU shards run the routed step through the fused native ops (csrc/router.hip);
        # the framework-op version (_serve_routed) is the CPU path and the test oracle
        self.fused = True
        self._engine = None
        # the native step's communicator (RCCL / mirror / gloo callbacks); False: none,
        # every step takes the multi-call path (collectives from Python)
        self._ncomm = None
        self._row = self._mat = None
        # the routed step's main-shard SET chain is joined by the NEXT step's owner probe
        # (RoutedStep::join_sets), so it runs under that step's planning; its buffers stay
        # referenced until then
        self._held = None
        self._asm = None      # side stream of the routed step's reply assembly
        # buffers the reply all-to-all (on the communicator's own stream) still reads or
        # writes after serve returns: released two steps later, once the current stream
        # has waited for that step's assembly (so the allocator never hands them out while
        # the transfer runs)
        self._inflight = []
        self._hot_dir = None  # 65537-entry directory into self._hot (built lazily)
        # incremental migration (set_ring): keys SET / DELETEd since the ring switch
        self._migrating = None
        self._touched = None
        self._touched_all = None
        # simulated world: request digests -> the digests their owners hold (see serve)
        self.probe_of = None
        # replica refresh: scores of the hot keys (aligned with _hot) and their decay per
        # refresh (_hot_candidates)
        self._hot_score = None
        self.hot_decay = 0.5
        # run SET chains on a side stream, concurrently with GET gathers (GPU shards)
        self.overlap_store = True
        # GET coalescing: the duplicate keys of a batch share one probe and one record
        # (ops.cache.coalesce); False probes and copies every request (bench --no-coalesce)
        self.coalesce = True
        # (Two other N=1 schedules were measured slower and removed: a compacting lookup
        # with bump-allocated response offsets, and the SET planning kernels ahead of the
        # lookup; profiles/archive/r2_step_schedule_ab.md.)
        # (Queuing the SET index insert after the host read the lookup total, with no
        # event between lookup and gather, needs the total published only once every
        # lookup workgroup has released its outputs: a device-scope fence per workgroup,
        # which cost ~30 us per step in k_offsets. Not adopted.)
        # fence scope of the events that order the main and side streams of a step:
        # "system" = torch's events (a system-scope release: L2 write-back + invalidate
        # at every record); "device" / "none" (default) = StreamEvent with a device-scope
        # release / no system fence (both streams are on one GPU; nothing on the host reads
        # what these events order, and every kernel dispatch carries its own release). One
        # box, two rounds: 0.309 / 0.308 ms per step with "device" vs 0.315 / 0.311 with
        # "system" (profiles/archive/r2_event_fence_ab.log); round 4, one box, two rounds each:
        # wrapped 0.3362 / 0.3363 "device" vs 0.3313 / 0.3304 "none", fresh 0.3008 / 0.3004
        # vs 0.2953 / 0.2952 (profiles/archive/r4h_fence)
        self.event_fence = "none"
        # the step's cross-stream events ride on the kernels' own completion signals: the
        # lookup's probe completes `probe` (the index insert's wait), the SET chain's index
        # fix-up completes the step's end (the next lookup's wait), and the log append waits
        # for the step's input event instead of a `start` marker behind the previous chain
        # — no marker packet on the main stream's critical path (each costs ~2.7 us; a stop
        # event is seen ~2.4 us sooner across streams than a recorded one: profiles/r6_hop).
        # Needs StreamEvents (event_fence != "system"). SHELLAC_STOP_EVENTS=0: markers.
        self.stop_events = os.environ.get("SHELLAC_STOP_EVENTS", "1") != "0"
        # fence scope of the events kernels complete as stop events (A/B: SHELLAC_STOP_FENCE)
        self.stop_fence = os.environ.get("SHELLAC_STOP_FENCE", "none")
        self._probe_stopped = False   # the last step lookup completed its `probe` itself
        # one GPU: the gather waits for the SET batch's log append (see serve)
        self.gather_after_append = False
        # one GPU, a full cache: where the SET batch's CLOCK hand runs (see serve).
        # "early": detached, on a stream of its own, as soon as the previous step's SET
        # planning is done — beside that step's log append, index insert and gather; its
        # reinsertions are indexed as moves (HbmCache::store). "inline": at the head of the
        # SET chain on the side stream, after the lookup is queued.
        if hand not in self.HANDS:
            raise ValueError(f"hand must be one of {self.HANDS}, not {hand!r}")
        self.hand = hand
        self._side_pending = False
        self._planned = False    # the serve pipeline orders the next hand (see serve)
        self._ends = [None, None]  # per step parity: recorded after the step's SET chain
        self._last_end = None
        self._held_steps = []    # the SET batches the last two steps' chains may still read
        self._hand_s = None
        self._events = {}
        self._side = None
        self._gather_cap = 0     # response buffer bytes for the unsynced gather
        self._co_table = None    # persistent GET-coalescing table (serve, side stream)
        # host edge (one rank): GET digests / SET payloads may be pinned host tensors and
        # responses are gathered straight into pinned host memory, as the proxy's HBM
        # tier does (bench.py --edge host)
        self.host_edge = False
        # host edge: the gather writes the response into HBM and a DMA engine copies it to
        # the pinned host buffer (56 GB/s D2H, scripts/pcie_d2h_micro.py) instead of the
        # gather kernel storing over PCIe itself (~38 GB/s)
        self.host_edge_dma = True
        self._dma = [None, None]       # per turn: (staging buffer, copy-done event)
        self._copy_stream = None
        self._last_pending = None
        self.gathered_bytes = 0  # response bytes the serving steps produced
        self._stats = {"get_requests": 0, "set_requests": 0, "remote_gets": 0,
                      "replica_hits": 0, "replica_refreshes": 0, "coalesced_gets": 0,
                      "slot_overflow_rows": 0, "reply_dropped_rows": 0}

    # ------------------------------------------------------------------------------
    @property
    def stats(self) -> dict:
        """Serving counters. The native routed step learns its own per-step numbers two
        steps late (it never waits for a step's matrix); reading them here collects every
        step issued so far (the host waits for the latest step's all-gather, not for the
        step)."""
        e = self._engine
        if e is not None:
            e.harvest_all()
            self._add_step_stats(e.take_stats())
        return self._stats

    def sync_sets(self) -> None:
        """Order the current stream after the SETs of the last routed ``serve`` (whose
        main-shard store may still be running on the executor's store stream). Every
        other ShardedCache method calls it; call it before using ``self.shard`` directly
        after a routed ``serve`` (a device synchronisation also does)."""
        if self._side_pending:
            # the last one-GPU serve's SET chain (serve leaves it for the next step)
            self._wait(torch.cuda.current_stream(self.device), self._last_end)
            self._side_pending = False
        self._held_steps = []
        # whatever runs next on the caller's stream (a set, a delete, ...) is not covered by
        # the last serve's plan event: the next early hand follows the caller's stream
        self._planned = False
        e = self._engine
        if e is not None and e.sets_pending:
            e.join_sets(torch.cuda.current_stream(self.device).cuda_stream)
            self._held = None
        if e is not None:
            # the native step's statistics run two steps behind: collect the rest
            e.harvest_all()
            self._add_step_stats(e.take_stats())

    def _add_step_stats(self, h) -> None:
        n_local, n_dup, off_rank, over, dropped = h
        self._stats["remote_gets"] += off_rank
        self._stats["replica_hits"] += n_local - n_dup
        self._stats["coalesced_gets"] += n_dup
        self._stats["slot_overflow_rows"] += over
        self._stats["reply_dropped_rows"] += dropped

    def _reset_exchange(self) -> None:
        """The traffic matrix changes (new ring, new hot set): the routed step's next
        serve recalibrates its slot capacities (collective: every rank calls it)."""
        if self._engine is not None:
            self._engine.reset_caps()

    def recalibrate(self) -> None:
        """Collective. The routed step sizes its per-peer exchange slots from the demand
        of earlier steps; after a change of batch shape (say, a much larger GET batch)
        the first steps would answer the rows that do not fit as misses until the
        capacities catch up. Calling this on every rank makes the next serve measure the
        new demand exactly (one step with two host reads) instead."""
        self.sync_sets()
        self._reset_exchange()

    def _route(self, keys: torch.Tensor):
        return R.route(keys, self.ring_pts, self.ring_own, self.world)

    def _sample(self, keys: torch.Tensor) -> None:
        if self.replica is None:
            return
        self._samples.append(keys[: self.sample_rows])
        if len(self._samples) > self.sample_batches:
            self._samples.pop(0)

    def _is_hot(self, keys: torch.Tensor) -> torch.Tensor:
        """Membership of each digest in the replicated hot set (device op, no sync)."""
        h = self._hot
        idx = torch.searchsorted(h[:, 0].contiguous(), keys[:, 0].contiguous())
        idx = torch.clamp(idx, max=h.shape[0] - 1)
        cand = h.index_select(0, idx)
        return (cand == keys).all(dim=1)

    def get(self, keys: torch.Tensor, now: Optional[int] = None,
            probe_keys: Optional[torch.Tensor] = None) -> GetResult:
        """GET a batch (collective when routed). ``probe_keys`` (simulated world only): the
        digests the owners probe for each request."""
        self.sync_sets()
        n = keys.shape[0]
        self._stats["get_requests"] += n
        if not self.routed:
            if self.coalesce:
                lk, first, _ = self.shard.lookup_coalesced(keys, now)
            else:
                lk, first = self.shard.lookup(keys, now), None
            data = self.shard.gather(lk)
            expand(first, lk.size, lk.off)
            return GetResult(data, lk.off[:n], lk.size[:n])
        self._sample(keys)
        w = self.world
        dest, _ = self._route(keys)
        rl = None
        if self.replica is not None:
            rl = self.replica.lookup(keys, now)           # local copies of hot objects
            local = rl.size[:n] > 0
            dest = torch.where(local, torch.full_like(dest, w), dest)
        counts = torch.bincount(dest.long(), minlength=w + 1)
        perm = R.scatter_positions(dest, counts)         # local hits sort to the tail
        send_keys = R.permute(keys if probe_keys is None else probe_keys, perm)
        recv_counts = exchange_counts(counts[:w].contiguous(), self.group)
        local_total = rl.off[n:n + 1] if rl is not None else torch.zeros(1, dtype=torch.int64,
                                                                           device=self.device)
        host = torch.cat([counts, recv_counts, local_total]).cpu()       # sync 1
        send_rows, n_local = host[:w].tolist(), int(host[w])
        recv_rows = host[w + 1: 2 * w + 1].tolist()
        local_bytes = int(host[2 * w + 1])
        n_remote = n - n_local
        req = all_to_all_rows(send_keys[:n_remote], send_rows, recv_rows, self.group)

        # owner side: probe my shard for everything I received
        lk = self.shard.lookup(req, now)
        m = req.shape[0]
        rc = torch.tensor(recv_rows, dtype=torch.int64, device=self.device)
        reply_bytes = segment_sums(lk.off, rc)                   # bytes I send back per source
        got_bytes = exchange_counts(reply_bytes, self.group)     # bytes I receive per owner
        nbytes = torch.cat([reply_bytes, got_bytes]).cpu()       # sync 2
        send_b, recv_b = nbytes[:w].tolist(), nbytes[w:].tolist()
        reply = torch.empty(max(int(sum(send_b)), 16), dtype=torch.uint8, device=self.device)
        self.shard.gather(lk, reply)
        sizes_back = all_to_all_rows(lk.size[:m], recv_rows, send_rows, self.group)
        # response buffer: [local replica hits | remote values]
        data = torch.empty(local_bytes + int(sum(recv_b)) + 16, dtype=torch.uint8,
                           device=self.device)
        if rl is not None and n_local:
            self.replica.gather(rl, data)
        all_to_all_single(data[local_bytes: local_bytes + int(sum(recv_b))],
                               reply[: int(sum(send_b))], output_split_sizes=recv_b,
                               input_split_sizes=send_b, group=self.group)
        # requester side: remote sizes arrive in grouped (perm) order
        goff = R.exclusive_scan(sizes_back)
        pos = torch.clamp(perm, max=max(n_remote - 1, 0))
        if n_remote:
            rsize = sizes_back.index_select(0, pos)
            roff = goff.index_select(0, pos) + local_bytes
        else:
            rsize = torch.zeros(n, dtype=torch.int64, device=self.device)
            roff = torch.zeros(n, dtype=torch.int64, device=self.device)
        if rl is not None:
            local = rl.size[:n] > 0
            size = torch.where(local, rl.size[:n], rsize)
            off = torch.where(local, rl.off[:n], roff)
        else:
            size, off = rsize, roff
        self._stats["remote_gets"] += n_remote - int(send_rows[self.rank])
        self._stats["replica_hits"] += n_local
        return GetResult(data, off, size)

    def serve(self, keys: torch.Tensor, batch: SetBatch, now: Optional[int] = None,
              inputs_ready=None, probe_keys: Optional[torch.Tensor] = None) -> GetResult:
        """One serving step: a GET batch and a SET batch, GETs ordered before SETs.

        ``inputs_ready`` (optional ``torch.cuda.Event``, routed GPU step): an event after
        which ``keys`` and ``batch`` are complete. The step's planning then starts as soon
        as the previous step's owner side allows, beside its reply gather, instead of after
        everything the caller queued on the current stream before this call.

        With one rank the GET's extent read (the only host sync) is hidden behind
        ``probe_keys`` / ``batch.probe_keys`` (simulated world, routed GPU step only): the
        digests owners probe and store (bench.py --simulate-world maps every key onto one
        the simulated rank owns, so its shard holds 1/N of the key space like a real one).

        the SET kernels: the lookup reserves the SET's log bytes (objects the SET may
        overwrite count as misses) and its kernel writes the total into a pinned host
        slot; the SET is queued, and only then does the host spin on that slot to size
        the gather (no event, no copy).
        With several ranks see ``_serve_routed``: 4-5 collectives and 2 host syncs for
        the whole step instead of 10 and 3 for get() followed by set()."""
        self._touch(batch.keys)
        if self.routed:
            if self.fused and self.device.type == "cuda":
                return self._serve_routed_fused(keys, batch, now, inputs_ready, probe_keys)
            return self._serve_routed(keys, batch, now)
        n = keys.shape[0]
        self._stats["get_requests"] += n
        self._stats["set_requests"] += batch.keys.shape[0]
        sh = self.shard
        bound = sh.set_bound(batch.keys.shape[0], batch.values.numel())
        if not sh.is_gpu:
            lk = sh.lookup(keys, now, reserve_bytes=bound)
            sh.store(batch.keys, batch.values, batch.val_off, batch.vlen, batch.flags,
                     batch.expire, now)
            data = sh.gather(lk)
            return GetResult(data, lk.off[:n], lk.size[:n])
        side = self._side_stream() if self.overlap_store else None
        stage = self.host_edge and self.host_edge_dma and keys.device.type == "cpu"
        if stage:
            # host edge: the GET digests into HBM by DMA on this stream (the lookup reads
            # them from HBM instead of across PCIe); the SET batch likewise on the stream
            # that first reads it, below
            t = self._stage_turn = 1 - getattr(self, "_stage_turn", 1)
            keys = self._staged(t, "keys", keys)

        def staged_batch(b):
            if not stage:
                return b
            return SetBatch(*(self._staged(t, f"s{i}", x) for i, x in enumerate(
                (b.keys, b.values, b.val_off, b.vlen, b.flags, b.expire))))

        if side is None:
            lk, first, cslot, _ = self._lookup_step(keys, now, bound, None)
            sh.store(batch.keys, batch.values, batch.val_off, batch.vlen, batch.flags,
                     batch.expire, now)
            data = self._gather_unsynced(lk)
            expand(first, lk.size, lk.off)
            return GetResult(data, lk.off[:n], lk.size[:n], self._take_pending())
        # The SET chain runs beside the GET path. Streams: the caller's (main: lookup,
        # gather), the SET stream (side: dedupe, sizing, log append, index insert) and, with
        # hand="early", a hand stream (the CLOCK hand of a full cache). Ordering:
        #  * everything that reads the request batches waits for `ready` (inputs_ready, or
        #    the caller's stream as of this call);
        #  * the lookup waits for the previous step's SET chain (a step's GETs see the
        #    previous step's SETs, never this step's);
        #  * the log append waits for the previous step's gather (it overwrites the oldest
        #    region, which that gather may still read; the lookup reserved the SET's bytes,
        #    so this step's gather never reads them); the index insert waits for the lookup;
        #  * the early hand waits for the previous step's SET planning only (it reads the
        #    hand position, the claimed head and the ring the planning leaves) and runs beside
        #    that step's append, index insert and gather; its reinsertions are moves, so a
        #    SET that lands after it read the index makes them no-ops, never stale values.
        main = torch.cuda.current_stream(self.device)
        now = sh.now() if now is None else now
        if inputs_ready is None:
            ready = self._event("inputs")
            ready.record(main)
        else:
            ready = inputs_ready
        early = self.hand == "early"
        k = self._nserve = getattr(self, "_nserve", -1) + 1   # this step's event parity
        planned = self._event("planned") if early else None
        if early:
            # the hand and the planning of this batch, on the hand stream: after the
            # previous batch's planning (the stream's order) and the chain of the batch
            # before that (its SET workspace and hand buffer, which this batch reuses)
            hs = self._hand_stream()
            self._wait(hs, ready)
            if self._planned:
                if self._ends[k % 2] is not None:
                    self._wait(hs, self._ends[k % 2])
            else:
                # no serve pipeline to follow (first step, or other work since): the
                # caller's stream as of now, which has joined every earlier SET chain
                self._xwait(hs, main, "mainpos")
            with torch.cuda.stream(hs):
                batch = staged_batch(batch)
                sh.store(batch.keys, batch.values, batch.val_off, batch.vlen, batch.flags,
                         batch.expire, now, phase=1, plan_done=planned)
        stop = self.stop_events and self.event_fence != "system"
        if self._side_pending:
            self._wait(main, self._ends[(k - 1) % 2])   # the previous step's SET chain
            self._side_pending = False
        if stop and inputs_ready is None:
            # the append follows the previous step's gather (and everything else queued on
            # main before this call: `ready` marks it); the previous chain precedes it on
            # the side stream itself
            start = ready
        else:
            start = self._event("start")
            start.record(main)               # ... and its gather: the append may overwrite
        ev = self._event("probe")
        try:
            lk, first, cslot, table = self._lookup_step(keys, now, bound, side,
                                                        ev if stop else None)
        except BaseException:
            if early:
                # the planned batch still runs its chain (the native store pairs phase 1
                # with the next phase 2), after the previous gather like any append
                with torch.cuda.stream(side):
                    self._wait(side, planned)
                    sh.store(batch.keys, batch.values, batch.val_off, batch.vlen, batch.flags,
                             batch.expire, now, append_after=start, phase=2)
                self._end_step(side, k, batch, early)
            raise
        # Safe by construction: the lookup reserved the SET's log bytes, so the gather
        # never reads a region the SET writes, and the gather does not read the index.
        if first is not None:
            out_size = torch.empty(n, dtype=torch.int64, device=self.device)
            out_off = torch.empty(n, dtype=torch.int64, device=self.device)
        if not (stop and self._probe_stopped):
            ev.record(main)
        appended = self._event("appended") if self.gather_after_append else None
        with torch.cuda.stream(side):
            if early:
                self._wait(side, planned)    # (the plan followed `ready`)
            else:
                self._wait(side, ready)
                batch = staged_batch(batch)
            end = self._end_event(k) if stop else None
            sh.store(batch.keys, batch.values, batch.val_off, batch.vlen, batch.flags,
                     batch.expire, now, index_after=ev, append_after=start, append_done=appended,
                     phase=2 if early else 0, done=end)
        self._end_step(side, k, batch, early, recorded=end is not None)
        if appended is not None:
            # the gather runs after the log append, not beside it: the two byte movers
            # contending for HBM are slower together than one after the other
            self._wait(main, appended)
        # per-request (size, off) and the table clean-up: the gather's workgroups do them
        # after their copies (no launch, and nothing on the side stream for the next
        # step's lookup to wait for but the SET chain)
        data = self._gather_unsynced(
            lk, None if first is None else (first, out_size, out_off, table, cslot))
        if first is not None:
            return GetResult(data, out_off, out_size, self._take_pending())
        return GetResult(data, lk.off[:n], lk.size[:n], self._take_pending())

    def _end_event(self, k: int):
        """The end event of step parity ``k % 2`` (created on first use)."""
        e = self._ends[k % 2]
        if e is None:
            e = self._ends[k % 2] = (torch.cuda.Event() if self.event_fence == "system"
                                     else StreamEvent(self._fence_of("end")))
        return e

    def _fence_of(self, name: str) -> str:
        """Fence scope of a StreamEvent: the stop events' own for those a kernel completes."""
        return (self.stop_fence if self.stop_events and name in ("end", "probe")
                else self.event_fence)

    def _end_step(self, side, k: int, batch, early: bool, recorded: bool = False) -> None:
        """After a step's SET chain is queued: its end event (the next step's lookup and the
        step after next's hand wait for it; ``recorded``: the chain's last kernel already
        completes it), the batch kept alive until the chain is joined (the next serve's
        lookup or sync_sets)."""
        e = self._end_event(k)
        if not recorded:
            e.record(side)
        self._last_end = e
        self._side_pending = True
        held = self._held_steps
        held.append(batch)
        while len(held) > 2:   # the chain of two steps back is joined by now
            held.pop(0)
        self._planned = early

    def _lookup_step(self, keys, now, bound, side, index_done=None):
        """The step's GET lookup (coalesced unless ``coalesce`` is off): (lookup, first,
        cslot, table). ``index_done`` (a StreamEvent): completed by the lookup's probe
        kernel when the coalescing lookup runs (``_probe_stopped`` says whether it did)."""
        sh = self.shard
        self._probe_stopped = False
        if self.coalesce:
            table = self._coalesce_table(keys.shape[0]) if side is not None else None
            # with the table (the step's path, whose gather carries the expand tail): block-
            # local offsets, no n-row offsets scan between the lookup and the gather
            lk, first, cslot = sh.lookup_coalesced(keys, now, reserve_bytes=bound, total_slot=0,
                                                   table=table, blocked=table is not None,
                                                   index_done=index_done)
            self._probe_stopped = index_done is not None and sh.is_gpu and keys.shape[0] > 0
            return lk, first, cslot, table
        return sh.lookup(keys, now, reserve_bytes=bound, total_slot=0), None, None, None

    @staticmethod
    def _wait(stream, ev) -> None:
        """``stream`` waits for a recorded event (a StreamEvent or a torch.cuda.Event)."""
        if isinstance(ev, StreamEvent):
            ev.wait(stream)
        else:
            stream.wait_event(ev)

    def _hand_stream(self):
        """The early CLOCK hand's stream: the executor's plan stream, a hardware queue of its
        own (reserve_step_streams), unused by the one-GPU step otherwise."""
        if self._hand_s is None:
            ss = [int(x) for x in _core().step_streams(self.device.index)]
            self._hand_s = torch.cuda.ExternalStream(ss[0], device=self.device)
        return self._hand_s

    def _event(self, name: str):
        e = self._events.get(name)
        if e is None:
            e = self._events[name] = (torch.cuda.Event() if self.event_fence == "system"
                                      else StreamEvent(self._fence_of(name)))
        return e

    def _xwait(self, waiter, signaler, name: str) -> None:
        """``waiter`` stream waits for the work queued so far on ``signaler``."""
        e = self._event(name)
        e.record(signaler)
        if isinstance(e, StreamEvent):
            e.wait(waiter)
        else:
            waiter.wait_event(e)

    def _coalesce_table(self, n: int) -> torch.Tensor:
        """Persistent, zeroed GET-coalescing table (every serve step leaves it zeroed:
        expand_out clears the slots its batch claimed). Coalescing the next batch
        under this step's gather on a third stream (two tables, ping-pong) was measured
        slower, 0.35 vs 0.30 ms/step: both passes compete for the same memory system."""
        slots = int(_core().coalesce_table_slots(n))
        t = self._co_table
        if t is None or t.numel() < slots:
            t = self._co_table = torch.zeros(slots, dtype=torch.int32, device=self.device)
        return t

    def _staged(self, turn: int, name: str, x: Optional[torch.Tensor]):
        """``x`` (pinned host) copied into a persistent HBM buffer of this turn by DMA on the
        current stream (which runs everything that reads the buffer, so the copy of turn t
        two steps later is ordered after those reads)."""
        if x is None:
            return None
        bufs = self._stage_bufs = getattr(self, "_stage_bufs", None) or [{}, {}]
        b = bufs[turn].get(name)
        if b is None or b.numel() < x.numel() or b.dtype != x.dtype:
            b = bufs[turn][name] = torch.empty(max(x.numel(), 1), dtype=x.dtype,
                                               device=self.device)
        d = b[: x.numel()].view(x.shape)
        d.copy_(x, non_blocking=True)
        return d

    def _take_pending(self):
        p, self._last_pending = self._last_pending, None
        return p

    def _gather_unsynced(self, lk, expand=None) -> torch.Tensor:
        """Gather a lookup given ``total_slot=0`` without stalling the GPU: the gather
        is queued at once into a buffer sized from earlier steps (the kernel writes
        nothing if the total exceeds it) and the host reads the kernel-written total
        while the gather runs; only an outgrown buffer costs a second gather."""
        if self.host_edge and self.host_edge_dma and self.device.type == "cuda":
            return self._gather_dma(lk, expand)
        sh = self.shard
        cap = self._gather_cap
        if cap:
            data = self._out_buffer(cap)
            sh.gather(lk, data, out_cap=cap, expand=expand)
        total = sh.host_total(0)
        self.gathered_bytes += total
        if cap and total <= cap:
            return data
        self._gather_cap = max(int(total * 1.25), 1 << 20) // 16 * 16
        # (the expand tail ran with the first gather too: it is idempotent)
        return sh.gather(lk, self._out_buffer(max(total, 16)), expand=expand)

    def _gather_dma(self, lk, expand=None) -> torch.Tensor:
        """Host edge: gather into an HBM staging buffer, then copy [0, total) to the pinned
        host buffer on a copy stream (a DMA engine; the next step's kernels run beside it).
        Two turns: the gather of step k+2 waits for the copy of step k out of its staging
        buffer. The result's ``wait()`` blocks the host until its copy is done."""
        sh = self.shard
        main = torch.cuda.current_stream(self.device)
        k = self._host_turn = 1 - getattr(self, "_host_turn", 1)
        cap = self._gather_cap or (64 << 20)
        stg, done = self._dma[k] if self._dma[k] is not None else (None, None)
        if done is not None:
            main.wait_event(done)  # that turn's copy has read its staging buffer
        if stg is None or stg.numel() < cap:
            stg = torch.empty(cap, dtype=torch.uint8, device=self.device)
        sh.gather(lk, stg, out_cap=cap, expand=expand)
        total = sh.host_total(0)
        self.gathered_bytes += total
        if total > cap:
            self._gather_cap = max(int(total * 1.25), 1 << 20) // 16 * 16
            stg = torch.empty(self._gather_cap, dtype=torch.uint8, device=self.device)
            sh.gather(lk, stg, out_cap=self._gather_cap, expand=expand)
        elif not self._gather_cap:
            self._gather_cap = cap
        n = max(total, 16)
        bufs = getattr(self, "_host_out", None) or [None, None]
        self._host_out = bufs
        if bufs[k] is None or bufs[k].numel() < n:
            bufs[k] = torch.empty(max(n, self._gather_cap), dtype=torch.uint8, pin_memory=True)
        host = bufs[k][:n]
        if self._copy_stream is None:
            self._copy_stream = torch.cuda.Stream(device=self.device)
        cs = self._copy_stream
        gathered = torch.cuda.Event()
        gathered.record(main)
        cs.wait_event(gathered)
        with torch.cuda.stream(cs):
            host.copy_(stg[:n], non_blocking=True)
        done = torch.cuda.Event()
        done.record(cs)
        self._dma[k] = (stg, done)
        self._last_pending = _HostCopy(done)
        return host

    def _out_buffer(self, nbytes: int) -> torch.Tensor:
        if self.host_edge:
            # pinned host memory the gather kernel writes over PCIe; two buffers taken in
            # turn, so a step's response stays valid while the next step runs
            bufs = getattr(self, "_host_out", None) or [None, None]
            self._host_out = bufs
            k = self._host_turn = 1 - getattr(self, "_host_turn", 1)
            if bufs[k] is None or bufs[k].numel() < nbytes:
                bufs[k] = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
            return bufs[k][:nbytes]
        return torch.empty(nbytes, dtype=torch.uint8, device=self.device)

    def _side_stream(self):
        """The one-GPU step's SET stream: the executor's SET stream, a hardware queue of its
        own (reserve_step_streams), so nothing queues behind the caller's gather."""
        if self.device.type != "cuda":
            return None
        if self._side is None:
            # (a high-priority side stream measured the same: 0.3156 vs 0.3161 ms/step)
            ss = [int(x) for x in _core().step_streams(self.device.index)]
            self._side = torch.cuda.ExternalStream(ss[1], device=self.device)
        return self._side

    def _serve_routed_fused(self, keys: torch.Tensor, batch: SetBatch,
                            now: Optional[int] = None, inputs_ready=None,
                            probe_keys: Optional[torch.Tensor] = None) -> GetResult:
        """``_serve_routed`` run by the native executor (csrc/router.hip, RoutedStep), with
        no host synchronisation between planning and the result (after one calibrating
        step): GET requests and replies travel in fixed-capacity per-peer slots whose
        counts and (size, offset) headers ride in-band, so the all-to-alls need no split
        sizes from the device; capacities every rank agrees on come from the demand the
        ranks all-gathered in earlier steps, and a row that does not fit is a counted
        miss. SETs travel with exact sizes the host reads mid-step, while the GPU is busy
        with the GET exchange queued before. Same results as the framework-op version
        (tests); the reply transfer and the per-request assembly finish on a side stream
        (``GetResult.wait()``), under the next step's planning."""
        c = _core()
        dev, w, me = self.device, self.world, self.rank
        cur = torch.cuda.current_stream(dev)
        st = cur.cuda_stream
        i64, u8 = torch.int64, torch.uint8
        n = keys.shape[0]
        ns_in = batch.keys.shape[0]
        self._stats["get_requests"] += n
        self._stats["set_requests"] += ns_in
        self._sample(keys)
        now = self.shard.now() if now is None else now
        e = self._engine
        if e is None:
            e = self._engine = c.RoutedStep(w, me, dev.index)
            e.single_comm = self.comm_mode == "single"
            k = e.row_words
            self._row = torch.zeros(k, dtype=i64, device=dev)
            self._mat = torch.zeros(w * k, dtype=i64, device=dev)
            # the executor's process-wide streams (plan, SET side, reply + assembly): the
            # multi-call path uses the same ones, so a process keeps to four streams, one
            # hardware queue each (4 per process, taken round robin)
            ss = [int(x) for x in c.step_streams(dev.index)]
            self._sset = torch.cuda.ExternalStream(ss[1], device=dev)
            self._asm = torch.cuda.ExternalStream(ss[2], device=dev)
        e.set_ring(self.ring_pts.data_ptr(), self.ring_own.data_ptr(), self.ring_pts.numel())
        e.set_probe_keys(probe_keys.data_ptr() if probe_keys is not None else 0,
                         batch.probe_keys.data_ptr() if batch.probe_keys is not None else 0)
        fanout = self.replica is not None and self._hot is not None
        changed = False
        if fanout and self._hot_dir is None:
            self._hot_dir = _hot_directory(self._hot)
            changed = True  # a new hot set: the executor rebuilds its hash set
        e.set_hot(self._hot.data_ptr() if fanout else 0, self._hot.shape[0] if fanout else 0,
                  self._hot_dir.data_ptr() if fanout else 0, changed)
        rep = self.replica._impl if self.replica is not None else None
        while len(self._inflight) >= 2:
            ev, _bufs = self._inflight.pop(0)
            cur.wait_event(ev)  # long complete: frees the buffers for reuse on this stream
        cap_g, cap_d, cap_l, cal, cal_l = e.prepare(n)
        if self._ncomm is None:
            self._ncomm = step_comm(self.group, dev) or False
            if self._ncomm is not False:
                e.set_comm(self._ncomm)
        # the path must be the same on every rank: `cal` is (every rank derives it from the
        # same all-gathered rows), `cal_l` is per rank (its own local-region history)
        if self._ncomm is not False and not cal:
            return self._serve_native(e, keys, batch, now, n, ns_in, cap_g, cap_d, cap_l,
                                      fanout, rep, inputs_ready)
        self._calibrations = getattr(self, "_calibrations", 0) + 1  # (the multi-call path)
        ph = _Phases("serve.")
        ph.next("plan")
        # G = [recv: w-1 slots | self slot | send: w-1 slots] of cap_g digests
        gslot = 16 * cap_g
        G = torch.empty((2 * w - 1) * gslot, dtype=u8, device=dev)
        e.plan(keys.data_ptr(), n, rep, now, batch.keys.data_ptr(), batch.vlen.data_ptr(),
               batch.flags.data_ptr() if batch.flags is not None else 0,
               batch.expire.data_ptr() if batch.expire is not None else 0,
               batch.val_off.data_ptr(), batch.values.data_ptr(), ns_in, fanout,
               G.data_ptr(), self._row.data_ptr(), st, self.coalesce)
        ph.next("row_allgather")
        all_gather_rows(self._mat, self._row, self.group, peer_blocks=4)
        e.publish(self._mat.data_ptr(), st)
        if cal_l:
            e.calibrate_local()                                   # calibration: host read
        ph.next("request_a2a")
        if w > 1:
            sp = [0 if p == me else gslot for p in range(w)]
            all_to_all_single(G[: (w - 1) * gslot], G[w * gslot:], output_split_sizes=sp,
                              input_split_sizes=sp, group=self.group)
        ph.next("owner")
        e.owner_probe(G.data_ptr(), self.shard._impl, now, st)
        # the SET stream forks here: the probe reserved this step's SET bytes, so the SET
        # exchange and the main-shard SET chain run beside the reply gather
        sset = self._sset
        self._xwait(sset, cur, "routed_probe")
        if cal:
            dem = torch.empty(w, dtype=i64, device=dev)
            e.owner_demand(dem.data_ptr(), st)
            dmat = torch.empty(w * w, dtype=i64, device=dev)
            all_gather_rows(dmat, dem, self.group, peer_blocks=1)
            e.calibrate_reply(dmat.data_ptr())                    # calibration: host read
        if cal or cal_l:
            cap_g, cap_d, cap_l = e.caps(n)[:3]
        slot_r = 8 * cap_g + cap_d
        # the response buffer: [local capL | w-1 reply slots (recv) | self reply slot]
        R = torch.empty(max((w - 1) * slot_r, 16), dtype=u8, device=dev)
        data = torch.empty(cap_l + w * slot_r + 16, dtype=u8, device=dev)
        e.owner_reply(self.shard._impl, R.data_ptr(), data.data_ptr(), st)
        work = None
        if w > 1:
            sp = [0 if p == me else slot_r for p in range(w)]
            work = all_to_all_single(data[cap_l: cap_l + (w - 1) * slot_r], R[: (w - 1) * slot_r],
                                     output_split_sizes=sp, input_split_sizes=sp,
                                     group=self.data_group, async_op=True)
        e.gather_local(data.data_ptr(), st)
        local_done = torch.cuda.Event()
        local_done.record(cur)
        ph.next("set_exchange")
        h = e.set_splits()           # waits for the published rows: the GPU is still busy
        send, recv = h[:w], h[w:2 * w]
        n_local, n_dup, off_rank, over, dropped = h[2 * w: 2 * w + 5]
        so, ro = sum(send) - send[me], sum(recv) - recv[me]
        # S: the other ranks' blocks only (own SETs are stored from the batch in place)
        S = torch.empty(so + 16, dtype=u8, device=dev)
        Rs = torch.empty(ro + 16, dtype=u8, device=dev)
        e.pack_sets(S.data_ptr(), sset.cuda_stream)
        if w > 1:
            with torch.cuda.stream(sset):
                all_to_all_single(Rs[:ro], S[:so],
                                  output_split_sizes=[0 if q == me else recv[q] for q in range(w)],
                                  input_split_sizes=[0 if p == me else send[p] for p in range(w)],
                                  group=self.group)
        e.store_sets(Rs.data_ptr(), self.shard._impl, rep, now, st, sset.cuda_stream)
        # the main-shard SET chain reads S / Rs and the batch until the next step's owner
        # probe joins it
        self._held = (S, Rs, batch) if e.sets_pending else None
        ph.next("assemble")
        out = torch.empty((2, n), dtype=i64, device=dev)
        side = self._asm
        side.wait_event(local_done)
        with torch.cuda.stream(side):
            if work is not None:
                work.wait()          # the side stream waits for the reply all-to-all
            e.assemble(data.data_ptr(), out[0].data_ptr(), out[1].data_ptr(), side.cuda_stream)
        data.record_stream(side)
        out.record_stream(side)
        done = torch.cuda.Event()
        done.record(side)
        self._inflight.append((done, (R, data)))
        self._add_step_stats((n_local, n_dup, off_rank, over, dropped))
        self._add_step_stats(e.take_stats())  # earlier native steps' (lagged)
        ph.end()
        return GetResult(data, out[1], out[0], _pending=_StreamDone(done))

    def _serve_native(self, e, keys, batch, now, n, ns_in, cap_g, cap_d, cap_l, fanout, rep,
                      inputs_ready=None):
        """The routed step as one native call (``RoutedStep.step``): every kernel launch
        and collective of the step is issued from C++, none from Python; only the response
        buffers are torch tensors (the caller keeps them). Calibrating steps take the
        multi-call path in ``_serve_routed_fused``."""
        dev, w = self.device, self.world
        cur = torch.cuda.current_stream(dev)
        slot_r = 8 * cap_g + cap_d
        data = torch.empty(cap_l + w * slot_r + 16, dtype=torch.uint8, device=dev)
        out = torch.empty((2, n), dtype=torch.int64, device=dev)
        # the reply transfer and the assembly run on the executor's assembly stream (one
        # per device for the process, never destroyed, so tensors recorded on it are safe)
        side = self._asm
        h = e.step(keys.data_ptr(), n, rep, now, batch.keys.data_ptr(), batch.vlen.data_ptr(),
                   batch.flags.data_ptr() if batch.flags is not None else 0,
                   batch.expire.data_ptr() if batch.expire is not None else 0,
                   batch.val_off.data_ptr(), batch.values.data_ptr(), ns_in, fanout,
                   self.coalesce, self.shard._impl, data.data_ptr(), out[0].data_ptr(),
                   out[1].data_ptr(), cur.cuda_stream, 0, 0,
                   _event_handle(inputs_ready), batch.values.numel())
        # the reply transfer and the assembly (both on `side`) and the local gather (SET
        # stream, awaited by the assembly) write and read these
        data.record_stream(side)
        out.record_stream(side)
        done = torch.cuda.Event()
        done.record(side)
        self._inflight.append((done, (data,)))
        # the main-shard SET chain (the executor's SET stream, a hardware queue of its own)
        # reads the batch until the next step's probe joins it
        self._held = (batch,) if e.sets_pending else None
        # statistics of the steps two back (the host never waits for this step's matrix)
        self._add_step_stats(h)
        return GetResult(data, out[1], out[0], _pending=_StreamDone(done))

    def _set_rows(self, batch: SetBatch):
        """Routing of a SET batch: (dest int32 [m], records int64 [m, 4], val_off [m]).
        A record is [digest lo, digest hi, vlen | flags << 32, expire | tier << 32];
        hot keys are fanned out to every rank (tier 1 = replica copy); dest == world
        marks rows that go nowhere."""
        dev, w, n = self.device, self.world, batch.keys.shape[0]
        owner, _ = self._route(batch.keys)
        meta = torch.zeros((n, 4), dtype=torch.int32, device=dev)
        meta[:, 0] = batch.vlen
        if batch.flags is not None:
            meta[:, 1] = batch.flags
        if batch.expire is not None:
            meta[:, 2] = batch.expire
        if self.replica is not None and self._hot is not None:
            hot = self._is_hot(batch.keys)
            r = torch.arange(w, device=dev, dtype=torch.int32).view(1, w)
            own = owner.view(n, 1)
            valid = (r == own) | hot.view(n, 1)
            dest = torch.where(valid, r.expand(n, w), torch.full((n, w), w, dtype=torch.int32,
                                                                 device=dev)).reshape(-1)
            keys = batch.keys.repeat_interleave(w, dim=0)
            meta = meta.repeat_interleave(w, dim=0)
            meta[:, 3] = (r != own).reshape(-1).to(torch.int32)
            val_off = batch.val_off.repeat_interleave(w)
        else:
            dest, keys, val_off = owner, batch.keys, batch.val_off
        rec = torch.cat([keys, meta.view(torch.int64)], dim=1)
        return dest, rec, val_off

    def _serve_routed(self, keys: torch.Tensor, batch: SetBatch,
                      now: Optional[int] = None) -> GetResult:
        """GET + SET step over all ranks with one request exchange and one reply exchange.

          1. route GETs (replica hits stay local) and SETs on the device; ONE tiny
             all-to-all of per-peer [get rows, set rows, set value bytes]; host sync 1.
          2. ONE all-to-all carries, per peer, [GET digests | SET records | SET values],
             assembled by a single gather_segments launch from three tensors.
          3. owner: de-interleave, lookup; all-to-all of reply sizes; host sync 2.
          4. owner gathers replies straight into the send buffer; the value all-to-all
             runs asynchronously while the SET stores and the local replica gather run
             on the compute stream (GETs of this step see the state before its SETs).
        """
        dev, w, me = self.device, self.world, self.rank
        n = keys.shape[0]
        self._stats["get_requests"] += n
        self._stats["set_requests"] += batch.keys.shape[0]
        self._sample(keys)
        i64 = torch.int64
        ph = _Phases("serve.")
        # ---- 1. routing + count exchange
        ph.next("route")
        dest_g, _ = self._route(keys)
        rl = None
        if self.replica is not None:
            rl = self.replica.lookup(keys, now)
            dest_g = torch.where(rl.size[:n] > 0, torch.full_like(dest_g, w), dest_g)
        cnt_g = torch.bincount(dest_g.long(), minlength=w + 1)
        perm_g = R.scatter_positions(dest_g, cnt_g)
        gk = R.permute(keys, perm_g)
        dest_s, rec, val_off = self._set_rows(batch)
        m = rec.shape[0]
        cnt_s = torch.bincount(dest_s.long(), minlength=w + 1)
        perm_s = R.scatter_positions(dest_s, cnt_s)
        srec = R.permute(rec, perm_s)
        sval = R.permute(val_off.view(-1, 1), perm_s).view(-1)
        vlen = srec[:, 2] & 0xFFFFFFFF
        vlen = torch.where(vlen >= 0x80000000, torch.zeros_like(vlen), vlen)  # skip rows: no bytes
        padded = torch.where(torch.arange(m, device=dev) < m - cnt_s[w], (vlen + 15) & ~15,
                             torch.zeros_like(vlen))
        vscan = R.exclusive_scan(padded)
        vb = segment_sums(vscan, cnt_s[:w].contiguous())
        table = torch.stack([cnt_g[:w], cnt_s[:w], vb], dim=1).contiguous()
        ph.next("count_exchange")
        rtable = torch.empty_like(table)
        all_to_all_single(rtable, table, group=self.group)
        ltot = rl.off[n:n + 1] if rl is not None else torch.zeros(1, dtype=i64, device=dev)
        host = torch.cat([table.view(-1), rtable.view(-1), cnt_g[w:w + 1], ltot]).cpu()  # sync 1
        t = host[: 3 * w].view(w, 3).tolist()
        rt = host[3 * w: 6 * w].view(w, 3).tolist()
        n_local, local_bytes = int(host[6 * w]), int(host[6 * w + 1])
        g_rows = [r[0] for r in t]
        s_rows = [r[1] for r in t]
        rg_rows = [r[0] for r in rt]
        rs_rows = [r[1] for r in rt]
        send_b = [16 * a + 32 * b + c for a, b, c in t]
        recv_b = [16 * a + 32 * b + c for a, b, c in rt]
        ns = sum(s_rows)

        # ---- 2. request exchange: per peer [G | R | V]
        ph.next("pack_requests")
        g_start = [0] * w
        s_start = [0] * w
        for p in range(1, w):
            g_start[p] = g_start[p - 1] + g_rows[p - 1]
            s_start[p] = s_start[p - 1] + s_rows[p - 1]
        nseg = 2 * w + ns
        seg_len = torch.empty(nseg, dtype=i64, device=dev)
        seg_src = torch.empty(nseg, dtype=i64, device=dev)
        hdr_idx, hdr_len, hdr_src = [], [], []
        for p in range(w):
            hdr_idx += [2 * p + s_start[p], 2 * p + 1 + s_start[p]]
            hdr_len += [16 * g_rows[p], 32 * s_rows[p]]
            hdr_src += [gk.data_ptr() + 16 * g_start[p], srec.data_ptr() + 32 * s_start[p]]
        hdr = torch.tensor([hdr_idx, hdr_len, hdr_src], dtype=i64).to(dev, non_blocking=True)
        seg_len.index_copy_(0, hdr[0], hdr[1])
        seg_src.index_copy_(0, hdr[0], hdr[2])
        if ns:
            peer = torch.repeat_interleave(torch.arange(w, device=dev), cnt_s[:w],
                                           output_size=ns)
            vidx = torch.arange(ns, device=dev) + 2 * peer + 2
            seg_len.index_copy_(0, vidx, padded[:ns])
            seg_src.index_copy_(0, vidx, sval[:ns] + batch.values.data_ptr())
        send = torch.empty(sum(send_b) + 16, dtype=torch.uint8, device=dev)
        R.gather_segments(seg_src, R.exclusive_scan(seg_len), send)
        recv = torch.empty(sum(recv_b) + 16, dtype=torch.uint8, device=dev)
        ph.next("request_a2a")
        all_to_all_single(recv[: sum(recv_b)], send[: sum(send_b)],
                               output_split_sizes=recv_b, input_split_sizes=send_b,
                               group=self.group)

        # ---- 3. owner: de-interleave digests and records, probe
        ph.next("owner_lookup")
        mg, ms = sum(rg_rows), sum(rs_rows)
        body = torch.empty(16 * mg + 32 * ms + 16, dtype=torch.uint8, device=dev)
        src_l, len_l = [], []
        q0 = 0
        blocks_g, blocks_r = [], []
        for q in range(w):
            blocks_g.append((recv.data_ptr() + q0, 16 * rg_rows[q]))
            blocks_r.append((recv.data_ptr() + q0 + 16 * rg_rows[q], 32 * rs_rows[q]))
            q0 += recv_b[q]
        for a, l in blocks_g + blocks_r:
            src_l.append(a)
            len_l.append(l)
        dl = torch.tensor([src_l, len_l], dtype=i64).to(dev, non_blocking=True)
        R.gather_segments(dl[0].contiguous(), R.exclusive_scan(dl[1]), body)
        req = body[: 16 * mg].view(i64).view(mg, 2)
        rrec = body[16 * mg: 16 * mg + 32 * ms].view(i64).view(ms, 4)
        lk = self.shard.lookup(req, now)
        rcv = torch.tensor(rg_rows, dtype=i64).to(dev, non_blocking=True)
        reply_bytes = segment_sums(lk.off, rcv)
        sizes_back = all_to_all_rows(lk.size[:mg], rg_rows, g_rows, self.group)
        n_remote = n - n_local
        gscan = R.exclusive_scan(sizes_back)
        got_bytes = segment_sums(gscan, torch.tensor(g_rows, dtype=i64).to(dev, non_blocking=True))
        ph.next("reply_sizes")
        nb = torch.cat([reply_bytes, got_bytes]).cpu()                    # sync 2
        rep_b, got_b = nb[:w].tolist(), nb[w:].tolist()

        # ---- 4. replies (async) overlapped with SET stores and the replica gather
        ph.next("reply_a2a+set_store")
        reply = torch.empty(max(sum(rep_b), 16), dtype=torch.uint8, device=dev)
        self.shard.gather(lk, reply)
        data = torch.empty(local_bytes + sum(got_b) + 16, dtype=torch.uint8, device=dev)
        work = all_to_all_single(data[local_bytes: local_bytes + sum(got_b)],
                                      reply[: sum(rep_b)], output_split_sizes=got_b,
                                      input_split_sizes=rep_b, group=self.group, async_op=True)
        if rl is not None and n_local:
            self.replica.gather(rl, data)
        if ms:
            meta = rrec[:, 2:].contiguous().view(torch.int32).view(ms, 4)
            rvlen = meta[:, 0].contiguous()
            tier = meta[:, 3]
            # value offsets inside `recv`: source block start + scan within the block
            vpad = (rvlen.to(i64) + 15) & ~15
            vs = R.exclusive_scan(vpad)
            vstart, r0, q0 = [], 0, 0
            for q in range(w):
                vstart.append(q0 + 16 * rg_rows[q] + 32 * rs_rows[q])
                q0 += recv_b[q]
            rs_t = torch.tensor(rs_rows, dtype=i64).to(dev, non_blocking=True)
            first = torch.cumsum(rs_t, 0) - rs_t
            delta = torch.tensor(vstart, dtype=i64).to(dev, non_blocking=True) - \
                vs.index_select(0, first)
            roff = (vs[:ms] + torch.repeat_interleave(delta, rs_t, output_size=ms)).contiguous()
            skip = torch.full_like(rvlen, SKIP_VLEN)
            rkeys = rrec[:, :2].contiguous()
            self.shard.store(rkeys, recv, roff, torch.where(tier == 0, rvlen, skip).contiguous(),
                             meta[:, 1].contiguous(), meta[:, 2].contiguous(), now)
            if self.replica is not None:
                self.replica.store(rkeys, recv, roff,
                                   torch.where(tier == 1, rvlen, skip).contiguous(),
                                   meta[:, 1].contiguous(), meta[:, 2].contiguous(), now)
        work.wait()

        # ---- requester: response offsets in request order
        ph.next("assemble")
        if n_remote:
            pos = torch.clamp(perm_g, max=n_remote - 1)
            rsize = sizes_back.index_select(0, pos)
            roff_g = gscan.index_select(0, pos) + local_bytes
        else:
            rsize = torch.zeros(n, dtype=i64, device=dev)
            roff_g = torch.zeros(n, dtype=i64, device=dev)
        if rl is not None:
            local = rl.size[:n] > 0
            size = torch.where(local, rl.size[:n], rsize)
            off = torch.where(local, rl.off[:n], roff_g)
        else:
            size, off = rsize, roff_g
        self._stats["remote_gets"] += n_remote - int(g_rows[me])
        self._stats["replica_hits"] += n_local
        ph.end()
        return GetResult(data, off, size)

    def set(self, batch: SetBatch, now: Optional[int] = None, if_absent: bool = False) -> None:
        """SET a batch (collective when routed). ``if_absent``: an owner stores a row only
        when it holds no live object of the key (a migration's delivery, which must never
        overwrite a newer value the owner received directly)."""
        self.sync_sets()
        if not if_absent:  # (a migration's own delivery is not a newer write)
            self._touch(batch.keys)
        n = batch.keys.shape[0]
        self._stats["set_requests"] += n
        if not self.routed:
            vlen = batch.vlen
            if if_absent and n:
                have = self.shard.lookup(batch.keys.contiguous(), now).size[:n] > 0
                vlen = torch.where(have, torch.full_like(vlen, SKIP_VLEN), vlen).contiguous()
            self.shard.store(batch.keys, batch.values, batch.val_off, vlen, batch.flags,
                             batch.expire, now)
            return
        dev, w = self.device, self.world
        owner, _ = self._route(batch.keys)
        # metadata records [vlen, flags, expire, tier] as int32x4 (16 B); tier 1 = replica copy
        meta = torch.zeros((n, 4), dtype=torch.int32, device=dev)
        meta[:, 0] = batch.vlen
        if batch.flags is not None:
            meta[:, 1] = batch.flags
        if batch.expire is not None:
            meta[:, 2] = batch.expire
        if self.replica is not None and self._hot is not None:
            # write-through: a replicated key goes to its owner AND to every other rank
            hot = self._is_hot(batch.keys)
            r = torch.arange(w, device=dev, dtype=torch.int32).view(1, w)
            own = owner.view(n, 1)
            valid = (r == own) | hot.view(n, 1)
            dest = torch.where(valid, r.expand(n, w), torch.full((n, w), w, dtype=torch.int32,
                                                                 device=dev)).reshape(-1)
            keys = batch.keys.repeat_interleave(w, dim=0)
            meta = meta.repeat_interleave(w, dim=0)
            meta[:, 3] = (r != own).reshape(-1).to(torch.int32)
            val_off = batch.val_off.repeat_interleave(w)
        else:
            dest, keys, val_off = owner, batch.keys, batch.val_off
        counts = torch.bincount(dest.long(), minlength=w + 1)
        perm = R.scatter_positions(dest, counts)
        send_keys = R.permute(keys, perm)
        send_meta = R.permute(meta, perm)
        nvalid = keys.shape[0] - counts[w:w + 1]
        padded = (send_meta[:, 0].to(torch.int64) + 15) & ~15
        padded = torch.where(torch.arange(keys.shape[0], device=dev) < nvalid, padded,
                             torch.zeros_like(padded))
        dst_off = R.exclusive_scan(padded)
        src_off = R.permute(val_off.view(-1, 1), perm).view(-1)
        seg_bytes = segment_sums(dst_off, counts[:w].contiguous())
        recv_counts = exchange_counts(counts[:w].contiguous(), self.group)
        recv_bytes = exchange_counts(seg_bytes, self.group)
        host = torch.cat([counts[:w], recv_counts, seg_bytes, recv_bytes]).cpu()  # sync 1
        send_rows, recv_rows = host[:w].tolist(), host[w: 2 * w].tolist()
        send_b, recv_b = host[2 * w: 3 * w].tolist(), host[3 * w:].tolist()
        ns = int(sum(send_rows))
        payload = torch.empty(int(sum(send_b)) + 16, dtype=torch.uint8, device=dev)
        R.segcopy(batch.values, src_off[:ns].contiguous(), dst_off[: ns + 1].contiguous(), payload)
        rkeys = all_to_all_rows(send_keys[:ns], send_rows, recv_rows, self.group)
        rmeta = all_to_all_rows(send_meta[:ns], send_rows, recv_rows, self.group)
        rvals = torch.empty(int(sum(recv_b)) + 16, dtype=torch.uint8, device=dev)
        all_to_all_single(rvals[: int(sum(recv_b))], payload[: int(sum(send_b))],
                               output_split_sizes=recv_b, input_split_sizes=send_b,
                               group=self.group)
        rvlen = rmeta[:, 0].contiguous()
        roff = R.exclusive_scan((rvlen.to(torch.int64) + 15) & ~15)[:-1].contiguous()
        tier = rmeta[:, 3]
        skip = torch.full_like(rvlen, SKIP_VLEN)
        main_vlen = torch.where(tier == 0, rvlen, skip)
        if if_absent and rkeys.shape[0]:
            # insert-if-absent (as HbmBackend's warm restore): keys this owner already holds
            # keep their (newer) value
            have = self.shard.lookup(rkeys.contiguous(), now).size[: rkeys.shape[0]] > 0
            main_vlen = torch.where(have, skip, main_vlen)
        self.shard.store(rkeys, rvals, roff, main_vlen.contiguous(),
                         rmeta[:, 1].contiguous(), rmeta[:, 2].contiguous(), now)
        if self.replica is not None and self._hot is not None:  # tier-1 rows only exist then
            self.replica.store(rkeys, rvals, roff, torch.where(tier == 1, rvlen, skip).contiguous(),
                               rmeta[:, 1].contiguous(), rmeta[:, 2].contiguous(), now)

    def delete(self, keys: torch.Tensor, now: Optional[int] = None) -> torch.Tensor:
        self.sync_sets()
        self._touch(keys)
        if not self.routed:
            return self.shard.remove(keys, now)
        if self.replica is not None:  # replicas are dropped everywhere (collective)
            cnt = torch.tensor([keys.shape[0]], dtype=torch.int64, device=self.device)
            all_reduce(cnt, op=dist.ReduceOp.MAX, group=self.group)
            pad = torch.zeros((int(cnt), 2), dtype=keys.dtype, device=self.device)
            pad[: keys.shape[0]] = keys
            allk = [torch.empty_like(pad) for _ in range(self.world)]
            all_gather(allk, pad, group=self.group)
            self.replica.remove(torch.cat(allk).contiguous(), now)
        dest, counts = self._route(keys)
        perm = R.scatter_positions(dest, counts)
        send_keys = R.permute(keys, perm)
        recv_counts = exchange_counts(counts, self.group)
        both = torch.cat([counts, recv_counts]).cpu()
        send_rows, recv_rows = both[: self.world].tolist(), both[self.world:].tolist()
        req = all_to_all_rows(send_keys, send_rows, recv_rows, self.group)
        found = self.shard.remove(req, now).to(torch.int32)
        back = all_to_all_rows(found, recv_rows, send_rows, self.group)
        return back.index_select(0, perm).bool()

    # ------------------------------------------------------------------------------
    def _hot_candidates(self, top_k: int, keys: Optional[torch.Tensor],
                        old: Optional[torch.Tensor] = None,
                        old_score: Optional[torch.Tensor] = None):
        """Collective: the global top-k digests by request count (from ``keys`` or the
        recent GET samples), the same on every rank, most requested first (ties in digest
        order: stable sorts of all-gathered / all-reduced counts, identical everywhere),
        and their scores. With the current hot set ``old`` (sorted by lo) and its scores
        from the last refresh, an old key scores decay * its old score + its requests now
        + 1 (hysteresis): the tail of a large hot set is seen a few times per sample at
        most, so a key only displaces a hot one when it is seen more often — the hot set
        follows a drift instead of churning on sampling noise."""
        dev, w = self.device, self.world
        if keys is None:
            keys = torch.cat(self._samples) if self._samples else torch.zeros((0, 2), dtype=torch.int64,
                                                                             device=dev)
        # count by the low digest word (a 1-D sort; two keys sharing it are vanishingly rare)
        if keys.shape[0]:
            ulo, inv, cnt = torch.unique(keys[:, 0].contiguous(), return_inverse=True,
                                         return_counts=True)
            uniq = torch.empty((ulo.numel(), 2), dtype=torch.int64, device=dev)
            uniq[inv] = keys
        else:
            ulo = torch.zeros(0, dtype=torch.int64, device=dev)
            uniq = torch.zeros((0, 2), dtype=torch.int64, device=dev)
            cnt = torch.zeros(0, dtype=torch.int64, device=dev)
        k = min(top_k, uniq.shape[0])
        top = torch.topk(cnt, k).indices if k else cnt[:0]
        cand = torch.zeros((top_k, 2), dtype=torch.int64, device=dev)
        ccnt = torch.zeros(top_k, dtype=torch.int64, device=dev)
        cand[:k] = uniq.index_select(0, top)
        ccnt[:k] = cnt.index_select(0, top)
        all_c = [torch.empty_like(cand) for _ in range(w)]
        all_n = [torch.empty_like(ccnt) for _ in range(w)]
        all_gather(all_c, cand, group=self.group)
        all_gather(all_n, ccnt, group=self.group)
        allc = torch.cat(all_c)
        alln = torch.cat(all_n)
        # merge by the low word (a 1-D sort), in digest order: identical on every rank
        ulo2, inv = torch.unique(allc[:, 0].contiguous(), return_inverse=True)
        u = torch.empty((ulo2.numel(), 2), dtype=torch.int64, device=dev)
        u[inv] = allc
        tot = torch.zeros(u.shape[0], dtype=torch.int64, device=dev).scatter_add_(0, inv, alln)
        # a key enters the hot set only once seen twice (a mirrored world counts every
        # sighting once per simulated rank)
        min_count = 2 * (w if isinstance(self.group, MirrorComm) else 1)
        keep = ((u != 0).any(dim=1)) & (tot >= min_count)  # (drops the padding rows too)
        u, score = u[keep], tot[keep].to(torch.float64)
        if old is not None and old.shape[0]:
            # the old keys' requests in this sample, summed over the ranks
            oc = torch.zeros(old.shape[0], dtype=torch.int64, device=dev)
            if ulo.numel():
                at = torch.clamp(torch.searchsorted(ulo, old[:, 0].contiguous()), max=ulo.numel() - 1)
                oc = torch.where(ulo.index_select(0, at) == old[:, 0], cnt.index_select(0, at), oc)
            all_reduce(oc, group=self.group)
            prev = old_score if old_score is not None else torch.zeros(old.shape[0], dtype=torch.float64,
                                                                       device=dev)
            osc = prev * self.hot_decay + oc.to(torch.float64) + 1.0
            fresh = ~self._member(u, old)
            u = torch.cat([old, u[fresh]])
            score = torch.cat([osc, score[fresh]])
        # (with an old hot set every old key stays in the ranking: the caller picks the
        # top-k among the keys it could put in place)
        order = torch.sort(-score, stable=True).indices
        if old is None or old.shape[0] == 0:
            order = order[:top_k]
        return u.index_select(0, order).contiguous(), score.index_select(0, order).contiguous()

    @staticmethod
    def _member(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
        """Rows of ``a`` that are rows of ``b`` (both [n, 2] digests; b sorted by lo)."""
        if a.shape[0] == 0 or b.shape[0] == 0:
            return torch.zeros(a.shape[0], dtype=torch.bool, device=a.device)
        at = torch.searchsorted(b[:, 0].contiguous(), a[:, 0].contiguous())
        at = torch.clamp(at, max=b.shape[0] - 1)
        return (b.index_select(0, at) == a).all(dim=1)

    def _fetch_into_replica(self, keys: torch.Tensor, now: Optional[int]) -> tuple:
        """Collective. GET ``keys`` through their owners (never the replica) and store the
        records in this rank's replica (keys this rank owns stay out: an owner serves its
        own keys from its main shard). Returns (objects stored, record bytes fetched)."""
        if keys.shape[0] == 0:
            return 0, 0
        saved = self.replica
        self.replica = None                               # fetch through the owners only
        try:
            res = self.get(keys, now, probe_keys=self.probe_of(keys) if self.probe_of else None)
        finally:
            self.replica = saved
        sb = records_to_set_batch(keys, res)
        owner, _ = self._route(keys)
        sb.vlen = torch.where(owner == self.rank, torch.full_like(sb.vlen, SKIP_VLEN), sb.vlen)
        # store in chunks with exact byte bounds (the records buffer can be GBs)
        k = keys.shape[0]
        chunk = 1 << 17
        cuts = list(range(0, k, chunk)) + [k]
        # records of a chunk are scattered in the response buffer: bound by their sizes
        sizes = torch.stack([res.size[cuts[i]:cuts[i + 1]].sum()
                             for i in range(len(cuts) - 1)]).tolist()
        for i in range(len(cuts) - 1):
            a, b = cuts[i], cuts[i + 1]
            self.replica.store(sb.keys[a:b], sb.values, sb.val_off[a:b], sb.vlen[a:b],
                               sb.flags[a:b], sb.expire[a:b], now,
                               bytes_bound=int(sizes[i]) + 48 * (b - a))
        return int((sb.vlen != SKIP_VLEN).sum()), int(sum(sizes))

    def refresh_replica(self, top_k: int, keys: Optional[torch.Tensor] = None,
                        now: Optional[int] = None, budget_bytes: Optional[int] = None,
                        chunk_keys: int = 1 << 16) -> int:
        """Collective. Move the replica tier towards the global top-k keys by request
        frequency (from ``keys`` or the recent GET samples), incrementally: keys that left
        the top-k are deleted from the replica and stop being written through; keys that
        entered it are fetched from their owners, most popular first, until
        ``budget_bytes`` of records have moved (None: all of them) — the rest stay
        un-replicated (served by their owners) and are candidates again at the next
        refresh (fetched ``chunk_keys`` at a time: the budget's granularity). Nothing is
        flushed: the replica keeps serving the keys that stay hot. The hot set changes
        identically on every rank. Returns #objects this call stored."""
        self.sync_sets()
        if self.replica is None:
            return 0
        dev = self.device
        old = self._hot if self._hot is not None else torch.zeros((0, 2), dtype=torch.int64,
                                                                    device=dev)
        ranked, rscore = self._hot_candidates(top_k, keys, old, self._hot_score)  # hottest first
        if ranked.shape[0] == 0 and old.shape[0] == 0:
            return 0
        # newly hot keys (in the top k, not in place yet), most requested first, fetched in
        # chunks under the byte budget
        top = ranked[:top_k]
        added = top[~self._member(top, old)]
        stored = fetched = 0
        took = []
        chunk = max(1, int(chunk_keys))
        for a in range(0, added.shape[0], chunk):
            if budget_bytes is not None and fetched >= budget_bytes:
                break
            part = added[a: a + chunk].contiguous()
            n_st, nb = self._fetch_into_replica(part, now)
            stored += n_st
            fetched += nb
            took.append(part)
        # the new hot set: the top-k of the ranking among the keys that are in place (old
        # ones and the ones fetched now); an old key leaves only for a fetched hotter one
        avail = torch.cat([old] + took) if took else old
        avail = avail.index_select(0, torch.argsort(avail[:, 0])).contiguous()
        new = ranked[self._member(ranked, avail)][:top_k] if avail.shape[0] else avail
        nsorted = new.index_select(0, torch.argsort(new[:, 0])).contiguous()
        dropped = old[~self._member(old, nsorted)].contiguous()
        if dropped.shape[0]:
            self.replica.remove(dropped, now)             # no longer written through
        if new.shape[0] == 0:
            self._hot = self._hot_score = None
        else:
            self._hot = nsorted
            # the scores of the hot keys, aligned with self._hot (the next refresh decays them)
            by_lo = torch.argsort(ranked[:, 0])
            rlo = ranked[:, 0].index_select(0, by_lo).contiguous()
            at = torch.clamp(torch.searchsorted(rlo, nsorted[:, 0].contiguous()), max=rlo.numel() - 1)
            self._hot_score = rscore.index_select(0, by_lo.index_select(0, at)).contiguous()
        self._hot_dir = None
        changed = dropped.shape[0] + sum(t.shape[0] for t in took)
        # a large change of the hot set changes the traffic matrix: measure it afresh (the
        # fixed-capacity exchange otherwise adapts within a few steps)
        if changed * 4 > max(old.shape[0], 1):
            self._reset_exchange()
        self._stats["replica_refreshes"] += 1
        self._stats["replica_added"] = self._stats.get("replica_added", 0) + sum(
            t.shape[0] for t in took)
        self._stats["replica_dropped"] = self._stats.get("replica_dropped", 0) + int(dropped.shape[0])
        self._stats["replica_fetched_bytes"] = self._stats.get("replica_fetched_bytes", 0) + fetched
        return stored

    # ------------------------------------------------------------------------------
    # membership changes: rebalancing, failure, warm recovery, snapshots
    # ------------------------------------------------------------------------------
    def set_ring(self, ring: ShardRing, migrate: bool = True, now: Optional[int] = None,
                 chunk_keys: int = 1 << 18, incremental: bool = False) -> int:
        """Collective. Switch every rank to ``ring``. With ``migrate`` each rank ships
        the live objects it holds that the new ring assigns elsewhere to their new
        owners through the routed SET path (warm rebalancing: no refetch from the
        origin), ``chunk_keys`` objects at a time (bounded memory). ``incremental``: only
        switch the ring and queue the migration; ``migrate_step`` then moves it a byte
        budget at a time between serving steps (meanwhile a moved key's GET misses at its
        new owner until its object arrives — a cache miss, never a wrong answer). Returns
        the number of objects this rank has to migrate."""
        self.sync_sets()
        mkeys = None
        if migrate and self.world > 1:
            keys = self.shard.export_keys(now)
            pts, own = ring.tensors(self.device)
            dest, _ = R.route(keys, pts, own, self.world)
            mkeys = keys[dest != self.rank].contiguous()
        self.ring = ring
        self.ring_pts, self.ring_own = ring.tensors(self.device)
        self._reset_exchange()
        self._migrating = mkeys if mkeys is not None else None
        self._migrate_chunk = chunk_keys
        # until the migration is done, every key a SET or DELETE names (on any rank, through
        # any path) is remembered: its migrated copy is older than what the new owner got
        self._touched = [] if migrate and self.world > 1 else None
        self._touched_all = None
        moved = int(mkeys.shape[0]) if mkeys is not None else 0
        if migrate and self.world > 1 and not incremental:
            while self.migrate_step(None, now):
                pass
        return moved

    def _touch(self, keys: torch.Tensor) -> None:
        """During an incremental migration: remember keys a SET / DELETE names."""
        t = getattr(self, "_touched", None)
        if t is not None and keys.shape[0]:
            t.append(keys.to(self.device).contiguous().clone())

    def _gather_touched(self) -> None:
        """Collective: merge every rank's keys SET or DELETEd since the ring switch into
        ``_touched_all`` (sorted by lo, the same on every rank), and drop them from this
        rank's migration queue (their old copies here are stale: the new owner has a newer
        value, or the key is gone)."""
        dev = self.device
        mine = (torch.cat(self._touched) if self._touched else
                torch.zeros((0, 2), dtype=torch.int64, device=dev))
        self._touched = []
        cnt = torch.tensor([mine.shape[0]], dtype=torch.int64, device=dev)
        all_reduce(cnt, op=dist.ReduceOp.MAX, group=self.group)
        m = int(cnt)
        if m == 0:
            return
        pad = torch.zeros((m, 2), dtype=torch.int64, device=dev)
        pad[: mine.shape[0]] = mine
        parts = [torch.empty_like(pad) for _ in range(self.world)]
        all_gather(parts, pad, group=self.group)
        allk = torch.cat(parts + ([self._touched_all] if self._touched_all is not None else []))
        allk = allk[(allk != 0).any(dim=1)]
        ulo, inv = torch.unique(allk[:, 0].contiguous(), return_inverse=True)
        u = torch.empty((ulo.numel(), 2), dtype=torch.int64, device=dev)
        u[inv] = allk
        self._touched_all = u  # torch.unique sorts by lo
        q = getattr(self, "_migrating", None)
        if q is not None and q.shape[0]:
            stale = self._member(q, u)
            if bool(stale.any()):
                self.shard.remove(q[stale].contiguous(), None)
                q = q[~stale].contiguous()
                self._migrating = q if q.shape[0] else None

    def migrate_step(self, budget_bytes: Optional[int] = None, now: Optional[int] = None) -> bool:
        """Collective. Move queued migration objects (``set_ring``) to their new owners:
        chunks of ``chunk_keys`` until ``budget_bytes`` of records have moved on this rank
        (None: one chunk). Returns whether any rank has objects left (the same on every
        rank). A key SET or DELETEd anywhere since the ring switch is not migrated (its
        copy here is older than what its new owner holds, or it was deleted), and a
        delivered object is stored only where the new owner holds nothing of the key."""
        self.sync_sets()
        moved_bytes = 0
        while True:
            if getattr(self, "_touched", None) is not None:
                self._gather_touched()
            q = getattr(self, "_migrating", None)
            left = torch.tensor([0 if q is None else int(q.shape[0])], dtype=torch.int64,
                                device=self.device)
            all_reduce(left, op=dist.ReduceOp.MAX, group=self.group)
            if int(left) == 0:
                self._migrating = None
                self._touched = self._touched_all = None
                return False
            part = (q[: self._migrate_chunk] if q is not None
                    else torch.zeros((0, 2), dtype=torch.int64, device=self.device)).contiguous()
            batch = None
            if part.shape[0]:
                lk = self.shard.lookup(part, now)
                data = self.shard.gather(lk)
                n = part.shape[0]
                batch = records_to_set_batch(part, GetResult(data, lk.off[:n], lk.size[:n]))
                moved_bytes += int(lk.off[n])
            else:
                empty = torch.zeros(0, dtype=torch.int64, device=self.device)
                batch = SetBatch(part, torch.zeros(16, dtype=torch.uint8, device=self.device),
                                 empty, empty.to(torch.int32))
            # lands on the new owners (collective), where they hold nothing of the key yet
            self.set(batch, now, if_absent=True)
            if part.shape[0]:
                self.shard.remove(part, now)      # this rank no longer owns them
                self._migrating = q[part.shape[0]:] if q.shape[0] > part.shape[0] else None
            # stop once any rank has used its budget (the decision is collective)
            q = getattr(self, "_migrating", None)
            st = torch.tensor([0 if q is None else int(q.shape[0]),
                               int(budget_bytes is None or moved_bytes >= budget_bytes)],
                              dtype=torch.int64, device=self.device)
            all_reduce(st, op=dist.ReduceOp.MAX, group=self.group)
            if int(st[0]) == 0:
                self._migrating = None
                self._touched = self._touched_all = None
                return False
            if int(st[1]):
                return True

    def fail_shard(self, rank: int) -> None:
        """Collective. Simulate (or react to) the loss of ``rank``'s shard: every rank
        drops it from the ring (its keys remap, like ketama auto-eject) and the lost
        shard's contents are discarded."""
        self.sync_sets()
        if rank not in self.ring.shards:
            return
        self.set_ring(self.ring.without(rank), migrate=False)
        if self.rank == rank:
            self.shard.flush()
        if self.replica is not None:
            self.replica.flush()
            self._hot = self._hot_score = None
            self._reset_exchange()

    def restore_shard(self, rank: int, now: Optional[int] = None) -> int:
        """Collective. Re-admit ``rank``; objects written while it was out migrate
        back to it from their interim owners (warm restore from peer shards)."""
        shards = sorted(set(self.ring.shards) | {rank})
        return self.set_ring(ShardRing(shards, self.ring.points_per_shard), migrate=True, now=now)

    def save(self, directory: str) -> str:
        """Snapshot this rank's shard to ``directory/shard-<rank>.snap``."""
        import os

        os.makedirs(directory, exist_ok=True)
        path = os.path.join(directory, f"shard-{self.rank}.snap")
        self.sync_sets()
        self.shard.save(path)
        return path

    def load(self, directory: str) -> None:
        import os

        self.sync_sets()
        self.shard.load(os.path.join(directory, f"shard-{self.rank}.snap"))

    def counters(self) -> dict:
        self.sync_sets()
        return allreduce_stats(self.shard.counters(), self.device, self.group)
