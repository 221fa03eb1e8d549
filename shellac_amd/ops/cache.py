"""Tensor-level batch operations on one cache shard (HBM on a GPU, DRAM on the CPU).

This is the compute path of the cache. A ``CacheShard`` on a ``cuda`` device
drives the hand-written HIP kernels in ``csrc/hbm_cache.hip`` (probe, load-
balanced gather, dedupe + scan-allocated log write, two-choice CAS insert); on
the CPU it drives ``csrc/host_cache.cc``, which implements the same layout and
policies and is the semantic reference the kernels are tested against.

Keys are 128-bit digests stored as ``int64`` tensors of shape ``[n, 2]`` (lo, hi)
(see ``csrc/digest.h``). The reference addresses objects by URL string through
pylibmc (src/python/shellac/server/Server.py:327, :335, :432); digests are what
let the GPU path move fixed 16-byte records.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Iterable, Optional, Sequence

import numpy as np
import torch

from .._native import core

ITEM_HEADER_BYTES = 32
ITEM_MAGIC = 0x5348A11C
MISS_LOC = (1 << 64) - 1


def _stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def item_bytes(vlen: int) -> int:
    return ITEM_HEADER_BYTES + ((vlen + 15) & ~15)


# ----------------------------------------------------------------------------------
# digests & packing helpers
# ----------------------------------------------------------------------------------
def pack_bytes(items: Sequence[bytes]) -> tuple[np.ndarray, np.ndarray]:
    """Concatenate byte strings -> (uint8 buffer, int64 offsets[n+1])."""
    offs = np.zeros(len(items) + 1, dtype=np.int64)
    np.cumsum([len(x) for x in items], out=offs[1:])
    buf = np.frombuffer(b"".join(items), dtype=np.uint8) if items else np.zeros(0, np.uint8)
    return buf, offs


def digest_strings(keys: Sequence[bytes], device: str | torch.device = "cpu") -> torch.Tensor:
    """128-bit digests of ``keys`` as an int64 tensor [n, 2] (computed on the host)."""
    c = core()
    buf, offs = pack_bytes(list(keys))
    buf = np.ascontiguousarray(buf)
    if buf.size == 0:
        buf = np.zeros(1, np.uint8)
    out = np.zeros((len(keys), 2), dtype=np.int64)
    c.host_digest_keys(buf.ctypes.data, offs.ctypes.data, len(keys), out.ctypes.data)
    return torch.from_numpy(out).to(device)


def digest_packed(buf: torch.Tensor, offs: torch.Tensor) -> torch.Tensor:
    """Digest packed key bytes on the tensors' device (HIP kernel on GPU)."""
    c = core()
    n = offs.numel() - 1
    out = torch.empty((n, 2), dtype=torch.int64, device=buf.device)
    if buf.is_cuda:
        c.digest_keys(buf.data_ptr(), offs.data_ptr(), n, out.data_ptr(), _stream_handle(buf.device))
    else:
        c.host_digest_keys(buf.data_ptr(), offs.data_ptr(), n, out.data_ptr())
    return out


def pack_values(values: Sequence[bytes], device: str | torch.device = "cpu"):
    """Pack values 16-byte aligned (+16 B readable slack) for ``CacheShard.store``.

    Returns (values uint8 tensor, val_off int64 tensor, vlen int32 tensor).
    """
    n = len(values)
    vlen = np.array([len(v) for v in values], dtype=np.int64)
    padded = (vlen + 15) & ~15
    val_off = np.zeros(n, dtype=np.int64)
    if n:
        np.cumsum(padded[:-1], out=val_off[1:])
    total = int(padded.sum()) + 16
    buf = np.zeros(total, dtype=np.uint8)
    for i, v in enumerate(values):
        buf[val_off[i] : val_off[i] + len(v)] = np.frombuffer(v, dtype=np.uint8)
    return (
        torch.from_numpy(buf).to(device),
        torch.from_numpy(val_off).to(device),
        torch.from_numpy(vlen.astype(np.int32)).to(device),
    )


def unpack_records(out: torch.Tensor, off: torch.Tensor, size: torch.Tensor) -> list:
    """Decode GET output ([ItemHeader | value | pad] per hit) -> list of (value, flags) or None."""
    o = out.cpu().numpy()
    offs = off.cpu().numpy()
    sizes = size.cpu().numpy()
    res = []
    for i in range(len(sizes)):
        if sizes[i] == 0:
            res.append(None)
            continue
        base = int(offs[i])
        hdr = o[base : base + ITEM_HEADER_BYTES].view(np.uint32)
        vl, flags, magic = int(hdr[4]), int(hdr[5]), int(hdr[7])
        if magic != ITEM_MAGIC:
            raise RuntimeError(f"corrupt item header at {base}: magic {magic:#x}")
        res.append((o[base + ITEM_HEADER_BYTES : base + ITEM_HEADER_BYTES + vl].tobytes(), flags))
    return res


def coalesce(keys: torch.Tensor, table: Optional[torch.Tensor] = None):
    """GET coalescing (request collapsing inside a batch). Returns ``first`` (int32
    [n]): the row that serves row i — one row per distinct digest claims it with a CAS
    in an open-addressing table (``k_coalesce``), its duplicates point at that row.
    Pass it to ``CacheShard.lookup(first=...)`` (duplicates skip the index probe and
    the gather) and call ``expand(first, lookup)`` after the gather, so every request
    addresses its claimer's record. CPU shards: ``None`` (the host engine probes every
    row; results are the same values).
    ``table`` (a caller-owned, zeroed table, see ``CacheShard.lookup_coalesced``):
    returns ``(first, cslot)`` and ``expand_out(..., table, cslot)`` must clean it."""
    if not keys.is_cuda or keys.shape[0] == 0:
        return None if table is None else (None, None)
    c = core()
    n = keys.shape[0]
    cslot = None
    if table is None:
        slots = int(c.coalesce_table_slots(n))
        table = torch.empty(slots, dtype=torch.int32, device=keys.device)
    else:
        slots = table.numel()
        if slots < int(c.coalesce_table_slots(n)) or slots & (slots - 1):
            raise ValueError("coalescing table too small or not a power of two")
        cslot = torch.empty(n, dtype=torch.int32, device=keys.device)
    first = torch.empty(n, dtype=torch.int32, device=keys.device)
    c.coalesce_keys(keys.data_ptr(), n, table.data_ptr(), slots, first.data_ptr(),
                    _stream_handle(keys.device), cslot.data_ptr() if cslot is not None else 0,
                    cslot is not None)
    return first if cslot is None else (first, cslot)


def expand(first: Optional[torch.Tensor], size: torch.Tensor, off: torch.Tensor) -> None:
    """After the gather of a coalesced lookup: duplicate rows take their claimer's
    (size, off), in place (``k_expand``). No-op when ``first`` is None."""
    if first is None:
        return
    n = first.numel()
    core().expand_coalesced(first.data_ptr(), n, size.data_ptr(), off.data_ptr(),
                            _stream_handle(first.device))


def expand_out(first: torch.Tensor, size: torch.Tensor, off: torch.Tensor,
               out_size: torch.Tensor, out_off: torch.Tensor,
               table: Optional[torch.Tensor] = None, cslot: Optional[torch.Tensor] = None) -> None:
    """Out-of-place ``expand`` (``k_expand_out``): out_size/out_off[i] := size/off of
    first[i]. It does not modify size/off, so it may run on another stream while the
    gather reads them. With ``table``/``cslot`` from ``lookup_coalesced(table=...)`` it
    also clears the claimed slots, leaving the table zeroed for the next batch."""
    n = first.numel()
    core().expand_coalesced_out(first.data_ptr(), n, size.data_ptr(), off.data_ptr(),
                                out_size.data_ptr(), out_off.data_ptr(),
                                table.data_ptr() if table is not None else 0,
                                cslot.data_ptr() if cslot is not None else 0,
                                _stream_handle(first.device))


class StreamEvent:
    """A HIP event with a chosen fence scope, for ordering two streams of one GPU.

    ``torch.cuda.Event`` records with the default system-scope release (an L2 write-back
    and invalidate every time); ``fence="device"`` releases to device scope only
    (``hipEventReleaseToDevice``), ``"none"`` disables the system fence
    (``hipEventDisableSystemFence``), ``"system"`` is the default. Both streams must be on
    the same GPU and nothing on the host may read what the event orders."""

    def __init__(self, fence: str = "device", timing: bool = False):
        c = core()
        flags = 0 if timing else int(c.EVENT_DISABLE_TIMING)
        if fence == "device":
            flags |= int(c.EVENT_RELEASE_TO_DEVICE)
        elif fence == "none":
            flags |= int(c.EVENT_DISABLE_SYSTEM_FENCE)
        elif fence != "system":
            raise ValueError(f"unknown fence {fence!r}")
        self.fence = fence
        self.handle = int(c.event_create(flags))

    def record(self, stream: "torch.cuda.Stream") -> None:
        core().event_record(self.handle, stream.cuda_stream)

    def wait(self, stream: "torch.cuda.Stream") -> None:
        """``stream`` waits for the work this event recorded."""
        core().stream_wait_event(stream.cuda_stream, self.handle)

    def query(self) -> bool:
        """Whether the work this event marks (or the kernel that completes it) is done."""
        return bool(core().event_query(self.handle))

    def elapsed_time(self, end: "StreamEvent") -> float:
        """Milliseconds from this event to ``end`` (both created with timing=True);
        waits for ``end``."""
        return float(core().event_elapsed_ms(self.handle, end.handle))

    def __del__(self):
        h = getattr(self, "handle", 0)
        if h:
            try:
                core().event_destroy(h)
            except Exception:  # interpreter shutdown
                pass


def _event_handle(ev) -> int:
    if ev is None:
        return 0
    if isinstance(ev, StreamEvent):
        return ev.handle
    return ev.cuda_event



def _stop_handle(ev) -> int:
    """hipEvent_t a launch completes as its stop event: a ``StreamEvent`` only (a
    ``torch.cuda.Event`` has no handle before its first record)."""
    if ev is None:
        return 0
    if not isinstance(ev, StreamEvent):
        raise TypeError("a stop event must be a StreamEvent")
    return ev.handle


@dataclass
class Lookup:
    loc: torch.Tensor   # int64 [n]  physical log offset (MISS_LOC as -1 on miss)
    size: torch.Tensor  # int64 [n+1] response bytes per key (0 = miss); size[n] = 0
    # the offsets buffer as the lookup wrote it: the exclusive scan of size (off_raw[n] =
    # total bytes), or, for a blocked lookup (lookup_coalesced(blocked=True)), row i's
    # offset within its lookup workgroup's rows [b << shift, (b + 1) << shift) with
    # off_raw[n] unwritten, `prefix[b]` the bytes of the workgroups before b (prefix[last +
    # 1] = the total). Read it through `off`, which refuses a blocked lookup: only gather()
    # (with its expand tail, which writes the per-request offsets) reads those.
    off_raw: torch.Tensor
    prefix: Optional[torch.Tensor] = None
    shift: int = 0

    @property
    def off(self) -> torch.Tensor:
        """int64 [n+1]: the exclusive scan of ``size`` (off[n] = total bytes)."""
        if self.prefix is not None:
            raise ValueError("a blocked lookup holds workgroup-local offsets: the per-request "
                             "offsets come from the gather's expand tail")
        return self.off_raw

    @property
    def n(self) -> int:
        return self.loc.numel()

    def total(self) -> torch.Tensor:
        """Total response bytes (a one-element device tensor)."""
        if self.prefix is None:
            return self.off_raw[self.n:self.n + 1]
        nb = ((self.n - 1) >> self.shift) + 1 if self.n else 0
        return self.prefix[nb:nb + 1]

    def hits(self) -> torch.Tensor:
        return self.size[: self.n] > 0


def reserve_step_streams(device) -> None:
    """Create the routed serving step's streams (plan, SET side, reply + assembly) for
    ``device`` now. A process gets four hardware queues, handed out round robin as
    streams are first used; the step keeps four streams busy at once (with the caller's),
    so it needs them created before anything else makes streams (torch.distributed's
    communicators, other libraries). Idempotent; bench.py calls it right after choosing the
    device, and every GPU ``CacheShard`` does."""
    dev = torch.device(device)
    if dev.type == "cuda":
        core().step_streams(dev.index if dev.index is not None else torch.cuda.current_device())


class CacheShard:
    """One cache shard: an HBM arena on ``cuda:i`` or a DRAM arena on ``cpu``.

    Args:
      log_bytes: capacity of the circular value log.
      nbuckets: index buckets (power of two); 4 entries each, two-choice hashing.
      max_item: largest storable value (memcached parity default 1 MiB).
      evict: "clock" (default: objects read since the eviction hand last passed are
        re-appended instead of overwritten — memcached-LRU-like hit ratios) or "fifo"
        (plain circular log).
      reinsert_max: CLOCK reinsertion budget per SET batch in bytes (0 = auto).
      serve_blocks: resident edge-server blocks (GPU; ``serve_get`` jobs side by side).
    """

    EVICT = {"fifo": 0, "clock": 1}

    def __init__(self, log_bytes: int, nbuckets: int, max_item: int = 1 << 20,
                 device: str | torch.device = "cpu", evict: str = "clock",
                 reinsert_max: int = 0, serve_blocks: int = 8):
        self.device = torch.device(device)
        self.log_bytes = int(log_bytes)
        self.nbuckets = int(nbuckets)
        self.max_item = int(max_item)
        self.evict = evict
        ev = self.EVICT[evict]
        c = core()
        if self.device.type == "cuda":
            idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
            self.device = torch.device("cuda", idx)
            reserve_step_streams(self.device)
            self._impl = c.HbmCache(self.log_bytes, self.nbuckets, self.max_item, idx, ev,
                                    int(reinsert_max), int(serve_blocks))
            self.is_gpu = True
        elif self.device.type == "cpu":
            self._impl = c.HostCache(self.log_bytes, self.nbuckets, self.max_item, ev,
                                     int(reinsert_max))
            self.is_gpu = False
        else:
            raise ValueError(f"unsupported device {self.device}")
        self.epoch = time.time()

    # -- time ---------------------------------------------------------------------
    def now(self) -> int:
        """Seconds since this shard's epoch (the unit of ``expire``)."""
        return int(time.time() - self.epoch) + 1

    def expire_at(self, ttl_seconds: int) -> int:
        return 0 if ttl_seconds <= 0 else self.now() + int(ttl_seconds)

    def _s(self) -> int:
        return _stream_handle(self.device)

    def _check(self, t: torch.Tensor, name: str):
        # a GPU shard also takes pinned host tensors: its kernels read and write them in
        # place over PCIe (the proxy's edge: keys, SET payloads and responses stay in host
        # memory, no staging copies)
        host_ok = self.is_gpu and t.device.type == "cpu" and t.is_pinned()
        if t.device != self.device and not host_ok:
            raise ValueError(f"{name} on {t.device}, shard on {self.device}")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")

    # -- GET ----------------------------------------------------------------------
    def lookup(self, keys: torch.Tensor, now: Optional[int] = None,
               reserve_bytes: int = 0, total_slot: int = -1,
               first: Optional[torch.Tensor] = None) -> Lookup:
        """Probe the index. ``reserve_bytes`` > 0 also misses objects that the next
        ``reserve_bytes`` of log appends would overwrite, so a SET of at most that many
        bytes (``set_bound``) may run between this lookup and its gather.
        ``total_slot`` >= 0 (GPU) has the kernel write off[n] into that pinned host slot
        (``host_total``), so the response size needs no device-to-host copy.
        ``first`` (GPU, from ``coalesce``): duplicate rows are answered as empty without
        a probe; ``expand`` fills them in after the gather."""
        self._check(keys, "keys")
        n = keys.shape[0]
        loc = torch.empty(n, dtype=torch.int64, device=self.device)
        size = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        off = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        now = self.now() if now is None else now
        if self.is_gpu:
            if first is not None:
                self._check(first, "first")
                if first.numel() != n or first.dtype != torch.int32:
                    raise ValueError("first must be int32 [n] from coalesce()")
            self._impl.lookup(keys.data_ptr(), n, loc.data_ptr(), size.data_ptr(), off.data_ptr(),
                              now, self._s(), int(reserve_bytes), int(total_slot),
                              first.data_ptr() if first is not None else 0)
        else:
            size[n] = 0
            self._impl.lookup(keys.data_ptr(), n, loc.data_ptr(), size.data_ptr(), off.data_ptr(),
                              now, int(reserve_bytes))
        return Lookup(loc, size, off)

    def lookup_coalesced(self, keys: torch.Tensor, now: Optional[int] = None,
                         reserve_bytes: int = 0, total_slot: int = -1,
                         table: Optional[torch.Tensor] = None, blocked: bool = False,
                         index_done=None):
        """``coalesce`` + ``lookup(first=...)`` fused into one kernel on GPU shards (the
        row that claims a digest probes the index for it). Returns (Lookup, first,
        cslot); duplicate rows have size 0 until ``expand(first, lk.size, lk.off)`` runs
        after the gather. ``table``: a caller-owned, zeroed coalescing table (int32,
        >= ``coalesce_table_slots(n)`` power-of-two slots) — then ``cslot`` holds each
        claimer's slot and ``expand_out`` must run to clean the table again; otherwise
        a temporary table is zeroed here and ``cslot`` is None. ``blocked`` (GPU): the
        Lookup holds block-local offsets (``Lookup.prefix``), which only ``gather`` with an
        ``expand`` tail reads — no n-row offsets scan between the lookup and the gather.
        ``index_done`` (GPU, a ``StreamEvent``): completes with the kernel that reads the
        index, as that kernel's own completion signal (a SET's ``index_after``).
        CPU shards: a plain lookup, ``first = cslot = None``."""
        if not self.is_gpu or keys.shape[0] == 0:
            return self.lookup(keys, now, reserve_bytes, total_slot), None, None
        self._check(keys, "keys")
        c = core()
        n = keys.shape[0]
        cslot = None
        if table is None:
            slots = int(c.coalesce_table_slots(n))
            table = torch.empty(slots, dtype=torch.int32, device=self.device)
        else:
            slots = table.numel()
            if slots < int(c.coalesce_table_slots(n)) or slots & (slots - 1):
                raise ValueError("coalescing table too small or not a power of two")
            cslot = torch.empty(n, dtype=torch.int32, device=self.device)
        first = torch.empty(n, dtype=torch.int32, device=self.device)
        loc = torch.empty(n, dtype=torch.int64, device=self.device)
        size = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        off = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        now = self.now() if now is None else now
        prefix = (torch.empty(int(c.LOOKUP_PREFIX_WORDS), dtype=torch.int64, device=self.device)
                  if blocked else None)
        shift = self._impl.lookup_coalesced(keys.data_ptr(), n, table.data_ptr(), slots,
                                            first.data_ptr(), loc.data_ptr(), size.data_ptr(),
                                            off.data_ptr(), now, self._s(), int(reserve_bytes),
                                            int(total_slot),
                                            cslot.data_ptr() if cslot is not None else 0,
                                            cslot is not None,
                                            prefix.data_ptr() if prefix is not None else 0,
                                            _stop_handle(index_done))
        return Lookup(loc, size, off, prefix, max(int(shift), 0)), first, cslot

    def host_total(self, slot: int, timeout_ms: int = 10000) -> int:
        """Total bytes of the last lookup given ``total_slot=slot``: spins on the pinned
        slot until the kernel has written it (no stream or event synchronisation)."""
        return int(self._impl.wait_host_slot(slot, timeout_ms))

    def small_get(self, keys: torch.Tensor, out_cap: int = 16 << 20,
                  now: Optional[int] = None, done_slot: int = -1):
        """GPU edge GET (the proxy's micro-batch path): probe + scan + gather in one
        kernel, each key probed once. Returns (out bytes, off[n+1]); off[n] > out_cap
        means nothing was copied. ``done_slot`` >= 0: the kernel's last workgroup
        publishes off[n] into that host slot once every output byte is visible;
        ``host_total(done_slot)`` then replaces a stream synchronisation."""
        assert self.is_gpu and keys.shape[0] <= int(core().SMALL_GET_MAX)
        self._check(keys, "keys")
        n = keys.shape[0]
        out = torch.empty(max(int(out_cap), 16), dtype=torch.uint8, device=self.device)
        off = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        self._impl.small_get(keys.data_ptr(), n, out.data_ptr(), int(out_cap), off.data_ptr(),
                             self.now() if now is None else now, self._s(), int(done_slot))
        return out, off

    def serve_get(self, keys: torch.Tensor, out_cap: int = 16 << 20,
                  now: Optional[int] = None, done_slot: int = 5, timeout_ms: int = 10000):
        """The same edge GET answered by the resident edge-server kernel (no launch):
        ``keys`` are host digests; returns (out bytes, off[n+1]) once the server has
        published the job's total into ``done_slot``. None when the job could not be
        queued (ring full, n > SERVE_KEYS). Records a concurrent SET overwrote while
        they were copied come back with a zeroed magic word (treat as misses). The job is
        ordered after the work queued so far on the current stream (the server runs on no
        stream: the binding polls an event recorded there before it queues the job)."""
        assert self.is_gpu
        keys = keys.to("cpu").contiguous()
        n = keys.shape[0]
        out = torch.zeros(max(int(out_cap), 16), dtype=torch.uint8, device=self.device)
        off = torch.zeros(n + 1, dtype=torch.int64, device=self.device)
        if not self._impl.serve_get(keys.data_ptr(), n, out.data_ptr(), int(out_cap),
                                    off.data_ptr(), self.now() if now is None else now,
                                    int(done_slot), self._s()):
            return None
        self._impl.serve_wait(int(done_slot), int(timeout_ms))
        return out, off

    def gather(self, lk: Lookup, out: Optional[torch.Tensor] = None,
               total: Optional[int] = None, out_cap: Optional[int] = None,
               expand=None) -> torch.Tensor:
        """Copy hits into ``out`` (allocated from off[n] if not given: one sync).
        ``out_cap`` (GPU): the kernel writes nothing when off[n] exceeds it, so a gather
        can be queued before the total is known. ``expand`` (GPU, a coalesced lookup):
        (first, out_size, out_off, table, cslot) — the gather also writes every request's
        (size, off) from its claimer and clears the coalescing table (``expand_out``)."""
        if out is None:
            total = int(lk.total().item()) if total is None else total
            out = torch.empty(max(total, 16), dtype=torch.uint8, device=self.device)
        self._check(out, "out")
        if self.is_gpu:
            cap = out.numel() if out_cap is None else min(int(out_cap), out.numel())
            ex = [0] * 6
            if expand is not None:
                first, osz, ooff, table, cslot = expand
                ex = [first.data_ptr(), lk.size.data_ptr(), osz.data_ptr(), ooff.data_ptr(),
                      table.data_ptr() if table is not None else 0,
                      cslot.data_ptr() if cslot is not None else 0]
            elif lk.prefix is not None:
                raise ValueError("a blocked lookup's offsets are read only with an expand tail")
            self._impl.gather(lk.loc.data_ptr(), lk.off_raw.data_ptr(), lk.n, out.data_ptr(),
                              self._s(), cap, *ex,
                              lk.prefix.data_ptr() if lk.prefix is not None else 0, lk.shift)
        else:
            self._impl.gather(lk.loc.data_ptr(), lk.off.data_ptr(), lk.n, out.data_ptr())
        return out

    def get(self, keys: torch.Tensor, now: Optional[int] = None):
        """lookup + gather. Returns (out bytes, off[n], size[n]); record i = out[off[i]:+size[i]]."""
        if not self.is_gpu:
            lk = self.lookup(keys, now)
            return self.gather(lk), lk.off[: lk.n], lk.size[: lk.n]
        lk = self.lookup(keys, now, total_slot=1)
        out = self.gather(lk, total=self.host_total(1))
        return out, lk.off[: lk.n], lk.size[: lk.n]

    # -- SET ----------------------------------------------------------------------
    @staticmethod
    def payload_bound(n: int, payload_bytes: int) -> int:
        """Upper bound of the log bytes ``n`` values from a ``payload_bytes`` buffer
        occupy (32-B header + value, 16-B aligned, per item)."""
        return 48 * int(n) + int(payload_bytes)

    def set_bound(self, n: int, payload_bytes: int) -> int:
        """Upper bound of the log bytes a SET of ``n`` values from a ``payload_bytes``
        buffer appends — its own records plus, under CLOCK, the reinsertions of
        referenced objects it triggers (the ``reserve_bytes`` a lookup that a SET may
        overtake needs)."""
        return self.payload_bound(n, payload_bytes) + int(self._impl.reinsert_max)

    def store(self, keys: torch.Tensor, values: torch.Tensor, val_off: torch.Tensor,
              vlen: torch.Tensor, flags: Optional[torch.Tensor] = None,
              expire: Optional[torch.Tensor] = None, now: Optional[int] = None,
              bytes_bound: Optional[int] = None,
              index_after=None, append_after=None, append_done=None, phase: int = 0,
              plan_done=None, done=None) -> None:
        """SET a batch (later duplicates win). ``bytes_bound`` bounds the log bytes the
        batch appends; the default assumes every byte of ``values`` is stored.
        ``index_after`` (GPU, a recorded ``torch.cuda.Event`` or a ``StreamEvent``):
        dedupe, sizing and the log append run at once, the index insert waits for the
        event — so a lookup followed by that event on another stream overlaps the SET's log
        write (see ``HbmCache::store``). ``append_after`` (GPU, an event): the log append
        waits for it, the CLOCK hand and the SET planning do not (a gather still reading the
        region the append overwrites may run meanwhile). ``append_done`` (GPU, an event):
        recorded right after the log append. ``phase`` (GPU): 1 queues only the batch's
        CLOCK hand (a full cache), 2 the rest of the chain for the same batch; 0 both. A
        phase-1 hand is *detached*: it may run as soon as the previous batch's planning is
        done (``plan_done`` of that batch's phase 2), beside that batch's append and index
        insert — its reinsertions are indexed as moves, dropped when the key's entry has
        moved on (``HbmCache::store``). ``plan_done`` (GPU, an event): recorded after the
        batch's planning kernels. ``done`` (GPU, a ``StreamEvent``): completes with everything
        the call queued, carried by the chain's last kernel as its completion signal."""
        for t, nm in ((keys, "keys"), (values, "values"), (val_off, "val_off"), (vlen, "vlen")):
            self._check(t, nm)
        if vlen.dtype != torch.int32 or val_off.dtype != torch.int64:
            raise TypeError("vlen must be int32 and val_off int64")
        n = keys.shape[0]
        if n == 0:
            if done is not None and self.is_gpu:
                done.record(torch.cuda.current_stream(self.device))   # nothing to carry it
            return
        now = self.now() if now is None else now
        fp = 0 if flags is None else flags.data_ptr()
        ep = 0 if expire is None else expire.data_ptr()
        # the same bound on both twins: the CLOCK hand's reinsertion cap follows from it
        bound = (self.payload_bound(n, values.numel()) if bytes_bound is None
                 else int(bytes_bound))
        if self.is_gpu:
            self._impl.store(keys.data_ptr(), values.data_ptr(), val_off.data_ptr(), vlen.data_ptr(),
                             fp, ep, n, bound, now, self._s(), _event_handle(index_after),
                             _event_handle(append_after), _event_handle(append_done), phase,
                             _event_handle(plan_done), _stop_handle(done))
        elif phase != 1:
            self._impl.store(keys.data_ptr(), values.data_ptr(), val_off.data_ptr(), vlen.data_ptr(),
                             fp, ep, n, now, bound)

    def set_many(self, keys: Sequence[bytes], values: Sequence[bytes], ttl: int = 0,
                 flags: int = 0) -> None:
        d = digest_strings(keys, self.device)
        v, vo, vl = pack_values(values, self.device)
        ex = torch.full((len(keys),), self.expire_at(ttl), dtype=torch.int32, device=self.device)
        fl = torch.full((len(keys),), flags, dtype=torch.int32, device=self.device)
        self.store(d, v, vo, vl, fl, ex)

    def get_many(self, keys: Sequence[bytes]) -> list:
        d = digest_strings(keys, self.device)
        out, off, size = self.get(d)
        return [None if r is None else r[0] for r in unpack_records(out, off, size)]

    # -- DELETE / maintenance ------------------------------------------------------
    def remove(self, keys: torch.Tensor, now: Optional[int] = None) -> torch.Tensor:
        self._check(keys, "keys")
        n = keys.shape[0]
        found = torch.zeros(n, dtype=torch.uint8, device=self.device)
        now = self.now() if now is None else now
        if self.is_gpu:
            self._impl.remove(keys.data_ptr(), n, found.data_ptr(), now, self._s())
        else:
            self._impl.remove(keys.data_ptr(), n, found.data_ptr(), now)
        return found.bool()

    def sweep(self, now: Optional[int] = None) -> tuple[int, int]:
        now = self.now() if now is None else now
        return tuple(self._impl.sweep(now, self._s()) if self.is_gpu else self._impl.sweep(now))

    def flush(self) -> None:
        if self.is_gpu:
            self._impl.flush(self._s())
        else:
            self._impl.flush()

    def export_keys(self, now: Optional[int] = None) -> torch.Tensor:
        """Digests of every live object in this shard, int64 [m, 2] on the shard's device."""
        now = self.now() if now is None else now
        cap = 1 << 16
        while True:
            out = torch.empty((cap, 2), dtype=torch.int64, device=self.device)
            if self.is_gpu:
                m = self._impl.export_keys(out.data_ptr(), cap, now, self._s())
            else:
                m = self._impl.export_keys(out.data_ptr(), cap, now)
            if m <= cap:
                return out[:m]
            cap = int(m * 1.25) + 1024

    def save(self, path: str) -> None:
        """Snapshot index + log + head to ``path`` (warm restart)."""
        import struct

        user = [struct.unpack("<Q", struct.pack("<d", self.epoch))[0], 0, 0, 0]
        if self.is_gpu:
            self._impl.save(path, user, self._s())
        else:
            self._impl.save(path, user)

    def load(self, path: str) -> None:
        """Restore a snapshot written by ``save`` (same geometry); expiry times
        stay relative to the saved epoch."""
        import struct

        user = self._impl.load(path, self._s()) if self.is_gpu else self._impl.load(path)
        self.epoch = struct.unpack("<d", struct.pack("<Q", int(user[0])))[0]

    def counters(self) -> dict:
        return self._impl.counters(self._s()) if self.is_gpu else self._impl.counters()

    def head(self) -> int:
        return self._impl.head(self._s()) if self.is_gpu else self._impl.head()

    def reserve(self, n: int) -> None:
        if self.is_gpu:
            self._impl.reserve(n)
