"""Semantics of a cache shard (DRAM engine on the CPU; the HBM kernels are checked
against the same engine in tests/test_hbm_gpu.py)."""
import numpy as np
import pytest
import torch

from shellac_amd.ops.cache import (CacheShard, digest_strings, item_bytes, pack_values,
                                   unpack_records)
from shellac_amd.ops import routing as R


def make(log=1 << 20, nb=1 << 10, max_item=8192):
    return CacheShard(log, nb, max_item, "cpu")


def test_set_get_roundtrip_and_flags():
    s = make()
    keys = [f"/p/{i}".encode() for i in range(200)]
    vals = [bytes([i % 251]) * (i * 7 % 300) for i in range(200)]
    d = digest_strings(keys)
    v, vo, vl = pack_values(vals)
    flags = torch.arange(200, dtype=torch.int32)
    s.store(d, v, vo, vl, flags=flags)
    out, off, size = s.get(d)
    recs = unpack_records(out, off, size)
    assert [r[0] for r in recs] == vals
    assert [r[1] for r in recs] == list(range(200))
    assert size.tolist() == [item_bytes(len(x)) for x in vals]


def test_overwrite_last_writer_wins_within_batch():
    s = make()
    s.set_many([b"/a", b"/b", b"/a", b"/a"], [b"1", b"2", b"3", b"4"])
    assert s.get_many([b"/a", b"/b"]) == [b"4", b"2"]
    c = s.counters()
    assert c["set_ops"] == 4 and c["set_dropped"] == 2
    s.set_many([b"/a"], [b"5"])
    assert s.get_many([b"/a"]) == [b"5"]


def test_miss_and_delete():
    s = make()
    s.set_many([b"/x", b"/y"], [b"xx", b"yy"])
    found = s.remove(digest_strings([b"/x", b"/nope"]))
    assert found.tolist() == [True, False]
    assert s.get_many([b"/x", b"/y"]) == [None, b"yy"]


def test_ttl_expiry_and_sweep():
    s = make()
    d = digest_strings([b"/t1", b"/t2"])
    v, vo, vl = pack_values([b"a", b"b"])
    now = 100
    s.store(d, v, vo, vl, expire=torch.tensor([105, 0], dtype=torch.int32), now=now)
    recs = unpack_records(*s.get(d, now=104))
    assert recs[0][0] == b"a" and recs[1][0] == b"b"
    recs = unpack_records(*s.get(d, now=105))
    assert recs[0] is None and recs[1][0] == b"b"
    live, _ = s.sweep(now=105)
    assert live == 1
    assert s.counters()["swept"] == 1


def test_fifo_log_eviction():
    # 64 KiB log, 1 KiB values: only the newest ~64 survive
    s = make(log=64 << 10, nb=1 << 8, max_item=4096)
    keys = [f"/e/{i}".encode() for i in range(300)]
    for i in range(0, 300, 10):
        s.set_many(keys[i : i + 10], [bytes([i % 256]) * 1000] * 10)
    got = s.get_many(keys)
    alive = [i for i, g in enumerate(got) if g is not None]
    assert alive, "nothing survived"
    assert min(alive) > 200 and max(alive) == 299
    assert all(got[i] == bytes([(i // 10 * 10) % 256]) * 1000 for i in alive)


def check_reserve_lookup_survives_queued_set(dev):
    """A lookup that reserves a SET's log bytes stays valid after that SET runs."""
    s = CacheShard(64 << 10, 1 << 8, 4096, dev)
    keys = [f"/r/{i}".encode() for i in range(60)]
    vals = [bytes([i]) * 1000 for i in range(60)]
    for i in range(0, 60, 10):
        s.set_many(keys[i : i + 10], vals[i : i + 10])
    d = digest_strings(keys, s.device)
    plain = s.lookup(d).hits().cpu()
    newk = [f"/n/{i}".encode() for i in range(12)]
    v, vo, vl = pack_values([b"x" * 1000] * 12, s.device)
    bound = s.set_bound(12, v.numel())
    lk = s.lookup(d, reserve_bytes=bound)
    res_hits = lk.hits().cpu()
    # the reserved lookup drops exactly the oldest objects (a prefix of the FIFO)
    assert res_hits.sum() < plain.sum()
    first = int(res_hits.nonzero()[0])
    assert not res_hits[:first].any() and res_hits[first:].all() and plain[first:].all()
    s.store(digest_strings(newk, s.device), v, vo, vl)   # overwrites the oldest objects
    out = s.gather(lk)
    recs = unpack_records(out, lk.off[: lk.n], lk.size[: lk.n])
    for i, r in enumerate(recs):
        assert (r is None) == (not bool(res_hits[i]))
        if r is not None:
            assert r[0] == vals[i]
    got = s.get_many(keys)
    assert sum(g is not None for g in got) >= int(res_hits.sum())  # the bound is conservative


def test_reserve_lookup_survives_queued_set():
    check_reserve_lookup_survives_queued_set("cpu")


def test_too_large_rejected():
    s = make(max_item=100)
    s.set_many([b"/big", b"/ok"], [b"z" * 101, b"z" * 100])
    assert s.get_many([b"/big", b"/ok"]) == [None, b"z" * 100]
    assert s.counters()["set_dropped"] == 1


def test_bucket_overflow_evicts_oldest():
    # 2 buckets x 4 entries = 8 slots: the 9th..20th keys must displace older ones
    s = make(log=1 << 20, nb=2, max_item=64)
    keys = [f"/o/{i}".encode() for i in range(20)]
    for k in keys:
        s.set_many([k], [k])
    got = s.get_many(keys)
    assert sum(g is not None for g in got) == 8
    assert got[-1] == keys[-1]
    assert s.counters()["set_evicted"] == 12


def test_flush():
    s = make()
    s.set_many([b"/f"], [b"v"])
    s.flush()
    assert s.get_many([b"/f"]) == [None]


def test_scan_and_segcopy_host():
    x = torch.tensor([16, 0, 32, 48], dtype=torch.int64)
    off = R.exclusive_scan(x)
    assert off.tolist() == [0, 16, 16, 48, 96]
    src = torch.arange(256, dtype=torch.int64).to(torch.uint8)
    src_off = torch.tensor([64, 0, 16, 128], dtype=torch.int64)
    dst = torch.zeros(96, dtype=torch.uint8)
    R.segcopy(src, src_off, off, dst)
    assert dst[:16].tolist() == list(range(64, 80))
    assert dst[16:48].tolist() == list(range(16, 48))
    assert dst[48:96].tolist() == list(range(128, 176))


def test_dram_backend_full_key_identity():
    """The DRAM tier stores each value with its key: a GET under another key's digest
    (a forged collision) misses instead of returning that object."""
    from shellac_amd import core

    be = core().dram_backend(16 << 20, 1 << 16, 4)
    be.set(b"/victim", b"private", 7, 0)
    assert be.get(b"/victim") == (b"private", 7)
    assert be.get_with_digest(b"/attacker", b"/victim") is None
    assert be.get_with_digest(b"/victim", b"/victim") == (b"private", 7)
    assert be.stats()["cache_key_mismatch"] == 1


def test_dram_object_cache_clock_keeps_read_objects():
    """The host tier evicts by bytes with CLOCK: an object read between fills survives
    a fill larger than the cache, unread ones of the same age do not."""
    import time as _t

    from shellac_amd import core

    be = core().dram_backend(1 << 20, 1 << 16, 1)  # 1 MiB, one stripe: exact CLOCK order
    be.set(b"/hot", b"h" * 2000, 0, 0)
    be.set(b"/cold", b"c" * 2000, 0, 0)
    for lap in range(4):
        assert be.get(b"/hot") is not None
        for i in range(200):
            be.set(b"/fill/%d/%d" % (lap, i), b"f" * 2000, 0, 0)
    assert be.get(b"/hot") == (b"h" * 2000, 0)
    assert be.get(b"/cold") is None
    st = be.stats()
    assert st["cache_evicted"] > 0 and st["cache_bytes"] <= (1 << 20)
    # TTL: expired objects read as misses
    be.set(b"/ttl", b"t", 0, 1)
    assert be.get(b"/ttl") == (b"t", 0)
    _t.sleep(2.1)
    assert be.get(b"/ttl") is None


def test_dram_hit_is_shared_not_copied():
    """Two hits of the same object return the same bytes (the tier hands out references
    to one immutable object) and a later SET replaces it without touching them."""
    from shellac_amd import core

    be = core().dram_backend(16 << 20, 1 << 16, 4)
    be.set(b"/obj", b"v1" * 100, 0, 0)
    a = be.get(b"/obj")
    be.set(b"/obj", b"v2" * 100, 0, 0)
    assert a == (b"v1" * 100, 0) and be.get(b"/obj") == (b"v2" * 100, 0)
    assert be.delete(b"/obj") is True and be.get(b"/obj") is None


def test_tiered_promotes_small_objects_only():
    """L2 hits are copied into the L1 up to promote_max bytes; larger objects keep being
    served by the L2 (no L1 churn, no copy)."""
    from shellac_amd import core

    c = core()
    l1 = c.dram_backend(16 << 20, 1 << 20, 4)
    l2 = c.dram_backend(64 << 20, 1 << 20, 4)
    t = c.tiered_backend(l1, l2, 60, 1024)
    l2.set(b"/small", b"s" * 100, 0, 0)
    l2.set(b"/big", b"b" * 5000, 0, 0)
    assert t.get(b"/small") == (b"s" * 100, 0)
    assert t.get(b"/big") == (b"b" * 5000, 0)
    assert l1.get(b"/small") == (b"s" * 100, 0) and l1.get(b"/big") is None
    st = t.stats()
    assert st["tier_promoted"] == 1 and st["tier_not_promoted_large"] == 1
