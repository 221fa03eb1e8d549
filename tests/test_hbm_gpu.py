"""HIP kernels vs the host (DRAM) engine / plain PyTorch references. GPU only."""
import dataclasses

import numpy as np

import pytest
import torch

from shellac_amd.ops.cache import (CacheShard, digest_packed, digest_strings, item_bytes,
                                   pack_values, unpack_records)
from shellac_amd.ops import routing as R

pytestmark = pytest.mark.gpu


def _pair(log=1 << 24, nb=1 << 12, max_item=1 << 16, dev=None):
    return CacheShard(log, nb, max_item, dev), CacheShard(log, nb, max_item, "cpu")


def _batch(keys, vals, dev):
    d = digest_strings(keys)
    v, vo, vl = pack_values(vals)
    return d, v, vo, vl


def _get_both(g, h, keys, now):
    d = digest_strings(keys)
    og, offg, sg = g.get(d.to(g.device), now=now)
    oh, offh, sh = h.get(d, now=now)
    return unpack_records(og, offg, sg), unpack_records(oh, offh, sh), sg.cpu(), sh


def test_native_extension_is_loaded(core):
    import shellac_amd

    assert core.device_count() >= 1
    assert core.__file__.startswith(shellac_amd.__path__[0])


def test_roundtrip_matches_host_engine(cuda_dev):
    g, h = _pair(dev=cuda_dev)
    rng = np.random.default_rng(0)
    keys = [f"/obj/{i}".encode() for i in range(3000)]
    vals = [rng.integers(0, 256, size=int(rng.integers(0, 5000)), dtype=np.uint8).tobytes()
            for _ in keys]
    d, v, vo, vl = _batch(keys, vals, cuda_dev)
    fl = torch.arange(len(keys), dtype=torch.int32)
    now = 10
    g.store(d.to(cuda_dev), v.to(cuda_dev), vo.to(cuda_dev), vl.to(cuda_dev), fl.to(cuda_dev), now=now)
    h.store(d, v, vo, vl, fl, now=now)
    probe = keys + [f"/miss/{i}".encode() for i in range(500)]
    rg, rh, sg, sh = _get_both(g, h, probe, now)
    assert torch.equal(sg, sh)
    assert rg == rh
    assert [r[0] for r in rg[:3000]] == vals
    assert g.head() == h.head()
    cg, ch = g.counters(), h.counters()
    for k in ("get_ops", "get_hits", "get_bytes", "set_ops", "set_bytes", "set_dropped"):
        assert cg[k] == ch[k], k


def test_duplicate_keys_in_batch_last_wins(cuda_dev):
    g, h = _pair(dev=cuda_dev)
    keys = [b"/dup"] * 50 + [f"/u/{i}".encode() for i in range(50)] + [b"/dup", b"/u/3"]
    vals = [f"v{i}".encode() * (i + 1) for i in range(len(keys))]
    d, v, vo, vl = _batch(keys, vals, cuda_dev)
    g.store(d.to(cuda_dev), v.to(cuda_dev), vo.to(cuda_dev), vl.to(cuda_dev), now=1)
    h.store(d, v, vo, vl, now=1)
    rg, rh, _, _ = _get_both(g, h, [b"/dup", b"/u/3", b"/u/4"], 1)
    assert rg == rh
    assert rg[0][0] == vals[100] and rg[1][0] == vals[101]


def test_many_batches_fifo_eviction_matches_host(cuda_dev):
    g, h = _pair(log=1 << 20, nb=1 << 14, max_item=1 << 14, dev=cuda_dev)
    rng = np.random.default_rng(1)
    allkeys = [f"/f/{i}".encode() for i in range(6000)]
    for b in range(24):
        ks = [allkeys[j] for j in rng.integers(0, len(allkeys), size=200)]
        vs = [rng.integers(0, 256, size=int(rng.integers(1, 3000)), dtype=np.uint8).tobytes()
              for _ in ks]
        d, v, vo, vl = _batch(ks, vs, cuda_dev)
        g.store(d.to(cuda_dev), v.to(cuda_dev), vo.to(cuda_dev), vl.to(cuda_dev), now=5)
        h.store(d, v, vo, vl, now=5)
    assert g.head() == h.head() and g.head() > (1 << 20)  # the log wrapped
    rg, rh, sg, sh = _get_both(g, h, allkeys, 5)
    assert rg == rh
    assert sum(r is not None for r in rg) > 100


def test_ttl_delete_sweep(cuda_dev):
    g, h = _pair(dev=cuda_dev)
    keys = [f"/t/{i}".encode() for i in range(1000)]
    d, v, vo, vl = _batch(keys, [b"x" * 33] * 1000, cuda_dev)
    ex = torch.tensor([0 if i % 3 == 0 else 50 + i % 7 for i in range(1000)], dtype=torch.int32)
    for s, dv in ((g, cuda_dev), (h, "cpu")):
        s.store(d.to(dv), v.to(dv), vo.to(dv), vl.to(dv), expire=ex.to(dv), now=40)
    fg = g.remove(d[:100].to(cuda_dev), now=40).cpu()
    fh = h.remove(d[:100], now=40)
    assert torch.equal(fg, fh) and bool(fg.all())
    for now in (40, 52, 54, 60):
        rg, rh, _, _ = _get_both(g, h, keys, now)
        assert rg == rh, now
    assert g.sweep(now=54) == h.sweep(now=54)


@pytest.mark.parametrize("evict", ["clock", "fifo"])
def test_small_set_kernel_matches_host_engine(cuda_dev, evict):
    """SET batches of <= 256 rows run as one fused kernel (k_set_small); batches above
    run the launched chain. Over a log that wraps many times — duplicates, skip rows,
    values above max_item, TTLs, CLOCK reinsertions fed by the ring entries the fused
    kernel appends — both engines end with the same head, records and counters."""
    from shellac_amd.models.sharded_cache import SKIP_VLEN

    g = CacheShard(1 << 21, 1 << 10, 1 << 11, cuda_dev, evict=evict)
    h = CacheShard(1 << 21, 1 << 10, 1 << 11, "cpu", evict=evict)
    rng = np.random.default_rng(7)
    allkeys = [f"/ss/{i}".encode() for i in range(3000)]
    for b in range(60):
        n = int(rng.choice([1, 5, 64, 255, 256, 257, 600]))
        ks = [allkeys[j] for j in rng.integers(0, 3000, size=n)]
        vs = [rng.integers(0, 256, size=int(rng.integers(0, 2600)), dtype=np.uint8).tobytes()
              for _ in ks]  # some above max_item (2 KiB): dropped
        d, v, vo, vl = _batch(ks, vs, cuda_dev)
        vl[::9] = SKIP_VLEN
        ex = torch.tensor([0 if i % 4 else 30 + i % 5 for i in range(n)], dtype=torch.int32)
        for s, dv in ((g, cuda_dev), (h, "cpu")):
            s.store(d.to(dv), v.to(dv), vo.to(dv), vl.to(dv), expire=ex.to(dv), now=20 + b // 8)
        if b % 5 == 4:  # reads set CLOCK bits: later hands reinsert those items
            _get_both(g, h, allkeys[:1500:3], 20 + b // 8)
    assert g.head() == h.head() and g.head() > (4 << 20)  # the log wrapped twice
    for now in (25, 40):
        rg, rh, sg, sh = _get_both(g, h, allkeys, now)
        assert torch.equal(sg, sh) and rg == rh
    cg, ch = g.counters(), h.counters()
    for k in ("set_ops", "set_bytes", "set_dropped", "set_evicted", "reinserted"):
        assert cg[k] == ch[k], k


def test_bucket_overflow_eviction_invariants(cuda_dev):
    g = CacheShard(1 << 20, 2, 64, cuda_dev)  # 8 slots total
    keys = [f"/o/{i}".encode() for i in range(20)]
    for k in keys:  # one key per batch: deterministic order
        g.set_many([k], [k])
    got = g.get_many(keys)
    assert sum(x is not None for x in got) == 8
    assert got[-1] == keys[-1]
    assert g.counters()["set_evicted"] == 12


def test_digest_kernel_matches_host(cuda_dev):
    keys = [f"/digest/{i}/".encode() * (i % 9) for i in range(777)]
    from shellac_amd.ops.cache import pack_bytes

    buf, offs = pack_bytes(keys)
    bt = torch.from_numpy(np.concatenate([buf, np.zeros(1, np.uint8)])).to(cuda_dev)
    ot = torch.from_numpy(offs).to(cuda_dev)
    assert torch.equal(digest_packed(bt, ot).cpu(), digest_strings(keys))


def test_routing_kernels_match_host(cuda_dev):
    from shellac_amd.parallel.ring import ShardRing

    ring = ShardRing(list(range(8)))
    keys = digest_strings([f"/route/{i}".encode() for i in range(20000)])
    pts, own = ring.tensors("cpu")
    dh, ch = R.route(keys, pts, own, 8)
    pg, og = ring.tensors(cuda_dev)
    dg, cgt = R.route(keys.to(cuda_dev), pg, og, 8)
    assert torch.equal(dg.cpu(), dh) and torch.equal(cgt.cpu(), ch)
    perm = R.scatter_positions(dg, cgt)
    assert sorted(perm.cpu().tolist()) == list(range(20000))
    grouped = R.permute(keys.to(cuda_dev), perm)
    gd = R.permute(dg.view(-1, 1), perm).view(-1)
    assert bool((gd[1:] >= gd[:-1]).all())
    assert torch.equal(grouped.index_select(0, perm).cpu(), keys)


def test_scan_and_segcopy_kernels(cuda_dev):
    g = torch.Generator().manual_seed(3)
    n = 50000
    sizes = (torch.randint(0, 200, (n,), generator=g) * 16) * (torch.rand(n, generator=g) > 0.3)
    off_h = R.exclusive_scan(sizes)
    off_d = R.exclusive_scan(sizes.to(cuda_dev))
    assert torch.equal(off_h, off_d.cpu())
    src = torch.randint(0, 256, (1 << 22,), generator=g, dtype=torch.uint8)
    src_off = (torch.randint(0, (1 << 22) - 4096, (n,), generator=g) // 16) * 16
    total = int(off_h[-1])
    dh = torch.zeros(total, dtype=torch.uint8)
    R.segcopy(src, src_off, off_h, dh)
    dd = torch.zeros(total, dtype=torch.uint8, device=cuda_dev)
    R.segcopy(src.to(cuda_dev), src_off.to(cuda_dev), off_d, dd)
    assert torch.equal(dh, dd.cpu())


def test_mfma_hello_matches_fp32_reference(cuda_dev):
    from shellac_amd.ops.smoke import mfma_hello

    a = torch.randn(16, 32, 16, device=cuda_dev).to(torch.bfloat16)
    # asymmetric B catches a transposed C write
    b = (torch.arange(16 * 32, device=cuda_dev, dtype=torch.float32).view(16, 32) / 97.0)
    b = (b.unsqueeze(0).repeat(16, 1, 1) + torch.randn(16, 16, 32, device=cuda_dev)).to(torch.bfloat16)
    c = mfma_hello(a, b)
    ref = torch.bmm(a.float(), b.float())
    torch.testing.assert_close(c, ref, atol=1e-3, rtol=1e-4)


def test_sharded_cache_single_rank_gpu(cuda_dev):
    from shellac_amd.bench.workload import Workload
    from shellac_amd.models.sharded_cache import ShardedCache

    wl = Workload(20000, cuda_dev, pool_bytes=1 << 20)
    shard = CacheShard(1 << 26, 1 << 14, 1 << 16, cuda_dev)
    sc = ShardedCache(shard)
    sc.set(wl.set_batch(torch.arange(20000, device=cuda_dev)))
    ids = wl.sample_ids(5000, 9)
    res = sc.get(wl.digests.index_select(0, ids).contiguous())
    recs = unpack_records(res.data, res.off, res.size)
    for i, r in zip(ids.tolist()[:500], recs[:500]):
        assert r is not None and r[0] == wl.expected_value(i)


def test_export_keys_and_snapshot_roundtrip(cuda_dev, tmp_path):
    g, h = _pair(log=1 << 22, nb=1 << 12, dev=cuda_dev)
    keys = [f"/snap/{i}".encode() for i in range(3000)]
    vals = [bytes([i % 251]) * (i % 700) for i in range(3000)]
    d, v, vo, vl = _batch(keys, vals, cuda_dev)
    g.store(d.to(cuda_dev), v.to(cuda_dev), vo.to(cuda_dev), vl.to(cuda_dev), now=3)
    h.store(d, v, vo, vl, now=3)
    g.remove(d[:100].to(cuda_dev), now=3)
    h.remove(d[:100], now=3)
    eg = {tuple(r) for r in g.export_keys(now=3).cpu().tolist()}
    eh = {tuple(r) for r in h.export_keys(now=3).tolist()}
    assert eg == eh and len(eg) == 2900
    path = str(tmp_path / "gpu.snap")
    g.save(path)
    g2 = CacheShard(1 << 22, 1 << 12, 1 << 16, cuda_dev)
    g2.load(path)
    rg, _, _, _ = _get_both(g2, h, keys, 3)
    assert [r[0] if r else None for r in rg] == [None] * 100 + vals[100:]


def test_reserve_lookup_survives_queued_set_gpu(cuda_dev):
    from test_cache_semantics import check_reserve_lookup_survives_queued_set

    check_reserve_lookup_survives_queued_set(cuda_dev)


@pytest.mark.parametrize("side_stream", [True, False])
def test_serve_overlapped_matches_get_then_set(cuda_dev, side_stream):
    """serve() (reserved lookup; SET chain on a side stream concurrently with the
    gather, or in stream order) returns what get() then set() returns."""
    from shellac_amd.bench.workload import Workload
    from shellac_amd.models.sharded_cache import ShardedCache

    wl = Workload(20000, cuda_dev)
    outs = []
    for mode in ("serve", "seq"):
        sc = ShardedCache(CacheShard(256 << 20, 1 << 14, 1 << 16, cuda_dev))
        sc.overlap_store = side_stream
        for s0 in range(0, 20000, 5000):
            sc.set(wl.set_batch(torch.arange(s0, s0 + 5000, device=cuda_dev)))
        keys = wl.digests.index_select(0, wl.sample_ids(4096, 3)).contiguous()
        sb = wl.set_batch(wl.uniform_ids(2048, 4))
        if mode == "serve":
            r = sc.serve(keys, sb)
        else:
            r = sc.get(keys)
            sc.set(sb)
        outs.append((r.size.cpu(), unpack_records(r.data, r.off, r.size)))
        after = sc.get(keys)
        outs.append((after.size.cpu(),))
    (s1, d1), (a1,), (s2, d2), (a2,) = outs
    # the reserved lookup may miss objects the SET could evict, never hit more
    hit1, hit2 = s1 > 0, s2 > 0
    assert not (hit1 & ~hit2).any()
    assert hit1.float().mean() > 0.5
    assert torch.equal(a1, a2)
    ids = wl.sample_ids(4096, 3).cpu()
    for i in range(0, 4096, 97):
        if hit1[i]:
            assert d1[i][0] == wl.expected_value(int(ids[i]))


@pytest.mark.parametrize("n", [1, 5, 17, 255, 2049, 40001, 300007])
def test_lookup_offsets_fused_scan(cuda_dev, n):
    """k_probe's per-workgroup partials + k_offsets == exclusive cumsum of sizes."""
    shard = CacheShard(64 << 20, 1 << 18, 1 << 12, cuda_dev)
    g = torch.Generator().manual_seed(n)
    keys = torch.randint(-2**62, 2**62, (n, 2), generator=g, dtype=torch.int64)
    vl = torch.randint(0, 200, (n,), generator=g, dtype=torch.int32)
    store = torch.rand(n, generator=g) < 0.6
    ks = keys[store].contiguous().to(cuda_dev)
    vls = vl[store].contiguous()
    vo = torch.cumsum(torch.cat([torch.zeros(1, dtype=torch.int64), vls.long()]), 0)[:-1]
    pay = torch.zeros(int(vls.sum()) + 16, dtype=torch.uint8, device=cuda_dev)
    if ks.shape[0]:
        shard.store(ks, pay, vo.contiguous().to(cuda_dev), vls.to(cuda_dev))
    lk = shard.lookup(keys.to(cuda_dev))
    size = lk.size[:n].cpu()
    assert torch.equal(size > 0, store)
    ref = torch.cumsum(torch.cat([torch.zeros(1, dtype=torch.int64), size]), 0)
    assert torch.equal(lk.off.cpu(), ref)
    # the kernel-written host slot carries the same total without a D2H copy
    shard.lookup(keys.to(cuda_dev), total_slot=3)
    assert shard.host_total(3) == int(ref[-1])


@pytest.mark.parametrize("world", [2, 4, 8])
def test_fused_routed_step_matches_framework_ops(cuda_dev, world):
    """The fused native routed step (csrc/router.hip) returns exactly what the
    framework-op version returns, on one GPU with mirrored all-to-alls."""
    from shellac_amd.bench.workload import Workload
    from shellac_amd.models.sharded_cache import ShardedCache
    from shellac_amd.parallel.exchange import MirrorComm

    wl = Workload(40000, cuda_dev)
    outs = []
    # (fused, coalesce, inputs-ready event): steps after the first (calibrating) one run
    # the native executor (RoutedStep::step); with the event its plan is pipelined
    for fused, co, ready in ((False, False, False), (True, False, False), (True, True, False),
                             (True, True, True)):
        sc = ShardedCache(CacheShard(256 << 20, 1 << 16, 1 << 16, cuda_dev), group=MirrorComm(world),
                          replica=CacheShard(64 << 20, 1 << 12, 1 << 16, cuda_dev))
        sc.fused = fused
        sc.coalesce = co
        for s0 in range(0, 40000, 10000):
            sc.set(wl.set_batch(torch.arange(s0, s0 + 10000, device=cuda_dev)))
        sc.refresh_replica(2000, keys=wl.digests.index_select(0, wl.sample_ids(50000, 1)))
        keys = wl.digests.index_select(0, wl.sample_ids(8192, 2)).contiguous()
        batches = [wl.set_batch(wl.uniform_ids(1024, 10 + step)) for step in range(4)]
        ev = None
        if ready:
            ev = torch.cuda.Event()
            ev.record()
        got, pend = [], []
        for step in range(4):
            pend.append(sc.serve(keys, batches[step], inputs_ready=ev))
        for r in pend:  # results stay valid while later steps run
            r.wait()
            got.append([None if x is None else x[0]
                        for x in unpack_records(r.data, r.off, r.size)])
        outs.append((got, dict(sc.stats), sc._engine.early_sets if sc._engine else 0))
    (g0, s0, e0), (g1, s1, e1), (g2, s2, e2), (g3, s3, e3) = outs
    assert g0 == g1
    assert s0 == s1
    assert g3 == g2 and s3 == s2
    # the native steps after the first two ran their SET appends early (look-ahead)
    assert e1 >= 1 and e2 >= 1 and e3 >= 1
    assert sum(v is not None for v in g1[0]) == 8192     # every GET hits
    assert s1["replica_hits"] > 0
    # coalesced: the same values; duplicates neither probed nor sent
    assert g2 == g1
    assert s2["coalesced_gets"] > 0 and s2["remote_gets"] < s1["remote_gets"]
    assert 0 < s2["replica_hits"] < s1["replica_hits"]


def test_routed_step_slot_overflow_is_a_counted_miss(cuda_dev):
    """Fixed-capacity exchange: GET rows past a peer slot's capacity and replies past its
    data capacity come back as misses (never wrong data) and are counted; with the
    capacities the executor learns from the observed demand, the next steps are exact."""
    from shellac_amd.bench.workload import Workload
    from shellac_amd.models.sharded_cache import ShardedCache
    from shellac_amd.parallel.exchange import MirrorComm

    wl = Workload(30000, cuda_dev)
    sc = ShardedCache(CacheShard(256 << 20, 1 << 16, 1 << 16, cuda_dev), group=MirrorComm(3),
                      replica=CacheShard(64 << 20, 1 << 12, 1 << 16, cuda_dev))
    sc.set(wl.set_batch(torch.arange(0, 30000, device=cuda_dev)))
    ids = wl.sample_ids(6000, 3)
    keys = wl.digests.index_select(0, ids).contiguous()
    expect = [wl.expected_value(i) for i in ids.tolist()]

    def step(k):
        r = sc.serve(keys, wl.set_batch(wl.uniform_ids(256, 20 + k))).wait()
        return [None if x is None else x[0] for x in unpack_records(r.data, r.off, r.size)]

    got = step(0)  # calibrating step: exact capacities
    assert got == expect
    assert sc.stats["slot_overflow_rows"] == 0
    e = sc._engine
    for cap_g, cap_d in ((64, 1 << 20), (1 << 14, 64 << 10)):  # full GET slots, full replies
        e.set_cap_override(cap_g, cap_d, 8 << 20)
        before = dict(sc.stats)
        got = step(1)
        wrong = [i for i, (g, w) in enumerate(zip(got, expect)) if g is not None and g != w]
        misses = sum(g is None for g in got)
        assert not wrong and misses > 0
        if cap_g == 64:
            assert sc.stats["slot_overflow_rows"] > before["slot_overflow_rows"]
    e.set_cap_override(0, 0, 0)
    step(2)  # the dropped replies of the last forced step are reported one step later
    assert sc.stats["reply_dropped_rows"] > 0
    for k in range(3, 5):
        assert step(k) == expect  # learned capacities: exact again


@pytest.mark.parametrize("comm_mode", ["single", "channels"])
def test_routed_step_set_overflow_is_carried_not_lost(cuda_dev, comm_mode):
    """Fixed-capacity SET slots: rows past a slot's capacity (records or value bytes, to a
    peer or to this rank's own store) are carried into the next step, never dropped. With
    forced tiny SET slots the carry is exercised, and once the capacities are learned again
    every SET of the forced steps is stored within two steps (ground truth for each key)."""
    from shellac_amd.bench.workload import Workload
    from shellac_amd.models.sharded_cache import ShardedCache
    from shellac_amd.parallel.exchange import MirrorComm

    wl = Workload(30000, cuda_dev)
    sc = ShardedCache(CacheShard(256 << 20, 1 << 16, 1 << 16, cuda_dev), group=MirrorComm(3),
                      replica=CacheShard(64 << 20, 1 << 12, 1 << 16, cuda_dev), comm_mode=comm_mode)
    sc.set(wl.set_batch(torch.arange(0, 30000, device=cuda_dev)))
    gets = wl.digests.index_select(0, wl.sample_ids(4000, 3)).contiguous()
    empty = wl.set_batch(torch.zeros(0, dtype=torch.int64, device=cuda_dev))
    sc.serve(gets, empty).wait()  # calibrating step
    sc.serve(gets, empty).wait()
    e = sc._engine
    e.set_set_cap_override(64, 96 << 10, 64, 96 << 10)
    # new values for 1500 keys over two forced steps (different bytes from the fill: the
    # workload's version 1)
    ids = [torch.arange(1000 + 1500 * k, 1000 + 1500 * k + 750, device=cuda_dev) for k in (0, 1)]
    for k in (0, 1):
        b = wl.set_batch(ids[k], version=1)
        sc.serve(gets, b).wait()
    carried, cbytes, lost = e.carry_stats()
    assert carried > 0 and cbytes > 0 and lost == 0
    e.set_set_cap_override(0, 0, 0, 0)
    for _ in range(2):
        sc.serve(gets, empty).wait()
    sc.sync_sets()
    allids = torch.cat(ids)
    r = sc.get(wl.digests.index_select(0, allids).contiguous())
    got = [None if x is None else x[0] for x in unpack_records(r.data, r.off, r.size)]
    want = [wl.expected_value(i, version=1) for i in allids.tolist()]
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, (len(bad), bad[:5])
    assert e.carry_stats()[2] == 0


def test_routed_comm_modes_give_identical_results(cuda_dev):
    """`comm_mode="single"` (every collective of a step on one stream, in issue order) and
    the default `"channels"` (three communicator channels on their own streams) are the
    same step: from identical caches, the same GET / SET batches give byte-identical
    answers every step (hot-replica fan-out included), and the caches end identical."""
    from shellac_amd.bench.workload import Workload
    from shellac_amd.models.sharded_cache import ShardedCache
    from shellac_amd.parallel.exchange import MirrorComm

    wl = Workload(40000, cuda_dev)
    caches = {}
    for mode in ("channels", "single"):
        sc = ShardedCache(CacheShard(256 << 20, 1 << 16, 1 << 16, cuda_dev), group=MirrorComm(3),
                          replica=CacheShard(64 << 20, 1 << 12, 1 << 16, cuda_dev),
                          comm_mode=mode)
        sc.set(wl.set_batch(torch.arange(0, 40000, device=cuda_dev)))
        sc.sync_sets()
        caches[mode] = sc
    outs = {m: [] for m in caches}
    for k in range(6):
        gets = wl.digests.index_select(0, wl.sample_ids(5000, 10 + k)).contiguous()
        sets = wl.set_batch(wl.uniform_ids(600, 30 + k), version=1 + k % 2)
        for m, sc in caches.items():
            r = sc.serve(gets, sets).wait()
            outs[m].append(unpack_records(r.data, r.off, r.size))
        if k == 2:  # from here on the hottest keys are also answered from the replica tier
            for sc in caches.values():
                sc.refresh_replica(256, gets)
    for k in range(6):
        assert outs["channels"][k] == outs["single"][k], k
        assert sum(x is not None for x in outs["channels"][k]) > 4000
    allk = wl.digests[:40000].contiguous()
    final = {}
    for m, sc in caches.items():
        sc.sync_sets()
        r = sc.get(allk)
        final[m] = unpack_records(r.data, r.off, r.size)
    assert final["channels"] == final["single"]


@pytest.mark.parametrize("n,nb", [(1, 2), (777, 3), (100003, 9), (300000, 65)])
def test_group_rows_counting_sort(cuda_dev, n, nb):
    """csrc/router.hip counting sort: bucket counts, a permutation, rows moved with it,
    every bucket contiguous and in bucket order."""
    from shellac_amd._native import core

    c = core()
    g = torch.Generator(device=cuda_dev).manual_seed(n)
    dest = torch.randint(0, nb, (n,), generator=g, device=cuda_dev, dtype=torch.int32)
    rows = torch.randint(-2**62, 2**62, (n, 2), generator=g, device=cuda_dev)
    out = torch.empty_like(rows)
    perm = torch.empty(n, dtype=torch.int64, device=cuda_dev)
    counts = torch.empty(nb, dtype=torch.int64, device=cuda_dev)
    ws = torch.empty(c.group_ws_words(n, nb), dtype=torch.int64, device=cuda_dev)
    st = torch.cuda.current_stream(cuda_dev).cuda_stream
    c.group_rows(dest.data_ptr(), n, nb, rows.data_ptr(), 16, out.data_ptr(), perm.data_ptr(),
                 counts.data_ptr(), ws.data_ptr(), st)
    assert torch.equal(counts.cpu(), torch.bincount(dest.long().cpu(), minlength=nb))
    assert torch.equal(torch.sort(perm).values.cpu(), torch.arange(n))
    assert torch.equal(out[perm], rows)
    starts = torch.cumsum(counts, 0) - counts
    grouped = torch.empty_like(dest)
    grouped[perm] = dest
    expect = torch.repeat_interleave(torch.arange(nb, device=cuda_dev, dtype=torch.int32), counts)
    assert torch.equal(grouped, expect)
    assert int(starts[0]) == 0


def test_fused_routed_step_edge_cases(cuda_dev):
    """Empty GET / SET batches, SET skip rows and an all-replica GET batch take the same
    path through the native executor and the framework-op version."""
    from shellac_amd.bench.workload import Workload
    from shellac_amd.models.sharded_cache import SKIP_VLEN, SetBatch, ShardedCache
    from shellac_amd.parallel.exchange import MirrorComm

    wl = Workload(20000, cuda_dev)
    empty_keys = torch.zeros((0, 2), dtype=torch.int64, device=cuda_dev)
    results = []
    for fused in (False, True):
        sc = ShardedCache(CacheShard(512 << 20, 1 << 15, 1 << 16, cuda_dev), group=MirrorComm(3),
                          replica=CacheShard(128 << 20, 1 << 12, 1 << 16, cuda_dev))
        sc.fused = fused
        sc.set(wl.set_batch(torch.arange(0, 20000, device=cuda_dev)))
        hot = wl.digests[:500].contiguous()
        sc.refresh_replica(500, keys=hot)
        sb = wl.set_batch(wl.uniform_ids(300, 5))
        sb.vlen[::7] = SKIP_VLEN
        empty_sb = SetBatch(empty_keys, sb.values, sb.val_off[:0].contiguous(),
                            sb.vlen[:0].contiguous())
        got = []
        for keys, batch in ((empty_keys, sb), (hot, empty_sb), (hot, sb),
                            (wl.digests[:4000].contiguous(), empty_sb)):
            sc.recalibrate()  # batch shapes jump between steps: measure each one exactly
            r = sc.serve(keys, batch).wait()
            got.append(([None if x is None else x[0]
                          for x in unpack_records(r.data, r.off, r.size)]))
        results.append((got, dict(sc.stats)))
    assert results[0] == results[1]
    # the same steps through the native executor (RoutedStep::step) every time: fixed
    # capacities large enough for every shape, so no step calibrates
    sc = ShardedCache(CacheShard(512 << 20, 1 << 15, 1 << 16, cuda_dev), group=MirrorComm(3),
                      replica=CacheShard(128 << 20, 1 << 12, 1 << 16, cuda_dev))
    sc.set(wl.set_batch(torch.arange(0, 20000, device=cuda_dev)))
    sc.refresh_replica(500, keys=hot)
    sc.serve(hot, empty_sb).wait()  # builds the executor
    sc._engine.set_cap_override(4096, 32 << 20, 16 << 20)
    got = []
    for keys, batch in ((empty_keys, sb), (hot, empty_sb), (hot, sb),
                        (wl.digests[:4000].contiguous(), empty_sb)):
        r = sc.serve(keys, batch).wait()
        got.append(([None if x is None else x[0] for x in unpack_records(r.data, r.off, r.size)]))
    assert got == results[0][0]
    assert all(v is not None for v in results[1][0][1])  # hot keys all served


@pytest.mark.parametrize("n", [0, 1, 31, 32, 33, 100, 777, 2048, 5000, 70000])
def test_small_get_matches_lookup_gather(cuda_dev, n):
    """The one-launch edge GET (decoupled look-back across workgroups) returns the same
    bytes and offsets as lookup + gather at every batch size, including ranges that
    straddle workgroups, and reports the full size when the capacity is too small."""
    shard = CacheShard(64 << 20, 1 << 14, 1 << 14, cuda_dev)
    keys = [f"/small/{i}".encode() for i in range(3000)]
    vals = [bytes([i % 251]) * (i * 13 % 3000) for i in range(3000)]
    shard.set_many(keys[:2000], vals[:2000])
    req = digest_strings([keys[(i * 7) % 3000] for i in range(n)], cuda_dev)
    lk = shard.lookup(req)
    ref = shard.gather(lk)
    out, off = shard.small_get(req, out_cap=max(int(lk.off[-1]), 16))
    assert torch.equal(off.cpu(), lk.off.cpu())
    total = int(off[-1])
    assert torch.equal(out[:total].cpu(), ref[:total].cpu())
    if total > 64:
        # too small a buffer: offsets still complete, nothing written past the capacity
        out2, off2 = shard.small_get(req, out_cap=total - 16)
        assert int(off2[-1]) == total
        out3, off3 = shard.small_get(req, out_cap=0)
        assert int(off3[-1]) == total


@pytest.mark.parametrize("n", [1, 64, 2048, 9000])
def test_small_get_completion_slot(cuda_dev, n):
    """With a done slot, the host learns the batch finished from the pinned slot (the
    last workgroup's system-scope store) and may read the output without a stream
    sync; repeated launches reuse the self-resetting workgroup counter."""
    shard = CacheShard(64 << 20, 1 << 14, 1 << 14, cuda_dev)
    keys = [f"/done/{i}".encode() for i in range(3000)]
    vals = [bytes([i % 251]) * (16 + i * 13 % 3000) for i in range(3000)]
    shard.set_many(keys[:2500], vals[:2500])
    torch.cuda.synchronize()
    for rep in range(3):
        idx = [(i * 7 + rep) % 3000 for i in range(n)]
        req = digest_strings([keys[i] for i in idx], cuda_dev)
        torch.cuda.synchronize()
        out, off = shard.small_get(req, done_slot=5)
        total = shard.host_total(5)  # spins on the slot; no torch.cuda.synchronize()
        assert total == int(off[-1])
        got = unpack_records(out, off[:-1], off[1:] - off[:-1])
        for i, g in zip(idx, got):
            assert (g is None) == (i >= 2500)
            if g is not None:
                assert g[0] == vals[i]


@pytest.mark.parametrize("n", [1, 7, 16, 29])
def test_serve_get_matches_small_get(cuda_dev, n):
    """The resident edge server answers a job with exactly the launched edge GET's bytes
    and offsets (misses and duplicates included, records over several copy rounds), reports the full
    size without writing when the buffer is too small, and rejects batches above
    SERVE_KEYS so the caller falls back to a launch."""
    from shellac_amd._native import core

    shard = CacheShard(64 << 20, 1 << 14, 1 << 14, cuda_dev)
    keys = [f"/srv/{i}".encode() for i in range(3000)]
    vals = [bytes([i % 251]) * (i * 13 % 3000) for i in range(3000)]
    shard.set_many(keys[:2000], vals[:2000])
    torch.cuda.synchronize()
    for rep in range(3):  # jobs back to back on the same resident kernel
        req = digest_strings([keys[(i * 7 + rep) % 3000] for i in range(n)], "cpu")
        out, off = shard.small_get(req.to(cuda_dev), out_cap=8 << 20)
        torch.cuda.synchronize()
        got = shard.serve_get(req, out_cap=8 << 20)
        assert got is not None
        out2, off2 = got
        assert torch.equal(off2.cpu(), off.cpu())
        total = int(off[-1])
        assert torch.equal(out2[:total].cpu(), out[:total].cpu())
    if total > 64:
        out3, off3 = shard.serve_get(req, out_cap=total - 16)
        assert int(off3[-1]) == total and int(out3.count_nonzero()) == 0
    big = digest_strings(keys[:int(core().SERVE_KEYS) + 1], "cpu")
    assert shard.serve_get(big) is None


@pytest.mark.parametrize("blocks", [1, 4, 8])
def test_serve_blocks_answer_concurrent_submitters(cuda_dev, blocks):
    """Several resident server blocks: ticket T goes to block T % blocks. Eight host
    threads (the proxy's reactors) submit small jobs with slots of their own, interleaved;
    every job is answered with its own keys' records, whichever block took it."""
    import threading

    shard = CacheShard(64 << 20, 1 << 14, 1 << 14, cuda_dev, serve_blocks=blocks)
    assert shard._impl.serve_blocks == blocks
    keys = [f"/blk/{i}".encode() for i in range(2000)]
    vals = [bytes([i % 251 + 1]) * (64 + i * 7 % 4000) for i in range(2000)]
    shard.set_many(keys, vals)   # (the jobs are ordered after it on the null stream)
    errors = []

    def worker(t):
        # the zero fills are queued on this thread's current stream and not waited for:
        # serve_get orders the job after them (a fill landing after the server wrote a
        # job's answer would wipe it)
        out = torch.zeros(1 << 18, dtype=torch.uint8, device=cuda_dev)
        off = torch.zeros(32, dtype=torch.int64, device=cuda_dev)
        stream = torch.cuda.current_stream(cuda_dev).cuda_stream
        slot = 20 + t
        try:
            for j in range(150):
                n = 1 + (t + j) % 5
                ids = [(t * 331 + j * 17 + k * 101) % 2000 for k in range(n)]
                dh = digest_strings([keys[i] for i in ids], "cpu").contiguous()
                while not shard._impl.serve_get(dh.data_ptr(), n, out.data_ptr(), out.numel(),
                                                off.data_ptr(), shard.now(), slot, stream):
                    pass  # this block's ring is full: retry
                total = shard._impl.serve_wait(slot, 10000)
                o, f = out[:total].cpu(), off[:n + 1].cpu()
                got = unpack_records(o, f[:-1], f[1:] - f[:-1])
                if [g[0] if g else None for g in got] != [vals[i] for i in ids]:
                    errors.append((t, j))
        except Exception as e:  # pragma: no cover
            errors.append(repr(e))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors[:5]
    assert shard._impl.serve_jobs == 8 * 150


def test_serve_get_orders_after_a_side_stream_fill(cuda_dev):
    """The response buffers are zero-filled on a side stream that is still busy (a slow
    kernel ahead of the fill) and the job is submitted at once from that stream: the
    stream-less server must answer after the fill, so the answer survives."""
    shard = CacheShard(16 << 20, 1 << 12, 1 << 14, cuda_dev)
    keys = [f"/ord/{i}".encode() for i in range(29)]
    vals = [bytes([i + 1]) * (100 + 37 * i) for i in range(29)]
    shard.set_many(keys, vals)
    dh = digest_strings(keys, "cpu").contiguous()
    side = torch.cuda.Stream(device=cuda_dev)
    side.wait_stream(torch.cuda.current_stream(cuda_dev))
    for rep in range(3):
        with torch.cuda.stream(side):
            torch.cuda._sleep(5_000_000)   # a few ms of work queued ahead of the fills
            out = torch.full((1 << 16,), 7, dtype=torch.uint8, device=cuda_dev)
            off = torch.full((30,), -1, dtype=torch.int64, device=cuda_dev)
            out.zero_()
            off.zero_()
            assert shard._impl.serve_get(dh.data_ptr(), 29, out.data_ptr(), out.numel(),
                                         off.data_ptr(), shard.now(), 6, side.cuda_stream)
        total = shard._impl.serve_wait(6, 10000)
        side.synchronize()
        o, f = out[:total].cpu(), off.cpu()
        got = unpack_records(o, f[:-1], f[1:] - f[:-1])
        assert [g[0] if g else None for g in got] == vals, rep
        # the Python wrapper orders after the current stream the same way
        with torch.cuda.stream(side):
            torch.cuda._sleep(2_000_000)
            r = shard.serve_get(dh)
        assert r is not None
        o, f = r[0].cpu(), r[1].cpu()
        assert [g[0] if g else None for g in unpack_records(o, f[:-1], f[1:] - f[:-1])] == vals


def test_serve_get_relaunches_and_sees_new_sets(cuda_dev):
    """The server exits when idle and the next job relaunches it; a SET chain that ran
    while it was resident (other CUs, no stream order with it) is visible to its next job
    (the per-job acquire), and keys the SET's log append overwrote miss."""
    import time

    shard = CacheShard(1 << 20, 1 << 12, 1 << 14, cuda_dev, evict="fifo")  # wraps quickly
    first = [f"/srv2/a{i}".encode() for i in range(29)]
    shard.set_many(first, [b"a" * 3000] * 29)
    torch.cuda.synchronize()
    req = digest_strings(first, "cpu")
    out, off = shard.serve_get(req)
    assert all(r is not None for r in unpack_records(out, off[:-1], off[1:] - off[:-1]))
    l0 = shard._impl.serve_launches
    time.sleep(0.05)  # past the idle timeout
    out, off = shard.serve_get(req)
    assert shard._impl.serve_launches == l0 + 1
    # overwrite the whole log with new keys while the server may still be resident
    newer = [f"/srv2/b{i}".encode() for i in range(400)]
    for k in range(0, 400, 100):  # each SET batch within half the log
        shard.set_many(newer[k:k + 100], [b"b" * 3000] * 100)
    torch.cuda.synchronize()
    out, off = shard.serve_get(req)
    assert all(r is None for r in unpack_records(out, off[:-1], off[1:] - off[:-1]))
    tail = digest_strings(newer[-29:], "cpu")
    out, off = shard.serve_get(tail)
    got = unpack_records(out, off[:-1], off[1:] - off[:-1])
    assert all(r is not None and r[0] == b"b" * 3000 for r in got)


def test_serve_get_multi_round_jobs_beside_wrapping_sets(cuda_dev):
    """Edge-server jobs whose records span several copy rounds (29 x 8 KiB = 232 KiB, a
    round is 112 KiB) answered while SET chains on another stream keep wrapping the log over
    them: every record that comes back with a valid magic word names its own key and holds
    its own bytes; torn ones are misses (magic zeroed). The server re-reads the claim after
    the last round before it publishes."""
    from shellac_amd.ops.cache import ITEM_MAGIC

    log = 1 << 20
    shard = CacheShard(log, 1 << 12, 1 << 14, cuda_dev, evict="fifo")
    K, V = 29, 8192
    ka = [f"/tear/a{i}".encode() for i in range(K)]
    da = digest_strings(ka, cuda_dev)
    va, vao, val = pack_values([bytes([i + 1]) * V for i in range(K)], cuda_dev)
    # filler batches: 32 x 8 KiB = 256 KiB of 0xEE bytes each, 4 per log lap
    fills = []
    for b in range(4):
        kb = [f"/tear/b{b}/{i}".encode() for i in range(32)]
        fills.append((digest_strings(kb, cuda_dev),) + pack_values([b"\xee" * V] * 32, cuda_dev))
    shard.store(da, va, vao, val)
    torch.cuda.synchronize()
    dh = da.cpu().contiguous()
    out = torch.zeros(1 << 20, dtype=torch.uint8, device=cuda_dev)
    off = torch.zeros(K + 1, dtype=torch.int64, device=cuda_dev)
    cur = torch.cuda.current_stream(cuda_dev).cuda_stream  # serve_get orders after the fills
    side = torch.cuda.Stream(device=cuda_dev)
    hits = torn = 0
    for rnd in range(6):
        with torch.cuda.stream(side):  # queued, not waited for: runs beside the jobs
            for rep in range(40):
                shard.store(da, va, vao, val)
                for f in fills[: 1 + rep % 4]:
                    shard.store(*f)
        for job in range(150):
            assert shard._impl.serve_get(dh.data_ptr(), K, out.data_ptr(), out.numel(),
                                         off.data_ptr(), shard.now(), 5, cur)
            shard._impl.serve_wait(5, 10000)
            o = out.cpu().numpy()
            offs = off.cpu().numpy()
            if int(offs[K]) > out.numel():
                continue
            for i in range(K):
                if offs[i + 1] == offs[i]:
                    continue
                base = int(offs[i])
                hdr = o[base: base + 32].view(np.uint32)
                if int(hdr[7]) != ITEM_MAGIC:
                    torn += 1
                    continue
                words = o[base: base + 16].view(np.int64)
                assert words[0] == int(dh[i, 0]) and words[1] == int(dh[i, 1])
                body = o[base + 32: base + 32 + V]
                assert int(hdr[4]) == V and bool((body == i + 1).all()), (rnd, job, i)
                hits += 1
        side.synchronize()
    assert hits > 0


def test_store_graph_matches_store(cuda_dev):
    """A SET replayed from a captured hipGraph (fixed size class, skip-row padding, one
    executable per head-slot parity) leaves the shard exactly as the launched SET
    chain does; the graph is captured once per (pointers, n, now) and then replayed."""
    from shellac_amd._native import core

    cls = 64
    a = CacheShard(8 << 20, 1 << 10, 1 << 12, cuda_dev)
    b = CacheShard(8 << 20, 1 << 10, 1 << 12, cuda_dev)
    g = core().StoreGraph()
    now = a.now()
    keys = torch.zeros((cls, 2), dtype=torch.int64, device=cuda_dev)
    vals = torch.zeros(cls * 1024 + 16, dtype=torch.uint8, device=cuda_dev)
    voff = torch.arange(cls, dtype=torch.int64, device=cuda_dev) * 1024
    vlen = torch.empty(cls, dtype=torch.int32, device=cuda_dev)
    flags = torch.zeros(cls, dtype=torch.int32, device=cuda_dev)
    expire = torch.zeros(cls, dtype=torch.int32, device=cuda_dev)
    side = torch.cuda.Stream(device=cuda_dev)  # the null stream cannot be captured
    side.wait_stream(torch.cuda.current_stream(cuda_dev))
    s = side.cuda_stream
    rng = np.random.default_rng(3)
    all_keys = []
    torch.cuda.set_stream(side)
    for step in range(40):  # several log wraps of the 8 MiB log
        n = int(rng.integers(1, cls + 1))
        ks = digest_strings([f"/g/{step}/{i % 23}".encode() for i in range(n)], cuda_dev)
        all_keys.append(ks)
        keys[:n] = ks
        vals.copy_(torch.from_numpy(rng.integers(0, 256, vals.numel(), dtype=np.uint8)))
        vlen.fill_(-1)  # skip rows
        vlen[:n] = torch.from_numpy(rng.integers(1, 1000, n).astype(np.int32))
        flags[:n] = step
        a.store(keys[:n].contiguous(), vals, voff[:n].contiguous(), vlen[:n].contiguous(),
                flags[:n].contiguous(), expire[:n].contiguous(), now)
        b._impl.store_graph(g, keys.data_ptr(), vals.data_ptr(), voff.data_ptr(), vlen.data_ptr(),
                            flags.data_ptr(), expire.data_ptr(), cls, 4 << 20, now, s)
    torch.cuda.synchronize()
    torch.cuda.set_stream(torch.cuda.default_stream(cuda_dev))
    assert g.launches == 40 and g.captures == 1
    assert a.head() == b.head()
    q = torch.cat(all_keys)
    la, lb = a.lookup(q, now), b.lookup(q, now)
    assert torch.equal(la.size, lb.size) and torch.equal(la.off, lb.off)
    assert torch.equal(a.gather(la), b.gather(lb))
    assert int((la.size > 0).sum()) > 0
    g.destroy()


@pytest.mark.parametrize("n", [1, 2, 1000, 65537, 1 << 20])
def test_coalesce_kernel_first_rows(cuda_dev, n):
    """k_coalesce: first[i] holds the same digest as row i, claimers point at
    themselves, and there is exactly one claimer per distinct digest."""
    from shellac_amd.ops.cache import coalesce

    g = torch.Generator().manual_seed(n)
    pool = torch.randint(-2**62, 2**62, (max(n // 3, 1), 2), generator=g, dtype=torch.int64)
    # Zipf-like skew: low pool ids repeat a lot
    ids = (torch.rand(n, generator=g) ** 3 * pool.shape[0]).long().clamp(max=pool.shape[0] - 1)
    keys = pool.index_select(0, ids).contiguous().to(cuda_dev)
    shard = CacheShard(16 << 20, 1 << 12, 1 << 12, cuda_dev)
    ar = torch.arange(n, device=cuda_dev)
    nuniq = torch.unique(keys, dim=0).shape[0]
    lk, f2, _ = shard.lookup_coalesced(keys)  # fused coalesce + probe (empty shard: misses)
    for first in (coalesce(keys).long(), f2.long()):
        assert torch.equal(keys.index_select(0, first), keys)
        assert torch.equal(first.index_select(0, first), first)
        assert int((first == ar).sum()) == nuniq
    assert int(lk.off[n]) == 0 and shard.counters()["get_ops"] == nuniq


def test_coalesced_get_and_serve_match_uncoalesced(cuda_dev):
    """A Zipf batch (many duplicates) coalesced: the same value for every request as
    the uncoalesced path, one probe per distinct key, and a smaller response buffer."""
    from shellac_amd.bench.workload import Workload
    from shellac_amd.models.sharded_cache import ShardedCache

    wl = Workload(50000, cuda_dev)
    ids = wl.sample_ids(200000, 5)
    keys = wl.digests.index_select(0, ids).contiguous()
    res = {}
    for co in (False, True):
        shard = CacheShard(512 << 20, 1 << 16, 1 << 16, cuda_dev)
        sc = ShardedCache(shard)
        sc.coalesce = co
        for s0 in range(0, 50000, 10000):
            sc.set(wl.set_batch(torch.arange(s0, s0 + 10000, device=cuda_dev)))
        c0 = shard.counters()["get_ops"]
        r = sc.get(keys)
        probes = shard.counters()["get_ops"] - c0
        s = sc.serve(keys, wl.set_batch(wl.uniform_ids(4096, 6)))
        torch.cuda.synchronize()
        if co:  # the persistent coalescing table is left zeroed by every step
            assert sc._co_table is not None and int(sc._co_table.abs().sum()) == 0
            s2 = sc.serve(keys, wl.set_batch(wl.uniform_ids(4096, 7)))
            assert int(sc._co_table.abs().sum()) == 0
            assert torch.equal(s2.size.cpu() > 0, s.size.cpu() > 0)
        res[co] = (unpack_records(r.data, r.off, r.size), r.size.cpu(), probes,
                   unpack_records(s.data, s.off, s.size), int(r.data.numel()))
    a, b = res[False], res[True]
    assert a[0] == b[0] and torch.equal(a[1], b[1])
    assert a[3] == b[3]
    assert a[2] == keys.shape[0]
    assert b[2] == torch.unique(keys, dim=0).shape[0] < keys.shape[0] // 2
    assert b[4] < a[4] // 2
    for i in range(0, 200000, 997):
        assert b[0][i] is not None and b[0][i][0] == wl.expected_value(int(ids[i]))



@pytest.mark.parametrize("bs,pad", [(300, 512), (1500, 2048), (3000, 4096)])
def test_set_index_under_same_bucket_contention(cuda_dev, bs, pad):
    """3000 keys into a 1024-slot index in large batches (~12 inserts per bucket pair per
    batch, padded with skip rows like the HTTP backend's micro-batches): every key that
    hits must return its own record (the insert claims an entry with a lock value before
    it writes the digest; a late digest write once paired keys with other keys' records)."""
    sh = CacheShard(64 << 20, 256, 1 << 16, cuda_dev)
    keys = [b"/pf/%d" % i for i in range(3000)]
    for s in range(0, 3000, bs):
        kk = keys[s:s + bs]
        d = torch.zeros((pad, 2), dtype=torch.int64)
        d[: len(kk)] = digest_strings(kk)
        v, vo, vl = pack_values([b"v%d" % i for i in range(s, s + len(kk))] + [b""] * (pad - len(kk)))
        vl[len(kk):] = -1  # kSkipVlen padding rows
        vo[len(kk):] = 0
        sh.store(d.to(cuda_dev), v.to(cuda_dev), vo.to(cuda_dev), vl.to(cuda_dev))
    lk = sh.lookup(digest_strings(keys).to(cuda_dev))
    recs = unpack_records(sh.gather(lk), lk.off[:3000], lk.size[:3000])
    hits = [i for i, r in enumerate(recs) if r is not None]
    assert len(hits) > 900
    assert all(recs[i][0] == b"v%d" % i for i in hits)


def test_set_index_resets_over_dead_entries_lose_nothing(cuda_dev):
    """Re-SET keys whose old entries are dead but still hold their digests (deleted), all
    in one batch under same-bucket contention: a row must never take another row's fresh
    claim (whose digest words have not landed) for its own entry. Every row of the batch
    either hits with its own new value or is accounted for as evicted / dropped."""
    sh = CacheShard(64 << 20, 256, 1 << 16, cuda_dev)
    keys = [b"/rz/%d" % i for i in range(3000)]
    d = digest_strings(keys).to(cuda_dev)
    for s in range(0, 3000, 500):
        v, vo, vl = pack_values([b"old%d" % i for i in range(s, s + 500)])
        sh.store(d[s:s + 500], v.to(cuda_dev), vo.to(cuda_dev), vl.to(cuda_dev))
    sh.remove(d)
    torch.cuda.synchronize()
    c0 = sh.counters()
    v, vo, vl = pack_values([b"new%d" % i for i in range(3000)])
    sh.store(d, v.to(cuda_dev), vo.to(cuda_dev), vl.to(cuda_dev))
    torch.cuda.synchronize()
    c1 = sh.counters()
    lk = sh.lookup(d)
    recs = unpack_records(sh.gather(lk), lk.off[:3000], lk.size[:3000])
    hits = [i for i, r in enumerate(recs) if r is not None]
    assert all(recs[i][0] == b"new%d" % i for i in hits)
    lost = (c1["set_evicted"] - c0["set_evicted"]) + (c1["set_dropped"] - c0["set_dropped"])
    assert len(hits) + lost == 3000, (len(hits), lost)
    assert len(hits) > 900


def _compact(b):
    """The SetBatch with its values gathered into a buffer of their own (its bytes, not
    the workload's whole pool, bound the log bytes the SET may append)."""
    import dataclasses

    vl = b.vlen.long()
    off = torch.cumsum(vl, 0) - vl
    src = torch.repeat_interleave(b.val_off - off, vl) + torch.arange(int(vl.sum()),
                                                                      device=vl.device)
    return dataclasses.replace(b, values=b.values[src].contiguous(), val_off=off.contiguous())


def _serve_steps_vs_truth(sc, wl, dev, steps=4, nget=100000, compact=False):
    """serve() steps of Zipf GETs over a filled cache; per step the number of requests
    that got a value other than the workload's ground truth, and of misses."""
    pool = wl.pool.cpu().numpy()  # ground truth on the host once (not one copy per request)
    voff, vlen = wl.val_off.cpu().tolist(), wl.vlen.cpu().tolist()

    def truth(i):
        return pool[voff[i]: voff[i] + vlen[i]].tobytes()

    out = []
    for step in range(steps):
        ids = wl.sample_ids(nget, 11 + step)
        keys = wl.digests.index_select(0, ids).contiguous()
        b = wl.set_batch(wl.uniform_ids(4096, 21 + step))
        r = sc.serve(keys, _compact(b) if compact else b)
        torch.cuda.synchronize()
        recs = unpack_records(r.data, r.off, r.size)
        wrong = [(k, i) for k, (i, x) in enumerate(zip(ids.tolist(), recs))
                 if x is not None and (x[0] != truth(i) or x[1] != i % 65536)]
        miss = [k for k, x in enumerate(recs) if x is None]
        out.append((len(wrong), len(miss), wrong[:3], miss[:3]))
    return out


def test_serve_steps_return_ground_truth_records(cuda_dev):
    """The N=1 serving step (coalesced lookup and gather on the main stream, SET chain on
    the side stream) serves the workload's ground-truth record (value and flags) for every
    request, step after step, over a cache that holds every key (no misses)."""
    from shellac_amd.bench.workload import Workload
    from shellac_amd.models.sharded_cache import ShardedCache

    wl = Workload(40000, cuda_dev)
    shard = CacheShard(256 << 20, 1 << 15, 1 << 16, cuda_dev)
    sc = ShardedCache(shard)
    for s0 in range(0, 40000, 10000):
        sc.set(wl.set_batch(torch.arange(s0, s0 + 10000, device=cuda_dev)))
    res = _serve_steps_vs_truth(sc, wl, cuda_dev)
    assert all(w == 0 and m == 0 for w, m, _, _ in res), res


@pytest.mark.parametrize("hand", ["early", "inline"])
def test_serve_wrapped_log_ground_truth_both_hand_schedules(cuda_dev, hand):
    """A log the key space overfills, so every serve step runs the CLOCK hand: with the
    hand detached on its own stream (early, the default) and at the head of the SET chain
    (inline), every request that hits gets its ground-truth record, the hand reinserts,
    and a later get() (which joins the pending SET chain) agrees with the last serve."""
    from shellac_amd.bench.workload import Workload
    from shellac_amd.models.sharded_cache import ShardedCache

    wl = Workload(100000, cuda_dev)  # ~100 MB of records into a 96 MiB log
    shard = CacheShard(96 << 20, 1 << 16, 1 << 13, cuda_dev)
    sc = ShardedCache(shard, hand=hand)
    for s0 in range(0, 100000, 5000):
        sc.set(_compact(wl.set_batch(torch.arange(s0, s0 + 5000, device=cuda_dev))))
    c0 = sc.counters()
    res = _serve_steps_vs_truth(sc, wl, cuda_dev, steps=6, nget=50000, compact=True)
    assert all(w == 0 for w, _, _, _ in res), res
    assert sum(m for _, m, _, _ in res) < 6 * 50000 // 2, res
    assert sc.counters()["reinserted"] > c0["reinserted"]
    ids = wl.sample_ids(20000, 99)
    keys = wl.digests.index_select(0, ids).contiguous()
    r = sc.serve(keys, _compact(wl.set_batch(wl.uniform_ids(4096, 98))))
    g = sc.get(keys)  # no device sync in between: get() joins the serve's SET chain
    torch.cuda.synchronize()
    a = unpack_records(r.data, r.off, r.size)
    b = unpack_records(g.data, g.off, g.size)
    pool, voff, vlen = wl.pool.cpu().numpy(), wl.val_off.cpu().tolist(), wl.vlen.cpu().tolist()
    for i, x, y in zip(ids.tolist(), a, b):
        t = pool[voff[i]: voff[i] + vlen[i]].tobytes()
        assert x is None or x[0] == t
        assert y is None or y[0] == t


@pytest.mark.parametrize("hand,lead", [("early", False), ("inline", False), ("early", True)])
def test_serve_back_to_back_updates_never_resurrect_stale_values(cuda_dev, hand, lead):
    """Steps queued back to back (no host sync) over a full cache whose SET batches UPDATE
    objects (new payload versions) and DELETE some: the early hand of step k+1 runs beside
    step k's index insert, so it may pick for reinsertion an object step k's SET or DELETE
    is superseding. Its reinsertion is a move that must then be dropped. Every GET of step
    k returns the version the SETs of steps < k left, or a miss — never an older version
    and never a deleted key — and the hand does reinsert. lead: a log 32x the SET batch, so
    the hand runs in lead mode (decisions two batches ahead, reinsertions copied straight
    from the log, layout.h hand_lead)."""
    from shellac_amd.bench.workload import Workload
    from shellac_amd.models.sharded_cache import ShardedCache

    N = 300000 if lead else 60000
    log = (128 << 20) if lead else (16 << 20)
    wl = Workload(N, cuda_dev, min_val=64, max_val=2048)
    # ~25 MB of records into a 16 MiB log (lead: ~185 MB into 128 MiB): the populate wraps
    # it, every step runs the hand
    shard = CacheShard(log, 1 << 18 if lead else 1 << 16, 1 << 13, cuda_dev)
    sc = ShardedCache(shard, hand=hand)
    rmax = shard._impl.reinsert_max
    for s0 in range(0, N, 5000):
        sc.set(_compact(wl.set_batch(torch.arange(s0, s0 + 5000, device=cuda_dev))))
    sc.sync_sets()
    c0 = sc.counters()
    # hot keys, so the hand finds referenced objects; SETs hit the hot keys too
    steps, results = 10, []
    version = [0] * N           # host truth: the version the SETs so far left
    deleted = set()
    truth_at = []               # per step: (ids, versions expected, deleted ids) at its GETs
    batches = []
    for k in range(steps):
        ids = wl.sample_ids(20000, 300 + k)
        up = torch.cat([wl.sample_ids(1500, 500 + k), wl.uniform_ids(1500, 700 + k)])
        truth_at.append((ids.tolist(), list(version), set(deleted)))
        b = _compact(wl.set_batch(up, version=k + 1))
        # layout.h hand_lead on this batch's byte bound (CacheShard.store's default)
        assert (log >= 16 * (shard.payload_bound(b.keys.shape[0], b.values.numel()) + rmax)) == lead
        batches.append(b)
        r = sc.serve(wl.digests.index_select(0, ids).contiguous(), b)
        results.append(r)
        for i in up.tolist():
            version[i] = k + 1
            deleted.discard(i)
        if k % 3 == 2:          # a DELETE between steps (joins the pending chain)
            dels = wl.sample_ids(300, 900 + k).unique()
            sc.delete(wl.digests.index_select(0, dels).contiguous())
            deleted |= set(dels.tolist())
    torch.cuda.synchronize()
    pool = wl.pool.cpu().numpy()
    vlen = wl.vlen.cpu().tolist()
    offs = {}

    def truth(i, v):
        if (i, v) not in offs:
            offs[(i, v)] = int(wl._offsets(torch.tensor([i], device=cuda_dev), v)[0])
        o = offs[(i, v)]
        return pool[o: o + vlen[i]].tobytes()

    stale = dead = hits = 0
    for (ids, ver, gone), r in zip(truth_at, results):
        for i, x in zip(ids, unpack_records(r.data, r.off, r.size)):
            if x is None:
                continue
            hits += 1
            if i in gone:
                dead += 1
            elif x[0] != truth(i, ver[i]):
                stale += 1
    c1 = sc.counters()
    assert stale == 0 and dead == 0, (stale, dead, hits)
    assert hits > steps * 20000 // 2
    assert c1["reinserted"] > c0["reinserted"]


def test_serve_waits_for_a_batch_the_caller_is_still_producing(cuda_dev):
    """The SET batch is finished on the caller's stream right before serve() (behind a slow
    kernel): the SET chain and the early hand must not read it before then. A later get()
    returns the new values of every key the batch set."""
    from shellac_amd.bench.workload import Workload
    from shellac_amd.models.sharded_cache import ShardedCache

    N = 30000
    wl = Workload(N, cuda_dev, min_val=64, max_val=1024)
    sc = ShardedCache(CacheShard(8 << 20, 1 << 15, 1 << 13, cuda_dev))  # ~11 MB of records
    for s0 in range(0, N, 5000):
        sc.set(_compact(wl.set_batch(torch.arange(s0, s0 + 5000, device=cuda_dev))))
    keys = wl.digests.index_select(0, wl.sample_ids(8000, 5)).contiguous()
    for k in range(3):   # the log is overfilled: every step runs the hand
        sc.serve(keys, _compact(wl.set_batch(wl.uniform_ids(2000, 40 + k))))
    ids = wl.uniform_ids(2000, 77).unique()
    real = _compact(wl.set_batch(ids, version=5))
    # the batch the caller passes: zero keys and values until a slow producer on the
    # current stream writes them, queued right before serve()
    b = dataclasses.replace(real, keys=torch.zeros_like(real.keys),
                            values=torch.zeros_like(real.values))
    torch.cuda.synchronize()
    torch.cuda._sleep(20_000_000)      # ~10 ms of GPU time ahead of the copies
    b.keys.copy_(real.keys)
    b.values.copy_(real.values)
    sc.serve(keys, b)
    del b                              # the cache keeps what its chain still reads
    g = sc.get(wl.digests.index_select(0, ids).contiguous())
    torch.cuda.synchronize()
    pool = wl.pool.cpu().numpy()
    vlen = wl.vlen.cpu().tolist()
    offs = wl._offsets(ids, 5).cpu().tolist()
    recs = unpack_records(g.data, g.off, g.size)
    got = sum(1 for i, o, x in zip(ids.tolist(), offs, recs)
              if x is not None and x[0] == pool[o: o + vlen[i]].tobytes())
    assert got == len(recs), (got, len(recs))


@pytest.mark.parametrize("fence", ["system", "device", "none"])
def test_serve_event_fences_return_the_same_records(cuda_dev, fence):
    """The events ordering the serving step's two streams, at every fence scope: each
    step's GETs see the previous step's SETs (index insert on the side stream) and the
    coalescing table is clean again."""
    from shellac_amd.bench.workload import Workload
    from shellac_amd.models.sharded_cache import ShardedCache

    wl = Workload(20000, cuda_dev)
    shard = CacheShard(512 << 20, 1 << 14, 1 << 16, cuda_dev)
    sc = ShardedCache(shard)
    sc.event_fence = fence
    sc.set(wl.set_batch(torch.arange(0, 10000, device=cuda_dev)))
    keys = wl.digests.index_select(0, wl.sample_ids(50000, 3)).contiguous()
    ids_new = torch.arange(10000, 20000, device=cuda_dev)
    r1 = sc.serve(keys, wl.set_batch(ids_new))  # ids >= 10000 miss now ...
    r2 = sc.serve(keys, wl.set_batch(ids_new[:16]))  # ... and hit one step later
    torch.cuda.synchronize()
    ids = wl.sample_ids(50000, 3).cpu().tolist()
    pool = wl.pool.cpu().numpy()
    voff, vlen = wl.val_off.cpu().tolist(), wl.vlen.cpu().tolist()
    v1 = unpack_records(r1.data, r1.off, r1.size)
    v2 = unpack_records(r2.data, r2.off, r2.size)
    assert all((v is None) == (i >= 10000) for v, i in zip(v1, ids))
    assert all(v is not None and v[0] == pool[voff[i]: voff[i] + vlen[i]].tobytes()
               for v, i in zip(v2, ids))
    assert int(sc._co_table.abs().sum()) == 0


@pytest.mark.parametrize("dma", [True, False])
def test_host_edge_serve_matches_device_edge(cuda_dev, dma):
    """Host edge (digests, SET payloads and responses in pinned host memory): the response
    lands in host memory — by a DMA copy of an HBM staging buffer (host_edge_dma, the
    default) or by the gather's own stores — and every step returns the same records as
    the device edge on the same inputs, across the two buffer turns."""
    from shellac_amd.bench.workload import Workload
    from shellac_amd.models.sharded_cache import SetBatch, ShardedCache

    wl = Workload(20000, cuda_dev, min_val=64, max_val=2048, pool_bytes=4 << 20)
    gets = [wl.digests.index_select(0, wl.sample_ids(3000 + 11 * i, 21 + i)).contiguous()
            for i in range(4)]
    sets = [wl.set_batch(wl.uniform_ids(500, 70 + i)) for i in range(4)]
    runs = []
    for host in (False, True):
        sc = ShardedCache(CacheShard(32 << 20, 1 << 14, 1 << 16, cuda_dev))
        sc.overlap_store = True
        sc.host_edge, sc.host_edge_dma = host, dma
        for s0 in range(0, 20000, 4000):
            sc.set(wl.set_batch(torch.arange(s0, s0 + 4000, device=cuda_dev)))
        out = []
        for step in range(6):
            g, b = gets[step % 4], sets[step % 4]
            if host:
                def pin(t):
                    return None if t is None else t.cpu().pin_memory()

                g = pin(g)
                b = SetBatch(pin(b.keys), pin(b.values), pin(b.val_off), pin(b.vlen),
                             pin(b.flags), pin(b.expire))
            r = sc.serve(g, b).wait()
            assert r.data.device.type == ("cpu" if host else "cuda")
            out.append((r.size.cpu().clone(), unpack_records(r.data, r.off, r.size)))
        torch.cuda.synchronize(cuda_dev)
        runs.append(out)
    for (s0, d0), (s1, d1) in zip(*runs):
        assert torch.equal(s0, s1)
        assert d0 == d1
    assert sum(int((s > 0).sum()) for s, _ in runs[1]) > 0


@pytest.mark.gpu
def test_set_workspace_grows_then_frees_retired_blocks(cuda_dev):
    """SET batches growing 8x (1000 -> 8000 rows, on two streams in turn): every grow
    retires the old SET workspace behind the last stores of the streams that used it, and once those
    chains have drained the next store frees it — retired bytes back to 0, no keep-forever
    and no device synchronisation in store. A store on the other
    stream is ordered after the grow's dedupe-table clears: every value lands."""
    from shellac_amd.ops.cache import CacheShard

    s = CacheShard(64 << 20, 1 << 15, 1 << 14, cuda_dev)
    ever0 = s._impl.retired_ever
    side = torch.cuda.Stream(cuda_dev)
    n, written = 1000, []
    for step in range(4):
        keys = [b"/grow/%d/%d" % (step, i) for i in range(n)]
        vals = [b"v%d-%d-" % (step, i) * 5 for i in range(n)]
        if step % 2:
            with torch.cuda.stream(side):
                s.set_many(keys, vals)
        else:
            s.set_many(keys, vals)
        written.append((keys, vals))
        n *= 2
    torch.cuda.synchronize()
    assert s._impl.retired_ever > ever0  # the workspace did grow (and retire) 3 times
    s.set_many([b"/grow/last"], [b"x" * 10])  # a store reaps the groups whose chains drained
    torch.cuda.synchronize()
    assert s._impl.retired_bytes() == 0
    for keys, vals in written:
        assert s.get_many(keys) == vals


def test_set_workspace_grow_after_a_store_stream_was_destroyed(cuda_dev):
    """A SET on a caller's raw stream that the caller then destroys, then SET batches that
    grow the workspace on the current stream: the retire must not touch the dead stream
    (it waits for that stream's last-store event instead), the retired blocks are freed
    once drained, and every value lands."""
    from shellac_amd import core
    from shellac_amd.ops.cache import CacheShard

    c = core()
    s = CacheShard(64 << 20, 1 << 15, 1 << 14, cuda_dev)
    raw = c.stream_create()
    ext = torch.cuda.ExternalStream(raw, device=cuda_dev)
    with torch.cuda.stream(ext):
        s.set_many([b"/dead/%d" % i for i in range(500)], [b"d%d" % i for i in range(500)])
    c.stream_destroy(raw)
    del ext
    ever0 = s._impl.retired_ever
    written = []
    for step, n in enumerate((1000, 4000, 16000)):
        keys = [b"/after/%d/%d" % (step, i) for i in range(n)]
        vals = [b"a%d-%d" % (step, i) for i in range(n)]
        s.set_many(keys, vals)
        written.append((keys, vals))
    torch.cuda.synchronize()
    assert s._impl.retired_ever > ever0
    s.set_many([b"/after/last"], [b"x"])
    torch.cuda.synchronize()
    assert s._impl.retired_bytes() == 0
    assert s.get_many([b"/dead/%d" % i for i in range(500)]) == [b"d%d" % i for i in range(500)]
    for keys, vals in written:
        assert s.get_many(keys) == vals


@pytest.mark.gpu
def test_reserve_presizes_the_clock_combined_batch(cuda_dev):
    """reserve(n) sizes the SET workspace, the hand's window workspace and both hand buffers
    for the combined batch (hand window + n rows) a SET of n runs once the log wraps, so a
    serving store never allocates in steady state: three laps of 2000-row SETs with the hand
    active grow (and retire) nothing."""
    from shellac_amd.ops.cache import CacheShard

    s = CacheShard(4 << 20, 1 << 14, 1 << 14, cuda_dev)
    s.reserve(2000)
    ever = s._impl.retired_ever
    for b in range(24):  # ~600 KB per batch: 3+ laps of the 4 MiB log
        s.set_many([b"/rsv/%d/%d" % (b, i) for i in range(2000)], [b"r" * 280] * 2000)
        if b % 4 == 0:
            s.get_many([b"/rsv/%d/%d" % (b, i) for i in range(0, 2000, 7)])  # referenced
    torch.cuda.synchronize()
    assert s.head() > 3 * (4 << 20) and s.counters()["reinserted"] > 0
    assert s._impl.retired_ever == ever


@pytest.mark.parametrize("n", [100, 3000])
def test_stop_events_order_a_second_stream(cuda_dev, n):
    """``store(done=)`` and ``lookup_coalesced(index_done=)`` complete the caller's event as
    their last / probing kernel's own completion signal (hipExtLaunchKernel stop event;
    the small-batch path records it instead): the event is pending while the call's kernels
    wait behind other work on their stream, and a second stream ordered by it sees the
    SETs (n = 100: the one-launch small path; n = 3000: the full chain, fix-up last)."""
    from shellac_amd.ops.cache import StreamEvent

    shard = CacheShard(32 << 20, 1 << 14, 1 << 14, cuda_dev)
    keys = [f"/stop/{n}/{i}".encode() for i in range(n)]
    vals = [bytes([i % 251 + 1]) * (40 + (i * 37) % 900) for i in range(n)]
    d, v, vo, vl = (t.to(cuda_dev) for t in _batch(keys, vals, "cpu"))
    main = torch.cuda.current_stream(cuda_dev)
    side = torch.cuda.Stream(device=cuda_dev)
    side.wait_stream(main)
    done = StreamEvent("none")
    with torch.cuda.stream(side):
        torch.cuda._sleep(20_000_000)   # the store's kernels queue behind ~10 ms of work
        shard.store(d, v, vo, vl, done=done)
    assert not done.query()
    done.wait(main)                     # main: the lookup follows the whole SET chain
    out, off, size = shard.get(d)
    got = unpack_records(out, off, size)
    assert [g[0] if g else None for g in got] == vals
    assert done.query()
    # the coalescing lookup's probe completes index_done
    probed = StreamEvent("none")
    dup = torch.cat([d, d[: n // 2]])
    with torch.cuda.stream(side):
        torch.cuda._sleep(20_000_000)
        lk, first, _ = shard.lookup_coalesced(dup, index_done=probed)
    assert not probed.query()
    side.synchronize()
    assert probed.query()
    assert int((lk.size[: dup.shape[0]] > 0).sum()) == n   # one claimer per distinct key
    # an empty batch queues no kernel: its done event is recorded on the stream instead
    empty = StreamEvent("none")
    with torch.cuda.stream(side):
        torch.cuda._sleep(20_000_000)
        shard.store(d[:0], v, vo[:0], vl[:0], done=empty)
    assert not empty.query()
    side.synchronize()
    assert empty.query()
