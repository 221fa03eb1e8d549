"""Host-routed topology routing (parallel/hotspread.py, csrc/host_router.cc) on the CPU:
the native HostRouter and the tensor routing make the same decisions, and spraying the
hot objects' GETs evens out a Zipf stream's per-rank load."""
import pytest
import torch

from shellac_amd.parallel.hotspread import HotSpread, cumulative, spray_ranks, water_fill


@pytest.mark.parametrize("lanes", [False, True])
@pytest.mark.parametrize("world", [1, 2, 3, 8, 20, 70])
def test_native_router_matches_tensor_routing(world, lanes):
    g = torch.Generator().manual_seed(world)
    keys = torch.randint(-2**63, 2**63 - 1, (50000, 2), dtype=torch.int64, generator=g)
    # crowded hot-table buckets: 40 hot objects on one home slot (long probe runs: the
    # lanes' second probe misses and the scalar rule redoes them)
    keys[260:300, 0] = (keys[260:300, 0] & ~0xFFFF) | 0x1234
    hs = HotSpread(world, "cpu")
    hs.router.lanes = lanes
    stream = keys[torch.randint(0, 3000, (200000,), generator=g)].contiguous()
    for hot in (None, keys[:300]):
        w = [1.0 + (r % 3) for r in range(world)]
        # designated ranks for most hot objects, sprayed (-1) for every fifth
        ranks = torch.tensor([-1 if i % 5 == 0 else i % world for i in range(300)],
                             dtype=torch.int32)
        hs.set_hot(hot, ranks if hot is not None else None, w if hot is not None else None)
        for seq0 in (0, 12345678901):
            d, c = hs.host_route_gets(stream, seq0=seq0, threads=3)
            assert torch.equal(d, hs.route_gets(stream, seq0=seq0))
            assert torch.equal(c, torch.bincount(d.long(), minlength=world))
            # an odd-sized slice (the lanes' scalar tail) at an odd stream position
            d1, _ = hs.host_route_gets(stream[7:1006], seq0=seq0 + 7)
            assert torch.equal(d1, d[7:1006])
        s, c = hs.host_route_sets(stream, threads=2)
        assert torch.equal(s, hs.route_sets(stream))
        fan = int((s < 0).sum())
        assert torch.equal(c, torch.bincount(s[s >= 0].long(), minlength=world) + fan)
        assert (fan > 0) == (hot is not None and world >= 1)
    # ownership alone is the ketama ring's (ShardRing, DigestRing)
    own = hs.owners(stream)
    for i in range(0, 200000, 20011):
        lo, hi = int(stream[i, 0]) & (2**64 - 1), int(stream[i, 1]) & (2**64 - 1)
        assert hs.router.owner(lo, hi) == int(own[i]) == hs.ring.owner_of_digest(lo, hi)


def test_spray_follows_the_weights():
    cw = torch.tensor(cumulative([1.0, 3.0, 0.0, 4.0]), dtype=torch.float64)
    r = spray_ranks(torch.arange(80000, dtype=torch.int64), cw)
    share = torch.bincount(r.long(), minlength=4).double() / 80000
    assert torch.allclose(share, torch.tensor([0.125, 0.375, 0.0, 0.5], dtype=torch.float64),
                          atol=2e-3)


def test_water_fill_levels_the_ranks():
    own = [0.10, 0.02, 0.20, 0.05]
    w = water_fill(own, 0.63)
    tot = sum(w)
    final = [o + 0.63 * x / tot for o, x in zip(own, w)]
    assert max(final) - min(final) < 1e-9 and abs(sum(final) - 1.0) < 1e-9
    # a rank the non-hot traffic already overloads gets no hot traffic
    w = water_fill([0.6, 0.1, 0.1], 0.2)
    assert w[0] == 0.0 and abs(w[1] - w[2]) < 1e-12


@pytest.mark.parametrize("policy", ["designate", "spray"])
def test_spreading_evens_out_a_zipf_stream(policy):
    """Zipf(0.99) over 400K keys on 8 ranks: ketama alone leaves the most loaded rank well
    above the mean (the hot keys' owners); the top 4096 objects designated to ranks (or
    sprayed) bring it within 2 %."""
    n, world = 400000, 8
    g = torch.Generator().manual_seed(3)
    keys = torch.randint(-2**63, 2**63 - 1, (n, 2), dtype=torch.int64, generator=g)
    ranks = torch.arange(1, n + 1, dtype=torch.float64)
    cdf = torch.cumsum(ranks.pow(-0.99), 0)
    cdf /= cdf[-1].clone()
    ids = torch.searchsorted(cdf, torch.rand(2_000_000, generator=g, dtype=torch.float64))
    stream = keys[ids.clamp_(max=n - 1)]
    hs = HotSpread(world, "cpu")
    c0 = torch.bincount(hs.route_gets(stream).long(), minlength=world).double()
    info = hs.plan(stream[:1_000_000], 4096, policy=policy)
    c1 = torch.bincount(hs.route_gets(stream[1_000_000:], seq0=1_000_000).long(),
                        minlength=world).double()
    assert float(c0.max() / c0.mean()) > 1.1
    assert float(c1.max() / c1.mean()) < 1.02, (c1 / c1.mean()).tolist()
    assert info["hot_share"] > 0.3


def test_router_tables_swap_under_concurrent_routing():
    """set_hot publishes a new immutable table while other threads route (the proxy's
    reactors route every request while the hot-set refresh thread re-plans): each
    route_gets call sees exactly one table, never a half-built one, and set_hot returns
    only after the old table has no readers (it is freed there)."""
    import threading

    from shellac_amd import core

    world = 4
    r = core().HostRouter(world)
    g = torch.Generator().manual_seed(3)
    hot = torch.randint(-2**63, 2**63 - 1, (512, 2), dtype=torch.int64, generator=g)
    # the routed batch: the hot objects only, so a call's ranks name its table
    stream = hot[torch.randint(0, 512, (70000,), generator=g)].contiguous()
    tables = []
    for t in range(world):  # table t designates every hot object to rank t
        ranks = torch.full((512,), t, dtype=torch.int32)
        tables.append(ranks)
    w = [1.0] * world
    stop = threading.Event()
    bad = []

    def route():
        dest = torch.empty(stream.shape[0], dtype=torch.int32)
        counts = torch.zeros(world, dtype=torch.int64)
        while not stop.is_set():
            counts.zero_()
            r.route_gets(stream.data_ptr(), stream.shape[0], 0, dest.data_ptr(),
                         counts.data_ptr(), 2)
            u = torch.unique(dest)
            if u.numel() != 1 or int(counts.max()) != stream.shape[0]:
                bad.append(u.tolist())

    r.set_hot(hot.data_ptr(), 512, tables[0].data_ptr(), w)  # before any reader starts
    ths = [threading.Thread(target=route) for _ in range(3)]
    for th in ths:
        th.start()
    try:
        for i in range(200):
            ranks = tables[i % world]
            r.set_hot(hot.data_ptr(), 512, ranks.data_ptr(), w)
            assert r.nhot == 512
            # after set_hot returned, every decision uses the new table
            lo, hi = int(hot[7, 0]) & (2**64 - 1), int(hot[7, 1]) & (2**64 - 1)
            assert r.hot_rank(lo, hi) == i % world
    finally:
        stop.set()
        for th in ths:
            th.join()
    assert not bad, bad[:5]
    assert r.publications == 201


@pytest.mark.parametrize("world", [2, 4, 8])
def test_native_hot_plan_matches_hotspread_design(world):
    """plan_hot (the proxy HBM tier's planner, host_router.cc) makes HotSpread.design's
    decisions on the same sample: the same hot set in the same order, the same designated
    ranks (sprayed -1 above 1/(4N)) and the same planned loads."""
    from shellac_amd import core

    g = torch.Generator().manual_seed(world)
    keys = torch.randint(-2**63, 2**63 - 1, (3000, 2), dtype=torch.int64, generator=g)
    p = 1.0 / torch.arange(1, 3001, dtype=torch.float64) ** 0.99
    sample = keys[torch.multinomial(p, 40000, replacement=True, generator=g)]
    hs = HotSpread(world, "cpu")
    hot, ranks, _, info = hs.design(sample, 200)
    u, cnt = torch.unique(sample, dim=0, return_counts=True)
    rows = [(int(a) & (2**64 - 1), int(b) & (2**64 - 1), int(c))
            for (a, b), c in zip(u.tolist(), cnt.tolist())]
    plan = core().plan_hot(hs.router, rows, 200, (1 << world) - 1, 1.0 / (4 * world), 1)
    want = [(int(a) & (2**64 - 1), int(b) & (2**64 - 1)) for a, b in hot.tolist()]
    assert [tuple(x) for x in plan["hot"]] == want
    assert plan["rank"] == ranks.tolist()
    assert abs(plan["hot_share"] - info["hot_share"]) < 1e-6  # (the tensor mean is fp32)
    assert plan["planned"] == pytest.approx(info["planned_load"], abs=1e-12)
    # only eligible ranks are designation / spray targets
    el = (1 << world) - 1 - 2
    plan = core().plan_hot(hs.router, rows, 200, el, 1.0 / (4 * world), 1)
    assert 1 not in plan["rank"] and plan["weights"][1] == 0.0


def test_native_hot_plan_hysteresis_keeps_the_replicated_tail():
    """The HBM tier re-plans its hot set every refresh from decayed sampled counts; objects
    already replicated rank at 2x (sticky), so a tail object is replaced only by one at least
    twice as hot — sampling noise does not churn fills and deletes."""
    from shellac_amd import core

    r = core().HostRouter(4)
    rows = [(1000 + i, 7 * i + 1, 100 - i) for i in range(60)]  # counts 100 .. 41
    top = core().plan_hot(r, rows, 10, 0b1111, 0.25, 1)
    assert [h[0] for h in top["hot"]] == list(range(1000, 1010))
    # a tail object of the current set (count 60) against colder newcomers above it
    cur = [(1040, 7 * 40 + 1)]
    plan = core().plan_hot(r, rows, 10, 0b1111, 0.25, 1, sticky=cur, sticky_factor=2.0)
    hot = [h[0] for h in plan["hot"]]
    assert 1040 in hot and 1009 not in hot  # 60 x 2 = 120 outranks the 91 of the newcomer
    # ... but not against one more than twice as hot
    rows2 = rows + [(5000, 3, 130)]
    plan = core().plan_hot(r, rows2, 10, 0b1111, 0.25, 1, sticky=cur, sticky_factor=2.0)
    hot = [h[0] for h in plan["hot"]]
    assert 5000 in hot and 1040 in hot
    # the designation loads use the true counts (the sticky factor ranks only)
    assert abs(sum(plan["planned"]) - 1.0) < 1e-9
