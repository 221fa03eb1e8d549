"""The HBM cache behind the proxy and the memcached-protocol node (GPU only)."""
import time

import pytest

from shellac_amd.server.cached import CacheNode
from shellac_amd.server.proxy import Server, make_backend
from shellac_amd.utils.fakemc import MemcacheClient
from shellac_amd.utils.httpclient import HttpClient
from shellac_amd.utils.origin import Origin

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hbm():
    return make_backend("hbm", gpus=[0], hbm_gb=1.0, batch_us=20)


def _wait_get(be, key, timeout=3.0):
    deadline = time.time() + timeout
    while time.time() < deadline:
        r = be.get(key)
        if r is not None:
            return r
        time.sleep(0.01)
    return None


def test_hbm_backend_roundtrip(hbm):
    assert hbm.name == "hbm"
    hbm.set(b"/gpu/a", b"A" * 5000, 3, 0)
    hbm.set(b"/gpu/b", b"", 0, 0)
    assert _wait_get(hbm, b"/gpu/a") == (b"A" * 5000, 3)
    assert _wait_get(hbm, b"/gpu/b") == (b"", 0)
    assert hbm.get(b"/gpu/none") is None
    assert hbm.delete(b"/gpu/a") is True
    assert hbm.get(b"/gpu/a") is None
    st = hbm.stats()
    assert st["hbm_gpus"] == 1 and st["hbm_batches"] >= 1


@pytest.mark.parametrize("edge_server", [True, False])
def test_hbm_backend_edge_server_paths(edge_server):
    """Small GET batches go to the resident edge-server kernel (no launch per batch) and
    return the same objects as the launched path; overwrites and deletes are seen by the
    next GET once they completed, and batches with a write of one of their keys still in
    flight fall back to the ordered stream path."""
    be = make_backend("hbm", gpus=[0], hbm_gb=0.25, edge_server=edge_server)
    keys = [b"/es/%d" % i for i in range(64)]
    for i, k in enumerate(keys):
        be.set(k, b"v%d-" % i * 100, i, 0)
    assert _wait_get(be, keys[-1]) is not None
    for rep in range(3):
        for i, k in enumerate(keys):
            assert be.get(k) == (b"v%d-" % i * 100, i)
    be.set(keys[0], b"new" * 50, 7, 0)
    deadline = time.time() + 3
    while be.get(keys[0]) != (b"new" * 50, 7) and time.time() < deadline:
        time.sleep(0.001)
    assert be.get(keys[0]) == (b"new" * 50, 7)
    assert be.delete(keys[1]) is True
    assert be.get(keys[1]) is None
    st = be.stats()
    if edge_server:
        assert st["hbm_served_batches"] > 0 and st["hbm_server_launches"] >= 1
    else:
        assert st["hbm_served_batches"] == 0 and st["hbm_server_launches"] == 0


def test_hbm_cache_node_over_memcached_protocol(hbm):
    with CacheNode(backend=hbm, port=0, threads=2) as node:
        c = MemcacheClient(port=node.port)
        for i in range(200):
            c.set(b"n%d" % i, b"v%d" % i * 10, flags=i)
        got = c.get_multi([b"n%d" % i for i in range(200)])
        assert len(got) == 200 and got[b"n7"] == b"v7" * 10
        assert c.get(b"n9") == (b"v9" * 10, 9)


def test_proxy_with_hbm_backend(hbm):
    o = Origin(body_bytes=3000).start()
    try:
        with Server([("127.0.0.1", o.port)], port=0, backend=hbm, threads=2) as px:
            c = HttpClient(port=px.port)
            paths = [f"/hbm/{i}" for i in range(50)]
            first = [c.get(p).body().read() for p in paths]
            time.sleep(0.2)
            rs = c.pipeline(paths)
            assert [r.body().read() for r in rs] == first
            assert all(o.hits[p] == 1 for p in paths)
            # repeated paths in one pipeline: batch-mates share a GPU row (host coalescing)
            c0 = hbm.stats()["hbm_coalesced_gets"]
            rs = c.pipeline(paths[:10] * 8)
            assert [r.body().read() for r in rs] == first[:10] * 8
            assert all(o.hits[p] == 1 for p in paths)
            st = px.stats()
            assert st["cache_hits"] >= 50 and st["backend"] == "hbm"
            # the batch-mates did share rows (not just correct bodies)
            assert hbm.stats()["hbm_coalesced_gets"] > c0
    finally:
        o.stop()


@pytest.mark.parametrize("direct", [True, False])
def test_proxy_reactor_direct_gets(direct):
    """Reactor-direct submission: each proxy reactor writes its own edge-server jobs and
    answers them from its loop. Bodies match the batcher path; a GET right after the miss
    that stored its key is ordered after that SET (it hits); pipelines with more distinct
    keys than one server job still go through the batcher."""
    be = make_backend("hbm", gpus=[0], hbm_gb=0.25, direct=direct)
    o = Origin(body_bytes=2500).start()
    try:
        with Server([("127.0.0.1", o.port)], port=0, backend=be, threads=2) as px:
            c = HttpClient(port=px.port)
            paths = [f"/rd/{i}" for i in range(60)]
            first = []
            for p in paths:
                first.append(c.get(p).body().read())
                assert c.get(p).body().read() == first[-1]  # read-your-write: a hit
            assert all(o.hits[p] == 1 for p in paths)
            for _ in range(3):
                assert [c.get(p).body().read() for p in paths] == first
            rs = c.pipeline(paths[:40] * 2)
            assert [r.body().read() for r in rs] == first[:40] * 2
            assert all(o.hits[p] == 1 for p in paths)
            st = be.stats()
            if direct:
                assert st["hbm_direct_jobs"] > 0 and st["hbm_direct_requests"] >= 180
                assert st["hbm_direct_timeouts"] == 0 and st["hbm_key_mismatch"] == 0
            else:
                assert st["hbm_direct_jobs"] == 0 and st["hbm_direct_requests"] == 0
    finally:
        o.stop()


def test_proxy_with_tiered_dram_hbm():
    be = make_backend("hbm", gpus=[0], hbm_gb=1.0, batch_us=20, l1_mb=16)
    o = Origin(body_bytes=1000).start()
    try:
        with Server([("127.0.0.1", o.port)], port=0, backend=be) as px:
            c = HttpClient(port=px.port)
            for i in range(20):
                c.get(f"/tier/{i}")
            time.sleep(0.2)
            for i in range(20):
                c.get(f"/tier/{i}")
            st = px.stats()["cache"]
            assert st["tier_l1_hits"] == 20 and st["l2_hbm_gpus"] == 1
            assert all(o.hits[f"/tier/{i}"] == 1 for i in range(20))
    finally:
        o.stop()


def test_hbm_backend_idle_sweep_expires_ttl():
    be = make_backend("hbm", gpus=[0], hbm_gb=0.25, sweep_s=1)
    be.set(b"/ttl/short", b"x" * 100, 0, 1)
    be.set(b"/ttl/long", b"y" * 100, 0, 3600)
    assert _wait_get(be, b"/ttl/long") == (b"y" * 100, 0)
    time.sleep(3.2)
    st = be.stats()
    assert st["hbm_sweeps"] >= 1
    assert be.get(b"/ttl/short") is None
    assert be.get(b"/ttl/long") == (b"y" * 100, 0)
    assert st["hbm_live_objects"] == 1


def test_hbm_presence_filter_skips_cold_misses_and_survives_rebuild():
    """GETs of never-stored digests are answered on the host (no GPU batch); once a
    full index worth of digests was added the filter is rebuilt from the shard's live
    keys, and every live object must still hit (no false negatives)."""
    from shellac_amd import core

    be = core().hbm_backend([0], 64 << 20, 256, 1 << 16, 0, sweep_interval_s=1)
    st0 = be.stats()
    assert be.get(b"/never/stored") is None
    assert be.stats()["hbm_filter_skips"] == st0["hbm_filter_skips"] + 1
    assert be.stats()["hbm_batches"] == st0["hbm_batches"]  # no GPU round trip
    keys = [b"/pf/%d" % i for i in range(3000)]  # > 1024 index slots: rebuilds + evictions
    for i, k in enumerate(keys):
        be.set(k, b"v%d" % i, 0, 0)
        if i % 500 == 499:
            assert _wait_get(be, k) == (b"v%d" % i, 0)
    assert _wait_get(be, keys[-1]) == (b"v2999", 0)
    for k in keys[:8]:  # trigger the rebuild check after the last SET batch
        be.get(k)
    time.sleep(2.5)  # idle sweep refreshes hbm_live_objects
    st = be.stats()
    assert st["hbm_filter_rebuilds"] >= 1
    hits = sum(1 for i, k in enumerate(keys) if be.get(k) == (b"v%d" % i, 0))
    assert hits == be.stats()["hbm_live_objects"] > 0
    skips = be.stats()["hbm_filter_skips"]
    cold = sum(be.get(b"/cold/%d" % i) is None for i in range(1000))
    assert cold == 1000
    assert be.stats()["hbm_filter_skips"] - skips > 900  # few false positives


def test_hbm_presence_filter_off_sends_every_get_to_the_gpu():
    from shellac_amd import core

    be = core().hbm_backend([0], 16 << 20, 256, 1 << 16, 0, presence_filter=False)
    b0 = be.stats()["hbm_batches"]
    assert be.get(b"/never/stored") is None
    st = be.stats()
    assert st["hbm_batches"] == b0 + 1 and "hbm_filter_skips" not in st


def test_hbm_forged_digest_collision_is_a_miss(hbm):
    """Objects are identified by their full key, not the digest: a GET for another key
    that arrives with this object's digest (a forged collision) misses."""
    hbm.set(b"/victim/page", b"secret" * 100, 5, 0)
    assert _wait_get(hbm, b"/victim/page") == (b"secret" * 100, 5)
    assert hbm.get_with_digest(b"/attacker/url", b"/victim/page") is None
    assert hbm.get_with_digest(b"/victim/page", b"/victim/page") == (b"secret" * 100, 5)
    assert hbm.stats()["hbm_key_mismatch"] >= 1


def test_hbm_concurrent_clients_pipelined_batches():
    """Many client threads against one GPU: batches overlap (depth 3), every GET gets
    its own key's value, SETs interleave."""
    import threading

    be = make_backend("hbm", gpus=[0], hbm_gb=0.5, depth=3)
    keys = [b"/cc/%d" % i for i in range(2000)]
    for i, k in enumerate(keys):
        be.set(k, b"%d:" % i + bytes([i % 251]) * (i % 3000), 0, 0)
    assert _wait_get(be, keys[-1]) is not None
    errors = []

    def worker(t):
        try:
            for j in range(400):
                i = (t * 7919 + j * 104729) % 2000
                r = be.get(keys[i])
                want = b"%d:" % i + bytes([i % 251]) * (i % 3000)
                if r is None or r[0] != want:
                    errors.append((i, r is None))
                if j % 50 == 0:
                    be.set(b"/cc/new/%d/%d" % (t, j), b"n" * 100, 0, 0)
        except Exception as e:  # pragma: no cover
            errors.append(repr(e))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors[:5]
    st = be.stats()
    assert st["hbm_batches"] > 0 and st["hbm_failures"] == 0 and st["hbm_regathers"] >= 0


def test_gpu_shard_ejection_drill_and_restore():
    """gpu_down=0: the shard leaves the ring, the proxy keeps answering (misses go to
    the origin), SETs to it are dropped; lifting the drill restores (and flushes) the
    shard, and hits resume once objects are cached again."""
    from shellac_amd.server.proxy import set_fault

    be = make_backend("hbm", gpus=[0], hbm_gb=0.5, fault="")
    o = Origin(body_bytes=2000).start()
    try:
        with Server([("127.0.0.1", o.port)], port=0, backend=be, threads=2) as px:
            c = HttpClient(port=px.port)
            paths = [f"/ej/{i}" for i in range(30)]
            for p in paths:
                assert c.get(p).status() == 200
            time.sleep(0.2)
            for p in paths:
                c.get(p)
            assert all(o.hits[p] == 1 for p in paths)  # cached
            set_fault(be, "gpu_down=0")
            for p in paths:
                assert c.get(p).status() == 200     # still served: misses -> origin
            assert all(o.hits[p] == 2 for p in paths)
            st = px.stats()["cache"]
            assert st["hbm_gpus_up"] == 0 and st["hbm_ejections"] >= 1
            set_fault(be, "")
            deadline = time.time() + 5
            while px.stats()["cache"]["hbm_gpus_up"] == 0 and time.time() < deadline:
                time.sleep(0.05)
            assert px.stats()["cache"]["hbm_gpus_up"] == 1
            for p in paths:
                c.get(p)                             # flushed on restore: refill
            time.sleep(0.3)
            for p in paths:
                assert c.get(p).status() == 200
            assert all(o.hits[p] == 3 for p in paths)  # hits resumed
            assert px.stats()["cache"]["hbm_restores"] >= 1
    finally:
        o.stop()


@pytest.mark.parametrize("peer_copy", ["auto", "staged"])
def test_gpu_shard_warm_restore_pulls_its_keys_back_from_peers(peer_copy):
    """Two shards (both on GPU 0 here; on a node they are two GPUs and the copy goes
    over xGMI). While shard 0 is ejected its key range is served by shard 1; when it
    returns it flushes, then pulls those objects back peer-to-peer, so they keep hitting
    (shard 1 drops them). Objects shard 1 owned all along are untouched."""
    from shellac_amd import core

    be = core().hbm_backend([0, 0], 64 << 20, 1 << 14, 1 << 16, 0, peer_copy=peer_copy)
    before = [b"/wr/before/%d" % i for i in range(300)]
    for i, k in enumerate(before):
        be.set(k, b"b%d" % i * 20, 1, 0)
    assert _wait_get(be, before[-1]) is not None
    core().inject_shard_down(be, 0, True)
    assert be.stats()["hbm_gpus_up"] == 1
    during = [b"/wr/during/%d" % i for i in range(400)]
    for i, k in enumerate(during):
        be.set(k, b"d%d" % i * 30, 2, 0)
    assert _wait_get(be, during[-1]) is not None
    assert all(be.get(k) == (b"d%d" % i * 30, 2) for i, k in enumerate(during))
    core().inject_shard_down(be, 0, False)
    deadline = time.time() + 10
    while be.stats()["hbm_gpus_up"] < 2 and time.time() < deadline:
        time.sleep(0.05)
    st = be.stats()
    assert st["hbm_gpus_up"] == 2 and st["hbm_restores"] >= 1
    # every object SET during the drill still hits (about half now live on shard 0)
    got = [be.get(k) for k in during]
    assert all(g == (b"d%d" % i * 30, 2) for i, g in enumerate(got)), \
        sum(g is None for g in got)
    st = be.stats()
    assert 100 < st["hbm_migrated"] < 300, st["hbm_migrated"]
    # "staged": the records went through pinned host memory (a pair without peer access)
    assert (st["hbm_staged_peer_copies"] > 0) == (peer_copy == "staged")
    # before the drill: shard 1's objects hit, shard 0's were flushed on restore
    hits = sum(be.get(k) == (b"b%d" % i * 20, 1) for i, k in enumerate(before))
    assert 80 < hits < 220, hits
