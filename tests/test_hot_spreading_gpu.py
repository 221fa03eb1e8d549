"""Hot-object spreading in the proxy's multi-GPU HBM tier (HbmBackend), GPU only.

The reference's ketama client sends each key to one memcached node
(/root/reference/src/python/shellac/server/Server.py:81-83), so a Zipf hot key loads one
node. HbmBackend replicates the most requested objects on every shard, spreads their GETs
(designated / sprayed ranks from host_router.cc plan_hot) and writes their SETs / DELETEs
through. These tests run 2 and 4 shards on GPU 0 (on a node they are separate GPUs and
the replica fills go over xGMI)."""
import threading
import time

import numpy as np
import pytest

from shellac_amd import core
from shellac_amd.server.proxy import Server, hot_refresh, make_backend
from shellac_amd.utils.httpclient import HttpClient
from shellac_amd.utils.origin import Origin

pytestmark = pytest.mark.gpu

NKEYS = 4000
# a key set whose ketama split is uneven under Zipf(0.99) at both 2 and 4 shards
# (owner shares max/mean 1.28 and 1.32, computed with HostRouter on the CPU)
KEYS = [b"/hs13/%d" % i for i in range(NKEYS)]
P = 1.0 / np.arange(1, NKEYS + 1) ** 0.99
P /= P.sum()


def _val(i, v=0):
    return b"v%d-%d-" % (v, i) * 6


def _backend(nshards, hot, **kw):
    return core().hbm_backend([0] * nshards, 64 << 20, 1 << 14, 1 << 16, 0, hot_objects=hot,
                              hot_refresh_ms=0, **kw)


def _fill(be, v=0):
    for i, k in enumerate(KEYS):
        be.set(k, _val(i, v), v, 0)
    deadline = time.time() + 5
    while be.get(KEYS[-1]) is None and time.time() < deadline:
        time.sleep(0.005)


def _shard_gets(be, n):
    st = be.stats()
    return np.array([st[f"hbm_shard_gets_{i}"] for i in range(n)], dtype=np.float64)


@pytest.mark.parametrize("nshards", [2, 4])
def test_hot_spreading_evens_out_per_shard_gets(nshards):
    """Per-shard GET share of a Zipf(0.99) stream: max/mean > 1.15 on plain ketama,
    <= 1.05 once the hot set is replicated and its GETs designated / sprayed; every GET
    returns its object's value either way."""
    rng = np.random.default_rng(5)
    ratio = {}
    for hot in (0, 256):
        be = _backend(nshards, hot, hot_sample=2)
        _fill(be)
        warm = rng.choice(NKEYS, size=20000, p=P)
        got = be.get_many([KEYS[i] for i in warm])
        assert all(g == (_val(i), 0) for g, i in zip(got, warm))
        if hot:
            info = hot_refresh(be)
            assert info["hot"] == 256 and info["added"] == 256, info
            assert info["failed_mask"] == 0 and info["spread_mask"] == (1 << nshards) - 1, info
        before = _shard_gets(be, nshards)
        idx = rng.choice(NKEYS, size=40000, p=P)
        got = be.get_many([KEYS[i] for i in idx])
        assert all(g == (_val(i), 0) for g, i in zip(got, idx)), \
            sum(g != (_val(i), 0) for g, i in zip(got, idx))
        d = _shard_gets(be, nshards) - before
        assert d.sum() == len(idx)
        ratio[hot] = d.max() / d.mean()
        print(f"[hot-spread] shards={nshards} hot_objects={hot} per-shard GET share "
              f"{(d / d.sum()).round(4).tolist()} max/mean {ratio[hot]:.4f}")
        st = be.stats()
        assert st["hbm_hot_spreading"] == (1 if hot else 0)
        if hot:
            assert st["hbm_hot_objects"] == 256 and st["hbm_hot_spread_gets"] > 0
            assert st["hbm_hot_filled_rows"] > 0 and st["hbm_key_mismatch"] == 0
    assert ratio[0] > 1.15, ratio
    assert ratio[256] <= 1.05, ratio


def test_hot_spreading_never_serves_stale_or_deleted_copies():
    """SETs and DELETEs of hot objects are written through: a GET issued after them sees
    them on whichever replica it lands. Hot-set refreshes while one writer updates versions
    and another SETs then DELETEs objects in turn never let a reader see a version older
    than one whose SET had returned before the GET, nor a version whose DELETE had returned;
    objects that cool lose their non-owner replicas (a later promotion refills)."""
    be = _backend(4, 64, hot_sample=1)
    _fill(be)
    rng = np.random.default_rng(11)
    be.get_many([KEYS[i] for i in rng.choice(NKEYS, size=20000, p=P)])
    info = hot_refresh(be)
    assert info["hot"] == 64, info
    top = KEYS[:32]  # the hottest ranks of the Zipf: all in the hot set
    for v in (1, 2, 3):
        for i, k in enumerate(top):
            be.set(k, _val(i, v), v, 0)
        got = be.get_many(top * 8)  # every replica the designation / spray can pick
        assert got == [(_val(i, v), v) for i in range(32)] * 8
        for k in top[:6]:
            assert be.delete(k) is True
        assert be.get_many(top[:6] * 8) == [None] * 48
        assert be.delete(top[0]) is False
        for i, k in enumerate(top[:6]):
            be.set(k, _val(i, v), v, 0)
    assert be.stats()["hbm_hot_spread_gets"] > 0

    # a writer bumps versions of 48 objects (hot and cold); readers check monotonicity
    # against the version committed before each GET, while the hot set drifts
    watched = list(range(0, 24)) + list(range(2000, 2024))
    committed = {i: 3 if i < 32 else 0 for i in watched}
    lock = threading.Lock()
    stop = threading.Event()
    errors = []

    def writer():
        v = 10
        while not stop.is_set():
            for i in watched:
                be.set(KEYS[i], _val(i, v), v, 0)
                with lock:
                    committed[i] = v
            v += 1

    # a second writer SETs and then DELETEs 16 more objects in turn (a DELETE returns once
    # every copy is gone): a GET issued after it must not return the deleted version
    churn = list(range(24, 32)) + list(range(2024, 2032))
    last = {i: (0, "set") for i in churn}

    def deleter():
        v = 10
        while not stop.is_set():
            for i in churn:
                be.set(KEYS[i], _val(i, v), v, 0)
                with lock:
                    last[i] = (v, "set")
                be.delete(KEYS[i])
                with lock:
                    last[i] = (v, "del")
            v += 1

    def reader():
        while not stop.is_set():
            with lock:
                snap = dict(committed)
                snap_c = dict(last)
            got = be.get_many([KEYS[i] for i in watched + churn])
            for i, g in zip(watched, got):
                if g is None or g[1] < snap[i] or g[0] != _val(i, g[1]):
                    errors.append((i, snap[i], g))
            for i, g in zip(churn, got[len(watched):]):
                v, kind = snap_c[i]
                if g is not None and (g[1] < v or (kind == "del" and g[1] == v) or
                                      g[0] != _val(i, g[1])):
                    errors.append((i, snap_c[i], g))

    th = [threading.Thread(target=writer), threading.Thread(target=deleter),
          threading.Thread(target=reader), threading.Thread(target=reader)]
    for t in th:
        t.start()
    totals = {"added": 0, "removed": 0, "replicas_dropped": 0}
    try:
        for shift in (1500, 3000, 0, 1500):  # the hot set moves, then comes back
            perm = (np.arange(NKEYS) + shift) % NKEYS
            for _ in range(3):
                be.get_many([KEYS[perm[i]] for i in rng.choice(NKEYS, size=20000, p=P)])
                info = hot_refresh(be)
                for k in totals:
                    totals[k] += info.get(k, 0)
    finally:
        stop.set()
        for t in th:
            t.join()
    assert not errors, errors[:5]
    assert totals["added"] > 0 and totals["removed"] > 0 and totals["replicas_dropped"] > 0, totals
    # a DELETE of every watched object is seen on every replica
    for i in watched:
        be.delete(KEYS[i])
    assert be.get_many([KEYS[i] for i in watched] * 8) == [None] * (len(watched) * 8)
    st = be.stats()
    assert st["hbm_key_mismatch"] == 0 and st["hbm_hot_fill_failures"] == 0


def test_hot_spreading_shard_ejection_drops_its_replicas_and_heals():
    """An ejected shard leaves the spread mask (its GETs go to the owners); back in
    service it is flushed, and the next refresh refills the whole hot set into it before
    GETs are spread to it again."""
    be = _backend(4, 64, hot_sample=1)
    _fill(be)
    rng = np.random.default_rng(3)
    be.get_many([KEYS[i] for i in rng.choice(NKEYS, size=20000, p=P)])
    assert hot_refresh(be)["spread_mask"] == 0b1111
    core().inject_shard_down(be, 2, True)
    st = be.stats()
    assert st["hbm_hot_spread_mask"] == 0b1011 and st["hbm_gpus_up"] == 3
    idx = rng.choice(NKEYS, size=5000, p=P)
    got = be.get_many([KEYS[i] for i in idx])
    # shard 2's own keys miss while it is out; nothing is answered from it, nothing stale
    assert all(g is None or g == (_val(i), 0) for g, i in zip(got, idx))
    g0 = _shard_gets(be, 4)
    be.get_many([KEYS[i] for i in idx])
    assert (_shard_gets(be, 4) - g0)[2] == 0
    core().inject_shard_down(be, 2, False)
    deadline = time.time() + 10
    while be.stats()["hbm_gpus_up"] < 4 and time.time() < deadline:
        time.sleep(0.05)
    assert be.stats()["hbm_gpus_up"] == 4
    for i, k in enumerate(KEYS[:40]):  # new versions while shard 2 holds no replicas
        be.set(k, _val(i, 5), 5, 0)
    info = hot_refresh(be)
    assert info["heal_mask"] == 0b0100 and info["spread_mask"] == 0b1111, info
    got = be.get_many(KEYS[:40] * 8)
    assert got == [(_val(i, 5), 5) for i in range(40)] * 8
    # hot objects not written since: back on every replica, shard 2's own ones included
    # (read from a peer's replica: shard 2 was flushed and migration left them be)
    got = be.get_many(KEYS[40:48] * 8)
    assert got == [(_val(i), 0) for i in range(40, 48)] * 8


def test_proxy_hbm_hot_spreading_over_http():
    """The same through the HTTP proxy: a Zipf stream of cached URLs, a refresh, then the
    GETs spread over both shards' replicas and every body is the origin's."""
    be = make_backend("hbm", gpus=[0, 0], hbm_gb=0.25, hot_objects=64, hot_refresh_ms=0,
                      hot_sample=1)
    o = Origin(body_bytes=1500).start()
    n = 600
    p = 1.0 / np.arange(1, n + 1) ** 0.99
    p /= p.sum()
    rng = np.random.default_rng(2)
    try:
        with Server([("127.0.0.1", o.port)], port=0, backend=be, threads=2,
                    client_max_reqs=1 << 30) as px:
            c = HttpClient(port=px.port)
            paths = [f"/hsp/{i}" for i in range(n)]
            body = {}
            for pth in paths:
                body[pth] = c.get(pth).body().read()
            time.sleep(0.2)
            for i in rng.choice(n, size=3000, p=p):
                assert c.get(paths[i]).body().read() == body[paths[i]]
            info = hot_refresh(be)
            assert info["hot"] > 0 and info["spread_mask"] == 0b11, info
            st0 = px.stats()["cache"]
            for i in rng.choice(n, size=6000, p=p):
                assert c.get(paths[i]).body().read() == body[paths[i]]
            st = px.stats()["cache"]
            assert st["hbm_hot_objects"] == info["hot"]
            assert st["hbm_hot_spread_gets"] > st0["hbm_hot_spread_gets"]
            d = np.array([st[f"hbm_shard_gets_{i}"] - st0[f"hbm_shard_gets_{i}"]
                          for i in range(2)], dtype=np.float64)
            print(f"[hot-spread] http shards=2 per-shard GETs {d.tolist()} "
                  f"max/mean {d.max() / d.mean():.4f} refresh {info}")
            assert d.max() / d.mean() <= 1.10, d
            assert all(o.hits[pth] == 1 for pth in paths)  # every request after the fill hit
    finally:
        o.stop()
