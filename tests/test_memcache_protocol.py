"""memcached binary protocol: shellac-cached (native server) vs the pure-Python client,
native client vs the fake server, and the ketama continuum (MD5)."""
import hashlib
import time

import pytest

from shellac_amd.server.cached import CacheNode
from shellac_amd.utils.fakemc import FakeMemcached, MemcacheClient


@pytest.fixture
def node():
    n = CacheNode(port=0, kind="dram", dram_mb=64, threads=2).start()
    yield n
    n.stop()


def test_set_get_delete_flags(node):
    c = MemcacheClient(port=node.port)
    assert c.set(b"k1", b"hello", flags=42) == 0
    assert c.get(b"k1") == (b"hello", 42)
    assert c.get(b"nope") is None
    assert c.delete(b"k1") is True
    assert c.get(b"k1") is None
    assert c.delete(b"k1") is False


def test_add_replace_append_incr_touch(node):
    c = MemcacheClient(port=node.port)
    assert c.add(b"a", b"1") == 0
    assert c.add(b"a", b"2") == 2          # KEY_EEXISTS
    assert c.replace(b"zz", b"x") == 1     # KEY_ENOENT
    assert c.replace(b"a", b"3") == 0
    assert c.get(b"a")[0] == b"3"
    assert c.append(b"a", b"45") == 0
    assert c.get(b"a")[0] == b"345"
    assert c.incr(b"a", 5) == 350
    assert c.incr(b"ctr", 1, initial=10) == 10
    assert c.incr(b"ctr", 7) == 17
    assert c.touch(b"ctr", 100) == 0
    assert c.touch(b"missing", 100) == 1


def test_expiry(node):
    c = MemcacheClient(port=node.port)
    c.set(b"e", b"v", exptime=1)
    assert c.get(b"e")[0] == b"v"
    time.sleep(2.2)
    assert c.get(b"e") is None


def test_multiget_pipelined_quiet_ops(node):
    c = MemcacheClient(port=node.port)
    for i in range(50):
        c.set(b"m%d" % i, b"v%d" % i)
    got = c.get_multi([b"m%d" % i for i in range(60)])
    assert got == {b"m%d" % i: b"v%d" % i for i in range(50)}


def test_version_stats_flush(node):
    c = MemcacheClient(port=node.port)
    assert c.version().startswith(b"shellac")
    c.set(b"s", b"1")
    st = c.stats()
    assert int(st["cache_set_ops"]) >= 1
    assert c.flush() == 0
    assert c.get(b"s") is None


def test_large_value_and_binary_keys(node):
    c = MemcacheClient(port=node.port)
    v = bytes(range(256)) * 3000
    c.set(b"\x01bin\xffkey", v)
    assert c.get(b"\x01bin\xffkey")[0] == v


def test_native_client_against_fake_server():
    from shellac_amd._native import core

    f = FakeMemcached().start()
    try:
        be = core().memcached_backend(f"127.0.0.1:{f.port}")
        be.set(b"x", b"payload", 7, 0)
        deadline = time.time() + 3
        while b"x" not in f.data and time.time() < deadline:
            time.sleep(0.01)
        assert be.get(b"x") == (b"payload", 7)
        assert be.get(b"y") is None
        long_key = b"/very/long/" + b"a" * 400  # > 250 bytes: hashed on the wire
        be.set(long_key, b"L")
        time.sleep(0.2)
        assert be.get(long_key)[0] == b"L"
        assert be.delete(b"x") is True and be.get(b"x") is None
    finally:
        f.stop()


def test_md5_and_ketama(core):
    for s in [b"", b"abc", b"hello world" * 20]:
        assert core.md5_hex(s) == hashlib.md5(s).hexdigest()
    names = [f"10.0.0.{i}:11211" for i in range(4)]
    r = core.KetamaRing(names)
    assert r.points() == 4 * 160
    # reference continuum computed independently in Python (libketama algorithm)
    pts = []
    for idx, n in enumerate(names):
        for k in range(40):
            d = hashlib.md5(f"{n}-{k}".encode()).digest()
            for h in range(4):
                pts.append((int.from_bytes(d[4 * h : 4 * h + 4], "little"), idx))
    pts.sort()
    import bisect

    for key in [b"/a", b"/index.html", b"/x/y/z?q=1"] + [b"/k%d" % i for i in range(200)]:
        hv = int.from_bytes(hashlib.md5(key).digest()[:4], "little")
        i = bisect.bisect_left(pts, (hv, -1))
        exp = pts[i % len(pts)][1]
        assert r.pick(key) == exp
    # ejecting a node moves only its keys
    before = {k: r.pick(b"/k%d" % k) for k in range(500)}
    r.set_alive(2, False)
    for k, o in before.items():
        n = r.pick(b"/k%d" % k)
        assert n != 2 and (o == 2 or n == o)
