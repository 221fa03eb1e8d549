"""GPU batch gzip (csrc/deflate.hip) against zlib: every member must decompress to its
input (gzip framing, CRC-32 and ISIZE checked by zlib), across empty, tiny, multi-block,
incompressible (stored-block fallback) and highly repetitive inputs."""
import gzip
import os
import random
import zlib

import pytest

pytestmark = pytest.mark.gpu


def _html(rng, n):
    words = [b"cache", b"proxy", b"<div class=\"item\">", b"</div>", b"memcached", b"GPU",
             b"<a href=\"/static/obj/", b"\">", b"</a>", b"HBM", b"\n", b"  "]
    out = bytearray()
    while len(out) < n:
        out += rng.choice(words)
        if rng.random() < 0.1:
            out += str(rng.randrange(10 ** 6)).encode()
    return bytes(out[:n])


@pytest.fixture
def gz(cuda_dev):
    from shellac_amd.ops.gzip import engine

    return engine(cuda_dev.index or 0)


def test_round_trip_mixed_batch(gz):
    rng = random.Random(5)
    block = 32768
    bodies = [b"", b"a", b"ab", b"abc", b"aaaa" * 100, b"x" * 258, b"x" * 259,
              os.urandom(1000), os.urandom(block), os.urandom(block + 1),
              _html(rng, 4096), _html(rng, block), _html(rng, block + 17),
              _html(rng, 3 * block + 5), bytes(range(256)) * 300, b"\x00" * 100000]
    out = gz.compress(bodies)
    assert len(out) == len(bodies)
    for b, o in zip(bodies, out):
        assert o[:2] == b"\x1f\x8b"
        assert zlib.decompress(o, 31) == b
        assert gzip.decompress(o) == b


def test_raw_deflate_and_ratio(gz):
    rng = random.Random(9)
    bodies = [_html(rng, 65536) for _ in range(8)]
    out = gz.deflate(bodies)
    for b, o in zip(bodies, out):
        assert zlib.decompress(o, -15) == b
    ratio = sum(map(len, out)) / sum(map(len, bodies))
    z1 = sum(len(zlib.compress(b, 1)) for b in bodies) / sum(map(len, bodies))
    # greedy single-candidate LZ77 + per-block dynamic Huffman codes: about zlib level 1
    assert ratio < 0.5 and ratio < 1.1 * z1, (ratio, z1)


def test_incompressible_falls_back_to_stored(gz):
    before = gz.stats().stored_blocks
    bodies = [os.urandom(20000) for _ in range(4)]
    out = gz.compress(bodies)
    for b, o in zip(bodies, out):
        assert zlib.decompress(o, 31) == b
        assert len(o) <= len(b) + 18 + 5 * (1 + len(b) // 32768)
    assert gz.stats().stored_blocks >= before + 4


def test_large_batch_many_blocks(gz):
    rng = random.Random(3)
    bodies = [_html(rng, rng.randrange(1, 200000)) for _ in range(300)]
    out = gz.compress(bodies)
    assert all(zlib.decompress(o, 31) == b for b, o in zip(bodies, out))


def test_proxy_compresses_misses_on_the_gpu(cuda_dev):
    """proxy -z --gzip-gpu 0: identity text responses of the miss path are gzipped by the
    GPU service in batches across reactor threads; pipelined order, cache fills and hits
    behave as with zlib on the reactor."""
    import json

    from shellac_amd.server.proxy import Server
    from shellac_amd.utils.httpclient import HttpClient
    from shellac_amd.utils.origin import Origin

    o = Origin(body_bytes=6000).start()
    try:
        with Server([("127.0.0.1", o.port)], port=0, backend_kind="dram", dram_mb=64,
                    compress=True, gzip_gpu=cuda_dev.index or 0, threads=2).start() as px:
            c = HttpClient(port=px.port)
            paths = [f"/zgpu/{i}.html" for i in range(24)]  # (the origin itself gzips /gz*)
            rs = c.pipeline(paths, headers={"Accept-Encoding": "gzip"})
            for p, r in zip(paths, rs):
                assert r.headers().get("content-encoding") == "gzip", p
                assert r.body().read().startswith(f"<html>{p} #1 ".encode()), p
            rs = c.pipeline(paths[:5], headers={"Accept-Encoding": "gzip"})  # cache hits
            for p, r in zip(paths, rs):
                assert r.body().read().startswith(f"<html>{p} #1 ".encode()), p
            st = px.stats()
            assert st["gzip_gpu"]["completed"] == len(paths) == st["gzip_gpu"]["bodies"] and st["gzip_gpu"]["errors"] == 0
            assert st["gzip_gpu"]["out_bytes"] < st["gzip_gpu"]["in_bytes"]
            assert all(o.hits[p] == 1 for p in paths)
            json.dumps(st)
    finally:
        o.stop()


def test_proxy_identity_variants_inflate_on_the_gpu(cuda_dev):
    """Under --policy rfc a client without Accept-Encoding: gzip gets the identity variant
    of a gzip-coded cached object; with --gzip-gpu the proxy's GPU service inflates those
    in batches (zlib on the service thread only for members the GPU path rejects), and the
    bytes match what the gzip client's response decodes to."""
    from shellac_amd.server.proxy import Server
    from shellac_amd.utils.httpclient import HttpClient
    from shellac_amd.utils.origin import Origin

    o = Origin(body_bytes=9000).start()
    try:
        with Server([("127.0.0.1", o.port)], port=0, backend_kind="dram", dram_mb=64,
                    compress=True, gzip_gpu=cuda_dev.index or 0, threads=2).start() as px:
            c = HttpClient(port=px.port)
            paths = [f"/zid/{i}.html" for i in range(16)] + [f"/gz/zid{i}" for i in range(4)]
            gz_bodies = [r.body().read() for r in
                         c.pipeline(paths, headers={"Accept-Encoding": "gzip"})]
            rs = c.pipeline(paths)  # no Accept-Encoding: identity variants, from the cache
            for p, r, want in zip(paths, rs, gz_bodies):
                assert r.status() == 200, p
                assert "content-encoding" not in r.headers(), p
                assert r.body().read() == want, p
            st = px.stats()
            assert st["identity_decoded"] == len(paths)
            assert st["gzip_gpu"]["identity_served"] == len(paths)
            assert st["gzip_gpu"]["inflated_gpu"] + st["gzip_gpu"]["inflated_cpu"] == len(paths)
            assert st["gzip_gpu"]["inflated_gpu"] >= 16 and st["gzip_gpu"]["inflate_errors"] == 0
            assert all(o.hits[p] == 1 for p in paths)
    finally:
        o.stop()


def test_gpu_inflate_matches_zlib(gz):
    """Batched GPU gunzip (one wave per member) against zlib-made members of every block
    type: stored (incompressible), fixed (tiny) and dynamic Huffman, multi-block, empty,
    long runs (distance 1 back-references), plus the GPU's own members; a corrupt member
    is rejected (None), never returned wrong."""
    rng = random.Random(11)
    bodies = [b"", b"a", b"hello world", b"x" * 100000, os.urandom(70000),
              _html(rng, 4096), _html(rng, 200000), bytes(range(256)) * 500,
              b"ab" * 40000 + os.urandom(300)]
    members = [gzip.compress(b, lvl) for b in bodies for lvl in (1, 6, 9)]
    members += gz.compress(bodies)
    want = [b for b in bodies for _ in (1, 6, 9)] + bodies
    got = gz.inflate(members)
    assert [g for g in got] == want
    bad = bytearray(members[15])
    bad[len(bad) // 2] ^= 0x40
    assert gz.inflate([bytes(bad)])[0] is None
    big = gzip.compress(b"\0" * (1 << 20))
    assert gz.inflate([big], 1000)[0] is None          # ISIZE over the cap: not decoded
    from shellac_amd.ops.gzip import gunzip_batch

    assert gunzip_batch([big, members[0]], max_out=2 << 20) == [b"\0" * (1 << 20), bodies[0]]


def test_gpu_ratio_close_to_zlib6(gz):
    """The lazy chained parse with per-block dynamic codes lands within 10 % of zlib -6's
    size on HTML-like text (verdict target: the miss path at a zlib-like ratio)."""
    rng = random.Random(3)
    bodies = [_html(rng, 8192) for _ in range(64)] + [_html(rng, 65536) for _ in range(8)]
    out = gz.compress(bodies)
    for b, o in zip(bodies, out):
        assert zlib.decompress(o, 31) == b
    ratio = sum(map(len, out)) / sum(map(len, bodies))
    z6 = sum(len(gzip.compress(b, 6)) for b in bodies) / sum(map(len, bodies))
    assert ratio <= 1.10 * z6, (ratio, z6)
