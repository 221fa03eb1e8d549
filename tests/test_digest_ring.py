"""Digest (MurmurHash3_x64_128) and consistent-hash ring tests (CPU)."""
import numpy as np
import pytest
import torch

M64 = (1 << 64) - 1


def _rotl(x, r):
    return ((x << r) | (x >> (64 - r))) & M64


def _fmix(k):
    k ^= k >> 33
    k = (k * 0xFF51AFD7ED558CCD) & M64
    k ^= k >> 33
    k = (k * 0xC4CEB9FE1A85EC53) & M64
    k ^= k >> 33
    return k


def murmur3_x64_128(data: bytes, seed: int):
    """Straight transcription of the public-domain reference algorithm."""
    c1, c2 = 0x87C37B91114253D5, 0x4CF5AD432745937F
    h1 = h2 = seed
    n = len(data) // 16
    for i in range(n):
        k1 = int.from_bytes(data[16 * i : 16 * i + 8], "little")
        k2 = int.from_bytes(data[16 * i + 8 : 16 * i + 16], "little")
        k1 = (k1 * c1) & M64; k1 = _rotl(k1, 31); k1 = (k1 * c2) & M64; h1 ^= k1
        h1 = _rotl(h1, 27); h1 = (h1 + h2) & M64; h1 = (h1 * 5 + 0x52DCE729) & M64
        k2 = (k2 * c2) & M64; k2 = _rotl(k2, 33); k2 = (k2 * c1) & M64; h2 ^= k2
        h2 = _rotl(h2, 31); h2 = (h2 + h1) & M64; h2 = (h2 * 5 + 0x38495AB5) & M64
    tail = data[16 * n :]
    k1 = k2 = 0
    if len(tail) > 8:
        k2 = int.from_bytes(tail[8:], "little")
        k2 = (k2 * c2) & M64; k2 = _rotl(k2, 33); k2 = (k2 * c1) & M64; h2 ^= k2
    if len(tail) > 0:
        k1 = int.from_bytes(tail[:8], "little")
        k1 = (k1 * c1) & M64; k1 = _rotl(k1, 31); k1 = (k1 * c2) & M64; h1 ^= k1
    h1 ^= len(data); h2 ^= len(data)
    h1 = (h1 + h2) & M64; h2 = (h2 + h1) & M64
    h1 = _fmix(h1); h2 = _fmix(h2)
    h1 = (h1 + h2) & M64; h2 = (h2 + h1) & M64
    return h1, h2


SEED = 0x5348454C4C414321


def test_digest_matches_reference_algorithm(core):
    rng = np.random.default_rng(0)
    cases = [b"", b"a", b"hello", b"/index.html", bytes(range(15)), bytes(range(16)),
             bytes(range(17)), bytes(range(33))]
    cases += [rng.integers(0, 256, size=int(n), dtype=np.uint8).tobytes()
              for n in rng.integers(0, 300, size=40)]
    for c in cases:
        assert core.digest(c) == murmur3_x64_128(c, SEED), c


def test_murmur_known_vector_seed0():
    # MurmurHash3_x64_128("", seed=0) is (0, 0) by construction of the algorithm.
    assert murmur3_x64_128(b"", 0) == (0, 0)


def test_digest_strings_batch(core):
    from shellac_amd.ops.cache import digest_strings

    keys = [f"/k/{i}".encode() * (i % 5 + 1) for i in range(100)]
    d = digest_strings(keys)
    for i, k in enumerate(keys):
        lo, hi = murmur3_x64_128(k, SEED)
        assert int(d[i, 0]) & M64 == lo and int(d[i, 1]) & M64 == hi


def test_ring_balance_and_minimal_remap():
    from shellac_amd.parallel.ring import ShardRing

    ring = ShardRing(list(range(8)), points_per_shard=160)
    rng = np.random.default_rng(1)
    pos = rng.integers(0, 2**32, size=40000, dtype=np.uint64)
    owners = np.array([ring.owner_of_position(int(p)) for p in pos])
    frac = np.bincount(owners, minlength=8) / len(owners)
    assert frac.min() > 0.08 and frac.max() < 0.17, frac
    # removing one shard moves ~1/8 of the key space, and only that shard's keys
    smaller = ring.without(3)
    moved = ring.moved_fraction(smaller)
    assert 0.08 < moved < 0.18, moved
    for p in pos[:3000]:
        a = ring.shards[ring.owner_of_position(int(p))]
        b = smaller.shards[smaller.owner_of_position(int(p))]
        assert a == b or a == 3


def test_ring_routing_op_matches_python(core):
    from shellac_amd.ops import routing as R
    from shellac_amd.ops.cache import digest_strings
    from shellac_amd.parallel.ring import ShardRing

    ring = ShardRing(list(range(5)), points_per_shard=40)
    keys = digest_strings([f"/r/{i}".encode() for i in range(500)])
    pts, own = ring.tensors("cpu")
    dest, counts = R.route(keys, pts, own, 5)
    for i in range(500):
        lo, hi = int(keys[i, 0]) & M64, int(keys[i, 1]) & M64
        assert int(dest[i]) == ring.owner_of_digest(lo, hi)
    assert counts.tolist() == torch.bincount(dest.long(), minlength=5).tolist()
    perm = R.scatter_positions(dest, counts)
    assert sorted(perm.tolist()) == list(range(500))
    grouped = R.permute(keys, perm)
    gd = R.permute(dest.view(-1, 1), perm).view(-1)
    assert torch.all(gd[1:] >= gd[:-1])
    assert torch.equal(grouped.index_select(0, perm), keys)
