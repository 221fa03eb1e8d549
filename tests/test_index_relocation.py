"""Index insert relocation: when all 8 slots of a new key's bucket pair are live, one entry
moves to a dead slot of its own other bucket (one cuckoo step) instead of the oldest being
evicted (hbm_cache.hip relocate_one / deferred_insert, host_cache.cc insert_locked).

A small Python model of the placement policy picks key sets on which the old policy
(evict at once) loses keys and the new one loses none; both engines must then keep every
key. The GPU batch path (k_set_index defers all-live rows to k_set_fixup) is checked on a
fill where racing inserts used to evict a live key in about 1 run in 4."""
import pytest
import torch

from shellac_amd.ops.cache import CacheShard, core, digest_strings, pack_values

M64 = (1 << 64) - 1


def _pairs(keys, nb):
    d = digest_strings(keys).tolist()
    return [tuple(core().bucket_pair(lo & M64, hi & M64, nb)) for lo, hi in d]


def _model_evictions(pairs, nb, relocate):
    """Sequential inserts of distinct keys, nothing expires: the engines' policy."""
    B = [[] for _ in range(nb)]
    ev = 0
    for k, (b1, b2) in enumerate(pairs):
        l1, l2 = len(B[b1]), len(B[b2])
        if l1 < 4 or l2 < 4:
            t = b1 if 4 - l1 >= 2 else (b2 if l2 < l1 and l2 < 4 else (b1 if l1 < 4 else b2))
            B[t].append(k)
            continue
        moved = False
        if relocate:
            for b in (b1, b2):
                for j, e in enumerate(B[b]):
                    x1, x2 = pairs[e]
                    ob = x2 if x1 == b else (x1 if x2 == b else b)
                    if ob != b and len(B[ob]) < 4:
                        B[ob].append(e)
                        B[b][j] = k
                        moved = True
                        break
                if moved:
                    break
        if not moved:
            ev += 1
            B[b1][0] = k  # (which one goes does not matter for the count)
    return ev


def _directed_keys(nb, n):
    for seed in range(500):
        keys = [f"/reloc/{seed}/{i}".encode() for i in range(n)]
        p = _pairs(keys, nb)
        if _model_evictions(p, nb, False) >= 2 and _model_evictions(p, nb, True) == 0:
            return keys
    raise AssertionError("no directed key set found")


def _check_keeps_every_key(dev):
    nb, n = 16, 44  # 69 % slot load
    keys = _directed_keys(nb, n)
    s = CacheShard(1 << 20, nb, 256, dev)
    for k in keys:  # one key per batch: the engines' sequential order
        s.set_many([k], [b"v1" + k])
    assert s.counters()["set_evicted"] == 0
    assert s.get_many(keys) == [b"v1" + k for k in keys]


def _check_no_stale_duplicates(dev):
    """A nearly full index (moves and evictions both happen), then every key updated, one
    at a time and then as one batch: no lookup may return an older value."""
    nb, n = 16, 60
    keys = [f"/dup/{i}".encode() for i in range(n)]
    s = CacheShard(1 << 22, nb, 256, dev)
    for gen in (1, 2):
        for k in keys:
            s.set_many([k], [b"v%d" % gen + k])
    s.set_many(keys, [b"v3" + k for k in keys])
    got = s.get_many(keys)
    live = [g for g in got if g is not None]
    assert all(g == b"v3" + k for g, k in zip(got, keys) if g is not None)
    assert 40 <= len(live) <= 64


def _model_place(pairs, nb):
    """The engines' placement of sequential distinct inserts (with one-step moves): the
    bucket lists, or None when some insert had to evict."""
    B = [[] for _ in range(nb)]
    for k, (b1, b2) in enumerate(pairs):
        l1, l2 = len(B[b1]), len(B[b2])
        if l1 < 4 or l2 < 4:
            t = b1 if 4 - l1 >= 2 else (b2 if l2 < l1 and l2 < 4 else (b1 if l1 < 4 else b2))
            B[t].append(k)
            continue
        moved = False
        for b in (b1, b2):
            for j, e in enumerate(B[b]):
                x1, x2 = pairs[e]
                ob = x2 if x1 == b else (x1 if x2 == b else b)
                if ob != b and len(B[ob]) < 4:
                    B[ob].append(e)
                    B[b][j] = k
                    moved = True
                    break
            if moved:
                break
        if not moved:
            return None
    return B


def _one_free_slot_setup(nb=16):
    """63 keys placed into 16 x 4 slots one at a time with no eviction (the index is full but
    for one slot, in bucket `free`), plus new keys whose pair excludes that bucket but holds
    an entry whose other bucket is it: inserting them in one batch makes every row of the
    batch race to relocate an entry into the same single free slot."""
    for seed in range(5000):
        keys = [f"/one/{seed}/{i}".encode() for i in range(63)]
        p = _pairs(keys, nb)
        B = _model_place(p, nb)
        if B is None:
            continue
        free = next(b for b in range(nb) if len(B[b]) < 4)
        movable = set()  # buckets holding an entry whose other bucket is `free`
        for b in range(nb):
            for e in B[b]:
                if free in p[e] and b != free:
                    movable.add(b)
        cand = [f"/one/{seed}/new{i}".encode() for i in range(4000)]
        cp = _pairs(cand, nb)
        new = [k for k, (b1, b2) in zip(cand, cp)
               if free not in (b1, b2) and (b1 in movable or b2 in movable)][:48]
        if len(movable) >= 3 and len(new) == 48:
            return keys, new
    raise AssertionError("no one-free-slot setup found")


def _check_single_free_slot_race(dev, pad=0):
    """Every row of one batch finds its pair all live and tries to move an entry into the
    one free slot of the index: at most one copy may land there, and no entry may pair one
    key's digest with another key's record (each hit returns its own value). `pad`: skip
    rows that make the batch a large one (GPU: k_set_index defers the rows, k_set_fixup's
    deferred_insert moves; unpadded it is the one-workgroup k_set_small)."""
    keys, new = _one_free_slot_setup()
    for trial in range(8):
        s = CacheShard(1 << 22, 16, 256, dev)
        for k in keys:
            s.set_many([k], [b"old" + k])
        assert s.counters()["set_evicted"] == 0
        vals = [b"new%d" % trial + k for k in new]
        if pad:
            d = torch.zeros((pad, 2), dtype=torch.int64)
            d[: len(new)] = digest_strings(new)
            v, vo, vl = pack_values(vals + [b""] * (pad - len(new)))
            vl[len(new):] = -1  # kSkipVlen rows
            vo[len(new):] = 0
            s.store(d.to(dev), v.to(dev), vo.to(dev), vl.to(dev))
        else:
            s.set_many(new, vals)
        allk = keys + new
        want = [b"old" + k for k in keys] + [b"new%d" % trial + k for k in new]
        got = s.get_many(allk)
        wrong = [(k, g) for k, g, w in zip(allk, got, want) if g is not None and g != w]
        assert not wrong, wrong[:4]
        assert sum(g is not None for g in got) >= len(new)
        c = s.counters()
        assert c["set_evicted"] + c["set_dropped"] >= len(new) - 1, c


@pytest.mark.parametrize("pad", [0, 1024])
def test_single_free_slot_relocation_race_host(pad):
    _check_single_free_slot_race("cpu", pad)


@pytest.mark.gpu
@pytest.mark.parametrize("pad", [0, 1024])
def test_single_free_slot_relocation_race_gpu(cuda_dev, pad):
    _check_single_free_slot_race(cuda_dev, pad)


def test_relocation_keeps_every_key_host():
    _check_keeps_every_key("cpu")


def test_relocation_no_stale_duplicates_host():
    _check_no_stale_duplicates("cpu")


@pytest.mark.gpu
def test_relocation_keeps_every_key_gpu(cuda_dev):
    _check_keeps_every_key(cuda_dev)


@pytest.mark.gpu
def test_relocation_no_stale_duplicates_gpu(cuda_dev):
    _check_no_stale_duplicates(cuda_dev)


@pytest.mark.gpu
def test_batch_fill_keeps_every_key_gpu(cuda_dev):
    """40K keys in 32K buckets (30 % slot load) in 10K-row batches: racing inserts may
    find a pair all live; k_set_fixup then moves an entry instead of evicting one."""
    from shellac_amd.bench.workload import Workload

    wl = Workload(40000, cuda_dev)
    for _ in range(4):
        shard = CacheShard(256 << 20, 1 << 15, 1 << 16, cuda_dev)
        for s0 in range(0, 40000, 10000):
            b = wl.set_batch(torch.arange(s0, s0 + 10000, device=cuda_dev))
            shard.store(b.keys, b.values, b.val_off, b.vlen, b.flags, b.expire)
        lk = shard.lookup(wl.digests)
        torch.cuda.synchronize()
        c = shard.counters()
        assert c["set_evicted"] == 0 and c["set_dropped"] == 0, c
        assert int((lk.size[:40000] == 0).sum()) == 0
