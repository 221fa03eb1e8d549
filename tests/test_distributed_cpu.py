"""Multi-process sharded cache over gloo (CPU shards, world_size 2 and 3)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_world(target, world, *args, timeout=240):
    """Spawn `world` ranks of target(rank, world, port, q, *args); fail fast if one dies."""
    import queue
    import time

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    results, t0 = [], time.time()
    try:
        while len(results) < world:
            try:
                results.append(q.get(timeout=1))
                if results[-1][1] != "ok":
                    break  # a failed rank: its peers may wait in a collective forever
            except queue.Empty:
                dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
                assert not dead, f"rank exited with {dead} before reporting"
                assert time.time() - t0 < timeout, "distributed test timed out"
    finally:
        failed = any(r[1] != "ok" for r in results)
        for p in procs:
            p.join(timeout=2 if failed else 30)
            if p.is_alive():
                p.kill()
    fails = [r for r in results if r[1] != "ok"]
    assert not fails, "\n".join(f"rank {r[0]}: {r[2]}" for r in fails)
    return results


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from shellac_amd.models.sharded_cache import SetBatch, ShardedCache
        from shellac_amd.ops.cache import CacheShard, digest_strings, pack_values, unpack_records

        shard = CacheShard(1 << 22, 1 << 12, 1 << 14, "cpu")
        sc = ShardedCache(shard)
        # every rank writes its own keys (some colliding keys written by all ranks)
        keys = [f"/r{rank}/{i}".encode() for i in range(300)] + [b"/shared"]
        vals = [f"{rank}:{i}".encode() * (1 + i % 11) for i in range(300)] + [b"s"]
        v, vo, vl = pack_values(vals)
        sc.set(SetBatch(digest_strings(keys), v, vo, vl,
                        flags=torch.full((301,), rank, dtype=torch.int32)))
        dist.barrier()
        # read everybody's keys
        allkeys, expect = [], []
        for r in range(world):
            allkeys += [f"/r{r}/{i}".encode() for i in range(300)]
            expect += [f"{r}:{i}".encode() * (1 + i % 11) for i in range(300)]
        allkeys += [b"/nothing-here", b"/shared"]
        res = sc.get(digest_strings(allkeys))
        recs = unpack_records(res.data, res.off, res.size)
        got = [r[0] if r else None for r in recs]
        assert got[: len(expect)] == expect
        assert got[-2] is None and got[-1] == b"s"
        # flags travel with the payload
        assert all(recs[r * 300][1] == r for r in range(world))
        # keys live only on their owner shard
        owned = shard.sweep()[0]
        total = sc.counters()
        gathered = [None] * world
        dist.all_gather_object(gathered, owned)
        assert sum(gathered) == 300 * world + 1
        # delete through the routed path
        found = sc.delete(digest_strings([f"/r{(rank + 1) % world}/0".encode(), b"/zz"]))
        assert found.tolist() == [True, False]
        dist.barrier()
        q.put((rank, "ok", total["get_ops"]))
    except BaseException as e:  # surface the failure in the parent
        import traceback

        q.put((rank, "fail", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_cache_gloo(world):
    results = _run_world(_worker, world)
    assert all(r[2] == world * (300 * world + 2) for r in results)


def _replica_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from shellac_amd.models.sharded_cache import SetBatch, ShardedCache
        from shellac_amd.ops.cache import CacheShard, digest_strings, pack_values, unpack_records

        shard = CacheShard(1 << 22, 1 << 12, 1 << 14, "cpu")
        replica = CacheShard(1 << 20, 1 << 10, 1 << 14, "cpu")
        sc = ShardedCache(shard, replica=replica)
        keys = [f"/k{i}".encode() for i in range(400)]
        if rank == 0:
            v, vo, vl = pack_values([b"v1-" + k for k in keys])
            batch = SetBatch(digest_strings(keys), v, vo, vl)
        else:
            v, vo, vl = pack_values([])
            batch = SetBatch(digest_strings([]), v, vo, vl)
        sc.set(batch)
        dist.barrier()
        hot = keys[:20]
        reqs = digest_strings(hot * 10 + keys[100:120])   # hot keys dominate the sample
        res = sc.get(reqs)
        nrep = sc.refresh_replica(20)
        owned = sum(sc.ring.owner_of_key(k) == rank for k in hot)
        assert nrep == 20 - owned, (nrep, owned)
        before = sc.stats["replica_hits"]
        res = sc.get(digest_strings(keys))
        got = [r[0] if r else None for r in unpack_records(res.data, res.off, res.size)]
        assert got == [b"v1-" + k for k in keys]
        assert sc.stats["replica_hits"] - before == 20 - owned  # hot keys served locally
        # write-through: rank 1 overwrites hot keys; everybody must see the new values
        if rank == 1:
            v, vo, vl = pack_values([b"v2-" + k for k in hot])
            batch = SetBatch(digest_strings(hot), v, vo, vl)
        else:
            v, vo, vl = pack_values([])
            batch = SetBatch(digest_strings([]), v, vo, vl)
        sc.set(batch)
        dist.barrier()
        res = sc.get(digest_strings(hot))
        got = [r[0] if r else None for r in unpack_records(res.data, res.off, res.size)]
        assert got == [b"v2-" + k for k in hot], got[:2]
        # deletes drop replicas everywhere
        found = sc.delete(digest_strings(hot[:5] if rank == 0 else []))
        dist.barrier()
        res = sc.get(digest_strings(hot[:6]))
        got = [r[0] if r else None for r in unpack_records(res.data, res.off, res.size)]
        assert got[:5] == [None] * 5 and got[5] == b"v2-" + hot[5]
        q.put((rank, "ok", 0))
    except BaseException:
        import traceback

        q.put((rank, "fail", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_hot_object_replication_gloo(world):
    _run_world(_replica_worker, world)


def _membership_worker(rank, world, port, q, snapdir):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from shellac_amd.models.sharded_cache import SetBatch, ShardedCache
        from shellac_amd.ops.cache import CacheShard, digest_strings, pack_values, unpack_records

        def mk():
            return CacheShard(1 << 22, 1 << 12, 1 << 14, "cpu")

        sc = ShardedCache(mk())
        def put(keys, tag):
            mine = keys if rank == 0 else []
            v, vo, vl = pack_values([tag + k for k in mine])
            sc.set(SetBatch(digest_strings(mine), v, vo, vl))
            dist.barrier()

        def read(keys):
            res = sc.get(digest_strings(keys))
            return [r[0] if r else None for r in unpack_records(res.data, res.off, res.size)]

        keys = [f"/m{i}".encode() for i in range(300)]
        put(keys, b"a-")
        owner = {k: sc.ring.owner_of_key(k) for k in keys}
        # shard 1 fails: its keys miss, everything else still hits
        sc.fail_shard(1)
        got = read(keys)
        for k, g in zip(keys, got):
            assert (g is None) == (owner[k] == 1), (k, g)
        # writes during the outage land on the interim owners
        late = [f"/late{i}".encode() for i in range(100)]
        put(late, b"b-")
        assert read(late) == [b"b-" + k for k in late]
        # warm restore: shard 1 rejoins and pulls back its keys from peers
        sc.restore_shard(1)
        assert read(late) == [b"b-" + k for k in late]
        full = sc.ring
        late_owned = sum(full.owner_of_key(k) == 1 for k in late)
        assert late_owned > 0
        if rank == 1:
            assert sc.shard.sweep()[0] >= late_owned
        # snapshot + warm restart of every shard
        sc.save(snapdir)
        dist.barrier()
        sc2 = ShardedCache(mk())
        sc2.load(snapdir)
        sc = sc2
        assert read(late) == [b"b-" + k for k in late]
        q.put((rank, "ok", 0))
    except BaseException:
        import traceback

        q.put((rank, "fail", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_shard_failure_rebalance_and_snapshot_gloo(tmp_path):
    _run_world(_membership_worker, 3, str(tmp_path))


def _serve_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from shellac_amd.models.sharded_cache import SKIP_VLEN, SetBatch, ShardedCache
        from shellac_amd.ops.cache import CacheShard, digest_strings, pack_values, unpack_records

        shard = CacheShard(1 << 22, 1 << 12, 1 << 14, "cpu")
        replica = CacheShard(1 << 20, 1 << 10, 1 << 14, "cpu")
        sc = ShardedCache(shard, replica=replica, routed=True)  # world 1: routed anyway

        def batch(keys, vals, skip_last=False):
            v, vo, vl = pack_values(vals)
            if skip_last and len(vals):
                vl[-1] = SKIP_VLEN          # a row with no value (e.g. a refetch miss)
            return SetBatch(digest_strings(keys), v, vo, vl,
                            flags=torch.full((len(keys),), rank, dtype=torch.int32))

        def values(res):
            return [r[0] if r else None for r in unpack_records(res.data, res.off, res.size)]

        keys = [f"/s{r}/{i}".encode() for r in range(world) for i in range(150)]
        mine = [k for k in keys if k.startswith(f"/s{rank}/".encode())]
        # step 1: GETs of everything (all misses) + every rank fills its own keys
        res = sc.serve(digest_strings(keys), batch(mine, [b"v1" + k * (1 + len(k) % 5)
                                                          for k in mine]))
        assert values(res) == [None] * len(keys)
        hot = keys[:10] + keys[-10:]
        sc.get(digest_strings(hot * 8))
        sc.refresh_replica(20)
        # step 2: GETs see the state before this step's SETs (hot and cold overwrites)
        upd = hot[:6] + keys[40:60] if rank == 1 else []
        v1 = [b"v1" + k * (1 + len(k) % 5) for k in keys]
        res = sc.serve(digest_strings(keys + [b"/none"]),
                       batch(upd + [b"/skipped"], [b"v2" + k for k in upd] + [b"x"],
                             skip_last=True))
        assert values(res) == v1 + [None]
        # step 3: the overwrites are visible everywhere (replicas written through)
        res = sc.serve(digest_strings(keys + [b"/skipped"]), batch([], []))
        expect = {k: b"v2" + k for k in hot[:6] + keys[40:60]} if world > 1 else {}
        assert values(res) == [expect.get(k, v) for k, v in zip(keys, v1)] + [None]
        flags = [r[1] if r else None for r in unpack_records(res.data, res.off, res.size)]
        assert (flags[40], flags[0]) == ((1, 1) if world > 1 else (0, 0))
        assert sc.stats["replica_hits"] > 0 or world == 1  # world 1: every key is local
        q.put((rank, "ok", 0))
    except BaseException:
        import traceback

        q.put((rank, "fail", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3])
def test_fused_serve_step_gloo(world):
    _run_world(_serve_worker, world)


def _drift_worker(rank, world, port, q):
    """Incremental replica maintenance: the hot set drifts; a refresh fetches newly hot keys
    under a byte budget (the rest follow at the next refresh) and drops as many keys that
    cooled (deleted from the replica, no longer written through: an update of one at its
    owner is never shadowed by a stale copy), without flushing the replica."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from shellac_amd.models.sharded_cache import SetBatch, ShardedCache
        from shellac_amd.ops.cache import CacheShard, digest_strings, pack_values, unpack_records

        sc = ShardedCache(CacheShard(1 << 22, 1 << 12, 1 << 14, "cpu"),
                          replica=CacheShard(1 << 21, 1 << 10, 1 << 14, "cpu"))
        keys = [f"/d{i}".encode() for i in range(600)]

        def put(ks, tag, who=0):
            mine = ks if rank == who else []
            v, vo, vl = pack_values([tag + k for k in mine])
            sc.set(SetBatch(digest_strings(mine), v, vo, vl))

        def read(ks):
            res = sc.get(digest_strings(ks))
            return [r[0] if r else None for r in unpack_records(res.data, res.off, res.size)]

        put(keys, b"a-" + b"x" * 200)
        a = keys[:40]
        b = keys[30:70]       # 10 stay hot, 30 cool down, 30 heat up
        sc.refresh_replica(40, keys=digest_strings(a * 5))
        assert sc._hot.shape[0] == 40
        r0 = sc.stats["replica_refreshes"]
        # the drift: b is hot now; a budget of ~10 records per call on every rank
        budget = 10 * 260
        sc.refresh_replica(40, keys=digest_strings(b * 5), budget_bytes=budget, chunk_keys=8)
        hot = {tuple(x) for x in sc._hot.tolist()}
        want_b = {tuple(x) for x in digest_strings(b).tolist()}
        gone = {tuple(x) for x in digest_strings(keys[:30]).tolist()}
        # the budget held some newly hot keys back: cooled keys leave only for fetched ones
        assert len(hot) == 40 and 10 < len(hot & want_b) < 40, len(hot & want_b)
        assert len(hot & gone) == 40 - len(hot & want_b)
        # a cooled key updated at its owner: nobody may see the stale replica copy
        put(keys[:5], b"c-", who=world - 1)
        assert read(keys[:5]) == [b"c-" + k for k in keys[:5]]
        # the next refreshes bring the rest of b in
        sc.refresh_replica(40, keys=digest_strings(b * 5), budget_bytes=budget, chunk_keys=8)
        sc.refresh_replica(40, keys=digest_strings(b * 5))
        hot = {tuple(x) for x in sc._hot.tolist()}
        assert hot == want_b and not (hot & gone)
        assert sc.stats["replica_refreshes"] == r0 + 3
        before = sc.stats["replica_hits"]
        got = read(b)
        assert got == [b"a-" + b"x" * 200 + k for k in b]
        owned = sum(sc.ring.owner_of_key(k) == rank for k in b)
        assert sc.stats["replica_hits"] - before == 40 - owned
        q.put((rank, "ok", 0))
    except BaseException:
        import traceback

        q.put((rank, "fail", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_incremental_replica_refresh_gloo(world):
    _run_world(_drift_worker, world)


def _migrate_worker(rank, world, port, q):
    """A ring change migrated incrementally (a byte budget per call between steps): every
    GET in the meantime returns the right value or a miss, never a wrong one, and once the
    migration is done every key hits on its new owner."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from shellac_amd.models.sharded_cache import SetBatch, ShardedCache
        from shellac_amd.ops.cache import CacheShard, digest_strings, pack_values, unpack_records
        from shellac_amd.parallel.ring import ShardRing

        sc = ShardedCache(CacheShard(1 << 22, 1 << 12, 1 << 14, "cpu"))
        keys = [f"/g{i}".encode() for i in range(900)]
        mine = keys[rank::world]
        v, vo, vl = pack_values([b"m-" + k for k in mine])
        sc.set(SetBatch(digest_strings(mine), v, vo, vl))

        def read(ks):
            res = sc.get(digest_strings(ks))
            return [r[0] if r else None for r in unpack_records(res.data, res.off, res.size)]

        new = ShardRing(list(range(world)), 97)   # another continuum: many keys move
        n = sc.set_ring(new, incremental=True, chunk_keys=16)
        # the value every key must end with: writes and deletes land on the new owners
        # between migrate_step calls (every rank issues a slice of them), and no migrated
        # (older) copy may overwrite a newer value or bring a deleted key back
        want = {k: b"m-" + k for k in keys}
        calls = 0
        while True:
            got = read(keys)
            assert all(g is None or g == want[k] for g, k in zip(got, keys)), calls
            calls += 1
            upd = keys[(37 * calls) % 900::53][:6]
            dele = keys[(11 * calls + 5) % 900::71][:4]
            v, vo, vl = pack_values([b"u%d-" % calls + k for k in upd[rank::world]])
            sc.set(SetBatch(digest_strings(upd[rank::world]), v, vo, vl))
            sc.delete(digest_strings(dele[rank::world]))
            for k in upd:
                want[k] = b"u%d-" % calls + k
            for k in dele:
                want[k] = None
            if not sc.migrate_step(budget_bytes=16 * 40):
                break
        assert calls > 2 or n == 0
        assert read(keys) == [want[k] for k in keys]
        q.put((rank, "ok", 0))
    except BaseException:
        import traceback

        q.put((rank, "fail", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_incremental_ring_migration_gloo(world):
    _run_world(_migrate_worker, world)


def _local_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from shellac_amd.models.sharded_cache import SetBatch, ShardedCache
        from shellac_amd.ops.cache import CacheShard, digest_strings, pack_values, unpack_records
        from shellac_amd.parallel.exchange import LocalComm

        # a host-routed rank: its cache serves the keys the host sent it and never takes
        # part in a collective, so ranks may make different numbers of calls
        sc = ShardedCache(CacheShard(1 << 22, 1 << 12, 1 << 14, "cpu"), group=LocalComm())
        assert (sc.world, sc.routed) == (1, False)
        n_batches = 1 + 2 * rank
        for b in range(n_batches):
            keys = [f"/r{rank}/{b}/{i}".encode() for i in range(50)]
            v, vo, vl = pack_values([k * 2 for k in keys])
            sc.set(SetBatch(digest_strings(keys), v, vo, vl))
        mine = [f"/r{rank}/{b}/{i}".encode() for b in range(n_batches) for i in range(50)]
        other = [f"/r{(rank + 1) % world}/0/{i}".encode() for i in range(50)]
        res = sc.get(digest_strings(mine + other))
        recs = unpack_records(res.data, res.off, res.size)
        assert [r[0] for r in recs[: len(mine)]] == [k * 2 for k in mine]
        assert all(r is None for r in recs[len(mine):])  # another rank's keys stay there
        assert sc.counters()["get_ops"] == len(mine) + len(other)  # this shard only
        dist.barrier()
        q.put((rank, "ok", None))
    except BaseException:
        import traceback

        q.put((rank, "fail", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_local_group_never_routes_gloo():
    """A host-routed rank (bench.py --route host) holds a default process group for the
    barriers and reductions around its steps; its cache must not route over it. With
    group=None it would (the default group), and ranks that made different numbers of
    SET calls deadlocked in the first count exchange (seen on a 2-rank GPU rehearsal)."""
    _run_world(_local_worker, 2, timeout=120)


def _spread_worker(rank, world, port, q, rank_policy):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import torch

        from shellac_amd.bench.workload import Workload
        from shellac_amd.models.sharded_cache import ShardedCache
        from shellac_amd.ops.cache import CacheShard, unpack_records
        from shellac_amd.parallel.exchange import LocalComm
        from shellac_amd.parallel.hotspread import HotSpread, member, replicate_hot, water_fill

        N = 6000 * world
        wl = Workload(N, "cpu", min_val=16, max_val=512, pool_bytes=1 << 20)
        hs = HotSpread(world, "cpu")
        owner = hs.owners(wl.digests).long()
        # the hot set and spray weights from an observed sample (the same on every rank)
        sample = wl.sample_ids(50000, 8)
        u, cnt = torch.unique(sample, return_counts=True)
        hot_ids = u[torch.sort(-cnt, stable=True).indices[:200]]
        hmask = torch.zeros(N, dtype=torch.bool)
        hmask[hot_ids] = True
        hsamp = hmask[sample]
        share = torch.bincount(owner[sample[~hsamp]], minlength=world).double() / sample.numel()
        if rank_policy == "spray":
            hs.set_hot(wl.digests[hot_ids], None,
                       water_fill(share.tolist(), float(hsamp.float().mean())))
        else:
            hs.plan(wl.digests[sample], 200)      # (ties at the cut may pick other keys)
            hot_ids = torch.nonzero(member(wl.digests, hs.hot)).flatten()
            hmask = torch.zeros(N, dtype=torch.bool)
            hmask[hot_ids] = True
            assert hot_ids.numel() == 200 and int((hs.hot_rank >= 0).sum()) > 150
        # a host-routed rank: its own keys, then the hot objects it does not own, fetched
        # from their owners with one all-gather of records
        sc = ShardedCache(CacheShard(16 << 20, 1 << 14, 1 << 12, "cpu"), group=LocalComm())
        sc.set(wl.set_batch(torch.nonzero(owner == rank).flatten()))
        got = replicate_hot(sc, hs.hot, hs.owners(hs.hot), rank, world)
        want = int((hmask & (owner != rank)).sum())
        assert got == want, (got, want)
        version = torch.zeros(N, dtype=torch.int64)
        served = torch.zeros(world, dtype=torch.int64)
        for step in range(3):
            g = wl.sample_ids(4000 * world, 100 + step)           # one global GET stream
            gd = hs.route_gets(wl.digests[g], seq0=step * 4000 * world)
            hd, _ = hs.host_route_gets(wl.digests[g].contiguous(), seq0=step * 4000 * world,
                                       threads=2)
            assert torch.equal(gd, hd)
            st = wl.uniform_ids(300 * world, 200 + step)           # one global SET stream
            st = torch.cat([st, hot_ids[step::7]])                 # hot objects are updated too
            sd = hs.route_sets(wl.digests[st])
            mine_g = g[gd == rank]
            mine_s = st[(sd == rank) | (sd < 0)]
            vb = wl.set_batch(mine_s, version=step + 1)
            r = sc.serve(wl.digests[mine_g].contiguous(), vb)
            recs = unpack_records(r.data, r.off, r.size)
            for i, x in zip(mine_g.tolist(), recs):
                assert x is not None, (step, i)                   # owners and replicas hit
                assert x[0] == wl.expected_value(i, int(version[i])), (step, i)
            version[st] = step + 1        # GETs of the next step see this step's SETs
            served[rank] += mine_g.numel() + mine_s.numel()
        dist.all_reduce(served)
        mean = served.double().mean()
        assert float(served.max() / mean) < 1.08, served.tolist()
        q.put((rank, "ok", 0))
    except BaseException:
        import traceback

        q.put((rank, "fail", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world,policy", [(2, "designate"), (3, "designate"), (3, "spray")])
def test_host_routed_true_shares_with_hot_spreading_gloo(world, policy):
    """The host-routed topology end to end on CPU ranks: one global Zipf stream routed by
    ketama with the hottest objects replicated on every rank (filled from their owners by an
    all-gather) and their GETs sprayed, their SETs written through everywhere. Every rank
    serves exactly its share, every GET of it returns the version the SETs of earlier steps
    left, wherever it was sent, and the ranks' loads stay within a few percent."""
    _run_world(_spread_worker, world, policy)


def _spread_refresh_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import torch

        from shellac_amd.bench.workload import Workload
        from shellac_amd.models.sharded_cache import ShardedCache
        from shellac_amd.ops.cache import CacheShard, unpack_records
        from shellac_amd.parallel.exchange import LocalComm
        from shellac_amd.parallel.hotspread import HotSpread, member, refresh_hot, replicate_hot

        N = 6000 * world
        wl = Workload(N, "cpu", min_val=16, max_val=512, pool_bytes=1 << 20)
        hs = HotSpread(world, "cpu")
        owner = hs.owners(wl.digests).long()
        sc = ShardedCache(CacheShard(16 << 20, 1 << 14, 1 << 12, "cpu"), group=LocalComm())
        sc.set(wl.set_batch(torch.nonzero(owner == rank).flatten()))
        hs.plan(wl.digests[wl.sample_ids(50000, 8)], 200)
        replicate_hot(sc, hs.hot, hs.owners(hs.hot), rank, world)
        version = torch.zeros(N, dtype=torch.int64)

        def steps(order, first, count):
            for step in range(first, first + count):
                g = wl.sample_ids(4000 * world, 100 + step, rank_to_id=order)
                gd = hs.route_gets(wl.digests[g], seq0=step * 4000 * world)
                st = torch.cat([wl.uniform_ids(300 * world, 200 + step),
                                order[step % 5:400:5]])      # hot (old and new) objects too
                sd = hs.route_sets(wl.digests[st])
                mine_g, mine_s = g[gd == rank], st[(sd == rank) | (sd < 0)]
                r = sc.serve(wl.digests[mine_g].contiguous(),
                             wl.set_batch(mine_s, version=step + 1))
                for i, x in zip(mine_g.tolist(), unpack_records(r.data, r.off, r.size)):
                    assert x is not None, (step, i)
                    assert x[0] == wl.expected_value(i, int(version[i])), (step, i)
                version[st] = step + 1

        order0 = wl.rank_to_id
        steps(order0, 0, 2)
        old_hot = hs.hot.clone()
        # the popularity drifts: 120 of the top 200 trade places with tail objects
        order1 = wl.drifted(order0, 200, 120, 4242)
        # a budget that admits about half of the newly hot objects' copies
        info = refresh_hot(sc, hs, wl.digests[wl.sample_ids(50000, 9, rank_to_id=order1)], 200,
                           rank, world, budget_bytes=60 * 260 * (world - 1))
        assert info["added"] > 20 and info["deferred"] > 20 and info["removed"] > 20, info
        # the cooled objects' replicas are gone from the ranks that do not own them
        cooled = old_hot[~member(old_hot, hs.hot)]
        not_mine = cooled[hs.owners(cooled).long() != rank]
        assert int((sc.shard.lookup(not_mine).size[: not_mine.shape[0]] > 0).sum()) == 0
        steps(order1, 2, 3)
        # back to the first order: objects demoted above (and SET meanwhile at their owners
        # only) are promoted again and must be fetched fresh
        refresh_hot(sc, hs, wl.digests[wl.sample_ids(50000, 10, rank_to_id=order0)], 200,
                    rank, world)
        steps(order0, 5, 2)
        q.put((rank, "ok", 0))
    except BaseException:
        import traceback

        q.put((rank, "fail", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_host_routed_hot_set_refresh_gloo(world):
    """The host-routed hot set follows a drifting popularity order incrementally
    (parallel/hotspread.py refresh_hot): only newly hot objects are fetched, within a byte
    budget (the rest wait), cooled objects' replicas are dropped, and every GET before,
    after and across two refreshes (one promoting objects demoted earlier, which were SET at
    their owners meanwhile) returns the version the SETs left."""
    _run_world(_spread_refresh_worker, world)
