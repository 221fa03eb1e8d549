"""The fused routed serving step across real processes (GPU): 2 and 3 ranks, each with
its own shard and replica on the box's one GPU, collectives bounced through gloo
(BounceComm: RCCL refuses two ranks on one device). Unlike the single-process mirror
(MirrorComm), traffic here is asymmetric and every owner is a different process —
the path the 8-GPU scaling run takes, minus RCCL itself."""
import os

import pytest
import torch
import torch.distributed as dist

from test_distributed_cpu import _run_world

pytestmark = pytest.mark.gpu


def _routed_worker(rank, world, port, q, backend="bounce"):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        stack_dir = os.environ.get("SHELLAC_TEST_STACKS")
        if stack_dir:  # a hung rank leaves its Python stack here (diagnostics)
            import faulthandler

            faulthandler.dump_traceback_later(
                60, exit=False, file=open(os.path.join(stack_dir, f"rank{rank}.stack"), "w"))
        from shellac_amd.models.sharded_cache import SetBatch, ShardedCache
        from shellac_amd.ops.cache import CacheShard, digest_strings, pack_values, unpack_records
        from shellac_amd.parallel.exchange import BounceComm

        dev = torch.device("cuda", 0)
        shard = CacheShard(64 << 20, 1 << 12, 1 << 14, dev)
        replica = CacheShard(16 << 20, 1 << 10, 1 << 14, dev)
        if backend == "rccl":
            # one rank on a real RCCL communicator (plus the second, data communicator
            # bench.py opens): every collective call of the routed step goes through RCCL
            torch.cuda.set_device(dev)
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
            data = dist.new_group(ranks=list(range(world)))
            sc = ShardedCache(shard, replica=replica, data_group=data, routed=True)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
            sc = ShardedCache(shard, group=BounceComm(), replica=replica)
        assert sc.fused and sc.coalesce and sc.routed

        def batch(keys, vals):
            v, vo, vl = pack_values(vals, dev)
            return SetBatch(digest_strings(keys, dev), v, vo, vl,
                            flags=torch.full((len(keys),), rank, dtype=torch.int32, device=dev))

        def values(res):
            res.wait()
            return [r[0] if r else None for r in unpack_records(res.data, res.off, res.size)]

        keys = [f"/m{r}/{i}".encode() for r in range(world) for i in range(200)]
        mine = [k for k in keys if k.startswith(f"/m{rank}/".encode())]
        v1 = {k: b"v1" + k * (1 + len(k) % 7) for k in keys}
        # step 1: every rank fills its own keys; GETs (with duplicates) all miss
        dup = keys[:50] * 3
        res = sc.serve(digest_strings(keys + dup, dev), batch(mine, [v1[k] for k in mine]))
        assert values(res) == [None] * (len(keys) + len(dup))
        # hot set from a skewed sample, replicated on every rank
        sc.get(digest_strings(keys[:20] * 10, dev))
        sc.refresh_replica(20)
        # step 2: duplicate-heavy GET batch, every key owned somewhere else or here;
        # the last rank overwrites some hot and cold keys (GETs see the state before the SETs)
        upd = keys[:5] + keys[100:110] if rank == world - 1 else []
        req = keys[:30] * 5 + keys + [b"/none"] * 3
        res = sc.serve(digest_strings(req, dev), batch(upd, [b"v2" + k for k in upd]))
        got = values(res)
        want = [v1[k] for k in req[:-3]] + [None] * 3
        bad = [(i, req[i], (g or b"")[:12], (w or b"")[:12]) for i, (g, w) in
               enumerate(zip(got, want)) if g != w]
        if bad:  # diagnostics: which owners, hot or not, and this rank's step counters
            owners, _ = sc._route(digest_strings([b[1] for b in bad], dev))
            hot = sc._is_hot(digest_strings([b[1] for b in bad], dev))
            by_owner = torch.bincount(owners.long(), minlength=world).tolist()
            info = (f"by owner {by_owner}, hot {int(hot.sum())}, stats {sc.stats}, "
                    f"counters {shard.counters()}")
        assert not bad, f"rank {rank}: {len(bad)} wrong GETs, first {bad[:6]}; {info}"
        # step 3: the overwrites are visible on every rank (replicas written through)
        res = sc.serve(digest_strings(req, dev), batch([], []))
        new = {k: b"v2" + k for k in keys[:5] + keys[100:110]}
        got = values(res)
        want = [new.get(k, v1[k]) for k in req[:-3]] + [None] * 3
        bad = [(i, req[i], (g or b"")[:12], (w or b"")[:12]) for i, (g, w) in
               enumerate(zip(got, want)) if g != w]
        assert not bad, f"rank {rank} step 3: {len(bad)} wrong GETs, first {bad[:6]}"
        # steps 4-9: the same shapes, the last rank updating 8 keys per step; from the third
        # native step on, SET appends start early under the previous probe's look-ahead
        # reserve. Every step's GETs see exactly the SETs of the steps before it.
        cur = dict(v1)
        cur.update(new)
        for t in range(6):
            upd_t = keys[120 + 8 * t: 128 + 8 * t]
            vals_t = {k: b"v3-%d-" % t + k for k in upd_t}
            mine_upd = upd_t if rank == world - 1 else []
            res = sc.serve(digest_strings(req, dev), batch(mine_upd, [vals_t[k] for k in mine_upd]))
            got = values(res)
            want = [cur[k] for k in req[:-3]] + [None] * 3
            bad = [(i, req[i], (g or b"")[:12], (w or b"")[:12]) for i, (g, w) in
                   enumerate(zip(got, want)) if g != w]
            assert not bad, f"rank {rank} step {4 + t}: {len(bad)} wrong GETs, first {bad[:6]}"
            cur.update(vals_t)
        # forced SET overflow: tiny SET slots (the same on every rank) for one step, in which
        # every rank updates 100 keys; the rows that do not fit are carried, and once the
        # capacities are learned again every update is visible within two steps
        e = sc._engine
        e.set_set_cap_override(16, 8 << 10, 16, 8 << 10)
        upd_f = keys[rank * 100: rank * 100 + 100]
        vals_f = {k: b"vf-%d-" % rank + k for k in upd_f}
        sc.serve(digest_strings(req, dev), batch(upd_f, [vals_f[k] for k in upd_f])).wait()
        e.set_set_cap_override(0, 0, 0, 0)
        for _ in range(2):
            sc.serve(digest_strings(req, dev), batch([], [])).wait()
        for r in range(world):
            cur.update({k: b"vf-%d-" % r + k for k in keys[r * 100: r * 100 + 100]})
        res = sc.serve(digest_strings(req, dev), batch([], []))
        got = values(res)
        want = [cur[k] for k in req[:-3]] + [None] * 3
        bad = [(i, req[i], (g or b"")[:12], (w or b"")[:12]) for i, (g, w) in
               enumerate(zip(got, want)) if g != w]
        assert not bad, f"rank {rank} after forced SET overflow: {len(bad)} wrong, {bad[:6]}"
        carried, _, lost = e.carry_stats()
        assert carried > 0 and lost == 0, (carried, lost)
        st = sc.stats
        assert st["coalesced_gets"] > 0
        # world 1: every key is local (no remote GETs, the replica is never consulted)
        assert (st["replica_hits"] > 0 and st["remote_gets"] > 0) or world == 1
        q.put((rank, "ok", 0))
    except BaseException:
        import traceback

        q.put((rank, "fail", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_fused_routed_step_multiprocess(world):
    _run_world(_routed_worker, world, timeout=120)


def test_routed_step_over_rccl_one_rank():
    """The fused routed step (routing, 5 all-to-alls with the SET payloads on a second
    communicator, replica refresh by all_gather, stats all-reduce) over a real RCCL
    communicator of one rank: the collective calls the 8-GPU scaling run makes, on the
    one GPU this box has."""
    _run_world(_routed_worker, 1, "rccl", timeout=180)
