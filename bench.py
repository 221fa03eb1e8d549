#!/usr/bin/env python3
"""Flagship benchmark: sharded HBM web-cache serving step (one process per GPU).

Contract (see task README): ``python bench.py --gpus N --steps K --warmup W``;
for N>1 launched by torch.distributed.run (one rank per GPU, RCCL). Prints ONE
JSON line on rank 0.

Step = one serving tick of the distributed cache on every rank: a GET batch of Zipf(0.99)
requests and a SET batch, probed / gathered and committed (dedupe, scan-allocate, log write
with CLOCK reinsertions, CAS index insert) by the HIP kernels on the shard's HBM.
  * One GPU: ``--batch`` GETs and ``--sets`` SETs over the ``--keys-per-gpu`` key space.
  * N>1 ranks (default ``--route host``, the HTTP path's topology): every step draws ONE
    global stream of N x --batch GETs and N x --sets SETs (same seeds on every rank); the
    host router (ketama, csrc/host_router.cc) sends each request to the GPU owning its key,
    the ``--spread`` hottest objects replicated on every GPU with their GETs spread to even
    out the load. Each rank serves its true, unequal share; the timed region ends at the
    slowest rank. No value crosses xGMI in the step. ``--route device``: the experimental
    all-to-all step (GPU-resident batches routed between GPUs over RCCL; see docs/PERF.md).
Per-GPU work is fixed as N grows (weak scaling): the key space is N x --keys-per-gpu.

Headline (``--headline pressured``): the full cache — a shard log sized to its working set
(every key it holds, one record each: --pressured-fill 1.0), wrapped, so every SET batch's
CLOCK hand re-appends the objects read since it last passed and evicts the rest. Its request
stream is the walk (``walk_batches``): the SETs walk a permutation of every key the shard
holds and the GETs are --walk-get-batches (256) fresh batches of the Zipf stream, more than
a log lap of steps, so the keys read over one lap of the log fill 3/4 of it
(``read_working_set_over_capacity`` 0.750 at the defaults) rather than the 0.40 the 16
cycled batches touched in round 5's headline. Secondary: the same full
cache on the 16 cycled GET / SET batches (``log_pressured_cycled``, the round-5 headline),
the fresh cache (``log_fresh``), a 16 GiB log that has wrapped with the working set at ~1/4
of it (``log_wrapped``), and a working set --overfull-fill (1.25) times the log
(``log_overfull``, on the walk too, so an evicted key misses until re-SET). The full-cache
blocks also report ``request_hit_ratio`` (duplicates included, untimed steps).
Pooled capacity (scripts/pooled_capacity.sh): ``--keys-total`` fixes the key space across N.
Host routing (N > 1): ``value`` is bounded by what the host routers can feed — the measured
native router rate times N — when that is below the job's rate. A simulated
host-routed world also runs ``spread_drift``: the spread hot set refreshed incrementally
(parallel/hotspread.py refresh_hot) under a drifting popularity order.

Metric: whole-job cache operations per second (GET+SET requests served).
The reference (kmacrow/Shellac) publishes no numbers, so vs_baseline is null.
Secondary (outside the timed region): the BASELINE.json platform smoke checks
— the MFMA hello tile and an RCCL all-reduce of a 1 GiB bf16 tensor.
"""
from __future__ import annotations

import argparse
import datetime
import faulthandler
import json
import os
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from shellac_amd.bench.workload import Workload  # noqa: E402
from shellac_amd.models.sharded_cache import ShardedCache  # noqa: E402
from shellac_amd.ops.cache import CacheShard  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1 << 20, help="GET requests per rank per step")
    ap.add_argument("--sets", type=int, default=1 << 16, help="SET requests per rank per step")
    ap.add_argument("--keys-per-gpu", type=int, default=4 << 20)
    ap.add_argument("--keys-total", type=int, default=None,
                    help="a fixed total key count (strong scaling of capacity): each of the N "
                         "ranks gets keys-total / N instead of --keys-per-gpu (with --set-walk "
                         "and a fixed --pressured-gb: hit ratio against the pooled capacity, "
                         "scripts/pooled_capacity.sh)")
    ap.add_argument("--walk-get-batches", type=int, default=256,
                    help="GET batches of the request stream pre-generated for --set-walk and "
                         "log_overfull (cycled; more than a log lap of steps, so a key's "
                         "re-reads are the stream's, not the cycle's)")
    ap.add_argument("--set-walk", dest="set_walk", action="store_true", default=True,
                    help="(default) the headline full-cache block runs on the walk: its SETs walk "
                         "a permutation of every key the shard holds (each re-SET once per "
                         "keys/sets steps) and its GETs are --walk-get-batches fresh batches")
    ap.add_argument("--cycled-headline", dest="set_walk", action="store_false",
                    help="the headline full-cache block cycles the 16 pre-generated GET / SET "
                         "batches instead (the round-5 headline: ~1/2 of the keys read)")
    ap.add_argument("--no-cycled", action="store_true",
                    help="skip the secondary log_pressured_cycled block")
    ap.add_argument("--zipf", type=float, default=0.99)
    ap.add_argument("--min-val", type=int, default=64)
    ap.add_argument("--max-val", type=int, default=4096)
    ap.add_argument("--log-gb", type=float, default=16.0, help="value-log GiB per shard")
    ap.add_argument("--set-dist", choices=["uniform", "zipf"], default="uniform",
                    help="SET popularity: uniform (TTL refresh fills, default) or zipf")
    ap.add_argument("--replicate", type=int, default=None,
                    help="--route device: hot objects replicated on every rank (0 = off; "
                         "default 1M, the per-N replica table in docs/PERF.md)")
    ap.add_argument("--replica-gb", type=float, default=None,
                    help="replica log GiB (default: 2 KiB per replicated object)")
    ap.add_argument("--sample-batches", type=int, default=32,
                    help="GET batches (independent of the timed ones) observed to pick the "
                         "replicated hot set")
    ap.add_argument("--simulate-world", type=int, default=0,
                    help="profiling only: run rank 0 of an N-rank job on one GPU with mirrored "
                         "all-to-alls (no interconnect); every key is mapped onto one rank 0 "
                         "owns, so its shard holds 1/N of the key space in one --log-gb log "
                         "like a real rank; prints a *_simulated metric")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu = functional rehearsal of the distributed path over gloo "
                         "(DRAM shards); never a performance number")
    ap.add_argument("--no-coalesce", action="store_true",
                    help="probe and copy every GET request (no in-batch request collapsing)")
    ap.add_argument("--bounce", action="store_true",
                    help="functional rehearsal of the N-rank GPU step on ONE GPU: every rank on "
                         "cuda:0, collectives bounced through gloo (RCCL refuses two ranks on "
                         "one device); never a performance number")
    ap.add_argument("--edge", choices=["device", "host"], default="device",
                    help="host: the product edge — GET digests and SET payloads in pinned host "
                         "memory, responses gathered into pinned host memory over PCIe "
                         "(as the proxy's HBM tier); one rank")
    ap.add_argument("--routed", action="store_true",
                    help="one rank: run the routed multi-GPU step anyway, over a real one-rank "
                         "RCCL communicator (every collective call of the N-GPU step; all keys "
                         "are local, so no interconnect traffic) — a rehearsal, not a scaling "
                         "number")
    ap.add_argument("--spread", type=int, default=None,
                    help="host-routed N>1: hot objects replicated on every GPU (the top of an "
                         "observed GET sample), their GETs sprayed over the GPUs to even out "
                         "the load and their SETs written through to every GPU (0 = off; "
                         "default 1024: the request shares are within 0.3 %% of the mean "
                         "with 1024 at N = 2-8, as with 65536, and the router stays faster)")
    ap.add_argument("--spread-sample", type=int, default=1 << 22,
                    help="GET requests of the observed sample that picks the hot set")
    ap.add_argument("--spread-policy", choices=["designate", "spray"], default="designate",
                    help="a hot object's GETs go to one rank designated to even out the load "
                         "(objects above 1/(4N) of the traffic sprayed), or every hot object's "
                         "GETs are sprayed over all ranks")
    ap.add_argument("--ring-points", type=int, default=1024,
                    help="host routing: ring points per GPU (the per-GPU key-space share, "
                         "hence the distinct-key work, is within ~5 %% of the mean at 1024 "
                         "for 8 GPUs, ~12 %% at 160)")
    ap.add_argument("--sim-rank", type=int, default=-1,
                    help="--simulate-world N --route host: the rank to simulate (default: the "
                         "most loaded one under the routing in force)")
    ap.add_argument("--route-threads", type=int, default=0,
                    help="threads of the measured host router (0: the CPUs this process may "
                         "use, at most 16, the box's share of one GPU)")
    ap.add_argument("--route", choices=["host", "device"], default=None,
                    help="N>1 ranks: 'host' — requests reach the GPU that owns their key (ketama "
                         "on the host proxy, as the HTTP path's HbmBackend routes; GPUs exchange "
                         "no values); 'device' — GPU-resident request batches routed between GPUs "
                         "by the all-to-all step (RCCL over xGMI). Default: host with real ranks, "
                         "device with --simulate-world (--simulate-world N --route host: rank "
                         "0's owner share of the stream on its 1/N of the key space)")
    ap.add_argument("--comm-mode", choices=["single", "channels"], default="channels",
                    help="routed step: every collective on one communicator and one stream in "
                         "a fixed order (single), or one communicator per channel (channels)")
    ap.add_argument("--evict", choices=["clock", "fifo"], default="clock",
                    help="value-log eviction policy of the shards")
    ap.add_argument("--batches", type=int, default=16,
                    help="distinct pre-generated GET/SET batch pairs cycled through the steps "
                         "(16 x 16 MiB of digests + 16 SET payload sets: more than the 256 MB MALL)")
    ap.add_argument("--pg-timeout", type=float, default=300.0,
                    help="process-group timeout in seconds: a stuck collective exits non-zero")
    ap.add_argument("--no-smoke", action="store_true")
    ap.add_argument("--no-uncoalesced", action="store_true",
                    help="skip the secondary uncoalesced-GET measurement")
    ap.add_argument("--no-wrapped", action="store_true",
                    help="skip the steady-state measurement (value log wrapped, so every SET "
                         "batch runs the eviction hand); the headline is then the fresh cache")
    ap.add_argument("--pressured-gb", type=float, default=None,
                    help="the full-cache steady state (the headline): a shard log of this many "
                         "GiB, wrapped, so the CLOCK hand re-appends read objects every step. "
                         "Default: sized so the shard's working set (every key it owns, one "
                         "record each) fills --pressured-fill of it (0 = skip)")
    ap.add_argument("--pressured-fill", type=float, default=1.0,
                    help="working set over log capacity of the default pressured shard")
    ap.add_argument("--overfull-fill", type=float, default=1.25,
                    help="secondary block log_overfull: a shard log the working set fills "
                         "this many times over (0 = skip; only with the default pressured log)")
    ap.add_argument("--headline", choices=["pressured", "wrapped", "fresh"], default="pressured",
                    help="which cache state the headline K steps run in: a full cache whose "
                         "working set fills --pressured-fill of the log (default: eviction with "
                         "CLOCK reinsertions in every SET batch, hit ratio < 1), the 16 GiB log "
                         "wrapped (eviction hand in every batch, nothing live to evict), or the "
                         "fresh cache before the first wrap")
    ap.add_argument("--drift-epochs", type=int, default=4,
                    help="hot_drift block (N>1 / simulated, replica on): epochs of drifted "
                         "popularity, each --drift-steps steps then an incremental replica "
                         "refresh (0 = skip)")
    ap.add_argument("--drift-steps", type=int, default=400)
    ap.add_argument("--spread-drift-steps", type=int, default=40,
                    help="spread_drift block (simulated host-routed world with --spread): steps per epoch of "
                         "drifted popularity after each incremental hot-set refresh "
                         "(--drift-epochs epochs; 0 = skip)")
    ap.add_argument("--spread-drift-swap", type=float, default=0.25,
                    help="share of the spread hot set whose objects trade places with tail "
                         "objects every spread_drift epoch")
    ap.add_argument("--drift-swap", type=float, default=0.05,
                    help="share of the replicated top ranks whose objects trade places with "
                         "tail objects every epoch (content cooling, new content heating up)")
    ap.add_argument("--drift-sample", type=int, default=16 << 20,
                    help="observed requests per rank the replica refresh ranks keys by")
    ap.add_argument("--drift-budget-mb", type=float, default=512.0,
                    help="replica refresh byte budget per epoch and rank (MiB)")
    ap.add_argument("--event-fence", choices=["device", "none", "system"], default=None,
                    help="one-GPU step: fence scope of the events ordering its two streams "
                         "(ShardedCache.event_fence; default: the cache's)")
    ap.add_argument("--gather-after-append", action="store_true",
                    help="one GPU: the GET gather waits for the SET batch's log append")
    ap.add_argument("--hand", choices=["early", "inline"], default="early",
                    help="one GPU, full cache: the CLOCK hand detached on a stream of its own, "
                         "beside the previous step's SET chain, its reinsertions indexed as "
                         "moves (early), or at the head of the SET chain (inline)")
    ap.add_argument("--check", action="store_true", help="verify a sample of GET values")
    return ap.parse_args()


def router_bound(out: dict, router_req_per_s: float, world: int) -> dict:
    """The host-routed headline bounded by its router: value =
    min(job rate, N x the measured native router rate); ms_per_step follows the value.
    Returns the updated fields (``value``, ``ms_per_step``, ``host_routing``)."""
    hr_ = dict(out["host_routing"])
    value, ms = out["value"], out["ms_per_step"]
    cap_ = router_req_per_s * world
    hr_["host_route_job_capacity_req_per_s"] = round(cap_, 1)
    hr_["router_feeds_job"] = bool(cap_ >= value)
    hr_["job_rate_req_per_s"] = value
    hr_["job_ms_per_step"] = ms
    if cap_ < value:
        ms = round(ms * value / cap_, 4)
        value = round(cap_, 1)
    hr_["value_bounded_by_router"] = not hr_["router_feeds_job"]
    return {"value": value, "ms_per_step": ms, "host_routing": hr_}


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def maybe_launch(args) -> None:
    """``--gpus N`` (N > 1) without a torch.distributed launcher: run the N ranks as a
    CHILD ``torch.distributed.run`` job and exit with its status. This happens before
    anything touches the GPU (no exec from a process with a live HIP context). With a
    launcher, the rank count must equal --gpus: a job that would silently report a
    1-rank number as an N-GPU run exits non-zero instead."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None:
        if args.gpus <= 1 or args.simulate_world:
            return
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
               "--master-port", str(_free_port()), os.path.abspath(__file__), *sys.argv[1:]]
        print(f"[bench] launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
        raise SystemExit(subprocess.run(cmd).returncode)
    if int(world_env) != args.gpus and not args.simulate_world:
        print(f"[bench] error: --gpus {args.gpus} but the launcher started WORLD_SIZE={world_env} "
              "ranks; refusing to report a number for the wrong GPU count", file=sys.stderr,
              flush=True)
        raise SystemExit(2)


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def smoke(rank, world, dev):
    out = {}
    try:
        from shellac_amd.ops.smoke import mfma_hello

        g = torch.Generator(device=dev).manual_seed(7)
        a = torch.randn(64, 32, 16, generator=g, device=dev).to(torch.bfloat16)
        b = torch.randn(64, 16, 32, generator=g, device=dev).to(torch.bfloat16)
        c = mfma_hello(a, b)
        ref = torch.bmm(a.float(), b.float())
        out["mfma_hello_max_abs_err"] = float((c - ref).abs().max())
    except Exception as e:  # report, never hide
        out["mfma_hello_error"] = repr(e)
    if world > 1:
        x = torch.ones(512 << 20, dtype=torch.bfloat16, device=dev)  # 1 GiB
        dist.all_reduce(x)
        torch.cuda.synchronize()
        # every element must equal the rank count (exact in bf16 for world <= 256)
        lo, hi = float(x.min()), float(x.max())
        if lo != world or hi != world:
            raise RuntimeError(f"RCCL all-reduce smoke wrong: min {lo} max {hi}, want {world}")
        out["allreduce_check"] = "ok"
        iters = 5
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(x)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / iters
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
        nbytes = x.numel() * 2
        out["allreduce_1GiB_bf16_ms"] = round(dt * 1e3, 3)
        out["allreduce_busbw_GBps"] = round(nbytes * 2 * (world - 1) / world / dt / 1e9, 1)
        del x
        torch.cuda.empty_cache()
    return out


def check_memory_budget(args, world, sim, dev) -> None:
    """Fail fast, with a clear message, when a rank's HBM cannot hold its shard: the value
    log, the index (128 B per bucket, ~4 per key), the replica tier, the workload's
    payload pool and pre-generated batches, the routed step's exchange buffers (about
    three steps of responses in flight) and the 1 GiB all-reduce of the smoke check."""
    gib = 1 << 30
    shard_keys = args.keys_per_gpu
    nb = 1
    while nb < shard_keys:
        nb *= 2
    need = args.log_gb * gib + nb * 128
    if world > 1 and args.replicate:
        rgb = args.replica_gb if args.replica_gb is not None else args.replicate * 2048 / gib
        need += rgb * gib + 2 * args.replicate * 128
    mean_val = (args.max_val - args.min_val) / max(1.0, __import__("math").log(
        max(args.max_val, 2) / max(args.min_val, 1)))
    need += args.keys_per_gpu * world * (mean_val + 64)          # payload pool
    need += max(1, args.batches) * (args.batch * 16 + args.sets * 64)
    need += 3 * args.batch * (mean_val + 48) * 1.2 + 2 * gib        # responses in flight
    if not args.no_smoke and world > 1:
        need += gib
    if (args.pressured_gb is None or args.pressured_gb > 0) and not sim:
        pgb = (args.pressured_gb if args.pressured_gb is not None else
               args.keys_per_gpu * (mean_val + 48) / max(args.pressured_fill, 0.1) / gib)
        need += pgb * gib + nb * 128
    if args.set_walk or (args.overfull_fill > 0 and args.pressured_gb is None):
        # walk_batches(): fresh GET batches (ids + digests) and SET batches over every key
        need += args.walk_get_batches * args.batch * 24 + args.keys_per_gpu * 48
    if sim:  # the probe digests of the key space and their sorted index
        need += args.keys_per_gpu * sim * 48
    free, total = torch.cuda.mem_get_info(dev)
    if need > free:
        print(f"[bench] error: this configuration needs ~{need / gib:.1f} GiB of HBM per rank "
              f"but {free / gib:.1f} of {total / gib:.1f} GiB are free on {dev}; lower --log-gb "
              f"or --keys-per-gpu", file=sys.stderr, flush=True)
        raise SystemExit(2)


def simulated_world_map(wl, sim: int, dev) -> dict:
    """--simulate-world N: rank 0 of N ranks on one GPU, all-to-alls mirrored (what rank 0
    sends to p comes back as what p sends to rank 0). Requests keep the whole key space
    (popularity, routing by the real ring, coalescing, the replica tier), but every key i is
    mapped onto a key f(i) that rank 0 owns — the j-th key (by id) rank p owns onto the j-th
    key rank 0 owns — and owners probe and store f(i). Rank 0's shard then holds only its
    1/N of the key space in one log, as a real rank's does, while receiving N-1 mirrored
    request slots of the real shape. Returns {mine: ids rank 0 owns, f: id -> owner key id,
    pdig: digests of f, probe_of: request digests -> probe digests}."""
    from shellac_amd.ops import routing as R
    from shellac_amd.parallel.ring import ShardRing

    pts, own = ShardRing(list(range(sim)), 160).tensors(dev)
    owners = R.route(wl.digests, pts, own, sim)[0].long()
    ids = torch.arange(wl.total_keys, device=dev)
    mine = ids[owners == 0].contiguous()
    f = ids.clone()
    for p in range(1, sim):
        ip = ids[owners == p]
        f[ip] = mine[torch.arange(ip.numel(), device=dev) % mine.numel()]
    pdig = wl.digests.index_select(0, f).contiguous()
    lo_sorted, order = torch.sort(wl.digests[:, 0].contiguous())

    def probe_of(keys):
        at = torch.searchsorted(lo_sorted, keys[:, 0].contiguous()).clamp_(max=lo_sorted.numel() - 1)
        return pdig.index_select(0, order.index_select(0, at)).contiguous()

    return {"mine": mine, "f": f, "pdig": pdig, "probe_of": probe_of}


def _claim_stdout():
    """The contract is ONE JSON line on rank 0's stdout, but RCCL prints a version banner
    to fd 1 when a communicator comes up. Keep a private handle on the real stdout for the
    JSON line and point fd 1 (C libraries, stray prints) at stderr."""
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    return out


def main():
    args = parse()
    maybe_launch(args)
    json_out = _claim_stdout()
    if os.environ.get("SHELLAC_BENCH_STACKS"):
        # debugging a hung rank: every rank prints all its threads' stacks every N seconds
        faulthandler.dump_traceback_later(float(os.environ["SHELLAC_BENCH_STACKS"]), repeat=True)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    sim = args.simulate_world
    if sim and world != 1:
        raise SystemExit("--simulate-world runs as a single process")
    bounce = args.bounce and args.device == "cuda" and world > 1
    routed1 = args.routed and world == 1 and not sim
    if routed1 and args.device != "cuda":
        raise SystemExit("--routed is the one-GPU RCCL rehearsal")
    pg_timeout = datetime.timedelta(seconds=args.pg_timeout)
    # a collective that outlives the timeout aborts the rank (non-zero exit), not a hang
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    if bounce:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", timeout=pg_timeout)
    elif args.device == "cuda":
        ndev = torch.cuda.device_count()
        if local >= ndev or (world > 1 and ndev < world and not sim):
            print(f"[bench] error: --gpus {args.gpus} needs {max(world, local + 1)} GPUs on this "
                  f"node, {ndev} visible; refusing to put several ranks on one device",
                  file=sys.stderr, flush=True)
            raise SystemExit(2)
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        # the serving step's streams take their hardware queues before the process
        # group's communicators make streams of their own
        from shellac_amd.ops.cache import reserve_step_streams

        reserve_step_streams(dev)
        if world > 1:
            dist.init_process_group("nccl", device_id=dev, timeout=pg_timeout)
        elif routed1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            dist.init_process_group("nccl", device_id=dev, timeout=pg_timeout, rank=0,
                                    world_size=1)
    else:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo", timeout=pg_timeout)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    group = None
    if sim:
        from shellac_amd.parallel.exchange import MirrorComm

        group = MirrorComm(sim)
        world = sim
    real_world = 1 if sim else world
    if args.keys_total:
        args.keys_per_gpu = max(1, args.keys_total // world)
    # N real ranks behind host proxies: each GPU serves the requests for the keys it owns
    # (a bounce rehearsal keeps the device-routed step unless --route host is given: then
    # every rank is a host-routed GPU server sharing cuda:0, its barriers and reductions
    # over gloo — the real N>1 default's flow, rehearsed on one GPU)
    host_route = ((real_world > 1 and (args.route or ("device" if bounce else "host")) == "host")
                  or (sim and args.route == "host"))
    msim = 0 if host_route else sim  # the mirrored (device-routed) simulation
    if host_route:
        from shellac_amd.parallel.exchange import LocalComm

        args.replicate = 0  # no device-routed replica tier (hot objects: --spread)
        # the rank's cache never routes (group=None would mean the world group here)
        group = LocalComm()
        if args.spread is None:
            args.spread = 1 << 10
    else:
        args.spread = 0
    if routed1:
        args.replicate = 0  # one rank owns every key: the replica tier is never consulted
    if bounce and not host_route:
        from shellac_amd.parallel.exchange import BounceComm

        group = BounceComm()

    if args.replicate is None:
        # device-routed step: the per-N table (profiles/archive/r4_sweep2, docs/PERF.md) — every
        # N is link-bound, and 1M replicated objects give the lowest max(compute, link) at
        # N=2 and N=8 and are within 1 % of it at N=4
        args.replicate = 1 << 20
    if args.replica_gb is None:
        args.replica_gb = args.replicate * 2048 / (1 << 30)
    total_keys = args.keys_per_gpu * world
    if dev.type == "cuda" and not bounce:
        check_memory_budget(args, world, msim, dev)
    t_setup = time.perf_counter()
    wl = Workload(total_keys, dev, zipf_s=args.zipf, min_val=args.min_val, max_val=args.max_val)
    sim_map = simulated_world_map(wl, sim, dev) if msim else None
    owner_of = mine = spread = None
    me = rank
    route_info = {}
    if host_route:
        # The host proxies' routing (HostRouter; its tensor twin prepares the batches here):
        # one global request stream per step, N x --batch GETs and N x --sets SETs drawn
        # with the same seeds on every rank, of which each rank serves what the router sends
        # it — its keys' true ketama share, hot objects sprayed when --spread is on
        from shellac_amd.parallel.hotspread import HotSpread, member

        spread = HotSpread(world, dev, points_per_shard=args.ring_points)
        owner_of = spread.owners(wl.digests).long()
        route_info["ring_points_per_gpu"] = args.ring_points
        # (at most 1/64 of the key space: every GPU holds the replicas on top of its share)
        args.spread = min(args.spread, total_keys // 64)
        if args.spread > 0:
            sample = wl.digests.index_select(0, wl.sample_ids(args.spread_sample, 8800))
            info = spread.plan(sample, args.spread, policy=args.spread_policy)
            hmask = member(wl.digests, spread.hot)
            route_info.update(spread_hot_objects=int(spread.hot.shape[0]),
                              spread_policy=args.spread_policy,
                              spread_hot_share_of_gets=round(info["hot_share"], 4),
                              spread_sprayed_objects=info.get("sprayed_objects"))
            del sample
        else:
            hmask = None

        def global_batch(p):
            """Batch pair p of the global stream, routed: (GET ids, GET dest, SET ids,
            SET dest) — dest -1 = every rank (a hot object's SET)."""
            g = wl.sample_ids(world * args.batch, 1000 + 97 * p)
            gd = spread.route_gets(wl.digests.index_select(0, g), seq0=p * world * args.batch)
            pick_ = wl.uniform_ids if args.set_dist == "uniform" else wl.sample_ids
            st = pick_(world * args.sets, 5000 + 97 * p)
            sd = spread.route_sets(wl.digests.index_select(0, st))
            return g, gd, st, sd

        # per-rank requests and distinct GET keys of the first batch pair: the shares, and
        # the rank a simulation runs. A step's work is mostly per distinct key (probe, record
        # copy; duplicates collapse): measured ~0.9 ns per distinct key and ~0.06 per request
        # (profiles/r5c_hostsim), so the simulated rank is the one with the most of that cost
        g0, gd0, st0, sd0 = global_batch(0)
        load = (torch.bincount(gd0.long(), minlength=world) +
                torch.bincount(sd0[sd0 >= 0].long(), minlength=world) +
                int((sd0 < 0).sum())).double()
        distinct = torch.tensor([float(torch.unique(g0[gd0 == r]).numel()) for r in range(world)],
                                dtype=torch.float64, device=dev)
        cost = 0.9 * distinct + 0.06 * load
        if sim:
            me = int(torch.argmax(cost)) if args.sim_rank < 0 else args.sim_rank
        route_info.update(rank_requests_share=[round(x, 5) for x in (load / load.sum()).tolist()],
                          rank_share_max_over_mean=round(float(load.max() / load.mean()), 4),
                          rank_distinct_gets=[int(x) for x in distinct.tolist()],
                          rank_distinct_max_over_mean=round(float(distinct.max() / distinct.mean()), 4),
                          rank_cost_max_over_mean=round(float(cost.max() / cost.mean()), 4))
        # the native router on the same stream (host memory), timed: what the host proxies
        # can feed
        import time as _t

        kh = wl.digests.index_select(0, g0).cpu().contiguous()
        th = args.route_threads or min(16, len(os.sched_getaffinity(0)))
        rates = {}
        hbuf = torch.empty(kh.shape[0], dtype=torch.int32)
        for t_ in sorted({1, th}):
            best = float("inf")
            for _ in range(3):
                t0_ = _t.perf_counter()
                hd, _hc = spread.host_route_gets(kh, seq0=0, threads=t_, out=hbuf)
                best = min(best, _t.perf_counter() - t0_)
            rates[t_] = kh.shape[0] / best
        route_info.update(host_route_threads=th, host_route_avx512_lanes=bool(spread.router.lanes),
                          host_route_req_per_s=round(rates[th], 1),
                          host_route_req_per_s_one_thread=round(rates[1], 1),
                          host_route_agrees_with_device=bool(torch.equal(hd, gd0.cpu())))
        del kh, g0, gd0, st0, sd0
        mine = torch.nonzero(owner_of == me).flatten().contiguous()
        if hmask is not None:   # replicas: hot objects this rank does not own
            rep_ids = torch.nonzero(hmask & (owner_of != me)).flatten().contiguous()
        else:
            rep_ids = None
    nb = 1
    shard_keys = (int(sim_map["mine"].numel()) if msim else
                  int(mine.numel()) + (int(rep_ids.numel()) if rep_ids is not None else 0)
                  if host_route else args.keys_per_gpu)
    while nb < shard_keys:  # ~25% slot load with 4-entry buckets (HBM is plentiful)
        nb *= 2
    log_bytes = int(args.log_gb * (1 << 30)) // 16 * 16
    shard = CacheShard(log_bytes, nb, max_item=1 << 20, device=dev, evict=args.evict)
    replica = None
    if world > 1 and args.replicate > 0:
        rnb = 1
        while rnb * 2 < args.replicate:
            rnb *= 2
        replica = CacheShard(int(args.replica_gb * (1 << 30)) // 16 * 16, max(rnb, 1024),
                             max_item=1 << 20, device=dev)
    data_group = None
    if (real_world > 1 or routed1) and not bounce and not host_route:
        # second communicator: the value all-to-all of step i overlaps step i+1's exchanges
        data_group = dist.new_group(ranks=list(range(real_world)))
    sc = ShardedCache(shard, group=group, replica=replica,
                      data_group=data_group, routed=True if routed1 else None,
                      comm_mode=args.comm_mode, hand=args.hand)
    if host_route and (sc.world, sc.routed) != (1, False):
        raise SystemExit("[bench] a host-routed rank's cache must serve only its own keys")
    sc.coalesce = not args.no_coalesce
    sc.gather_after_append = args.gather_after_append
    if args.event_fence:
        sc.event_fence = args.event_fence
    if msim:
        sc.probe_of = sim_map["probe_of"]

    # populate: every rank SETs its slice of the key space through the routed path
    chunk = 1 << 18
    lo, hi = rank * args.keys_per_gpu, (rank + 1) * args.keys_per_gpu
    # (the simulated rank and a host-routed rank fill what they own)
    fill_ids = sim_map["mine"] if msim else mine

    def populate(cache):
        n_own = int(fill_ids.numel()) if fill_ids is not None else hi - lo
        for s0 in range(0, n_own, chunk):
            ids = (fill_ids[s0: s0 + chunk] if fill_ids is not None else
                   torch.arange(lo + s0, min(lo + s0 + chunk, hi), device=dev))
            cache.set(wl.set_batch(ids))
        if host_route and rep_ids is not None and rep_ids.numel():
            # the hot objects this rank does not own, fetched from their owners
            if real_world > 1:
                from shellac_amd.parallel.hotspread import replicate_hot

                hot_d = spread.hot
                replicate_hot(cache, hot_d, spread.owners(hot_d), rank, world,
                              group=dist.group.WORLD)
            else:  # a simulated rank: its peers' copies are the workload's objects
                for s0 in range(0, int(rep_ids.numel()), chunk):
                    cache.set(wl.set_batch(rep_ids[s0: s0 + chunk]))
        sync()

    populate(sc)
    if real_world > 1:
        dist.barrier()
    log(rank, f"[bench] populated {total_keys} keys in {time.perf_counter() - t_setup:.1f}s")

    # pre-generated request batches (the "data loader"), cycled through the steps: 16
    # distinct pairs by default, so the GET digests alone (16 x 16 MiB) outgrow the 256 MB
    # MALL and each step reads its batch from HBM rather than from the last-level cache
    P = max(1, args.batches)
    pick = wl.uniform_ids if args.set_dist == "uniform" else wl.sample_ids
    if host_route:
        # what the router sends this rank out of each batch pair of the global stream
        get_ids, set_ids = [], []
        rank_req = torch.zeros(world, dtype=torch.float64, device=dev)
        for i in range(P):
            g, gd, st, sd = global_batch(i)
            get_ids.append(g[gd == me].contiguous())
            set_ids.append(st[(sd == me) | (sd < 0)].contiguous())
            rank_req += (torch.bincount(gd.long(), minlength=world) +
                         torch.bincount(sd[sd >= 0].long(), minlength=world) +
                         int((sd < 0).sum())).double()
            del g, gd, st, sd
        route_info["rank_requests_per_step"] = [round(x / P) for x in rank_req.tolist()]
        route_info["rank_share_max_over_mean"] = round(float(rank_req.max() / rank_req.mean()), 4)
    else:
        get_ids = [wl.sample_ids(args.batch, 1000 + 97 * rank + i) for i in range(P)]
        set_ids = [pick(args.sets, 5000 + 97 * rank + i) for i in range(P)]
    gets = [wl.digests.index_select(0, g).contiguous() for g in get_ids]
    sets = [wl.set_batch(x) for x in set_ids]
    gprobe = [None] * P
    if msim:  # what the (mirrored) owners probe and store: keys the simulated rank owns
        pd = sim_map["pdig"]
        gprobe = [pd.index_select(0, wl.sample_ids(args.batch, 1000 + 97 * rank + i)).contiguous()
                  for i in range(P)]
        for i in range(P):
            sets[i].probe_keys = pd.index_select(
                0, pick(args.sets, 5000 + 97 * rank + i)).contiguous()
    if replica is not None:
        # hot-object replica tier from an observed request stream (periodic in a server);
        # the observed batches are independent samples, not the timed ones
        seen = torch.cat([wl.digests.index_select(0, wl.sample_ids(args.batch, 9000 + 97 * rank + i))
                          for i in range(args.sample_batches)])
        nrep = sc.refresh_replica(args.replicate, keys=seen)
        del seen
        log(rank, f"[bench] replicated {nrep} hot objects on every rank")
    shard.reserve(max(args.sets * 2, chunk))
    host_edge = args.edge == "host"
    if host_edge:
        if real_world > 1 or sim or dev.type != "cuda":
            raise SystemExit("--edge host runs one GPU rank")
        from shellac_amd.models.sharded_cache import SetBatch

        def pin(t):
            return None if t is None else t.cpu().pin_memory()

        pool_h = pin(wl.pool)
        gets = [pin(g) for g in gets]
        sets = [SetBatch(pin(b.keys), pool_h, pin(b.val_off), pin(b.vlen), pin(b.flags),
                         pin(b.expire)) for b in sets]
        sc.host_edge = True

    # the request batches are complete from here on (the routed step may plan a batch
    # beside the previous step's reply gather)
    ready = torch.cuda.Event() if dev.type == "cuda" else None
    if ready is not None:
        ready.record()

    # the batches the steps cycle (a phase may swap in its own): GET digests, their ids
    # (for --check) and the SET batches
    cyc = {"gets": gets, "get_ids": get_ids, "sets": sets}

    def serve_i(cache, i):
        # GET batch then SET batch; with one rank the GET's host sync overlaps the SET
        gl, sl = cyc["gets"], cyc["sets"]
        return cache.serve(gl[i % len(gl)], sl[i % len(sl)], inputs_ready=ready,
                           probe_keys=gprobe[i % P] if msim else None)

    def step(i):
        return serve_i(sc, i)

    # Per-step GPU timing events are recorded in a separate pass after the timed one: an
    # event record is a marker packet on the stream, and one between every two steps cost
    # ~6 us of a 0.32 ms step (profiles/archive/r2_bench_events_ab.log)
    use_events = dev.type == "cuda"
    rdev = torch.device("cpu") if bounce else dev  # gloo reduces host tensors

    last_rank_ms = []   # each rank's own ms/step of the last timed() (before the barrier)

    def timed(steps, first, events=False, cache=None):
        """Run `steps` steps bracketed by barrier + device sync; returns (max-over-ranks
        wall seconds, per-step GPU-event intervals in ms if `events`, last result)."""
        cache = sc if cache is None else cache
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)] if events else []
        cur = torch.cuda.current_stream(dev) if events else None
        if real_world > 1:
            dist.barrier()
        sync()
        t0 = time.perf_counter()
        res = None
        for i in range(steps):
            if events:
                evs[i].record(cur)
            res = serve_i(cache, first + i)
        if events:
            evs[steps].record(cur)
        sync()
        own = time.perf_counter() - t0   # this rank's steps, before it waits for the others
        if real_world > 1:
            dist.barrier()
        sync()
        el = time.perf_counter() - t0
        t = torch.tensor([el], dtype=torch.float64, device=rdev)
        if real_world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ot = torch.zeros(max(real_world, 1), dtype=torch.float64, device=rdev)
        ot[rank if real_world > 1 else 0] = own
        if real_world > 1:
            dist.all_reduce(ot)
        last_rank_ms[:] = [round(x / steps * 1e3, 4) for x in ot.tolist()]
        iv = [evs[i].elapsed_time(evs[i + 1]) for i in range(steps)] if events else []
        return float(t), iv, res

    def window(cache, shard_, first):
        """The headline protocol on `cache`: K steps from batch `first`, bracketed by a
        barrier and device syncs (timed), and the counters of exactly those steps."""
        cache.sync_sets()
        c0 = shard_.counters()
        st0 = dict(cache.stats)
        gb0 = cache.gathered_bytes
        h0 = shard_.head()
        # SHELLAC_BENCH_WINDOW_EVENTS=1 (diagnostic): per-step GPU events inside the timed
        # window itself (they cost a few us per step), reported as window_step_ms
        wev = bool(os.environ.get("SHELLAC_BENCH_WINDOW_EVENTS")) and use_events
        el, wiv, res = timed(args.steps, first, events=wev, cache=cache)
        rank_ms = list(last_rank_ms)
        gathered = cache.gathered_bytes - gb0
        cache.sync_sets()
        c1 = shard_.counters()
        st1 = cache.stats
        # owner-shard counters cover the GETs that left the replica tier; replica hits
        # are counted by the serving step
        agg = torch.tensor([c1["get_hits"] - c0["get_hits"], c1["get_ops"] - c0["get_ops"],
                            c1["get_bytes"] - c0["get_bytes"],
                            st1["replica_hits"] - st0["replica_hits"],
                            st1["get_requests"] - st0["get_requests"],
                            c1["reinsert_bytes"] - c0["reinsert_bytes"]],
                           dtype=torch.int64, device=rdev)
        if real_world > 1:
            dist.all_reduce(agg)
        hits, gops, gbytes, rep, greq, rbytes = (int(v) for v in agg.tolist())
        return {"el": el, "res": res, "last": (first + args.steps - 1) % len(cyc["gets"]),
                "hits": hits,
                "gops": gops, "gbytes": gbytes, "rep": rep, "greq": greq, "rbytes": rbytes,
                "head0": h0, "head1": shard_.head(), "gathered": gathered, "c0": c0, "c1": c1,
                "rank_ms": rank_ms, "wiv": wiv}

    def check(w):
        """Verify the window's last GET batch against the workload's ground truth (before
        any later step can reuse its response buffer)."""
        from shellac_amd.ops.cache import unpack_records

        res, last_batch = w["res"], w["last"]
        k = 200
        ids = cyc["get_ids"][last_batch][:k]
        res.wait()
        recs = unpack_records(res.data, res.off[:k], res.size[:k])
        if msim:
            # the owner holds key f(i) for request i: several requests alias one owner key
            # (and a SET of any of them updates it), so values are informational here
            fmap = sim_map["f"]
            bad = sum(1 for i, r in zip(ids.tolist(), recs)
                      if r is not None and r[0] != wl.expected_value(int(fmap[i])))
            log(rank, f"[bench] check (simulated world, aliased values): {bad} of {k} sampled "
                      f"GETs differ from the owner key's first value")
        else:
            bad = sum(1 for i, r in zip(ids.tolist(), recs)
                      if r is not None and r[0] != wl.expected_value(i))
            log(rank, f"[bench] check: {bad} mismatches in {k} sampled GETs")
        # every hit of the whole last batch: its record's header names the requested digest
        words = res.data[: res.data.numel() // 8 * 8].view(torch.int64)
        wd = words.device  # pinned host memory under --edge host
        keys_last = cyc["gets"][last_batch].to(wd)
        hit = (res.size > 0).to(wd)
        at = torch.where(hit, torch.div(res.off.to(wd), 8, rounding_mode="floor"),
                         torch.zeros_like(res.off, device=wd))
        w0, w1 = words.index_select(0, at), words.index_select(0, at + 1)
        wrong = hit & ((w0 != keys_last[:, 0]) | (w1 != keys_last[:, 1]))
        if msim:  # an owner's record names the probe digest (a replica's the request's)
            pk = gprobe[last_batch].to(wd)
            wrong &= (w0 != pk[:, 0]) | (w1 != pk[:, 1])
        log(rank, f"[bench] check: {int(wrong.sum())} of {int(hit.sum())} hit records name "
                  f"another key")

    def median(iv):
        return round(sorted(iv)[len(iv) // 2], 4) if iv else None

    def summary(w, iv=None, log_bytes_=log_bytes, fill=None):
        out_ = {"ms_per_step": round(w["el"] / args.steps * 1e3, 4),
                "cache_ops_per_s": round((args.batch + args.sets) * world * args.steps / w["el"], 1),
                "log_gib_per_shard": round(log_bytes_ / (1 << 30), 2),
                "log_head_laps": round(w["head1"] / log_bytes_, 3),
                "working_set_over_capacity": round(ws_bytes / log_bytes_, 4),
                "owner_hit_ratio": round(w["hits"] / max(w["gops"], 1), 4),
                "reinserted_bytes_per_step_per_rank": round(w["rbytes"] / world / args.steps)}
        if fill is not None:
            out_["fill_steps"] = fill
        if host_route:
            out_["rank_ms_per_step"] = w["rank_ms"]
        if iv:
            out_["ms_per_step_median_gpu_events"] = median(iv)
        if w.get("wiv"):
            out_["window_step_ms"] = [round(x, 4) for x in w["wiv"]]
        return out_

    # The log fills at ~66 MB per step and rank; a serving cache is full, and then every
    # SET batch runs the eviction hand (CLOCK second chances) first. Steps run until every
    # rank's log has wrapped by a quarter lap (untimed).
    def fill_to_wrap(cache, shard_, log_bytes_, base, per_step):
        need = torch.tensor([max(0.0, (1.25 * log_bytes_ - shard_.head()) / per_step)],
                            dtype=torch.float64, device=rdev)
        if real_world > 1:
            dist.all_reduce(need, op=dist.ReduceOp.MAX)
        nfill = int(float(need)) + 2
        if nfill > 20000:
            return None
        for i in range(nfill):
            serve_i(cache, base + i)
        sync()
        return nfill

    def hot_drift():
        E, K = args.drift_epochs, args.drift_steps
        R_ = args.replicate
        swap = max(1, int(R_ * args.drift_swap))
        order = wl.rank_to_id
        budget = int(args.drift_budget_mb * (1 << 20))
        PB = 4
        # The refresh ranks keys by the requests of the epoch: the steps cycle a few batches,
        # so the traffic the epoch stands for is sampled afresh from its popularity order
        # (--drift-sample requests per rank; a 2M-key hot set cannot be ranked from a few
        # batches: its tail is seen about once)
        epochs = []
        t_steps = t_ref = 0.0
        for e in range(1, E + 1):
            order = wl.drifted(order, R_, swap, 4242 + e)   # the same drift on every rank
            ids_e = [wl.sample_ids(args.batch, 7000 + 97 * rank + 13 * e + i, rank_to_id=order)
                     for i in range(PB)]
            g = [wl.digests.index_select(0, x).contiguous() for x in ids_e]
            gp = ([sim_map["pdig"].index_select(0, x).contiguous() for x in ids_e] if msim
                  else [None] * PB)
            del ids_e
            ev = torch.cuda.Event()
            ev.record()
            sc.sync_sets()
            c0, st0 = shard.counters(), dict(sc.stats)
            cal0 = int(getattr(sc, "_calibrations", 0))
            if real_world > 1:
                dist.barrier()
            sync()
            t0 = time.perf_counter()
            for i in range(K):
                sc.serve(g[i % PB], sets[i % P], inputs_ready=ev, probe_keys=gp[i % PB])
            sync()
            t1 = time.perf_counter()
            sc.sync_sets()
            c1, st1 = shard.counters(), sc.stats
            rep = st1["replica_hits"] - st0["replica_hits"]
            ops = c1["get_ops"] - c0["get_ops"]
            seen = wl.digests.index_select(0, wl.sample_ids(args.drift_sample, 9100 + 97 * rank + e,
                                                            rank_to_id=order))
            sync()
            t2 = time.perf_counter()
            sc.refresh_replica(args.replicate, keys=seen, budget_bytes=budget)
            del seen
            sync()
            t3 = time.perf_counter()
            # how much of this epoch's true top-R (ground truth) the refreshed hot set holds
            truth = wl.digests.index_select(0, order[:R_])
            hotset = sc._hot if sc._hot is not None else truth[:0]
            prec = float(ShardedCache._member(truth, hotset).float().mean()) if R_ else 0.0
            agg = torch.tensor([t1 - t0, t3 - t2, rep, ops], dtype=torch.float64, device=rdev)
            if real_world > 1:
                dist.all_reduce(agg, op=dist.ReduceOp.MAX)  # (times: the slowest rank)
            ts, tr, rep, ops = agg.tolist()
            t_steps += ts
            t_ref += tr
            epochs.append({"ms_per_step": round(ts / K * 1e3, 4), "refresh_ms": round(tr * 1e3, 1),
                           "replica_hit_fraction": round(rep / max(rep + ops, 1), 4),
                           "hot_set_size_after_refresh": int(hotset.shape[0]),
                           "top_covered_after_refresh": round(prec, 4),
                           "slot_overflow_rows": st1["slot_overflow_rows"] - st0["slot_overflow_rows"],
                           "calibrating_steps": int(getattr(sc, "_calibrations", 0)) - cal0,
                           "replica_log_laps": round(replica.head() / (args.replica_gb * (1 << 30)), 3),
                           "reinsert_mib": round((c1["reinsert_bytes"] - c0["reinsert_bytes"]) / (1 << 20), 1)})
            del g, gp
        st = sc.stats
        return {"epochs": E, "steps_per_epoch": K, "hot_objects_replaced_per_epoch": swap,
                "refresh_budget_mib": args.drift_budget_mb,
                "ms_per_step": round(t_steps / (E * K) * 1e3, 4),
                "ms_per_step_with_refresh": round((t_steps + t_ref) / (E * K) * 1e3, 4),
                "per_epoch": epochs,
                "replica_added": st.get("replica_added", 0),
                "replica_dropped": st.get("replica_dropped", 0),
                "replica_fetched_gib": round(st.get("replica_fetched_bytes", 0) / (1 << 30), 3)}

    steady_ok = not host_edge and dev.type == "cuda" and not args.no_wrapped
    # the shard's working set: one record of every key it holds (its owner share, plus the
    # replicas of spread hot objects), as the log stores it (header + 16-B aligned value)
    held = (torch.arange(lo, hi, device=dev) if fill_ids is None else
            fill_ids if rep_ids is None else torch.cat([fill_ids, rep_ids]))
    ws_bytes = int((32 + ((wl.vlen.index_select(0, held).long() + 15) & ~15)).sum())
    del held
    p_gb = args.pressured_gb
    if p_gb is None:
        p_gb = ws_bytes / max(args.pressured_fill, 0.1) / (1 << 30)
    do_pressured = p_gb > 0 and steady_ok and not msim
    headline = args.headline if steady_ok else "fresh"
    if headline == "pressured" and not do_pressured:
        headline = "wrapped"
    for i in range(args.warmup):
        step(i)
    sync()
    # the log not yet wrapped (the first K steps after the warmup)
    fresh = window(sc, shard, args.warmup)
    if args.check and headline == "fresh":
        check(fresh)
    diag = None
    if sc._engine is not None:
        # the routed step's SET exchange: early appends (look-ahead), carried rows
        e = sc._engine
        carried, cbytes, clost = e.carry_stats()
        cg = e.prepare(args.batch)
        scp = [int(x) for x in e.set_caps()]
        # bytes per step on each link (one per peer, each direction): request slot, reply
        # slot (headers + data), SET slot: fixed sizes, whatever the step carries
        per_peer = 16 * cg[0] + 8 * cg[0] + cg[1] + 16 + 32 * scp[0] + scp[1]
        diag = {"early_set_steps": int(e.early_sets), "set_rows_carried": carried,
                "set_bytes_carried": cbytes, "set_rows_lost": clost, "set_slot_caps": scp,
                "get_slot_caps": [int(cg[0]), int(cg[1])],
                "link_bytes_per_peer_per_step": int(per_peer) if world > 1 else 0,
                "link_ms_per_step_at_55GBps": round(per_peer / 55e9 * 1e3, 3) if world > 1 else 0}
        if replica is not None:
            diag["replica_head_gib"] = round(replica.head() / (1 << 30), 3)
            diag["replica_log_gib"] = round(args.replica_gb, 3)
        if args.check and clost:
            # a SET row that neither fit its slot nor the carry leaves the owner's older
            # value in place (a stale hit, not a miss): a checked run must not have any
            raise SystemExit(f"[bench] check: {clost} routed SET rows were lost (carry full)")
    fresh_iv = timed(args.steps, args.warmup + args.steps, events=True)[1] if use_events else []
    # secondary: the same steps with every GET probed and copied (no in-batch request
    # collapsing)
    unco = None
    if sc.coalesce and not args.no_uncoalesced:
        sc.coalesce = False
        step(0)
        unco_el, _, _ = timed(args.steps, args.warmup)
        sc.coalesce = True
        unco = (args.batch + args.sets) * world * args.steps / unco_el
    per_step = max((fresh["head1"] - fresh["head0"]) / max(args.steps, 1), 1.0)

    # the 16 GiB log wrapped: every SET batch runs the eviction hand, but the working set
    # fills only ~1/4 of the log, so nothing live is evicted or re-appended
    wrapped = wrapped_iv = nfill = None
    if steady_ok:
        base = args.warmup + 3 * args.steps
        nfill = fill_to_wrap(sc, shard, log_bytes, base, per_step)
        if nfill is not None:
            wrapped = window(sc, shard, base + nfill)
            if args.check and headline == "wrapped":
                check(wrapped)
            if use_events:
                wrapped_iv = timed(args.steps, base + nfill + args.steps, events=True)[1]
    if headline == "wrapped" and wrapped is None:
        raise SystemExit("[bench] the value log could not be wrapped for the headline; "
                         "pass --headline fresh")
    # the full cache (the headline): a shard whose working set fills --pressured-fill of its
    # log, wrapped, so the CLOCK hand re-appends the objects the steps read (reinsertions)
    # and evicts the rest: the state a serving cache runs in (memcached evicts under load)
    def full_cache(gb, check_it, min_fill=0, walk=None):
        """A shard of `gb` GiB populated with this rank's keys, wrapped (fill steps, at least
        `min_fill`), then the headline protocol (K timed steps), a GPU-event pass and one
        whole lap timed: (summary, window, event intervals, fill steps). `walk`: the
        (GET digests, GET ids, SET batches) the steps cycle instead of the default ones."""
        if walk is not None:
            cyc["gets"], cyc["get_ids"], cyc["sets"] = walk
        f_log = int(gb * (1 << 30)) // 16 * 16
        f_shard = CacheShard(f_log, nb, max_item=1 << 20, device=dev, evict=args.evict)
        f_sc = ShardedCache(f_shard, group=group, replica=replica,
                            data_group=data_group, routed=True if routed1 else None,
                            comm_mode=args.comm_mode, hand=args.hand)
        f_sc.coalesce = sc.coalesce
        f_sc.event_fence = sc.event_fence
        f_sc.gather_after_append = sc.gather_after_append
        if replica is not None:
            f_sc._hot, f_sc._hot_dir = sc._hot, None
        populate(f_sc)
        f_shard.reserve(max(args.sets * 2, chunk))
        sync()
        if real_world > 1:
            dist.barrier()
        fbase = 3 * args.warmup + 2 * args.steps

        def debug_hot(when):
            # SHELLAC_BENCH_DEBUG_HOT=1 (diagnostic): which of the 16 most popular objects
            # this shard holds (host routing: their owner and GET rank)
            if not os.environ.get("SHELLAC_BENCH_DEBUG_HOT"):
                return
            f_sc.sync_sets()
            sync()
            top = wl.rank_to_id[:16]
            d = wl.digests.index_select(0, top).contiguous()
            _, _, sz = f_shard.get(d)
            extra = ""
            if host_route:
                extra = (f" owners {owner_of.index_select(0, top).tolist()} GET ranks "
                         f"{spread.route_gets(d).tolist()}")
            hand, tail, head, hloc, *rest = f_shard._impl.debug_hand()
            lag = (hloc - (head - f_log)) / 2**20 if hloc != 2**64 - 1 else None
            log(rank, f"[debug] {when}: top-16 present {(sz > 0).int().tolist()}{extra}; hand "
                      f"{tail - hand} entries behind the ring tail, its item {lag} MiB past "
                      f"the overwrite point; consumed / windows {rest}; reinserted "
                      f"{f_shard.counters()['reinserted']}")

        debug_hot("after populate")
        ffill = fill_to_wrap(f_sc, f_shard, f_log, fbase, per_step)
        debug_hot("after fill")
        if ffill is not None and ffill < min_fill:
            for i in range(ffill, min_fill):
                serve_i(f_sc, fbase + i)
                if i % 64 == 0 or (os.environ.get("SHELLAC_BENCH_DEBUG_HOT") == "2" and i < 24):
                    debug_hot(f"fill step {i}")
            sync()
            ffill = min_fill
        out_ = fw = fiv = None
        if ffill is not None:
            fw = window(f_sc, f_shard, fbase + ffill)
            debug_hot("after window")
            if check_it:
                check(fw)
            fiv = timed(args.steps, fbase + ffill + args.steps, events=True,
                        cache=f_sc)[1] if use_events else []
            out_ = summary(fw, fiv, f_log, ffill)
            # what a client sees: the share of GET requests (duplicates included) answered
            # with a record, over K more steps (untimed: a reduction per step)
            hit_n = torch.zeros(2, dtype=torch.int64, device=dev)
            for i in range(args.steps):
                res = serve_i(f_sc, fbase + ffill + 2 * args.steps + i).wait()
                hit_n[0] += (res.size > 0).sum().to(dev)
                hit_n[1] += res.size.numel()
            if real_world > 1:
                hr = hit_n.to(rdev)
                dist.all_reduce(hr)
                hit_n = hr
            out_["request_hit_ratio"] = round(float(hit_n[0]) / max(float(hit_n[1]), 1.0), 4)
            # the cost of a step varies with where the hand is in the lap (the objects it
            # re-appended one lap earlier come round together): one whole lap, timed
            lap_steps = int(f_log / max(1.0, (fw["head1"] - fw["head0"]) / args.steps)) + 1
            if real_world > 1:  # one step count on every rank (the longest lap)
                lt = torch.tensor([lap_steps], dtype=torch.int64, device=rdev)
                dist.all_reduce(lt, op=dist.ReduceOp.MAX)
                lap_steps = int(lt)
            lap_el = timed(lap_steps, fbase + ffill + 3 * args.steps, cache=f_sc)[0]
            out_["lap_steps"] = lap_steps
            out_["lap_ms_per_step"] = round(lap_el / lap_steps * 1e3, 4)
            # the read working set: distinct keys the GET batches of one lap of steps read
            # (the stream's, the batches cycled when a lap is longer), as records over the log
            nb_ = len(cyc["get_ids"])
            seen = torch.zeros(int(wl.vlen.numel()), dtype=torch.bool, device=dev)
            for j in range(min(lap_steps, nb_)):
                seen[cyc["get_ids"][(fbase + ffill + j) % nb_].to(dev)] = True
            rid = seen.nonzero().flatten()
            rbytes = int((32 + ((wl.vlen.index_select(0, rid).long() + 15) & ~15)).sum())
            rk = torch.tensor([rbytes, int(rid.numel())], dtype=torch.int64, device=rdev)
            if real_world > 1:
                dist.all_reduce(rk, op=dist.ReduceOp.MAX)  # (the rank that reads the most)
            out_["read_working_set_over_capacity"] = round(int(rk[0]) / f_log, 4)
            out_["read_keys_per_lap"] = int(rk[1])
            out_["get_batches_per_lap"] = min(lap_steps, nb_)
            del seen, rid
        f_sc.sync_sets()
        cyc["gets"], cyc["get_ids"], cyc["sets"] = gets, get_ids, sets
        del f_sc, f_shard
        return out_, fw, fiv, ffill

    def walk_batches():
        """For a cache that cannot hold every key: (GET digests, GET ids, SET batches) where
        the SETs walk a random permutation of every key this rank holds (an evicted key comes
        back when the walk reaches it, like a cache-aside refill of the whole key space) and
        the GETs are --walk-get-batches fresh batches of the request stream. The 16 default
        GET batches repeat every 16 steps, so the keys they touch (~1/3 of 16M requests)
        would be the whole read working set: a log far smaller than the key space would
        still hold all of it."""
        own = torch.arange(lo, hi, device=dev) if fill_ids is None else fill_ids
        g = torch.Generator(device="cpu").manual_seed(777 + rank)
        own = own.index_select(0, torch.randperm(int(own.numel()), generator=g).to(own.device))
        ws_ = [wl.set_batch(own[s0: s0 + args.sets].contiguous())
               for s0 in range(0, max(1, int(own.numel()) - args.sets + 1), args.sets)]
        del own
        gi = []
        for i in range(max(args.walk_get_batches, 1)):
            if host_route:   # this rank's share of batch P + i of the global stream
                gg, gd, _, _ = global_batch(P + i)
                gi.append(gg[gd == me].contiguous())
                del gg, gd
            else:
                gi.append(wl.sample_ids(args.batch, 200000 + 1009 * rank + i))
        gd_ = [wl.digests.index_select(0, x).contiguous() for x in gi]
        return gd_, gi, ws_

    pressured = pw = piv = pfill = None
    pressured_cycled = None
    wb = None  # the walk: built once, shared by the headline and log_overfull
    if do_pressured and (args.set_walk or (args.overfull_fill > 0 and args.pressured_gb is None)):
        wb = walk_batches()
    if do_pressured:
        walk = wb if args.set_walk else None
        pressured, pw, piv, pfill = full_cache(
            p_gb, args.check and headline == "pressured",
            min_fill=2 * len(walk[2]) if walk else 0, walk=walk)
        if pressured is not None:
            pressured["stream"] = "walk" if walk else "cycled"
            pressured["set_batches_cycled"] = len(walk[2]) if walk else len(cyc["sets"])
            pressured["get_batches_cycled"] = len(walk[0]) if walk else len(cyc["gets"])
        if walk is not None and not args.no_cycled and world == 1:
            # secondary (N = 1): the same full cache on the 16 cycled batches (round 5's
            # headline); skipped with more ranks, where each block repopulates every shard
            pressured_cycled = full_cache(p_gb, False)[0]
            if pressured_cycled is not None:
                pressured_cycled["stream"] = "cycled"
    # secondary: a working set larger than the log (--overfull-fill x the log): the hit ratio
    # when the cache cannot hold every key
    overfull = None
    if do_pressured and args.overfull_fill > 0 and args.pressured_gb is None:
        # An evicted key comes back only when it is SET again (the default steps cycle 16
        # SET batches, 1M of the 4M keys), and 16 cycled GET batches read only ~1/3 of the
        # keys: walk_batches() (every key re-SET in turn, 256 fresh GET batches). The
        # populate itself wraps this log, evicting unread objects in key order: two passes
        # of the walk run before the window, so it sees the steady state, not the populate's
        # transient.
        overfull = full_cache(ws_bytes / args.overfull_fill / (1 << 30), False,
                              min_fill=2 * len(wb[2]), walk=wb)[0]
        if overfull is not None:
            overfull["set_batches_cycled"] = len(wb[2])
            overfull["get_batches_cycled"] = len(wb[0])
    del wb
    if headline == "pressured" and pw is None:
        raise SystemExit("[bench] the pressured log could not be wrapped for the headline; "
                         "pass --headline wrapped")
    hw, hw_iv, hw_log, hw_fill = {"pressured": (pw, piv, p_gb, pfill),
                                  "wrapped": (wrapped, wrapped_iv, None, nfill),
                                  "fresh": (fresh, fresh_iv, None, None)}[headline]

    # secondary (host routing): the spread hot set follows a drifting popularity order, one
    # incremental refresh per epoch (parallel/hotspread.py refresh_hot: only newly hot objects
    # fetched, within --drift-budget-mb, cooled replicas dropped), then steps of the drifted
    # stream routed by the new table
    def spread_drift():
        from shellac_amd.parallel.hotspread import refresh_hot

        E, K, PB = args.drift_epochs, args.spread_drift_steps, 4
        order = wl.rank_to_id
        swap = max(1, int(args.spread * args.spread_drift_swap))
        budget = int(args.drift_budget_mb * (1 << 20))
        fetch = sizes = None
        if sim:
            # the simulated rank's peers: their copies are the workload's objects
            lo_sorted, lo_order = torch.sort(wl.digests[:, 0].contiguous())

            def ids_of(dg):
                at = torch.searchsorted(lo_sorted, dg[:, 0].contiguous()).clamp_(
                    max=lo_sorted.numel() - 1)
                return lo_order.index_select(0, at)

            def fetch(dg, own):
                ids = ids_of(dg[own.to(dg.device) != me])
                if ids.numel():
                    sc.set(wl.set_batch(ids), if_absent=True)
                return int(ids.numel())

            def sizes(dg):
                return 32 + ((wl.vlen.index_select(0, ids_of(dg)).long() + 15) & ~15)
        epochs = []
        for e in range(1, E + 1):
            order = wl.drifted(order, args.spread, swap, 5151 + e)   # the same on every rank
            sample = wl.digests.index_select(0, wl.sample_ids(args.spread_sample, 8800 + e,
                                                              rank_to_id=order))
            sc.sync_sets()
            if real_world > 1:
                dist.barrier()
            sync()
            t0 = time.perf_counter()
            info = refresh_hot(sc, spread, sample, args.spread, me, world, budget_bytes=budget,
                               fetch=fetch, sizes=sizes)
            sync()
            t_ref = time.perf_counter() - t0
            del sample
            g_e, s_e = [], []
            req = torch.zeros(world, dtype=torch.float64, device=dev)
            for i in range(PB):
                g = wl.sample_ids(world * args.batch, 7700 + 97 * e + i, rank_to_id=order)
                gd = spread.route_gets(wl.digests.index_select(0, g), seq0=i * world * args.batch)
                st = wl.uniform_ids(world * args.sets, 7900 + 97 * e + i)
                sd = spread.route_sets(wl.digests.index_select(0, st))
                g_e.append(wl.digests.index_select(0, g[gd == me]).contiguous())
                s_e.append(wl.set_batch(st[(sd == me) | (sd < 0)].contiguous()))
                req += (torch.bincount(gd.long(), minlength=world) +
                        torch.bincount(sd[sd >= 0].long(), minlength=world) +
                        int((sd < 0).sum())).double()
                del g, gd, st, sd
            ev = torch.cuda.Event()
            ev.record()
            sc.sync_sets()
            c0 = shard.counters()
            if real_world > 1:
                dist.barrier()
            sync()
            t0 = time.perf_counter()
            for i in range(K):
                sc.serve(g_e[i % PB], s_e[i % PB], inputs_ready=ev)
            sync()
            t_steps = time.perf_counter() - t0
            sc.sync_sets()
            c1 = shard.counters()
            hit_n = [0, 0]
            for i in range(PB):   # what a client sees (untimed)
                r = sc.serve(g_e[i], s_e[i], inputs_ready=ev).wait()
                hit_n[0] += int((r.size > 0).sum())
                hit_n[1] += int(r.size.numel())
            agg = torch.tensor([t_steps, t_ref], dtype=torch.float64, device=rdev)
            if real_world > 1:
                dist.all_reduce(agg, op=dist.ReduceOp.MAX)
            epochs.append({"ms_per_step": round(float(agg[0]) / K * 1e3, 4),
                           "refresh_ms": round(float(agg[1]) * 1e3, 1),
                           "hot_added": info["added"], "hot_deferred": info["deferred"],
                           "hot_removed": info["removed"],
                           "replicas_dropped": info["replicas_dropped"],
                           "rank_share_max_over_mean": round(float(req.max() / req.mean()), 4),
                           "owner_hit_ratio": round((c1["get_hits"] - c0["get_hits"]) /
                                                    max(c1["get_ops"] - c0["get_ops"], 1), 4),
                           "request_hit_ratio": round(hit_n[0] / max(hit_n[1], 1), 4)})
            del g_e, s_e
        return {"epochs": E, "steps_per_epoch": K, "hot_objects_replaced_per_epoch": swap,
                "refresh_budget_mib": args.drift_budget_mb, "per_epoch": epochs}

    sdrift = None
    # (simulated worlds only: the real N-rank job's collectives in refresh_hot are covered by
    # the gloo test, and a secondary block must not put the driver's scaling run at risk)
    if (host_route and sim and args.spread and args.drift_epochs > 0
            and args.spread_drift_steps > 0 and steady_ok):
        sdrift = spread_drift()

    # secondary: a drifting hot set (hot objects replaced every epoch) with the replica tier
    # maintained incrementally between epochs (refresh under a byte budget, no flush)
    drift = None
    if (args.drift_epochs > 0 and replica is not None and dev.type == "cuda" and not bounce
            and sc._hot is not None):
        drift = hot_drift()

    t_sm = time.perf_counter()
    sm = {} if (args.no_smoke or dev.type != "cuda" or sim or bounce) else smoke(rank, world, dev)
    if sm:
        # BASELINE.json's headline: wall clock of the platform smoke checks
        sm["smoke_wallclock_s"] = round(time.perf_counter() - t_sm, 3)

    elapsed, gathered = hw["el"], hw["gathered"]
    hits, gops, gbytes, rep_hits, greq = hw["hits"], hw["gops"], hw["gbytes"], hw["rep"], hw["greq"]
    ops_per_step = (args.batch + args.sets) * world
    ms = elapsed / args.steps * 1e3
    value = ops_per_step * args.steps / elapsed
    if world == 1 and not routed1:
        parallelism = "shard1 (one GPU, no routing)"
    elif host_route:
        parallelism = (f"shard{world} (host-routed: ketama on the host proxies sends each "
                       f"request to the GPU owning its key"
                       + (f", the {args.spread} hottest objects replicated on every GPU and "
                          f"their GETs spread over the GPUs ({args.spread_policy})"
                          if args.spread else "") +
                       "; no GPU-to-GPU value traffic in the step)")
    else:
        parallelism = f"shard{world} (all-to-all routed, {args.comm_mode} communicator mode)"
    out = {
        "metric": "cache_ops_per_s",
        "value": round(value, 1),
        "unit": "requests/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "uint8",
        "data": "synthetic (device-generated Zipf web-object workload; random payloads)",
        "config": {
            "model": f"shellac-hbm-cache: ketama-ring sharded, 1 shard/GPU, {args.evict.upper()} log "
                     "+ 2-choice index",
            "global_batch": ops_per_step,
            "seq_len": None,
            "parallelism": parallelism,
            "get_per_rank": args.batch,
            "set_per_rank": args.sets,
            "keys_total": total_keys,
            "zipf_s": args.zipf,
            "value_bytes": [args.min_val, args.max_val],
            # the headline phase's shard log
            "log_gib_per_shard": round(hw_log, 3) if hw_log else args.log_gb,
            "set_dist": args.set_dist,
            "replicated_hot_objects": args.replicate if world > 1 else 0,
            "routing": ("none" if world == 1 and not sim and not routed1 else
                        "host" if host_route else "device (all-to-all)"),
            "spread_hot_objects": args.spread if host_route else 0,
        },
        # host routing (N > 1): each rank's true share of the one global stream (ketama
        # owners, hot objects sprayed with --spread), the per-rank steps of the headline
        # window, and the measured rate of the native host router on the box's cores
        "host_routing": (dict(route_info, simulated_rank=me if sim else None)
                         if host_route else None),
        # which cache state the headline steps ran in: "log_pressured" = a full cache (the
        # working set fills --pressured-fill of the log: CLOCK reinsertions and evictions in
        # every SET batch), "log_wrapped" = the 16 GiB log wrapped (the hand runs, nothing
        # live is evicted), "log_fresh" = before the first wrap
        "headline_phase": "log_" + headline,
        "working_set_over_capacity": round(ws_bytes / (hw_log * (1 << 30) if hw_log else log_bytes), 4),
        "warmup_detail": (f"{args.warmup} warmup steps, {args.steps} pre-wrap steps (log_fresh), "
                          f"{2 * args.steps} more, {nfill} fill steps to wrap the 16 GiB log, 2 x "
                          f"{args.steps} steps there (log_wrapped); a {hw_log:.2f} GiB shard "
                          f"populated and {hw_fill} fill steps to wrap it; then the {args.steps} "
                          f"timed steps") if headline == "pressured" else
                         (f"{args.warmup} warmup steps, {args.steps} pre-wrap steps (log_fresh), "
                          f"{2 * args.steps} more, {nfill} fill steps to wrap the log; then the "
                          f"{args.steps} timed steps") if headline == "wrapped" else None,
        "get_coalescing": sc.coalesce,
        # owner-shard probes (+ replica hits) per GET request: < 1 when duplicate
        # requests of a batch share one probe and one response record
        "get_probes_per_request": round((gops + rep_hits) / max(greq, 1), 4),
        "get_hit_ratio": round((hits + rep_hits) / max(gops + rep_hits, 1), 4),
        # share of the distinct-key lookups (after coalescing) a local replica answered
        "replica_hit_fraction": round(rep_hits / max(gops + rep_hits, 1), 4),
        "get_value_GBps_owner_shards": round(gbytes / elapsed / 1e9, 2),
        # distinct keys looked up per second (owner probes + replica hits), i.e. requests
        # that were not answered from a batch-mate's record
        "get_unique_per_s": round((gops + rep_hits) / elapsed, 1),
        "uncoalesced_ops_per_s": round(unco, 1) if unco else None,
        "batches_cycled": P,
        # CLOCK second chances per step (objects re-appended ahead of the log overwrite):
        # 0 until the value log has wrapped
        "reinserted_bytes_per_step": round(hw["rbytes"] / args.steps),
        "edge": args.edge,
        "routed_diag": diag,
        # the step before the value log first wraps (no eviction work)
        "log_fresh": summary(fresh, fresh_iv),
        # the 16 GiB log wrapped (the hand in every SET batch; ~1/4 of it live)
        "log_wrapped": summary(wrapped, wrapped_iv, fill=nfill) if wrapped else None,
        # the full cache (the default headline): reinsertions and evictions every step
        "log_pressured": pressured,
        # the same full cache on the 16 cycled GET / SET batches (~1/2 of the keys read)
        "log_pressured_cycled": pressured_cycled,
        # the working set --overfull-fill x the log (more keys than the cache holds)
        "log_overfull": overfull,
        # a drifting hot set with the replica maintained between epochs (N>1 / simulated)
        "hot_drift": drift,
        # host routing: the spread hot set refreshed incrementally under drift
        "spread_drift": sdrift,
        "smoke": sm,
    }
    if host_route and out["host_routing"] and "host_route_req_per_s" in out["host_routing"]:
        # what the host proxies can feed: one router per GPU share of the host's cores (the
        # measured rate is this process's, on its share), against the job's request rate.
        # The routing of the timed steps' batches was done beforehand, so the job rate alone
        # could claim more than the routers deliver: the headline is the smaller of the two.
        out.update(router_bound(out, route_info["host_route_req_per_s"], world))
    if host_edge:
        # responses delivered into pinned host memory (GPU -> host over PCIe) against the
        # PCIe 5.0 x16 roofline (~63 GB/s per direction); the keys and SET payloads
        # travel the other way (host -> GPU)
        out["host_delivered_GBps"] = round(gathered / elapsed / 1e9, 2)
        out["pcie_roofline_GBps"] = 63.0
        out["host_read_GBps"] = round(
            (args.batch * 16 + args.sets * (16 + 8 + 12) + int(wl.vlen.float().mean()) * args.sets)
            * args.steps / elapsed / 1e9, 2)
    if hw_iv:
        out["ms_per_step_median_gpu_events"] = median(hw_iv)
    if dev.type != "cuda":
        out["data"] = "cpu rehearsal over gloo: functional only, not a performance number"
    if bounce:
        out["metric"] = "cache_ops_per_s_rehearsal"
        out["data"] = (f"functional rehearsal: {world} ranks on one GPU, collectives bounced "
                       "through gloo; not a performance number")
    if routed1:
        out["metric"] = "cache_ops_per_s_routed_rehearsal"
        out["config"]["parallelism"] = "shard1, routed step over a one-rank RCCL communicator"
        out["data"] += "; routed one-rank rehearsal: not the N=1 headline"
    if sim:
        out["metric"] = "cache_ops_per_s_simulated"
        out["data"] = ((f"single-GPU simulation of rank 0 of {sim} host-routed ranks: its owner "
                        "share of the Zipf stream on its 1/N of the key space; profiling only, "
                        "not a scaling result") if host_route else
                       (f"single-GPU simulation of rank 0 of {sim} ranks: all-to-alls mirrored "
                        "locally (no interconnect), keys mapped onto the simulated rank's 1/N "
                        "of the key space; profiling only, not a scaling result"))
        out["n_gpus"] = 1
        out["simulated_world"] = sim
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    if real_world > 1:
        dist.barrier()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
