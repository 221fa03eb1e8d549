"""bench.py contract on the CPU: the distributed serving step rehearsed over gloo
(world 2, DRAM shards) must print exactly one well-formed JSON line and return
correct values (--check)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("route", ["host", "device"])
def test_bench_cpu_rehearsal_world2(route):
    """host: each rank serves the requests for the keys it owns (the default); device: the
    all-to-all routed step over gloo."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--device", "cpu", "--batch", "4096", "--sets", "512", "--keys-per-gpu", "32768",
           "--log-gb", "0.125", "--replicate", "4096", "--replica-gb", "0.03",
           "--sample-batches", "2", "--check", "--route", route]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd="/tmp")
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["warmup"] == 1
    assert out["config"]["global_batch"] == 2 * (4096 + 512)
    assert out["get_hit_ratio"] == 1.0
    assert out["config"]["routing"] == ("host" if route == "host" else "device (all-to-all)")
    assert out["config"]["replicated_hot_objects"] == (0 if route == "host" else 4096)
    assert "0 mismatches" in p.stderr
    if route == "host":
        # each rank serves its true share of the one global stream (unequal batches), hot
        # objects sprayed: the shares stay within 5 % of the mean, and the native host
        # router sends every request where the tensor routing did
        import re

        assert re.search(r"check: 0 of \d+ hit records name another key", p.stderr)
        hr = out["host_routing"]
        assert hr["rank_share_max_over_mean"] <= 1.05
        assert hr["host_route_agrees_with_device"] is True and hr["host_route_req_per_s"] > 0
        assert hr["spread_hot_objects"] > 0 and len(out["log_fresh"]["rank_ms_per_step"]) == 2
        assert sum(hr["rank_requests_per_step"]) >= 2 * (4096 + 512)
        # the headline never claims more than the host routers can feed
        cap = hr["host_route_job_capacity_req_per_s"]
        assert out["value"] == pytest.approx(min(hr["job_rate_req_per_s"], cap), rel=1e-6)
        assert hr["router_feeds_job"] == (cap >= hr["job_rate_req_per_s"])
        assert hr["value_bounded_by_router"] == (not hr["router_feeds_job"])
    else:
        assert "check: 0 of 4096 hit records name another key" in p.stderr


def test_router_bound_caps_the_host_routed_headline():
    """value = min(job rate, N x the measured router rate): router_feeds_job == False can
    no longer coexist with a headline above the routers' capacity."""
    sys.path.insert(0, ROOT)
    import bench

    out = {"value": 100.0, "ms_per_step": 2.0, "host_routing": {"rank_share_max_over_mean": 1.0}}
    r = bench.router_bound(out, 30.0, 2)  # the routers feed 60 requests/s
    hr = r["host_routing"]
    assert r["value"] == 60.0 and r["ms_per_step"] == round(2.0 * 100 / 60, 4)
    assert hr["router_feeds_job"] is False and hr["value_bounded_by_router"] is True
    assert hr["job_rate_req_per_s"] == 100.0 and hr["rank_share_max_over_mean"] == 1.0
    r = bench.router_bound(out, 80.0, 2)  # 160 >= 100: the job rate stands
    assert r["value"] == 100.0 and r["ms_per_step"] == 2.0
    assert r["host_routing"]["router_feeds_job"] is True
    assert r["host_routing"]["value_bounded_by_router"] is False


SMALL = ["--steps", "2", "--warmup", "1", "--device", "cpu", "--batch", "2048", "--sets", "256",
         "--keys-per-gpu", "8192", "--log-gb", "0.0625", "--replicate", "1024",
         "--replica-gb", "0.01", "--sample-batches", "1", "--batches", "2", "--no-uncoalesced"]


def test_bench_self_launches_ranks_without_torchrun():
    """--gpus 4 with no launcher: bench.py starts its own 4-rank child job (no exec) and
    the JSON reports 4 GPUs' worth of work."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", *SMALL],
                       capture_output=True, text=True, timeout=600, cwd="/tmp", env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 4
    assert out["config"]["global_batch"] == 4 * (2048 + 256)
    assert "launching 4 ranks" in p.stderr


def test_bench_rank_count_mismatch_exits_nonzero():
    """A launcher that started fewer ranks than --gpus must not yield a number."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", *SMALL],
                       capture_output=True, text=True, timeout=300, cwd="/tmp", env=env)
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert "refusing" in p.stderr


def test_bench_more_gpus_than_devices_exits_nonzero():
    """--gpus N on a node with fewer devices: a clear message and no number, instead of
    several ranks silently sharing a device (here: no GPU at all)."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", HIP_VISIBLE_DEVICES="")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=300, cwd="/tmp", env=env)
    assert p.returncode == 2, p.stderr[-2000:]
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert "GPUs on this node" in p.stderr


def test_bench_simulated_host_routed_world_cpu():
    """--simulate-world 4 --route host: rank 0's owner share of the Zipf stream over its
    1/4 of a 4x key space (one process, no mirrored collectives)."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2",
                        "--warmup", "1", "--device", "cpu", "--batch", "2048", "--sets", "256",
                        "--keys-per-gpu", "8192", "--log-gb", "0.125", "--batches", "2",
                        "--no-uncoalesced", "--simulate-world", "4", "--route", "host",
                        "--check"], capture_output=True, text=True, timeout=600, cwd="/tmp")
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert out["config"]["routing"] == "host" and out["simulated_world"] == 4
    assert out["config"]["keys_total"] == 4 * 8192
    assert out["get_hit_ratio"] == 1.0
    assert "0 mismatches" in p.stderr


@pytest.mark.gpu
def test_bench_host_routed_ranks_on_one_gpu():
    """The N>1 default's flow (host-routed ranks, barriers and reductions between steps,
    per-rank shard populate of different sizes) with two processes sharing the box's GPU
    over gloo: one JSON line, --check clean. (The flow once deadlocked in populate: each
    rank's cache routed over the default group.)"""
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--bounce", "--route", "host", "--check", "--steps", "3", "--warmup",
                        "1", "--no-uncoalesced"],
                       capture_output=True, text=True, timeout=300, cwd="/tmp",
                       env={**os.environ, "SHELLAC_BENCH_STACKS": "60"})
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["config"]["routing"] == "host" and out["n_gpus"] == 2
    # the headline is the full cache (working set 0.8 of the log: evictions, hit ratio < 1);
    # the fresh cache holds every key
    assert out["headline_phase"] == "log_pressured"
    assert out["working_set_over_capacity"] >= 0.8
    assert 0.9 <= out["get_hit_ratio"] <= 1.0
    assert out["log_fresh"]["owner_hit_ratio"] == 1.0
    assert "check: 0 mismatches in 200 sampled GETs" in p.stderr
    assert " 0 of " in p.stderr and "hit records name another key" in p.stderr


@pytest.mark.gpu
def test_bench_pooled_capacity_mode_on_one_gpu():
    """scripts/pooled_capacity.sh's mode, smaller: a fixed total key space (--keys-total) over a
    simulated 2-rank host-routed job, a 4 GiB shard log half the rank's working set (large
    enough for the hand's lead mode, layout.h hand_lead, as the bench's logs), SETs walking
    every key and fresh GET batches (--set-walk): evictions miss some requests, the replicas
    of spread hot objects stay (they are read every step), --check clean."""
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"),
                        "--simulate-world", "2", "--route", "host", "--keys-total", str(16 << 20),
                        "--pressured-gb", "4", "--log-gb", "2", "--set-walk",
                        "--walk-get-batches", "32", "--overfull-fill", "0", "--check",
                        "--steps", "3", "--warmup", "1", "--no-uncoalesced", "--no-smoke"],
                       capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    pr = out["log_pressured"]
    assert out["config"]["keys_total"] == 16 << 20
    assert pr["working_set_over_capacity"] > 1.5
    assert pr["get_batches_cycled"] == 32 and pr["set_batches_cycled"] >= 120
    # a cache holding half the keys: some misses, but the Zipf head (hot replicas included)
    # stays resident (0.67 when the CLOCK hand fell behind the overwrite and lost them)
    assert 0.85 < pr["request_hit_ratio"] < 1.0, pr
    assert "check: 0 mismatches in 200 sampled GETs" in p.stderr


@pytest.mark.gpu
def test_bench_spread_drift_block_on_one_gpu():
    """The spread_drift block (simulated host-routed world): each epoch drifts the
    popularity order, refreshes the spread hot set incrementally (hotspread.refresh_hot) and
    times steps of the drifted stream; the request shares stay even and every epoch reports
    what the refresh added and dropped."""
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"),
                        "--simulate-world", "2", "--route", "host", "--keys-per-gpu", str(1 << 20),
                        "--drift-epochs", "2", "--spread-drift-steps", "4", "--overfull-fill", "0",
                        "--steps", "3", "--warmup", "1", "--no-uncoalesced", "--no-smoke"],
                       capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    sd = out["spread_drift"]
    assert sd is not None and sd["epochs"] == 2 and len(sd["per_epoch"]) == 2
    for e in sd["per_epoch"]:
        assert e["hot_added"] > 0 and e["hot_added"] == e["hot_removed"]
        assert e["rank_share_max_over_mean"] < 1.05
        assert e["ms_per_step"] > 0 and 0.0 < e["request_hit_ratio"] <= 1.0
