#!/usr/bin/env python3
"""HTTP-level parity benchmark (BASELINE.md metrics 1, 2 and 4).

The reference's benchmark is ApacheBench against the proxy with a warm memcached
cluster (README.md:47-65; benchmarks/run-shellac.sh: ``ab -k -n N -c C -H
"Accept-Encoding: gzip"``). This runs the same shape with three processes:

  * the origin — native epoll server in its own process (``utils/origin.py``), serving
    *incompressible* per-URL bodies of ``--body`` bytes (random bytes seeded by the
    path), so a cached object is ``--body`` bytes on the wire;
  * the proxy — shellac_amd's native reactors in THIS process, with the cache backend
    under test (its peak RSS is reported alone);
  * the load generator — ``shellac-ab`` in its own process, keep-alive clients issuing
    Zipf(``--zipf``) requests over ``--objects`` URLs (paths generated natively).

Flow: fill pass (every object fetched once through the proxy, so it is cached), then
for each concurrency a short warm pass and a measured run: hit RPS, p50/p99/p99.9
latency, the proxy's hit ratio over the run (cache hits / requests — with a working
set larger than the cache some requests miss and go to the origin), bytes on the wire.

Backends: ``dram`` (host-DRAM cache of ``--dram-mb``), ``hbm`` (HBM shards only),
``tiered`` (``--l1-mb`` host L1 in front of the HBM shards).
Example: python benchmarks/http_bench.py --backend tiered --objects 4000000 --l1-mb 256
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from shellac_amd.server.proxy import Server, make_backend  # noqa: E402
from shellac_amd.utils import cpus as cpu_plan  # noqa: E402

# the origin and the load generator never touch the GPU: no torch / HIP runtime in them
HOST_ONLY = dict(os.environ, SHELLAC_NO_TORCH="1")


def rss_mb() -> tuple[float, float]:
    """(current, peak) resident MiB of this process (the proxy)."""
    cur = peak = 0.0
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                cur = int(line.split()[1]) / 1024
            elif line.startswith("VmHWM:"):
                peak = int(line.split()[1]) / 1024
    return cur, peak


def thread_cpu() -> dict:
    """CPU seconds of this process's threads grouped by name (reactors, GPU batchers,
    the rest)."""
    tick = os.sysconf("SC_CLK_TCK")
    out: dict = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/comm") as f:
                name = f.read().strip()
            with open(f"/proc/self/task/{tid}/stat") as f:
                fields = f.read().rsplit(")", 1)[1].split()
        except OSError:
            continue
        cpu = (int(fields[11]) + int(fields[12])) / tick
        grp = ("reactors" if name.startswith("shellac-rx") else
               "gpu_batcher" if name.startswith("shellac-hbm") else "other")
        out[grp] = out.get(grp, 0.0) + cpu
    return out


def cgroup_cpus() -> int:
    """CPUs the cgroup's CPU quota grants (0 when unlimited or unknown)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return 0 if q == "max" else max(1, int(q) // int(per))
    except (OSError, ValueError):
        return 0


def cgroup_throttle() -> dict:
    """nr_throttled / throttled_usec of this cgroup (CPU quota enforcement)."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            st = dict(l.split() for l in f if l.strip())
        return {k: int(st[k]) for k in ("nr_throttled", "throttled_usec") if k in st}
    except (OSError, ValueError):
        return {}


def cpu_ticks(cpus) -> dict:
    """/proc/stat jiffies per CPU: {cpu: (user, system, irq, softirq, idle)}."""
    out = {}
    try:
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("cpu") and line[3].isdigit():
                    v = line.split()
                    c = int(v[0][3:])
                    if c in cpus:
                        out[c] = (int(v[1]) + int(v[2]), int(v[3]), int(v[6]), int(v[7]), int(v[4]))
    except OSError:
        pass
    return out


def start_origin(body: int, threads: int, cpus=()) -> tuple[subprocess.Popen, int]:
    p = subprocess.Popen([sys.executable, "-m", "shellac_amd.utils.origin", "--body", str(body),
                          "--threads", str(threads), "--random-body",
                          "--cpus", cpu_plan.format_cpus(cpus)],
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, cwd=ROOT,
                         env=HOST_ONLY)
    line = p.stdout.readline().split()
    if len(line) != 2 or line[0] != "port":
        p.kill()
        raise RuntimeError(f"origin failed to start: {line}")
    return p, int(line[1])


def load(port: int, n: int, conc: int, threads: int, objects: int, zipf: float, prefix: str,
         seed: int, timeout: float, cpus=(), spin_us: int = 0) -> dict:
    """One shellac-ab run in its own process; returns its JSON summary."""
    cmd = [sys.executable, "-m", "shellac_amd.bench.ab", "-n", str(n), "-c", str(conc), "-k",
           "--threads", str(threads), "--objects", str(objects), "--zipf", str(zipf),
           "--prefix", prefix, "--suffix", "", "--seed", str(seed), "--timeout", str(timeout),
           "-H", "Accept-Encoding: gzip", "--json", "--cpus", cpu_plan.format_cpus(cpus),
           "--spin-us", str(spin_us),
           f"http://127.0.0.1:{port}/"]
    p = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT, timeout=timeout + 120,
                       env=HOST_ONLY)
    if p.returncode != 0:
        raise RuntimeError(f"load generator failed: {p.stderr[-2000:]}")
    return json.loads(p.stdout.strip().splitlines()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", choices=["dram", "hbm", "tiered", "none"], default="tiered")
    ap.add_argument("--threads", type=int, default=9, help="proxy reactor threads")
    ap.add_argument("--client-threads", type=int, default=6)
    ap.add_argument("--origin-threads", type=int, default=2)
    ap.add_argument("--objects", type=int, default=1000000)
    ap.add_argument("--body", type=int, default=4096, help="origin body bytes (incompressible)")
    ap.add_argument("--zipf", type=float, default=0.99)
    ap.add_argument("--requests", type=int, default=1000000)
    ap.add_argument("--conc", type=int, nargs="+", default=[10, 1000])
    ap.add_argument("--fill-conc", type=int, default=256)
    ap.add_argument("--dram-mb", type=int, default=256, help="--backend dram: cache MiB")
    ap.add_argument("--l1-mb", type=int, default=256, help="--backend tiered: host L1 MiB")
    ap.add_argument("--hbm-gb", type=float, default=0.0,
                    help="HBM log GiB per GPU (default: 1.25x the working set, >= 4)")
    ap.add_argument("--hbm-depth", type=int, default=3)
    ap.add_argument("--evict", choices=["clock", "fifo"], default="clock")
    ap.add_argument("--batch-us", type=int, default=0)
    ap.add_argument("--timeout", type=float, default=300.0)
    ap.add_argument("--pin", choices=["auto", "off"], default="auto",
                    help="auto: each reactor and load-generator worker on its own core of "
                         "the lowest allowed CPUs (one socket); the GPU batcher and the origin "
                         "on the last cores of the CPU budget")
    ap.add_argument("--rx-spin-us", type=int, default=None,
                    help="reactor busy-poll window (proxy --spin-us; default 200 when pinned, "
                         "else 0)")
    ap.add_argument("--lg-spin-us", type=int, default=None,
                    help="load-generator busy-poll window (shellac-ab --spin-us; default 200 "
                         "when pinned, else 0)")
    ap.add_argument("--cpu-budget", type=int, default=0,
                    help="CPUs to lay the processes over (default: the cgroup CPU quota)")
    ap.add_argument("--misc-cpus", type=int, default=0,
                    help="cores for the GPU batcher, the proxy's other threads and the origin "
                         "(default 1: the origin idles once the cache is filled)")
    ap.add_argument("--batcher-core", choices=["auto", "off"], default="auto",
                    help="auto (pinned GPU backends): the GPU batcher on a core of its own, "
                         "next to the misc core")
    ap.add_argument("--no-edge-server", action="store_true",
                    help="HBM: a kernel launch per GET batch instead of the resident server")
    ap.add_argument("--no-direct", action="store_true",
                    help="HBM: every GET through the batcher thread (no reactor-direct jobs)")
    ap.add_argument("--serve-blocks", type=int, default=8,
                    help="HBM: resident edge-server blocks per GPU (jobs served side by side)")
    ap.add_argument("--serve-backlog", type=int, default=2,
                    help="HBM: server jobs that may be ahead of a batch sent to the server")
    ap.add_argument("--layouts", nargs="+", default=None,
                    help="RxC pairs (reactor threads x load-generator threads), each measured "
                         "with its own proxy over the same filled cache (default: "
                         "--threads x --client-threads)")
    ap.add_argument("--shards", type=int, default=1,
                    help="HBM shards (all on GPU 0, a stand-in for that many GPUs: the ketama "
                         "split and hot-object spreading run as on a node)")
    ap.add_argument("--hot-objects", type=int, default=1024,
                    help="with --shards > 1: the replicated hot set (0: plain ketama)")
    ap.add_argument("--hot-refresh-ms", type=int, default=500)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    item = a.body + 400  # record + key + response headers, roughly
    hbm_gb = a.hbm_gb or max(4.0, 1.25 * a.objects * item / (1 << 30))
    gpu = a.backend in ("hbm", "tiered")
    layouts = [tuple(int(x) for x in l.split("x")) for l in
               (a.layouts or [f"{a.threads}x{a.client_threads}"])]
    budget = a.cpu_budget or cgroup_cpus() or len(cpu_plan.allowed_cpus())
    allowed = cpu_plan.allowed_cpus()[:budget]
    pin = a.pin == "auto" and len(allowed) >= 4
    nmisc = a.misc_cpus or 1
    misc_cpus = allowed[-nmisc:] if pin else []
    # the GPU batcher spins on its queue and on the GPU: a core of its own, not the
    # origin's / the proxy's other threads'
    batcher_cpus = []
    if pin and gpu and a.batcher_core == "auto":
        shards = a.shards if a.backend in ("hbm", "tiered") else 1
        batcher_cpus = allowed[len(allowed) - nmisc - shards: len(allowed) - nmisc]
        nmisc += shards
    # busy-polling only on dedicated (pinned) cores
    if a.rx_spin_us is None:
        a.rx_spin_us = 200 if pin else 0
    if a.lg_spin_us is None:
        a.lg_spin_us = 200 if pin else 0
    or_cpus = allowed[-1:] if pin else []  # the origin idles once the cache is filled

    def layout_cpus(r, c):
        if not pin:
            return [], []
        if r + c > len(allowed) - nmisc:
            raise SystemExit(f"layout {r}x{c} does not fit {len(allowed)} CPUs")
        return allowed[:r], allowed[r:r + c]

    origin, oport = start_origin(a.body, a.origin_threads, or_cpus)
    # threads created from here on (GPU batchers, HIP runtime) stay on the last cores;
    # each reactor pins itself to its own core
    cpu_plan.pin_process(misc_cpus)
    rss0, _ = rss_mb()
    if a.backend == "none":
        backend = None
    elif a.backend == "dram":
        backend = make_backend("dram", dram_mb=a.dram_mb)
    else:
        backend = make_backend("hbm", gpus=[0] * a.shards, hbm_gb=hbm_gb / a.shards,
                               batch_us=a.batch_us, hot_objects=a.hot_objects,
                               hot_refresh_ms=a.hot_refresh_ms,
                               l1_mb=a.l1_mb if a.backend == "tiered" else 0,
                               depth=a.hbm_depth, evict=a.evict,
                               edge_server=not a.no_edge_server, batcher_cpus=batcher_cpus,
                               serve_backlog=a.serve_backlog, direct=not a.no_direct,
                               serve_blocks=a.serve_blocks)
    prefix = "/o/"  # no /gz prefix: the origin sends the incompressible body as is
    out = {"backend": a.backend, "proxy_threads": layouts[0][0], "objects": a.objects,
           "body_bytes": a.body, "zipf": a.zipf, "working_set_MB": a.objects * item / 1e6,
           "dram_mb": a.dram_mb if a.backend == "dram" else None,
           "l1_mb": a.l1_mb if a.backend == "tiered" else None,
           "hbm_gb": hbm_gb if a.backend in ("hbm", "tiered") else None,
           "hbm_shards": a.shards if a.backend in ("hbm", "tiered") else None,
           "hot_objects": a.hot_objects if a.shards > 1 else 0,
           "cpu_count": os.cpu_count(), "cpu_budget": budget,
           "processes": "origin | proxy | load generator",
           "cpus": {"proxy_other": misc_cpus, "origin": or_cpus, "gpu_batcher": batcher_cpus},
           "edge_server": gpu and not a.no_edge_server, "serve_backlog": a.serve_backlog, "serve_blocks": a.serve_blocks,
           "reactor_direct": gpu and not a.no_edge_server and not a.no_direct,
           "spin_us": {"reactors": a.rx_spin_us, "load_generator": a.lg_spin_us}}
    px = None
    try:
        for li, (nrx, ncl) in enumerate(layouts):
            rx_cpus, lg_cpus = layout_cpus(nrx, ncl)
            px = Server([("127.0.0.1", oport)], port=0, backend=backend, threads=nrx,
                        client_max_reqs=1 << 30, cpus=rx_cpus,
                        spin_us=a.rx_spin_us).start()
            tag = "" if li == 0 else f"{nrx}x{ncl}_"
            out[f"{tag}layout"] = {"reactors": rx_cpus, "load_generator": lg_cpus}
            if li == 0:
                t0 = time.time()
                fill = load(px.port, a.objects, a.fill_conc, ncl, a.objects, 0.0, prefix, 1,
                            a.timeout, lg_cpus)
                out["fill"] = {"s": time.time() - t0, "rps": fill["rps"], "errors": fill["errors"]}
                print(f"[http] fill {a.objects} objects: {fill['rps']:.0f} rps", file=sys.stderr)
                time.sleep(1.0)
            for conc in a.conc:
                load(px.port, min(50000, a.requests), conc, ncl, a.objects, a.zipf,
                     prefix, 100 + conc, a.timeout, lg_cpus, a.lg_spin_us)
                s0 = px.stats()
                c0, l0, g0 = thread_cpu(), os.times(), cgroup_throttle()
                k0 = cpu_ticks(set(allowed))
                r = load(px.port, a.requests, conc, ncl, a.objects, a.zipf, prefix,
                         200 + conc, a.timeout, lg_cpus, a.lg_spin_us)
                c1, l1, g1 = thread_cpu(), os.times(), cgroup_throttle()
                r["cgroup_throttled"] = {k: g1[k] - g0.get(k, 0) for k in g1}
                k1 = cpu_ticks(set(allowed))
                # per core: (user, system, irq, softirq, idle) jiffies during the run
                r["core_ticks"] = {c: [b - a for a, b in zip(k0[c], k1[c])] for c in k1 if c in k0}
                s1 = px.stats()
                # where the CPU went during the run: proxy threads and the load generator
                r["cpu_s"] = {k: round(c1.get(k, 0) - c0.get(k, 0), 2) for k in c1}
                r["cpu_s"]["load_generator"] = round((l1.children_user + l1.children_system) -
                                                     (l0.children_user + l0.children_system), 2)
                reqs = s1["requests"] - s0["requests"]
                hits = s1["cache_hits"] - s0["cache_hits"]
                r["hit_ratio"] = hits / max(reqs, 1)
                r["origin_requests"] = s1["upstream_requests"] - s0["upstream_requests"]
                r["layout"] = f"{nrx}x{ncl}"
                sg = [s1.get("cache", {}).get(f"hbm_shard_gets_{i}", 0) -
                      s0.get("cache", {}).get(f"hbm_shard_gets_{i}", 0) for i in range(a.shards)]
                if a.shards > 1 and sum(sg):
                    # per-shard GET share (ketama split, evened out by hot-object spreading)
                    r["shard_get_share"] = [round(x / sum(sg), 4) for x in sg]
                    r["shard_get_max_over_mean"] = round(max(sg) / (sum(sg) / len(sg)), 4)
                out[f"{tag}c{conc}"] = r
                lm = r["latency_ms"]
                print(f"[http] {a.backend} {nrx}x{ncl} c={conc}: {r['rps']:.0f} rps "
                      f"(steady {r['steady_rps']:.0f}) hit ratio {r['hit_ratio']:.4f} "
                      f"p50 {lm['p50']:.3f} ms p99 {lm['p99']:.3f} ms "
                      f"{r['transfer_MBps']:.0f} MB/s errors {r['errors']} cpu {r['cpu_s']} "
                      f"elapsed {r['elapsed_s']:.2f}s connect {r.get('connect_lat_ms')} "
                      f"connect() {r.get('connect_call_ms')} open {r.get('open_loop_ms')} "
                      f"throttled {r['cgroup_throttled']}", file=sys.stderr)
            st = px.stats()
            if li + 1 < len(layouts):
                px.stop()
                px = None
        out["proxy_stats"] = st
        cur, peak = rss_mb()
        out["proxy_rss_MB"] = {"before_proxy": rss0, "end": cur, "peak": peak,
                               "peak_minus_baseline": peak - rss0}
    finally:
        if px is not None:
            px.stop()
        origin.stdin.close()
        origin.wait(timeout=30)
    js = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js)
    print(js)


if __name__ == "__main__":
    main()
