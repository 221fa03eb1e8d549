"""``shellac-ab``: ApacheBench-style driver for the native load generator.

Mirrors the reference's benchmark invocation (benchmarks/run-shellac.sh:
``ab -k -n 400 -c 10 -g shellac.dat -H "Accept-Encoding: gzip" http://127.0.0.1:8080/``)
and adds pipelining depth, worker threads and percentile output. ``-g`` writes an
ab-compatible gnuplot TSV (column 9 = ttime in ms, as benchmarks/requests.p plots).
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from typing import Optional, Sequence
from urllib.parse import urlparse

import numpy as np

from .._native import core
from ..utils.cpus import parse_cpus


def run(url: str, requests: int = 1000, concurrency: int = 10, keepalive: bool = True,
        headers: Sequence[str] = (), depth: int = 1, threads: int = 1,
        paths: Optional[Sequence[str]] = None, method: str = "GET", timeout_s: float = 120.0,
        objects: int = 0, zipf_s: float = 0.99, path_prefix: str = "/obj/",
        path_suffix: str = ".html", seed: int = 1, cpus: Sequence[int] = (),
        spin_us: int = 0) -> dict:
    """``objects`` > 0: request paths are generated natively — ``path_prefix + id +
    path_suffix`` with ids drawn Zipf(``zipf_s``) over ``objects`` objects, or in order
    (a cache-fill pass) when ``zipf_s`` is 0."""
    u = urlparse(url)
    host = u.hostname or "127.0.0.1"
    port = u.port or 80
    path = u.path or "/"
    if u.query:
        path += "?" + u.query
    res = core().run_load(host, port, list(paths) if paths else [path], int(requests),
                          int(concurrency), int(depth), int(threads), bool(keepalive),
                          list(headers), method, float(timeout_s), int(objects), float(zipf_s),
                          path_prefix, path_suffix, int(seed), [int(c) for c in cpus],
                          int(spin_us))
    lat = np.asarray(res["latency"]) * 1e3
    done = int(res["completed"])
    el = float(res["elapsed_s"])
    # steady state: completions between the 10th and 90th percentile completion times
    # (excludes connection setup, which ab's total time includes: ~80 ms for 1000
    # connections here, 10 % of a 200K-request run)
    steady = 0.0
    starts = np.sort(np.asarray(res["start"])) if done else np.zeros(1)
    # ramp: when the c-th request left, i.e. every connection is up and busy
    ramp_ms = float(starts[min(int(concurrency), len(starts)) - 1]) * 1e3
    if done >= 100:
        end = np.asarray(res["start"]) + np.asarray(res["latency"])
        a, b = np.percentile(end, [10, 90])
        steady = 0.8 * done / (b - a) if b > a else 0.0
    out = {
        "completed": done,
        "elapsed_s": el,
        "rps": done / el if el > 0 else 0.0,
        "steady_rps": steady,
        "ramp_ms": ramp_ms,
        "connect_ms": float(res["connected_s"]) * 1e3,
        # per connection, connect() -> writable: a handshake the server's accept queue
        # dropped shows here as a SYN retransmission (>= 1 s)
        "connect_lat_ms": ({"p50": float(np.percentile(res["connect_lat"], 50)) * 1e3,
                            "p99": float(np.percentile(res["connect_lat"], 99)) * 1e3,
                            "max": float(np.max(res["connect_lat"])) * 1e3}
                           if len(res["connect_lat"]) else None),
        "connect_call_ms": ({"p50": float(np.percentile(res["connect_call"], 50)) * 1e3,
                             "max": float(np.max(res["connect_call"])) * 1e3}
                            if len(res["connect_call"]) else None),
        "open_loop_ms": float(res["open_loop_s"]) * 1e3,
        "transfer_MBps": res["bytes"] / el / 1e6 if el > 0 else 0.0,
        "errors": int(res["errors"]),
        "non2xx": int(res["non2xx"]),
        "reconnects": int(res["reconnects"]),
        "latency_ms": {
            "mean": float(lat.mean()) if done else 0.0,
            "p50": float(np.percentile(lat, 50)) if done else 0.0,
            "p90": float(np.percentile(lat, 90)) if done else 0.0,
            "p99": float(np.percentile(lat, 99)) if done else 0.0,
            "p999": float(np.percentile(lat, 99.9)) if done else 0.0,
            "max": float(lat.max()) if done else 0.0,
        },
        "_start": res["start"],
        "_latency": res["latency"],
        "_status": res["status"],
    }
    return out


def write_gnuplot(path: str, result: dict, t0: float) -> None:
    """ab -g format: starttime seconds ctime dtime ttime wait (ttime in column 9 ms)."""
    with open(path, "w") as f:
        f.write("starttime\tseconds\tctime\tdtime\tttime\twait\n")
        for s, l in zip(result["_start"], result["_latency"]):
            ts = t0 + float(s)
            ms = int(round(float(l) * 1e3))
            f.write(f"{time.strftime('%a %b %d %H:%M:%S %Y', time.localtime(ts))}\t{int(ts)}\t0\t{ms}\t{ms}\t{ms}\n")


def main(argv: Optional[Sequence[str]] = None) -> int:
    p = argparse.ArgumentParser(prog="shellac-ab", description="ab-style HTTP load generator (native)")
    p.add_argument("-n", type=int, default=1000, help="number of requests")
    p.add_argument("-c", type=int, default=10, help="concurrency (connections)")
    p.add_argument("-k", action="store_true", help="HTTP keep-alive")
    p.add_argument("-g", default=None, help="gnuplot TSV output")
    p.add_argument("-H", action="append", default=[], help="extra header 'Name: value'")
    p.add_argument("--depth", type=int, default=1, help="pipelined requests per connection")
    p.add_argument("--threads", type=int, default=1)
    p.add_argument("--json", action="store_true")
    p.add_argument("--objects", type=int, default=0,
                   help="generate paths over this many objects (prefix + id + suffix)")
    p.add_argument("--zipf", type=float, default=0.99, help="popularity skew (0 = in order)")
    p.add_argument("--prefix", default="/obj/")
    p.add_argument("--suffix", default=".html")
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--timeout", type=float, default=120.0)
    p.add_argument("--cpus", default="", help="pin worker threads to these CPUs ('0-3,8')")
    p.add_argument("--spin-us", type=int, default=0,
                   help="workers busy-poll this long after their last event (pinned cores)")
    p.add_argument("url")
    a = p.parse_args(argv)
    t0 = time.time()
    r = run(a.url, a.n, a.c, a.k, a.H, a.depth, a.threads, timeout_s=a.timeout,
            objects=a.objects, zipf_s=a.zipf, path_prefix=a.prefix, path_suffix=a.suffix,
            seed=a.seed, cpus=parse_cpus(a.cpus), spin_us=a.spin_us)
    if a.g:
        write_gnuplot(a.g, r, t0)
    pub = {k: v for k, v in r.items() if not k.startswith("_")}
    if a.json:
        print(json.dumps(pub))
    else:
        print(f"Complete requests:      {pub['completed']}")
        print(f"Failed requests:        {pub['errors']} (non-2xx {pub['non2xx']})")
        print(f"Time taken for tests:   {pub['elapsed_s']:.3f} seconds")
        print(f"Requests per second:    {pub['rps']:.2f} [#/sec] (mean)")
        print(f"Transfer rate:          {pub['transfer_MBps']:.2f} MB/s")
        lm = pub["latency_ms"]
        print(f"Latency (ms):           mean {lm['mean']:.3f}  p50 {lm['p50']:.3f}  "
              f"p90 {lm['p90']:.3f}  p99 {lm['p99']:.3f}  max {lm['max']:.3f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
