#!/usr/bin/env python3
"""The proxy's compressing miss path (-z): zlib -6 on the reactor threads vs the GPU batch
gzip service (--gzip-gpu 0) vs no compression, on compressible HTML-like bodies.

Every request of the first pass is a miss (distinct objects in order, like the fill pass
of http_bench.py): origin fetch, compression of the identity text body, cache store,
response. The second pass reads the same objects back as hits (served gzip-encoded from
the DRAM cache). Origin, proxy and load generator are separate processes; the load
generator sends Accept-Encoding: gzip.

usage: python benchmarks/http_compress_bench.py [--body 8192] [--objects 200000]"""
import argparse
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import http_bench as hb  # noqa: E402
from shellac_amd.server.proxy import Server, make_backend  # noqa: E402


def start_text_origin(body: int, threads: int):
    p = subprocess.Popen([sys.executable, "-m", "shellac_amd.utils.origin", "--body", str(body),
                          "--threads", str(threads), "--text-body"],
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, cwd=hb.ROOT,
                         env=hb.HOST_ONLY)
    line = p.stdout.readline().split()
    if len(line) != 2 or line[0] != "port":
        p.kill()
        raise RuntimeError(f"origin failed to start: {line}")
    return p, int(line[1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--body", type=int, default=8192)
    ap.add_argument("--objects", type=int, default=200000)
    ap.add_argument("--threads", type=int, default=8, help="proxy reactor threads")
    ap.add_argument("--client-threads", type=int, default=4)
    ap.add_argument("--origin-threads", type=int, default=3)
    ap.add_argument("--conc", type=int, default=256)
    ap.add_argument("--modes", nargs="+", default=["none", "cpu", "gpu"])
    ap.add_argument("--gzip-batch-us", type=int, default=200, help="GPU service batch window")
    ap.add_argument("--timeout", type=float, default=300.0)
    a = ap.parse_args()
    origin, oport = start_text_origin(a.body, a.origin_threads)
    try:
        for i, mode in enumerate(a.modes):
            backend = make_backend("dram", dram_mb=max(512, 2 * a.objects * (a.body + 512) >> 20))
            prefix = f"/m{i}/"  # fresh objects per mode: every first-pass request misses
            with Server([("127.0.0.1", oport)], port=0, backend=backend, threads=a.threads,
                        client_max_reqs=1 << 30, compress=mode != "none",
                        gzip_gpu=0 if mode == "gpu" else -1,
                        gzip_batch_us=a.gzip_batch_us).start() as px:
                c0 = hb.thread_cpu()
                t0 = time.time()
                miss = hb.load(px.port, a.objects, a.conc, a.client_threads, a.objects, 0.0,
                               prefix, 1, a.timeout)
                dt = time.time() - t0
                c1 = hb.thread_cpu()
                st = px.stats()
                hit = hb.load(px.port, a.objects, a.conc, a.client_threads, a.objects, 0.0,
                              prefix, 2, a.timeout)
                res = {"mode": mode, "body_bytes": a.body, "objects": a.objects,
                       "gzip_batch_us": a.gzip_batch_us if mode == "gpu" else None,
                       "miss_rps": round(miss["rps"]),
                       "miss_p50_ms": round(miss["latency_ms"]["p50"], 3),
                       "miss_p99_ms": round(miss["latency_ms"]["p99"], 3),
                       "miss_errors": miss["errors"],
                       "hit_rps": round(hit["rps"]), "hit_errors": hit["errors"],
                       "proxy_cpu_s_during_misses": {k: round(c1.get(k, 0) - c0.get(k, 0), 2)
                                                     for k in c1},
                       "miss_wall_s": round(dt, 2),
                       "hit_MBps_on_wire": round(hit["transfer_MBps"]),
                       "gzip_gpu": st.get("gzip_gpu")}
                print(json.dumps(res), flush=True)
    finally:
        origin.stdin.close()
        origin.wait(timeout=10)


if __name__ == "__main__":
    main()
