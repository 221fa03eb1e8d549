#!/usr/bin/env python3
"""GPU batch gzip (csrc/deflate.hip) vs CPU zlib on HTML-like text bodies.

The miss path of a caching proxy compresses identity text responses before storing them
(the reference does gunzip + gzip level 6 on every miss, HttpParser.py:124-127,
:343-351). This measures one MI355X compressing a batch of bodies end to end — pinned
staging, H2D, kernel, D2H, host CRC-32 and member assembly — against single-core zlib at
levels 1 and 6, and reports the compression ratios. Every GPU member is checked with
zlib.decompress.

usage: python benchmarks/gzip_bench.py [--sizes 4096 65536] [--count 4096] [--reps 5]"""
import argparse
import json
import os
import random
import sys
import time
import zlib

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def html(rng, n):
    words = [b"cache", b"proxy", b"<div class=\"item\">", b"</div>", b"memcached", b"GPU",
             b"<a href=\"/static/obj/", b"\">", b"</a>", b"HBM", b"\n", b"  ", b"the", b"of",
             b"<span>", b"</span>", b"<li>", b"</li>"]
    out = bytearray()
    while len(out) < n:
        out += rng.choice(words)
        if rng.random() < 0.15:
            out += str(rng.randrange(10 ** 7)).encode()
        out += b" "
    return bytes(out[:n])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="+", default=[4096, 65536])
    ap.add_argument("--count", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu-sample", type=int, default=256, help="bodies timed with zlib")
    a = ap.parse_args()
    from shellac_amd.ops.gzip import engine

    assert torch.cuda.is_available()
    gz = engine(0)
    rng = random.Random(1)
    for size in a.sizes:
        count = max(1, min(a.count, (1 << 30) // size))
        bodies = [html(rng, size) for _ in range(count)]
        total = sum(map(len, bodies))
        out = gz.compress(bodies)  # warm-up (allocations)
        bad = sum(zlib.decompress(o, 31) != b for b, o in zip(bodies, out))
        ts = []
        for _ in range(a.reps):
            t = time.perf_counter()
            out = gz.compress(bodies)
            ts.append(time.perf_counter() - t)
        t_gpu = sorted(ts)[len(ts) // 2]
        st = gz.stats()
        sample = bodies[: a.cpu_sample]
        sb = sum(map(len, sample))
        res = {"body_bytes": size, "bodies": count, "batch_MB": round(total / 1e6, 1),
               "gpu_ms": round(t_gpu * 1e3, 2), "gpu_GBps": round(total / t_gpu / 1e9, 2),
               "gpu_ratio": round(sum(map(len, out)) / total, 4), "gpu_mismatches": bad,
               "last_call_ms": {"host_pack": round(st.last_pack_ms, 2),
                                "gpu_copies_and_kernel": round(st.last_gpu_ms, 2),
                                "host_assemble": round(st.last_assemble_ms, 2)}}
        for lvl in (1, 6):
            t = time.perf_counter()
            z = [zlib.compress(b, lvl) for b in sample]
            dt = time.perf_counter() - t
            res[f"zlib{lvl}_1core_MBps"] = round(sb / dt / 1e6, 1)
            res[f"zlib{lvl}_ratio"] = round(sum(map(len, z)) / sb, 4)
        res["gpu_vs_zlib6_1core"] = round(res["gpu_GBps"] * 1e3 / res["zlib6_1core_MBps"], 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
