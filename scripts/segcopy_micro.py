#!/usr/bin/env python3
"""Microbenchmark of the segmented byte mover (k_segcopy, the GET gather): ~317K records
of log-uniform 96 B-4 KiB (the bench step's distinct GETs), copied into a contiguous
buffer from sources laid out several ways, to separate the kernel's own cost from the
cost of random reads over a large log. Prints median µs and GB/s (read + write)."""
import math
import sys

import torch

from shellac_amd._native import core


def main():
    dev = torch.device("cuda", 0)
    c = core()
    g = torch.Generator().manual_seed(1)
    n = 317_000
    lo, hi = math.log(64), math.log(4096)
    vals = torch.exp(torch.rand(n, generator=g) * (hi - lo) + lo).long()
    sizes = ((vals + 32 + 15) // 16 * 16)
    total = int(sizes.sum())
    dst_off = torch.zeros(n + 1, dtype=torch.int64)
    dst_off[1:] = torch.cumsum(sizes, 0)
    span_max = 16 << 30
    src = torch.empty(span_max + (1 << 20), dtype=torch.uint8, device=dev)
    dst = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream

    def run(name, soff, doff, nseg):
        # the kernel trusts its arguments: check every shape and bound on the host first
        assert soff.numel() == nseg and doff.numel() == nseg + 1
        assert int(soff.max()) + int((doff[1:] - doff[:-1]).max()) <= src.numel()
        assert int(doff[-1]) <= dst.numel()
        so = soff.to(dev)
        do = doff.to(dev)
        for _ in range(3):
            c.segcopy(src.data_ptr(), so.data_ptr(), do.data_ptr(), nseg, dst.data_ptr(), st)
        ts = []
        for _ in range(10):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            c.segcopy(src.data_ptr(), so.data_ptr(), do.data_ptr(), nseg, dst.data_ptr(), st)
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        us = sorted(ts)[len(ts) // 2]
        print(f"{name:48s} {us:8.1f} us  {2 * total / us / 1e3:7.0f} GB/s", flush=True)

    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        dst[:total].copy_(src[:total])
    a.record()
    for _ in range(10):
        dst[:total].copy_(src[:total])
    b.record()
    b.synchronize()
    us = a.elapsed_time(b) * 1e2
    print(f"{'torch copy (same bytes, contiguous)':48s} {us:8.1f} us  {2 * total / us / 1e3:7.0f} GB/s")
    run("sequential sources", dst_off[:n].clone(), dst_off, n)
    for span in (256 << 20, 1 << 30, 4 << 30, 16 << 30):
        # random 16-B aligned starts (with replacement: small spans hold fewer records)
        pos = torch.randint(0, (span - 8192) // 16, (n,), generator=g) * 16
        run(f"random sources over {span >> 20} MiB", pos, dst_off, n)
    # the N=1 step's segment list: 1M rows, ~70 % empty (coalesced duplicates)
    m = 1_048_576
    keep = torch.randperm(m, generator=g)[:n].sort().values
    sz = torch.zeros(m, dtype=torch.int64)
    sz[keep] = sizes
    doff = torch.zeros(m + 1, dtype=torch.int64)
    doff[1:] = torch.cumsum(sz, 0)
    pos = torch.zeros(m, dtype=torch.int64)
    pos[keep] = torch.randint(0, ((16 << 30) - 8192) // 16, (n,), generator=g) * 16
    run("random over 16 GiB, 1M rows of which 70% empty", pos, doff, m)
    return 0


if __name__ == "__main__":
    sys.exit(main())
