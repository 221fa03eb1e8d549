#!/usr/bin/env python3
"""D2H bandwidth into pinned host memory on one MI355X: SDMA copy (hipMemcpyAsync via
torch copy_) vs kernel stores over PCIe (k_segcopy gather into a pinned buffer), for the
sizes of a bench step's response (~330 MB) and smaller."""
import os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shellac_amd._native import core  # noqa: E402

dev = torch.device("cuda", 0)
c = core()
for mb in (16, 64, 330):
    n = mb << 20
    src = torch.randint(0, 255, (n,), dtype=torch.uint8, device=dev)
    dst = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    for _ in range(2):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter(); reps = 5
    for _ in range(reps):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    sdma = n * reps / (time.perf_counter() - t0) / 1e9
    # kernel stores: one segment covering the buffer, 64 KiB segments
    seg = 64 << 10
    m = n // seg
    src_off = torch.arange(m, dtype=torch.int64, device=dev) * seg
    dst_off = torch.arange(m + 1, dtype=torch.int64, device=dev) * seg
    s = torch.cuda.current_stream().cuda_stream
    c.segcopy(src.data_ptr(), src_off.data_ptr(), dst_off.data_ptr(), m, dst.data_ptr(), s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        c.segcopy(src.data_ptr(), src_off.data_ptr(), dst_off.data_ptr(), m, dst.data_ptr(), s)
    torch.cuda.synchronize()
    kern = n * reps / (time.perf_counter() - t0) / 1e9
    ok = bool(torch.equal(dst[:1 << 20].to(dev), src[:1 << 20]))
    print(f"{mb} MB: SDMA D2H {sdma:.1f} GB/s, kernel stores {kern:.1f} GB/s, check {ok}", flush=True)
