#!/usr/bin/env python3
"""PCIe DMA rates on one MI355X: hipMemcpyAsync (torch's non_blocking copy_) of an HBM
buffer into pinned host memory and back, for the response sizes of the N=1 step (64 and
320 MiB). Prints GB/s. The gather kernel's own stores into pinned memory ran at ~38 GB/s
(bench.py --edge host, round 3); profiles/archive/r4s_edge_host compares the two in the step."""
import time

import torch


def rate(fn, nbytes, iters=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return nbytes * iters / (time.perf_counter() - t) / 1e9


def main():
    dev = torch.device("cuda", 0)
    for mb in (64, 320):
        n = mb << 20
        d = torch.randint(0, 255, (n,), dtype=torch.uint8, device=dev)
        h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        print(f"{mb} MiB: DMA D2H {rate(lambda: h.copy_(d, non_blocking=True), n):.1f} GB/s, "
              f"DMA H2D {rate(lambda: d.copy_(h, non_blocking=True), n):.1f} GB/s", flush=True)
        del d, h


if __name__ == "__main__":
    main()
