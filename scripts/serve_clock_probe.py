#!/usr/bin/env python3
"""Edge-server diagnostics: the device wall-clock rate the server's idle / lifetime
timers assume (hipDeviceAttributeWallClockRate) against the rate measured from two jobs
a host sleep apart, and how often back-to-back jobs relaunch the server."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shellac_amd.ops.cache import CacheShard, digest_strings  # noqa: E402

dev = torch.device("cuda", 0)
shard = CacheShard(1 << 28, 1 << 14, 1 << 16, dev)
keys = [f"/clk/{i}".encode() for i in range(64)]
shard.set_many(keys, [b"x" * 4096] * 64)
torch.cuda.synchronize()
imp = shard._impl
req = digest_strings(keys[:1], "cpu").pin_memory()
out = torch.empty(1 << 20, dtype=torch.uint8).pin_memory()
off = torch.empty(8, dtype=torch.int64).pin_memory()


def job():
    assert imp.serve_get(req.data_ptr(), 1, out.data_ptr(), out.numel(), off.data_ptr(),
                         shard.now(), 7)
    imp.serve_wait(7, 10000)
    t = time.perf_counter()
    tr = imp.serve_trace()
    rows = [tr[i * 8:(i + 1) * 8] for i in range(64)]
    last = max(rows, key=lambda r: r[0])  # (stamps land before the slot is published)
    return t, last[5]


job()
ta, ka = job()
time.sleep(0.05)
tb, kb = job()
print(f"wall clock: attribute {imp.wall_khz} kHz, measured {(kb - ka) / (tb - ta) / 1e3:.0f} kHz "
      f"(two jobs {1e3 * (tb - ta):.1f} ms apart)", flush=True)
for gap_us in (0, 20, 100, 300, 1000):
    l0 = imp.serve_launches
    lat = []
    for _ in range(300):
        t0 = time.perf_counter()
        job()
        lat.append((time.perf_counter() - t0) * 1e6)
        if gap_us:
            t1 = time.perf_counter() + gap_us * 1e-6
            while time.perf_counter() < t1:
                pass
    lat.sort()
    print(f"gap {gap_us} us: p50 {lat[150]:.1f} us p99 {lat[297]:.1f} us, "
          f"{imp.serve_launches - l0} relaunches in 300 jobs", flush=True)
