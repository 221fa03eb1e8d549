#!/usr/bin/env python3
"""Host-observed latency of one micro-batch GET (the proxy's HBM hit path) against the
floor of a launch round trip: k_small_get with the completion slot, with a stream sync,
the resident edge server (serve_get: no launch), and an empty-ish kernel (torch fill of
one element) + sync; (p50, p99) of 2000 runs in us."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shellac_amd.ops.cache import CacheShard, digest_strings  # noqa: E402
from shellac_amd._native import core  # noqa: E402


def med(fn, iters=2000):
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return round(ts[len(ts) // 2] * 1e6, 1), round(ts[int(len(ts) * 0.99)] * 1e6, 1)


dev = torch.device("cuda", 0)
shard = CacheShard(1 << 30, 1 << 16, 1 << 16, dev)
keys = [f"/lat/{i}".encode() for i in range(4096)]
shard.set_many(keys, [b"x" * 4096] * 4096)
torch.cuda.synchronize()
s = torch.cuda.current_stream(dev).cuda_stream
imp = shard._impl
x = torch.zeros(1, device=dev)
print("empty kernel + sync (p50, p99 us)", med(lambda: (x.fill_(1.0), torch.cuda.synchronize())))
for n in (1, 10, 29, 100, 1000):
    req = digest_strings(keys[:n], "cpu")
    pin_k = req.pin_memory()
    out = torch.empty(n * 4200 + 4096, dtype=torch.uint8).pin_memory()
    off = torch.empty(n + 1, dtype=torch.int64).pin_memory()
    now = shard.now()

    def sync_path():
        imp.small_get(pin_k.data_ptr(), n, out.data_ptr(), out.numel(), off.data_ptr(), now, s, -1)
        torch.cuda.synchronize()

    def slot_path():
        imp.small_get(pin_k.data_ptr(), n, out.data_ptr(), out.numel(), off.data_ptr(), now, s, 7)
        imp.wait_host_slot(7, 10000)

    def serve_path():  # the resident edge server: a ring write, no launch
        assert imp.serve_get(pin_k.data_ptr(), n, out.data_ptr(), out.numel(), off.data_ptr(),
                             now, 7)
        imp.serve_wait(7, 10000)

    srv = f"  serve_get+slot {med(serve_path)}" if n <= int(core().SERVE_KEYS) else ""
    print(f"n={n}: small_get+sync {med(sync_path)}  small_get+slot {med(slot_path)}{srv}",
          flush=True)
    if srv:  # slow server samples vs relaunches (idle / lifetime exits)
        slow = relaunch_slow = 0
        for _ in range(2000):
            l0 = imp.serve_launches
            t0 = time.perf_counter()
            serve_path()
            dt = (time.perf_counter() - t0) * 1e6
            if dt > 50:
                slow += 1
                relaunch_slow += imp.serve_launches != l0
        print(f"   slow (>50 us) server samples: {slow} of 2000, {relaunch_slow} of them "
              f"relaunched the server", flush=True)
    if srv:  # where a server job's time goes (device wall clock, median of the last 64)
        tr = imp.serve_trace()
        rows = [tr[i * 8:(i + 1) * 8] for i in range(64)]
        rows = [r for r in rows if r[0] and r[6] == n]
        us = 1000.0 / imp.wall_khz
        def pm(a, b):
            v = sorted((r[b] - r[a]) * us for r in rows)
            return round(v[len(v) // 2], 2) if v else None
        print(f"   server phases (us): poll load {pm(1, 2)}  probe+scan {pm(2, 3)}  "
              f"copy+claim+drain {pm(3, 4)}  publish {pm(4, 5)}", flush=True)

# SET micro-batches: the launched chain (5 kernels) vs one replayed graph, both reading
# zero-copy staging in mapped pinned memory, + stream sync

cls = 64
hk = torch.zeros((cls, 2), dtype=torch.int64).pin_memory()
hv = torch.zeros(cls * 4096 + 16, dtype=torch.uint8).pin_memory()
ho = (torch.arange(cls, dtype=torch.int64) * 4096).pin_memory()
hm = torch.zeros(3 * cls, dtype=torch.int32).pin_memory()
hk[:] = digest_strings([f"/set/{i}".encode() for i in range(cls)], "cpu")
hm[:cls] = 4000
g = core().StoreGraph()
now = shard.now()
side = torch.cuda.Stream(device=dev)  # capturable (not the legacy default stream)
s = side.cuda_stream
p = [t.data_ptr() for t in (hk, hv, ho)] + [hm.data_ptr(), hm.data_ptr() + 4 * cls,
                                            hm.data_ptr() + 8 * cls]


def set_launch():
    imp.store(p[0], p[1], p[2], p[3], p[4], p[5], cls, 1 << 20, now, s)
    torch.cuda.synchronize()


def set_graph():
    imp.store_graph(g, p[0], p[1], p[2], p[3], p[4], p[5], cls, 1 << 20, now, s)
    torch.cuda.synchronize()


print(f"SET n={cls}: launched chain + sync {med(set_launch, 1000)}  graph + sync "
      f"{med(set_graph, 1000)} (captures {g.captures})", flush=True)
g.destroy()
