"""Diagnose slow connection setup against a GPU-tiered proxy holding many objects:
fill N objects, then time bursts of 1000 connections (each sending one request) with
and without a proxy stats() call right before the burst."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
import http_bench as hb  # noqa: E402
from shellac_amd.server.proxy import Server, make_backend  # noqa: E402

objects = int(sys.argv[1]) if len(sys.argv) > 1 else 2000000
backend_kind = sys.argv[2] if len(sys.argv) > 2 else "tiered"
origin, oport = hb.start_origin(4096, 2)
if backend_kind == "dram":
    be = make_backend("dram", dram_mb=256)
else:
    be = make_backend("hbm", gpus=[0], hbm_gb=max(4.0, 1.25 * objects * 4496 / (1 << 30)),
                      l1_mb=256 if backend_kind == "tiered" else 0)
px = Server([("127.0.0.1", oport)], port=0, backend=be, threads=int(os.environ.get("RX", 9)), client_max_reqs=1 << 30,
            cpus=list(range(int(os.environ.get("RX", 9))))).start()
lg = list(range(int(os.environ.get("RX", 9)), int(os.environ.get("RX", 9)) + int(os.environ.get("LG", 5))))
try:
    t0 = time.time()
    hb.load(px.port, objects, 256, 5, objects, 0.0, "/o/", 1, 600, lg)
    print(f"fill {objects}: {time.time() - t0:.1f}s", flush=True)
    def throttled():
        try:
            with open("/sys/fs/cgroup/cpu.stat") as f:
                return dict(l.split() for l in f)
        except OSError:
            return {}

    def show(tag):
        st = px.stats()
        c = st.get("cache", {})
        th = throttled()
        print(f"  [{tag}] loop_max_us {st.get('loop_max_us')} phases {st.get('loop_phase_max_us')} "
              f"loop_slow {st.get('loop_slow')} "
              f"accepts {st.get('accepts')} arena allocs {c.get('hbm_arena_allocs')} frees "
              f"{c.get('hbm_arena_frees')} bytes {c.get('hbm_arena_bytes')} "
              f"nr_throttled {th.get('nr_throttled')} throttled_usec {th.get('throttled_usec')}",
              flush=True)

    show("after fill")
    for i in range(3):
        if i % 2:
            t = time.time()
            px.stats()
            print(f"  stats() {1e3 * (time.time() - t):.1f} ms", flush=True)
        r = hb.load(px.port, 1000, 1000, 5, objects, 0.99, "/o/", 300 + i, 120, lg)
        print(f"burst {i}: connect {r['connect_ms']:.1f} ms ramp {r['ramp_ms']:.1f} ms "
              f"elapsed {1e3 * r['elapsed_s']:.1f} ms", flush=True)
        show(f"burst {i}")
        r = hb.load(px.port, 200000, 1000, 5, objects, 0.99, "/o/", 400 + i, 120, lg)
        print(f"run {i}: connect {r['connect_ms']:.1f} ms rps {r['rps']:.0f} steady {r['steady_rps']:.0f}",
              flush=True)
        show(f"run {i}")
finally:
    px.stop()
    origin.stdin.close()
    origin.wait(timeout=30)
