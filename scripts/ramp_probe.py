#!/usr/bin/env python3
"""Connection ramp of the load generator at c=1000: against the native origin directly
and through the proxy (diagnoses where 1000 keep-alive connections spend their setup)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shellac_amd.bench.ab import run  # noqa: E402
from shellac_amd.server.proxy import Server, make_backend  # noqa: E402
from shellac_amd.utils.origin import NativeOrigin  # noqa: E402

o = NativeOrigin(body_bytes=4096, threads=4).start()
hdr = ["Accept-Encoding: gzip"]
paths = [f"/gz/obj{i}.html" for i in range(1000)]
for c in (100, 1000):
    r = run(f"http://127.0.0.1:{o.port}", 100000, c, True, hdr, 1, 8, paths=paths)
    print("origin", c, round(r["ramp_ms"], 1), "ms ramp", round(r["connect_ms"], 1), "ms connected",
          round(r["steady_rps"]), flush=True)
def show(tag, r):
    print(tag, "ramp", round(r["ramp_ms"], 1), "ms, connected", round(r["connect_ms"], 1),
          "ms, steady", round(r["steady_rps"]), flush=True)


for th in (8,):
    px = Server([("127.0.0.1", o.port)], port=0, backend=make_backend("dram", dram_mb=256),
                threads=th, client_max_reqs=1 << 30).start()
    run(f"http://127.0.0.1:{px.port}", 1000, 8, True, hdr, 1, 1, paths=paths)
    for c in (10, 1000, 1000, 100, 1000):
        r = run(f"http://127.0.0.1:{px.port}", 500000, c, True, hdr, 1, 8, paths=paths)
        show(f"proxy threads {th} c={c}", r)
    px.stop()
o.stop()
for f in ("/proc/sys/net/core/somaxconn", "/proc/sys/net/ipv4/tcp_max_syn_backlog",
          "/proc/sys/net/ipv4/tcp_syncookies"):
    try:
        print(f, open(f).read().strip())
    except OSError as e:
        print(f, e)
