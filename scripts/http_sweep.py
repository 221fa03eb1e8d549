#!/usr/bin/env python3
"""Thread-count sweep of the HTTP hit path (DRAM backend, native origin):
usage: http_sweep.py PROXY_THREADS CLIENT_THREADS -> one line per concurrency
(threads, client threads, c, rps, p50 ms, p99 ms)."""
import os
import sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shellac_amd.bench.ab import run
from shellac_amd.server.proxy import Server, make_backend
from shellac_amd.utils.origin import NativeOrigin
o=NativeOrigin(body_bytes=4096,threads=1).start()
be=make_backend("dram", dram_mb=256)
pt=int(sys.argv[1]); ct=int(sys.argv[2])
px=Server([("127.0.0.1",o.port)],port=0,backend=be,threads=pt,client_max_reqs=1<<30).start()
url=f"http://127.0.0.1:{px.port}"
paths=[f"/gz/obj{i}.html" for i in range(1000)]
run(url,1000,8,True,["Accept-Encoding: gzip"],1,1,paths=paths)
for c in (10,100,1000):
    r=run(url,200000,c,True,["Accept-Encoding: gzip"],1,ct,paths=paths)
    print(pt,ct,c,round(r['rps']),round(r['latency_ms']['p50'],3),round(r['latency_ms']['p99'],3))
px.stop(); o.stop()
