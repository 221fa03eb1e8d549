"""``shellac-cached``: a cache node speaking the memcached binary protocol.

Exports this node's HBM shards (one per local MI355X) or a DRAM shard to the
rest of the cluster; proxies list it in ``-c host:port,...`` exactly like the
memcached nodes of the reference deployment (README.md:12, :30; Server.py:81-83).
"""
from __future__ import annotations

import argparse
import signal
import sys
import threading
from typing import Optional, Sequence

from .._native import core
from .proxy import make_backend


class CacheNode:
    def __init__(self, backend=None, port: int = 11211, bind: str = "0.0.0.0", threads: int = 1,
                 kind: str = "dram", **backend_opts):
        self.backend = backend if backend is not None else make_backend(kind, **backend_opts)
        self._srv = core().CacheServer(self.backend, port=port, bind=bind, threads=threads)

    @property
    def port(self) -> int:
        return self._srv.port

    def start(self) -> "CacheNode":
        self._srv.start()
        return self

    def stop(self) -> None:
        self._srv.stop()
        self._srv.wait()

    def running(self) -> bool:
        return self._srv.running

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()


def main(argv: Optional[Sequence[str]] = None) -> int:
    p = argparse.ArgumentParser(prog="shellac-cached", description="Shellac cache node (memcached binary protocol)")
    p.add_argument("-p", "--port", type=int, default=11211)
    p.add_argument("--bind", default="0.0.0.0")
    p.add_argument("--threads", type=int, default=2)
    p.add_argument("--cache", choices=["dram", "hbm"], default="dram")
    p.add_argument("--dram-mb", type=int, default=1024)
    p.add_argument("--gpus", type=str, default=None)
    p.add_argument("--hbm-gb", type=float, default=16.0)
    p.add_argument("--batch-us", type=int, default=0)
    p.add_argument("--no-hbm-filter", action="store_true",
                   help="send every GET to the GPUs (no host presence filter)")
    p.add_argument("--hbm-spin-us", type=int, default=50)
    p.add_argument("--hot-objects", type=int, default=1024,
                   help="--cache hbm on several GPUs: replicate this many of the most requested "
                        "objects on every GPU and spread their GETs (0: plain ketama)")
    p.add_argument("--hot-refresh-ms", type=int, default=1000)
    a = p.parse_args(argv)
    opts = ({"dram_mb": a.dram_mb} if a.cache == "dram" else
            {"gpus": [int(x) for x in a.gpus.split(",")] if a.gpus else None, "hbm_gb": a.hbm_gb,
             "batch_us": a.batch_us, "hbm_filter": not a.no_hbm_filter,
             "spin_us": a.hbm_spin_us, "hot_objects": a.hot_objects,
             "hot_refresh_ms": a.hot_refresh_ms})
    node = CacheNode(port=a.port, bind=a.bind, threads=a.threads, kind=a.cache, **opts).start()
    print(f"shellac-cached on port {node.port} ({a.cache})", flush=True)
    stop = threading.Event()
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    while not stop.is_set():
        stop.wait(0.5)
    node.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
