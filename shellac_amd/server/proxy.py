"""Python API and CLI of the caching reverse proxy.

``Server`` keeps the reference constructor (src/python/shellac/server/Server.py:30,
``Server(servers, caches, port=8080, ttl=170, compress=False, cache=False)``) and
``run()`` (Server.py:442); the event loop itself is the native multi-threaded
reactor in ``csrc/proxy.cc``. ``main()`` keeps the reference CLI
(Server.py:490-547: ``-s/--servers``, ``-c/--caches``, ``-p/--port``, ``-t/--ttl``,
``-z/--compress``) and adds flags for the promoted constants and the GPU cache.
"""
from __future__ import annotations

import argparse
import signal
import socket
import sys
import threading
from typing import Iterable, Optional, Sequence, Union

from .._native import core
from ..utils.cpus import parse_cpus

ServerSpec = Union[str, tuple]


def _csv(items: Iterable[ServerSpec], default_port: int) -> str:
    out = []
    for it in items:
        if isinstance(it, tuple):
            out.append(f"{it[0]}:{int(it[1])}")
        elif ":" in str(it):
            out.append(str(it))
        else:
            out.append(f"{it}:{default_port}")
    return ",".join(out)


def parse_server_list(slist: str, default_port: int) -> list:
    """``"a:1,b"`` -> ``[(ip, 1), (ip, default_port)]`` with DNS resolution
    (reference: parse_server_list, Server.py:493-505)."""
    result = []
    for srv in [s for s in (slist or "").split(",") if s]:
        if ":" in srv:
            host, port = srv.rsplit(":", 1)
            result.append((socket.gethostbyname(host), int(port)))
        else:
            result.append((socket.gethostbyname(srv), default_port))
    return result


def make_backend(kind: str = "dram", *, caches: Sequence[ServerSpec] = (),
                 dram_mb: int = 1024, gpus: Optional[Sequence[int]] = None,
                 hbm_gb: float = 16.0, max_item: int = 1 << 20, batch_us: int = 0,
                 retry_s: int = 2, l1_mb: int = 0, promote_ttl: int = 60,
                 fault: Optional[str] = None,
                 sweep_s: int = 10, hbm_filter: bool = True, spin_us: int = 50,
                 depth: int = 3, evict: str = "clock", batch_timeout_ms: int = 2000,
                 edge_server: bool = True, batcher_cpus: Sequence[int] = (),
                 serve_backlog: int = 2, direct: bool = True, serve_blocks: int = 8,
                 hot_objects: int = 1024, hot_refresh_ms: int = 1000, hot_sample: int = 8):
    """Build a native cache backend.

    kind: ``memcached`` (ketama over ``caches``; the reference's configuration),
    ``dram`` (local host memory), ``hbm`` (one HBM shard per GPU in ``gpus``) or
    ``none``. ``l1_mb > 0`` puts a host-DRAM L1 of that size in front of the
    ``hbm`` / ``memcached`` tier (``TieredBackend``: L1 hits never wait for a GPU
    batch or a network round trip). ``fault`` (e.g. ``"get_miss=0.1,delay_us=500"``,
    ``"down"``) wraps the stack in a fault-injection backend; see ``set_fault``.
    ``hbm_filter`` keeps a host presence filter of stored digests so cold-key GETs miss
    without a GPU batch; ``spin_us`` is how long the HBM batcher polls before blocking;
    ``depth`` is how many batches each GPU keeps in flight; ``evict`` is the log policy
    (``clock``: read objects get a second chance, memcached-LRU-like; ``fifo``); a GPU
    whose batch fails or stalls past ``batch_timeout_ms`` is ejected for ``retry_s``.
    ``edge_server`` sends small GET batches to each GPU's resident edge-server kernel
    (no launch per batch); ``batcher_cpus`` pins the GPU batcher threads. ``direct``
    lets each proxy reactor write its own small GET batches to the edge server and poll
    their completion in its loop (no batcher-thread hop; larger batches still batch).
    ``fault="gpu_down=K"`` ejects GPU shard K as a drill. With several GPUs,
    ``hot_objects`` (0: off) is the size of the replicated hot set: the most requested
    objects of a sampled GET stream live on every GPU, their GETs spread over the GPUs and
    their SETs / DELETEs written through, re-planned every ``hot_refresh_ms`` (0: only on
    ``hot_refresh(backend)``) from one GET in ``hot_sample``.
    """
    c = core()
    if kind == "none":
        return None
    if fault is not None:
        # fault injection wraps the whole cache stack (set_fault() changes it live; ""
        # starts healthy)
        inner = make_backend(kind, caches=caches, dram_mb=dram_mb, gpus=gpus, hbm_gb=hbm_gb,
                             max_item=max_item, batch_us=batch_us, retry_s=retry_s, l1_mb=l1_mb,
                             promote_ttl=promote_ttl, sweep_s=sweep_s, hbm_filter=hbm_filter,
                             spin_us=spin_us, depth=depth, evict=evict,
                             batch_timeout_ms=batch_timeout_ms, edge_server=edge_server,
                             batcher_cpus=batcher_cpus, serve_backlog=serve_backlog,
                             direct=direct, serve_blocks=serve_blocks,
                             hot_objects=hot_objects, hot_refresh_ms=hot_refresh_ms,
                             hot_sample=hot_sample)
        return c.fault_backend(inner, fault)
    if l1_mb and kind in ("hbm", "memcached"):
        l2 = make_backend(kind, caches=caches, gpus=gpus, hbm_gb=hbm_gb, max_item=max_item,
                          batch_us=batch_us, retry_s=retry_s, sweep_s=sweep_s,
                          hbm_filter=hbm_filter, spin_us=spin_us, depth=depth, evict=evict,
                          batch_timeout_ms=batch_timeout_ms, edge_server=edge_server,
                          batcher_cpus=batcher_cpus, serve_backlog=serve_backlog,
                          direct=direct, serve_blocks=serve_blocks,
                          hot_objects=hot_objects, hot_refresh_ms=hot_refresh_ms,
                             hot_sample=hot_sample)
        return c.tiered_backend(c.dram_backend(int(l1_mb) << 20, max_item), l2, promote_ttl)
    if kind == "memcached":
        if not caches:
            raise ValueError("memcached backend needs cache servers (-c host:port,...)")
        return c.memcached_backend(_csv(caches, 11211), retry_s=retry_s)
    if kind == "dram":
        return c.dram_backend(int(dram_mb) << 20, max_item)
    if kind == "hbm":
        devs = list(gpus) if gpus is not None else list(range(max(1, c.device_count())))
        log_bytes = int(hbm_gb * (1 << 30)) // 16 * 16
        nb = 1
        while nb * 4 * 1024 < log_bytes:  # ~2 KiB/object at <=50% slot load
            nb *= 2
        return c.hbm_backend(devs, log_bytes, nb, max_item, batch_us, sweep_interval_s=sweep_s,
                             spin_us=spin_us, presence_filter=hbm_filter, depth=depth,
                             evict=evict, retry_s=retry_s, batch_timeout_ms=batch_timeout_ms,
                             edge_server=edge_server,
                             batcher_cpus=[int(x) for x in batcher_cpus],
                             serve_backlog=int(serve_backlog), direct=bool(direct),
                             serve_blocks=int(serve_blocks), hot_objects=int(hot_objects),
                             hot_refresh_ms=int(hot_refresh_ms), hot_sample=int(hot_sample))
    raise ValueError(f"unknown cache backend {kind!r}")


def hot_refresh(backend) -> dict:
    """Re-plan an HBM tier's replicated hot set now (what its refresh thread does every
    ``hot_refresh_ms``); returns the refresh's counts ({} when the tier has no hot set)."""
    return dict(core().hot_refresh(backend))


def set_fault(backend, spec: str) -> None:
    """Change the faults of a backend built with ``make_backend(..., fault=...)`` live:
    ``get_miss=P``, ``set_drop=P``, ``delay_us=N``, ``down`` (``""`` = healthy)."""
    core().set_fault(backend, spec)


class Server:
    """Shellac caching reverse proxy (reference-compatible constructor)."""

    def __init__(self, servers: Sequence[ServerSpec], caches: Sequence[ServerSpec] = (),
                 port: int = 8080, ttl: int = 170, compress: bool = False, cache: bool = False,
                 *, backend=None, backend_kind: Optional[str] = None, threads: int = 1,
                 policy: str = "rfc", kill_switch: bool = True, key_host: Optional[bool] = None,
                 client_timeout: int = 30, client_max_reqs: int = 1000,
                 balance: str = "random", bind: str = "0.0.0.0", decode_gzip: bool = False,
                 stream_bytes: int = 1 << 20, stream_high_water: int = 8 << 20,
                 health_path: str = "", health_interval_ms: int = 1000,
                 health_timeout_ms: int = 500, health_fails: int = 2,
                 cpus: Sequence[int] = (), spin_us: int = 0, gzip_gpu: int = -1,
                 gzip_batch_us: int = 200, gzip_workers: int = 2,
                 max_inflate_bytes: int = 64 << 20, **backend_opts):
        if not servers:
            raise ValueError("No upstream web servers specified.")
        self._backend = backend
        if self._backend is None and (cache or backend_kind):
            kind = backend_kind or ("memcached" if caches else "dram")
            self._backend = make_backend(kind, caches=caches, **backend_opts)
        if key_host is None:
            # rfc: virtual hosts never share an entry; reference: URL-only keys (Server.py:327)
            key_host = policy == "rfc"
        self._proxy = core().Proxy(
            _csv(servers, 80), self._backend, port=port, bind=bind, threads=threads, ttl=ttl,
            compress=compress, policy=policy, kill_switch=kill_switch, key_host=key_host,
            client_timeout=client_timeout, client_max_reqs=client_max_reqs, balance=balance,
            decode_gzip=decode_gzip, stream_bytes=stream_bytes,
            stream_high_water=stream_high_water, health_path=health_path,
            health_interval_ms=health_interval_ms, health_timeout_ms=health_timeout_ms,
            health_fails=health_fails, cpus=[int(c) for c in cpus], spin_us=int(spin_us),
            gzip_gpu=int(gzip_gpu), gzip_batch_us=int(gzip_batch_us),
            max_inflate_bytes=int(max_inflate_bytes), gzip_workers=int(gzip_workers))
        self._started = False

    @property
    def port(self) -> int:
        return self._proxy.port

    def set_fault(self, spec: str) -> None:
        """Live fault injection on the cache tier (requires ``fault=`` at construction)."""
        set_fault(self._backend, spec)

    @property
    def backend(self):
        return self._backend

    def start(self) -> "Server":
        if not self._started:
            self._proxy.start()
            self._started = True
        return self

    def run(self) -> None:
        """Serve until ``stop()`` / ``GET /kill`` / SIGTERM (blocking)."""
        self.start()
        self._proxy.wait()

    def stop(self) -> None:
        self._proxy.stop()
        if self._started:
            self._proxy.wait()

    def running(self) -> bool:
        return self._proxy.running

    def stats(self) -> dict:
        import json

        return json.loads(self._proxy.stats_json())

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()


def build_arg_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="shellac", description="Shellac Accelerator (MI355X-native)")
    p.add_argument("-s", "--servers", help="Web servers to cache: host:port,host:port,... (port defaults to 80)")
    p.add_argument("-c", "--caches", help="Cache servers to use: host:port,host:port,... (port defaults to 11211)")
    p.add_argument("-p", "--port", type=int, default=8080, help="Port to listen for connections on.")
    p.add_argument("-t", "--ttl", type=int, default=170, help="Lifetime of cached objects.")
    p.add_argument("-z", "--compress", action="store_true", help="Compress cached objects.")
    p.add_argument("--gzip-gpu", type=int, default=-1, metavar="GPU",
                   help="with -z: compress on this GPU, batched across reactor threads "
                        "(ops/gzip.py; default: zlib on the reactor threads)")
    p.add_argument("--gzip-batch-us", type=int, default=200,
                   help="collection window of one GPU gzip batch")
    # beyond the reference
    p.add_argument("--cache", choices=["memcached", "dram", "hbm", "none"], default=None,
                   help="cache backend (default: memcached if -c is given, else dram)")
    p.add_argument("--gpus", type=str, default=None, help="GPU ids for --cache hbm, e.g. 0,1,2,3")
    p.add_argument("--hbm-gb", type=float, default=16.0, help="HBM value-log GiB per GPU")
    p.add_argument("--dram-mb", type=int, default=1024, help="host cache MiB for --cache dram")
    p.add_argument("--no-hbm-filter", action="store_true",
                   help="send every GET to the GPUs (default: a host presence filter answers "
                        "GETs of never-stored keys without a GPU batch)")
    p.add_argument("--hbm-spin-us", type=int, default=50,
                   help="HBM batcher polls for new requests this long before sleeping")
    p.add_argument("--batch-us", type=int, default=0,
                   help="HBM batch linger (us); 0 = natural batching (what queued during the "
                        "previous batch)")
    p.add_argument("--l1-mb", type=int, default=256,
                   help="host-DRAM L1 in front of --cache hbm/memcached (0 = off)")
    p.add_argument("--threads", type=int, default=1, help="reactor threads (SO_REUSEPORT)")
    p.add_argument("--bind", default="0.0.0.0")
    p.add_argument("--cpus", default="",
                   help="pin reactor i to the i-th of these CPUs, e.g. 0-7 (default: unpinned)")
    p.add_argument("--spin-us", type=int, default=0,
                   help="reactors busy-poll this long after their last event before sleeping "
                        "(with --cpus: dedicated cores)")
    p.add_argument("--policy", choices=["rfc", "reference"], default="rfc",
                   help="rfc: cache GET 200/301/404.. honouring Cache-Control; reference: cache everything")
    p.add_argument("--balance", choices=["random", "roundrobin", "leastconn"], default="random")
    p.add_argument("--client-timeout", type=int, default=30)
    p.add_argument("--client-max-reqs", type=int, default=1000)
    p.add_argument("--key-host", dest="key_host", action="store_true", default=None,
                   help="include Host in the cache key (default: on with --policy rfc)")
    p.add_argument("--no-key-host", dest="key_host", action="store_false",
                   help="URL-only cache keys (the reference's, Server.py:327)")
    p.add_argument("--max-inflate-mb", type=int, default=64,
                   help="cap on any body the proxy inflates (identity variants for clients "
                        "without gzip, --decode-gzip); larger bodies answer 502")
    p.add_argument("--health-check", default="", metavar="PATH",
                   help="actively probe every upstream with GET PATH (the reference's TODO "
                        "'check that servers are responsive', Server.py:532)")
    p.add_argument("--health-interval-ms", type=int, default=1000)
    p.add_argument("--health-fails", type=int, default=2,
                   help="consecutive failed probes that take an upstream out of rotation")
    p.add_argument("--no-kill-switch", action="store_true", help="disable GET /kill")
    p.add_argument("--fault", default="",
                   help="fault injection on the cache tier, e.g. get_miss=0.1,set_drop=0.5,"
                        "delay_us=500, down, or gpu_down=K (eject GPU shard K; drills; "
                        "default off)")
    p.add_argument("--hbm-depth", type=int, default=3,
                   help="GET/SET batches each GPU keeps in flight (--cache hbm)")
    p.add_argument("--evict", choices=["clock", "fifo"], default="clock",
                   help="HBM log eviction: clock (read objects get a second chance, "
                        "memcached-LRU-like; default) or fifo")
    p.add_argument("--no-edge-server", action="store_true",
                   help="--cache hbm: launch a kernel per GET batch instead of feeding the "
                        "resident edge-server kernel")
    p.add_argument("--no-hbm-direct", action="store_true",
                   help="--cache hbm: every GET goes through the GPU batcher thread (default: "
                        "reactors send small GET batches to the edge server themselves)")
    p.add_argument("--batcher-cpus", default="",
                   help="--cache hbm: pin the GPU batcher threads to these CPUs")
    p.add_argument("--hot-objects", type=int, default=1024,
                   help="--cache hbm on several GPUs: replicate this many of the most requested "
                        "objects on every GPU and spread their GETs (0: plain ketama)")
    p.add_argument("--hot-refresh-ms", type=int, default=1000,
                   help="--cache hbm: how often the replicated hot set follows the traffic")
    p.add_argument("--stream-bytes", type=int, default=1 << 20,
                   help="stream responses larger than this to the client without caching them")
    p.add_argument("--decode-gzip", action="store_true",
                   help="inflate + re-deflate every miss like the reference (default: passthrough)")
    return p


def main(argv: Optional[Sequence[str]] = None) -> int:
    args = build_arg_parser().parse_args(argv)
    servers = parse_server_list(args.servers, 80) if args.servers else []
    caches = parse_server_list(args.caches, 11211) if args.caches else []
    if not servers:
        print("No upstream web servers specified. See shellac -h for help.")
        return 1
    kind = args.cache or ("memcached" if caches else "dram")
    if kind == "memcached" and not caches:
        print("No cache servers specified. See shellac -h for help.")
        return 1
    gpus = [int(x) for x in args.gpus.split(",")] if args.gpus else None
    srv = Server(servers, caches, port=args.port, ttl=args.ttl, compress=args.compress,
                 backend_kind=kind, threads=args.threads, policy=args.policy,
                 kill_switch=not args.no_kill_switch, key_host=args.key_host,
                 client_timeout=args.client_timeout, client_max_reqs=args.client_max_reqs,
                 balance=args.balance, bind=args.bind, decode_gzip=args.decode_gzip,
                 stream_bytes=args.stream_bytes, health_path=args.health_check,
                 health_interval_ms=args.health_interval_ms, health_fails=args.health_fails,
                 cpus=parse_cpus(args.cpus), spin_us=args.spin_us,
                 gzip_gpu=args.gzip_gpu, gzip_batch_us=args.gzip_batch_us,
                 max_inflate_bytes=args.max_inflate_mb << 20,
                 **({"fault": args.fault} if args.fault else {}),
                 **({"dram_mb": args.dram_mb} if kind == "dram" else {}),
                 **({"gpus": gpus, "hbm_gb": args.hbm_gb, "batch_us": args.batch_us,
                     "hbm_filter": not args.no_hbm_filter, "spin_us": args.hbm_spin_us,
                     "depth": args.hbm_depth, "evict": args.evict,
                     "edge_server": not args.no_edge_server,
                     "direct": not args.no_hbm_direct,
                     "batcher_cpus": parse_cpus(args.batcher_cpus),
                     "hot_objects": args.hot_objects, "hot_refresh_ms": args.hot_refresh_ms}
                    if kind == "hbm" else {}),
                 **({"l1_mb": args.l1_mb} if kind in ("hbm", "memcached") else {}))
    print(f"Running Shellac on port {args.port} (cache: {kind})...", flush=True)
    stop = threading.Event()

    def _sig(signum, frame):  # SIGINT/SIGTERM: clean shutdown (ref installs a no-op SIGINT)
        stop.set()
        srv.stop()

    signal.signal(signal.SIGINT, _sig)
    signal.signal(signal.SIGTERM, _sig)
    try:
        srv.start()
        while srv.running() and not stop.is_set():
            stop.wait(0.2)
    finally:
        srv.stop()
        print("\nShutting down...")
    return 0


if __name__ == "__main__":
    sys.exit(main())
