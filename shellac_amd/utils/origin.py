"""A tiny HTTP/1.1 origin server for tests and benchmarks (stands in for the
reference's Apache upstream, benchmarks/run-baseline.sh). Counts requests per
path so tests can prove which requests the cache absorbed."""
from __future__ import annotations

import gzip
import threading
from collections import Counter
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer


class Origin:
    def __init__(self, port: int = 0, body_bytes: int = 1024, delay_s: float = 0.0,
                 keep_alive: bool = True):
        self.hits: Counter = Counter()
        self.lock = threading.Lock()
        self.healthy = True  # GET /health answers 200, or 503 when False
        outer = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1" if keep_alive else "HTTP/1.0"
            disable_nagle_algorithm = True

            def log_message(self, *a):
                pass

            def _reply(self, head: bool):
                with outer.lock:
                    outer.hits[self.path] += 1
                    n = outer.hits[self.path]
                if delay_s:
                    import time

                    time.sleep(delay_s)
                path = self.path
                if path == "/health":
                    code = 200 if outer.healthy else 503
                    body = b"ok\n" if outer.healthy else b"sick\n"
                    self.send_response(code)
                    self.send_header("Content-Length", str(len(body)))
                    self.end_headers()
                    if not head:
                        self.wfile.write(body)
                    return
                if path == "/badcl":  # malformed framing: the proxy must not pass it on
                    self.send_response(200)
                    self.send_header("Content-Length", "5x")
                    self.end_headers()
                    if not head:
                        self.wfile.write(b"hello")
                    return
                if path.startswith("/bomb"):  # 64 MiB of zeros, ~64 KB gzipped
                    z = outer.bomb()
                    self.send_response(200)
                    self.send_header("Content-Type", "text/html")
                    self.send_header("Content-Encoding", "gzip")
                    self.send_header("Content-Length", str(len(z)))
                    self.end_headers()
                    if not head:
                        self.wfile.write(z)
                    return
                if path.startswith("/status/"):
                    code = int(path.split("/")[2])
                    body = f"status {code}\n".encode()
                else:
                    code = 200
                    nb = body_bytes
                    if "/big/" in path:  # /big/<bytes>: a large object
                        nb = int(path.rsplit("/", 1)[1])
                    body = (f"<html>{path} #{n} ".encode() + b"x" * nb + b"</html>\n")
                headers = {"Content-Type": "text/html"}
                if path.startswith("/vary/ua"):  # one variant per User-Agent
                    headers["Vary"] = "User-Agent, Accept-Encoding"
                    body = body.replace(b"</html>", f"ua={self.headers.get('User-Agent')}</html>".encode())
                if path.startswith("/vary/star"):
                    headers["Vary"] = "*"
                if path.startswith("/nocache"):
                    headers["Cache-Control"] = "no-store"
                if path.startswith("/cookie"):
                    headers["Set-Cookie"] = "a=1"
                if path.startswith("/gz") and "gzip" in (self.headers.get("Accept-Encoding") or ""):
                    body = gzip.compress(body)
                    headers["Content-Encoding"] = "gzip"
                if path.startswith("/chunked"):
                    self.send_response(code)
                    for k, v in headers.items():
                        self.send_header(k, v)
                    self.send_header("Transfer-Encoding", "chunked")
                    self.end_headers()
                    if not head:
                        step = 100 if len(body) < 100000 else 65536
                        for i in range(0, len(body), step):
                            part = body[i : i + step]
                            self.wfile.write(b"%x\r\n" % len(part) + part + b"\r\n")
                        self.wfile.write(b"0\r\n\r\n")
                    return
                self.send_response(code)
                for k, v in headers.items():
                    self.send_header(k, v)
                self.send_header("Content-Length", str(len(body)))
                if not keep_alive:
                    self.send_header("Connection", "close")
                self.end_headers()
                if not head:
                    self.wfile.write(body)

            def do_GET(self):
                self._reply(False)

            def do_HEAD(self):
                self._reply(True)

            def do_POST(self):
                n = int(self.headers.get("Content-Length") or 0)
                data = self.rfile.read(n)
                with outer.lock:
                    outer.hits["POST " + self.path] += 1
                body = b"posted " + data
                self.send_response(200)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        class S(ThreadingHTTPServer):
            daemon_threads = True
            allow_reuse_address = True

        self._srv = S(("127.0.0.1", port), H)
        self.port = self._srv.server_address[1]
        self._th = threading.Thread(target=self._srv.serve_forever, daemon=True)

    _bomb = None

    def bomb(self) -> bytes:
        if Origin._bomb is None:
            Origin._bomb = gzip.compress(bytes(64 << 20), 9)
        return Origin._bomb

    def start(self) -> "Origin":
        self._th.start()
        return self

    def stop(self) -> None:
        self._srv.shutdown()
        self._srv.server_close()


class NativeOrigin:
    """C++ epoll origin (csrc/origin.cc) with the same response shape as ``Origin``
    for GET/HEAD: ``<html>{path} #1 xxx…</html>``, gzip-encoded for ``/gz*`` paths
    when the request accepts gzip. Used by ``benchmarks/http_bench.py`` so the
    miss-path RPS measures the proxy, not Python's ``http.server``."""

    def __init__(self, port: int = 0, body_bytes: int = 1024, threads: int = 2,
                 gzip_level: int = 1, random_body: bool = False, text_body: bool = False):
        from .._native import core

        # random_body: incompressible per-path bodies of exactly body_bytes;
        # text_body: compressible HTML-like bodies of exactly body_bytes
        self._o = core().NativeOrigin(port=port, threads=threads, body_bytes=body_bytes,
                                      gzip_level=gzip_level, random_body=random_body,
                                      text_body=text_body)
        self.port = self._o.port

    @property
    def requests(self) -> int:
        return self._o.requests

    def start(self) -> "NativeOrigin":
        self._o.start()
        return self

    def stop(self) -> None:
        self._o.stop()


def serve_native_origin(argv=None) -> int:
    """Run a NativeOrigin in its own process (benchmarks: the origin's CPU and memory stay
    out of the proxy process). Prints ``port <n>`` and serves until stdin closes."""
    import argparse
    import sys

    ap = argparse.ArgumentParser()
    ap.add_argument("--body", type=int, default=4096)
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--random-body", action="store_true")
    ap.add_argument("--text-body", action="store_true")
    ap.add_argument("--gzip-level", type=int, default=1)
    ap.add_argument("--cpus", default="", help="run on these CPUs only ('0-3,8')")
    a = ap.parse_args(argv)
    from .cpus import parse_cpus, pin_process
    pin_process(parse_cpus(a.cpus))
    o = NativeOrigin(body_bytes=a.body, threads=a.threads, gzip_level=a.gzip_level,
                     random_body=a.random_body, text_body=a.text_body).start()
    print(f"port {o.port}", flush=True)
    try:
        sys.stdin.read()
    finally:
        o.stop()
    return 0


if __name__ == "__main__":
    import sys

    sys.exit(serve_native_origin())
