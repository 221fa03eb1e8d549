"""Pure-Python memcached binary protocol: an in-process fake server and a client.

The reference's only test dependencies were a live memcached and Apache
(devenv:10; README.md:87-100). These let the native memcached *client*
(``csrc/backend.cc``) and *server* (``csrc/mcserver.cc``) be tested against an
independent implementation without daemons: the fake server is a dict-backed
subset (GET/GETK/GETQ/GETKQ/SET/SETQ/ADD/DELETE/NOOP/VERSION/FLUSH/QUIT) and the
client covers what tests and tools need.
"""
from __future__ import annotations

import socket
import socketserver
import struct
import threading
import time
from typing import Optional

HDR = struct.Struct(">BBHBBHIIQ")
GET, SET, ADD, REPLACE, DELETE, INCR, DECR, QUIT, FLUSH, GETQ, NOOP, VERSION, GETK, GETKQ = (
    0x00, 0x01, 0x02, 0x03, 0x04, 0x05, 0x06, 0x07, 0x08, 0x09, 0x0A, 0x0B, 0x0C, 0x0D)
APPEND, PREPEND, STAT, SETQ, DELETEQ, TOUCH = 0x0E, 0x0F, 0x10, 0x11, 0x14, 0x1C


def frame(magic, op, key=b"", extras=b"", value=b"", status=0, opaque=0, cas=0) -> bytes:
    return HDR.pack(magic, op, len(key), len(extras), 0, status,
                    len(extras) + len(key) + len(value), opaque, cas) + extras + key + value


def read_frame(sock) -> tuple:
    hdr = _recvn(sock, 24)
    magic, op, kl, el, _, status, bl, opaque, cas = HDR.unpack(hdr)
    body = _recvn(sock, bl)
    return op, status, opaque, cas, body[:el], body[el : el + kl], body[el + kl :]


def _recvn(sock, n) -> bytes:
    buf = b""
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("connection closed")
        buf += chunk
    return buf


class FakeMemcached:
    """Threaded dict-backed memcached (binary protocol) on 127.0.0.1:<port>."""

    def __init__(self, port: int = 0):
        self.data: dict = {}
        self.ops = 0
        self.lock = threading.Lock()
        outer = self

        class Handler(socketserver.BaseRequestHandler):
            def handle(self):
                s = self.request
                s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                try:
                    while True:
                        op, _, opaque, _, extras, key, value = read_frame(s)
                        out = outer._handle(op, opaque, extras, key, value)
                        if out is None:
                            return
                        if out:
                            s.sendall(out)
                except (ConnectionError, OSError):
                    return

        class TS(socketserver.ThreadingTCPServer):
            allow_reuse_address = True
            daemon_threads = True

        self._srv = TS(("127.0.0.1", port), Handler)
        self.port = self._srv.server_address[1]
        self._th = threading.Thread(target=self._srv.serve_forever, daemon=True)

    def _handle(self, op, opaque, extras, key, value) -> Optional[bytes]:
        now = time.time()
        with self.lock:
            self.ops += 1
            if op in (GET, GETQ, GETK, GETKQ):
                item = self.data.get(key)
                if item and item[2] and item[2] < now:
                    del self.data[key]
                    item = None
                k = key if op in (GETK, GETKQ) else b""
                if item:
                    return frame(0x81, op, k, struct.pack(">I", item[1]), item[0], opaque=opaque)
                return b"" if op in (GETQ, GETKQ) else frame(0x81, op, k, value=b"Not found",
                                                             status=1, opaque=opaque)
            if op in (SET, SETQ, ADD):
                flags, exp = struct.unpack(">II", extras[:8])
                if op == ADD and key in self.data:
                    return frame(0x81, op, status=2, opaque=opaque)
                self.data[key] = (value, flags, (now + exp) if exp else 0)
                return b"" if op == SETQ else frame(0x81, op, opaque=opaque)
            if op in (DELETE, DELETEQ):
                found = self.data.pop(key, None) is not None
                if op == DELETEQ and found:
                    return b""
                return frame(0x81, op, status=0 if found else 1, opaque=opaque)
            if op == NOOP:
                return frame(0x81, op, opaque=opaque)
            if op == VERSION:
                return frame(0x81, op, value=b"fake-1.0", opaque=opaque)
            if op == FLUSH:
                self.data.clear()
                return frame(0x81, op, opaque=opaque)
            if op == QUIT:
                return None
            return frame(0x81, op, status=0x81, opaque=opaque)

    def start(self) -> "FakeMemcached":
        self._th.start()
        return self

    def stop(self) -> None:
        self._srv.shutdown()
        self._srv.server_close()


class MemcacheClient:
    """Minimal blocking binary-protocol client (tests, tools, benchmarks)."""

    def __init__(self, host: str = "127.0.0.1", port: int = 11211, timeout: float = 5.0):
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._opaque = 0

    def _rpc(self, op, key=b"", extras=b"", value=b""):
        self._opaque += 1
        self.sock.sendall(frame(0x80, op, key, extras, value, opaque=self._opaque))
        return read_frame(self.sock)

    def get(self, key: bytes):
        op, status, _, _, extras, _, value = self._rpc(GET, key)
        if status:
            return None
        return value, struct.unpack(">I", extras)[0] if extras else 0

    def set(self, key: bytes, value: bytes, flags: int = 0, exptime: int = 0) -> int:
        return self._rpc(SET, key, struct.pack(">II", flags, exptime), value)[1]

    def add(self, key: bytes, value: bytes, flags: int = 0, exptime: int = 0) -> int:
        return self._rpc(ADD, key, struct.pack(">II", flags, exptime), value)[1]

    def replace(self, key: bytes, value: bytes, flags: int = 0, exptime: int = 0) -> int:
        return self._rpc(REPLACE, key, struct.pack(">II", flags, exptime), value)[1]

    def append(self, key: bytes, value: bytes) -> int:
        return self._rpc(APPEND, key, b"", value)[1]

    def incr(self, key: bytes, delta: int = 1, initial: int = 0, exptime: int = 0):
        _, status, _, _, _, _, value = self._rpc(INCR, key, struct.pack(">QQI", delta, initial, exptime))
        return None if status else struct.unpack(">Q", value)[0]

    def delete(self, key: bytes) -> bool:
        return self._rpc(DELETE, key)[1] == 0

    def touch(self, key: bytes, exptime: int) -> int:
        return self._rpc(TOUCH, key, struct.pack(">I", exptime))[1]

    def version(self) -> bytes:
        return self._rpc(VERSION)[6]

    def flush(self) -> int:
        return self._rpc(FLUSH)[1]

    def stats(self) -> dict:
        self._opaque += 1
        self.sock.sendall(frame(0x80, STAT, opaque=self._opaque))
        out = {}
        while True:
            _, _, _, _, _, key, value = read_frame(self.sock)
            if not key:
                return out
            out[key.decode()] = value.decode()

    def get_multi(self, keys) -> dict:
        """GETKQ x n + NOOP (how libmemcached pipelines a multiget)."""
        buf = b"".join(frame(0x80, GETKQ, k, opaque=i + 1) for i, k in enumerate(keys))
        self.sock.sendall(buf + frame(0x80, NOOP, opaque=0xFFFF))
        out = {}
        while True:
            op, status, opaque, _, extras, key, value = read_frame(self.sock)
            if op == NOOP:
                return out
            if status == 0:
                out[key] = value

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass
