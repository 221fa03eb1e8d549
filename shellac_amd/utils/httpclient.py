"""Raw-socket HTTP/1.1 keep-alive client with pipelining (tests, load generator)."""
from __future__ import annotations

import socket
from typing import List, Optional, Sequence

from ..server.http import HttpParser


class HttpClient:
    def __init__(self, host: str = "127.0.0.1", port: int = 8080, timeout: float = 10.0):
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._buf = b""

    @staticmethod
    def request_bytes(path: str, method: str = "GET", headers: Optional[dict] = None,
                      body: bytes = b"", host: str = "localhost") -> bytes:
        h = {"Host": host, "User-Agent": "shellac-test"}
        h.update(headers or {})
        if body:
            h["Content-Length"] = str(len(body))
        lines = [f"{method} {path} HTTP/1.1"] + [f"{k}: {v}" for k, v in h.items()]
        return ("\r\n".join(lines) + "\r\n\r\n").encode() + body

    def send(self, data: bytes) -> None:
        self.sock.sendall(data)

    def read_response(self, head: bool = False) -> HttpParser:
        p = HttpParser(decode_gzip=True, eof_body=True, no_body=head)
        while True:
            if self._buf:
                n = p.parse(self._buf)
                self._buf = self._buf[n:]
                if p.message_complete():
                    return p
            chunk = self.sock.recv(1 << 16)
            if not chunk:
                if p.finish():
                    return p
                raise ConnectionError("connection closed before a full response")
            self._buf += chunk

    def get(self, path: str, **kw) -> HttpParser:
        head = kw.get("method", "GET") == "HEAD"
        self.send(self.request_bytes(path, **kw))
        return self.read_response(head=head)

    def pipeline(self, paths: Sequence[str], **kw) -> List[HttpParser]:
        self.send(b"".join(self.request_bytes(p, **kw) for p in paths))
        return [self.read_response() for _ in paths]

    def closed_by_peer(self) -> bool:
        self.sock.settimeout(2.0)
        try:
            return self.sock.recv(1) == b""
        except (socket.timeout, OSError):
            return False

    def close(self) -> None:
        try:
            self.sock.close()
        except OSError:
            pass
