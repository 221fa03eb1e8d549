"""Python API of the native HTTP/1.1 codec and StreamBuf.

Method-for-method parity with the reference's ``HttpParser``
(src/python/shellac/server/HttpParser.py:43-138) and ``StreamBuf``
(src/python/shellac/server/StreamBuf.py:35-78); the work happens in the native
core (``csrc/http.cc``, ``csrc/stream_buf.h``). Python 3 bytes replace Python 2
``str``; ``str`` inputs are accepted and encoded as latin-1.
"""
from __future__ import annotations

import io
from typing import Optional, Union

from .._native import core

BytesLike = Union[bytes, bytearray, memoryview, str]


def _b(data: BytesLike) -> bytes:
    if isinstance(data, str):
        return data.encode("latin-1")
    return bytes(data) if not isinstance(data, bytes) else data


class HttpParser:
    """Incremental HTTP/1.1 request/response parser (see csrc/http.h for the list of
    deliberate fixes relative to the reference)."""

    def __init__(self, decode_gzip: bool = True, eof_body: bool = False, no_body: bool = False):
        self._p = core().NativeHttpParser(decode_gzip)
        if eof_body:
            self._p.set_eof_body(True)
        if no_body:  # parsing the response to a HEAD request
            self._p.set_no_body(True)
        self._headers: Optional[dict] = None
        self._body: Optional[io.BytesIO] = None

    # -- parsing --------------------------------------------------------------------
    def parse(self, data: BytesLike, length: Optional[int] = None) -> int:
        """Parse ``data``; return the number of bytes consumed."""
        b = _b(data)
        n = self._p.parse(b, -1 if length is None else int(length))
        if self._p.error():
            raise ValueError(f"HTTP parse error: {self._p.error_message()}")
        self._body = None
        return n

    def finish(self) -> bool:
        """Signal EOF (close-delimited bodies); returns message_complete()."""
        self._body = None
        return self._p.finish()

    # -- accessors (HttpParser.py:67-98) --------------------------------------------
    def method(self):
        return self._p.method()

    def url(self):
        return self._p.url()

    def status(self):
        return self._p.status()

    def version(self) -> float:
        return self._p.version()

    def message(self):
        return self._p.message()

    def headers(self) -> dict:
        if self._headers is None:
            d: dict = {}
            for k, v in self._p.header_list():
                if k in d:
                    if isinstance(d[k], list):
                        d[k].append(v)
                    else:
                        d[k] = [d[k], v]
                else:
                    d[k] = v
            if not self._p.headers_complete():
                return d
            self._headers = d
        return self._headers

    def body(self) -> io.BytesIO:
        if self._body is None:
            self._body = io.BytesIO(self._p.body_bytes())
        return self._body

    def is_request(self) -> bool:
        return self._p.is_request()

    def is_response(self) -> bool:
        return not self._p.is_request()

    def headers_complete(self) -> bool:
        return self._p.headers_complete()

    def message_complete(self) -> bool:
        return self._p.message_complete()

    def keep_alive(self) -> bool:
        self._sync_headers()
        return self._p.keep_alive()

    def keep_alive_params(self) -> tuple:
        self._sync_headers()
        return tuple(self._p.keep_alive_params())

    # -- serialization (HttpParser.py:111-138) --------------------------------------
    def _sync_headers(self):
        if self._headers is None:
            return
        hl = []
        for k, v in self._headers.items():
            k = str(k).lower()
            if isinstance(v, list):
                hl.extend((k, str(x)) for x in v)
            else:
                hl.append((k, str(v)))
        self._p.set_header_list(hl)

    def __bytes__(self) -> bytes:
        self._sync_headers()
        return self._p.serialize()

    def serialize(self) -> bytes:
        return bytes(self)

    def __str__(self) -> str:
        return bytes(self).decode("latin-1")


class StreamBuf:
    """Append-only stream with an acknowledged read cursor (StreamBuf.py:35-78)."""

    def __init__(self, data: Optional[BytesLike] = None):
        self._s = core().NativeStreamBuf()
        if data:
            self.write(data)

    def write(self, data: BytesLike) -> None:
        self._s.write(_b(data))

    def ack(self, nbytes: int) -> None:
        self._s.ack(int(nbytes))

    def seek(self, pos: int) -> None:
        self._s.seek(int(pos))

    def read(self) -> bytes:
        return self._s.read()

    def close(self) -> None:
        self._s.close()

    def buffer(self) -> bytes:
        return self._s.buffer()

    def clear(self) -> None:
        self._s.clear()

    def complete(self) -> bool:
        return self._s.complete()

    def closed(self) -> bool:
        return self._s.closed()

    def ready(self) -> bool:
        return self._s.ready()

    def __len__(self) -> int:
        return self._s.size()
