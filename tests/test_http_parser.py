"""Port of the reference's test/HttpParserTests.py + StreamBufTests.py to pytest,
plus the SURVEY.md §4 edge cases the native codec fixes.

The reference reads test/data/fish.jpg (HttpParserTests.py:257), which is missing
from the snapshot (.MISSING_LARGE_BLOBS); a 3.5 MiB synthetic binary blob of the
same role stands in for it."""
import math
import zlib

import numpy as np
import pytest

from shellac_amd.server import HttpParser, StreamBuf


def parse_all(req: bytes) -> list:
    out = []
    while len(req):
        h = HttpParser()
        while not h.message_complete():
            c = h.parse(req, len(req))
            req = req[c:]
            if c == 0 and not h.message_complete():
                raise AssertionError("parser made no progress")
        out.append(h)
    return out


def gz(b: bytes) -> bytes:
    z = zlib.compressobj(6, zlib.DEFLATED, 31)
    return z.compress(b) + z.flush()


def test_get_request():
    req = b"GET /get-request.html HTTP/1.1\r\nUser-Agent: Safari\r\nDate: Jul 25, 2013 5:14:11 GMT\r\n\r\n"
    p = HttpParser()
    while not p.message_complete():
        c = p.parse(req, len(req))
        req = req[c:]
    assert p.method() == "GET"
    assert p.url() == "/get-request.html"
    assert p.version() == 1.1
    assert p.headers()["user-agent"] == "Safari"
    assert p.is_request() and not p.is_response()


def test_post_request_with_body():
    req = (b"POST /post-request.html HTTP/1.1\r\nUser-Agent: Safari\r\nContent-Length: 10\r\n"
           b"Date: Jul 25, 2013 5:14:11 GMT\r\n\r\nXXXXXXXXXX")
    (p,) = parse_all(req)
    assert p.method() == "POST" and p.url() == "/post-request.html"
    assert p.headers()["user-agent"] == "Safari"
    assert p.body().read() == b"XXXXXXXXXX"


def test_pipelined_requests():
    req = (b"GET /stream1.html HTTP/1.1\r\nUser-Agent: Safari\r\nDate: Jul 25, 2013 5:14:11 GMT\r\n\r\n"
           b"POST /stream2.html HTTP/1.1\r\nUser-Agent: Safari\r\nContent-Length: 10\r\n"
           b"Date: Jul 25, 2013 5:14:11 GMT\r\n\r\nXXXXXXXXXX"
           b"POST /stream3.html HTTP/1.1\r\nUser-Agent: Safari\r\nContent-Length: 20\r\n"
           b"Date: Jul 25, 2013 5:14:11 GMT\r\n\r\nXXXXXXXXXXXXXXXXXXXX")
    ps = parse_all(req)
    assert len(ps) == 3
    assert [p.url() for p in ps] == ["/stream1.html", "/stream2.html", "/stream3.html"]
    assert all(p.message_complete() for p in ps)
    assert ps[2].body().read() == b"X" * 20


def test_pipelined_responses_including_gzip():
    req = b""
    for n in (10, 20, 30):
        req += (b"HTTP/1.1 200 OK\r\nUser-Agent: Safari\r\nDate: Jul 25, 2013 5:14:11 GMT\r\n"
                b"Content-Length: %d\r\n\r\n" % n) + b"X" * n
    req += b"HTTP/1.1 200 OK\r\nUser-Agent: Safari\r\nContent-Length: 0\r\nDate: x\r\n\r\n"
    req += b"HTTP/1.1 302 Not Modified\r\nUser-Agent: Safari\r\nDate: Jul 25, 2013 5:14:11 GMT\r\n\r\n"
    data = gz(b"A certain kind of magic.")
    req += (b"HTTP/1.1 200 OK\r\nUser-Agent: gws\r\nDate: Jan 4, 1989 2:51:12 GMT\r\n"
            b"Content-Encoding: gzip\r\nContent-Length: %d\r\n\r\n" % len(data)) + data
    ps = parse_all(req)
    assert len(ps) == 6
    assert [p.status() for p in ps] == [200, 200, 200, 200, 302, 200]
    assert ps[4].message() == "Not Modified"
    assert ps[5].body().read() == b"A certain kind of magic."


def test_parse_in_pieces():
    p = HttpParser()
    for req in (b"HTTP/1.1 200 OK\r\nUser-Agent: Safari\r\nDate: Jul 25, 2013 5:14:11 GMT\r\n",
                b"Content-Length: 10\r\n\r\nXXXXX"):
        while len(req):
            c = p.parse(req, len(req))
            req = req[c:]
    assert p.headers_complete()
    req = b"AAAAA"
    while len(req):
        c = p.parse(req, len(req))
        req = req[c:]
    assert p.message_complete()
    assert p.body().read() == b"XXXXXAAAAA"


def test_chunked_with_extensions_and_repeated_header():
    req = (b"HTTP/1.1 200 OK\r\nUser-Agent: Safari\r\nUser-Agent: Mac OS 10.8\r\n"
           b"Transfer-Encoding: chunked\r\nDate: Jul 25, 2013 5:14:11 GMT\r\n\r\n"
           b"A;ext=foo\r\nAAAAAAAAAA\r\n8;ext=\"foo\"\r\nBBBBBBBB\r\n6;ext=foo7\r\nCCCCCC\r\n0\r\n\r\n")
    (p,) = parse_all(req)
    assert p.body().read() == b"AAAAAAAAAABBBBBBBBCCCCCC"
    assert p.headers()["user-agent"] == ["Safari", "Mac OS 10.8"]


def test_gzip_chunked_split_stream():
    data = gz(b"Romeo, oh Romeo, why are thou so fair.")
    k = int(math.floor(len(data) / 3))
    parts = [data[:k], data[k : 2 * k], data[2 * k :]]
    assert zlib.decompress(b"".join(parts), 31) == b"Romeo, oh Romeo, why are thou so fair."
    req = (b"HTTP/1.1 200 OK\r\nUser-Agent: Safari\r\nTransfer-Encoding: chunked\r\n"
           b"Content-Encoding: gzip\r\nDate: Jul 25, 2013 5:14:11 GMT\r\n\r\n")
    for ext, part in zip((b";ext=foo", b';ext="foo"', b";ext=foo7"), parts):
        req += b"%x" % len(part) + ext + b"\r\n" + part + b"\r\n"
    req += b"0\r\n\r\n"
    (p,) = parse_all(req)
    assert p.body().read() == b"Romeo, oh Romeo, why are thou so fair."


def test_large_binary_body_in_1mib_pieces():
    # stands in for the missing test/data/fish.jpg (HttpParserTests.py:257-292)
    data = np.random.default_rng(5).integers(0, 256, size=3_500_000, dtype=np.uint8).tobytes()
    req = b"HTTP/1.1 200 OK\r\nUser-Agent: IE 6\r\nContent-Length: %d\r\n\r\n" % len(data) + data
    pieces = [req[i : i + (1 << 20)] for i in range(0, len(req), 1 << 20)]
    p = HttpParser()
    for chunk in pieces:
        if p.message_complete():
            break
        while len(chunk) and not p.message_complete():
            c = p.parse(chunk, len(chunk))
            chunk = chunk[c:]
    assert p.message_complete()
    assert p.body().read() == data


def test_serialize_response_and_request():
    req = (b"HTTP/1.1 500 Internal Server Error\r\nServer: Apache 2.2\r\nDate: Never\r\n"
           b"Content-Length: 12\r\n\r\nRRRRRRRRRRRR")
    (p,) = parse_all(req)
    s = bytes(p)
    assert s.startswith(b"HTTP/1.1 500 Internal Server Error\r\n")
    assert b"Server: Apache 2.2\r\n" in s and b"Content-Length: 12\r\n" in s
    assert s.endswith(b"\r\n\r\nRRRRRRRRRRRR")
    (q,) = parse_all(s)  # round trip
    assert q.status() == 500 and q.body().read() == b"R" * 12
    req = b"GET /index.html HTTP/1.1\r\nUser-Agent: Mozilla/WebKit 2.11\r\nDate: Never\r\n\r\n"
    (p,) = parse_all(req)
    assert str(p) == "GET /index.html HTTP/1.1\r\nUser-Agent: Mozilla/WebKit 2.11\r\nDate: Never\r\n\r\n"


def test_serialize_rechunks_and_regzips():
    data = gz(b"hello " * 100)
    req = (b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\nContent-Encoding: gzip\r\n\r\n"
           + b"%x\r\n" % len(data) + data + b"\r\n0\r\n\r\n")
    (p,) = parse_all(req)
    p.headers()["x-cache"] = "MISS"
    s = bytes(p)
    assert b"Transfer-Encoding" not in s and b"X-Cache: MISS" in s
    (q,) = parse_all(s)
    assert q.body().read() == b"hello " * 100
    assert int(q.headers()["content-length"]) == len(s.split(b"\r\n\r\n", 1)[1])


def test_keep_alive_params():
    (p,) = parse_all(b"HTTP/1.1 200 OK\r\nConnection: Keep-Alive\r\nKeep-Alive: timeout=15, max=99\r\n"
                     b"Content-Length: 0\r\n\r\n")
    assert p.keep_alive() and p.keep_alive_params() == (15, 99)
    (p,) = parse_all(b"HTTP/1.1 200 OK\r\nConnection: close\r\nContent-Length: 0\r\n\r\n")
    assert not p.keep_alive() and p.keep_alive_params() == (0, 1)
    (p,) = parse_all(b"HTTP/1.1 200 OK\r\nContent-Length: 0\r\n\r\n")
    assert p.keep_alive() and p.keep_alive_params() == (5, 100)
    (p,) = parse_all(b"HTTP/1.0 200 OK\r\nContent-Length: 0\r\n\r\n")
    assert not p.keep_alive()


# ---- SURVEY.md §4 edge cases the reference gets wrong -------------------------------
def test_zero_header_request_completes():
    (p,) = parse_all(b"GET / HTTP/1.1\r\n\r\n")
    assert p.url() == "/" and p.headers() == {}


def test_header_value_with_colon_space_and_no_space():
    (p,) = parse_all(b"GET / HTTP/1.1\r\nX-A: b: c\r\nX-B:nospace\r\n\r\n")
    assert p.headers()["x-a"] == "b: c" and p.headers()["x-b"] == "nospace"


def test_parse_zero_length_returns_zero():
    assert HttpParser().parse(b"", 0) == 0


def test_set_cookie_not_joined():
    (p,) = parse_all(b"HTTP/1.1 200 OK\r\nSet-Cookie: a=1; Path=/\r\nSet-Cookie: b=2\r\n"
                     b"Content-Length: 0\r\n\r\n")
    s = bytes(p)
    assert b"Set-Cookie: a=1; Path=/\r\nSet-Cookie: b=2\r\n" in s


def test_eof_delimited_body():
    p = HttpParser(eof_body=True)
    p.parse(b"HTTP/1.0 200 OK\r\nServer: x\r\n\r\nbody bytes ")
    p.parse(b"more")
    assert not p.message_complete()
    assert p.finish()
    assert p.body().read() == b"body bytes more"


@pytest.mark.parametrize("step", [1, 2, 3, 5, 7, 11, 13])
def test_slices_of_every_size(step):
    body = b"0123456789" * 7
    req = (b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n" + b"%x;x=y\r\n" % len(body) + body
           + b"\r\n0\r\nTrailer: t\r\n\r\n" + b"HTTP/1.1 200 OK\r\nContent-Length: 3\r\n\r\nabc")
    ps, p = [], HttpParser()
    for i in range(0, len(req), step):
        piece = req[i : i + step]
        while piece:
            c = p.parse(piece)
            piece = piece[c:]
            if p.message_complete():
                ps.append(p)
                p = HttpParser()
    assert [x.body().read() for x in ps] == [body, b"abc"]


def test_malformed_raises():
    with pytest.raises(ValueError):
        HttpParser().parse(b"garbage\r\n")
    with pytest.raises(ValueError):
        HttpParser().parse(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\nzz\r\n")


@pytest.mark.parametrize("head", [
    b"POST / HTTP/1.1\r\nContent-Length: 12abc\r\n\r\n",           # trailing garbage
    b"POST / HTTP/1.1\r\nContent-Length: -1\r\n\r\n",
    b"POST / HTTP/1.1\r\nContent-Length: 3\r\nContent-Length: 4\r\n\r\n",  # conflicting
    b"POST / HTTP/1.1\r\nContent-Length: 3, 4\r\n\r\n",
    b"POST / HTTP/1.1\r\nTransfer-Encoding: gzip\r\n\r\n",       # no final chunked
    b"POST / HTTP/1.1\r\nTransfer-Encoding: chunked, gzip\r\n\r\n",
    b"POST / HTTP/1.1\r\nTransfer-Encoding: xchunked\r\n\r\n",   # not a substring match
    b"POST / HTTP/1.1\r\nTransfer-Encoding: chunked\r\nContent-Length: 4\r\n\r\n",  # both
])
def test_ambiguous_request_framing_is_an_error(head):
    """RFC 7230 §3.3.3: a request the proxy and the origin could frame differently is
    rejected (the proxy answers 400), never guessed at."""
    with pytest.raises(ValueError):
        HttpParser().parse(head + b"abcd")


def test_strict_framing_accepts_valid_forms():
    # identical repeated Content-Length values and a chunked final coding are fine
    p = parse_all(b"POST /a HTTP/1.1\r\nContent-Length: 3\r\nContent-Length: 3\r\n\r\nabc")[0]
    assert p.body().read() == b"abc"
    p = parse_all(b"POST /b HTTP/1.1\r\nTransfer-Encoding: Chunked\r\n\r\n3\r\nabc\r\n0\r\n\r\n")[0]
    assert p.body().read() == b"abc"
    # a response with both: transfer-encoding wins (RFC 7230 §3.3.3 rule 3)
    p = HttpParser()
    p.parse(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\nContent-Length: 99\r\n\r\n"
            b"2\r\nhi\r\n0\r\n\r\n")
    assert p.message_complete() and p.body().read() == b"hi"


def test_gzip_body_with_pending_output_fully_inflated():
    # 1 MiB of one byte gzips to ~1 KB: after the last input byte most of the output is
    # still inside zlib and must be drained, not dropped
    body = b"a" * (1 << 20)
    z = gz(body)
    p = HttpParser(decode_gzip=True)
    p.parse(b"HTTP/1.1 200 OK\r\nContent-Encoding: gzip\r\nContent-Length: %d\r\n\r\n" % len(z) + z)
    assert p.message_complete() and p.body().read() == body


def test_decoded_gzip_body_is_capped():
    """--decode-gzip inflates every gzip body: a decompression bomb fails the parse
    instead of allocating the whole output."""
    bomb = gz(bytes(80 << 20))  # 80 MiB of zeros, ~80 KB compressed
    p = HttpParser(decode_gzip=True)
    with pytest.raises(ValueError, match="too large"):
        p.parse(b"HTTP/1.1 200 OK\r\nContent-Encoding: gzip\r\nContent-Length: %d\r\n\r\n"
                % len(bomb) + bomb)


# ---- StreamBufTests.py port -------------------------------------------------------
def test_streambuf_reference_behaviour():
    s = StreamBuf()
    assert s.ready() is False and s.closed() is False
    s.write(b"Hello")
    assert s.ready() is True
    assert s.read() == b"Hello" and s.read() == b"Hello"
    s.ack(2)
    assert s.read() == b"llo"
    s.ack(3)
    assert s.read() == b""
    s.close()
    assert s.closed() is True
    assert s.buffer() == b"Hello"
    s.clear()
    assert s.buffer() == b"" and s.ready() is False and s.closed() is False
    s.write(b"Romeo, oh Romeo.")
    s.close()
    s.ack(16)
    assert s.complete() is True


def test_streambuf_seek_and_segments():
    s = StreamBuf(b"abc")
    s.write("def")
    s.ack(4)
    assert s.read() == b"ef"
    s.seek(1)
    assert s.read() == b"bcdef"
    assert len(s) == 6
