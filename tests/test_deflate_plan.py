"""Host-side DEFLATE planning of the GPU batch gzip (csrc/huffman.cc), on the CPU:
length-limited Huffman codes are complete and within the limit, and token streams encoded
with the planner's stored / fixed / dynamic choice decompress with zlib."""
import os
import random
import zlib

import pytest


@pytest.fixture(scope="module")
def core():
    from shellac_amd._native import core as _core

    return _core()


def greedy_tokens(data: bytes, window: int = 32768):
    """A tiny greedy LZ77 (one candidate per 4-byte hash), tokens as in huffman.h."""
    toks, head, i, n = [], {}, 0, len(data)
    while i < n:
        best = 0
        if i + 3 < n:
            key = data[i:i + 4]
            c = head.get(key)
            head[key] = i
            if c is not None and i - c <= window:
                m = 0
                while m < 258 and i + m < n and data[c + m] == data[i + m]:
                    m += 1
                best = m
        if best >= 3:
            toks.append(0x80000000 | (best << 16) | (i - c - 1))
            i += best
        else:
            toks.append(data[i])
            i += 1
    return toks


@pytest.mark.parametrize("n,max_len", [(286, 15), (30, 15), (19, 7), (2, 15), (286, 9)])
def test_huffman_lengths_complete_and_limited(core, n, max_len):
    rng = random.Random(n * 31 + max_len)
    for trial in range(30):
        # skewed (Fibonacci-like) frequencies force deep trees and the length limit
        freq = [0] * n
        for k in rng.sample(range(n), rng.randrange(2, n + 1)):
            freq[k] = int(1.6 ** rng.randrange(0, 40)) + 1
        ln = core.huffman_lengths(freq, max_len)
        used = [l for f, l in zip(freq, ln) if f]
        assert all(1 <= l <= max_len for l in used)
        assert all(l == 0 for f, l in zip(freq, ln) if not f)
        assert sum(2.0 ** -l for l in used) == pytest.approx(1.0)


def test_single_and_no_symbol_codes_are_complete(core):
    for freq in ([0] * 30, [0] * 5 + [7] + [0] * 24):
        ln = core.huffman_lengths(freq, 15)
        assert sum(2.0 ** -l for l in ln if l) == pytest.approx(1.0)


def _text(rng, n):
    words = [b"<div>", b"</div>", b"cache", b"proxy", b" ", b"\n", b"<a href=\"/x/", b"\">"]
    out = bytearray()
    while len(out) < n:
        out += rng.choice(words)
        if rng.random() < 0.2:
            out += str(rng.randrange(10 ** 6)).encode()
    return bytes(out[:n])


@pytest.mark.parametrize("kind", ["text", "random", "runs", "tiny", "empty"])
def test_token_streams_decompress_with_zlib(core, kind):
    rng = random.Random(hash(kind) & 0xFFFF)
    data = {"text": _text(rng, 30000), "random": os.urandom(5000), "runs": b"a" * 20000 + b"b" * 7,
            "tiny": b"hello", "empty": b""}[kind]
    toks = greedy_tokens(data)
    out = core.deflate_tokens_cpu(toks, data, True)
    assert zlib.decompress(out, -15) == data
    if kind == "text":  # dynamic codes beat zlib -1 on this text with the same window
        assert len(out) < len(zlib.compress(data, 1))


def test_fixed_codes_for_high_literals(core):
    """Tiny blocks take the fixed code; literals >= 144 use its 9-bit codes, whose
    canonical assignment counts the unused literal/length symbols 286-287."""
    rng = random.Random(11)
    for _ in range(300):
        data = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 6)))
        out = core.deflate_tokens_cpu(greedy_tokens(data), data, True)
        assert zlib.decompress(out, -15) == data, data


def test_non_final_blocks_concatenate(core):
    rng = random.Random(4)
    parts = [_text(rng, 12000), os.urandom(3000), _text(rng, 9000)]
    stream = b"".join(core.deflate_tokens_cpu(greedy_tokens(p), p, i == len(parts) - 1)
                      for i, p in enumerate(parts))
    assert zlib.decompress(stream, -15) == b"".join(parts)
