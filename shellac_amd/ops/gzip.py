"""Batch gzip / gunzip on the GPU (csrc/deflate.hip). Compression: one wave per 32 KiB
block, a lane-parallel lazy LZ77 parse over LDS hash chains, per-block stored / fixed /
dynamic Huffman codes planned on the device (csrc/deflate_plan.h), lane-parallel emission;
members decompress with zlib / gzip. Decompression: one wave per member (serial Huffman
decoding, lane-parallel copies and CRC-32), zlib fallback for anything it rejects.

The reference gunzips and re-gzips every cached origin response at level 6 on the CPU
(src/python/shellac/server/HttpParser.py:124-127, :343-351). Here whole batches of bodies
are compressed by one kernel launch (SURVEY.md §7.3 stretch item). GPU only: without a
GPU the native engine is not constructed and the call raises."""
from __future__ import annotations

from typing import Dict, List, Sequence

from .._native import core

_engines: Dict[int, object] = {}


def engine(device: int = 0):
    e = _engines.get(device)
    if e is None:
        e = _engines[device] = core().GpuGzip(device)
    return e


def gzip_batch(bodies: Sequence[bytes], device: int = 0) -> List[bytes]:
    """One gzip member per body (RFC 1952), compressed on ``cuda:device``."""
    return engine(device).compress(list(bodies))


def deflate_batch(bodies: Sequence[bytes], device: int = 0) -> List[bytes]:
    """Raw DEFLATE streams (RFC 1951), e.g. for ``zlib.decompress(x, -15)``."""
    return engine(device).deflate(list(bodies))


def gunzip_batch(members: Sequence[bytes], device: int = 0, max_out: int = 64 << 20) -> List[bytes]:
    """Inflate gzip members on ``cuda:device``. A member the GPU path rejects (corrupt,
    unusual framing, ISIZE over ``max_out``, CRC mismatch) goes through zlib, which
    raises on a corrupt one."""
    import zlib

    got = engine(device).inflate(list(members), max_out)
    out = []
    for m, g in zip(members, got):
        if g is None:
            d = zlib.decompressobj(31)
            g = d.decompress(m, max_out)
            if d.unconsumed_tail:
                raise ValueError("gzip member inflates past max_out")
        out.append(g)
    return out
