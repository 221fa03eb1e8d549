"""Batch gzip on the GPU (csrc/deflate.hip): one wave per 32 KiB block, greedy LZ77 over
an LDS hash table, per-block stored / fixed / dynamic Huffman codes planned on the host
(csrc/huffman.cc); members decompress with zlib / gzip.

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
