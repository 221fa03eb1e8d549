"""Batch compute ops (HIP kernels on GPU tensors, C++ host code on CPU tensors)."""
from .cache import (CacheShard, Lookup, digest_packed, digest_strings, item_bytes, pack_values,
                    unpack_records)
from . import routing

__all__ = ["CacheShard", "Lookup", "digest_packed", "digest_strings", "item_bytes", "pack_values",
           "unpack_records", "routing"]
