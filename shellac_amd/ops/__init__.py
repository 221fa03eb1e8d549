"""Batch compute ops (HIP kernels on GPU tensors, C++ host code on CPU tensors)."""
from .cache import (CacheShard, Lookup, coalesce, digest_packed, digest_strings, expand, item_bytes,
                    pack_values, unpack_records)
from . import routing

__all__ = ["CacheShard", "Lookup", "coalesce", "expand", "digest_packed", "digest_strings", "item_bytes", "pack_values",
           "unpack_records", "routing"]
