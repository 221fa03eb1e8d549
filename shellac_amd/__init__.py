"""shellac_amd — an MI355X-native distributed web accelerator.

Same capabilities as kmacrow/Shellac (an HTTP/1.1 caching reverse proxy with a
consistent-hashed distributed cache), re-designed for MI355X: a native C++
epoll proxy, a native HTTP/1.1 codec, and a cache that lives in HBM, sharded
over the GPUs and driven by hand-written CDNA4 HIP kernels, with RCCL over
xGMI moving request batches between shards.
"""
__version__ = "0.2.0"

SERVER_NAME = "Shellac/0.2.0"


def core():
    """The native extension module (built in-tree; raises if unavailable)."""
    from ._native import core as _core

    return _core()
