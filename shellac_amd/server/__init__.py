"""Server-side API: HTTP codec, StreamBuf, the proxy Server and the CLI.

Mirrors ``shellac.server`` of the reference (src/python/shellac/server/__init__.py:5-6,
which exports HttpParser and StreamBuf)."""
from .http import HttpParser, StreamBuf

__all__ = ["HttpParser", "StreamBuf"]
