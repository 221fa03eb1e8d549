"""Loader for the native core. Fails loudly: there is no silent Python fallback.

``torch`` (when installed) is imported first so that the process has exactly one
HIP runtime: the core's ``libamdhip64.so.7`` then resolves to the copy PyTorch
already loaded instead of a second one from ``/opt/rocm``.
"""
from __future__ import annotations

import importlib
import os
import shutil

_core = None


def _try_import():
    return importlib.import_module("shellac_amd._shellac_core")


def core():
    """Return the ``_shellac_core`` extension module, building it in-tree if absent."""
    global _core
    if _core is not None:
        return _core
    if not os.environ.get("SHELLAC_NO_TORCH"):  # host-only helpers (load generator, origin)
        try:
            import torch  # noqa: F401  (one HIP runtime per process; see module doc)
        except ImportError:
            pass
    try:
        _core = _try_import()
    except ImportError as first:
        if os.environ.get("SHELLAC_NO_AUTOBUILD") or not shutil.which(
            os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
        ):
            raise ImportError(
                "shellac_amd native core (_shellac_core) is not built; run "
                "`python -m shellac_amd._build`"
            ) from first
        from . import _build

        _build.build()
        _core = _try_import()
    return _core
