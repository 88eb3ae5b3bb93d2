"""Loader for the native extension ``distriflow_amd._C`` (gfx950 HIP kernels + C++ runtime).

The extension is built in-tree (``python -m distriflow_amd._build``).  GPU tensors ALWAYS go
through it: if it is missing or stale on a GPU box the ops raise instead of silently falling
back to eager PyTorch.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None
_err: Exception | None = None


def _try_import():
    global _mod, _err
    try:
        import torch  # noqa: F401  (loads libamdhip64 / libc10 first, so _C binds to the same runtime)

        _mod = importlib.import_module("distriflow_amd._C")
        _err = None
    except Exception as e:  # pragma: no cover - reported by require()
        _mod, _err = None, e


def get(build_if_missing: bool | None = None):
    """Return the ``_C`` module, building it first if allowed (default: DISTRIFLOW_AUTOBUILD=1)."""
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        _try_import()
        if _mod is None:
            if build_if_missing is None:
                build_if_missing = os.environ.get("DISTRIFLOW_AUTOBUILD", "1") == "1"
            if build_if_missing:
                from . import _build

                _build.build()
                _try_import()
    return _mod


def require():
    m = get()
    if m is None:
        raise RuntimeError(
            "distriflow_amd native extension (_C.so) is not available; build it with "
            f"`python -m distriflow_amd._build` (import error: {_err!r})"
        )
    return m


def available() -> bool:
    return get(build_if_missing=False) is not None
