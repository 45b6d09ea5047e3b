"""Loader for the in-tree native extension (``_C.so``).

The HIP kernels are the compute path on GPU: if the extension is missing or fails to load,
GPU callers get a loud error (``require()``) — there is no silent eager fallback.  CPU
callers (tests, the gloo oracle) never touch it.
"""
from __future__ import annotations

import importlib
import os

_mod = None
_err: Exception | None = None


def _load():
    global _mod, _err
    if _mod is not None or _err is not None:
        return
    import torch  # noqa: F401  (loads torch's vendored libamdhip64 / librccl first)

    try:
        _mod = importlib.import_module("distributed_pytorch_amd._C")
    except Exception as e:  # pragma: no cover - depends on build state
        _err = e


def available() -> bool:
    _load()
    return _mod is not None


def require():
    """Return the native module or raise with build instructions."""
    _load()
    if _mod is None:
        so = os.path.join(os.path.dirname(__file__), "_C.so")
        raise RuntimeError(
            f"distributed_pytorch_amd native extension not loadable ({so}): {_err!r}. "
            "Build it with `python -m distributed_pytorch_amd._build` (hipcc, gfx950)."
        )
    return _mod
