"""Loader for the in-tree native extension (``_C.so``).

The HIP kernels are the compute path on GPU: if the extension is missing or fails to load,
GPU callers get a loud error (``require()``) — there is no silent eager fallback.  CPU
callers (tests, the gloo oracle) never touch it.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys

_mod = None
_err: Exception | None = None


def _load():
    global _mod, _err
    if _mod is not None or _err is not None:
        return
    import torch  # noqa: F401  (loads torch's vendored libamdhip64 / librccl first)

    try:
        alt = os.environ.get("DPA_EXT_SO")  # an A/B build of the same sources (_build.py)
        if alt:
            spec = importlib.util.spec_from_file_location("distributed_pytorch_amd._C", alt)
            _mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(_mod)
            sys.modules["distributed_pytorch_amd._C"] = _mod
        else:
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
