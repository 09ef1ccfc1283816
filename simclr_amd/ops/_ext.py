"""Loader for the in-tree HIP extension ``simclr_amd/_C.so`` (built by ``simclr_amd.csrc.build``).

The library is loaded with ``torch.ops.load_library`` (plain dlopen of the in-tree file — never a
site-packages or JIT-cache copy) and registers ``torch.ops.simclr_amd.*``.  On a GPU tensor an op
that needs the library raises if it is missing instead of silently running torch ops.
"""
from __future__ import annotations

import os
import threading
from pathlib import Path

import torch

_LIB = Path(__file__).resolve().parent.parent / "_C.so"
_lock = threading.Lock()
_loaded = False
_error: Exception | None = None


def lib_path() -> Path:
    return _LIB


def load(build_if_missing: bool = False) -> bool:
    global _loaded, _error
    if _loaded:
        return True
    with _lock:
        if _loaded:
            return True
        if not _LIB.exists() and build_if_missing:
            from ..csrc import build as _b
            _b.build()
        if not _LIB.exists():
            _error = FileNotFoundError(
                f"{_LIB} not found; build it with `python -m simclr_amd.csrc.build`")
            return False
        try:
            torch.ops.load_library(str(_LIB))
            _loaded = True
        except Exception as e:  # pragma: no cover - surfaced by require()
            _error = e
            return False
    return True


def available() -> bool:
    return load(build_if_missing=False)


def require() -> None:
    if not load(build_if_missing=os.environ.get("SIMCLR_AUTOBUILD", "1") == "1"):
        raise RuntimeError(f"simclr_amd HIP extension unavailable: {_error}")


class _DebugOps:
    """``SIMCLR_DEBUG=1`` / ``runtime.debug``: every op is followed by a device synchronise, so
    an asynchronous fault or launch error is reported at the op that caused it, and every
    floating-point tensor argument (inputs and outputs alike) is checked for NaN: the first op
    whose arguments hold a NaN is named in the error.  (±Inf is legitimate in some scratch
    buffers, e.g. the -inf "no positive in this column split" of the NT-Xent partials.)"""

    def __init__(self, real):
        self._real = real

    def __getattr__(self, name):
        f = getattr(self._real, name)
        if not callable(f):
            return f

        def run(*args, **kw):
            out = f(*args, **kw)
            if torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing():
                torch.cuda.synchronize()
                for i, a in enumerate(list(args) + list(kw.values())):
                    if (isinstance(a, torch.Tensor) and a.is_floating_point() and a.numel()
                            and bool(torch.isnan(a).any())):
                        raise FloatingPointError(
                            f"simclr_amd.{name} [{TAG}]: argument {i} {tuple(a.shape)} "
                            f"{a.dtype} holds NaN")
            return out

        return run


DEBUG = os.environ.get("SIMCLR_DEBUG", "0") == "1"


def set_debug(on: bool) -> None:
    global DEBUG
    DEBUG = bool(on)


def ops():
    require()
    return _DebugOps(torch.ops.simclr_amd) if DEBUG else torch.ops.simclr_amd


# Semantic label of the op being issued (set by the fused executor, read by profilers such as
# tools/layer_profile.py); plain attribute, no cost on the hot path.
TAG = ""
