"""Loader for the native extension ``beforeholiday_amd._C`` (HIP kernels for gfx950).

Policy (so a GPU run can never silently fall back to eager PyTorch):

* GPU tensors always go through the native kernels; if the extension is missing that is a hard
  error (``require_native``), never a fallback.
* CPU tensors use the pure-PyTorch reference implementations in ``beforeholiday_amd.ops._ref``
  (that is the "python-only build" the reference also supports, and the oracle the GPU tests
  compare the kernels against).
"""
from __future__ import annotations

import importlib
import os

_C = None
_err: Exception | None = None
_tried = False


def native():
    """Return the ``_C`` module or ``None`` if it is not built/importable."""
    global _C, _err, _tried
    if not _tried:
        _tried = True
        try:
            _C = importlib.import_module("beforeholiday_amd._C")
            _register_exit_cleanup(_C)
        except Exception as e:  # pragma: no cover - depends on the build
            _err = e
            _C = None
            if os.environ.get("BH_AUTOBUILD", "0") == "1":
                from . import _build

                _build.build()
                _C = importlib.import_module("beforeholiday_amd._C")
                _err = None
        if _C is not None:  # the native run-time switches come from the typed config (config.py)
            from . import config

            config.push_native(_C)
    return _C


def loaded() -> bool:
    """Whether the extension has been imported already (without importing it)."""
    return _C is not None


def module():
    return native()


def _register_exit_cleanup(mod):
    """Release the multi-tensor plan cache (device + pinned tensors) at interpreter exit while
    PyTorch's allocators are still alive (the C++ cache itself is never destroyed)."""
    import atexit

    fn = getattr(getattr(mod, "amp_C", None), "clear_plan_cache", None)
    if fn is not None:
        atexit.register(fn)


def available() -> bool:
    return native() is not None


def require_native(what: str = "this op"):
    mod = native()
    if mod is None:
        raise RuntimeError(
            f"beforeholiday_amd: {what} needs the native HIP extension (beforeholiday_amd._C) for GPU "
            f"tensors, but it failed to import: {_err!r}. Build it with "
            f"`python -m beforeholiday_amd._build`."
        )
    return mod


def submodule(name: str):
    return getattr(require_native(name), name)


def import_error():
    native()
    return _err
