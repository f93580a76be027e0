"""Loaders for the two in-tree native extensions.

``hip()`` returns the gfx950 kernel module and ``cpu()`` the native CPU
runtime.  Both are built in-tree by :mod:`cme213_sp18_amd._build`; if a module
is missing it is built on first use.  There is NO silent eager/PyTorch
fallback for the GPU path: if the HIP extension cannot be loaded, every GPU op
raises.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mods: dict[str, object] = {}


class NativeExtensionError(RuntimeError):
    pass


def _load(name: str):
    with _lock:
        if name in _mods:
            return _mods[name]
        if name == "_hip":
            import torch  # noqa: F401  -- torch's HIP runtime must be loaded first (shared SONAME)
        try:
            mod = importlib.import_module(f"cme213_sp18_amd.{name}")
        except ImportError:
            from . import _build

            try:
                _build.build(verbose=True, diag=name == "_hip_diag")
            except Exception as e:  # pragma: no cover - surfaced to the caller
                raise NativeExtensionError(f"could not build native extension {name}: {e}") from e
            importlib.invalidate_caches()
            try:
                mod = importlib.import_module(f"cme213_sp18_amd.{name}")
            except ImportError as e:
                raise NativeExtensionError(f"native extension {name} failed to load: {e}") from e
        _mods[name] = mod
        return mod


def hip():
    """The gfx950 kernel module (``cme213_sp18_amd._hip``; with ``CME_DIAG=1`` the diagnostics build
    ``_hip_diag`` -- the same kernels with the two-launch kernels' timing stamps compiled in)."""
    return _load("_hip_diag" if os.environ.get("CME_DIAG") == "1" else "_hip")


def cpu():
    """The native CPU runtime module (``cme213_sp18_amd._cpu``)."""
    return _load("_cpu")


DTYPE_CODES = {"f32": 0, "f64": 1, "bf16": 2}
