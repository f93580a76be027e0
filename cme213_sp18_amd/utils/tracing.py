"""Tracing / profiling hooks.

The reference times phases with CUDA events and host clocks only
(fpcode/inc/gpu_func.h:24-40, fpcode/main.cpp:218-250).  Here:

* :class:`Roctx` -- ROCm tracer ranges (``roctxRangePushA`` / ``roctxRangePop``) loaded with ctypes
  from the rocprofiler-sdk roctx library, so ``rocprofv3 --marker-trace -- python -m
  cme213_sp18_amd.train ...`` shows epochs / steps / collectives on the timeline.  Enabled by
  ``CME_ROCTX=1`` or ``--profile``; a no-op when the library is missing (CPU boxes).
* :class:`PhaseTimer` -- stream-ordered event timing per phase (forward+head, weight gradients,
  all-reduce, SGD), aggregated per run; host clocks on CPU.  No host synchronisation until
  :meth:`summary`, so it measures the device time of each phase without serialising the step
  (beyond the eager, graph-free execution that per-phase events need).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from collections import defaultdict

_LIBS = ("librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", "libroctx64.so.4",
         "/opt/rocm/lib/libroctx64.so.4")


class Roctx:
    """roctx range push/pop (ctypes).  ``enabled`` is False when no roctx library loads."""

    def __init__(self, enabled: bool | None = None):
        if enabled is None:
            enabled = os.environ.get("CME_ROCTX") == "1"
        self._lib = None
        if enabled:
            for name in _LIBS:
                try:
                    lib = ctypes.CDLL(name)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.restype = ctypes.c_int
                    lib.roctxRangePop.restype = ctypes.c_int
                    self._lib = lib
                    break
                except OSError:
                    continue

    @property
    def enabled(self) -> bool:
        return self._lib is not None

    def push(self, name: str) -> None:
        if self._lib is not None:
            self._lib.roctxRangePushA(name.encode())

    def pop(self) -> None:
        if self._lib is not None:
            self._lib.roctxRangePop()

    @contextlib.contextmanager
    def range(self, name: str):
        self.push(name)
        try:
            yield
        finally:
            self.pop()


_NULL = Roctx(enabled=False)


class PhaseTimer:
    """Per-phase device time: ``with timer.phase("wgrad"): ...`` records an event pair on the
    current stream (GPU) or host clocks (CPU); :meth:`summary` syncs once and reports mean / total
    milliseconds per phase.  ``roctx``: an optional :class:`Roctx` that also brackets each phase."""

    def __init__(self, device=None, roctx: Roctx | None = None):
        import torch

        self.device = device
        self.gpu = device is not None and torch.device(device).type == "cuda"
        self.roctx = roctx or _NULL
        self._ev: dict[str, list] = defaultdict(list)
        self._host: dict[str, list[float]] = defaultdict(list)

    @contextlib.contextmanager
    def phase(self, name: str):
        import torch

        self.roctx.push(name)
        if self.gpu:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            try:
                yield
            finally:
                e.record()
                self._ev[name].append((s, e))
                self.roctx.pop()
        else:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self._host[name].append((time.perf_counter() - t0) * 1e3)
                self.roctx.pop()

    def summary(self) -> dict[str, dict[str, float]]:
        import torch

        out = {}
        if self.gpu:
            torch.cuda.synchronize(self.device)
            for k, evs in self._ev.items():
                ms = [s.elapsed_time(e) for s, e in evs]
                out[k] = {"count": len(ms), "mean_ms": sum(ms) / len(ms), "total_ms": sum(ms)}
        for k, ms in self._host.items():
            out[k] = {"count": len(ms), "mean_ms": sum(ms) / len(ms), "total_ms": sum(ms)}
        return out

    def reset(self) -> None:
        self._ev.clear()
        self._host.clear()

    def format(self) -> str:
        s = self.summary()
        tot = sum(v["mean_ms"] for v in s.values()) or 1.0
        return "  ".join(f"{k}={v['mean_ms'] * 1e3:.1f}us({100 * v['mean_ms'] / tot:.0f}%)" for k, v in s.items())
