"""Small device helpers shared by the homework-suite wrappers."""
from __future__ import annotations

import time

import torch

from .._native import cpu, hip


def kernels():
    """``_hip.suite`` -- raises NativeExtensionError if the extension is missing."""
    return hip().suite


def host():
    """``_cpu.suite`` -- OpenMP algorithms and host oracles."""
    return cpu().suite


def stream_handle(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def require_cuda(*tensors: torch.Tensor) -> None:
    for t in tensors:
        if not t.is_cuda:
            raise ValueError("expected a cuda tensor")
        if not t.is_contiguous():
            raise ValueError("expected a contiguous tensor")


class EventTimer:
    """HIP-event timer (the reference's start_timer/stop_timer, hw2code/common/mp1-util.h:14-40)."""

    def __init__(self):
        self.a = torch.cuda.Event(enable_timing=True)
        self.b = torch.cuda.Event(enable_timing=True)

    def __enter__(self):
        self.a.record()
        return self

    def __exit__(self, *exc):
        self.b.record()
        self.b.synchronize()
        self.ms = self.a.elapsed_time(self.b)
        return False


class WallTimer:
    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        self.ms = (time.perf_counter() - self.t0) * 1e3
        return False
