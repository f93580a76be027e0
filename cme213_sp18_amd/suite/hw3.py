"""hw3: 2-D heat diffusion stencil (orders 2/4/8) on gfx950.

Reference capabilities:
  * simParams: params.in parsing, dx/dy/dt/CFL, calcBytes   hw3code/simParams.cpp:7-93
  * Grid: host + device buffers, swap, text dump           hw3code/Grid.h, Grid.cu:14-101
  * boundary conditions curr = prev * exp(-2 dt)            hw3code/BC.h:7-73
  * global / "block" (loop) / shared stencil kernels        hw3code/gpuStencil.cu:15-308
  * CPU reference, initGrid sin*sin, ULP-512 checker        hw3code/main.cu:74-293
  * CLI -g/-b/-s with time and GB/s                         hw3code/main.cu:295-412

The reference's shared-memory variant was an empty kernel (gpuStencil.cu:263-268);
here "shared" is a real LDS-tiled halo stencil.  The boundary convention is the
GPU driver's (next.border = curr.border * exp(-2 dt), then next.interior from
curr); the reference's CPU loop applied it one step out of phase
(main.cu:184 writes curr.border from next), so our CPU oracle follows the GPU
semantics and the two agree to a few ULP.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

from ..utils.common import ulp_distance
from ._dev import EventTimer, host, kernels, require_cuda, stream_handle

VARIANTS = {"global": 0, "block": 1, "shared": 2, "vec": 3, "shared2": 4}  # shared2: LDS walk, 2 steps per sweep
MAX_ULPS = 512  # main.cu:229


@dataclass
class SimParams:
    nx: int
    ny: int
    lx: float
    ly: float
    iters: int
    order: int

    def __post_init__(self):
        if self.nx <= 0 or self.ny <= 0 or self.lx <= 0 or self.ly <= 0 or self.iters < 0:
            raise ValueError("SimParams: sizes must be positive")
        if self.order not in (2, 4, 8):
            raise ValueError("SimParams: order must be 2, 4 or 8")

    @classmethod
    def from_file(cls, path: str) -> "SimParams":
        """``nx ny / lx ly / iters / order`` (hw3code/params.in)."""
        tok = open(path).read().split()
        if len(tok) < 6:
            raise ValueError(f"{path}: expected 'nx ny lx ly iters order'")
        return cls(int(tok[0]), int(tok[1]), float(tok[2]), float(tok[3]), int(tok[4]), int(tok[5]))

    @property
    def border(self) -> int:
        return self.order // 2

    @property
    def gx(self) -> int:
        return self.nx + 2 * self.border

    @property
    def gy(self) -> int:
        return self.ny + 2 * self.border

    # double-precision parameters, as simParams stores them (simParams.h:55-63)
    @property
    def dx(self) -> float:
        return self.lx / (self.gx - 1)

    @property
    def dy(self) -> float:
        return self.ly / (self.gy - 1)

    def _dt_cfl(self):
        dx2, dy2 = self.dx * self.dx, self.dy * self.dy
        k = {2: (1, 1), 4: (12, 16), 8: (5040, 8064)}[self.order]  # simParams.cpp:53-77
        dt = (0.5 - 0.01) * (k[0] * dx2 * dy2) / (k[1] * (dx2 + dy2))
        return dt, dt / (k[0] * dx2), dt / (k[0] * dy2)

    @property
    def dt(self) -> float:
        return self._dt_cfl()[0]

    @property
    def xcfl(self) -> float:
        return self._dt_cfl()[1]

    @property
    def ycfl(self) -> float:
        return self._dt_cfl()[2]

    @property
    def bc_scale(self) -> float:
        return math.exp(-2 * self.dt)  # narrowed to float at the kernel call, as BC.h:67

    def calc_bytes(self) -> int:
        """Stencil traffic model: iters * nx * ny * {6,10,18} words (simParams.cpp:79-93).  It counts every
        stencil tap as a memory read, so it exceeds what any kernel that reuses neighbours moves."""
        return self.iters * self.nx * self.ny * {2: 6, 4: 10, 8: 18}[self.order] * 4

    def compulsory_bytes(self) -> int:
        """The bytes an ideal kernel moves: per iteration the whole current grid (halo included) read once and
        the next grid's interior written once."""
        return self.iters * (self.gx * self.gy + self.nx * self.ny) * 4


def init_grid(p: SimParams) -> np.ndarray:
    """sin(i dx) sin(j dy) on the full grid, [gy][gx] row-major (main.cu:116-130)."""
    i = np.arange(p.gx, dtype=np.float64)
    j = np.arange(p.gy, dtype=np.float64)
    return (np.sin(j * p.dy)[:, None] * np.sin(i * p.dx)[None, :]).astype(np.float32)


def cpu_computation(grid: np.ndarray, p: SimParams) -> np.ndarray:
    """CPU oracle (OpenMP, native): ``iters`` BC + stencil updates."""
    return host().stencil(np.ascontiguousarray(grid, np.float32), p.order, p.xcfl, p.ycfl, p.bc_scale, p.iters)


class Grid:
    """Device ping-pong pair for the stencil (Grid.h/Grid.cu: host+device, swap)."""

    def __init__(self, host_grid: np.ndarray, device="cuda"):
        self.curr = torch.from_numpy(np.ascontiguousarray(host_grid, np.float32)).to(device)
        self.next = self.curr.clone()

    def swap(self):
        self.curr, self.next = self.next, self.curr

    def to_host(self) -> np.ndarray:
        return self.curr.cpu().numpy()

    def save_text(self, path: str) -> None:
        """Text dump of the current grid (Grid.cu:85-101: one row per line)."""
        np.savetxt(path, self.to_host(), fmt="%.8g")


def gpu_step(grid: Grid, p: SimParams, variant: int, fused: bool = True) -> None:
    """One time step: BC on the border + stencil on the interior -- one fused launch (default), or the
    reference's two launches (BC kernel then stencil kernel, gpuStencil.cu:113-131)."""
    k = kernels()
    s = stream_handle()
    if fused:
        k.stencil_step_bc(grid.next.data_ptr(), grid.curr.data_ptr(), p.gx, p.gy, p.order, p.xcfl, p.ycfl, variant,
                          p.bc_scale, s)
    else:
        k.stencil_bc(grid.next.data_ptr(), grid.curr.data_ptr(), p.gx, p.gy, p.border, p.bc_scale, s)
        k.stencil_step(grid.next.data_ptr(), grid.curr.data_ptr(), p.gx, p.gy, p.order, p.xcfl, p.ycfl, variant, s)
    grid.swap()


def gpu_step2(grid: Grid, p: SimParams) -> None:
    """TWO time steps in one sweep (the temporal-blocked LDS walk, order 8): bitwise two ``gpu_step`` calls."""
    kernels().stencil_step2_bc(grid.next.data_ptr(), grid.curr.data_ptr(), p.gx, p.gy, p.order, p.xcfl, p.ycfl,
                               p.bc_scale, stream_handle())
    grid.swap()


def gpu_computation(host_grid: np.ndarray, p: SimParams, variant: str | int = "shared",
                    fused: bool = True) -> tuple[np.ndarray, float]:
    """Run ``iters`` steps on the GPU; returns (final grid, milliseconds).  ``shared2`` (order 8): pairs of steps
    per sweep, an odd last step by the one-step LDS walk."""
    v = VARIANTS[variant] if isinstance(variant, str) else int(variant)
    if v == 4 and p.order != 8:
        v = VARIANTS["shared"]
    g = Grid(host_grid)
    require_cuda(g.curr)
    with EventTimer() as t:
        if v == 4:
            for _ in range(p.iters // 2):
                gpu_step2(g, p)
            if p.iters % 2:
                gpu_step(g, p, VARIANTS["shared"], fused)
        else:
            for _ in range(p.iters):
                gpu_step(g, p, v, fused)
    return g.to_host(), t.ms


def check_errors(ref: np.ndarray, out: np.ndarray, max_ulps: int = MAX_ULPS) -> dict:
    """Mismatch count (> max_ulps ULP), L2 of the reference, relative L-inf and L2 error (main.cu:217-266)."""
    ref = np.asarray(ref, np.float32)
    out = np.asarray(out, np.float32)
    mism = int(np.count_nonzero(ulp_distance(ref, out) > max_ulps))
    r64, o64 = ref.astype(np.float64), out.astype(np.float64)
    l2ref = float(np.sum(r64 * r64))
    nz = r64 != 0
    linf = float(np.max(np.abs((r64[nz] - o64[nz]) / r64[nz]))) if nz.any() else 0.0
    l2err = float(np.sum((r64 - o64) ** 2))
    return {"mismatches": mism, "l2ref": l2ref, "linf": linf, "l2err": math.sqrt(l2err / l2ref) if l2ref else 0.0}
