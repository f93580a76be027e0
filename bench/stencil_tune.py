#!/usr/bin/env python3
"""The LDS stencil's knobs at order 8 on an HBM-sized grid (csrc/suite/stencil.hip stencil_lds_tune): rows per wave,
rows loaded ahead, non-temporal streamed loads.  Interior sweeps only, ping-ponged; every form's result after the
sweeps is compared BITWISE with the production LDS variant's (same arithmetic, so any difference is a bug).  GB/s of
compulsory bytes (read the grid, write the interior once per sweep).

    python bench/stencil_tune.py [--n 12288] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=12288)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--forms", default="all", choices=["all", "stores", "two_step"])
    a = ap.parse_args(argv)
    import torch

    from cme213_sp18_amd._native import hip

    k = hip().suite
    g = a.n
    torch.manual_seed(0)
    init = torch.rand(g * g, dtype=torch.float32, device="cuda")
    A, Bf = torch.empty_like(init), torch.empty_like(init)
    st = torch.cuda.current_stream().cuda_stream
    xcfl = ycfl = 0.0001

    def run(fn):
        A.copy_(init)
        Bf.copy_(init)
        src, dst = A, Bf
        for _ in range(a.iters):
            fn(dst, src)
            src, dst = dst, src
        return src

    def timeit(fn):
        run(fn)
        best = float("inf")
        for _ in range(a.reps):
            A.copy_(init)
            Bf.copy_(init)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            src, dst = A, Bf
            for _ in range(a.iters):
                fn(dst, src)
                src, dst = dst, src
            e1.record()
            e1.synchronize()
            best = min(best, e0.elapsed_time(e1))
        return best

    nx = g - 8
    comp = a.iters * (g * g + nx * nx) * 4  # read the grid, write the interior
    if a.forms == "two_step":
        # the temporal-blocked walk (two time steps per sweep, stencil_step2_bc) against two one-step LDS launches,
        # both with the boundary condition; --iters counts time steps (even)
        scale = 0.999
        steps = a.iters // 2
        one = lambda d, s: k.stencil_step_bc(d.data_ptr(), s.data_ptr(), g, g, 8, xcfl, ycfl, 2, scale, st)  # noqa: E731
        it0 = a.iters
        ref = run(one).clone()
        ms = timeit(one)
        print(json.dumps({"form": "one-step lds + bc, per time step", "ms": round(ms, 3),
                          "compulsory_GBps": round(comp / (ms * 1e-3) / 1e9, 1)}), flush=True)
        a.iters = steps
        for rows, ahead in ((64, 4), (64, 2), (32, 4), (96, 4), (128, 4), (128, 2), (32, 2), (64, 3), (64, 1), (96, 2),
                            (64, 2), (32, 2), (64, 4)):
            fn = lambda d, s, r=rows, h=ahead: k.stencil_step2_bc(d.data_ptr(), s.data_ptr(), g, g, 8, xcfl, ycfl,  # noqa: E731
                                                                  scale, st, r, h)
            out = run(fn)
            same = bool(torch.equal(out, ref))
            ms = timeit(fn)
            print(json.dumps({"two_step_rows": rows, "ahead": ahead, "time_steps": it0, "ms": round(ms, 3),
                              "bitwise_equal": same, "compulsory_GBps": round(comp / (ms * 1e-3) / 1e9, 1)}),
                  flush=True)
        return
    prod = lambda d, s: k.stencil_step(d.data_ptr(), s.data_ptr(), g, g, 8, xcfl, ycfl, 2, st)  # noqa: E731
    ref = run(prod).clone()
    ms = timeit(prod)
    print(json.dumps({"form": "production lds (32 rows, 4 ahead)", "ms": round(ms, 3),
                      "compulsory_GBps": round(comp / (ms * 1e-3) / 1e9, 1)}), flush=True)
    # nt: bit 0 non-temporal streamed loads, bit 1 the alternate-direction walk (ALT), bit 2 plain stores
    forms = ((32, 4, 0), (32, 8, 0), (32, 8, 1), (64, 8, 0), (32, 4, 2), (32, 8, 2), (64, 8, 2), (16, 8, 2))
    if a.forms == "stores":
        forms = ((32, 4, 2), (32, 4, 6), (32, 6, 2), (32, 6, 6), (64, 4, 6), (16, 4, 2), (32, 4, 2), (32, 4, 6))
    for rows, ahead, nt in forms:
        fn = lambda d, s, r=rows, h=ahead, t=nt: k.stencil_lds_tune(d.data_ptr(), s.data_ptr(), g, g, xcfl, ycfl,  # noqa: E731
                                                                    r, h, t, st)
        out = run(fn)
        same = bool(torch.equal(out, ref))
        ms = timeit(fn)
        print(json.dumps({"rows": rows, "ahead": ahead, "nt": nt, "ms": round(ms, 3), "bitwise_equal": same,
                          "compulsory_GBps": round(comp / (ms * 1e-3) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
