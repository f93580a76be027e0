#!/usr/bin/env python3
"""Why the wide configs run slower for their first few hundred steps (profiles/r5/wide_warmup/README.md): the native
step loop in blocks of --block steps, each block event-timed and followed by a shader-clock probe
(bench/micro/clockprobe.hip: s_memtime cycles over s_memrealtime), under four conditions, each in a FRESH engine:

  walk        consecutive batches over the whole dataset (what bench.py times)
  same        the same batch every step (N_end = n: no new pixels, no new pages)
  pretouch    walk, after one pass that reads the whole dataset (every page of X / XT / their bf16 copies touched
              once, by torch reductions, before the first step)
  walk_again  walk, in a second engine created after the first ran (a warm process, new buffers)
  reset       walk, then the SAME engine (same buffers) set back to the initial weights and walked again: a ramp that
              comes back follows the weights' values (data-dependent power), one that does not follows the buffers

If the slow start follows new pages (first touch of the dataset's pages / TLB), `same` and `pretouch` start fast; if it
follows the shader clock, the probe shows it; if neither, it is something in the engine's own state.

    python bench/wide_warmup.py --hidden 4096 --dtype f32 --blocks 24 --block 25
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--n", type=int, default=800)
    ap.add_argument("--blocks", type=int, default=24)
    ap.add_argument("--block", type=int, default=25)
    ap.add_argument("--modes", nargs="*", default=["walk", "same", "pretouch", "walk_again"])
    ap.add_argument("--probe-during", action="store_true",
                    help="also probe the shader clock DURING each block (one 64-thread workgroup on a side stream)")
    ap.add_argument("--prewarm-ms", type=float, default=0.0,
                    help="before each mode's first block: this long of a memory-bound load (1 GiB copies) and, "
                         "separately reported, of the step itself -- does a sustained load, not the step, lift it")
    a = ap.parse_args(argv)
    import torch

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import MlpEngine
    from cme213_sp18_amd.utils.data import synthetic_mnist

    lib = ctypes.CDLL(os.path.join(ROOT, "bench", "micro", "libclockprobe.so"))
    probe_buf = torch.zeros(2 * 256, dtype=torch.int64, device="cuda")

    def sclk_mhz():
        torch.cuda.synchronize()
        rc = lib.clock_probe(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream),
                             ctypes.c_void_p(probe_buf.data_ptr()), 256, 20)
        assert rc == 0
        torch.cuda.synchronize()
        v = probe_buf.view(256, 2).double()
        return round(float((100.0 * v[:, 0] / v[:, 1]).median()), 1)

    side = torch.cuda.Stream()
    during_buf = torch.zeros(2, dtype=torch.int64, device="cuda")

    def probe_during_start(us):
        rc = lib.clock_probe(ctypes.c_void_p(side.cuda_stream), ctypes.c_void_p(during_buf.data_ptr()), 1, int(us))
        assert rc == 0

    def probe_during_read():
        side.synchronize()
        v = during_buf.double()
        return round(float(100.0 * v[0] / v[1]), 1)

    x, y = synthetic_mnist(54000, seed=0)
    n = a.n
    for mode in a.modes:
        nn = NeuralNetwork([784, a.hidden, 10])
        e = MlpEngine(nn.H, dtype=a.dtype, max_cols=n, device="cuda")
        e.set_params(*nn.params)
        e.load_dataset(x, y)
        e.set_store_a1(False)
        if mode == "walk_again":  # a second engine in the same (warm) process: new buffers, new pages
            e2 = MlpEngine(nn.H, dtype=a.dtype, max_cols=n, device="cuda")
            e2.set_params(*nn.params)
            e2.load_dataset(x, y)
            e2.set_store_a1(False)
            e = e2
        st = e._hip_step()
        N = e.num_samples
        n_end = n if mode == "same" else N
        if mode == "pretouch":
            with torch.no_grad():
                tot = 0.0
                for t in (e.X, e.XT, e.Xw, e.XTw, e.Xs):
                    if t is not None:
                        tot += float(t.view(-1)[:: 64].float().sum().item()) + float(t.float().sum().item())
        stream = torch.cuda.current_stream().cuda_stream
        if a.prewarm_ms > 0:  # a sustained HBM load first (fabric / memory clocks ramp with load, not with time)
            import time as _time

            src = torch.empty(1 << 28, dtype=torch.float32, device="cuda")
            dst = torch.empty_like(src)
            t_end = _time.perf_counter() + a.prewarm_ms * 1e-3
            while _time.perf_counter() < t_end:
                dst.copy_(src)
                torch.cuda.synchronize()
            del src, dst
        def walk_blocks():
            blocks, g0 = [], 0
            for b in range(a.blocks):
                s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                if a.probe_during:
                    probe_during_start(a.block * 40)
                s0.record()
                st.run_steps(g0 % (N - N % n) if n_end == N else 0, a.block, n, 0, n, n_end, 1.0 / n, 1e-4, 1e-3, 1,
                             stream)
                s1.record()
                s1.synchronize()
                g0 += a.block * n
                r = {"us_per_step": round(s0.elapsed_time(s1) * 1e3 / a.block, 2)}
                if a.probe_during:
                    r["sclk_during_mhz"] = probe_during_read()
                r["sclk_mhz"] = sclk_mhz()
                blocks.append(r)
            return blocks

        passes = [walk_blocks()]
        if mode == "reset":  # the same engine and buffers, back to the initial weights
            e.set_params(*nn.params)
            passes.append(walk_blocks())
        for k, blocks in enumerate(passes):
            print(json.dumps({"H": a.hidden, "dtype": a.dtype, "n": n, "mode": mode, "pass": k, "block_steps": a.block,
                              "prewarm_ms": a.prewarm_ms,
                              "us_per_step": [r["us_per_step"] for r in blocks],
                              "sclk_mhz": [r["sclk_mhz"] for r in blocks],
                              **({"sclk_during_mhz": [r["sclk_during_mhz"] for r in blocks]} if a.probe_during else {}),
                              "planes_stale": bool(st.planes_stale), "kernel_error": bool(e.kernel_error())}),
                  flush=True)
        del e


if __name__ == "__main__":
    main()
