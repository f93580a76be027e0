#!/usr/bin/env python3
"""Timeline of the small-layer weight-gradient launch (wgrad_split_kernel, dW1 tiles) from the wave-split-K
engine's s_memrealtime stamps (mma_tile.h: per wave entry, K loop done, reduction barrier, end; 100 MHz),
with the GEMM reading fp32 dZ1 (split in registers) or the stored bf16 planes.  Diagnostic.

    python bench/stamps_wgrad.py [--n 800] [--hidden 100]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the two-launch kernels' stamps exist only in the diagnostics library (_hip_diag: `python -m cme213_sp18_amd._build
# --diag`, built on first use)
os.environ.setdefault("CME_DIAG", "1")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=800)
    ap.add_argument("--hidden", type=int, default=100)
    a = ap.parse_args(argv)
    import numpy as np
    import torch

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import MlpEngine
    from cme213_sp18_amd.utils.data import synthetic_mnist

    x, y = synthetic_mnist(4000, seed=0)
    nn = NeuralNetwork([784, a.hidden, 10])
    pct = lambda v: [round(float(np.percentile(v, q)), 3) for q in (0, 50, 90, 100)]  # noqa: E731
    def xcd_remap(orig, nwg):  # csrc/common/hip_common.h
        if nwg <= 8:
            return orig
        q, r, x = nwg // 8, nwg % 8, orig % 8
        return (x * (q + 1) if x < r else r * (q + 1) + (x - r) * q) + orig // 8

    t1n = (785 + 31) // 32
    t1 = ((a.hidden + 15) // 16) * t1n
    for a32 in (1, 1):  # (two identical runs: the spread between them is the noise)
        e = MlpEngine(nn.H, dtype="f32", max_cols=a.n, device="cuda", path="split3")
        e.set_params(*nn.params)
        e.load_dataset(x, y)
        step = e._hip_step()
        st = torch.cuda.current_stream().cuda_stream
        buf = torch.zeros(4096 * 8 * 4, dtype=torch.int64, device="cuda")
        for _ in range(20):
            step.run(0, a.n, 1.0 / a.n, 1e-4, 0.0, 1, 0, st, 3)
        torch.cuda.synchronize()
        step.stamps = buf.data_ptr()
        step.run_wgrad(0, a.n, 1.0 / a.n, 1e-4, 0.0, 1, 1, 0, -1, st)
        step.stamps = 0
        torch.cuda.synchronize()
        s = buf.view(-1, 4).cpu().numpy().astype(np.int64)
        s = s[s[:, 0] > 0]
        t0 = s[:, 0].min()
        rel = (s - t0) * 10.0 / 1000.0
        print(json.dumps({"run": a32, "waves": int(len(s)), "entry": pct(rel[:, 0]), "kloop_done": pct(rel[:, 1]),
                          "kloop": pct(rel[:, 1] - rel[:, 0]), "reduced": pct(rel[:, 2]), "end": pct(rel[:, 3])}))
        # per workgroup (wave 0): which dW1 tiles end last -- (row tile, column tile, XCD, end us)
        raw = buf.view(-1, 8, 4)[:t1].cpu().numpy().astype(np.int64)
        ends = [((raw[b, :, 3].max() - t0) * 10.0 / 1000.0, b) for b in range(t1) if raw[b, 0, 0] > 0]
        ends.sort(reverse=True)
        slow = [{"row_tile": xcd_remap(b, t1) // t1n, "col_tile": xcd_remap(b, t1) % t1n, "xcd": b % 8,
                 "end_us": round(float(t_), 2)} for t_, b in ends[:12]]
        cols = {}
        for t_, b in ends:
            cols.setdefault(xcd_remap(b, t1) % t1n, []).append(float(t_))
        print(json.dumps({"slowest": slow, "median_end_by_col_tile": {k: round(float(np.median(v)), 2)
                                                                     for k, v in sorted(cols.items())}}), flush=True)


if __name__ == "__main__":
    main()
