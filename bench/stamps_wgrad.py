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
    for a32 in (3, 1, 3, 1):
        e = MlpEngine(nn.H, dtype="f32", max_cols=a.n, device="cuda", path="split3")
        e.set_params(*nn.params)
        e.load_dataset(x, y)
        step = e._hip_step()
        step.a_fp32 = a32
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
        print(json.dumps({"a_fp32": a32, "waves": int(len(s)), "entry": pct(rel[:, 0]), "kloop_done": pct(rel[:, 1]),
                          "kloop": pct(rel[:, 1] - rel[:, 0]), "reduced": pct(rel[:, 2]), "end": pct(rel[:, 3])}))


if __name__ == "__main__":
    main()
