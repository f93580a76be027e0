#!/usr/bin/env python3
"""Timeline of the wide fused forward + head launch (mlp_fwd1_wide_ag) from s_memrealtime stamps (100 MHz,
thread 0 of every workgroup; csrc/mlp/mlp_split.hip ag_stamp): entry -> K loop done -> z2 granules stored ->
hand-off 1 (reducers: the tm partials arrived) -> D stored -> D arrived -> end.  Percentiles over workgroups
(min / median / p90 / max, us from the first entry), plus the same per column tile.  Diagnostic.

    python bench/stamps_wide_ag.py [--hidden 4096] [--n 800] [--dtype f32]
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

NAMES = ("entry", "kloop", "z2_stored", "handoff1", "d_stored", "d_arrived", "end")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--n", type=int, default=800)
    ap.add_argument("--dtype", default="f32")
    a = ap.parse_args(argv)
    import numpy as np
    import torch

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import MlpEngine
    from cme213_sp18_amd.utils.data import synthetic_mnist

    x, y = synthetic_mnist(4 * a.n, seed=0)
    nn = NeuralNetwork([784, a.hidden, 10])
    e = MlpEngine(nn.H, dtype=a.dtype, max_cols=a.n, device="cuda")
    e.set_params(*nn.params)
    e.load_dataset(x, y)
    e.set_store_a1(False)
    step = e._hip_step()
    st = torch.cuda.current_stream().cuda_stream
    buf = torch.zeros(8192 * 8, dtype=torch.int64, device="cuda")
    pct = lambda v: [round(float(np.percentile(v, q)), 3) for q in (0, 50, 90, 100)]  # noqa: E731
    for rep in range(4):
        for _ in range(20):
            step.run(0, a.n, 1.0 / a.n, 1e-4, 0.0, 1, 0, st, 3)
        torch.cuda.synchronize()
        buf.zero_()
        step.stamps = buf.data_ptr()
        step.run(0, a.n, 1.0 / a.n, 1e-4, 0.0, 1, 0, st, 1)
        step.stamps = 0
        torch.cuda.synchronize()
        s = buf.view(-1, 8).cpu().numpy().astype(np.int64)
        live = s[:, 0] > 0
        s = s[live]
        t0 = s[:, 0].min()
        rel = np.where(s > 0, (s - t0) * 10.0 / 1000.0, np.nan)
        rec = {"H": a.hidden, "n": a.n, "dtype": a.dtype, "wgs": int(len(s)), "kernel_error": bool(e.kernel_error())}
        for i, nm in enumerate(NAMES):
            col = rel[:, i]
            col = col[~np.isnan(col)]
            if len(col):
                rec[nm] = pct(col)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
