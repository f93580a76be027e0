#!/usr/bin/env python3
"""Where does a tile kernel spend its time?  Diagnostic timeline from
per-wave s_memrealtime stamps (100 MHz) recorded by wsk_tile (mma_tile.h):
entry -> K loop done -> reduction barrier passed -> epilogue stored.

    python bench/stamps.py [--n 800] [--hidden 100]
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
    e = MlpEngine(nn.H, dtype="f32", max_cols=a.n, device="cuda", path="split3")
    e.set_params(*nn.params)
    e.load_dataset(x, y)
    step = e._hip_step()
    st = torch.cuda.current_stream().cuda_stream
    buf = torch.zeros(4096 * 8 * 4, dtype=torch.int64, device="cuda")
    out = {}
    for name, part in (("fwd1(+head)", 1), ("wgrad", 2)):
        for _ in range(50):  # warm
            step.run(0, a.n, 1.0 / a.n, 1e-4, 0.0, 1, 0, st, 3)
        torch.cuda.synchronize()
        buf.zero_()
        step.stamps = buf.data_ptr()
        step.run(0, a.n, 1.0 / a.n, 1e-4, 0.0, 1, 0, st, part)
        step.stamps = 0
        torch.cuda.synchronize()
        s = buf.view(-1, 4).cpu().numpy().astype(np.int64)
        s = s[s[:, 0] > 0]
        t0 = s[:, 0].min()
        rel = (s - t0) * 10.0 / 1000.0  # us
        pct = lambda v: [round(float(np.percentile(v, q)), 3) for q in (0, 50, 90, 100)]  # noqa: E731
        out[name] = {
            "waves": int(len(s)),
            "entry_us_p0_50_90_100": pct(rel[:, 0]),
            "kloop_us": pct(rel[:, 1] - rel[:, 0]),
            "reduce_wait_us": pct(rel[:, 2] - rel[:, 1]),
            "epilogue_us": pct(rel[:, 3] - rel[:, 2]),
            "end_us_p0_50_90_100": pct(rel[:, 3]),
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
