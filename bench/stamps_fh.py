#!/usr/bin/env python3
"""Timeline of the single-launch forward + head kernel (mlp_fwd1_head) from s_memrealtime stamps
(100 MHz): per workgroup entry -> GEMM + a1 stores drained -> counter add returned -> (last
arriver only) head done.  Diagnostic: where the launch's time goes.

    python bench/stamps_fh.py [--n 800] [--hidden 100]
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
    assert e.fh_counters is not None, "single-launch forward + head not enabled"
    step = e._hip_step()
    st = torch.cuda.current_stream().cuda_stream
    buf = torch.zeros(4096 * 4, dtype=torch.int64, device="cuda")
    hb = torch.zeros(4096 * 8, dtype=torch.int64, device="cuda")
    res = []
    for rep in range(5):
        for _ in range(20):
            step.run(0, a.n, 1.0 / a.n, 1e-4, 0.0, 1, 0, st, 3)
        torch.cuda.synchronize()
        buf.zero_()
        hb.zero_()
        step.stamps = buf.data_ptr()
        step.hstamps = hb.data_ptr()
        step.run(0, a.n, 1.0 / a.n, 1e-4, 0.0, 1, 0, st, 1)
        step.stamps = 0
        step.hstamps = 0
        torch.cuda.synchronize()
        s = buf.view(-1, 4).cpu().numpy().astype(np.int64)
        s = s[s[:, 0] > 0]
        t0 = s[:, 0].min()
        rel = (s - t0) * 10.0 / 1000.0  # us
        last = s[:, 3] > 0
        pct = lambda v: [round(float(np.percentile(v, q)), 3) for q in (0, 50, 90, 100)]  # noqa: E731
        hs = hb.view(-1, 8).cpu().numpy().astype(np.int64)
        hs = hs[hs[:, 0] > 0]
        hd = (hs[:, 1:4] - hs[:, 0:1]) * 10.0 / 1000.0
        hs0 = (hs[:, 0] - t0) * 10.0 / 1000.0 if len(hs) else hs[:, 0]
        res.append({
            "head_loads_drained_at": pct(hs0) if len(hs) else None,
            "head_after_loads_us(softmax,barrier,pass2+stores)": ([round(float(np.median(hd[:, i])), 3)
                                                                  for i in range(3)] if len(hd) else None),
            "wgs": int(len(s)), "last": int(last.sum()),
            "entry": pct(rel[:, 0]),
            "gemm_done": pct(rel[:, 1]),
            "gemm_dur": pct(rel[:, 1] - rel[:, 0]),
            "atomic_dur": pct(rel[:, 2] - rel[:, 1]),
            "head_start": pct(rel[last, 2]),
            "head_dur": pct(rel[last, 3] - rel[last, 2]),
            "end": pct(rel[last, 3]),
        })
    for r in res:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
