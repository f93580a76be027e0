#!/usr/bin/env python3
"""Timeline of the wide head (head_wide_kernel: z2 partial sums -> softmax -> dZ1 + dW2 partials) from its
s_memrealtime stamps (100 MHz): per workgroup entry -> operand burst landed (z2 summed) -> softmax / D done
-> last store drained (wave 0 of the block).  One full step first, then the head alone is stamped.  Diagnostic.

    python bench/stamps_hw.py [--hidden 4096] [--n 800] [--dtype f32]
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
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--n", type=int, default=800)
    ap.add_argument("--dtype", default="f32")
    a = ap.parse_args(argv)
    import numpy as np
    import torch

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import MlpEngine
    from cme213_sp18_amd.utils.data import synthetic_mnist

    x, y = synthetic_mnist(4000, seed=0)
    nn = NeuralNetwork([784, a.hidden, 10])
    e = MlpEngine(nn.H, dtype=a.dtype, max_cols=a.n, device="cuda")
    e.set_params(*nn.params)
    e.load_dataset(x, y)
    step = e._hip_step()
    st = torch.cuda.current_stream().cuda_stream
    buf = torch.zeros(8192 * 8, dtype=torch.int64, device="cuda")
    pct = lambda v: [round(float(np.percentile(v, q)), 3) for q in (0, 50, 90, 100)]  # noqa: E731
    for rep in range(4):
        for _ in range(10):
            step.run(0, a.n, 1.0 / a.n, 1e-4, 0.0, 1, 0, st, 3)
        torch.cuda.synchronize()
        buf.zero_()
        step.hstamps = buf.data_ptr()
        step.run(0, a.n, 1.0 / a.n, 1e-4, 0.0, 1, 0, st, 1)  # forward + head
        step.hstamps = 0
        torch.cuda.synchronize()
        s = buf.view(-1, 8)[:, :4].cpu().numpy().astype(np.int64)
        s = s[s[:, 0] > 0]
        t0 = s[:, 0].min()
        rel = (s - t0) * 10.0 / 1000.0
        done = rel[:, 3][s[:, 3] > 0]
        print(json.dumps({"wgs": int(len(s)), "entry": pct(rel[:, 0]), "burst_landed": pct(rel[:, 1]),
                          "softmax_done": pct(rel[:, 2]), "drained": pct(done) if len(done) else None,
                          "burst": pct(rel[:, 1] - rel[:, 0])}), flush=True)


if __name__ == "__main__":
    main()
