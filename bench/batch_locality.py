#!/usr/bin/env python3
"""What a new batch per step costs the headline step: the native step loop (MlpStep.run_steps) over K steps
that walk the resident dataset (bench.py's form) against K steps that re-read ONE batch (N_end = one batch:
the loop wraps to offset 0 every step, so the batch's X / XT bytes are cache-hot from the previous step).

    python bench/batch_locality.py [--k 400] [--trials 5] [--mode walk|same|both]

One JSON line per form: best-of-trials us/step.  Under rocprofv3 --kernel-trace --stats use --mode walk or
--mode same so the kernel statistics belong to one form.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=400)
    ap.add_argument("--trials", type=int, default=5)
    ap.add_argument("--mode", default="both", choices=["walk", "same", "both"])
    ap.add_argument("--hidden", type=int, default=100)
    a = ap.parse_args(argv)
    import torch

    from cme213_sp18_amd.models.mlp import NeuralNetwork
    from cme213_sp18_amd.parallel.trainer import DataParallelTrainer
    from cme213_sp18_amd.utils.data import synthetic_mnist

    x, y = synthetic_mnist(54000, seed=0)
    tr = DataParallelTrainer(NeuralNetwork([784, a.hidden, 10]), batch_size=800)
    tr.load(x, y)
    e = tr.engine
    s = e._hip_step()
    st = torch.cuda.current_stream().cuda_stream
    n, lr, reg = 800, 1e-3, 1e-4
    forms = {"walk": e.num_samples, "same": n}
    for name in (["walk", "same"] if a.mode == "both" else [a.mode]):
        n_end = forms[name]
        s.run_steps(0, 50, n, 0, n, n_end, 1.0 / n, reg, lr, 1, st)  # warm-up
        best = float("inf")
        for _ in range(a.trials):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            s.run_steps(0, a.k, n, 0, n, n_end, 1.0 / n, reg, lr, 1, st)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        print(json.dumps({"form": name, "hidden": a.hidden, "K": a.k, "us_per_step": round(best * 1e6 / a.k, 3),
                          "finite": bool(torch.isfinite(e.params).all().item())}), flush=True)


if __name__ == "__main__":
    main()
