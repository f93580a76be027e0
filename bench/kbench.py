#!/usr/bin/env python3
"""Per-kernel microbenchmark of the MLP step (graph-replayed, event-timed).

Each measurement captures ``reps`` back-to-back launches of one kernel into a
HIP graph and replays it; time per launch = elapsed / reps, so host launch
overhead is excluded and the number is the on-device cost INCLUDING the
dependent-kernel boundary (what a training step actually pays).

    python bench/kbench.py [--hidden 100] [--cols 800] [--dtype f32]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden", type=int, nargs="*", default=[100])
    ap.add_argument("--cols", type=int, nargs="*", default=[800, 100])
    ap.add_argument("--dtype", nargs="*", default=["f32"])
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    import torch

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd._native import DTYPE_CODES, hip
    from cme213_sp18_amd.parallel import MlpEngine
    from cme213_sp18_amd.utils.data import synthetic_mnist

    m = hip()
    x, y = synthetic_mnist(8000, seed=0)
    results = []

    def timeit(fn, reps):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(5):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            g.replay()
            e.record()
            e.synchronize()
            best = min(best, s.elapsed_time(e) * 1e3 / reps)
        return best

    for dt in a.dtype:
        for H in a.hidden:
            nn = NeuralNetwork([784, H, 10])
            for n in a.cols:
                e = MlpEngine(nn.H, dtype=dt, max_cols=n, device="cuda")
                e.set_params(*nn.params)
                e.load_dataset(x, y)
                code = DTYPE_CODES[dt]
                st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
                step = e._hip_step()

                def fwd():
                    m.mlp_forward1(code, e.W1g.data_ptr(), e.b1.data_ptr(), e.X.data_ptr(), 784, H, n,
                                   e.a1.data_ptr(), e.ld, 1, st())

                def head():
                    m.mlp_head(code, 0, e.a1.data_ptr(), e.ld, e.W2.data_ptr(), e.b2.data_ptr(),
                               labels=e.labels.data_ptr(), H=H, C=10, n=n, scale=1.0 / n, D=e.D.data_ptr(),
                               ldd=e.ld, dZ1=e.dZ1.data_ptr(), ldz=e.ld,
                               dZ1_bf16=e.dZ1g.data_ptr() if dt == "bf16" else 0, stream=st())

                def wgrad(sgd, roles=7, use_xt=True):
                    def f():
                        m.mlp_wgrad(code, e.dZ1g.data_ptr(), e.ld, e.X.data_ptr(), 784, e.dZ1.data_ptr(),
                                    e.D.data_ptr(), e.ld, e.a1.data_ptr(), e.ld, H, 10, n, 1e-4, 0.0, sgd,
                                    e.W1.data_ptr(), e.b1.data_ptr(), e.W2.data_ptr(), e.b2.data_ptr(),
                                    e.gW1.data_ptr(), e.gb1.data_ptr(), e.gW2.data_ptr(), e.gb2.data_ptr(),
                                    e.W1g.data_ptr() if dt == "bf16" else 0,
                                    XT=e.XT.data_ptr() if use_xt else 0, ldxt=e.num_samples, roles=roles,
                                    stream=st())
                    return f

                def sgd():
                    m.sgd_flat(code, e.params.data_ptr(), e.grads.data_ptr(), e.layout.total, 0.0,
                               e.W1g.data_ptr() if dt == "bf16" else 0, H * 784 if dt == "bf16" else 0, st())

                def full_step():
                    step.run(0, n, 1.0 / n, 1e-4, 0.0, 1, 0, st())

                row = {"dtype": dt, "H": H, "n": n}
                for name, fn in (("fwd1", fwd), ("head", head), ("wgrad_sgd", wgrad(1)), ("wgrad_grads", wgrad(0)),
                                 ("wgrad_dW1", wgrad(0, 1)), ("wgrad_dW1_noXT", wgrad(0, 1, False)),
                                 ("wgrad_dW2", wgrad(0, 2)), ("wgrad_bias", wgrad(0, 4)), ("wgrad_none", wgrad(0, 0)),
                                 ("sgd_flat", sgd), ("step_fused", full_step)):
                    row[name + "_us"] = round(timeit(fn, a.reps), 3)
                flops = 2 * n * (784 * H * 2 + 10 * H * 3)
                row["step_tflops"] = round(flops / (row["step_fused_us"] * 1e-6) / 1e12, 3)
                print(json.dumps(row), flush=True)
                results.append(row)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
