#!/usr/bin/env python3
"""Numerics of the wave-split-K GEMMs' paired 16-byte pixel loads (SplitStepArgs.u8_pairs): gradients with the
pairs on and off against the fp32 torch engine, per (H, n, offset).  One JSON line per case.

    python bench/diag_pairs.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import MlpEngine
    from cme213_sp18_amd.utils.data import synthetic_mnist

    def rel(a, b):
        a, b = a.double(), b.double()
        return float((a - b).abs().max() / b.abs().max().clamp_min(1e-300))

    for H, n, off in ((4096, 160, 64), (4096, 160, 0), (100, 800, 64), (100, 800, 0), (1024, 100, 64), (300, 800, 0)):
        x, y = synthetic_mnist(2 * n + 64, seed=3)
        nn = NeuralNetwork([784, H, 10])
        out = {}
        for tag, backend, pairs in (("torch", "torch", None), ("p0", "hip", 0), ("p1", "hip", 1)):
            e = MlpEngine(nn.H, dtype="f32", max_cols=n, device="cuda", backend=backend, path="auto")
            e.set_params(*nn.params)
            e.load_dataset(x, y)
            if pairs is not None:
                e._hip_step().u8_pairs = pairs
            e.run(off, n, 1.0 / n, 1e-4, 0.0, sgd=False, with_loss=True)
            torch.cuda.synchronize()
            out[tag] = {k: getattr(e, k).clone() for k in ("gW1", "gb1", "gW2", "gb2", "dZ1", "a1", "D")}
        row = {"H": H, "n": n, "off": off}
        for k in ("gW1", "gb1", "gW2", "dZ1", "D"):
            row[k + "_p0"] = rel(out["p0"][k], out["torch"][k])
            row[k + "_p1"] = rel(out["p1"][k], out["torch"][k])
        d = (out["p1"]["gW1"] - out["p0"]["gW1"]).abs()
        i = int(d.argmax())
        row["gW1_p1_vs_p0"] = rel(out["p1"]["gW1"], out["p0"]["gW1"])
        row["gW1_worst"] = [i // out["p0"]["gW1"].shape[1], i % out["p0"]["gW1"].shape[1]]
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
