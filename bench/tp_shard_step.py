#!/usr/bin/env python3
"""Compute time of ONE tensor-parallel rank's step (no collective): the hidden shard H / R of a 784-H-10 MLP over
the whole global batch B -- BASELINE config 4 on 8 GPUs is H = 4096, R = 8, B = 6400 (512 hidden rows x 6400
columns per rank).  The rank's step is then this plus the z2 all-reduce (16 x B fp32 over xGMI).  Graph-replayed,
with and without the split-K weight gradient (MlpEngine.enable_splitk).  One JSON line per row.

    python bench/tp_shard_step.py [--hidden 4096] [--ranks 8] [--batch 6400]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--batch", type=int, default=6400)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args(argv)
    import torch

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import MlpEngine
    from cme213_sp18_amd.utils.data import synthetic_mnist

    Hs, B = a.hidden // a.ranks, a.batch
    x, y = synthetic_mnist(B + 64, seed=0)
    nn = NeuralNetwork([784, Hs, 10])
    for split in (True, False):
        e = MlpEngine(nn.H, dtype=a.dtype, max_cols=B, device="cuda")
        e.set_params(*nn.params)
        e.load_dataset(x, y)
        e.set_store_a1(False)
        if split:
            e.enable_splitk(8)
        st = e._hip_step()

        def step(parts):  # (the stream read at call time: inside the capture it is the capture stream)
            st.run(0, B, 1.0 / B, 1e-4, 1e-3, 1, 0, torch.cuda.current_stream().cuda_stream, parts)

        row = {"hidden_shard": Hs, "global_batch": B, "dtype": a.dtype, "splitk": split}
        for name, parts in (("step", 3), ("fwd_head", 1), ("wgrad", 2)):
            step(parts)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(a.reps):
                    step(parts)
            g.replay()
            torch.cuda.synchronize()
            best = float("inf")
            for _ in range(5):
                t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0.record()
                g.replay()
                t1.record()
                t1.synchronize()
                best = min(best, t0.elapsed_time(t1) * 1e3 / a.reps)
            row[name + "_us"] = round(best, 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
