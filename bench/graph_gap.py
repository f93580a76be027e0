#!/usr/bin/env python3
"""Kernel-to-kernel gaps of the headline step (784-100-10, n = 800) replayed as a HIP graph vs launched from the
native loop, the same batch every step (diagnostic for `profiles/kbench_graph_vs_stream_r4.jsonl`, where only the
same-batch graph reaches 13.2 us).  Run under `rocprofv3 --kernel-trace`; then `--parse DIR` prints, per phase, the
median kernel durations and the median gap from one kernel's end to the next one's start (negative = overlap).

    rocprofv3 --kernel-trace -d OUT -o gg --output-format csv -- python3 bench/graph_gap.py
    python3 bench/graph_gap.py --parse OUT
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run():
    import torch

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import MlpEngine
    from cme213_sp18_amd.utils.data import synthetic_mnist

    n, reps = 800, 20
    x, y = synthetic_mnist(8000, seed=0)
    nn = NeuralNetwork([784, 100, 10])
    e = MlpEngine(nn.H, dtype="f32", max_cols=n, device="cuda", path="split3")
    e.set_params(*nn.params)
    e.load_dataset(x, y)
    step = e._hip_step()
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    one = lambda: step.run_steps(0, 1, n, 0, n, n, 1.0 / n, 1e-4, 0.0, 1, st())  # noqa: E731
    one()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            one()
    torch.cuda.synchronize()
    marker = torch.zeros(1, device="cuda")
    for _ in range(5):  # phase A: graph replays
        g.replay()
    torch.cuda.synchronize()
    marker.add_(1)  # a torch kernel between the phases
    torch.cuda.synchronize()
    for _ in range(5):  # phase B: native loop, same batch
        step.run_steps(0, reps, n, 0, n, n, 1.0 / n, 1e-4, 0.0, 1, st())
    torch.cuda.synchronize()


def parse(d):
    import csv
    import glob
    import statistics as s

    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    phases, cur = [], []
    for r in rows:
        name = r["Kernel_Name"]
        if "fwd1_head_ag" in name or "wgrad_split" in name:
            cur.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "fwd" if "fwd1" in name else "wgrad"))
        elif cur:
            phases.append(cur)
            cur = []
    if cur:
        phases.append(cur)
    for label, ks in zip(("graph, same batch", "native loop, same batch"), phases[-2:]):
        ks = ks[2:]  # (the first step of the phase)
        gaps = [(b[0] - a[1]) / 1e3 for a, b in zip(ks, ks[1:])]
        fwd = [(k[1] - k[0]) / 1e3 for k in ks if k[2] == "fwd"]
        wg = [(k[1] - k[0]) / 1e3 for k in ks if k[2] == "wgrad"]
        step = (ks[-1][1] - ks[0][0]) / 1e3 / (len(ks) / 2)
        print(f"{label}: kernels {len(ks)}, fwd median {s.median(fwd):.2f} us, wgrad median {s.median(wg):.2f} us, "
              f"gap median {s.median(gaps):.2f} us (min {min(gaps):.2f}), step {step:.2f} us")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--parse", default=None)
    a = ap.parse_args()
    parse(a.parse) if a.parse else run()
