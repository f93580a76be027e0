#!/usr/bin/env python3
"""Fixed cost of a short timed run of the headline step (bench.py's driver form: sync, t0, K steps, sync).

For K in a sweep, the host wall time of K steps (best of ``--trials``) three ways:
  * graph:  one captured K-step HIP graph, replayed (bench.py / DataParallelTrainer.run_plan);
  * native: MlpStep.run_steps -- the same kernels launched from a C++ loop, no graph;
  * graph-warm: the K-step graph replayed right after an untimed replay of itself (back-to-back),
    i.e. what a graph costs once its upload/first-replay work is done.
A least-squares fit t(K) = a + b K gives the fixed cost a (launch latency + final sync) and the
per-step cost b.

    python bench/launch_overhead.py [--ks 1 2 5 10 20 50 100] [--trials 10]
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
    ap.add_argument("--ks", type=int, nargs="*", default=[1, 2, 5, 10, 20, 50])
    ap.add_argument("--trials", type=int, default=10)
    ap.add_argument("--spin", action="store_true",
                    help="hipSetDeviceFlags(hipDeviceScheduleSpin) before the runtime creates its context")
    a = ap.parse_args(argv)
    if a.spin:
        import ctypes

        hip = ctypes.CDLL("libamdhip64.so")
        print(json.dumps({"hipSetDeviceFlags_spin": int(hip.hipSetDeviceFlags(1))}), flush=True)
    import numpy as np
    import torch

    from cme213_sp18_amd.models.mlp import NeuralNetwork
    from cme213_sp18_amd.parallel.trainer import DataParallelTrainer, EpochPlan
    from cme213_sp18_amd.utils.data import synthetic_mnist

    x, y = synthetic_mnist(54000, seed=0)
    tr = DataParallelTrainer(NeuralNetwork([784, 100, 10]), batch_size=800)
    tr.load(x, y)
    e = tr.engine
    s = e._hip_step()
    st = torch.cuda.current_stream().cuda_stream
    n, lr, reg = 800, 1e-3, 1e-4
    rows = []

    def wall(fn):
        best = float("inf")
        for _ in range(a.trials):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best * 1e6

    for k in a.ks:
        plan = EpochPlan([((i * n) % (e.num_samples - e.num_samples % n), n) for i in range(k)])
        g = tr.capture(plan, lr, reg)
        g.replay()
        t_graph = wall(lambda: g.replay())
        t_warm = wall(lambda: (g.replay(), g.replay())) - t_graph  # second replay queued behind the first
        t_native = wall(lambda: s.run_steps(0, k, n, 0, n, e.num_samples, 1.0 / n, reg, lr, 1, st))
        runner = tr.plan_runner(plan, lr, reg)
        t_runner = wall(runner)
        rows.append({"K": k, "graph_us": round(t_graph, 2), "graph_back_to_back_us": round(t_warm, 2),
                     "native_us": round(t_native, 2), "plan_runner_us": round(t_runner, 2)})
        print(json.dumps(rows[-1]), flush=True)
    K = np.array([r["K"] for r in rows], dtype=float)
    for key in ("graph_us", "native_us", "plan_runner_us", "graph_back_to_back_us"):
        b, c = np.polyfit(K, np.array([r[key] for r in rows]), 1)
        print(json.dumps({"fit": key, "fixed_us": round(c, 2), "per_step_us": round(b, 3)}), flush=True)


if __name__ == "__main__":
    main()
