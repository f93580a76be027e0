#!/usr/bin/env python3
"""A/B of the wide-layer head forms on one GPU: the forward launch + head_wide_kernel ("head") against the
head fused into the forward launch (mlp_fwd1_wide_ag: "ag", "ag_noa1" without the a1 store).  Each form: whole training steps (forward + head + wgrad + fused SGD) captured into a HIP graph of
`reps` steps, best of 5 replays, plus the forward + head launch alone (parts=1).  One JSON line per form.

    python bench/wide_ag_ab.py [--hidden 4096] [--cols 800] [--cfg f32:split3 bf16:split1]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden", type=int, nargs="*", default=[4096])
    ap.add_argument("--cols", type=int, default=800)
    ap.add_argument("--cfg", nargs="*", default=["f32:split3", "bf16:split1"])
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--modes", nargs="*", default=["head", "ag", "ag_noa1"],
                    help="head | ag | ag_noa1, each optionally +l0 / +l1 (MlpStep.lazy_planes off / on: the in-place "
                         "W1 update skips the W1-plane refresh; default: the engine's); a mode may repeat (A/B alternation)")
    a = ap.parse_args(argv)
    import torch

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import MlpEngine
    from cme213_sp18_amd.utils.data import synthetic_mnist

    n = a.cols
    x, y = synthetic_mnist(8 * n, seed=0)

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
            torch.cuda.synchronize()
            best = min(best, s.elapsed_time(e) * 1e3 / reps)
        return best

    for H in a.hidden:
        nn = NeuralNetwork([784, H, 10])
        for cfg in a.cfg:
            dt, path = cfg.split(":")
            ref = ref_ag = None
            for mode_q in a.modes:
                mode, *opts = mode_q.split("+")
                e = MlpEngine(nn.H, dtype=dt, max_cols=n, device="cuda", path=path)
                e.set_params(*nn.params)
                e.load_dataset(x, y)
                e.set_fh_allgather(mode != "head")
                e.set_store_a1(not mode.endswith("noa1"))
                e._hip_step().ag_tiles64 = 1
                if "l0" in opts or "l1" in opts:  # (else the engine's default, MlpEngine.lazy_planes)
                    e.set_lazy_planes("l1" in opts)
                off = [0]

                def step():
                    e.run(off[0], n, 1.0 / n, 1e-4, 0.01, sgd=True)
                    off[0] = (off[0] + n) % (7 * n)

                def fwd_head():
                    e.run(0, n, 1.0 / n, 1e-4, 0.0, sgd=False, parts=1)

                r = {"H": H, "n": n, "cfg": cfg, "mode": mode_q, "step_us": round(timeit(step, a.reps), 3)}
                # every form runs the same 6 * reps + 2 steps: the fused forms must leave BITWISE equal params
                # (a stale hand-off read would show here), the head form equal to fp32 rounding
                p = e.params.clone()
                if mode == "head" and ref is None:
                    ref = p
                if ref is not None:
                    r["params_rel_vs_head"] = float((p - ref).abs().max() / ref.abs().max())
                if mode != "head" and ref_ag is None:
                    ref_ag = p
                if mode != "head":
                    r["params_bitwise_eq_ag"] = bool(torch.equal(p, ref_ag))
                r["fwd_head_us"] = round(timeit(fwd_head, a.reps), 3)
                r["kernel_error"] = bool(e.kernel_error())
                print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
