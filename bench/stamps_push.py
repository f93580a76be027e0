#!/usr/bin/env python3
"""Timeline of the small-layer weight-gradient launch in its three forms -- SGD fused (one process), the xGMI
all-reduce fused in as the one-shot pull, and as the owner-tile push (both at world 1: the protocol with no
peers) -- from per-workgroup s_memrealtime stamps (SplitStepArgs::wstamps: entry, dW1 tile + epilogue done,
exchange done, end; 100 MHz).  Diagnostic: where the fused forms' extra time goes.

    python bench/stamps_push.py [--n 100 800]
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
    ap.add_argument("--n", type=int, nargs="*", default=[100, 800])
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args(argv)
    import numpy as np
    import torch

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd._native import hip
    from cme213_sp18_amd.parallel import MlpEngine
    from cme213_sp18_amd.utils.data import synthetic_mnist

    x, y = synthetic_mnist(4000, seed=0)
    nn = NeuralNetwork([784, 100, 10])
    pct = lambda v: [round(float(np.percentile(v, q)), 3) for q in (0, 50, 90, 100)]  # noqa: E731
    for n in a.n:
        e = MlpEngine(nn.H, dtype="f32", max_cols=n, device="cuda", path="split3")
        e.set_params(*nn.params)
        e.load_dataset(x, y)
        step = e._hip_step()
        st = torch.cuda.current_stream().cuda_stream
        slots = e.fused_allreduce_slots()
        t1 = 7 * 25
        buf = torch.zeros(1024 * 8, dtype=torch.int64, device="cuda")
        for form in ("sgd", "pull", "push"):
            xc = None
            sgd = 1
            if form != "sgd":
                xc = hip().comm.XgmiComm(0, 1, e.params.numel(), 4, slots, slots if form == "push" else 0)

                class _B:
                    c = xc
                e.attach_xgmi(_B, push=form == "push")
                sgd = 2
            rows = []
            for r in range(a.reps):
                for _ in range(5):
                    step.run(0, n, 1.0 / n, 1e-4, 0.0, sgd, 0, st, 3)
                step.run(0, n, 1.0 / n, 1e-4, 0.0, sgd, 0, st, 1)  # this step's forward, then the stamped wgrad
                torch.cuda.synchronize()
                buf.zero_()
                step.wstamps = buf.data_ptr()
                step.run(0, n, 1.0 / n, 1e-4, 0.0, sgd, 0, st, 2)
                step.wstamps = 0
                torch.cuda.synchronize()
                s = buf.view(-1, 8).cpu().numpy().astype(np.int64)
                live = s[:, 0] > 0
                t0 = s[live, 0].min()
                rel = np.where(s > 0, (s - t0) * 10.0 / 1000.0, np.nan)
                tiles = rel[:8 * 25]  # the dW1 slots (XCD-row placement: 8 x t1n slots; XCD 7's are idle)
                tiles = tiles[~np.isnan(tiles[:, 3])]
                roles = rel[8 * 25:8 * 25 + 9]
                sub = {}
                if form == "push":  # the exchange's phases (xp_exchange stamps): words waited, poll done, barrier
                    sub = {"words_ready": pct(tiles[:, 4]), "polled": pct(tiles[:, 5]), "barrier": pct(tiles[:, 6])}
                rows.append({**sub, "entry": pct(tiles[:, 0]), "tile_done": pct(tiles[:, 1]), "exchanged": pct(tiles[:, 2]),
                             "end": pct(tiles[:, 3]), "roles_end": pct(roles[~np.isnan(roles[:, 3]), 3]),
                             "launch_end": round(float(np.nanmax(rel[:, 3])), 3)})
            med = {k: [round(float(np.median([r[k][i] for r in rows])), 3) for i in range(4)] for k in rows[0]
                   if k != "launch_end"}
            med["launch_end"] = round(float(np.median([r["launch_end"] for r in rows])), 3)
            print(json.dumps({"n": n, "form": form, "err": xc.error() if xc else 0, **med}), flush=True)
            if xc is not None:
                e.attach_xgmi(None)
                xc.close()


if __name__ == "__main__":
    main()
