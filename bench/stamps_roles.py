#!/usr/bin/env python3
"""Timeline of the small-layer weight-gradient launch's ROLE workgroups (dW2 tiles / slices, db2 rows) from
per-workgroup and per-wave s_memrealtime stamps (SplitStepArgs::wstamps: entry / end; SplitStepArgs::stamps inside
wsk_tile: wave entry, K loop done, reduction barrier, epilogue done; 100 MHz), with and without the head's dW2
partials (MlpStep.head_dw2) and for the roles alone (run_wgrad parts = 2) or the whole launch (run parts = 2, SGD
fused).  Diagnostic only.  (The dW2 role split over workgroups this script also timed, MlpStep.w2_ks, measured no
faster and was removed: profiles/r5/stamps_roles_w2_split.jsonl.)

    python bench/stamps_roles.py [--n 400 800]
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
    ap.add_argument("--n", type=int, nargs="*", default=[400, 800])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--head-dw2", type=int, nargs="*", default=[0, 1])
    a = ap.parse_args(argv)
    import numpy as np
    import torch

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import MlpEngine
    from cme213_sp18_amd.utils.data import synthetic_mnist

    x, y = synthetic_mnist(4000, seed=0)
    nn = NeuralNetwork([784, 100, 10])
    pct = lambda v: [round(float(np.percentile(v, q)), 3) for q in (0, 50, 100)] if len(v) else []  # noqa: E731
    for n in a.n:
        e = MlpEngine(nn.H, dtype="f32", max_cols=n, device="cuda", path="split3")
        e.set_params(*nn.params)
        e.load_dataset(x, y)
        step = e._hip_step()
        st = torch.cuda.current_stream().cuda_stream
        wbuf = torch.zeros(1024 * 8, dtype=torch.int64, device="cuda")
        sbuf = torch.zeros(1024 * 8 * 4, dtype=torch.int64, device="cuda")
        for hd in a.head_dw2:
            step.head_dw2 = hd
            for whole in (False, True):
                rows = []
                for r in range(a.reps):
                    for _ in range(5):
                        step.run(0, n, 1.0 / n, 1e-4, 0.0, 1, 0, st, 3)
                    step.run(0, n, 1.0 / n, 1e-4, 0.0, 1, 0, st, 1)
                    torch.cuda.synchronize()
                    wbuf.zero_()
                    sbuf.zero_()
                    step.wstamps, step.stamps = wbuf.data_ptr(), sbuf.data_ptr()
                    if whole:
                        step.run(0, n, 1.0 / n, 1e-4, 0.0, 1, 0, st, 2)
                    else:
                        step.run_wgrad(0, n, 1.0 / n, 1e-4, 0.0, 1, 2, 0, -1, st)
                    step.wstamps = step.stamps = 0
                    torch.cuda.synchronize()
                    w = wbuf.view(-1, 8).cpu().numpy().astype(np.int64)
                    s = sbuf.view(-1, 8, 4).cpu().numpy().astype(np.int64)  # [block][wave][4]
                    live = w[:, 0] > 0
                    t0 = w[live, 0].min()
                    us = lambda v: (v - t0) * 10.0 / 1000.0  # noqa: E731
                    nb = int(live.nonzero()[0].max()) + 1
                    first_role = 8 * 25 if whole else 0
                    t2 = 7
                    roles = [b for b in range(first_role, first_role + t2) if w[b, 0] > 0]
                    bias = [b for b in range(first_role + t2, nb) if w[b, 0] > 0 and w[b, 3] > 0 and b < first_role + t2 + 2]
                    kdone = [us(s[b, :, 1].max()) for b in roles if s[b, 0, 0] > 0]
                    red = [us(s[b, :, 2].max()) for b in roles if s[b, 0, 0] > 0]
                    rows.append({"role_entry": pct([us(w[b, 0]) for b in roles]),
                                 "kloop_done": pct(kdone), "reduced": pct(red),
                                 "role_end": pct([us(w[b, 3]) for b in roles]),
                                 "bias_end": pct([us(w[b, 3]) for b in bias]),
                                 "launch_end": round(float(us(w[live, 3][w[live, 3] > 0].max())), 3)})
                med = {k: [round(float(np.median([r[k][i] for r in rows if r[k]])), 3) for i in range(3)]
                       for k in rows[0] if k != "launch_end" and rows[0][k]}
                med["launch_end"] = round(float(np.median([r["launch_end"] for r in rows])), 3)
                print(json.dumps({"n": n, "head_dw2": hd, "launch": "whole" if whole else "roles", **med}), flush=True)


if __name__ == "__main__":
    main()
