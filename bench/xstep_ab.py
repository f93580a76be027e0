#!/usr/bin/env python3
"""The XCD-local step pipeline (csrc/mlp/xstep.hip) against the two-launch native step loop, alternated.

For each batch size: the walking native loop (``MlpStep.run_steps`` over consecutive batches, as bench.py's timed
region runs it) with ``xstep = 0`` (two launches per step) and ``xstep = -1`` (the whole plan in one persistent
launch; its XCD-local barrier's form from --bar), ``--rounds`` times alternated; us/step = best of 5 event-timed plans
of --reps steps.  With --stamps K, the pipeline also records per-workgroup phase stamps of its first K steps
(s_memrealtime): forward + head, first barrier, dW1 / role, second barrier -- medians per XCD.

    python bench/xstep_ab.py [--cols 800] [--reps 200] [--rounds 2] [--bar 0 1] [--stamps 40] [--fha-stamps 30]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

# (CME_PKG_ROOT: a variant copy of the package, bench/flags_ab_build.py)
sys.path.insert(0, os.environ.get("CME_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden", type=int, default=100)
    ap.add_argument("--cols", type=int, nargs="*", default=[800])
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--bar", type=int, nargs="*", default=[3], help="MlpStep.xstep_bar values (XStepPlan::bar)")
    ap.add_argument("--pf", type=int, nargs="*", default=[0], help="MlpStep.xstep_pf values (XStepPlan::npf)")
    ap.add_argument("--rm", action="store_true",
                    help="also the pipeline's row-major form on plans the fragment-ordered form takes (MlpStep.dz_swz = 0)")
    ap.add_argument("--stamps", type=int, default=0)
    ap.add_argument("--fha-stamps", type=int, default=0, help="forward + head body stamps of the last of K steps")
    ap.add_argument("--gemm-stamps", action="store_true",
                    help="with --fha-stamps: also the forward K loop's per-wave stamps (stored mid-body: they perturb)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    import numpy as np
    import torch

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import MlpEngine
    from cme213_sp18_amd.utils.data import synthetic_mnist

    x, y = synthetic_mnist(54000, seed=0)
    out = open(a.json, "a") if a.json else None

    def emit(row):
        print(json.dumps(row), flush=True)
        if out:
            out.write(json.dumps(row) + "\n")
            out.flush()

    for n in a.cols:
        nn = NeuralNetwork([784, a.hidden, 10])
        e = MlpEngine(nn.H, dtype="f32", max_cols=n, device="cuda", path="split3")
        e.set_params(*nn.params)
        e.load_dataset(x, y)
        e.set_store_a1(False)
        st = e._hip_step()
        N = e.num_samples
        stream = torch.cuda.current_stream().cuda_stream

        def walk(count, g0=0):
            st.run_steps(g0, count, n, 0, n, N, 1.0 / n, 1e-4, 1e-3, 1, stream)

        forms = [("two_launch", 0, 1, 0)] + [(f"xstep_bar{b}_pf{q}", -1, b, q) for b in a.bar for q in a.pf
                                             if b == 1 or q == 0]
        if a.rm:
            forms.append(("xstep_rm", -1, 3, 0))
        dz0 = st.dz_swz
        for rnd in range(a.rounds):
            for name, xs, b, q in forms:
                st.xstep, st.xstep_bar, st.xstep_pf = xs, b, q
                st.dz_swz = 0 if name == "xstep_rm" else dz0
                walk(20)
                torch.cuda.synchronize()
                best = float("inf")
                for _ in range(5):
                    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s0.record()
                    walk(a.reps, 8 * n)
                    s1.record()
                    s1.synchronize()
                    best = min(best, s0.elapsed_time(s1) * 1e3 / a.reps)
                emit({"n": n, "H": a.hidden, "form": name, "round": rnd, "reps": a.reps, "us_per_step": round(best, 3),
                      "xstep_used": int(st.xstep_used), "kernel_error": bool(e.kernel_error())})
        if a.stamps:
            # phase stamps of the first K steps, relative to each step's GLOBAL start (the earliest workgroup entry
            # into the step on any XCD): per XCD, medians over its workers (and the role workgroup)
            k = a.stamps
            buf = torch.zeros(k * 8 * 32 * 4, dtype=torch.int64, device="cuda")
            st.xstep, st.xstep_bar, st.xstep_pf = -1, a.bar[-1], a.pf[-1]
            st.xs_stamps, st.xs_stamp_steps = buf.data_ptr(), k
            walk(k)
            torch.cuda.synchronize()
            st.xs_stamps, st.xs_stamp_steps = 0, 0
            s4 = buf.view(k, 8, 32, 4).cpu().numpy().astype(np.int64)
            nw = max((n + 31) // 32, (784 + 1 + 31) // 32)
            live = [x for x in range(8) if (s4[:, x, 0, 0] > 0).all()]
            g0 = np.array([min(s4[i, x, :nw + 1, 0].min() for x in live) for i in range(k)])[:, None]
            rows = {}
            for x in live:
                w = s4[:, x, :nw, :] - g0[:, :, None]
                r = s4[:, x, nw, :] - g0
                rows[x] = {"entry": np.median(w[:, :, 0]), "fwd_head_done": np.median(w[:, :, 1]),
                           "fwd_head_done_last": np.median(w[:, :, 1].max(axis=1)),
                           "barrier1_passed": np.median(w[:, :, 2]), "dw1_done": np.median(w[:, :, 3]),
                           "dw1_done_last": np.median(w[:, :, 3].max(axis=1)), "role_done": np.median(r[:, 3])}
                rows[x] = {kk: round(float(v) / 100, 3) for kk, v in rows[x].items()}
            per = np.diff(g0[:, 0]) / 100
            emit({"n": n, "H": a.hidden, "bar": a.bar[-1], "stamps_steps": k, "step_period_median_us": round(float(np.median(per)), 3),
                  "per_xcd_median_us_from_step_start": rows})
        if a.fha_stamps:
            # the forward + head body's own stamps (fha_body: entry, z2 partial published, all partials gathered,
            # end) and the K loop's per-wave stamps (wsk_tile) for the LAST step of a K-step plan, relative to the
            # earliest entry
            k = a.fha_stamps
            fst = torch.zeros(2 * 256 * 4, dtype=torch.int64, device="cuda")
            hst = torch.zeros(256 * 8 * 4, dtype=torch.int64, device="cuda")
            st.xstep, st.xstep_bar, st.xstep_pf = -1, a.bar[-1], a.pf[-1]
            st.stamps, st.hstamps = fst.data_ptr(), hst.data_ptr() if a.gemm_stamps else 0
            walk(k)
            torch.cuda.synchronize()
            st.stamps, st.hstamps = 0, 0
            f8 = fst.view(2, 256, 4).cpu().numpy().astype(np.int64)
            f4, f4b = f8[0], f8[1]  # [slot * 8 + xcd]: fha_body's four stamps, then its PS extras
            h4 = hst.view(256, 8, 4).cpu().numpy().astype(np.int64)  # [blockIdx][wave] (physical block)
            used = f4[:, 0] > 0
            t0 = f4[used, 0].min()
            hb = h4[h4[:, 0, 0] > 0]  # the forward K loop's per-wave stamps: entry, K loop done, reduced, epilogue done
            kst = {f"gemm_{nm}": np.median(hb[:, :, i].max(axis=1) - t0) if len(hb) else None
                   for i, nm in enumerate(("entry", "kloop_done", "reduced", "epilogue_done"))}
            kst["gemm_kloop_done_first_wave"] = np.median(hb[:, :, 1].min(axis=1) - t0) if len(hb) else None
            rows = {"entry": np.median(f4[used, 0] - t0), **kst,
                    "fwd_tile_returned": np.median(f4b[used, 0] - t0), "w2_staged": np.median(f4b[used, 1] - t0),
                    "z2_partial_formed": np.median(f4b[used & (f4b[:, 2] > 0), 2] - t0),
                    "z2_published": np.median(f4[used, 1] - t0), "z2_published_last": (f4[used, 1] - t0).max(),
                    "gathered": np.median(f4[used, 2] - t0), "end": np.median(f4[used, 3] - t0),
                    "end_last": (f4[used, 3] - t0).max()}
            per_xcd = {}
            for x in range(8):
                m = used & (np.arange(256) % 8 == x)
                if m.any():
                    per_xcd[x] = {"entry": round(float(np.median(f4[m, 0] - t0)) / 100, 3),
                                  "published": round(float(np.median(f4[m, 1] - t0)) / 100, 3),
                                  "gathered": round(float(np.median(f4[m, 2] - t0)) / 100, 3),
                                  "end": round(float(np.median(f4[m, 3] - t0)) / 100, 3)}
            emit({"n": n, "H": a.hidden, "bar": st.xstep_bar, "fha_stamps_last_of": k,
                  "fha_median_us": {kk: (round(float(v) / 100, 3) if v is not None else None) for kk, v in rows.items()},
                  "fha_per_xcd_median_us": per_xcd})
    if out:
        out.close()


if __name__ == "__main__":
    main()
