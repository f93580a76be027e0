#!/usr/bin/env python3
"""Per-kernel microbenchmark of the MLP step (graph-replayed, event-timed).

Each measurement captures ``reps`` back-to-back launches into a HIP graph and
replays it; time per launch = elapsed / reps, so host launch overhead is
excluded and the number is the on-device cost INCLUDING the dependent-kernel
boundary (what a training step actually pays).

    python bench/kbench.py [--hidden 100] [--cols 800 100] [--cfg f32:split3 f32:mfma ...]
"""
from __future__ import annotations

import argparse
import re
import json
import os
import sys

# (CME_PKG_ROOT: a variant copy of the package, bench/flags_ab_build.py)
sys.path.insert(0, os.environ.get("CME_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden", type=int, nargs="*", default=[100])
    ap.add_argument("--cols", type=int, nargs="*", default=[800, 100])
    ap.add_argument("--cfg", nargs="*", default=["f32:split3", "f32:mfma", "bf16:split1", "f64:mfma"])
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    import torch

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import MlpEngine
    from cme213_sp18_amd.utils.data import synthetic_mnist

    x, y = synthetic_mnist(8000, seed=0)
    results = []

    join = None

    def timeit(fn, reps):
        fn()
        if join is not None:
            join()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
            if join is not None:
                join()
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

    for cfg in a.cfg:
        dt, path = cfg.split(":")
        # "+s0": no a1 store (the trainer's setting); "+d0": no dW2 partials from the head (dw2p = 0);
        # "+x0" / "+x1": the XCD-row placement of the H <= 128 launches off / on (MlpStep.xcd_rows)
        no_a1, no_dw2 = "+s0" in path, "+d0" in path
        m = re.search(r"\+x(\d)", path)
        xrows = int(m.group(1)) if m else None
        m = re.search(r"\+p(\d)", path)  # "+pK": K prefetch workgroups per XCD for X (MlpStep.prefetch)
        pref = int(m.group(1)) if m else None
        m = re.search(r"\+t(\d)", path)  # "+tK": K prefetch workgroups per XCD for XT (MlpStep.prefetch_xt)
        pref_xt = int(m.group(1)) if m else None
        m = re.search(r"\+g(\d)", path)  # "+gK": the wide 128 x 128 K loop's engine (MlpStep.wide_eng)
        weng = int(m.group(1)) if m else None
        m = re.search(r"\+l(\d)", path)  # "+lK": the g64 engine's L2 pre-touch off / on (MlpStep.g64_touch)
        gtouch = int(m.group(1)) if m else None
        m = re.search(r"\+h(\d)", path)  # "+hK": the H <= 128 head's dW2 partials off / on (MlpStep.head_dw2)
        hdw2 = int(m.group(1)) if m else None
        m = re.search(r"\+q(\d)", path)  # "+qK": the forward's packed XCD rows off / on (MlpStep.xcd_pack)
        xpack = int(m.group(1)) if m else None
        m = re.search(r"\+z(\d)", path)  # "+zK": the fragment-ordered W1 copy for the forward (MlpStep.w1_swz)
        wswz = int(m.group(1)) if m else None
        m = re.search(r"\+a(\d)", path)  # "+aK": SplitStepArgs::a_fp32 (bit0 fp32 W1, bit1 fp32 dZ1; MlpStep.a_fp32)
        afp = int(m.group(1)) if m else None
        m = re.search(r"\+v(\d)", path)  # "+vK": fp32 dZ1 in the dW1 GEMM's fragment order (MlpStep.dz_swz; needs +a3)
        dzs = int(m.group(1)) if m else None
        m = re.search(r"\+y(\d)", path)  # "+yK": the fragment-ordered pixel copy for the forward (MlpStep.x_swz)
        xswz = int(m.group(1)) if m else None
        path = re.sub(r"\+[sdxptglwhqzyav]\d", "", path)
        for H in a.hidden:
            nn = NeuralNetwork([784, H, 10])
            for n in a.cols:
                e = MlpEngine(nn.H, dtype=dt, max_cols=n, device="cuda", path=path)
                e.set_params(*nn.params)
                e.load_dataset(x, y)
                step = e._hip_step()
                join = e.join
                if xrows is not None:
                    step.xcd_rows = xrows
                if pref is not None:
                    step.prefetch = pref
                if weng is not None:
                    step.wide_eng = weng
                if gtouch is not None:
                    step.g64_touch = gtouch
                if hdw2 is not None:
                    step.head_dw2 = hdw2
                if xpack is not None:
                    step.xcd_pack = xpack
                if wswz is not None:
                    step.w1_swz = wswz
                if xswz is not None:
                    step.x_swz = xswz
                if afp is not None:
                    step.a_fp32 = afp
                if dzs is not None:
                    step.dz_swz = dzs
                if pref_xt is not None:
                    step.prefetch_xt = pref_xt
                if no_a1:
                    e.set_store_a1(False)
                if no_dw2:
                    step.dw2p = 0
                st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731

                def part(p, sgd=1):
                    return lambda: step.run(0, n, 1.0 / n, 1e-4, 0.0, sgd, 0, st(), p)

                row = {"dtype": dt, "path": e.path + ("+s0" if no_a1 else "") + ("+d0" if no_dw2 else "") + (f"+x{xrows}" if xrows is not None else "") + (f"+p{pref}" if pref is not None else "") + (f"+t{pref_xt}" if pref_xt is not None else "") + (f"+g{weng}" if weng is not None else "") + (f"+l{gtouch}" if gtouch is not None else "") + (f"+h{hdw2}" if hdw2 is not None else "") + (f"+q{xpack}" if xpack is not None else "") + (f"+z{wswz}" if wswz is not None else "") + (f"+y{xswz}" if xswz is not None else "") + (f"+a{afp}" if afp is not None else "") + (f"+v{dzs}" if dzs is not None else ""), "H": H, "n": n}
                if e.np:  # split paths: the weight-gradient launch's two halves on their own
                    for name, prt in (("wgrad_w1", 1), ("wgrad_roles", 2)):
                        row[name + "_us"] = round(timeit(
                            lambda prt=prt: step.run_wgrad(0, n, 1.0 / n, 1e-4, 0.0, 0, prt, 0, -1, st()), a.reps), 3)
                for name, fn in (("fwd_head", part(1)), ("fwd1", part(1 | 4)), ("head", part(1 | 8)),
                                 ("wgrad_sgd", part(2)), ("wgrad_grads", part(2, 0)),
                                 ("step_fused", part(3)), ("sgd_flat", lambda: e.sgd(0.0))):
                    row[name + "_us"] = round(timeit(fn, a.reps), 3)
                if e.np:  # the native step loop over consecutive batches (new pixels every step, as in training)
                    import torch as _t

                    N = e.num_samples
                    step.run_steps(0, 4, n, 0, n, N, 1.0 / n, 1e-4, 0.0, 1, st())
                    best = float("inf")
                    for _ in range(5):
                        s0, s1 = _t.cuda.Event(enable_timing=True), _t.cuda.Event(enable_timing=True)
                        s0.record()
                        step.run_steps(0, a.reps, n, 0, n, N, 1.0 / n, 1e-4, 0.0, 1, st())
                        s1.record()
                        s1.synchronize()
                        best = min(best, s0.elapsed_time(s1) * 1e3 / a.reps)
                    row["step_walk_us"] = round(best, 3)
                    best = float("inf")  # the same native loop over ONE batch (N_end = n): host loop vs data walk
                    for _ in range(5):
                        s0, s1 = _t.cuda.Event(enable_timing=True), _t.cuda.Event(enable_timing=True)
                        s0.record()
                        step.run_steps(0, a.reps, n, 0, n, n, 1.0 / n, 1e-4, 0.0, 1, st())
                        s1.record()
                        s1.synchronize()
                        best = min(best, s0.elapsed_time(s1) * 1e3 / a.reps)
                    row["step_loop_same_us"] = round(best, 3)
                    # the same two loops captured into a HIP graph and replayed: stream launches vs graph nodes
                    # for identical kernels and arguments
                    cnt = [0]

                    def walk1():  # one step of the walk per call: consecutive batches across the captured nodes
                        step.run_steps(cnt[0] * n % (N - N % n), 1, n, 0, n, N, 1.0 / n, 1e-4, 0.0, 1, st())
                        cnt[0] += 1
                    row["step_walk_graph_us"] = round(timeit(walk1, a.reps), 3)
                    row["step_same_graph_us"] = round(timeit(
                        lambda: step.run_steps(0, 1, n, 0, n, n, 1.0 / n, 1e-4, 0.0, 1, st()), a.reps), 3)
                    import time as _time  # host time to ENQUEUE the loop's launches (no sync inside)

                    _t.cuda.synchronize()
                    h0 = _time.perf_counter()
                    step.run_steps(0, a.reps, n, 0, n, N, 1.0 / n, 1e-4, 0.0, 1, st())
                    row["host_enqueue_us"] = round((_time.perf_counter() - h0) * 1e6 / a.reps, 3)
                    _t.cuda.synchronize()
                slots = e.fused_allreduce_slots()
                if slots:  # wgrad with the xGMI all-reduce fused in, world 1 (the flag protocol, no peers)
                    from cme213_sp18_amd._native import hip as _hip

                    xc = _hip().comm.XgmiComm(0, 1, e.params.numel(), 4, slots)

                    class _B:  # minimal bucket view for attach_xgmi
                        c = xc

                    e.attach_xgmi(_B)
                    row["wgrad_xgmi1_us"] = round(timeit(part(2, 2), a.reps), 3)
                    row["step_xgmi1_us"] = round(timeit(part(3, 2), a.reps), 3)
                    torch.cuda.synchronize()
                    row["xgmi1_sep_us"] = round(timeit(lambda: xc.run(0, e.grads.data_ptr(), e.params.data_ptr(), 0.0,
                                                                      e.W1p.data_ptr(), e.np, e.H * e.P, 0,
                                                                      e.params.numel(), st()), a.reps), 3)
                    row["xgmi1_err"] = xc.error()
                    e.attach_xgmi(None)
                    xc.close()
                    # the owner-tile push form at world 1 (XgmiFuse::push): this rank owns every tile, nothing leaves
                    # the workgroup -- what is left is the LDS staging of the gradient tile
                    xp = _hip().comm.XgmiComm(0, 1, e.params.numel(), 4, slots, slots)

                    class _P:
                        c = xp

                    e.attach_xgmi(_P, push=True)
                    row["wgrad_push1_us"] = round(timeit(part(2, 2), a.reps), 3)
                    row["step_push1_us"] = round(timeit(part(3, 2), a.reps), 3)
                    # ablations (SplitStepArgs::xp_dbg): 1 no dW1 exchange, 2 no dW1 put, 3 neither, 4 no dW2 exchange,
                    # 8 no db2 row sums, 16 dW1 tiles stop after the GEMM, 32 dW2 tiles stop after the GEMM
                    # (compiled only into the diagnostics instantiations of the headline shapes: other shapes raise)
                    for dbg in (16, 20, 24, 32, 33, 34, 35, 48):
                        step.xp_dbg = dbg
                        try:
                            row[f"wgrad_push1_dbg{dbg}_us"] = round(timeit(part(2, 2), a.reps), 3)
                        except ValueError:
                            break
                    step.xp_dbg = 0
                    torch.cuda.synchronize()
                    row["push1_err"] = xp.error()
                    e.attach_xgmi(None)
                    xp.close()
                flops = 2 * n * (784 * H * 2 + 10 * H * 3)
                row["step_tflops"] = round(flops / (row["step_fused_us"] * 1e-6) / 1e12, 3)
                print(json.dumps(row), flush=True)
                results.append(row)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
