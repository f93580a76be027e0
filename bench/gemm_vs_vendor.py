#!/usr/bin/env python3
"""Our GEMMs against the vendor BLAS (hipBLASLt / rocBLAS through torch) on MI355X.

Two tables, both graph-replayed and event-timed (``reps`` launches captured in one HIP graph, time per
launch = elapsed / reps: no host launch overhead, the dependent-kernel boundary included):

1. The reference's grade-4 GEMM benchmark shapes (fpcode/utils/tests.cpp:261-280, main.cpp:154-161):
   column-major ``C = 2 A B + 5 C`` at (M, N, K) = (800, 1000, 784) and (800, 10, 1000), f64 / f32 /
   bf16: ``myGEMM`` (ops/gemm.py) vs ``torch.addmm`` with the same alpha / beta.
2. The training GEMMs of the wide configs (784-4096-10 and 784-1024-10, 800 samples per GPU):
   forward ``Z1 = W1 X^T`` (H x 800 x 784, both operands K-contiguous) and ``dW1 = dZ1 X`` (H x 784 x 800).
   Ours is the fused engine kernel (sigmoid / z2-partials or reg + SGD + plane-refresh epilogue
   included); the vendor column is the bare GEMM in bf16, in fp32, and the fp32-exact equivalent of
   our split3 path (three bf16 planes of W1 stacked: a 3H x 800 x 784 bf16 GEMM).

    python bench/gemm_vs_vendor.py [--reps 50] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def graph_time_us(fn, reps: int) -> float:
    import torch

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


def reference_shapes(reps: int) -> list:
    import torch

    from cme213_sp18_amd.ops.gemm import create_mats, myGEMM

    rows = []
    for dt in (torch.float64, torch.float32, torch.bfloat16):
        for (M, N, K) in ((800, 1000, 784), (800, 10, 1000)):
            A, B, C = create_mats(M, N, K, dt, "cuda")
            Am, Bm = A.view(K, M).t(), B.view(N, K).t()
            Cm = C.view(N, M).t()
            out = torch.empty(M, N, dtype=dt, device="cuda")
            Cw = C.clone()
            lib = graph_time_us(lambda: torch.addmm(Cm, Am, Bm, beta=5.0, alpha=2.0, out=out), reps)
            mine = graph_time_us(lambda: myGEMM(A, B, Cw, 2.0, 5.0, M, N, K), reps)
            # numerics of one call from the same C
            Cw.copy_(C)
            myGEMM(A, B, Cw, 2.0, 5.0, M, N, K)
            ref = torch.addmm(Cm.double(), Am.double(), Bm.double(), beta=5.0, alpha=2.0)
            err = float((Cw.view(N, M).t().double() - ref).abs().max() / ref.abs().max())
            fl = 2.0 * M * N * K
            rows.append({"table": "reference", "dtype": str(dt).replace("torch.", ""), "M": M, "N": N, "K": K,
                         "lib_us": round(lib, 3), "mine_us": round(mine, 3),
                         "lib_tflops": round(fl / lib / 1e6, 2), "mine_tflops": round(fl / mine / 1e6, 2),
                         "speedup_vs_lib": round(lib / mine, 3), "max_rel_err_vs_f64": err})
            print(json.dumps(rows[-1]), flush=True)
    return rows


def training_shapes(reps: int, hiddens=(1024, 4096), n: int = 800) -> list:
    import torch

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import MlpEngine
    from cme213_sp18_amd.utils.data import synthetic_mnist

    x, y = synthetic_mnist(4000, seed=0)
    P = 784
    rows = []
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    for H in hiddens:
        W = torch.randn(H, P, device="cuda")
        X = torch.randint(0, 256, (n, P), device="cuda").float()
        dZ = torch.randn(H, n, device="cuda")
        vendor = {}
        for name, dt in (("bf16", torch.bfloat16), ("fp32", torch.float32)):
            Wd, Xd, dZd = W.to(dt), X.to(dt), dZ.to(dt)
            o1 = torch.empty(H, n, dtype=dt, device="cuda")
            o2 = torch.empty(H, P, dtype=dt, device="cuda")
            vendor[f"fwd_{name}"] = graph_time_us(lambda: torch.matmul(Wd, Xd.t(), out=o1), reps)
            vendor[f"dw1_{name}"] = graph_time_us(lambda: torch.matmul(dZd, Xd, out=o2), reps)
        W3 = torch.cat([W.bfloat16()] * 3)
        Xb = X.bfloat16()
        dZ3 = torch.cat([dZ.bfloat16()] * 3)
        o1 = torch.empty(3 * H, n, dtype=torch.bfloat16, device="cuda")
        o2 = torch.empty(3 * H, P, dtype=torch.bfloat16, device="cuda")
        vendor["fwd_bf16x3"] = graph_time_us(lambda: torch.matmul(W3, Xb.t(), out=o1), reps)
        vendor["dw1_bf16x3"] = graph_time_us(lambda: torch.matmul(dZ3, Xb, out=o2), reps)
        nn = NeuralNetwork([P, H, 10])
        for dt, path, planes, vkey in (("f32", "split3", 3, "bf16x3"), ("bf16", "split1", 1, "bf16")):
            e = MlpEngine(nn.H, dtype=dt, max_cols=n, device="cuda", path=path)
            e.set_params(*nn.params)
            e.load_dataset(x, y)
            s = e._hip_step()
            ours_fwd = graph_time_us(lambda: s.run(0, n, 1.0 / n, 1e-4, 0.0, 1, 0, st(), 1 | 4), reps)
            ours_dw1 = graph_time_us(lambda: s.run_wgrad(0, n, 1.0 / n, 1e-4, 0.0, 0, 1, 0, -1, st()), reps)
            fl = 2.0 * planes * H * n * P
            for op, ours, lib in (("fwd", ours_fwd, vendor[f"fwd_{vkey}"]), ("dw1", ours_dw1, vendor[f"dw1_{vkey}"])):
                rows.append({"table": "training", "op": op, "H": H, "n": n, "K": P if op == "fwd" else n,
                             "ours": f"{dt}:{path}", "mine_us": round(ours, 3), "lib_us": round(lib, 3),
                             "lib_op": f"torch.matmul {vkey}", "lib_fp32_us": round(vendor[f"{op}_fp32"], 3),
                             "mine_tflops": round(fl / ours / 1e6, 1), "lib_tflops": round(fl / lib / 1e6, 1),
                             "speedup_vs_lib": round(lib / ours, 3)})
                print(json.dumps(rows[-1]), flush=True)
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", choices=["reference", "training"], default=None)
    a = ap.parse_args(argv)
    rows = []
    if a.only in (None, "reference"):
        rows += reference_shapes(a.reps)
    if a.only in (None, "training"):
        rows += training_shapes(a.reps)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
