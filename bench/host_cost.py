#!/usr/bin/env python3
"""Host-side cost of one native-loop call (MlpStep.run_steps with one step): back-to-back calls without a
synchronise, so the GPU never holds the host up (the launches queue), timed by the host clock -- the part of the
driver form's fixed cost that is the Python -> pybind -> argument setup -> launch path.  Pipeline (xstep auto) and
two-launch (xstep = 0), alternated.

    python bench/host_cost.py [--calls 200] [--rounds 3]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.environ.get("CME_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args(argv)
    import torch

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import MlpEngine
    from cme213_sp18_amd.utils.data import synthetic_mnist

    n = 800
    x, y = synthetic_mnist(54000, seed=0)
    nn = NeuralNetwork([784, 100, 10])
    e = MlpEngine(nn.H, dtype="f32", max_cols=n, device="cuda", path="split3")
    e.set_params(*nn.params)
    e.load_dataset(x, y)
    e.set_store_a1(False)
    st = e._hip_step()
    N = e.num_samples
    stream = torch.cuda.current_stream().cuda_stream
    for rnd in range(a.rounds):
        for xs in (-1, 0):
            st.xstep = xs
            for _ in range(20):
                st.run_steps(0, 1, n, 0, n, N, 1.0 / n, 1e-4, 1e-3, 1, stream)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.calls):
                st.run_steps((i * n) % (N - n), 1, n, 0, n, N, 1.0 / n, 1e-4, 1e-3, 1, stream)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(json.dumps({"form": "xstep" if xs else "two_launch", "round": rnd, "calls": a.calls,
                              "host_us_per_call": round(1e6 * (t1 - t0) / a.calls, 2),
                              "wall_us_per_call_incl_drain": round(1e6 * (t2 - t0) / a.calls, 2),
                              "xstep_used": int(st.xstep_used)}), flush=True)


if __name__ == "__main__":
    main()
