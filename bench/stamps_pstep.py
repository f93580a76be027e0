"""Per-phase timeline of the persistent small-batch engine (csrc/mlp/pstep.hip) from s_memrealtime stamps (100 MHz):
workgroup 0, the first 16 steps of one run_steps launch; prints the median duration of every phase (us).

    python bench/stamps_pstep.py [--n 100] [--steps 16]
"""
import argparse
import json
import statistics

import torch

from cme213_sp18_amd import NeuralNetwork
from cme213_sp18_amd.parallel import MlpEngine
from cme213_sp18_amd.utils.data import synthetic_mnist

PHASES = ["forward (a1)", "z2 partial store", "z2 gather", "softmax / D", "dZ1", "dW2 + dW1 + update", "W2 update"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[100])
    ap.add_argument("--steps", type=int, default=16)
    a = ap.parse_args()
    for n in a.n:
        N = 16 * n
        x, y = synthetic_mnist(N, seed=1)
        nn = NeuralNetwork([784, 100, 10])
        e = MlpEngine(nn.H, dtype="f32", max_cols=n, device="cuda")
        e.set_params(*nn.params)
        e.load_dataset(x, y)
        st = e._hip_step()
        st.persistent = 1
        assert st.uses_persistent(n, 1)
        buf = torch.zeros(16 * 8, dtype=torch.int64, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        st.run_steps(0, 4, n, 0, n, N, 1.0 / n, 1e-4, 0.0, 1, s)  # warm-up
        st.stamps = buf.data_ptr()
        st.run_steps(0, a.steps, n, 0, n, N, 1.0 / n, 1e-4, 0.0, 1, s)
        torch.cuda.synchronize()
        st.stamps = 0
        t = buf.view(16, 8).cpu().tolist()
        k = min(a.steps, 16)
        rows = [[(t[i][j + 1] - t[i][j]) / 100.0 for j in range(7)] for i in range(k)]
        step = [(t[i][7] - t[i][0]) / 100.0 for i in range(k)]
        gap = [(t[i + 1][0] - t[i][7]) / 100.0 for i in range(k - 1)]
        out = {"n": n, "step_us_median": statistics.median(step), "between_steps_us": statistics.median(gap) if gap else 0}
        for j, name in enumerate(PHASES):
            out[name] = round(statistics.median(r[j] for r in rows), 3)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
