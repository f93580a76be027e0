"""Per-block comparison of the persistent small-batch engine (csrc/mlp/pstep.hip) with the two-launch step:
the parameter DELTAS of `steps` steps from one initialisation, block by block (W1, b1, W2, b2), for a few batch
sizes.  Diagnostic for tests/test_gpu_mlp.py::test_persistent_engine_matches_two_launch_steps."""
import argparse
import json

import torch

from cme213_sp18_amd import NeuralNetwork
from cme213_sp18_amd.parallel import MlpEngine
from cme213_sp18_amd.utils.data import synthetic_mnist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[100])
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--reg", type=float, default=1e-4)
    ap.add_argument("--chunk", type=int, default=0, help="persistent: run the steps as launches of this many (0: one)")
    a = ap.parse_args()
    for n in a.n:
        N = 4 * n
        x, y = synthetic_mnist(N, seed=n)
        nn = NeuralNetwork([784, 100, 10])
        res = {}
        for mode in ("persistent", "two-launch", "torch"):
            e = MlpEngine(nn.H, dtype="f32", max_cols=n, device="cuda", backend="torch" if mode == "torch" else "hip")
            e.set_params(*nn.params)
            e.load_dataset(x, y)
            init = [v.clone() for v in (e.W1, e.b1, e.W2, e.b2)]
            if mode == "torch":
                gs = 0
                for i in range(a.steps):
                    gs = 0 if gs + n > N else gs
                    e.run(gs, n, 1.0 / n, a.reg, a.lr, sgd=True)
                    gs += n
            else:
                st = e._hip_step()
                st.persistent = int(mode == "persistent")
                s = torch.cuda.current_stream().cuda_stream
                ch = a.chunk if (a.chunk and mode == "persistent") else a.steps
                done, gs = 0, 0
                while done < a.steps:
                    k = min(ch, a.steps - done)
                    st.run_steps(gs, k, n, 0, n, N, 1.0 / n, a.reg, a.lr, 1, s)
                    for _ in range(k):
                        gs = 0 if gs + n > N else gs
                        gs += n
                    gs = 0 if gs + n > N else gs
                    done += k
            torch.cuda.synchronize()
            res[mode] = [v - i for v, i in zip((e.W1, e.b1, e.W2, e.b2), init)]
            res[mode + "_err"] = bool(e.kernel_error())
        out = {"n": n, "steps": a.steps, "chunk": a.chunk, "err": [res["persistent_err"], res["two-launch_err"]]}
        for name, p, q, r in zip(("W1", "b1", "W2", "b2"), res["persistent"], res["two-launch"], res["torch"]):
            out[name] = {"norm_p": float(p.norm()), "norm_2": float(q.norm()), "norm_t": float(r.norm()),
                         "rel_p2": float((p - q).norm() / q.norm().clamp_min(1e-30)),
                         "rel_pt": float((p - r).norm() / r.norm().clamp_min(1e-30)),
                         "rel_2t": float((q - r).norm() / r.norm().clamp_min(1e-30))}
        # where the W1 delta differs: by hidden row and by feature
        d = (res["persistent"][0] - res["two-launch"][0]).abs()
        out["W1_rows_bad"] = [int(i) for i in torch.nonzero(d.amax(1) > 1e-3 * d.max().clamp_min(1e-30) + 1e-9).flatten()[:20]]
        out["W1_cols_bad"] = [int(i) for i in torch.nonzero(d.amax(0) > 1e-3 * d.max().clamp_min(1e-30) + 1e-9).flatten()[:40]]
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
