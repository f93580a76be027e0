"""n = 100 step forms against the torch backend: planes / fp32 dZ1, head dW2 partials on / off, the pipeline's
row-major form.  Relative max-norm error of every parameter after one step and after a 10-step plan."""
import json
import sys

import torch

from cme213_sp18_amd.models.mlp import NeuralNetwork
from cme213_sp18_amd.parallel.engine import MlpEngine
from cme213_sp18_amd.utils.data import synthetic_mnist

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
H = 100
N = 5 * n + 48
x, y = synthetic_mnist(N, seed=5)
nn = NeuralNetwork([784, H, 10])
forms = {"torch": None, "planes_h-1": (-1, -1, 0), "planes_h1": (-1, 1, 0), "fp32_h1": (3, 1, 0),
         "fp32_h-1": (3, -1, 0), "xstep": (-1, -1, -1)}
eng = {}
for k, f in forms.items():
    e = MlpEngine(nn.H, "f32", max_cols=n, device="cuda", path="split3", backend="torch" if f is None else "hip")
    e.set_params(*nn.params)
    e.load_dataset(x, y)
    if f is not None:
        e.set_store_a1(False)
        st = e._hip_step()
        st.a_fp32, st.head_dw2, st.xstep = f
    eng[k] = e
s = torch.cuda.current_stream().cuda_stream


def rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max())


def torch_plan(e, count):
    gs = 0
    for _ in range(count):
        e.run(gs, n, 1.0 / n, 1e-4, 0.05, sgd=True)
        gs = 0 if gs + 2 * n > N else gs + n


for label, fn in (("one_step", lambda e: e.run(0, n, 1.0 / n, 1e-4, 0.05, sgd=True)),
                  ("plan10", lambda e: e._hip_step().run_steps(0, 10, n, 0, n, N, 1.0 / n, 1e-4, 0.05, 1, s)
                   if e.backend == "hip" else torch_plan(e, 10))):
    for k, e in eng.items():
        fn(e)
    torch.cuda.synchronize()
    ref = eng["torch"]
    row = {"n": n, "after": label}
    for k, e in eng.items():
        if k == "torch":
            continue
        row[k] = {p: rel(getattr(e, p), getattr(ref, p)) for p in ("W1", "b1", "W2", "b2")}
        if k == "xstep":
            row["xstep_used"] = e._hip_step().xstep_used
    print(json.dumps(row), flush=True)
