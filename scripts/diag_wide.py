"""Wide-path diagnostic: every intermediate of one hip step against the torch backend (rel max-norm)."""
import sys

import torch

sys.path.insert(0, ".")
from cme213_sp18_amd import NeuralNetwork  # noqa: E402
from cme213_sp18_amd.parallel import MlpEngine  # noqa: E402
from cme213_sp18_amd.utils.data import synthetic_mnist  # noqa: E402


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-300))


for H, n, dt, path in [(4096, 800, "f32", "split3"), (2048, 800, "f32", "split3"), (4096, 800, "bf16", "split1")]:
    x, y = synthetic_mnist(2 * n + 64, seed=3)
    nn = NeuralNetwork([784, H, 10])
    for ag in (True, False):
        es = []
        for backend in ("hip", "torch"):
            e = MlpEngine(nn.H, dtype=dt, max_cols=n, device="cuda", backend=backend, path=path)
            e.set_params(*nn.params)
            e.load_dataset(x, y)
            if backend == "hip":
                e.set_fh_allgather(ag)
            e.run(64, n, 1.0 / n, 1e-4, 0.0, sgd=False, with_loss=True)
            es.append(e)
        torch.cuda.synchronize()
        h, t = es
        r = {k: rel(getattr(h, k)[:, :n], getattr(t, k)[:, :n]) for k in ("a1", "D", "dZ1")}
        r.update({k: rel(getattr(h, k), getattr(t, k)) for k in ("gW1", "gb1", "gW2", "gb2")})
        print(H, n, dt, "ag" if ag else "head", {k: f"{v:.2e}" for k, v in r.items()}, flush=True)
