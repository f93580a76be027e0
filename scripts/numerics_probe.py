import json, sys
sys.path.insert(0, '/root/repo')
import numpy as np, torch
from cme213_sp18_amd import NeuralNetwork
from cme213_sp18_amd.models import mlp as cpu_mlp
from cme213_sp18_amd.parallel import DataParallelTrainer, MlpEngine
from cme213_sp18_amd.utils.data import synthetic_mnist

def rel(a, b):
    a = a.double(); b = b.double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-300))

for H in (100, 300, 1024, 4096):
    for n in (800, 100, 37):
        x, y = synthetic_mnist(2 * n + 64, seed=3)
        nn = NeuralNetwork([784, H, 10])
        res = {"H": H, "n": n}
        ref = MlpEngine(nn.H, dtype="f64", max_cols=n, device="cuda", backend="torch")
        ref.set_params(*nn.params); ref.load_dataset(x, y)
        ref.run(64, n, 1.0 / n, 1e-4, 0.0, sgd=False)
        for dt, path in (("f32", "split3"), ("f32", "mfma")):
            for backend in ("hip", "torch"):
                if backend == "torch" and path == "mfma": continue
                e = MlpEngine(nn.H, dtype=dt, max_cols=n, device="cuda", backend=backend, path=path)
                e.set_params(*nn.params); e.load_dataset(x, y)
                e.run(64, n, 1.0 / n, 1e-4, 0.0, sgd=False)
                torch.cuda.synchronize()
                key = f"{backend}:{path}"
                res[key] = {k: float(f"{rel(getattr(e, k), getattr(ref, k)):.3g}") for k in ("gW1", "gb1", "gW2", "gb2")}
        print(json.dumps(res), flush=True)

# multi-epoch drift: split3 (GPU) vs fp64 CPU oracle
x, y = synthetic_mnist(8000, seed=7)
nn = NeuralNetwork([784, 100, 10])
seq = nn.copy()
cpu_mlp.train(seq, x, y, 0.01, 1e-4, epochs=4, batch_size=800)
for dt in ("f32", "f64"):
    par = nn.copy()
    t = DataParallelTrainer(par, dtype=dt)
    t.load(x, y)
    t.train(4, 0.01, 1e-4)
    print(json.dumps({"drift_epochs": 4, "dtype": dt, "W": [float(f"{np.abs(par.W[i] - seq.W[i]).max() / np.abs(seq.W[i]).max():.3g}") for i in range(2)],
                      "b": [float(f"{np.abs(par.b[i] - seq.b[i]).max() / np.abs(seq.b[i]).max():.3g}") for i in range(2)]}), flush=True)
