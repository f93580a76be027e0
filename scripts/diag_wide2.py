"""Wide-path diagnostic 2: the forward launch's z2 partials (parts=5: forward GEMM only) vs W2 . a1."""
import sys

import torch

sys.path.insert(0, ".")
from cme213_sp18_amd import NeuralNetwork  # noqa: E402
from cme213_sp18_amd.parallel import MlpEngine  # noqa: E402
from cme213_sp18_amd.utils.data import synthetic_mnist  # noqa: E402

for H, n in [(4096, 800), (2048, 800)]:
    x, y = synthetic_mnist(2 * n + 64, seed=3)
    nn = NeuralNetwork([784, H, 10])
    e = MlpEngine(nn.H, dtype="f32", max_cols=n, device="cuda", path="split3")
    e.set_params(*nn.params)
    e.load_dataset(x, y)
    e.z2buf.fill_(float("nan"))
    e.run(64, n, 1.0 / n, 1e-4, 0.0, sgd=False, parts=5)
    torch.cuda.synchronize()
    bm = 128 if H == 4096 else 64
    tm = (H + bm - 1) // bm
    z = e.z2buf[: tm * 16 * e.ld].view(tm, 16, e.ld)[:, :10, :n].double()
    ref = e.W2.double() @ e.a1[:, :n].double()
    print(H, "nan tiles:", [int(torch.isnan(z[t]).any()) for t in range(tm)], flush=True)
    zs = torch.nan_to_num(z).sum(0)
    print(H, "rel", float((zs - ref).abs().max() / ref.abs().max()), flush=True)
    per = [(W2t := e.W2.double()[:, t * bm:(t + 1) * bm]) @ e.a1[t * bm:(t + 1) * bm, :n].double() for t in range(tm)]
    bad = [t for t in range(tm) if float((torch.nan_to_num(z[t]) - per[t]).abs().max()) > 1e-4]
    print(H, "bad tiles", bad[:40], flush=True)
    if bad:
        t = bad[0]
        d = (torch.nan_to_num(z[t]) - per[t]).abs()
        cols = (d.max(0).values > 1e-4).nonzero().flatten().tolist()
        print(H, "tile", t, "bad cols", cols[:20], "...", len(cols), flush=True)
