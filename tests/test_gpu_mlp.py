"""GPU numerics of the gfx950 MLP kernels vs plain PyTorch / the fp64 oracle.

Every HIP kernel is compared against a PyTorch fp64 (or fp32) reference of the
same op, on shapes from the reference's call sites plus ragged
edges.  Tolerances: f64 1e-12 (fpcode/utils/tests.cpp:13), f32 ~1e-5 rel,
bf16 ~2e-2 rel.
"""
import numpy as np
import pytest
import torch

from cme213_sp18_amd import NeuralNetwork
from cme213_sp18_amd._native import hip
from cme213_sp18_amd.models import mlp as cpu_mlp
from cme213_sp18_amd.parallel import DataParallelTrainer, MlpEngine
from cme213_sp18_amd.utils.data import synthetic_mnist

pytestmark = pytest.mark.gpu

DT = {"f32": (0, torch.float32), "f64": (1, torch.float64), "bf16": (2, torch.bfloat16)}


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _rel(a, b):
    a = a.double()
    b = b.double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-300))


@pytest.mark.parametrize("dt", ["f64", "f32", "bf16"])
@pytest.mark.parametrize("tA,tB", [(False, False), (True, False), (False, True), (True, True)])
@pytest.mark.parametrize("M,N,K", [(100, 200, 784), (10, 100, 200), (100, 784, 200), (33, 17, 10), (1, 1, 1),
                                   (800, 1000, 784), (800, 10, 1000)])
def test_gemm_all_ops(dt, tA, tB, M, N, K):
    code, tdt = DT[dt]
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N * 3 + K)
    A = torch.randn((K, M) if tA else (M, K), generator=g, dtype=torch.float64)
    B = torch.randn((N, K) if tB else (K, N), generator=g, dtype=torch.float64)
    C = torch.randn(M, N, generator=g, dtype=torch.float64)
    alpha, beta = 2.0, 5.0  # fpcode/utils/tests.cpp:169
    Ad, Bd = A.to(tdt), B.to(tdt)
    opA = Ad.double().t() if tA else Ad.double()
    opB = Bd.double().t() if tB else Bd.double()
    ref = alpha * opA @ opB + beta * C.to(tdt).double()
    # column-major device buffers: a row-major (r x c) tensor's transpose storage
    Acm = Ad.t().contiguous().cuda()
    Bcm = Bd.t().contiguous().cuda()
    Ccm = C.to(tdt).t().contiguous().cuda()
    lda = Ad.shape[0]
    ldb = Bd.shape[0]
    hip().gemm(code, tA, tB, M, N, K, alpha, Acm.data_ptr(), lda, Bcm.data_ptr(), ldb, beta, Ccm.data_ptr(), M,
               _stream())
    out = Ccm.t().double().cpu()
    tol = {"f64": 1e-12, "f32": 2e-6, "bf16": 2e-2}[dt]
    assert _rel(out, ref) < tol * max(1.0, K ** 0.5 / 8)


@pytest.mark.parametrize("dt", ["f64", "f32", "bf16"])
@pytest.mark.parametrize("H,n", [(100, 800), (100, 100), (1024, 200), (37, 45)])
def test_forward1_bias_sigmoid(dt, H, n):
    code, tdt = DT[dt]
    P = 784
    pdt = torch.float64 if dt == "f64" else torch.float32
    g = torch.Generator().manual_seed(H + n)
    W = (0.01 * torch.randn(H, P, generator=g, dtype=torch.float64)).to(tdt)
    X = torch.randint(0, 256, (n, P), generator=g).to(tdt)
    b = torch.randn(H, generator=g, dtype=torch.float64).to(pdt)
    ld = (n + 15) // 16 * 16
    a1 = torch.zeros(H, ld, dtype=pdt, device="cuda")
    Wd, Xd, bd = W.cuda(), X.cuda(), b.cuda()
    hip().mlp_forward1(code, Wd.data_ptr(), bd.data_ptr(), Xd.data_ptr(), P, H, n, a1.data_ptr(), ld, 1, _stream())
    ref = torch.sigmoid(W.double() @ X.double().t() + b.double()[:, None])
    # f32: |z| ~ 30 from raw 0-255 pixels; fp32 accumulation over K=784 -> ~1e-5 abs in sigmoid
    tol = {"f64": 1e-12, "f32": 1e-4, "bf16": 1e-4}[dt]
    assert (a1[:, :n].double().cpu() - ref).abs().max().item() < tol


def _engine_pair(dt, H=100, n=800, N=1600):
    x, y = synthetic_mnist(N, seed=3)
    nn = NeuralNetwork([784, H, 10])
    engines = []
    for backend in ("hip", "torch"):
        e = MlpEngine(nn.H, dtype=dt, max_cols=n, device="cuda", backend=backend)
        e.set_params(*nn.params)
        e.load_dataset(x, y)
        engines.append(e)
    return engines


@pytest.mark.parametrize("dt", ["f64", "f32", "bf16"])
@pytest.mark.parametrize("n", [800, 100, 37])
def test_step_gradients_match_torch(dt, n):
    hipe, te = _engine_pair(dt, n=max(n, 16))
    scale, reg = 1.0 / n, 1e-4
    for e in (hipe, te):
        e.run(64, n, scale, reg, 0.0, sgd=False, with_loss=True)
    torch.cuda.synchronize()
    tol = {"f64": 1e-11, "f32": 2e-4, "bf16": 3e-2}[dt]
    for name in ("gW1", "gb1", "gW2", "gb2"):
        assert _rel(getattr(hipe, name), getattr(te, name)) < tol, name
    assert abs(hipe.loss_sum() - te.loss_sum()) / te.loss_sum() < 1e-4
    for name in ("a1", "dZ1", "D"):
        a = getattr(hipe, name)[:, :n]
        b = getattr(te, name)[:, :n]
        assert _rel(a, b) < max(tol, 1e-5), name


@pytest.mark.parametrize("dt", ["f64", "f32", "bf16"])
def test_fused_sgd_matches_torch(dt):
    hipe, te = _engine_pair(dt)
    for it in range(5):
        for e in (hipe, te):
            e.run(800 * (it % 2), 800, 1 / 800, 1e-4, 0.01, sgd=True)
    torch.cuda.synchronize()
    tol = {"f64": 1e-11, "f32": 1e-5, "bf16": 1e-2}[dt]
    assert _rel(hipe.params, te.params) < tol


def test_predict_matches_cpu_oracle():
    x, y = synthetic_mnist(3000, seed=5)
    nn = NeuralNetwork([784, 100, 10])
    e = MlpEngine(nn.H, dtype="f64", max_cols=800, device="cuda")
    e.set_params(*nn.params)
    pg = e.predict(x)
    pc = cpu_mlp.predict(nn, x)
    assert (pg == pc).mean() > 0.999


@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_graph_replay_equals_eager(dt):
    x, y = synthetic_mnist(4000, seed=2)
    nn = NeuralNetwork([784, 100, 10])
    a = DataParallelTrainer(nn.copy(), dtype=dt, use_graphs=True)
    b = DataParallelTrainer(nn.copy(), dtype=dt, use_graphs=False)
    for t in (a, b):
        t.load(x, y)
        t.train(2, 0.01, 1e-4)
    for i in range(2):
        np.testing.assert_array_equal(a.nn.W[i], b.nn.W[i])
        np.testing.assert_array_equal(a.nn.b[i], b.nn.b[i])


def test_gpu_f64_matches_cpu_oracle_reference_threshold():
    """Grade-preset-style check: GPU fp64 training vs the fp64 CPU oracle, max-norm rel <= 1e-7
    (fpcode/utils/tests.cpp:39)."""
    from cme213_sp18_amd.utils.checkpoint import checkNNErrors
    x, y = synthetic_mnist(8000, seed=7)
    nn = NeuralNetwork([784, 100, 10])
    seq = nn.copy()
    cpu_mlp.train(seq, x, y, 0.025, 1e-4, epochs=1, batch_size=800)
    par = nn.copy()
    t = DataParallelTrainer(par, dtype="f64")
    t.load(x, y)
    t.train(1, 0.025, 1e-4)
    assert checkNNErrors(seq, par, "/tmp/cme_nnerrors.txt", verbose=False)


def test_gpu_f32_close_to_cpu_oracle():
    x, y = synthetic_mnist(8000, seed=7)
    nn = NeuralNetwork([784, 100, 10])
    seq = nn.copy()
    cpu_mlp.train(seq, x, y, 0.01, 1e-4, epochs=2, batch_size=800)
    par = nn.copy()
    t = DataParallelTrainer(par, dtype="f32")
    t.load(x, y)
    t.train(2, 0.01, 1e-4)
    for i in range(2):
        assert np.abs(par.W[i] - seq.W[i]).max() / np.abs(seq.W[i]).max() < 1e-4
