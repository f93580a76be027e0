"""CPU tests of the MLP: native fp64 oracle vs an independent PyTorch fp64
implementation, numerical gradients, checkpoints, data I/O (no GPU needed)."""
import os

import numpy as np
import pytest
import torch

from cme213_sp18_amd import NeuralNetwork
from cme213_sp18_amd.models import mlp
from cme213_sp18_amd.parallel import DataParallelTrainer, MlpEngine
from cme213_sp18_amd.utils import checkpoint as ck
from cme213_sp18_amd.utils.common import gradcheck, precision, rel_error
from cme213_sp18_amd.utils.data import label_to_y, split_train_dev, synthetic_mnist


def _torch_forward(nn, X, shift=True):
    W1, b1, W2, b2 = (torch.as_tensor(p) for p in nn.params)
    X = torch.as_tensor(np.asarray(X, np.float64))
    a1 = torch.sigmoid(X @ W1.t() + b1)
    z2 = a1 @ W2.t() + b2
    if shift:
        z2 = z2 - z2.max(1, keepdim=True).values
    e = torch.exp(z2)
    return a1, e / e.sum(1, keepdim=True)


def test_init_deterministic_and_shapes():
    a = NeuralNetwork([784, 100, 10])
    b = NeuralNetwork([784, 100, 10])
    assert a.W[0].shape == (100, 784) and a.W[1].shape == (10, 100)
    assert a.b[0].shape == (100,) and a.b[1].shape == (10,)
    np.testing.assert_array_equal(a.W[0], b.W[0])
    np.testing.assert_array_equal(a.W[1], b.W[1])
    assert np.all(a.b[0] == 0) and np.all(a.b[1] == 0)
    # 0.01 * N(0,1)
    assert 0.008 < a.W[0].std() < 0.012 and abs(a.W[0].mean()) < 1e-3
    # layer seeds differ (seed(i) per layer) -> W1's first entries are not W0's
    assert not np.allclose(a.W[0].T.ravel()[:10], a.W[1].T.ravel()[:10])


@pytest.mark.parametrize("shift", [True, False])
def test_feedforward_matches_torch(shift):
    x, _ = synthetic_mnist(300, seed=1)
    nn = NeuralNetwork([784, 50, 10])
    c = mlp.feedforward(nn, x / 255.0, shift=shift)
    a1, yc = _torch_forward(nn, x / 255.0, shift)
    np.testing.assert_allclose(c.a1, a1.numpy(), rtol=1e-13, atol=1e-15)
    np.testing.assert_allclose(c.yc, yc.numpy(), rtol=1e-12, atol=1e-15)


def test_backprop_matches_autograd():
    x, y = synthetic_mnist(200, seed=2)
    X = x / 255.0
    nn = NeuralNetwork([784, 30, 10])
    reg = 1e-3
    c = mlp.feedforward(nn, X)
    g = mlp.backprop(nn, y, reg, c)
    W1, b1, W2, b2 = (torch.tensor(p, requires_grad=True) for p in nn.params)
    Xt = torch.tensor(X)
    z2 = torch.sigmoid(Xt @ W1.t() + b1) @ W2.t() + b2
    loss = torch.nn.functional.cross_entropy(z2, torch.tensor(y, dtype=torch.long)) + 0.5 * reg * (
        (W1 ** 2).sum() + (W2 ** 2).sum())
    loss.backward()
    for mine, ref in ((g.dW[0], W1.grad), (g.dW[1], W2.grad), (g.db[0], b1.grad), (g.db[1], b2.grad)):
        np.testing.assert_allclose(mine, ref.numpy(), rtol=1e-10, atol=1e-14)
    assert abs(mlp.loss(nn, c.yc, y, reg) - loss.item()) < 1e-12


def test_numgrad_gradcheck_small_net():
    x, y = synthetic_mnist(40, seed=3)
    X = (x[:, :20] / 255.0)
    nn = NeuralNetwork([20, 6, 4])
    c = mlp.feedforward(nn, X)
    g = mlp.backprop(nn, y % 4, 1e-2, c)
    ng = mlp.numgrad(nn, X, y % 4, 1e-2)
    assert gradcheck(ng, g, threshold=1e-6)
    # a wrong gradient must FAIL (the reference's threshold of 1000 never did)
    g.dW[0] = g.dW[0] * 1.01
    assert not gradcheck(ng, g, threshold=1e-6)


def test_cpu_train_matches_torch_engine():
    x, y = synthetic_mnist(3000, seed=4)
    nn = NeuralNetwork([784, 32, 10])
    ref = nn.copy()
    losses = mlp.train(ref, x, y, 0.01, 1e-4, epochs=2, batch_size=800, print_every=2)
    assert len(losses) == 4  # 4 batches/epoch (last partial) x 2 epochs / 2
    t = DataParallelTrainer(nn.copy(), backend="torch", dtype="f64", device="cpu", batch_size=800)
    t.load(x, y)
    st = t.train(2, 0.01, 1e-4, print_every=2, log=lambda *_: None)
    assert st.steps == 8
    for i in range(2):
        assert rel_error(t.nn.W[i], ref.W[i]) < 1e-14
        assert rel_error(t.nn.b[i], ref.b[i]) < 1e-14
    np.testing.assert_allclose(st.losses, losses, rtol=1e-6)


def test_training_learns_synthetic_task():
    x, y = synthetic_mnist(6000, seed=5)
    xtr, ytr, xd, yd = split_train_dev(x, y)
    nn = NeuralNetwork([784, 32, 10])
    mlp.train(nn, xtr / 255.0, ytr, 0.5, 1e-4, epochs=3, batch_size=100)
    acc = precision(mlp.predict(nn, xd / 255.0), yd)
    assert acc > 0.9, acc


def test_engine_flat_layout_alignment():
    e = MlpEngine([784, 100, 10], dtype="f32", device="cpu", backend="torch")
    assert all(o % 64 == 0 for o in e.layout.offsets)
    assert e.W1.data_ptr() == e.params.data_ptr()
    assert e.layout.total >= 784 * 100 + 100 + 1000 + 10


def test_label_to_y_and_split():
    y = np.array([3, 0, 9, 3])
    Y = label_to_y(y)
    assert Y.shape == (10, 4) and Y.sum() == 4 and Y[3, 0] == 1 and Y[9, 2] == 1
    x = np.arange(20).reshape(10, 2)
    a, b, c, d = split_train_dev(x, np.arange(10))
    assert a.shape[0] == 9 and c.shape[0] == 1 and c[0, 0] == 18  # last 10% is dev (main.cpp:197-204)


def test_raw_ascii_format_and_roundtrip(tmp_path):
    a = np.array([[1.0, -2.5e-7, 3.14159265358979], [0.0, 123456.789, -1e-300]])
    p = tmp_path / "m.mat"
    ck.save_raw_ascii(str(p), a)
    lines = p.read_text().splitlines()
    assert len(lines) == 2
    assert lines[0] == " %20.12e %20.12e %20.12e" % tuple(a[0])
    back = ck.load_raw_ascii(str(p))
    np.testing.assert_allclose(back, a, rtol=1e-12)
    ck.save_raw_ascii(str(p), a, precision=17)
    np.testing.assert_array_equal(ck.load_raw_ascii(str(p)), a)
    v = np.arange(5.0)
    ck.save_raw_ascii(str(p), v)  # column vector: one value per line
    assert ck.load_raw_ascii(str(p)).shape == (5, 1)


def test_cpu_debug_snapshots_and_diff_report(tmp_path):
    x, y = synthetic_mnist(1700, seed=6)
    nn = NeuralNetwork([784, 20, 10])
    seq = nn.copy()
    mlp.train(seq, x, y, 0.01, 1e-4, epochs=2, batch_size=800, debug=True, outdir=str(tmp_path))
    files = sorted(os.listdir(tmp_path / "CPUmats"))
    # print_every <= 0 -> first batch of each epoch: iters 0 and 3 (3 batches/epoch)
    assert files == sorted(f"Sequential{n}-{i}.mat" for n in ("W0", "W1", "b0", "b1") for i in (0, 3))
    W0 = ck.load_raw_ascii(str(tmp_path / "CPUmats" / "SequentialW0-0.mat"))
    assert W0.shape == (20, 784)
    par = nn.copy()
    t = DataParallelTrainer(par, backend="torch", dtype="f64", device="cpu", batch_size=800)
    t.load(x, y)
    t.train(2, 0.01, 1e-4, debug=True, outdir=str(tmp_path))
    rep = (tmp_path / "CpuGpuDiff.txt").read_text().splitlines()
    assert rep[0].startswith("Iteration") and len(rep) == 3
    vals = [float(v) for v in rep[1].split()[1:]]
    assert max(vals) < 1e-9  # precision-12 snapshots vs exact fp64 params
    assert ck.checkNNErrors(seq, par, str(tmp_path / "NNErrors.txt"), verbose=False)


def test_checkpoint_resume_roundtrip(tmp_path):
    nn = NeuralNetwork([784, 16, 10])
    ck.save_checkpoint(nn, str(tmp_path / "c"), meta={"epoch": 3, "lr": 0.1})
    nn2, meta = ck.load_checkpoint(str(tmp_path / "c"))
    assert meta["epoch"] == 3 and meta["H"] == [784, 16, 10]
    for i in range(2):
        np.testing.assert_array_equal(nn.W[i], nn2.W[i])
    os.remove(tmp_path / "c" / "params.npz")  # raw_ascii (precision 17) path is exact too
    nn3, _ = ck.load_checkpoint(str(tmp_path / "c"))
    np.testing.assert_array_equal(nn.W[0], nn3.W[0])


def test_idx_reader_roundtrip(tmp_path):
    from cme213_sp18_amd._native import cpu

    x, y = synthetic_mnist(50, seed=8)
    cpu().write_idx_images(str(tmp_path / "train-images-idx3-ubyte"), x, 28, 28)
    cpu().write_idx_labels(str(tmp_path / "train-labels-idx1-ubyte"), y.astype(np.uint8))
    xi, r, c = cpu().read_idx_images(str(tmp_path / "train-images-idx3-ubyte"))
    assert (r, c) == (28, 28)
    np.testing.assert_array_equal(xi, x)
    np.testing.assert_array_equal(cpu().read_idx_labels(str(tmp_path / "train-labels-idx1-ubyte")), y)
    raw = (tmp_path / "train-images-idx3-ubyte").read_bytes()
    assert raw[:4] == bytes([0, 0, 8, 3])  # big-endian magic 2051


def test_save_label_format(tmp_path):
    from cme213_sp18_amd.utils.common import save_label

    save_label(str(tmp_path / "p.txt"), np.array([7, 2, 1, 0]))
    assert (tmp_path / "p.txt").read_text() == "7210"
