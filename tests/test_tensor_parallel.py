"""Tensor parallelism over the hidden dimension (parallel/tensor_parallel.py) against single-process
full-model training: gloo world 2 (multi-process) and LoopbackComm world 4 (threads), fp64 torch ops."""
import threading

import numpy as np
import pytest
import torch

from cme213_sp18_amd import NeuralNetwork
from cme213_sp18_amd.parallel import DataParallelTrainer, LoopbackComm, TensorParallelTrainer
from cme213_sp18_amd.parallel.launcher import spawn
from cme213_sp18_amd.utils.data import synthetic_mnist

from .dist_workers import tp_train_worker


def _single(H, N, B, E, lr, reg):
    x, y = synthetic_mnist(N, seed=11)
    nn = NeuralNetwork([784, H, 10])
    tr = DataParallelTrainer(nn, device="cpu", dtype="f64", batch_size=B, backend="torch", use_graphs=False)
    tr.load(x, y)
    st = tr.train(E, lr, reg, print_every=2, log=lambda *_: None)
    return nn, st


def _close(a, b, tol=1e-11):
    return np.abs(a - b).max() <= tol * max(1.0, np.abs(b).max())


def test_gloo_tp_equals_single_process(tmp_path):
    H, N, B, E, lr, reg = 32, 2000, 800, 2, 0.05, 1e-3  # 800, 800, 400 (partial last batch)
    spawn(tp_train_worker, 2, args=(str(tmp_path), H, N, B, E, lr, reg, "f64"), backend="gloo")
    ref, st = _single(H, N, B, E, lr, reg)
    r0, r1 = (np.load(tmp_path / f"tp{r}.npz") for r in range(2))
    for k, w in (("W0", ref.W[0]), ("W1", ref.W[1]), ("b0", ref.b[0]), ("b1", ref.b[1])):
        np.testing.assert_array_equal(r0[k], r1[k])  # every rank gathers the same model
        assert _close(r0[k], w), k
    np.testing.assert_allclose(r0["losses"], st.losses, rtol=1e-9)
    np.testing.assert_array_equal(r0["pred"], r1["pred"])


def test_loopback_tp_world4_and_divisibility():
    H, N, B, E, lr, reg = 48, 1600, 800, 2, 0.1, 1e-4
    comms = LoopbackComm.create(4)
    x, y = synthetic_mnist(N, seed=11)
    nets = [NeuralNetwork([784, H, 10]) for _ in range(4)]
    errs = []

    def work(r):
        try:
            torch.set_num_threads(1)
            tr = TensorParallelTrainer(nets[r], comm=comms[r], device="cpu", dtype="f64", batch_size=B,
                                       backend="torch")
            assert tr.Hs == H // 4
            tr.load(x, y)
            tr.train(E, lr, reg)
        except Exception as ex:  # pragma: no cover - surfaced below
            errs.append(ex)

    ts = [threading.Thread(target=work, args=(r,)) for r in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    ref, _ = _single(H, N, B, E, lr, reg)
    for r in range(4):
        assert _close(nets[r].W[0], ref.W[0]) and _close(nets[r].W[1], ref.W[1])
        assert _close(nets[r].b[1], ref.b[1])
    with pytest.raises(ValueError):
        TensorParallelTrainer(NeuralNetwork([784, 30, 10]), comm=LoopbackComm.create(4)[0], device="cpu",
                              dtype="f64", backend="torch")


def test_cli_tensor_parallel_gloo(tmp_path):
    """python -m torch.distributed.run ... cme213_sp18_amd.train --parallel tp on 2 CPU ranks (gloo):
    trains, prints the loss, predicts on rank 0 only (no collective) and exits cleanly."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root)
    port = 29000 + (os.getpid() * 7) % 2000
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "cme213_sp18_amd.train",
                        "--parallel", "tp", "--preset", "cpu_plumbing", "-n", "16", "-e", "1", "-p", "1",
                        "--num-train", "1700", "--num-test", "100", "--outdir", str(tmp_path / "Outputs")],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "Loss at iteration 0" in r.stdout
    out = json.loads([line for line in r.stdout.splitlines() if line.startswith("{")][-1])
    assert out["allreduce"].startswith("z2 all-reduce") and 0.0 <= out["par_dev_precision"] <= 1.0
