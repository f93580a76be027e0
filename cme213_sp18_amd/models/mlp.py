"""The 2-layer MLP model (784-H-10, sigmoid hidden layer, softmax output).

Parity with the reference's ``class NeuralNetwork`` (fpcode/inc/neural_network.h:8-31):
  * ``H = [784, hidden, 10]``, ``W[i]`` is ``H[i+1] x H[i]``, ``b[i]`` has ``H[i+1]`` entries.
  * Init: layer i is seeded with ``i``, ``W[i] = 0.01 * randn``, ``b[i] = 0`` -- identical on every
    rank, so data-parallel replicas need no broadcast (native C++ init, see csrc/cpu/mlp_cpu.cpp).

Parameters are host float64 numpy arrays (the oracle's precision); GPU engines
copy them to device in their own dtype and write them back on ``sync``.
CPU math below (feedforward/backprop/loss/predict/numgrad/train) runs in the
native fp64 OpenMP runtime (``_cpu``): the reference's sequential trainer
(fpcode/neural_network.cpp:91-279).
"""
from __future__ import annotations

import dataclasses

import numpy as np

from .._native import cpu


class NeuralNetwork:
    num_layers = 2

    def __init__(self, H=(784, 100, 10), init: bool = True):
        H = [int(h) for h in H]
        if len(H) != 3:
            raise ValueError("NeuralNetwork is a 2-layer MLP: H must be [inputs, hidden, classes]")
        if H[2] > 16:
            raise ValueError("at most 16 output classes are supported by the fused softmax head")
        self.H = H
        self.W = [np.zeros((H[1], H[0])), np.zeros((H[2], H[1]))]
        self.b = [np.zeros(H[1]), np.zeros(H[2])]
        if init:
            cpu().init_params(self.W[0], self.b[0], self.W[1], self.b[1])

    # -- convenience -------------------------------------------------------
    @property
    def params(self):
        return self.W[0], self.b[0], self.W[1], self.b[1]

    def copy(self) -> "NeuralNetwork":
        nn = NeuralNetwork(self.H, init=False)
        for i in range(2):
            nn.W[i][...] = self.W[i]
            nn.b[i][...] = self.b[i]
        return nn

    def num_params(self) -> int:
        return sum(w.size for w in self.W) + sum(b.size for b in self.b)

    def __repr__(self) -> str:
        return f"NeuralNetwork(H={self.H})"


@dataclasses.dataclass
class Cache:
    """Forward cache (fpcode/utils/common.h:15-20): a1 [n][H], yc [n][C] (sample-major)."""
    X: np.ndarray
    a1: np.ndarray
    yc: np.ndarray


@dataclasses.dataclass
class Grads:
    dW: list
    db: list


def _x64(X) -> np.ndarray:
    return np.ascontiguousarray(X, dtype=np.float64)


def feedforward(nn: NeuralNetwork, X, shift: bool = True) -> Cache:
    """z1 = W1 x + b1; a1 = sigmoid(z1); z2 = W2 a1 + b2; yc = softmax(z2) per sample."""
    X = _x64(X)
    a1, yc = cpu().feedforward(*nn.params, X, shift)
    return Cache(X, a1, yc)


def backprop(nn: NeuralNetwork, labels, reg: float, cache: Cache, scale: float | None = None) -> Grads:
    """Gradients of the regularised cross-entropy (neural_network.cpp:123-139); scale = 1/N."""
    labels = np.ascontiguousarray(labels, dtype=np.int32)
    n = labels.shape[0]
    dW1, db1, dW2, db2 = cpu().backprop(*nn.params, cache.X, labels, float(reg), cache.a1, cache.yc,
                                        1.0 / n if scale is None else float(scale))
    return Grads([dW1, dW2], [db1, db2])


def loss(nn: NeuralNetwork, yc, labels, reg: float) -> float:
    return float(cpu().loss(*nn.params, np.ascontiguousarray(yc, np.float64),
                            np.ascontiguousarray(labels, np.int32), float(reg)))


def predict(nn: NeuralNetwork, X, shift: bool = True) -> np.ndarray:
    """argmax class per sample (neural_network.cpp:159-169)."""
    return cpu().predict(*nn.params, _x64(X), shift)


def numgrad(nn: NeuralNetwork, X, labels, reg: float, shift: bool = True) -> Grads:
    dW1, db1, dW2, db2 = cpu().numgrad(*nn.params, _x64(X), np.ascontiguousarray(labels, np.int32), float(reg),
                                       shift)
    return Grads([dW1, dW2], [db1, db2])


def train(nn: NeuralNetwork, X, labels, learning_rate: float, reg: float = 0.0, epochs: int = 15,
          batch_size: int = 800, grad_check: bool = False, print_every: int = -1, debug: bool = False,
          outdir: str = "Outputs", shift: bool = True, ckpt_precision: int = 12, iter0: int = 0) -> list[float]:
    """Sequential fp64 minibatch SGD on the CPU -- the oracle (neural_network.cpp:219-279).

    ``iter0``: the iteration counter at the start -- a resumed run continues the loss / snapshot numbering.

    ``grad_check`` runs a numerical gradient check on the first batch (the
    reference's threshold of 1000 made it a no-op; we assert a real bound).
    """
    X = _x64(X)
    labels = np.ascontiguousarray(labels, dtype=np.int32)
    if grad_check:
        from ..utils.common import gradcheck

        n = min(batch_size, X.shape[0])
        c = feedforward(nn, X[:n], shift)
        g = backprop(nn, labels[:n], reg, c)
        ng = numgrad(nn, X[:n], labels[:n], reg, shift)
        if not gradcheck(ng, g):
            raise AssertionError("gradient check failed")
    return list(cpu().train(*nn.params, X, labels, float(learning_rate), float(reg), int(epochs), int(batch_size),
                            int(print_every), bool(debug), outdir, shift, int(ckpt_precision), int(iter0)))
