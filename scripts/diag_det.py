"""Determinism diagnostics: graph vs eager, repeated runs, role-overlap on/off (prints max |diff|)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cme213_sp18_amd import NeuralNetwork
from cme213_sp18_amd.parallel import DataParallelTrainer
from cme213_sp18_amd.utils.data import synthetic_mnist


def run(graphs, epochs=2, steps=None):
    x, y = synthetic_mnist(4000, seed=2)
    nn = NeuralNetwork([784, 100, 10])
    t = DataParallelTrainer(nn, dtype="f32", use_graphs=graphs)
    t.load(x, y)
    t.train(epochs, 0.01, 1e-4)
    return np.concatenate([w.ravel() for w in nn.W] + [b.ravel() for b in nn.b])


def d(a, b):
    return float(np.abs(a - b).max())


g1, g2, e1, e2 = run(True), run(True), run(False), run(False)
print("overlap", os.environ.get("CME_NO_ROLE_OVERLAP") != "1")
print("graph-graph", d(g1, g2), "eager-eager", d(e1, e2), "graph-eager", d(g1, e1))
g1, e1 = run(True, 1), run(False, 1)
print("1 epoch graph-eager", d(g1, e1))
