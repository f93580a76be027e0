"""Model families: the 2-layer sigmoid/softmax MLP of the final project."""
from .mlp import NeuralNetwork, Cache, Grads, feedforward, backprop, loss, predict, numgrad, train  # noqa: F401
