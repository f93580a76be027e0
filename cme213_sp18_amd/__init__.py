"""cme213_sp18_amd -- an MI355X-native (gfx950) framework with the capabilities of
the Stanford CME213 (Spring 2018) coursework: a 2-layer MLP training engine with
hand-written CDNA4 MFMA kernels and RCCL data parallelism, plus a HIP kernel
suite for the homework workloads (streaming cipher, PageRank, heat stencil,
radix sort, Vigenere cryptanalysis).

The package directory uses underscores (``cme213_sp18_amd``) because a Python
package name cannot contain ``-``.
"""
__version__ = "0.1.0"

from .models.mlp import NeuralNetwork, feedforward, backprop, loss, predict, numgrad, train  # noqa: F401
