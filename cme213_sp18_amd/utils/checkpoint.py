"""Checkpoints and the CPU-vs-GPU diff protocol.

Reference behaviour (fpcode/neural_network.cpp:27-88, fpcode/utils/tests.cpp:17-75):
  * ``write_cpudata_tofile`` saves W0, W1, b0, b1 in Armadillo ``raw_ascii`` to
    ``Outputs/CPUmats/Sequential{W0,W1,b0,b1}-<iter>.mat`` (one matrix row per line).
  * ``write_diff_gpu_cpu`` reloads those and appends max-norm and L2 relative
    errors of the parallel network to ``Outputs/CpuGpuDiff.txt``.
  * ``checkNNErrors`` compares two final networks, lists elements differing by
    more than 1e-4 and flags max-norm relative error > 1e-7.

Layout (kept byte-compatible): W0 = W1 of the MLP (H x 784), W1 = W2 (10 x H),
b0 (H x 1), b1 (10 x 1); the native writer emits `` %20.12e`` per element
(Armadillo's raw_ascii stream setup: scientific, precision 12, width 20).
``precision=17`` switches to an exact fp64 round trip.

On top of that: ``save_checkpoint``/``load_checkpoint`` write the same four
files plus a JSON sidecar ``{epoch, iter, lr, reg, seed, H}`` for resume, and
an ``.npz`` fast path.  Only rank 0 writes; callers barrier afterwards.
"""
from __future__ import annotations

import json
import os

import numpy as np

from .._native import cpu

RAW_ASCII_PRECISION = 12
NN_ERROR_ELEM_TOL = 1e-4   # tests.cpp:32
NN_ERROR_MAX_REL = 1e-7    # tests.cpp:39

_NAMES = ("W0", "W1", "b0", "b1")


def save_raw_ascii(path: str, a, precision: int = RAW_ASCII_PRECISION) -> None:
    a = np.asarray(a, np.float64)
    if a.ndim == 1:
        a = a.reshape(-1, 1)
    cpu().save_raw_ascii(path, np.ascontiguousarray(a), precision)


def load_raw_ascii(path: str) -> np.ndarray:
    return cpu().load_raw_ascii(path)


def _mats(nn):
    return (nn.W[0], nn.W[1], nn.b[0].reshape(-1, 1), nn.b[1].reshape(-1, 1))


def write_cpudata_tofile(nn, it: int, outdir: str = "Outputs", precision: int = RAW_ASCII_PRECISION) -> None:
    d = os.path.join(outdir, "CPUmats")
    os.makedirs(d, exist_ok=True)
    for name, m in zip(_NAMES, _mats(nn)):
        save_raw_ascii(os.path.join(d, f"Sequential{name}-{it}.mat"), m, precision)


def _inf_norm(a) -> float:
    """Armadillo norm(X, "inf") = max row sum of |X| (vectors: max |x|)."""
    a = np.asarray(a, np.float64)
    if a.ndim == 1 or 1 in a.shape:
        return float(np.max(np.abs(a)))
    return float(np.max(np.sum(np.abs(a), axis=1)))


def _two_norm(a) -> float:
    """Armadillo norm(X, 2): spectral norm for matrices, Euclidean for vectors."""
    a = np.asarray(a, np.float64)
    if a.ndim == 1 or 1 in a.shape:
        return float(np.linalg.norm(a.ravel()))
    return float(np.linalg.norm(a, 2))


def _rel(num: float, den: float) -> float:
    return num / den if den != 0 else (0.0 if num == 0 else float("inf"))


def write_diff_gpu_cpu(nn, it: int, error_file, outdir: str = "Outputs") -> dict:
    """Append one row of max-norm / L2 relative errors vs the CPU snapshot of iteration ``it``."""
    d = os.path.join(outdir, "CPUmats")
    errs = {}
    for name, m in zip(_NAMES, _mats(nn)):
        ref = load_raw_ascii(os.path.join(d, f"Sequential{name}-{it}.mat"))
        diff = np.asarray(m) - ref
        errs[f"max_{name}"] = _rel(_inf_norm(diff), _inf_norm(ref))
        errs[f"l2_{name}"] = _rel(_two_norm(diff), _two_norm(ref))
    ow = 15
    if it == 0:
        hdr = ["Iteration"] + [f"Max Err {n}" for n in _NAMES] + [f"L2 Err {n}" for n in _NAMES]
        error_file.write("".join(h.ljust(ow) for h in hdr) + "\n")
    vals = [str(it)] + [f"{errs['max_' + n]:.6g}" for n in _NAMES] + [f"{errs['l2_' + n]:.6g}" for n in _NAMES]
    error_file.write("".join(v.ljust(ow) for v in vals) + "\n")
    error_file.flush()
    return errs


def check_errors(a, b, name: str, fh=None, elem_tol: float = NN_ERROR_ELEM_TOL) -> tuple[float, float]:
    """tests.cpp:17-49: list |a-b| > elem_tol, return (max-norm rel, L2 rel)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if fh is not None:
        bad = np.argwhere(np.abs(a - b) > elem_tol)
        for idx in bad[:1000]:
            fh.write(f"{name}{tuple(int(i) for i in idx)}: {a[tuple(idx)]} vs {b[tuple(idx)]}\n")
    diff = a - b
    return _rel(_inf_norm(diff), _inf_norm(b)), _rel(_two_norm(diff), _two_norm(b))


def checkNNErrors(seq_nn, par_nn, path: str = "Outputs/NNErrors.txt", verbose: bool = True) -> bool:
    """Compare a CPU (sequential) and a GPU (parallel) network; True when correct (tests.cpp:51-75)."""
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    ok = True
    with open(path, "w") as fh:
        rows = []
        for i in range(2):
            mw, lw = check_errors(par_nn.W[i], seq_nn.W[i], f"W[{i}]", fh)
            mb, lb = check_errors(par_nn.b[i], seq_nn.b[i], f"b[{i}]", fh)
            rows.append((i, mw, lw, mb, lb))
            ok &= mw <= NN_ERROR_MAX_REL and mb <= NN_ERROR_MAX_REL
    if verbose:
        print("Max norm of diff b/w seq and par: W[0]: %.6g, b[0]: %.6g" % (rows[0][1], rows[0][3]))
        print("l2  norm of diff b/w seq and par: W[0]: %.6g, b[0]: %.6g" % (rows[0][2], rows[0][4]))
        print("Max norm of diff b/w seq and par: W[1]: %.6g, b[1]: %.6g" % (rows[1][1], rows[1][3]))
        print("l2  norm of diff b/w seq and par: W[1]: %.6g, b[1]: %.6g" % (rows[1][2], rows[1][4]))
        if not ok:
            print("Correctness test failed")
    return bool(ok)


def save_checkpoint(nn, directory: str, meta: dict | None = None, precision: int = 17,
                    binary: bool = True) -> None:
    """Resume checkpoint: W0/W1/b0/b1 raw_ascii (exact fp64 by default) + JSON sidecar (+ .npz)."""
    os.makedirs(directory, exist_ok=True)
    for name, m in zip(_NAMES, _mats(nn)):
        save_raw_ascii(os.path.join(directory, f"{name}.mat"), m, precision)
    if binary:
        np.savez(os.path.join(directory, "params.npz"), W0=nn.W[0], W1=nn.W[1], b0=nn.b[0], b1=nn.b[1])
    m = dict(meta or {})
    m["H"] = list(nn.H)
    with open(os.path.join(directory, "meta.json"), "w") as f:
        json.dump(m, f, indent=1, sort_keys=True)


def load_checkpoint(directory: str):
    """Returns (NeuralNetwork, meta).  Uses the .npz fast path when present (allow_pickle=False)."""
    from ..models.mlp import NeuralNetwork

    with open(os.path.join(directory, "meta.json")) as f:
        meta = json.load(f)
    nn = NeuralNetwork(meta["H"], init=False)
    npz = os.path.join(directory, "params.npz")
    if os.path.exists(npz):
        with np.load(npz, allow_pickle=False) as z:
            nn.W[0][...] = z["W0"]
            nn.W[1][...] = z["W1"]
            nn.b[0][...] = z["b0"]
            nn.b[1][...] = z["b1"]
    else:
        nn.W[0][...] = load_raw_ascii(os.path.join(directory, "W0.mat"))
        nn.W[1][...] = load_raw_ascii(os.path.join(directory, "W1.mat"))
        nn.b[0][...] = load_raw_ascii(os.path.join(directory, "b0.mat")).ravel()
        nn.b[1][...] = load_raw_ascii(os.path.join(directory, "b1.mat")).ravel()
    return nn, meta
