"""Datasets: synthetic MNIST-shaped data (default) and the MNIST IDX reader.

The reference loads MNIST from IDX files on rank 0 only and scatters column
slices every batch (fpcode/main.cpp:170-210, fpcode/utils/mnist.cpp:9-65,
fpcode/neural_network.cpp:460-481).  There is no network access here, so the
default is a deterministic synthetic set with MNIST's exact shape and value
range (28x28 uint8 pixels in [0, 255], 10 classes), generated identically on
every rank (no broadcast needed) and uploaded ONCE to each GPU.

Layout: images are ``[N][784]`` (one sample per row) == the reference's
784 x N column-major Armadillo matrix; labels are int32 ``[N]``.
"""
from __future__ import annotations

import dataclasses
import os

import numpy as np

NUM_TRAIN = 60000  # fpcode/main.cpp:21
NUM_TEST = 10000   # fpcode/main.cpp:24
IMAGE_SIZE = 784   # fpcode/main.cpp:22
NUM_CLASSES = 10   # fpcode/main.cpp:23
DEV_FRACTION = 0.1  # fpcode/main.cpp:197


@dataclasses.dataclass
class MnistSplit:
    x_train: np.ndarray  # uint8 [N_train][784]
    y_train: np.ndarray  # int32 [N_train]
    x_dev: np.ndarray
    y_dev: np.ndarray
    x_test: np.ndarray
    y_test: np.ndarray | None
    source: str

    @property
    def num_features(self) -> int:
        return int(self.x_train.shape[1])


def synthetic_mnist(n: int, seed: int = 0, num_classes: int = NUM_CLASSES, side: int = 28,
                    noise: float = 40.0) -> tuple[np.ndarray, np.ndarray]:
    """Deterministic MNIST-shaped data: class prototypes (smooth blobs) plus
    per-sample shifts and pixel noise, clipped to uint8 [0, 255].

    Learnable (a 784-100-10 MLP separates the classes) so accuracy numbers are
    meaningful, and cheap enough to regenerate on every rank.
    """
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:side, 0:side].astype(np.float32)
    protos = np.zeros((num_classes, side, side), np.float32)
    prng = np.random.default_rng(1234)  # prototypes fixed across seeds: same task, different samples
    for c in range(num_classes):
        for _ in range(3):
            cy, cx = prng.uniform(6, side - 6, size=2)
            sy, sx = prng.uniform(2.0, 5.0, size=2)
            protos[c] += np.exp(-((yy - cy) ** 2 / (2 * sy**2) + (xx - cx) ** 2 / (2 * sx**2)))
        protos[c] *= 255.0 / protos[c].max()
    labels = rng.integers(0, num_classes, size=n, dtype=np.int32)
    out = np.empty((n, side * side), np.uint8)
    chunk = 8192
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        lab = labels[s:e]
        img = protos[lab]
        dy, dx = rng.integers(-2, 3, size=(2, e - s))
        for k in range(e - s):  # small integer shifts (cheap roll per sample)
            img[k] = np.roll(img[k], (dy[k], dx[k]), axis=(0, 1))
        img = img + rng.normal(0.0, noise, size=img.shape).astype(np.float32)
        out[s:e] = np.clip(img, 0, 255).astype(np.uint8).reshape(e - s, -1)
    return out, labels


def split_train_dev(x: np.ndarray, y: np.ndarray, dev_fraction: float = DEV_FRACTION):
    """First (1-f)·N samples train, last f·N dev -- fpcode/main.cpp:197-204."""
    n = x.shape[0]
    dev = int(dev_fraction * n)
    return x[: n - dev], y[: n - dev], x[n - dev:], y[n - dev:]


def load_mnist_idx(data_dir: str, max_train: int = -1, max_test: int = -1) -> MnistSplit:
    from .._native import cpu

    c = cpu()
    x, _, _ = c.read_idx_images(os.path.join(data_dir, "train-images-idx3-ubyte"), max_train)
    y = c.read_idx_labels(os.path.join(data_dir, "train-labels-idx1-ubyte"), max_train).astype(np.int32)
    xt, _, _ = c.read_idx_images(os.path.join(data_dir, "t10k-images-idx3-ubyte"), max_test)
    lt = os.path.join(data_dir, "t10k-labels-idx1-ubyte")
    yt = c.read_idx_labels(lt, max_test).astype(np.int32) if os.path.exists(lt) else None
    xtr, ytr, xd, yd = split_train_dev(x, y)
    return MnistSplit(xtr, ytr, xd, yd, xt, yt, source=f"mnist:{data_dir}")


def load_synthetic(num_train: int = NUM_TRAIN, num_test: int = NUM_TEST, seed: int = 0) -> MnistSplit:
    x, y = synthetic_mnist(num_train + num_test, seed=seed)
    xtr, ytr, xd, yd = split_train_dev(x[:num_train], y[:num_train])
    return MnistSplit(xtr, ytr, xd, yd, x[num_train:], y[num_train:], source=f"synthetic(seed={seed})")


def load_dataset(kind: str = "synthetic", data_dir: str = "data", num_train: int = NUM_TRAIN,
                 num_test: int = NUM_TEST, seed: int = 0) -> MnistSplit:
    if kind == "mnist":
        return load_mnist_idx(data_dir, num_train, num_test)
    if kind == "synthetic":
        return load_synthetic(num_train, num_test, seed)
    raise ValueError(f"unknown dataset kind {kind!r} (expected 'synthetic' or 'mnist')")


def label_to_y(labels: np.ndarray, num_classes: int = NUM_CLASSES) -> np.ndarray:
    """One-hot C x N matrix (fpcode/utils/common.cpp:61-68)."""
    y = np.zeros((num_classes, labels.shape[0]), np.float64)
    y[labels.astype(np.int64), np.arange(labels.shape[0])] = 1.0
    return y
