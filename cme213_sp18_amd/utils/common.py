"""Host-side helpers mirroring fpcode/utils/common.cpp and fpcode/utils/test_utils.h."""
from __future__ import annotations

import numpy as np

# The reference's MAX_REL_ERROR_THRESHOLD is 1000 (common.cpp:5), which accepts
# any gradient.  We keep its rel_error definition but default to a bound that
# actually detects a wrong gradient.
GRADCHECK_THRESHOLD = 1e-6
MAX_ULPS_DIFF = 512  # fpcode/utils/test_utils.h


def rel_error(a, b) -> float:
    """max |a-b| / max(1, |a|, |b|)  (common.cpp:23-30)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.maximum(np.abs(a), np.abs(b)))))


def gradcheck(g1, g2, threshold: float = GRADCHECK_THRESHOLD, verbose: bool = False) -> bool:
    """Compare two Grads (numerical vs analytical) layer by layer (common.cpp:33-56)."""
    ok = True
    for i in reversed(range(len(g1.dW))):
        e = rel_error(g1.dW[i], g2.dW[i])
        if verbose:
            print(f"dW[{i}] rel error: {e}")
        ok &= e <= threshold
    for i in reversed(range(len(g1.db))):
        e = rel_error(g1.db[i], g2.db[i])
        if verbose:
            print(f"db[{i}] rel error: {e}")
        ok &= e <= threshold
    return bool(ok)


def precision(pred, label) -> float:
    """Fraction of equal entries (common.cpp:78-80)."""
    pred = np.asarray(pred).ravel()
    label = np.asarray(label).ravel()
    return float(np.mean(pred.astype(np.int64) == label.astype(np.int64)))


def save_label(path: str, labels) -> None:
    """Digits concatenated without separator (common.cpp:82-94), via the native writer."""
    from .._native import cpu

    cpu().save_label(path, np.ascontiguousarray(labels, np.int32))


def relu(x):
    return np.maximum(x, 0)


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-np.asarray(x)))


def softmax_cols(z, shift: bool = True):
    """Column softmax of a C x N matrix (common.cpp:13-18 has no max shift)."""
    z = np.asarray(z, np.float64)
    if shift:
        z = z - z.max(axis=0, keepdims=True)
    e = np.exp(z)
    return e / e.sum(axis=0, keepdims=True)


def ulp_distance(a, b) -> np.ndarray:
    """Elementwise distance in units-in-the-last-place (test_utils.h:18-58)."""
    a = np.asarray(a)
    b = np.asarray(b)
    if a.dtype == np.float64:
        ia, ib = a.view(np.int64), b.view(np.int64)
        lim = np.int64(np.iinfo(np.int64).min)
    else:
        a = a.astype(np.float32)
        b = b.astype(np.float32)
        ia, ib = a.view(np.int32).astype(np.int64), b.view(np.int32).astype(np.int64)
        lim = np.int64(np.iinfo(np.int32).min)
    # map sign-magnitude to a monotonically ordered integer line
    ia = np.where(ia < 0, lim - ia, ia)
    ib = np.where(ib < 0, lim - ib, ib)
    return np.abs(ia - ib)


def almost_equal_ulps(a, b, max_ulps: int = MAX_ULPS_DIFF) -> bool:
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape:
        return False
    same_sign = np.signbit(a) == np.signbit(b)
    close = (ulp_distance(a, b) <= max_ulps) & same_sign
    close |= a == b  # +0 == -0
    return bool(np.all(close))
