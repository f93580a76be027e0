"""The exact-split argument behind the split3 GEMMs, checked on the host in IEEE fp32 (numpy).

csrc/mlp/mma_tile.h `split_trunc` splits an fp32 value into three bf16 values by TRUNCATION:
hi = top 16 bits of x, r = x - hi, mid = top 16 bits of r, lo = r - mid.  The GEMMs rely on every step being
exact: hi + mid + lo == x bit for bit, and lo already a bf16 (its low 16 bits zero), so three bf16 MFMA
products against an exact bf16 operand (raw 0..255 pixels) reproduce the fp32 operand exactly.  The
round-to-nearest split the stored planes use (mlp_split.hip split_store) has the same property."""
import numpy as np


def _bits(a):
    return a.view(np.uint32)


def _f(b):
    return b.astype(np.uint32).view(np.float32)


def _trunc16(a):
    return _f(_bits(a) & np.uint32(0xFFFF0000))


def _rne_bf16(a):
    b = _bits(a).astype(np.uint64)
    b = (b + 0x7FFF + ((b >> 16) & 1)) & 0xFFFF0000
    return _f(b.astype(np.uint32))


def _values(n=200_000, seed=0):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal(n) * np.exp2(rng.integers(-40, 40, n))).astype(np.float32)
    # every mantissa pattern class: random bits with exponents well inside the normal range
    raw = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    raw = (raw & np.uint32(0x807FFFFF)) | (rng.integers(64, 190, n).astype(np.uint32) << 23)
    return np.concatenate([x, _f(raw), np.array([0.0, -0.0, 1.0, -1.0, 255.0, 1e-30, 3.4e38], np.float32)])


def test_truncation_split_is_exact():
    x = _values()
    hi = _trunc16(x)
    r = (x - hi).astype(np.float32)
    mid = _trunc16(r)
    lo = (r - mid).astype(np.float32)
    assert np.all(_bits(lo) & np.uint32(0xFFFF) == 0)  # lo is a bf16 as computed: no rounding in the pack
    recon = (hi.astype(np.float64) + mid.astype(np.float64) + lo.astype(np.float64))
    assert np.array_equal(recon, x.astype(np.float64))


def test_round_to_nearest_split_is_exact():
    x = _values(seed=1)
    x = x[np.abs(x) < 3e38]  # (RNE of the largest finite values rounds up to inf)
    hi = _rne_bf16(x)
    r = (x - hi).astype(np.float32)
    mid = _rne_bf16(r)
    lo = (r - mid).astype(np.float32)
    assert np.all(_bits(lo) & np.uint32(0xFFFF) == 0)
    recon = (hi.astype(np.float64) + mid.astype(np.float64) + lo.astype(np.float64))
    assert np.array_equal(recon, x.astype(np.float64))


def test_products_with_pixels_are_exact_in_fp32():
    """Each plane times a 0..255 pixel is exact in fp32 (8 + 8 significant bits <= 24), so the bf16 MFMA's
    fp32 products carry no rounding; only the accumulation order differs from an fp32 GEMM."""
    x = _values(20_000, seed=2)
    x = x[(np.abs(x) < 1e30) & (np.abs(x) > 1e-30)]
    px = np.random.default_rng(3).integers(0, 256, x.size).astype(np.float32)
    for plane in (_trunc16(x), _trunc16((x - _trunc16(x)).astype(np.float32))):
        prod32 = (plane * px).astype(np.float32)
        assert np.array_equal(prod32.astype(np.float64), plane.astype(np.float64) * px.astype(np.float64))
