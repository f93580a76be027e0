"""The fragment orders of the split kernels: the forward's pixel copy (MlpEngine.load_dataset -> engine.fragment_order_pixels) holds every
pixel where the kernel's xs_off (csrc/mlp/mma_tile.h) looks for it, and zeros in the padding.  CPU only."""
import torch

from cme213_sp18_amd.parallel.engine import fragment_order_pixels, fragment_rows_to_rowmajor


def xs_off(s, k, npair):  # mma_tile.h xs_off
    p, w = k >> 6, k & 63
    lane = (w >> 4) * 16 + (s & 15)
    return (((s >> 4) * npair + p) * 64 + lane) * 16 + (w & 15)


def test_fragment_order_pixels_matches_the_kernel_offsets():
    for n, P in ((37, 208), (48, 784), (5, 64)):
        x = torch.randint(1, 256, (n, P), dtype=torch.uint8, generator=torch.Generator().manual_seed(n))
        xs = fragment_order_pixels(x)
        npair = (P + 63) // 64
        assert xs.numel() == (n + 15) // 16 * 16 * npair * 64
        s = torch.arange(n).view(-1, 1).expand(n, P)
        k = torch.arange(P).view(1, -1).expand(n, P)
        idx = xs_off(s, k, npair)
        assert torch.equal(xs[idx], x)
        pad = torch.ones_like(xs, dtype=torch.bool)
        pad[idx.reshape(-1)] = False
        assert int(xs[pad].count_nonzero()) == 0


def w1s_off(row, col, npair):  # mma_tile.h w1s_off (fp32 W1 copy, fragment-ordered dZ1)
    rt, c, p, w = row >> 4, row & 15, col >> 6, col & 63
    lane, i, e = (w >> 4) * 16 + c, (w & 15) >> 2, w & 3
    return (((rt * npair + p) * 4 + i) * 64 + lane) * 4 + e


def test_fragment_rows_to_rowmajor_inverts_w1s_off():
    for rows, cols in ((100, 800), (37, 96), (128, 784)):
        npair = (cols + 63) // 64
        src = torch.randn(rows, cols, dtype=torch.float64, generator=torch.Generator().manual_seed(rows))
        buf = torch.zeros((rows + 15) // 16 * 16 * npair * 64, dtype=torch.float64)
        r = torch.arange(rows).view(-1, 1).expand(rows, cols)
        c = torch.arange(cols).view(1, -1).expand(rows, cols)
        buf[w1s_off(r, c, npair).reshape(-1)] = src.reshape(-1)
        assert torch.equal(fragment_rows_to_rowmajor(buf, rows, cols), src)


def dzr_off(row, col, nst):  # rega_gemm.h dzr_off (the wide fp32 dZ1 in the A-in-registers K loop's order)
    kt, w = col >> 5, col & 31
    lane = (w >> 3) * 16 + (row & 15)
    return ((((row >> 4) * nst + kt) * 2 + ((w >> 2) & 1)) * 64 + lane) * 4 + (w & 3)


def test_fragment_rows_to_rowmajor_inverts_dzr_off():
    for rows, cols in ((512, 800), (37, 96), (100, 40)):
        nst = (cols + 31) // 32
        src = torch.randn(rows, cols, dtype=torch.float64, generator=torch.Generator().manual_seed(cols))
        buf = torch.zeros((rows + 15) // 16 * 16 * nst * 32, dtype=torch.float64)
        r = torch.arange(rows).view(-1, 1).expand(rows, cols)
        c = torch.arange(cols).view(1, -1).expand(rows, cols)
        buf[dzr_off(r, c, nst).reshape(-1)] = src.reshape(-1)
        assert torch.equal(fragment_rows_to_rowmajor(buf, rows, cols, 32), src)
