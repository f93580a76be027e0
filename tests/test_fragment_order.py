"""The forward's fragment-ordered pixel copy (MlpEngine.load_dataset -> engine.fragment_order_pixels) holds every
pixel where the kernel's xs_off (csrc/mlp/mma_tile.h) looks for it, and zeros in the padding.  CPU only."""
import torch

from cme213_sp18_amd.parallel.engine import fragment_order_pixels


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
