"""GPU tests of the homework kernel suite: each HIP kernel against its CPU oracle."""
import numpy as np
import pytest
import torch

from cme213_sp18_amd.suite import hw1, hw2, hw3, hw4

pytestmark = pytest.mark.gpu

def _text(n=300_000):
    return hw4.read_text()[:n]  # the reference's Moby Dick, shipped as tests/fixtures/mobydick.txt.gz


# ------------------------------------------------------------------ hw1
@pytest.mark.parametrize("n", [1, 5, 1000, 30_000_000])
def test_sum_even_odd_gpu(n):
    v = hw1.init_sum_input(n, seed=n)
    got = hw1.sum_even_odd_gpu(torch.from_numpy(v.view(np.int32)).cuda()).cpu().tolist()
    assert tuple(got) == hw1.sum_even_odd_parallel(v)


def test_sum_even_odd_gpu_repeated_calls_rearm():
    """Back-to-back calls of different inputs (and an empty one)
    each return their own sums, into a preallocated output."""
    out = torch.empty(2, dtype=torch.int64, device="cuda")
    for n in (3, 1_000_003, 0, 77):
        v = hw1.init_sum_input(n, seed=n + 1) if n else np.zeros(0, np.uint32)
        got = hw1.sum_even_odd_gpu(torch.from_numpy(v.view(np.int32)).cuda(), out).cpu().tolist()
        assert tuple(got) == (hw1.sum_even_odd_parallel(v) if n else (0, 0))


@pytest.mark.parametrize("n", [1, 100, 4096, 4097, 40000, 1 << 22, 3_000_001])
def test_radix_sort_gpu(n):
    keys = np.random.default_rng(n).integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    d = torch.from_numpy(keys.view(np.int32)).cuda()
    out = hw1.radix_sort_gpu(d).cpu().numpy().view(np.uint32)
    assert np.array_equal(out, np.sort(keys))


def test_radix_pass_gpu_matches_golden_stage5():
    f = hw1.make_golden_fixtures()
    d = torch.from_numpy(f["input"].view(np.int32)).cuda()
    dst = torch.empty_like(d)
    srt = hw1.GpuRadixSorter(d.numel())
    srt.pass_(d, dst, 0)
    assert np.array_equal(dst.cpu().numpy().view(np.uint32), f["sorted"])


def test_radix_sort_gpu_few_distinct_keys():
    keys = (np.arange(1 << 20, dtype=np.uint32) % 3) << 24
    d = torch.from_numpy(keys.view(np.int32)).cuda()
    assert np.array_equal(hw1.radix_sort_gpu(d).cpu().numpy().view(np.uint32), np.sort(keys))


# ------------------------------------------------------------------ hw2
@pytest.mark.parametrize("width", hw2.SHIFT_WIDTHS)
@pytest.mark.parametrize("n", [1, 15, 16, 1000, 1_235_157])
def test_shift_gpu_exact_all_bytes(width, n):
    t = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8)  # full byte range: carries must not leak
    out = hw2.shift_gpu(torch.from_numpy(t).cuda(), 200, width).cpu().numpy()
    assert np.array_equal(out, hw2.shift_host(t, 200))


def test_shift_benchmark_runs():
    r = hw2.benchmark_shift(hw2.doubled_text(_text(100_000), 2), reps=2)
    assert set(r["gbps"]) == set(hw2.SHIFT_WIDTHS)


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
@pytest.mark.parametrize("nodes,edges", [(1000, 2), (1 << 15, 7), (1 << 17, 19), (1 << 20, 19), (4097, 4)])
def test_pagerank_gpu(variant, nodes, edges):
    g = hw2.generate_graph(nodes, edges, seed=nodes + edges)
    out = hw2.pagerank_gpu(g, 6, variant)
    assert hw2.check_pagerank(out, hw2.pagerank_host(g, 6)) == 0


# ------------------------------------------------------------------ hw3
@pytest.mark.parametrize("variant", ["global", "block", "shared", "vec", "shared2"])
@pytest.mark.parametrize("order", [2, 4, 8])
@pytest.mark.parametrize("shape", [(64, 64), (257, 131), (1000, 77), (1023, 5)])
def test_stencil_gpu(variant, order, shape):
    p = hw3.SimParams(shape[0], shape[1], 1.0, 1.0, 20, order)
    g0 = hw3.init_grid(p)
    ref = hw3.cpu_computation(g0, p)
    out, _ = hw3.gpu_computation(g0, p, variant)
    err = hw3.check_errors(ref, out)
    assert err["mismatches"] == 0, err


# ------------------------------------------------------------------ hw4
def test_sanitize_gpu_matches_host():
    t = _text()
    clean = hw4.sanitize(t)
    assert np.array_equal(clean.cpu().numpy(), hw4.sanitize_host(t))


def test_letter_frequency_gpu_vs_cpu():
    t = _text()
    g = hw4.letter_frequency_gpu(hw4.sanitize(t))
    c = hw4.letter_frequency_cpu(t)
    assert len(g) == len(c) == 5
    assert max(abs(a - b) for a, b in zip(g, c)) < 1e-14  # create_cipher.cu:200 eps


def test_byte_histogram_gpu():
    t = np.random.default_rng(3).integers(0, 256, 1_000_003, dtype=np.uint8)
    h = hw4.byte_histogram(torch.from_numpy(t).cuda()).cpu().numpy()
    assert np.array_equal(h, np.bincount(t, minlength=256))


def test_shifted_matches_gpu():
    t = np.random.default_rng(4).integers(97, 100, 50_000, dtype=np.uint8)
    m = hw4.shifted_matches(torch.from_numpy(t).cuda(), 1, 300)
    exp = [int(np.count_nonzero(t[:-s] == t[s:])) for s in range(1, 300)]
    assert m.tolist() == exp


@pytest.mark.parametrize("period", [1, 7, 64])
def test_residue_histogram_gpu(period):
    t = np.random.default_rng(period).integers(0, 256, 100_000, dtype=np.uint8)
    h = hw4.residue_histogram(torch.from_numpy(t).cuda(), period).cpu().numpy()
    exp = np.stack([np.bincount(t[r::period], minlength=256) for r in range(period)])
    assert np.array_equal(h, exp)


@pytest.mark.parametrize("wrap", [True, False])
@pytest.mark.parametrize("period", [4, 8, 11])
def test_cipher_roundtrip(period, wrap):
    t = _text(600_000)
    cipher, shifts, clean = hw4.create_cipher(t, period, wrap=wrap)
    assert np.array_equal(cipher.cpu().numpy(), hw4.vigenere_host(clean.cpu().numpy(), shifts, 1, wrap))
    plain, rec, k = hw4.solve_cipher(cipher, wrap=wrap)
    assert k == period
    assert np.array_equal(rec % 26, shifts % 26)
    assert torch.equal(plain, clean)


@pytest.mark.parametrize("variant", ["global", "block", "shared"])
@pytest.mark.parametrize("order", [2, 8])
def test_stencil_fused_bc_equals_two_launches(variant, order):
    p = hw3.SimParams(300, 211, 1.0, 1.0, 7, order)
    g0 = hw3.init_grid(p)
    a, _ = hw3.gpu_computation(g0, p, variant, fused=True)
    b, _ = hw3.gpu_computation(g0, p, variant, fused=False)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("iters", [1, 2, 7, 8])
@pytest.mark.parametrize("shape", [(9, 9), (248, 256), (249, 257), (1000, 77), (600, 600), (2100, 530)])
def test_stencil_two_steps_per_sweep_is_bitwise_two_launches(shape, iters):
    """The temporal-blocked LDS walk (two time steps per sweep, order 8: strips of 248 output columns over 256 of
    the intermediate grid, 64-row blocks reading 16 rows of halo) against the one-step LDS walk: the same bits,
    across strip and block edges, grids narrower than one strip, and an odd last step."""
    p = hw3.SimParams(shape[0], shape[1], 1.0, 1.0, iters, 8)
    g0 = hw3.init_grid(p)
    a, _ = hw3.gpu_computation(g0, p, "shared")
    b, _ = hw3.gpu_computation(g0, p, "shared2")
    assert np.array_equal(a, b)
