"""CPU tests of the homework suite (hw1-hw4 capabilities): native OpenMP algorithms,
host oracles and the golden radix fixtures (hw1code/tests_q2.cpp:80-157)."""
import os

import numpy as np
import pytest

from cme213_sp18_amd.suite import hw1, hw2, hw3, hw4
from cme213_sp18_amd.utils.common import ulp_distance

REF_FIXTURES = "/root/reference/hw1code/test_files"


# ------------------------------------------------------------------ hw1
def test_sum_even_odd_serial_parallel_agree():
    v = hw1.init_sum_input(1_000_003)
    ev = int(v[v % 2 == 0].astype(np.uint64).sum())
    od = int(v[v % 2 == 1].astype(np.uint64).sum())
    assert hw1.sum_even_odd_serial(v) == (ev, od)
    assert hw1.sum_even_odd_parallel(v) == (ev, od)


def test_vector_file_roundtrip(tmp_path):
    v = hw1.glibc_rand(1000)
    hw1.write_vector(str(tmp_path / "v"), v)
    assert np.array_equal(hw1.read_vector(str(tmp_path / "v")), v)
    assert open(tmp_path / "v").readline().strip() == "1804289383"  # first rand() after srand(1)


@pytest.fixture(scope="module")
def golden():
    return hw1.make_golden_fixtures()


def test_golden_fixtures_match_reference_files(golden):
    ref = hw1.load_fixtures(REF_FIXTURES)
    if ref is None:
        pytest.skip("reference fixtures not present")
    for name in hw1.FIXTURE_NAMES:
        assert np.array_equal(golden[name], ref[name]), name


@pytest.mark.parametrize("stage", [1, 2, 3, 4, 5])
def test_radix_stage(stage, golden):
    """Test1..Test5 of tests_q2.cpp: each stage from the previous stage's golden output."""
    f = golden
    keys = f["input"]
    bs, nb = hw1.radix_geometry(len(keys), 8)
    if stage == 1:
        out, exp = hw1.compute_block_histograms(keys, nb, 256, 0, bs), f["blockhistograms"]
    elif stage == 2:
        out, exp = hw1.reduce_local_histo_to_global(f["blockhistograms"], nb, 256), f["globalhisto"]
    elif stage == 3:
        out, exp = hw1.scan_global_histo(f["globalhisto"]), f["globalhistoexscan"]
    elif stage == 4:
        out = hw1.compute_block_exscan_from_global_histo(256, nb, f["globalhistoexscan"], f["blockhistograms"])
        exp = f["blockexscan"]
    else:
        out = hw1.populate_output_from_block_exscan(f["blockexscan"], nb, 256, 0, bs, keys)
        exp = f["sorted"]
    assert np.array_equal(out, exp)


def test_stage5_is_stable_digit_partition(golden):
    s = golden["sorted"]
    d = s & 255
    assert np.all(np.diff(d.astype(np.int64)) >= 0)
    keys = golden["input"]
    exp = keys[np.argsort(keys & 255, kind="stable")]
    assert np.array_equal(s, exp)


@pytest.mark.parametrize("n", [0, 1, 7, 40000, 1 << 20])
@pytest.mark.parametrize("bits,blocks", [(8, 8), (4, 3), (16, 64), (8, 1)])
def test_radix_sort_parallel(n, bits, blocks):
    keys = hw1.glibc_rand(n, seed=n + 3) * np.uint32(3)  # spread into the top bit too
    assert np.array_equal(hw1.radix_sort_parallel(keys, bits, blocks), np.sort(keys))


@pytest.mark.parametrize("n", [0, 1, 7, 65535, 300_001])
def test_radix_sort_lsd_and_std_sort(n):
    keys = hw1.glibc_rand(n, seed=n + 5) * np.uint32(3)
    ref = np.sort(keys)
    assert np.array_equal(hw1.radix_sort_lsd(keys), ref)
    assert np.array_equal(hw1.std_sort(keys), ref)
    same = np.full(n, 7, np.uint32)  # every pass trivial (skipped)
    assert np.array_equal(hw1.radix_sort_lsd(same), same)


@pytest.mark.parametrize("bits", [4, 8, 11, 16])
def test_radix_sort_serial(bits):
    keys = np.random.default_rng(0).integers(0, 2**32, 100_001, dtype=np.uint64).astype(np.uint32)
    assert np.array_equal(hw1.radix_sort_serial(keys, bits), np.sort(keys))


# ------------------------------------------------------------------ hw2
def test_shift_host_wraps():
    t = np.arange(256, dtype=np.uint8)
    assert np.array_equal(hw2.shift_host(t, 3), ((np.arange(256) + 3) % 256).astype(np.uint8))


def test_doubled_text():
    t = b"abc"
    assert hw2.doubled_text(t, 2).tobytes() == b"abc" * 4


def _pagerank_numpy(g, iters):
    v = g.values.copy()
    src = np.repeat(np.arange(g.num_nodes), np.diff(g.indptr.astype(np.int64)))
    for _ in range(iters):
        contrib = (v[g.edges] * g.inv_deg[g.edges]).astype(np.float64)
        s = np.bincount(src, weights=contrib, minlength=g.num_nodes)
        v = (0.5 / g.num_nodes + 0.5 * s).astype(np.float32)
    return v


def test_generate_graph_ramp():
    g = hw2.generate_graph(1000, 4)
    deg = np.diff(g.indptr.astype(np.int64))
    assert deg[0] == 1 and deg.max() <= 2 * 4 - 1 and np.all(np.diff(deg) >= 0)
    assert np.allclose(g.inv_deg, 1.0 / deg)
    assert g.edges.max() < 1000


@pytest.mark.parametrize("iters", [1, 6, 7])
def test_pagerank_host(iters):
    g = hw2.generate_graph(5000, 5, seed=1)
    out = hw2.pagerank_host(g, iters)
    assert hw2.check_pagerank(out, _pagerank_numpy(g, iters)) == 0


def test_pagerank_bytes_model():
    assert hw2.pagerank_bytes(10, 3, 6) == 2 * 10 * 6 * 4 * 4 + 10 * 6 * 7 * 4


# ------------------------------------------------------------------ hw3
def _stencil_numpy(grid, p):
    b = p.border
    co = {2: [1, -2, 1], 4: [-1, 16, -30, 16, -1], 8: [-9, 128, -1008, 8064, -14350, 8064, -1008, 128, -9]}[p.order]
    cur = grid.astype(np.float64)
    for _ in range(p.iters):
        nxt = cur.copy() * p.bc_scale
        c = cur
        sx = sum(co[k + b] * c[b:-b, b + k:c.shape[1] - b + k] for k in range(-b, b + 1))
        sy = sum(co[k + b] * c[b + k:c.shape[0] - b + k, b:-b] for k in range(-b, b + 1))
        nxt[b:-b, b:-b] = c[b:-b, b:-b] + p.xcfl * sx + p.ycfl * sy
        cur = nxt
    return cur


def test_simparams_file(tmp_path):
    f = tmp_path / "params.in"
    f.write_text("4096 4096\n1 1\n400\n8\n")
    p = hw3.SimParams.from_file(str(f))
    assert (p.nx, p.ny, p.iters, p.order, p.border, p.gx) == (4096, 4096, 400, 8, 4, 4104)
    assert p.dx == pytest.approx(1 / 4103)
    assert p.dt == pytest.approx(0.49 * 5040 * p.dx**4 / (8064 * 2 * p.dx**2))
    assert p.xcfl == pytest.approx(p.dt / (5040 * p.dx**2))
    assert p.calc_bytes() == 400 * 4096 * 4096 * 18 * 4
    with pytest.raises(ValueError):
        hw3.SimParams(10, 10, 1, 1, 1, 3)


@pytest.mark.parametrize("order", [2, 4, 8])
def test_stencil_cpu_oracle(order):
    p = hw3.SimParams(61, 37, 1.0, 1.0, 5, order)
    g0 = hw3.init_grid(p)
    out = hw3.cpu_computation(g0, p)
    ref = _stencil_numpy(g0, p)
    assert out.shape == (p.gy, p.gx)
    np.testing.assert_allclose(out, ref, rtol=2e-5, atol=2e-6)
    err = hw3.check_errors(ref.astype(np.float32), out)
    assert err["l2err"] < 1e-5


def test_stencil_check_errors_counts():
    a = np.ones((4, 4), np.float32)
    b = a.copy()
    b[1, 1] = np.nextafter(np.float32(1), np.float32(2))
    b[2, 2] = 1.5
    e = hw3.check_errors(a, b)
    assert e["mismatches"] == 1 and e["linf"] == pytest.approx(0.5)
    assert int(ulp_distance(a, b)[1, 1]) == 1


# ------------------------------------------------------------------ hw4
def test_sanitize_and_frequency_host():
    t = b"Hello, World! EEE"
    assert hw4.sanitize_host(t).tobytes() == b"helloworldeee"
    f = hw4.letter_frequency_cpu(t)
    assert f[0] == pytest.approx(4 / 13) and len(f) == 5


@pytest.mark.parametrize("wrap", [True, False])
def test_vigenere_host_roundtrip(wrap):
    t = hw4.sanitize_host(b"the quick brown fox jumps over the lazy dog" * 3)
    sh = hw4.make_shifts(7)
    assert sh.min() >= 1 and sh.max() <= 25
    c = hw4.vigenere_host(t, sh, 1, wrap)
    if wrap:
        assert c.min() >= 97 and c.max() <= 122
    assert np.array_equal(hw4.vigenere_host(c, sh, -1, wrap), t)


def test_make_shifts_rejects_short_period():
    with pytest.raises(ValueError):
        hw4.make_shifts(3)


def test_synthetic_english_ioc_separates_period():
    t = hw4.sanitize_host(hw4.synthetic_english(200_000, seed=1))
    x = hw4.vigenere_host(t, hw4.make_shifts(6), 1, True)
    s = np.arange(4, 20)
    m = np.array([np.count_nonzero(x[:-k] == x[k:]) for k in s])
    ioc = hw4.index_of_coincidence(m, len(x), s)
    assert list(s[ioc > hw4.IOC_THRESHOLD]) == [6, 12, 18]


def test_moby_dick_fixture_and_period():
    """The shipped plaintext is the reference's mobydick.txt (1,235,150 bytes); the host Vigenere
    + kappa IoC pipeline on it recovers the period, as hw4code/solve_cipher.cu:75-109 does."""
    raw = hw4.read_text()
    assert len(raw) == 1_235_150 and raw.count(b"Ishmael") > 10
    t = hw4.sanitize_host(raw)
    x = hw4.vigenere_host(t, hw4.make_shifts(7), 1, True)
    s = np.arange(4, 16)
    m = np.array([np.count_nonzero(x[:-k] == x[k:]) for k in s])
    assert list(s[hw4.index_of_coincidence(m, len(x), s) > hw4.IOC_THRESHOLD]) == [7, 14]


def test_stencil_byte_models():
    """calcBytes (simParams.cpp:79-93) counts every tap; the compulsory model reads the grid and writes the
    interior once per iteration, so it is the smaller (and the one HBM bandwidth applies to)."""
    p = hw3.SimParams(256, 128, 1.0, 1.0, 10, 8)
    assert p.calc_bytes() == 10 * 256 * 128 * 18 * 4
    assert p.compulsory_bytes() == 10 * (p.gx * p.gy + 256 * 128) * 4
    assert p.compulsory_bytes() < p.calc_bytes()
