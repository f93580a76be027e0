"""hw1: even/odd sum and LSD radix sort (CPU OpenMP + gfx950).

Reference capabilities:
  * even/odd sum, serial and OpenMP            hw1code/main_q1.cpp:16-45
  * vector file I/O (one uint per line)          hw1code/tests_q1.cpp:8-38
  * serial radix sort                            hw1code/main_q2.cpp:174-218
  * OpenMP radix sort and its five stages        hw1code/main_q2.cpp:26-159
  * golden stage tests on test_files/            hw1code/tests_q2.cpp:80-157

The CPU algorithms live in the native ``_cpu.suite`` module; the GPU versions
(``sum_even_odd_gpu``, ``radix_sort_gpu``) are HIP kernels in
csrc/suite/stream_kernels.hip and csrc/suite/radix_cipher.hip.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ._dev import host, kernels, require_cuda, stream_handle

N_SUM = 30_000_000  # main_q1.cpp:14
RADIX_NUM_BITS = 8  # tests_q2.cpp: 8-bit digits, 8 blocks
RADIX_NUM_BLOCKS = 8


# ------------------------------------------------------------------ I/O
def read_vector(path: str) -> np.ndarray:
    """One unsigned int per line (tests_q1.cpp:8-24)."""
    return np.loadtxt(path, dtype=np.uint32, ndmin=1)


def write_vector(path: str, v) -> None:
    """One unsigned int per line (tests_q1.cpp:26-38)."""
    np.savetxt(path, np.asarray(v, np.uint32), fmt="%u")


def init_sum_input(n: int = N_SUM, seed: int = 0) -> np.ndarray:
    """uints uniform in [0, 100] (main_q1.cpp:47-57 uses std::default_random_engine; any
    fixed generator serves -- the test compares serial, OpenMP and GPU sums of the same data)."""
    return np.random.default_rng(seed).integers(0, 101, n, dtype=np.uint32)


def glibc_rand(n: int, seed: int = 1) -> np.ndarray:
    """The C library rand() stream after srand(seed) -- the generator behind the reference fixtures."""
    return host().glibc_rand(n, seed)


# ------------------------------------------------------------------ sums
def sum_even_odd_serial(v) -> tuple[int, int]:
    return tuple(int(x) for x in host().sum_even_odd(np.ascontiguousarray(v, np.uint32), False))


def sum_even_odd_parallel(v) -> tuple[int, int]:
    return tuple(int(x) for x in host().sum_even_odd(np.ascontiguousarray(v, np.uint32), True))


def sum_even_odd_gpu(v: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """(even_sum, odd_sum) as a uint64-valued int64 tensor of 2 (a zeroing memset node + one
    wave-reduction kernel).  ``out``: a preallocated int64 tensor of 2 (timed loops allocate nothing)."""
    require_cuda(v)
    if v.dtype not in (torch.int32, torch.uint32):
        raise TypeError("sum_even_odd_gpu: need a 32-bit integer tensor")
    if out is None:
        out = torch.empty(2, dtype=torch.int64, device=v.device)
    kernels().sum_even_odd(v.data_ptr(), v.numel(), out.data_ptr(), stream_handle())
    return out


# ------------------------------------------------------------------ radix (CPU)
def radix_sort_serial(keys, num_bits: int = 16) -> np.ndarray:
    return host().radix_sort_serial(np.ascontiguousarray(keys, np.uint32), num_bits)


def radix_sort_parallel(keys, num_bits: int = RADIX_NUM_BITS, num_blocks: int = RADIX_NUM_BLOCKS) -> np.ndarray:
    return host().radix_sort_parallel(np.ascontiguousarray(keys, np.uint32), num_bits, num_blocks)


def radix_sort_lsd(keys) -> np.ndarray:
    """The production OpenMP LSD sort (8-bit digits, one parallel region, write-combined scatter)."""
    return host().radix_sort_lsd(np.ascontiguousarray(keys, np.uint32))


def std_sort(keys) -> np.ndarray:
    """C++ std::sort of the keys: the reference's baseline (hw1code/main_q2.cpp:249-256)."""
    return host().std_sort(np.ascontiguousarray(keys, np.uint32))


def radix_geometry(n: int, num_blocks: int = RADIX_NUM_BLOCKS) -> tuple[int, int]:
    """(block_size, num_blocks) as the stage tests derive them: ``blockSize = n / 8``,
    ``numBlocks = ceil(n / blockSize)`` (tests_q2.cpp:84-85)."""
    bs = max(1, n // num_blocks)
    return bs, -(-n // bs)


def compute_block_histograms(keys, num_blocks, num_buckets, start_bit, block_size):
    keys = np.ascontiguousarray(keys, np.uint32)
    return host().block_histograms(keys, num_blocks, num_buckets, start_bit, block_size)


def reduce_local_histo_to_global(block_hist, num_blocks=RADIX_NUM_BLOCKS, num_buckets=1 << RADIX_NUM_BITS):
    return host().reduce_to_global(np.ascontiguousarray(block_hist, np.uint32), num_blocks, num_buckets)


def scan_global_histo(global_hist):
    return host().scan_global(np.ascontiguousarray(global_hist, np.uint32))


def compute_block_exscan_from_global_histo(num_buckets, num_blocks, global_exscan, block_hist):
    return host().block_exscan(num_buckets, num_blocks, np.ascontiguousarray(global_exscan, np.uint32),
                               np.ascontiguousarray(block_hist, np.uint32))


def populate_output_from_block_exscan(block_exscan, num_blocks, num_buckets, start_bit, block_size, keys):
    keys = np.ascontiguousarray(keys, np.uint32)
    return host().populate(np.ascontiguousarray(block_exscan, np.uint32), num_blocks, num_buckets, start_bit,
                           block_size, keys)


# ------------------------------------------------------------------ radix (GPU)
class GpuRadixSorter:
    """Stable LSD sort of uint32 keys (4 x 8-bit passes) with reusable scratch."""

    def __init__(self, capacity: int, device="cuda"):
        self.capacity = int(capacity)
        self.tmp = torch.empty(self.capacity, dtype=torch.int32, device=device)
        self.ws = torch.empty(max(1, kernels().radix_workspace_bytes(self.capacity)), dtype=torch.uint8,
                              device=device)

    def sort_(self, keys: torch.Tensor) -> torch.Tensor:
        require_cuda(keys)
        if keys.element_size() != 4 or keys.numel() > self.capacity:
            raise ValueError("GpuRadixSorter: 32-bit keys within capacity")
        kernels().radix_sort_u32(keys.data_ptr(), self.tmp.data_ptr(), keys.numel(), self.ws.data_ptr(),
                                 stream_handle())
        return keys

    def pass_(self, src: torch.Tensor, dst: torch.Tensor, start_bit: int) -> torch.Tensor:
        require_cuda(src, dst)
        kernels().radix_pass_u32(src.data_ptr(), dst.data_ptr(), src.numel(), start_bit, self.ws.data_ptr(),
                                 stream_handle())
        return dst


def radix_sort_gpu(keys: torch.Tensor) -> torch.Tensor:
    """Sort a copy of ``keys`` (int32 storage holding uint32 bit patterns)."""
    out = keys.clone()
    GpuRadixSorter(out.numel(), out.device).sort_(out)
    return out


# ------------------------------------------------------------------ golden fixtures
FIXTURE_NAMES = ("input", "blockhistograms", "globalhisto", "globalhistoexscan", "blockexscan", "sorted")


def make_golden_fixtures(n: int = 40000, num_bits: int = RADIX_NUM_BITS, num_blocks: int = RADIX_NUM_BLOCKS,
                         seed: int = 1) -> dict[str, np.ndarray]:
    """Stage outputs for the first pass (start_bit 0) on the C rand() keys, as in tests_q2.cpp:80-157."""
    keys = glibc_rand(n, seed)
    nb = 1 << num_bits
    bs, blocks = radix_geometry(n, num_blocks)
    bh = compute_block_histograms(keys, blocks, nb, 0, bs)
    g = reduce_local_histo_to_global(bh, blocks, nb)
    gs = scan_global_histo(g)
    bex = compute_block_exscan_from_global_histo(nb, blocks, gs, bh)
    return {"input": keys, "blockhistograms": bh, "globalhisto": g, "globalhistoexscan": gs,
            "blockexscan": bex, "sorted": populate_output_from_block_exscan(bex, blocks, nb, 0, bs, keys)}


def load_fixtures(directory: str) -> dict[str, np.ndarray] | None:
    """Read the reference's text fixtures (hw1code/test_files) if present."""
    if not all(os.path.exists(os.path.join(directory, f)) for f in FIXTURE_NAMES):
        return None
    return {f: read_vector(os.path.join(directory, f)) for f in FIXTURE_NAMES}
