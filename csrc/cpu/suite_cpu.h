// Native CPU side of the homework suite: hw1 OpenMP algorithms and the host
// oracles of hw2/hw3 (reference: hw1code/main_q1.cpp, main_q2.cpp,
// hw2code/main_q2.cu:30-85, hw3code/main.cu:74-214).  No Python here; the
// bindings live in csrc/bindings_suite_cpu.cpp and the native test driver in
// csrc/tests/ links this file directly.
#pragma once
#include <cstdint>
#include <utility>
#include <vector>

namespace pybind11 {
class module_;
}

namespace cme::cpu {
void bind_suite_cpu(pybind11::module_& m);  // defined in bindings_suite_cpu.cpp
}

namespace cme::cpu::suite {

using u32vec = std::vector<uint32_t>;

// hw1 Q1: (sum of even values, sum of odd values)
std::pair<uint64_t, uint64_t> sum_even_odd_serial(const uint32_t* v, int64_t n);
std::pair<uint64_t, uint64_t> sum_even_odd_parallel(const uint32_t* v, int64_t n);

// hw1 Q2: the five stages of one parallel LSD pass (main_q2.cpp:26-117)
u32vec block_histograms(const uint32_t* keys, int64_t n, int num_blocks, int num_buckets, int start_bit,
                        int64_t block_size);
u32vec reduce_to_global(const u32vec& block_hist, int num_blocks, int num_buckets);
u32vec exclusive_scan(const u32vec& global_hist);
u32vec block_exscan(int num_buckets, int num_blocks, const u32vec& global_exscan, const u32vec& block_hist);
void populate(const u32vec& block_exscan, int num_blocks, int num_buckets, int start_bit, int64_t block_size,
              const uint32_t* keys, int64_t n, uint32_t* sorted);
void radix_parallel_pass(const uint32_t* keys, uint32_t* sorted, int64_t n, int num_bits, int start_bit,
                         int64_t block_size);
// full sorts: result in keys, tmp is n-element scratch
void radix_parallel(uint32_t* keys, uint32_t* tmp, int64_t n, int num_bits, int num_blocks);
void radix_serial(uint32_t* keys, uint32_t* tmp, int64_t n, int num_bits);
// the production OpenMP sort (8-bit digits, fused histograms, write-combined scatter; see suite_cpu.cpp)
void radix_parallel_lsd(uint32_t* keys, uint32_t* tmp, int64_t n);
// std::sort of the same keys (the reference's baseline, hw1code/main_q2.cpp:249-256)
void std_sort(uint32_t* keys, int64_t n);

// hw3: `iters` steps of next.border = curr.border * bc_scale, next.interior = stencil(curr); grid [gy][gx]
void stencil_cpu(float* grid, int gx, int gy, int order, float xcfl, float ycfl, float bc_scale, int iters);

// hw2: `iters` PageRank propagations, ping-pong, result in vals
void pagerank_cpu(const uint32_t* indptr, const uint32_t* edges, const float* inv, float* vals, int n, int iters);

}  // namespace cme::cpu::suite
