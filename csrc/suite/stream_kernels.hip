// hw2 (shift cipher, PageRank) and hw1 (even/odd sum) on gfx950.
#include <algorithm>

#include "../common/hip_common.h"
#include "suite_kernels.h"

namespace cme::suite {

namespace {

// SWAR byte-wise add of the same byte `s` to every byte of `a` (mod 256 per byte,
// no carry between bytes).
__device__ __forceinline__ uint32_t add_bytes(uint32_t a, uint32_t sx) {
  return ((a & 0x7f7f7f7fu) + (sx & 0x7f7f7f7fu)) ^ ((a ^ sx) & 0x80808080u);
}

__global__ void shift_u8_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, int64_t n, uint8_t s) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = in[i] + s;
}

template <int W>  // bytes per lane: 4, 8, 16
__global__ void shift_wide_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, int64_t n, uint8_t s) {
  constexpr int WORDS = W / 4;
  const uint32_t sx = 0x01010101u * s;
  const int64_t lanes = n / W;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t i = t0; i < lanes; i += stride) {
    uint32_t w[WORDS];
    __builtin_memcpy(w, in + i * W, W);
#pragma unroll
    for (int q = 0; q < WORDS; ++q) w[q] = add_bytes(w[q], sx);
    __builtin_memcpy(out + i * W, w, W);
  }
  // tail (< W bytes) by the first threads
  const int64_t tail = lanes * W;
  if (t0 < n - tail) out[tail + t0] = in[tail + t0] + s;
}

// ---------------------------------------------------------------- PageRank
template <int LPN>  // lanes per node: 1 (thread per node) .. 64 (wave per node)
__global__ void pagerank_kernel(const uint32_t* __restrict__ indptr, const uint32_t* __restrict__ edges,
                                const float* __restrict__ in, float* __restrict__ out,
                                const float* __restrict__ inv_deg, int n) {
  const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int sub = threadIdx.x % LPN;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x / LPN;
  const float base = 0.5f / (float)n;
  for (int64_t node = gt / LPN; node < n; node += stride) {
    const uint32_t b = indptr[node], e = indptr[node + 1];
    float sum = 0.f;
    for (uint32_t j = b + sub; j < e; j += LPN) {
      const uint32_t src = edges[j];
      sum += in[src] * inv_deg[src];
    }
    if constexpr (LPN > 1) {
#pragma unroll
      for (int o = LPN / 2; o > 0; o >>= 1) sum += __shfl_xor(sum, o, LPN);
    }
    if (sub == 0) out[node] = base + 0.5f * sum;
  }
}

// ---- PageRank, pre-multiplied gather operand (variant 3).  The pull kernel above gathers TWO random floats per
// edge, in[src] and inv_deg[src]: an 8 MB random working set at 1 M nodes, twice one XCD's 4 MB L2, so every
// other gather misses to the Infinity Cache (1 M nodes x degree 19: 478 GB/s on the reference's bytes model).
// Here each propagation also writes w_out[i] = out[i] * inv_deg[i] (a coalesced read and write), and the next
// one gathers w[src] alone: one random float per edge from a 4 MB array -- half the gathers, half the working
// set.  The streamed operands (row pointers, edge lists) are read non-temporally so they do not push w out of L2.
// LPN lanes per row; each lane keeps UNR edge loads, then UNR gathers, in flight per trip.  The product
// in[src] * inv_deg[src] is the same rounded fp32 value whether formed here or when gathered (the reference's
// host loop adds the rounded products too, hw2code/main_q2.cu:49-85).
template <typename T>
__device__ __forceinline__ T ld_nt(const T* p) {
  return __builtin_nontemporal_load(p);
}

__global__ __launch_bounds__(256) void pagerank_premul_kernel(const float* __restrict__ in,
                                                              const float* __restrict__ inv_deg,
                                                              float* __restrict__ w, int n) {
  const int stride = gridDim.x * blockDim.x;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) w[i] = in[i] * inv_deg[i];
}

template <int LPN, int UNR>
__global__ __launch_bounds__(256) void pagerank_w_kernel(const uint32_t* __restrict__ indptr,
                                                         const uint32_t* __restrict__ edges,
                                                         const float* __restrict__ w_in, float* __restrict__ out,
                                                         float* __restrict__ w_out,
                                                         const float* __restrict__ inv_deg, int n) {
  const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int sub = threadIdx.x % LPN;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x / LPN;
  const float base = 0.5f / (float)n;
  for (int64_t node = gt / LPN; node < n; node += stride) {
    const uint32_t b = ld_nt(indptr + node), e = ld_nt(indptr + node + 1);
    float sum = 0.f;
    for (uint32_t j0 = b + sub; j0 < e; j0 += LPN * UNR) {
      uint32_t src[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const uint32_t j = j0 + u * LPN;
        src[u] = j < e ? ld_nt(edges + j) : 0xFFFFFFFFu;
      }
      float v[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) v[u] = src[u] != 0xFFFFFFFFu ? w_in[src[u]] : 0.f;
#pragma unroll
      for (int u = 0; u < UNR; ++u) sum += v[u];  // (edge order per lane: j0, j0 + LPN, ...)
    }
    if constexpr (LPN > 1) {
#pragma unroll
      for (int o = LPN / 2; o > 0; o >>= 1) sum += __shfl_xor(sum, o, LPN);
    }
    if (sub == 0) {
      const float r = base + 0.5f * sum;
      out[node] = r;
      w_out[node] = r * inv_deg[node];
    }
  }
}

// ------------------------------------------------------------ even/odd sum
// Streaming reduction: every thread keeps UNR independent 16-byte loads in flight per iteration
// (contiguous chunk of the array per workgroup, coalesced across the wave) and accumulates the
// total and the odd sum (even = total - odd: one masked add per element instead of a branch);
// wave shuffles + one atomic per workgroup and value.
constexpr int kSumUnr = 4;

__global__ __launch_bounds__(256) void sum_even_odd_kernel(const uint32_t* __restrict__ v, int64_t n,
                                                           unsigned long long* __restrict__ sums) {
  unsigned long long tot = 0, odd = 0;
  const int64_t n4 = n / 4;
  const uint4* v4 = reinterpret_cast<const uint4*>(v);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (kSumUnr - 1) * stride < n4; i += kSumUnr * stride) {
    uint4 w[kSumUnr];
#pragma unroll
    for (int u = 0; u < kSumUnr; ++u) w[u] = v4[i + u * stride];
#pragma unroll
    for (int u = 0; u < kSumUnr; ++u) {
      const uint32_t x[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        tot += x[q];
        odd += x[q] & (0u - (x[q] & 1u));
      }
    }
  }
  for (; i < n4; i += stride) {
    const uint4 w = v4[i];
    const uint32_t x[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      tot += x[q];
      odd += x[q] & (0u - (x[q] & 1u));
    }
  }
  for (int64_t j = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
    tot += v[j];
    odd += v[j] & (0u - (v[j] & 1u));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    tot += __shfl_xor(tot, off, 64);
    odd += __shfl_xor(odd, off, 64);
  }
  __shared__ unsigned long long part[2][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    part[0][wave] = tot;
    part[1][wave] = odd;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t = part[0][0] + part[0][1] + part[0][2] + part[0][3];
    const unsigned long long o = part[1][0] + part[1][1] + part[1][2] + part[1][3];
    atomicAdd(&sums[0], t - o);
    atomicAdd(&sums[1], o);
  }
}

}  // namespace

void shift_bytes(const uint8_t* in, uint8_t* out, int64_t n, uint8_t shift, int width, int block, int grid_cap,
                 hipStream_t s) {
  if (n <= 0) return;
  CME_REQUIRE(block > 0 && block % 64 == 0 && block <= 1024, "shift_bytes: block must be a multiple of 64");
  const int64_t lanes = width == 1 ? n : n / width;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((lanes + block - 1) / block, grid_cap));
  switch (width) {
    case 1: shift_u8_kernel<<<grid, block, 0, s>>>(in, out, n, shift); break;
    case 4: shift_wide_kernel<4><<<grid, block, 0, s>>>(in, out, n, shift); break;
    case 8: shift_wide_kernel<8><<<grid, block, 0, s>>>(in, out, n, shift); break;
    case 16: shift_wide_kernel<16><<<grid, block, 0, s>>>(in, out, n, shift); break;
    default: CME_REQUIRE(false, "shift_bytes: width must be 1, 4, 8 or 16");
  }
  CME_LAUNCH_CHECK(s);
}

void pagerank_propagate(const uint32_t* indptr, const uint32_t* edges, const float* in, float* out,
                        const float* inv_deg, int n, int variant, hipStream_t s) {
  if (n <= 0) return;
  if (variant == 2) variant = 0;  // auto: short rows (avg degree < ~32) favour one thread per node
  const int block = 256;
  if (variant == 0) {
    const int grid = std::min((n + block - 1) / block, 8192);
    pagerank_kernel<1><<<grid, block, 0, s>>>(indptr, edges, in, out, inv_deg, n);
  } else {
    const int grid = std::min((int)(((int64_t)n * 8 + block - 1) / block), 8192);
    pagerank_kernel<8><<<grid, block, 0, s>>>(indptr, edges, in, out, inv_deg, n);
  }
  CME_LAUNCH_CHECK(s);
}

void pagerank_premul(const float* in, const float* inv_deg, float* w, int n, hipStream_t s) {
  if (n <= 0) return;
  pagerank_premul_kernel<<<std::min((n + 255) / 256, 8192), 256, 0, s>>>(in, inv_deg, w, n);
  CME_LAUNCH_CHECK(s);
}

void pagerank_propagate_w(const uint32_t* indptr, const uint32_t* edges, const float* w_in, float* out, float* w_out,
                          const float* inv_deg, int n, int lpn, hipStream_t s) {
  if (n <= 0) return;
  const int block = 256;
  const int grid = (int)std::min<int64_t>(((int64_t)n * lpn + block - 1) / block, 16384);
  switch (lpn) {
    case 1: pagerank_w_kernel<1, 4><<<grid, block, 0, s>>>(indptr, edges, w_in, out, w_out, inv_deg, n); break;
    case 2: pagerank_w_kernel<2, 4><<<grid, block, 0, s>>>(indptr, edges, w_in, out, w_out, inv_deg, n); break;
    case 4: pagerank_w_kernel<4, 4><<<grid, block, 0, s>>>(indptr, edges, w_in, out, w_out, inv_deg, n); break;
    case 8: pagerank_w_kernel<8, 2><<<grid, block, 0, s>>>(indptr, edges, w_in, out, w_out, inv_deg, n); break;
    default: CME_REQUIRE(false, "pagerank_propagate_w: lanes per node must be 1, 2, 4 or 8");
  }
  CME_LAUNCH_CHECK(s);
}

void sum_even_odd(const uint32_t* v, int64_t n, unsigned long long* sums, hipStream_t s) {
  // (a self-resetting single-kernel form -- returning atomics + last-ticket publish, no memset -- measured
  // 54 us vs 42 us per call at 30M: the serial atomic round trips of the last workgroup cost more than
  // the memset node)
  HIP_CHECK(hipMemsetAsync(sums, 0, 2 * sizeof(unsigned long long), s));
  if (n <= 0) return;
  CME_REQUIRE((reinterpret_cast<uintptr_t>(v) & 15) == 0, "sum_even_odd: input must be 16-byte aligned");
  // 4 workgroups per CU, each thread kSumUnr 16-byte loads in flight
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (n / 4 + 256 * kSumUnr - 1) / (256 * kSumUnr)));
  sum_even_odd_kernel<<<grid, 256, 0, s>>>(v, n, sums);
  CME_LAUNCH_CHECK(s);
}

}  // namespace cme::suite
