// Wave-split-K MFMA tile engine for the small / skinny GEMMs of the MLP.
//
// Why this shape (MI355X-first, not a port of the reference's 32x32 shared-
// memory DGEMM, fpcode/gpu_func.cu:92-256):
//   * The MLP GEMMs are tiny (e.g. 100x800x784).  The whole step is ~0.26
//     GFLOP, so the limit is how many of the 1024 SIMDs get work, not tile
//     reuse.  We therefore give every wave its own K-slice of one small output
//     tile (KS waves per workgroup) and reduce the KS partial tiles through
//     LDS once at the end.  Operands go straight from global/L2 into VGPRs
//     (cdna_hip_programming.md §5, "GEMV / M <= 16" row): there is no
//     cross-wave reuse inside a workgroup, so an LDS round trip would be pure
//     overhead.
//   * One MFMA family per dtype, 16x16 output blocks:
//       f32  -> v_mfma_f32_16x16x4_f32   (exact f32, fmaf-chain numerics)
//       f64  -> v_mfma_f64_16x16x4_f64   (parity mode vs the fp64 reference)
//       bf16 -> v_mfma_f32_16x16x32_bf16 (f32 accumulate)
//   * K is permuted inside each 16-deep chunk so that each lane's four k
//     values are CONTIGUOUS in memory (lane group g owns k = kc+4g..kc+4g+3 and
//     instruction j consumes element j).  A K-contiguous operand is then one
//     16-byte load per lane per 4 MFMAs instead of four 4-byte loads.
//
// Lane map (l = lane, c = l & 15, g = l >> 4):
//   A operand: A(m0 + c, kc + V*g + j)     B operand: B(kc + V*g + j, n0 + c)
//   result   : C(m0 + row(g, i), n0 + c)    row = 4g+i (f32/bf16), g+4i (f64)
#pragma once

#include "../common/hip_common.h"

namespace cme {

template <typename T>
struct MmaTraits;

template <>
struct MmaTraits<float> {
  using in_t = float;
  using acc_t = float;
  using accv_t = f32x4;
  static constexpr int V = 4;   // contiguous k-elements per lane per chunk
  static constexpr int KC = 16; // k covered by one chunk (4 lane groups x V)
  __device__ static __forceinline__ void mma(const float (&a)[4], const float (&b)[4], accv_t& c) {
#pragma unroll
    for (int j = 0; j < 4; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], c, 0, 0, 0);
  }
  __device__ static __forceinline__ int row(int g, int i) { return 4 * g + i; }
};

template <>
struct MmaTraits<double> {
  using in_t = double;
  using acc_t = double;
  using accv_t = f64x4;
  static constexpr int V = 4;
  static constexpr int KC = 16;
  __device__ static __forceinline__ void mma(const double (&a)[4], const double (&b)[4], accv_t& c) {
#pragma unroll
    for (int j = 0; j < 4; ++j) c = __builtin_amdgcn_mfma_f64_16x16x4f64(a[j], b[j], c, 0, 0, 0);
  }
  // f64 MFMA C/D layout differs from every other dtype (cdna_hip_programming.md §3).
  __device__ static __forceinline__ int row(int g, int i) { return g + 4 * i; }
};

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

template <>
struct MmaTraits<__hip_bfloat16> {
  using in_t = __hip_bfloat16;
  using acc_t = float;
  using accv_t = f32x4;
  static constexpr int V = 8;
  static constexpr int KC = 32;
  __device__ static __forceinline__ void mma(const __hip_bfloat16 (&a)[8], const __hip_bfloat16 (&b)[8],
                                             accv_t& c) {
    bf16x8_t av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c, 0, 0, 0);
  }
  __device__ static __forceinline__ int row(int g, int i) { return 4 * g + i; }
};

template <typename T>
__device__ __forceinline__ T zero_val() { return T(0); }
template <>
__device__ __forceinline__ __hip_bfloat16 zero_val<__hip_bfloat16>() { return __float2bfloat16(0.f); }

// Operand loads go through BUFFER loads (cdna_hip_programming.md §5.5 T8):
// a wave-uniform 128-bit descriptor built from the kernel-argument pointer +
// a 32-bit per-lane byte offset.  Anything outside the operand (row >= rmax,
// k >= kend) gets the out-of-range offset kOOB and the hardware range check
// returns ZERO -- no branches, no clamping, no select.  (A guarded load, or a
// "load; ok ? v : 0" select that LLVM turns back into a guarded load, makes
// hipcc branch around every load and wait vmcnt(0) per element -- measured:
// a 10x100x800 dW2 took 17 us that way.)
constexpr int kOOB = 0x7FFFFFF0;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, kOOB, 0x00020000);
}

template <typename T>
__device__ __forceinline__ T buf_load1(__amdgpu_buffer_rsrc_t r, int off);
template <>
__device__ __forceinline__ float buf_load1<float>(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
template <>
__device__ __forceinline__ double buf_load1<double>(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
template <>
__device__ __forceinline__ __hip_bfloat16 buf_load1<__hip_bfloat16>(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(__hip_bfloat16, (unsigned short)__builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0));
}

// Load V logical elements X(r, k..k+V-1) of an operand stored either with k
// contiguous (KCONTIG: X[r*ld + k]) or r contiguous (X[k*ld + r]).
// VEC: 16-byte vector loads; the caller guarantees 16-byte alignment of every
// full vector and that kend is a multiple of V (a vector is fully in or out).
template <typename T, int V, bool KCONTIG, bool VEC>
__device__ __forceinline__ void load_frag(__amdgpu_buffer_rsrc_t rs, int ld, int r, int rmax, int k, int kend,
                                          T (&out)[V], int base_off = 0) {
  const bool rok = r < rmax;
  if constexpr (KCONTIG && VEC) {
    static_assert((V * sizeof(T)) % 16 == 0, "vector fragment must be a multiple of 16 B");
    const int off = (rok && k < kend) ? (r * ld + k) * (int)sizeof(T) + base_off : kOOB;
#pragma unroll
    for (int q = 0; q < (int)(V * sizeof(T) / 16); ++q) {
      const auto w = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 16 * q, 0);
      __builtin_memcpy(reinterpret_cast<char*>(out) + 16 * q, &w, 16);
    }
  } else {
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int kj = k + j;
      const int idx = KCONTIG ? r * ld + kj : kj * ld + r;
      out[j] = buf_load1<T>(rs, (rok && kj < kend) ? idx * (int)sizeof(T) + base_off : kOOB);
    }
  }
}

struct TileGeom {
  int M, N, K;
  int m0, n0;
};

// One workgroup = KS waves computing the (16*MB) x (16*NB) tile at (m0, n0)
// of C = A * B with K split across the waves.  On return, `epi(row, col, v)`
// has been called exactly once for every in-bounds element of the tile.
// `red` must point at >= KS*MB*NB*4*64 accumulators of LDS (unused if KS==1).
//
// NPA > 1: A is the exact sum of NPA planes stored `plane_bytes` apart
// (A = A_0 + A_1 + ...; the split-bf16 representation of an fp32 operand,
// see mlp_split.hip) and every plane is multiplied into the same accumulator.
template <typename T, int MB, int NB, int KS, bool AK, bool BK, bool VEC, int U, int NPA = 1, class Epi>
__device__ __forceinline__ void wsk_tile(const T* __restrict__ A, int lda, const T* __restrict__ B, int ldb,
                                         TileGeom g, Epi& epi,
                                         typename MmaTraits<T>::acc_t* __restrict__ red, int plane_bytes = 0) {
  using Tr = MmaTraits<T>;
  using accv_t = typename Tr::accv_t;
  using acc_t = typename Tr::acc_t;
  constexpr int V = Tr::V, KC = Tr::KC;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int c = lane & 15, grp = lane >> 4;

  accv_t acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = accv_t{0, 0, 0, 0};

  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(A), rsB = make_rsrc(B);
  const int nch = (g.K + KC - 1) / KC;
  const int cpw = (nch + KS - 1) / KS;
  const int kbeg = wave * cpw * KC;
  const int kend = min(g.K, (wave + 1) * cpw * KC);

  for (int kc = kbeg; kc < kend; kc += KC * U) {
    T af[U][NPA][MB][V];
    T bf[U][NB][V];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = kc + u * KC + V * grp;
#pragma unroll
      for (int p = 0; p < NPA; ++p)
#pragma unroll
        for (int i = 0; i < MB; ++i)
          load_frag<T, V, AK, VEC>(rsA, lda, g.m0 + 16 * i + c, g.M, k, kend, af[u][p][i], p * plane_bytes);
#pragma unroll
      for (int j = 0; j < NB; ++j)
        load_frag<T, V, BK, VEC>(rsB, ldb, g.n0 + 16 * j + c, g.N, k, kend, bf[u][j]);
    }
    // Keep every load of this burst ahead of the first MFMA: without the fence
    // the scheduler sinks each load next to its consumer to save VGPRs, which
    // turns the burst into U dependent memory round trips (measured: 25
    // vmcnt(0) waits per wave in fwd1).  With it: one wait ladder per burst.
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int p = 0; p < NPA; ++p)
#pragma unroll
        for (int i = 0; i < MB; ++i)
#pragma unroll
          for (int j = 0; j < NB; ++j) Tr::mma(af[u][p][i], bf[u][j], acc[i][j]);
  }

  if constexpr (KS == 1) {
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = g.m0 + 16 * i + Tr::row(grp, r);
          const int col = g.n0 + 16 * j + c;
          if (row < g.M && col < g.N) epi(row, col, acc[i][j][r]);
        }
  } else {
    constexpr int E = MB * NB * 4 * 64;  // accumulators per wave
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wave * E + (((i * NB + j) * 4 + r) << 6) + lane] = acc[i][j][r];
    __syncthreads();
    for (int e = threadIdx.x; e < E; e += 64 * KS) {
      acc_t s = red[e];
#pragma unroll
      for (int w = 1; w < KS; ++w) s += red[w * E + e];
      const int ln = e & 63, r = (e >> 6) & 3, blk = e >> 8;
      const int i = blk / NB, j = blk % NB;
      const int row = g.m0 + 16 * i + Tr::row(ln >> 4, r);
      const int col = g.n0 + 16 * j + (ln & 15);
      if (row < g.M && col < g.N) epi(row, col, s);
    }
    __syncthreads();  // `red` may be reused by the caller
  }
}

}  // namespace cme
