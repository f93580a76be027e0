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

#include <type_traits>
#include <utility>

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
constexpr int kSc1 = 16;  // buffer cache-policy bit sc1: write-through stores / L1-bypassing loads

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
// CP: the loads' cache policy (kSc1: L1-bypassing, for an operand another workgroup of the launch rewrote)
template <typename T, int V, bool KCONTIG, int VEC, int CP = 0>
__device__ __forceinline__ void load_frag(__amdgpu_buffer_rsrc_t rs, int ld, int r, int rmax, int k, int kend,
                                          T (&out)[V], int base_off = 0) {
  // VEC == 1: 16-byte loads, every vector fully in or out (kend % V == 0)
  // VEC == 2: two 8-byte halves with separate range checks (kend % (V/2) == 0)
  // VEC == 0: element loads
  // VEC == 4: 16-byte loads with the tail past kend zeroed in registers (fp32)
  const bool rok = r < rmax;
  if constexpr (KCONTIG && VEC == 1) {
    static_assert((V * sizeof(T)) % 16 == 0, "vector fragment must be a multiple of 16 B");
    const int off = (rok && k < kend) ? (r * ld + k) * (int)sizeof(T) + base_off : kOOB;
#pragma unroll
    for (int q = 0; q < (int)(V * sizeof(T) / 16); ++q) {
      const auto w = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 16 * q, CP);
      __builtin_memcpy(reinterpret_cast<char*>(out) + 16 * q, &w, 16);
    }
  } else if constexpr (KCONTIG && VEC == 4) {
    // VEC == 4 (fp32): 16-byte loads for kend % 4 == 0 -- a vector that starts in range is loaded whole (the row's
    // pitch covers it) and its elements past kend are zeroed in registers: the same MFMA operands as element loads
    // (out-of-range elements read 0), 2 loads instead of 8 per fragment
    static_assert(std::is_same_v<T, float> && V == 8, "tail-masked vectors: 8 fp32 per fragment");
    const int off = (rok && k < kend) ? (r * ld + k) * (int)sizeof(T) + base_off : kOOB;
    const auto w0 = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, CP);
    const auto w1 = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 16, CP);
    __builtin_memcpy(reinterpret_cast<char*>(out), &w0, 16);
    __builtin_memcpy(reinterpret_cast<char*>(out) + 16, &w1, 16);
#pragma unroll
    for (int j = 0; j < V; ++j)
      if (k + j >= kend) out[j] = 0.f;
  } else if constexpr (KCONTIG && VEC == 2) {
    constexpr int HV = V / 2;  // elements per 8-byte half
    static_assert(HV * sizeof(T) == 8, "half-vector path expects 8-byte halves");
    const int base = (r * ld + k) * (int)sizeof(T) + base_off;
    const int o0 = (rok && k + HV <= kend) ? base : kOOB;
    const int o1 = (rok && k + V <= kend) ? base + 8 : kOOB;
    const auto w0 = __builtin_amdgcn_raw_buffer_load_b64(rs, o0, 0, CP);
    const auto w1 = __builtin_amdgcn_raw_buffer_load_b64(rs, o1, 0, CP);
    __builtin_memcpy(reinterpret_cast<char*>(out), &w0, 8);
    __builtin_memcpy(reinterpret_cast<char*>(out) + 8, &w1, 8);
  } else {
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int kj = k + j;
      const int idx = KCONTIG ? r * ld + kj : kj * ld + r;
      const int o = (rok && kj < kend) ? idx * (int)sizeof(T) + base_off : kOOB;
      if constexpr (CP != 0) {
        static_assert(std::is_same_v<T, float>, "a cache policy on element loads: fp32 only");
        out[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, o, 0, CP));
      } else {
        out[j] = buf_load1<T>(rs, o);
      }
    }
  }
}

// B operand stored as uint8 (raw MNIST pixels, exact in bf16): 8 bytes per lane
// (two 4-byte buffer loads, OOB -> 0) widened to 8 bf16 in registers.  Halves
// the operand bytes of a bf16 copy; the per-CU L2->L1 fill rate (~70 GB/s) is
// what bounds these small GEMMs.  VEC: 4-byte aligned rows, kend % 8 == 0.
__device__ __forceinline__ unsigned int u8x2_to_bf16x2(unsigned int w, int hi) {
  // bytes (2*hi, 2*hi+1) of w -> two bf16 (upper halves of the exact floats)
  const float f0 = (float)((w >> (16 * hi)) & 0xffu);
  const float f1 = (float)((w >> (16 * hi + 8)) & 0xffu);
  return (__builtin_bit_cast(unsigned int, f0) >> 16) | (__builtin_bit_cast(unsigned int, f1) & 0xffff0000u);
}

// The same 8 bytes as two raw words (VEC != 0) or 8 byte-loads (VEC == 0, one byte per word), widened later
// by widen_u8: the burst loads of wsk_tile stay ahead of every wait (widening right after the load makes
// hipcc wait for the bytes in the middle of the burst -- two memory round trips instead of one).
template <int VEC>
struct U8Raw {
  unsigned int w[VEC != 0 ? 2 : 8];
};

template <int VEC>
__device__ __forceinline__ void load_u8_raw(__amdgpu_buffer_rsrc_t rs, int ld, int r, int rmax, int k, int kend,
                                            U8Raw<VEC>& out) {
  const bool rok = r < rmax;
  if constexpr (VEC != 0) {
    const int base = r * ld + k;
    out.w[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, (rok && k + 4 <= kend) ? base : kOOB, 0, 0);
    out.w[1] = __builtin_amdgcn_raw_buffer_load_b32(rs, (rok && k + 8 <= kend) ? base + 4 : kOOB, 0, 0);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      out.w[j] = __builtin_amdgcn_raw_buffer_load_b8(rs, (rok && k + j < kend) ? r * ld + k + j : kOOB, 0, 0);
  }
}

template <int VEC>
__device__ __forceinline__ void widen_u8(const U8Raw<VEC>& in, __hip_bfloat16 (&out)[8]) {
  unsigned int w[4];
  if constexpr (VEC != 0) {
    w[0] = u8x2_to_bf16x2(in.w[0], 0);
    w[1] = u8x2_to_bf16x2(in.w[0], 1);
    w[2] = u8x2_to_bf16x2(in.w[1], 0);
    w[3] = u8x2_to_bf16x2(in.w[1], 1);
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) w[q] = u8x2_to_bf16x2(in.w[2 * q] | (in.w[2 * q + 1] << 8), 0);
  }
  __builtin_memcpy(out, w, 16);
}

template <int VEC>
__device__ __forceinline__ void load_frag_u8(__amdgpu_buffer_rsrc_t rs, int ld, int r, int rmax, int k, int kend,
                                             __hip_bfloat16 (&out)[8]) {
  // VEC != 0: two 4-byte loads, each range-checked on its own (kend % 4 == 0, rows 4-byte aligned)
  const bool rok = r < rmax;
  unsigned int w[4];
  if constexpr (VEC != 0) {
    const int base = r * ld + k;
    const unsigned int lo = __builtin_amdgcn_raw_buffer_load_b32(rs, (rok && k + 4 <= kend) ? base : kOOB, 0, 0);
    const unsigned int hi = __builtin_amdgcn_raw_buffer_load_b32(rs, (rok && k + 8 <= kend) ? base + 4 : kOOB, 0, 0);
    w[0] = u8x2_to_bf16x2(lo, 0);
    w[1] = u8x2_to_bf16x2(lo, 1);
    w[2] = u8x2_to_bf16x2(hi, 0);
    w[3] = u8x2_to_bf16x2(hi, 1);
  } else {
    unsigned int b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      b[j] = __builtin_amdgcn_raw_buffer_load_b8(rs, (rok && k + j < kend) ? r * ld + k + j : kOOB, 0, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q) w[q] = u8x2_to_bf16x2(b[2 * q] | (b[2 * q + 1] << 8), 0);
  }
  __builtin_memcpy(out, w, 16);
}

// Exact split of V fp32 values into NP bf16 planes BY TRUNCATION (x = hi + mid + lo for NP = 3):
// hi = the top 16 bits of x, r = x - hi (exact: < 2^-7 ulp-relative, <= 16 significant bits),
// mid = the top 16 bits of r, lo = r - mid (exact, <= 8 significant bits: a bf16).  Cheaper than the
// round-to-nearest split (an AND and a SUB per plane; packing takes the upper halves directly) and just
// as exact: 3 bf16 significands hold the 24 of an fp32.  NP = 1 is NOT exact (a truncated bf16); the
// callers use this only for NP = 3.
template <int NP, int V>
__device__ __forceinline__ void split_trunc(const float (&x)[V], __hip_bfloat16 (&p)[NP][V]) {
  static_assert(V % 2 == 0, "pairs of values per 32-bit word");
  unsigned w[NP][V / 2];
#pragma unroll
  for (int j = 0; j < V; j += 2) {
    unsigned cur0 = __builtin_bit_cast(unsigned, x[j]), cur1 = __builtin_bit_cast(unsigned, x[j + 1]);
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      w[q][j / 2] = (cur0 >> 16) | (cur1 & 0xffff0000u);
      if (q + 1 < NP) {
        const float r0 = __builtin_bit_cast(float, cur0) - __builtin_bit_cast(float, cur0 & 0xffff0000u);
        const float r1 = __builtin_bit_cast(float, cur1) - __builtin_bit_cast(float, cur1 & 0xffff0000u);
        cur0 = __builtin_bit_cast(unsigned, r0);
        cur1 = __builtin_bit_cast(unsigned, r1);
      }
    }
  }
  __builtin_memcpy(p, w, sizeof(w));
}

constexpr int kEpiMaxQ = 16;  // max output elements per thread in a tile epilogue

// Epilogue protocol used by wsk_tile:
//   epi.prefetch(q, row, col, valid)  -- before the K loop (issue independent loads)
//   epi(q, row, col, value)           -- once per in-bounds output element
struct EpiNoPrefetch {
  __device__ __forceinline__ void prefetch(int, int, int, bool) {}
};

struct TileGeom {
  int M, N, K;
  int m0, n0;
};

// An epilogue may also gate the K loop: epi.before_kloop(kbeg, kend) -- this wave's K range -- is called by every wave
// right before its first K-loop load, after the epilogue prefetch (the XCD-local step pipeline's dW1 waves wait there
// for the dZ1 column tiles their range reads, xstep.hip).  Epilogues without it compile to the plain loop.
template <class E, class = void>
struct HasBeforeKloop : std::false_type {};
template <class E>
struct HasBeforeKloop<E, std::void_t<decltype(std::declval<E&>().before_kloop(0, 0))>> : std::true_type {};

// One workgroup = KS waves computing the (16*MB) x (16*NB) tile at (m0, n0)
// of C = A * B with K split across the waves.  On return, `epi(row, col, v)`
// has been called exactly once for every in-bounds element of the tile.
// `red` must point at >= KS*MB*NB*4*64 accumulators of LDS (unused if KS==1).
//
// NPA > 1: A is the exact sum of NPA planes stored `plane_bytes` apart
// (A = A_0 + A_1 + ...; the split-bf16 representation of an fp32 operand,
// see mlp_split.hip) and every plane is multiplied into the same accumulator.
//
// stamps != nullptr (diagnostic builds only): lane 0 of every wave records
// s_memrealtime (100 MHz wall clock) at entry, after the K loop, after the
// reduction barrier and at the end: stamps[(block*KS + wave)*4 + i].
//
// TB = uint8_t (with T = bf16): the B operand is raw bytes, widened in registers.
// TA = float (with T = bf16, NPA = 3, AK): A is the fp32 operand itself, 4 B per element pulled instead of
// the 6 B of three stored planes, split into its exact planes in registers (split_trunc) while the MFMAs
// of the previous unroll step run.
//
// ASWZ (fp32 A, VEC == 3, MB == 1): A is the fragment-ordered copy of the fp32 operand (SplitStepArgs::w1_swz): for
// row tile rt, K pair p (64 k) and load i (0..3), lane l's 4 floats A(16 rt + (l & 15), 64 p + 16 (l >> 4) + 4 i ..
// + 3) at float offset (((rt * lda + p) * 4 + i) * 64 + l) * 4, lda = the number of K pairs -- every 16-byte load
// instruction of a wave reads 1 KB of contiguous memory instead of 16 rows x 64 B.
// Float offset of A(row, col) in that copy (npair = cdiv(K, 64)).
__host__ __device__ __forceinline__ int64_t w1s_off(int row, int col, int npair) {
  const int rt = row >> 4, c = row & 15, p = col >> 6, w = col & 63;
  const int lane = (w >> 4) * 16 + c, i = (w & 15) >> 2, e = w & 3;
  return ((((int64_t)rt * npair + p) * 4 + i) * 64 + lane) * 4 + e;
}
// BSWZ (u8 B, VEC == 3): B is the fragment-ordered copy of the pixels (SplitStepArgs::x_swz), ldb = the number of K
// pairs: sample tile st (16 samples), K pair p, lane l's 16 bytes at byte ((st * ldb + p) * 64 + l) * 16 (xs_off),
// st counted from the tile geometry's n0 = 0 -- again 1 KB per wave load instruction.  Needs g.n0 % 16 == 0.
__host__ __device__ __forceinline__ int64_t xs_off(int64_t s, int k, int npair) {
  const int p = k >> 6, w = k & 63;
  const int lane = (w >> 4) * 16 + (int)(s & 15);
  return (((s >> 4) * npair + p) * 64 + lane) * 16 + (w & 15);
}
//
// CPA (fp32 A only): the A loads' cache policy -- kSc1 for an operand another workgroup of the same launch rewrote
// since this CU last read it (the XCD-local step pipeline, xstep.hip: W1s and dZ1 -- fragment-ordered or row-major --
// are read with L1-bypassing, L2-served loads; a plain load could return this CU's stale L1 line)
template <typename T, int MB, int NB, int KS, bool AK, bool BK, int VEC, int U, int NPA = 1, typename TB = T,
          typename TA = T, bool ASWZ = false, bool BSWZ = false, int CPA = 0, class Epi>
__device__ __forceinline__ void wsk_tile(const TA* __restrict__ A, int lda, const TB* __restrict__ B, int ldb,
                                         TileGeom g, Epi& epi,
                                         typename MmaTraits<T>::acc_t* __restrict__ red, int plane_bytes = 0,
                                         unsigned long long* stamps = nullptr) {
  using Tr = MmaTraits<T>;
  using accv_t = typename Tr::accv_t;
  using acc_t = typename Tr::acc_t;
  constexpr int V = Tr::V, KC = Tr::KC;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int c = lane & 15, grp = lane >> 4;

  unsigned long long* st = stamps ? stamps + ((size_t)blockIdx.x * KS + wave) * 4 : nullptr;
  auto stamp = [&](int i) {
    if (st) {
      const unsigned long long tt = __builtin_amdgcn_s_memrealtime();
      if (lane == 0) st[i] = tt;
    }
  };
  stamp(0);
  accv_t acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = accv_t{0, 0, 0, 0};

  // Output elements owned by this thread in the epilogue: q = 0..NQ-1.
  constexpr int E = MB * NB * 4 * 64;  // accumulators per wave
  constexpr int NQ = KS == 1 ? MB * NB * 4 : (E + 64 * KS - 1) / (64 * KS);
  static_assert(NQ <= kEpiMaxQ, "epilogue prefetch slots exceeded");
  auto coord = [&](int q, int& row, int& col, int& e) -> bool {
    if constexpr (KS == 1) {
      const int i = q / (NB * 4), j = (q / 4) % NB, r = q % 4;
      row = g.m0 + 16 * i + Tr::row(grp, r);
      col = g.n0 + 16 * j + c;
      e = 0;
    } else {
      e = threadIdx.x + q * 64 * KS;
      const int ln = e & 63, r = (e >> 6) & 3, blk = e >> 8;
      const int i = blk / NB, j = blk % NB;
      row = g.m0 + 16 * i + Tr::row(ln >> 4, r);
      col = g.n0 + 16 * j + (ln & 15);
      if (e >= E) return false;
    }
    return row < g.M && col < g.N;
  };
  // Epilogue operands that do not depend on the GEMM (bias, the weight being
  // updated, ...) are fetched now, so their latency hides under the K loop
  // instead of adding a dependent round trip after the reduction.
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    int row, col, e;
    const bool ok = coord(q, row, col, e);
    epi.prefetch(q, row, col, ok);
  }

  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(A), rsB = make_rsrc(B);
  const int nch = (g.K + KC - 1) / KC;
  const int cpw = (nch + KS - 1) / KS;
  const int kbeg = wave * cpw * KC;
  const int kend = min(g.K, (wave + 1) * cpw * KC);

  if constexpr (HasBeforeKloop<Epi>::value) epi.before_kloop(kbeg, kend);
  constexpr bool AF32 = std::is_same_v<TA, float> && !std::is_same_v<T, float>;
  static_assert(!AF32 || (std::is_same_v<T, __hip_bfloat16> && NPA == 3 && AK), "fp32 A: split3 bf16, K-contiguous");
  constexpr bool BU8 = std::is_same_v<TB, uint8_t>;
  static_assert(CPA == 0 || AF32, "an A cache policy only on the fp32 A loads");
  // VEC == 3 (u8 B only): chunks go in PAIRS.  Lane group grp of chunk pair (u, u + 1) covers the 16 k
  // kp + 16 grp .. kp + 16 grp + 15 (kp = the pair's first k): chunk u takes the first 8, chunk u + 1 the
  // last 8 (the MFMA sums over its chunk, so any bijection of k onto (lane group, element) that A and B
  // share is the same product).  B is then ONE 16-byte load per lane per pair instead of four 4-byte loads
  // (the u8 rows are 16 B per lane group); A keeps its 16-byte vectors.  Needs kend % 16 == 0 and 16-byte
  // aligned B rows.
  static_assert(VEC != 3 || (BU8 && U % 2 == 0 && V == 8), "paired chunks: u8 B, even U");
  // VEC == 4 (fp32 A, u8 B): A as 16-byte vectors with the tail zeroed in registers (load_frag), B as VEC 1 / 2
  static_assert(VEC != 4 || (AF32 && BU8), "tail-masked vectors: fp32 A, u8 B");
  constexpr int VECA = VEC == 3 ? 1 : VEC;  // the A operand's load form
  constexpr int VA = VECA == 1 ? 1 : VECA == 4 ? 4 : 0;  // fp32 A: 2 x 16-byte loads (tail-masked), or element loads
  for (int kc = kbeg; kc < kend; kc += KC * U) {
    T af[U][NPA][MB][V];
    float ar[AF32 ? U : 1][MB][V];
    T bf[U][NB][V];
    U8Raw<VEC == 3 ? 1 : VEC> braw[BU8 ? U : 1][NB];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = VEC == 3 ? kc + (u & ~1) * KC + 2 * V * grp + (u & 1) * V : kc + u * KC + V * grp;
      if constexpr (AF32 && ASWZ) {
        static_assert(MB == 1 && VEC == 3 && V == 8, "fragment-ordered A: one row block, chunk pairs");
        const int kp = kc + (u & ~1) * KC;  // the pair's first k (a multiple of 64)
        const bool ok = g.m0 + c < g.M && k < kend;
        const int base = ((((g.m0 >> 4) * lda + (kp >> 6)) * 4 + 2 * (u & 1)) * 64 + lane) * 16;
        const auto w0 = __builtin_amdgcn_raw_buffer_load_b128(rsA, ok ? base : kOOB, 0, CPA);
        const auto w1 = __builtin_amdgcn_raw_buffer_load_b128(rsA, ok ? base + 1024 : kOOB, 0, CPA);
        __builtin_memcpy(ar[u][0], &w0, 16);
        __builtin_memcpy(reinterpret_cast<char*>(ar[u][0]) + 16, &w1, 16);
      } else if constexpr (AF32) {
#pragma unroll
        for (int i = 0; i < MB; ++i)
          load_frag<float, V, true, VA, CPA>(rsA, lda, g.m0 + 16 * i + c, g.M, k, kend, ar[u][i]);
      } else {
#pragma unroll
        for (int p = 0; p < NPA; ++p)
#pragma unroll
          for (int i = 0; i < MB; ++i)
            load_frag<T, V, AK, VECA>(rsA, lda, g.m0 + 16 * i + c, g.M, k, kend, af[u][p][i], p * plane_bytes);
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        if constexpr (BU8) {
          static_assert(std::is_same_v<T, __hip_bfloat16> && BK, "u8 B operand: bf16 MFMA, K-contiguous");
          if constexpr (VEC == 3) {
            if ((u & 1) == 0) {  // the pair's 16 bytes: words 0-1 -> chunk u, words 2-3 -> chunk u + 1
              const int r = g.n0 + 16 * j + c;
              int off = r * ldb + k;
              if constexpr (BSWZ) off = ((((g.n0 >> 4) + j) * ldb + ((kc + u * KC) >> 6)) * 64 + lane) * 16;
              const auto w = __builtin_amdgcn_raw_buffer_load_b128(rsB, (r < g.N && k + 16 <= kend) ? off : kOOB, 0, 0);
              braw[u][j].w[0] = w[0];
              braw[u][j].w[1] = w[1];
              braw[u + 1][j].w[0] = w[2];
              braw[u + 1][j].w[1] = w[3];
            }
          } else {
            load_u8_raw<VEC>(rsB, ldb, g.n0 + 16 * j + c, g.N, k, kend, braw[u][j]);
          }
        } else {
          load_frag<T, V, BK, VECA>(rsB, ldb, g.n0 + 16 * j + c, g.N, k, kend, bf[u][j]);
        }
      }
    }
    // Keep every load of this burst ahead of the first MFMA: without the fence
    // the scheduler sinks each load next to its consumer to save VGPRs, which
    // turns the burst into U dependent memory round trips (measured: 25
    // vmcnt(0) waits per wave in fwd1).  With it: one wait ladder per burst.
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (BU8) {
#pragma unroll
        for (int j = 0; j < NB; ++j) widen_u8<VEC == 3 ? 1 : VEC>(braw[u][j], bf[u][j]);
      }
      if constexpr (AF32) {
#pragma unroll
        for (int i = 0; i < MB; ++i) {
          T pl[NPA][V];
          split_trunc<NPA, V>(ar[u][i], pl);
#pragma unroll
          for (int p = 0; p < NPA; ++p)
#pragma unroll
            for (int v = 0; v < V; ++v) af[u][p][i][v] = pl[p][v];
        }
      }
#pragma unroll
      for (int p = 0; p < NPA; ++p)
#pragma unroll
        for (int i = 0; i < MB; ++i)
#pragma unroll
          for (int j = 0; j < NB; ++j) Tr::mma(af[u][p][i], bf[u][j], acc[i][j]);
    }
  }

  if (st) {  // make the K-loop stamp wait for the MFMA results
    float sink = 0.f;
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) sink += (float)acc[i][j][0];
    asm volatile("" ::"v"(sink));
  }
  stamp(1);
  if constexpr (KS == 1) {
    stamp(2);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      int row, col, e;
      if (coord(q, row, col, e)) epi(q, row, col, acc[q / (NB * 4)][(q / 4) % NB][q % 4]);
    }
    stamp(3);
  } else {
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wave * E + (((i * NB + j) * 4 + r) << 6) + lane] = acc[i][j][r];
    __syncthreads();
    stamp(2);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      int row, col, e;
      const bool ok = coord(q, row, col, e);
      if (e < E) {
        acc_t s = red[e];
#pragma unroll
        for (int w = 1; w < KS; ++w) s += red[w * E + e];
        if (ok) epi(q, row, col, s);
      }
    }
    if (st) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(3);
    __syncthreads();  // `red` may be reused by the caller
  }
}

}  // namespace cme
