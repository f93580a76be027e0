// LDS double-buffered MFMA tile engine for the WIDE MLP configs (H >= 512:
// BASELINE configs 4 and 5, 784-4096-10 and 784-1024-10).
//
// At H=100 the step's GEMMs are too small for operand reuse and the
// wave-split-K engine (mma_tile.h) wins; at H=4096 the same tiles re-read W1
// 25x and X 256x through L2 (~640 MB per step) -- there the classic blocked
// GEMM is the right shape (cdna_hip_programming.md §5):
//   * C[m][n] = sum_k A[m][k] B[n][k], both operands K-contiguous ("NT");
//     A = NPA exact bf16 planes (split-fp32, see mlp_split.h), B = uint8 pixels
//     (exact in bf16, converted at fragment read) or bf16.
//   * BM x BN workgroup tile, 4 waves as 2x2 (or 8 as 4x2), each wave's share built from
//     16x16 blocks of v_mfma_f32_16x16x32_bf16; BK = 64 per stage.
//   * global -> VGPR -> LDS staging with 16-byte buffer loads (out-of-range
//     rows / k return zero: no edge branches), two LDS buffers and two register
//     stages: the loads of stage k+2 are in flight while stages k and k+1 are
//     multiplied, ONE barrier per stage.
//   * A rows padded +32 B: the 16-row ds_read_b128 fragment reads are bank-conflict
//     free (modelled per the gfx950 lane groups); B rows +16 B (ds_read_b64).
//   * XCD-aware tile order (tiles sharing A rows land on one XCD's L2).
#pragma once

#include "mma_tile.h"

#include <type_traits>

#ifndef CME_LDS_SETPRIO
#define CME_LDS_SETPRIO 0  // measured: -1.5 us bf16 H=4096, +0.9 us fp32 H=4096 (kbench) -- off
#endif

namespace cme {

namespace lg {

constexpr int kBK = 64;
constexpr int kThreads = 256;
constexpr int kARow = kBK * 2 + 32;  // bytes per A row in LDS (bf16, +32 B: conflict-free ds_read_b128 fragments)

template <typename TB>
struct BTraits;
template <>
struct BTraits<uint8_t> {
  // uint8 pixels are widened to bf16 ONCE, when a stage is written to LDS (16 conversions per thread per
  // stage), instead of at every fragment read (measured: ~95 VALU conversions per 40 MFMAs per wave)
  static constexpr int kRow = kBK * 2 + 16;   // bytes per B row in LDS (bf16)
  static constexpr int kChunksPerRow = kBK / 16;  // 16-byte global chunks (16 pixels) per row
  static constexpr int kLdsChunk = 32;        // bytes one global chunk occupies in LDS
};
template <>
struct BTraits<__hip_bfloat16> {
  static constexpr int kRow = kBK * 2 + 16;
  static constexpr int kChunksPerRow = kBK * 2 / 16;
  static constexpr int kLdsChunk = 16;
};

template <int BM, int BN, int NPA, typename TB>
constexpr int lds_bytes() {
  return 2 * (NPA * BM * kARow + BN * BTraits<TB>::kRow);
}

__device__ __forceinline__ bf16x8_t u8x8_to_bf16(uint2 w) {
  // bytes -> bf16 exactly: bf16(x) for 0 <= x <= 255 via the float bit pattern
  bf16x8_t r;
  const uint32_t lo = w.x, hi = w.y;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = (__bf16)(float)((lo >> (8 * j)) & 255u);
    r[4 + j] = (__bf16)(float)((hi >> (8 * j)) & 255u);
  }
  return r;
}

// Epi::kTileHook present -> lds_gemm_tile calls epi.tile<MB, NB, WRN>(acc, wr, wc, fr, fg, row0, col0, lds)
// once per workgroup after the element epilogue (row0/col0: this wave's first row / column)
template <class E, class = void>
struct HasTileHook : std::false_type {};
template <class E>
struct HasTileHook<E, std::void_t<decltype(E::kTileHook)>> : std::true_type {};

}  // namespace lg

// One BM x BN output tile at (m0, n0).  `lds` must hold lg::lds_bytes<...>()
// bytes (16-byte aligned).  Requirements (checked by the launcher): K % 16 == 0,
// lda % 8 == 0 (bf16) and ldb % 16 == 0 bytes, 16-byte aligned operand bases.
// epi(row, col, v) is called for every in-range element of the tile.
// NKS > 0: the K loop has exactly NKS stages (K in ((NKS-1)*64, NKS*64]) and is fully unrolled -- in a
// runtime-trip-count loop the compiler's vmcnt tracking merges at the back-edge and drains every load
// (vmcnt(0)) before the stage-(k+1) LDS stores, i.e. the stage-(k+2) prefetch never stays in flight.
template <int BM, int BN, int NPA, typename TB, class Epi, int NT = lg::kThreads, int NKS = 0>
__device__ __forceinline__ void lds_gemm_tile(const __hip_bfloat16* __restrict__ A, int lda, int plane_bytes,
                                              const TB* __restrict__ B, int ldb, int M, int N, int K, int m0, int n0,
                                              Epi& epi, char* __restrict__ lds) {
  using namespace lg;
  // NT = 256: 4 waves as 2x2; NT = 512: 8 waves as 4x2 (two waves per SIMD hide more of the L2
  // latency at one workgroup per CU)
  constexpr int WRN = NT / 64 / 2, WM = BM / WRN, WN = BN / 2, MB = WM / 16, NB = WN / 16;
  static_assert(MB >= 1 && NB >= 1, "tile too small for the wave layout");
  constexpr int BROW = BTraits<TB>::kRow, BCPR = BTraits<TB>::kChunksPerRow;
  constexpr int A_CHUNKS = BM * (kBK * 2 / 16);  // 16-byte chunks per plane per stage
  constexpr int B_CHUNKS = BN * BCPR;
  constexpr int AJ = (A_CHUNKS + NT - 1) / NT, BJ = (B_CHUNKS + NT - 1) / NT;
  static_assert(A_CHUNKS % NT == 0 && (B_CHUNKS % NT == 0 || B_CHUNKS < NT), "tile/thread mismatch");
  // B_CHUNKS < NT (narrow uint8 B tiles at 8 waves): only the first B_CHUNKS threads stage B
  auto b_mine = [&](int j) { return B_CHUNKS % NT == 0 || (int)threadIdx.x + j * NT < B_CHUNKS; };
  constexpr int A_BUF = NPA * BM * kARow, B_BUF = BN * BROW;

  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int fr = lane & 15, fg = lane >> 4;

  const __amdgpu_buffer_rsrc_t ra = make_rsrc(A), rb = make_rsrc(B);
  char* ldsA = lds;
  char* ldsB = lds + 2 * A_BUF;

  // per-thread staging coordinates (fixed across stages)
  int a_off[AJ], a_lds[AJ], b_off[BJ], b_lds[BJ];
  bool a_ok[AJ], b_ok[BJ];
#pragma unroll
  for (int j = 0; j < AJ; ++j) {
    const int c = t + j * NT, r = c >> 3, kc = c & 7;  // 8 chunks of 8 bf16 per row
    a_ok[j] = m0 + r < M;
    a_off[j] = ((m0 + r) * lda + kc * 8) * 2;
    a_lds[j] = r * kARow + kc * 16;
  }
#pragma unroll
  for (int j = 0; j < BJ; ++j) {
    const int c = t + j * NT, r = c / BCPR, kc = c % BCPR;
    b_ok[j] = n0 + r < N;
    b_off[j] = (n0 + r) * ldb * (int)sizeof(TB) + kc * 16;
    b_lds[j] = r * BROW + kc * BTraits<TB>::kLdsChunk;
  }

  // two register stages: the loads of K-stage k+2 are issued before stage k is multiplied and are
  // only consumed (written to LDS) after stage k+1 -- two compute phases of cover for L2 latency
  uint4 ra_reg[2][NPA][AJ], rb_reg[2][BJ];
  auto load_stage = [&](int k0, uint4 (&rA)[NPA][AJ], uint4 (&rB)[BJ]) {
    const int kb = k0 * 2;  // byte offset of k0 in an A row
#pragma unroll
    for (int j = 0; j < AJ; ++j) {
      const int kc = (t + j * NT) & 7;
      const bool ok = a_ok[j] && k0 + kc * 8 < K;
#pragma unroll
      for (int p = 0; p < NPA; ++p) {
        const auto w = __builtin_amdgcn_raw_buffer_load_b128(ra, ok ? a_off[j] + kb + p * plane_bytes : kOOB, 0, 0);
        __builtin_memcpy(&rA[p][j], &w, 16);
      }
    }
#pragma unroll
    for (int j = 0; j < BJ; ++j) {
      const int kc = (t + j * NT) % BCPR;
      constexpr int EPC = 16 / (int)sizeof(TB);  // elements per chunk
      const bool ok = b_ok[j] && k0 + kc * EPC < K;
      if (!b_mine(j)) continue;
      const auto w = __builtin_amdgcn_raw_buffer_load_b128(rb, ok ? b_off[j] + k0 * (int)sizeof(TB) : kOOB, 0, 0);
      __builtin_memcpy(&rB[j], &w, 16);
    }
  };
  auto store_stage = [&](int buf, const uint4 (&rA)[NPA][AJ], const uint4 (&rB)[BJ]) {
#pragma unroll
    for (int p = 0; p < NPA; ++p)
#pragma unroll
      for (int j = 0; j < AJ; ++j)
        *reinterpret_cast<uint4*>(ldsA + buf * A_BUF + p * BM * kARow + a_lds[j]) = rA[p][j];
#pragma unroll
    for (int j = 0; j < BJ; ++j)
      if (b_mine(j)) {
        if constexpr (sizeof(TB) == 1) {  // 16 pixels -> 16 bf16 (32 bytes)
          const bf16x8_t lo = lg::u8x8_to_bf16(uint2{rB[j].x, rB[j].y});
          const bf16x8_t hi = lg::u8x8_to_bf16(uint2{rB[j].z, rB[j].w});
          *reinterpret_cast<bf16x8_t*>(ldsB + buf * B_BUF + b_lds[j]) = lo;
          *reinterpret_cast<bf16x8_t*>(ldsB + buf * B_BUF + b_lds[j] + 16) = hi;
        } else {
          *reinterpret_cast<uint4*>(ldsB + buf * B_BUF + b_lds[j]) = rB[j];
        }
      }
  };

  f32x4 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const char* sA = ldsA + buf * A_BUF + (wr * WM + fr) * kARow;
    const char* sB = ldsB + buf * B_BUF + (wc * WN + fr) * BROW;
#pragma unroll
    for (int kk = 0; kk < kBK / 32; ++kk) {
      bf16x8_t bf[NB];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        bf[nb] = *reinterpret_cast<const bf16x8_t*>(sB + nb * 16 * BROW + (kk * 32 + fg * 8) * 2);
      }
      // issue every A fragment read of this k-step before the first MFMA: one LDS round trip per
      // k-step instead of one per fragment (the reads are independent; counted lgkmcnt waits)
      bf16x8_t af[NPA][MB];
#pragma unroll
      for (int p = 0; p < NPA; ++p)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          af[p][mb] =
              *reinterpret_cast<const bf16x8_t*>(sA + p * BM * kARow + mb * 16 * kARow + (kk * 32 + fg * 8) * 2);
#if CME_LDS_SETPRIO
      __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
      for (int p = 0; p < NPA; ++p)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
            acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[p][mb], bf[nb], acc[mb][nb], 0, 0, 0);
#if CME_LDS_SETPRIO
      __builtin_amdgcn_s_setprio(0);
#endif
    }
  };

  const int nk = NKS > 0 ? NKS : (K + kBK - 1) / kBK;
  load_stage(0, ra_reg[0], rb_reg[0]);
  if (nk > 1) load_stage(kBK, ra_reg[1], rb_reg[1]);
  store_stage(0, ra_reg[0], rb_reg[0]);
  __syncthreads();
  // stage kt lives in LDS buffer kt&1 and (before its store) in register set kt&1
  // LDS-only barrier: __syncthreads() would also drain vmcnt, i.e. wait for the stage-(k+2) global
  // loads that are meant to stay in flight across it (cdna_hip_programming.md §5, "Pipelining
  // across barriers"); the LDS writes only need lgkmcnt(0) before the s_barrier
  auto lds_barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto step = [&](int kt, uint4 (&rA_cur)[NPA][AJ], uint4 (&rB_cur)[BJ], uint4 (&rA_nxt)[NPA][AJ],
                  uint4 (&rB_nxt)[BJ]) {
    if (kt + 2 < nk) load_stage((kt + 2) * kBK, rA_cur, rB_cur);  // set kt&1 is free again
    // keep the stage-(k+2) loads ahead of this stage's MFMAs: without the fence the scheduler sinks them
    // below the stage-(k+1) LDS stores (one register set instead of two), so only one compute phase
    // covers the load latency (measured in the ISA: loads issued right before the barrier)
    __builtin_amdgcn_sched_barrier(0);
    compute(kt & 1);
    if (kt + 1 < nk) store_stage((kt + 1) & 1, rA_nxt, rB_nxt);
    lds_barrier();
  };
#pragma unroll
  for (int kt = 0; kt < (NKS > 0 ? NKS : nk); kt += 2) {
    step(kt, ra_reg[0], rb_reg[0], ra_reg[1], rb_reg[1]);
    if (kt + 1 < nk) step(kt + 1, ra_reg[1], rb_reg[1], ra_reg[0], rb_reg[0]);
  }

  // epilogue: C layout of 16x16 f32 MFMA -- lane holds col fr, rows 4*fg + i
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + wr * WM + mb * 16 + 4 * fg + i;
        const int col = n0 + wc * WN + nb * 16 + fr;
        if (row < M && col < N) epi(row, col, acc[mb][nb][i]);
      }
  // optional whole-tile hook on the raw accumulators (e.g. a second tiny MFMA contraction of the tile);
  // every LDS read of the main loop has passed the last lds_barrier, so `lds` is free for it
  if constexpr (lg::HasTileHook<Epi>::value)
    epi.template tile<MB, NB, WRN>(acc, wr, wc, fr, fg, m0 + wr * WM, n0 + wc * WN, lds);
}

}  // namespace cme
