// The wide forward / dW1 K loop with BOTH operands staged global -> LDS by LDS-DMA in 64-deep K steps ("g64"),
// for the 128 x 128 tiles of H >= 2048.  Same contract and accumulator layout as rega_gemm_mainloop<AT, 128, 1>
// (8 waves, wave w owns rows m0 + 16 w + [0, 16) and all 128 columns: acc[1][8]), so the epilogues -- the fused
// head, the dW1 update -- are unchanged, and the same MFMA sequence per accumulator (32-deep halves in K order,
// planes hi / mid / lo innermost, the same in-register split): BITWISE the rega engine's result.
//
// What it changes against rega_gemm.h (bench/kbench.py wide rows, docs/PERFORMANCE.md round 5):
//   * A (W1 / dZ1) no longer goes straight into fragment registers: each lane's fragment load covered 16 rows x
//     64 B per wave instruction -- a fragment-shaped load, which costs the CU's texture path twice the work of a
//     full-line load for the same bytes (cdna_hip_programming.md §5, projection-GEMM table: +18-45 %).  Here A and
//     B land in LDS as whole 128-B / 256-B rows, 1 KB per DMA instruction, and fragments come back by
//     ds_read_b128;
//   * 64-deep K steps (12.25 per K = 784 instead of 25 32-deep stages): half the barriers and counted waits,
//     and 2 (fp32 A) / 3 (bf16 A) K steps -- 96 KB -- in flight behind each barrier;
//   * the LDS images are lane-linear per DMA instruction; the bank-conflict swizzle is applied to the per-lane
//     GLOBAL address and undone on the fragment read: logical 16-byte chunk c of row r sits in physical chunk
//     c ^ (r & 15) (fp32 rows: 256 B, 16 chunks) or c ^ ((r >> 1) & 7) (bf16 rows: 128 B, 8 chunks).  Either way
//     the 16 (row, chunk) pairs of each of ds_read_b128's four lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}
//     and the same + 32) land in 16 different 16-byte slots of the 256-byte bank row: conflict-free;
//   * one raw s_barrier per K step after a counted vmcnt (the younger steps' DMAs stay in flight) and
//     lgkmcnt(0) (this wave's fragment reads of the buffer about to be refilled have retired).
// Requirements (launcher, as rega): K % 8 == 0, lda % 4 (fp32) / 8 (bf16), ldb % 8, 16-byte aligned bases, the
// caller's ONE dynamic LDS array of >= g64::lds_bytes<AT>() bytes.
#pragma once

#include "l2_touch.h"
#include "rega_gemm.h"

namespace cme {

namespace g64 {

constexpr int kBK = 64;
template <typename AT>
constexpr int stages() {
  return sizeof(AT) == 4 ? 3 : 4;  // 3 x 48 KB (fp32 A) / 4 x 32 KB (bf16 A): K steps in flight = stages - 1
}
template <typename AT>
constexpr int a_bytes() {
  return 128 * kBK * (int)sizeof(AT);
}
constexpr int kBBytes = 128 * kBK * 2;
template <typename AT>
constexpr int stage_bytes() {
  return a_bytes<AT>() + kBBytes;
}
constexpr int kJunk = 8 * 1024;  // the L2 pre-touch's landing slot (1 KB per wave, never read)
template <typename AT>
constexpr int lds_bytes() {
  return stages<AT>() * stage_bytes<AT>() + kJunk;
}

// L2 pre-touch (g64_gemm_mainloop): the workgroups of one XCD that read the same A rows / B rows split pulling
// ALL of them into the XCD's L2 at entry, so only the first K step waits a memory latency and the rest stream from
// L2.  a_part / a_parts: this workgroup's share of its A rows [m0, m0 + 128) x K (parts 0: no touch); b_* the same
// for B.  Speed only: any split is correct.
struct Touch {
  int a_part = 0, a_parts = 0, b_part = 0, b_parts = 0;
};

}  // namespace g64

template <typename AT, int NKS = 0>
__device__ __forceinline__ void g64_gemm_mainloop(const AT* __restrict__ A, int lda, const __hip_bfloat16* __restrict__ B,
                                                  int ldb, int M, int N, int K, int m0, int n0, char* __restrict__ lds,
                                                  f32x4 (&acc)[1][8], g64::Touch touch = {}) {
  using namespace g64;
  constexpr bool F32 = sizeof(AT) == 4;
  constexpr int S = stages<AT>();
  constexpr int SB = stage_bytes<AT>(), AB = a_bytes<AT>();
  constexpr int LA = AB / 1024 / 8, LB = kBBytes / 1024 / 8;  // DMA instructions per wave per K step
  constexpr int LS = LA + LB;
  constexpr int NB = 8;
  constexpr int AROWB = kBK * (int)sizeof(AT);  // LDS bytes per A row (256 / 128)
  constexpr int AROWS_PER_I = 1024 / AROWB;     // A rows per DMA instruction (4 / 8)

  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const __amdgpu_buffer_rsrc_t rsa = make_rsrc(A), rsb = make_rsrc(B);

  // ---- DMA sources (per lane) for this wave's instructions: A instruction j covers image rows
  // (wave + 8 j) * AROWS_PER_I + [0, AROWS_PER_I); lane -> (row, physical chunk) in image order, logical chunk by
  // the swizzle (its k offset is added per K step)
  int asrc[LA], bsrc[LB];
#pragma unroll
  for (int j = 0; j < LA; ++j) {
    int row, c;
    if constexpr (F32) {
      row = (wave + 8 * j) * AROWS_PER_I + (lane >> 4);
      c = (lane & 15) ^ (row & 15);
      asrc[j] = m0 + row < M ? ((m0 + row) * lda + 4 * c) * 4 : -1;
    } else {
      row = (wave + 8 * j) * AROWS_PER_I + (lane >> 3);
      c = (lane & 7) ^ ((row >> 1) & 7);
      asrc[j] = m0 + row < M ? ((m0 + row) * lda + 8 * c) * 2 : -1;
    }
  }
  int bkc[LB];  // (the logical chunk's first k, for the K-tail check)
  int akc[LA];
#pragma unroll
  for (int j = 0; j < LA; ++j) {
    const int row = (wave + 8 * j) * AROWS_PER_I + (F32 ? (lane >> 4) : (lane >> 3));
    akc[j] = F32 ? 4 * ((lane & 15) ^ (row & 15)) : 8 * ((lane & 7) ^ ((row >> 1) & 7));
  }
#pragma unroll
  for (int j = 0; j < LB; ++j) {
    const int row = (wave + 8 * j) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    bsrc[j] = n0 + row < N ? ((n0 + row) * ldb + 8 * c) * 2 : -1;
    bkc[j] = 8 * c;
  }
  auto issue = [&](int ks) {
    const int k0 = ks * kBK;
    char* base = lds + (ks % S) * SB;
#pragma unroll
    for (int j = 0; j < LA; ++j)
      gl::dma16(rsa, base + (wave + 8 * j) * 1024,
                (asrc[j] >= 0 && k0 + akc[j] < K) ? asrc[j] + k0 * (int)sizeof(AT) : kOOB);
#pragma unroll
    for (int j = 0; j < LB; ++j)
      gl::dma16(rsb, base + AB + (wave + 8 * j) * 1024, (bsrc[j] >= 0 && k0 + bkc[j] < K) ? bsrc[j] + k0 * 2 : kOOB);
  };

#pragma unroll
  for (int j = 0; j < NB; ++j) acc[0][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets inside a stage: A row 16 wave + fr; B row (column) 16 nb + fr
  const int arow = 16 * wave + fr;
  auto a_off = [&](int c) { return arow * AROWB + ((F32 ? (c ^ fr) : (c ^ ((arow >> 1) & 7))) << 4); };
  auto b_off = [&](int nb, int c) {
    const int r = 16 * nb + fr;
    return AB + r * 128 + ((c ^ ((r >> 1) & 7)) << 4);
  };

  const int nk = NKS > 0 ? NKS : (K + kBK - 1) / kBK;
  const int nh = (K + 31) / 32;  // 32-deep halves with any k < K (a K step's second half past K is skipped)

  auto barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // K step ks landed for this wave with `younger` later steps still allowed in flight
  auto wait_step = [&](int younger) {
    if (younger >= 2) gl::wait_vm<2 * LS>();
    else if (younger == 1) gl::wait_vm<LS>();
    else gl::wait_vm<0>();
  };

  if (touch.a_parts > 0) {  // (older than every DMA below: the first K step's counted wait covers them)
    char* junk = lds + S * SB;
    l2_touch_nowait(A, (int64_t)m0 * lda * (int)sizeof(AT), min(128, M - m0), (int64_t)lda * (int)sizeof(AT),
                    (int64_t)K * (int)sizeof(AT), touch.a_part, touch.a_parts, junk);
    l2_touch_nowait(B, (int64_t)n0 * ldb * 2, min(128, N - n0), (int64_t)ldb * 2, (int64_t)K * 2, touch.b_part,
                    touch.b_parts, junk);
  }
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue(s);

  auto step = [&](int ks) {
    wait_step(min(S - 2, nk - 1 - ks));
    barrier();  // step ks visible to every wave; every wave's reads of step ks - 1's buffer retired
    if (ks + S - 1 < nk) issue(ks + S - 1);  // into the buffer of step ks - 1
    const char* st = lds + (ks % S) * SB;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (2 * ks + h >= nh) break;  // (uniform: the K tail's empty half)
      bf16x8_t b[NB], ap[F32 ? 3 : 1];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) b[nb] = *reinterpret_cast<const bf16x8_t*>(st + b_off(nb, 4 * h + fg));
      if constexpr (F32) {
        const ra::u32x4 w0 = *reinterpret_cast<const ra::u32x4*>(st + a_off(8 * h + 2 * fg));
        const ra::u32x4 w1 = *reinterpret_cast<const ra::u32x4*>(st + a_off(8 * h + 2 * fg + 1));
        ra::split3(w0, w1, ap[0], ap[1], ap[2]);
      } else {
        ap[0] = *reinterpret_cast<const bf16x8_t*>(st + a_off(4 * h + fg));
      }
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int p = 0; p < (F32 ? 3 : 1); ++p)  // planes innermost: hi, mid, lo (rega's order)
          acc[0][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ap[p], b[nb], acc[0][nb], 0, 0, 0);
    }
  };
  if constexpr (NKS > 0) {
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) step(ks);
  } else {
    for (int ks = 0; ks < nk; ++ks) step(ks);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

}  // namespace cme
