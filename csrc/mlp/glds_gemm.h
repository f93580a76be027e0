// Direct-to-LDS (buffer_load ... lds) MFMA tile engine for the WIDE MLP GEMMs (H >= 512: BASELINE
// configs 4 and 5, 784-4096-10 and 784-1024-10) -- the successor of round 1's register-staged engine (removed
// in round 4: never selected once the bf16 copies of X existed).
//
// What limited that engine (profiles/wide4096_pmc.md): global -> VGPR -> LDS staging with two LDS buffers
// leaves ONE stage of loads in flight behind each barrier, the waves spend ~45 % parked at the per-stage
// barrier / vmcnt wait and MFMA is busy ~20-30 %.  Here (cdna_hip_programming.md §5 "Pipelining across
// barriers", the glds row of its staging table):
//   * every operand byte goes global -> LDS by the LDS-DMA form of the buffer load (16 B per lane, no
//     VGPR round trip, no ds_write pass), so four 32-deep K stages fit in 128 KB of LDS and THREE of them
//     are in flight while the fourth is multiplied;
//   * one raw s_barrier per stage, preceded by a COUNTED vmcnt (the loads of the two younger stages stay
//     in flight across it) and lgkmcnt(0) (this wave's fragment reads of the previous stage retired, so
//     the buffer the next DMA overwrites is free);
//   * all LDS is the caller's ONE dynamic array (a second __shared__ object can make hipcc wait vmcnt(0)
//     before every fragment read, §5 item 4(a));
//   * the LDS image is lane-linear per DMA instruction (16 rows x 64 B), so the bank-conflict swizzle is
//     applied to the per-lane GLOBAL address and undone on the fragment read (rule 21): logical 16-byte
//     k-chunk kc of row r lives in physical slot kc ^ gl::swz(r), which spreads each of ds_read_b128's four
//     NON-contiguous 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31} and the same + 32,
//     MI355X_MICROARCH.md LDS table) over all 16 slots of the 256-byte bank row: conflict-free.  (The plain
//     kc ^ ((r >> 2) & 3) is right for contiguous groups and 2-way on these: 1.4-1.7 M conflict cycles per
//     H = 4096 launch, profiles/wide4096_pmc_r3.md);
//   * out-of-range rows and the K tail (k >= K) are zero-filled by the buffer range check (kOOB offset).
//
// Operands: C[m][n] = sum_k A[m][k] B[n][k], both K-contiguous ("NT"); A = NPA exact bf16 planes of an
// fp32 matrix stored plane_bytes apart (split-fp32, mlp_split.h) or one bf16 plane; B bf16.  The
// accumulator layout is the 16x16x32 MFMA's (8 waves as 4 x 2); the epilogue is the caller's, with
// its operand loads issued before the K loop and branch-free buffer stores (an element functor that loads
// b1[row] / W1[i] behind a bounds branch serialises one dependent L2 round trip per output element).
#pragma once

#include "mma_tile.h"

#include <type_traits>

namespace cme {

namespace gl {

constexpr int kBK = 32;        // K per stage (64 bytes of bf16 per row)
constexpr int kRowB = kBK * 2;  // LDS bytes per row per stage
constexpr int kStages = 4;     // LDS buffers; kStages - 1 stages in flight

template <int BM, int BN, int NPA>
constexpr int stage_bytes() {
  return (NPA * BM + BN) * kRowB;
}
template <int BM, int BN, int NPA>
constexpr int lds_bytes() {
  return kStages * stage_bytes<BM, BN, NPA>();
}

// physical 16-byte slot of logical k-chunk kc in row r: kc ^ swz(r).  With rows 64 B apart a row's slots are
// 4 (r & 3) + 0..3; for the 16x16x32 fragment read (lane l: row l & 15, chunk l >> 4) each ds_read_b128 lane group
// holds, per r & 3, rows with r >> 2 = {0, 3} at chunk g and {1, 2} at chunk g ^ 1 (or the reverse), and
// swz = [0, 2, 3, 1] by r >> 2 gives those four (row, chunk) pairs four different slots
__device__ __forceinline__ int swz(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds_base, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_base, 16, voff, 0, 0,
                                           0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

}  // namespace gl

// Wave layout of the engine: 8 waves as 4 (rows) x 2 (columns); wave (wr, wc) owns rows
// m0 + wr * WM + [0, WM) and columns n0 + wc * WN + [0, WN) as MB x NB 16x16 accumulator blocks (16x16 f32
// MFMA layout: lane holds column fr = lane & 15, rows 4 * (lane >> 4) + i).
template <int BM, int BN>
struct GldsGeom {
  static constexpr int WRN = 4, WM = BM / WRN, WN = BN / 2, MB = WM / 16, NB = WN / 16;
};

// The K loop of one BM x BN tile at (m0, n0) into acc (zeroed here); NT = 512.  `lds` must hold
// gl::lds_bytes bytes.  Requirements (checked by the launcher): K % 8 == 0, lda and ldb multiples of 8
// elements, 16-byte aligned operand bases.  On return every wave's fragment reads have retired but other
// waves may still read `lds`: __syncthreads() before reusing it.  The epilogue is the caller's: it knows
// which operands to prefetch (issue them BEFORE this call: their latency then hides under the K loop).
template <int BM, int BN, int NPA, int NT = 512>
__device__ __forceinline__ void glds_gemm_mainloop(const __hip_bfloat16* __restrict__ A, int lda, int plane_bytes,
                                                   const __hip_bfloat16* __restrict__ B, int ldb, int M, int N, int K,
                                                   int m0, int n0, char* __restrict__ lds,
                                                   f32x4 (&acc)[GldsGeom<BM, BN>::MB][GldsGeom<BM, BN>::NB]) {
  using namespace gl;
  using G = GldsGeom<BM, BN>;
  constexpr int NW = NT / 64;
  static_assert(NW == 8, "8 waves (4 x 2)");
  constexpr int WM = G::WM, WN = G::WN, MB = G::MB, NB = G::NB;
  static_assert(MB >= 1 && NB >= 1 && BM % 64 == 0 && BN % 32 == 0, "tile too small for the wave layout");
  // 16-row DMA chunks per stage: A planes first, then B
  constexpr int ACH = NPA * BM / 16, BCH = BN / 16, CH = ACH + BCH;
  static_assert(CH % NW == 0, "DMA chunks must divide evenly over the waves");
  constexpr int L = CH / NW;  // DMA instructions per wave per stage
  constexpr int SB = stage_bytes<BM, BN, NPA>();

  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int fr = lane & 15, fg = lane >> 4;

  const __amdgpu_buffer_rsrc_t ra = make_rsrc(A), rb = make_rsrc(B);

  // this lane's DMA sources: chunk c = wave + NW * j; lane -> (row r = lane >> 2, physical slot lane & 3)
  const int dr = lane >> 2, dps = lane & 3;
  const int dkc = dps ^ gl::swz(dr);  // logical k-chunk this lane fetches
  int src[L];
  bool isA[L];
  int ldsoff[L];
#pragma unroll
  for (int j = 0; j < L; ++j) {
    const int c = wave + NW * j;  // wave-uniform
    if (c < ACH) {
      const int p = c / (BM / 16), rb16 = (c % (BM / 16)) * 16;
      const int row = m0 + rb16 + dr;
      isA[j] = true;
      src[j] = row < M ? p * plane_bytes + (row * lda + dkc * 8) * 2 : -1;
      ldsoff[j] = (p * BM + rb16) * kRowB;
    } else {
      const int rb16 = (c - ACH) * 16;
      const int row = n0 + rb16 + dr;
      isA[j] = false;
      src[j] = row < N ? (row * ldb + dkc * 8) * 2 : -1;
      ldsoff[j] = (NPA * BM + rb16) * kRowB;
    }
  }
  auto issue = [&](int kt) {
    const int k0 = kt * kBK;
    char* base = lds + (kt % kStages) * SB;
    const bool kok = k0 + dkc * 8 < K;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const int off = (src[j] >= 0 && kok) ? src[j] + k0 * 2 : kOOB;
      dma16(isA[j] ? ra : rb, base + ldsoff[j], off);
    }
  };

#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment reads: the 16x16x32 MFMA lane reads k = 8 fg .. 8 fg + 7 of the 32-deep stage = logical
  // chunk fg of row fr of a 16-row block, stored in physical slot fg ^ swz(fr)
  const int frag = fr * kRowB + ((fg ^ gl::swz(fr)) << 4);
  auto compute = [&](int kt) {
    const char* sA = lds + (kt % kStages) * SB + (wr * WM) * kRowB + frag;
    const char* sB = lds + (kt % kStages) * SB + (NPA * BM + wc * WN) * kRowB + frag;
    bf16x8_t bf[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) bf[nb] = *reinterpret_cast<const bf16x8_t*>(sB + nb * 16 * kRowB);
    bf16x8_t af[NPA][MB];
#pragma unroll
    for (int p = 0; p < NPA; ++p)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        af[p][mb] = *reinterpret_cast<const bf16x8_t*>(sA + (p * BM + mb * 16) * kRowB);
#pragma unroll
    for (int p = 0; p < NPA; ++p)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[p][mb], bf[nb], acc[mb][nb], 0, 0, 0);
  };

  const int nk = (K + kBK - 1) / kBK;
  // prologue: stages 0 .. kStages-2 in flight
#pragma unroll
  for (int s = 0; s < kStages - 1; ++s)
    if (s < nk) issue(s);

  for (int kt = 0; kt < nk; ++kt) {
    // stage kt landed (this wave's share): the younger issued stages may stay in flight
    const int younger = min(kStages - 2, nk - 1 - kt);
    if (younger >= 2) gl::wait_vm<2 * L>();
    else if (younger == 1) gl::wait_vm<L>();
    else gl::wait_vm<0>();
    // this wave's reads of stage kt-1 retired (its buffer is the next DMA target), then every wave's
    // share of stage kt is in LDS
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + kStages - 1 < nk) issue(kt + kStages - 1);
    compute(kt);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

}  // namespace cme
