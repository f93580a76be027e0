// "A in registers" MFMA tile engine for the wide fp32 (split3) MLP GEMMs -- the fastest of the three wide
// engines at H = 4096 (round 1 register-staged, glds_gemm.h: direct-to-LDS, this one).
//
// Why (bench/micro/glds_fill.hip, profiles/wide_engines_r2.md): at the ~128 x 128 tile that ~224
// workgroups on 256 CUs allow, the wide GEMMs are bound by how many operand bytes each CU pulls from L2
// per FLOP, not by the MFMA pipe -- a CU takes in ~45-55 GB/s whether the bytes arrive by LDS-DMA or by
// vector loads.  The split3 operand stored as three bf16 planes costs 6 B per fp32 weight; read as fp32
// and split into the three exact bf16 planes in registers it costs 4 B (-25 % bytes per stage with a
// bf16 B operand), and the planes never have to be written at all.
//
// Layout: 8 waves, wave w owns the 16 rows m0 + 16 w + [0, 16) and all BN columns (NB = BN / 16 MFMA
// column blocks).  Rows are private to a wave, so A needs no LDS: each lane loads its 16x16x32 fragment
// (row lane & 15, k = 8 (lane >> 4) .. + 7 of the 32-deep stage) straight into registers -- 32 B of fp32
// (two dwordx4) or 16 B of bf16 -- into a 4-slot register ring, three stages ahead.  B (shared by the 8
// waves) goes global -> LDS by LDS-DMA into a 4-buffer ring, three stages in flight, with the XOR swizzle
// of glds_gemm.h (conflict-free ds_read_b128).  One counted vmcnt + lgkmcnt(0) + s_barrier per stage.
//
// fp32 A: the lane splits its 8 values into hi = bf16(x), mid = bf16(x - hi), lo = bf16(x - hi - mid)
// (exact: an fp32 significand is three bf16 significands; the same split as mlp_split.hip split_store),
// and multiplies hi, mid, lo against the same B fragment -- bit-identical to reading stored planes.
#pragma once

#include "glds_gemm.h"

namespace cme {

namespace ra {

constexpr int kBK = 32;
constexpr int kRowB = kBK * 2;  // LDS bytes per B row per stage (bf16)
constexpr int kBufs = 5;        // B LDS buffers and A register slots; 4 stages in flight

template <int BN>
constexpr int lds_bytes() {
  return kBufs * BN * kRowB;
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// one stage's A operand of one lane: MB row blocks x 8 k-values (fp32: two dwordx4 per block; bf16: one)
// (round 3 also read the three stored bf16 planes of an fp32 operand here; measured slower than the split in
// registers at 784-4096-10 -- profiles/wide_ag_ab_operand_forms_r3.jsonl -- and removed in round 4)
template <typename AT, int MB>
struct AFrag {
  static constexpr int Q = (sizeof(AT) == 4 ? 2 : 1) * MB;  // dwordx4 per lane
  u32x4 v[Q];
};

// A fragment loads are inline asm, hidden from hipcc's vmcnt bookkeeping (cdna_hip_programming.md §5
// 'Three .s-level traps' (b), §5.7 item 1 form (ii)): beside LDS-DMA in one K loop hipcc otherwise waits
// for them -- and for every DMA issued before them -- long before their registers are used, which cuts
// the pipeline to ~1 stage in flight.  Their completion is counted by hand (the per-stage vmcnt), and the
// wait statement names the destination registers ("+v"), so no consumer is scheduled above it.
template <int IMM>
__device__ __forceinline__ u32x4 load16_asm(__amdgpu_buffer_rsrc_t r, int voff) {
  u32x4 v;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3" : "=v"(v) : "v"(voff), "s"(r), "i"(IMM) : "memory");
  return v;
}

template <int N, typename AT, int MB>
__device__ __forceinline__ void wait_vm_regs(AFrag<AT, MB>& f) {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
#pragma unroll
  for (int q = 0; q < AFrag<AT, MB>::Q; ++q) asm volatile("" : "+v"(f.v[q]));
}

// the three exact bf16 planes of 8 fp32 values (two dwordx4)
__device__ __forceinline__ void split3(const u32x4& w0, const u32x4& w1, bf16x8_t& hi, bf16x8_t& mid,
                                       bf16x8_t& lo) {
  float x[8];
  __builtin_memcpy(x, &w0, 16);
  __builtin_memcpy(x + 4, &w1, 16);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h = (__bf16)x[j];
    const float r1 = x[j] - (float)h;
    const __bf16 m = (__bf16)r1;
    const float r2 = r1 - (float)m;
    hi[j] = h;
    mid[j] = m;
    lo[j] = (__bf16)r2;
  }
}

}  // namespace ra

// 8 waves as WR (rows) x WC (columns): wave (wr, wc) owns rows m0 + wr * 16 * MB + [0, 16 * MB) and
// columns n0 + wc * 16 * NB + [0, 16 * NB).  WC = 1: each wave 16 rows x all BN columns (every wave reads
// the whole B stage from LDS: 8 KB per wave per stage at BN = 128); WC = 2: 32 rows x BN / 2 columns (half
// the B fragment reads, each A row block loaded by the two column waves -- the second load hits L1).
template <int BN, int WC = 1>
struct RegaGeom {
  static constexpr int BM = 128, WR = 8 / WC, MB = WC, NB = BN / (16 * WC);
  static_assert(WR * 16 * MB == BM && NB >= 1, "8 waves cover 128 rows");
};

// K loop of the 128 x BN tile at (m0, n0) into acc[MB][NB] (zeroed here): C[m][n] = sum_k A[m][k] B[n][k].
// AT = float: A is fp32 split into 3 exact bf16 planes on the fly; AT = bf16: A is one bf16 plane.  B is
// bf16.  Requirements (launcher): K % 8 == 0, lda % 4 == 0 (fp32) / % 8 (bf16), ldb % 8 == 0, 16-byte
// aligned bases.  Ends with this wave's LDS reads retired (other waves may still read `lds`:
// __syncthreads() before reusing it).
// NKS > 0: exactly NKS stages (K in ((NKS-1)*32, NKS*32]), loop fully unrolled -- with a runtime trip
// count hipcc's vmcnt tracking merges at the back-edge and drains every load in flight (vmcnt(0)) once
// per trip before the A registers are used.
// ABLATE (bench/micro/rega_ablate.hip only): 1 = no MFMA (fragments still read and split, kept live),
// 2 = no loads after the prologue (the MFMAs run on whatever the ring holds)
// ASWZ (fp32 A): A is in the K loop's fragment order (dzr_off; the wide head's dZ1, SplitStepArgs::dz_swz == 2) and
// lda is the number of 32-k stages per 16-row block: each 16-byte load instruction of a wave reads 1 KB of contiguous
// memory instead of 16 rows x 64 B.
// Float offset of A(row, col) in that order (nst = stages per row block = cdiv(row length, 32)).
__host__ __device__ __forceinline__ int64_t dzr_off(int row, int col, int nst) {
  const int kt = col >> 5, w = col & 31, lane = (w >> 3) * 16 + (row & 15);
  return (((((int64_t)(row >> 4) * nst + kt) * 2 + ((w >> 2) & 1)) * 64 + lane) * 4) + (w & 3);
}
template <typename AT, int BN, int WC = 1, int NKS = 0, int ABLATE = 0, bool ASWZ = false>
__device__ __forceinline__ void rega_gemm_mainloop(const AT* __restrict__ A, int lda,
                                                   const __hip_bfloat16* __restrict__ B, int ldb, int M, int N,
                                                   int K, int m0, int n0, char* __restrict__ lds,
                                                   f32x4 (&acc)[RegaGeom<BN, WC>::MB][RegaGeom<BN, WC>::NB]) {
  using namespace ra;
  using G = RegaGeom<BN, WC>;
  constexpr int MB = G::MB, NB = G::NB, NW = 8;
  constexpr bool F32 = sizeof(AT) == 4;
  constexpr int SB = BN * kRowB;  // B bytes per stage
  static_assert(SB % (1024 * NW) == 0, "B DMA instructions must divide over the 8 waves");
  constexpr int LB = SB / 1024 / NW;            // B DMA instructions per wave per stage
  constexpr int LA = AFrag<AT, MB>::Q;          // A loads per lane per stage
  constexpr int LS = LB + LA;                   // vmcnt per stage per wave
  using AF = AFrag<AT, MB>;

  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = wave / WC, wc = wave % WC;
  const int fr = lane & 15, fg = lane >> 4;
  const __amdgpu_buffer_rsrc_t rsa = make_rsrc(A), rsb = make_rsrc(B);

  // A: rows m0 + 16 (MB wr + mb) + fr, k = 8 fg .. 8 fg + 7 of each stage
  int abase[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int arow = m0 + 16 * (MB * wr + mb) + fr;
    if constexpr (ASWZ) {
      static_assert(F32, "fragment-ordered A: fp32");
      abase[mb] = arow < M ? (((m0 >> 4) + MB * wr + mb) * lda * 2 * 64 + lane) * 16 : -1;
    } else {
      abase[mb] = arow < M ? (arow * lda + 8 * fg) * (int)sizeof(AT) : -1;
    }
  }
  // B DMA: chunk c = wave + 8 j of 16 rows; lane -> row lane >> 2, physical slot lane & 3 holding logical
  // k-chunk slot ^ gl::swz(row)
  const int dr = lane >> 2, dkc = (lane & 3) ^ gl::swz(dr);
  int bsrc[LB], blds[LB];
#pragma unroll
  for (int j = 0; j < LB; ++j) {
    const int rb16 = (wave + NW * j) * 16;
    const int row = n0 + rb16 + dr;
    bsrc[j] = row < N ? (row * ldb + dkc * 8) * 2 : -1;
    blds[j] = rb16 * kRowB;
  }

  auto issue = [&](int kt, AF& fa) {
    const int k0 = kt * kBK;
    char* base = lds + (kt % kBufs) * SB;
    const bool bk = k0 + dkc * 8 < K;
#pragma unroll
    for (int j = 0; j < LB; ++j) gl::dma16(rsb, base + blds[j], (bsrc[j] >= 0 && bk) ? bsrc[j] + k0 * 2 : kOOB);
    const bool ak = k0 + 8 * fg < K;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int ao = (abase[mb] >= 0 && ak) ? abase[mb] + (ASWZ ? kt * 2048 : k0 * (int)sizeof(AT)) : kOOB;
      if constexpr (ASWZ) {
        fa.v[2 * mb] = load16_asm<0>(rsa, ao);
        fa.v[2 * mb + 1] = load16_asm<1024>(rsa, ao);
      } else if constexpr (F32) {
        fa.v[2 * mb] = load16_asm<0>(rsa, ao);
        fa.v[2 * mb + 1] = load16_asm<16>(rsa, ao);
      } else {
        fa.v[mb] = load16_asm<0>(rsa, ao);
      }
    }
  };

#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int frag = (wc * 16 * NB + fr) * kRowB + ((fg ^ gl::swz(fr)) << 4);
  // one stage's MFMA operands in registers: NB B fragments (LDS) and the A planes (split of the A ring slot)
  constexpr int NPL = F32 ? 3 : 1;
  struct Frags {
    bf16x8_t b[NB];
    bf16x8_t a[MB][NPL];
  };
  auto load_frags = [&](int kt, Frags& F, const AF& fa) {
    const char* sB = lds + (kt % kBufs) * SB + frag;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) F.b[nb] = *reinterpret_cast<const bf16x8_t*>(sB + nb * 16 * kRowB);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      if constexpr (F32) {
        split3(fa.v[2 * mb], fa.v[2 * mb + 1], F.a[mb][0], F.a[mb][1], F.a[mb][2]);
      } else {
        __builtin_memcpy(&F.a[mb][0], &fa.v[mb], 16);
      }
    }
  };
  auto mma = [&](const Frags& F) {
    if constexpr (ABLATE == 1) {
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) asm volatile("" ::"v"(F.b[nb]));
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int p = 0; p < NPL; ++p) asm volatile("" ::"v"(F.a[mb][p]));
    } else {
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
          for (int p = 0; p < NPL; ++p)  // planes innermost: hi, mid, lo into the same accumulator
            acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(F.a[mb][p], F.b[nb], acc[mb][nb], 0, 0, 0);
    }
  };

  const int nk = NKS > 0 ? NKS : (K + kBK - 1) / kBK;
  AF ring[kBufs];
  Frags F[2];
  // stage s landed for this wave, with `younger` later stages allowed to stay in flight
  auto wait_stage = [&](int younger, AF& slot) {
    if (younger >= 3) wait_vm_regs<3 * LS>(slot);
    else if (younger == 2) wait_vm_regs<2 * LS>(slot);
    else if (younger == 1) wait_vm_regs<LS>(slot);
    else wait_vm_regs<0>(slot);
  };
  auto barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  asm volatile("s_nop 4" ::: "memory");  // descriptor SGPRs just written -> the asm loads read them
#pragma unroll
  for (int s = 0; s < kBufs - 1; ++s)
    if (s < nk) issue(s, ring[s]);
  wait_stage(min(kBufs - 2, nk - 1), ring[0]);
  barrier();
  load_frags(0, F[0], ring[0]);

  // Stage kt: its operands are already in registers (F[kt & 1], read during stage kt-1).  Wait for stage
  // kt+1 to land, barrier (it is visible to every wave; every wave's reads of stage kt-1's buffer are
  // retired), refill that buffer with stage kt+kBufs-1, read stage kt+1's fragments into the other
  // register set, and multiply stage kt.
  auto stage = [&](int kt, int slot_next, Frags& Fcur, Frags& Fnext) {
    if (kt + 1 < nk) wait_stage(min(kBufs - 3, nk - 2 - kt), ring[slot_next]);
    barrier();
    if (ABLATE != 2 && kt + kBufs - 1 < nk) issue(kt + kBufs - 1, ring[(slot_next + kBufs - 2) % kBufs]);
    if (kt + 1 < nk) load_frags(kt + 1, Fnext, ring[slot_next]);
    mma(Fcur);
  };
  if constexpr (NKS > 0) {
#pragma unroll
    for (int kt = 0; kt < NKS; ++kt) stage(kt, (kt + 1) % kBufs, F[kt & 1], F[(kt + 1) & 1]);
  } else {
    // 2 * kBufs stages per trip: every ring slot and register set index is a compile-time constant
    for (int k0 = 0; k0 < nk; k0 += 2 * kBufs) {
#pragma unroll
      for (int d = 0; d < 2 * kBufs; ++d) {
        if (k0 + d >= nk) break;
        stage(k0 + d, (d + 1) % kBufs, F[d & 1], F[(d + 1) & 1]);
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

}  // namespace cme
