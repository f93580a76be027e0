// "A in registers" MFMA tile engine for the wide fp32 (split3) MLP GEMMs -- the fastest of the three wide
// engines at H = 4096 (lds_gemm.h: register-staged, glds_gemm.h: direct-to-LDS, this one).
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
constexpr int kBufs = 4;        // B LDS buffers and A register slots; 3 stages in flight

template <int BN>
constexpr int lds_bytes() {
  return kBufs * BN * kRowB;
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <typename AT>
struct AFrag;
template <>
struct AFrag<float> {
  u32x4 v[2];  // 8 fp32
};
template <>
struct AFrag<__hip_bfloat16> {
  u32x4 v[1];  // 8 bf16
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

template <int N, typename AT>
__device__ __forceinline__ void wait_vm_regs(AFrag<AT>& f) {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  if constexpr (sizeof(AT) == 4)
    asm volatile("s_waitcnt vmcnt(%2)" : "+v"(f.v[0]), "+v"(f.v[1]) : "n"(N) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%1)" : "+v"(f.v[0]) : "n"(N) : "memory");
}

// the three exact bf16 planes of 8 fp32 values
__device__ __forceinline__ void split3(const AFrag<float>& f, bf16x8_t& hi, bf16x8_t& mid, bf16x8_t& lo) {
  float x[8];
  __builtin_memcpy(x, f.v, 32);
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

template <int BN>
struct RegaGeom {
  static constexpr int BM = 128, NB = BN / 16;
};

// K loop of the BM(=128) x BN tile at (m0, n0) into acc[NB] (zeroed here): C[m][n] = sum_k A[m][k] B[n][k].
// AT = float: A is fp32 split into NPA (= 3) exact bf16 planes on the fly; AT = bf16: A is one bf16
// plane (NPA = 1).  B is bf16.  Requirements (launcher): K % 8 == 0, lda % 4 == 0 (fp32) / % 8 (bf16),
// ldb % 8 == 0, 16-byte aligned bases.  Ends with this wave's LDS reads retired (other waves may still
// read `lds`: __syncthreads() before reusing it).
// NKS > 0: exactly NKS stages (K in ((NKS-1)*32, NKS*32]), loop fully unrolled -- with a runtime trip
// count hipcc's vmcnt tracking merges at the back-edge and drains every load in flight (vmcnt(0)) once
// per trip before the A registers are used.
template <typename AT, int BN, int NKS = 0>
__device__ __forceinline__ void rega_gemm_mainloop(const AT* __restrict__ A, int lda,
                                                   const __hip_bfloat16* __restrict__ B, int ldb, int M, int N,
                                                   int K, int m0, int n0, char* __restrict__ lds,
                                                   f32x4 (&acc)[RegaGeom<BN>::NB]) {
  using namespace ra;
  constexpr int NB = RegaGeom<BN>::NB, NW = 8;
  constexpr bool F32 = sizeof(AT) == 4;
  constexpr int SB = BN * kRowB;  // B bytes per stage
  static_assert(SB % (1024 * NW) == 0, "B DMA instructions must divide over the 8 waves");
  constexpr int LB = SB / 1024 / NW;            // B DMA instructions per wave per stage
  constexpr int LA = F32 ? 2 : 1;               // A loads per lane per stage
  constexpr int LS = LB + LA;                   // vmcnt per stage per wave

  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const __amdgpu_buffer_rsrc_t rsa = make_rsrc(A), rsb = make_rsrc(B);

  // A: row m0 + 16 wave + fr, k = 8 fg .. 8 fg + 7 of each stage
  const int arow = m0 + 16 * wave + fr;
  const int abase = arow < M ? (arow * lda + 8 * fg) * (int)sizeof(AT) : -1;
  // B DMA: chunk c = wave + 8 j of 16 rows; lane -> row lane >> 2, physical slot lane & 3 holding logical
  // k-chunk slot ^ ((row >> 2) & 3)
  const int dr = lane >> 2, dkc = (lane & 3) ^ ((dr >> 2) & 3);
  int bsrc[LB], blds[LB];
#pragma unroll
  for (int j = 0; j < LB; ++j) {
    const int rb16 = (wave + NW * j) * 16;
    const int row = n0 + rb16 + dr;
    bsrc[j] = row < N ? (row * ldb + dkc * 8) * 2 : -1;
    blds[j] = rb16 * kRowB;
  }

  auto issue = [&](int kt, AFrag<AT>& fa) {
    const int k0 = kt * kBK;
    char* base = lds + (kt % kBufs) * SB;
    const bool bk = k0 + dkc * 8 < K;
#pragma unroll
    for (int j = 0; j < LB; ++j) gl::dma16(rsb, base + blds[j], (bsrc[j] >= 0 && bk) ? bsrc[j] + k0 * 2 : kOOB);
    const int ao = (abase >= 0 && k0 + 8 * fg < K) ? abase + k0 * (int)sizeof(AT) : kOOB;
    fa.v[0] = load16_asm<0>(rsa, ao);
    if constexpr (LA == 2) fa.v[1] = load16_asm<16>(rsa, ao);
  };

#pragma unroll
  for (int j = 0; j < NB; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int frag = fr * kRowB + ((fg ^ ((fr >> 2) & 3)) << 4);
  auto compute = [&](int kt, const AFrag<AT>& fa) {
    const char* sB = lds + (kt % kBufs) * SB + frag;
    bf16x8_t bf[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) bf[nb] = *reinterpret_cast<const bf16x8_t*>(sB + nb * 16 * kRowB);
    if constexpr (F32) {
      bf16x8_t h, m, l;
      split3(fa, h, m, l);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h, bf[nb], acc[nb], 0, 0, 0);
        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(m, bf[nb], acc[nb], 0, 0, 0);
        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(l, bf[nb], acc[nb], 0, 0, 0);
      }
    } else {
      bf16x8_t a;
      __builtin_memcpy(&a, fa.v, 16);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bf[nb], acc[nb], 0, 0, 0);
    }
  };

  const int nk = NKS > 0 ? NKS : (K + kBK - 1) / kBK;
  AFrag<AT> ring[kBufs];
  asm volatile("s_nop 4" ::: "memory");  // descriptor SGPRs just written -> the asm loads read them
#pragma unroll
  for (int s = 0; s < kBufs - 1; ++s)
    if (s < nk) issue(s, ring[s]);

  auto stage = [&](int kt, int d) {
    const int younger = min(kBufs - 2, nk - 1 - kt);
    if (younger >= 2) wait_vm_regs<2 * LS>(ring[d]);
    else if (younger == 1) wait_vm_regs<LS>(ring[d]);
    else wait_vm_regs<0>(ring[d]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // stage kt + 3 reuses B buffer (kt - 1) % 4 (every wave is past its reads: the barrier) and A slot
    // (kt + 3) % 4 == (kt - 1) % 4, consumed by the previous stage's compute
    if (kt + kBufs - 1 < nk) issue(kt + kBufs - 1, ring[(d + kBufs - 1) % kBufs]);
    compute(kt, ring[d]);
  };
  if constexpr (NKS > 0) {
#pragma unroll
    for (int kt = 0; kt < NKS; ++kt) stage(kt, kt % kBufs);
  } else {
    // 4 stages per trip so every ring slot index is a compile-time constant
    for (int k4 = 0; k4 < nk; k4 += kBufs) {
#pragma unroll
      for (int d = 0; d < kBufs; ++d) {
        if (k4 + d >= nk) break;
        stage(k4 + d, d);
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

}  // namespace cme
