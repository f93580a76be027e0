// The forward GEMM tile of the small-layer kernels (fwd1_split_kernel, fwd1_head_kernel,
// fwd1_head_ag_kernel): a1 tile = W1[rows] . X[cols]^T on the wave-split-K engine (mma_tile.h), W1 either
// from its stored bf16 planes or (AF, split3) straight from fp32 W1, split into the exact planes in
// registers -- 4 B per weight through the CU's ~50 GB/s L2 fill instead of 6 B.
//
// img != nullptr (SplitStepArgs::fwd_lds, the all-gather forward + head): the tile's operands are first staged
// WHOLE into LDS by LDS-DMA -- the 16 W1 rows (one contiguous block of global memory: 16 x P x 4 B) and the 32
// pixel rows (one contiguous block: 32 x P B) as 1-KB lane-linear DMA instructions, every 128-B line read in full
// once -- and the K loop reads its fragments from there.  The per-wave fragment loads of the global form touch
// 16 rows x 64 B per instruction (fragment-shaped: cdna_hip_programming.md §5, the projection-GEMM table), and
// the headline forward's K loop is bound by that fill (~75 KB per CU, bench/stamps_fha.py per-wave K loops).
// Same K ranges, pairing, split and MFMA order as the global form: bitwise the same a1.
#pragma once

#include "glds_gemm.h"
#include "mlp_split.h"
#include "mma_tile.h"

namespace cme {

namespace fimg {
// 16-byte slots per LDS row of the A image: the row's slots rounded up to an ODD count (rows 16 B apart in bank
// terms modulo 256 B, fewer b128 conflicts)
__host__ __device__ constexpr int a_slots(int P, int es) { return ((P * es / 16) | 1); }
__host__ __device__ constexpr int a_bytes(int P, int es) { return (16 * a_slots(P, es) * 16 + 1023) / 1024 * 1024; }
__host__ __device__ constexpr int b_bytes(int P, int NB) { return (16 * NB * P + 1023) / 1024 * 1024; }
// the image for an NB-block tile (caller's dynamic LDS)
__host__ __device__ constexpr int bytes(int P, int es, int NB) { return a_bytes(P, es) + b_bytes(P, NB); }
// the form applies: P a multiple of 16 (whole 16-byte slots, and the u8 rows 16-byte aligned)
__host__ __device__ constexpr bool ok(int P) { return P % 16 == 0; }
}  // namespace fimg

// Stage the tile's A rows [m0, m0 + 16) (row pitch P elements of es bytes, rows >= M zero) and B rows
// [n0, n0 + 16 NB) (uint8, pitch P, rows >= N zero) into img; returns after every wave's DMAs landed and the
// workgroup's barrier (the image is then complete for every wave).
template <int NB>
__device__ __forceinline__ void fwd_stage(const void* A, int es, const uint8_t* X, int P, int M, int N, int m0,
                                          int n0, char* img) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int SR = fimg::a_slots(P, es), rowb = P * es;
  const int ia = fimg::a_bytes(P, es) / 1024, ib = fimg::b_bytes(P, NB) / 1024;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(static_cast<const char*>(A) + (size_t)m0 * rowb);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(X + (size_t)n0 * P);
  const int arows = min(16, M - m0), bbytes = min(16 * NB, N - n0) * P;
  for (int j = wave; j < ia; j += 8) {
    const int slot = j * 64 + lane, r = slot / SR, c = slot - r * SR;
    gl::dma16(ra, img + j * 1024, (r < arows && c * 16 < rowb) ? r * rowb + c * 16 : kOOB);
  }
  char* bimg = img + fimg::a_bytes(P, es);
  for (int j = wave; j < ib; j += 8) {
    const int off = (j * 64 + lane) * 16;
    gl::dma16(rb, bimg + j * 1024, off < bbytes ? off : kOOB);
  }
  gl::wait_vm<0>();
  __syncthreads();
}

template <int NPW, int NB, int VEC, int U, bool AF, class Epi>
__device__ __forceinline__ void fwd_tile(const SplitStepArgs& f, const TileGeom& g, Epi& epi, float* red,
                                         unsigned long long* stamps = nullptr, char* img = nullptr) {
  const uint8_t* X = static_cast<const uint8_t*>(f.X);
  const int krot = f.k_rot ? (g.n0 / (16 * NB)) % 7 : -1;  // (SplitStepArgs::k_rot)
  if constexpr (AF) {
    static_assert(NPW == 3, "fp32 W1 is split into three planes");
    if constexpr (VEC == 1 || VEC == 3) {
      if (img) {
        fwd_stage<NB>(f.W1, 4, X, f.P, g.M, g.N, g.m0, g.n0, img);
        wsk_tile<__hip_bfloat16, 1, NB, 8, true, true, VEC, U, 3, uint8_t, float, true>(
            f.W1, f.P, X, f.P, g, epi, red, 0, stamps, krot, img, fimg::a_slots(f.P, 4) * 16, img + fimg::a_bytes(f.P, 4),
            f.P);
        return;
      }
    }
    wsk_tile<__hip_bfloat16, 1, NB, 8, true, true, VEC, U, 3, uint8_t>(f.W1, f.P, X, f.P, g, epi, red, 0, stamps,
                                                                       krot);
  } else {
    if constexpr (NPW == 1 && (VEC == 1 || VEC == 3)) {
      if (img) {
        const __hip_bfloat16* W = static_cast<const __hip_bfloat16*>(f.W1p);
        fwd_stage<NB>(W, 2, X, f.P, g.M, g.N, g.m0, g.n0, img);
        wsk_tile<__hip_bfloat16, 1, NB, 8, true, true, VEC, U, 1, uint8_t, __hip_bfloat16, true>(
            W, f.P, X, f.P, g, epi, red, 0, stamps, krot, img, fimg::a_slots(f.P, 2) * 16, img + fimg::a_bytes(f.P, 2),
            f.P);
        return;
      }
    }
    wsk_tile<__hip_bfloat16, 1, NB, 8, true, true, VEC, U, NPW, uint8_t>(
        static_cast<const __hip_bfloat16*>(f.W1p), f.P, X, f.P, g, epi, red, f.H * f.P * (int)sizeof(__hip_bfloat16),
        stamps, krot);
  }
}

}  // namespace cme
