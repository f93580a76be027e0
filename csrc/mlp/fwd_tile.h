// The forward GEMM tile of the small-layer kernels (fwd1_split_kernel, fwd1_head_kernel,
// fwd1_head_ag_kernel): a1 tile = W1[rows] . X[cols]^T on the wave-split-K engine (mma_tile.h), W1 either
// from its stored bf16 planes or (AF, split3) straight from fp32 W1, split into the exact planes in
// registers -- 4 B per weight through the CU's ~50 GB/s L2 fill instead of 6 B.
#pragma once

#include "mlp_split.h"
#include "mma_tile.h"

namespace cme {

// SWZ (AF, VEC == 3; a template argument, not a runtime test: the kernels that never read the copies carry none of
// their code): bit0 reads fp32 W1 from its fragment-ordered copy f.W1s, bit1 also the pixels from theirs, f.Xs
// (SplitStepArgs::w1_swz / x_swz; both need K pairs that start at multiples of 64: mlp_fwd_swz_ok)
// CPA: the W1-copy loads' cache policy (wsk_tile; kSc1 in the XCD-local step pipeline, where other workgroups of the
// same launch rewrite W1s between steps)
template <int NPW, int NB, int VEC, int U, bool AF, int SWZ = 0, int CPA = 0, class Epi>
__device__ __forceinline__ void fwd_tile(const SplitStepArgs& f, const TileGeom& g, Epi& epi, float* red,
                                         unsigned long long* stamps = nullptr) {
  const uint8_t* X = static_cast<const uint8_t*>(f.X);
  if constexpr (AF) {
    static_assert(NPW == 3, "fp32 W1 is split into three planes");
    if constexpr (SWZ != 0) {  // the fragment-ordered fp32 copy of W1 (SplitStepArgs::w1_swz)
      static_assert(VEC == 3 && (SWZ & 1), "fragment-ordered W1 (+ pixels): 16-byte pixel pairs");
      const int npair = (f.P + 63) / 64;
      if constexpr ((SWZ & 2) != 0)
        wsk_tile<__hip_bfloat16, 1, NB, 8, true, true, VEC, U, 3, uint8_t, float, true, true, CPA>(
            f.W1s, npair, static_cast<const uint8_t*>(f.Xs), npair, g, epi, red, 0, stamps);
      else
        wsk_tile<__hip_bfloat16, 1, NB, 8, true, true, VEC, U, 3, uint8_t, float, true, false, CPA>(
            f.W1s, npair, X, f.P, g, epi, red, 0, stamps);
    } else {
      static_assert(CPA == 0, "a W1 cache policy only on the fragment-ordered copy");
      wsk_tile<__hip_bfloat16, 1, NB, 8, true, true, VEC, U, 3, uint8_t>(f.W1, f.P, X, f.P, g, epi, red, 0, stamps);
    }
  } else {
    static_assert(CPA == 0, "a W1 cache policy only on the fragment-ordered copy");
    wsk_tile<__hip_bfloat16, 1, NB, 8, true, true, VEC, U, NPW, uint8_t>(
        static_cast<const __hip_bfloat16*>(f.W1p), f.P, X, f.P, g, epi, red, f.H * f.P * (int)sizeof(__hip_bfloat16),
        stamps);
  }
}

}  // namespace cme
