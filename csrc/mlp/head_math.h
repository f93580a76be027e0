// The per-element arithmetic of the softmax / cross-entropy head (fpcode/gpu_func.cu gpuSoftmax +
// gpuElementwiseSum: D = (softmax(z2) - onehot) / batch), shared by every head that must produce BITWISE the same
// D: head_wide_kernel (mlp_kernels.hip) and the head fused into the wide forward launch (mlp_split.hip
// wide_head_ag).  Contraction is off inside: hipcc's default -ffp-contract=fast-honor-pragmas would otherwise
// fuse e * inv - 1 into an FMA in one kernel and not in the other (HIP's __fmul_rn is a plain multiply, so it
// does not prevent that), which made the two heads' D differ by an ulp.
#pragma once

namespace cme {

// The fp32 sigmoid of every forward epilogue (split and MFMA paths alike, so that the forms that tests pin
// BITWISE against each other agree): 1 / (1 + e^-x) with the hardware reciprocal (v_rcp_f32, 1 ulp) instead
// of the IEEE division, which hipcc expands to ~10 dependent instructions (v_div_scale x2, v_div_fmas,
// v_div_fixup and their FMAs) -- 32 of them per lane in the wide forward epilogue, on the critical path before
// the z2 hand-off.  x -> -inf: rcp(inf) = 0; x -> +inf: rcp(1) = 1.
__device__ __forceinline__ float sigmoid_f32(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

// y = e / sum as e * (1 / sum); d = (y - [class == label]) * scale.  Returns y (for the loss term).
__device__ __forceinline__ float head_prob_grad(float e, float inv, bool hit, float scale, float& d) {
#pragma clang fp contract(off)
  const float y = e * inv;
  d = (y - (hit ? 1.f : 0.f)) * scale;
  return y;
}

}  // namespace cme
