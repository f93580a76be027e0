// The per-element arithmetic of the softmax / cross-entropy head (fpcode/gpu_func.cu gpuSoftmax +
// gpuElementwiseSum: D = (softmax(z2) - onehot) / batch), shared by every head that must produce BITWISE the same
// D: head_wide_kernel (mlp_kernels.hip) and the head fused into the wide forward launch (mlp_split.hip
// wide_head_ag).  Contraction is off inside: hipcc's default -ffp-contract=fast-honor-pragmas would otherwise
// fuse e * inv - 1 into an FMA in one kernel and not in the other (HIP's __fmul_rn is a plain multiply, so it
// does not prevent that), which made the two heads' D differ by an ulp.
#pragma once

namespace cme {

// y = e / sum as e * (1 / sum); d = (y - [class == label]) * scale.  Returns y (for the loss term).
__device__ __forceinline__ float head_prob_grad(float e, float inv, bool hit, float scale, float& d) {
#pragma clang fp contract(off)
  const float y = e * inv;
  d = (y - (hit ? 1.f : 0.f)) * scale;
  return y;
}

}  // namespace cme
