// The weight-gradient epilogues and the small helpers they share (split planes, the fused exchange's
// system-coherent gradient store, the forward-timed-out word): used by the two-launch step's weight-gradient
// kernels (mlp_split.hip) and by the XCD-local step pipeline (xstep.hip), so both apply bit-identical updates.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include "mlp_split.h"
#include "mma_tile.h"

namespace cme {
namespace wg {

using bf16 = __hip_bfloat16;

// exact np-way split of an fp32 value into bf16 planes (np = 1: plain rounding)
template <int NP>
__device__ __forceinline__ void split_store(float v, bf16* base, size_t plane_stride, size_t idx) {
  float r = v;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const bf16 h = __float2bfloat16(r);
    base[p * plane_stride + idx] = h;
    r -= __bfloat162float(h);
  }
}

constexpr int kXfSys = 1 | 16;  // cache policy sc0 | sc1: system coherent

// The forward + head launch of this step timed out (SplitStepArgs::ag_err): the word is loaded (a vector
// atomic load from L2) BEFORE the K loop, like the epilogue's other operands, and tested only by the epilogue
// (poisoned()), so its latency hides behind the loop.
__device__ __forceinline__ int ag_err_load(const int* e) {
  return e ? __hip_atomic_load(e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
}
__device__ __forceinline__ bool poisoned(int v) { return __builtin_amdgcn_readfirstlane(v) != 0; }

__device__ __forceinline__ void xf_store(float* base, int64_t idx, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), make_rsrc(base), (int)(idx * 4), 0, kXfSys);
}

// this lane's share of sum(src[0:n]) (combine with wave_sum); CP: the loads' cache policy (kSc1 where another
// workgroup of the same launch wrote src: the XCD-local step pipeline's db2)
template <int CP = 0>
__device__ __forceinline__ float row_sum(const float* src, int n, int lane) {
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(src);
  float s = 0.f;
  for (int j0 = 0; j0 < n; j0 += 64 * 16) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int j = j0 + u * 64 + lane;
      v[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, j < n ? j * 4 : kOOB, 0, CP));
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) s += v[u];
  }
  return s;
}

struct EpiW2 {
  float* W2;
  float* gW2;
  int H, sgd;
  int sys;  // gradients into a peer-visible IPC buffer (write-through)
  float reg, lr;
  float pre[kEpiMaxQ];
  const int* ag_err;  // the step's forward timed out: no update (the gradient goes to gW2, unused)
  int perr = 0;
  // sys == 2 (the push form): gradient / current weight into LDS xs / xo[class * 16 + column - n0]
  float *xs = nullptr, *xo = nullptr;
  int n0 = 0;
  __device__ __forceinline__ void prefetch(int q, int row, int col, bool ok) {
    pre[q] = buf_load1<float>(make_rsrc(W2), ok ? (row * H + col) * 4 : kOOB);
    if (q == 0) perr = ag_err_load(ag_err);
  }
  __device__ __forceinline__ void operator()(int q, int row, int col, float v) {
    const size_t i = (size_t)row * H + col;
    const float w = pre[q];
    const float g = v + reg * w;
    if (sgd && !poisoned(perr)) W2[i] = w - lr * g;
    else if (sys == 2) {
      xs[row * 16 + col - n0] = g;
      xo[row * 16 + col - n0] = w;
    }
    else if (sys) xf_store(gW2, (int64_t)i, g);
    else gW2[i] = g;
  }
};

struct EpiW1 {
  float* W1;
  float* gW1;
  bf16* W1p;
  size_t plane;  // H*P
  int P, sgd, npw;
  float reg, lr, xscale;
  float pre[kEpiMaxQ];
  float* b1;
  float* gb1;
  int sys;  // gradients into a peer-visible IPC buffer (write-through)
  const int* ag_err;  // the step's forward timed out: no update (the gradient goes to gW1, unused)
  int perr = 0;
  // sys == 2 (the push form): the gradient into LDS xs[(row - m0) * 32 + col - n0] and the current weight (or b1)
  // into xo
  float *xs = nullptr, *xo = nullptr;
  int m0 = 0, n0 = 0;
  float* W1s = nullptr;  // the fragment-ordered copy the forward reads (SplitStepArgs::W1s): updated with W1
  __device__ __forceinline__ void prefetch(int q, int row, int col, bool ok) {
    // (the all-ones feature column P: b1[row], so its update is not a dependent load after the K loop)
    if (col == P) pre[q] = buf_load1<float>(make_rsrc(b1), ok ? row * 4 : kOOB);
    else pre[q] = buf_load1<float>(make_rsrc(W1), (ok && col < P) ? (row * P + col) * 4 : kOOB);
    if (q == 0) perr = ag_err_load(ag_err);
  }
  __device__ __forceinline__ void operator()(int q, int row, int col, float v) {
    const bool upd = sgd && !poisoned(perr);
    if (col == P) {  // the all-ones feature: db1[row] (no input scale, no regulariser)
      if (upd) b1[row] = pre[q] - lr * v;
      else if (sys == 2) {
        xs[(row - m0) * 32 + col - n0] = v;
        xo[(row - m0) * 32 + col - n0] = pre[q];
      } else if (sys) xf_store(gb1, row, v);
      else gb1[row] = v;
      return;
    }
    const size_t i = (size_t)row * P + col;
    const float w = pre[q];
    const float g = v * xscale + reg * w;
    if (upd) {
      const float nw = w - lr * g;
      W1[i] = nw;
      if (W1s) W1s[w1s_off(row, col, (P + 63) >> 6)] = nw;
      if (npw == 3) split_store<3>(nw, W1p, plane, i);
      else if (npw == 1) split_store<1>(nw, W1p, plane, i);  // (0: no forward kernel reads the planes)
    } else if (sys == 2) {
      xs[(row - m0) * 32 + col - n0] = g;
      xo[(row - m0) * 32 + col - n0] = w;
    } else if (sys) {
      xf_store(gW1, (int64_t)i, g);
    } else {
      gW1[i] = g;
    }
  }
};

}  // namespace wg
}  // namespace cme
