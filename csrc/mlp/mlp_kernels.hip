// Fused MLP step kernels for MI355X (gfx950).  See mlp_kernels.h for the
// step decomposition and mma_tile.h for the MFMA tile engine.
#include "mlp_kernels.h"
#include "mlp_split.h"

#include "mma_tile.h"
#include "fwd_tile.h"
#include "fha_body.h"
#include "l2_touch.h"
#include "head_math.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace cme {

namespace {

template <typename T>
__device__ __forceinline__ T dev_exp(T x);
template <>
__device__ __forceinline__ float dev_exp<float>(float x) { return __expf(x); }
template <>
__device__ __forceinline__ double dev_exp<double>(double x) { return exp(x); }

template <typename T>
__device__ __forceinline__ T dev_log(T x);
template <>
__device__ __forceinline__ float dev_log<float>(float x) { return __logf(x); }
template <>
__device__ __forceinline__ double dev_log<double>(double x) { return log(x); }

template <typename T>
__device__ __forceinline__ T sigmoid_(T x) { return T(1) / (T(1) + dev_exp<T>(-x)); }
template <>
__device__ __forceinline__ float sigmoid_<float>(float x) { return sigmoid_f32(x); }  // (head_math.h)

// ---------------------------------------------------------------- K1: forward
template <typename P>  // param / activation type
struct EpiBiasAct {
  const P* __restrict__ bias;
  P* __restrict__ out;
  int ldo;
  int act;  // 0 none, 1 sigmoid, 2 relu
  P pre[kEpiMaxQ];
  __device__ __forceinline__ void prefetch(int q, int row, int, bool ok) {
    pre[q] = buf_load1<P>(make_rsrc(bias), ok ? row * (int)sizeof(P) : kOOB);
  }
  template <typename A>
  __device__ __forceinline__ void operator()(int q, int row, int col, A v) {
    P z = P(v) + pre[q];
    if (act == 1) z = sigmoid_<P>(z);
    else if (act == 2) z = z > P(0) ? z : P(0);
    out[(size_t)row * ldo + col] = z;
  }
};

constexpr int kFwdMB = 1, kFwdNB = 2, kKS = 8;
constexpr int kThreads = 64 * kKS;

// chunks-per-iteration: enough to issue a wave's whole K-slice in one burst
template <typename T>
constexpr int unroll_for() { return sizeof(T) == 4 ? 8 : 4; }

template <typename T, typename P, bool VEC>
__global__ __launch_bounds__(kThreads) void fwd1_kernel(const T* __restrict__ W1, const P* __restrict__ b1,
                                                   const T* __restrict__ X, int Pdim, int H, int n,
                                                   P* __restrict__ a1, int lda, int act, int tiles_n) {
  using acc_t = typename MmaTraits<T>::acc_t;
  __shared__ acc_t red[kKS * kFwdMB * kFwdNB * 4 * 64];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  TileGeom g{H, n, Pdim, (bid / tiles_n) * 16 * kFwdMB, (bid % tiles_n) * 16 * kFwdNB};
  EpiBiasAct<P> epi{b1, a1, lda, act, {}};
  constexpr int U = unroll_for<T>();
  wsk_tile<T, kFwdMB, kFwdNB, kKS, true, true, VEC, U>(W1, Pdim, X, Pdim, g, epi, red);
}

// ------------------------------------------------------------------ K2: head
// One workgroup = COLS columns (samples) x (256/COLS) parts of the hidden dim.
// NC = number of classes padded to a compile-time constant (10 or 16): class
// loops are fully unrolled with no data-dependent branches around loads.
// W2^T is staged once per workgroup in LDS ([h][NC]) when it fits, so every
// weight read in both passes is an LDS broadcast instead of a global load.
constexpr int kHeadCols = 16;
constexpr int kCMax = 16;
constexpr int kHeadLdsMax = 64 * 1024;

// Stage W2^T ([h][NC], zero past C) and b2 (NC values, zero past C) into LDS: ws[H*NC] then b2s[NC]
// (head_lds_elems).  Every load is a range-checked buffer load issued in one burst per thread
// (a guarded `c < C ? W2[..] : 0` becomes a branch + vmcnt(0) wait per element).  nthr threads.
__host__ __device__ inline int head_lds_elems(int H, int NC) { return H * NC + NC; }

template <typename P, int NC>
__device__ __forceinline__ void head_stage(const HeadArgs& a, int t, int nthr, P* ws) {
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.W2), rb = make_rsrc(a.b2);
  const int H = a.H, C = a.C, tot = H * NC;
  for (int i0 = t; i0 < tot; i0 += 4 * nthr) {
    P v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * nthr, h = i / NC, c = i - h * NC;
      v[u] = buf_load1<P>(rw, (i < tot && c < C) ? (c * H + h) * (int)sizeof(P) : kOOB);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i0 + u * nthr < tot) ws[i0 + u * nthr] = v[u];
  }
  if (t < NC) ws[tot + t] = buf_load1<P>(rb, t < C ? t * (int)sizeof(P) : kOOB);
}

template <typename P, int NC, bool LDSW>
__device__ __forceinline__ void head_block(const HeadArgs& a, const int vb, const int t, char* head_dyn,
                                           P (*zred)[NC][kHeadCols], float* lred) {
  // One head block (kHeadCols columns, 256 threads) -- vb: the block index, t: thread in [0, 256);
  // every barrier below is reached by all threads of the workgroup.  (fp64 and the head-alone profiling hook
  // only: the fp32 / bf16 training steps take the MFMA heads)
  constexpr int COLS = kHeadCols;
  constexpr int NPART = 256 / COLS;
  const P* __restrict__ a1 = static_cast<const P*>(a.a1);
  const P* __restrict__ W2 = static_cast<const P*>(a.W2);
  const P* __restrict__ b2 = static_cast<const P*>(a.b2);
  P* ws = reinterpret_cast<P*>(head_dyn);
  const int lane = t & 63, wave = t >> 6;
  const int col = t % COLS, part = t / COLS;
  const int H = a.H, C = a.C;
  const int bcol = vb * COLS + col;
  const bool valid = bcol < a.n;
  const int b = valid ? bcol : a.n - 1;  // clamped: loads stay in bounds, results discarded
  const int lab = a.mode == HEAD_TRAIN ? a.labels[b] : 0;

  if constexpr (LDSW) {
    head_stage<P, NC>(a, t, 256, ws);
    __syncthreads();
  }
  auto w2 = [&](int c, int h) -> P {
    if constexpr (LDSW) return ws[h * NC + c];
    else return c < C ? W2[(c < C ? c : C - 1) * H + h] : P(0);
  };

  // ---- pass 1: z2 partial sums over this thread's hidden units
  P z[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) z[c] = P(0);
  {
    int h = part;
    for (; h + 3 * NPART < H; h += 4 * NPART) {
      P x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) x[u] = a1[(size_t)(h + u * NPART) * a.lda + b];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int c = 0; c < NC; ++c) z[c] += w2(c, h + u * NPART) * x[u];
    }
    for (; h < H; h += NPART) {
      const P x = a1[(size_t)h * a.lda + b];
#pragma unroll
      for (int c = 0; c < NC; ++c) z[c] += w2(c, h) * x;
    }
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
#pragma unroll
    for (int o = COLS; o < 64; o <<= 1) z[c] += __shfl_xor(z[c], o, 64);
  }
  if (lane < COLS) {
#pragma unroll
    for (int c = 0; c < NC; ++c) zred[wave][c][col] = z[c];
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < NC; ++c)
    z[c] = zred[0][c][col] + zred[1][c][col] + zred[2][c][col] + zred[3][c][col] +
           (LDSW ? ws[H * NC + c] : (c < C ? b2[c < C ? c : 0] : P(0)));

  if (a.mode == HEAD_PREDICT) {
    if (part == 0 && valid) {
      int best = 0;
      P bv = z[0];
#pragma unroll
      for (int c = 1; c < NC; ++c)
        if (c < C && z[c] > bv) { bv = z[c]; best = c; }
      a.pred[bcol] = best;
    }
    return;
  }

  // ---- softmax over the C classes of this column (registers only)
  P m = P(0);
  if (a.shift) {
    m = z[0];
#pragma unroll
    for (int c = 1; c < NC; ++c) m = (c < C && z[c] > m) ? z[c] : m;
  }
  P s = P(0);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    z[c] = c < C ? dev_exp<P>(z[c] - m) : P(0);
    s += z[c];
  }
  const P inv = P(1) / s;
#pragma unroll
  for (int c = 0; c < NC; ++c) z[c] *= inv;  // yhat

  if (a.mode == HEAD_PROBS) {
    if (part == 0 && valid) {
      P* probs = static_cast<P*>(a.probs);
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (c < C) probs[(size_t)c * a.ldp + bcol] = z[c];
    }
    return;
  }

  // ---- train: D = (yhat - onehot) * scale  (fused softmax + cross-entropy gradient)
  float lpart = 0.f;
  if (a.loss_partial && part == 0 && valid) {
    P pl = P(0);
#pragma unroll
    for (int c = 0; c < NC; ++c) pl = c == lab ? z[c] : pl;
    lpart = -(float)dev_log<P>(pl);
  }
  const P sc = P(a.scale);
#pragma unroll
  for (int c = 0; c < NC; ++c) z[c] = (z[c] - (c == lab ? P(1) : P(0))) * sc;  // D
  if (part == 0 && valid) {
    P* D = static_cast<P*>(a.D);
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (c < C) D[(size_t)c * a.ldd + bcol] = z[c];
  }
  if (a.loss_partial) {
    const float v = wave_sum(lpart);
    if (lane == 0) lred[wave] = v;
    __syncthreads();
    if (t == 0 && vb * COLS < a.n) a.loss_partial[vb] = lred[0] + lred[1] + lred[2] + lred[3];
  }
  // ---- pass 2: dZ1 = (W2^T D) .* a1 .* (1 - a1)
  if (!valid) return;
  P* dZ1 = static_cast<P*>(a.dZ1);
  __hip_bfloat16* dZlo = static_cast<__hip_bfloat16*>(a.dZ1_bf16);
  __hip_bfloat16* dZp = static_cast<__hip_bfloat16*>(a.dZ1_planes);
  const size_t pstride = (size_t)a.H * a.ldz;
  auto emit = [&](int h, P x) {
    P da = P(0);
#pragma unroll
    for (int c = 0; c < NC; ++c) da += w2(c, h) * z[c];
    const P dz = da * x * (P(1) - x);
    const size_t zi = (size_t)h * a.ldz + bcol;
    dZ1[zi] = dz;
    if (dZlo) dZlo[zi] = __float2bfloat16((float)dz);
    if (dZp) {  // exact split into npz bf16 planes (mlp_split.h)
      float r = (float)dz;
      for (int p = 0; p < a.npz; ++p) {
        const __hip_bfloat16 q = __float2bfloat16(r);
        dZp[p * pstride + zi] = q;
        r -= __bfloat162float(q);
      }
    }
  };
  for (int h = part; h < H; h += NPART) emit(h, a1[(size_t)h * a.lda + bcol]);
}

template <typename P, int NC, bool LDSW>
__global__ __launch_bounds__(256) void head_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) char head_dyn[];
  __shared__ P zred[4][NC][kHeadCols];
  __shared__ float lred[4];
  head_block<P, NC, LDSW>(a, blockIdx.x, threadIdx.x, head_dyn, zred, lred);
}

// ------------------------------------------------ K2 on MFMA: 32 columns per 512-thread workgroup
// (fp32 params, train mode, H <= 128, C <= 16).  The VALU head above is latency-bound at these sizes
// (per thread 80 dependent LDS reads + FMAs per pass: 1.4 us per pass measured with s_memrealtime
// stamps), so both of its contractions run as v_mfma_f32_16x16x4_f32 tiles instead:
//   pass 1  z2 (16 x 32) = W2 (16 x H) . a1 (H x 32): wave w -> column half nt = w & 1, hidden quarter
//           kq = w >> 1 (32 rows, 8 MFMAs); partial tiles summed through LDS by waves 0/1, which then do
//           softmax / loss / D across the 4 lane groups (classes 4g+i live in lane group g).
//   pass 2  dA1 (H x 32) = W2^T . D: the K index of step i in lane group g is class 4g+i, which is
//           EXACTLY where pass 1 left D in the accumulator -> D goes to the other waves as one float4
//           per lane; each wave then owns (up to) two 16x16 tiles and applies a1 (1 - a1) in place.
// Lane map of v_mfma_f32_16x16x4f32 (mma_tile.h): lane l gives A[l&15][l>>4], B[l>>4][l&15] and
// receives C[4(l>>4) + i][l&15].  W2 is staged as [16][kW2S] in LDS (zero past C and past H).
// SC1: a1 was stored earlier in the same launch with write-through stores (fwd1_head_kernel).
constexpr int kW2S = 132;      // LDS row stride of the staged W2 (bank spread)
constexpr int kH32MaxH = 128;  // 8 row tiles = 2 per wave
constexpr int kH32Cols = 32;

struct Head32Lds {
  float w2[16 * kW2S];    // W2 [class][hidden], zero past C and past H
  float b2[16];
  float zp[3][2][64][4];  // pass-1 partial tiles of hidden quarters 1..3
  float ds[2][64][4];     // D in accumulator layout, per column half
};

// Stage W2 / b2 into LDS (512 threads, one burst of range-checked buffer loads).  Measured faster than
// loading the pass operands straight into registers, in the head kernel and before the fused GEMM.
__device__ __forceinline__ void head32_stage(const HeadArgs& a, int t, Head32Lds& L) {
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.W2), rb = make_rsrc(a.b2);
  float v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = t + u * 512, c = i >> 7, h = i & 127;
    v[u] = buf_load1<float>(rw, (c < a.C && h < a.H) ? (c * a.H + h) * 4 : kOOB);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = t + u * 512;
    L.w2[(i >> 7) * kW2S + (i & 127)] = v[u];
  }
  if (t < 16) L.b2[t] = buf_load1<float>(rb, t < a.C ? t * 4 : kOOB);
}

// ct: 32-column tile index; 512 threads; W2 / b2 staged in L (head32_stage) and a barrier since
template <bool SC1>
__device__ __forceinline__ void head32(const HeadArgs& a, int ct, int t, Head32Lds& L) {
  const int lane = t & 63, w = t >> 6, c16 = lane & 15, g = lane >> 4;
  const int nt = w & 1, kq = w >> 1;
  const int col = ct * kH32Cols + nt * 16 + c16;
  const bool cval = col < a.n;
  const int H = a.H, C = a.C, ld = a.lda;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(a.a1);
  auto ld_a1 = [&](int h) -> float {
    const int off = (h < H && cval) ? (h * ld + col) * 4 : kOOB;
    if constexpr (SC1) return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ra, off, 0, kSc1));
    else return buf_load1<float>(ra, off);
  };
  // one burst: pass-1 B operands and the pass-2 epilogue activations
  float bop[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) bop[s] = ld_a1(kq * 32 + 4 * s + g);
  float xe[2][4];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt)
#pragma unroll
    for (int j = 0; j < 4; ++j) xe[tt][j] = ld_a1((kq + 4 * tt) * 16 + 4 * g + j);
  const int lab = (int)__builtin_amdgcn_raw_buffer_load_b32(make_rsrc(a.labels), cval ? col * 4 : kOOB, 0, 0);
  auto hstamp = [&](int i) {  // diagnostics (HeadArgs::stamps): drained, wave 0 lane 0 (the diagnostics library only)
    if (CME_DIAG_STAMPS && a.stamps) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      const unsigned long long tt = __builtin_amdgcn_s_memrealtime();
      if (t == 0) a.stamps[(size_t)ct * 8 + i] = tt;
    }
  };
  hstamp(0);

  // ---- pass 1: this wave's hidden quarter of z2
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 8; ++s)
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(L.w2[c16 * kW2S + kq * 32 + 4 * s + g], bop[s], acc, 0, 0, 0);
  if (kq > 0) *reinterpret_cast<f32x4*>(L.zp[kq - 1][nt][lane]) = acc;
  __syncthreads();
  if (w < 2) {  // ---- softmax + cross-entropy gradient for the 16 columns of half nt
#pragma unroll
    for (int q = 0; q < 3; ++q) acc += *reinterpret_cast<const f32x4*>(L.zp[q][nt][lane]);
    float z[4];
    float m = 0.f;
    bool any = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cls = 4 * g + i;
      z[i] = acc[i] + L.b2[cls];
      if (a.shift && cls < C) {
        m = any ? fmaxf(m, z[i]) : z[i];
        any = true;
      }
    }
    if (a.shift) {  // class 0 is in lane group 0: every column has a valid entry there
      float mo = any ? m : -3.402823466e38f;
      mo = fmaxf(mo, __shfl_xor(mo, 16, 64));
      mo = fmaxf(mo, __shfl_xor(mo, 32, 64));
      m = mo;
    }
    float e[4], ssum = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      e[i] = (4 * g + i) < C ? __expf(z[i] - m) : 0.f;
      ssum += e[i];
    }
    ssum += __shfl_xor(ssum, 16, 64);
    ssum += __shfl_xor(ssum, 32, 64);
    const float inv = 1.f / ssum;
    const float sc = (float)a.scale;
    float lp = 0.f;
    f32x4 dv;
    float* Dg = static_cast<float*>(a.D);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cls = 4 * g + i;
      const float yh = e[i] * inv;
      const bool hit = cval && cls == lab;
      if (hit) lp = -__logf(yh);
      const float d = (cval && cls < C) ? (yh - (hit ? 1.f : 0.f)) * sc : 0.f;
      dv[i] = d;
      if (cval && cls < C) Dg[(size_t)cls * a.ldd + col] = d;
    }
    *reinterpret_cast<f32x4*>(L.ds[nt][lane]) = dv;
    if (a.loss_partial) {
      const float v = wave_sum(lp);
      const int vb = 2 * ct + nt;
      if (lane == 0 && vb * 16 < a.n) a.loss_partial[vb] = v;
    }
  }
  hstamp(1);
  __syncthreads();
  hstamp(2);
  // ---- pass 2: dZ1 = (W2^T D) .* a1 .* (1 - a1) on row tiles kq and kq + 4 of half nt
  const f32x4 dv = *reinterpret_cast<const f32x4*>(L.ds[nt][lane]);
  float* dZ1 = static_cast<float*>(a.dZ1);
  __hip_bfloat16* dZlo = static_cast<__hip_bfloat16*>(a.dZ1_bf16);
  __hip_bfloat16* dZp = static_cast<__hip_bfloat16*>(a.dZ1_planes);
  const size_t pstride = (size_t)H * a.ldz;
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int mt = kq + 4 * tt;
    if (mt * 16 >= H) break;  // wave-uniform
    f32x4 r = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i)
      r = __builtin_amdgcn_mfma_f32_16x16x4f32(L.w2[(4 * g + i) * kW2S + mt * 16 + c16], dv[i], r, 0, 0, 0);
    if (!cval) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int h = mt * 16 + 4 * g + j;
      if (h >= H) continue;
      const float x = xe[tt][j];
      const float dz = r[j] * x * (1.f - x);
      const size_t zi = (size_t)h * a.ldz + col;
      dZ1[zi] = dz;
      if (dZlo) dZlo[zi] = __float2bfloat16(dz);
      if (dZp) {
        float rr = dz;
        for (int p = 0; p < a.npz; ++p) {
          const __hip_bfloat16 q = __float2bfloat16(rr);
          dZp[p * pstride + zi] = q;
          rr -= __bfloat162float(q);
        }
      }
    }
  }
  hstamp(3);
}

__global__ __launch_bounds__(512) void head32_kernel(HeadArgs a) {
  __shared__ __attribute__((aligned(16))) Head32Lds L;
  head32_stage(a, threadIdx.x, L);
  __syncthreads();
  head32<false>(a, blockIdx.x, threadIdx.x, L);
}

bool head32_ok(const HeadArgs& a) {
  return a.mode == HEAD_TRAIN && a.H <= kH32MaxH && a.C <= 16;
}

// ------------------------------------- forward GEMM + head in ONE launch (split path, H <= 128)
// Workgroups compute 16x32 tiles of a1 = sigmoid(W1 X + b1) exactly as fwd1_split_kernel does, but
// store them write-through (sc1).  Per 32-column tile, the tm row-tile workgroups each add 1 to a
// counter after all their stores drained; the workgroup whose add completes the tile (old + 1 == tm)
// re-arms the counter to 0 and runs the head for those 32 columns (two 256-thread head blocks) with sc1
// loads of a1.  This is the "last arriver" hand-off of MI355X_MICROARCH.md (sc1 stores, vmcnt(0) in
// every storing wave, barrier, one agent-scope add per workgroup, sc1 loads; no fences), and it
// removes the head launch and its kernel boundary from the step (reference: gpuFeedforward +
// gpuBackprop's first half, fpcode/neural_network.cpp:281-378, were 8 launches with syncs).
// Placement for speed only: the tm workgroups of a column tile share blockIdx % 8 (one XCD under
// round-robin dispatch), so the hand-off normally stays inside one L2; correctness does not depend
// on it.
struct EpiSigWT {
  const float* b1;
  float* a1;
  int ld;
  float xscale;
  float pre[kEpiMaxQ];
  __device__ __forceinline__ void prefetch(int q, int row, int, bool ok) {
    pre[q] = buf_load1<float>(make_rsrc(b1), ok ? row * 4 : kOOB);
  }
  __device__ __forceinline__ void operator()(int q, int row, int col, float v) {
    const float s = sigmoid_<float>(v * xscale + pre[q]);
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, s), make_rsrc(a1), (row * ld + col) * 4, 0,
                                          kSc1);
  }
};

// 32-column a1 tiles (64-column tiles measured 15.4 vs 10.3 us at 784-100-10, n = 800: the last arriver then
// runs two head passes back to back)
template <int NPW, int VEC, bool AF>
__global__ __launch_bounds__(512) void fwd1_head_kernel(SplitStepArgs f, HeadArgs h, unsigned* __restrict__ counters,
                                                        int tm, int tn) {
  __shared__ __attribute__((aligned(16))) float red[8 * 1 * 2 * 4 * 64];
  __shared__ __attribute__((aligned(16))) Head32Lds L;
  __shared__ int s_last;
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int ct = xcd + 8 * (slot / tm), rt = slot % tm;
  if (ct >= tn) return;  // padding workgroup of the XCD-grouped grid (uniform: no barrier reached)
  unsigned long long* st = f.stamps ? f.stamps + (size_t)blockIdx.x * 4 : nullptr;  // diagnostics only
  auto stamp = [&](int i) {
    if (st && threadIdx.x == 0) st[i] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  // W2 / b2 for the head, staged by every workgroup before its GEMM (independent of a1; wsk_tile's
  // internal barrier orders these LDS writes before any head read)
  head32_stage(h, threadIdx.x, L);
  TileGeom g{f.H, f.n, f.P, rt * 16, ct * kH32Cols};
  EpiSigWT epi{f.b1, f.a1, f.ld, f.xscale, {}};
  fwd_tile<NPW, 2, VEC, 4, AF>(f, g, epi, red);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its sc1 stores are done
  __syncthreads();
  stamp(1);
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(counters + ct, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old + 1u == (unsigned)tm;
    // the last arriver re-arms the tile's counter for the next launch (every other workgroup of this tile
    // has already added; the next launch starts after this one ends) -- no wrap-around after 2^32 adds
    if (s_last) __hip_atomic_store(counters + ct, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  stamp(2);
  if (!s_last) return;
  head32<true>(h, ct, threadIdx.x, L);
  if (st) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(3);
  }
}

// ------------------------------------- forward GEMM + head in ONE launch, all-gather form (H <= 128)
// (body: fha_body.h)
template <int NPW, int VEC, bool AF, int SWZ = 0>
__global__ __launch_bounds__(512) void fwd1_head_ag_kernel(SplitStepArgs f, HeadArgs h,
                                                           unsigned long long* __restrict__ counters,
                                                           gran_t* __restrict__ slabs, int* __restrict__ err, int tm,
                                                           int tn) {
  __shared__ __attribute__((aligned(16))) float red[8 * 1 * 2 * 4 * 64];
  if (f.pf_wgs_xt && (int)blockIdx.x >= (int)gridDim.x - 8 * f.pf_wgs_xt) {  // a prefetch workgroup (pf_wgs_xt):
    // this step's XT into the L2 of an XCD whose dW1 tiles read it next (all P + 1 features x n columns)
    const int xcd = blockIdx.x & 7, part = ((int)blockIdx.x - ((int)gridDim.x - 8 * f.pf_wgs_xt)) >> 3;
    if (xcd < tm) l2_touch(f.XT, 0, f.P + f.bias_col, f.ldxt, f.n, part, f.pf_wgs_xt, reinterpret_cast<char*>(red));
    return;
  }
  fha_body<NPW, VEC, AF, SWZ>(f, h, counters, slabs, err, tm, tn, blockIdx.x, red);
}

template <typename P, int NC>
void launch_head(const HeadArgs& a, hipStream_t s) {
  const dim3 grid((a.n + kHeadCols - 1) / kHeadCols);
  const size_t lds = (size_t)head_lds_elems(a.H, NC) * sizeof(P);
  if (lds <= (size_t)kHeadLdsMax) head_kernel<P, NC, true><<<grid, 256, lds, s>>>(a);
  else head_kernel<P, NC, false><<<grid, 256, 0, s>>>(a);
}

// ------------------------------------------------ K2 for wide layers (H >= 512)
// scratch for the forward GEMM's z2 row-tile partials: [chunk][16][ld], 64-row chunks at most
constexpr int kHBCols = 64;
inline int hb_cdiv(int a, int b) { return (a + b - 1) / b; }
inline int hb_cols_pad(int n) { return hb_cdiv(n, kHBCols) * kHBCols; }

// ----------------------------------- K2 for wide layers when the forward GEMM left z2 partials
// (HeadArgs::z2_chunks > 0, see EpiSigBig::tile in mlp_split.hip).  One 512-thread workgroup per
// (128 RT hidden rows x 32 columns): it reduces the partials of its 32 columns (every row block
// recomputes the same softmax, a 16 x 32 x chunks sum), then each wave forms dZ1 for 16 RT rows x 32
// columns as 2 RT tiles of v_mfma_f32_16x16x4_f32 (dA1 = W2^T D, K = the 16 classes, class 4g+i in lane
// group g at step i) and applies a1 (1 - a1).  a1 is read once (the old two-kernel head read it twice).
constexpr int kHWCols = 32;

// RT row tiles of 16 per wave: 8 * 16 * RT hidden rows per workgroup (launcher picks RT for >= 256 workgroups)
template <int RT>
__global__ __launch_bounds__(512) void head_wide_kernel(HeadArgs a, int nrb) {
  __shared__ float zs[16][kHWCols + 1];
  __shared__ float Ds[16][kHWCols + 1];
  __shared__ float ls[kHWCols];
  __shared__ float ts[8][16][kHWCols + 1];  // per wave: one 16 x 32 dZ1 tile, re-read as 8-column rows
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, c16 = lane & 15, g = lane >> 4;
  const int rb = blockIdx.x % nrb, ct = blockIdx.x / nrb;
  const int H = a.H, C = a.C, ld = a.lda;
  const int row0 = (rb * 8 + w) * 16 * RT;
  auto hstamp = [&](int i) {  // diagnostics (HeadArgs::stamps, bench/stamps_hw.py): wave 0 lane 0 of the block
    if (CME_DIAG_STAMPS && a.stamps && t == 0) a.stamps[(size_t)blockIdx.x * 8 + i] = __builtin_amdgcn_s_memrealtime();
  };
  hstamp(0);
  // ---- one burst: the z2 partial sums of (class t>>5, column t&31), W2^T operands, a1 of the tiles
  const int zc = t >> 5, zcol = ct * kHWCols + (t & 31);
  // the label of softmax column t, fetched with the burst: loaded where it is used it was a dependent
  // memory round trip inside the single-wave softmax (bench/stamps_hw.py: softmax phase 2.3 us)
  const int lab_pre = (int)__builtin_amdgcn_raw_buffer_load_b32(
      make_rsrc(a.labels), (t < kHWCols && ct * kHWCols + t < a.n) ? (ct * kHWCols + t) * 4 : kOOB, 0, 0);
  const __amdgpu_buffer_rsrc_t rz = make_rsrc(a.z2part);
  float zsum = 0.f;
  {
    // every partial of this (class, column) in ONE burst of kZ2Burst loads (chunks past z2_chunks read the
    // range-checked zero) instead of z2_chunks / 8 dependent round trips: 32 chunks at H = 4096 (128-row
    // forward tiles), 16 at H = 1024.  Summed in chunk order as before (adding the zeros changes no bit).
    constexpr int kZ2Burst = 32;
    float v[kZ2Burst];
#pragma unroll
    for (int u = 0; u < kZ2Burst; ++u)
      v[u] = buf_load1<float>(rz, (zcol < a.n && u < a.z2_chunks && zc < C) ? ((u * 16 + zc) * ld + zcol) * 4 : kOOB);
#pragma unroll
    for (int u = 0; u < kZ2Burst; ++u) zsum += v[u];
    for (int k = kZ2Burst; k < a.z2_chunks; ++k)  // (classes past C: never stored, read as the range-checked 0)
      zsum += buf_load1<float>(rz, (zcol < a.n && zc < C) ? ((k * 16 + zc) * ld + zcol) * 4 : kOOB);
  }
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.W2), ra = make_rsrc(a.a1);
  // a1: each wave's 16 x 32 tiles as two 16-byte loads per lane (row lane >> 2, 8 columns from (lane & 3) * 8),
  // re-read from the wave's LDS tile in the MFMA layout below -- 4x fewer load instructions than 4-byte loads
  // in that layout (rows ld apart).  Columns past n (inside the ld padding) hold finite stale values or zeros:
  // they only meet D = 0 or masked stores.
  const int sr = lane >> 2, sc = (lane & 3) * 8;
  float wv[RT][4];
  f32x4 xr[RT][2];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int hA = row0 + rt * 16 + c16;
#pragma unroll
    for (int i = 0; i < 4; ++i) wv[rt][i] = buf_load1<float>(rw, (4 * g + i < C && hA < H) ? ((4 * g + i) * H + hA) * 4 : kOOB);
    const int h = row0 + rt * 16 + sr, col = ct * kHWCols + sc;
    const int off = (h < H && col < ld) ? (h * ld + col) * 4 : kOOB;
#pragma unroll
    for (int q = 0; q < 2; ++q)
      xr[rt][q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, off, 16 * q, 0));
  }
  zs[zc][t & 31] = zsum + (zc < C ? static_cast<const float*>(a.b2)[zc < C ? zc : 0] : 0.f);
  __syncthreads();
  hstamp(1);
  if (t < kHWCols) {  // ---- softmax / loss / D for column t
    const int col = ct * kHWCols + t;
    const bool ok = col < a.n;
    const int lab = ok ? lab_pre : -1;
    float m = 0.f;
    if (a.shift) {
      m = zs[0][t];
      for (int c = 1; c < C; ++c) m = fmaxf(m, zs[c][t]);
    }
    float e[16], sum = 0.f;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      e[c] = c < C ? __expf(zs[c][t] - m) : 0.f;
      sum += e[c];
    }
    const float inv = 1.f / sum, sc = (float)a.scale;
    float lp = 0.f;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      float d;
      const float y = head_prob_grad(e[c], inv, c == lab, sc, d);  // the fused wide head's arithmetic
      if (c == lab) lp = -__logf(y);
      if (!(ok && c < C)) d = 0.f;
      Ds[c][t] = d;
      if (rb == 0 && ok && c < C) static_cast<float*>(a.D)[(size_t)c * a.ldd + col] = d;
    }
    ls[t] = lp;
  }
  __syncthreads();
  hstamp(2);
  if (rb == 0 && a.loss_partial && t < 2) {  // the column head's layout: one partial per 16 columns
    const int vb = ct * 2 + t;
    if (vb * 16 < a.n) {
      float s = 0.f;
      for (int k = 0; k < 16; ++k) s += ls[t * 16 + k];
      a.loss_partial[vb] = s;
    }
  }
  if (row0 >= H) return;  // wave-uniform; no barrier follows
  float* dZ1 = static_cast<float*>(a.dZ1);
  __hip_bfloat16* dZlo = static_cast<__hip_bfloat16*>(a.dZ1_bf16);
  __hip_bfloat16* dZp = static_cast<__hip_bfloat16*>(a.dZ1_planes);
  const size_t pstride = (size_t)H * a.ldz;
  float dv[2][4];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int i = 0; i < 4; ++i) dv[cb][i] = Ds[4 * g + i][cb * 16 + c16];
  // The MFMA leaves each lane 4 ROWS of one column; stored straight from there every plane store is a
  // 2-byte scatter (32-byte row pieces).  The tile goes through this wave's LDS tile instead and comes
  // back as 8 consecutive columns per lane: one 16-byte store per plane (64-byte row pieces).
  const int scol = ct * kHWCols + sc;
  const bool vec = a.ldz % 8 == 0;  // 16-byte aligned rows (ld is padded to 16)
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    // this row tile's a1, row-major into the wave's LDS tile, then read back in the MFMA C layout
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int u = 0; u < 4; ++u) ts[w][sr][sc + 4 * q + u] = xr[rt][q][u];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float xv[2][4];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int j = 0; j < 4; ++j) xv[cb][j] = ts[w][4 * g + j][cb * 16 + c16];
    if (a.dw2part) {
      // this column tile's share of dW2: P[c][h] = sum over its 32 columns of D[c][col] a1[h][col], one
      // 16 x 16 x 32 v_mfma_f32_16x16x4_f32 chain per 16 rows (A = D from LDS, B = the row-major a1 tile);
      // the weight-gradient launch sums the column tiles' partials instead of re-reading all of a1
      // (mlp_split.hip wgrad_roles)
      f32x4 pw = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s8 = 0; s8 < 8; ++s8)
        pw = __builtin_amdgcn_mfma_f32_16x16x4f32(Ds[c16][4 * s8 + g], ts[w][c16][4 * s8 + g], pw, 0, 0, 0);
      const int hh = row0 + rt * 16 + c16;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * g + r < C && hh < H) a.dw2part[((size_t)ct * 16 + 4 * g + r) * H + hh] = pw[r];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // every read of the a1 tile is done
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      f32x4 r = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) r = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[rt][i], dv[cb][i], r, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x = xv[cb][j];
        ts[w][4 * g + j][cb * 16 + c16] = r[j] * x * (1.f - x);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int h = row0 + rt * 16 + sr;
    if (h < H) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ts[w][sr][sc + u];
      const size_t zi = (size_t)h * a.ldz + scol;
      if (vec && scol + 8 <= a.n) {
        if (dZ1) {  // nullptr: fp32 dZ1 not needed (planes only)
          *reinterpret_cast<f32x4*>(dZ1 + zi) = f32x4{v[0], v[1], v[2], v[3]};
          *reinterpret_cast<f32x4*>(dZ1 + zi + 4) = f32x4{v[4], v[5], v[6], v[7]};
        }
        if (dZlo) {
          __hip_bfloat16 q[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) q[u] = __float2bfloat16(v[u]);
          uint4 qw;
          __builtin_memcpy(&qw, q, 16);
          *reinterpret_cast<uint4*>(dZlo + zi) = qw;
        }
        if (dZp) {
          for (int p = 0; p < a.npz; ++p) {
            __hip_bfloat16 q[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              q[u] = __float2bfloat16(v[u]);
              v[u] -= __bfloat162float(q[u]);
            }
            uint4 qw;
            __builtin_memcpy(&qw, q, 16);
            *reinterpret_cast<uint4*>(dZp + p * pstride + zi) = qw;
          }
        }
      } else {  // ragged last columns / unpadded rows
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (scol + u >= a.n) break;
          const float dz = v[u];
          if (dZ1) dZ1[zi + u] = dz;
          if (dZlo) dZlo[zi + u] = __float2bfloat16(dz);
          if (dZp) {
            float rr = dz;
            for (int p = 0; p < a.npz; ++p) {
              const __hip_bfloat16 q = __float2bfloat16(rr);
              dZp[p * pstride + zi + u] = q;
              rr -= __bfloat162float(q);
            }
          }
        }
      }
    }
    // every lane's reads of this tile are done before the next row tile overwrites it
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (CME_DIAG_STAMPS && a.stamps) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    hstamp(3);
  }
}

// ----------------------------------------------------------------- K3: wgrad
template <typename P>
struct EpiWgrad {
  P* __restrict__ W;       // params [rows][ldw]
  P* __restrict__ G;       // gradient out (sgd == 0)
  __hip_bfloat16* __restrict__ Wlo;  // optional bf16 shadow of W
  int ldw;
  P reg, lr;
  int sgd;
  P pre[kEpiMaxQ];
  __device__ __forceinline__ void prefetch(int q, int row, int col, bool ok) {
    pre[q] = buf_load1<P>(make_rsrc(W), ok ? (row * ldw + col) * (int)sizeof(P) : kOOB);
  }
  template <typename A>
  __device__ __forceinline__ void operator()(int q, int row, int col, A v) {
    const size_t i = (size_t)row * ldw + col;
    const P w = pre[q];
    const P gr = P(v) + reg * w;
    if (sgd) {
      const P nw = w - lr * gr;
      W[i] = nw;
      if (Wlo) Wlo[i] = __float2bfloat16((float)nw);
    } else {
      G[i] = gr;
    }
  }
};

constexpr int kW1MB = 1, kW1NB = 2, kW2MB = 1, kW2NB = 2;

template <typename T, typename P>
__global__ __launch_bounds__(kThreads) void wgrad_kernel(WgradArgs a, int t1, int t1n, int t2, int t2n,
                                                    int vec1) {
  using acc1_t = typename MmaTraits<T>::acc_t;
  using acc2_t = typename MmaTraits<P>::acc_t;
  constexpr int R1 = kKS * kW1MB * kW1NB * 4 * 64 * sizeof(acc1_t);
  constexpr int R2 = kKS * kW2MB * kW2NB * 4 * 64 * sizeof(acc2_t);
  __shared__ __attribute__((aligned(16))) char smem[R1 > R2 ? R1 : R2];
  const int bid = blockIdx.x;
  const P reg = P(a.reg), lr = P(a.lr);

  if (bid < t1) {  // ---- dW1 = dZ1 * X^T  (K = batch)
    if (!(a.roles & 1)) return;
    const int tb = xcd_remap(bid, t1);
    TileGeom g{a.H, a.P, a.n, (tb / t1n) * 16 * kW1MB, (tb % t1n) * 16 * kW1NB};
    EpiWgrad<P> epi{static_cast<P*>(a.W1), static_cast<P*>(a.gW1),
                    static_cast<__hip_bfloat16*>(a.W1_bf16), a.P, reg, lr, a.sgd, {}};
    const T* A = static_cast<const T*>(a.dZ1g);
    constexpr int U = unroll_for<T>();
    if (a.XT) {  // B(k=b, n=p) = XT[p*ldxt + b]: K-contiguous, 16-byte loads
      const T* B = static_cast<const T*>(a.XT);
      if (vec1)
        wsk_tile<T, kW1MB, kW1NB, kKS, true, true, true, U>(A, a.ldz, B, a.ldxt, g, epi, (acc1_t*)smem);
      else
        wsk_tile<T, kW1MB, kW1NB, kKS, true, true, false, U>(A, a.ldz, B, a.ldxt, g, epi, (acc1_t*)smem);
    } else {     // B(k=b, n=p) = X[b*P + p]: n-contiguous, coalesced scalar loads
      const T* B = static_cast<const T*>(a.X);
      wsk_tile<T, kW1MB, kW1NB, kKS, true, false, false, U>(A, a.ldz, B, a.P, g, epi, (acc1_t*)smem);
    }
    return;
  }
  if (bid < t1 + t2) {  // ---- dW2 = D * a1^T
    if (!(a.roles & 2)) return;
    const int tb = bid - t1;
    TileGeom g{a.C, a.H, a.n, (tb / t2n) * 16 * kW2MB, (tb % t2n) * 16 * kW2NB};
    EpiWgrad<P> epi{static_cast<P*>(a.W2), static_cast<P*>(a.gW2), nullptr, a.H, reg, lr, a.sgd, {}};
    constexpr int U = unroll_for<P>();
    wsk_tile<P, kW2MB, kW2NB, kKS, true, true, false, U>(static_cast<const P*>(a.D), a.ldd,
                                                          static_cast<const P*>(a.a1), a.lda, g, epi,
                                                          (acc2_t*)smem);
    return;
  }
  // ---- bias gradients: one wave per row; rows [0,H) -> db1 from dZ1, [H,H+C) -> db2 from D.
  // Burst of 16 coalesced buffer loads per lane (OOB -> 0 past n), then a wave reduction.
  const int row = (bid - t1 - t2) * kKS + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= a.H + a.C || !(a.roles & 4)) return;
  const bool first = row < a.H;
  const P* src = first ? static_cast<const P*>(a.dZ1) + (size_t)row * a.ldz
                       : static_cast<const P*>(a.D) + (size_t)(row - a.H) * a.ldd;
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(src);
  P s = P(0);
  for (int j0 = 0; j0 < a.n; j0 += 64 * 16) {
    P v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int j = j0 + u * 64 + lane;
      v[u] = buf_load1<P>(rs, j < a.n ? j * (int)sizeof(P) : kOOB);
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) s += v[u];
  }
  s = wave_sum(s);
  if (lane == 0) {
    P* bp = static_cast<P*>(first ? a.b1 : a.b2);
    const int r = first ? row : row - a.H;
    if (a.sgd) bp[r] -= lr * s;
    else static_cast<P*>(first ? a.gb1 : a.gb2)[r] = s;
  }
}

// -------------------------------------------------------------- SGD (flat)
template <typename P>
__global__ __launch_bounds__(256) void sgd_flat_kernel(P* __restrict__ p, const P* __restrict__ g, int64_t n,
                                                       P lr, __hip_bfloat16* __restrict__ shadow,
                                                       int64_t shadow_n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const P v = p[i] - lr * g[i];
    p[i] = v;
    if (shadow && i < shadow_n) shadow[i] = __float2bfloat16((float)v);
  }
}

template <>
__global__ __launch_bounds__(256) void sgd_flat_kernel<float>(float* __restrict__ p, const float* __restrict__ g,
                                                              int64_t n, float lr,
                                                              __hip_bfloat16* __restrict__ shadow,
                                                              int64_t shadow_n) {
  // 16-byte vectorised body (flat arena segments are 64-element aligned)
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float4* p4 = reinterpret_cast<float4*>(p);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = p4[i];
    const float4 d = g4[i];
    v.x -= lr * d.x; v.y -= lr * d.y; v.z -= lr * d.z; v.w -= lr * d.w;
    p4[i] = v;
    if (shadow && 4 * i < shadow_n) {
      const int64_t b = 4 * i;
      shadow[b] = __float2bfloat16(v.x);
      if (b + 1 < shadow_n) shadow[b + 1] = __float2bfloat16(v.y);
      if (b + 2 < shadow_n) shadow[b + 2] = __float2bfloat16(v.z);
      if (b + 3 < shadow_n) shadow[b + 3] = __float2bfloat16(v.w);
    }
  }
  for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    p[i] -= lr * g[i];
    if (shadow && i < shadow_n) shadow[i] = __float2bfloat16(p[i]);
  }
}

__global__ void f32_to_bf16_kernel(const float* __restrict__ s, __hip_bfloat16* __restrict__ d, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    d[i] = __float2bfloat16(s[i]);
}

// ----------------------------------------------------------- generic GEMM
template <typename T>
struct EpiColMajor {  // C = alpha op(A) op(B) + beta C, column-major; S: the arithmetic type (fp32 for bf16)
  using S = std::conditional_t<std::is_same_v<T, __hip_bfloat16>, float, T>;
  T* __restrict__ C;
  int ldc;
  S alpha, beta;
  S pre[kEpiMaxQ];
  __device__ __forceinline__ void prefetch(int q, int row, int col, bool ok) {
    pre[q] = S(buf_load1<T>(make_rsrc(C), (ok && beta != S(0)) ? (row + col * ldc) * (int)sizeof(T) : kOOB));
  }
  template <typename A>
  __device__ __forceinline__ void operator()(int q, int row, int col, A v) {
    S r = alpha * S(v);
    if (beta != S(0)) r += beta * pre[q];
    C[(size_t)row + (size_t)col * ldc] = T(r);
  }
};

constexpr int kGMB = 2, kGNB = 2;

template <typename T, bool AK, bool BK, bool VEC>
__global__ __launch_bounds__(kThreads) void gemm_kernel(const T* __restrict__ A, int lda, const T* __restrict__ B,
                                                   int ldb, int M, int N, int K, EpiColMajor<T> epi,
                                                   int tiles_n) {
  using acc_t = typename MmaTraits<T>::acc_t;
  __shared__ acc_t red[kKS * kGMB * kGNB * 4 * 64];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  TileGeom g{M, N, K, (bid / tiles_n) * 16 * kGMB, (bid % tiles_n) * 16 * kGNB};
  constexpr int U = sizeof(T) == 4 ? 4 : 2;
  wsk_tile<T, kGMB, kGNB, kKS, AK, BK, VEC, U>(A, lda, B, ldb, g, epi, red);
}

inline int cdiv(int a, int b) { return (a + b - 1) / b; }
inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

template <typename T>
void launch_fwd1(const void* W1, const void* b1, const void* X, int P, int H, int n, void* a1, int lda, int act,
                 hipStream_t s) {
  using Par = std::conditional_t<std::is_same_v<T, __hip_bfloat16>, float, T>;
  const int tn = cdiv(n, 16 * kFwdNB), tm = cdiv(H, 16 * kFwdMB);
  constexpr int V = MmaTraits<T>::V;
  const bool vec = aligned16(W1) && aligned16(X) && (P % V == 0);
  if (vec)
    fwd1_kernel<T, Par, true><<<tm * tn, kThreads, 0, s>>>((const T*)W1, (const Par*)b1, (const T*)X, P, H, n,
                                                       (Par*)a1, lda, act, tn);
  else
    fwd1_kernel<T, Par, false><<<tm * tn, kThreads, 0, s>>>((const T*)W1, (const Par*)b1, (const T*)X, P, H, n,
                                                        (Par*)a1, lda, act, tn);
  CME_LAUNCH_CHECK(s);
}

template <typename T, typename Par>
void launch_wgrad(const WgradArgs& a, hipStream_t s) {
  const int t1n = cdiv(a.P, 16 * kW1NB), t1 = cdiv(a.H, 16 * kW1MB) * t1n;
  const int t2n = cdiv(a.H, 16 * kW2NB), t2 = cdiv(a.C, 16 * kW2MB) * t2n;
  const int tb = cdiv(a.H + a.C, kKS);
  constexpr int V = MmaTraits<T>::V;
  const int vec1 = aligned16(a.dZ1g) && (a.ldz % V == 0) && (a.n % V == 0) &&
                   (!a.XT || (aligned16(a.XT) && a.ldxt % V == 0));
  wgrad_kernel<T, Par><<<t1 + t2 + tb, kThreads, 0, s>>>(a, t1, t1n, t2, t2n, vec1);
  CME_LAUNCH_CHECK(s);
}

template <typename T>
void launch_gemm(bool tA, bool tB, int M, int N, int K, double alpha, const void* A, int lda, const void* B,
                 int ldb, double beta, void* C, int ldc, hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  using E = EpiColMajor<T>;
  E epi;
  epi.C = (T*)C;
  epi.ldc = ldc;
  epi.alpha = (typename E::S)alpha;
  epi.beta = (typename E::S)beta;
  const int tn = cdiv(N, 16 * kGNB), tm = cdiv(M, 16 * kGMB);
  const dim3 grid(tm * tn);
  constexpr int V = MmaTraits<T>::V;
  // column-major: A(m,k) = A[m + k*lda] (k strided) unless transposed.
  const bool AK = tA, BK = !tB;
  const bool vec = aligned16(A) && aligned16(B) && (!AK || lda % V == 0) && (!BK || ldb % V == 0) && (K % V == 0);
  const T* a = (const T*)A;
  const T* b = (const T*)B;
#define CME_GEMM_CASE(ak, bk)                                                                      \
  if (AK == ak && BK == bk) {                                                                      \
    if (vec) gemm_kernel<T, ak, bk, true><<<grid, kThreads, 0, s>>>(a, lda, b, ldb, M, N, K, epi, tn); \
    else gemm_kernel<T, ak, bk, false><<<grid, kThreads, 0, s>>>(a, lda, b, ldb, M, N, K, epi, tn);    \
  }
  CME_GEMM_CASE(true, true)
  CME_GEMM_CASE(true, false)
  CME_GEMM_CASE(false, true)
  CME_GEMM_CASE(false, false)
#undef CME_GEMM_CASE
  CME_LAUNCH_CHECK(s);
}

}  // namespace

// ================================================================ public API
void mlp_forward1(DType dt, const void* W1g, const void* b1, const void* X, int P, int H, int n, void* a1,
                  int lda, int act, hipStream_t s) {
  if (n <= 0) return;
  CME_REQUIRE(lda >= n, "mlp_forward1: lda < n");
  switch (dt) {
    case DType::F32: launch_fwd1<float>(W1g, b1, X, P, H, n, a1, lda, act, s); break;
    case DType::F64: launch_fwd1<double>(W1g, b1, X, P, H, n, a1, lda, act, s); break;
    case DType::BF16: launch_fwd1<__hip_bfloat16>(W1g, b1, X, P, H, n, a1, lda, act, s); break;
  }
}

int mlp_head_num_blocks(int n) { return cdiv(n, kHeadCols); }

bool mlp_fwd1_head_ok(const SplitStepArgs& f, const HeadArgs& h) {
  return head32_ok(h) && f.H == h.H && f.n == h.n && f.ld % 4 == 0 && h.lda == f.ld &&
         (int64_t)f.H * f.ld * 4 < (int64_t)kOOB && f.a1 == h.a1;
}

void mlp_fwd1_head(const SplitStepArgs& f, const HeadArgs& h, unsigned* counters, int max_tiles, hipStream_t s) {
  if (f.n <= 0) return;
  CME_REQUIRE(mlp_fwd1_head_ok(f, h), "fwd1_head: H <= 128, C <= 16, train-mode head over the same a1");
  CME_REQUIRE((int64_t)f.H * f.P * 2 * f.npw < (int64_t)kOOB && (int64_t)f.n * f.P < (int64_t)kOOB,
              "fwd1_head: operand too large for 32-bit buffer offsets");
  const int tm = cdiv(f.H, 16), tn = cdiv(f.n, kH32Cols);
  CME_REQUIRE(counters != nullptr && tn <= max_tiles, "fwd1_head: counter array too small");
  const bool af = mlp_split_fwd_fp32_w(f);
  const bool vec = reinterpret_cast<uintptr_t>(f.X) % 4 == 0 &&
                   reinterpret_cast<uintptr_t>(af ? (const void*)f.W1 : f.W1p) % 16 == 0 && f.P % 8 == 0;
  const int nwg = 8 * tm * cdiv(tn, 8);
#define CME_FH(np, af)                                                                     \
  if (vec) fwd1_head_kernel<np, 1, af><<<nwg, 512, 0, s>>>(f, h, counters, tm, tn);   \
  else fwd1_head_kernel<np, 0, af><<<nwg, 512, 0, s>>>(f, h, counters, tm, tn);
  if (af) { CME_FH(3, true) } else if (f.npw == 3) { CME_FH(3, false) } else { CME_FH(1, false) }
#undef CME_FH
  CME_LAUNCH_CHECK(s);
}

namespace {
template <auto Kern>
int resident_per_cu(int threads) {  // workgroups of Kern one CU holds at once (static LDS only), cached
  static int occ = -1;
  if (occ < 0) HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, Kern, threads, 0));
  return occ;
}
}  // namespace

// the wave-split-K forward's operand form: 3 = 16-byte pixel loads over chunk pairs (16-byte X rows), 1 = 4-byte
// pixel loads, 0 = element loads (mma_tile.h VEC)
static int fha_vec(const SplitStepArgs& f) {
  const bool af = mlp_split_fwd_fp32_w(f);
  const uintptr_t x = reinterpret_cast<uintptr_t>(f.X);
  if (x % 4 != 0 || reinterpret_cast<uintptr_t>(af ? (const void*)f.W1 : f.W1p) % 16 != 0 || f.P % 8 != 0) return 0;
  return x % 16 == 0 && f.P % 16 == 0 ? 3 : 1;
}

// the fragment-ordered operand copies (SplitStepArgs::w1_swz / x_swz) are laid out in 64-k pairs: the forward's
// waves must start their K ranges on pair boundaries, i.e. an even number of 32-k chunks per wave (8 waves):
// P = 784 / 800 / 1024 yes (4 chunks), P <= 256 or 513..768 no -- those take the row-major forms
bool mlp_fwd_swz_ok(const SplitStepArgs& f) {
  return f.H <= 128 && mlp_split_fwd_fp32_w(f) && fha_vec(f) == 3 && cdiv(cdiv(f.P, 32), 8) % 2 == 0;
}

bool mlp_fwd1_head_ag_fits(const SplitStepArgs& f) {
  if (f.n <= 0) return true;
  const int tm = cdiv(f.H, 16), tn = cdiv(f.n, 32), nwg = tm * tn;
  const bool af = mlp_split_fwd_fp32_w(f);
  const int vec = fha_vec(f);
#define CME_OCC(np, af)                                                            \
  (vec == 3   ? resident_per_cu<fwd1_head_ag_kernel<np, 3, af>>(512)               \
   : vec == 1 ? resident_per_cu<fwd1_head_ag_kernel<np, 1, af>>(512)               \
              : resident_per_cu<fwd1_head_ag_kernel<np, 0, af>>(512))
  const int occ = af ? CME_OCC(3, true) : (f.npw == 3 ? CME_OCC(3, false) : CME_OCC(1, false));
#undef CME_OCC
  return nwg <= occ * device_cu_count();
}

void mlp_fwd1_head_ag(const SplitStepArgs& f, const HeadArgs& h, unsigned long long* counters,
                      unsigned long long* slabs, int* err, int max_tiles, hipStream_t s) {
  if (f.n <= 0) return;
  CME_REQUIRE(mlp_fwd1_head_ok(f, h), "fwd1_head_ag: H <= 128, C <= 16, train-mode head over the same a1");
  CME_REQUIRE((int64_t)f.H * f.P * 2 * f.npw < (int64_t)kOOB && (int64_t)f.n * f.P < (int64_t)kOOB,
              "fwd1_head_ag: operand too large for 32-bit buffer offsets");
  const int tm = cdiv(f.H, 16), tn = cdiv(f.n, 32);
  CME_REQUIRE(tm <= 8, "fwd1_head_ag: H <= 128");
  CME_REQUIRE(counters && slabs && err && tn <= max_tiles, "fwd1_head_ag: counter / slab arrays too small");
  CME_REQUIRE(mlp_fwd1_head_ag_fits(f), "fwd1_head_ag: grid larger than the device holds at once (use the "
                                        "last-arriver form, mlp_fwd1_head)");
  const bool af = mlp_split_fwd_fp32_w(f);
  const int vec = fha_vec(f);
  const bool swz = f.w1_swz && f.W1s && mlp_fwd_swz_ok(f);
  CME_REQUIRE(!f.x_swz || (swz && f.Xs), "fwd1_head_ag: the fragment-ordered pixels need the W1 copy's form too");
  CME_REQUIRE(!h.dz_swz || (swz && h.dZ1 && !h.dZ1_planes && mlp_wgrad_dz_swz_ok(f)),
              "fwd1_head_ag: the fragment-ordered dZ1 needs the W1 copy's form, fp32 dZ1 and pair-aligned K ranges");
  // (prefetch workgroups last; xcd_rows == 2: cdiv(tm, 4) slots of tn per XCD, XCDs 4-7 padding)
  const int nwg = f.xcd_rows == 2 ? 8 * cdiv(tm, 4) * tn + 8 * f.pf_wgs_xt
                  : f.xcd_rows    ? 8 * tn + 8 * f.pf_wgs_xt
                                  : 8 * tm * cdiv(tn, 8);
#define CME_FHA(np, af)                                                                                  \
  if (swz && f.x_swz && h.dz_swz)                                                                       \
    fwd1_head_ag_kernel<3, 3, true, 7><<<nwg, 512, 0, s>>>(f, h, counters, slabs, err, tm, tn);           \
  else if (swz && h.dz_swz)                                                                             \
    fwd1_head_ag_kernel<3, 3, true, 5><<<nwg, 512, 0, s>>>(f, h, counters, slabs, err, tm, tn);           \
  else if (swz && f.x_swz)                                                                              \
    fwd1_head_ag_kernel<3, 3, true, 3><<<nwg, 512, 0, s>>>(f, h, counters, slabs, err, tm, tn);           \
  else if (swz)                                                                                         \
    fwd1_head_ag_kernel<3, 3, true, 1><<<nwg, 512, 0, s>>>(f, h, counters, slabs, err, tm, tn);           \
  else if (vec == 3) fwd1_head_ag_kernel<np, 3, af><<<nwg, 512, 0, s>>>(f, h, counters, slabs, err, tm, tn);  \
  else if (vec == 1) fwd1_head_ag_kernel<np, 1, af><<<nwg, 512, 0, s>>>(f, h, counters, slabs, err, tm, tn); \
  else fwd1_head_ag_kernel<np, 0, af><<<nwg, 512, 0, s>>>(f, h, counters, slabs, err, tm, tn);
  if (af) { CME_FHA(3, true) } else if (f.npw == 3) { CME_FHA(3, false) } else { CME_FHA(1, false) }
#undef CME_FHA
  CME_LAUNCH_CHECK(s);
}

// the forward GEMM's row-tile partials (64-row tiles at most, pitch = the activation ld <= hb_cols_pad(n) for
// ld = n rounded to 16)
int64_t head_big_scratch_floats(int H, int n) { return (int64_t)cdiv(H, 64) * kCMax * hb_cols_pad(n); }

void mlp_head(DType dt, const HeadArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  CME_REQUIRE(a.C >= 1 && a.C <= kCMax, "mlp_head: 1 <= C <= 16 required");
  if (a.z2part && a.z2_chunks > 0 && dt != DType::F64 && a.mode == HEAD_TRAIN && a.C <= 16) {
    // partials left by the forward GEMM
    CME_REQUIRE((int64_t)a.z2_chunks * 16 * a.lda < (int64_t)kOOB / 4 && (int64_t)a.H * a.lda < (int64_t)kOOB / 4,
                "mlp_head: z2 partials too large for 32-bit buffer offsets");
    const int nct = cdiv(a.n, kHWCols);
    // row tiles per wave: the largest RT that still gives >= 256 workgroups (RT 1/2/4 measured at H=1024
    // and 4096: this choice is the best or tied)
    const int rt = cdiv(a.H, 512) * nct >= 256 ? 4 : (cdiv(a.H, 256) * nct >= 256 ? 2 : 1);
    if (rt == 4) head_wide_kernel<4><<<cdiv(a.H, 512) * nct, 512, 0, s>>>(a, cdiv(a.H, 512));
    else if (rt == 2) head_wide_kernel<2><<<cdiv(a.H, 256) * nct, 512, 0, s>>>(a, cdiv(a.H, 256));
    else head_wide_kernel<1><<<cdiv(a.H, 128) * nct, 512, 0, s>>>(a, cdiv(a.H, 128));
    CME_LAUNCH_CHECK(s);
    return;
  }
  // (a wide head without the forward's partials -- only the head-alone profiling hook, MlpStep.run parts & 8 --
  // takes the column head below)
  if (dt != DType::F64 && head32_ok(a) && (int64_t)a.H * a.lda < (int64_t)kOOB / 4) {  // MFMA head
    head32_kernel<<<cdiv(a.n, kH32Cols), 512, 0, s>>>(a);
    CME_LAUNCH_CHECK(s);
    return;
  }
  if (dt == DType::F64) {
    if (a.C == 10) launch_head<double, 10>(a, s);
    else launch_head<double, 16>(a, s);
  } else {
    if (a.C == 10) launch_head<float, 10>(a, s);
    else launch_head<float, 16>(a, s);
  }
  CME_LAUNCH_CHECK(s);
}

void mlp_wgrad(DType dt, const WgradArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  switch (dt) {
    case DType::F32: launch_wgrad<float, float>(a, s); break;
    case DType::F64: launch_wgrad<double, double>(a, s); break;
    case DType::BF16: launch_wgrad<__hip_bfloat16, float>(a, s); break;
  }
}

void sgd_flat(DType dt, void* params, const void* grads, int64_t count, double lr, void* shadow,
              int64_t shadow_count, hipStream_t s) {
  if (count <= 0) return;
  const int grid = (int)std::min<int64_t>(2048, (count / 4 + 255) / 256 + 1);
  if (dt == DType::F64)
    sgd_flat_kernel<double><<<grid, 256, 0, s>>>((double*)params, (const double*)grads, count, lr,
                                                 (__hip_bfloat16*)shadow, shadow_count);
  else {
    CME_REQUIRE(aligned16(params) && aligned16(grads), "sgd_flat: f32 arena must be 16-byte aligned");
    sgd_flat_kernel<float><<<grid, 256, 0, s>>>((float*)params, (const float*)grads, count, (float)lr,
                                                (__hip_bfloat16*)shadow, shadow_count);
  }
  CME_LAUNCH_CHECK(s);
}

void gemm(DType dt, bool tA, bool tB, int M, int N, int K, double alpha, const void* A, int lda, const void* B,
          int ldb, double beta, void* C, int ldc, hipStream_t s) {
  switch (dt) {
    case DType::F32: launch_gemm<float>(tA, tB, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, s); break;
    case DType::F64: launch_gemm<double>(tA, tB, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, s); break;
    case DType::BF16:
      launch_gemm<__hip_bfloat16>(tA, tB, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, s);
      break;
  }
}

void convert_f32_to_bf16(const float* src, void* dst, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  const int grid = (int)std::min<int64_t>(2048, (n + 255) / 256);
  f32_to_bf16_kernel<<<grid, 256, 0, s>>>(src, (__hip_bfloat16*)dst, n);
  CME_LAUNCH_CHECK(s);
}

}  // namespace cme
