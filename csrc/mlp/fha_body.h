// Forward GEMM + head, all-gather form (H <= 128): the body of fwd1_head_ag_kernel (mlp_kernels.hip).
//
// The 16 x 32 a1 tiles of the forward GEMM; each of the tm row-tile workgroups of a 32-column tile
//   0. makes ONE agent-scope add to the tile's monotonic 64-bit counter at entry: every launch adds exactly tm
//      per tile (tm = cdiv(H, 16) is fixed for an engine), so old / tm + 1 is this launch's epoch, never 0;
//   1. forms its z2 partial W2[:, its 16 rows] . a1[its rows, cols] (16 classes x 32 columns) and publishes
//      it as data-tagged granules {value, epoch} (granule.h: one 8-byte sc1 store each, no drain, no flag);
//   2. polls the tm partials of its (class, column) until every tag is the epoch (bounded, s_sleep between
//      passes) and sums them in row-tile order (bit-identical z2 in every workgroup), softmax, D (row tile 0
//      stores it and the loss partial);
//   3. forms dZ1 for ITS OWN 16 rows from the a1 tile it still holds in LDS and stores it (fp32 and / or
//      the bf16 planes, two columns per 4-byte word).
// Requires every workgroup of the launch to be resident at once (mlp_fwd1_head_ag_fits); a poll that outlasts
// ag_wait_us of wall time sets *err: the launch's results are not trusted, and the weight-gradient launch that
// follows reads *err and applies nothing (SplitStepArgs::ag_err; MlpEngine.kernel_error(), KernelHandoffTimeout).
//
// PS (the XCD-local step pipeline, xstep.hip): the same body as one phase of a persistent multi-step launch -- the
// caller names the tile (rt, ct) and the step's granule tag, and the operands other workgroups of that launch rewrite
// between steps (b1, W2, b2; W1s in the K loop) are read with sc1 (L1-bypassing) loads; every row tile stores D
// (h.D: its own XCD's copy).  Returns false when a hand-off wait timed out (nothing after it was written).
#pragma once

#include "fwd_tile.h"
#include "granule.h"
#include "head_math.h"
#include "mlp_kernels.h"
#include "mlp_split.h"
#include "mma_tile.h"

namespace cme {

constexpr int kAgCounterStride = 32;  // uint64 words: one 256-byte line per tile counter (polls and adds of
                                      // different tiles must not share a line)

__device__ __forceinline__ float ag_sigmoid(float x) { return sigmoid_f32(x); }  // (head_math.h)

template <int CP = 0>  // CP: the b1 load's cache policy (kSc1 under PS)
struct EpiSigLdsT {
  const float* b1;
  float* a1;
  float (*a1s)[33];  // [16][32 + 1] this workgroup's a1 tile
  int ld, r0, c0;
  float xscale;
  float pre[kEpiMaxQ];
  __device__ __forceinline__ void prefetch(int q, int row, int, bool ok) {
    pre[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(make_rsrc(b1), ok ? row * 4 : kOOB, 0, CP));
  }
  __device__ __forceinline__ void operator()(int q, int row, int col, float v) {
    const float s = ag_sigmoid(v * xscale + pre[q]);
    a1s[row - r0][col - c0] = s;
    if (a1)  // (nullptr: nothing after the launch reads a1 -- the dW2 partials below replace it)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, s), make_rsrc(a1), (row * ld + col) * 4, 0, 0);
  }
};

// ---- the XCD-local step pipeline's flag line (xstep.hip XsBar): one 32-bit word per participant of an XCD in one
// 128-byte line of that XCD's L2, word 31 the launch's stop word.  ONE WAVE (every lane) waits until the words of
// participants [lo, hi) -- and `extra` when >= 0 -- carry `tag` (wrap-safe >=).  False when the launch stops: the
// stop word, or a wait past limit_us (then *err is set and the stop word written); *s_stop (LDS) is set either way.
__device__ __forceinline__ bool xcd_flags_wait(unsigned* line, unsigned tag, unsigned stop_tag, int lo, int hi,
                                               int extra, int* s_stop, int* err, uint32_t limit_us) {
  const int l = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t rl = make_rsrc(line);
  const uint64_t limit = (uint64_t)limit_us * kTicksPerUs;
  uint64_t t0 = 0;
  for (uint32_t pass = 1;; ++pass) {
    const unsigned v = __builtin_amdgcn_raw_buffer_load_b32(rl, l < 32 ? l * 4 : kOOB, 0, kSc1);
    if (__any(l == 31 && v == stop_tag)) {
      if (l == 0) *s_stop = 1;
      return false;
    }
    if (__all(!((l >= lo && l < hi) || l == extra) || v - tag < 0x80000000u)) return true;
    if (pass == 1) t0 = wall_ticks();
    else if ((pass & 7) == 0 && wall_ticks() - t0 > limit) {
      if (l == 0) {
        atomicExch(err, 1);
        line[31] = stop_tag;
        *s_stop = 1;
      }
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// PS with a gate (PSG): instead of a barrier between the previous step's weight update and this forward, each wave
// of the forward GEMM waits for the flags of the dW1 tiles that wrote the W1 columns of its K range (dW1 feature tile
// j = features [32 j, 32 j + 32)); the wave with no K range (wave 7) waits for every dW1 tile and the role workgroup
// -- this step's head then overwrites what they read (dZ1, D, the dW2 partials) -- and then stages b1 (this tile's
// rows), W2[:, rows] and b2 into LDS for the epilogue and the head (nobody else loads them).  line == nullptr: the
// plan's first step, nothing to wait for.
struct PsGate {
  unsigned* line = nullptr;
  unsigned tag = 0, stop_tag = 0;  // the previous step's second-barrier tag, this launch's stop value
  int ntiles = 0, role = 0;        // dW1 tiles of the XCD (slots [0, ntiles)), the role's slot
  int* s_stop = nullptr;
  int* err = nullptr;
  uint32_t limit_us = 0;
};

template <int CP, bool A1 = false>
struct EpiSigGate {  // (EpiSigLdsT's arithmetic; b1 from LDS, staged by wave 7; A1: the a1 store's test compiled in)
  float* a1;
  float (*a1s)[33];
  int ld, r0, c0;
  float xscale;
  const PsGate* gate;
  float* b1s;                      // [16]
  float (*w2s)[17];                // [16][17]
  float* b2s;                      // [16]
  const float *b1, *W2, *b2;
  int H, C;
  __device__ __forceinline__ void prefetch(int, int, int, bool) {}
  __device__ void before_kloop(int kbeg, int kend) {
    const PsGate& g = *gate;
    if (kend > kbeg) {
      if (g.line) xcd_flags_wait(g.line, g.tag, g.stop_tag, kbeg / 32, min(g.ntiles, (kend + 31) / 32), -1, g.s_stop,
                                 g.err, g.limit_us);
      return;
    }
    if (g.line) xcd_flags_wait(g.line, g.tag, g.stop_tag, 0, g.ntiles, g.role, g.s_stop, g.err, g.limit_us);
    const int l = threadIdx.x & 63;
    if (l < 16)
      b1s[l] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(make_rsrc(b1), r0 + l < H ? (r0 + l) * 4 : kOOB,
                                                                              0, CP));
    for (int e = l; e < 256; e += 64) {  // W2[class][tile row], zero past C / H
      const int c = e >> 4, r = e & 15;
      w2s[c][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                make_rsrc(W2), (c < C && r0 + r < H) ? (c * H + r0 + r) * 4 : kOOB, 0, CP));
    }
    if (l < 16)
      b2s[l] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(make_rsrc(b2), l < C ? l * 4 : kOOB, 0,
                                                                              CP));
  }
  __device__ __forceinline__ void operator()(int, int row, int col, float v) {
    const float s = ag_sigmoid(v * xscale + b1s[row - r0]);
    a1s[row - r0][col - c0] = s;
    if constexpr (A1) {
      if (a1) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, s), make_rsrc(a1), (row * ld + col) * 4, 0, 0);
    }
  }
};

// blk: the workgroup's slot in the XCD-grouped grid (the hardware XCD is blk & 7).  red: >= 8 * 2 * 4 * 64
// floats of LDS.
// DG (PS only): the diagnostics build -- the stamps and the hand-off test hook (SplitStepArgs::ag_test_skip); a
// production PS body compiles neither, nor the a1 store and the loss partials (the pipeline takes neither: mlp_xstep_ok)
// HK (PS only): the non-PS body's runtime tests kept in the build -- bit 0 the hand-off hook, bit 1 the loss
// partials, bit 2 the a1 store; each is a no-op in the pipeline (mlp_xstep_ok), but with all three the compiler's
// schedule of the body is 0.25 us faster per step (xstep.hip's launcher, profiles/r6/hk/)
template <int NPW, int VEC, bool AF, int SWZ = 0, bool PS = false, bool PSG = false, bool DG = !PS, int HK = 0>
__device__ __forceinline__ bool fha_body(const SplitStepArgs& f, const HeadArgs& h,
                                         unsigned long long* __restrict__ counters, gran_t* __restrict__ slabs,
                                         int* __restrict__ err, int tm, int tn, int blk, float* red, int ps_rt = 0,
                                         int ps_ct = 0, unsigned ps_ep = 0, const PsGate* ps_gate = nullptr) {
  static_assert(!PSG || PS, "the gate is a persistent-pipeline form");
  constexpr int CP = PS ? kSc1 : 0;
  constexpr int kCols = 32;
  __shared__ float a1s[16][kCols + 1];
  __shared__ float w2s[16][17];        // W2[class][row of this tile], zero past C / H
  __shared__ float b2s[16];
  __shared__ float zs[16][kCols + 1];  // z2 (+ b2), then D
  __shared__ float ls[kCols];
  __shared__ int s_bad;
  __shared__ unsigned s_ep;
  const int xcd = blk & 7, slot = blk >> 3;
  // column-tile grouping (the tm row tiles of a column tile on one XCD) or, xcd_rows, row tile rt on XCD rt -- or,
  // xcd_rows == 2 (the packed form for small batches), row tiles rt and rt + 4 on XCD rt < 4: the first four XCDs
  // start a launch up to ~1 us before the others (bench/stamps_fha.py per row tile), and every column tile's
  // all-gather waits for its last row tile
  int ct, rt;
  if constexpr (PS) {
    ct = ps_ct;
    rt = ps_rt;
  } else if (f.xcd_rows == 2) {
    const int j = slot / tn;
    ct = slot - j * tn;
    rt = xcd < 4 ? xcd + 4 * j : tm;  // (XCDs 4-7: padding)
  } else {
    ct = f.xcd_rows ? slot : xcd + 8 * (slot / tm);
    rt = f.xcd_rows ? xcd : slot % tm;
  }
  if (ct >= tn || rt >= tm) return true;  // padding workgroup of the XCD-grouped grid (uniform: no barrier reached)
  const int t = threadIdx.x, H = f.H, C = h.C, n = f.n;
  const int r0 = rt * 16, c0 = ct * kCols;
  constexpr bool kStamps = PS ? DG : (CME_DIAG_STAMPS != 0);  // (PS: the pipeline's DIAG build; else the diag library)
  unsigned long long* st = (kStamps && f.stamps) ? f.stamps + (size_t)blk * 4 : nullptr;  // diagnostics
  // (PS: the stamps are held in registers and stored at the end -- a store in the middle of the body puts its
  // completion in front of the next vmcnt wait -- with three more per workgroup after the first 256 x 4: the GEMM
  // returned, W2 staged, z2 partial formed)
  unsigned long long ts[8] = {};
  auto stamp = [&](int i) {
    if constexpr (PS) {
      if (st && t == 0) ts[i] = __builtin_amdgcn_s_memrealtime();
    } else {
      if (st && t == 0) st[i] = __builtin_amdgcn_s_memrealtime();
    }
  };
  auto stamp2 = [&](int i) {
    if constexpr (PS) {
      if (st && t == 0) ts[4 + i] = __builtin_amdgcn_s_memrealtime();
    }
  };
  auto stamps_out = [&]() {
    if constexpr (PS) {
      if (st && t == 0)
        for (int i = 0; i < 4; ++i) {
          st[i] = ts[i];
          st[1024 + i] = ts[4 + i];
        }
    }
  };
  stamp(0);
  // the launch epoch: one add per workgroup now, by wave 7, which has no K range at K = 784 or 800 -- so it also
  // WAITS for the add here, while the other waves run their K loop, and publishes the epoch to LDS before the
  // GEMM's reduction barrier.  (Waited for after the GEMM, the same vmcnt(0) also covered wave 7's a1 epilogue
  // stores: a store round trip in front of the z2 publication of every workgroup, bench/stamps_fha.py.)
  constexpr int kEpochThread = 448;
  if (t == kEpochThread) {
    if constexpr (PS) {
      s_ep = ps_ep;
    } else {
      gran_t ep_old = gran_epoch_add(counters + (size_t)ct * kAgCounterStride);
      gran_epoch_wait(ep_old);
      s_ep = (unsigned)(ep_old / (unsigned)tm) + 1u;
    }
    s_bad = 0;
  }
  // the label of this thread's softmax column (t >> 4), fetched now: loaded where the softmax uses it, it was
  // a dependent memory round trip after the all-gather wait
  const int lab_pre = (int)__builtin_amdgcn_raw_buffer_load_b32(
      make_rsrc(h.labels), c0 + (t >> 4) < n ? (c0 + (t >> 4)) * 4 : kOOB, 0, 0);
  // W2 slice of this tile's rows (read by the z2 partial and by dZ1) and b2: loaded now, written to LDS after
  // the GEMM (written here, each wave waited for its W2 load before its K-loop burst: a dependent memory round
  // trip in front of the GEMM, ~0.5 us of the launch per bench/stamps_fha.py)
  const int wc = t >> 4, wr = t & 15;
  TileGeom g{H, n, f.P, r0, c0};
  if constexpr (PSG) {  // (wave 7 stages b1, W2 and b2 into LDS inside the GEMM, after its wait: EpiSigGate)
    __shared__ float b1s[16];
    EpiSigGate<CP, (HK & 4) != 0> epi{f.a1, a1s, f.ld, r0, c0, f.xscale, ps_gate, b1s, w2s, b2s, f.b1, static_cast<const float*>(h.W2),
                       static_cast<const float*>(h.b2), H, C};
    fwd_tile<NPW, 2, VEC, 4, AF, SWZ, CP>(f, g, epi, red, kStamps ? h.stamps : nullptr);
    stamp2(0);
    if (*ps_gate->s_stop) {  // (a wait of this step's gate saw the launch stop: nothing is written)
      stamps_out();
      return false;
    }
  } else {
    const float w2v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
        make_rsrc(h.W2), (t < 256 && wc < C && r0 + wr < H) ? (wc * H + r0 + wr) * 4 : kOOB, 0, CP));
    const float b2v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
        make_rsrc(h.b2), (t >= 256 && t < 256 + 16 && t - 256 < C) ? (t - 256) * 4 : kOOB, 0, CP));
    EpiSigLdsT<CP> epi{f.b1, f.a1, a1s, f.ld, r0, c0, f.xscale, {}};
    fwd_tile<NPW, 2, VEC, 4, AF, SWZ, CP>(f, g, epi, red, kStamps ? h.stamps : nullptr);  // (per-wave GEMM timeline)
    stamp2(0);
    // wsk_tile ends with a barrier: a1s is complete.  Rows past H / columns past n: a1s holds stale LDS, so
    // they are masked below.  w2s / b2s are complete after the barrier below.
    if (t < 256) w2s[wc][wr] = w2v;
    else if (t < 256 + 16) b2s[t - 256] = b2v;
  }
  __syncthreads();
  stamp2(1);
  const unsigned ep = s_ep;
  // ---- 1. z2 partial W2[:, tile rows] . a1[tile rows, 32 columns] on MFMA (waves 0 and 1: 16 columns each,
  // 4 x v_mfma_f32_16x16x4_f32 over the 16 rows), published as tagged granules (lane: classes 4 g + i of
  // column 16 w + (lane & 15)).  Rows past H and columns past n read 0 (a1s holds stale LDS there).
  const int c = t >> 5, col = t & 31;
  if (t < 128) {
    const int w = t >> 6, l16 = t & 15, kg = (t & 63) >> 4, zc = 16 * w + l16;
    const bool colok = c0 + zc < n;
    f32x4 p = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int r = 4 * s + kg;
      p = __builtin_amdgcn_mfma_f32_16x16x4f32(w2s[l16][r], (colok && r0 + r < H) ? a1s[r][zc] : 0.f, p, 0, 0, 0);
    }
    if constexpr (PS) {
      if (st) {  // (diagnostics: the partial is formed)
        float sink = p[0];
        asm volatile("" ::"v"(sink));
        stamp2(2);
      }
    }
    // (test hook: one workgroup of column tile 0 never publishes, so that tile's polls time out)
    if (!((DG || (HK & 1)) && f.ag_test_skip == rt && ct == 0)) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (4 * kg + i < C) gran_store(slabs + (size_t)(ct * tm + rt) * 16 * kCols + (4 * kg + i) * kCols + zc, p[i], ep);
    }
  }
  stamp(1);
  // ---- 2. z2 = sum of the tm partials (row-tile order: the same bits in every workgroup) + b2
  {
    float z = 0.f;
    const bool good = gran_poll<8>(slabs, (unsigned)(ct * tm * 16 * kCols + c * kCols + col), 16u * kCols, tm,
                                   c < C, ep, (uint32_t)f.ag_wait_us, [&](int, float v) { z += v; });
    if (!good && (t & 63) == 0) {
      atomicExch(err, 1);
      s_bad = 1;
    }
    zs[c][col] = z + b2s[c];
  }
  __syncthreads();
  stamp(2);
  // softmax + cross-entropy gradient: 16 lanes (classes) per column, 4 columns per wave
  {
    const int col2 = t >> 4, cls = t & 15;
    const int gcol = c0 + col2;
    const bool cval = gcol < n;
    const float z = zs[cls][col2];
    float m = cls < C ? z : -3.402823466e38f;
    if (h.shift) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    } else {
      m = 0.f;
    }
    const float e = cls < C ? __expf(z - m) : 0.f;
    float ssum = e;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) ssum += __shfl_xor(ssum, o, 64);
    const int lab = cval ? lab_pre : -1;
    const float yh = e / ssum;
    const bool hit = cls == lab;
    const float d = (cval && cls < C) ? (yh - (hit ? 1.f : 0.f)) * (float)h.scale : 0.f;
    __syncthreads();  // every lane has read zs before it is overwritten with D
    zs[cls][col2] = d;
    if (PS || rt == 0)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, d), make_rsrc(h.D),
                                            (cval && cls < C) ? (cls * h.ldd + gcol) * 4 : kOOB, 0, 0);
    if ((!PS || (HK & 2)) && rt == 0 && h.loss_partial) {
      float lp = (cval && hit) ? -__logf(yh) : 0.f;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) lp += __shfl_xor(lp, o, 64);
      if (cls == 0) ls[col2] = lp;
    }
  }
  __syncthreads();
  if ((!PS || (HK & 2)) && rt == 0 && h.loss_partial && t < 2) {  // one partial per 16 columns (the column head's layout)
    const int vb = ct * 2 + t;
    if (vb * 16 < n) {
      float sl = 0.f;
      for (int k = 0; k < 16; ++k) sl += ls[t * 16 + k];
      h.loss_partial[vb] = sl;
    }
  }
  if (s_bad) {  // (zs holds D) a timed-out wait: nothing more is written
    stamps_out();
    return false;
  }
  // ---- 4a. (h.dw2part) this tile's dW2 partials D[:, 16 columns] . a1[tile rows, 16 columns]^T into
  // dw2part[16-column block][16 classes][H] (SplitStepArgs::dw2part, dw2_cols = 16): the weight-gradient launch's
  // dW2 role then sums cdiv(n, 16) partials per element (32 KB per 16-row tile at n = 800) instead of pulling D and
  // its a1 rows over the whole batch (~114 KB through one CU: the launch's critical path, bench/stamps_roles.py),
  // and nothing reads a1 after this launch.  Two waves, 4 x v_mfma_f32_16x16x4_f32 each from the LDS tiles (lane:
  // class l & 15 / row l & 15, k = column 4 s + (l >> 4)); zs holds D (0 past n and past C).  (One wave over all
  // 32 columns: forward + head +0.37 us; the 8 MFMAs' chain sat in front of that wave's dZ1 stores.)
  if (h.dw2part && t >= 384) {  // waves 6 and 7: columns [16 (w - 6), + 16) each, its own partial
    const int l = t & 63, l16 = l & 15, kg = l >> 4, half = (t >> 6) - 6;
    const bool rok = r0 + l16 < H;
    // (every LDS operand read first, unmasked -- the addresses are inside the tiles -- and masked by a select, so
    // the 8 reads issue back to back and the 4 MFMAs follow without a wait between them)
    float za[4], ab[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      za[s] = zs[l16][16 * half + 4 * s + kg];
      ab[s] = a1s[l16][16 * half + 4 * s + kg];
    }
    f32x4 p = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s)
      p = __builtin_amdgcn_mfma_f32_16x16x4f32(za[s], (rok && c0 + 16 * half + 4 * s + kg < n) ? ab[s] : 0.f, p, 0,
                                               0, 0);
    const __amdgpu_buffer_rsrc_t rp = make_rsrc(h.dw2part);
    const int pt = 2 * ct + half;  // partial index: 16 columns each
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cls = 4 * kg + i;
      const float v = p[i];  // (a copy: hipcc bit-casts an ext-vector element lvalue as element 0)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rp,
                                            (rok && cls < C) ? ((pt * 16 + cls) * H + r0 + l16) * 4 : kOOB, 0, 0);
    }
  }
  // ---- 4b. dZ1 = (W2^T D) .* a1 .* (1 - a1) for this tile's 16 rows, one element per thread
  {
    const int r = t >> 5;  // (col as above)
    const int row = r0 + r, gcol = c0 + col;
    const bool rok = row < H, ok = rok && gcol < n;
    float dz = 0.f;
    if (ok) {
      float da = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) da += w2s[k][r] * zs[k][col];
      const float x = a1s[r][col];
      dz = da * x * (1.f - x);
    }
    const size_t zi = (size_t)row * h.ldz + gcol;
    int zoff = (int)(zi * 4);
    if constexpr ((SWZ & 4) != 0) zoff = (int)(w1s_off(row, gcol, (h.ldz + 63) >> 6) * 4);  // (HeadArgs::dz_swz)
    if (h.dZ1)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, dz), make_rsrc(h.dZ1), ok ? zoff : kOOB, 0,
                                            0);
    // the planes two columns per 4-byte word: lanes col and col ^ 1 (same row) both split both values;
    // the even lane stores the even planes' words, the odd lane the odd ones (the pair's second column
    // lies inside the ld padding when it is past n; the dW1 GEMM never reads past n)
    const float dzn = __shfl_xor(dz, 1, 64);
    if (h.dZ1_planes) {
      const float ve = (col & 1) ? dzn : dz, vo = (col & 1) ? dz : dzn;
      const int ce = gcol & ~1;
      const bool pok = rok && ce < n;
      const __amdgpu_buffer_rsrc_t rp = make_rsrc(h.dZ1_planes);
      const size_t pstride = (size_t)H * h.ldz;
      float re = ve, ro = vo;
      for (int p = 0; p < h.npz; ++p) {
        const __hip_bfloat16 qe = __float2bfloat16(re), qo = __float2bfloat16(ro);
        re -= __bfloat162float(qe);
        ro -= __bfloat162float(qo);
        const unsigned w = (unsigned)__builtin_bit_cast(unsigned short, qe) |
                           ((unsigned)__builtin_bit_cast(unsigned short, qo) << 16);
        const int off = (int)((p * pstride + (size_t)row * h.ldz + ce) * 2);
        if ((p & 1) == (col & 1)) __builtin_amdgcn_raw_buffer_store_b32(w, rp, pok ? off : kOOB, 0, 0);
      }
    }
  }
  if (st) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    stamp(3);
    stamps_out();
  }
  return true;
}

}  // namespace cme
