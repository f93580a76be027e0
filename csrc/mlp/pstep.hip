// Persistent small-batch training engine (H <= 128, per-GPU batch n <= 256, split3 = fp32, one process):
// `count` SGD steps in ONE launch of tm = cdiv(H, 16) workgroups.
//
// Why (profiles/stamps_fha_xcd_rows_r4.jsonl, profiles/kbench_small_n_r4_start.jsonl): at n = 100 the two-launch
// step (forward + head, weight gradient) takes ~12 us although it moves ~1 MB and does ~50 MFLOP -- two kernel
// boundaries (~1.9 us each), a forward K loop that pulls ~75 KB of fp32 W1 + pixels into every workgroup's CU
// (~2 us, at the die-level cache's per-CU rate), the z2 all-gather hand-off (~1.6 us) and the head.  The
// reference's strong-scaling run (global batch 800 over N ranks, fpcode/run.sh:39, neural_network.cpp:458) lives
// exactly there: n = 100 per rank at N = 8.
//
// Design: workgroup r OWNS hidden rows [16 r, 16 r + 16): its W1 rows (+ b1), the matching W2 columns and a copy
// of b2 stay in LDS for the whole launch, so a step reads only the batch's pixels from memory and the only
// cross-CU traffic is the z2 all-gather (one data-tagged granule hand-off, granule.h).  Per step:
//   1. z1 = W1_r . X_b^T on v_mfma_f32_16x16x32_bf16: the fp32 W1 rows split into their three exact bf16 planes
//      in registers (mma_tile.h split_trunc), the uint8 pixels exact in one bf16; waves split K (KG groups) and
//      the columns (8 / KG groups); partial sums reduced through LDS;
//   2. a1 = sigmoid(z1 xscale + b1); this tile's z2 partial W2[:, rows] . a1 published as granules {value, tag}
//      (double-buffered by step parity);
//   3. every workgroup polls all tm partials of every (class, column), sums them in tile order (+ b2: the same bits
//      in every workgroup), softmax, D = (yhat - y) scale;
//   4. dZ1 = (W2_r^T D) .* a1 .* (1 - a1) into LDS; dW1 rows = dZ1 . XT_b (the feature-major pixel copy with its
//      all-ones feature: column 784 is db1) on the same MFMA, each wave owning whole 16-column blocks -- the SGD
//      update of W1 / b1 is applied to the LDS copy straight from the accumulators; dW2 = D . a1^T and db2 = D 1
//      on the fp32 MFMA (every workgroup computes db2 identically, so the b2 copies stay equal bit for bit).
// At the end every workgroup publishes its status, waits for all tm, and (no error anywhere) writes its rows back.
// A poll that outlasts SplitStepArgs::ag_wait_us sets *err: every workgroup then stops and NOTHING is written back
// (the parameters stay as they were before the launch; MlpEngine.kernel_error(), KernelHandoffTimeout).
// All tm <= 8 workgroups sit on one XCD (blockIdx = 8 r): they read the same batch, which one L2 then serves.
#include "mlp_split.h"

#include "granule.h"
#include "head_math.h"
#include "mma_tile.h"

namespace cme {

namespace {

using bf16 = __hip_bfloat16;

constexpr int kPT = 512;          // threads: 8 waves
constexpr int kPMaxN = 256;       // batch columns
constexpr int kPW1S = 804;        // LDS row stride of the W1 rows (>= 800: 25 whole K chunks; zero past P)
constexpr int kPCols = 785;       // dW1 columns: 784 features + the all-ones feature (db1)
constexpr int kPAS = kPMaxN + 1;  // LDS row stride of the [16][n] activation tiles

struct PLds {
  float w1[16][kPW1S];                       // W1 rows of this tile (fp32 master)
  float red[8 * 16 * 128];                   // z1 partial sums [wave][16][128 columns]; then D, dZ1 [16][kPAS]
  float a1[16][kPAS];
  float w2[16][16];                          // W2[class][row of this tile], zero past C / H
  float b1[16], b2[16];
  int bad;
};
static_assert(sizeof(PLds) <= 160 * 1024, "LDS budget");

__device__ __forceinline__ unsigned int widen2(unsigned int w, int hi) { return u8x2_to_bf16x2(w, hi); }

}  // namespace

// KN: 32-deep K chunks of the dW1 GEMM (n <= 32 KN).  The forward splits K = P (<= 784: 25 chunks of 32) over the
// 8 waves (chunk kg + 8 u of wave kg, u < 4) and walks the columns in halves of 8 blocks of 16.
template <int KN>
__global__ __launch_bounds__(kPT) void pstep_kernel(PStepArgs p) {
  extern __shared__ __attribute__((aligned(16))) char pst_lds[];
  if (blockIdx.x & 7) return;  // one workgroup per 8 blocks: all tm on one XCD (speed only)
  PLds& L = *reinterpret_cast<PLds*>(pst_lds);
  const SplitStepArgs& a = p.a;
  const int r = blockIdx.x >> 3, tm = (a.H + 15) / 16;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, fr = lane & 15, fg = lane >> 4;
  const int H = a.H, C = a.C, P = a.P, n = a.n, r0 = 16 * r;
  const int npad = (n + 15) & ~15, nb = npad / 16;  // column blocks of 16
  const float xs = a.xscale, sc = (float)a.scale, reg = (float)a.reg, lr = (float)a.lr;

  // ---- the launch's tag base: one add of `count` to this workgroup's own counter (every launch adds the same
  // amount to every counter, so every workgroup gets the same base; no host sequence number: graph-safe)
  __shared__ unsigned s_base;
  if (t == 0) {
    const unsigned long long old =
        __hip_atomic_fetch_add(p.counters + (size_t)r * 32, (unsigned long long)p.count, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    s_base = (unsigned)old;
    // the error word is sticky (as for the two-launch step): set by an earlier launch, this one applies nothing
    L.bad = __hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  }
  // ---- parameters of this tile into LDS
  for (int i = t; i < 16 * kPW1S; i += kPT) {
    const int rr = i / kPW1S, c = i - rr * kPW1S;
    L.w1[rr][c] = (r0 + rr < H && c < P) ? a.W1[(size_t)(r0 + rr) * P + c] : 0.f;
  }
  if (t < 256) {
    const int c = t >> 4, h = t & 15;
    L.w2[c][h] = (c < C && r0 + h < H) ? a.W2[(size_t)c * H + r0 + h] : 0.f;
  } else if (t < 256 + 16) {
    const int h = t - 256;
    L.b1[h] = r0 + h < H ? a.b1[r0 + h] : 0.f;
  } else if (t < 256 + 32) {
    const int c = t - 272;
    L.b2[c] = c < C ? a.b2[c] : 0.f;
  }
  __syncthreads();
  const unsigned base = s_base;
  const __amdgpu_buffer_rsrc_t rX = make_rsrc(a.X), rXT = make_rsrc(a.XT), rL = make_rsrc(a.labels);
  const int kch = (P + 31) / 32;  // forward K chunks (<= 25)
  int64_t gs = p.gstart0;
  bool ok = !L.bad;
  // diagnostics (SplitStepArgs::stamps, bench/stamps_pstep.py): workgroup 0, thread 0, steps < 16: s_memrealtime at
  // 0 step start, 1 a1 done, 2 z2 partials stored, 3 z2 gathered, 4 D done, 5 dZ1 done, 6 dW1 applied, 7 step end
  auto stamp = [&](int64_t s, int i) {
    if (a.stamps && r == 0 && t == 0 && s < 16) a.stamps[s * 8 + i] = __builtin_amdgcn_s_memrealtime();
  };

  for (int64_t s = 0; s < p.count && ok; ++s) {
    if (gs + p.B > p.N_end) gs = 0;
    const int64_t off = gs + p.shard_off;  // this step's first sample
    gs += p.B;
    const unsigned tag = base + (unsigned)s + 1u;
    stamp(s, 0);
    // (this step's label of column t, fetched now: loaded where the softmax uses it, it was a dependent round trip)
    const int lab_pre = (int)__builtin_amdgcn_raw_buffer_load_b32(rL, t < n ? (int)((off + t) * 4) : kOOB, 0, 0);
    // ================= 1. z1 = W1_r . X_b^T, then a1: per half of <= 8 column blocks, the wave's 4 K chunks as ONE
    // burst of pixel loads (issued before any MFMA), partial sums of the 8 waves reduced through LDS
    for (int hb = 0; hb < nb; hb += 8) {
      unsigned int bw[4][8][2];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = (wave + 8 * u) * 32 + 8 * fg;
#pragma unroll
        for (int j = 0; j < 8; ++j) {  // pixels of sample (block hb + j, lane column fr), k .. k + 7
          const int col = (hb + j) * 16 + fr;
          const bool rok = hb + j < nb && col < n && k + 8 <= P;
          const int o = rok ? (int)((off + col) * P + k) : kOOB;
          bw[u][j][0] = __builtin_amdgcn_raw_buffer_load_b32(rX, o, 0, 0);
          bw[u][j][1] = __builtin_amdgcn_raw_buffer_load_b32(rX, rok ? o + 4 : kOOB, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // (the burst stays ahead of the first MFMA)
      f32x4 acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int kc = wave + 8 * u;
        if (kc >= kch) break;  // (wave-uniform)
        const int k = kc * 32 + 8 * fg;
        float av[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) av[j] = L.w1[fr][k + j];  // (zero past P)
        bf16 pl[3][8];
        split_trunc<3, 8>(av, pl);
        bf16x8_t A[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) __builtin_memcpy(&A[q], pl[q], 16);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (hb + j >= nb) break;  // (wave-uniform: no MFMA on column blocks past n)
          unsigned int w[4] = {widen2(bw[u][j][0], 0), widen2(bw[u][j][0], 1), widen2(bw[u][j][1], 0),
                               widen2(bw[u][j][1], 1)};
          bf16x8_t B;
          __builtin_memcpy(&B, w, 16);
#pragma unroll
          for (int q = 0; q < 3; ++q) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[q], B, acc[j], 0, 0, 0);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) L.red[(wave * 16 + 4 * fg + i) * 128 + j * 16 + fr] = acc[j][i];
      __syncthreads();
      for (int i = t; i < 16 * 128; i += kPT) {  // a1 = sigmoid(z1 xscale + b1), the waves' partials in wave order
        const int h = i >> 7, cl = i & 127, col = hb * 16 + cl;
        if (col >= npad) continue;
        float z = 0.f;
#pragma unroll
        for (int g = 0; g < 8; ++g) z += L.red[(g * 16 + h) * 128 + cl];
        L.a1[h][col] = (r0 + h < H && col < n) ? sigmoid_f32(z * xs + L.b1[h]) : 0.f;
      }
      __syncthreads();
    }
    stamp(s, 1);
    // ---- the dW1 GEMM's B operand (XT words of this wave's feature blocks w, w + 8, ...), issued NOW: its latency
    // hides behind the z2 hand-off, the softmax and dZ1 instead of one round trip per feature block later.  All of
    // them up to n = 128 (56 VGPRs); above, the first kPD, the rest kPD blocks ahead inside the loop.
    constexpr int kFB = (kPCols + 15) / 16;  // 50 feature blocks
    constexpr int kFBW = (kFB + 7) / 8;      // per wave
    constexpr int kPD = KN <= 4 ? kFBW : 2;
    auto load_xt = [&](int fb, unsigned int (&w)[KN][2]) {
      const int feat = fb * 16 + fr;
#pragma unroll
      for (int kc = 0; kc < KN; ++kc) {
        const int k = kc * 32 + 8 * fg;
        const bool rok = fb < kFB && feat < kPCols;
        const int o = (int)((int64_t)feat * a.ldxt + off + k);
        w[kc][0] = __builtin_amdgcn_raw_buffer_load_b32(rXT, rok && k < n ? o : kOOB, 0, 0);
        w[kc][1] = __builtin_amdgcn_raw_buffer_load_b32(rXT, rok && k + 4 < n ? o + 4 : kOOB, 0, 0);
      }
    };
    unsigned int xw[kFBW][KN][2];
#pragma unroll
    for (int v = 0; v < kPD; ++v) load_xt(wave + 8 * v, xw[v]);
    // ================= 2. this tile's z2 partial W2[:, rows] . a1 -> granules (double-buffered by step parity)
    gran_t* z2g = p.gran + (size_t)(s & 1) * 8 * 16 * kPMaxN;  // [parity][tile][class][column]
    // (test hook, SplitStepArgs::ag_test_skip: this workgroup withholds its partials, every poll really times out)
    for (int i = t; i < (a.ag_test_skip == r ? 0 : C * n); i += kPT) {
      const int c = i / n, col = i - c * n;
      float z = 0.f;
#pragma unroll
      for (int h = 0; h < 16; ++h) z += L.w2[c][h] * L.a1[h][col];
      gran_store(z2g + ((size_t)r * 16 + c) * kPMaxN + col, z, tag);
    }
    stamp(s, 2);
    // ================= 3. z2 = sum of the tm partials (tile order) + b2; softmax; D (into red, [16][kPAS])
    float* Ds = L.red;
    float* dzs = L.red + 16 * kPAS;
    // every (class, column) item's tm partials; a lane takes kIG items (granule j * 8 + tile) per poll pass, so
    // ONE round trip per pass gathers them all (item i = i0 + j kPT + t: a wave's lanes read consecutive columns)
    constexpr int kIG = 2;
    for (int i0 = 0; i0 < C * n; i0 += kIG * kPT) {  // (uniform trip count)
      unsigned offs[kIG * 8], need = 0u;
#pragma unroll
      for (int j = 0; j < kIG; ++j) {
        const int i = i0 + j * kPT + t, c = i / n, col = i - c * n;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          offs[j * 8 + k] = (unsigned)((k * 16 + c) * kPMaxN + col);
          if (i < C * n && k < tm) need |= 1u << (j * 8 + k);
        }
      }
      float z[kIG] = {};
      const bool good = gran_poll_set<kIG * 8>(z2g, offs, need, tag, (uint32_t)a.ag_wait_us,
                                               [&](int k, float v) { z[k >> 3] += v; });  // (tile order)
      if (!good) {
        atomicExch(p.err, 1);
        L.bad = 1;
      }
#pragma unroll
      for (int j = 0; j < kIG; ++j) {
        const int i = i0 + j * kPT + t, c = i / n, col = i - c * n;
        if (i < C * n) Ds[c * kPAS + col] = z[j] + L.b2[c];  // (z2 for now)
      }
    }
    __syncthreads();
    stamp(s, 3);
    if (L.bad) {
      ok = false;
      break;
    }
    for (int col = t; col < npad; col += kPT) {  // one column per thread: softmax + cross-entropy gradient
      if (col >= n) {  // (D is zero past n: the dW2 / db2 chains read whole 4-column steps)
#pragma unroll
        for (int c = 0; c < 16; ++c) Ds[c * kPAS + col] = 0.f;
        continue;
      }
      const int lab = lab_pre;  // (col == t: n <= 256 < kPT)
      float m = 0.f;
      if (a.shift) {
        m = Ds[col];
        for (int c = 1; c < C; ++c) m = fmaxf(m, Ds[c * kPAS + col]);
      }
      float e[16], ssum = 0.f;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        e[c] = c < C ? __expf(Ds[c * kPAS + col] - m) : 0.f;
        ssum += e[c];
      }
      const float inv = 1.f / ssum;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        float d = 0.f;
        if (c < C) head_prob_grad(e[c], inv, c == lab, sc, d);
        Ds[c * kPAS + col] = d;  // (classes past C: 0)
      }
    }
    __syncthreads();
    stamp(s, 4);
    // ================= 4. dZ1 (LDS); dW2 / db2 (fp32 loops); dW1 (MFMA) + the SGD update of the LDS copies
    for (int i = t; i < 16 * 32 * KN; i += kPT) {
      const int h = i / (32 * KN), col = i - h * (32 * KN);
      float dz = 0.f;
      if (col < n && r0 + h < H) {
        float da = 0.f;
#pragma unroll
        for (int c = 0; c < 16; ++c) da += L.w2[c][h] * Ds[c * kPAS + col];
        const float x = L.a1[h][col];
        dz = da * x * (1.f - x);
      }
      dzs[h * kPAS + col] = dz;  // (zero past n: the dW1 K loop reads whole 32-deep chunks)
    }
    __syncthreads();
    stamp(s, 5);
    // dW2 = D . a1^T and db2 = D 1 on v_mfma_f32_16x16x4_f32, waves 6 and 7 (they own 6 feature blocks, waves 0 and 1
    // own 7) taking one half of the batch columns each: A(c, k) = D[c][k], B(k, h) = a1[h][k] (or 1 for db2); the two
    // halves' 16 x 16 partials meet in LDS and are summed (half 0 + half 1) by the W2 / b2 update below
    float* w2s = L.red + 32 * kPAS;  // [2][16][16] dW2 partials, then [2][16] db2 partials
    if (wave >= 6) {
      const int half = wave - 6, kh = npad / 2, k0 = half * kh;  // (npad % 16 == 0: kh % 4 == 0)
      f32x4 gw = {0.f, 0.f, 0.f, 0.f}, gb = {0.f, 0.f, 0.f, 0.f};
      for (int k = k0 + fg; k < k0 + kh; k += 4) {
        const float dv = Ds[fr * kPAS + k];
        gw = __builtin_amdgcn_mfma_f32_16x16x4f32(dv, L.a1[fr][k], gw, 0, 0, 0);
        gb = __builtin_amdgcn_mfma_f32_16x16x4f32(dv, 1.f, gb, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        w2s[(half * 16 + 4 * fg + i) * 16 + fr] = gw[i];  // dW2[class 4 fg + i][row fr]
        if (fr == 0) w2s[512 + half * 16 + 4 * fg + i] = gb[i];
      }
    }
    // dW1 = dZ1 . XT_b: the dZ1 chunks split into their exact planes ONCE (registers), then wave w walks the
    // 16-feature blocks w, w + 8, ... (feature 784 is the all-ones db1 column) over the prefetched XT words
    bf16x8_t Az[KN][3];
#pragma unroll
    for (int kc = 0; kc < KN; ++kc) {
      float av[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) av[j] = dzs[fr * kPAS + kc * 32 + 8 * fg + j];
      bf16 pl[3][8];
      split_trunc<3, 8>(av, pl);
#pragma unroll
      for (int q = 0; q < 3; ++q) __builtin_memcpy(&Az[kc][q], pl[q], 16);
    }
#pragma unroll
    for (int v = 0; v < kFBW; ++v) {
      const int fb = wave + 8 * v;
      if (v + kPD < kFBW) load_xt(fb + 8 * kPD, xw[v + kPD]);
      f32x4 g = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KN; ++kc) {
        unsigned int w[4] = {widen2(xw[v][kc][0], 0), widen2(xw[v][kc][0], 1), widen2(xw[v][kc][1], 0),
                             widen2(xw[v][kc][1], 1)};
        bf16x8_t B;
        __builtin_memcpy(&B, w, 16);
#pragma unroll
        for (int q = 0; q < 3; ++q) g = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Az[kc][q], B, g, 0, 0, 0);
      }
      // the update, straight from the accumulators: element (row 4 fg + i, feature feat)
      const int feat = fb * 16 + fr;
      if (fb < kFB && feat < kPCols) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int h = 4 * fg + i;
          if (r0 + h >= H) continue;
          if (feat == P) {  // all-ones feature: db1 (no input scale, no regulariser)
            L.b1[h] -= lr * g[i];
          } else if (feat < P) {
            const float w = L.w1[h][feat];
            L.w1[h][feat] = w - lr * (g[i] * xs + reg * w);
          }
        }
      }
    }
    __syncthreads();  // every read of w2 / Ds / a1 / the old W1 done
    stamp(s, 6);
    if (t < 256) {
      const int c = t >> 4, h = t & 15;
      if (c < C && r0 + h < H) {
        const float w = L.w2[c][h], gw2 = w2s[c * 16 + h] + w2s[256 + c * 16 + h];
        L.w2[c][h] = w - lr * (gw2 + reg * w);
      }
    } else if (t < 256 + 16) {
      const int c = t - 256;
      if (c < C) L.b2[c] -= lr * (w2s[512 + c] + w2s[512 + 16 + c]);
    }
    __syncthreads();
    stamp(s, 7);
  }
  // ---- every workgroup's status (tag base + count + 1), then all agree: write back only if none failed
  const unsigned stag = base + (unsigned)p.count + 1u;
  if (t == 0) gran_store(p.status + r, ok ? 0.f : 1.f, stag);
  __shared__ int s_err;
  if (t < 64) {
    float e = 0.f;
    const bool good = gran_poll<8>(p.status, 0u, 1u, tm, t == 0, stag, (uint32_t)a.ag_wait_us,
                                   [&](int, float v) { e += v; });
    if (t == 0) {
      s_err = (!good || e != 0.f) ? 1 : 0;
      if (s_err) atomicExch(p.err, 1);
    }
  }
  __syncthreads();
  if (s_err) return;  // (the parameters keep their values from before the launch)
  for (int i = t; i < 16 * P; i += kPT) {
    const int rr = i / P, c = i - rr * P;
    if (r0 + rr < H) a.W1[(size_t)(r0 + rr) * P + c] = L.w1[rr][c];
  }
  if (t < 256) {
    const int c = t >> 4, h = t & 15;
    if (c < C && r0 + h < H) a.W2[(size_t)c * H + r0 + h] = L.w2[c][h];
  } else if (t < 256 + 16) {
    const int h = t - 256;
    if (r0 + h < H) a.b1[r0 + h] = L.b1[h];
  } else if (t < 256 + 32 && r == 0) {
    const int c = t - 272;
    if (c < C) a.b2[c] = L.b2[c];
  }
}

bool mlp_pstep_ok(const SplitStepArgs& a) {
  // (split3 only: the bf16 path's single rounded W1 / dZ1 planes stay on the two-launch step)
  return a.npw == 3 && a.npz == 3 && a.H >= 1 && a.H <= 128 && a.C >= 1 && a.C <= 16 && a.n >= 1 &&
         a.n <= kPMaxN && a.P <= 784 &&
         a.n % 4 == 0 && a.P % 8 == 0 && a.bias_col && a.XT && a.X && a.W1 && a.xf.world == 0 && a.sgd == 1 &&
         (int64_t)(a.P + 1) * a.ldxt < (int64_t)kOOB;
}

template <int KN>
void launch_pstep(const PStepArgs& p, int tm, hipStream_t s) {
  constexpr int L = (int)sizeof(PLds);
  static bool done = false;  // one attribute call per instantiation
  if (!done) {
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(pstep_kernel<KN>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, L));
    done = true;
  }
  pstep_kernel<KN><<<8 * tm, kPT, L, s>>>(p);
}

void mlp_pstep(const PStepArgs& p, hipStream_t s) {
  const SplitStepArgs& a = p.a;
  CME_REQUIRE(mlp_pstep_ok(a), "pstep: H <= 128, C <= 16, n <= 256 and n % 4 == 0, P <= 784, the all-ones XT feature, sgd = 1");
  CME_REQUIRE(p.counters && p.gran && p.status && p.err && p.count >= 1 && p.B >= a.n && p.N_end >= p.B,
              "pstep: buffers / plan");
  CME_REQUIRE((int64_t)p.N_end * a.P < (int64_t)kOOB, "pstep: dataset too large for 32-bit buffer offsets");
  const int tm = (a.H + 15) / 16;
  if (a.n <= 64) launch_pstep<2>(p, tm, s);
  else if (a.n <= 128) launch_pstep<4>(p, tm, s);
  else launch_pstep<8>(p, tm, s);
  CME_LAUNCH_CHECK(s);
}

}  // namespace cme
