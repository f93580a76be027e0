// Split-bf16 MLP step kernels (see mlp_split.h for the numerics argument).
#include "mlp_split.h"
#include "mlp_kernels.h"

#include <algorithm>

#include "glds_gemm.h"
#include "granule.h"
#include "head_math.h"
#include "l2_touch.h"
#include "rega_gemm.h"
#include "g64_gemm.h"
#include "mma_tile.h"
#include "fwd_tile.h"
#include "wgrad_epi.h"

namespace cme {

namespace {

using bf16 = __hip_bfloat16;
using namespace wg;  // (wgrad_epi.h: split_store, kXfSys, ag_err_load, poisoned, xf_store, row_sum, EpiW1, EpiW2)

__device__ __forceinline__ float sigm(float x) { return sigmoid_f32(x); }  // (head_math.h)


// Kernel A1 (tiled): a1 = sigmoid(W1 X + b1) on 16x32 tiles, K split over 8 waves, W1 as fp32 split in
// registers or NPW exact bf16 planes; with the separate head kernel where the fused forward + head launch does
// not apply (H > 128, predict).
constexpr int kF1MB = 1, kF1NB = 2, kF1KS = 8;

struct EpiSig {
  const float* b1;
  float* a1;
  int ld;
  float xscale;
  float pre[kEpiMaxQ];
  __device__ __forceinline__ void prefetch(int q, int row, int, bool ok) {
    pre[q] = buf_load1<float>(make_rsrc(b1), ok ? row * 4 : kOOB);
  }
  __device__ __forceinline__ void operator()(int q, int row, int col, float v) {
    a1[(size_t)row * ld + col] = sigm(v * xscale + pre[q]);
  }
};

template <int NPW, int VEC, bool AF>
__global__ __launch_bounds__(64 * kF1KS) void fwd1_split_kernel(SplitStepArgs a, int tiles_n) {
  static_assert(kF1MB == 1 && kF1KS == 8, "fwd_tile: one 16-row block, 8 K-waves");
  __shared__ __attribute__((aligned(16))) float red[kF1KS * kF1MB * kF1NB * 4 * 64];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  TileGeom g{a.H, a.n, a.P, (bid / tiles_n) * 16 * kF1MB, (bid % tiles_n) * 16 * kF1NB};
  EpiSig epi{a.b1, a.a1, a.ld, a.xscale, {}};
  fwd_tile<NPW, kF1NB, VEC, 4, AF>(a, g, epi, red, CME_DIAG_STAMPS ? a.stamps : nullptr);
}


// ---- gradient all-reduce fused into the wgrad launch (XgmiFuse, see mlp_split.h) ------------------
// Protocol per gradient tile (same as csrc/comm/xgmi_allreduce.hip per chunk): epoch e = epochs[tile]+1;
// the tile's gradients go WRITE-THROUGH (sc0 sc1) into half e&1 of my IPC buffer; drain, barrier,
// system-scope release flag store into every peer's slot [tile][rank]; bounded wait for every peer's
// flag; rank-order sum with system-coherent loads (bit-identical on every rank).  Double
// buffering + per-tile epochs: half e&1 of a tile is rewritten only after every peer passed e-1.
constexpr uint64_t kXfWaitTicks = kPeerWaitUs * kTicksPerUs;  // 2 s of wall time (hip_common.h)


// sgd = 0: the dW1 launch marks the gradient bucket's status element (one lane of workgroup 0, after its
// epilogue): 1.f when this rank's step is untrusted
__device__ __forceinline__ void mark_status(const SplitStepArgs& a, int err) {
  if (a.gstatus && blockIdx.x == 0 && threadIdx.x == 0) *a.gstatus = poisoned(err) ? 1.f : 0.f;
}


__device__ __forceinline__ float xf_load(const void* base, int64_t idx) {
  const auto w = __builtin_amdgcn_raw_buffer_load_b32(make_rsrc(base), (int)(idx * 4), 0, kXfSys);
  return __builtin_bit_cast(float, w);
}

// s_xf[0]: the tile's epoch; s_xf[1]: 1 = the tile is NOT exchanged or applied (block-uniform via LDS).
// A rank whose earlier wait timed out stops taking part altogether: it neither writes its IPC buffer (a
// peer may still be reading the other epoch's half there) nor publishes flags nor applies updates, so
// its peers time out too and every rank reports the error instead of stepping on stale data.
// An untrusted step of this rank (its forward + head launch timed out: ag_err) is treated the same way.
__device__ __forceinline__ bool xf_begin(const XgmiFuse& x, int tile, uint32_t* s_xf, const int* ag_err) {
  if (threadIdx.x == 0) {
    s_xf[0] = x.epochs[tile] + 1;
    s_xf[1] = (__hip_atomic_load(x.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) | ag_err_load(ag_err)) != 0;
  }
  __syncthreads();
  return s_xf[1] == 0;
}

// every thread's gradient stores of this tile are complete -> publish, wait for the peers.  Returns false
// (block-uniform) when a peer's flag never arrived: the caller then applies nothing for this tile.
__device__ __forceinline__ bool xf_exchange(const XgmiFuse& x, int tile, uint32_t* s_xf) {
  const uint32_t ep = s_xf[0];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int t = threadIdx.x;
  if (t < x.world) {
    // relaxed, not release: every byte a peer reads was stored write-through at system scope (xf_store)
    // and drained by every wave above, so a release would only write back the L2's OTHER dirty lines
    // (W1/plane updates no peer reads) once per tile.  bench.py checks the replicas bitwise after warm-up.
    __hip_atomic_store(x.peerflags[t] + tile * 8 + x.rank, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint64_t t0 = 0;  // (the clock only once the flag is missing: granule.h gran_poll)
    const uint32_t* f = x.myflags + tile * 8 + t;
    while ((int32_t)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - ep) < 0) {
      if (t0 == 0) t0 = wall_ticks();
      else if (wall_ticks() - t0 > kXfWaitTicks) {
        atomicExch(x.err, 1);
        s_xf[1] = 1;  // (the waiting lanes may race here: they all store 1)
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  // no acquire fence: every peer datum is read with system-coherent loads (xf_load) issued after the
  // flag was observed; a full L2 invalidation per tile measured +9 us per step (182 tiles)
  return s_xf[1] == 0;
}

__device__ __forceinline__ float xf_sum(const XgmiFuse& x, int64_t idx) {
  float s = xf_load(x.peers[0], idx);
  for (int r = 1; r < x.world; ++r) s += xf_load(x.peers[r], idx);
  return s;
}

__device__ __forceinline__ void xf_end(const XgmiFuse& x, int tile, const uint32_t* s_xf) {
  if (threadIdx.x == 0) x.epochs[tile] = s_xf[0];
}

// ---- the owner-tile push form (XgmiFuse::push) ------------------------------------------------------------
constexpr int kXpTile = 512;  // granule slots per tile (a dW1 tile is 16 x 32; a dW2 tile 16 x 16 + C)

__device__ __forceinline__ gran_t* xp_grad_slot(gran_t* slab, int tile, int src) {
  return slab + ((size_t)tile * 8 + src) * kXpTile;
}
__device__ __forceinline__ gran_t* xp_result_slot(const XgmiFuse& x, gran_t* slab, int tile) {
  return slab + ((size_t)x.slab_tiles * 8 + tile) * kXpTile;
}

// The push form's per-tile words, issued at workgroup entry by thread 0 WITHOUT a wait and waited for after the K
// loop (xp_words_wait): the tile's exchange epoch -- one returning add to epochs[tile] per launch (old + 1 is this
// launch's epoch on every rank: each launch adds one) -- and the bucket's and the forward's error words.  As inline
// asm they are counted by the hardware in issue order (every later vmcnt wait only gets stricter) and hipcc can
// neither sink them to their use after the K loop nor wait for them early: plain loads there were sunk behind the
// loop, a cold memory round trip (the words were written by the previous launch) in front of every exchange --
// 1.25 us per tile at world 1 (bench/stamps_push.py).
struct XpWords {
  uint32_t ep_old = 0;
  int err = 0, agerr = 0;
};
__device__ __forceinline__ XpWords xp_words_issue(const XgmiFuse& x, int tile, const int* ag_err) {
  XpWords w;
  asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(w.ep_old) : "v"(x.epochs + tile), "v"(1u) : "memory");
  asm volatile("global_load_dword %0, %1, off sc1" : "=v"(w.err) : "v"(x.err) : "memory");
  if (ag_err) asm volatile("global_load_dword %0, %1, off sc1" : "=v"(w.agerr) : "v"(ag_err) : "memory");
  return w;
}
__device__ __forceinline__ void xp_words_wait(XpWords& w) {
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(w.ep_old), "+v"(w.err), "+v"(w.agerr)::"memory");
}

// Bounded poll of the granules p[k] with bit k of `need` set until each carries tag ep (system-coherent loads of
// this rank's own receive area); v[k] = their values.  Wave-uniform; false once the wait outlasts the peer bound.
template <int N>
__device__ __forceinline__ bool xp_poll(const gran_t* const (&p)[N], unsigned need, unsigned ep, float (&v)[N]) {
  constexpr unsigned kAll = (1u << N) - 1u;
  unsigned rdy = ~need & kAll;
  gran_t g[N];
  uint64_t t0 = 0;  // (the clock only once a pass comes back incomplete: granule.h gran_poll)
  for (uint32_t pass = 1;; ++pass) {
    if (rdy != kAll) {
#pragma unroll
      for (int k = 0; k < N; ++k)
        if (!(rdy & (1u << k))) g[k] = gran_load_sys(p[k]);
#pragma unroll
      for (int k = 0; k < N; ++k)
        if (!(rdy & (1u << k))) rdy |= (unsigned)((unsigned)(g[k] >> 32) == ep) << k;
    }
    if (__all(rdy == kAll)) break;
    if (pass == 1) t0 = wall_ticks();
    else if ((pass & 7) == 0 && wall_ticks() - t0 > kXfWaitTicks) return false;
    __builtin_amdgcn_s_sleep(1);
  }
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] = (need & (1u << k)) ? __builtin_bit_cast(float, (unsigned)g[k]) : 0.f;
  return true;
}

// One tile through the owner-tile exchange.  Thread e < ne holds tile element e; xs[e] (LDS, complete) is this
// rank's gradient of it and `old` (owner only, loaded by the caller before the exchange) its current value.
// Returns true (block-uniform) with *nv the element's new value -- the owner's old - lr * (rank-order sum), the
// one-shot's expression, so both forms leave the same bits -- or false when a wait timed out (err set; the
// caller applies nothing, and a non-owner that times out never hears of it: its owner's wait times out too).
__device__ __forceinline__ bool xp_exchange(const XgmiFuse& x, int tile, uint32_t* s_xf, const float* xs, int ne,
                                            bool valid, float old, float lr, float* nv,
                                            unsigned long long* st = nullptr) {  // (st: diagnostics only)
  const unsigned ep = s_xf[0];
  const int owner = tile % x.world, e = threadIdx.x;
  const bool mine = valid && e < ne;
  bool ok;
  if (x.rank != owner) {
    if (mine) gran_store_sys(xp_grad_slot(x.peerslab[owner], tile, x.rank) + e, xs[e], ep);
    const gran_t* p[1] = {xp_result_slot(x, x.myslab, tile) + (mine ? e : 0)};
    float v[1];
    ok = xp_poll<1>(p, mine ? 1u : 0u, ep, v);
    *nv = v[0];
  } else {
    const gran_t* p[8];
    unsigned need = 0;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const bool want = mine && r < x.world && r != x.rank;
      p[r] = xp_grad_slot(x.myslab, tile, want ? r : 0) + (mine ? e : 0);
      need |= (unsigned)want << r;
    }
    float v[8];
    ok = xp_poll<8>(p, need, ep, v);
    if (ok && mine) {
      const float own = xs[e];
      float sum = x.rank == 0 ? own : v[0];
      for (int r = 1; r < x.world; ++r) sum += r == x.rank ? own : v[r];
      *nv = old - lr * sum;
    }
  }
  if (st && e == 0) st[5] = __builtin_amdgcn_s_memrealtime();
  if (!ok && (e & 63) == 0) {
    atomicExch(x.err, 1);
    s_xf[1] = 1;
  }
  __syncthreads();
  if (st && e == 0) st[6] = __builtin_amdgcn_s_memrealtime();
  if (s_xf[1]) return false;
  if (x.rank == owner && mine) {  // the update to every other rank
    for (int r = 0; r < x.world; ++r)
      if (r != x.rank) gran_store_sys(xp_result_slot(x, x.peerslab[r], tile) + e, *nv, ep);
  }
  return true;
}

// ======================================================================
// Kernel B: dW1 (MFMA over dZ1 planes x X^T) + fused reg/SGD/plane refresh,
//           dW2 and bias gradients as extra workgroup roles.
// ======================================================================
constexpr int kWMB = 1, kWNB = 2, kWKS = 8, kWT = 64 * kWKS;


template <int FU, int PV = 32, bool XPD = false>
__device__ __forceinline__ void wgrad_roles(const SplitStepArgs& a, int bid, int t1, int t2, float* red,
                                            uint32_t* s_xf, float* xs);

// AF (split3): dZ1 read in fp32 and split into its exact planes in registers (the head then writes no planes).
// FU: the gradient all-reduce fused in -- 0 none (SGD or the gradient bucket), 1 the one-shot pull, 2 the
// owner-tile push (SplitStepArgs::xf).  A template, not a runtime test: with the xGMI forms compiled into the one
// kernel, the single-process step's weight-gradient launch ran 0.8 us longer (rocprofv3, 784-100-10 at n = 800:
// 5.70 -> 6.51 us on one box, profiles/r5/regression_bisect.md) for code it never executes.
// DSWZ (AF, VEC == 3): dZ1 is read from the fragment-ordered buffer the head wrote (SplitStepArgs::dz_swz)
// XPD (FU == 2 only): the diagnostics instantiation that honours SplitStepArgs::xp_dbg (bench/kbench.py's push-form
// ablations).  Every production instantiation has XPD = false: the ablation tests fold away and the multi-GPU kernel
// carries none of them (a runtime branch of this kind cost a launch 0.8 us, profiles/r5/regression_bisect.md).
template <int NPZ, int VEC, bool AF, int FU, bool DSWZ = false, bool XPD = false>
__global__ __launch_bounds__(kWT) void wgrad_split_kernel(SplitStepArgs a, int t1, int t1n, int t2) {
  static_assert(!XPD || FU == 2, "the push-form ablations exist only in the push form");
  const int xdbg = XPD ? a.xp_dbg : 0;
  __shared__ __attribute__((aligned(16))) float red[kWKS * kWMB * kWNB * 4 * 64];
  __shared__ uint32_t s_xf[2];
  // the push form's staged gradient tile, then the current values (FU = 2); otherwise xs is the upper half of
  // `red`, which the dW2 role's GEMM leaves unused (the dW2 slices' partial tile)
  __shared__ float xsx[FU == 2 ? 2 * kXpTile : 1];
  float* xs = FU == 2 ? xsx : red + kWKS * 4 * 64;
  float* xo = xs + kXpTile;
  unsigned long long* wst = (CME_DIAG_STAMPS && a.wstamps) ? a.wstamps + (size_t)blockIdx.x * 8 : nullptr;  // diagnostics
  auto wstamp = [&](int i) {
    if (wst && threadIdx.x == 0) wst[i] = __builtin_amdgcn_s_memrealtime();
  };
  wstamp(0);
  if (a.pf_wgs && (int)blockIdx.x >= (int)gridDim.x - 8 * a.pf_wgs) {  // a prefetch workgroup (SplitStepArgs::pf_wgs):
    // the next step's X into the L2 of an XCD whose forward row tile reads all of it next
    const int xcd = blockIdx.x & 7, part = ((int)blockIdx.x - ((int)gridDim.x - 8 * a.pf_wgs)) >> 3;
    if (a.pf_X && a.pf_bytes > 0 && xcd < (a.H + 15) / 16)
      l2_touch(a.pf_X, 0, 1, 0, a.pf_bytes, part, a.pf_wgs, reinterpret_cast<char*>(red));
    return;
  }
  // logical workgroup id: dW1 tiles [0, t1) row-major, then the roles.  xcd_rows: the first 8 * t1n blocks are the
  // dW1 tiles with row tile rt on XCD rt (blockIdx % 8; slots of XCDs past the last row tile idle), roles after
  int bid = blockIdx.x, tb;
  if (a.xcd_rows) {
    const int grid1 = 8 * t1n, xcd = bid & 7, slot = bid >> 3;
    if (bid >= grid1) bid = t1 + (bid - grid1);
    else if (xcd * t1n + slot >= t1) return;  // (uniform)
    else bid = xcd * t1n + slot;
    tb = bid;
  } else {
    tb = bid < t1 ? xcd_remap(bid, t1) : bid;
  }
  const float reg = (float)a.reg, lr = (float)a.lr;
  constexpr bool fused = FU > 0;
  if (bid < t1) {  // ---- dW1 tile
    const int r1 = a.w1_rows < 0 ? a.H : a.w1_row0 + a.w1_rows;
    TileGeom g{r1, a.P + a.bias_col, a.n, a.w1_row0 + (tb / t1n) * 16 * kWMB, (tb % t1n) * 16 * kWNB};
    float *gw = a.gW1, *gb = a.gb1;
    // fused: gradients straight into this step's half of the IPC buffer (unless this rank is in error); the push
    // form stages them in LDS and decides whether to take part after the K loop (its words are prefetched)
    constexpr bool push = FU == 2;
    const bool live = fused && !push && xf_begin(*a.xf, bid, s_xf, a.ag_err);
    if (live) {
      gw = static_cast<float*>(a.xf->mybuf) + (int64_t)(s_xf[0] & 1u) * a.xf->npad;
      gb = gw + a.xf->off_b1;
    }
    EpiW1 epi{a.W1, gw, static_cast<bf16*>(a.W1p), (size_t)a.H * a.P, a.P, fused ? 0 : a.sgd, a.w1_planes ? a.npw : 0, reg, lr,
              a.xscale, {}, a.b1, gb, push ? 2 : (live ? 1 : 0), a.ag_err};
    if (a.w1_swz) epi.W1s = a.W1s;
    XpWords xw;
    if (push) {
      epi.xs = xs;
      epi.xo = xo;
      epi.m0 = g.m0;
      epi.n0 = g.n0;
      if (threadIdx.x == 0) xw = xp_words_issue(*a.xf, bid, a.ag_err);
    }
    constexpr int U = 4;
    if constexpr (AF && DSWZ)
      wsk_tile<bf16, kWMB, kWNB, kWKS, true, true, VEC, U, 3, uint8_t, float, true>(
          a.dZ1, (a.ld + 63) / 64, static_cast<const uint8_t*>(a.XT), a.ldxt, g, epi, red, 0, CME_DIAG_STAMPS ? a.stamps : nullptr);
    else if constexpr (AF)
      wsk_tile<bf16, kWMB, kWNB, kWKS, true, true, VEC, U, 3, uint8_t>(a.dZ1, a.ld, static_cast<const uint8_t*>(a.XT),
                                                                       a.ldxt, g, epi, red, 0, CME_DIAG_STAMPS ? a.stamps : nullptr);
    else
      wsk_tile<bf16, kWMB, kWNB, kWKS, true, true, VEC, U, NPZ, uint8_t>(static_cast<const bf16*>(a.dZ1p), a.ld,
                                                                static_cast<const uint8_t*>(a.XT), a.ldxt, g, epi,
                                                                red, a.H * a.ld * (int)sizeof(bf16), CME_DIAG_STAMPS ? a.stamps : nullptr);
    wstamp(1);
    if (push && (xdbg & 16)) return;  // (diagnostics: no exchange work at all after the tile)
    if (push) {  // the owner-tile exchange: thread e holds element (e / 32, e % 32) of the tile
      const int e = threadIdx.x, row = g.m0 + e / 32, col = g.n0 + e % 32;
      const bool ok = e < 512 && row < g.M && col < g.N;
      const int64_t i = (int64_t)row * a.P + col;
      if (threadIdx.x == 0) {  // (thread 0's words decide for the whole workgroup)
        xp_words_wait(xw);
        s_xf[0] = xw.ep_old + 1;
        s_xf[1] = (xw.err | xw.agerr) != 0;
      }
      __syncthreads();  // xs / xo complete
      wstamp(4);
      float nv = ok ? xo[e] - lr * xs[e] : 0.f;
      if (!s_xf[1] && ((xdbg & 1) || xp_exchange(*a.xf, bid, s_xf, xs, 512, ok, ok ? xo[e] : 0.f, lr, &nv, wst)) &&
          ok && !(xdbg & 2)) {
        if (col < a.P) {
          a.W1[i] = nv;
          if (a.w1_swz) a.W1s[w1s_off(row, col, (a.P + 63) >> 6)] = nv;
          if (a.w1_planes) {
            if (a.npw == 3) split_store<3>(nv, static_cast<bf16*>(a.W1p), (size_t)a.H * a.P, (size_t)i);
            else split_store<1>(nv, static_cast<bf16*>(a.W1p), (size_t)a.H * a.P, (size_t)i);
          }
        } else {
          a.b1[row] = nv;
        }
      }
    } else if (live && xf_exchange(*a.xf, bid, s_xf)) {  // all-reduced with the peers: SGD + bf16 planes
      const int64_t half = (int64_t)(s_xf[0] & 1u) * a.xf->npad;
      constexpr int TW = 16 * kWNB;
      for (int e = threadIdx.x; e < 16 * kWMB * TW; e += kWT) {
        const int row = g.m0 + e / TW, col = g.n0 + e % TW;
        if (row >= g.M || col >= g.N) continue;
        if (col < a.P) {
          const int64_t i = (int64_t)row * a.P + col;
          const float w = a.W1[i] - lr * xf_sum(*a.xf, half + i);
          a.W1[i] = w;
          if (a.w1_swz) a.W1s[w1s_off(row, col, (a.P + 63) >> 6)] = w;
          if (!a.w1_planes) continue;
          if (a.npw == 3) split_store<3>(w, static_cast<bf16*>(a.W1p), (size_t)a.H * a.P, (size_t)i);
          else split_store<1>(w, static_cast<bf16*>(a.W1p), (size_t)a.H * a.P, (size_t)i);
        } else {
          a.b1[row] -= lr * xf_sum(*a.xf, half + a.xf->off_b1 + row);
        }
      }
      xf_end(*a.xf, bid, s_xf);
    }
    wstamp(2);
    mark_status(a, epi.perr);
    if (wst) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      wstamp(3);
    }
    return;
  }
  wgrad_roles<FU, 32, XPD>(a, bid, t1, t2, red, s_xf, xs);
  if (wst) {  // (no barrier: the roles' returns are not block-uniform)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wstamp(3);
  }
}

// The weight-gradient launch's workgroups past its t1 dW1 tiles: t2 dW2 tiles (+ the fused xGMI exchange)
// followed by the bias-row workgroups.  `red`: kWKS * 4 * 64 floats of LDS, `s_xf`: 2 words of LDS.
// Shared by wgrad_split_kernel and the wide engines' launches (their extra workgroups).
// PV: dW2 partial loads in flight per lane (the small launch sums cdiv(n, 16) partials: 32; the wide launches' roles,
// which share their CUs with the GEMM tiles, sum cdiv(n, 32 or 128): 8)
template <int FU, int PV, bool XPD>
__device__ __forceinline__ void wgrad_roles(const SplitStepArgs& a, int bid, int t1, int t2, float* red,
                                            uint32_t* s_xf, float* xs) {
  const float reg = (float)a.reg, lr = (float)a.lr;
  const int xdbg = XPD ? a.xp_dbg : 0;  // (diagnostics instantiation only: wgrad_split_kernel XPD)
  constexpr bool fused = FU > 0;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (bid < t1 + t2) {  // ---- dW2 = D a1^T on MFMA (exact f32 16x16x4): one 16x16 tile per workgroup,
    //                        the 8 waves split K = batch; fused reg + SGD (or gradient) epilogue
    const int tb = bid - t1;
    TileGeom g{a.C, a.H, a.n, 0, tb * 16};
    float* gw = a.gW2;
    constexpr bool push = FU == 2;
    const bool live = fused && (push || xf_begin(*a.xf, bid, s_xf, a.ag_err));
    const int64_t half = push ? 0 : (int64_t)(s_xf[0] & 1u) * a.xf->npad;
    if (live && !push) gw = static_cast<float*>(a.xf->mybuf) + half + a.xf->off_W2;
    EpiW2 epi{a.W2, gw, a.H, fused ? 0 : a.sgd, push ? 2 : (live ? 1 : 0), reg, lr, {}, a.ag_err};
    XpWords xw;
    if (push) {
      epi.xs = xs;
      epi.xo = xs + kXpTile;
      epi.n0 = tb * 16;
      if (threadIdx.x == 0) xw = xp_words_issue(*a.xf, bid, a.ag_err);
    }
    if (a.dw2part) {  // the head's per-column-tile partials, summed in tile order (16 rows x C classes)
      const int nct = (a.n + a.dw2_cols - 1) / a.dw2_cols, e = threadIdx.x, c = e >> 4, h = tb * 16 + (e & 15);
      const bool ok = e < 256 && c < a.C && h < a.H;
      epi.prefetch(0, c, h, ok);
      const __amdgpu_buffer_rsrc_t rp = make_rsrc(a.dw2part);
      float v = 0.f;
      for (int k0 = 0; k0 < nct; k0 += PV) {  // (PV = 32 loads in flight per lane: n <= 1024 is one round trip)
        float pv[PV];
#pragma unroll
        for (int u = 0; u < PV; ++u)
          pv[u] = buf_load1<float>(rp, (ok && k0 + u < nct) ? (((k0 + u) * 16 + c) * a.H + h) * 4 : kOOB);
#pragma unroll
        for (int u = 0; u < PV; ++u) v += pv[u];
      }
      if (ok) epi(0, c, h, v);
    } else if (a.n % 4 == 0) {
      wsk_tile<float, 1, 1, kWKS, true, true, 1, 8>(a.D, a.ld, a.a1, a.ld, g, epi, red, 0, CME_DIAG_STAMPS ? a.stamps : nullptr);
    } else {
      wsk_tile<float, 1, 1, kWKS, true, true, 0, 8>(a.D, a.ld, a.a1, a.ld, g, epi, red, 0, CME_DIAG_STAMPS ? a.stamps : nullptr);
    }
    if (!live || (push && (xdbg & 32))) return;  // (xp_dbg 32: diagnostics, the roles stop after the GEMM)
    if (push) {  // the owner-tile exchange: element e < 256 is W2[e / 16][tb * 16 + e % 16]
      const int e = threadIdx.x, c = e / 16, h = tb * 16 + e % 16;
      const bool ok = e < 256 && c < a.C && h < a.H;
      const int64_t i = (int64_t)c * a.H + h;
      if (threadIdx.x == 0) {
        xp_words_wait(xw);
        s_xf[0] = xw.ep_old + 1;
        s_xf[1] = (xw.err | xw.agerr) != 0;
      }
      __syncthreads();  // xs / xo complete
      const float old = ok ? xs[kXpTile + e] : 0.f;
      float nv = ok ? old - lr * xs[e] : 0.f;  // (xp_dbg 4: diagnostics, no exchange -- world 1's own value)
      if (!s_xf[1] && ((xdbg & 4) || xp_exchange(*a.xf, bid, s_xf, xs, 256, ok, old, lr, &nv)) && ok) a.W2[i] = nv;
      return;
    }
    if (!xf_exchange(*a.xf, bid, s_xf)) return;
    for (int e = threadIdx.x; e < 256; e += kWT) {
      const int c = e / 16, h = tb * 16 + e % 16;
      if (c >= a.C || h >= a.H) continue;
      const int64_t i = (int64_t)c * a.H + h;
      a.W2[i] -= lr * xf_sum(*a.xf, half + a.xf->off_W2 + i);
    }
    xf_end(*a.xf, bid, s_xf);
    return;
  }
  if (fused) {  // ---- db2 (the fused launch's last role, exchange tile t1 + t2): one wave per class, in parallel
    //               with the dW1 / dW2 tiles (inside the first dW2 tile it was a dependent pass over D after the
    //               tile's GEMM, on the launch's critical path: -0.9 us at world 1, bench/kbench.py xp_dbg rows)
    if (bid != t1 + t2) return;
    constexpr bool push = FU == 2;
    const bool live = push || xf_begin(*a.xf, bid, s_xf, a.ag_err);
    if (!live) return;
    const int64_t half = push ? 0 : (int64_t)(s_xf[0] & 1u) * a.xf->npad;
    XpWords xw;
    if (push && threadIdx.x == 0) xw = xp_words_issue(*a.xf, bid, a.ag_err);
    const float bold = (int)threadIdx.x < a.C ? a.b2[threadIdx.x] : 0.f;
    for (int c = wv; c < a.C; c += kWKS) {
      const float sc = wave_sum(row_sum(a.D + (size_t)c * a.ld, a.n, lane));
      if (lane == 0) {
        if (push) xs[c] = sc;
        else xf_store(static_cast<float*>(a.xf->mybuf), half + a.xf->off_b2 + c, sc);
      }
    }
    if (push) {
      const int e = threadIdx.x;
      const bool ok = e < a.C;
      if (threadIdx.x == 0) {
        xp_words_wait(xw);
        s_xf[0] = xw.ep_old + 1;
        s_xf[1] = (xw.err | xw.agerr) != 0;
      }
      __syncthreads();  // xs complete
      float nv = ok ? bold - lr * xs[e] : 0.f;
      if (!s_xf[1] && ((xdbg & 8) || xp_exchange(*a.xf, bid, s_xf, xs, a.C, ok, bold, lr, &nv)) && ok) a.b2[e] = nv;
      return;
    }
    if (!xf_exchange(*a.xf, bid, s_xf)) return;
    for (int c = threadIdx.x; c < a.C; c += kWT) a.b2[c] = bold - lr * xf_sum(*a.xf, half + a.xf->off_b2 + c);
    xf_end(*a.xf, bid, s_xf);
    return;
  }
  // ---- bias gradients: one wave per row; rows [0,H) -> db1 from dZ1, [H,H+C) -> db2 from D
  const int row = (bid - t1 - t2) * kWKS + wv + (a.bias_col ? a.H : 0);  // db1 fused into dW1: db2 rows only
  if (row >= a.H + a.C) return;
  const bool first = row < a.H;
  const float* src = first ? a.dZ1 + (size_t)row * a.ld : a.D + (size_t)(row - a.H) * a.ld;
  const float bpre = buf_load1<float>(make_rsrc(first ? a.b1 : a.b2), (first ? row : row - a.H) * 4);
  const int perr = ag_err_load(a.ag_err);
  const float s = wave_sum(row_sum(src, a.n, lane));
  if (lane == 0) {
    float* bp = first ? a.b1 : a.b2;
    const int r = first ? row : row - a.H;
    if (a.sgd && !poisoned(perr)) bp[r] = bpre - lr * s;
    else (first ? a.gb1 : a.gb2)[r] = s;
  }
}

// the fragment-ordered copy of W1 rebuilt from W1 (padding slots: 0)
__global__ __launch_bounds__(256) void w1s_kernel(const float* __restrict__ W, float* __restrict__ Ws, int H, int P,
                                                  int64_t total) {
  const int npair = (P + 63) >> 6;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int e = (int)(t & 3), lane = (int)((t >> 2) & 63), i = (int)((t >> 8) & 3);
    const int64_t rp = t >> 10;  // rt * npair + p
    const int p = (int)(rp % npair), rt = (int)(rp / npair);
    const int row = rt * 16 + (lane & 15), col = p * 64 + (lane >> 4) * 16 + i * 4 + e;
    Ws[t] = (row < H && col < P) ? W[(int64_t)row * P + col] : 0.f;
  }
}

template <int NP>
__global__ __launch_bounds__(256) void planes_kernel(const float* __restrict__ W, bf16* __restrict__ p, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    split_store<NP>(W[i], p, (size_t)n, (size_t)i);
}

template <int NP>
__global__ __launch_bounds__(256) void sgd_planes_kernel(float* __restrict__ prm, const float* __restrict__ g,
                                                         int64_t n, float lr, bf16* __restrict__ planes,
                                                         int64_t w1n, const float* __restrict__ status) {
  // the bucket's status element (summed over the ranks): some rank's step is untrusted -> no update anywhere
  if (status && __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, *status)) != 0) return;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float v = prm[i] - lr * g[i];
    prm[i] = v;
    if (planes && i < w1n) split_store<NP>(v, planes, (size_t)w1n, (size_t)i);
  }
}

// ---- the same two GEMMs on the direct-to-LDS engine (glds_gemm.h): bf16 copies of X / XT as B.
// Epilogues are written out here (not element functors): every operand they need is loaded BEFORE the K
// loop, out-of-range elements go to the kOOB offset (loads return 0, stores are dropped), no branches.
__device__ __forceinline__ void st_f32(__amdgpu_buffer_rsrc_t r, int off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0, 0);
}
__device__ __forceinline__ void st_bf16(__amdgpu_buffer_rsrc_t r, int off, bf16 v) {
  __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, v), r, off, 0, 0);
}

// ---- wide layers: the head fused into the forward launch (all-gather form, H >= 512).
// Every BM x BN a1 tile is still in its workgroup's accumulators when the forward GEMM ends, so instead of
// storing z2 partials for head_wide_kernel to reduce (and re-reading all of a1 there), the tm row-tile
// workgroups of a column tile hand off twice, both times through DATA-TAGGED GRANULES -- 8 bytes {value,
// epoch}, each written by ONE sc1 store (MI355X_MICROARCH.md price list 'handoff-1to1'; cdna_hip_programming.md
// Guideline 16 R2): the data is its own flag, so a hand-off is one poll that returns the payload, with no
// store drain, no counter add and no separate payload load behind it.
//   0. before its K loop every workgroup makes ONE agent-scope add to its column tile's monotonic counter.
//      Each launch adds exactly tm per tile (every workgroup adds, whatever happens later; one counter array
//      per tiling, so a partial batch switching 128 x 128 <-> 64 x 64 keeps both aligned), hence the launch
//      epoch is old / tm + 1, never 0 (a kernel argument cannot carry it: graph replays freeze them); the tag
//      is 2 epoch + tiling, so the two tilings' launches never accept each other's granules;
//   1. every workgroup stores its z2 partial as granules tagged with the epoch (RegaAgArgs::z2g);
//   2. row tile rt < BN / 16 polls the tm partials of its 16 columns until every tag is the epoch, sums them in
//      tile order (+ b2) and forms softmax / D / the loss partial of those columns exactly as head_wide_kernel
//      does (same operation order: bit-identical D, loss and dZ1); D goes out as tagged granules (dg) and as
//      plain fp32 for the weight-gradient launch;
//   3. every workgroup polls the tile's 16 x BN D granules and forms dZ1 = (W2^T D) .* a1 .* (1 - a1) for its
//      own tile on the f32 MFMA, plus the tile's dW2 partial D . a1^T (SplitStepArgs::dw2_cols = BN).
// Every workgroup must be resident at once (one per CU: the launcher's LDS request and tm * tn <= CUs).  A poll
// that outlasts ag_wait_us of wall time sets *err (MlpEngine.kernel_error()) and the workgroup writes nothing
// more; the weight-gradient launch that follows applies nothing (SplitStepArgs::ag_err).
}  // namespace
// (outside the anonymous namespace: the fp32 launchers of mlp_wide_f32.hip, the same source compiled apart, take it)
struct RegaAgArgs {
  HeadArgs h{};
  unsigned long long* counters = nullptr;  // [column tile * kRegaAgCounterStride], monotonic: the launch epoch
  unsigned long long* z2g = nullptr;       // z2 partial granules [tm][16][ld]
  unsigned long long* dg = nullptr;        // D granules [16][ld]
  int* err = nullptr;
  int store_a1 = 1;  // 0: a1 is not stored (nothing after the fused head reads it)
  int tm = 0;        // row tiles
  int ep_off = 0;    // LDS byte offset of the epoch + 2 flag words (past every other LDS use of the launch)
  int tiling = 0;    // 0: 128 x 128, 1: 64 x 64 -- the low bit of every tag (both tilings share the granules)
};
namespace {
constexpr int kRegaAgCounterStride = 32;  // uint64 words: one 256-byte line per column-tile counter
// LDS of the fused head for a BM x BN tile: the D tile [16][BN + 4], the a1 tile [BM][BN + 4] (row pitch BN + 4:
// conflict-free MFMA-layout reads), z2 [16][17], loss [16]
template <int BM, int BN>
constexpr int wide_ag_lds_bytes() {
  return (16 * (BN + 4) + BM * (BN + 4) + 16 * 17 + 16) * 4;
}
// the launch's dynamic LDS: > 80 KB keeps it at one workgroup per CU (the hand-off's measured form), and the
// last 16 bytes hold the epoch and the two timeout flags (no other use reaches them)
constexpr int wide_ag_launch_lds(int used) { return (used + 16 > 84 * 1024 ? used + 16 : 84 * 1024) / 16 * 16; }

__device__ __forceinline__ void ag_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// diagnostics (SplitStepArgs::stamps, bench/stamps_wide_ag.py): thread 0 records s_memrealtime (100 MHz) as
// stamp i of this workgroup's 8: 0 entry, 1 K loop done, 2 z2 granules stored, 3 hand-off 1 done, 4 D stored
// (reducers), 5 D arrived, 6 end (stores drained)
__device__ __forceinline__ void ag_stamp(const SplitStepArgs& a, int i, bool drain = false) {
  if (!CME_DIAG_STAMPS || !a.stamps) return;  // (the diagnostics library only)
  if (drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) a.stamps[(size_t)blockIdx.x * 8 + i] = __builtin_amdgcn_s_memrealtime();
}

// kernel entry, thread 0 only: this workgroup's epoch add (the returned count is used after the K loop)
__device__ __forceinline__ gran_t ag_epoch_add(const RegaAgArgs& g, int ct) {
  return gran_epoch_add(g.counters + (size_t)ct * kRegaAgCounterStride);  // (no wait: granule.h)
}
// after the K loop, before the first barrier that follows it, thread 0: the epoch + zeroed flags into LDS
__device__ __forceinline__ void ag_epoch_publish(const RegaAgArgs& g, char* lds, gran_t old) {
  gran_epoch_wait(old);
  unsigned* w = reinterpret_cast<unsigned*>(lds + g.ep_off);
  w[0] = (((unsigned)(old / (unsigned)g.tm) + 1u) << 1) | (unsigned)g.tiling;
  w[1] = 0u;
  w[2] = 0u;
}

// BM x BN tile at (m0, n0); this wave holds a1v[nb][j] = a1(row rw + 4 fg + j, column cw + 16 nb + fr) (16 rows x
// 16 NB columns); tm row tiles; ct = column tile.  BN / 16 row tiles reduce 16 columns each (tm >= BN / 16).
// Called after the barrier that follows ag_epoch_publish and the z2 granule stores.
template <int BM, int BN, int NB>
__device__ __forceinline__ void wide_head_ag(const SplitStepArgs& a, const RegaAgArgs& g, const f32x4 (&a1v)[NB],
                                             char* lds, int m0, int n0, int rw, int cw, int tm, int ct) {
  constexpr int LD = BN + 4, NU = BN / 16, NDS = 16 * BN / 512;
  static_assert(NDS * 512 == 16 * BN && BM % 16 == 0 && BM / 16 <= 8, "tile shape");
  const HeadArgs& h = g.h;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, fr = lane & 15, fg = lane >> 4;
  const int H = a.H, n = a.n, C = a.C, rt = m0 / BM;
  float* Ds = reinterpret_cast<float*>(lds);  // [16][LD] the column tile's D
  float* ts = Ds + 16 * LD;                     // [BM][LD] the a1 tile
  float* zs = ts + BM * LD;                     // [16][17] z2 (+ b2) of the reduced 16 columns
  float* ls = zs + 16 * 17;                         // [16] loss of those columns
  unsigned* sw = reinterpret_cast<unsigned*>(lds + g.ep_off);  // [0] epoch, [1] [2] timeout flags
  const unsigned ep = sw[0];
  const uint32_t limit = (uint32_t)a.ag_wait_us;
  // independent loads first: the W2^T operand of dZ1 (class 4 fg + i, row rw + fr), the reducer's labels, b2
  float wv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    wv[i] = buf_load1<float>(make_rsrc(a.W2), (4 * fg + i < C && rw + fr < H) ? ((4 * fg + i) * H + rw + fr) * 4 : kOOB);
  const int u0 = n0 + 16 * rt;  // the 16 columns row tile rt < NU reduces
  const bool red = rt < NU && u0 < n;
  // (the label of this thread's softmax column u0 + (t >> 4), fetched now)
  const int lab_pre = (int)__builtin_amdgcn_raw_buffer_load_b32(
      make_rsrc(h.labels), (red && t < 256 && u0 + (t >> 4) < n) ? (u0 + (t >> 4)) * 4 : kOOB, 0, 0);
  const int zc = t >> 4, zcol = u0 + (t & 15);
  const float b2v = buf_load1<float>(make_rsrc(h.b2), (red && t < 256 && zc < C) ? zc * 4 : kOOB);
  // ---- hand-off 1 (reducers): the tm z2 partials of (class zc, column zcol), in tile order, 32 per poll
  if (red && t < 256) {
    const bool need = zc < C && zcol < n;
    const unsigned stride = 16u * (unsigned)a.ld;
    float zsum = 0.f;
    bool good = true;
    for (int k0 = 0; k0 < tm && good; k0 += 16)  // the partials summed in tile order, 16 per poll
      good = gran_poll<16>(g.z2g, (unsigned)(k0 * 16 + zc) * a.ld + zcol, stride, min(16, tm - k0), need, ep, limit,
                           [&](int, float v) { zsum += v; });
    if (!good && lane == 0) {
      atomicExch(g.err, 1);
      sw[1] = 1u;
    }
    zs[zc * 17 + (t & 15)] = zsum + (zc < C ? b2v : 0.f);
  }
  __syncthreads();  // (also: every wave's reads of the z2 reduction scratch in lds are done)
  ag_stamp(a, 3);
  if (sw[1]) return;  // workgroup-uniform: a partial never arrived
  // ---- softmax / loss / D of columns u0 .. u0 + 15
  if (red) {
    if (t < 256) {  // softmax / loss / D: 16 lanes (classes) per column, 4 columns per wave
      const int col2 = t >> 4, cls = t & 15, col = u0 + col2, lb = lane & ~15;
      const bool ok = col < n;
      const int lab = ok ? lab_pre : -1;
      const float z = zs[cls * 17 + col2];
      float m = 0.f;
      if (h.shift) {  // (max is exact: any order gives head_wide_kernel's value)
        m = cls < C ? z : -3.402823466e38f;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
      }
      const float e = cls < C ? __expf(z - m) : 0.f;
      // the class sum in class order, as head_wide_kernel adds it: bit-identical D, loss and dZ1
      float sum = 0.f;
#pragma unroll
      for (int c = 0; c < 16; ++c) sum += __shfl(e, lb + c, 64);
      const float inv = 1.f / sum, sc = (float)h.scale;
      const bool hit = cls == lab;
      float d;
      const float y = head_prob_grad(e, inv, hit, sc, d);  // head_wide_kernel's arithmetic (head_math.h)
      if (!(ok && cls < C)) d = 0.f;
      float lp = hit ? -__logf(y) : 0.f;  // one non-zero lane per column: any summation order is exact
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) lp += __shfl_xor(lp, o, 64);
      const bool hooked = a.ag_test_skip == rt && ct == 0;  // test hook: this tile's D never arrives
      if (ok && cls < C) {
        st_f32(make_rsrc(h.D), (cls * h.ldd + col) * 4, d);  // for the weight-gradient launch
        if (!hooked) gran_store(g.dg + (size_t)cls * a.ld + col, d, ep);
      }
      if (cls == 0) ls[col2] = lp;
    }
    __syncthreads();
    ag_stamp(a, 4, true);
    if (t == 0 && h.loss_partial) {  // the column head's layout: one partial per 16 columns
      float s = 0.f;
      for (int k = 0; k < 16; ++k) s += ls[k];
      h.loss_partial[u0 / 16] = s;
    }
  }
  // ---- hand-off 2: the tile's 16 x BN D granules.  Lane t's NDS granules are D rows c = t / BN + q * 512 / BN
  // of column n0 + t % BN: the needed ones (c < C, column < n) are the first `cnt`
  {
    constexpr int kRowsPerQ = 512 / BN;
    const int c0 = t / BN, j = t % BN;
    int cnt = 0;
#pragma unroll
    for (int q = 0; q < NDS; ++q) cnt += (c0 + kRowsPerQ * q < C && n0 + j < n) ? 1 : 0;
    float v[NDS];
#pragma unroll
    for (int q = 0; q < NDS; ++q) v[q] = 0.f;
    const bool good = gran_poll<NDS>(g.dg, (unsigned)c0 * a.ld + n0 + j, (unsigned)(kRowsPerQ * a.ld), cnt, cnt > 0,
                                     ep, limit, [&](int q, float x) { v[q] = x; });
    if (!good && lane == 0) {
      atomicExch(g.err, 1);
      sw[2] = 1u;
    }
#pragma unroll
    for (int q = 0; q < NDS; ++q) Ds[(c0 + kRowsPerQ * q) * LD + j] = q < cnt ? v[q] : 0.f;
  }
  // this wave's a1 block into the row-major a1 tile, for the dW2 partial's B operand
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int j = 0; j < 4; ++j) ts[(rw - m0 + 4 * fg + j) * LD + cw - n0 + 16 * nb + fr] = a1v[nb][j];
  __syncthreads();
  ag_stamp(a, 5);
  if (sw[2]) return;  // workgroup-uniform: the tile's D never arrived
  if (h.dw2part && wave < BM / 16) {
    // P[c][row m0 + 16 wave + fr] = sum over the tile's BN columns of D[c][col] a1[row][col] (head_wide_kernel's
    // chain over BN columns instead of 32): A = D, B = the row-major a1 rows
    const float* tr = ts + 16 * wave * LD;
    f32x4 pw = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < BN / 4; ++s)
      pw = __builtin_amdgcn_mfma_f32_16x16x4f32(Ds[fr * LD + 4 * s + fg], tr[fr * LD + 4 * s + fg], pw, 0, 0, 0);
    const int hh = m0 + 16 * wave + fr;
    const __amdgpu_buffer_rsrc_t rp = make_rsrc(h.dw2part);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      st_f32(rp, (4 * fg + r < C && hh < H) ? ((ct * 16 + 4 * fg + r) * H + hh) * 4 : kOOB, pw[r]);
  }
  // dZ1 of this wave's block, written over its a1 block in the LDS tile (every dW2 read of it is done after the
  // barrier), then read back as 4 consecutive columns per lane: 16-byte fp32 stores / 8-byte plane stores along
  // rows instead of a 4-byte (2-byte) scatter in the MFMA layout
  __syncthreads();
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    f32x4 r = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i)
      r = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[i], Ds[(4 * fg + i) * LD + cw - n0 + 16 * nb + fr], r, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x = a1v[nb][j];
      ts[(rw - m0 + 4 * fg + j) * LD + cw - n0 + 16 * nb + fr] = r[j] * x * (1.f - x);
    }
  }
  ag_wave_sync();  // (each wave re-reads only its own block)
  constexpr int CPR = 4 * NB;  // 4-column chunks per row of the wave's block
  const __amdgpu_buffer_rsrc_t rdz = make_rsrc(h.dZ1), rpl = make_rsrc(h.dZ1_planes);
  if (NB % 2 == 0 && !h.dZ1 && h.npz == 1 && h.ldz % 8 == 0) {  // bf16 (split1): 8 columns per lane, one 16-byte store
    constexpr int CPR8 = 2 * NB;
#pragma unroll
    for (int q = 0; q < 16 * CPR8 / 64; ++q) {
      const int c = q * 64 + lane, rr = c / CPR8, c8 = (c % CPR8) * 8;
      const int row = rw + rr, col = cw + c8;
      const float* src = ts + (rw - m0 + rr) * LD + cw - n0 + c8;
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(src), v1 = *reinterpret_cast<const f32x4*>(src + 4);
      const bool rok = row < H;
      unsigned short qb[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        qb[e] = __builtin_bit_cast(unsigned short, __float2bfloat16(v0[e]));
        qb[4 + e] = __builtin_bit_cast(unsigned short, __float2bfloat16(v1[e]));
      }
      const int base = (row * h.ldz + col) * 2;
      if (rok && col + 8 <= n) {
        __attribute__((ext_vector_type(4))) unsigned w;
        __builtin_memcpy(&w, qb, 16);
        __builtin_amdgcn_raw_buffer_store_b128(w, rpl, base, 0, 0);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          __builtin_amdgcn_raw_buffer_store_b16(qb[e], rpl, (rok && col + e < n) ? base + 2 * e : kOOB, 0, 0);
      }
    }
  } else
#pragma unroll
  for (int q = 0; q < 16 * CPR / 64; ++q) {
    const int c = q * 64 + lane, rr = c / CPR, c4 = (c % CPR) * 4;
    const int row = rw + rr, col = cw + c4;
    const f32x4 v = *reinterpret_cast<const f32x4*>(ts + (rw - m0 + rr) * LD + cw - n0 + c4);
    const bool rok = row < H, full = rok && col + 4 <= n;
    if (h.dZ1) {  // (dz_swz == 2: in the weight-gradient K loop's fragment order, rega_gemm.h dzr_off; the 4 columns
      //            col .. col + 3 stay one 16-byte group there)
      const int nst = (h.ldz + 31) >> 5;
      if (full) {
        __attribute__((ext_vector_type(4))) unsigned w;
        __builtin_memcpy(&w, &v, 16);
        const int off = h.dz_swz == 2 ? (int)dzr_off(row, col, nst) : row * h.ldz + col;
        __builtin_amdgcn_raw_buffer_store_b128(w, rdz, off * 4, 0, 0);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float ve = v[e];
          const int off = h.dz_swz == 2 ? (int)dzr_off(row, col + e, nst) : row * h.ldz + col + e;
          st_f32(rdz, (rok && col + e < n) ? off * 4 : kOOB, ve);
        }
      }
    }
    if (h.dZ1_planes) {
      float rem[4] = {v[0], v[1], v[2], v[3]};
      for (int p = 0; p < h.npz; ++p) {
        unsigned short qb[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bf16 qv = __float2bfloat16(rem[e]);
          qb[e] = __builtin_bit_cast(unsigned short, qv);
          rem[e] -= __bfloat162float(qv);
        }
        const int base = ((p * H + row) * h.ldz + col) * 2;
        if (full) {
          __attribute__((ext_vector_type(2))) unsigned w;
          w.x = (unsigned)qb[0] | ((unsigned)qb[1] << 16);
          w.y = (unsigned)qb[2] | ((unsigned)qb[3] << 16);
          __builtin_amdgcn_raw_buffer_store_b64(w, rpl, base, 0, 0);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            __builtin_amdgcn_raw_buffer_store_b16(qb[e], rpl, (rok && col + e < n) ? base + 2 * e : kOOB, 0, 0);
        }
      }
    }
  }
  if (CME_DIAG_STAMPS && a.stamps) {
    __syncthreads();
    ag_stamp(a, 6, true);
  }
}

// a1 = sigmoid(W1 X + b1) and (z2p != nullptr) the head's z2 partials of this tile's rows:
// z2p[row tile][class][col] = sum over the tile rows h of W2[class][h] a1[h][col]
template <int BM, int BN, int NPW, bool AG = false>
__global__ __launch_bounds__(512) void fwd1_glds_kernel(SplitStepArgs a, int tn, RegaAgArgs ag = {}) {
  extern __shared__ __attribute__((aligned(16))) char lds_dyn[];
  using G = GldsGeom<BM, BN>;
  constexpr int MB = G::MB, NB = G::NB;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (id / tn) * BM, n0 = (id % tn) * BN;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1, fr = lane & 15, fg = lane >> 4;
  const int rw = m0 + wr * G::WM, cw = n0 + wc * G::WN;  // this wave's first row / column
  const int H = a.H, n = a.n, C = a.C;
  const bool z2 = a.z2part != nullptr || AG;
  gran_t ep_old = 0;  // the fused head's launch epoch (wide_head_ag step 0): one add per workgroup, now
  if (AG && threadIdx.x == 0) ep_old = ag_epoch_add(ag, n0 / BN);
  if (AG) ag_stamp(a, 0);
  // epilogue operands, issued before the K loop: b1 of this lane's rows, W2[class fr][those rows]
  const __amdgpu_buffer_rsrc_t rb1 = make_rsrc(a.b1), rw2 = make_rsrc(a.W2);
  float bb[MB][4], w2[MB][4];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int h = rw + 16 * mb + 4 * fg + i;
      bb[mb][i] = buf_load1<float>(rb1, h < H ? h * 4 : kOOB);
      w2[mb][i] = buf_load1<float>(rw2, (z2 && fr < C && h < H) ? (fr * H + h) * 4 : kOOB);
    }
  f32x4 acc[MB][NB];
  glds_gemm_mainloop<BM, BN, NPW>(static_cast<const bf16*>(a.W1p), a.P, H * a.P * (int)sizeof(bf16),
                                  static_cast<const bf16*>(a.Xw), a.P, H, n, a.P, m0, n0, lds_dyn, acc);
  if (AG) ag_stamp(a, 1);
  const __amdgpu_buffer_rsrc_t ra1 = make_rsrc(a.a1);
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = rw + 16 * mb + 4 * fg + i, col = cw + 16 * nb + fr;
        const float sv = sigm(acc[mb][nb][i] * a.xscale + bb[mb][i]);
        acc[mb][nb][i] = sv;
        if (!AG || ag.store_a1) st_f32(ra1, (row < H && col < n) ? (row * a.ld + col) * 4 : kOOB, sv);
      }
  if (!z2) return;
  // z2 partials on the f32 MFMA: step i of block mb takes B[k = fg][n = fr] = a1(row rw + 16 mb + 4 fg + i,
  // col fr) -- exactly accumulator element i -- and A[m = fr][k = fg] = W2[class fr][that row]; the 4 row
  // waves are summed through LDS (all K-loop reads of lds_dyn are done after the barrier)
  f32x4 z[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) z[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        z[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(w2[mb][i], acc[mb][nb][i], z[nb], 0, 0, 0);
  if (AG && threadIdx.x == 0) ag_epoch_publish(ag, lds_dyn, ep_old);
  __syncthreads();
  f32x4* red = reinterpret_cast<f32x4*>(lds_dyn);  // [4][2][NB][64]
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) red[((wr * 2 + wc) * NB + nb) * 64 + lane] = z[nb];
  __syncthreads();
  if (wr == 0) {
    const int tile = m0 / BM;
    const __amdgpu_buffer_rsrc_t rz = make_rsrc(a.z2part);
    const unsigned ep = AG ? reinterpret_cast<const unsigned*>(lds_dyn + ag.ep_off)[0] : 0u;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      f32x4 sz = red[(wc * NB + nb) * 64 + lane];
#pragma unroll
      for (int r = 1; r < G::WRN; ++r) sz += red[((r * 2 + wc) * NB + nb) * 64 + lane];
      const int col = cw + 16 * nb + fr;
#pragma unroll
      for (int i = 0; i < 4; ++i) {  // (classes past C are zero: not stored, the head does not read them)
        const float zv = sz[i];      // (a scalar copy: see fwd1_rega_kernel)
        if constexpr (AG) {  // tagged granules for the fused head (hand-off 1)
          if (col < n && 4 * fg + i < a.C) gran_store(ag.z2g + (size_t)(tile * 16 + 4 * fg + i) * a.ld + col, zv, ep);
        } else {
          __builtin_amdgcn_raw_buffer_store_b32(
              __builtin_bit_cast(unsigned, zv), rz,
              (col < n && 4 * fg + i < a.C) ? ((tile * 16 + 4 * fg + i) * a.ld + col) * 4 : kOOB, 0, 0);
        }
      }
    }
  }
  if constexpr (AG) {
    static_assert(MB == 1 && BM == 64 && BN == 64, "fused head: the 64 x 64 tiling (4 x 2 waves of 16 x 32)");
    f32x4 a1v[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) a1v[nb] = acc[0][nb];
    ag_stamp(a, 2, true);
    wide_head_ag<BM, BN, NB>(a, ag, a1v, lds_dyn, m0, n0, rw, cw, ag.tm, n0 / BN);
  }
}

// The wide dW1 launches' epilogue in ROW-CONTIGUOUS 4-column chunks: the BM x BN accumulator tile goes through
// an LDS transpose after the K loop, so W1 and the gradient move as 16-byte vectors and the planes as 8-byte
// vectors instead of a 4-byte (2-byte) scatter in the MFMA layout (at 128 x 128: 8 instead of 32 memory
// instructions per lane per array; 784-4096-10 step -1.1 us fp32, -0.8 us bf16).  Chunk q = t + 512 k: row
// q / (BN / 4), columns 4 (q % (BN / 4)) .. + 3.  P % 4 == 0 (the launchers check it), so a chunk is all weights,
// or -- the chunk at column P -- the all-ones feature's db1 in its first element.
typedef float f32x4v __attribute__((ext_vector_type(4)));
template <int BM, int BN>
struct W1Chunks {
  static constexpr int kCh = BM * BN / 4 / 512, CPR = BN / 4, LDT = BN + 4;
  static constexpr int kLdsBytes = BM * LDT * 4;
  static_assert(kCh * 512 * 4 == BM * BN, "tile of whole chunks per thread");
  f32x4v wq[kCh];
  float bq[kCh];
  // the weights (and b1 for the all-ones column) of this thread's chunks: issue BEFORE the K loop
  __device__ __forceinline__ void prefetch(const SplitStepArgs& a, int m0, int n0, int M) {
    const __amdgpu_buffer_rsrc_t rW = make_rsrc(a.W1), rb1 = make_rsrc(a.b1);
#pragma unroll
    for (int k = 0; k < kCh; ++k) {
      const int q = (int)threadIdx.x + 512 * k, row = m0 + q / CPR, col = n0 + 4 * (q % CPR);
      const bool rok = row < M;
      wq[k] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(
                                             rW, (rok && col + 4 <= a.P) ? (row * a.P + col) * 4 : kOOB, 0, 0));
      bq[k] = buf_load1<float>(rb1, (rok && a.bias_col && col == a.P) ? row * 4 : kOOB);
    }
  }
  // the MFMA-layout accumulators (this wave: rows rw + 16 mb + 4 fg + i, columns cw + 16 nb + fr) into the
  // transposed tile; call after the K loop (its LDS reads are then done once the first barrier passes)
  template <int MB, int NB>
  __device__ __forceinline__ void stage(char* lds, const f32x4 (&acc)[MB][NB], int rw, int cw, int m0, int n0, int fg,
                                        int fr) const {
    float* T = reinterpret_cast<float*>(lds);
    __syncthreads();
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int i = 0; i < 4; ++i) T[(rw - m0 + 16 * mb + 4 * fg + i) * LDT + cw - n0 + 16 * nb + fr] = acc[mb][nb][i];
    __syncthreads();
  }
  // reg + SGD (+ nps planes) in place (upd), or the pre-scaled gradient into gW1 / gb1
  __device__ __forceinline__ void apply(const SplitStepArgs& a, const char* lds, int m0, int n0, int M, bool upd,
                                        int nps) const {
    const float* T = reinterpret_cast<const float*>(lds);
    const float reg = (float)a.reg, lr = (float)a.lr, xs = a.xscale;
    const int P = a.P;
    const size_t plane = (size_t)a.H * P;
    const __amdgpu_buffer_rsrc_t rW = make_rsrc(a.W1), rg = make_rsrc(a.gW1), rp = make_rsrc(a.W1p);
#pragma unroll
    for (int k = 0; k < kCh; ++k) {
      const int q = (int)threadIdx.x + 512 * k, r = q / CPR, c4 = 4 * (q % CPR);
      const int row = m0 + r, col = n0 + c4;
      if (row >= M) continue;
      const f32x4v v = *reinterpret_cast<const f32x4v*>(T + r * LDT + c4);
      if (col + 4 <= P) {
        const int idx = row * P + col;
        f32x4v g, nw;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          g[e] = v[e] * xs + reg * wq[k][e];
          nw[e] = wq[k][e] - lr * g[e];
        }
        if (upd) {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ra::u32x4, nw), rW, idx * 4, 0, 0);
          float rem[4] = {nw[0], nw[1], nw[2], nw[3]};
          for (int pl = 0; pl < nps; ++pl) {
            unsigned short qb[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const bf16 hb = __float2bfloat16(rem[e]);
              qb[e] = __builtin_bit_cast(unsigned short, hb);
              rem[e] -= __bfloat162float(hb);
            }
            __attribute__((ext_vector_type(2))) unsigned w2;
            w2.x = (unsigned)qb[0] | ((unsigned)qb[1] << 16);
            w2.y = (unsigned)qb[2] | ((unsigned)qb[3] << 16);
            __builtin_amdgcn_raw_buffer_store_b64(w2, rp, (int)((pl * plane + idx) * 2), 0, 0);
          }
        } else {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ra::u32x4, g), rg, idx * 4, 0, 0);
        }
      } else if (a.bias_col && col == P) {  // all-ones feature: db1 (no input scale, no regulariser)
        if (upd) a.b1[row] = bq[k] - lr * v[0];
        else a.gb1[row] = v[0];
      }
    }
  }
};

// dW1 = dZ1 XT (+ the all-ones feature column P = db1) with the fused reg + SGD + bf16-plane refresh (sgd)
// or the pre-scaled gradient (sgd == 0); the dW2 / db2 role workgroups ride in the same launch
template <int BM, int BN, int NPZ>
__global__ __launch_bounds__(512) void wgrad_glds_kernel(SplitStepArgs a, int tn, int tbig, int t2) {
  extern __shared__ __attribute__((aligned(16))) char lds_dyn[];
  if ((int)blockIdx.x >= tbig) {  // the dW2 / db2 roles riding in this launch
    wgrad_roles<0, 8>(a, (int)blockIdx.x - tbig, 0, t2, reinterpret_cast<float*>(lds_dyn),
                reinterpret_cast<uint32_t*>(lds_dyn + kWKS * 4 * 64 * sizeof(float)),
                reinterpret_cast<float*>(lds_dyn + kWKS * 4 * 64 * sizeof(float) + 16));  // (never fused: unused;
                                                                                            //  2 x kXpTile floats)
    return;
  }
  using G = GldsGeom<BM, BN>;
  constexpr int MB = G::MB, NB = G::NB;
  // split-K (a.wg_ksplit > 1): workgroup -> (tile, K slice ks); the slice's columns [ks kc, ks kc + kc) of dZ1 and
  // XT are the GEMM's whole K, and the raw partial goes to slab ks (splitk_sgd_kernel applies the update)
  const int ksplit = a.wg_ksplit, tiles = tbig / ksplit;
  const int id0 = xcd_remap(blockIdx.x, tbig), id = id0 % tiles, ks = id0 / tiles;
  const int k0 = ks * a.wg_kchunk, klen = ksplit > 1 ? min(a.n - k0, a.wg_kchunk) : a.n;
  const int m0 = a.w1_row0 + (id / tn) * BM, n0 = (id % tn) * BN;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1, fr = lane & 15, fg = lane >> 4;
  const int rw = m0 + wr * G::WM, cw = n0 + wc * G::WN;
  const int M = a.w1_rows < 0 ? a.H : a.w1_row0 + a.w1_rows, P = a.P;
  const float reg = (float)a.reg, lr = (float)a.lr, xs = a.xscale;
  if (ksplit > 1) {
    f32x4 acc[MB][NB];
    glds_gemm_mainloop<BM, BN, NPZ>(static_cast<const bf16*>(a.dZ1p) + k0, a.ld, a.H * a.ld * (int)sizeof(bf16),
                                    static_cast<const bf16*>(a.XTw) + k0, a.ldxt, M, P + a.bias_col, klen, m0, n0,
                                    lds_dyn, acc);
    const int W = P + a.bias_col;
    const __amdgpu_buffer_rsrc_t rk = make_rsrc(a.kpart + (size_t)ks * (M - a.w1_row0) * W);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = rw + 16 * mb + 4 * fg + i, col = cw + 16 * nb + fr;
          st_f32(rk, (row < M && col < W) ? ((row - a.w1_row0) * W + col) * 4 : kOOB, acc[mb][nb][i]);
        }
    return;
  }
  // the weights this thread updates (and b1 for the all-ones column), before the K loop
  W1Chunks<BM, BN> wc1;
  wc1.prefetch(a, m0, n0, M);
  const int perr = ag_err_load(a.ag_err);  // the step's forward timed out: no update
  f32x4 acc[MB][NB];
  glds_gemm_mainloop<BM, BN, NPZ>(static_cast<const bf16*>(a.dZ1p), a.ld, a.H * a.ld * (int)sizeof(bf16),
                                  static_cast<const bf16*>(a.XTw), a.ldxt, M, P + a.bias_col, a.n, m0, n0, lds_dyn,
                                  acc);
  wc1.stage(lds_dyn, acc, rw, cw, m0, n0, fg, fr);
  wc1.apply(a, lds_dyn, m0, n0, M, a.sgd && !poisoned(perr), NPZ);  // (the W1 planes: npw == npz)
  mark_status(a, perr);
}

// a1 = sigmoid(W1 X + b1) on the A-in-registers engine (rega_gemm.h): W1 read as fp32 and split into the
// exact bf16 planes in registers (AT = float), or the bf16 plane 0 (AT = bf16, split1); z2 partials of
// this 128-row tile as in fwd1_glds_kernel
// The g64 engine's L2 pre-touch shares (g64::Touch) for a 128 x 128 tiling of `nwg` workgroups, tn column tiles,
// remapped by xcd_remap (each XCD holds a contiguous id range, i.e. whole rows of tiles when its range is a multiple
// of tn): the tn workgroups of a tile row share its A rows, the tile rows of one XCD share each B column tile.
// SplitStepArgs::g64_touch 0: none.
__device__ __forceinline__ g64::Touch g64_touch(const SplitStepArgs& a, int id, int nwg, int tn) {
  g64::Touch t;
  if (!a.g64_touch) return t;
  const int per_xcd = (nwg + 7) / 8, rows_per_xcd = per_xcd / tn;
  if (rows_per_xcd < 1 || per_xcd % tn != 0) return t;
  t.a_part = id % tn;
  t.a_parts = tn;
  t.b_part = (id / tn) % rows_per_xcd;
  t.b_parts = rows_per_xcd;
  return t;
}

template <typename AT, int WC, int NKS, bool AG = false, int ENG = 0>
__global__ __launch_bounds__(512) void fwd1_rega_kernel(SplitStepArgs a, int tn, RegaAgArgs ag = {}) {
  extern __shared__ __attribute__((aligned(16))) char lds_dyn[];
  using G = RegaGeom<128, WC>;
  constexpr int MB = G::MB, NB = G::NB, WR = G::WR, BM = G::BM;
  // (a column tile's row tiles span XCDs: measured faster than an XCD-grouped grid, where every XCD reads all
  // of W1 -- profiles/wide_fused_head_r2.md)
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (id / tn) * BM, n0 = (id % tn) * 128;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave / WC, wc = wave % WC, fr = lane & 15, fg = lane >> 4;
  const int rw = m0 + 16 * MB * wr, cw = n0 + 16 * NB * wc;  // this wave's first row / column
  const int H = a.H, n = a.n, C = a.C;
  const bool z2 = a.z2part != nullptr || AG;
  gran_t ep_old = 0;  // the fused head's launch epoch (wide_head_ag step 0): one add per workgroup, now
  if (AG && threadIdx.x == 0) ep_old = ag_epoch_add(ag, n0 / 128);
  if (AG) ag_stamp(a, 0);
  const __amdgpu_buffer_rsrc_t rb1 = make_rsrc(a.b1), rw2 = make_rsrc(a.W2);
  float bb[MB][4], w2[MB][4];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int h = rw + 16 * mb + 4 * fg + i;
      bb[mb][i] = buf_load1<float>(rb1, h < H ? h * 4 : kOOB);
      w2[mb][i] = buf_load1<float>(rw2, (z2 && fr < C && h < H) ? (fr * H + h) * 4 : kOOB);
    }
  f32x4 acc[MB][NB];
  const AT* A = sizeof(AT) == 4 ? reinterpret_cast<const AT*>(a.W1) : reinterpret_cast<const AT*>(a.W1p);
  if constexpr (ENG == 1) {
    static_assert(WC == 1, "g64 engine: the 8 x 1 wave layout");
    g64_gemm_mainloop<AT, (NKS > 0 ? (NKS * 32 + 63) / 64 : 0)>(A, a.P, static_cast<const bf16*>(a.Xw), a.P, H, n, a.P, m0,
                                                               n0, lds_dyn, acc, g64_touch(a, id, gridDim.x, tn));
  } else {
    rega_gemm_mainloop<AT, 128, WC, NKS>(A, a.P, static_cast<const bf16*>(a.Xw), a.P, H, n, a.P, m0, n0, lds_dyn, acc);
  }
  if (AG) ag_stamp(a, 1);
  const __amdgpu_buffer_rsrc_t ra1 = make_rsrc(a.a1);
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = rw + 16 * mb + 4 * fg + i, col = cw + 16 * nb + fr;
        const float sv = sigm(acc[mb][nb][i] * a.xscale + bb[mb][i]);
        acc[mb][nb][i] = sv;
        if (!AG || ag.store_a1) st_f32(ra1, (row < H && col < n) ? (row * a.ld + col) * 4 : kOOB, sv);
      }
  if (!z2) return;
  // z2 partials on the f32 MFMA: step i of block mb takes B[k = fg][n = fr] = a1(row rw + 16 mb + 4 fg + i,
  // col fr) -- exactly accumulator element i -- and A[m = fr][k = fg] = W2[class fr][that row]; the WR row
  // waves are summed through LDS (every K-loop read of lds_dyn is done after the barrier)
  f32x4 z[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    z[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        z[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(w2[mb][i], acc[mb][nb][i], z[nb], 0, 0, 0);
  }
  if (AG && threadIdx.x == 0) ag_epoch_publish(ag, lds_dyn, ep_old);
  __syncthreads();
  f32x4* red = reinterpret_cast<f32x4*>(lds_dyn);  // [WR][WC][NB][64]
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) red[((wr * WC + wc) * NB + nb) * 64 + lane] = z[nb];
  __syncthreads();
  // the tile's 8 column blocks, one per wave
  static_assert(WC * NB == 8, "8 column blocks of 16");
  const int oc = wave / NB, onb = wave % NB;
  f32x4 sz = red[(oc * NB + onb) * 64 + lane];
#pragma unroll
  for (int r = 1; r < WR; ++r) sz += red[((r * WC + oc) * NB + onb) * 64 + lane];
  const int col = n0 + 16 * wave + fr;
  const int tile = m0 / BM;
  if constexpr (AG) {  // tagged granules for the fused head (hand-off 1)
    const unsigned ep = reinterpret_cast<const unsigned*>(lds_dyn + ag.ep_off)[0];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (col < n && 4 * fg + i < C) {
        const float zv = sz[i];  // (a scalar copy: see below)
        gran_store(ag.z2g + (size_t)(tile * 16 + 4 * fg + i) * a.ld + col, zv, ep);
      }
  } else {
    const __amdgpu_buffer_rsrc_t rz = make_rsrc(a.z2part);
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // (classes past C are zero: not stored, the head does not read them)
      // (the element is copied to a scalar first: hipcc (ROCm 7.2) lowered __builtin_bit_cast of the vector
      // element sz[i] to element 0 for every i -- all four z2 rows stored the same value)
      const float zv = sz[i];
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, zv), rz,
                                            (col < n && 4 * fg + i < C) ? ((tile * 16 + 4 * fg + i) * a.ld + col) * 4 : kOOB,
                                            0, 0);
    }
  }
  if constexpr (AG) {
    static_assert(MB == 1 && NB == 8, "all-gather head: 8 row waves of 16 rows x 128 columns");
    f32x4 a1v[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) a1v[nb] = acc[0][nb];
    ag_stamp(a, 2, true);
    wide_head_ag<128, 128, NB>(a, ag, a1v, lds_dyn, m0, n0, rw, cw, ag.tm, n0 / 128);
  }
}

// dW1 = dZ1 XT on the A-in-registers engine: dZ1 read as fp32 (AT = float; the head writes it instead of
// the three bf16 planes: 4 B per element stored and loaded instead of 6) or as its one bf16 plane (split1),
// with wgrad_glds_kernel's fused reg + SGD + plane-refresh epilogue; the dW2 / db2 roles ride along
// DSWZ (fp32, rega engine): dZ1 is read in the K loop's fragment order from the buffer the wide head wrote
// (SplitStepArgs::dz_swz == 2, rega_gemm.h dzr_off)
template <typename AT, int WC, int NKS, int ENG = 0, bool DSWZ = false>
__global__ __launch_bounds__(512) void wgrad_rega_kernel(SplitStepArgs a, int tn, int tbig, int t2) {
  extern __shared__ __attribute__((aligned(16))) char lds_dyn[];
  if ((int)blockIdx.x >= tbig) {
    wgrad_roles<0, 8>(a, (int)blockIdx.x - tbig, 0, t2, reinterpret_cast<float*>(lds_dyn),
                reinterpret_cast<uint32_t*>(lds_dyn + kWKS * 4 * 64 * sizeof(float)),
                reinterpret_cast<float*>(lds_dyn + kWKS * 4 * 64 * sizeof(float) + 16));  // (never fused: unused;
                                                                                            //  2 x kXpTile floats)
    return;
  }
  using G = RegaGeom<128, WC>;
  constexpr int MB = G::MB, NB = G::NB, BM = G::BM, NP = sizeof(AT) == 4 ? 3 : 1;
  const int id = xcd_remap(blockIdx.x, tbig);
  const int m0 = a.w1_row0 + (id / tn) * BM, n0 = (id % tn) * 128;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave / WC, wc = wave % WC, fr = lane & 15, fg = lane >> 4;
  const int rw = m0 + 16 * MB * wr, cw = n0 + 16 * NB * wc;
  const int M = a.w1_rows < 0 ? a.H : a.w1_row0 + a.w1_rows, P = a.P;
  const float reg = (float)a.reg, lr = (float)a.lr, xs = a.xscale;
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(a.W1), rb1 = make_rsrc(a.b1);
  W1Chunks<128, 128> wc1;  // (the epilogue: row-contiguous chunks through an LDS transpose)
  wc1.prefetch(a, m0, n0, M);
  const int perr = ag_err_load(a.ag_err);  // the step's forward timed out: no update
  f32x4 acc[MB][NB];
  // fp32 dZ1 split in registers (AT = float), or its one bf16 plane (split1)
  const AT* A = sizeof(AT) == 4 ? reinterpret_cast<const AT*>(a.dZ1) : reinterpret_cast<const AT*>(a.dZ1p);
  if constexpr (ENG == 1) {
    static_assert(WC == 1, "g64 engine: the 8 x 1 wave layout");
    g64_gemm_mainloop<AT, (NKS > 0 ? (NKS * 32 + 63) / 64 : 0)>(A, a.ld, static_cast<const bf16*>(a.XTw), a.ldxt, M,
                                                               P + a.bias_col, a.n, m0, n0, lds_dyn, acc,
                                                               g64_touch(a, id, tbig, tn));
  } else if constexpr (DSWZ) {
    static_assert(sizeof(AT) == 4, "fragment-ordered dZ1: fp32");
    rega_gemm_mainloop<AT, 128, WC, NKS, 0, true>(A, (a.ld + 31) / 32, static_cast<const bf16*>(a.XTw), a.ldxt, M,
                                                  P + a.bias_col, a.n, m0, n0, lds_dyn, acc);
  } else {
    rega_gemm_mainloop<AT, 128, WC, NKS>(A, a.ld, static_cast<const bf16*>(a.XTw), a.ldxt, M, P + a.bias_col, a.n, m0,
                                         n0, lds_dyn, acc);
  }
  wc1.stage(lds_dyn, acc, rw, cw, m0, n0, fg, fr);
  // the W1 planes (npw == npz); split3 w1_planes_lazy: none (the 128 x 128 forward reads fp32 W1)
  wc1.apply(a, lds_dyn, m0, n0, M, a.sgd && !poisoned(perr), (NP == 3 && a.w1_planes_lazy) ? 0 : NP);
  mark_status(a, perr);
}

template <auto Kern>
void set_lds_limit(int bytes) {
  static bool done = false;  // one attribute call per kernel instantiation
  if (!done) {
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(Kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  bytes));
    done = true;
  }
}

inline int cdiv(int a, int b) { return (a + b - 1) / b; }
inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
inline bool al4(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 3) == 0; }

constexpr int kBigMinH = 512;  // below this the wave-split-K kernels win (too few tiles to fill the chip)

// the wide (blocked-GEMM) weight-gradient engines apply: wide hidden layer, 16-byte aligned K-contiguous rows
bool big_wgrad_ok(const SplitStepArgs& a) {
  return a.H >= kBigMinH && a.n % 16 == 0 && a.ld % 8 == 0 && a.ldxt % 16 == 0 && al16(a.dZ1p) && al16(a.XT);
}
// the direct-to-LDS engine: bf16 copies present, rows a whole number of 16-byte chunks, 16-byte bases
bool glds_fwd_ok(const SplitStepArgs& a) {
  return a.H >= kBigMinH && a.Xw && a.P % 8 == 0 && al16(a.W1p) && al16(a.Xw);
}
bool glds_wgrad_ok(const SplitStepArgs& a) {
  return a.H >= kBigMinH && a.npw == a.npz && a.XTw && a.n % 8 == 0 && a.ld % 8 == 0 && a.ldxt % 8 == 0 && al16(a.dZ1p) &&
         al16(a.XTw) && a.P % 4 == 0 && al16(a.W1);  // (W1Chunks: 16-byte W1 rows chunks)
}

// the A-in-registers engine: 128 x 128 tiles only, and only when they still give ~200+ workgroups
bool rega_fwd_ok(const SplitStepArgs& a) {
  return glds_fwd_ok(a) && cdiv(a.H, 128) * cdiv(a.n, 128) >= 192 && a.P % 4 == 0 && al16(a.W1);
}

constexpr int kRegaWC = 1;  // wave layout of the A-in-registers kernels: 8 (rows) x 1 (bench/micro/rega_ablate.hip: WC = 2 splits every A value twice, +25 % at H = 4096)

template <typename AT, int NKS>
void launch_fwd1_rega_k(const SplitStepArgs& a, hipStream_t s) {
  constexpr int L = std::max({ra::lds_bytes<128>(), g64::lds_bytes<AT>(), 8 * 8 * 64 * 16});  // (z2 reduction scratch)
  const int grid = cdiv(a.H, 128) * cdiv(a.n, 128);
  if (a.wide_eng == 1) {
    set_lds_limit<fwd1_rega_kernel<AT, kRegaWC, NKS, false, 1>>(L);
    fwd1_rega_kernel<AT, kRegaWC, NKS, false, 1><<<grid, 512, L, s>>>(a, cdiv(a.n, 128));
  } else {
    set_lds_limit<fwd1_rega_kernel<AT, kRegaWC, NKS, false>>(L);
    fwd1_rega_kernel<AT, kRegaWC, NKS, false><<<grid, 512, L, s>>>(a, cdiv(a.n, 128));
  }
}

// the fused all-gather head: > 80 KB of LDS keeps it at one workgroup per CU (the hand-off's measured form)
template <typename AT, int NKS>
void launch_fwd1_rega_ag_k(const SplitStepArgs& a, RegaAgArgs g, hipStream_t s) {
  constexpr int L = wide_ag_launch_lds(
      std::max({ra::lds_bytes<128>(), g64::lds_bytes<AT>(), 8 * 8 * 64 * 16, wide_ag_lds_bytes<128, 128>()}));
  static_assert(L <= 160 * 1024, "fused wide head: LDS");
  g.ep_off = L - 16;
  g.tiling = 0;
  const int tn = cdiv(a.n, 128);
  if (a.wide_eng == 1) {
    set_lds_limit<fwd1_rega_kernel<AT, kRegaWC, NKS, true, 1>>(L);
    fwd1_rega_kernel<AT, kRegaWC, NKS, true, 1><<<g.tm * tn, 512, L, s>>>(a, tn, g);
  } else {
    set_lds_limit<fwd1_rega_kernel<AT, kRegaWC, NKS, true>>(L);
    fwd1_rega_kernel<AT, kRegaWC, NKS, true><<<g.tm * tn, 512, L, s>>>(a, tn, g);
  }
}

// K = P = 784 (MNIST) is 25 stages of 32: the fully unrolled K loop; anything else the runtime loop
template <typename AT>
void launch_fwd1_rega(const SplitStepArgs& a, hipStream_t s) {
  if (cdiv(a.P, ra::kBK) == 25) launch_fwd1_rega_k<AT, 25>(a, s);
  else launch_fwd1_rega_k<AT, 0>(a, s);
}

// the direct-to-LDS forward where the A-in-registers one does not apply (its 128 x 128 tiles would give < 192
// workgroups: H = 512-1024 at a per-GPU batch of 800): 64 x 64 tiles
template <int NP>
void launch_fwd1_glds(const SplitStepArgs& a, hipStream_t s) {
  constexpr int L = std::max(gl::lds_bytes<64, 64, NP>(), 4 * 2 * 2 * 64 * 16);  // (tile hook scratch)
  set_lds_limit<fwd1_glds_kernel<64, 64, NP>>(L);
  const int tn = cdiv(a.n, 64);
  fwd1_glds_kernel<64, 64, NP><<<cdiv(a.H, 64) * tn, 512, L, s>>>(a, tn);
}

// the A-in-registers dW1 (and the head writing fp32 dZ1 instead of its planes, split3): wide layers whose
// full 128 x 128 dW1 tiling gives ~200+ workgroups.  Decided on the whole layer (not the row range of a
// bucketed call) so the head and every wgrad call of a step agree on what dZ1 form exists.
bool rega_wgrad_ok(const SplitStepArgs& a) {
  return a.H >= kBigMinH && a.npw == a.npz && a.XTw && cdiv(a.H, 128) * cdiv(a.P + a.bias_col, 128) >= 192 &&
         a.P % 4 == 0 &&
         a.n % 8 == 0 && a.ld % 8 == 0 && a.ldxt % 8 == 0 && al16(a.XTw) && al16(a.W1) &&
         (a.npz == 3 ? (a.dZ1 != nullptr && al16(a.dZ1)) : al16(a.dZ1p));
}

template <typename AT, int NKS>
void launch_wgrad_rega_k(const SplitStepArgs& a, int t2, int tb, hipStream_t s) {
  const int rows = a.w1_rows < 0 ? a.H : a.w1_rows;
  const int tn = cdiv(a.P + a.bias_col, 128), tbig = cdiv(rows, 128) * tn;
  // (the K-loop ring, the epilogue's transposed 128 x (128 + 4) fp32 tile, the role workgroups' scratch)
  constexpr int L = std::max({ra::lds_bytes<128>(), g64::lds_bytes<AT>(), W1Chunks<128, 128>::kLdsBytes,
                              kWKS * 4 * 64 * (int)sizeof(float) + 16 + 2 * kXpTile * (int)sizeof(float)});
  if constexpr (sizeof(AT) == 4) {
    if (a.dz_swz == 2) {
      CME_REQUIRE(a.wide_eng == 0, "wgrad_rega: the fragment-ordered dZ1 is read by the A-in-registers engine");
      set_lds_limit<wgrad_rega_kernel<AT, kRegaWC, NKS, 0, true>>(L);
      wgrad_rega_kernel<AT, kRegaWC, NKS, 0, true><<<tbig + t2 + tb, 512, L, s>>>(a, tn, tbig, t2);
      return;
    }
  }
  CME_REQUIRE(a.dz_swz == 0, "wgrad_rega: fragment-ordered dZ1 with bf16 planes");
  if (a.wide_eng == 1) {
    set_lds_limit<wgrad_rega_kernel<AT, kRegaWC, NKS, 1>>(L);
    wgrad_rega_kernel<AT, kRegaWC, NKS, 1><<<tbig + t2 + tb, 512, L, s>>>(a, tn, tbig, t2);
  } else {
    set_lds_limit<wgrad_rega_kernel<AT, kRegaWC, NKS>>(L);
    wgrad_rega_kernel<AT, kRegaWC, NKS><<<tbig + t2 + tb, 512, L, s>>>(a, tn, tbig, t2);
  }
}

template <typename AT>
void launch_wgrad_rega(const SplitStepArgs& a, int t2, int tb, hipStream_t s) {
  if (cdiv(a.n, ra::kBK) == 25) launch_wgrad_rega_k<AT, 25>(a, t2, tb, s);
  else launch_wgrad_rega_k<AT, 0>(a, t2, tb, s);
}

// split-K dW1, second half: sum the ksplit partial slabs in slab order (deterministic), then the fused
// epilogue of wgrad_glds_kernel: reg + SGD + the W1 planes (or the gradient), db1 from the all-ones column.
template <int NPZ>
__global__ __launch_bounds__(256) void splitk_sgd_kernel(SplitStepArgs a) {
  const int M = a.w1_rows < 0 ? a.H - a.w1_row0 : a.w1_rows, P = a.P, W = P + a.bias_col;
  const int64_t total = (int64_t)M * W, slab = total;
  const float reg = (float)a.reg, lr = (float)a.lr, xs = a.xscale;
  const int perr = ag_err_load(a.ag_err);  // the step's forward timed out: no update
  const bool upd = a.sgd && !poisoned(perr);
  const size_t plane = (size_t)a.H * P;
  mark_status(a, perr);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    float v = a.kpart[e];
    for (int k = 1; k < a.wg_ksplit; ++k) v += a.kpart[k * slab + e];
    const int row = a.w1_row0 + (int)(e / W), col = (int)(e % W);
    if (col == P) {  // all-ones feature: db1 (no input scale, no regulariser)
      if (upd) a.b1[row] -= lr * v;
      else a.gb1[row] = v;
      continue;
    }
    const size_t idx = (size_t)row * P + col;
    const float wv = a.W1[idx], g = v * xs + reg * wv;
    if (upd) {
      const float nw = wv - lr * g;
      a.W1[idx] = nw;
      split_store<NPZ>(nw, static_cast<bf16*>(a.W1p), plane, idx);
    } else {
      a.gW1[idx] = g;
    }
  }
}

template <int NP>
void launch_wgrad_glds(const SplitStepArgs& a, int t2, int tb, hipStream_t s) {
  const int rows = a.w1_rows < 0 ? a.H : a.w1_rows;
  const int NW = a.P + a.bias_col;
  const int t128 = cdiv(rows, 128) * cdiv(NW, 128);
  const int tn64 = cdiv(NW, 64), t64 = cdiv(rows, 64) * tn64;
  constexpr int kRoleLds = kWKS * 4 * 64 * (int)sizeof(float) + 16;
  constexpr int L128 = std::max({gl::lds_bytes<128, 128, NP>(), W1Chunks<128, 128>::kLdsBytes, kRoleLds});
  constexpr int L64 = std::max({gl::lds_bytes<64, 64, NP>(), W1Chunks<64, 64>::kLdsBytes, kRoleLds});
  // split-K when the output tiles cannot fill the chip and K is long (the tensor-parallel shard at a large
  // global batch): K slices of whole 32-deep stages, the 128 x 128 tiles first (the data-parallel launch's
  // per-workgroup shape when 8 slices of K = 6400 give 200+ workgroups), else the 64 x 64 ones
  auto slices = [&](int tiles, int& kc) {
    if (!a.kpart || a.sgd == 2 || a.n < 2048) return 1;
    int ks = std::min(8, 256 / tiles);
    kc = cdiv(cdiv(a.n, ks), 32) * 32;
    ks = cdiv(a.n, kc);
    return (int64_t)ks * rows * NW <= a.kpart_cap ? ks : 1;
  };
  auto split_launch = [&](auto kern, int L, int tn, int tiles, int ks, int kc) {
    SplitStepArgs b = a;
    b.wg_ksplit = ks;
    b.wg_kchunk = kc;
    kern<<<tiles * ks + t2 + tb, 512, L, s>>>(b, tn, tiles * ks, t2);
    const int64_t total = (int64_t)rows * NW;
    splitk_sgd_kernel<NP><<<(unsigned)std::min<int64_t>(2048, (total + 255) / 256), 256, 0, s>>>(b);
  };
  int kc = a.n;
  if (t128 >= 192) {
    set_lds_limit<wgrad_glds_kernel<128, 128, NP>>(L128);
    wgrad_glds_kernel<128, 128, NP><<<t128 + t2 + tb, 512, L128, s>>>(a, cdiv(NW, 128), t128, t2);
  } else if (int ks = slices(t128, kc); ks > 1 && t128 * ks >= 192) {
    set_lds_limit<wgrad_glds_kernel<128, 128, NP>>(L128);
    split_launch(wgrad_glds_kernel<128, 128, NP>, L128, cdiv(NW, 128), t128, ks, kc);
  } else if (int ks64 = t64 < 128 ? slices(t64, kc) : 1; ks64 > 1) {
    set_lds_limit<wgrad_glds_kernel<64, 64, NP>>(L64);
    split_launch(wgrad_glds_kernel<64, 64, NP>, L64, tn64, t64, ks64, kc);
  } else {
    set_lds_limit<wgrad_glds_kernel<64, 64, NP>>(L64);
    wgrad_glds_kernel<64, 64, NP><<<t64 + t2 + tb, 512, L64, s>>>(a, tn64, t64, t2);
  }
}

}  // namespace

// The fp32 (split3) launches of the A-in-registers engine are compiled in their own translation unit,
// mlp_wide_f32.hip (this file again under CME_WIDE_F32_TU), with the machine scheduler's max-ILP strategy: its
// K loops (MFMA + the in-register split VALU) run 784-4096-10 fp32 2.2 us per step faster that way, while the same
// strategy makes the bf16 engines and the small-layer kernels of this file slower (profiles/r6/flags_split/).
namespace wide_f32 {
void fwd1_rega(const SplitStepArgs& a, hipStream_t s);
void fwd1_rega_ag(const SplitStepArgs& a, RegaAgArgs g, hipStream_t s);
void wgrad_rega(const SplitStepArgs& a, int t2, int tb, hipStream_t s);
}  // namespace wide_f32

#ifdef CME_WIDE_F32_TU
namespace wide_f32 {
void fwd1_rega(const SplitStepArgs& a, hipStream_t s) { launch_fwd1_rega<float>(a, s); }
void fwd1_rega_ag(const SplitStepArgs& a, RegaAgArgs g, hipStream_t s) {
  if (cdiv(a.P, ra::kBK) == 25) launch_fwd1_rega_ag_k<float, 25>(a, g, s);
  else launch_fwd1_rega_ag_k<float, 0>(a, g, s);
}
void wgrad_rega(const SplitStepArgs& a, int t2, int tb, hipStream_t s) { launch_wgrad_rega<float>(a, t2, tb, s); }
}  // namespace wide_f32
#else

// the wave-split-K dW1 reads fp32 dZ1 (split3, a_fp32, 16-byte rows)
bool small_wgrad_fp32_ok(const SplitStepArgs& a) {
  return a.npz == 3 && (a.a_fp32 & 2) && a.dZ1 != nullptr && al16(a.dZ1) && a.ld % 4 == 0;
}

// the wide form (SplitStepArgs::dz_swz == 2): the whole layer's dW1 on the A-in-registers engine reading fp32 dZ1, no
// fused exchange, db1 from the all-ones XT row
bool mlp_wgrad_dzr_ok(const SplitStepArgs& a) {
  return a.npz == 3 && a.xf_world == 0 && big_wgrad_ok(a) && rega_wgrad_ok(a) && a.wide_eng == 0 && a.bias_col &&
         a.w1_row0 == 0 && a.w1_rows < 0 && a.dZ1 != nullptr && al16(a.dZ1);
}

// the fragment-ordered fp32 dZ1 (SplitStepArgs::dz_swz): the wave-split-K dW1 GEMM over 16-byte pixel pairs whose
// waves start their K (= batch) ranges on 64-column pairs: an even number of 32-column chunks per wave (n = 257-512,
// 769-1024, ...)
bool mlp_wgrad_dz_swz_ok(const SplitStepArgs& a) {
  // (bias_col: db1 comes out of the dW1 GEMM; without the all-ones XT row a bias role would read dZ1 row-major)
  return a.H <= 128 && a.bias_col && small_wgrad_fp32_ok(a) && a.n % 16 == 0 && al16(a.XT) && a.ldxt % 16 == 0 &&
         a.ld % 8 == 0 && cdiv(cdiv(a.n, 32), kWKS) % 2 == 0;
}

// Decided on the whole step (not the row range of a bucketed call; the xGMI-fused launch always takes the
// wave-split-K kernel) so that the head and every wgrad call of a step agree on what dZ1 form exists.
bool mlp_split_wgrad_fp32_dz(const SplitStepArgs& a) {
  if (a.npz != 3) return false;
  const bool big = big_wgrad_ok(a) && a.xf_world == 0;
  // (wide: the A-in-registers dW1 always splits fp32 dZ1 -- profiles/wide_ag_ab_operand_forms_r3.jsonl)
  return big ? rega_wgrad_ok(a) : small_wgrad_fp32_ok(a);
}

bool mlp_split_fwd_fp32_w(const SplitStepArgs& a) { return a.npw == 3 && (a.a_fp32 & 1) && a.W1 != nullptr && al16(a.W1); }

// below kBigMinH every forward kernel (fwd1_split, fwd1_head(_ag)) takes fp32 W1 when
// mlp_split_fwd_fp32_w holds: nothing reads the W1 planes, so the weight update stops refreshing them
bool mlp_split_w1_planes_read(const SplitStepArgs& a) { return a.H >= kBigMinH || !mlp_split_fwd_fp32_w(a); }

int mlp_split_fwd1_z2_chunks(const SplitStepArgs& a) {
  if (!a.z2part || a.C > 16 || a.n <= 0 || !glds_fwd_ok(a)) return 0;
  return rega_fwd_ok(a) ? cdiv(a.H, 128) : cdiv(a.H, 64);  // the forward's tiles: rega 128 rows, glds 64
}

// the tile the fused head runs on: 128 (A-in-registers engine), 64 (the direct-to-LDS 64 x 64 tiling), 0 (none)
// (64 x 64: faster than forward + head_wide_kernel only without the a1 store -- 784-1024-10 bf16 25.33 -> 25.06 us,
// 784-512-10 f32 32.20 -> 31.13 us, profiles/wide_ag_ab_64_r2.jsonl; MlpStep.ag_tiles64 decides)
static int wide_ag_bm(const SplitStepArgs& a, int allow64) {
  if (rega_fwd_ok(a)) return 128;
  if (allow64 && glds_fwd_ok(a) && cdiv(a.H, 128) * cdiv(a.n, 128) < 192) return 64;
  return 0;
}

bool mlp_split_wide_fwd_reads_planes(const SplitStepArgs& a, int ag, int allow64) {
  if (a.npw != 3) return true;
  if (ag) return wide_ag_bm(a, allow64) != 128;  // 128: fwd1_rega_kernel (fp32 W1); 64: glds (planes)
  // mirrors mlp_split_fwd1's dispatch: rega (fp32 W1), glds (planes), the small kernels (fp32 W1 or planes)
  if (rega_fwd_ok(a)) return false;
  if (glds_fwd_ok(a)) return true;
  return !mlp_split_fwd_fp32_w(a);
}

bool mlp_split_wgrad_leaves_planes_stale(const SplitStepArgs& a) {
  return a.w1_planes_lazy && a.npw == 3 && a.npz == 3 && a.sgd && (a.wg_parts & 1) && a.w1_rows != 0 &&
         a.xf_world == 0 && big_wgrad_ok(a) && rega_wgrad_ok(a);
}

bool mlp_fwd1_wide_ag_ok(const SplitStepArgs& a, const HeadArgs& h, int allow64) {
  const int bm = wide_ag_bm(a, allow64);
  if (bm == 0 || a.n <= 0) return false;
  const int tm = cdiv(a.H, bm), tn = cdiv(a.n, bm);
  return a.z2part != nullptr && h.mode == HEAD_TRAIN && a.C >= 1 && a.C <= 16 && h.C == a.C && h.H == a.H &&
         h.n == a.n && h.W2 == a.W2 && tm >= bm / 16 && tm * tn <= device_cu_count() && h.dZ1_bf16 == nullptr &&
         (h.dZ1 || h.dZ1_planes) && h.D && h.labels && h.b2 && h.dw2part &&
         (int64_t)a.H * h.ldz * 4 < (int64_t)kOOB && (int64_t)h.npz * a.H * h.ldz * 2 < (int64_t)kOOB &&
         (int64_t)16 * tn * a.H * 4 < (int64_t)kOOB && (int64_t)16 * h.ldd * 4 < (int64_t)kOOB &&
         (int64_t)tm * 16 * a.ld * 4 < (int64_t)kOOB;
}

template <int NP>
void launch_fwd1_glds64_ag(const SplitStepArgs& a, RegaAgArgs g, hipStream_t s) {
  constexpr int L = wide_ag_launch_lds(std::max({gl::lds_bytes<64, 64, NP>(), 4 * 2 * 2 * 64 * 16, wide_ag_lds_bytes<64, 64>()}));
  set_lds_limit<fwd1_glds_kernel<64, 64, NP, true>>(L);
  g.ep_off = L - 16;
  g.tiling = 1;
  const int tn = cdiv(a.n, 64);
  fwd1_glds_kernel<64, 64, NP, true><<<g.tm * tn, 512, L, s>>>(a, tn, g);
}

int mlp_fwd1_wide_ag(const SplitStepArgs& a, const HeadArgs& h, unsigned long long* counters, int max_tiles,
                     unsigned long long* gran, int64_t gran_count, int* err, int store_a1, int allow64,
                     hipStream_t s) {
  CME_REQUIRE(mlp_fwd1_wide_ag_ok(a, h, allow64), "fwd1_wide_ag: wide split path (128 x 128 A-in-registers or 64 x 64 "
                                         "direct-to-LDS tiles, grid <= CU count), train-mode head, C <= 16");
  CME_REQUIRE((int64_t)a.H * a.P * 2 * a.npw < (int64_t)kOOB && (int64_t)a.n * a.P * 2 < (int64_t)kOOB,
              "fwd1_wide_ag: operand too large for 32-bit buffer offsets");
  const int bm = wide_ag_bm(a, allow64);
  CME_REQUIRE(counters && err && cdiv(a.n, bm) <= max_tiles, "fwd1_wide_ag: counter array too small");
  RegaAgArgs g;
  g.h = h;
  // [2][max_tiles][kRegaAgCounterStride]: the 64 x 64 tiling's counters after the 128 x 128 tiling's
  g.counters = counters + (bm == 64 ? (size_t)max_tiles * kRegaAgCounterStride : 0);
  g.err = err;
  g.store_a1 = store_a1;
  g.tm = cdiv(a.H, bm);
  // granules: the z2 partials [tm][16][ld], then D [16][ld]
  CME_REQUIRE(gran && (int64_t)(g.tm * 16 + 16) * a.ld <= gran_count, "fwd1_wide_ag: granule buffer too small");
  g.z2g = gran;
  g.dg = gran + (size_t)g.tm * 16 * a.ld;
  if (bm == 128) {
    const bool k25 = cdiv(a.P, ra::kBK) == 25;
    if (a.npw == 3) {
      wide_f32::fwd1_rega_ag(a, g, s);
    } else {
      if (k25) launch_fwd1_rega_ag_k<bf16, 25>(a, g, s);
      else launch_fwd1_rega_ag_k<bf16, 0>(a, g, s);
    }
  } else if (a.npw == 3) {
    launch_fwd1_glds64_ag<3>(a, g, s);
  } else {
    launch_fwd1_glds64_ag<1>(a, g, s);
  }
  CME_LAUNCH_CHECK(s);
  return bm;
}

void mlp_split_fwd1(const SplitStepArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  CME_REQUIRE((int64_t)a.H * a.P * 2 * a.npw < (int64_t)kOOB && (int64_t)a.n * a.P * 2 < (int64_t)kOOB,
              "split path: operand too large for 32-bit buffer offsets");
  CME_REQUIRE(a.ld >= a.n, "split path: ld >= n");
  if (rega_fwd_ok(a)) {
    if (a.npw == 3) wide_f32::fwd1_rega(a, s);
    else launch_fwd1_rega<bf16>(a, s);
    CME_LAUNCH_CHECK(s);
    return;
  }
  if (glds_fwd_ok(a)) {
    if (a.npw == 3) launch_fwd1_glds<3>(a, s);
    else launch_fwd1_glds<1>(a, s);
    CME_LAUNCH_CHECK(s);
    return;
  }
  const int tn = cdiv(a.n, 16 * kF1NB), tm = cdiv(a.H, 16 * kF1MB);
  const bool af = mlp_split_fwd_fp32_w(a);
  const bool vec = al4(a.X) && al16(af ? (const void*)a.W1 : a.W1p) && a.P % 8 == 0;
  const dim3 grid(tm * tn);
#define CME_F1(np, af)                                                                     \
  if (vec) fwd1_split_kernel<np, 1, af><<<grid, 64 * kF1KS, 0, s>>>(a, tn);               \
  else fwd1_split_kernel<np, 0, af><<<grid, 64 * kF1KS, 0, s>>>(a, tn);
  if (af) { CME_F1(3, true) } else if (a.npw == 3) { CME_F1(3, false) } else { CME_F1(1, false) }
#undef CME_F1
  CME_LAUNCH_CHECK(s);
}

void mlp_split_wgrad(const SplitStepArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  CME_REQUIRE((int64_t)a.H * a.ld * 2 * a.npz < (int64_t)kOOB && (int64_t)a.P * a.ldxt < (int64_t)kOOB,
              "split path: operand too large for 32-bit buffer offsets");
  CME_REQUIRE(a.w1_row0 >= 0 && (a.w1_rows < 0 || a.w1_row0 + a.w1_rows <= a.H), "wgrad: bad dW1 row range");
  const bool fused = a.xf_world > 0;
  const bool big = big_wgrad_ok(a) && !fused;
  const bool do_w1 = (a.wg_parts & 1) && a.w1_rows != 0, do_roles = (a.wg_parts & 2) != 0;
  if (big && do_w1) {  // dW1 as a blocked GEMM; the dW2 / db2 roles ride in the same launch as extra
    // workgroups: one launch and its boundary fewer, and they run on the CUs the dW1 tiles leave idle
    const int t2f = do_roles ? cdiv(a.H, 16) : 0;
    const int tbf = do_roles ? cdiv((a.bias_col ? 0 : a.H) + a.C, kWKS) : 0;
    const SplitStepArgs& c = a;
    if (rega_wgrad_ok(c)) {
      if (c.npz == 3) wide_f32::wgrad_rega(c, t2f, tbf, s);
      else launch_wgrad_rega<bf16>(c, t2f, tbf, s);
      CME_LAUNCH_CHECK(s);
      return;
    }
    CME_REQUIRE(c.dz_swz == 0, "wgrad: fragment-ordered dZ1 outside the A-in-registers engine");
    if (glds_wgrad_ok(c)) {
      if (c.npz == 3) launch_wgrad_glds<3>(c, t2f, tbf, s);
      else launch_wgrad_glds<1>(c, t2f, tbf, s);
      CME_LAUNCH_CHECK(s);
      return;
    }
    // (no direct-to-LDS copies: the wave-split-K kernel below)
  }
  const int w1rows = a.w1_rows < 0 ? a.H : a.w1_rows;
  const int t1n = cdiv(a.P + a.bias_col, 16 * kWNB), t1 = do_w1 ? cdiv(w1rows, 16 * kWMB) * t1n : 0;
  const int t2 = do_roles ? cdiv(a.H, 16) : 0;
  if (fused)
    CME_REQUIRE(do_w1 && do_roles && a.bias_col && a.w1_row0 == 0 && a.w1_rows < 0 && a.C <= 16 &&
                    a.xf_world <= 8 && t1 + t2 + 1 <= mlp_split_fused_tiles(a.P, a.H, 1 << 30),
                "wgrad: fused all-reduce needs the whole small-layer step with the all-ones XT feature");
  // fused mode: db2 is one role workgroup of its own (exchange tile t1 + t2)
  const int tb = !do_roles ? 0 : fused ? 1 : cdiv((a.bias_col ? 0 : a.H) + a.C, kWKS);
  if (t1 + t2 + tb == 0) {
    CME_LAUNCH_CHECK(s);
    return;
  }
  // dZ1 planes: 16-byte vectors when n % 8 == 0, 8-byte halves when n % 4 == 0; XT bytes need 4-byte rows
  // (fp32 dZ1: 2 x 16-byte vectors when n % 8 == 0, else element loads -- mma_tile.h VA)
  const bool af = small_wgrad_fp32_ok(a);
  const bool base_ok = al16(af ? (const void*)a.dZ1 : a.dZ1p) && al4(a.XT) && a.ld % 8 == 0 && a.ldxt % 4 == 0;
  // (3: the XT bytes as 16-byte loads over chunk pairs, mma_tile.h: 16-byte XT rows, n % 16 == 0)
  const bool pairs = al16(a.XT) && a.ldxt % 16 == 0 && a.n % 16 == 0;
  const int vec = !base_ok ? 0 : (a.n % 8 == 0 ? (pairs ? 3 : 1) : (a.n % 4 == 0 ? 2 : 0));
  SplitStepArgs b = a;
  b.w1_planes = mlp_split_w1_planes_read(a) ? 1 : 0;
  // the XCD-row placement only for the whole layer's dW1 (a bucketed row range keeps the plain order)
  // (the forward's packed form, xcd_rows == 2, is the forward's alone: 2 x 25 dW1 tiles would not fit 4 XCDs)
  b.xcd_rows = a.xcd_rows && do_w1 && a.w1_row0 == 0 && a.w1_rows < 0 && cdiv(a.H, 16 * kWMB) <= 8 ? 1 : 0;
  b.pf_wgs = b.xcd_rows ? a.pf_wgs : 0;
  const dim3 grid((b.xcd_rows ? 8 * t1n : t1) + t2 + tb + 8 * b.pf_wgs);  // (prefetch workgroups last)
  const int fu = !fused ? 0 : a.xf_push ? 2 : 1;
#define CME_WG3(npz, af, FU)                                                                    \
  if (vec == 3) wgrad_split_kernel<npz, 3, af, FU><<<grid, kWT, 0, s>>>(b, t1, t1n, t2);      \
  else if (vec == 1) wgrad_split_kernel<npz, 1, af, FU><<<grid, kWT, 0, s>>>(b, t1, t1n, t2); \
  else if (vec == 2) wgrad_split_kernel<npz, 2, af, FU><<<grid, kWT, 0, s>>>(b, t1, t1n, t2); \
  else wgrad_split_kernel<npz, 0, af, FU><<<grid, kWT, 0, s>>>(b, t1, t1n, t2);
#define CME_WG(npz, af)     \
  if (fu == 2) {            \
    CME_WG3(npz, af, 2)     \
  } else if (fu == 1) {     \
    CME_WG3(npz, af, 1)     \
  } else {                  \
    CME_WG3(npz, af, 0)     \
  }
  CME_REQUIRE(!a.dz_swz || (af && vec == 3 && do_w1 && mlp_wgrad_dz_swz_ok(a)),
              "wgrad: the fragment-ordered dZ1 needs fp32 dZ1, 16-byte pixel pairs and pair-aligned K ranges");
  if (a.xp_dbg) {  // diagnostics (bench/kbench.py xp rows): the push form's two headline shapes only
    CME_REQUIRE(fu == 2 && vec == 3 && (a.dz_swz || af || a.npz == 3),
                "wgrad: xp_dbg ablations exist for the push form at 16-byte pixel pairs with fp32 dZ1 (fragment-ordered "
                "or row-major: n = 800) or the three dZ1 planes (n = 100)");
    if (a.dz_swz) wgrad_split_kernel<3, 3, true, 2, true, true><<<grid, kWT, 0, s>>>(b, t1, t1n, t2);
    else if (af) wgrad_split_kernel<3, 3, true, 2, false, true><<<grid, kWT, 0, s>>>(b, t1, t1n, t2);
    else wgrad_split_kernel<3, 3, false, 2, false, true><<<grid, kWT, 0, s>>>(b, t1, t1n, t2);
  } else if (a.dz_swz) {
    if (fu == 2) wgrad_split_kernel<3, 3, true, 2, true><<<grid, kWT, 0, s>>>(b, t1, t1n, t2);
    else if (fu == 1) wgrad_split_kernel<3, 3, true, 1, true><<<grid, kWT, 0, s>>>(b, t1, t1n, t2);
    else wgrad_split_kernel<3, 3, true, 0, true><<<grid, kWT, 0, s>>>(b, t1, t1n, t2);
  } else if (af) { CME_WG(3, true) } else if (a.npz == 3) { CME_WG(3, false) } else { CME_WG(1, false) }
#undef CME_WG
#undef CME_WG3
  CME_LAUNCH_CHECK(s);
}

bool mlp_split_xcd_rows_packed_ok(const SplitStepArgs& a) {
  const int tm = cdiv(a.H, 16), tn = cdiv(a.n, 32);
  return mlp_split_xcd_rows_ok(a) && tm > 4 && tm <= 8 && cdiv(tm, 4) * tn <= device_cu_count() / 8;
}

bool mlp_split_xcd_rows_ok(const SplitStepArgs& a) {
  return a.H <= 16 * 8 && a.n > 0 && cdiv(a.n, 32) <= device_cu_count() / 8;
}

int mlp_split_fused_tiles(int P, int H, int cap) {
  // dW1 tiles, dW2 tiles, the db2 workgroup
  const int t = cdiv(P + 1, 16 * kWNB) * cdiv(H, 16 * kWMB) + cdiv(H, 16) + 1;
  return t <= cap ? t : -1;
}

int64_t mlp_split_w1s_floats(int H, int P) { return (int64_t)cdiv(H, 16) * 16 * cdiv(P, 64) * 64; }

void mlp_split_w1s_refresh(const float* W1, float* W1s, int H, int P, hipStream_t s) {
  const int64_t total = mlp_split_w1s_floats(H, P);
  const int grid = (int)std::min<int64_t>(2048, (total + 255) / 256);
  w1s_kernel<<<grid, 256, 0, s>>>(W1, W1s, H, P, total);
  CME_LAUNCH_CHECK(s);
}

void mlp_split_planes(const float* W, void* planes, int64_t n, int np, hipStream_t s) {
  if (n <= 0) return;
  const int grid = (int)std::min<int64_t>(2048, (n + 255) / 256);
  if (np == 3) planes_kernel<3><<<grid, 256, 0, s>>>(W, (bf16*)planes, n);
  else planes_kernel<1><<<grid, 256, 0, s>>>(W, (bf16*)planes, n);
  CME_LAUNCH_CHECK(s);
}

void mlp_split_sgd(float* params, const float* grads, int64_t count, double lr, void* W1p, int64_t w1_count,
                   int npw, hipStream_t s, const float* status) {
  if (count <= 0) return;
  const int grid = (int)std::min<int64_t>(2048, (count + 255) / 256);
  if (npw == 3)
    sgd_planes_kernel<3><<<grid, 256, 0, s>>>(params, grads, count, (float)lr, (bf16*)W1p, w1_count, status);
  else
    sgd_planes_kernel<1><<<grid, 256, 0, s>>>(params, grads, count, (float)lr, (bf16*)W1p, w1_count, status);
  CME_LAUNCH_CHECK(s);
}

#endif  // CME_WIDE_F32_TU

}  // namespace cme
