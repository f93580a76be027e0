// The XCD-local step pipeline (H <= 128, split3, one process): every step of a native step-loop plan in ONE
// persistent launch, with no grid-wide seam anywhere.
//
// The two-launch step (forward + head, then weight gradient) pays at both kernel boundaries of every step: the XCDs
// start a launch 0.6-1.5 us apart and every z2 all-gather waits for the last one (profiles/r5/stamps_fha_per_xcd.jsonl),
// and whatever the previous launch WROTE -- the updated W1, dZ1, the dW2 partials -- is read back at the die-level
// cache's rate, 2.44 us against 0.92 us for an L2-resident 2 MiB (docs/PERFORMANCE.md "Data written by one kernel is
// cold for the next").  Under the XCD-row placement, row tile rt of W1 is both forward-read and updated on XCD rt,
// dZ1 rows rt are written and read there, and so are W2[:, rt rows] and their dW2 partials.  The only cross-XCD
// dependency of a step is the z2 all-gather of the head, already an in-launch hand-off.  So here:
//
//   * every workgroup reads its XCD from HW_REG_XCC_ID and takes a ticket on that XCD's counter: row tile rt = XCD,
//     slot j = ticket (placement decides only which XCD serves which row tile: every hand-off below is between
//     workgroups that read the same XCC id, i.e. that share one L2);
//   * slot j < nw is a worker: the forward + head of tile (rt, column tile j) -- fha_body, the two-launch forward's
//     own body, in its PS form: z2 partials out as data-tagged granules (tag = the plan's step number, slab by step
//     parity), the all-gather, softmax, D, the dW2 partials and dZ1 -- then, after the XCD's first barrier, the dW1
//     tile (rt, feature tile j) over the whole batch with the fused reg + SGD update of W1 / W1s / b1 (EpiW1, the
//     two-launch epilogue);
//   * slot nw is the XCD's role workgroup: after the first barrier it sums the dW2 partials of W2[:, rt rows] (EpiW2)
//     and reduces D into db2 -- redundantly on every XCD, in the same order, into that XCD's own copy of b2 (XCD 0
//     also writes the master b2 at the plan's last step);
//   * the other slots idle.  (Extra workgroups pulling the pixels each XCD reads next into its L2 -- this step's XT,
//     the next step's X -- measured slower, +1.5 us per step, and so did the workers' own LDS-DMA pull during the z2
//     wait and an LDS-DMA of the dW1 tile's pixels ahead of its GEMM (the DMAs share the in-order vmcnt with the
//     critical loads): profiles/r6/xstep_ab_r6b.jsonl, xstep_ab_r6c_prefetch_rejected.jsonl, xpf_rejected/.)
//
// Synchronisation is XCD-local (XsBar), in four forms (XStepPlan::bar; the default, 3, has no full barrier left):
// each participant drains its stores (s_waitcnt vmcnt(0) + workgroup barrier) and signals on its XCD's flag line (one
// 128-byte line, a plain-store tag per slot) or counter; in form 3 each dW1 wave waits only for the column tiles its
// K range reads (EpiW1Gate) and each forward wave of the next step only for the dW1 tiles its K range reads (fha_body
// PsGate; its wave 7, which has no K range, waits for all of them and the role and stages b1 / W2 / b2).  Every read
// of data another workgroup of the launch wrote goes through sc1 (L1-bypassing, L2-served) loads, so a CU never reuses
// a stale L1 line, and the producer's plain stores stay in the XCD's L2 (bench/micro/xcd_barrier.hip: the same-XCD
// read-back checked word by word, and priced, profiles/r6/xcd_barrier_micro*.jsonl).  Arithmetic and summation
// orders are those of the two-launch step, so the parameters are bitwise equal to it (tests/test_gpu_xstep.py).
// Walking step at n = 800: 9.4-9.5 us against the two-launch loop's 14.0 (profiles/r6/flags/, docs/ROUND6_STATUS.md);
// n = 100 (the row-major form, RM below): 8.90 us against 12.33 (profiles/r6/rm_form/).
//
// Failure semantics: a z2 hand-off wait that outlasts SplitStepArgs::ag_wait_us sets *err and makes its workgroup
// arrive "bad" at the first barrier; every XCD's workgroup of that column tile waits for the same missing granule,
// so every XCD stops there and the step applies nothing (the launch ends; the steps before it stay applied).  A
// barrier wait that times out (a workgroup that never arrives) sets *err and stops the launch.
// Reference: the hot loop of fpcode/neural_network.cpp:449-555 (forward/backward :281-394) -- here one launch.
#include "mlp_split.h"
#include "mlp_kernels.h"

#include "fha_body.h"
#include "granule.h"
#include "l2_touch.h"
#include "mma_tile.h"
#include "wgrad_epi.h"

namespace cme {

namespace {

using bf16 = __hip_bfloat16;
using namespace wg;

constexpr int kXsWgsPerXcd = 32;                 // 256 CUs / 8 XCDs: one workgroup per CU
constexpr unsigned long long kXsBad = 1ull << 40;  // a barrier arrival that stops the XCD (added to the count)
constexpr int kXsCols = 32;                      // the forward's column tile (fha_body)

inline int xs_cdiv(int a, int b) { return (a + b - 1) / b; }

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 15u;
}

// control words: [2 banks][8 XCDs][64] uint64 -- ticket at [0], barrier counter at [32] (separate 256-byte lines)
__device__ __forceinline__ unsigned long long* xs_ticket(unsigned long long* ctl, int bank, int x) {
  return ctl + ((size_t)bank * 8 + x) * 64;
}
__device__ __forceinline__ unsigned long long* xs_counter(unsigned long long* ctl, int bank, int x) {
  return ctl + ((size_t)bank * 8 + x) * 64 + 32;
}
// ... then [8 XCDs][16] uint64: one 128-byte flag line per XCD (XsBar<1>), never reset
__device__ __forceinline__ unsigned* xs_flags(unsigned long long* ctl, int x) {
  return reinterpret_cast<unsigned*>(ctl + 2 * 8 * 64 + (size_t)x * 16);
}

// The XCD-local barriers.  Every participant first drains its stores (s_waitcnt vmcnt(0) in every wave, then a
// workgroup barrier); lane 0 then signals and wave 0 waits; the other waves wait at a workgroup barrier.  sync(q, bad)
// is the plan's q-th barrier (two per step: q = 2 s + b); false (block-uniform) when the XCD must stop -- a bad
// arrival (a timed-out z2 hand-off upstream) or a wait past `limit_us` (then *err is set and the stop is signalled
// to every other waiter).
//
// BAR 0: one monotonic 64-bit counter per XCD (ctl bank launch & 1), an agent-scope atomic add per arrival, lane 0
//        polling it with sc1 loads (bench/micro/xcd_barrier.hip mode 2: 0.64 us from arrival to release); a stop
//        adds kXsBad.
// BAR 1: a FLAG LINE per XCD: one 32-bit word per participant in a single 128-byte line, written with a PLAIN
//        store -- the line stays in this XCD's L2, no trip to the memory-side atomic unit -- holding the barrier's tag
//        2 (ep0 + s) + b (tags only grow over the buffer's life, so nothing is ever reset); lanes 0-31 of wave 0 poll
//        the whole line with sc1 (L2-served) loads.  Word 31 is the stop word: launch + 1 when this launch stopped.
//        Valid because every participant of a line is on the XCD whose L2 holds it (they all read the same XCC id).
template <int BAR>
struct XsBar {
  unsigned long long* cnt;  // BAR 0
  unsigned* line;           // BAR 1: 32 words
  unsigned long long np;    // participants
  unsigned ep0, stop_tag;   // BAR 1: the first step's granule tag, this launch's stop value
  int slot;
  int* err;
  uint32_t limit_us;
  int* s_stop;
  __device__ unsigned tag_of(int q) const { return 2u * (ep0 + (unsigned)(q >> 1)) + (unsigned)(q & 1); }
  // BAR 1: this workgroup's stores drained (every wave), then lane 0 publishes its flag (and the stop word first when
  // its step is bad).  Returns after the workgroup barrier that follows the drain: the flag may still be in flight.
  __device__ void arrive(int q, bool bad) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      if (bad) line[31] = stop_tag;
      line[slot] = tag_of(q);
    }
  }
  // BAR 1, one WAVE (all its lanes): wait until the flags of participants [lo, hi) carry barrier q's tag.  False when
  // the launch stops (the stop word, or a wait past limit_us: then *err is set and the stop word written); *s_stop is
  // then set for the workgroup (read after its next workgroup barrier).
  __device__ bool poll(int q, int lo, int hi) {
    const int l = threadIdx.x & 63;
    const unsigned tag = tag_of(q);
    const __amdgpu_buffer_rsrc_t rl = make_rsrc(line);
    const uint64_t limit = (uint64_t)limit_us * kTicksPerUs;
    uint64_t t0 = 0;
    for (uint32_t pass = 1;; ++pass) {
      const unsigned v = __builtin_amdgcn_raw_buffer_load_b32(rl, l < 32 ? l * 4 : kOOB, 0, kSc1);
      if (__any(l == 31 && v == stop_tag)) {
        if (l == 0) *s_stop = 1;
        return false;
      }
      if (__all(l < lo || l >= hi || v - tag < 0x80000000u)) return true;  // (wrap-safe v >= tag)
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
  // the whole barrier: arrive, wave 0 waits for every participant, the workgroup joins it
  __device__ bool sync(int q, bool bad) {
    const int t = threadIdx.x;
    if constexpr (BAR == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const uint64_t limit = (uint64_t)limit_us * kTicksPerUs;
      if (t == 0) {
        const unsigned long long target = (unsigned long long)(q + 1) * np;
        __hip_atomic_fetch_add(cnt, bad ? 1ull + kXsBad : 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint64_t t0 = 0;
        for (uint32_t pass = 1;; ++pass) {
          const unsigned long long v = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (v >= kXsBad) {
            *s_stop = 1;
            break;
          }
          if (v >= target) break;
          if (pass == 1) t0 = wall_ticks();
          else if ((pass & 7) == 0 && wall_ticks() - t0 > limit) {
            atomicExch(err, 1);
            __hip_atomic_fetch_add(cnt, kXsBad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *s_stop = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
    } else {
      arrive(q, bad);
      if (t < 64) poll(q, 0, (int)np);
    }
    __syncthreads();
    return *s_stop == 0;
  }
};

// FG (fine-grained first barrier, BAR 1): the dW1 tile's epilogue, gated.  Each wave of the tile waits only for the
// forward + head workgroups whose dZ1 column tiles its K range reads (samples [kbeg, kend) = column tiles
// [kbeg / 32, ceil(kend / 32))), instead of the whole XCD; a wave that sees the launch stop marks the workgroup and
// the update is then not applied (the K loop's reduction barrier orders that mark before the epilogue).
struct EpiW1Gate : EpiW1 {
  XsBar<1>* bar;
  int q, tn;
  const int* s_stop;
  __device__ void before_kloop(int kbeg, int kend) {
    if (kend > kbeg) bar->poll(q, kbeg / kXsCols, min(tn, (kend + kXsCols - 1) / kXsCols));
  }
  __device__ __forceinline__ void operator()(int qq, int row, int col, float v) {
    if (!*s_stop) EpiW1::operator()(qq, row, col, v);
  }
};

// The samples of a run_steps plan's steps: consecutive global batches of B from gstart0, wrapping to 0 when one
// would pass N_end (MlpStep::run_steps), this rank's shard at +shard_off.  off() is the current step's first sample,
// next() the following step's; advance() moves on by one step.
struct XsWalk {
  int64_t gs;
  const XStepPlan& p;
  __device__ explicit XsWalk(const XStepPlan& q) : gs(q.gstart0 + q.B > q.N_end ? 0 : q.gstart0), p(q) {}
  __device__ int64_t off() const { return gs + p.shard_off; }
  __device__ int64_t next() const { return (gs + 2 * p.B > p.N_end ? 0 : gs + p.B) + p.shard_off; }
  __device__ void advance() { gs = gs + 2 * p.B > p.N_end ? 0 : gs + p.B; }
};

// FG: 0 two full XCD barriers per step; 1 the first fine-grained (EpiW1Gate); 2 both (the forward's waves wait for
// their own dW1 tiles: fha_body's PsGate) -- no full barrier left, only flags.
// DIAG: the diagnostics instantiation that honours the stamp buffers (XStepPlan::stamps, SplitStepArgs::stamps,
// HeadArgs::stamps) and the hand-off test hook (SplitStepArgs::ag_test_skip); the production one has none of their
// branches (dropping the stamps' took the walking step 9.86 -> 9.55 us, profiles/r6/xstep_ab_r6k_diag_templated.jsonl) (a runtime diagnostics branch in a production
// kernel cost a launch 0.8 us in round 5, profiles/r5/regression_bisect.md).
// RM: the operand form.  0: the fragment-ordered pixels and dZ1 (steps on the 16-sample grid, n % 16 == 0, n >= 257);
// 1 / 2 / 3: the row-major form for every other step -- the forward reads the pixels row-major (fha_body SWZ = 1),
// the head writes fp32 dZ1 row-major and the dW1 tile reads it with sc1 loads, 2 x 16-byte vectors (RM 1, n % 8 == 0)
// or 16-byte pixel pairs (RM 3: a plan on the 16-sample grid, n % 16 == 0) -- the two-launch step's own forms for such
// a step (mlp_split_wgrad vec 1 / 3) -- or, n % 4 == 0, 2 x 16-byte vectors with the tail past n zeroed in registers
// (RM 4: the same MFMA operands as the two-launch step's element loads, vec 2; n = 100 walking step 9.25 -> 8.90 us,
// profiles/r6/rm_form/), so the bits are its bits.
template <int BAR, int FG, bool DIAG = false, int HK = 0, int RM = 0>
__global__ __launch_bounds__(512) void xstep_kernel(SplitStepArgs a, HeadArgs h, XStepPlan p, int tm, int tn,
                                                    int t1n) {
  static_assert(FG == 0 || BAR == 1, "the fine-grained barriers need the flag line");
  static_assert(RM == 0 || (BAR == 1 && FG == 2), "the row-major form: barrier form 3");
  constexpr int kSwz = RM == 0 ? 7 : 1;  // fha_body: fragment-ordered W1 (+ pixels and dZ1 in form 0)
  __shared__ __attribute__((aligned(16))) float red[8 * 1 * 2 * 4 * 64];  // both GEMM tiles' K reductions
  __shared__ int s_slot, s_stop;
  __shared__ unsigned s_x;
  const int t = threadIdx.x;
  const int bank = (int)(p.launch & 1u);
  if (t == 0) {
    const unsigned x = xcc_id();
    int slot = -1;
    if (x < 8) {
      slot = (int)__hip_atomic_fetch_add(xs_ticket(p.ctl, bank, (int)x), 1ull, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
      if (slot == 0) {  // the other bank, for the next launch (the previous launch that used it has ended)
        __hip_atomic_store(xs_ticket(p.ctl, bank ^ 1, (int)x), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(xs_counter(p.ctl, bank ^ 1, (int)x), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    s_x = x;
    s_slot = slot;
    s_stop = 0;
  }
  __syncthreads();
  const int x = (int)s_x, slot = s_slot;
  if (x >= tm || slot < 0 || slot > p.nw + p.npf) return;  // (uniform) XCDs past the last row tile, spare CUs
  const uint32_t limit_us = (uint32_t)a.ag_wait_us;
  // barrier participants: the workers + the role
  XsBar<BAR> bar{xs_counter(p.ctl, bank, x), xs_flags(p.ctl, x), (unsigned long long)p.nw + 1, p.ep0, p.launch + 1u,
                 slot, p.err, limit_us, &s_stop};
  const int n = a.n, ld = a.ld;
  const float reg = (float)a.reg, lr = (float)a.lr;
  unsigned long long* st = DIAG ? p.stamps : nullptr;  // diagnostics: [step][8][32][4]
  auto stamp = [&](int s, int i) {
    if (st && t == 0 && s < p.stamp_steps)
      st[(((size_t)s * 8 + x) * kXsWgsPerXcd + slot) * 4 + i] = __builtin_amdgcn_s_memrealtime();
  };

  if (slot > p.nw) {  // ---- prefetch (BAR 1): the pixels this XCD reads next, pulled into its L2 by idle CUs
    if constexpr (BAR == 1 && FG == 0) {
      // at the start of step s (the flag line says the previous step's second barrier is complete): this step's XT
      // (the dW1 tiles read it after the first barrier) and the next step's fragment-ordered X (the next forward)
      const int part = slot - p.nw - 1;
      const unsigned* line = xs_flags(p.ctl, x);
      XsWalk w(p);
      for (int s = 0; s < p.count; ++s, w.advance()) {
        if (s > 0 && t < 64) {
          const unsigned tag = 2u * (p.ep0 + (unsigned)(s - 1)) + 1u, stop = p.launch + 1u;
          const __amdgpu_buffer_rsrc_t rl = make_rsrc(line);
          const uint64_t t0 = wall_ticks();
          for (;;) {
            const unsigned v = __builtin_amdgcn_raw_buffer_load_b32(rl, t < 32 ? t * 4 : kOOB, 0, kSc1);
            if (__any(t == 31 && v == stop) || wall_ticks() - t0 > (uint64_t)limit_us * kTicksPerUs) {
              if (t == 0) s_stop = 1;
              break;
            }
            if (__all(t > p.nw || v - tag < 0x80000000u)) break;
            __builtin_amdgcn_s_sleep(4);
          }
        }
        __syncthreads();
        if (s_stop) return;
        l2_touch(p.XT0, w.off(), a.P + a.bias_col, a.ldxt, n, part, p.npf, reinterpret_cast<char*>(red));
        if (s + 1 < p.count)
          l2_touch(p.Xs0, w.next() / 16 * p.xs_tile, 1, 0, (int64_t)((n + 15) / 16) * p.xs_tile, part, p.npf,
                   reinterpret_cast<char*>(red));
      }
    }
    return;
  }

  XsWalk w(p);
  for (int s = 0; s < p.count; ++s, w.advance()) {
    const int64_t off = w.off();
    stamp(s, 0);
    // ---- forward + head of tile (x, slot)
    bool bad = false;
    if (slot < p.nw && slot < tn) {
      SplitStepArgs f = a;
      if constexpr (!DIAG) f.stamps = nullptr;  // (fha_body's per-workgroup stamps)
      f.X = p.X0 + off * a.P;
      if constexpr (RM == 0) f.Xs = p.Xs0 + off / 16 * p.xs_tile;
      f.XT = p.XT0 + off;
      HeadArgs hh = h;
      if constexpr (!DIAG) hh.stamps = nullptr;  // (the forward K loop's per-wave stamps)
      hh.labels = p.lab0 + off;
      hh.D = p.Dx + (size_t)x * 16 * ld;  // this XCD's copy of D (the role's db2 reads it)
      hh.b2 = s == 0 ? (const void*)a.b2 : (const void*)(p.b2x + x * 16);
      gran_t* slabs = p.gran + (size_t)(s & 1) * 32 * 8 * 16 * kXsCols;
      if constexpr (FG == 2) {  // (the previous step's dW1 tiles and role, waited for per wave inside the GEMM)
        PsGate gate;
        gate.line = s > 0 ? xs_flags(p.ctl, x) : nullptr;
        gate.tag = bar.tag_of(2 * s - 1);
        gate.stop_tag = p.launch + 1u;
        gate.ntiles = t1n;
        gate.role = p.nw;
        gate.s_stop = &s_stop;
        gate.err = p.err;
        gate.limit_us = limit_us;
        bad = !fha_body<3, 3, true, kSwz, true, true, DIAG, HK>(f, hh, nullptr, slabs, p.err, tm, tn, slot * 8 + x, red,
                                                             x, slot, p.ep0 + (unsigned)s, &gate);
      } else {
        bad = !fha_body<3, 3, true, 7, true, false, DIAG>(f, hh, nullptr, slabs, p.err, tm, tn, slot * 8 + x, red, x,
                                                          slot, p.ep0 + (unsigned)s);
      }
    }  // (FG 2, a worker without a forward tile: the heads that overwrite what its dW1 tile read waited for it)
    stamp(s, 1);
    if constexpr (FG > 0) {
      bar.arrive(2 * s, bad);  // (the dW1 waves wait for their own column tiles, the role for all of them)
    } else {
      if (!bar.sync(2 * s, bad)) return;
    }
    stamp(s, 2);
    if (slot < p.nw) {
      if (slot < t1n) {  // ---- dW1 tile (x, slot) over the whole batch + reg + SGD (W1, W1s, b1)
        TileGeom g{a.H, a.P + a.bias_col, n, x * 16, slot * 32};
        const EpiW1 e1{a.W1, a.gW1, static_cast<bf16*>(a.W1p), (size_t)a.H * a.P, a.P, 1, 0, reg, lr, a.xscale, {},
                       a.b1, a.gb1, 0, nullptr};
        if constexpr (FG > 0) {
          EpiW1Gate epi{e1, &bar, 2 * s, tn, &s_stop};
          epi.W1s = a.W1s;
          if constexpr (RM == 0)
            wsk_tile<bf16, 1, 2, 8, true, true, 3, 4, 3, uint8_t, float, true, false, kSc1>(
                a.dZ1, (ld + 63) / 64, static_cast<const uint8_t*>(p.XT0) + off, a.ldxt, g, epi, red, 0, nullptr);
          else
            wsk_tile<bf16, 1, 2, 8, true, true, RM, 4, 3, uint8_t, float, false, false, kSc1>(
                a.dZ1, ld, static_cast<const uint8_t*>(p.XT0) + off, a.ldxt, g, epi, red, 0, nullptr);
        } else {
          EpiW1 epi = e1;
          epi.W1s = a.W1s;
          wsk_tile<bf16, 1, 2, 8, true, true, 3, 4, 3, uint8_t, float, true, false, kSc1>(
              a.dZ1, (ld + 63) / 64, static_cast<const uint8_t*>(p.XT0) + off, a.ldxt, g, epi, red, 0, nullptr);
        }
      }
    } else {
      if constexpr (FG > 0) {  // (the role reads every column tile's dW2 partials and D: it waits for all of them)
        if (t < 64) bar.poll(2 * s, 0, tn);
        __syncthreads();
      }
    }
    if (slot == p.nw && !s_stop) {  // ---- the role: W2[:, x rows] from the dW2 partials and db2 into this XCD's b2
      // copy, side by side
      // (waves [0, dw): dW2, one element per lane; waves [dw, 8): db2, up to 4 classes per wave with every row's
      // loads in flight at once -- one after the other they were this workgroup's 4.2 us critical path,
      // profiles/r6/xstep_ab_r6a.jsonl)
      const int lane = t & 63, wv = __builtin_amdgcn_readfirstlane(t >> 6);
      const int dw = (16 * a.C + 63) / 64;
      if (wv < dw) {
        const int nct = (n + 15) / 16, e = t, c = e >> 4, hr = x * 16 + (e & 15);
        const bool ok = c < a.C && hr < a.H;
        EpiW2 epi{a.W2, a.gW2, a.H, 1, 0, reg, lr, {}, nullptr};
        epi.prefetch(0, c, hr, ok);
        const __amdgpu_buffer_rsrc_t rp = make_rsrc(a.dw2part);
        float v = 0.f;
        for (int k0 = 0; k0 < nct; k0 += 32) {  // (the two-launch role's summation order: k ascending)
          float pv[32];
#pragma unroll
          for (int u = 0; u < 32; ++u)
            pv[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                  rp, (ok && k0 + u < nct) ? (((k0 + u) * 16 + c) * a.H + hr) * 4 : kOOB,
                                                  0, kSc1));
#pragma unroll
          for (int u = 0; u < 32; ++u) v += pv[u];
        }
        if (ok) epi(0, c, hr, v);
      } else {
        // db2 as the two-launch step's bias-row workgroups compute it (row_sum's lane-strided order, then wave_sum)
        const int nd = 8 - dw, c0 = wv - dw;
        const float* b2src = s == 0 ? a.b2 : p.b2x + x * 16;
        const __amdgpu_buffer_rsrc_t rb = make_rsrc(b2src);
        float bpre[4], acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int cc = c0 + k * nd;
          bpre[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb, cc < a.C ? cc * 4 : kOOB, 0,
                                                                                   kSc1));
        }
        for (int j0 = 0; j0 < n; j0 += 64 * 16) {
          float v[4][16];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int cc = c0 + k * nd;
            const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.Dx + ((size_t)x * 16 + (cc < a.C ? cc : 0)) * ld);
#pragma unroll
            for (int u = 0; u < 16; ++u) {
              const int jj = j0 + u * 64 + lane;
              v[k][u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                      rs, (cc < a.C && jj < n) ? jj * 4 : kOOB, 0, kSc1));
            }
          }
#pragma unroll
          for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int u = 0; u < 16; ++u) acc[k] += v[k][u];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int cc = c0 + k * nd;
          const float sum = wave_sum(acc[k]);
          if (cc < a.C && lane == 0) {
            const float nb = bpre[k] - lr * sum;
            p.b2x[x * 16 + cc] = nb;
            if (x == 0 && s + 1 == p.count) a.b2[cc] = nb;
          }
        }
      }
    }
    stamp(s, 3);
    if constexpr (FG == 2) {
      bar.arrive(2 * s + 1, s_stop != 0);  // (the next forward's waves wait for the flags they need)
      if (s_stop) return;
    } else {
      if (!bar.sync(2 * s + 1, s_stop != 0)) return;
    }
  }
}

}  // namespace

// The row-major form's dW1 vector form (xstep_kernel RM): 1 (n % 8 == 0), 2 (n % 4 == 0), 0 none -- fp32 dZ1 and
// 4-byte pixel rows, as the two-launch weight gradient takes them (mlp_split_wgrad: base_ok, vec)
int mlp_xstep_rm(const SplitStepArgs& a) {
  const bool ok = a.npz == 3 && (a.a_fp32 & 2) && a.dZ1 && ((uintptr_t)a.dZ1 & 15) == 0 && a.ld % 8 == 0 &&
                  ((uintptr_t)a.XT & 3) == 0 && a.ldxt % 4 == 0;
  const bool pairs = ((uintptr_t)a.XT & 15) == 0 && a.ldxt % 16 == 0 && a.n % 16 == 0;
  return !ok ? 0 : a.n % 8 == 0 ? (pairs ? 3 : 1) : a.n % 4 == 0 ? 4 : 0;
}

bool mlp_xstep_ok(const SplitStepArgs& a, const HeadArgs& h) {
  const int tm = xs_cdiv(a.H, 16), tn = xs_cdiv(a.n, kXsCols), t1n = xs_cdiv(a.P + a.bias_col, 32);
  const int nw = std::max(tn, t1n);
  const bool common =
      a.H <= 128 && tm <= 8 && a.C <= 16 && a.bias_col && a.sgd == 1 && a.xf_world == 0 && a.npw == 3 &&
      a.npz == 3 && a.w1_swz && a.W1s && a.dZ1 && h.dZ1 == a.dZ1 && !h.dZ1_planes && a.dw2part &&
      h.dw2part == a.dw2part && a.dw2_cols == 16 && !h.a1 && !a.a1 && !h.loss_partial && a.n > 0 &&
      nw + 1 <= kXsWgsPerXcd && nw + 1 <= 31 && device_cu_count() == 8 * kXsWgsPerXcd &&
      // (the forward GEMM's wave 7 has no K range: the gated forward stages b1 / W2 / b2 there, fha_body PsGate)
      xs_cdiv(xs_cdiv(a.P, 32), 8) * 7 * 32 >= a.P && (int64_t)a.P * a.ldxt < (int64_t)kOOB &&
      (int64_t)xs_cdiv(a.H, 16) * 16 * a.ld < (int64_t)kOOB / 4;
  if (!common) return false;
  if (a.dz_swz == 1)  // the fragment-ordered form
    return a.x_swz && a.Xs && h.dz_swz == 1 && a.n % 16 == 0 && mlp_wgrad_dz_swz_ok(a);
  return a.dz_swz == 0 && h.dz_swz == 0 && !a.x_swz && mlp_xstep_rm(a) > 0;  // the row-major form
}

int mlp_xstep_workers(const SplitStepArgs& a) { return std::max(xs_cdiv(a.n, kXsCols), xs_cdiv(a.P + a.bias_col, 32)); }

void mlp_xstep(const SplitStepArgs& a, const HeadArgs& h, const XStepPlan& p, hipStream_t s) {
  if (p.count <= 0) return;
  CME_REQUIRE(mlp_xstep_ok(a, h), "xstep: the plan's step is not the XCD-local pipeline's shape");
  const int tm = xs_cdiv(a.H, 16), tn = xs_cdiv(a.n, kXsCols), t1n = xs_cdiv(a.P + a.bias_col, 32);
  CME_REQUIRE(p.nw == mlp_xstep_workers(a) && p.nw + 1 + p.npf <= kXsWgsPerXcd && p.nw + 1 <= 31 && p.npf >= 0 &&
                  (p.npf == 0 || p.bar == 1) && p.bar >= 0 && p.bar <= 3,
              "xstep: the workers + the role (+ prefetch workgroups, flag-line barrier only) must fit one XCD's CUs");
  CME_REQUIRE(p.gran && p.ctl && p.Dx && p.b2x && p.err && p.X0 && p.XT0 && p.Xs0 && p.lab0 && p.xs_tile > 0,
              "xstep: scratch buffers missing");
  const bool grid16 = p.gstart0 % 16 == 0 && p.B % 16 == 0 && p.shard_off % 16 == 0;
  int rm = a.dz_swz ? 0 : mlp_xstep_rm(a);
  if (rm == 3 && !grid16) rm = 1;  // (16-byte pixel pairs need every step's columns 16-byte aligned)
  const int grid = rm ? 4 : 16;
  CME_REQUIRE(p.gstart0 % grid == 0 && p.B % grid == 0 && p.shard_off % grid == 0 && p.B >= a.n && p.N_end >= p.B,
              "xstep: every step must start a 16-sample tile of the fragment-ordered pixels (row-major form: 4-byte "
              "aligned pixel columns)");
  CME_REQUIRE(a.ld >= a.n && a.ld % 16 == 0, "xstep: activation pitch");
  const bool diag = p.stamps || a.stamps || h.stamps || a.ag_test_skip >= 0;
  CME_REQUIRE(!diag || p.bar == 3 || p.bar == 1,
              "xstep: the stamps and the hand-off test hook exist in the diagnostics builds of barrier forms 1 and 3");
  CME_REQUIRE(!rm || (p.bar == 3 && p.npf == 0 && !diag), "xstep: the row-major form exists in barrier form 3 only");
  if (rm == 1) xstep_kernel<1, 2, false, 7, 1><<<8 * kXsWgsPerXcd, 512, 0, s>>>(a, h, p, tm, tn, t1n);
  else if (rm == 4) xstep_kernel<1, 2, false, 7, 4><<<8 * kXsWgsPerXcd, 512, 0, s>>>(a, h, p, tm, tn, t1n);
  else if (rm == 3) xstep_kernel<1, 2, false, 7, 3><<<8 * kXsWgsPerXcd, 512, 0, s>>>(a, h, p, tm, tn, t1n);
  else if (diag && p.bar == 3) xstep_kernel<1, 2, true><<<8 * kXsWgsPerXcd, 512, 0, s>>>(a, h, p, tm, tn, t1n);
  else if (diag) xstep_kernel<1, 0, true><<<8 * kXsWgsPerXcd, 512, 0, s>>>(a, h, p, tm, tn, t1n);
  // (the production form keeps fha_body's three no-op runtime tests, HK = 7: measured 9.55-9.61 us against 9.81-9.86
  // without them and 9.62-9.94 with any one or two -- the compiler schedules the body differently; alternated four
  // and three times on two boxes, profiles/r6/hk/)
  else if (p.bar == 3) xstep_kernel<1, 2, false, 7><<<8 * kXsWgsPerXcd, 512, 0, s>>>(a, h, p, tm, tn, t1n);
  else if (p.bar == 2) xstep_kernel<1, 1><<<8 * kXsWgsPerXcd, 512, 0, s>>>(a, h, p, tm, tn, t1n);
  else if (p.bar == 1) xstep_kernel<1, 0><<<8 * kXsWgsPerXcd, 512, 0, s>>>(a, h, p, tm, tn, t1n);
  else xstep_kernel<0, 0><<<8 * kXsWgsPerXcd, 512, 0, s>>>(a, h, p, tm, tn, t1n);
  CME_LAUNCH_CHECK(s);
}

}  // namespace cme
