// Split-bf16 fast path for the MLP step ("bf16 planes").
//
// gfx950 has no xf32/TF32 MFMA and its f32-input MFMA runs at the f32 VECTOR
// rate (1/16 of bf16).  An fp32 value has a 24-bit significand = exactly three
// bf16 significands, so w = w0 + w1 + w2 with w_i = bf16 EXACTLY
// (w0 = rn_bf16(w), w1 = rn_bf16(w - w0), w2 = w - w0 - w1).  MNIST pixels are
// integers 0..255, exact in ONE bf16.  Hence
//      W1 . x  =  w0 . x + w1 . x + w2 . x
// with every product exact and fp32 accumulation inside the bf16 MFMA: the
// GEMM reads the same fp32 operands as an f32 GEMM and only the accumulation
// order differs -- 3 v_mfma_f32_16x16x32_bf16 (48 cycles) instead of 8
// v_mfma_f32_16x16x4_f32 (256 cycles) per 16x16x32 block.  The same identity
// is used for dW1 = dZ1 . X^T with dZ1 split into 3 planes.
// With npw = npz = 1 the identical kernels ARE the bf16 mixed-precision path.
//
// The step becomes TWO kernels:
//   A  forward GEMM + head (mlp_fwd1_head_ag at H <= 128, mlp_fwd1_wide_ag for the
//      wide layers): z1 (MFMA) -> sigmoid -> z2 -> softmax -> D -> dZ1 in one launch;
//   B  mlp_split_wgrad : dW1 (MFMA) with fused reg + SGD (+ W1-plane refresh where
//      a forward reads the planes), dW2 and bias gradients as extra roles.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

#include "../common/hip_common.h"

// The two-launch kernels' per-wave / per-workgroup s_memrealtime stamps (SplitStepArgs::stamps / wstamps,
// HeadArgs::stamps; bench/stamps_*.py) exist only in the diagnostics library (`python -m cme213_sp18_amd._build
// --diag` -> _hip_diag, loaded when CME_DIAG=1): their runtime tests cost the production launches 0.3-0.55 us per
// step (profiles/r6/flags_stamps/).  The XCD-local pipeline has its own diagnostics instantiation (xstep.hip DIAG).
#ifndef CME_DIAG_STAMPS
#define CME_DIAG_STAMPS 0
#endif

namespace cme {

// Gradient all-reduce fused into the weight-gradient launch (data parallel over xGMI, one process per
// GPU): every gradient tile is written into this step's half of the rank's IPC buffer, published,
// and, once every peer has published the same tile, summed in rank order and applied (SGD + bf16
// planes) by the same workgroup.  world == 0: off.  Buffers/handles: csrc/comm (XgmiComm).
struct XgmiFuse {
  void* mybuf = nullptr;
  const void* peers[8] = {};
  uint32_t* myflags = nullptr;
  uint32_t* peerflags[8] = {};
  uint32_t* epochs = nullptr;
  int* err = nullptr;
  int rank = 0, world = 0;
  int64_t npad = 0;
  int64_t off_b1 = 0, off_W2 = 0, off_b2 = 0;  // flat-arena offsets ([W1|b1|W2|b2], 64-aligned)
  // Owner-tile push form (push != 0; XgmiComm created with slab_tiles >= the launch's tiles): gradient tile t is
  // reduced and applied by rank t % world alone.  Every other rank PUSHES its tile there as system-scope data-tagged
  // granules (one 8-byte {value, epoch} store each, into the owner's receive area), the owner polls its OWN memory,
  // sums the R tiles in rank order (its own from LDS: the one-shot's bits), applies the update and pushes the new
  // values back the same way.  Two one-way hops per tile, 2 S / R payload bytes per link (x2 for the tags), no
  // write-through drain, no flag, no remote read; at world 1 nothing leaves the workgroup.  Receive areas, in
  // every rank's IPC buffer: [slab_tiles][8][512] gradient granules, then [slab_tiles][512] result granules.
  int push = 0;
  unsigned long long* myslab = nullptr;
  unsigned long long* peerslab[8] = {};
  int64_t slab_tiles = 0;
};

struct SplitStepArgs {
  int P = 784, H = 100, C = 10, n = 0, ld = 0;
  int npw = 3, npz = 3;          // planes of W1 and of dZ1 (3: exact fp32, 1: bf16)
  const void* X = nullptr;       // uint8 shard [n][P] (raw pixels, exact in bf16)
  const void* XT = nullptr;      // uint8 feature-major shard (XT + off) [P][ldxt]
  int ldxt = 0;
  float xscale = 1.f;            // inputs are X * xscale (1/255 = normalised); applied in the epilogues
  const int* labels = nullptr;   // shard
  float *W1 = nullptr, *b1 = nullptr, *W2 = nullptr, *b2 = nullptr;  // fp32 master params
  void* W1p = nullptr;           // bf16 planes [npw][H][P]
  float *gW1 = nullptr, *gb1 = nullptr, *gW2 = nullptr, *gb2 = nullptr;
  float *a1 = nullptr, *D = nullptr, *dZ1 = nullptr;  // [H][ld], [C][ld], [H][ld]
  void* dZ1p = nullptr;          // bf16 planes [npz][H][ld]
  float* loss_partial = nullptr; // one per fwdhead block (optional)
  double scale = 1.0, reg = 0.0, lr = 0.0;
  int sgd = 1, shift = 1;
  int mode = 0;                  // HeadMode: 0 train, 1 predict (pred), 2 probs
  int* pred = nullptr;
  float* probs = nullptr;
  int ldp = 0;
  unsigned long long* stamps = nullptr;  // diagnostics: per-wave s_memrealtime stamps (see mma_tile.h)
  // diagnostics: per-workgroup stamps of the small weight-gradient launch (thread 0: entry, tile + epilogue done,
  // exchange done, end; [blockIdx][4]) -- bench/stamps_push.py
  unsigned long long* wstamps = nullptr;
  // weight-gradient launch selection (bucketed all-reduce overlap): wg_parts bit0 = dW1 rows
  // [w1_row0, w1_row0 + w1_rows) (w1_rows < 0: all), bit1 = dW2 + bias gradients
  int wg_parts = 3, w1_row0 = 0, w1_rows = -1;
  // split-K dW1 (wide layers, few output tiles and a long K: the tensor-parallel shard at a large global batch,
  // e.g. 512 hidden rows x 6400 columns): fp32 partial slabs [ksplit][rows][P + 1] of kpart_cap floats; the
  // launcher takes it when the tiles alone cannot fill the chip, and a second kernel sums the slabs in slab order
  // and applies the update.  nullptr: never split.
  float* kpart = nullptr;
  int64_t kpart_cap = 0;
  int wg_ksplit = 1, wg_kchunk = 0;  // (set by the launcher)
  // XT carries an extra all-ones feature row P: the dW1 GEMM's column P is then sum_b dZ1[h][b] = db1[h]
  // (exact, same planes), so db1 / b1 come out of the dW1 launch and the role kernel only does dW2 / db2
  int bias_col = 0;
  // the fused all-reduce (run(sgd = 2)): a DEVICE copy of the XgmiFuse, uploaded once by MlpStep::set_xgmi, and its
  // two scalars the launcher tests.  (By value it was 288 of the launch's ~950 kernel-argument bytes, written by
  // the host on every launch: the native loop's host enqueue time per step is what that costs.)
  const XgmiFuse* xf = nullptr;
  int xf_world = 0, xf_push = 0;
  // H <= 128 split3: the forward reads fp32 W1 from its fragment-ordered copy W1s (mma_tile.h ASWZ: every 16-byte
  // load instruction of a wave reads 1 KB of contiguous memory instead of 16 rows x 64 B), and the weight-gradient
  // launch's in-place update writes W1s next to W1 (w1s_off).  Set by MlpStep::run after refreshing a stale copy
  int w1_swz = 0;
  float* W1s = nullptr;
  // ... and (with w1_swz) the pixels from their fragment-ordered copy Xs: this step's first sample tile of the
  // [cdiv(N, 16)][cdiv(P, 64)][64 lanes][16 B] copy (mma_tile.h BSWZ / xs_off; the step's first sample a multiple of 16)
  int x_swz = 0;
  const void* Xs = nullptr;
  // ... and (fp32 dZ1, a_fp32 bit1) the weight-gradient GEMM reads dZ1 from the fragment-ordered buffer the head
  // wrote (a.dZ1 then points at it).  1: H <= 128, [cdiv(H, 16)][cdiv(ld, 64)][4][64 lanes][4 floats] (mma_tile.h
  // w1s_off); 2: the wide A-in-registers engine, [cdiv(H, 16)][cdiv(ld, 32)][2][64 lanes][4 floats] (rega_gemm.h dzr_off)
  int dz_swz = 0;
  // wide layers (LDS GEMM forward): when set, the forward GEMM's tile epilogue also leaves the head's
  // z2 partial sums, z2part[row tile][16][ld] = W2[:, tile rows] . a1[tile rows, :] (v_mfma_f32_16x16x4
  // on the activated accumulators), so the head never re-reads a1 for z2 (mlp_split_fwd1_z2_chunks)
  float* z2part = nullptr;
  // wide layers: bf16 copies of the shard (Xw = Xw_base + off*P, [n][P]; XTw = XTw_base + off, [P+1][ldxt])
  // for the direct-to-LDS GEMM engines (glds_gemm.h, rega_gemm.h); nullptr: the wave-split-K kernels read the uint8s
  const void* Xw = nullptr;
  const void* XTw = nullptr;
  // small layers (wave-split-K kernels), split3 only: bit0 = the forward GEMM reads fp32 W1, bit1 = the dW1
  // GEMM reads fp32 dZ1 (4 B per element, split into the exact bf16 planes in registers; the head then
  // writes no dZ1 planes); clear bits: the stored planes (6 B per element, split once by their writer).
  // Policy (MlpStep::split_args, measured: bench/kbench.py): at H <= 128 1 below n = 200 columns, 3 from there; 3 above
  int a_fp32 = 1;
  // wide layers (the 128 x 128 A-in-registers tiling): the K loop's engine -- 0 rega_gemm.h (A fragments straight
  // into registers, 32-deep stages), 1 g64_gemm.h (both operands LDS-DMA'd in full rows, 64-deep steps); the same
  // bits either way (MlpStep.wide_eng)
  int wide_eng = 0;
  // diagnostics only (bench/kbench.py xp rows): ablations of the push form at world 1 -- bit0: no exchange
  // (old - lr * own), bit1: no W1 / b1 put, bit2: dW1 tiles skip the LDS staging wait (no barrier)
  int xp_dbg = 0;
  // the g64 wide engine pulls each XCD's A and B tiles into its L2 at entry (g64::Touch; MlpStep.g64_touch)
  int g64_touch = 1;
  // wide layers: the head left dW2 partials [cdiv(n, 32)][16][H] (HeadArgs::dw2part); the dW2 role then sums
  // them in column-tile order instead of forming D . a1^T from all of a1
  float* dw2part = nullptr;
  int dw2_cols = 32;  // columns per dW2 partial: 32 (head_wide_kernel), 128 (the fused all-gather head)
  int w1_planes = 1;  // (set by mlp_split_wgrad) the small-layer W1 update refreshes the W1 planes
  // wide split3 layers: the A-in-registers dW1 launch's in-place update (sgd = 1) leaves the W1 planes alone (the
  // 128 x 128 forward reads fp32 W1); the caller marks them stale and refreshes them before a forward that reads them
  int w1_planes_lazy = 0;
  // The all-gather forward + head launches' timed-out-wait word (MlpEngine.ag_err).  The weight-gradient
  // launch reads it and, when set, APPLIES NOTHING: no SGD / plane refresh (sgd = 1), no xGMI exchange (the
  // fused all-reduce: this rank stops taking part, its peers time out), and the gradient status word below
  // marks the bucket (sgd = 0) so the separate SGD / all-reduce kernels apply nothing on any rank.
  const int* ag_err = nullptr;
  // sgd = 0: the flat gradient bucket's status element (after b2): 0.f good, 1.f = this rank's step is
  // untrusted.  Summed by the all-reduce with the gradients; the SGD kernels skip the update when non-zero.
  float* gstatus = nullptr;
  // the all-gather hand-off's wait bound in microseconds of wall time (hip_common.h kHandoffWaitUs) and a TEST
  // hook: row tile ag_test_skip of column tile 0 withholds its granules, so that tile's wait really times out
  // (-1: off)
  int ag_wait_us = (int)kHandoffWaitUs;
  int ag_test_skip = -1;
  // H <= 128 (at most 8 row tiles): the forward + head and the dW1 launches place the workgroups of row tile rt on
  // XCD rt (blockIdx % 8, speed only): the W1 rows the dW1 launch updates and the dZ1 rows the forward writes are
  // then read back by the next launch from the same XCD's L2 instead of the die-level cache.  Set by the launcher
  // (mlp_split_xcd_rows_ok); 0: the column-tile grouping; 2 (the forward + head launch only, small batches): row
  // tiles rt and rt + 4 on XCD rt < 4 (mlp_split_xcd_rows_packed_ok; MlpStep.xcd_pack)
  int xcd_rows = 0;
  // H <= 128 under xcd_rows: pf_wgs extra workgroups per XCD in each launch pull the pixels that XCD's workgroups
  // read next into its L2, on CUs the step leaves idle: the forward + head launch this step's feature-major XT (for
  // the weight-gradient launch), the weight-gradient launch the next step's X at pf_X (nullptr: none) for the next
  // forward (MlpStep.prefetch; 0: off)
  int pf_wgs = 0;     // ... in the weight-gradient launch (the next step's X)
  int pf_wgs_xt = 0;  // ... in the forward + head launch (this step's XT)
  const void* pf_X = nullptr;
  int64_t pf_bytes = 0;  // bytes of pf_X to pull: the next step's rows that exist (a partial last batch is shorter)
};


// true when a forward kernel of this configuration reads the W1 planes (false: fp32 W1 everywhere)
bool mlp_split_w1_planes_read(const SplitStepArgs& a);

// the small-layer forward GEMM reads fp32 W1 (split in registers) instead of the W1 planes
bool mlp_split_fwd_fp32_w(const SplitStepArgs& a);
// the weight-gradient GEMM can read fp32 dZ1 in fragment order (SplitStepArgs::dz_swz)
bool mlp_wgrad_dz_swz_ok(const SplitStepArgs& a);
// ... and the wide A-in-registers dW1 in its own fragment order (SplitStepArgs::dz_swz == 2, rega_gemm.h dzr_off)
bool mlp_wgrad_dzr_ok(const SplitStepArgs& a);

// number of z2 row-tile partials mlp_split_fwd1 writes for `a` (0: the forward does not produce them)
int mlp_split_fwd1_z2_chunks(const SplitStepArgs& a);
// true when the weight-gradient launch of this (whole-layer) step reads dZ1 in fp32 and splits it in
// registers (rega_gemm.h): the head then writes fp32 dZ1 and no dZ1 planes
bool mlp_split_wgrad_fp32_dz(const SplitStepArgs& a);
// true when mlp_split_wgrad(a) leaves the W1 planes stale (a.w1_planes_lazy on the A-in-registers dW1 update)
bool mlp_split_wgrad_leaves_planes_stale(const SplitStepArgs& a);
// true when the wide forward launch of `a` (ag: the fused all-gather head form, allow64 as for it) reads the W1
// planes; false when it reads fp32 W1 only (the split3 128 x 128 A-in-registers engine)
bool mlp_split_wide_fwd_reads_planes(const SplitStepArgs& a, int ag, int allow64);

// the XCD-row placement (SplitStepArgs::xcd_rows) applies to this small-layer step: at most 8 row tiles of 16 and
// at most one workgroup per CU of the XCD for each row tile's column tiles
bool mlp_split_xcd_rows_ok(const SplitStepArgs& a);
// ... and its packed form for the forward + head launch (xcd_rows == 2: row tiles rt and rt + 4 on XCD rt < 4, when
// both fit the XCD's CUs: small batches)
bool mlp_split_xcd_rows_packed_ok(const SplitStepArgs& a);

// the fragment-ordered fp32 copy of W1 (SplitStepArgs::W1s): floats for an H x P layer, and a full rebuild from W1
int64_t mlp_split_w1s_floats(int H, int P);
void mlp_split_w1s_refresh(const float* W1, float* W1s, int H, int P, hipStream_t s);


// flag slots (workgroup tiles) of the fused-all-reduce wgrad launch for a P-H layer with the all-ones
// feature; -1 when above `cap`
int mlp_split_fused_tiles(int P, int H, int cap);

// tiled forward only: a1 = sigmoid(W1 X + b1) (pair with mlp_head for the 3-kernel step)
void mlp_split_fwd1(const SplitStepArgs& a, hipStream_t s);
// wide layers: the forward GEMM with the head fused in (all-gather form; fwd1_rega_kernel<..., AG> on 128 x 128
// tiles, fwd1_glds_kernel<64, 64, ..., AG> on 64 x 64): one launch leaves a1 (store_a1), D, the loss partials,
// dZ1 (fp32 and / or planes) and the dW2 partials per column tile (h.dw2part).  Returns the tile width: the
// weight-gradient launch then needs a.dw2_cols = it.  Every workgroup must be resident at once (off when
// processes share a GPU); a timed-out poll sets *err.  counters: [2][max_tiles][32] uint64 (one array per tiling);
// the hand-offs are data-tagged granules (gran) whose epoch comes from those counters.
struct HeadArgs;
// allow64: also the 64 x 64 tiling (MlpStep.ag_tiles64: by default only when a1 is not stored)
bool mlp_fwd1_wide_ag_ok(const SplitStepArgs& a, const HeadArgs& h, int allow64);
// gran: >= (cdiv(H, 64) * 16 + 16) * ld uint64 granules (z2 partials, then D), tags never reused
int mlp_fwd1_wide_ag(const SplitStepArgs& a, const HeadArgs& h, unsigned long long* counters, int max_tiles,
                     unsigned long long* gran, int64_t gran_count, int* err, int store_a1, int allow64,
                     hipStream_t s);
void mlp_split_wgrad(const SplitStepArgs& a, hipStream_t s);

// The XCD-local step pipeline (xstep.hip): every step of a native step-loop plan (MlpStep::run_steps) in ONE
// persistent launch -- row tile rt's forward + head, dW1 tiles and W2 rows on XCD rt, two XCD-local barriers per step,
// the z2 all-gather the only cross-XCD hand-off.  `a` / `h` are the plan's step as the two-launch form would run it
// (fragment-ordered W1, pixels and dZ1 -- or, a.dz_swz == 0, row-major pixels and fp32 dZ1 for steps off the
// 16-sample grid such as n = 100 -- the head's dW2 partials, fused SGD; their pixel / label pointers are re-based per
// step from the plan's bases).
struct XStepPlan {
  int64_t gstart0 = 0, B = 0, shard_off = 0, N_end = 0;  // MlpStep::run_steps's walk over the dataset
  int count = 0;
  const uint8_t* X0 = nullptr;   // row-major pixels [N][P]
  const uint8_t* XT0 = nullptr;  // feature-major pixels [P + 1][ldxt] (the all-ones row last)
  const uint8_t* Xs0 = nullptr;  // fragment-ordered pixels (mma_tile.h xs_off), xs_tile bytes per 16 samples
  const int* lab0 = nullptr;
  int64_t xs_tile = 0;
  unsigned ep0 = 1;        // the first step's granule tag; step s uses ep0 + s (tags never repeat over a buffer's life)
  unsigned launch = 0;     // launches so far: control bank launch & 1
  unsigned long long* gran = nullptr;  // z2 partial granules [2 step parities][32][8][16][32]
  unsigned long long* ctl = nullptr;   // [2 banks][8 XCDs][64] ticket / barrier words, zeroed once at allocation
  float* Dx = nullptr;     // [8 XCDs][16][ld]: each XCD's copy of D (its role workgroup's db2 reads it)
  float* b2x = nullptr;    // [8 XCDs][16]: each XCD's copy of b2 (updated in the same order on every XCD)
  int* err = nullptr;      // the sticky timed-out word (MlpEngine.ag_err)
  int nw = 0;              // workers per XCD (mlp_xstep_workers)
  int npf = 0;             // prefetch workgroups per XCD (idle CUs pulling the pixels the XCD reads next into its L2)
  int bar = 3;             // the XCD-local barriers: 0 an atomic counter, 1 a flag line in the XCD's L2 (xstep.hip XsBar),
                           // 2 the flag line with the first barrier fine-grained (each dW1 wave waits for its own
                           // column tiles' dZ1: EpiW1Gate), 3 both fine-grained (the next step's forward waves wait
                           // for their own dW1 tiles, wave 7 for all of them and the role: fha_body PsGate)
                           // -- n = 800 walking step: 0 ~14, 1 11.0, 2 10.8, 3 9.85 us (profiles/r6/xstep_ab_r6i.jsonl)
  unsigned long long* stamps = nullptr;  // diagnostics: [stamp_steps][8][32][4] s_memrealtime per workgroup
  int stamp_steps = 0;
};
bool mlp_xstep_ok(const SplitStepArgs& a, const HeadArgs& h);
int mlp_xstep_rm(const SplitStepArgs& a);  // the row-major form's dW1 vector form (0: the form does not apply)
int mlp_xstep_workers(const SplitStepArgs& a);
void mlp_xstep(const SplitStepArgs& a, const HeadArgs& h, const XStepPlan& p, hipStream_t s);
constexpr int64_t kXstepGranules = 2 * 32 * 8 * 16 * 32;
constexpr int64_t kXstepCtlWords = 2 * 8 * 64 + 8 * 16;

// planes[p][i] for i < n: exact np-way bf16 split of W[i] (np = 1: plain rounding).
void mlp_split_planes(const float* W, void* planes, int64_t n, int np, hipStream_t s);
// params[i] -= lr * grads[i]; then refresh the W1 planes (first w1_count params).
// status: the bucket's status element (nullptr: none) -- non-zero (an untrusted step on some rank) skips the update
void mlp_split_sgd(float* params, const float* grads, int64_t count, double lr, void* W1p, int64_t w1_count,
                   int npw, hipStream_t s, const float* status = nullptr);

}  // namespace cme
