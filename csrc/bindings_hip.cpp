// pybind11 bindings for the gfx950 kernels (module cme213_sp18_amd._hip).
//
// Tensors cross the boundary as raw device pointers (int) and the HIP stream
// as an int handle (torch.cuda.current_stream().cuda_stream), so any launch
// issued while torch is capturing a HIP graph is recorded into that graph.
// No torch headers: the extension only depends on the HIP runtime, which it
// shares with torch (same SONAME, torch is always imported first).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>


#include "comm/xgmi_allreduce.h"
#include "common/hip_common.h"
#include "mlp/mlp_kernels.h"
#include "mlp/mlp_split.h"
#include "suite/suite_kernels.h"

namespace py = pybind11;
using cme::DType;

namespace {

template <typename T>
inline T* P(uintptr_t p) { return reinterpret_cast<T*>(p); }
inline hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
inline DType to_dt(int d) {
  if (d < 0 || d > 2) throw std::invalid_argument("dtype code must be 0 (f32), 1 (f64) or 2 (bf16)");
  return static_cast<DType>(d);
}

// Hot-path step object: everything a training step needs, bound once.  One
// Python call launches the whole fused step (3 kernels), keeping host overhead
// out of eager-mode steps; graph capture records the same launches.
struct MlpStep {
  int dt = 0;
  int P = 784, H = 100, C = 10, ld = 0;
  uintptr_t X = 0, labels = 0;            // device-resident dataset (gemm dtype) + int32 labels
  uintptr_t XT = 0;                       // optional feature-major copy [P][N]
  uintptr_t Xw = 0, XTw = 0;              // wide layers: bf16 copies of X [N][P] / XT [P+1][N] (0: none)
  int64_t N = 0;                          // samples in the resident dataset (ld of XT)
  uintptr_t W1 = 0, b1 = 0, W2 = 0, b2 = 0, W1g = 0;  // params (+ bf16 shadow of W1)
  uintptr_t gW1 = 0, gb1 = 0, gW2 = 0, gb2 = 0;       // gradient bucket views
  uintptr_t a1 = 0, D = 0, dZ1 = 0, dZ1g = 0;         // activations [rows][ld]
  uintptr_t loss = 0;                                 // float partials, >= head blocks
  int shift = 1, act = 1;
  // split-bf16 path (mlp_split.h): X/XT are bf16, W1p/dZ1p hold npw/npz bf16 planes
  int split = 0, npw = 3, npz = 3;
  uintptr_t stamps = 0;  // diagnostics only
  uintptr_t hstamps = 0;  // diagnostics only: head-block stamps
  uintptr_t wstamps = 0;  // diagnostics only: weight-gradient workgroup stamps (SplitStepArgs::wstamps)
  uintptr_t z2p = 0;     // wide-layer head scratch (head_big_scratch_floats), 0: column head
  uintptr_t dw2p = 0;    // wide layers: dW2 partials [cdiv(ld, 32)][16][H] left by the head (0: the dW2 GEMM)
  int bias_col = 0;      // XT has an all-ones feature row P: db1 comes out of the dW1 GEMM
  // split path, H <= 128: uint32 tile counters (>= fh_tiles, zeroed) enable the single-launch forward +
  // head (mlp_fwd1_head); 0: separate fwd1 + head kernels
  uintptr_t fh_counters = 0;
  int fh_tiles = 0;
  // the all-gather form of that launch (mlp_fwd1_head_ag): uint64 counters, z2 partial slabs and an error
  // word (>= fh_tiles each); fh_allgather = 1 selects it when all three are set
  uintptr_t ag_counters = 0, ag_slabs = 0, ag_err = 0;
  int fh_allgather = 0;
  // the gradient bucket's status element (float, after b2): written by the wgrad launch in gradient mode
  uintptr_t gstatus = 0;
  // the all-gather hand-offs' wait bound (microseconds of wall time) and the forced-timeout test hook
  // (SplitStepArgs::ag_test_skip; -1 off)
  int ag_wait_us = (int)cme::kHandoffWaitUs, ag_test_skip = -1;
  // wide split layers: the all-gather head fused into the forward launch (fh_allgather, ag_counters, ag_err;
  // mlp_fwd1_wide_ag) leaves dW2 partials per 128 / 64 columns (32 from head_wide_kernel): what run_wgrad sums
  int dw2_cols_last = 32;
  int dw2_left = 0;  // the last run(parts & 1) left dW2 partials in dw2p (the H <= 128 all-gather head or wide)
  int store_a1 = 1;  // the fused wide head: 0 skips the a1 store (nothing in the step reads it)
  // the fused wide head's hand-off granules ([cdiv(H, 64)][16][ld] z2 partials, then [16][ld] D; uint64)
  uintptr_t ag_gran = 0;
  int64_t ag_gran_count = 0;
  // the fused wide head on the 64 x 64 tiling (H = 512-1024): -1 = when a1 is not stored (measured faster only
  // then: profiles/wide_fused_head_r2.md), 1 = always, 0 = never
  int ag_tiles64 = -1;
  // H <= 128: the XCD-row placement of the forward + head and dW1 launches (SplitStepArgs::xcd_rows; on: the W1
  // rows and dZ1 rows each launch writes are read back by the next one from the same XCD's L2 -- step 14.0 ->
  // 13.1-13.2 us at n = 800, 12.3 -> 11.7 us at n = 100, profiles/kbench_xcd_rows_r4.jsonl; 0 for A/B)
  int xcd_rows = 1;
  // SplitStepArgs::xcd_rows == 2 for the forward + head when it fits (small batches): the first four XCDs start a
  // launch up to ~1 us before the other four (profiles/r5/stamps_fha_per_xcd.jsonl), but two row tiles per XCD
  // measured SLOWER, off: walking step +0.3-0.7 us at n = 100-512 (profiles/r5/kbench_xcd_pack.jsonl, alternated
  // twice) -- each XCD then pulls twice the W1 rows and pixels through its L2
  int xcd_pack = 0;
  // SplitStepArgs::w1_swz / W1s: the forward (H <= 128 split3, 16-byte pixel pairs) reads fp32 W1 from its
  // fragment-ordered copy w1s; the in-place update keeps the copy fresh, every other W1 write marks it stale
  // (swz_stale: MlpEngine.refresh_shadow / sgd / mark_planes_stale, run_wgrad with an update) and run() rebuilds it
  // before the next forward that reads it
  int w1_swz = 1;
  uintptr_t w1s = 0;
  int a_fp32 = -1;  // SplitStepArgs::a_fp32 (-1: the measured policy in split_args; A/B knob)
  // SplitStepArgs::dz_swz: with fp32 dZ1 (a_fp32 bit1) and the W1 copy's forward, the all-gather head writes dZ1 in
  // the weight-gradient GEMM's fragment order into dz1s and that GEMM reads it from there (whole steps only: a
  // bucketed run_wgrad reads the row-major dZ1)
  int dz_swz = 1;
  uintptr_t dz1s = 0;
  int dz_left_swz = 0;  // the last forward + head left dZ1 in dz1s (fragment order), not in dZ1 (MlpEngine.dz1())
  // SplitStepArgs::x_swz / Xs: with w1_swz, the forward also reads the pixels from their fragment-ordered copy xs
  // (MlpEngine.load_dataset builds it once; a step whose first sample is not a multiple of 16 reads the row-major X)
  int x_swz = 1;
  uintptr_t xs = 0;
  bool swz_stale = true;
  void refresh_swz(uintptr_t stream) {
    if (!swz_stale || !w1s) return;
    cme::mlp_split_w1s_refresh(P_<float>(W1), P_<float>(w1s), H, P, S(stream));
    swz_stale = false;
  }
  // SplitStepArgs::pf_wgs, prefetch workgroups per XCD (0: off).  Walking-batch step (kbench step_walk_us, A/B twice):
  // 0 -> 4: 14.55-14.63 -> 14.11-14.14 us at n = 800, 13.0-13.1 -> 12.64-12.66 at n = 100; 2 and 6 slower at n = 800
  // (profiles/kbench_prefetch_wgs_r4.jsonl)
  int prefetch = 4;
  // SplitStepArgs::pf_wgs_xt (this step's XT pulled by extra workgroups of the forward + head launch): on in round 4,
  // OFF since the end of round 5 -- with the fragment-ordered forward operands and fp32 dZ1 they cost the forward more
  // than they save the weight-gradient launch: walking step 14.01-14.06 -> 13.73-13.85 us at n = 800, -0.13 at 512,
  // -0.15 at 400, -0.03 to -0.1 at 100-200 (profiles/r5/kbench_prefetch_xt_r5.jsonl, alternated three times)
  int prefetch_xt = 0;
  int wide_eng = -1;    // SplitStepArgs::wide_eng: the 128 x 128 wide K loop's engine (0 rega, 1 g64; -1: g64 for bf16
                        // A, rega for fp32 -- 784-4096-10 step bf16 39.1 -> 38.1 us, fp32 55.4 -> 58.0 with g64,
                        // profiles/r5/kbench_wide_engines.jsonl)
  // H <= 128, the all-gather forward + head: it also leaves the dW2 partials per 32 columns (fha_body step 4a) for
  // the weight-gradient launch's dW2 role (needs dw2p); 0: the role forms D . a1^T over the batch itself; -1 (auto):
  // from n = 768 columns (it was 512 when it went in; re-measured on the final round-5 forms, walking step: n = 512
  // h0 12.90-13.04 vs h1 13.24-13.25 us, n = 800 equal, 13.76-13.91 either way -- profiles/r5/kbench_head_dw2_r5end.jsonl)
  int head_dw2 = -1;
  int xp_dbg = 0;       // SplitStepArgs::xp_dbg (diagnostics)
  int g64_touch = 0;    // SplitStepArgs::g64_touch (measured slower: 784-4096-10 bf16 38.1 -> 41.7 us,
                        // fp32 57.5 -> 62.6, profiles/r5/kbench_wide_touch.jsonl)
  int ag64() const { return ag_tiles64 >= 0 ? ag_tiles64 : (store_a1 ? 0 : 1); }
  // data-parallel step with the xGMI gradient all-reduce + SGD fused into the wgrad launch (run(sgd=2))
  cme::XgmiFuse xf;
  // push != 0: the owner-tile push form (XgmiFuse::push; the bucket must have slab_tiles >= the launch's tiles)
  cme::XgmiFuse* xf_dev = nullptr;  // its device copy (SplitStepArgs::xf): allocated once, so captured graphs stay valid
  // The XCD-local step pipeline (mlp_xstep, csrc/mlp/xstep.hip): run_steps runs the whole plan in ONE persistent
  // launch when the plan's step has the pipeline's shape (H <= 128 split3, fragment-ordered operands, the head's dW2
  // partials, fused SGD, one process, steps on the 16-sample grid); -1 auto (on), 0 off, 1 required (an error if
  // the plan does not qualify).  xstep_bar: XStepPlan::bar (the XCD-local barrier's form).
  int xstep = -1, xstep_bar = 3, xstep_pf = 0;  // xstep_pf: XStepPlan::npf
  int xstep_used = 0;     // the last run_steps ran as one xstep launch (tests, bench records)
  unsigned xs_ep = 1, xs_launch = 0;  // the next step's granule tag; launches so far (control bank)
  unsigned long long *xs_gran = nullptr, *xs_ctl = nullptr;
  float *xs_dx = nullptr, *xs_b2x = nullptr;
  uintptr_t xs_stamps = 0;  // diagnostics: [xs_stamp_steps][8][32][4] uint64 (bench/stamps_xstep.py)
  int xs_stamp_steps = 0;
  ~MlpStep() {
    if (xf_dev) (void)hipFree(xf_dev);
    for (void* q : {(void*)xs_gran, (void*)xs_ctl, (void*)xs_dx, (void*)xs_b2x})
      if (q) (void)hipFree(q);
  }
  void set_xgmi(uintptr_t desc, int64_t slots, int64_t off_b1, int64_t off_W2, int64_t off_b2, int push = 0) {
    if (!desc) {
      xf = cme::XgmiFuse{};  // (the device copy is read only by sgd = 2 launches, which now refuse to run)
      return;
    }
    CME_REQUIRE(split && bias_col && XT, "MlpStep.set_xgmi: split path with the all-ones XT feature only");
    CME_REQUIRE(cme::mlp_split_fused_tiles(P, H, (int)std::min<int64_t>(slots, 1 << 30)) > 0,
                "MlpStep.set_xgmi: the bucket has fewer flag slots than the wgrad launch has tiles");
    const auto* d = reinterpret_cast<const cme::comm::XgmiDesc*>(desc);
    CME_REQUIRE(d->world >= 1 && d->world <= 8 && d->mybuf && d->n >= off_b2 + C,
                "MlpStep.set_xgmi: bucket not open or smaller than the flat gradient");
    cme::XgmiFuse f;
    f.mybuf = d->mybuf;
    for (int r = 0; r < d->world; ++r) {
      CME_REQUIRE(d->peers[r] && d->peerflags[r], "MlpStep.set_xgmi: peer handles not opened");
      f.peers[r] = d->peers[r];
      f.peerflags[r] = d->peerflags[r];
    }
    f.myflags = d->myflags;
    f.epochs = d->epochs;
    f.err = d->err;
    f.rank = d->rank;
    f.world = d->world;
    f.npad = d->npad;
    f.off_b1 = off_b1;
    f.off_W2 = off_W2;
    f.off_b2 = off_b2;
    if (push) {
      CME_REQUIRE(d->myslab && d->slab_tiles >= cme::mlp_split_fused_tiles(P, H, 1 << 30),
                  "MlpStep.set_xgmi(push): the bucket's receive areas are missing or smaller than the launch's tiles");
      f.push = 1;
      f.myslab = d->myslab;
      f.slab_tiles = d->slab_tiles;
      for (int r = 0; r < d->world; ++r) {
        CME_REQUIRE(d->peerslabs[r], "MlpStep.set_xgmi(push): peer receive areas not mapped");
        f.peerslab[r] = d->peerslabs[r];
      }
    }
    xf = f;
    if (!xf_dev) HIP_CHECK(hipMalloc(&xf_dev, sizeof(cme::XgmiFuse)));
    // every launch already enqueued (on any stream, or replayed from a graph) reads the device copy: it finishes
    // before the copy changes under it.  A graph captured against the old bucket must not be replayed afterwards --
    // DataParallelTrainer drops its captured graphs wherever it attaches or detaches a bucket.
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipMemcpy(xf_dev, &xf, sizeof(cme::XgmiFuse), hipMemcpyHostToDevice));
  }
  float xscale = 1.f;    // split path: inputs are uint8 * xscale
  uintptr_t W1p = 0, dZ1p = 0;
  // wide split3 layers: the in-place dW1 update skips the W1-plane refresh (SplitStepArgs::w1_planes_lazy) and
  // planes_stale records it; refresh_planes() re-splits W1 before any forward that reads the planes
  int lazy_planes = 0;
  bool planes_stale = false;
  void refresh_planes(uintptr_t stream) {
    if (!planes_stale) return;
    cme::mlp_split_planes(P_<float>(W1), reinterpret_cast<void*>(W1p), (int64_t)H * P, npw, S(stream));
    planes_stale = false;
  }
  uintptr_t kpart = 0;  // split-K dW1 partial slabs (SplitStepArgs::kpart), kpart_cap floats; 0: no split-K
  int64_t kpart_cap = 0;

  // Binds the engine's buffers and shapes in ONE call (MlpEngine._hip_step): every device pointer, count and
  // layout flag the step reads, by name; an unknown name is an error.  The runtime switches stay plain fields
  // (fh_allgather, store_a1, lazy_planes, ag_*, diagnostics).
  void bind(const py::dict& d) {
    for (const auto& kv : d) {
      const std::string k = py::str(kv.first);
      const py::handle v = kv.second;
      auto u = [&] { return v.cast<uintptr_t>(); };
      auto i = [&] { return v.cast<int>(); };
      if (k == "dt") dt = i(); else if (k == "P") P = i(); else if (k == "H") H = i(); else if (k == "C") C = i();
      else if (k == "ld") ld = i(); else if (k == "N") N = v.cast<int64_t>();
      else if (k == "X") X = u(); else if (k == "labels") labels = u(); else if (k == "XT") XT = u();
      else if (k == "Xw") Xw = u(); else if (k == "XTw") XTw = u();
      else if (k == "W1") W1 = u(); else if (k == "b1") b1 = u(); else if (k == "W2") W2 = u();
      else if (k == "b2") b2 = u(); else if (k == "W1g") W1g = u();
      else if (k == "gW1") gW1 = u(); else if (k == "gb1") gb1 = u(); else if (k == "gW2") gW2 = u();
      else if (k == "gb2") gb2 = u(); else if (k == "gstatus") gstatus = u();
      else if (k == "a1") a1 = u(); else if (k == "D") D = u(); else if (k == "dZ1") dZ1 = u();
      else if (k == "dZ1g") dZ1g = u(); else if (k == "loss") loss = u();
      else if (k == "act") act = i(); else if (k == "split") split = i(); else if (k == "npw") npw = i();
      else if (k == "npz") npz = i(); else if (k == "xscale") xscale = v.cast<float>();
      else if (k == "W1p") W1p = u(); else if (k == "dZ1p") dZ1p = u();
      else if (k == "z2p") z2p = u(); else if (k == "bias_col") bias_col = i();
      else if (k == "fh_counters") fh_counters = u(); else if (k == "fh_tiles") fh_tiles = i();
      else if (k == "ag_counters") ag_counters = u(); else if (k == "ag_slabs") ag_slabs = u();
      else if (k == "ag_gran") ag_gran = u(); else if (k == "ag_gran_count") ag_gran_count = v.cast<int64_t>();
      else if (k == "kpart") kpart = u(); else if (k == "kpart_cap") kpart_cap = v.cast<int64_t>();
      else if (k == "w1s") w1s = u();
      else if (k == "xs") xs = u();
      else if (k == "dz1s") dz1s = u();
      else throw std::invalid_argument("MlpStep.bind: unknown name '" + k + "'");
    }
  }

  cme::SplitStepArgs split_args(int64_t off, int n, double scale, double reg, double lr, int sgd,
                                int with_loss) const {
    cme::SplitStepArgs a;
    a.P = P; a.H = H; a.C = C; a.n = n; a.ld = ld; a.npw = npw; a.npz = npz;
    a.X = reinterpret_cast<const char*>(X) + (size_t)off * P;  // uint8 dataset
    a.XT = reinterpret_cast<const char*>(XT) + (size_t)off;
    a.xscale = xscale;
    a.ldxt = (int)N;
    if (Xw) a.Xw = reinterpret_cast<const char*>(Xw) + (size_t)off * P * 2;
    if (XTw) a.XTw = reinterpret_cast<const char*>(XTw) + (size_t)off * 2;
    a.labels = P_<int>(labels) + off;
    a.W1 = P_<float>(W1); a.b1 = P_<float>(b1); a.W2 = P_<float>(W2); a.b2 = P_<float>(b2);
    a.W1p = reinterpret_cast<void*>(W1p);
    a.gW1 = P_<float>(gW1); a.gb1 = P_<float>(gb1); a.gW2 = P_<float>(gW2); a.gb2 = P_<float>(gb2);
    a.a1 = P_<float>(a1); a.D = P_<float>(D); a.dZ1 = P_<float>(dZ1);
    a.dZ1p = reinterpret_cast<void*>(dZ1p);
    a.loss_partial = with_loss ? P_<float>(loss) : nullptr;
    a.scale = scale; a.reg = reg; a.lr = lr; a.sgd = sgd; a.shift = shift; a.mode = 0;
    a.stamps = reinterpret_cast<unsigned long long*>(stamps);
    a.wstamps = reinterpret_cast<unsigned long long*>(wstamps);
    a.bias_col = bias_col;
    // split3 small layers, measured (bench/kbench.py): fp32 W1 split in registers always (one split per weight
    // per column tile is cheaper than pulling 6 B); fp32 dZ1 above H = 128, where the separate head's plane
    // stores cost ~2 us at H = 300, and -- since round 5 (the head's dW2 partials, the fragment-ordered forward
    // operands and dZ1, dz_swz) -- at H <= 128 from n = 200 columns: the head's three plane stores cost more than the
    // dW1 tiles' re-split (walking step at n = 800 14.24 -> 14.02-14.07 us, n = 512 14.09-14.15 -> 13.33-13.36,
    // n = 400 12.94-12.96 -> 12.67-12.76; n = 100 +0.04-0.16 us, so planes there: profiles/r5/kbench_dz_fp32_r5.jsonl).
    // The decision depends only on the step's shape, so the head and every weight-gradient call of a step agree.
    // (The wide engines always split fp32 operands.)
    a.a_fp32 = a_fp32 >= 0 ? a_fp32 : (H <= 128 ? (n >= 200 ? 3 : 1) : 3);
    a.kpart = P_<float>(kpart);
    a.kpart_cap = kpart_cap;
    // a timed-out all-gather forward + head launch (sticky word) makes every later update a no-op
    a.ag_err = P_<const int>(ag_err);
    a.gstatus = P_<float>(gstatus);
    a.ag_wait_us = ag_wait_us;
    a.ag_test_skip = ag_test_skip;
    a.xcd_rows = xcd_rows && cme::mlp_split_xcd_rows_ok(a) ? 1 : 0;
    if (a.xcd_rows && xcd_pack && cme::mlp_split_xcd_rows_packed_ok(a)) a.xcd_rows = 2;
    a.pf_wgs = (a.xcd_rows && bias_col) ? prefetch : 0;
    a.pf_wgs_xt = (a.xcd_rows && bias_col) ? prefetch_xt : 0;
    a.wide_eng = wide_eng >= 0 ? wide_eng : (npw == 1 ? 1 : 0);
    a.xp_dbg = xp_dbg;
    a.g64_touch = g64_touch;
    return a;
  }

  // Forward + backward for samples [off, off+n) of the resident dataset.
  // sgd=1 applies the update in place (single process); sgd=0 writes the
  // pre-scaled gradients into the bucket for the all-reduce; sgd=2 all-reduces over xGMI and applies
  // the update inside the wgrad launch (set_xgmi, split path).
  // parts: bit0 = forward + head, bit1 = weight gradients / update (profiling hook; default both);
  //        with bit0: +4 skips the head (forward GEMM only), +8 skips the forward GEMM (head only)
  void run(int64_t off, int n, double scale, double reg, double lr, int sgd, int with_loss, uintptr_t stream,
           int parts = 3, int64_t pf_next = -1) {
    CME_REQUIRE(n > 0 && n <= ld, "MlpStep.run: 0 < n <= ld required");
    if (split) {
      CME_REQUIRE(XT != 0 && W1p != 0 && dZ1p != 0, "MlpStep.run: split path needs XT, W1p, dZ1p");
      cme::SplitStepArgs a = split_args(off, n, scale, reg, lr, sgd == 2 ? 0 : sgd, with_loss);
      // the next step's first sample (the native step loop knows it): its pixels are prefetched by this step's
      // weight-gradient launch (SplitStepArgs::pf_X)
      // (only the rows that exist: the next step's shard may be shorter than this one, or past the dataset's end)
      // the forward reads the fragment-ordered W1 copy (rebuilt first if anything but this step's update wrote W1)
      const bool swz = w1_swz && w1s && cme::mlp_fwd_swz_ok(a);
      if (swz) {
        refresh_swz(stream);
        a.w1_swz = 1;
        a.W1s = P_<float>(w1s);
      } else if (sgd) {
        swz_stale = true;  // (this step's update does not write the copy)
      }
      // ... and the pixels from theirs when this step's samples start a 16-sample tile of it
      const int64_t xs_tile = (int64_t)((P + 63) / 64) * 1024;  // bytes per 16 samples
      const bool xsw = swz && x_swz && xs;
      if (xsw && off % 16 == 0) {
        a.x_swz = 1;
        a.Xs = reinterpret_cast<const char*>(xs) + off / 16 * xs_tile;
      }
      if (pf_next >= 0 && pf_next < N && a.pf_wgs) {  // (the copy the next step's forward will read)
        const int64_t rows = std::min<int64_t>(n, N - pf_next);
        if (xsw && pf_next % 16 == 0) {
          a.pf_X = reinterpret_cast<const char*>(xs) + pf_next / 16 * xs_tile;
          a.pf_bytes = (rows + 15) / 16 * xs_tile;
        } else {
          a.pf_X = reinterpret_cast<const char*>(X) + (size_t)pf_next * P;
          a.pf_bytes = rows * P;
        }
      }
      if (sgd == 2) {  // all-reduce + SGD inside the wgrad launch
        CME_REQUIRE(xf.world > 0 && xf_dev, "MlpStep.run(sgd=2): set_xgmi() first");
        a.xf = xf_dev;
        a.xf_world = xf.world;
        a.xf_push = xf.push;
      }
      if (parts & 1) {
        {  // the forward GEMM + the head (fused into one launch where the shapes allow)
          cme::HeadArgs h{};
          h.a1 = a.a1; h.lda = ld; h.W2 = a.W2; h.b2 = a.b2; h.labels = a.labels; h.H = H; h.C = C; h.n = n;
          h.scale = scale; h.D = a.D; h.ldd = ld; h.dZ1 = a.dZ1; h.ldz = ld; h.dZ1_bf16 = nullptr;
          h.dZ1_planes = a.dZ1p; h.npz = npz;
          h.loss_partial = a.loss_partial; h.shift = shift; h.mode = cme::HEAD_TRAIN;
          h.z2part = P_<float>(z2p);
          h.stamps = hstamps ? reinterpret_cast<unsigned long long*>(hstamps) : nullptr;
          // the dW1 GEMM splits fp32 dZ1 in registers: the head writes fp32 dZ1 and no planes
          const bool dz32 = cme::mlp_split_wgrad_fp32_dz(a);
          if (dz32) h.dZ1_planes = nullptr;
          // (the small forms read the planes unless they split fp32 W1 in registers; the wide forms below decide
          // by their kernel)
          if (H < 512 && !cme::mlp_split_fwd_fp32_w(a)) refresh_planes(stream);
          if (fh_allgather && ag_counters && ag_slabs && ag_err && !(parts & 12) && cme::mlp_fwd1_head_ok(a, h) &&
              cme::mlp_fwd1_head_ag_fits(a)) {
            // training (store_a1 off): with the all-ones XT feature the dW1 launch reads only the dZ1 planes (db1 is
            // its column P) unless it splits fp32 dZ1 itself -- the fp32 dZ1 store is then skipped
            cme::HeadArgs hg = h;
            cme::SplitStepArgs fa = a;
            if (!store_a1 && bias_col && !dz32 && hg.dZ1_planes) hg.dZ1 = nullptr;
            if (dz_swz && dz1s && dz32 && swz && (parts & 3) == 3 && !hg.dZ1_planes) {
              cme::SplitStepArgs t = a;
              t.dZ1 = P_<float>(dz1s);
              if (cme::mlp_wgrad_dz_swz_ok(t)) {  // the head writes the fragment-ordered dZ1, the dW1 GEMM reads it
                a.dZ1 = t.dZ1;
                a.dz_swz = 1;
                hg.dZ1 = a.dZ1;
                hg.dz_swz = 1;
              }
            }
            if ((head_dw2 > 0 || (head_dw2 < 0 && n >= 768)) && dw2p && C <= 16) {  // the head leaves the dW2 partials (fha_body step 5); then
              // nothing after this launch reads a1: not stored in training (store_a1 off)
              hg.dw2part = P_<float>(dw2p);
              a.dw2part = hg.dw2part;
              a.dw2_cols = 16;  // (fha_body step 4a: two partials per 32-column tile)
              if (!store_a1) {
                fa.a1 = nullptr;
                hg.a1 = nullptr;
              }
            }
            cme::mlp_fwd1_head_ag(fa, hg, P_<unsigned long long>(ag_counters), P_<unsigned long long>(ag_slabs),
                                  P_<int>(ag_err), fh_tiles, S(stream));
          } else if (fh_counters && !(parts & 12) && cme::mlp_fwd1_head_ok(a, h)) {  // one launch
            cme::mlp_fwd1_head(a, h, P_<unsigned>(fh_counters), fh_tiles, S(stream));
          } else {
            // wide layers: the forward GEMM also leaves the head's z2 partials (unless only the head runs)
            cme::SplitStepArgs f = a;
            f.z2part = (z2p && !(parts & 8)) ? P_<float>(z2p) : nullptr;
            h.z2_chunks = f.z2part ? cme::mlp_split_fwd1_z2_chunks(f) : 0;
            // with the all-ones XT feature nothing reads dZ1 in fp32 on the wide path (db1 comes out of
            // the dW1 GEMM over the planes): skip those 4 B/element of HBM writes
            if (h.z2_chunks > 0 && bias_col) h.dZ1 = nullptr;
            // ... unless the dW1 GEMM splits fp32 dZ1 in registers: then fp32 dZ1 and no planes
            if (dz32) h.dZ1 = a.dZ1;
            if (h.z2_chunks > 0 && dw2p && !(parts & 4)) {  // the head leaves dW2 partials for the wgrad launch
              h.dw2part = P_<float>(dw2p);
              a.dw2part = h.dw2part;
            }
            const bool ag = fh_allgather && ag_counters && ag_err && ag_gran && h.dw2part && !(parts & 12) &&
                            cme::mlp_fwd1_wide_ag_ok(f, h, ag64());
            if (!(parts & 8) && cme::mlp_split_wide_fwd_reads_planes(f, ag, ag64())) refresh_planes(stream);
            if (ag && dz_swz && dz1s && dz32 && h.dZ1 && (parts & 3) == 3) {
              cme::SplitStepArgs t = a;
              t.dZ1 = P_<float>(dz1s);
              if (cme::mlp_wgrad_dzr_ok(t)) {  // the wide head writes dZ1 in the dW1 K loop's fragment order
                a.dZ1 = t.dZ1;
                a.dz_swz = 2;
                h.dZ1 = a.dZ1;
                h.dz_swz = 2;
              }
            }
            if (ag) {  // one launch: forward GEMM + the all-gather head
              a.dw2_cols = cme::mlp_fwd1_wide_ag(f, h, P_<unsigned long long>(ag_counters), fh_tiles,
                                                 P_<unsigned long long>(ag_gran), ag_gran_count, P_<int>(ag_err),
                                                 store_a1, ag64(), S(stream));
            } else {
              if (!(parts & 8)) cme::mlp_split_fwd1(f, S(stream));
              if (!(parts & 4)) cme::mlp_head(DType::F32, h, S(stream));
            }
          }
        }
        // what run_wgrad (the rest of this step's backward) reads: did this forward leave dW2 partials
        dw2_left = a.dw2part != nullptr;
        dz_left_swz = a.dz_swz;
        dw2_cols_last = a.dw2_cols;
      } else if (dw2p && dw2_left) {  // the backward half alone (profiling): the partials of the last forward
        a.dw2part = P_<float>(dw2p);
        a.dw2_cols = dw2_cols_last;
      }
      if (parts & 2) {
        a.w1_planes_lazy = lazy_planes;
        a.w1_planes_lazy = cme::mlp_split_wgrad_leaves_planes_stale(a) ? 1 : 0;  // (only where nothing reads them)
        cme::mlp_split_wgrad(a, S(stream));
        if (a.w1_planes_lazy) planes_stale = true;
      }
      return;
    }
    CME_REQUIRE(sgd != 2, "MlpStep.run(sgd=2): split paths only");
    const DType d = to_dt(dt);
    const size_t xe = d == DType::F64 ? 8 : (d == DType::BF16 ? 2 : 4);
    const void* Xb = reinterpret_cast<const char*>(X) + (size_t)off * P * xe;
    const int* lab = P_<int>(labels) + off;
    if (parts & 1)
      cme::mlp_forward1(d, reinterpret_cast<void*>(W1g), reinterpret_cast<void*>(b1), Xb, P, H, n,
                        reinterpret_cast<void*>(a1), ld, act, S(stream));
    cme::HeadArgs h{};
    h.a1 = reinterpret_cast<void*>(a1); h.lda = ld;
    h.W2 = reinterpret_cast<void*>(W2); h.b2 = reinterpret_cast<void*>(b2);
    h.labels = lab; h.H = H; h.C = C; h.n = n; h.scale = scale;
    h.D = reinterpret_cast<void*>(D); h.ldd = ld;
    h.dZ1 = reinterpret_cast<void*>(dZ1); h.ldz = ld;
    h.dZ1_bf16 = d == DType::BF16 ? reinterpret_cast<void*>(dZ1g) : nullptr;
    h.loss_partial = with_loss ? P_<float>(loss) : nullptr;
    h.shift = shift; h.mode = cme::HEAD_TRAIN;
    h.z2part = P_<float>(z2p);
    if (parts & 1) cme::mlp_head(d, h, S(stream));
    cme::WgradArgs w{};
    w.roles = 7;
    w.dZ1g = reinterpret_cast<void*>(d == DType::BF16 ? dZ1g : dZ1); w.ldz = ld;
    w.X = Xb; w.P = P;
    w.XT = XT ? reinterpret_cast<const char*>(XT) + (size_t)off * xe : nullptr;
    w.ldxt = (int)N;
    w.dZ1 = reinterpret_cast<void*>(dZ1);
    w.D = reinterpret_cast<void*>(D); w.ldd = ld;
    w.a1 = reinterpret_cast<void*>(a1); w.lda = ld;
    w.H = H; w.C = C; w.n = n; w.reg = reg; w.lr = lr; w.sgd = sgd;
    w.W1 = reinterpret_cast<void*>(W1); w.b1 = reinterpret_cast<void*>(b1);
    w.W2 = reinterpret_cast<void*>(W2); w.b2 = reinterpret_cast<void*>(b2);
    w.gW1 = reinterpret_cast<void*>(gW1); w.gb1 = reinterpret_cast<void*>(gb1);
    w.gW2 = reinterpret_cast<void*>(gW2); w.gb2 = reinterpret_cast<void*>(gb2);
    w.W1_bf16 = d == DType::BF16 ? reinterpret_cast<void*>(W1g) : nullptr;
    if (parts & 2) cme::mlp_wgrad(d, w, S(stream));
  }

  // The plan's step as the two-launch form would run it (run(): the all-gather forward + head with the fragment-ordered
  // operands, fp32 dZ1 in fragment order, the head's dW2 partials, SGD fused into the weight-gradient launch), or false
  // when any of those choices would differ -- the XCD-local pipeline then does not apply and run_steps launches per step.
  // grid16: every step of the plan starts a 16-sample tile.  Otherwise (or below 257 columns, where dZ1 has no
  // fragment order) the pipeline's row-major form: the pixels read row-major and fp32 dZ1 row-major -- as run() takes
  // such a step with a_fp32 bit 1 (n = 100 takes dZ1 planes by default there: the pipeline has no plane form).
  const char* xstep_args(int64_t off, int n, double scale, double reg, double lr, uintptr_t stream, bool grid16,
                         cme::SplitStepArgs& a, cme::HeadArgs& h) {
    if (!split || !XT || !W1p || !dZ1p || !w1s || !dw2p || !bias_col) return "not the split3 H <= 128 layout";
    if (!fh_allgather || !ag_counters || !ag_slabs || !ag_err) return "the all-gather forward + head is off";
    if (!w1_swz) return "the fragment-ordered W1 is off";
    // (head_dw2 auto: the pipeline always takes the head's dW2 partials -- its role workgroup sums them; below 768
    // columns the two-launch form forms dW2 in its own role instead, so the bits there match head_dw2 = 1)
    if (C > 16 || head_dw2 == 0) return "the head leaves no dW2 partials";
    a = split_args(off, n, scale, reg, lr, 1, 0);
    if (!cme::mlp_fwd_swz_ok(a) || cme::mlp_split_w1_planes_read(a)) return "the forward would not read fp32 W1";
    a.w1_swz = 1;
    a.W1s = P_<float>(w1s);
    h = cme::HeadArgs{};
    h.a1 = a.a1; h.lda = ld; h.W2 = a.W2; h.b2 = a.b2; h.labels = a.labels; h.H = H; h.C = C;
    h.n = n; h.scale = scale; h.D = a.D; h.ldd = ld; h.dZ1 = a.dZ1; h.ldz = ld; h.dZ1_bf16 = nullptr;
    h.dZ1_planes = nullptr; h.npz = npz; h.loss_partial = nullptr; h.shift = shift; h.mode = cme::HEAD_TRAIN;
    h.z2part = P_<float>(z2p);
    h.stamps = hstamps ? reinterpret_cast<unsigned long long*>(hstamps) : nullptr;  // (diagnostics)
    bool frag = grid16 && x_swz && dz_swz && xs && dz1s && cme::mlp_split_wgrad_fp32_dz(a);
    if (frag) {
      cme::SplitStepArgs t = a;
      t.x_swz = 1;
      t.dZ1 = P_<float>(dz1s);
      frag = cme::mlp_wgrad_dz_swz_ok(t);
    }
    if (frag) {
      a.x_swz = 1;
      a.Xs = reinterpret_cast<const char*>(xs) + off / 16 * ((int64_t)((P + 63) / 64) * 1024);
    } else {
      a.a_fp32 |= 2;  // (fp32 dZ1, row-major)
      if (xs_stamps || hstamps || ag_test_skip >= 0) return "the row-major form has no diagnostics build";
      if (xstep_bar != 3 || xstep_pf != 0) return "the row-major form exists in barrier form 3 only";
      if (!cme::mlp_xstep_rm(a)) return "the row-major form needs n % 4 == 0 and 4-byte aligned pixel columns";
    }
    if (!cme::mlp_fwd1_head_ok(a, h) || !cme::mlp_fwd1_head_ag_fits(a)) return "the all-gather head does not fit";
    if (frag) {
      a.dZ1 = P_<float>(dz1s);
      a.dz_swz = 1;
      h.dz_swz = 1;
    } else {
      a.dz_swz = 0;
      h.dz_swz = 0;
    }
    h.dZ1 = a.dZ1;
    h.dw2part = P_<float>(dw2p);
    a.dw2part = h.dw2part;
    a.dw2_cols = 16;
    if (!store_a1) {  // (run(): nothing after the forward reads a1 once the head leaves the dW2 partials)
      a.a1 = nullptr;
      h.a1 = nullptr;
    }
    if (!cme::mlp_xstep_ok(a, h)) return "mlp_xstep_ok";
    refresh_swz(stream);
    return nullptr;
  }
  std::string xstep_reason = "";  // why the last run_steps did not take the pipeline ("" when it did)

  // the whole plan as one XCD-local pipeline launch; false (nothing enqueued) when the plan does not qualify
  bool run_xstep(int64_t gstart0, int64_t count, int64_t B, int64_t shard_off, int n, int64_t N_end, double scale,
                 double reg, double lr, uintptr_t stream) {
    xstep_reason = "off";
    if (xstep == 0) return false;
    xstep_reason = "the plan's steps start off 4-byte aligned pixel columns";
    if (count <= 0 || count > (1 << 30) || gstart0 % 4 || B % 4 || shard_off % 4) return false;
    const bool grid16 = gstart0 % 16 == 0 && B % 16 == 0 && shard_off % 16 == 0;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIP_CHECK(hipStreamIsCapturing(S(stream), &cap));
    xstep_reason = "the stream is capturing a graph";
    if (cap != hipStreamCaptureStatusNone) return false;  // (granule tags come from the host: never replayed)
    int64_t g0 = gstart0 + B > N_end ? 0 : gstart0;
    cme::SplitStepArgs a;
    cme::HeadArgs h;
    if (const char* why = xstep_args(g0 + shard_off, n, scale, reg, lr, stream, grid16, a, h)) {
      xstep_reason = why;
      return false;
    }
    xstep_reason.clear();
    if (!xs_gran) {
      HIP_CHECK(hipMalloc(&xs_gran, cme::kXstepGranules * 8));
      HIP_CHECK(hipMemset(xs_gran, 0, cme::kXstepGranules * 8));
      HIP_CHECK(hipMalloc(&xs_ctl, cme::kXstepCtlWords * 8));
      HIP_CHECK(hipMemset(xs_ctl, 0, cme::kXstepCtlWords * 8));
      HIP_CHECK(hipMalloc(&xs_dx, (size_t)8 * 16 * ld * 4));
      HIP_CHECK(hipMalloc(&xs_b2x, (size_t)8 * 16 * 4));
      HIP_CHECK(hipDeviceSynchronize());
    }
    cme::XStepPlan p;
    p.gstart0 = gstart0; p.B = B; p.shard_off = shard_off; p.N_end = N_end; p.count = (int)count;
    p.X0 = P_<const uint8_t>(X); p.XT0 = P_<const uint8_t>(XT); p.Xs0 = P_<const uint8_t>(xs);
    p.lab0 = P_<const int>(labels);
    p.xs_tile = (int64_t)((P + 63) / 64) * 1024;
    p.ep0 = xs_ep; p.launch = xs_launch;
    p.gran = xs_gran; p.ctl = xs_ctl; p.Dx = xs_dx; p.b2x = xs_b2x; p.err = P_<int>(ag_err);
    p.nw = cme::mlp_xstep_workers(a);
    p.bar = xstep_bar;
    p.npf = std::max(0, std::min(xstep_pf, 32 - p.nw - 1));
    p.stamps = reinterpret_cast<unsigned long long*>(xs_stamps);
    p.stamp_steps = xs_stamps ? xs_stamp_steps : 0;
    cme::mlp_xstep(a, h, p, S(stream));
    xs_ep += (unsigned)count;
    xs_launch += 1;
    dw2_left = 1;
    dz_left_swz = a.dz_swz;
    dw2_cols_last = 16;
    return true;
  }

  // Native step loop: `count` consecutive global batches of B samples starting at gstart0 (wrapping to 0
  // when a batch would pass N_end), this rank's shard [gstart + shard_off, +n) of each, every kernel
  // launched from here with no Python between steps.  sgd = 1: single process, SGD fused into wgrad;
  // sgd = 2: the xGMI all-reduce + SGD fused into wgrad (set_xgmi).  The eager counterpart of a captured
  // epoch graph: the first kernel starts one launch after the call instead of after a whole-graph
  // submission (bench/launch_overhead.py: ~7 us less fixed cost per timed run, equal per-step cost).
  void run_steps(int64_t gstart0, int64_t count, int64_t B, int64_t shard_off, int n, int64_t N_end, double scale,
                 double reg, double lr, int sgd, uintptr_t stream) {
    CME_REQUIRE(count >= 0 && n > 0 && n <= ld && B >= n && N_end >= B && (sgd == 1 || sgd == 2),
                "MlpStep.run_steps: bad step plan");
    if (count == 0) return;
    xstep_used = sgd == 1 && run_xstep(gstart0, count, B, shard_off, n, N_end, scale, reg, lr, stream) ? 1 : 0;
    CME_REQUIRE(xstep_used || xstep != 1 || sgd != 1,
                "MlpStep.run_steps: xstep = 1 but the plan's step does not qualify: " + xstep_reason);
    if (xstep_used) return;
    int64_t gs = gstart0;
    for (int64_t i = 0; i < count; ++i) {
      if (gs + B > N_end) gs = 0;
      const int64_t nx = gs + B + B > N_end ? 0 : gs + B;  // (the next step's batch, wrap included)
      run(gs + shard_off, n, scale, reg, lr, sgd, 0, stream, 3, nx + shard_off);
      gs += B;
    }
  }

  // Weight-gradient pieces of a step whose forward + head already ran (parts=1): used by the
  // trainer to overlap per-bucket all-reduces with the rest of the backward pass.
  // parts bit0 = dW1 rows [row0, row0+rows), bit1 = dW2 + bias gradients.  Split paths only.
  void run_wgrad(int64_t off, int n, double scale, double reg, double lr, int sgd, int parts, int row0, int rows,
                 uintptr_t stream) {
    CME_REQUIRE(split, "MlpStep.run_wgrad: split (bf16-plane) paths only");
    CME_REQUIRE(n > 0 && n <= ld, "MlpStep.run_wgrad: 0 < n <= ld required");
    cme::SplitStepArgs a = split_args(off, n, scale, reg, lr, sgd, 0);
    if (sgd) swz_stale = true;  // (an in-place update here does not maintain the forward's W1 copy)
    a.wg_parts = parts;
    a.w1_row0 = row0;
    a.w1_rows = rows;
    if (dw2p && dw2_left) {  // the forward + head half (run(parts=1)) of this step left dW2 partials
      a.dw2part = P_<float>(dw2p);
      a.dw2_cols = dw2_cols_last;
    }
    cme::mlp_split_wgrad(a, S(stream));
  }

  // ---- tensor parallel over the hidden dimension (split paths; parallel/tensor_parallel.py)
  // forward GEMM of this rank's hidden shard only; with z2p != 0 the LDS GEMM also leaves the z2 row-tile
  // partials there.  Returns how many it wrote (0: the caller forms W2_s . a1_s itself).
  int tp_forward(int64_t off, int n, uintptr_t z2p_, uintptr_t stream) {
    CME_REQUIRE(split && n > 0 && n <= ld, "MlpStep.tp_forward: split path, 0 < n <= ld");
    cme::SplitStepArgs a = split_args(off, n, 1.0, 0.0, 0.0, 1, 0);
    a.z2part = z2p_ ? P_<float>(z2p_) : nullptr;
    refresh_planes(stream);
    cme::mlp_split_fwd1(a, S(stream));
    return a.z2part ? cme::mlp_split_fwd1_z2_chunks(a) : 0;
  }
  // head on the all-reduced pre-activation z2 ([16][ld], without b2): softmax / loss / D for every
  // column, dZ1 (+ planes) for this rank's hidden rows
  void tp_head(int64_t off, int n, double scale, int with_loss, uintptr_t z2full, uintptr_t stream) {
    CME_REQUIRE(split && n > 0 && n <= ld && z2full, "MlpStep.tp_head: split path, 0 < n <= ld, z2 buffer");
    const cme::SplitStepArgs a = split_args(off, n, scale, 0.0, 0.0, 1, with_loss);
    cme::HeadArgs h{};
    h.a1 = a.a1; h.lda = ld; h.W2 = a.W2; h.b2 = a.b2; h.labels = a.labels; h.H = H; h.C = C; h.n = n;
    h.scale = scale; h.D = a.D; h.ldd = ld; h.dZ1 = a.dZ1; h.ldz = ld; h.dZ1_bf16 = nullptr;
    h.dZ1_planes = a.dZ1p; h.npz = npz; h.loss_partial = a.loss_partial; h.shift = shift;
    h.mode = cme::HEAD_TRAIN;
    h.z2part = P_<float>(z2full);
    h.z2_chunks = 1;
    cme::mlp_head(DType::F32, h, S(stream));
  }

  template <typename T>
  static T* P_(uintptr_t p) { return reinterpret_cast<T*>(p); }
};

}  // namespace

void bind_suite(py::module_& m);  // suite_bindings.cpp
void bind_comm(py::module_& m);   // comm/comm_bindings.cpp

#ifndef CME_HIP_MODULE
#define CME_HIP_MODULE _hip  // (_hip_diag: the diagnostics library, cme213_sp18_amd/_build.py --diag)
#endif
PYBIND11_MODULE(CME_HIP_MODULE, m) {
  m.attr("diag_stamps") = CME_DIAG_STAMPS;
  m.doc() = "cme213_sp18_amd gfx950 HIP kernels (MFMA MLP engine + homework kernel suite)";

  m.def(
      "mlp_forward1",
      [](int dt, uintptr_t W1g, uintptr_t b1, uintptr_t X, int Pd, int H, int n, uintptr_t a1, int lda, int act,
         uintptr_t s) {
        cme::mlp_forward1(to_dt(dt), P<void>(W1g), P<void>(b1), P<void>(X), Pd, H, n, P<void>(a1), lda, act, S(s));
      },
      py::arg("dt"), py::arg("W1g"), py::arg("b1"), py::arg("X"), py::arg("P"), py::arg("H"), py::arg("n"),
      py::arg("a1"), py::arg("lda"), py::arg("act"), py::arg("stream"));

  m.def(
      "mlp_head",
      [](int dt, int mode, uintptr_t a1, int lda, uintptr_t W2, uintptr_t b2, uintptr_t labels, int H, int C,
         int n, double scale, uintptr_t Dp, int ldd, uintptr_t dZ1, int ldz, uintptr_t dZ1_bf16, uintptr_t loss,
         uintptr_t pred, uintptr_t probs, int ldp, int shift, uintptr_t s) {
        cme::HeadArgs h{};
        h.a1 = P<void>(a1); h.lda = lda; h.W2 = P<void>(W2); h.b2 = P<void>(b2);
        h.labels = P<int>(labels); h.H = H; h.C = C; h.n = n; h.scale = scale;
        h.D = P<void>(Dp); h.ldd = ldd; h.dZ1 = P<void>(dZ1); h.ldz = ldz; h.dZ1_bf16 = P<void>(dZ1_bf16);
        h.loss_partial = P<float>(loss); h.pred = P<int>(pred); h.probs = P<void>(probs); h.ldp = ldp;
        h.shift = shift; h.mode = mode;
        cme::mlp_head(to_dt(dt), h, S(s));
      },
      py::arg("dt"), py::arg("mode"), py::arg("a1"), py::arg("lda"), py::arg("W2"), py::arg("b2"),
      py::arg("labels") = 0, py::arg("H"), py::arg("C"), py::arg("n"), py::arg("scale") = 1.0,
      py::arg("D") = 0, py::arg("ldd") = 0, py::arg("dZ1") = 0, py::arg("ldz") = 0, py::arg("dZ1_bf16") = 0,
      py::arg("loss") = 0, py::arg("pred") = 0, py::arg("probs") = 0, py::arg("ldp") = 0,
      py::arg("shift") = 1, py::arg("stream") = 0);
  m.def("mlp_head_num_blocks", &cme::mlp_head_num_blocks);
  m.def("head_big_scratch_floats", &cme::head_big_scratch_floats);

  m.def(
      "mlp_wgrad",
      [](int dt, uintptr_t dZ1g, int ldz, uintptr_t X, int Pd, uintptr_t dZ1, uintptr_t Dp, int ldd, uintptr_t a1,
         int lda, int H, int C, int n, double reg, double lr, int sgd, uintptr_t W1, uintptr_t b1, uintptr_t W2,
         uintptr_t b2, uintptr_t gW1, uintptr_t gb1, uintptr_t gW2, uintptr_t gb2, uintptr_t W1_bf16,
         uintptr_t XT, int ldxt, int roles, uintptr_t s) {
        cme::WgradArgs w{};
        w.XT = P<void>(XT); w.ldxt = ldxt; w.roles = roles;
        w.dZ1g = P<void>(dZ1g); w.ldz = ldz; w.X = P<void>(X); w.P = Pd; w.dZ1 = P<void>(dZ1);
        w.D = P<void>(Dp); w.ldd = ldd; w.a1 = P<void>(a1); w.lda = lda; w.H = H; w.C = C; w.n = n;
        w.reg = reg; w.lr = lr; w.sgd = sgd; w.W1 = P<void>(W1); w.b1 = P<void>(b1); w.W2 = P<void>(W2);
        w.b2 = P<void>(b2); w.gW1 = P<void>(gW1); w.gb1 = P<void>(gb1); w.gW2 = P<void>(gW2);
        w.gb2 = P<void>(gb2); w.W1_bf16 = P<void>(W1_bf16);
        cme::mlp_wgrad(to_dt(dt), w, S(s));
      },
      py::arg("dt"), py::arg("dZ1g"), py::arg("ldz"), py::arg("X"), py::arg("P"), py::arg("dZ1"), py::arg("D"),
      py::arg("ldd"), py::arg("a1"), py::arg("lda"), py::arg("H"), py::arg("C"), py::arg("n"), py::arg("reg"),
      py::arg("lr"), py::arg("sgd"), py::arg("W1"), py::arg("b1"), py::arg("W2"), py::arg("b2"),
      py::arg("gW1") = 0, py::arg("gb1") = 0, py::arg("gW2") = 0, py::arg("gb2") = 0, py::arg("W1_bf16") = 0,
      py::arg("XT") = 0, py::arg("ldxt") = 0, py::arg("roles") = 7, py::arg("stream") = 0);

  m.def(
      "sgd_flat",
      [](int dt, uintptr_t params, uintptr_t grads, int64_t count, double lr, uintptr_t shadow,
         int64_t shadow_count, uintptr_t s) {
        cme::sgd_flat(to_dt(dt), P<void>(params), P<void>(grads), count, lr, P<void>(shadow), shadow_count, S(s));
      },
      py::arg("dt"), py::arg("params"), py::arg("grads"), py::arg("count"), py::arg("lr"), py::arg("shadow") = 0,
      py::arg("shadow_count") = 0, py::arg("stream") = 0);

  m.def(
      "gemm",
      [](int dt, bool tA, bool tB, int M, int N, int K, double alpha, uintptr_t A, int lda, uintptr_t B, int ldb,
         double beta, uintptr_t Cp, int ldc, uintptr_t s) {
        cme::gemm(to_dt(dt), tA, tB, M, N, K, alpha, P<void>(A), lda, P<void>(B), ldb, beta, P<void>(Cp), ldc, S(s));
      },
      py::arg("dt"), py::arg("transA"), py::arg("transB"), py::arg("M"), py::arg("N"), py::arg("K"),
      py::arg("alpha"), py::arg("A"), py::arg("lda"), py::arg("B"), py::arg("ldb"), py::arg("beta"), py::arg("C"),
      py::arg("ldc"), py::arg("stream") = 0);

  m.def(
      "convert_f32_to_bf16",
      [](uintptr_t src, uintptr_t dst, int64_t n, uintptr_t s) {
        cme::convert_f32_to_bf16(P<const float>(src), P<void>(dst), n, S(s));
      },
      py::arg("src"), py::arg("dst"), py::arg("n"), py::arg("stream") = 0);

  py::class_<MlpStep>(m, "MlpStep")
      .def(py::init<>())
      .def("bind", &MlpStep::bind, py::arg("buffers"))
      .def_readonly("dt", &MlpStep::dt)
      .def_readonly("P", &MlpStep::P)
      .def_readonly("H", &MlpStep::H)
      .def_readonly("C", &MlpStep::C)
      .def_readonly("ld", &MlpStep::ld)
      .def_readonly("split", &MlpStep::split)
      .def_readwrite("shift", &MlpStep::shift)
      .def_readwrite("ag_err", &MlpStep::ag_err)
      .def_readwrite("head_dw2", &MlpStep::head_dw2)
      .def_readwrite("fh_allgather", &MlpStep::fh_allgather)
      .def_readwrite("ag_wait_us", &MlpStep::ag_wait_us)
      .def_readwrite("ag_test_skip", &MlpStep::ag_test_skip)
      .def_readwrite("store_a1", &MlpStep::store_a1)
      .def_readwrite("ag_tiles64", &MlpStep::ag_tiles64)
      .def_readwrite("xcd_rows", &MlpStep::xcd_rows)
      .def_readwrite("xcd_pack", &MlpStep::xcd_pack)
      .def_readwrite("w1_swz", &MlpStep::w1_swz)
      .def_readwrite("x_swz", &MlpStep::x_swz)
      .def_readwrite("a_fp32", &MlpStep::a_fp32)
      .def_readwrite("dz_swz", &MlpStep::dz_swz)
      .def_readonly("dz_left_swz", &MlpStep::dz_left_swz)
      .def_readwrite("swz_stale", &MlpStep::swz_stale)
      .def_readwrite("prefetch", &MlpStep::prefetch)
      .def_readwrite("prefetch_xt", &MlpStep::prefetch_xt)
      .def_readwrite("wide_eng", &MlpStep::wide_eng)
      .def_readwrite("xp_dbg", &MlpStep::xp_dbg)
      .def_readwrite("g64_touch", &MlpStep::g64_touch)
      .def_readwrite("xstep", &MlpStep::xstep)
      .def_readwrite("xstep_bar", &MlpStep::xstep_bar)
      .def_readwrite("xstep_pf", &MlpStep::xstep_pf)
      .def_readonly("xstep_used", &MlpStep::xstep_used)
      .def_readonly("xstep_reason", &MlpStep::xstep_reason)
      .def_readwrite("xs_stamps", &MlpStep::xs_stamps)
      .def_readwrite("xs_stamp_steps", &MlpStep::xs_stamp_steps)
      .def_readwrite("lazy_planes", &MlpStep::lazy_planes)
      .def_readwrite("planes_stale", &MlpStep::planes_stale)
      .def_readwrite("dw2p", &MlpStep::dw2p)
      .def_readwrite("stamps", &MlpStep::stamps)
      .def_readwrite("hstamps", &MlpStep::hstamps)
      .def_readwrite("wstamps", &MlpStep::wstamps)
      .def("refresh_planes", &MlpStep::refresh_planes, py::arg("stream"))
      .def("w1_planes_read",
           [](const MlpStep& st) {  // a forward kernel of this step reads the W1 planes (else: not refreshed)
             return st.split != 0 && cme::mlp_split_w1_planes_read(st.split_args(0, st.ld, 1.0, 0.0, 0.0, 1, 0));
           })
      .def("lazy_planes_apply",
           [](const MlpStep& st) {  // this step's in-place W1 update leaves the planes stale (lazy_planes on)
             if (!st.split || !st.lazy_planes) return false;
             cme::SplitStepArgs a = st.split_args(0, st.ld, 1.0, 0.0, 0.0, 1, 0);
             a.w1_planes_lazy = 1;
             return cme::mlp_split_wgrad_leaves_planes_stale(a);
           })
      .def("tp_forward", &MlpStep::tp_forward)
      .def("tp_head", &MlpStep::tp_head)
      .def("set_xgmi", &MlpStep::set_xgmi, py::arg("desc"), py::arg("slots"), py::arg("off_b1"), py::arg("off_W2"),
           py::arg("off_b2"), py::arg("push") = 0)
      .def_property_readonly("xgmi_push", [](const MlpStep& st) { return st.xf.push; })
      .def("run_steps", &MlpStep::run_steps, py::arg("gstart0"), py::arg("count"), py::arg("B"), py::arg("shard_off"),
           py::arg("n"), py::arg("N_end"), py::arg("scale"), py::arg("reg"), py::arg("lr"), py::arg("sgd"),
           py::arg("stream"),
           py::call_guard<py::gil_scoped_release>())
      .def("run_wgrad", &MlpStep::run_wgrad, py::arg("off"), py::arg("n"), py::arg("scale"), py::arg("reg"),
           py::arg("lr"), py::arg("sgd"), py::arg("parts"), py::arg("row0"), py::arg("rows"), py::arg("stream"))
      .def("predict",
           [](MlpStep& st, uintptr_t x, int n, uintptr_t a1buf, int lda, uintptr_t pred, uintptr_t s) {
             // split path forward + argmax for n samples at x (uint8 [n][P]); a1buf: [H][lda] scratch.  The
             // tiled forward (wave-split-K: the wide engines' bf16 copies are of the training set, not of x)
             // into a1buf, then the column head in predict mode
             st.refresh_planes(s);
             cme::SplitStepArgs a = st.split_args(0, n, 1.0, 0.0, 0.0, 0, 0);
             a.X = reinterpret_cast<const void*>(x);
             a.Xw = nullptr;
             a.a1 = reinterpret_cast<float*>(a1buf);
             a.ld = lda;
             cme::mlp_split_fwd1(a, S(s));
             cme::HeadArgs h{};
             h.a1 = a.a1; h.lda = lda; h.W2 = a.W2; h.b2 = a.b2; h.H = st.H; h.C = st.C; h.n = n;
             h.shift = st.shift; h.mode = cme::HEAD_PREDICT; h.pred = reinterpret_cast<int*>(pred);
             cme::mlp_head(DType::F32, h, S(s));
           },
           py::arg("x"), py::arg("n"), py::arg("a1buf"), py::arg("lda"), py::arg("pred"), py::arg("stream"))
      .def("run", &MlpStep::run, py::arg("off"), py::arg("n"), py::arg("scale"), py::arg("reg"), py::arg("lr"),
           py::arg("sgd"), py::arg("with_loss"), py::arg("stream"), py::arg("parts") = 3, py::arg("pf_next") = -1);

  m.def(
      "occupy_cus",
      [](int wgs, int lds_bytes, int64_t ns, uintptr_t s, uintptr_t running) {
        cme::occupy_cus(wgs, lds_bytes, ns, S(s), reinterpret_cast<int*>(running));
      },
      py::arg("wgs"), py::arg("lds_bytes"), py::arg("ns"), py::arg("stream"), py::arg("running") = 0);
  m.def(
      "mlp_split_w1s_floats", [](int H, int Pd) { return cme::mlp_split_w1s_floats(H, Pd); }, py::arg("H"),
      py::arg("P"));

  m.def(
      "split_planes",
      [](uintptr_t W, uintptr_t planes, int64_t n, int np, uintptr_t s) {
        cme::mlp_split_planes(P<const float>(W), P<void>(planes), n, np, S(s));
      },
      py::arg("W"), py::arg("planes"), py::arg("n"), py::arg("np"), py::arg("stream") = 0);
  m.def(
      "split_sgd",
      [](uintptr_t params, uintptr_t grads, int64_t count, double lr, uintptr_t W1p, int64_t w1n, int npw,
         uintptr_t s, uintptr_t status) {
        cme::mlp_split_sgd(P<float>(params), P<const float>(grads), count, lr, P<void>(W1p), w1n, npw, S(s),
                           P<const float>(status));
      },
      py::arg("params"), py::arg("grads"), py::arg("count"), py::arg("lr"), py::arg("W1p"), py::arg("w1n"),
      py::arg("npw"), py::arg("stream") = 0, py::arg("status") = 0);
  m.def("mlp_split_fused_tiles", &cme::mlp_split_fused_tiles, py::arg("P"), py::arg("H"), py::arg("cap"));

  bind_suite(m);
  bind_comm(m);
}
