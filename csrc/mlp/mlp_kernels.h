// Host-side launchers for the fused MLP training step on gfx950.
//
// The reference's per-rank step is 13 separate kernels, each followed by a
// device-wide sync, plus 3 device-to-device copies (fpcode/neural_network.cpp
// :281-394, fpcode/gpu_func.cu:259-466).  Here a step is:
//   K1 mlp_forward1 : a1 = sigmoid(W1 X + b1)                     (MFMA GEMM + fused epilogue)
//   K2 mlp_head     : z2 = W2 a1 + b2, softmax, D = (yhat - y) * scale,
//                     dZ1 = (W2^T D) .* a1 .* (1 - a1), loss partials  (one pass per column)
//   K3 mlp_wgrad    : dW1 = dZ1 X^T + reg W1, dW2 = D a1^T + reg W2, db1, db2 -- all in ONE
//                     launch; either written to the flat gradient bucket (data parallel,
//                     all-reduced next) or applied as SGD in place (single process).
//   (DP only) sgd_flat: params -= lr * grads over the flat [W1|b1|W2|b2] arena.
// No host synchronisation anywhere, so the whole step is HIP-graph capturable.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace cme {

enum class DType : int { F32 = 0, F64 = 1, BF16 = 2 };

// a1[h*lda + b] = act(sum_p W1[h*P + p] * X[b*P + p] + b1[h]),  b < n.
// dt == BF16: W1g and X are bf16, b1/a1 are f32.  Otherwise all of dtype dt.
void mlp_forward1(DType dt, const void* W1g, const void* b1, const void* X, int P, int H, int n, void* a1,
                  int lda, int act, hipStream_t stream);

enum HeadMode : int { HEAD_TRAIN = 0, HEAD_PREDICT = 1, HEAD_PROBS = 2 };

struct HeadArgs {
  const void* a1;  int lda;      // [H][lda], param dtype
  const void* W2;  const void* b2;  // [C][H], [C]
  const int* labels;              // [n] (train mode)
  int H, C, n;
  double scale;                   // D = (yhat - y) * scale, scale = 1/(n*R) (fpcode/neural_network.cpp:333)
  void* D;   int ldd;             // [C][ldd]
  void* dZ1; int ldz;             // [H][ldz]
  void* dZ1_bf16;                 // optional bf16 shadow of dZ1 for the bf16 weight-gradient GEMM
  void* dZ1_planes = nullptr;     // optional exact bf16 planes of dZ1 ([npz][H][ldz]) for the split path
  int npz = 0;
  // the H <= 128 all-gather head (fha_body SWZ & 4): dZ1 is stored in the weight-gradient GEMM's fragment order
  // (mma_tile.h w1s_off over [H][cdiv(ldz, 64) pairs]) instead of row-major -- SplitStepArgs::dz_swz
  int dz_swz = 0;
  float* loss_partial;            // optional: one sum of -log(yhat[label]) per workgroup
  int* pred;                      // predict mode: argmax labels [n]
  void* probs; int ldp;           // probs mode: [C][ldp]
  int shift;                      // 1: max-shifted softmax; 0: reference form (common.cpp:13-18)
  int mode;
  // wide layers (H >= 512, fp32 params, train mode): scratch of head_big_scratch_floats(H, n) floats for the
  // z2 row-tile partial sums the forward GEMM leaves (z2_chunks below)
  float* z2part = nullptr;
  // > 0: z2part already holds z2_chunks row-tile partials [chunk][16][lda] left by the forward GEMM
  // (SplitStepArgs::z2part); the head then only reduces them and never re-reads a1 for z2
  int z2_chunks = 0;
  // diagnostics only: s_memrealtime stamps [block][8] (bench/stamps_fh.py)
  unsigned long long* stamps = nullptr;
  // wide head (z2_chunks > 0) only: when set, each 32-column tile also leaves its dW2 partial
  // dw2part[column tile][16][H] = D[:, tile cols] . a1[:, tile cols]^T (classes < C) for the weight-gradient
  // launch to sum (SplitStepArgs::dw2part)
  float* dw2part = nullptr;
};
int64_t head_big_scratch_floats(int H, int n);

struct SplitStepArgs;
void mlp_head(DType dt, const HeadArgs& a, hipStream_t stream);
// split path, H <= 128: forward GEMM (a1 = sigmoid(W1 X + b1), f) and the train-mode head (h, same a1) in
// ONE launch -- the last workgroup of every 32-column tile runs the head for it.  counters: >= max_tiles
// zero-initialised uint32 (one per 32-column tile; each launch leaves them at 0 again).
bool mlp_fwd1_head_ok(const SplitStepArgs& f, const HeadArgs& h);
void mlp_fwd1_head(const SplitStepArgs& f, const HeadArgs& h, unsigned* counters, int max_tiles, hipStream_t s);
// the same launch in the all-gather form (every row-tile workgroup of a column tile sums the tile's z2
// partials and forms dZ1 for its own rows): counters >= max_tiles * 32 uint64 (one 256-byte line per tile,
// only ever incremented: the launch epoch), slabs >= max_tiles * 8 * 16 * 32 uint64 granules (tags only grow:
// never re-zeroed), err: set to 1 if a poll for the tile's partials timed out
void mlp_fwd1_head_ag(const SplitStepArgs& f, const HeadArgs& h, unsigned long long* counters,
                      unsigned long long* slabs, int* err, int max_tiles, hipStream_t s);
// the all-gather form's grid fits on the device at once (occupancy x CU count): every workgroup waits for the
// others of its column tile, so a larger grid (a large per-GPU batch) must take the last-arriver form
bool mlp_fwd1_head_ag_fits(const SplitStepArgs& f);
// its forward can read the fragment-ordered copies of W1 and of the pixels (SplitStepArgs::w1_swz / x_swz): fp32 W1,
// 16-byte pixel pairs, and K ranges per wave that start on 64-k pair boundaries
bool mlp_fwd_swz_ok(const SplitStepArgs& f);
// TEST SUPPORT (occupy.hip): `wgs` workgroups of `lds_bytes` LDS each, sleeping for `ns` (bounded): keeps CUs busy;
// `running` (host-pinned, may be null) is set to 1 once the first workgroup runs
void occupy_cus(int wgs, int lds_bytes, int64_t ns, hipStream_t s, int* running = nullptr);
int mlp_head_num_blocks(int n);

struct WgradArgs {
  // gemm inputs (bf16 when dt == BF16, else param dtype)
  const void* dZ1g; int ldz;      // [H][ldz]
  const void* X;   int P;         // [n][P] sample-major
  const void* XT;  int ldxt;      // optional feature-major copy X^T [P][ldxt] (shard-offset applied):
                                  // makes the dW1 B operand K-contiguous (16-byte loads)
  // param-dtype inputs
  const void* dZ1;                // [H][ldz] (for db1)
  const void* D;   int ldd;       // [C][ldd]
  const void* a1;  int lda;       // [H][lda]
  int H, C, n;
  double reg, lr;
  int sgd;                        // 1: update params in place; 0: write gradients
  void *W1, *b1, *W2, *b2;        // params (param dtype)
  void *gW1, *gb1, *gW2, *gb2;    // gradient outputs (sgd == 0)
  void* W1_bf16;                  // optional bf16 shadow of W1 refreshed by the in-place update
  int roles = 7;                  // bit0 dW1, bit1 dW2, bit2 bias grads (profiling hook; default all)
};
void mlp_wgrad(DType dt, const WgradArgs& a, hipStream_t stream);

// params[i] -= lr * grads[i] for i < count;  optionally refresh a bf16 shadow of
// the first `shadow_count` params (W1 is first in the flat arena).
void sgd_flat(DType dt, void* params, const void* grads, int64_t count, double lr, void* shadow,
              int64_t shadow_count, hipStream_t stream);

// Column-major GEMM with the reference's myGEMM contract (fpcode/gpu_func.cu:259):
//   C := alpha * op(A) * op(B) + beta * C,  op(X) = X or X^T.
// All four transpose combinations are honoured (the reference silently drops
// BT when AT && BT, gpu_func.cu:263-273).
void gemm(DType dt, bool transA, bool transB, int M, int N, int K, double alpha, const void* A, int lda,
          const void* B, int ldb, double beta, void* C, int ldc, hipStream_t stream);

// Row-major copy with conversion (f32 -> bf16) used to build bf16 shadows.
void convert_f32_to_bf16(const float* src, void* dst, int64_t n, hipStream_t stream);

}  // namespace cme
