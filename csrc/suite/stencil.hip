// hw3: 2-D heat diffusion finite-difference stencil (orders 2/4/8) on gfx950.
//
// Reference: hw3code/gpuStencil.cu (global: one thread per point, 32x6 blocks;
// "block"/loop: 6 rows per thread; shared: EMPTY kernel, never launched).
// Here, wave64-shaped tiles (x is the lane axis -> 256-byte coalesced rows):
//   variant 0 global : one thread per interior point
//   variant 1 loop   : each thread walks ROWS consecutive y points keeping the
//                      2b+1-tall column window in registers (1 new load per row)
//   variant 2 lds    : 256-column strip per wave, register column window for y,
//                      the centre row exchanged through LDS for the x-neighbours
//   variant 3 vec    : 4 x-points per lane with 16-byte loads/stores + the
//                      register column window (fewest instructions per byte)
#include <algorithm>

#include "../common/hip_common.h"
#include "suite_kernels.h"

namespace cme::suite {

namespace {

template <int ORDER>
struct Coef;
template <>
struct Coef<2> {
  static constexpr int B = 1;
  __device__ static constexpr float c(int k) { return k == 0 ? -2.f : 1.f; }
};
template <>
struct Coef<4> {
  static constexpr int B = 2;
  __device__ static constexpr float c(int k) { return k == 0 ? -30.f : (k == 1 || k == -1 ? 16.f : -1.f); }
};
template <>
struct Coef<8> {
  static constexpr int B = 4;
  __device__ static constexpr float c(int k) {
    const int a = k < 0 ? -k : k;
    return a == 0 ? -14350.f : a == 1 ? 8064.f : a == 2 ? -1008.f : a == 3 ? 128.f : -9.f;
  }
};

// value at (x, y) given accessors for the x-line and the y-column.  Explicit FMAs: every kernel that inlines this
// (one-step, two-step, any walk direction) evaluates the same chain -- with contraction left to the compiler the
// one- and two-step walks differed by 1-3 ULP at scattered points (bench/dbg/stencil2_diag.py)
template <int ORDER, class FX, class FY>
__device__ __forceinline__ float apply_stencil(float center, FX fx, FY fy, float xcfl, float ycfl) {
  constexpr int B = Coef<ORDER>::B;
  float sx = 0.f, sy = 0.f;
#pragma unroll
  for (int k = -B; k <= B; ++k) {
    sx = __builtin_fmaf(Coef<ORDER>::c(k), fx(k), sx);
    sy = __builtin_fmaf(Coef<ORDER>::c(k), fy(k), sy);
  }
  return __builtin_fmaf(ycfl, sy, __builtin_fmaf(xcfl, sx, center));
}

template <int ORDER>
__device__ __forceinline__ void stencil_global_body(float* __restrict__ next, const float* __restrict__ curr, int gx,
                                                    int nx, int ny, float xcfl, float ycfl, int bx, int by) {
  constexpr int B = Coef<ORDER>::B;
  const int x = bx * 64 + threadIdx.x;
  const int y = by * 4 + threadIdx.y;
  if (x >= nx || y >= ny) return;
  const int64_t i = (int64_t)(y + B) * gx + (x + B);
  const float* c = curr + i;
  next[i] = apply_stencil<ORDER>(
      c[0], [&](int k) { return c[k]; }, [&](int k) { return c[(int64_t)k * gx]; }, xcfl, ycfl);
}

template <int ORDER, int ROWS>
__device__ __forceinline__ void stencil_loop_body(float* __restrict__ next, const float* __restrict__ curr, int gx,
                                                  int nx, int ny, float xcfl, float ycfl, int bx, int by) {
  constexpr int B = Coef<ORDER>::B;
  constexpr int WIN = 2 * B + 1;
  const int x = bx * 64 + threadIdx.x;
  const int y0 = (by * 4 + threadIdx.y) * ROWS;
  if (x >= nx || y0 >= ny) return;
  const int64_t col = x + B;
  float win[WIN];  // column window rows y-B .. y+B (grid coordinates y0 .. y0+2B)
#pragma unroll
  for (int k = 0; k < WIN - 1; ++k) win[k] = curr[(int64_t)(y0 + k) * gx + col];
#pragma unroll
  for (int r = 0; r < ROWS; ++r) {
    const int y = y0 + r;
    if (y >= ny) break;
    win[WIN - 1] = curr[(int64_t)(y + 2 * B) * gx + col];
    const int64_t i = (int64_t)(y + B) * gx + col;
    const float* c = curr + i;
    next[i] = apply_stencil<ORDER>(
        win[B], [&](int k) { return c[k]; }, [&](int k) { return win[B + k]; }, xcfl, ycfl);
#pragma unroll
    for (int k = 0; k < WIN - 1; ++k) win[k] = win[k + 1];
  }
}

// variant 3 "vec": 4 consecutive x points per lane (16-byte loads / stores), ROWS rows per thread with
// the (2B+1)-tall float4 column window in registers; the x-neighbours of the centre row come from the
// two adjacent float4s (B <= 4).  A wave covers 256 consecutive floats of a row (1 KB per instruction).
// Loads are buffer loads range-checked against the whole grid (4-byte aligned, any B): nothing past
// the allocation is touched and the interior-only stores are masked per element at the right edge.
__device__ __forceinline__ f32x4 ld4(__amdgpu_buffer_rsrc_t r, int64_t elem) {
  const auto w = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(elem * 4), 0, 0);
  return __builtin_bit_cast(f32x4, w);
}

template <int ORDER, int ROWS>
__device__ __forceinline__ void stencil_vec_body(float* __restrict__ next, const float* __restrict__ curr, int gx,
                                                 int gy, int nx, int ny, float xcfl, float ycfl, int bx, int by) {
  constexpr int B = Coef<ORDER>::B;
  constexpr int WIN = 2 * B + 1;
  const int x0 = (bx * 64 + threadIdx.x) * 4;  // first of this lane's 4 interior x
  const int y0 = (by * 4 + threadIdx.y) * ROWS;
  if (x0 >= nx || y0 >= ny) return;
  const __amdgpu_buffer_rsrc_t rc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(curr), (short)0, (int)((int64_t)gx * gy * 4), 0x00020000);
  const int64_t col = x0 + B;
  f32x4 win[WIN];
#pragma unroll
  for (int k = 0; k < WIN - 1; ++k) win[k] = ld4(rc, (int64_t)(y0 + k) * gx + col);
#pragma unroll
  for (int r = 0; r < ROWS; ++r) {
    const int y = y0 + r;
    if (y >= ny) break;
    const int64_t rowc = (int64_t)(y + B) * gx + col;
    win[WIN - 1] = ld4(rc, (int64_t)(y + 2 * B) * gx + col);
    const f32x4 lf = ld4(rc, rowc - 4), rt = ld4(rc, rowc + 4);
    float line[12];  // x = x0 + B - 4 .. x0 + B + 7
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      line[j] = lf[j];
      line[4 + j] = win[B][j];
      line[8 + j] = rt[j];
    }
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      o[j] = apply_stencil<ORDER>(
          line[4 + j], [&](int k) { return line[4 + j + k]; }, [&](int k) { return win[B + k][j]; }, xcfl, ycfl);
    float* dst = next + rowc;
    if (x0 + 4 <= nx && (rowc & 3) == 0) {
      *reinterpret_cast<f32x4*>(dst) = o;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (x0 + j < nx) dst[j] = o[j];
    }
#pragma unroll
    for (int k = 0; k < WIN - 1; ++k) win[k] = win[k + 1];
  }
}

constexpr int kVecRows = 8;

// variant 2 "lds" -- the capability the reference left empty (hw3code/gpuStencil.cu:263-308), built so that every
// grid value is fetched from memory ONCE per sweep and every x-neighbour comes out of LDS:
//   * a wave owns a 256-column strip (4 x points per lane, 16-byte loads) and walks kLdsRows rows down it with the
//     (2b+1)-tall float4 column window in registers (the y-stencil: one new 16-byte load per lane per row);
//   * the centre row goes through the wave's own LDS row buffer (64 float4 + a float4 of halo on each side, loaded
//     by lanes 0 / 63 only), and each lane reads its left / right neighbour float4 back with ds_read_b128 -- the
//     x-stencil costs 1 write + 2 16-byte LDS reads instead of vec's two extra 16-byte global loads per lane per
//     row (the same bytes from L1 / L2 a second and third time);
//   * the row buffer is double-buffered by row parity (one wave barrier per row, no workgroup barrier: the
//     buffer is wave-private), stores are non-temporal (the next grid is written once and read one sweep later,
//     after >> 256 MB of other traffic at the HBM-sized grids);
//   * rows are loaded kLdsAhead rows ahead of their use (a register queue of float4s, halo included): each row's
//     load was otherwise waited for in its own iteration -- one memory latency per row per wave (4096^2 x 400:
//     13.8 -> 13.0 ms);
//   * 32 rows per wave: the 2b rows of y-halo a wave reads beyond its own rows cost 25 % instead of 50 % (order 8).
//     (64 rows on the HBM-sized grids measured the same as 32: 5.54 vs 5.57 ms at 12288^2 x 20.)
constexpr int kLdsRows = 32;
constexpr int kLdsAhead = 4;
constexpr bool kLdsAlt = true;  // the production variant's walk (stencil_lds_body ALT; bench/stencil_tune.py)

// 16-byte load with a cache policy (CP: 0 default, 2 non-temporal: streamed, read once)
template <int CP>
__device__ __forceinline__ f32x4 ld4p(__amdgpu_buffer_rsrc_t r, int64_t elem) {
  const auto w = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(elem * 4), 0, CP);
  return __builtin_bit_cast(f32x4, w);
}

// ALT: waves of odd global index (by * 4 + w) walk their rows bottom-up.  A wave re-reads the 2b rows of y-halo past
// each end of its block; walking down, a block's bottom halo is its lower neighbour's first rows, read ~a block's
// time apart -- long enough at the HBM-sized grids for the XCD's L2 to have dropped them (25 % more HBM reads at
// 32 rows, order 8).  Walking in alternate directions, two neighbouring blocks reach their shared boundary at the
// same time (both at the start, or both at the end), so one of the two reads of each halo row hits L2 (the
// neighbouring workgroup is blockIdx + nbx: the same XCD whenever nbx % 8 == 0, e.g. 12288-wide grids).  The window
// is indexed by grid offset (win[B + dir * k] is row center + k), so every output is the same sum in the same order:
// bitwise the one-direction kernel.
template <int ORDER, int ROWS, int AHEAD = kLdsAhead, int CP = 0, int DIR = 1, bool NTST = true>
__device__ __forceinline__ void stencil_lds_walk(float* __restrict__ next, const float* __restrict__ curr, int gx,
                                                 int gy, int nx, int ny, float xcfl, float ycfl, int bx, int by,
                                                 f32x4 (*xrow)[66]) {
  constexpr int kLdsAhead = AHEAD;
  constexpr int B = Coef<ORDER>::B;
  constexpr int WIN = 2 * B + 1;
  static_assert(B <= 4, "x-neighbours within one float4 of each side");
  const int lane = threadIdx.x, w = threadIdx.y;
  const int x0 = (bx * 64 + lane) * 4;  // first of this lane's 4 interior x
  const int y0 = (by * 4 + w) * ROWS;
  if (y0 >= ny) return;  // wave-uniform (no workgroup barrier below)
  const int nrows = min(ROWS, ny - y0);
  constexpr int dir = DIR;  // (a compile-time walk direction: the window's indices stay static, in registers)
  // interior row of walk step r, and the grid row each step's window gains (its new edge row)
  const int yfirst = dir > 0 ? y0 : y0 + nrows - 1;
  auto ystep = [&](int r) { return yfirst + dir * r; };
  auto qrow = [&](int r) { return ystep(r) + B + dir * B; };
  const __amdgpu_buffer_rsrc_t rc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(curr), (short)0, (int)((int64_t)gx * gy * 4), 0x00020000);
  const int64_t col = x0 + B;
  constexpr int64_t kOffOOB = (int64_t)0x7FFFFFF0 / 4;
  f32x4 win[WIN];  // walk order: win[k] = grid row (center + (k - B) * dir)
#pragma unroll
  for (int k = 0; k < WIN - 1; ++k) win[k] = ld4(rc, (int64_t)(ystep(0) + B + (k - B) * dir) * gx + col);
  // the strip's halo float4s of the centre row: lane 0 the one left of the strip, lane 63 the one right of it
  auto halo = [&](int r) {
    const int64_t rc0 = (int64_t)(ystep(r) + B) * gx + col;
    return ld4p<CP>(rc, r < nrows ? (lane == 0 ? rc0 - 4 : (lane == 63 ? rc0 + 4 : kOffOOB)) : kOffOOB);
  };
  // queues: q[i] = the window's new edge row for walk step i, hq[i] its halo (steps past the block read the
  // range-checked 0 and are never used)
  f32x4 q[kLdsAhead], hq[kLdsAhead];
#pragma unroll
  for (int i = 0; i < kLdsAhead; ++i) {
    q[i] = ld4p<CP>(rc, i < nrows ? (int64_t)qrow(i) * gx + col : kOffOOB);
    hq[i] = halo(i);
  }
  auto wave_sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
#pragma unroll
  for (int r = 0; r < ROWS; ++r) {
    if (r >= nrows) break;
    const int y = ystep(r);
    const int64_t rowc = (int64_t)(y + B) * gx + col;
    win[WIN - 1] = q[0];
    const f32x4 hv = hq[0];
#pragma unroll
    for (int i = 0; i < kLdsAhead - 1; ++i) {
      q[i] = q[i + 1];
      hq[i] = hq[i + 1];
    }
    const int ra = r + kLdsAhead;  // the walk step whose loads go out now
    q[kLdsAhead - 1] = ld4p<CP>(rc, ra < nrows ? (int64_t)qrow(ra) * gx + col : kOffOOB);
    hq[kLdsAhead - 1] = halo(ra);
    f32x4* row = xrow[r & 1];
    row[1 + lane] = win[B];
    if (lane == 0) row[0] = hv;
    if (lane == 63) row[65] = hv;
    wave_sync();
    const f32x4 lf = row[lane], rt = row[lane + 2];
    float line[12];  // x = x0 + B - 4 .. x0 + B + 7
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      line[j] = lf[j];
      line[4 + j] = win[B][j];
      line[8 + j] = rt[j];
    }
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      o[j] = apply_stencil<ORDER>(
          line[4 + j], [&](int k) { return line[4 + j + k]; }, [&](int k) { return win[B + dir * k][j]; }, xcfl,
          ycfl);
    float* dst = next + rowc;
    if (x0 + 4 <= nx && (rowc & 3) == 0) {
      if constexpr (NTST) __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(dst));
      else *reinterpret_cast<f32x4*>(dst) = o;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (x0 + j < nx) dst[j] = o[j];
    }
#pragma unroll
    for (int k = 0; k < WIN - 1; ++k) win[k] = win[k + 1];
  }
}

template <int ORDER, int ROWS, int AHEAD = kLdsAhead, int CP = 0, bool ALT = false, bool NTST = true>
__device__ __forceinline__ void stencil_lds_body(float* __restrict__ next, const float* __restrict__ curr, int gx,
                                                 int gy, int nx, int ny, float xcfl, float ycfl, int bx, int by,
                                                 f32x4 (*xrow)[66]) {
  if (ALT && ((by * 4 + threadIdx.y) & 1))  // (wave-uniform)
    stencil_lds_walk<ORDER, ROWS, AHEAD, CP, -1, NTST>(next, curr, gx, gy, nx, ny, xcfl, ycfl, bx, by, xrow);
  else
    stencil_lds_walk<ORDER, ROWS, AHEAD, CP, 1, NTST>(next, curr, gx, gy, nx, ny, xcfl, ycfl, bx, by, xrow);
}

// variant 4 "lds2" (order 8): TWO time steps per sweep of the grid -- temporal blocking on the LDS walk above, so
// the grid crosses HBM once per two iterations instead of once per iteration.  A wave owns a 256-column strip of the
// INTERMEDIATE grid u1 (4 columns per lane) and writes u2 for the inner 248 columns (lanes 1..62); lanes 0 and 63
// carry u1 only, as the x-halo of the second step (strips overlap by 8 columns: 3 % of the work done twice).  Walking
// down, each new u0 row (loaded kLdsAhead rows ahead) completes a 9-row u0 window: stage 1 forms u1 of its centre
// row -- the stencil, or the boundary condition u0 * scale on the border rows / columns, exactly as the one-step
// launch forms them -- and pushes it into a 9-row u1 window; once that is full, stage 2 forms u2 of ITS centre row.
// The x-neighbours of both stages come from the wave's LDS rows (u0 with the strip's halo float4s; u1 needs none).
// A block of ROWS output rows reads ROWS + 16 u0 rows (the halo of both steps).  Every value is the same expression
// on the same operands as in two one-step launches: bitwise those (tests/test_gpu_suite.py).
template <int ORDER, int ROWS, int AHEAD = kLdsAhead>
__device__ __forceinline__ void stencil_lds2_walk(float* __restrict__ next, const float* __restrict__ curr, int gx,
                                                  int gy, int nx, int ny, float xcfl, float ycfl, float scale, int bx,
                                                  int by, f32x4 (*xr0)[66], f32x4 (*xr1)[66]) {
  constexpr int B = Coef<ORDER>::B;
  static_assert(B == 4, "the two-step walk's strip geometry is order 8's (a float4 of halo per side and step)");
  constexpr int WIN = 2 * B + 1;
  constexpr int OUTW = 256 - 2 * B * 1;  // u2 columns per strip (lanes 1..62)
  const int lane = threadIdx.x, w = threadIdx.y;
  const int s0 = B + OUTW * bx;          // first u2 column of the strip (grid coordinates)
  const int colL = s0 - 4 + 4 * lane;    // this lane's 4 grid columns [colL, colL + 4) of u0 / u1
  const int yo0 = B + (by * 4 + w) * ROWS;
  if (yo0 >= B + ny) return;  // wave-uniform (no workgroup barrier below)
  const int nout = min(ROWS, B + ny - yo0);
  const int g0 = yo0 - 2 * B, nin = nout + 4 * B;  // u0 rows [g0, g0 + nin)
  const __amdgpu_buffer_rsrc_t rc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(curr), (short)0, (int)((int64_t)gx * gy * 4), 0x00020000);
  constexpr int64_t kOffOOB = (int64_t)0x7FFFFFF0 / 4;
  auto at = [&](int g, int col) -> int64_t {
    return (g >= 0 && g < gy && col >= 0) ? (int64_t)g * gx + col : kOffOOB;
  };
  auto centre = [&](int i) { return ld4p<0>(rc, i < nin ? at(g0 + i, colL) : kOffOOB); };
  // the strip's halo float4s (lane 0 the one left of the strip, lane 63 the one right of it) of the u0 window's
  // CENTRE row at iteration i (row g0 + i - B, where stage 1 uses them), queued with the window's new rows
  auto halo = [&](int i) {
    const int g = g0 + i - B;
    return ld4p<0>(rc, i < nin ? (lane == 0 ? at(g, colL - 4) : (lane == 63 ? at(g, colL + 4) : kOffOOB)) : kOffOOB);
  };
  f32x4 q[AHEAD], hq[AHEAD];
#pragma unroll
  for (int i = 0; i < AHEAD; ++i) {
    q[i] = centre(i);
    hq[i] = halo(i);
  }
  f32x4 w0[WIN], w1[WIN];  // w0[k] = u0 row (a - B + k), w1[k] = u1 row (o - B + k)
  auto wave_sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  for (int i = 0; i < nin; ++i) {
#pragma unroll
    for (int k = 0; k < WIN - 1; ++k) w0[k] = w0[k + 1];
    w0[WIN - 1] = q[0];
    const f32x4 hv = hq[0];
#pragma unroll
    for (int k = 0; k < AHEAD - 1; ++k) {
      q[k] = q[k + 1];
      hq[k] = hq[k + 1];
    }
    q[AHEAD - 1] = centre(i + AHEAD);
    hq[AHEAD - 1] = halo(i + AHEAD);
    if (i < 2 * B) continue;  // (uniform) the u0 window is not full yet
    // ---- stage 1: u1 of row a
    const int a = g0 + i - B;
    f32x4* r0 = xr0[i & 1];
    r0[1 + lane] = w0[B];
    if (lane == 0) r0[0] = hv;
    if (lane == 63) r0[65] = hv;
    wave_sync();
    const f32x4 lf = r0[lane], rt = r0[lane + 2];
    const bool brow = a < B || a >= gy - B;
    float line[12];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      line[j] = lf[j];
      line[4 + j] = w0[B][j];
      line[8 + j] = rt[j];
    }
    f32x4 u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = colL + j;
      u[j] = (brow || c < B || c >= gx - B)
                 ? w0[B][j] * scale
                 : apply_stencil<ORDER>(
                       line[4 + j], [&](int k) { return line[4 + j + k]; }, [&](int k) { return w0[B + k][j]; },
                       xcfl, ycfl);
    }
#pragma unroll
    for (int k = 0; k < WIN - 1; ++k) w1[k] = w1[k + 1];
    w1[WIN - 1] = u;
    if (i < 4 * B) continue;  // (uniform) the u1 window is not full yet
    // ---- stage 2: u2 of row o (an interior row of this block)
    const int o = a - B;
    f32x4* r1 = xr1[i & 1];
    r1[1 + lane] = w1[B];
    wave_sync();
    const f32x4 lf1 = r1[lane], rt1 = r1[lane + 2];
    if (lane >= 1 && lane <= 62) {
      float l1[12];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        l1[j] = lf1[j];
        l1[4 + j] = w1[B][j];
        l1[8 + j] = rt1[j];
      }
      f32x4 v;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        v[j] = apply_stencil<ORDER>(
            l1[4 + j], [&](int k) { return l1[4 + j + k]; }, [&](int k) { return w1[B + k][j]; }, xcfl, ycfl);
      const int64_t rowc = (int64_t)o * gx + colL;
      float* dst = next + rowc;
      if (colL + 4 <= B + nx && (rowc & 3) == 0) {
        __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(dst));
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (colL + j < B + nx) dst[j] = v[j];
      }
    }
  }
}

// the border of u2: next = (curr * scale) * scale -- the boundary condition applied twice, as two one-step launches
// apply it (two roundings)
__device__ __forceinline__ void bc2_cells(float* __restrict__ next, const float* __restrict__ curr, int gx, int gy,
                                          int b, float scale, int64_t first, int64_t stride);

template <int ORDER, int ROWS, int AHEAD = kLdsAhead>
__global__ __launch_bounds__(256) void stencil_lds2_fused(float* __restrict__ next, const float* __restrict__ curr,
                                                          int gx, int gy, int nx, int ny, float xcfl, float ycfl,
                                                          int nbx, int nint, float scale) {
  const int id = blockIdx.x;
  if (id >= nint) {
    const int64_t tid = (int64_t)(id - nint) * 256 + threadIdx.y * 64 + threadIdx.x;
    bc2_cells(next, curr, gx, gy, Coef<ORDER>::B, scale, tid, (int64_t)(gridDim.x - nint) * 256);
    return;
  }
  __shared__ f32x4 x0[4][2][66], x1[4][2][66];
  stencil_lds2_walk<ORDER, ROWS, AHEAD>(next, curr, gx, gy, nx, ny, xcfl, ycfl, scale, id % nbx, id / nbx,
                                        x0[threadIdx.y], x1[threadIdx.y]);
}

// border strips: rows [0,b) and [gy-b,gy) (full width), columns [0,b) and [gx-b,gx) of the middle rows;
// `first`/`stride` enumerate the border cells over the calling threads
__device__ __forceinline__ void bc_cells(float* __restrict__ next, const float* __restrict__ curr, int gx, int gy,
                                         int b, float scale, int64_t first, int64_t stride) {
  const int64_t n_top = (int64_t)gx * b;
  const int64_t n_side = (int64_t)(gy - 2 * b) * b;
  const int64_t total = 2 * n_top + 2 * n_side;
  for (int64_t t = first; t < total; t += stride) {
    int64_t idx;
    if (t < n_top) idx = t;
    else if (t < 2 * n_top) idx = (t - n_top) + (int64_t)gx * (gy - b);
    else {
      const int64_t u = t - 2 * n_top;
      const bool left = u < n_side;
      const int64_t v = left ? u : u - n_side;
      const int64_t j = v / b, i = v % b;
      idx = (left ? i : i + (gx - b)) + (int64_t)gx * (b + j);
    }
    next[idx] = curr[idx] * scale;
  }
}

__device__ __forceinline__ void bc2_cells(float* __restrict__ next, const float* __restrict__ curr, int gx, int gy,
                                          int b, float scale, int64_t first, int64_t stride) {
  const int64_t n_top = (int64_t)gx * b;
  const int64_t n_side = (int64_t)(gy - 2 * b) * b;
  const int64_t total = 2 * n_top + 2 * n_side;
  for (int64_t t = first; t < total; t += stride) {
    int64_t idx;
    if (t < n_top) idx = t;
    else if (t < 2 * n_top) idx = (t - n_top) + (int64_t)gx * (gy - b);
    else {
      const int64_t u = t - 2 * n_top;
      const bool left = u < n_side;
      const int64_t v = left ? u : u - n_side;
      const int64_t j = v / b, i = v % b;
      idx = (left ? i : i + (gx - b)) + (int64_t)gx * (b + j);
    }
    const float u1 = curr[idx] * scale;
    next[idx] = u1 * scale;
  }
}

__global__ __launch_bounds__(256) void stencil_bc_kernel(float* __restrict__ next, const float* __restrict__ curr,
                                                         int gx, int gy, int b, float scale) {
  bc_cells(next, curr, gx, gy, b, scale, (int64_t)blockIdx.x * blockDim.x + threadIdx.x,
           (int64_t)gridDim.x * blockDim.x);
}

// Fused iteration: workgroups [0, nint) run the interior variant, the remaining nbc workgroups apply the
// boundary condition -- one launch per time step instead of two (the reference launched BC + stencil).
template <int ORDER, int VARIANT>
__global__ __launch_bounds__(256) void stencil_fused(float* __restrict__ next, const float* __restrict__ curr, int gx,
                                                     int gy, int nx, int ny, float xcfl, float ycfl, int nbx, int nint,
                                                     float scale) {
  const int id = blockIdx.x;
  if (id >= nint) {
    const int64_t tid = (int64_t)(id - nint) * 256 + threadIdx.y * 64 + threadIdx.x;
    bc_cells(next, curr, gx, gy, Coef<ORDER>::B, scale, tid, (int64_t)(gridDim.x - nint) * 256);
    return;
  }
  const int bx = id % nbx, by = id / nbx;
  if constexpr (VARIANT == 0) stencil_global_body<ORDER>(next, curr, gx, nx, ny, xcfl, ycfl, bx, by);
  else if constexpr (VARIANT == 1) stencil_loop_body<ORDER, 8>(next, curr, gx, nx, ny, xcfl, ycfl, bx, by);
  else if constexpr (VARIANT == 2) {
    __shared__ f32x4 xrow[4][2][66];  // per wave: the centre row (+ halo), double-buffered by row parity
    stencil_lds_body<ORDER, kLdsRows, kLdsAhead, 0, kLdsAlt>(next, curr, gx, gy, nx, ny, xcfl, ycfl, bx, by,
                                                            xrow[threadIdx.y]);
  }
  else stencil_vec_body<ORDER, kVecRows>(next, curr, gx, gy, nx, ny, xcfl, ycfl, bx, by);
}

template <int ORDER, int VARIANT>
void launch_v(float* next, const float* curr, int gx, int gy, float xcfl, float ycfl, float scale, bool with_bc,
              hipStream_t s) {
  constexpr int B = Coef<ORDER>::B;
  const int nx = gx - 2 * B, ny = gy - 2 * B;
  const int rows_per_block = VARIANT == 0 ? 4 : (VARIANT == 1 ? 4 * 8 : (VARIANT == 2 ? 4 * kLdsRows : 4 * kVecRows));
  const int cols_per_block = VARIANT >= 2 ? 256 : 64;
  const int nbx = (nx + cols_per_block - 1) / cols_per_block, nby = (ny + rows_per_block - 1) / rows_per_block;
  const int nint = nbx * nby;
  const int64_t bc_cells_total = 2 * ((int64_t)gx * B + (int64_t)(gy - 2 * B) * B);
  const int nbc = with_bc ? (int)std::min<int64_t>((bc_cells_total + 255) / 256, 1024) : 0;
  stencil_fused<ORDER, VARIANT><<<nint + nbc, dim3(64, 4), 0, s>>>(next, curr, gx, gy, nx, ny, xcfl, ycfl, nbx, nint,
                                                                   scale);
}

template <int ORDER>
void launch(float* next, const float* curr, int gx, int gy, float xcfl, float ycfl, int variant, float scale,
            bool with_bc, hipStream_t s) {
  if (variant == 0) launch_v<ORDER, 0>(next, curr, gx, gy, xcfl, ycfl, scale, with_bc, s);
  else if (variant == 1) launch_v<ORDER, 1>(next, curr, gx, gy, xcfl, ycfl, scale, with_bc, s);
  else if (variant == 2) launch_v<ORDER, 2>(next, curr, gx, gy, xcfl, ycfl, scale, with_bc, s);
  else launch_v<ORDER, 3>(next, curr, gx, gy, xcfl, ycfl, scale, with_bc, s);
}

// the LDS variant's knobs, order 8, interior only (bench/stencil_tune.py): rows per wave, rows loaded ahead,
// the streamed loads' cache policy
template <int ROWS, int AHEAD, int CP, bool ALT, bool NTST>
__global__ __launch_bounds__(256) void stencil_lds_tune_kernel(float* __restrict__ next, const float* __restrict__ curr,
                                                               int gx, int gy, int nx, int ny, float xcfl, float ycfl,
                                                               int nbx) {
  __shared__ f32x4 xrow[4][2][66];
  const int id = blockIdx.x;
  stencil_lds_body<8, ROWS, AHEAD, CP, ALT, NTST>(next, curr, gx, gy, nx, ny, xcfl, ycfl, id % nbx, id / nbx,
                                                  xrow[threadIdx.y]);
}

template <int ROWS, int AHEAD, int CP, bool ALT = false, bool NTST = true>
void launch_lds_tune(float* next, const float* curr, int gx, int gy, float xcfl, float ycfl, hipStream_t s) {
  const int nx = gx - 8, ny = gy - 8;
  const int nbx = (nx + 255) / 256, nby = (ny + 4 * ROWS - 1) / (4 * ROWS);
  stencil_lds_tune_kernel<ROWS, AHEAD, CP, ALT, NTST><<<nbx * nby, dim3(64, 4), 0, s>>>(next, curr, gx, gy, nx, ny,
                                                                                        xcfl, ycfl, nbx);
}

}  // namespace

void stencil_lds_tune(float* next, const float* curr, int gx, int gy, float xcfl, float ycfl, int rows, int ahead,
                      int nt, hipStream_t s) {
  CME_REQUIRE((int64_t)gx * gy * 4 < (int64_t)0x7FFFFFF0, "stencil_lds_tune: grid too large for 32-bit offsets");
  // nt bit 0: non-temporal streamed loads, bit 1: alternate walk, bit 2: plain (not non-temporal) stores
  const int key = rows * 100 + ahead * 10 + (nt & 1) + (nt & 2 ? 100000 : 0) + (nt & 4 ? 1000000 : 0);
  switch (key) {
    case 1103240: launch_lds_tune<32, 4, 0, true, false>(next, curr, gx, gy, xcfl, ycfl, s); break;
    case 1103260: launch_lds_tune<32, 6, 0, true, false>(next, curr, gx, gy, xcfl, ycfl, s); break;
    case 1106440: launch_lds_tune<64, 4, 0, true, false>(next, curr, gx, gy, xcfl, ycfl, s); break;
    case 103260: launch_lds_tune<32, 6, 0, true>(next, curr, gx, gy, xcfl, ycfl, s); break;
    case 101640: launch_lds_tune<16, 4, 0, true>(next, curr, gx, gy, xcfl, ycfl, s); break;
    case 103240: launch_lds_tune<32, 4, 0, true>(next, curr, gx, gy, xcfl, ycfl, s); break;
    case 103280: launch_lds_tune<32, 8, 0, true>(next, curr, gx, gy, xcfl, ycfl, s); break;
    case 106480: launch_lds_tune<64, 8, 0, true>(next, curr, gx, gy, xcfl, ycfl, s); break;
    case 101680: launch_lds_tune<16, 8, 0, true>(next, curr, gx, gy, xcfl, ycfl, s); break;
    case 3240: launch_lds_tune<32, 4, 0>(next, curr, gx, gy, xcfl, ycfl, s); break;
    case 3241: launch_lds_tune<32, 4, 2>(next, curr, gx, gy, xcfl, ycfl, s); break;
    case 3280: launch_lds_tune<32, 8, 0>(next, curr, gx, gy, xcfl, ycfl, s); break;
    case 3281: launch_lds_tune<32, 8, 2>(next, curr, gx, gy, xcfl, ycfl, s); break;
    case 6440: launch_lds_tune<64, 4, 0>(next, curr, gx, gy, xcfl, ycfl, s); break;
    case 6480: launch_lds_tune<64, 8, 0>(next, curr, gx, gy, xcfl, ycfl, s); break;
    case 6481: launch_lds_tune<64, 8, 2>(next, curr, gx, gy, xcfl, ycfl, s); break;
    case 12880: launch_lds_tune<128, 8, 0>(next, curr, gx, gy, xcfl, ycfl, s); break;
    case 12881: launch_lds_tune<128, 8, 2>(next, curr, gx, gy, xcfl, ycfl, s); break;
    default: CME_REQUIRE(false, "stencil_lds_tune: (rows, ahead, nt) not instantiated");
  }
  CME_LAUNCH_CHECK(s);
}

void stencil_step(float* next, const float* curr, int gx, int gy, int order, float xcfl, float ycfl, int variant,
                  hipStream_t s) {
  stencil_step_bc(next, curr, gx, gy, order, xcfl, ycfl, variant, 1.f, false, s);
}

void stencil_step_bc(float* next, const float* curr, int gx, int gy, int order, float xcfl, float ycfl, int variant,
                     float scale, bool with_bc, hipStream_t s) {
  CME_REQUIRE(variant >= 0 && variant <= 3, "stencil_step: variant 0 (global), 1 (loop), 2 (lds), 3 (vec)");
  CME_REQUIRE((int64_t)gx * gy * 4 < (int64_t)0x7FFFFFF0, "stencil_step: grid too large for 32-bit buffer offsets");
  switch (order) {
    case 2: launch<2>(next, curr, gx, gy, xcfl, ycfl, variant, scale, with_bc, s); break;
    case 4: launch<4>(next, curr, gx, gy, xcfl, ycfl, variant, scale, with_bc, s); break;
    case 8: launch<8>(next, curr, gx, gy, xcfl, ycfl, variant, scale, with_bc, s); break;
    default: CME_REQUIRE(false, "stencil_step: order must be 2, 4 or 8");
  }
  CME_LAUNCH_CHECK(s);
}

namespace {
template <int ROWS, int AHEAD>
void launch_lds2(float* next, const float* curr, int gx, int gy, float xcfl, float ycfl, float scale, hipStream_t s) {
  constexpr int B = 4;
  const int nx = gx - 2 * B, ny = gy - 2 * B;
  const int nbx = (nx + 247) / 248, nby = (ny + 4 * ROWS - 1) / (4 * ROWS);
  const int nint = nbx * nby;
  const int64_t bc_cells_total = 2 * ((int64_t)gx * B + (int64_t)(gy - 2 * B) * B);
  const int nbc = (int)std::min<int64_t>((bc_cells_total + 255) / 256, 1024);
  stencil_lds2_fused<8, ROWS, AHEAD><<<nint + nbc, dim3(64, 4), 0, s>>>(next, curr, gx, gy, nx, ny, xcfl, ycfl, nbx,
                                                                        nint, scale);
}
}  // namespace

void stencil_step2_bc(float* next, const float* curr, int gx, int gy, int order, float xcfl, float ycfl, float scale,
                      hipStream_t s, int rows, int ahead) {
  CME_REQUIRE(order == 8, "stencil_step2_bc: the two-step LDS walk is built for order 8");
  CME_REQUIRE((int64_t)gx * gy * 4 < (int64_t)0x7FFFFFF0, "stencil_step2_bc: grid too large for 32-bit buffer offsets");
  CME_REQUIRE(gx > 8 && gy > 8, "stencil_step2_bc: grid smaller than its border");
  if (rows <= 0) {  // rows per wave: one round of resident workgroups (~4 per CU) with >= 2 per CU if any does
    // (bench/stencil_tune.py --forms two_step, profiles/r6/stencil/: 4096^2 -> 32, 8192^2 -> 96, 12288^2 -> 64)
    const int nbx = (gx - 8 + 247) / 248;
    auto wgs = [&](int r) { return nbx * ((gy - 8 + 4 * r - 1) / (4 * r)); };
    rows = 64;
    for (int r : {96, 64, 32})
      if (wgs(r) >= 512 && wgs(r) <= 1024) {
        rows = r;
        break;
      }
    if (wgs(32) < 512) rows = 32;
  }
  if (ahead <= 0) ahead = 2;  // (2 rows of loads ahead: fewer registers, more waves -- faster than 4 at every size)
  // (rows, ahead): the production choice and the tuning grid of bench/stencil_tune.py --two-step
  switch (rows * 10 + ahead) {
    case 644: launch_lds2<64, 4>(next, curr, gx, gy, xcfl, ycfl, scale, s); break;
    case 642: launch_lds2<64, 2>(next, curr, gx, gy, xcfl, ycfl, scale, s); break;
    case 324: launch_lds2<32, 4>(next, curr, gx, gy, xcfl, ycfl, scale, s); break;
    case 964: launch_lds2<96, 4>(next, curr, gx, gy, xcfl, ycfl, scale, s); break;
    case 1284: launch_lds2<128, 4>(next, curr, gx, gy, xcfl, ycfl, scale, s); break;
    case 1282: launch_lds2<128, 2>(next, curr, gx, gy, xcfl, ycfl, scale, s); break;
    case 322: launch_lds2<32, 2>(next, curr, gx, gy, xcfl, ycfl, scale, s); break;
    case 643: launch_lds2<64, 3>(next, curr, gx, gy, xcfl, ycfl, scale, s); break;
    case 641: launch_lds2<64, 1>(next, curr, gx, gy, xcfl, ycfl, scale, s); break;
    case 962: launch_lds2<96, 2>(next, curr, gx, gy, xcfl, ycfl, scale, s); break;
    default: CME_REQUIRE(false, "stencil_step2_bc: (rows, ahead) not instantiated");
  }
  CME_LAUNCH_CHECK(s);
}

void stencil_bc(float* next, const float* curr, int gx, int gy, int b, float scale, hipStream_t s) {
  const int64_t total = 2 * ((int64_t)gx * b + (int64_t)(gy - 2 * b) * b);
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 4096));
  stencil_bc_kernel<<<grid, 256, 0, s>>>(next, curr, gx, gy, b, scale);
  CME_LAUNCH_CHECK(s);
}

}  // namespace cme::suite
