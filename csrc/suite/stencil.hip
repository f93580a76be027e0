// hw3: 2-D heat diffusion finite-difference stencil (orders 2/4/8) on gfx950.
//
// Reference: hw3code/gpuStencil.cu (global: one thread per point, 32x6 blocks;
// "block"/loop: 6 rows per thread; shared: EMPTY kernel, never launched).
// Here, wave64-shaped tiles (x is the lane axis -> 256-byte coalesced rows):
//   variant 0 global : one thread per interior point
//   variant 1 loop   : each thread walks ROWS consecutive y points keeping the
//                      2b+1-tall column window in registers (1 new load per row)
//   variant 2 lds    : (64 x 16) tile + b-wide halo staged in LDS, every
//                      stencil read served from LDS
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

// value at (x, y) given accessors for the x-line and the y-column
template <int ORDER, class FX, class FY>
__device__ __forceinline__ float apply_stencil(float center, FX fx, FY fy, float xcfl, float ycfl) {
  constexpr int B = Coef<ORDER>::B;
  float sx = 0.f, sy = 0.f;
#pragma unroll
  for (int k = -B; k <= B; ++k) {
    sx += Coef<ORDER>::c(k) * fx(k);
    sy += Coef<ORDER>::c(k) * fy(k);
  }
  return center + xcfl * sx + ycfl * sy;
}

template <int ORDER>
__global__ __launch_bounds__(256) void stencil_global(float* __restrict__ next, const float* __restrict__ curr,
                                                      int gx, int nx, int ny, float xcfl, float ycfl) {
  constexpr int B = Coef<ORDER>::B;
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= nx || y >= ny) return;
  const int64_t i = (int64_t)(y + B) * gx + (x + B);
  const float* c = curr + i;
  next[i] = apply_stencil<ORDER>(
      c[0], [&](int k) { return c[k]; }, [&](int k) { return c[(int64_t)k * gx]; }, xcfl, ycfl);
}

template <int ORDER, int ROWS>
__global__ __launch_bounds__(256) void stencil_loop(float* __restrict__ next, const float* __restrict__ curr,
                                                    int gx, int nx, int ny, float xcfl, float ycfl) {
  constexpr int B = Coef<ORDER>::B;
  constexpr int WIN = 2 * B + 1;
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y0 = (blockIdx.y * 4 + threadIdx.y) * ROWS;
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

constexpr int kTX = 64, kTY = 16;

template <int ORDER>
__global__ __launch_bounds__(256) void stencil_lds(float* __restrict__ next, const float* __restrict__ curr, int gx,
                                                   int gy, int nx, int ny, float xcfl, float ycfl) {
  constexpr int B = Coef<ORDER>::B;
  constexpr int W = kTX + 2 * B, Hh = kTY + 2 * B;
  __shared__ float tile[Hh][W + 1];
  const int bx = blockIdx.x * kTX, by = blockIdx.y * kTY;  // interior-coordinate origin
  // stage the tile + halo: grid rows by .. by+Hh-1, cols bx .. bx+W-1 (grid coordinates)
  for (int idx = threadIdx.y * 64 + threadIdx.x; idx < Hh * W; idx += 256) {
    const int r = idx / W, cc = idx - r * W;
    const int gr = by + r, gc = bx + cc;
    tile[r][cc] = (gr < gy && gc < gx) ? curr[(int64_t)gr * gx + gc] : 0.f;
  }
  __syncthreads();
  const int lx = threadIdx.x;
  for (int ly = threadIdx.y; ly < kTY; ly += 4) {
    const int x = bx + lx, y = by + ly;
    if (x < nx && y < ny) {
      const int tr = ly + B, tc = lx + B;
      next[(int64_t)(y + B) * gx + (x + B)] = apply_stencil<ORDER>(
          tile[tr][tc], [&](int k) { return tile[tr][tc + k]; }, [&](int k) { return tile[tr + k][tc]; }, xcfl,
          ycfl);
    }
  }
}

__global__ __launch_bounds__(256) void stencil_bc_kernel(float* __restrict__ next, const float* __restrict__ curr,
                                                         int gx, int gy, int b, float scale) {
  // border strips: rows [0,b) and [gy-b,gy) (full width), columns [0,b) and [gx-b,gx) of the middle rows
  const int64_t n_top = (int64_t)gx * b;
  const int64_t n_side = (int64_t)(gy - 2 * b) * b;
  const int64_t total = 2 * n_top + 2 * n_side;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
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

template <int ORDER>
void launch(float* next, const float* curr, int gx, int gy, float xcfl, float ycfl, int variant, hipStream_t s) {
  constexpr int B = Coef<ORDER>::B;
  const int nx = gx - 2 * B, ny = gy - 2 * B;
  const dim3 block(64, 4);
  if (variant == 0) {
    stencil_global<ORDER><<<dim3((nx + 63) / 64, (ny + 3) / 4), block, 0, s>>>(next, curr, gx, nx, ny, xcfl, ycfl);
  } else if (variant == 1) {
    constexpr int ROWS = 8;
    stencil_loop<ORDER, ROWS>
        <<<dim3((nx + 63) / 64, (ny + 4 * ROWS - 1) / (4 * ROWS)), block, 0, s>>>(next, curr, gx, nx, ny, xcfl, ycfl);
  } else {
    stencil_lds<ORDER><<<dim3((nx + kTX - 1) / kTX, (ny + kTY - 1) / kTY), block, 0, s>>>(next, curr, gx, gy, nx, ny,
                                                                                         xcfl, ycfl);
  }
}

}  // namespace

void stencil_step(float* next, const float* curr, int gx, int gy, int order, float xcfl, float ycfl, int variant,
                  hipStream_t s) {
  CME_REQUIRE(variant >= 0 && variant <= 2, "stencil_step: variant 0 (global), 1 (loop), 2 (lds)");
  switch (order) {
    case 2: launch<2>(next, curr, gx, gy, xcfl, ycfl, variant, s); break;
    case 4: launch<4>(next, curr, gx, gy, xcfl, ycfl, variant, s); break;
    case 8: launch<8>(next, curr, gx, gy, xcfl, ycfl, variant, s); break;
    default: CME_REQUIRE(false, "stencil_step: order must be 2, 4 or 8");
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
