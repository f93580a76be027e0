// Native CPU side of the homework suite: the OpenMP algorithms of hw1 and the
// host references / oracles of hw2-hw4 (the GPU kernels are in csrc/suite).
//
// hw1 radix-sort stage functions keep the reference's decomposition
// (hw1code/main_q2.cpp:26-159) so the golden stage fixtures can be checked
// stage by stage; the implementation is our own (OpenMP, flat vectors).
#include "suite_cpu.h"

#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace cme::cpu::suite {

// ------------------------------------------------------------- hw1 sums
std::pair<uint64_t, uint64_t> sum_even_odd_serial(const uint32_t* v, int64_t n) {
  uint64_t e = 0, o = 0;
  for (int64_t i = 0; i < n; ++i) (v[i] & 1u ? o : e) += v[i];
  return {e, o};
}

std::pair<uint64_t, uint64_t> sum_even_odd_parallel(const uint32_t* v, int64_t n) {
  uint64_t e = 0, o = 0;
#pragma omp parallel for reduction(+ : e, o) schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t x = v[i];
    if (x & 1u) o += x;
    else e += x;
  }
  return {e, o};
}

// ------------------------------------------------------------- hw1 radix
u32vec block_histograms(const uint32_t* keys, int64_t n, int num_blocks, int num_buckets, int start_bit,
                        int64_t block_size) {
  u32vec h((size_t)num_blocks * num_buckets, 0);
  const uint32_t mask = (uint32_t)num_buckets - 1;
#pragma omp parallel for schedule(static)
  for (int b = 0; b < num_blocks; ++b) {
    const int64_t lo = (int64_t)b * block_size, hi = std::min<int64_t>(n, lo + block_size);
    uint32_t* hb = h.data() + (size_t)b * num_buckets;
    for (int64_t i = lo; i < hi; ++i) ++hb[(keys[i] >> start_bit) & mask];
  }
  return h;
}

u32vec reduce_to_global(const u32vec& bh, int num_blocks, int num_buckets) {
  u32vec g(num_buckets, 0);
  for (int b = 0; b < num_blocks; ++b)
    for (int k = 0; k < num_buckets; ++k) g[k] += bh[(size_t)b * num_buckets + k];
  return g;
}

u32vec exclusive_scan(const u32vec& g) {
  u32vec s(g.size(), 0);
  for (size_t i = 1; i < g.size(); ++i) s[i] = s[i - 1] + g[i - 1];
  return s;
}

u32vec block_exscan(int num_buckets, int num_blocks, const u32vec& gscan, const u32vec& bh) {
  u32vec o((size_t)num_blocks * num_buckets, 0);
  for (int k = 0; k < num_buckets; ++k) {
    uint32_t run = gscan[k];
    for (int b = 0; b < num_blocks; ++b) {
      o[(size_t)b * num_buckets + k] = run;
      run += bh[(size_t)b * num_buckets + k];
    }
  }
  return o;
}

void populate(const u32vec& bex, int num_blocks, int num_buckets, int start_bit, int64_t block_size,
              const uint32_t* keys, int64_t n, uint32_t* sorted) {
  const uint32_t mask = (uint32_t)num_buckets - 1;
#pragma omp parallel for schedule(static)
  for (int b = 0; b < num_blocks; ++b) {
    std::vector<uint32_t> pos(bex.begin() + (size_t)b * num_buckets, bex.begin() + (size_t)(b + 1) * num_buckets);
    const int64_t lo = (int64_t)b * block_size, hi = std::min<int64_t>(n, lo + block_size);
    for (int64_t i = lo; i < hi; ++i) sorted[pos[(keys[i] >> start_bit) & mask]++] = keys[i];
  }
}

void radix_parallel_pass(const uint32_t* keys, uint32_t* sorted, int64_t n, int num_bits, int start_bit,
                         int64_t block_size) {
  const int nb = (int)((n + block_size - 1) / block_size);
  const int buckets = 1 << num_bits;
  const u32vec bh = block_histograms(keys, n, nb, buckets, start_bit, block_size);
  const u32vec g = reduce_to_global(bh, nb, buckets);
  const u32vec gs = exclusive_scan(g);
  const u32vec bex = block_exscan(buckets, nb, gs, bh);
  populate(bex, nb, buckets, start_bit, block_size, keys, n, sorted);
}

void radix_parallel(uint32_t* keys, uint32_t* tmp, int64_t n, int num_bits, int num_blocks) {
  const int64_t bs = std::max<int64_t>(1, (n + num_blocks - 1) / num_blocks);
  for (int sb = 0; sb < 32; sb += 2 * num_bits) {
    radix_parallel_pass(keys, tmp, n, num_bits, sb, bs);
    radix_parallel_pass(tmp, keys, n, num_bits, sb + num_bits, bs);
  }
}

void radix_serial(uint32_t* keys, uint32_t* tmp, int64_t n, int num_bits) {
  const int buckets = 1 << num_bits;
  const uint32_t mask = (uint32_t)buckets - 1;
  std::vector<uint32_t> cnt(buckets);
  auto pass = [&](const uint32_t* in, uint32_t* out, int sb) {
    std::fill(cnt.begin(), cnt.end(), 0);
    for (int64_t i = 0; i < n; ++i) ++cnt[(in[i] >> sb) & mask];
    uint32_t run = 0;
    for (int k = 0; k < buckets; ++k) {
      const uint32_t c = cnt[k];
      cnt[k] = run;
      run += c;
    }
    for (int64_t i = 0; i < n; ++i) out[cnt[(in[i] >> sb) & mask]++] = in[i];
  };
  for (int sb = 0; sb < 32; sb += 2 * num_bits) {
    pass(keys, tmp, sb);
    pass(tmp, keys, sb + num_bits);
  }
}

// ------------------------------------------------------------- hw3 stencil
static float stencil_point(const float* c, int64_t gx, int order, float xcfl, float ycfl) {
  // same coefficient order as the GPU kernels (csrc/suite/stencil.hip)
  static const float c2[3] = {1.f, -2.f, 1.f};
  static const float c4[5] = {-1.f, 16.f, -30.f, 16.f, -1.f};
  static const float c8[9] = {-9.f, 128.f, -1008.f, 8064.f, -14350.f, 8064.f, -1008.f, 128.f, -9.f};
  const int B = order / 2;
  const float* co = order == 2 ? c2 : (order == 4 ? c4 : c8);
  float sx = 0.f, sy = 0.f;
  for (int k = -B; k <= B; ++k) {
    sx += co[k + B] * c[k];
    sy += co[k + B] * c[(int64_t)k * gx];
  }
  return c[0] + xcfl * sx + ycfl * sy;
}

void stencil_cpu(float* grid, int gx, int gy, int order, float xcfl, float ycfl, float bc_scale, int iters) {
  const int B = order / 2;
  std::vector<float> next(grid, grid + (size_t)gx * gy);
  float* cur = grid;
  float* nxt = next.data();
  for (int it = 0; it < iters; ++it) {
    // border of next = border of curr * scale   (the GPU's convention; the reference's
    // CPU code updated curr's border from next, one step out of phase: hw3code/main.cu:184)
    for (int y = 0; y < gy; ++y)
      for (int x = 0; x < gx; ++x)
        if (y < B || y >= gy - B || x < B || x >= gx - B) nxt[(int64_t)y * gx + x] = cur[(int64_t)y * gx + x] * bc_scale;
#pragma omp parallel for schedule(static)
    for (int y = B; y < gy - B; ++y)
      for (int x = B; x < gx - B; ++x) {
        const int64_t i = (int64_t)y * gx + x;
        nxt[i] = stencil_point(cur + i, gx, order, xcfl, ycfl);
      }
    std::swap(cur, nxt);
  }
  if (cur != grid) std::memcpy(grid, cur, sizeof(float) * (size_t)gx * gy);
}

// ------------------------------------------------------------- hw2 pagerank
void pagerank_cpu(const uint32_t* indptr, const uint32_t* edges, const float* inv, float* vals, int n, int iters) {
  std::vector<float> other(vals, vals + n);
  float* in = vals;
  float* out = other.data();
  for (int it = 0; it < iters; ++it) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
      float sum = 0.f;
      for (uint32_t j = indptr[i]; j < indptr[i + 1]; ++j) sum += in[edges[j]] * inv[edges[j]];
      out[i] = 0.5f / (float)n + 0.5f * sum;
    }
    std::swap(in, out);
  }
  if (in != vals) std::memcpy(vals, in, sizeof(float) * n);
}

}  // namespace cme::cpu::suite
