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

// Software write-combining for the scatter: each bucket's next keys are staged in a 64-byte (one cache
// line) slot of a per-thread buffer and written out a full line at a time, so the 2^num_bits scattered
// output streams cost one line write each per 16 keys instead of a read-for-ownership per key.  Used when
// the slots fit in ~L2 (<= 4096 buckets: 256 KB); larger digits scatter directly.
namespace {
constexpr int kWc = 16;  // keys per slot (64 bytes)
constexpr int kWcMaxBuckets = 4096;

struct WcScatter {
  std::vector<uint32_t> buf;  // [bucket][kWc]
  std::vector<uint8_t> fill;  // keys staged per bucket
  uint32_t* pos;              // next output index per bucket (advanced as lines are written)
  uint32_t* out;
  WcScatter(int buckets, uint32_t* pos_, uint32_t* out_)
      : buf((size_t)buckets * kWc), fill(buckets, 0), pos(pos_), out(out_) {}
  inline void put(uint32_t b, uint32_t key) {
    uint32_t* slot = buf.data() + (size_t)b * kWc;
    slot[fill[b]++] = key;
    if (fill[b] == kWc) {
      std::memcpy(out + pos[b], slot, kWc * sizeof(uint32_t));
      pos[b] += kWc;
      fill[b] = 0;
    }
  }
  void flush(int buckets) {
    for (int b = 0; b < buckets; ++b) {
      std::memcpy(out + pos[b], buf.data() + (size_t)b * kWc, fill[b] * sizeof(uint32_t));
      pos[b] += fill[b];
      fill[b] = 0;
    }
  }
};

// stable scatter of keys[lo, hi) by digit (keys >> start_bit) & mask to out[pos[digit]++]
void scatter_range(const uint32_t* keys, int64_t lo, int64_t hi, int start_bit, uint32_t mask, int buckets,
                   uint32_t* pos, uint32_t* out) {
  if (buckets <= kWcMaxBuckets && hi - lo >= 8 * (int64_t)buckets) {
    WcScatter wc(buckets, pos, out);
    for (int64_t i = lo; i < hi; ++i) wc.put((keys[i] >> start_bit) & mask, keys[i]);
    wc.flush(buckets);
  } else {
    for (int64_t i = lo; i < hi; ++i) out[pos[(keys[i] >> start_bit) & mask]++] = keys[i];
  }
}
}  // namespace

void populate(const u32vec& bex, int num_blocks, int num_buckets, int start_bit, int64_t block_size,
              const uint32_t* keys, int64_t n, uint32_t* sorted) {
  const uint32_t mask = (uint32_t)num_buckets - 1;
#pragma omp parallel for schedule(static)
  for (int b = 0; b < num_blocks; ++b) {
    std::vector<uint32_t> pos(bex.begin() + (size_t)b * num_buckets, bex.begin() + (size_t)(b + 1) * num_buckets);
    const int64_t lo = (int64_t)b * block_size, hi = std::min<int64_t>(n, lo + block_size);
    scatter_range(keys, lo, hi, start_bit, mask, num_buckets, pos.data(), sorted);
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

// Serial LSD sort: every digit's histogram from ONE read of the keys, passes whose digit is the same for
// every key skipped, write-combined scatter.  num_bits divides 32 in pairs of passes (ping-pong), as the
// reference's loop does (hw1code/main_q2.cpp:174-206).
void radix_serial(uint32_t* keys, uint32_t* tmp, int64_t n, int num_bits) {
  const int buckets = 1 << num_bits;
  const uint32_t mask = (uint32_t)buckets - 1;
  const int passes = (32 + num_bits - 1) / num_bits;
  std::vector<uint32_t> hist((size_t)passes * buckets, 0);
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t k = keys[i];
    for (int p = 0; p < passes; ++p) ++hist[(size_t)p * buckets + ((k >> (p * num_bits)) & mask)];
  }
  uint32_t* in = keys;
  uint32_t* out = tmp;
  for (int p = 0; p < passes; ++p) {
    uint32_t* h = hist.data() + (size_t)p * buckets;
    bool trivial = false;
    uint32_t run = 0;
    for (int k = 0; k < buckets; ++k) {
      const uint32_t c = h[k];
      trivial |= c == (uint32_t)n;
      h[k] = run;
      run += c;
    }
    if (trivial) continue;  // one digit value for every key: the pass is the identity
    scatter_range(in, 0, n, p * num_bits, mask, buckets, h, out);
    std::swap(in, out);
  }
  if (in != keys) std::memcpy(keys, in, (size_t)n * sizeof(uint32_t));
}

// The production OpenMP LSD sort for 32-bit keys: 8-bit digits, ONE parallel region for the whole sort (per
// pass: each thread histograms its chunk, one thread forms every (thread, digit) output offset, each thread
// scatters its chunk stably through write-combining slots), passes whose digit is the same for every key
// skipped.  radix_parallel keeps the reference's block decomposition for the stage tests and the threads x
// blocks sweep (hw1code/main_q2.cpp:123-148, :282-309).
void radix_parallel_lsd(uint32_t* keys, uint32_t* tmp, int64_t n) {
  constexpr int B = 8, NBK = 1 << B, P = 4;
  if (n <= 1) return;
  const int T = std::max(1, std::min<int>(omp_get_max_threads(), (int)std::max<int64_t>(1, n / 65536)));
  const int64_t chunk = (n + T - 1) / T;
  std::vector<uint32_t> hist((size_t)T * NBK), pos((size_t)T * NBK);
  uint32_t* bufs[2] = {keys, tmp};
  int cur = 0;  // bufs[cur] holds the keys
  bool skip = false;
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num(), nt = omp_get_num_threads();
    for (int p = 0; p < P; ++p) {
      const uint32_t* in = bufs[cur];
      // (nt < T only when the runtime refuses threads: thread t then covers chunks t, t + nt, ...)
      for (int c = t; c < T; c += nt) {
        uint32_t* h = hist.data() + (size_t)c * NBK;
        std::fill(h, h + NBK, 0u);
        const int64_t lo = std::min<int64_t>(n, c * chunk), hi = std::min<int64_t>(n, lo + chunk);
        for (int64_t i = lo; i < hi; ++i) ++h[(in[i] >> (p * B)) & (NBK - 1)];
      }
#pragma omp barrier
#pragma omp single
      {
        uint32_t run = 0;
        skip = false;
        for (int d = 0; d < NBK; ++d) {
          uint32_t tot = 0;
          for (int c = 0; c < T; ++c) {
            const uint32_t k = hist[(size_t)c * NBK + d];
            pos[(size_t)c * NBK + d] = run;
            run += k;
            tot += k;
          }
          skip |= tot == (uint32_t)n;
        }
      }  // (implicit barrier)
      if (!skip) {
        for (int c = t; c < T; c += nt) {
          const int64_t lo = std::min<int64_t>(n, c * chunk), hi = std::min<int64_t>(n, lo + chunk);
          scatter_range(in, lo, hi, p * B, NBK - 1, NBK, pos.data() + (size_t)c * NBK, bufs[cur ^ 1]);
        }
      }
#pragma omp barrier
#pragma omp single
      if (!skip) cur ^= 1;
    }
  }
  if (cur) std::memcpy(keys, tmp, (size_t)n * sizeof(uint32_t));
}

void std_sort(uint32_t* keys, int64_t n) { std::sort(keys, keys + n); }

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
