// hw1 radix sort and hw4 Vigenere cryptanalysis on gfx950 (no Thrust).
//
// Radix (reference: hw1code/main_q2.cpp:26-159, OpenMP): per 8-bit pass
//   1. digit histogram per 4096-key tile, LDS atomics, stored digit-major
//   2. exclusive scan of the [256][tiles] table (one workgroup)
//   3. stable scatter: per 256-key chunk, each key's rank among equal digits is
//      found with eight 64-bit ballots (wave-local match mask + popcount), the
//      per-wave digit counts are prefix-summed through LDS.
// Cipher (reference: hw4code/create_cipher.cu, solve_cipher.cu with Thrust
// sort/reduce_by_key): histograms are LDS-privatised counting (no sort), the
// key-length search evaluates a whole range of shifts in one launch, and the
// per-residue frequency analysis is one [period][256] histogram.
#include <algorithm>

#include "../common/hip_common.h"
#include "suite_kernels.h"

namespace cme::suite {

namespace {

constexpr int kRT = 256;        // threads per radix block
constexpr int kRItems = 16;     // keys per thread per tile
constexpr int kRTile = kRT * kRItems;

int64_t radix_tiles(int64_t n) { return (n + kRTile - 1) / kRTile; }

// Pass structure (one 8-bit digit): hist -> scan -> scatter, three launches.
//   hist    : per 4096-key tile an LDS histogram, written digit-major counts[d][tile]; the per-digit
//             totals are accumulated with one atomic per (tile, digit) into totals[d]
//   scan    : one workgroup per digit: base(d) = sum of totals[0..d) (block reduction), then an
//             exclusive block scan of counts[d][0..tiles) + base -- 256 workgroups in parallel instead
//             of one workgroup walking 256 x tiles values
//   scatter : the tile is first sorted by digit IN LDS (stable: 16 rounds of 256 keys, ballot-ranked
//             within a wave, per-wave digit counts prefix-summed across waves), then written out so
//             that consecutive threads write consecutive keys of one digit run -- coalesced stores
//             instead of one scattered 4-byte store per key.
__global__ __launch_bounds__(kRT) void radix_hist_kernel(const uint32_t* __restrict__ keys, int64_t n, int shift,
                                                         uint32_t* __restrict__ counts, int64_t tiles,
                                                         uint32_t* __restrict__ totals) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kRTile;
  uint32_t k[kRItems];
#pragma unroll
  for (int j = 0; j < kRItems; ++j) {
    const int64_t i = base + j * kRT + threadIdx.x;
    k[j] = i < n ? keys[i] : 0u;
  }
#pragma unroll
  for (int j = 0; j < kRItems; ++j)
    if (base + j * kRT + threadIdx.x < n) atomicAdd(&h[(k[j] >> shift) & 255u], 1u);
  __syncthreads();
  const uint32_t c = h[threadIdx.x];
  counts[(int64_t)threadIdx.x * tiles + blockIdx.x] = c;  // digit-major
  if (c) atomicAdd(&totals[threadIdx.x], c);
}

// block-wide exclusive scan of one value per thread (256 threads); returns the exclusive prefix,
// *total = sum over the block
__device__ __forceinline__ uint32_t block_exscan256(uint32_t v, uint32_t* sh, uint32_t* total) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[wave] = x;
  __syncthreads();
  uint32_t pre = 0;
  for (int w = 0; w < wave; ++w) pre += sh[w];
  *total = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  return pre + x - v;
}

__global__ __launch_bounds__(kRT) void radix_scan_kernel(uint32_t* __restrict__ counts, int64_t tiles,
                                                         const uint32_t* __restrict__ totals) {
  __shared__ uint32_t sh[4];
  const int d = blockIdx.x, t = threadIdx.x;
  uint32_t tot;
  const uint32_t pre = block_exscan256(totals[t], sh, &tot);
  __shared__ uint32_t s_base;
  if (t == d) s_base = pre;  // exclusive prefix of digit d over the digit totals
  __syncthreads();
  uint32_t run = s_base;
  uint32_t* row = counts + (int64_t)d * tiles;
  for (int64_t c0 = 0; c0 < tiles; c0 += 4 * kRT) {  // 4 consecutive tiles per thread per round
    uint32_t v[4], s = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t i = c0 + (int64_t)t * 4 + q;
      v[q] = i < tiles ? row[i] : 0u;
      s += v[q];
    }
    uint32_t rtot;
    uint32_t ex = block_exscan256(s, sh, &rtot) + run;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t i = c0 + (int64_t)t * 4 + q;
      if (i < tiles) row[i] = ex;
      ex += v[q];
    }
    run += rtot;
  }
}

__device__ __forceinline__ unsigned long long lanemask_lt() {
  const int lane = threadIdx.x & 63;
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

__global__ __launch_bounds__(kRT) void radix_scatter_kernel(const uint32_t* __restrict__ in,
                                                            uint32_t* __restrict__ out, int64_t n, int shift,
                                                            const uint32_t* __restrict__ offsets, int64_t tiles) {
  __shared__ uint32_t sorted[kRTile];
  __shared__ uint32_t loc[256];    // tile-local exclusive offset of each digit
  __shared__ uint32_t glob[256];   // global offset of this tile's first key of each digit
  __shared__ uint32_t run[256];    // keys of each digit placed so far (tile-local)
  __shared__ uint32_t wcnt[4][256];
  __shared__ uint32_t sh[4];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t base = (int64_t)blockIdx.x * kRTile;
  const int cnt = (int)std::min<int64_t>(kRTile, n - base);
  uint32_t k[kRItems];
#pragma unroll
  for (int j = 0; j < kRItems; ++j) {
    const int64_t i = base + j * kRT + t;
    k[j] = i < n ? in[i] : 0u;
  }
  // tile-local digit histogram -> exclusive offsets
  run[t] = 0;
  glob[t] = offsets[(int64_t)t * tiles + blockIdx.x];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kRItems; ++j)
    if (j * kRT + t < cnt) atomicAdd(&run[(k[j] >> shift) & 255u], 1u);
  __syncthreads();
  uint32_t tot;
  loc[t] = block_exscan256(run[t], sh, &tot);
  run[t] = 0;
  __syncthreads();
  // stable rank of every key inside the tile: rounds of 256 keys in index order
  for (int j = 0; j < kRItems; ++j) {
#pragma unroll
    for (int w = 0; w < 4; ++w) wcnt[w][t] = 0;
    __syncthreads();
    const bool valid = j * kRT + t < cnt;
    const uint32_t d = (k[j] >> shift) & 255u;
    unsigned long long match = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
      const bool set = (d >> bit) & 1u;
      const unsigned long long bal = __ballot(set);
      match &= set ? bal : ~bal;
    }
    const int rank = __popcll(match & lanemask_lt());
    if (valid && rank == 0) wcnt[wave][d] = (uint32_t)__popcll(match);  // group leader
    __syncthreads();
    if (valid) {
      uint32_t before = 0;
      for (int w = 0; w < wave; ++w) before += wcnt[w][d];
      sorted[loc[d] + run[d] + before + rank] = k[j];
    }
    __syncthreads();
    run[t] += wcnt[0][t] + wcnt[1][t] + wcnt[2][t] + wcnt[3][t];
  }
  __syncthreads();
  // write-out in tile order: consecutive threads -> consecutive keys of the same digit run
#pragma unroll
  for (int j = 0; j < kRItems; ++j) {
    const int p = j * kRT + t;
    if (p < cnt) {
      const uint32_t key = sorted[p];
      const uint32_t d = (key >> shift) & 255u;
      out[glob[d] + (p - loc[d])] = key;
    }
  }
}

// exclusive scan of `a` (length L) in place, single workgroup of 1024 threads (small arrays: the
// cipher's per-block counts)
__global__ __launch_bounds__(1024) void scan_exclusive_kernel(uint32_t* __restrict__ a, int64_t L) {
  __shared__ uint32_t part[1024];
  const int t = threadIdx.x;
  const int64_t per = (L + 1023) / 1024;
  const int64_t b = t * per, e = std::min<int64_t>(L, b + per);
  uint32_t s = 0;
  for (int64_t i = b; i < e; ++i) s += a[i];
  part[t] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
    const uint32_t v = t >= off ? part[t - off] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - s;  // exclusive prefix of this thread's segment
  for (int64_t i = b; i < e; ++i) {
    const uint32_t v = a[i];
    a[i] = run;
    run += v;
  }
}

// ------------------------------------------------------------------ cipher
constexpr int kCT = 256, kCItems = 16, kCTile = kCT * kCItems;

__device__ __forceinline__ uint8_t to_lower(uint8_t c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }
__device__ __forceinline__ bool is_lower(uint8_t c) { return c >= 'a' && c <= 'z'; }

__global__ __launch_bounds__(kCT) void letters_count_kernel(const uint8_t* __restrict__ in, int64_t n,
                                                            uint32_t* __restrict__ counts) {
  const int64_t base = (int64_t)blockIdx.x * kCTile + (int64_t)threadIdx.x * kCItems;
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < kCItems; ++j)
    if (base + j < n && is_lower(to_lower(in[base + j]))) ++c;
  // block sum
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  __shared__ uint32_t p[4];
  if ((threadIdx.x & 63) == 0) p[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = p[0] + p[1] + p[2] + p[3];
}

__global__ __launch_bounds__(kCT) void letters_compact_kernel(const uint8_t* __restrict__ in, int64_t n,
                                                              const uint32_t* __restrict__ offs,
                                                              const uint32_t* __restrict__ counts, int nb,
                                                              uint8_t* __restrict__ out, int64_t* count) {
  __shared__ uint32_t sc[kCT];
  const int64_t base = (int64_t)blockIdx.x * kCTile + (int64_t)threadIdx.x * kCItems;
  uint8_t v[kCItems];
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < kCItems; ++j) {
    v[j] = base + j < n ? to_lower(in[base + j]) : 0;
    c += is_lower(v[j]);
  }
  sc[threadIdx.x] = c;
  __syncthreads();
  for (int off = 1; off < kCT; off <<= 1) {
    const uint32_t x = threadIdx.x >= off ? sc[threadIdx.x - off] : 0u;
    __syncthreads();
    sc[threadIdx.x] += x;
    __syncthreads();
  }
  uint32_t pos = offs[blockIdx.x] + sc[threadIdx.x] - c;
#pragma unroll
  for (int j = 0; j < kCItems; ++j)
    if (is_lower(v[j])) out[pos++] = v[j];
  if (blockIdx.x == nb - 1 && threadIdx.x == 0) *count = (int64_t)offs[nb - 1] + counts[nb - 1];
}

__global__ void vigenere_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, int64_t n,
                                const int* __restrict__ shifts, int period, int sign, int wrap) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int sh = sign * shifts[i % period];
    if (wrap) {
      int v = (int)in[i] - 'a' + sh;
      v %= 26;
      if (v < 0) v += 26;
      out[i] = (uint8_t)('a' + v);
    } else {
      out[i] = (uint8_t)((int)in[i] + sh);  // reference apply_shift: plain byte add
    }
  }
}

__global__ __launch_bounds__(256) void byte_hist_kernel(const uint8_t* __restrict__ in, int64_t n,
                                                        uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 4 <= n) {
      const uint32_t w = *reinterpret_cast<const uint32_t*>(in + i);
      atomicAdd(&h[w & 255u], 1u);
      atomicAdd(&h[(w >> 8) & 255u], 1u);
      atomicAdd(&h[(w >> 16) & 255u], 1u);
      atomicAdd(&h[w >> 24], 1u);
    } else {
      for (int64_t k = i; k < n; ++k) atomicAdd(&h[in[k]], 1u);
    }
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}

constexpr int kMChunk = 4096;
constexpr int kMaxShiftSpan = 4096;

__global__ __launch_bounds__(256) void shifted_matches_kernel(const uint8_t* __restrict__ t, int64_t n, int lo,
                                                              int hi, unsigned long long* __restrict__ counts) {
  __shared__ uint8_t buf[kMChunk + kMaxShiftSpan];
  __shared__ uint32_t part[4];
  const int64_t base = (int64_t)blockIdx.x * kMChunk;
  const int span = kMChunk + hi;
  for (int k = threadIdx.x; k < span; k += 256) buf[k] = base + k < n ? t[base + k] : 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int s = lo; s < hi; ++s) {
    uint32_t c = 0;
    for (int k = threadIdx.x; k < kMChunk; k += 256) {
      const int64_t i = base + k;
      if (i + s < n) c += buf[k] == buf[k + s];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if (lane == 0) part[wave] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long tot = part[0] + part[1] + part[2] + part[3];
      if (tot) atomicAdd(&counts[s - lo], tot);
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void residue_hist_kernel(const uint8_t* __restrict__ t, int64_t n, int period,
                                                           uint32_t* __restrict__ hist) {
  extern __shared__ uint32_t h[];  // [period][256]
  for (int k = threadIdx.x; k < period * 256; k += 256) h[k] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    atomicAdd(&h[(i % period) * 256 + t[i]], 1u);
  __syncthreads();
  for (int k = threadIdx.x; k < period * 256; k += 256)
    if (h[k]) atomicAdd(&hist[k], h[k]);
}

}  // namespace

// ---------------------------------------------------------------- radix API
// counts [256][tiles] + totals [256]
int64_t radix_workspace_bytes(int64_t n) { return ((int64_t)256 * std::max<int64_t>(1, radix_tiles(n)) + 256) * 4; }

void radix_pass_u32(const uint32_t* in, uint32_t* out, int64_t n, int start_bit, void* ws, hipStream_t s) {
  if (n <= 0) return;
  CME_REQUIRE(n < (int64_t)1 << 32, "radix_pass_u32: n must fit in 32 bits");
  const int64_t tiles = radix_tiles(n);
  uint32_t* counts = static_cast<uint32_t*>(ws);
  uint32_t* totals = counts + 256 * tiles;
  HIP_CHECK(hipMemsetAsync(totals, 0, 256 * sizeof(uint32_t), s));
  radix_hist_kernel<<<(unsigned)tiles, kRT, 0, s>>>(in, n, start_bit, counts, tiles, totals);
  radix_scan_kernel<<<256, kRT, 0, s>>>(counts, tiles, totals);
  radix_scatter_kernel<<<(unsigned)tiles, kRT, 0, s>>>(in, out, n, start_bit, counts, tiles);
  CME_LAUNCH_CHECK(s);
}

void radix_sort_u32(uint32_t* keys, uint32_t* tmp, int64_t n, void* ws, hipStream_t s) {
  for (int bit = 0; bit < 32; bit += 16) {  // 4 passes, ping-pong, result back in keys
    radix_pass_u32(keys, tmp, n, bit, ws, s);
    radix_pass_u32(tmp, keys, n, bit + 8, ws, s);
  }
}

// --------------------------------------------------------------- cipher API
int64_t cipher_workspace_bytes(int64_t n) {
  const int64_t nb = std::max<int64_t>(1, (n + kCTile - 1) / kCTile);
  return 2 * nb * 4;
}

void sanitize_lower(const uint8_t* in, int64_t n, uint8_t* out, int64_t* count, void* ws, hipStream_t s) {
  if (n <= 0) {
    HIP_CHECK(hipMemsetAsync(count, 0, sizeof(int64_t), s));
    return;
  }
  const int64_t nb = (n + kCTile - 1) / kCTile;
  CME_REQUIRE(nb < (1ll << 31), "sanitize_lower: input too large");
  uint32_t* counts = static_cast<uint32_t*>(ws);
  uint32_t* offs = counts + nb;
  letters_count_kernel<<<(unsigned)nb, kCT, 0, s>>>(in, n, counts);
  HIP_CHECK(hipMemcpyAsync(offs, counts, nb * 4, hipMemcpyDeviceToDevice, s));
  scan_exclusive_kernel<<<1, 1024, 0, s>>>(offs, nb);
  letters_compact_kernel<<<(unsigned)nb, kCT, 0, s>>>(in, n, offs, counts, (int)nb, out, count);
  CME_LAUNCH_CHECK(s);
}

void vigenere_apply(const uint8_t* in, uint8_t* out, int64_t n, const int* shifts, int period, int sign, int wrap,
                    hipStream_t s) {
  if (n <= 0) return;
  CME_REQUIRE(period > 0, "vigenere_apply: period must be positive");
  const int grid = (int)std::min<int64_t>(4096, (n + 255) / 256);
  vigenere_kernel<<<grid, 256, 0, s>>>(in, out, n, shifts, period, sign, wrap);
  CME_LAUNCH_CHECK(s);
}

void byte_histogram(const uint8_t* in, int64_t n, uint32_t* hist, hipStream_t s) {
  HIP_CHECK(hipMemsetAsync(hist, 0, 256 * 4, s));
  if (n <= 0) return;
  CME_REQUIRE((reinterpret_cast<uintptr_t>(in) & 3) == 0, "byte_histogram: input must be 4-byte aligned");
  const int grid = (int)std::min<int64_t>(1024, (n / 4 + 255) / 256 + 1);
  byte_hist_kernel<<<grid, 256, 0, s>>>(in, n, hist);
  CME_LAUNCH_CHECK(s);
}

void shifted_matches(const uint8_t* t, int64_t n, int lo, int hi, unsigned long long* counts, hipStream_t s) {
  CME_REQUIRE(0 < lo && lo <= hi && hi <= kMaxShiftSpan, "shifted_matches: need 0 < lo <= hi <= 4096");
  HIP_CHECK(hipMemsetAsync(counts, 0, (size_t)(hi - lo) * 8, s));
  if (n <= 0 || hi == lo) return;
  const int64_t nb = (n + kMChunk - 1) / kMChunk;
  shifted_matches_kernel<<<(unsigned)nb, 256, 0, s>>>(t, n, lo, hi, counts);
  CME_LAUNCH_CHECK(s);
}

void residue_histogram(const uint8_t* t, int64_t n, int period, uint32_t* hist, hipStream_t s) {
  CME_REQUIRE(period >= 1 && period <= 64, "residue_histogram: 1 <= period <= 64");
  HIP_CHECK(hipMemsetAsync(hist, 0, (size_t)period * 256 * 4, s));
  if (n <= 0) return;
  const int grid = (int)std::min<int64_t>(512, (n + 255) / 256);
  residue_hist_kernel<<<grid, 256, (size_t)period * 256 * 4, s>>>(t, n, period, hist);
  CME_LAUNCH_CHECK(s);
}

}  // namespace cme::suite
