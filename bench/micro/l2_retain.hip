// Does an XCD's L2 keep lines across a kernel boundary?  A launch whose 32 workgroups per XCD read a
// 2 MiB part of a 16 MiB buffer, then the same launch again: the second read of the SAME
// buffer vs a read of another buffer that was last touched several launches earlier (still in the
// Infinity Cache, not in L2).  Also: the same buffer read by the next launch on a DIFFERENT XCD mapping
// (workgroup i reads the slice workgroup i+1 read), and a buffer the previous launch WROTE.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o bench/micro/l2_retain bench/micro/l2_retain.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int kBytes = 16 << 20;  // 2 MiB per XCD: fits its 4 MiB L2
constexpr int kWG = 256;  // 32 per XCD
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// workgroup b (XCD x = b % 8, slot s = b / 8) reads 8 KiB piece s of part (x + shift) % 8 of the buffer:
// with shift 0 every XCD re-reads the 256 KiB part it read before, with shift 1 a part another XCD read
__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ buf, unsigned* __restrict__ sink, int shift) {
  const int x = blockIdx.x % 8, s = blockIdx.x / 8;
  constexpr int kPart = kBytes / 8 / 16, kPiece = kPart / 32;  // in 16-B units
  const u32x4* p = buf + (size_t)((x + shift) % 8) * kPart + (size_t)s * kPiece;
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll 2
  for (int i = threadIdx.x; i < kPiece; i += 256) acc ^= p[i];
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[blockIdx.x] = 1;  // keep the loads
}

__global__ __launch_bounds__(256) void k_write(u32x4* __restrict__ buf) {
  const int x = blockIdx.x % 8, s = blockIdx.x / 8;
  constexpr int kPart = kBytes / 8 / 16, kPiece = kPart / 32;
  u32x4* p = buf + (size_t)x * kPart + (size_t)s * kPiece;
  for (int i = threadIdx.x; i < kPiece; i += 256) p[i] = u32x4{(unsigned)i, 1u, 2u, 3u};
}

int main() {
  u32x4 *a, *b, *c, *flush;
  unsigned* sink;
  CK(hipMalloc(&a, kBytes));
  CK(hipMalloc(&b, kBytes));
  CK(hipMalloc(&c, kBytes));
  CK(hipMalloc(&flush, 128 << 20));
  CK(hipMalloc(&sink, kWG * 4));
  CK(hipMemset(a, 1, kBytes));
  CK(hipMemset(b, 2, kBytes));
  CK(hipMemset(c, 3, kBytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timed = [&](auto launch) {
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return 1e3f * ms;
  };
  auto rd = [&](const u32x4* buf, int shift) { k_read<<<kWG, 256>>>(buf, sink, shift); };
  auto evict = [&] {  // 8 launches over 128 MiB of other data: 16 MiB per XCD, four times its L2
    for (int i = 0; i < 8; ++i) k_read<<<kWG, 256>>>(flush + (size_t)i * (kBytes / 16), sink, 0);
  };
  for (int rep = 0; rep < 6; ++rep) {
    // same buffer, same mapping, back to back
    rd(a, 0);
    const float same = timed([&] { rd(a, 0); });
    // the other buffer, last read before 8 launches over 128 MiB of other data
    evict();
    const float other = timed([&] { rd(b, 0); });
    // same buffer, each XCD now reads the part another XCD read before
    rd(a, 0);
    const float shifted = timed([&] { rd(a, 1); });
    // a buffer the previous launch wrote (same XCD per slice)
    k_write<<<kWG, 256>>>(c);
    const float written = timed([&] { rd(c, 0); });
    CK(hipDeviceSynchronize());
    printf("{\"rep\": %d, \"same_us\": %.2f, \"cold_us\": %.2f, \"other_xcd_us\": %.2f, \"after_write_us\": %.2f}\n",
           rep, same, other, shifted, written);
  }
  return 0;
}
