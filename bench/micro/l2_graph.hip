// Does an XCD's L2 keep a buffer from one kernel to the next differently for stream launches and graph nodes?
// (The headline step's same-batch graph runs the SAME two kernels ~0.6 us shorter each than the native loop does,
// profiles/graph_gap_r4/summary.txt.)  Kernel k_read: 256 workgroups (32 per XCD) read a 2 MiB-per-XCD part of a
// 16 MiB buffer and record their own read time (s_memrealtime, 10 ns).  Sequence: read A, read A again -- as two
// stream launches, and as two nodes of a captured graph.  The second read's per-workgroup time is reported; a
// third case reads a buffer last touched before 128 MiB of other reads (cold in L2) for scale, and a pair
// write A -> read A checks data the previous kernel WROTE.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o bench/micro/l2_graph bench/micro/l2_graph.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int kBytes = 16 << 20;
constexpr int kWG = 256;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ buf, unsigned* __restrict__ t_out) {
  const int x = blockIdx.x % 8, s = blockIdx.x / 8;
  constexpr int kPart = kBytes / 8 / 16, kPiece = kPart / 32;  // 16-B units
  const u32x4* p = buf + (size_t)x * kPart + (size_t)s * kPiece;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll 4
  for (int i = threadIdx.x; i < kPiece; i += 256) acc ^= p[i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  const unsigned v = (acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u ? 1u : (unsigned)(t1 - t0);
  if (threadIdx.x == 0) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(t_out, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(v, r, blockIdx.x * 4, 0, 0);
  }
}

__global__ __launch_bounds__(256) void k_write(u32x4* __restrict__ buf) {  // the same per-workgroup part, written
  const int x = blockIdx.x % 8, s = blockIdx.x / 8;
  constexpr int kPart = kBytes / 8 / 16, kPiece = kPart / 32;
  u32x4* p = buf + (size_t)x * kPart + (size_t)s * kPiece;
  for (int i = threadIdx.x; i < kPiece; i += 256) p[i] = u32x4{(unsigned)i, 1u, 2u, 3u};
}

static void report(const char* name, unsigned* d_t) {
  std::vector<unsigned> h(kWG);
  CK(hipMemcpy(h.data(), d_t, kWG * 4, hipMemcpyDeviceToHost));
  std::sort(h.begin(), h.end());
  printf("{\"case\": \"%s\", \"read_us\": [%.2f, %.2f, %.2f]}\n", name, h[kWG / 10] / 100.0, h[kWG / 2] / 100.0,
         h[kWG * 9 / 10] / 100.0);
}

int main() {
  u32x4 *a, *b, *flush;
  unsigned *t1, *t2;
  CK(hipMalloc(&a, kBytes));
  CK(hipMalloc(&b, kBytes));
  CK(hipMalloc(&flush, 128 << 20));
  CK(hipMalloc(&t1, kWG * 4));
  CK(hipMalloc(&t2, kWG * 4));
  CK(hipMemset(a, 1, kBytes));
  CK(hipMemset(b, 2, kBytes));
  CK(hipMemset(flush, 3, 128 << 20));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto evict = [&] {
    for (int i = 0; i < 8; ++i) k_read<<<kWG, 256, 0, s>>>(flush + (size_t)i * (kBytes / 16), t1);
  };
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  k_read<<<kWG, 256, 0, s>>>(a, t1);
  k_read<<<kWG, 256, 0, s>>>(a, t2);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  hipGraph_t gw;
  hipGraphExec_t gwe;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  k_write<<<kWG, 256, 0, s>>>(a);
  k_read<<<kWG, 256, 0, s>>>(a, t2);
  CK(hipStreamEndCapture(s, &gw));
  CK(hipGraphInstantiate(&gwe, gw, nullptr, nullptr, 0));
  for (int rep = 0; rep < 3; ++rep) {
    evict();
    k_write<<<kWG, 256, 0, s>>>(a);
    k_read<<<kWG, 256, 0, s>>>(a, t2);
    CK(hipStreamSynchronize(s));
    report("stream: read of the buffer the previous kernel WROTE", t2);
    evict();
    CK(hipGraphLaunch(gwe, s));
    CK(hipStreamSynchronize(s));
    report("graph: read of the buffer the previous node WROTE", t2);
    evict();
    k_read<<<kWG, 256, 0, s>>>(a, t1);
    k_read<<<kWG, 256, 0, s>>>(a, t2);
    CK(hipStreamSynchronize(s));
    report("stream: second read of the same buffer", t2);
    evict();
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    report("graph: second read of the same buffer", t2);
    evict();
    k_read<<<kWG, 256, 0, s>>>(b, t2);
    CK(hipStreamSynchronize(s));
    report("stream: a buffer cold in L2", t2);
  }
  CK(hipGraphExecDestroy(gwe));
  CK(hipGraphDestroy(gw));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return 0;
}
