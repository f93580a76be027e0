// Microbenchmark: cost of a software grid barrier on MI355X (all workgroups resident), to price a
// persistent multi-phase training step against kernel boundaries.
//   mode 0: atomics only (counter + generation, agent scope, relaxed) -- data must then move with
//           coherent (sc1) loads/stores
//   mode 1: + agent-scope release/acquire fences (L2 write-back / invalidate per workgroup)
//   mode 2: empty kernel launches (one per "barrier") for comparison, in a HIP graph
// Usage: grid_barrier [blocks=256] [threads=512] [iters=2000]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

template <int MODE>
__device__ __forceinline__ void grid_barrier(unsigned* count, unsigned* gen, unsigned nblocks, int* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (MODE == 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned prev = __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == nblocks - 1) {
      __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gen, g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned spins = 0;
      while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
        if (++spins > (1u << 24)) {
          atomicExch(err, 1);
          break;
        }
        __builtin_amdgcn_s_sleep(0);
      }
    }
    if (MODE == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

template <int MODE>
__global__ void barrier_kernel(unsigned* count, unsigned* gen, int iters, int* err, float* sink) {
  float acc = threadIdx.x;
  for (int i = 0; i < iters; ++i) {
    acc = acc * 1.0001f + 1.f;
    grid_barrier<MODE>(count, gen, gridDim.x, err);
  }
  if (acc == -1.f) sink[0] = acc;
}

__global__ void empty_kernel(float* sink) {
  if (threadIdx.x == 1u << 30) sink[0] = 1.f;
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? std::atoi(argv[1]) : 256;
  const int threads = argc > 2 ? std::atoi(argv[2]) : 512;
  const int iters = argc > 3 ? std::atoi(argv[3]) : 2000;
  unsigned *count, *gen;
  int* err;
  float* sink;
  CHECK(hipMalloc(&count, 256));
  CHECK(hipMalloc(&gen, 256));
  CHECK(hipMalloc(&err, 4));
  CHECK(hipMalloc(&sink, 4));
  CHECK(hipMemset(count, 0, 256));
  CHECK(hipMemset(gen, 0, 256));
  CHECK(hipMemset(err, 0, 4));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  for (int mode = 0; mode < 2; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {  // first rep warms up
      CHECK(hipEventRecord(a, s));
      if (mode == 0) barrier_kernel<0><<<blocks, threads, 0, s>>>(count, gen, iters, err, sink);
      else barrier_kernel<1><<<blocks, threads, 0, s>>>(count, gen, iters, err, sink);
      CHECK(hipEventRecord(b, s));
      CHECK(hipStreamSynchronize(s));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      int e = 0;
      CHECK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
      if (rep) std::printf("mode %d (%s): %d blocks x %d threads: %.3f us per barrier (err %d)\n", mode,
                           mode ? "atomics + agent fences" : "atomics only", blocks, threads, ms * 1e3 / iters, e);
    }
  }
  // kernel boundaries: `iters` empty launches of the same grid captured in one graph
  hipGraph_t g;
  hipGraphExec_t ge;
  CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < 200; ++i) empty_kernel<<<blocks, threads, 0, s>>>(sink);
  CHECK(hipStreamEndCapture(s, &g));
  CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CHECK(hipGraphLaunch(ge, s));
  CHECK(hipStreamSynchronize(s));
  CHECK(hipEventRecord(a, s));
  for (int r = 0; r < 10; ++r) CHECK(hipGraphLaunch(ge, s));
  CHECK(hipEventRecord(b, s));
  CHECK(hipStreamSynchronize(s));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  std::printf("mode 2 (empty kernels in a graph): %d blocks x %d threads: %.3f us per launch\n", blocks, threads,
              ms * 1e3 / 2000);
  return 0;
}
