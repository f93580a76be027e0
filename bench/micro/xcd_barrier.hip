// Microbenchmark: the price of an XCD-LOCAL hand-off inside one persistent launch -- the seam the XCD-local step
// pipeline (csrc/mlp/xstep.hip) puts where the two-launch step has a kernel boundary.
//
// Every workgroup reads its XCD from HW_REG_XCC_ID and takes a ticket on its XCD's counter (slot); slots < NW are
// the XCD's workers.  Each round, every worker stores a 2 KB payload (one float per thread), drains its stores
// (s_waitcnt vmcnt(0) + barrier), adds one to its XCD's round counter (agent-scope atomic, no return), lane 0 polls
// that counter with sc1 loads until all NW workers of the XCD have arrived, and then EVERY worker reads all NW
// payloads of its XCD (NW x 2 KB, like the forward reading its row tile's whole W1 slice) with sc1 loads
// (L1-bypassing, L2-served) and checks every word.  Payloads are double-buffered by round parity.
//   mode 0: plain payload stores (the lines stay dirty in the XCD's L2: a same-XCD reader hits them)
//   mode 1: sc1 (write-through) payload stores (the lines leave the L2: read back at the die-level cache's rate)
//   mode 2: the counter alone (no payload)
//   mode 3: plain payload stores, and the arrival is a per-workgroup FLAG word in one line per XCD written with a
//           plain store (the line stays in the XCD's L2: no trip to the memory-side atomic unit), polled with sc1 loads
//   mode 4: the same flag line written with sc1 (write-through) stores
// Per-round phase stamps (s_memrealtime, 100 MHz) of every worker: stores drained -> last arrival seen -> payload
// read.  Usage: xcd_barrier [rounds=2000] [workers per XCD=25]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

constexpr int kThreads = 512, kPB = 512;  // payload floats per worker (one per thread)
constexpr unsigned long long kLimit = 100ull * 100000;  // 100 ms of s_memrealtime ticks

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 15u;
}

__device__ __forceinline__ float val(int r, int slot, int t) { return (float)(r * 131 + slot * 7 + t); }

template <int MODE>
__global__ __launch_bounds__(kThreads) void xcd_kernel(unsigned long long* ctl, float* payload, int rounds, int nw,
                                                       int* err, unsigned long long* stamps, int stamp_round) {
  __shared__ int s_slot, s_to;
  __shared__ unsigned s_x;
  const int t = threadIdx.x;
  if (t == 0) {
    const unsigned x = xcc_id();
    s_x = x;
    s_to = 0;
    // ctl: [x * 32] ticket, [x * 32 + 16] round counter (separate 128-B halves of a 256-B line pair)
    s_slot = (int)__hip_atomic_fetch_add(ctl + x * 64, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const int slot = s_slot;
  const unsigned x = s_x;
  if (slot >= nw || x >= 8) return;
  unsigned long long* cnt = ctl + x * 64 + 32;
  float* mine = payload + ((size_t)x * 2 * nw + slot) * kPB;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(payload + (size_t)x * 2 * nw * kPB, (short)0,
                                                                        0x7FFFFFF0, 0x00020000);
  int bad = 0;
  for (int r = 0; r < rounds; ++r) {
    const int par = r & 1;
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if constexpr (MODE == 0 || MODE >= 3) mine[(size_t)par * nw * kPB + t] = val(r, slot, t);
    if constexpr (MODE == 1)
      __hip_atomic_store(mine + (size_t)par * nw * kPB + t, val(r, slot, t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned long long t1 = 0, t2 = 0;
    if (MODE >= 3) {
      // flags: 32 words (128 B) per XCD at ctl + x * 64 + 16 .. (the ticket line's second half); lane 0 stores this
      // workgroup's round + 1, wave 0's lanes 0-7 each load 16 B and compare
      unsigned* flags = reinterpret_cast<unsigned*>(ctl + x * 64 + 16);
      if (t == 0) {
        t1 = __builtin_amdgcn_s_memrealtime();
        if (MODE == 3) flags[slot] = (unsigned)(r + 1);
        else __hip_atomic_store(flags + slot, (unsigned)(r + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (t < 64) {
        const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(flags, (short)0, 128, 0x00020000);
        const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
          const unsigned v = __builtin_amdgcn_raw_buffer_load_b32(rf, t < nw ? t * 4 : 0x7FFFFFF0, 0, 16);
          const bool ok = t >= nw || v >= (unsigned)(r + 1);
          if (__all(ok)) break;
          if (__builtin_amdgcn_s_memrealtime() - w0 > kLimit) {
            if (t == 0) {
              atomicOr(err, 1);
              s_to = 1;
            }
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (t == 0) t2 = __builtin_amdgcn_s_memrealtime();
      }
    } else if (t == 0) {
      t1 = __builtin_amdgcn_s_memrealtime();
      __hip_atomic_fetch_add(cnt, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long target = (unsigned long long)(r + 1) * nw;
      const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        if (__builtin_amdgcn_s_memrealtime() - w0 > kLimit) {
          atomicOr(err, 1);
          s_to = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      t2 = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    if (s_to) return;  // (a timed-out wait ends this workgroup: the others time out in turn)
    if (MODE != 2) {
      // every payload of this XCD: nw * kPB floats as 16-byte sc1 loads, all issued before the checks
      constexpr int kMax = 8;  // 16-B loads per thread per pass
      const int total4 = nw * kPB / 4;
      for (int i0 = 0; i0 < total4; i0 += kMax * kThreads) {
        unsigned __attribute__((ext_vector_type(4))) v[kMax];
#pragma unroll
        for (int k = 0; k < kMax; ++k) {
          const int i = i0 + k * kThreads + t;
          v[k] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, i < total4 ? ((par * nw * kPB) + 4 * i) * 4 : 0x7FFFFFF0,
                                                       0, 16);
        }
#pragma unroll
        for (int k = 0; k < kMax; ++k) {
          const int i = i0 + k * kThreads + t;
          if (i < total4) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int f = 4 * i + e, s = f / kPB, tt = f % kPB;
              const unsigned w = v[k][e];  // (a copy: hipcc bit-casts an ext-vector element lvalue as element 0)
              bad += __builtin_bit_cast(float, w) != val(r, s, tt);
            }
          }
        }
      }
    }
    if (t == 0 && r == stamp_round && stamps) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
      unsigned long long* st = stamps + ((size_t)x * nw + slot) * 4;
      st[0] = t0;
      st[1] = t1;
      st[2] = t2;
      st[3] = t3;
    }
  }
  if (bad) atomicAdd(err + 1, bad);
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 2000;
  const int nw = argc > 2 ? std::atoi(argv[2]) : 25;
  unsigned long long *ctl, *stamps;
  float* payload;
  int* err;
  CHECK(hipMalloc(&ctl, 8 * 64 * 8));
  CHECK(hipMalloc(&payload, (size_t)8 * 2 * nw * kPB * 4));
  CHECK(hipMalloc(&err, 8));
  CHECK(hipMalloc(&stamps, (size_t)8 * nw * 4 * 8));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  const char* names[5] = {"plain payload stores + sc1 reads", "sc1 payload stores + sc1 reads", "counter only",
                          "plain payload; plain-store flag line polled with sc1 loads",
                          "plain payload; sc1-store flag line polled with sc1 loads"};
  for (int mode = 0; mode < 5; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {  // rep 0 warms up
      CHECK(hipMemset(ctl, 0, 8 * 64 * 8));
      CHECK(hipMemset(err, 0, 8));
      CHECK(hipMemset(stamps, 0, (size_t)8 * nw * 4 * 8));
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(a, s));
      if (mode == 0) xcd_kernel<0><<<256, kThreads, 0, s>>>(ctl, payload, rounds, nw, err, stamps, rounds / 2);
      else if (mode == 1) xcd_kernel<1><<<256, kThreads, 0, s>>>(ctl, payload, rounds, nw, err, stamps, rounds / 2);
      else if (mode == 2) xcd_kernel<2><<<256, kThreads, 0, s>>>(ctl, payload, rounds, nw, err, stamps, rounds / 2);
      else if (mode == 3) xcd_kernel<3><<<256, kThreads, 0, s>>>(ctl, payload, rounds, nw, err, stamps, rounds / 2);
      else xcd_kernel<4><<<256, kThreads, 0, s>>>(ctl, payload, rounds, nw, err, stamps, rounds / 2);
      CHECK(hipEventRecord(b, s));
      CHECK(hipStreamSynchronize(s));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      int e[2];
      CHECK(hipMemcpy(e, err, 8, hipMemcpyDeviceToHost));
      std::vector<unsigned long long> c(8 * 64), st((size_t)8 * nw * 4);
      CHECK(hipMemcpy(c.data(), ctl, c.size() * 8, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost));
      if (!rep) continue;
      // phases of the stamped round, median over the workers of every XCD
      std::vector<double> drain, wait, read, total;
      for (int i = 0; i < 8 * nw; ++i) {
        const unsigned long long* p = &st[(size_t)i * 4];
        if (!p[0]) continue;
        drain.push_back((p[1] - p[0]) / 100.0);
        wait.push_back((p[2] - p[1]) / 100.0);
        read.push_back((p[3] - p[2]) / 100.0);
        total.push_back((p[3] - p[0]) / 100.0);
      }
      auto med = [](std::vector<double> v) {
        if (v.empty()) return -1.0;
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
      };
      std::printf("{\"mode\": %d, \"what\": \"%s\", \"workers_per_xcd\": %d, \"rounds\": %d, \"us_per_round\": %.3f, "
                  "\"timeout\": %d, \"bad_words\": %d, \"census\": [",
                  mode, names[mode], nw, rounds, ms * 1e3 / rounds, e[0], e[1]);
      for (int x = 0; x < 8; ++x) std::printf("%llu%s", c[x * 64], x < 7 ? ", " : "");
      std::printf("], \"stamped_round_median_us\": {\"stores_drained\": %.3f, \"arrivals_seen\": %.3f, "
                  "\"payload_read\": %.3f, \"round\": %.3f}}\n",
                  med(drain), med(wait), med(read), med(total));
      std::fflush(stdout);
    }
  }
  return 0;
}
