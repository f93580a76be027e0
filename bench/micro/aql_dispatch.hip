// What does the HIP runtime add to one idle-GPU launch + wait, against an AQL packet written straight into an HSA
// queue of our own?  The driver's 20-step bench form pays ~23 us from its timer start to the first kernel and ~7 us
// from the last kernel's end to the host's return (profiles/r6/driver_gap/analysis_xstep.jsonl); the launch itself
// is one kernel.  Each sample: the host idles 200 us (the GPU drains), then times launch -> completion seen on the host
// for a trivial 256-workgroup x 512-thread kernel taking an 848-byte argument block (the pipeline's size):
//
//   hip          hipLaunchKernel + hipDeviceSynchronize                (what bench.py's timed region does)
//   hip_event    hipLaunchKernel + hipEventRecord + hipEventSynchronize
//   aql_sys      AQL dispatch packet on our own HSA queue, kernarg in the system kernarg region, completion signal
//                polled (HSA_WAIT_STATE_ACTIVE); system-scope acquire + release fences
//   aql_dev      the same with the kernarg block in device memory written by the host (large BAR)
//   aql_agent    aql_dev with agent-scope acquire fence (release stays system: the host reads the results)
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o bench/micro/aql_dispatch bench/micro/aql_dispatch.hip -lhsa-runtime64
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 --genco -o /tmp/b.hsaco bench/micro/aql_dispatch.hip &&
//     clang-offload-bundler --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=/tmp/b.hsaco \
//     --output=bench/micro/aql_dispatch.hsaco
//   bench/micro/aql_dispatch bench/micro/aql_dispatch.hsaco [samples]
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

struct Args {
  unsigned* out;
  unsigned pad[210];
};

extern "C" __global__ __launch_bounds__(512) void aql_probe_kernel(Args a) {
  if (threadIdx.x == 0) a.out[blockIdx.x] = a.pad[blockIdx.x % 210] + 1u;
}

#ifndef __HIP_DEVICE_COMPILE__
#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)
#define HK(x)                                                           \
  do {                                                                  \
    hsa_status_t s_ = (x);                                              \
    if (s_ != HSA_STATUS_SUCCESS) {                                     \
      const char* m_ = nullptr;                                         \
      hsa_status_string(s_, &m_);                                       \
      fprintf(stderr, "%s:%d hsa %d %s\n", __FILE__, __LINE__, (int)s_, m_ ? m_ : ""); \
      exit(1);                                                          \
    }                                                                   \
  } while (0)

using clk = std::chrono::steady_clock;
static double us_since(clk::time_point t0) {
  return std::chrono::duration<double, std::micro>(clk::now() - t0).count();
}
static void idle(double us) {
  const auto t0 = clk::now();
  while (us_since(t0) < us) {
  }
}

struct Found {
  hsa_agent_t gpu{};
  bool have = false;
  hsa_region_t kernarg{};
  bool have_karg = false;
  hsa_amd_memory_pool_t dev_pool{};
  bool have_pool = false;
};

static hsa_status_t on_agent(hsa_agent_t agent, void* data) {
  auto* f = static_cast<Found*>(data);
  hsa_device_type_t t;
  HK(hsa_agent_get_info(agent, HSA_AGENT_INFO_DEVICE, &t));
  if (t == HSA_DEVICE_TYPE_GPU && !f->have) {
    f->gpu = agent;
    f->have = true;
  }
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t on_region(hsa_region_t r, void* data) {
  auto* f = static_cast<Found*>(data);
  uint32_t flags = 0;
  HK(hsa_region_get_info(r, HSA_REGION_INFO_GLOBAL_FLAGS, &flags));
  if ((flags & HSA_REGION_GLOBAL_FLAG_KERNARG) && !f->have_karg) {
    f->kernarg = r;
    f->have_karg = true;
  }
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t on_pool(hsa_amd_memory_pool_t p, void* data) {
  auto* f = static_cast<Found*>(data);
  hsa_amd_segment_t seg;
  HK(hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg));
  uint32_t flags = 0;
  HK(hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags));
  if (seg == HSA_AMD_SEGMENT_GLOBAL && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && !f->have_pool) {
    f->dev_pool = p;
    f->have_pool = true;
  }
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t on_cpu(hsa_agent_t agent, void* data) {
  hsa_device_type_t t;
  HK(hsa_agent_get_info(agent, HSA_AGENT_INFO_DEVICE, &t));
  if (t == HSA_DEVICE_TYPE_CPU) *static_cast<hsa_agent_t*>(data) = agent;
  return HSA_STATUS_SUCCESS;
}

static void report(const char* name, std::vector<double>& v) {
  std::sort(v.begin(), v.end());
  const size_t n = v.size();
  printf("{\"case\": \"%s\", \"samples\": %zu, \"p10_us\": %.2f, \"median_us\": %.2f, \"p90_us\": %.2f}\n", name, n,
         v[n / 10], v[n / 2], v[n * 9 / 10]);
  fflush(stdout);
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: aql_dispatch <code object> [samples]\n");
    return 2;
  }
  const int samples = argc > 2 ? atoi(argv[2]) : 200;
  CK(hipSetDevice(0));
  unsigned* out = nullptr;
  CK(hipMalloc(&out, 256 * sizeof(unsigned)));
  Args a{};
  a.out = out;
  for (int i = 0; i < 210; ++i) a.pad[i] = (unsigned)i;

  {  // HIP
    std::vector<double> v, ve;
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (int i = 0; i < 20; ++i) aql_probe_kernel<<<256, 512>>>(a);
    CK(hipDeviceSynchronize());
    for (int i = 0; i < samples; ++i) {
      idle(200);
      auto t0 = clk::now();
      aql_probe_kernel<<<256, 512>>>(a);
      CK(hipDeviceSynchronize());
      v.push_back(us_since(t0));
      idle(200);
      t0 = clk::now();
      aql_probe_kernel<<<256, 512>>>(a);
      CK(hipEventRecord(ev, 0));
      CK(hipEventSynchronize(ev));
      ve.push_back(us_since(t0));
    }
    report("hip", v);
    report("hip_event", ve);
  }

  HK(hsa_init());
  Found f;
  HK(hsa_iterate_agents(on_agent, &f));
  if (!f.have) {
    fprintf(stderr, "no GPU agent\n");
    return 1;
  }
  HK(hsa_agent_iterate_regions(f.gpu, on_region, &f));
  HK(hsa_amd_agent_iterate_memory_pools(f.gpu, on_pool, &f));
  hsa_agent_t cpu{};
  HK(hsa_iterate_agents(on_cpu, &cpu));
  hsa_queue_t* q = nullptr;
  HK(hsa_queue_create(f.gpu, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));

  std::ifstream in(argv[1], std::ios::binary);
  std::string co((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  if (co.empty()) {
    fprintf(stderr, "empty code object %s\n", argv[1]);
    return 1;
  }
  hsa_code_object_reader_t rd;
  HK(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &rd));
  hsa_executable_t exe;
  HK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
  HK(hsa_executable_load_agent_code_object(exe, f.gpu, rd, nullptr, nullptr));
  HK(hsa_executable_freeze(exe, nullptr));
  hsa_executable_symbol_t sym;
  HK(hsa_executable_get_symbol_by_name(exe, "aql_probe_kernel.kd", &f.gpu, &sym));
  uint64_t kobj = 0;
  uint32_t kargsz = 0, gseg = 0, pseg = 0;
  HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &kobj));
  HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &kargsz));
  HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &gseg));
  HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &pseg));
  fprintf(stderr, "kernarg segment %u B (Args %zu B), group %u, private %u\n", kargsz, sizeof(Args), gseg, pseg);

  void* karg_sys = nullptr;
  HK(hsa_memory_allocate(f.kernarg, std::max<uint32_t>(kargsz, sizeof(Args)), &karg_sys));
  void* karg_dev = nullptr;
  HK(hsa_amd_memory_pool_allocate(f.dev_pool, 4096, 0, &karg_dev));
  HK(hsa_amd_agents_allow_access(1, &cpu, nullptr, karg_dev));
  std::memset(karg_sys, 0, kargsz);
  hsa_signal_t sig;
  HK(hsa_signal_create(1, 0, nullptr, &sig));

  auto dispatch = [&](void* karg, bool dev, int acq) {
    std::memcpy(karg, &a, sizeof(Args));
    if (dev) {  // (the host's writes through the BAR: read one back so they have landed before the doorbell)
      volatile unsigned* pk = static_cast<volatile unsigned*>(karg);
      (void)pk[sizeof(Args) / 4 - 1];
    }
    hsa_signal_store_relaxed(sig, 1);
    const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
    auto* pkt = static_cast<hsa_kernel_dispatch_packet_t*>(q->base_address) + (idx & (q->size - 1));
    pkt->workgroup_size_x = 512;
    pkt->workgroup_size_y = 1;
    pkt->workgroup_size_z = 1;
    pkt->grid_size_x = 256 * 512;
    pkt->grid_size_y = 1;
    pkt->grid_size_z = 1;
    pkt->private_segment_size = pseg;
    pkt->group_segment_size = gseg;
    pkt->kernel_object = kobj;
    pkt->kernarg_address = karg;
    pkt->completion_signal = sig;
    const uint16_t header = (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                       (1 << HSA_PACKET_HEADER_BARRIER) |
                                       (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                       (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
    const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
    __atomic_store_n(reinterpret_cast<uint32_t*>(pkt), (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
    hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)idx);
    hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
  };
  struct Case {
    const char* name;
    void* karg;
    bool dev;
    int acq;
  } cases[] = {{"aql_sys", karg_sys, false, HSA_FENCE_SCOPE_SYSTEM},
               {"aql_dev", karg_dev, true, HSA_FENCE_SCOPE_SYSTEM},
               {"aql_agent", karg_dev, true, HSA_FENCE_SCOPE_AGENT}};
  for (const Case& c : cases) {
    for (int i = 0; i < 20; ++i) dispatch(c.karg, c.dev, c.acq);
    std::vector<double> v;
    for (int i = 0; i < samples; ++i) {
      idle(200);
      const auto t0 = clk::now();
      dispatch(c.karg, c.dev, c.acq);
      v.push_back(us_since(t0));
    }
    unsigned host[256];
    CK(hipMemcpy(host, out, sizeof host, hipMemcpyDeviceToHost));
    bool ok = true;
    for (int b = 0; b < 256; ++b) ok &= host[b] == (unsigned)(b % 210) + 1u;
    if (!ok) fprintf(stderr, "%s: wrong results\n", c.name);
    report(c.name, v);
    CK(hipMemset(out, 0, 256 * sizeof(unsigned)));
    CK(hipDeviceSynchronize());
  }
  HK(hsa_signal_destroy(sig));
  HK(hsa_queue_destroy(q));
  HK(hsa_executable_destroy(exe));
  HK(hsa_code_object_reader_destroy(rd));
  HK(hsa_memory_free(karg_sys));
  HK(hsa_amd_memory_pool_free(karg_dev));
  CK(hipFree(out));
  HK(hsa_shut_down());
  return 0;
}
#endif
