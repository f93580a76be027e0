// pybind11 bindings for the xGMI peer all-reduce: IPC buffer ownership,
// handle export/import and the launch (submodule `_hip.comm`).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../common/hip_common.h"
#include "xgmi_allreduce.h"

namespace py = pybind11;

namespace cme::comm {

namespace {

constexpr size_t kIpcGranule = 2u << 20;
size_t round_alloc(size_t b) { return (b + kIpcGranule - 1) / kIpcGranule * kIpcGranule; }

py::bytes handle_bytes(void* p, const char* what) {
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) {
    char buf[256];
    std::snprintf(buf, sizeof(buf), "hipIpcGetMemHandle(%s) failed: %s (is HSA_ENABLE_IPC_MODE_LEGACY=0 set?)",
                  what, hipGetErrorString(e));
    throw std::runtime_error(buf);
  }
  return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
}

void* open_handle(const std::string& b) {
  CME_REQUIRE(b.size() == sizeof(hipIpcMemHandle_t), "xgmi: bad IPC handle size");
  hipIpcMemHandle_t h;
  std::memcpy(&h, b.data(), sizeof(h));
  void* p = nullptr;
  HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  return p;
}

// Process-wide pool of exported IPC allocations.  A bucket's buffer is never hipFree'd: closing returns
// it here and the next bucket of a similar size takes it back (same allocation, same IPC handle).
// Reason (measured, 4 ranks sharing one GPU): after buffers were freed and re-allocated, a peer's
// hipIpcOpenMemHandle of a NEW handle returned a mapping of a different rank's buffer -- the runtime's
// import cache keyed on recycled memory.  Reusing allocations removes the churn; the signature check
// in open() catches any remaining mix-up loudly instead of summing the wrong gradients.
struct IpcPool {
  std::vector<std::pair<void*, size_t>> free_;
  void* take(size_t bytes, size_t* got) {
    size_t best = 0;
    for (size_t i = 1; i < free_.size(); ++i)
      if (free_[i].second >= bytes && (free_[best].second < bytes || free_[i].second < free_[best].second)) best = i;
    if (!free_.empty() && free_[best].second >= bytes && free_[best].second <= 2 * bytes + kIpcGranule) {
      void* p = free_[best].first;
      *got = free_[best].second;
      free_.erase(free_.begin() + best);
      return p;
    }
    void* p = nullptr;
    HIP_CHECK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained));
    *got = bytes;
    return p;
  }
  // Fine-grained device memory for the exported buffers.  Peers store flags into this buffer and read
  // gradients from it across xGMI; in fine-grained memory the owner's polls are coherent with those
  // remote stores by construction, instead of depending on how the owner's L2 treats a coarse-grained
  // line that another GPU wrote.  Measured with ranks sharing one GPU: same step time and all-reduce
  // latency as plain hipMalloc memory (profiles/xgmi_fused_notes.md).
  void give(void* p, size_t bytes) { free_.emplace_back(p, bytes); }
};
IpcPool& ipc_pool() {
  static IpcPool* p = new IpcPool();  // never destroyed: buffers live until the process exits
  return *p;
}

struct Signature {
  uint64_t magic, rank, nonce, bytes;
};
constexpr uint64_t kSigMagic = 0x43'4D'45'58'47'4D'49'31ull;  // "CMEXGMI1"

// Owns this rank's IPC buffers and the peers' mappings.
class XgmiComm {
 public:
  // flag_slots: minimum number of [kMaxRanks]-word flag rows (a kernel that signals per workgroup tile
  // -- the wgrad launch with the all-reduce fused in -- needs one per tile; default one per chunk)
  // slab_tiles: tiles of the owner-tile push form's receive areas (0: none; XgmiDesc::myslab)
  XgmiComm(int rank, int world, int64_t n, int elt_bytes, int64_t flag_slots = 0, int64_t slab_tiles = 0) {
    CME_REQUIRE(world >= 1 && world <= kMaxRanks, "XgmiComm: 1 <= world <= 8");
    CME_REQUIRE(rank >= 0 && rank < world, "XgmiComm: bad rank");
    CME_REQUIRE(elt_bytes == 2 || elt_bytes == 4 || elt_bytes == 8, "XgmiComm: bf16 wire, f32 or f64");
    elt_ = elt_bytes;
    d_.rank = rank;
    d_.world = world;
    d_.n = n;
    d_.npad = xgmi_padded_count(n);
    nblocks_ = std::max<int64_t>({1, xgmi_num_blocks(n), flag_slots});
    // ONE dedicated allocation per rank, [data: 2 x npad | flags: nblocks x 8 words], exported with one
    // IPC handle.  Rounded to 2 MiB so the runtime never sub-allocates it (hipIpcGetMemHandle rejects
    // sub-allocated pointers); fine-grained device memory (IpcPool::fine_grained; hipDeviceMallocUncached
    // pages did not export reliably), with every flag access a system-scope atomic.
    CME_REQUIRE(slab_tiles >= 0, "XgmiComm: slab_tiles >= 0");
    flags_off_ = (2 * d_.npad * elt_bytes + 4095) / 4096 * 4096;
    slab_off_ = flags_off_ + (flag_bytes() + 4095) / 4096 * 4096;
    const size_t slab_bytes = (size_t)slab_tiles * (kMaxRanks + 1) * kSlabTile * sizeof(unsigned long long);
    sig_off_ = slab_off_ + (slab_bytes + 4095) / 4096 * 4096;
    d_.mybuf = ipc_pool().take(round_alloc(sig_off_ + sizeof(Signature)), &alloc_bytes_);
    HIP_CHECK(hipMemset(d_.mybuf, 0, alloc_bytes_));
    std::random_device rd;
    sig_ = Signature{kSigMagic, (uint64_t)rank, ((uint64_t)rd() << 32) ^ rd(), alloc_bytes_};
    HIP_CHECK(hipMemcpy(static_cast<char*>(d_.mybuf) + sig_off_, &sig_, sizeof(sig_), hipMemcpyHostToDevice));
    d_.myflags = reinterpret_cast<uint32_t*>(static_cast<char*>(d_.mybuf) + flags_off_);
    d_.slab_tiles = slab_tiles;
    if (slab_tiles) d_.myslab = reinterpret_cast<unsigned long long*>(static_cast<char*>(d_.mybuf) + slab_off_);
    HIP_CHECK(hipMalloc(&d_.epochs, nblocks_ * sizeof(uint32_t)));
    HIP_CHECK(hipMemset(d_.epochs, 0, nblocks_ * sizeof(uint32_t)));
    HIP_CHECK(hipMalloc(&d_.err, sizeof(int)));
    HIP_CHECK(hipMemset(d_.err, 0, sizeof(int)));
    HIP_CHECK(hipDeviceSynchronize());
    d_.peers[rank] = d_.mybuf;
    d_.peerflags[rank] = d_.myflags;
    d_.peerslabs[rank] = d_.myslab;
  }
  ~XgmiComm() { close(); }

  // (IPC handle, signature) -- the signature lets every peer verify what its mapping shows
  py::tuple handles() const {
    return py::make_tuple(handle_bytes(d_.mybuf, "buffer"),
                          py::bytes(reinterpret_cast<const char*>(&sig_), sizeof(sig_)));
  }

  void open(const std::vector<std::pair<std::string, std::string>>& all) {
    CME_REQUIRE((int)all.size() == d_.world, "XgmiComm.open: need one handle pair per rank");
    for (int r = 0; r < d_.world; ++r) {
      if (r == d_.rank) continue;
      d_.peers[r] = open_handle(all[r].first);
      opened_.push_back(d_.peers[r]);
      d_.peerflags[r] = reinterpret_cast<uint32_t*>(static_cast<char*>(d_.peers[r]) + flags_off_);
      if (d_.slab_tiles)
        d_.peerslabs[r] = reinterpret_cast<unsigned long long*>(static_cast<char*>(d_.peers[r]) + slab_off_);
      // the mapping must show THAT rank's buffer (its signature, written at its construction)
      CME_REQUIRE(all[r].second.size() == sizeof(Signature), "XgmiComm.open: bad signature size");
      Signature want, seen;
      std::memcpy(&want, all[r].second.data(), sizeof(want));
      HIP_CHECK(hipMemcpy(&seen, static_cast<char*>(d_.peers[r]) + sig_off_, sizeof(seen), hipMemcpyDeviceToHost));
      if (std::memcmp(&want, &seen, sizeof(want)) != 0) {
        char buf[200];
        std::snprintf(buf, sizeof(buf), "XgmiComm.open: the IPC mapping of rank %d shows another buffer "
                      "(magic %llx rank %llu)", r, (unsigned long long)seen.magic, (unsigned long long)seen.rank);
        throw std::runtime_error(buf);
      }
    }
    ready_ = true;
  }

  void run(int dtype, uintptr_t grads, uintptr_t params, double lr, uintptr_t planes, int np, int64_t w1n, int mode,
           int64_t n, uintptr_t stream, uintptr_t status) {
    CME_REQUIRE(ready_ || d_.world == 1, "XgmiComm.run: open() the peer handles first");
    CME_REQUIRE(n == d_.n, "XgmiComm.run: element count differs from the one the buffers were sized for");
    CME_REQUIRE((dtype == 0 && elt_ == 4) || (dtype == 1 && elt_ == 8) || (dtype == 2 && elt_ == 2),
                "XgmiComm.run: dtype does not match the buffer's wire element size");
    xgmi_allreduce(d_, dtype, reinterpret_cast<const void*>(grads), reinterpret_cast<void*>(params), lr,
                   reinterpret_cast<void*>(planes), np, w1n, mode, reinterpret_cast<hipStream_t>(stream),
                   reinterpret_cast<const void*>(status));
  }

  int error() const {
    int e = 0;
    HIP_CHECK(hipMemcpy(&e, d_.err, sizeof(int), hipMemcpyDeviceToHost));
    return e;
  }

  // teardown in two phases across the group: every rank unmaps its peers (close_peers), a barrier,
  // then every rank frees its own buffers (close) -- never free while a peer still maps them
  void close_peers() {
    if (!opened_.empty()) HIP_CHECK(hipDeviceSynchronize());
    for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
    opened_.clear();
    for (int r = 0; r < d_.world; ++r)
      if (r != d_.rank) {
        d_.peers[r] = nullptr;
        d_.peerflags[r] = nullptr;
        d_.peerslabs[r] = nullptr;
      }
    ready_ = false;
  }

  void close() {
    close_peers();
    if (d_.mybuf) {  // back to the pool (see IpcPool); its signature is cleared
      (void)hipDeviceSynchronize();
      (void)hipMemset(d_.mybuf, 0, alloc_bytes_);
      ipc_pool().give(d_.mybuf, alloc_bytes_);
    }
    if (d_.epochs) (void)hipFree(d_.epochs);
    if (d_.err) (void)hipFree(d_.err);
    d_ = XgmiDesc{};
    ready_ = false;
  }

  int64_t nblocks() const { return nblocks_; }
  int64_t npad() const { return d_.npad; }
  // address of the descriptor, for a kernel that fuses this all-reduce in (MlpStep.set_xgmi); valid
  // while this object is open
  uintptr_t desc_address() const { return reinterpret_cast<uintptr_t>(&d_); }
  // address of the sticky timed-out-wait word (int, device): a launch that must apply nothing once a peer
  // wait of this bucket timed out reads it (the tensor-parallel weight-gradient launch, SplitStepArgs::ag_err)
  uintptr_t err_address() const { return reinterpret_cast<uintptr_t>(d_.err); }

 private:
  size_t flag_bytes() const { return (size_t)nblocks_ * kMaxRanks * sizeof(uint32_t); }
  XgmiDesc d_;
  int64_t nblocks_ = 0;
  int elt_ = 4;  // wire element bytes: 2 (bf16), 4 (f32), 8 (f64)
  static constexpr int kSlabTile = 512;  // granules per tile slot (mlp_split.hip kXpTile)
  size_t flags_off_ = 0, slab_off_ = 0, sig_off_ = 0, alloc_bytes_ = 0;
  Signature sig_{};
  bool ready_ = false;
  std::vector<void*> opened_;
};

}  // namespace

}  // namespace cme::comm

void bind_comm(py::module_& m) {
  using cme::comm::XgmiComm;
  auto sm = m.def_submodule("comm", "xGMI peer-to-peer all-reduce (IPC buffers, SGD fused)");
  py::class_<XgmiComm>(sm, "XgmiComm")
      .def(py::init<int, int, int64_t, int, int64_t, int64_t>(), py::arg("rank"), py::arg("world"), py::arg("n"),
           py::arg("elt_bytes"), py::arg("flag_slots") = 0, py::arg("slab_tiles") = 0)
      .def("handles", &XgmiComm::handles)
      .def("open", &XgmiComm::open)
      .def("run", &XgmiComm::run, py::arg("dtype"), py::arg("grads"), py::arg("params"), py::arg("lr"),
           py::arg("planes"), py::arg("np"), py::arg("w1n"), py::arg("mode"), py::arg("n"), py::arg("stream"),
           py::arg("status") = 0)
      .def("error", &XgmiComm::error)
      .def("close", &XgmiComm::close)
      .def("close_peers", &XgmiComm::close_peers)
      .def_property_readonly("nblocks", &XgmiComm::nblocks)
      .def_property_readonly("npad", &XgmiComm::npad)
      .def_property_readonly("desc_address", &XgmiComm::desc_address)
      .def_property_readonly("err_address", &XgmiComm::err_address);
  sm.attr("MODE_SGD") = cme::comm::kModeSgd;
  sm.attr("MODE_ALLREDUCE") = cme::comm::kModeAllReduce;
  sm.attr("MAX_RANKS") = cme::comm::kMaxRanks;
}
