// Peer-to-peer (xGMI) all-reduce for small gradient buckets, SGD fused.
// See xgmi_allreduce.hip for the protocol.  The IPC plumbing (allocation,
// handle export/import) lives in xgmi_ipc.cpp; Python drives the handle
// exchange through any torch.distributed group (cme213_sp18_amd/parallel/xgmi.py).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace cme::comm {

constexpr int kMaxRanks = 8;  // one xGMI hive
constexpr int kModeSgd = 0;        // params -= lr * sum(grads)   (+ bf16 plane/shadow refresh)
constexpr int kModeAllReduce = 1;  // grads  := sum(grads)
// two-shot forms (reduce-scatter + all-gather over peer reads, exact wire only): chunk c is owned by rank
// c % world, which sums the R gradient chunks (rank order: the one-shot's bits) and applies the update
// (sharded SGD) or keeps the sum; every other rank then copies the owner's result.  Each xGMI link carries
// 2 S / R bytes instead of the one-shot's S: the form for buckets of a few MB at 8 ranks.
constexpr int kModeSgd2 = 2;
constexpr int kModeAllReduce2 = 3;

struct XgmiDesc {
  int rank = 0, world = 1;
  int64_t n = 0, npad = 0;            // elements, padded elements per buffer half
  void* mybuf = nullptr;              // [2][npad] my IPC data buffer
  void* peers[kMaxRanks] = {};        // every rank's data buffer as mapped here (peers[rank] == mybuf)
  uint32_t* myflags = nullptr;        // [nblocks][kMaxRanks] uncached, IPC-exported
  uint32_t* peerflags[kMaxRanks] = {};
  uint32_t* epochs = nullptr;         // [nblocks] local
  int* err = nullptr;                 // set to 1 when a wait timed out
  // the owner-tile push form's receive areas (XgmiFuse::push), [slab_tiles][8 + 1][512] 8-byte granules inside
  // every rank's IPC allocation; slab_tiles == 0: none
  unsigned long long* myslab = nullptr;
  unsigned long long* peerslabs[kMaxRanks] = {};
  int64_t slab_tiles = 0;
};

int64_t xgmi_padded_count(int64_t n);
int64_t xgmi_num_blocks(int64_t n);

// dtype: 0 f32, 1 f64, 2 f32 gradients over a bf16 wire (the IPC buffers hold bf16; summed in fp32).  planes: bf16 [np][w1n] refreshed from the first w1n params (np 1 or 3), or null.
// status: this rank's gradient status element (the T-typed word after b2, or null): non-zero = this rank's
// step is untrusted -> the rank takes no part (publishes nothing, applies nothing); its peers' waits then
// time out and apply nothing either, exactly as for a stalled rank.
void xgmi_allreduce(const XgmiDesc& d, int dtype, const void* grads, void* params, double lr, void* planes, int np,
                    int64_t w1n, int mode, hipStream_t s, const void* status = nullptr);

}  // namespace cme::comm
