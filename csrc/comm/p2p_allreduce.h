// One-shot peer-to-peer all-reduce for small buckets on a single xGMI node (host side of
// csrc/kernels/p2p.hip).  Owned by an RcclPG when RINGDP_P2P_ALLREDUCE_MAX_BYTES > 0; the PG routes
// eligible all-reduces (fp32/bf16, SUM/AVG, size <= the threshold, 16-B multiple) here and
// everything else to RCCL.  Setup is collective over the group: every rank allocates uncached
// staging + flag memory, exports it by IPC handle through the store, maps every peer's, and the
// ranks agree (through the store) that all of them succeeded; otherwise the path stays off on all.
#pragma once

#include <hip/hip_runtime_api.h>

#include <memory>
#include <string>
#include <vector>

#include <ATen/ATen.h>

#include "../kernels/kernels.h"
#include "../store/store.h"

namespace ringdp {

class P2PAllReduce {
 public:
  // Returns nullptr (on every rank) when the group cannot use the path: more than 8 ranks,
  // ranks on different hosts, or an allocation/IPC failure on any rank.
  static std::unique_ptr<P2PAllReduce> create(const std::shared_ptr<Store>& store, int rank, int world,
                                              int device, int64_t max_bytes, int64_t timeout_ms);
  ~P2PAllReduce();

  bool eligible(const at::Tensor& t) const;
  // In place; `average` divides by the world size.  Stream-ordered on `s`, graph-capturable.
  void run(at::Tensor& t, bool average, hipStream_t s);
  // Host-blocking check of the kernel's timeout word (true: some peer never arrived).
  bool failed();
  int64_t max_bytes() const { return max_bytes_; }

 private:
  P2PAllReduce() = default;
  int rank_ = 0, world_ = 1, device_ = 0;
  int64_t max_bytes_ = 0, slot_bytes_ = 0;
  int seg_bytes_ = 8192;
  uint64_t timeout_ticks_ = 0;
  char* my_buf_ = nullptr;
  unsigned* my_flags_ = nullptr;
  unsigned* epochs_ = nullptr;
  int* error_ = nullptr;
  std::vector<void*> opened_;  // peer mappings to close
  kern::P2PArgs base_{};
};

}  // namespace ringdp
