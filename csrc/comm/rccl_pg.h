// RCCL process group: GPU collectives over xGMI, issued on a side HIP stream.
//
// Parity target: c10d ProcessGroupNCCL (c10d/ProcessGroupNCCL.hpp:318; SURVEY.md §2.3 U4,
// §2.4): comm-per-PG created eagerly from a store-exchanged unique id, dedicated comm stream
// fenced against the caller's stream by events, async Work, a watchdog thread that aborts a
// hung communicator after the PG timeout, new_group via ncclCommSplit.
#pragma once

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <deque>
#include <thread>

#include "p2p_allreduce.h"
#include "process_group.h"

namespace ringdp {

using HipStream = c10::hip::HIPStreamMasqueradingAsCUDA;

class RcclPG;

// Completion beacon of a captured step (hipGraph).  The graph's last node (kern::replay_beacon_mark)
// writes the number of finished replays into host-coherent memory; the host counts replays it
// issued.  The watchdog compares the two with plain loads: watching a replay costs no HIP call on
// either thread (an event created + recorded per replay and queried/destroyed by the watchdog thread
// deadlocked inside the HIP runtime, ~1 in 3 ViT bench runs).
class ReplayBeacon {
 public:
  explicit ReplayBeacon(int device);
  ~ReplayBeacon();
  ReplayBeacon(const ReplayBeacon&) = delete;
  ReplayBeacon& operator=(const ReplayBeacon&) = delete;
  // Enqueue the marker on `stream` (call while capturing, after the step).
  void mark(hipStream_t stream);
  // The host issued one more replay.
  void issued() { issued_.fetch_add(1, std::memory_order_relaxed); }
  uint64_t issued_count() const { return issued_.load(std::memory_order_relaxed); }
  uint64_t completed() const { return __atomic_load_n(host_, __ATOMIC_ACQUIRE); }
  int device() const { return device_; }

  // watchdog bookkeeping (watchdog thread only)
  uint64_t last_done_ = 0;
  int64_t progress_us_ = 0;

 private:
  int device_;
  unsigned long long* host_ = nullptr;  // hipHostMalloc'd, coherent + mapped
  unsigned long long* dev_ = nullptr;   // device counter
  std::atomic<uint64_t> issued_{0};
};

class RcclWork : public Work {
 public:
  RcclWork(OpType op, uint64_t seq, RcclPG* pg, bool captured, bool timing);
  ~RcclWork() override;
  void wait(bool blocking = false) override;
  bool is_completed() override;
  double duration_us() override;

  hipEvent_t done_ = nullptr;
  hipEvent_t start_ = nullptr;  // only when timing is enabled
  int64_t deadline_us_ = 0;
  bool captured_ = false;

 private:
  RcclPG* pg_;
};

class RcclPG : public ProcessGroup {
 public:
  // Bootstraps a communicator: rank 0 publishes the unique id in `store` under "rccl/uid".
  RcclPG(std::shared_ptr<Store> store, int rank, int size, int device,
         std::chrono::milliseconds timeout);
  // Wraps an already-initialised communicator (ncclCommSplit result).
  RcclPG(ncclComm_t comm, int rank, int size, int device, std::chrono::milliseconds timeout);
  ~RcclPG() override;

  std::string backend_name() const override { return "rccl"; }
  int device() const { return device_; }
  hipStream_t comm_stream() const { return comm_stream_.stream(); }

  std::shared_ptr<Work> allreduce(std::vector<at::Tensor>& tensors, ReduceOp op) override;
  std::shared_ptr<Work> allreduce_coalesced(std::vector<at::Tensor>& tensors,
                                            ReduceOp op) override;
  std::shared_ptr<Work> broadcast(std::vector<at::Tensor>& tensors, int root) override;
  std::shared_ptr<Work> allgather(std::vector<at::Tensor>& outputs,
                                  const at::Tensor& input) override;
  std::shared_ptr<Work> allgather_into_tensor(at::Tensor& output,
                                              const at::Tensor& input) override;
  std::shared_ptr<Work> reduce_scatter_tensor(at::Tensor& output, const at::Tensor& input,
                                              ReduceOp op) override;
  std::shared_ptr<Work> reduce(at::Tensor& tensor, int root, ReduceOp op) override;
  std::shared_ptr<Work> gather(std::vector<at::Tensor>& outputs, const at::Tensor& input,
                               int root) override;
  std::shared_ptr<Work> scatter(at::Tensor& output, std::vector<at::Tensor>& inputs,
                                int root) override;
  std::shared_ptr<Work> alltoall_base(at::Tensor& output, const at::Tensor& input,
                                      const AllToAllSplits& splits) override;
  std::shared_ptr<Work> send(at::Tensor& tensor, int dst, int tag) override;
  std::shared_ptr<Work> recv(at::Tensor& tensor, int src, int tag) override;
  std::shared_ptr<Work> barrier() override;
  std::shared_ptr<Work> coalesced(std::vector<CollOp>& ops) override;
  std::shared_ptr<ProcessGroup> split(const std::vector<int>& ranks,
                                      const std::string& tag) override;
  void shutdown() override;
  void abort() override;

  // Host-blocks until every eagerly issued op has completed and clears the watchdog list, so
  // no event query can race a subsequent hipGraph capture.
  void drain();
  // Puts the replays of a captured step (whose collectives the per-op watchdog entries cannot see)
  // under this group's watchdog: while replays are outstanding, one must complete within the group
  // timeout, else the communicator is aborted and the process exits non-zero like any other hung
  // collective.
  void watch_beacon(const std::shared_ptr<ReplayBeacon>& beacon);
  bool aborted() const { return aborted_.load(); }
  std::string error_message() {
    std::lock_guard<std::mutex> lk(wd_mu_);
    return error_;
  }
  void set_timing(bool on) { timing_ = on; }
  bool timing() const { return timing_; }
  void set_async_error_handling(bool on) { async_error_handling_ = on; }
  // One-shot P2P all-reduce for small buckets (RINGDP_P2P_ALLREDUCE_MAX_BYTES > 0 at creation).
  int64_t p2p_max_bytes() const { return p2p_ ? p2p_->max_bytes() : 0; }
  bool same_stream() const { return same_stream_; }
  void set_p2p_enabled(bool on) { p2p_on_ = on; }
  std::chrono::milliseconds timeout() const { return timeout_; }

 private:
  template <typename Fn>
  std::shared_ptr<Work> launch(OpType op, const std::vector<at::Tensor>& tensors, Fn&& body);
  void init_common();
  void watchdog_loop();
  void fail(const std::string& msg);
  void check_tensor(const at::Tensor& t, const char* what) const;

  ncclComm_t comm_ = nullptr;
  std::unique_ptr<P2PAllReduce> p2p_;
  bool p2p_on_ = true;
  int device_;
  std::chrono::milliseconds timeout_;
  // Normal priority by default: on gfx950 an eager step with its collectives on a high-priority
  // stream measured 1.26 ms vs 0.55 ms (ConvNet B=4096, one rank, forced comm); graph replay is
  // unaffected.  RINGDP_COMM_HIGH_PRIORITY=1 restores the high-priority stream.
  HipStream comm_stream_;
  hipEvent_t ready_ = nullptr;
  bool timing_ = false;
  bool same_stream_ = false;  // issue collectives on the caller's stream (see init_common)
  bool async_error_handling_ = true;

  std::mutex launch_mu_;
  std::mutex wd_mu_;
  std::condition_variable wd_cv_;
  std::deque<std::shared_ptr<RcclWork>> inflight_;
  std::mutex beacon_mu_;
  std::vector<std::weak_ptr<ReplayBeacon>> beacons_;
  std::thread watchdog_;
  std::atomic<bool> stop_{false};
  std::atomic<bool> aborted_{false};
  std::string error_;
  friend class RcclWork;
};

ncclDataType_t to_nccl_dtype(at::ScalarType t);
ncclRedOp_t to_nccl_op(ReduceOp op);

}  // namespace ringdp
