// ringdp process-group abstraction: collectives returning async Work handles.
//
// Parity target: c10d::ProcessGroup / Work as used by the reference through
// init_process_group + DDP.  Two backends implement it:
//   * RcclPG   (rccl_pg.cpp)  - GPU tensors, RCCL over xGMI on a side HIP stream + watchdog
//   * HostRingPG (host_ring.cpp) - CPU tensors, TCP ring collectives on a worker thread
#pragma once

#include <ATen/ATen.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../common.h"
#include "../store/store.h"

namespace ringdp {

enum class ReduceOp : int { SUM = 0, PRODUCT = 1, MIN = 2, MAX = 3, AVG = 4, BAND = 5, BOR = 6, BXOR = 7 };

enum class OpType : int {
  ALLREDUCE = 0,
  BROADCAST,
  ALLGATHER,
  ALLGATHER_BASE,
  REDUCE_SCATTER_BASE,
  REDUCE,
  GATHER,
  SCATTER,
  ALLTOALL_BASE,
  SEND,
  RECV,
  BARRIER,
  COALESCED,
  GRAPH_REPLAY,  // a captured step (hipGraph) that contains this group's collectives
};

const char* op_name(OpType t);

class Work {
 public:
  Work(OpType op, uint64_t seq) : op_(op), seq_(seq), start_us_(now_us()) {}
  virtual ~Work() = default;

  // CPU backends: blocks until done.  GPU backends: makes the caller's current stream wait on
  // completion (no host block) unless `blocking` is set.  Raises the op's error if any.
  virtual void wait(bool blocking = false) = 0;
  virtual bool is_completed() = 0;
  // Host-blocking completion.
  virtual void synchronize() { wait(true); }
  std::vector<at::Tensor>& result() { return outputs_; }
  OpType op() const { return op_; }
  uint64_t seq() const { return seq_; }
  int64_t start_us() const { return start_us_; }
  // Wall time (us) between enqueue and observed completion (GPU: device-side duration when known).
  virtual double duration_us() { return -1.0; }

 protected:
  OpType op_;
  uint64_t seq_;
  int64_t start_us_;
  std::vector<at::Tensor> outputs_;
  friend class HostRingPG;
  friend class GpuPG;
  friend class FakePG;
};

// A Work completed on a host thread (promise-style).
class HostWork : public Work {
 public:
  using Work::Work;
  void wait(bool blocking = false) override;
  bool is_completed() override { return done_.load(); }
  void finish(std::exception_ptr err = nullptr);
  double duration_us() override { return duration_us_; }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::atomic<bool> done_{false};
  std::exception_ptr err_;
  double duration_us_ = -1.0;
};

// Several Works completed together (the default coalesced() of host backends).
class CompositeWork : public Work {
 public:
  CompositeWork(std::vector<std::shared_ptr<Work>> parts, uint64_t seq)
      : Work(OpType::COALESCED, seq), parts_(std::move(parts)) {}
  void wait(bool blocking = false) override {
    for (auto& p : parts_) p->wait(blocking);
  }
  bool is_completed() override {
    for (auto& p : parts_)
      if (!p->is_completed()) return false;
    return true;
  }

 private:
  std::vector<std::shared_ptr<Work>> parts_;
};

// One collective of a coalesced batch (ringdp.distributed._coalescing_manager).
struct CollOp {
  enum Kind : int { ALLREDUCE = 0, BROADCAST = 1, ALLGATHER_INTO = 2, REDUCE_SCATTER = 3 };
  int kind = ALLREDUCE;
  at::Tensor out;  // in-place tensor for ALLREDUCE / BROADCAST
  at::Tensor in;   // ALLGATHER_INTO / REDUCE_SCATTER input
  int root = 0;
  ReduceOp op = ReduceOp::SUM;
};

struct AllToAllSplits {
  std::vector<int64_t> output_split_sizes;
  std::vector<int64_t> input_split_sizes;
};

class ProcessGroup : public std::enable_shared_from_this<ProcessGroup> {
 public:
  ProcessGroup(int rank, int size) : rank_(rank), size_(size) {}
  virtual ~ProcessGroup() = default;

  int rank() const { return rank_; }
  int size() const { return size_; }
  virtual std::string backend_name() const = 0;
  // While on, collectives are issued on the caller's current stream even in side-stream mode (GPU groups;
  // the reducer's inline buckets inside a segmented hipGraph capture).  No-op elsewhere.
  virtual void set_caller_stream_ops(bool /*on*/) {}

  virtual std::shared_ptr<Work> allreduce(std::vector<at::Tensor>& tensors, ReduceOp op) = 0;
  // Many tensors reduced as one fused op (one flat buffer / one RCCL group).
  virtual std::shared_ptr<Work> allreduce_coalesced(std::vector<at::Tensor>& tensors,
                                                    ReduceOp op) = 0;
  virtual std::shared_ptr<Work> broadcast(std::vector<at::Tensor>& tensors, int root) = 0;
  virtual std::shared_ptr<Work> allgather(std::vector<at::Tensor>& outputs,
                                          const at::Tensor& input) = 0;
  virtual std::shared_ptr<Work> allgather_into_tensor(at::Tensor& output,
                                                      const at::Tensor& input) = 0;
  virtual std::shared_ptr<Work> reduce_scatter_tensor(at::Tensor& output, const at::Tensor& input,
                                                      ReduceOp op) = 0;
  virtual std::shared_ptr<Work> reduce(at::Tensor& tensor, int root, ReduceOp op) = 0;
  virtual std::shared_ptr<Work> gather(std::vector<at::Tensor>& outputs, const at::Tensor& input,
                                       int root) = 0;
  virtual std::shared_ptr<Work> scatter(at::Tensor& output, std::vector<at::Tensor>& inputs,
                                        int root) = 0;
  virtual std::shared_ptr<Work> alltoall_base(at::Tensor& output, const at::Tensor& input,
                                              const AllToAllSplits& splits) = 0;
  virtual std::shared_ptr<Work> send(at::Tensor& tensor, int dst, int tag) = 0;
  virtual std::shared_ptr<Work> recv(at::Tensor& tensor, int src, int tag) = 0;
  virtual std::shared_ptr<Work> barrier() = 0;

  // A batch of collectives issued as one unit.  GPU backends fuse it into one RCCL group (one
  // launch, one completion event); the default issues them in order and waits for all.
  virtual std::shared_ptr<Work> coalesced(std::vector<CollOp>& ops) {
    std::vector<std::shared_ptr<Work>> parts;
    for (auto& c : ops) {
      switch (c.kind) {
        case CollOp::ALLREDUCE: {
          std::vector<at::Tensor> v{c.out};
          parts.push_back(allreduce(v, c.op));
          break;
        }
        case CollOp::BROADCAST: {
          std::vector<at::Tensor> v{c.out};
          parts.push_back(broadcast(v, c.root));
          break;
        }
        case CollOp::ALLGATHER_INTO:
          parts.push_back(allgather_into_tensor(c.out, c.in));
          break;
        case CollOp::REDUCE_SCATTER:
          parts.push_back(reduce_scatter_tensor(c.out, c.in, c.op));
          break;
      }
    }
    return std::make_shared<CompositeWork>(std::move(parts), next_seq());
  }

  // Collective creation of a sub-group.  Every member of this group must call it with the same
  // `ranks`; non-members receive nullptr.
  virtual std::shared_ptr<ProcessGroup> split(const std::vector<int>& ranks,
                                              const std::string& tag) = 0;
  virtual void shutdown() {}
  virtual void abort() { shutdown(); }

  uint64_t next_seq() { return ++seq_; }
  uint64_t seq() const { return seq_.load(); }

 protected:
  int rank_;
  int size_;
  std::atomic<uint64_t> seq_{0};
};

// Elementwise in-place reduction dst = op(dst, src) on CPU tensors of identical dtype / numel.
void host_reduce_inplace(at::Tensor& dst, const at::Tensor& src, ReduceOp op);
void host_reduce_raw(void* dst, const void* src, int64_t numel, at::ScalarType dtype, ReduceOp op);

}  // namespace ringdp
