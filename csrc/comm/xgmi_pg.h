// xGMI process group: every collective on ringdp's own kernels over IPC-mapped peer memory
// (csrc/kernels/xgmi.hip) - no RCCL.  Backend name "xgmi" (init_process_group("xgmi"), or
// RINGDP_GPU_BACKEND=xgmi to serve "nccl").
//
// Scope: ranks on one node (an 8x MI355X xGMI node, or several ranks sharing one GPU, which RCCL
// refuses).  Same Work / side stream / watchdog / hipGraph beacon contract as RcclPG (GpuPG).
// Every op is issued on the comm stream, so this group's ops execute in issue order (the kernels'
// slot reuse relies on it); one-rank groups skip the kernels (copies only).
#pragma once

#include "gpu_pg.h"
#include "xgmi_engine.h"

namespace ringdp {

class XgmiPG : public GpuPG {
 public:
  XgmiPG(std::shared_ptr<Store> store, int rank, int size, int device, std::chrono::milliseconds timeout);
  ~XgmiPG() override;

  std::string backend_name() const override { return "xgmi"; }

  std::shared_ptr<Work> allreduce(std::vector<at::Tensor>& tensors, ReduceOp op) override;
  std::shared_ptr<Work> allreduce_coalesced(std::vector<at::Tensor>& tensors, ReduceOp op) override;
  std::shared_ptr<Work> broadcast(std::vector<at::Tensor>& tensors, int root) override;
  std::shared_ptr<Work> allgather(std::vector<at::Tensor>& outputs, const at::Tensor& input) override;
  std::shared_ptr<Work> allgather_into_tensor(at::Tensor& output, const at::Tensor& input) override;
  std::shared_ptr<Work> reduce_scatter_tensor(at::Tensor& output, const at::Tensor& input,
                                              ReduceOp op) override;
  std::shared_ptr<Work> reduce(at::Tensor& tensor, int root, ReduceOp op) override;
  std::shared_ptr<Work> gather(std::vector<at::Tensor>& outputs, const at::Tensor& input, int root) override;
  std::shared_ptr<Work> scatter(at::Tensor& output, std::vector<at::Tensor>& inputs, int root) override;
  std::shared_ptr<Work> alltoall_base(at::Tensor& output, const at::Tensor& input,
                                      const AllToAllSplits& splits) override;
  std::shared_ptr<Work> send(at::Tensor& tensor, int dst, int tag) override;
  std::shared_ptr<Work> recv(at::Tensor& tensor, int src, int tag) override;
  std::shared_ptr<Work> barrier() override;
  std::shared_ptr<ProcessGroup> split(const std::vector<int>& ranks, const std::string& tag) override;
  void shutdown() override;
  std::string backend_failure() override;

  const XgmiConfig& config() const { return eng_->config(); }

 private:
  // in-place all-reduce of one contiguous tensor on stream s (16-B aligned data pointer)
  void allreduce_one(at::Tensor& t, ReduceOp op, hipStream_t s);
  at::Tensor scratch(int64_t nbytes);  // uint8, allocated on the comm stream

  // Sends run on a stream of their own: a send waits (on the device) only for its receiver to have
  // read the slot it refills, so with sends and receives on one in-order stream a send-then-recv
  // exchange of multi-slot messages would deadlock; receives and collectives stay on the comm stream.
  hipStream_t send_on(hipStream_t cs);   // fences the send stream after `cs`, returns it
  void join_sends(hipStream_t cs);       // `cs` waits for every send issued so far

  std::shared_ptr<Store> store_;
  std::unique_ptr<XgmiEngine> eng_;
  HipStream send_stream_;
  hipEvent_t send_fence_ = nullptr;
  hipEvent_t send_done_ = nullptr;
};

}  // namespace ringdp
