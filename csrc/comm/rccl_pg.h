// RCCL process group: GPU collectives over xGMI through RCCL, issued on a side HIP stream.
//
// Parity target: c10d ProcessGroupNCCL (c10d/ProcessGroupNCCL.hpp:318; SURVEY.md §2.3 U4,
// §2.4): comm-per-PG created eagerly from a store-exchanged unique id, dedicated comm stream
// fenced against the caller's stream by events, async Work, a watchdog thread that aborts a
// hung communicator after the PG timeout, new_group via ncclCommSplit.  The stream / Work /
// watchdog machinery is GpuPG (gpu_pg.h), shared with the xGMI backend.
#pragma once

#include <rccl/rccl.h>

#include "gpu_pg.h"
#include "xgmi_engine.h"

namespace ringdp {

class RcclPG : public GpuPG {
 public:
  // Bootstraps a communicator: rank 0 publishes the unique id in `store` under "rccl/uid".
  RcclPG(std::shared_ptr<Store> store, int rank, int size, int device, std::chrono::milliseconds timeout);
  // Wraps an already-initialised communicator (ncclCommSplit result); `store` (may be null) serves
  // the optional small-message xGMI path of the child group.
  RcclPG(ncclComm_t comm, std::shared_ptr<Store> store, int rank, int size, int device,
         std::chrono::milliseconds timeout);
  ~RcclPG() override;

  std::string backend_name() const override { return "rccl"; }

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
  std::shared_ptr<Work> coalesced(std::vector<CollOp>& ops) override;
  // `timeout_ms` > 0 overrides the parent's timeout for the child group.
  std::shared_ptr<ProcessGroup> split(const std::vector<int>& ranks, const std::string& tag) override;
  std::shared_ptr<ProcessGroup> split_with_timeout(const std::vector<int>& ranks, const std::string& tag,
                                                   int64_t timeout_ms);
  void shutdown() override;
  std::string backend_failure() override;

  // Small all-reduces on the xGMI one-shot kernel (RINGDP_P2P_ALLREDUCE_MAX_BYTES > 0 at creation).
  int64_t p2p_max_bytes() const { return xg_ ? p2p_max_bytes_ : 0; }
  void set_p2p_enabled(bool on) { p2p_on_ = on; }

 protected:
  void abort_backend() override;
  std::string poll_async_error() override;

 private:
  void setup_small_path(const std::shared_ptr<Store>& store);

  ncclComm_t comm_ = nullptr;
  std::shared_ptr<Store> store_;
  std::unique_ptr<XgmiEngine> xg_;
  int64_t p2p_max_bytes_ = 0;
  bool p2p_on_ = true;
};

ncclDataType_t to_nccl_dtype(at::ScalarType t);
ncclRedOp_t to_nccl_op(ReduceOp op);
// kern::XgDtype for a tensor dtype (-1: unsupported)
int to_xg_dtype(at::ScalarType t);

}  // namespace ringdp
