// Host (CPU) ring backend: the `gloo`-compatible CPU path (BASELINE config #1).
#pragma once

#include <deque>
#include <functional>
#include <thread>

#include "process_group.h"

namespace ringdp {

class HostRingPG : public ProcessGroup {
 public:
  HostRingPG(std::shared_ptr<Store> store, int rank, int size, std::chrono::milliseconds timeout,
             const std::string& bind_hint);
  ~HostRingPG() override;

  std::string backend_name() const override { return "host_ring"; }

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
  std::shared_ptr<ProcessGroup> split(const std::vector<int>& ranks,
                                      const std::string& tag) override;
  void shutdown() override;

 private:
  struct Queue {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<void()>> tasks;
    // Finished tasks, still holding their captures (tensors, the Work).  The worker thread never destroys
    // them: the last reference to a tensor whose Python object was already dropped must be released on a
    // thread that may take the GIL, and a worker taking it while the interpreter finalises is terminated
    // (pthread_exit through a noexcept frame: "terminate called without an active exception").  The
    // caller's thread frees them on its next enqueue and at shutdown.
    std::vector<std::function<void()>> done;
    std::thread th;
    bool stop = false;
  };
  void start_queue(Queue& q);
  void stop_queue(Queue& q);
  std::shared_ptr<Work> enqueue(Queue& q, OpType op, std::function<void(HostWork&)> fn);

  // Ring / mesh primitives (run on the collective worker thread).
  void sendrecv(int send_peer, const void* sbuf, size_t sbytes, int recv_peer, void* rbuf,
                size_t rbytes, uint64_t seq, OpType op);
  void send_to(int peer, const void* buf, size_t bytes, uint64_t seq, OpType op,
               const std::vector<int>& mesh);
  void recv_from(int peer, void* buf, size_t bytes, uint64_t seq, OpType op,
                 const std::vector<int>& mesh);
  void ring_allreduce(at::Tensor& flat, ReduceOp op, uint64_t seq);
  void ring_reduce_scatter(char* data, const std::vector<int64_t>& counts,
                           const std::vector<int64_t>& offs, at::ScalarType dtype, size_t esize,
                           ReduceOp op, uint64_t seq, OpType optype);
  void ring_allgather(char* data, const std::vector<int64_t>& bytes_per_rank,
                      const std::vector<int64_t>& byte_offs, uint64_t seq, OpType optype);
  void ring_broadcast(char* data, size_t bytes, int root, uint64_t seq);

  std::shared_ptr<Store> store_;
  std::chrono::milliseconds timeout_;
  std::string bind_hint_;
  std::vector<int> coll_fds_;  // full mesh for collectives (index = peer rank)
  std::vector<int> p2p_fds_;   // full mesh for point-to-point
  Queue coll_q_, send_q_, recv_q_;
  bool shut_ = false;
};

}  // namespace ringdp
