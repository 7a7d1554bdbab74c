// FakePG: the "fake" backend (upstream torch/testing/_internal/distributed/fake_pg.py:7-30).
// Every collective completes immediately and leaves its tensors untouched, so single-process
// tests can drive DDP / the reducer / sharding logic as rank r of an N-rank world without peers.
#pragma once

#include "process_group.h"

namespace ringdp {

class DoneWork : public Work {
 public:
  using Work::Work;
  void wait(bool) override {}
  bool is_completed() override { return true; }
  double duration_us() override { return 0.0; }
};

class FakePG : public ProcessGroup {
 public:
  FakePG(int rank, int size) : ProcessGroup(rank, size) {}
  std::string backend_name() const override { return "fake"; }

  std::shared_ptr<Work> allreduce(std::vector<at::Tensor>& t, ReduceOp) override {
    return done(OpType::ALLREDUCE, t);
  }
  std::shared_ptr<Work> allreduce_coalesced(std::vector<at::Tensor>& t, ReduceOp) override {
    return done(OpType::COALESCED, t);
  }
  std::shared_ptr<Work> broadcast(std::vector<at::Tensor>& t, int) override {
    return done(OpType::BROADCAST, t);
  }
  std::shared_ptr<Work> allgather(std::vector<at::Tensor>& outs, const at::Tensor&) override {
    return done(OpType::ALLGATHER, outs);
  }
  std::shared_ptr<Work> allgather_into_tensor(at::Tensor& out, const at::Tensor&) override {
    std::vector<at::Tensor> v{out};
    return done(OpType::ALLGATHER_BASE, v);
  }
  std::shared_ptr<Work> reduce_scatter_tensor(at::Tensor& out, const at::Tensor&, ReduceOp) override {
    std::vector<at::Tensor> v{out};
    return done(OpType::REDUCE_SCATTER_BASE, v);
  }
  std::shared_ptr<Work> reduce(at::Tensor& t, int, ReduceOp) override {
    std::vector<at::Tensor> v{t};
    return done(OpType::REDUCE, v);
  }
  std::shared_ptr<Work> gather(std::vector<at::Tensor>& outs, const at::Tensor&, int) override {
    return done(OpType::GATHER, outs);
  }
  std::shared_ptr<Work> scatter(at::Tensor& out, std::vector<at::Tensor>&, int) override {
    std::vector<at::Tensor> v{out};
    return done(OpType::SCATTER, v);
  }
  std::shared_ptr<Work> alltoall_base(at::Tensor& out, const at::Tensor&, const AllToAllSplits&) override {
    std::vector<at::Tensor> v{out};
    return done(OpType::ALLTOALL_BASE, v);
  }
  std::shared_ptr<Work> send(at::Tensor& t, int, int) override {
    std::vector<at::Tensor> v{t};
    return done(OpType::SEND, v);
  }
  std::shared_ptr<Work> recv(at::Tensor& t, int, int) override {
    std::vector<at::Tensor> v{t};
    return done(OpType::RECV, v);
  }
  std::shared_ptr<Work> barrier() override {
    std::vector<at::Tensor> v;
    return done(OpType::BARRIER, v);
  }
  std::shared_ptr<ProcessGroup> split(const std::vector<int>& ranks, const std::string&) override {
    for (size_t i = 0; i < ranks.size(); ++i)
      if (ranks[i] == rank_) return std::make_shared<FakePG>(static_cast<int>(i), static_cast<int>(ranks.size()));
    return nullptr;
  }

 private:
  std::shared_ptr<Work> done(OpType op, std::vector<at::Tensor>& t) {
    auto w = std::make_shared<DoneWork>(op, next_seq());
    w->outputs_ = t;
    return w;
  }
};

}  // namespace ringdp
