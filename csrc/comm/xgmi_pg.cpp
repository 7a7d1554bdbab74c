// xGMI process group (see xgmi_pg.h).  Collective semantics follow c10d/RCCL: in-place all-reduce and
// broadcast, out-of-place all-gather / reduce-scatter / all-to-all, paired send/recv.  Tensors whose
// data pointer or per-rank block is not 16-B aligned go through aligned scratch copies on the comm
// stream (the kernels move 16-B vectors); DDP buckets are aligned and never take that path.
#include "xgmi_pg.h"

#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>

#include <algorithm>

#include "rccl_pg.h"  // to_xg_dtype

namespace ringdp {

namespace {

bool aligned16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }
int64_t round16(int64_t x) { return (x + 15) / 16 * 16; }
void d2d(void* dst, const void* src, int64_t n, hipStream_t s) {
  if (n > 0 && dst != src) RINGDP_HIP_CHECK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, s));
}

int xg_red(ReduceOp op, at::ScalarType t) {
  const bool is_bool = t == at::kBool;
  switch (op) {
    case ReduceOp::SUM:
    case ReduceOp::AVG: return is_bool ? kern::XG_MAX : kern::XG_SUM;  // bool: logical or
    case ReduceOp::PRODUCT: return is_bool ? kern::XG_MIN : kern::XG_PROD;
    case ReduceOp::MIN: return kern::XG_MIN;
    case ReduceOp::MAX: return kern::XG_MAX;
    default: throw RingdpError("[ringdp] xgmi: bitwise reduce ops are not supported");
  }
}

int xg_dtype(const at::Tensor& t) {
  const int d = to_xg_dtype(t.scalar_type());
  RINGDP_CHECK(d >= 0, "xgmi backend: unsupported dtype ", t.scalar_type());
  return d;
}

}  // namespace

XgmiPG::XgmiPG(std::shared_ptr<Store> store, int rank, int size, int device, std::chrono::milliseconds timeout)
    : GpuPG(rank, size, device, timeout),
      store_(store),
      send_stream_(c10::hip::getStreamFromPoolMasqueradingAsCUDA(false, device)) {
  DeviceScope ds(device_);
  RINGDP_HIP_CHECK(hipEventCreateWithFlags(&send_fence_, hipEventDisableTiming));
  RINGDP_HIP_CHECK(hipEventCreateWithFlags(&send_done_, hipEventDisableTiming));
  std::string why;
  eng_ = XgmiEngine::create(std::make_shared<PrefixStore>("xgmi", store), rank, size, device,
                            XgmiConfig::from_env(), timeout.count(), &why);
  RINGDP_CHECK(eng_ != nullptr, "xgmi backend unavailable: ", why,
               " (it serves ranks on one node; use backend 'nccl' across nodes)");
  // one-rank groups launch no kernels; larger groups keep every op on the comm stream (issue order)
  init_common(size == 1);
}

XgmiPG::~XgmiPG() { shutdown(); }

void XgmiPG::shutdown() {
  stop_common();
  DeviceScope ds(device_);
  if (!aborted_.load()) (void)hipStreamSynchronize(send_stream_.stream());
  if (eng_) {
    // every rank's streams are drained: meet through the store before freeing memory peers map
    if (aborted_.load() || eng_->failed()) eng_->mark_unsafe();
    else (void)eng_->quiesce(std::min<int64_t>(timeout_.count(), 60000));
  }
  eng_.reset();
  if (send_fence_) hipEventDestroy(send_fence_);
  if (send_done_) hipEventDestroy(send_done_);
  send_fence_ = send_done_ = nullptr;
}

hipStream_t XgmiPG::send_on(hipStream_t cs) {
  RINGDP_HIP_CHECK(hipEventRecord(send_fence_, cs));
  RINGDP_HIP_CHECK(hipStreamWaitEvent(send_stream_.stream(), send_fence_, 0));
  return send_stream_.stream();
}

void XgmiPG::join_sends(hipStream_t cs) {
  RINGDP_HIP_CHECK(hipEventRecord(send_done_, send_stream_.stream()));
  RINGDP_HIP_CHECK(hipStreamWaitEvent(cs, send_done_, 0));
}

std::string XgmiPG::backend_failure() {
  if (eng_ && eng_->failed()) return "a peer did not arrive within the timeout (its process died or desynchronised)";
  return "";
}

at::Tensor XgmiPG::scratch(int64_t nbytes) {
  auto opts = at::TensorOptions().dtype(at::kByte).device(at::kCUDA, device_);
  if (on_caller_stream()) return at::empty({std::max<int64_t>(nbytes, 16)}, opts);
  c10::hip::HIPStreamGuardMasqueradingAsCUDA g(comm_stream_);
  return at::empty({std::max<int64_t>(nbytes, 16)}, opts);
}

void XgmiPG::allreduce_one(at::Tensor& t, ReduceOp op, hipStream_t s) {
  const int64_t nb = t.numel() * static_cast<int64_t>(t.element_size());
  if (size_ == 1 || nb == 0) return;  // every reduction over one rank is the identity (AVG included)
  const int dt = xg_dtype(t), red = xg_red(op, t.scalar_type());
  const bool avg = op == ReduceOp::AVG;
  if (aligned16(t.data_ptr())) {
    eng_->allreduce(t.data_ptr(), t.data_ptr(), nb, dt, red, avg, s);
    return;
  }
  at::Tensor tmp = scratch(nb);
  d2d(tmp.data_ptr(), t.data_ptr(), nb, s);
  eng_->allreduce(tmp.data_ptr(), tmp.data_ptr(), nb, dt, red, avg, s);
  d2d(t.data_ptr(), tmp.data_ptr(), nb, s);
}

std::shared_ptr<Work> XgmiPG::allreduce(std::vector<at::Tensor>& tensors, ReduceOp op) {
  for (auto& t : tensors) {
    check_tensor(t, "all_reduce");
    (void)xg_red(op, t.scalar_type());
    (void)xg_dtype(t);
  }
  return launch(OpType::ALLREDUCE, tensors, [&](hipStream_t s) {
    for (auto& t : tensors) allreduce_one(t, op, s);
  });
}

std::shared_ptr<Work> XgmiPG::allreduce_coalesced(std::vector<at::Tensor>& tensors, ReduceOp op) {
  return allreduce(tensors, op);
}

std::shared_ptr<Work> XgmiPG::broadcast(std::vector<at::Tensor>& tensors, int root) {
  for (auto& t : tensors) check_tensor(t, "broadcast");
  RINGDP_CHECK(root >= 0 && root < size_, "broadcast: invalid root ", root);
  return launch(OpType::BROADCAST, tensors, [&](hipStream_t s) {
    if (size_ == 1) return;
    for (auto& t : tensors) {
      const int64_t nb = t.numel() * static_cast<int64_t>(t.element_size());
      if (nb == 0) continue;
      if (aligned16(t.data_ptr())) {
        eng_->broadcast(t.data_ptr(), t.data_ptr(), nb, root, s);
      } else {
        at::Tensor tmp = scratch(nb);
        if (rank_ == root) d2d(tmp.data_ptr(), t.data_ptr(), nb, s);
        eng_->broadcast(tmp.data_ptr(), tmp.data_ptr(), nb, root, s);
        if (rank_ != root) d2d(t.data_ptr(), tmp.data_ptr(), nb, s);
      }
    }
  });
}

std::shared_ptr<Work> XgmiPG::allgather_into_tensor(at::Tensor& output, const at::Tensor& input) {
  check_tensor(input, "all_gather_into_tensor");
  check_tensor(output, "all_gather_into_tensor");
  RINGDP_CHECK(output.numel() == input.numel() * size_ && output.scalar_type() == input.scalar_type(),
               "all_gather_into_tensor: output must hold world_size * input numel of the same dtype");
  return launch(OpType::ALLGATHER_BASE, {output, input}, [&](hipStream_t s) {
    const int64_t M = input.numel() * static_cast<int64_t>(input.element_size());
    if (M == 0) return;
    if (size_ == 1) {
      d2d(output.data_ptr(), input.data_ptr(), M, s);
      return;
    }
    if (M % 16 == 0 && aligned16(input.data_ptr()) && aligned16(output.data_ptr())) {
      eng_->allgather(input.data_ptr(), output.data_ptr(), M, s);
      return;
    }
    const int64_t Mp = round16(M);
    at::Tensor tin = scratch(Mp), tout = scratch(Mp * size_);
    d2d(tin.data_ptr(), input.data_ptr(), M, s);
    eng_->allgather(tin.data_ptr(), tout.data_ptr(), Mp, s);
    RINGDP_HIP_CHECK(hipMemcpy2DAsync(output.data_ptr(), M, tout.data_ptr(), Mp, M, size_,
                                      hipMemcpyDeviceToDevice, s));
  });
}

std::shared_ptr<Work> XgmiPG::allgather(std::vector<at::Tensor>& outputs, const at::Tensor& input) {
  check_tensor(input, "all_gather");
  RINGDP_CHECK(static_cast<int>(outputs.size()) == size_, "all_gather: expected ", size_, " outputs");
  for (auto& o : outputs)
    RINGDP_CHECK(o.is_cuda() && o.numel() == input.numel() && o.scalar_type() == input.scalar_type() &&
                     o.is_contiguous(),
                 "all_gather: bad output tensor");
  std::vector<at::Tensor> all = outputs;
  all.push_back(input);
  return launch(OpType::ALLGATHER, all, [&](hipStream_t s) {
    const int64_t M = input.numel() * static_cast<int64_t>(input.element_size());
    if (M == 0) return;
    if (size_ == 1) {
      d2d(outputs[0].data_ptr(), input.data_ptr(), M, s);
      return;
    }
    const int64_t Mp = round16(M);
    at::Tensor tout = scratch(Mp * size_);
    if (M % 16 == 0 && aligned16(input.data_ptr())) {
      eng_->allgather(input.data_ptr(), tout.data_ptr(), Mp, s);
    } else {
      at::Tensor tin = scratch(Mp);
      d2d(tin.data_ptr(), input.data_ptr(), M, s);
      eng_->allgather(tin.data_ptr(), tout.data_ptr(), Mp, s);
    }
    for (int r = 0; r < size_; ++r)
      d2d(outputs[r].data_ptr(), static_cast<char*>(tout.data_ptr()) + r * Mp, M, s);
  });
}

std::shared_ptr<Work> XgmiPG::reduce_scatter_tensor(at::Tensor& output, const at::Tensor& input, ReduceOp op) {
  check_tensor(input, "reduce_scatter_tensor");
  check_tensor(output, "reduce_scatter_tensor");
  RINGDP_CHECK(input.numel() == output.numel() * size_ && output.scalar_type() == input.scalar_type(),
               "reduce_scatter_tensor: input must hold world_size * output numel of the same dtype");
  const int dt = xg_dtype(input), red = xg_red(op, input.scalar_type());
  return launch(OpType::REDUCE_SCATTER_BASE, {output, input}, [&](hipStream_t s) {
    const int64_t M = output.numel() * static_cast<int64_t>(output.element_size());
    if (M == 0) return;
    if (size_ == 1) {
      d2d(output.data_ptr(), input.data_ptr(), M, s);
      return;
    }
    const bool avg = op == ReduceOp::AVG;
    if (M % 16 == 0 && aligned16(input.data_ptr()) && aligned16(output.data_ptr())) {
      eng_->reduce_scatter(input.data_ptr(), output.data_ptr(), M, dt, red, avg, s);
      return;
    }
    const int64_t Mp = round16(M);
    at::Tensor tin = scratch(Mp * size_), tout = scratch(Mp);
    RINGDP_HIP_CHECK(hipMemcpy2DAsync(tin.data_ptr(), Mp, input.data_ptr(), M, M, size_,
                                      hipMemcpyDeviceToDevice, s));
    eng_->reduce_scatter(tin.data_ptr(), tout.data_ptr(), Mp, dt, red, avg, s);
    d2d(output.data_ptr(), tout.data_ptr(), M, s);
  });
}

std::shared_ptr<Work> XgmiPG::reduce(at::Tensor& tensor, int root, ReduceOp op) {
  check_tensor(tensor, "reduce");
  RINGDP_CHECK(root >= 0 && root < size_, "reduce: invalid root ", root);
  (void)xg_red(op, tensor.scalar_type());
  return launch(OpType::REDUCE, {tensor}, [&](hipStream_t s) {
    const int64_t nb = tensor.numel() * static_cast<int64_t>(tensor.element_size());
    if (size_ == 1 || nb == 0) return;
    // all-reduce a copy; only the root's tensor receives the result (c10d: non-roots keep theirs)
    at::Tensor tmp = scratch(nb);
    d2d(tmp.data_ptr(), tensor.data_ptr(), nb, s);
    eng_->allreduce(tmp.data_ptr(), tmp.data_ptr(), nb, xg_dtype(tensor), xg_red(op, tensor.scalar_type()),
                    op == ReduceOp::AVG, s);
    if (rank_ == root) d2d(tensor.data_ptr(), tmp.data_ptr(), nb, s);
  });
}

std::shared_ptr<Work> XgmiPG::gather(std::vector<at::Tensor>& outputs, const at::Tensor& input, int root) {
  check_tensor(input, "gather");
  RINGDP_CHECK(root >= 0 && root < size_, "gather: invalid root ", root);
  if (rank_ == root) RINGDP_CHECK(static_cast<int>(outputs.size()) == size_, "gather: root needs world_size outputs");
  std::vector<at::Tensor> all = outputs;
  all.push_back(input);
  return launch(OpType::GATHER, all, [&](hipStream_t s) {
    const int64_t M = input.numel() * static_cast<int64_t>(input.element_size());
    if (M == 0) return;
    if (size_ == 1) {
      d2d(outputs[0].data_ptr(), input.data_ptr(), M, s);
      return;
    }
    const int64_t Mp = round16(M);
    at::Tensor tin = scratch(Mp), tout = scratch(Mp * size_);
    d2d(tin.data_ptr(), input.data_ptr(), M, s);
    eng_->allgather(tin.data_ptr(), tout.data_ptr(), Mp, s);
    if (rank_ == root)
      for (int r = 0; r < size_; ++r)
        d2d(outputs[r].data_ptr(), static_cast<char*>(tout.data_ptr()) + r * Mp, M, s);
  });
}

std::shared_ptr<Work> XgmiPG::scatter(at::Tensor& output, std::vector<at::Tensor>& inputs, int root) {
  check_tensor(output, "scatter");
  RINGDP_CHECK(root >= 0 && root < size_, "scatter: invalid root ", root);
  if (rank_ == root) RINGDP_CHECK(static_cast<int>(inputs.size()) == size_, "scatter: root needs world_size inputs");
  std::vector<at::Tensor> all = inputs;
  all.push_back(output);
  return launch(OpType::SCATTER, all, [&](hipStream_t s) {
    const int64_t M = output.numel() * static_cast<int64_t>(output.element_size());
    if (rank_ == root) {
      std::vector<at::Tensor> keep;
      for (int r = 0; r < size_; ++r) {
        if (r == root) continue;
        at::Tensor tin = scratch(round16(M));
        d2d(tin.data_ptr(), inputs[r].data_ptr(), M, s);
        eng_->send(tin.data_ptr(), M, r, send_on(s));
        keep.push_back(tin);
      }
      d2d(output.data_ptr(), inputs[root].data_ptr(), M, s);
      join_sends(s);  // the scratch copies live on s: keep them until the sends have read them
    } else {
      at::Tensor tout = scratch(round16(M));
      eng_->recv(tout.data_ptr(), M, root, s);
      d2d(output.data_ptr(), tout.data_ptr(), M, s);
    }
  });
}

std::shared_ptr<Work> XgmiPG::alltoall_base(at::Tensor& output, const at::Tensor& input,
                                            const AllToAllSplits& splits) {
  check_tensor(input, "all_to_all_single");
  check_tensor(output, "all_to_all_single");
  return launch(OpType::ALLTOALL_BASE, {output, input}, [&](hipStream_t s) {
    const int n = size_;
    const int64_t row = input.dim() > 0 ? input.numel() / std::max<int64_t>(input.size(0), 1) : 1;
    const int64_t es = input.element_size();
    std::vector<int64_t> soff(n), sbytes(n), roff(n), rbytes(n);
    int64_t io = 0, oo = 0;
    for (int i = 0; i < n; ++i) {
      const int64_t isz = splits.input_split_sizes.empty() ? input.size(0) / n : splits.input_split_sizes[i];
      const int64_t osz = splits.output_split_sizes.empty() ? output.size(0) / n : splits.output_split_sizes[i];
      soff[i] = io * row * es;
      sbytes[i] = isz * row * es;
      roff[i] = oo * row * es;
      rbytes[i] = osz * row * es;
      io += isz;
      oo += osz;
    }
    char* in = static_cast<char*>(input.data_ptr());
    char* out = static_cast<char*>(output.data_ptr());
    d2d(out + roff[rank_], in + soff[rank_], sbytes[rank_], s);
    // step k: send to rank+k (send stream), receive from rank-k (comm stream): a send waits only for
    // its receiver to have read the slot it refills, which no send of the receiver can hold up
    std::vector<at::Tensor> keep;
    for (int k = 1; k < n; ++k) {
      const int dst = (rank_ + k) % n, src = (rank_ - k + n) % n;
      at::Tensor tin = scratch(round16(sbytes[dst])), tout = scratch(round16(rbytes[src]));
      d2d(tin.data_ptr(), in + soff[dst], sbytes[dst], s);
      eng_->send(tin.data_ptr(), sbytes[dst], dst, send_on(s));
      eng_->recv(tout.data_ptr(), rbytes[src], src, s);
      d2d(out + roff[src], tout.data_ptr(), rbytes[src], s);
      keep.push_back(tin);
    }
    join_sends(s);  // scratch inputs of the sends stay allocated (stream-ordered on s) until here
  });
}

std::shared_ptr<Work> XgmiPG::send(at::Tensor& tensor, int dst, int /*tag*/) {
  check_tensor(tensor, "send");
  RINGDP_CHECK(dst >= 0 && dst < size_ && dst != rank_, "send: invalid peer ", dst);
  return launch(OpType::SEND, {tensor}, [&](hipStream_t s) -> hipStream_t {
    const int64_t nb = tensor.numel() * static_cast<int64_t>(tensor.element_size());
    if (on_caller_stream()) {  // one stream by request: the caller orders sends and receives
      eng_->send(tensor.data_ptr(), nb, dst, s);
      return s;
    }
    hipStream_t ss = send_on(s);
    if (aligned16(tensor.data_ptr())) {
      eng_->send(tensor.data_ptr(), nb, dst, ss);
    } else {
      // stage through an aligned copy made ON the send stream, so the comm stream never waits for a
      // send (a send blocks until its receiver drains the P2P slots; a comm stream held behind it would
      // keep this rank's own recv from running: two ranks exchanging > 2 slots would deadlock)
      at::Tensor tin = scratch(round16(nb));
      d2d(tin.data_ptr(), tensor.data_ptr(), nb, ss);
      eng_->send(tin.data_ptr(), nb, dst, ss);
      c10::hip::HIPCachingAllocatorMasqueradingAsCUDA::recordStreamMasqueradingAsCUDA(tin.storage().data_ptr(),
                                                                                      send_stream_);
    }
    // the op completes on the send stream; the tensor is kept alive by the Work, and the caching
    // allocator learns about the second stream here
    c10::hip::HIPCachingAllocatorMasqueradingAsCUDA::recordStreamMasqueradingAsCUDA(tensor.storage().data_ptr(),
                                                                                    send_stream_);
    return send_stream_.stream();
  });
}

std::shared_ptr<Work> XgmiPG::recv(at::Tensor& tensor, int src, int /*tag*/) {
  check_tensor(tensor, "recv");
  RINGDP_CHECK(src >= 0 && src < size_ && src != rank_, "recv: invalid peer ", src);
  return launch(OpType::RECV, {tensor}, [&](hipStream_t s) {
    const int64_t nb = tensor.numel() * static_cast<int64_t>(tensor.element_size());
    if (aligned16(tensor.data_ptr())) {
      eng_->recv(tensor.data_ptr(), nb, src, s);
    } else {
      at::Tensor tout = scratch(round16(nb));
      eng_->recv(tout.data_ptr(), nb, src, s);
      d2d(tensor.data_ptr(), tout.data_ptr(), nb, s);
    }
  });
}

std::shared_ptr<Work> XgmiPG::barrier() {
  return launch(OpType::BARRIER, {}, [&](hipStream_t s) {
    if (size_ > 1) eng_->barrier(s);
  });
}

std::shared_ptr<ProcessGroup> XgmiPG::split(const std::vector<int>& ranks, const std::string& tag) {
  int new_rank = -1;
  for (size_t i = 0; i < ranks.size(); ++i)
    if (ranks[i] == rank_) new_rank = static_cast<int>(i);
  if (new_rank < 0) return nullptr;
  return std::make_shared<XgmiPG>(std::make_shared<PrefixStore>("split/" + tag, store_), new_rank,
                                  static_cast<int>(ranks.size()), device_, timeout_);
}

}  // namespace ringdp
