// RCCL process group implementation (see rccl_pg.h).
#include "rccl_pg.h"

#include "../kernels/kernels.h"

#include <ATen/hip/impl/HIPCachingAllocatorMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace ringdp {

#define RINGDP_NCCL_CHECK(expr)                                                              \
  do {                                                                                       \
    ncclResult_t _r = (expr);                                                                \
    if (_r != ncclSuccess && _r != ncclInProgress) {                                         \
      throw ::ringdp::RingdpError(::ringdp::strcat_all("[ringdp] RCCL error '",              \
                                                       ncclGetErrorString(_r), "' at ",      \
                                                       __FILE__, ":", __LINE__));            \
    }                                                                                        \
  } while (0)

ncclDataType_t to_nccl_dtype(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return ncclFloat32;
    case at::kDouble: return ncclFloat64;
    case at::kHalf: return ncclFloat16;
    case at::kBFloat16: return ncclBfloat16;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kChar: return ncclInt8;
    case at::kByte: return ncclUint8;
    case at::kBool: return ncclUint8;
    default:
      throw RingdpError(strcat_all("[ringdp] RCCL: unsupported dtype ", c10::toString(t)));
  }
}

ncclRedOp_t to_nccl_op(ReduceOp op) {
  switch (op) {
    case ReduceOp::SUM: return ncclSum;
    case ReduceOp::PRODUCT: return ncclProd;
    case ReduceOp::MIN: return ncclMin;
    case ReduceOp::MAX: return ncclMax;
    case ReduceOp::AVG: return ncclAvg;
    default:
      throw RingdpError("[ringdp] RCCL: bitwise reduce ops are not supported");
  }
}

namespace {

bool env_flag(const char* name, bool dflt) {
  const char* v = std::getenv(name);
  if (!v || !*v) return dflt;
  return !(std::strcmp(v, "0") == 0 || std::strcmp(v, "false") == 0);
}

class DeviceScope {
 public:
  explicit DeviceScope(int dev) {
    hipGetDevice(&prev_);
    if (prev_ != dev) hipSetDevice(dev);
  }
  ~DeviceScope() { hipSetDevice(prev_); }

 private:
  int prev_ = 0;
};

}  // namespace

// ------------------------------------------------------------------ RcclWork
RcclWork::RcclWork(OpType op, uint64_t seq, RcclPG* pg, bool captured, bool timing)
    : Work(op, seq), captured_(captured), pg_(pg) {
  RINGDP_HIP_CHECK(hipEventCreateWithFlags(&done_, timing ? hipEventDefault
                                                           : hipEventDisableTiming));
  if (timing) RINGDP_HIP_CHECK(hipEventCreateWithFlags(&start_, hipEventDefault));
}

RcclWork::~RcclWork() {
  if (done_) hipEventDestroy(done_);
  if (start_) hipEventDestroy(start_);
}

bool RcclWork::is_completed() {
  if (captured_) return false;
  return hipEventQuery(done_) == hipSuccess;
}

void RcclWork::wait(bool blocking) {
  if (pg_->aborted())
    throw RingdpError("[ringdp] RCCL communicator aborted: " + pg_->error_message());
  HipStream cur = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(pg_->device());
  RINGDP_HIP_CHECK(hipStreamWaitEvent(cur.stream(), done_, 0));
  if (blocking && !captured_) {
    auto deadline = now_us() + pg_->timeout().count() * 1000;
    while (hipEventQuery(done_) == hipErrorNotReady) {
      if (pg_->aborted())
        throw RingdpError("[ringdp] RCCL communicator aborted: " + pg_->error_message());
      if (now_us() > deadline)
        throw TimeoutError(strcat_all("[ringdp] RCCL ", op_name(op_), " seq ", seq_,
                                      " timed out after ", pg_->timeout().count(), " ms"));
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
}

double RcclWork::duration_us() {
  if (!start_ || captured_) return -1.0;
  if (hipEventQuery(done_) != hipSuccess) return -1.0;
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, start_, done_) != hipSuccess) return -1.0;
  return static_cast<double>(ms) * 1000.0;
}

// ------------------------------------------------------------------ ReplayBeacon
ReplayBeacon::ReplayBeacon(int device) : device_(device) {
  DeviceScope ds(device_);
  RINGDP_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&host_), sizeof(*host_),
                                 hipHostMallocCoherent | hipHostMallocMapped));
  *host_ = 0;
  RINGDP_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&dev_), sizeof(*dev_)));
  RINGDP_HIP_CHECK(hipMemset(dev_, 0, sizeof(*dev_)));
  RINGDP_HIP_CHECK(hipDeviceSynchronize());
}

ReplayBeacon::~ReplayBeacon() {
  DeviceScope ds(device_);
  (void)hipDeviceSynchronize();  // no replay may still write the counters
  if (dev_) (void)hipFree(dev_);
  if (host_) (void)hipHostFree(host_);
}

void ReplayBeacon::mark(hipStream_t stream) {
  unsigned long long* hdev = nullptr;
  RINGDP_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hdev), host_, 0));
  kern::replay_beacon_mark(dev_, hdev, stream);
  RINGDP_HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------ RcclPG
RcclPG::RcclPG(std::shared_ptr<Store> store, int rank, int size, int device,
               std::chrono::milliseconds timeout)
    : ProcessGroup(rank, size),
      device_(device),
      timeout_(timeout),
      comm_stream_(c10::hip::getStreamFromPoolMasqueradingAsCUDA(env_flag("RINGDP_COMM_HIGH_PRIORITY", false), device)) {
  DeviceScope ds(device_);
  ncclUniqueId uid;
  if (rank == 0) {
    RINGDP_NCCL_CHECK(ncclGetUniqueId(&uid));
    store->set("rccl/uid", std::string(reinterpret_cast<const char*>(&uid), sizeof(uid)));
  } else {
    std::string s = store->get("rccl/uid");
    RINGDP_CHECK(s.size() == sizeof(uid), "RCCL unique id has wrong size");
    std::memcpy(&uid, s.data(), sizeof(uid));
  }
  RINGDP_NCCL_CHECK(ncclCommInitRank(&comm_, size, uid, rank));
  if (const char* e = std::getenv("RINGDP_P2P_ALLREDUCE_MAX_BYTES")) {
    const int64_t max_bytes = std::atoll(e);
    if (max_bytes > 0) {
      // the kernel's own spin bound: the group timeout, capped so a dead peer ends it in minutes
      const int64_t tmo = std::min<int64_t>(timeout_.count(), 300000);
      p2p_ = P2PAllReduce::create(store, rank, size, device, max_bytes, tmo);
      if (!p2p_ && rank == 0)
        std::fprintf(stderr, "[ringdp] P2P all-reduce unavailable for this group (not one host, >8 ranks, "
                             "or IPC setup failed); using RCCL for every size\n");
    }
  }
  init_common();
}

RcclPG::RcclPG(ncclComm_t comm, int rank, int size, int device, std::chrono::milliseconds timeout)
    : ProcessGroup(rank, size),
      comm_(comm),
      device_(device),
      timeout_(timeout),
      comm_stream_(c10::hip::getStreamFromPoolMasqueradingAsCUDA(env_flag("RINGDP_COMM_HIGH_PRIORITY", false), device)) {
  init_common();
}

void RcclPG::init_common() {
  DeviceScope ds(device_);
  // Collectives of a one-rank group have nothing to overlap with, and a side-stream fork/join inside
  // a hipGraph is not free on ROCm 7 (ResNet-18 step: 3.52 ms forked vs 3.10 ms on the compute
  // stream, ConvNet unchanged): one-rank groups issue on the caller's stream.
  // RINGDP_COMM_SAME_STREAM=1 / 0 forces either choice for any group size.
  if (const char* v = std::getenv("RINGDP_COMM_SAME_STREAM"))
    same_stream_ = std::strcmp(v, "1") == 0;
  else
    same_stream_ = size_ == 1;
  RINGDP_HIP_CHECK(hipEventCreateWithFlags(&ready_, hipEventDisableTiming));
  timing_ = env_flag("RINGDP_COMM_TIMING", false);
  async_error_handling_ = env_flag("RINGDP_ASYNC_ERROR_HANDLING", true);
  watchdog_ = std::thread([this] { watchdog_loop(); });
}

RcclPG::~RcclPG() { shutdown(); }

void RcclPG::shutdown() {
  if (stop_.exchange(true)) return;
  wd_cv_.notify_all();
  if (watchdog_.joinable()) watchdog_.join();
  if (comm_) {
    DeviceScope ds(device_);
    if (!aborted_.load()) {
      (void)hipStreamSynchronize(comm_stream_.stream());
      ncclCommDestroy(comm_);
    }
    comm_ = nullptr;
  }
  inflight_.clear();
  if (p2p_) {
    DeviceScope ds(device_);
    (void)hipStreamSynchronize(comm_stream_.stream());
    p2p_.reset();
  }
  if (ready_) {
    hipEventDestroy(ready_);
    ready_ = nullptr;
  }
}

void RcclPG::drain() {
  std::lock_guard<std::mutex> lk(wd_mu_);
  DeviceScope ds(device_);
  for (auto& w : inflight_) (void)hipEventSynchronize(w->done_);
  inflight_.clear();
}

void RcclPG::watch_beacon(const std::shared_ptr<ReplayBeacon>& beacon) {
  std::lock_guard<std::mutex> bl(beacon_mu_);
  beacon->last_done_ = beacon->completed();
  beacon->progress_us_ = now_us();
  beacons_.push_back(beacon);
}

void RcclPG::abort() {
  if (comm_ && !aborted_.exchange(true)) {
    ncclCommAbort(comm_);
  }
  aborted_.store(true);
}

void RcclPG::fail(const std::string& msg) {
  {
    std::lock_guard<std::mutex> lk(wd_mu_);
    error_ = msg;
  }
  std::fprintf(stderr, "%s\n", msg.c_str());
  std::fflush(stderr);
  if (comm_ && !aborted_.exchange(true)) ncclCommAbort(comm_);
  if (async_error_handling_) {
    std::fprintf(stderr,
                 "[ringdp] rank %d: tearing the process down after a communicator failure "
                 "(set RINGDP_ASYNC_ERROR_HANDLING=0 to raise instead)\n",
                 rank_);
    std::fflush(stderr);
    std::_Exit(1);
  }
}

void RcclPG::watchdog_loop() {
  hipSetDevice(device_);
  while (!stop_.load()) {
    {
      std::unique_lock<std::mutex> lk(wd_mu_);
      wd_cv_.wait_for(lk, std::chrono::milliseconds(50), [&] { return stop_.load(); });
    }
    if (stop_.load() || aborted_.load()) break;
    std::string failure;
    {
      std::lock_guard<std::mutex> lk(wd_mu_);
      int64_t now = now_us();
      while (!inflight_.empty()) {
        auto& w = inflight_.front();
        hipError_t q = hipEventQuery(w->done_);
        if (q == hipSuccess) {
          inflight_.pop_front();
          continue;
        }
        if (now > w->deadline_us_) {
          failure = strcat_all("[ringdp] watchdog: rank ", rank_, " RCCL ", op_name(w->op()),
                               " (seq ", w->seq(), ") did not complete within ",
                               timeout_.count(), " ms; aborting communicator");
        }
        // Entries are queued in issue order with deadlines in the same order: an incomplete
        // head that is within its deadline means everything behind it is too.
        break;
      }
    }
    if (failure.empty()) {
      // captured steps: plain loads of the replay beacons (no HIP call on this thread)
      std::lock_guard<std::mutex> bl(beacon_mu_);
      const int64_t now = now_us();
      for (auto it = beacons_.begin(); it != beacons_.end();) {
        auto b = it->lock();
        if (!b) {
          it = beacons_.erase(it);
          continue;
        }
        const uint64_t done = b->completed(), issued = b->issued_count();
        if (done >= issued || done != b->last_done_) {
          b->last_done_ = done;
          b->progress_us_ = now;  // idle, or a replay finished since the last look
        } else if (now - b->progress_us_ > timeout_.count() * 1000) {
          failure = strcat_all("[ringdp] watchdog: rank ", rank_, " ", op_name(OpType::GRAPH_REPLAY), " ",
                               done + 1, " of ", issued, " did not complete within ", timeout_.count(),
                               " ms; aborting communicator");
          break;
        }
        ++it;
      }
    }
    if (failure.empty() && p2p_ && p2p_->failed()) {
      failure = strcat_all("[ringdp] watchdog: rank ", rank_, " P2P all-reduce: a peer did not arrive "
                           "within the timeout; aborting communicator");
    }
    if (failure.empty() && comm_) {
      ncclResult_t async_err = ncclSuccess;
      if (ncclCommGetAsyncError(comm_, &async_err) == ncclSuccess && async_err != ncclSuccess &&
          async_err != ncclInProgress) {
        failure = strcat_all("[ringdp] watchdog: rank ", rank_, " RCCL async error: ",
                             ncclGetErrorString(async_err));
      }
    }
    if (!failure.empty()) fail(failure);
  }
}

void RcclPG::check_tensor(const at::Tensor& t, const char* what) const {
  RINGDP_CHECK(t.is_cuda(), what, ": rccl backend expects GPU tensors, got ", t.device());
  RINGDP_CHECK(t.get_device() == device_, what, ": tensor on device ", t.get_device(),
               " but process group is bound to device ", device_);
  RINGDP_CHECK(t.is_contiguous(), what, ": tensor must be contiguous");
}

template <typename Fn>
std::shared_ptr<Work> RcclPG::launch(OpType op, const std::vector<at::Tensor>& tensors, Fn&& body) {
  RINGDP_CHECK(!aborted_.load(), "RCCL communicator was aborted: ", error_message());
  RINGDP_CHECK(comm_ != nullptr, "process group has been shut down");
  std::lock_guard<std::mutex> lk(launch_mu_);
  DeviceScope ds(device_);
  HipStream cur = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(device_);
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  RINGDP_HIP_CHECK(hipStreamIsCapturing(cur.stream(), &cap));
  const bool captured = cap == hipStreamCaptureStatusActive;
  auto work = std::make_shared<RcclWork>(op, next_seq(), this, captured, timing_ && !captured);
  const bool same_stream = same_stream_;
  hipStream_t cs = same_stream ? cur.stream() : comm_stream_.stream();
  // Fence: the comm stream waits for everything queued so far on the producer stream.
  if (!same_stream) {
    RINGDP_HIP_CHECK(hipEventRecord(ready_, cur.stream()));
    RINGDP_HIP_CHECK(hipStreamWaitEvent(cs, ready_, 0));
  }
  if (work->start_) RINGDP_HIP_CHECK(hipEventRecord(work->start_, cs));
  for (auto& t : tensors) {
    if (!same_stream && t.defined() && t.is_cuda() && t.numel() > 0)
      c10::hip::HIPCachingAllocatorMasqueradingAsCUDA::recordStreamMasqueradingAsCUDA(
          t.storage().data_ptr(), comm_stream_);
  }
  body(cs);
  RINGDP_HIP_CHECK(hipEventRecord(work->done_, cs));
  work->outputs_ = tensors;
  if (!captured) {
    work->deadline_us_ = now_us() + timeout_.count() * 1000;
    std::lock_guard<std::mutex> wl(wd_mu_);
    inflight_.push_back(work);
  }
  return work;
}

std::shared_ptr<Work> RcclPG::allreduce(std::vector<at::Tensor>& tensors, ReduceOp op) {
  for (auto& t : tensors) check_tensor(t, "all_reduce");
  if (p2p_ && p2p_on_ && tensors.size() == 1 && (op == ReduceOp::SUM || op == ReduceOp::AVG) &&
      p2p_->eligible(tensors[0])) {
    // small bucket on one xGMI node: one-shot read of every peer instead of 2(N-1) ring steps
    return launch(OpType::ALLREDUCE, tensors, [&](hipStream_t s) {
      p2p_->run(tensors[0], op == ReduceOp::AVG, s);
    });
  }
  auto red = to_nccl_op(op);
  return launch(OpType::ALLREDUCE, tensors, [&](hipStream_t s) {
    if (tensors.size() > 1) RINGDP_NCCL_CHECK(ncclGroupStart());
    for (auto& t : tensors)
      RINGDP_NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(),
                                      to_nccl_dtype(t.scalar_type()), red, comm_, s));
    if (tensors.size() > 1) RINGDP_NCCL_CHECK(ncclGroupEnd());
  });
}

std::shared_ptr<Work> RcclPG::allreduce_coalesced(std::vector<at::Tensor>& tensors, ReduceOp op) {
  return allreduce(tensors, op);
}

std::shared_ptr<Work> RcclPG::broadcast(std::vector<at::Tensor>& tensors, int root) {
  for (auto& t : tensors) check_tensor(t, "broadcast");
  RINGDP_CHECK(root >= 0 && root < size_, "broadcast: invalid root ", root);
  return launch(OpType::BROADCAST, tensors, [&](hipStream_t s) {
    if (tensors.size() > 1) RINGDP_NCCL_CHECK(ncclGroupStart());
    for (auto& t : tensors)
      RINGDP_NCCL_CHECK(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(),
                                      to_nccl_dtype(t.scalar_type()), root, comm_, s));
    if (tensors.size() > 1) RINGDP_NCCL_CHECK(ncclGroupEnd());
  });
}

std::shared_ptr<Work> RcclPG::allgather(std::vector<at::Tensor>& outputs, const at::Tensor& input) {
  check_tensor(input, "all_gather");
  RINGDP_CHECK(static_cast<int>(outputs.size()) == size_, "all_gather: expected ", size_,
               " outputs");
  for (auto& o : outputs) {
    RINGDP_CHECK(o.is_cuda() && o.numel() == input.numel(), "all_gather: bad output tensor");
  }
  // Gather into a flat staging buffer allocated on the comm stream, then scatter-copy out.
  at::Tensor flat;
  {
    c10::hip::HIPStreamGuardMasqueradingAsCUDA g(comm_stream_);
    flat = at::empty({size_ * input.numel()}, input.options());
  }
  std::vector<at::Tensor> all = outputs;
  all.push_back(input);
  all.push_back(flat);
  return launch(OpType::ALLGATHER, all, [&](hipStream_t s) {
    RINGDP_NCCL_CHECK(ncclAllGather(input.data_ptr(), flat.data_ptr(), input.numel(),
                                    to_nccl_dtype(input.scalar_type()), comm_, s));
    c10::hip::HIPStreamGuardMasqueradingAsCUDA g(comm_stream_);
    for (int i = 0; i < size_; ++i)
      outputs[i].copy_(flat.narrow(0, i * input.numel(), input.numel()).view(outputs[i].sizes()),
                       /*non_blocking=*/true);
  });
}

std::shared_ptr<Work> RcclPG::allgather_into_tensor(at::Tensor& output, const at::Tensor& input) {
  check_tensor(input, "all_gather_into_tensor");
  check_tensor(output, "all_gather_into_tensor");
  RINGDP_CHECK(output.numel() == input.numel() * size_,
               "all_gather_into_tensor: output numel must be world_size * input numel");
  return launch(OpType::ALLGATHER_BASE, {output, input}, [&](hipStream_t s) {
    RINGDP_NCCL_CHECK(ncclAllGather(input.data_ptr(), output.data_ptr(), input.numel(),
                                    to_nccl_dtype(input.scalar_type()), comm_, s));
  });
}

std::shared_ptr<Work> RcclPG::reduce_scatter_tensor(at::Tensor& output, const at::Tensor& input,
                                                    ReduceOp op) {
  check_tensor(input, "reduce_scatter_tensor");
  check_tensor(output, "reduce_scatter_tensor");
  RINGDP_CHECK(input.numel() == output.numel() * size_,
               "reduce_scatter_tensor: input numel must be world_size * output numel");
  auto red = to_nccl_op(op);
  return launch(OpType::REDUCE_SCATTER_BASE, {output, input}, [&](hipStream_t s) {
    RINGDP_NCCL_CHECK(ncclReduceScatter(input.data_ptr(), output.data_ptr(), output.numel(),
                                        to_nccl_dtype(input.scalar_type()), red, comm_, s));
  });
}

std::shared_ptr<Work> RcclPG::reduce(at::Tensor& tensor, int root, ReduceOp op) {
  check_tensor(tensor, "reduce");
  auto red = to_nccl_op(op);
  return launch(OpType::REDUCE, {tensor}, [&](hipStream_t s) {
    RINGDP_NCCL_CHECK(ncclReduce(tensor.data_ptr(), tensor.data_ptr(), tensor.numel(),
                                 to_nccl_dtype(tensor.scalar_type()), red, root, comm_, s));
  });
}

std::shared_ptr<Work> RcclPG::gather(std::vector<at::Tensor>& outputs, const at::Tensor& input,
                                     int root) {
  check_tensor(input, "gather");
  std::vector<at::Tensor> all = outputs;
  all.push_back(input);
  return launch(OpType::GATHER, all, [&](hipStream_t s) {
    auto dt = to_nccl_dtype(input.scalar_type());
    RINGDP_NCCL_CHECK(ncclGroupStart());
    if (rank_ == root) {
      RINGDP_CHECK(static_cast<int>(outputs.size()) == size_, "gather: root needs world_size outputs");
      for (int i = 0; i < size_; ++i) {
        if (i == root) continue;
        RINGDP_NCCL_CHECK(ncclRecv(outputs[i].data_ptr(), outputs[i].numel(), dt, i, comm_, s));
      }
    } else {
      RINGDP_NCCL_CHECK(ncclSend(input.data_ptr(), input.numel(), dt, root, comm_, s));
    }
    RINGDP_NCCL_CHECK(ncclGroupEnd());
    if (rank_ == root) {
      c10::hip::HIPStreamGuardMasqueradingAsCUDA g(comm_stream_);
      outputs[root].copy_(input, true);
    }
  });
}

std::shared_ptr<Work> RcclPG::scatter(at::Tensor& output, std::vector<at::Tensor>& inputs,
                                      int root) {
  check_tensor(output, "scatter");
  std::vector<at::Tensor> all = inputs;
  all.push_back(output);
  return launch(OpType::SCATTER, all, [&](hipStream_t s) {
    auto dt = to_nccl_dtype(output.scalar_type());
    RINGDP_NCCL_CHECK(ncclGroupStart());
    if (rank_ == root) {
      RINGDP_CHECK(static_cast<int>(inputs.size()) == size_, "scatter: root needs world_size inputs");
      for (int i = 0; i < size_; ++i) {
        if (i == root) continue;
        RINGDP_NCCL_CHECK(ncclSend(inputs[i].data_ptr(), inputs[i].numel(), dt, i, comm_, s));
      }
    } else {
      RINGDP_NCCL_CHECK(ncclRecv(output.data_ptr(), output.numel(), dt, root, comm_, s));
    }
    RINGDP_NCCL_CHECK(ncclGroupEnd());
    if (rank_ == root) {
      c10::hip::HIPStreamGuardMasqueradingAsCUDA g(comm_stream_);
      output.copy_(inputs[root], true);
    }
  });
}

std::shared_ptr<Work> RcclPG::alltoall_base(at::Tensor& output, const at::Tensor& input,
                                            const AllToAllSplits& splits) {
  check_tensor(input, "all_to_all_single");
  check_tensor(output, "all_to_all_single");
  return launch(OpType::ALLTOALL_BASE, {output, input}, [&](hipStream_t s) {
    const int n = size_;
    const int64_t row = input.dim() > 0 ? input.numel() / std::max<int64_t>(input.size(0), 1) : 1;
    const size_t es = input.element_size();
    auto dt = to_nccl_dtype(input.scalar_type());
    int64_t ioff = 0, ooff = 0;
    RINGDP_NCCL_CHECK(ncclGroupStart());
    for (int i = 0; i < n; ++i) {
      int64_t isz = splits.input_split_sizes.empty() ? input.size(0) / n : splits.input_split_sizes[i];
      int64_t osz = splits.output_split_sizes.empty() ? output.size(0) / n : splits.output_split_sizes[i];
      char* ip = static_cast<char*>(input.data_ptr()) + ioff * row * es;
      char* op = static_cast<char*>(output.data_ptr()) + ooff * row * es;
      if (isz) RINGDP_NCCL_CHECK(ncclSend(ip, isz * row, dt, i, comm_, s));
      if (osz) RINGDP_NCCL_CHECK(ncclRecv(op, osz * row, dt, i, comm_, s));
      ioff += isz;
      ooff += osz;
    }
    RINGDP_NCCL_CHECK(ncclGroupEnd());
  });
}

std::shared_ptr<Work> RcclPG::send(at::Tensor& tensor, int dst, int /*tag*/) {
  check_tensor(tensor, "send");
  return launch(OpType::SEND, {tensor}, [&](hipStream_t s) {
    RINGDP_NCCL_CHECK(ncclSend(tensor.data_ptr(), tensor.numel(),
                               to_nccl_dtype(tensor.scalar_type()), dst, comm_, s));
  });
}

std::shared_ptr<Work> RcclPG::recv(at::Tensor& tensor, int src, int /*tag*/) {
  check_tensor(tensor, "recv");
  return launch(OpType::RECV, {tensor}, [&](hipStream_t s) {
    RINGDP_NCCL_CHECK(ncclRecv(tensor.data_ptr(), tensor.numel(),
                               to_nccl_dtype(tensor.scalar_type()), src, comm_, s));
  });
}

std::shared_ptr<Work> RcclPG::barrier() {
  at::Tensor t;
  {
    c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, static_cast<c10::DeviceIndex>(device_)));
    t = at::zeros({1}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device_));
  }
  std::vector<at::Tensor> v{t};
  auto w = allreduce(v, ReduceOp::SUM);
  return w;
}

std::shared_ptr<Work> RcclPG::coalesced(std::vector<CollOp>& ops) {
  std::vector<at::Tensor> all;
  for (auto& c : ops) {
    check_tensor(c.out, "coalesced");
    all.push_back(c.out);
    if (c.kind == CollOp::ALLGATHER_INTO || c.kind == CollOp::REDUCE_SCATTER) {
      check_tensor(c.in, "coalesced");
      all.push_back(c.in);
    }
    if (c.kind == CollOp::ALLGATHER_INTO)
      RINGDP_CHECK(c.out.numel() == c.in.numel() * size_, "coalesced all_gather_into_tensor: bad sizes");
    if (c.kind == CollOp::REDUCE_SCATTER)
      RINGDP_CHECK(c.in.numel() == c.out.numel() * size_, "coalesced reduce_scatter_tensor: bad sizes");
    if (c.kind == CollOp::BROADCAST)
      RINGDP_CHECK(c.root >= 0 && c.root < size_, "coalesced broadcast: invalid root ", c.root);
  }
  // One ncclGroupStart/End: RCCL fuses the batch into a single launch on the comm stream.
  return launch(OpType::COALESCED, all, [&](hipStream_t s) {
    RINGDP_NCCL_CHECK(ncclGroupStart());
    for (auto& c : ops) {
      auto dt = to_nccl_dtype(c.out.scalar_type());
      switch (c.kind) {
        case CollOp::ALLREDUCE:
          RINGDP_NCCL_CHECK(ncclAllReduce(c.out.data_ptr(), c.out.data_ptr(), c.out.numel(), dt,
                                          to_nccl_op(c.op), comm_, s));
          break;
        case CollOp::BROADCAST:
          RINGDP_NCCL_CHECK(ncclBroadcast(c.out.data_ptr(), c.out.data_ptr(), c.out.numel(), dt,
                                          c.root, comm_, s));
          break;
        case CollOp::ALLGATHER_INTO:
          RINGDP_NCCL_CHECK(ncclAllGather(c.in.data_ptr(), c.out.data_ptr(), c.in.numel(), dt,
                                          comm_, s));
          break;
        case CollOp::REDUCE_SCATTER:
          RINGDP_NCCL_CHECK(ncclReduceScatter(c.in.data_ptr(), c.out.data_ptr(), c.out.numel(), dt,
                                              to_nccl_op(c.op), comm_, s));
          break;
      }
    }
    RINGDP_NCCL_CHECK(ncclGroupEnd());
  });
}

std::shared_ptr<ProcessGroup> RcclPG::split(const std::vector<int>& ranks, const std::string&) {
  int new_rank = -1;
  for (size_t i = 0; i < ranks.size(); ++i)
    if (ranks[i] == rank_) new_rank = static_cast<int>(i);
  DeviceScope ds(device_);
  (void)hipStreamSynchronize(comm_stream_.stream());
  ncclComm_t nc = nullptr;
  RINGDP_NCCL_CHECK(ncclCommSplit(comm_, new_rank >= 0 ? 0 : NCCL_SPLIT_NOCOLOR,
                                  new_rank >= 0 ? new_rank : rank_, &nc, nullptr));
  if (new_rank < 0) return nullptr;
  return std::make_shared<RcclPG>(nc, new_rank, static_cast<int>(ranks.size()), device_, timeout_);
}

}  // namespace ringdp
