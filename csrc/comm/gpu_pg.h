// GPU process-group machinery shared by the RCCL and xGMI backends: a dedicated comm HIP stream
// fenced against the caller's stream by events, async Work handles with completion events, a watchdog
// thread (per-op deadlines, hipGraph replay beacons, backend error words) that aborts and tears the
// process down on a hang, and the capture-aware launch path.
//
// Parity target: c10d ProcessGroupNCCL's stream/event/Work/watchdog contract
// (c10d/ProcessGroupNCCL.hpp:318, watchdog :683, heartbeat :603; SURVEY.md §2.3 U4, §5 failure row).
#pragma once

#include <hip/hip_runtime_api.h>

#include <ATen/hip/impl/HIPCachingAllocatorMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <deque>
#include <thread>
#include <type_traits>

#include "process_group.h"

namespace ringdp {

using HipStream = c10::hip::HIPStreamMasqueradingAsCUDA;

class GpuPG;

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

class GpuWork : public Work {
 public:
  GpuWork(OpType op, uint64_t seq, GpuPG* pg, bool captured, bool timing);
  ~GpuWork() override;
  void wait(bool blocking = false) override;
  bool is_completed() override;
  double duration_us() override;

  hipEvent_t done_ = nullptr;
  hipEvent_t start_ = nullptr;  // only when timing is enabled
  int64_t deadline_us_ = 0;
  bool captured_ = false;

 private:
  GpuPG* pg_;
};

class GpuPG : public ProcessGroup {
 public:
  GpuPG(int rank, int size, int device, std::chrono::milliseconds timeout);
  ~GpuPG() override;

  int device() const { return device_; }
  hipStream_t comm_stream() const { return comm_stream_.stream(); }
  std::chrono::milliseconds timeout() const { return timeout_; }
  bool same_stream() const { return same_stream_; }
  void set_caller_stream_ops(bool on) override { caller_ops_ = on; }
  // ops go to the caller's stream: same-stream mode, or an inline op (set_caller_stream_ops)
  bool on_caller_stream() const { return same_stream_ || caller_ops_; }
  // Switch between the caller's stream and the side stream for later ops (drains the device first:
  // nothing issued under the old placement is still in flight).  For A/B placement tuning.
  void set_same_stream(bool v);
  // the stream the next op will be issued on (the caller's in same-stream mode, else the comm stream)
  c10::hip::HIPStreamMasqueradingAsCUDA op_stream() const {
    return on_caller_stream() ? c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(device_) : comm_stream_;
  }

  // Host-blocks until every eagerly issued op has completed and clears the watchdog list, so
  // no event query can race a subsequent hipGraph capture.
  void drain();
  // Puts the replays of a captured step (whose collectives the per-op watchdog entries cannot see)
  // under this group's watchdog: while replays are outstanding, one must complete within the group
  // timeout, else the group is aborted and the process exits non-zero like any other hung collective.
  void watch_beacon(const std::shared_ptr<ReplayBeacon>& beacon);
  // Makes `stream` wait for the last op this group issued eagerly since the previous call (a graph
  // replay launched on `stream` then cannot overlap an eager collective still running on the comm
  // stream).  No HIP call when nothing was issued since.
  void join_into(hipStream_t stream);
  bool aborted() const { return aborted_.load(); }
  std::string error_message() {
    std::lock_guard<std::mutex> lk(wd_mu_);
    return error_;
  }
  void set_timing(bool on) { timing_ = on; }
  bool timing() const { return timing_; }
  void set_async_error_handling(bool on) { async_error_handling_ = on; }
  void shutdown() override;
  void abort() override;

  // Backend failure seen by a host-side check (e.g. a kernel's timeout word); "" when healthy.
  virtual std::string backend_failure() { return ""; }

 protected:
  // Must be called at the end of the derived constructor (starts the watchdog thread).
  void init_common(bool same_stream_default);
  // Stops the watchdog and drains the comm stream (derived destructors call shutdown()).
  void stop_common();
  // Backend hooks (watchdog thread / failure path).
  virtual std::string poll_async_error() { return backend_failure(); }
  virtual void abort_backend() {}

  template <typename Fn>
  std::shared_ptr<Work> launch(OpType op, const std::vector<at::Tensor>& tensors, Fn&& body);
  void fail(const std::string& msg);
  void check_tensor(const at::Tensor& t, const char* what) const;
  void watchdog_loop();

  int device_;
  std::chrono::milliseconds timeout_;
  // Normal priority by default: on gfx950 an eager step with its collectives on a high-priority
  // stream measured 1.26 ms vs 0.55 ms (ConvNet B=4096, one rank, forced comm); graph replay is
  // unaffected.  RINGDP_COMM_HIGH_PRIORITY=1 restores the high-priority stream.
  HipStream comm_stream_;
  hipEvent_t ready_ = nullptr;
  hipEvent_t last_ = nullptr;      // recorded after every eager op on the comm stream (join_into)
  hipEvent_t last_aux_ = nullptr;  // ... and after eager ops that complete on an auxiliary stream
  bool eager_since_join_ = false;
  bool eager_aux_since_join_ = false;
  bool timing_ = false;
  bool same_stream_ = false;  // issue collectives on the caller's stream (see init_common)
  bool caller_ops_ = false;   // ... for the ops issued while set_caller_stream_ops(true)
  bool async_error_handling_ = true;
  std::atomic<bool> stopped_{false};

  std::mutex launch_mu_;
  std::mutex wd_mu_;
  std::condition_variable wd_cv_;
  std::deque<std::shared_ptr<GpuWork>> inflight_;
  // Works the watchdog saw complete.  They keep their output tensors; the watchdog thread never drops the
  // last reference (that may release a tensor's Python object, which needs the GIL - fatal for a native
  // thread while the interpreter finalises).  Freed on the caller's thread by the next launch / drain.
  std::vector<std::shared_ptr<GpuWork>> retired_;
  std::mutex beacon_mu_;
  std::vector<std::weak_ptr<ReplayBeacon>> beacons_;
  std::thread watchdog_;
  std::atomic<bool> stop_{false};
  std::atomic<bool> aborted_{false};
  std::string error_;
  friend class GpuWork;
};

bool env_flag(const char* name, bool dflt);

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

template <typename Fn>
std::shared_ptr<Work> GpuPG::launch(OpType op, const std::vector<at::Tensor>& tensors, Fn&& body) {
  RINGDP_CHECK(!aborted_.load(), "communicator was aborted: ", error_message());
  RINGDP_CHECK(!stopped_.load(), "process group has been shut down");
  std::lock_guard<std::mutex> lk(launch_mu_);
  DeviceScope ds(device_);
  HipStream cur = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(device_);
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  RINGDP_HIP_CHECK(hipStreamIsCapturing(cur.stream(), &cap));
  const bool captured = cap == hipStreamCaptureStatusActive;
  auto work = std::make_shared<GpuWork>(op, next_seq(), this, captured, timing_ && !captured);
  const bool same_stream = on_caller_stream();
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
  // The body may finish the op on another stream (the xGMI sends): it then returns that stream, and
  // the op's completion event is recorded there instead of on the comm stream.
  hipStream_t done_stream = cs;
  if constexpr (std::is_void_v<decltype(body(cs))>) {
    body(cs);
  } else {
    hipStream_t r = body(cs);
    if (r) done_stream = r;
  }
  RINGDP_HIP_CHECK(hipEventRecord(work->done_, done_stream));
  work->outputs_ = tensors;
  if (!captured) {
    if (!same_stream) {
      RINGDP_HIP_CHECK(hipEventRecord(done_stream == cs ? last_ : last_aux_, done_stream));
      if (done_stream == cs) eager_since_join_ = true;
      else eager_aux_since_join_ = true;
    }
    work->deadline_us_ = now_us() + timeout_.count() * 1000;
    std::vector<std::shared_ptr<GpuWork>> retired;
    {
      std::lock_guard<std::mutex> wl(wd_mu_);
      inflight_.push_back(work);
      retired.swap(retired_);
    }
  }
  return work;
}

}  // namespace ringdp
