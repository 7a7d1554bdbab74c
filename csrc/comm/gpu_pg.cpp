// Shared GPU process-group machinery (see gpu_pg.h).
#include "gpu_pg.h"

#include "../kernels/kernels.h"

#include <c10/core/DeviceGuard.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace ringdp {

bool env_flag(const char* name, bool dflt) {
  const char* v = std::getenv(name);
  if (!v || !*v) return dflt;
  return !(std::strcmp(v, "0") == 0 || std::strcmp(v, "false") == 0);
}

// ------------------------------------------------------------------ GpuWork
GpuWork::GpuWork(OpType op, uint64_t seq, GpuPG* pg, bool captured, bool timing)
    : Work(op, seq), captured_(captured), pg_(pg) {
  RINGDP_HIP_CHECK(hipEventCreateWithFlags(&done_, timing ? hipEventDefault : hipEventDisableTiming));
  if (timing) RINGDP_HIP_CHECK(hipEventCreateWithFlags(&start_, hipEventDefault));
}

GpuWork::~GpuWork() {
  if (done_) hipEventDestroy(done_);
  if (start_) hipEventDestroy(start_);
}

bool GpuWork::is_completed() {
  if (captured_) return false;
  return hipEventQuery(done_) == hipSuccess;
}

void GpuWork::wait(bool blocking) {
  if (pg_->aborted()) throw RingdpError("[ringdp] communicator aborted: " + pg_->error_message());
  HipStream cur = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(pg_->device());
  RINGDP_HIP_CHECK(hipStreamWaitEvent(cur.stream(), done_, 0));
  if (blocking && !captured_) {
    auto deadline = now_us() + pg_->timeout().count() * 1000;
    while (hipEventQuery(done_) == hipErrorNotReady) {
      if (pg_->aborted()) throw RingdpError("[ringdp] communicator aborted: " + pg_->error_message());
      if (now_us() > deadline)
        throw TimeoutError(strcat_all("[ringdp] ", pg_->backend_name(), " ", op_name(op_), " seq ", seq_,
                                      " timed out after ", pg_->timeout().count(), " ms"));
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    // a completed op whose kernel gave up on a peer left unreduced data: never return it silently
    const std::string f = pg_->backend_failure();
    if (!f.empty()) throw RingdpError("[ringdp] " + pg_->backend_name() + " " + op_name(op_) + " failed: " + f);
  }
}

double GpuWork::duration_us() {
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

// ------------------------------------------------------------------ GpuPG
GpuPG::GpuPG(int rank, int size, int device, std::chrono::milliseconds timeout)
    : ProcessGroup(rank, size),
      device_(device),
      timeout_(timeout),
      comm_stream_(c10::hip::getStreamFromPoolMasqueradingAsCUDA(env_flag("RINGDP_COMM_HIGH_PRIORITY", false),
                                                                 device)) {}

GpuPG::~GpuPG() { stop_common(); }

void GpuPG::init_common(bool same_stream_default) {
  DeviceScope ds(device_);
  // RINGDP_COMM_SAME_STREAM=1 / 0 forces the caller's stream / the side stream for any group size.
  if (const char* v = std::getenv("RINGDP_COMM_SAME_STREAM"))
    same_stream_ = std::strcmp(v, "1") == 0;
  else
    same_stream_ = same_stream_default;
  RINGDP_HIP_CHECK(hipEventCreateWithFlags(&ready_, hipEventDisableTiming));
  RINGDP_HIP_CHECK(hipEventCreateWithFlags(&last_, hipEventDisableTiming));
  RINGDP_HIP_CHECK(hipEventCreateWithFlags(&last_aux_, hipEventDisableTiming));
  timing_ = env_flag("RINGDP_COMM_TIMING", false);
  async_error_handling_ = env_flag("RINGDP_ASYNC_ERROR_HANDLING", true);
  watchdog_ = std::thread([this] { watchdog_loop(); });
}

void GpuPG::set_same_stream(bool v) {
  std::lock_guard<std::mutex> lk(launch_mu_);
  if (v == same_stream_) return;
  DeviceScope ds(device_);
  RINGDP_HIP_CHECK(hipDeviceSynchronize());
  same_stream_ = v;
}

void GpuPG::stop_common() {
  if (stopped_.exchange(true)) return;
  stop_.store(true);
  wd_cv_.notify_all();
  if (watchdog_.joinable()) watchdog_.join();
  {
    DeviceScope ds(device_);
    // every op issued so far, on the comm stream or (same-stream mode) on callers' streams
    if (!aborted_.load()) {
      (void)hipStreamSynchronize(comm_stream_.stream());
      if (same_stream_) (void)hipDeviceSynchronize();
    }
    std::lock_guard<std::mutex> lk(wd_mu_);
    inflight_.clear();
    retired_.clear();
    if (ready_) hipEventDestroy(ready_);
    if (last_) hipEventDestroy(last_);
    if (last_aux_) hipEventDestroy(last_aux_);
    ready_ = last_ = last_aux_ = nullptr;
  }
}

void GpuPG::shutdown() { stop_common(); }

void GpuPG::drain() {
  std::lock_guard<std::mutex> lk(wd_mu_);
  DeviceScope ds(device_);
  for (auto& w : inflight_) (void)hipEventSynchronize(w->done_);
  inflight_.clear();
  retired_.clear();
}

void GpuPG::watch_beacon(const std::shared_ptr<ReplayBeacon>& beacon) {
  std::lock_guard<std::mutex> bl(beacon_mu_);
  beacon->last_done_ = beacon->completed();
  beacon->progress_us_ = now_us();
  beacons_.push_back(beacon);
}

void GpuPG::join_into(hipStream_t stream) {
  std::lock_guard<std::mutex> lk(launch_mu_);
  if (eager_since_join_ && last_) RINGDP_HIP_CHECK(hipStreamWaitEvent(stream, last_, 0));
  if (eager_aux_since_join_ && last_aux_) RINGDP_HIP_CHECK(hipStreamWaitEvent(stream, last_aux_, 0));
  eager_since_join_ = eager_aux_since_join_ = false;
}

void GpuPG::abort() {
  if (!aborted_.exchange(true)) abort_backend();
}

void GpuPG::fail(const std::string& msg) {
  {
    std::lock_guard<std::mutex> lk(wd_mu_);
    error_ = msg;
  }
  std::fprintf(stderr, "%s\n", msg.c_str());
  std::fflush(stderr);
  if (!aborted_.exchange(true)) abort_backend();
  if (async_error_handling_) {
    std::fprintf(stderr,
                 "[ringdp] rank %d: tearing the process down after a communicator failure "
                 "(set RINGDP_ASYNC_ERROR_HANDLING=0 to raise instead)\n",
                 rank_);
    std::fflush(stderr);
    std::_Exit(1);
  }
}

void GpuPG::watchdog_loop() {
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
          retired_.push_back(std::move(w));  // freed on the caller's thread (see retired_)
          inflight_.pop_front();
          continue;
        }
        if (now > w->deadline_us_) {
          failure = strcat_all("[ringdp] watchdog: rank ", rank_, " ", backend_name(), " ", op_name(w->op()),
                               " (seq ", w->seq(), ") did not complete within ", timeout_.count(),
                               " ms; aborting communicator");
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
    if (failure.empty()) {
      const std::string be = poll_async_error();
      if (!be.empty()) failure = strcat_all("[ringdp] watchdog: rank ", rank_, " ", backend_name(), ": ", be);
    }
    if (!failure.empty()) fail(failure);
  }
}

void GpuPG::check_tensor(const at::Tensor& t, const char* what) const {
  RINGDP_CHECK(t.is_cuda(), what, ": ", backend_name(), " backend expects GPU tensors, got ", t.device());
  RINGDP_CHECK(t.get_device() == device_, what, ": tensor on device ", t.get_device(),
               " but process group is bound to device ", device_);
  RINGDP_CHECK(t.is_contiguous(), what, ": tensor must be contiguous");
}

}  // namespace ringdp
