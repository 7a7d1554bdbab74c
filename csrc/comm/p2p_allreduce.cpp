// One-shot P2P all-reduce: setup (IPC exchange through the store) and launch (see p2p_allreduce.h
// and csrc/kernels/p2p.hip for the protocol).
#include "p2p_allreduce.h"

#include <cstdio>
#include <cstring>
#include <fstream>
#include <unistd.h>

#include "../common.h"

namespace ringdp {

namespace {

std::string host_identity() {
  // boot_id identifies the running kernel (shared by every container on one machine); the
  // hostname separates machines that happen to boot identically.
  std::string id;
  std::ifstream f("/proc/sys/kernel/random/boot_id");
  std::getline(f, id);
  char hn[256] = {0};
  gethostname(hn, sizeof(hn) - 1);
  return id + "/" + hn;
}

struct Handles {
  hipIpcMemHandle_t buf;
  hipIpcMemHandle_t flags;
};

bool all_agree(const std::shared_ptr<Store>& store, const std::string& key, int rank, int world, bool ok) {
  store->set(key + "/" + std::to_string(rank), ok ? "1" : "0");
  bool all = true;
  for (int r = 0; r < world; ++r) all &= store->get(key + "/" + std::to_string(r)) == "1";
  return all;
}

}  // namespace

std::unique_ptr<P2PAllReduce> P2PAllReduce::create(const std::shared_ptr<Store>& store, int rank, int world,
                                                   int device, int64_t max_bytes, int64_t timeout_ms) {
  if (world < 1 || world > kern::kP2PMaxRanks || max_bytes <= 0) return nullptr;
  // same machine?
  const std::string me = host_identity();
  store->set("p2p/host/" + std::to_string(rank), me);
  bool same_host = true;
  for (int r = 0; r < world; ++r) same_host &= store->get("p2p/host/" + std::to_string(r)) == me;
  if (!all_agree(store, "p2p/samehost", rank, world, same_host)) return nullptr;

  std::unique_ptr<P2PAllReduce> p(new P2PAllReduce());
  p->rank_ = rank;
  p->world_ = world;
  p->device_ = device;
  p->max_bytes_ = max_bytes;
  p->slot_bytes_ = (max_bytes + p->seg_bytes_ - 1) / p->seg_bytes_ * p->seg_bytes_;
  p->timeout_ticks_ = static_cast<uint64_t>(timeout_ms) * 100000ull;  // wall_clock64 runs at 100 MHz
  const int64_t nseg = p->slot_bytes_ / p->seg_bytes_;
  const size_t flag_bytes = static_cast<size_t>(nseg) * kern::kP2PMaxRanks * sizeof(unsigned);

  bool ok = true;
  Handles mine{};
  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(device);
  ok &= hipExtMallocWithFlags(reinterpret_cast<void**>(&p->my_buf_), 2 * p->slot_bytes_, hipDeviceMallocUncached) == hipSuccess;
  ok &= ok && hipExtMallocWithFlags(reinterpret_cast<void**>(&p->my_flags_), flag_bytes, hipDeviceMallocUncached) == hipSuccess;
  ok &= ok && hipMalloc(reinterpret_cast<void**>(&p->epochs_), nseg * sizeof(unsigned)) == hipSuccess;
  ok &= ok && hipHostMalloc(reinterpret_cast<void**>(&p->error_), sizeof(int), hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess;
  if (ok) {
    ok &= hipMemset(p->my_flags_, 0, flag_bytes) == hipSuccess;
    ok &= hipMemset(p->epochs_, 0, nseg * sizeof(unsigned)) == hipSuccess;
    *p->error_ = 0;
    ok &= hipIpcGetMemHandle(&mine.buf, p->my_buf_) == hipSuccess;
    ok &= hipIpcGetMemHandle(&mine.flags, p->my_flags_) == hipSuccess;
    ok &= hipDeviceSynchronize() == hipSuccess;
  }
  store->set("p2p/ipc/" + std::to_string(rank),
             ok ? std::string(reinterpret_cast<const char*>(&mine), sizeof(mine)) : std::string("FAIL"));
  kern::P2PArgs& a = p->base_;
  for (int r = 0; r < world; ++r) {
    if (r == rank) {
      a.bufs[r] = p->my_buf_;
      a.flags[r] = p->my_flags_;
      continue;
    }
    std::string s = store->get("p2p/ipc/" + std::to_string(r));
    if (!ok || s.size() != sizeof(Handles)) {
      ok = false;
      continue;
    }
    Handles h;
    std::memcpy(&h, s.data(), sizeof(h));
    void* pb = nullptr;
    void* pf = nullptr;
    if (hipIpcOpenMemHandle(&pb, h.buf, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
      ok = false;
      continue;
    }
    p->opened_.push_back(pb);
    if (hipIpcOpenMemHandle(&pf, h.flags, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
      ok = false;
      continue;
    }
    p->opened_.push_back(pf);
    a.bufs[r] = static_cast<char*>(pb);
    a.flags[r] = static_cast<unsigned*>(pf);
  }
  hipSetDevice(prev);
  if (!all_agree(store, "p2p/ready", rank, world, ok)) {
    (void)hipGetLastError();
    return nullptr;  // destructor releases whatever was mapped / allocated
  }
  int* dev_err = nullptr;
  hipHostGetDevicePointer(reinterpret_cast<void**>(&dev_err), p->error_, 0);
  a.epochs = p->epochs_;
  a.error = dev_err;
  a.slot_bytes = p->slot_bytes_;
  a.seg_bytes = p->seg_bytes_;
  a.world = world;
  a.rank = rank;
  a.timeout_ticks = p->timeout_ticks_;
  return p;
}

P2PAllReduce::~P2PAllReduce() {
  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(device_);
  for (void* q : opened_) hipIpcCloseMemHandle(q);
  if (my_buf_) hipFree(my_buf_);
  if (my_flags_) hipFree(my_flags_);
  if (epochs_) hipFree(epochs_);
  if (error_) hipHostFree(error_);
  hipSetDevice(prev);
}

bool P2PAllReduce::eligible(const at::Tensor& t) const {
  const auto st = t.scalar_type();
  if (st != at::kFloat && st != at::kBFloat16) return false;
  const int64_t nb = t.numel() * static_cast<int64_t>(t.element_size());
  return t.is_contiguous() && nb > 0 && nb <= max_bytes_ && nb % 16 == 0 &&
         reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0;
}

void P2PAllReduce::run(at::Tensor& t, bool average, hipStream_t s) {
  kern::P2PArgs a = base_;
  a.data = t.data_ptr();
  a.nbytes = t.numel() * static_cast<int64_t>(t.element_size());
  a.dtype = t.scalar_type() == at::kBFloat16 ? 1 : 0;
  a.scale = average ? 1.0f / static_cast<float>(world_) : 1.0f;
  kern::p2p_allreduce(a, s);
}

bool P2PAllReduce::failed() { return __atomic_load_n(error_, __ATOMIC_ACQUIRE) != 0; }

}  // namespace ringdp
