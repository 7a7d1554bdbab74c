// xGMI collective engine: setup (IPC exchange through the store) and op launch (see xgmi_engine.h and
// csrc/kernels/xgmi.hip for the protocol).
#include "xgmi_engine.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <unistd.h>

#include <chrono>
#include <thread>

#include "../common.h"

namespace ringdp {

namespace {

int64_t env_i64(const char* name, int64_t dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::atoll(v) : dflt;
}

std::string host_identity() {
  // boot_id identifies the running kernel (shared by every container on one machine); the hostname
  // separates machines that happen to boot identically.
  std::string id;
  std::ifstream f("/proc/sys/kernel/random/boot_id");
  std::getline(f, id);
  char hn[256] = {0};
  gethostname(hn, sizeof(hn) - 1);
  return id + "/" + hn;
}

struct Handles {
  hipIpcMemHandle_t stage;
  hipIpcMemHandle_t flags;
};

bool all_agree(const std::shared_ptr<Store>& store, const std::string& key, int rank, int world, bool ok) {
  store->set(key + "/" + std::to_string(rank), ok ? "1" : "0");
  bool all = true;
  for (int r = 0; r < world; ++r) all &= store->get(key + "/" + std::to_string(r)) == "1";
  return all;
}

int64_t round16(int64_t x) { return (x + 15) / 16 * 16; }

}  // namespace

XgmiConfig XgmiConfig::from_env() {
  XgmiConfig c;
  c.blocks_set = getenv("RINGDP_XGMI_BLOCKS") && *getenv("RINGDP_XGMI_BLOCKS");
  c.slot_set = getenv("RINGDP_XGMI_SLOT_MB") && *getenv("RINGDP_XGMI_SLOT_MB");
  c.nblocks = static_cast<int>(std::clamp<int64_t>(env_i64("RINGDP_XGMI_BLOCKS", c.nblocks), 1, 1024));
  c.slot_bytes = round16(std::max<int64_t>(env_i64("RINGDP_XGMI_SLOT_MB", c.slot_bytes >> 20), 1) << 20);
  c.p2p_slot_bytes = round16(std::max<int64_t>(env_i64("RINGDP_XGMI_P2P_SLOT_MB", 1), 1) << 20);
  c.oneshot_max = std::max<int64_t>(env_i64("RINGDP_XGMI_ONESHOT_KB", 512), 0) << 10;
  return c;
}

std::unique_ptr<XgmiEngine> XgmiEngine::create(const std::shared_ptr<Store>& store, int rank, int world,
                                               int device, const XgmiConfig& cfg, int64_t timeout_ms,
                                               std::string* why) {
  auto say = [&](const char* m) {
    if (why) *why = m;
    return nullptr;
  };
  if (world < 1 || world > kern::kXgMaxRanks) return say("more than 16 ranks");
  const std::string me = host_identity();
  store->set("xgmi/host/" + std::to_string(rank), me);
  bool same_host = true;
  for (int r = 0; r < world; ++r) same_host &= store->get("xgmi/host/" + std::to_string(r)) == me;
  if (!all_agree(store, "xgmi/samehost", rank, world, same_host)) return say("ranks are not on one host");

  // ranks sharing a device (same PCI bus id): the shared-GPU defaults unless the environment says otherwise
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus) - 1, device) != hipSuccess) std::snprintf(bus, sizeof(bus), "dev%d", device);
  store->set("xgmi/bus/" + std::to_string(rank), bus);
  bool shared = false;
  for (int r = 0; r < world; ++r)
    if (r != rank) shared |= store->get("xgmi/bus/" + std::to_string(r)) == std::string(bus);
  shared = !all_agree(store, "xgmi/distinct", rank, world, !shared);
  XgmiConfig c = cfg;
  if (shared && !c.blocks_set) c.nblocks = 64;
  if (shared && !c.slot_set) c.slot_bytes = 4 << 20;
  if (!c.slot_set) {
    // cap the two staging regions (4 x world x slot per rank, plus every peer's IPC mapping of them) at
    // RINGDP_XGMI_STAGING_MB (256): 16 MiB slots are 128 MiB at ws2 but would be 512 MiB at ws8, and
    // small sub-groups from new_group get their own engine; above the cap the slot shrinks (ws8: 8 MiB,
    // a 26 MB bucket then takes one two-shot pass in world x slot = 64 MiB pieces - still one piece)
    const int64_t cap = std::max<int64_t>(env_i64("RINGDP_XGMI_STAGING_MB", 256), 4) << 20;
    const int64_t per = cap / (4 * static_cast<int64_t>(world));
    if (c.slot_bytes > per) c.slot_bytes = std::max<int64_t>(1 << 20, per >> 20 << 20);
  }

  std::unique_ptr<XgmiEngine> p(new XgmiEngine());
  p->rank_ = rank;
  p->world_ = world;
  p->device_ = device;
  p->cfg_ = c;
  p->cfg_.oneshot_max = std::min(c.oneshot_max, c.slot_bytes);
  const int G = c.nblocks;
  const int64_t region = 2 * static_cast<int64_t>(world) * c.slot_bytes;
  const int64_t off_a = 0, off_b = region, off_p2p = 2 * region;
  const int64_t stage_bytes = off_p2p + static_cast<int64_t>(kern::kXgMaxRanks) * 2 * c.p2p_slot_bytes;
  const size_t flag_bytes = static_cast<size_t>(4) * G * kern::kXgMaxRanks * sizeof(unsigned);
  const size_t epoch_bytes = static_cast<size_t>(1 + 2 * kern::kXgMaxRanks) * G * sizeof(unsigned);

  bool ok = true;
  Handles mine{};
  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(device);
  // uncached (fine-grained on every agent): peers' pushes are never hidden behind a stale L2 line
  ok &= hipExtMallocWithFlags(reinterpret_cast<void**>(&p->stage_), stage_bytes, hipDeviceMallocUncached) == hipSuccess;
  ok = ok && hipExtMallocWithFlags(reinterpret_cast<void**>(&p->flags_), flag_bytes, hipDeviceMallocUncached) == hipSuccess;
  ok = ok && hipMalloc(reinterpret_cast<void**>(&p->epochs_), epoch_bytes) == hipSuccess;
  ok = ok && hipHostMalloc(reinterpret_cast<void**>(&p->error_), sizeof(int),
                           hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess;
  if (ok) {
    ok &= hipMemset(p->flags_, 0, flag_bytes) == hipSuccess;
    ok &= hipMemset(p->epochs_, 0, epoch_bytes) == hipSuccess;
    *p->error_ = 0;
    ok &= hipIpcGetMemHandle(&mine.stage, p->stage_) == hipSuccess;
    ok &= hipIpcGetMemHandle(&mine.flags, p->flags_) == hipSuccess;
    ok &= hipDeviceSynchronize() == hipSuccess;
  }
  store->set("xgmi/ipc/" + std::to_string(rank),
             ok ? std::string(reinterpret_cast<const char*>(&mine), sizeof(mine)) : std::string("FAIL"));
  kern::XgArgs& a = p->base_;
  for (int r = 0; r < world; ++r) {
    if (r == rank) {
      a.stage[r] = p->stage_;
      a.flags[r] = p->flags_;
      continue;
    }
    std::string s = store->get("xgmi/ipc/" + std::to_string(r));
    if (!ok || s.size() != sizeof(Handles)) {
      ok = false;
      continue;
    }
    Handles h;
    std::memcpy(&h, s.data(), sizeof(h));
    void* ps = nullptr;
    void* pf = nullptr;
    if (hipIpcOpenMemHandle(&ps, h.stage, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
      ok = false;
      continue;
    }
    p->opened_.push_back(ps);
    if (hipIpcOpenMemHandle(&pf, h.flags, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
      ok = false;
      continue;
    }
    p->opened_.push_back(pf);
    a.stage[r] = static_cast<char*>(ps);
    a.flags[r] = static_cast<unsigned*>(pf);
  }
  hipSetDevice(prev);
  if (!all_agree(store, "xgmi/ready", rank, world, ok)) {
    (void)hipGetLastError();
    return say("staging allocation or IPC mapping failed on some rank");  // the destructor releases it
  }
  int* dev_err = nullptr;
  hipHostGetDevicePointer(reinterpret_cast<void**>(&dev_err), p->error_, 0);
  a.epochs = p->epochs_;
  a.error = dev_err;
  // the per-rank pointers as a device-memory table: the kernels index it by peer (a kernel-argument
  // array indexed by a run-time value is copied to scratch first in every thread)
  {
    void* tab[2 * kern::kXgMaxRanks];
    for (int r = 0; r < kern::kXgMaxRanks; ++r) {
      tab[r] = a.stage[r];
      tab[kern::kXgMaxRanks + r] = a.flags[r];
    }
    if (hipMalloc(reinterpret_cast<void**>(&p->ptr_tab_), sizeof(tab)) != hipSuccess ||
        hipMemcpy(p->ptr_tab_, tab, sizeof(tab), hipMemcpyHostToDevice) != hipSuccess)
      return say("pointer table allocation failed");
    a.stage_tab = reinterpret_cast<char* const*>(p->ptr_tab_);
    a.flag_tab = reinterpret_cast<unsigned* const*>(p->ptr_tab_ + kern::kXgMaxRanks);
  }
  // the kernels' own spin bound is the group timeout itself (s_memrealtime: 100 MHz ticks), uncapped,
  // so a slow but healthy peer (evaluation, checkpointing) gets the same grace as under c10d
  a.timeout_ticks = static_cast<uint64_t>(std::max<int64_t>(timeout_ms, 1)) * 100000ull;
  a.world = world;
  a.rank = rank;
  a.nblocks = G;
  a.slot = c.slot_bytes;
  a.p2p_slot = c.p2p_slot_bytes;
  a.off_a = off_a;
  a.off_b = off_b;
  a.off_p2p = off_p2p;
  a.scale = 1.0f / static_cast<float>(world);
  p->store_ = store;
  return p;
}

bool XgmiEngine::quiesce(int64_t timeout_ms) {
  if (quiesced_) return !leak_exported_;
  quiesced_ = true;
  if (world_ == 1) return true;
  try {
    store_->add("xgmi/fin", 1);
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(std::max<int64_t>(timeout_ms, 1));
    while (store_->add("xgmi/fin", 0) < world_) {
      if (std::chrono::steady_clock::now() > deadline) {
        leak_exported_ = true;
        return false;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    return true;
  } catch (const std::exception&) {
    leak_exported_ = true;
    return false;
  }
}

XgmiEngine::~XgmiEngine() {
  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(device_);
  for (void* q : opened_) hipIpcCloseMemHandle(q);
  // memory that peers map: freed only after a group-wide quiesce (a peer kernel could still push)
  const bool free_exported = world_ == 1 || (quiesced_ && !leak_exported_);
  if (stage_ && free_exported) hipFree(stage_);
  if (flags_ && free_exported) hipFree(flags_);
  if (epochs_) hipFree(epochs_);
  if (ptr_tab_) hipFree(ptr_tab_);
  if (error_) hipHostFree(error_);
  hipSetDevice(prev);
}

bool XgmiEngine::failed() const { return error_ && __atomic_load_n(error_, __ATOMIC_ACQUIRE) != 0; }

void XgmiEngine::launch(kern::XgArgs& a, hipStream_t s) {
  kern::xgmi_collective(a, s);
  RINGDP_HIP_CHECK(hipGetLastError());
}

void XgmiEngine::allreduce(const void* in, void* out, int64_t nbytes, int dtype, int red, bool average,
                           hipStream_t s) {
  if (nbytes <= 0) return;
  kern::XgArgs a = base_;
  a.dtype = dtype;
  a.red = red;
  a.average = average ? 1 : 0;
  if (nbytes <= cfg_.oneshot_max) {
    a.kind = kern::XG_ONESHOT;
    a.in = static_cast<const char*>(in);
    a.out = static_cast<char*>(out);
    a.nbytes = nbytes;
    launch(a, s);
    return;
  }
  // two-shot in pieces of at most world * slot bytes (each rank's chunk fits one slot)
  a.kind = kern::XG_TWOSHOT;
  const int64_t piece_max = static_cast<int64_t>(world_) * cfg_.slot_bytes;
  for (int64_t o = 0; o < nbytes; o += piece_max) {
    const int64_t ps = std::min(piece_max, nbytes - o);
    a.in = static_cast<const char*>(in) + o;
    a.out = static_cast<char*>(out) + o;
    a.nbytes = ps;
    a.chunk = round16((ps + world_ - 1) / world_);
    launch(a, s);
  }
}

void XgmiEngine::reduce_scatter(const void* in, void* out, int64_t block_bytes, int dtype, int red,
                                bool average, hipStream_t s) {
  if (block_bytes <= 0) return;
  kern::XgArgs a = base_;
  a.kind = kern::XG_REDUCE_SCATTER;
  a.dtype = dtype;
  a.red = red;
  a.average = average ? 1 : 0;
  a.stride = block_bytes;
  for (int64_t o = 0; o < block_bytes; o += cfg_.slot_bytes) {
    a.in = static_cast<const char*>(in) + o;
    a.out = static_cast<char*>(out) + o;
    a.nbytes = std::min(cfg_.slot_bytes, block_bytes - o);
    launch(a, s);
  }
}

void XgmiEngine::allgather(const void* in, void* out, int64_t block_bytes, hipStream_t s) {
  if (block_bytes <= 0) return;
  kern::XgArgs a = base_;
  a.kind = kern::XG_ALLGATHER;
  a.stride = block_bytes;
  for (int64_t o = 0; o < block_bytes; o += cfg_.slot_bytes) {
    a.in = static_cast<const char*>(in) + o;
    a.out = static_cast<char*>(out) + o;
    a.nbytes = std::min(cfg_.slot_bytes, block_bytes - o);
    launch(a, s);
  }
}

void XgmiEngine::broadcast(const void* in, void* out, int64_t nbytes, int root, hipStream_t s) {
  if (nbytes <= 0) return;
  kern::XgArgs a = base_;
  a.kind = kern::XG_BROADCAST;
  a.root = root;
  for (int64_t o = 0; o < nbytes; o += cfg_.slot_bytes) {
    a.in = static_cast<const char*>(in) + o;
    a.out = static_cast<char*>(out) + o;
    a.nbytes = std::min(cfg_.slot_bytes, nbytes - o);
    launch(a, s);
  }
}

void XgmiEngine::send(const void* in, int64_t nbytes, int dst, hipStream_t s) {
  kern::XgArgs a = base_;
  a.kind = kern::XG_SEND;
  a.peer = dst;
  int64_t o = 0;
  do {  // a zero-byte message still pairs with its recv
    a.in = static_cast<const char*>(in) + o;
    a.nbytes = std::min(cfg_.p2p_slot_bytes, nbytes - o);
    launch(a, s);
    o += cfg_.p2p_slot_bytes;
  } while (o < nbytes);
}

void XgmiEngine::recv(void* out, int64_t nbytes, int src, hipStream_t s) {
  kern::XgArgs a = base_;
  a.kind = kern::XG_RECV;
  a.peer = src;
  int64_t o = 0;
  do {
    a.out = static_cast<char*>(out) + o;
    a.nbytes = std::min(cfg_.p2p_slot_bytes, nbytes - o);
    launch(a, s);
    o += cfg_.p2p_slot_bytes;
  } while (o < nbytes);
}

void XgmiEngine::barrier(hipStream_t s) {
  kern::XgArgs a = base_;
  a.kind = kern::XG_BARRIER;
  launch(a, s);
}

}  // namespace ringdp
