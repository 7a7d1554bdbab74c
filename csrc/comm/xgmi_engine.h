// xGMI collective engine: IPC-mapped symmetric staging memory + the kernels of csrc/kernels/xgmi.hip.
//
// Owned by an XgmiPG (every collective) or by an RcclPG (small all-reduces, when
// RINGDP_P2P_ALLREDUCE_MAX_BYTES > 0).  Creation is collective over the group: every rank allocates an
// uncached staging buffer and a flag block on its GPU, exports both by IPC handle through the store,
// maps every peer's, and all ranks agree through the store that every one of them succeeded.  Ranks
// may share a GPU (IPC within one device).  Every op is stream-ordered on the stream it is given,
// hipGraph-capturable (epochs live in device memory), and issues exactly `nblocks` workgroups.
//
// Staging layout (each rank, one allocation):
//   region A  [2 parities][world][slot]   one-shot / reduce-scatter / all-gather / broadcast inbound
//   region B  [2 parities][world][slot]   two-shot all-gather inbound
//   region P  [16 sources][2 parities][p2p_slot]   send/recv
// Messages larger than a slot are cut into pieces, each one op (one epoch).
#pragma once

#include <hip/hip_runtime_api.h>

#include <memory>
#include <string>
#include <vector>

#include "../kernels/kernels.h"
#include "../store/store.h"

namespace ringdp {

struct XgmiConfig {
  // defaults from the ws2 sweep (profiles/r05/xgmi/): 26 MB all-reduce 164 us at 64 blocks / 4 MiB slots,
  // 82 us at 128 / 16 MiB (69 us at 256 blocks, whose per-workgroup handshakes cost small messages +50 %)
  int nblocks = 128;                 // RINGDP_XGMI_BLOCKS
  int64_t slot_bytes = 16 << 20;     // RINGDP_XGMI_SLOT_MB (staging: 4 x world x slot per rank, capped at
                                     // RINGDP_XGMI_STAGING_MB = 256 unless the slot size is set explicitly)
  int64_t p2p_slot_bytes = 1 << 20;  // RINGDP_XGMI_P2P_SLOT_MB
  int64_t oneshot_max = 512 << 10;   // RINGDP_XGMI_ONESHOT_KB: all-reduces up to this size are one-shot
  // set from the environment: otherwise ranks that SHARE a GPU (a one-GPU box running the multi-process
  // protocol) get the round-4 64 blocks / 4 MiB - 4 ranks x 128 spinning workgroups on one device starved
  // the other ranks' compute in the ws4 DDP test
  bool blocks_set = false, slot_set = false;
  static XgmiConfig from_env();
};

class XgmiEngine {
 public:
  // nullptr on every rank when the path cannot be used (ranks on different hosts, more than 16
  // ranks, an allocation or IPC failure on any rank); `why` says which.
  static std::unique_ptr<XgmiEngine> create(const std::shared_ptr<Store>& store, int rank, int world,
                                            int device, const XgmiConfig& cfg, int64_t timeout_ms,
                                            std::string* why = nullptr);
  ~XgmiEngine();

  int rank() const { return rank_; }
  int world() const { return world_; }
  const XgmiConfig& config() const { return cfg_; }

  // dtype: kern::XgDtype; red: kern::XgRed.  Pointers 16-B aligned, sizes in bytes.
  // In place (in == out allowed).
  void allreduce(const void* in, void* out, int64_t nbytes, int dtype, int red, bool average,
                 hipStream_t s);
  // in: world blocks of block_bytes (multiple of 16), out: block_bytes.
  void reduce_scatter(const void* in, void* out, int64_t block_bytes, int dtype, int red, bool average,
                      hipStream_t s);
  // in: block_bytes, out: world blocks of block_bytes (multiple of 16).
  void allgather(const void* in, void* out, int64_t block_bytes, hipStream_t s);
  void broadcast(const void* in, void* out, int64_t nbytes, int root, hipStream_t s);
  void send(const void* in, int64_t nbytes, int dst, hipStream_t s);
  void recv(void* out, int64_t nbytes, int src, hipStream_t s);
  void barrier(hipStream_t s);

  // Host-side check of the kernels' timeout word (true: some peer did not arrive in time).
  bool failed() const;

  // Group-wide quiesce before teardown: every rank has drained its streams and arrived through the
  // store, so no peer kernel can still be writing into this rank's exported staging / flag memory.
  // Call it (collectively) before destroying the engine of a healthy group.  On failure (a peer never
  // arrives within `timeout_ms`, or the store is gone) the exported buffers are leaked rather than
  // freed under a possibly live writer.
  bool quiesce(int64_t timeout_ms);
  // Aborted groups skip the quiesce: peers are dead or desynchronised; leak the exported memory.
  void mark_unsafe() { leak_exported_ = true; }

 private:
  XgmiEngine() = default;
  void launch(kern::XgArgs& a, hipStream_t s);

  int rank_ = 0, world_ = 1, device_ = 0;
  XgmiConfig cfg_;
  char* stage_ = nullptr;
  unsigned* flags_ = nullptr;
  unsigned* epochs_ = nullptr;
  void** ptr_tab_ = nullptr;  // device copy of the stage / flag pointer tables (XgArgs::stage_tab)
  int* error_ = nullptr;  // hipHostMalloc'd, mapped
  std::vector<void*> opened_;
  kern::XgArgs base_{};
  std::shared_ptr<Store> store_;
  bool quiesced_ = false, leak_exported_ = false;
};

}  // namespace ringdp
