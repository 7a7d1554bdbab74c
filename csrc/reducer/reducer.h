// ringdp gradient Reducer: bucketed, ordered, overlapped gradient all-reduce.
//
// Parity target: c10d Reducer (c10d/reducer.hpp).  Behaviour kept:
//   * per-parameter hooks on the AccumulateGrad node fire as gradients become ready;
//   * a bucket launches when all its gradients are ready, and buckets launch strictly in index
//     order (every rank issues the same collective sequence whatever the readiness order);
//   * finalize at the end of backward (engine callback) waits for every bucket;
//   * "marked ready twice" / unused-parameter errors; no_sync; bucket rebuild from the
//     observed ready order after iteration 0 (limits [first_bucket, bucket_cap]).
// MI355X-first differences:
//   * gradients ALWAYS live in the flat bucket (grad-as-bucket-view): the reducer hands out
//     per-parameter "grad slots" that ringdp kernels write into directly, so there is no
//     copy-in (K23) or copy-out (K24) kernel;
//   * averaging is done by the collective (ncclAvg) - no 1/N scale kernel;
//   * optional bf16/fp16 wire compression uses ringdp's cast kernels on the comm path.
#pragma once

#include <ATen/ATen.h>
#include <torch/csrc/autograd/function.h>

#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "../comm/process_group.h"

namespace ringdp {

enum class CommHook : int { ALLREDUCE = 0, BF16_COMPRESS = 1, FP16_COMPRESS = 2, PYTHON = 3, NONE = 4 };

// Mirrors c10d::compute_bucket_assignment_by_size (returns bucket indices + per-bucket limits).
std::pair<std::vector<std::vector<int64_t>>, std::vector<int64_t>> compute_bucket_assignment_by_size(
    const std::vector<at::Tensor>& tensors, const std::vector<int64_t>& bucket_size_limits,
    const std::vector<bool>& expect_sparse_gradient, const std::vector<int64_t>& tensor_indices);

struct BucketStats {
  int64_t numel = 0;
  int64_t bytes = 0;
  double last_ready_us = 0;     // since first hook of the iteration
  double last_launch_us = 0;
  double last_comm_us = -1;     // device-measured when RINGDP_COMM_TIMING=1
  double total_comm_us = 0;
  int64_t comm_samples = 0;
};

class Reducer {
 public:
  using PyHook = std::function<std::shared_ptr<Work>(int64_t bucket_index, at::Tensor flat)>;

  Reducer(std::vector<at::Tensor> params, std::vector<std::vector<int64_t>> bucket_indices,
          std::shared_ptr<ProcessGroup> pg, bool find_unused_parameters, int64_t pad_elems);
  ~Reducer();

  // Called by DDP around forward / backward.
  void prepare_for_forward();
  void prepare_for_backward();
  void set_require_sync(bool v);
  bool require_sync() const { return require_sync_; }

  void set_comm_hook(CommHook h) { hook_ = h; }
  void set_python_hook(PyHook fn) {
    py_hook_ = std::move(fn);
    hook_ = CommHook::PYTHON;
  }
  CommHook comm_hook() const { return hook_; }

  // Layout: per param (bucket id, offset in the flat buffer of its dtype key).
  std::vector<at::Tensor> grad_slots() const { return views_; }
  std::vector<at::Tensor> flat_buffers() const;
  std::vector<int64_t> param_offsets() const { return offsets_; }
  std::vector<std::vector<int64_t>> bucket_indices() const { return bucket_indices_; }
  std::vector<int64_t> bucket_numels() const;

  // Ready order recorded during the first backward (rebuild input).
  std::vector<int64_t> ready_order() const { return ready_order_; }
  bool rebuilt() const { return rebuilt_; }
  void rebuild_buckets(std::vector<std::vector<int64_t>> new_indices);

  int64_t iteration() const { return iteration_; }
  std::vector<BucketStats> stats() const;
  // Device-measured duration of each bucket's last collective (-1 where unknown: no timing
  // events, captured in a hipGraph, or not complete).  Call after synchronising the device;
  // also folds the samples into stats().
  std::vector<double> collect_comm_times();

  // Segmented hipGraph capture (ringdp.utils.graph.StepGraph, split mode): while a split function is set,
  // each bucket whose collective would be issued (ALLREDUCE / BF16 / FP16 hook) asks split(index) first.
  // true: the capture ended its current graph segment there (or defers the bucket to the next boundary) and
  // the replay issues the collective between segments on the comm stream (launch_collective), overlapping
  // the rest of backward; false: the collective is captured inline on the compute stream (worth less than a
  // segment boundary, or the last bucket, which nothing follows).  The end of backward calls split(-1), the
  // join point before the optimizer segment.  Every segment stays a single-stream chain: no fork inside a
  // graph.  Compressed hooks keep their casts on the compute stream: the bf16/fp16 wire copy is captured in
  // the segment that produced the gradients, the split collective all-reduces the wire buffer, and the
  // decompression is captured after the join (finalize_backward), ahead of the optimizer.
  using SplitFn = std::function<bool(int64_t)>;
  void set_capture_split(SplitFn fn) {
    std::lock_guard<std::mutex> lk(mu_);
    split_ = std::move(fn);
  }
  std::shared_ptr<Work> launch_collective(int64_t index);

  // Internal: invoked from the AccumulateGrad post hook.
  void autograd_hook(int64_t index);

 private:
  struct Bucket {
    std::vector<int64_t> params;
    at::Tensor flat;       // view into the per-dtype flat grad buffer
    at::Tensor wire;       // compressed copy for BF16/FP16 hooks
    int64_t pending = 0;
    bool launched = false;
    bool split_wire = false;  // split capture of a compressed bucket: decompress after the join
    std::shared_ptr<Work> work;
    BucketStats st;
  };

  void build(const std::vector<std::vector<int64_t>>& bucket_indices);
  void launch_ready_buckets();
  void launch_bucket(Bucket& b, int64_t index);
  void finalize_backward();
  void install_hooks();
  void remove_hooks();

  std::vector<at::Tensor> params_;
  std::shared_ptr<ProcessGroup> pg_;
  bool find_unused_;
  int64_t pad_elems_;

  std::vector<std::vector<int64_t>> bucket_indices_;
  std::vector<Bucket> buckets_;
  std::vector<int64_t> param_bucket_;  // param -> bucket
  std::vector<at::Tensor> views_;      // per param grad slot
  std::vector<int64_t> offsets_;       // per param offset in its dtype's flat buffer
  std::map<int, at::Tensor> flat_by_dtype_;

  // Tensor-level post-accumulate-grad hooks (one per parameter).  Hooks are attached to the
  // parameter, not to an AccumulateGrad node, so the reducer never pins a node created on another
  // stream (which would break hipGraph capture of backward).
  std::vector<bool> hooked_;

  std::mutex mu_;
  CommHook hook_ = CommHook::ALLREDUCE;
  PyHook py_hook_;
  SplitFn split_;
  bool split_this_iter_ = false;
  bool expect_hooks_ = false;
  bool require_sync_ = true;
  bool finalize_queued_ = false;
  std::vector<char> ready_;
  int64_t next_bucket_ = 0;
  int64_t iteration_ = 0;
  int64_t backward_start_us_ = 0;
  bool record_order_ = true;
  bool rebuilt_ = false;
  std::vector<int64_t> ready_order_;
};

}  // namespace ringdp
