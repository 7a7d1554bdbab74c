// ringdp gradient Reducer implementation (see reducer.h).
#include "reducer.h"

#include "../trace/trace.h"

#include <torch/csrc/autograd/engine.h>
#include <torch/csrc/autograd/functions/accumulate_grad.h>
#include <torch/csrc/autograd/utils/lambda_post_hook.h>
#include <torch/csrc/autograd/variable.h>

#include <algorithm>
#include <cstdlib>
#include <unordered_map>

#include "../ops/ops.h"

namespace ringdp {

// ------------------------------------------------------------------ bucket assignment
std::pair<std::vector<std::vector<int64_t>>, std::vector<int64_t>> compute_bucket_assignment_by_size(
    const std::vector<at::Tensor>& tensors, const std::vector<int64_t>& limits,
    const std::vector<bool>& expect_sparse, const std::vector<int64_t>& tensor_indices) {
  RINGDP_CHECK(!tensors.empty(), "compute_bucket_assignment_by_size: no tensors");
  RINGDP_CHECK(!limits.empty(), "compute_bucket_assignment_by_size: no size limits");
  RINGDP_CHECK(expect_sparse.empty() || expect_sparse.size() == tensors.size(),
               "expect_sparse_gradient must match tensors");
  struct Acc {
    std::vector<int64_t> indices;
    int64_t size = 0;
    int64_t limit = 0;
  };
  using Key = std::pair<int, std::string>;
  std::vector<std::pair<std::vector<int64_t>, int64_t>> result;
  std::map<Key, size_t> limit_it;
  std::map<Key, Acc> buckets;
  std::vector<Key> key_order;  // first-seen order for the remainder flush
  for (size_t i = 0; i < tensors.size(); ++i) {
    const auto& t = tensors[i];
    int64_t idx = tensor_indices.empty() ? static_cast<int64_t>(i) : tensor_indices[i];
    if (!expect_sparse.empty() && expect_sparse[idx]) {
      result.push_back({{idx}, 0});
      continue;
    }
    Key key{static_cast<int>(t.scalar_type()), t.device().str()};
    if (!buckets.count(key)) key_order.push_back(key);
    auto& b = buckets[key];
    b.indices.push_back(idx);
    b.size += t.numel() * static_cast<int64_t>(t.element_size());
    if (!limit_it.count(key)) limit_it[key] = 0;
    size_t& li = limit_it[key];
    b.limit = limits[li];
    if (b.size >= b.limit) {
      result.push_back({std::move(b.indices), b.limit});
      b = Acc();
      if (li + 1 < limits.size()) ++li;
    }
  }
  // Remainder flush: most recently first-seen key first (the iteration order c10d's
  // unordered_map yields with libstdc++, so mixed-dtype layouts match upstream too).
  for (auto it = key_order.rbegin(); it != key_order.rend(); ++it) {
    auto& b = buckets[*it];
    if (!b.indices.empty()) result.push_back({std::move(b.indices), b.limit});
  }
  if (tensor_indices.empty()) {
    std::stable_sort(result.begin(), result.end(), [](const auto& a, const auto& b) {
      return *std::min_element(a.first.begin(), a.first.end()) <
             *std::min_element(b.first.begin(), b.first.end());
    });
  }
  std::vector<std::vector<int64_t>> idx;
  std::vector<int64_t> lims;
  for (auto& r : result) {
    idx.push_back(std::move(r.first));
    lims.push_back(r.second);
  }
  return {idx, lims};
}

// ------------------------------------------------------------------ construction
Reducer::Reducer(std::vector<at::Tensor> params, std::vector<std::vector<int64_t>> bucket_indices,
                 std::shared_ptr<ProcessGroup> pg, bool find_unused_parameters, int64_t pad_elems)
    : params_(std::move(params)),
      pg_(std::move(pg)),
      find_unused_(find_unused_parameters),
      pad_elems_(std::max<int64_t>(pad_elems, 1)) {
  RINGDP_CHECK(!params_.empty(), "Reducer: no parameters");
  for (auto& p : params_) RINGDP_CHECK(p.requires_grad(), "Reducer: parameter without requires_grad");
  build(bucket_indices);
  install_hooks();
}

Reducer::~Reducer() { remove_hooks(); }

void Reducer::build(const std::vector<std::vector<int64_t>>& bucket_indices) {
  const size_t n = params_.size();
  std::vector<char> seen(n, 0);
  for (auto& b : bucket_indices)
    for (auto i : b) {
      RINGDP_CHECK(i >= 0 && static_cast<size_t>(i) < n, "bucket index out of range: ", i);
      RINGDP_CHECK(!seen[i], "parameter ", i, " assigned to two buckets");
      seen[i] = 1;
    }
  for (size_t i = 0; i < n; ++i) RINGDP_CHECK(seen[i], "parameter ", i, " not assigned to a bucket");

  // Pass 1: per-dtype offsets in bucket order, each param padded to pad_elems_ (alignment for
  // vector loads and for the single-kernel optimizer over the flat buffer).
  std::map<int, int64_t> total;
  std::vector<int64_t> offsets(n, 0);
  std::vector<std::pair<int64_t, int64_t>> bucket_range(bucket_indices.size());
  for (size_t b = 0; b < bucket_indices.size(); ++b) {
    int key = static_cast<int>(params_[bucket_indices[b][0]].scalar_type());
    int64_t start = total[key];
    for (auto i : bucket_indices[b]) {
      RINGDP_CHECK(static_cast<int>(params_[i].scalar_type()) == key,
                   "a bucket must hold a single dtype");
      offsets[i] = total[key];
      int64_t ne = params_[i].numel();
      total[key] += (ne + pad_elems_ - 1) / pad_elems_ * pad_elems_;
    }
    bucket_range[b] = {start, total[key] - start};
  }

  // Keep any existing gradient values across a rebuild.
  std::vector<at::Tensor> old_grads(n);
  for (size_t i = 0; i < n; ++i) old_grads[i] = params_[i].grad();

  flat_by_dtype_.clear();
  for (auto& kv : total) {
    const at::Tensor* proto = nullptr;
    for (auto& p : params_)
      if (static_cast<int>(p.scalar_type()) == kv.first) {
        proto = &p;
        break;
      }
    flat_by_dtype_[kv.first] = at::zeros({kv.second}, proto->options().requires_grad(false));
  }

  buckets_.clear();
  buckets_.resize(bucket_indices.size());
  param_bucket_.assign(n, -1);
  views_.assign(n, at::Tensor());
  for (size_t b = 0; b < bucket_indices.size(); ++b) {
    auto& bk = buckets_[b];
    bk.params = bucket_indices[b];
    int key = static_cast<int>(params_[bk.params[0]].scalar_type());
    at::Tensor& flat = flat_by_dtype_[key];
    bk.flat = flat.narrow(0, bucket_range[b].first, bucket_range[b].second);
    bk.st.numel = bk.flat.numel();
    bk.st.bytes = bk.flat.nbytes();
    for (auto i : bk.params) {
      param_bucket_[i] = static_cast<int64_t>(b);
      views_[i] = flat.narrow(0, offsets[i], params_[i].numel()).view(params_[i].sizes());
    }
  }
  offsets_ = offsets;
  bucket_indices_ = bucket_indices;
  ready_.assign(n, 0);

  // Re-point every parameter's .grad at its slot (grad-as-bucket-view).
  at::NoGradGuard ng;
  for (size_t i = 0; i < n; ++i) {
    if (old_grads[i].defined()) {
      views_[i].copy_(old_grads[i]);
      params_[i].mutable_grad() = views_[i];
    }
  }
}

namespace {

// Calls the reducer after the parameter's gradient has been accumulated; chains any hook that was
// installed before (e.g. a user's register_post_accumulate_grad_hook).
class ReducerAccHook : public torch::autograd::PostAccumulateGradHook {
 public:
  ReducerAccHook(Reducer* r, int64_t index,
                 std::unique_ptr<torch::autograd::PostAccumulateGradHook> prev)
      : reducer_(r), index_(index), prev_(std::move(prev)) {}
  void operator()(const torch::autograd::Variable& tensor) override {
    if (prev_) (*prev_)(tensor);
    reducer_->autograd_hook(index_);
  }
  std::unique_ptr<torch::autograd::PostAccumulateGradHook> take_prev() { return std::move(prev_); }
  const Reducer* owner() const { return reducer_; }

 private:
  Reducer* reducer_;
  int64_t index_;
  std::unique_ptr<torch::autograd::PostAccumulateGradHook> prev_;
};

}  // namespace

void Reducer::install_hooks() {
  hooked_.assign(params_.size(), false);
  for (size_t i = 0; i < params_.size(); ++i) {
    RINGDP_CHECK(params_[i].is_leaf(), "Reducer: parameter ", i, " is not a leaf tensor");
    auto& slot = torch::autograd::impl::post_acc_grad_hooks(params_[i]);
    std::unique_ptr<torch::autograd::PostAccumulateGradHook> prev = std::move(slot);
    torch::autograd::impl::set_post_acc_grad_hooks(
        params_[i], std::make_unique<ReducerAccHook>(this, static_cast<int64_t>(i), std::move(prev)));
    hooked_[i] = true;
  }
}

void Reducer::remove_hooks() {
  for (size_t i = 0; i < hooked_.size(); ++i) {
    if (!hooked_[i]) continue;
    auto& slot = torch::autograd::impl::post_acc_grad_hooks(params_[i]);
    auto* mine = dynamic_cast<ReducerAccHook*>(slot.get());
    if (mine && mine->owner() == this) {
      auto prev = mine->take_prev();
      slot = std::move(prev);
    }
    hooked_[i] = false;
  }
}

std::vector<at::Tensor> Reducer::flat_buffers() const {
  std::vector<at::Tensor> out;
  for (auto& kv : flat_by_dtype_) out.push_back(kv.second);
  return out;
}

std::vector<int64_t> Reducer::bucket_numels() const {
  std::vector<int64_t> out;
  for (auto& b : buckets_) out.push_back(b.flat.numel());
  return out;
}

std::vector<BucketStats> Reducer::stats() const {
  std::vector<BucketStats> out;
  for (auto& b : buckets_) out.push_back(b.st);
  return out;
}

std::vector<double> Reducer::collect_comm_times() {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<double> out;
  for (auto& b : buckets_) {
    double d = b.work ? b.work->duration_us() : -1.0;
    if (d >= 0 && b.st.last_comm_us != d) {
      b.st.last_comm_us = d;
      b.st.total_comm_us += d;
      b.st.comm_samples += 1;
    }
    out.push_back(d);
  }
  return out;
}

void Reducer::rebuild_buckets(std::vector<std::vector<int64_t>> new_indices) {
  std::lock_guard<std::mutex> lk(mu_);
  RINGDP_CHECK(!expect_hooks_, "cannot rebuild buckets during backward");
  build(new_indices);
  rebuilt_ = true;
  record_order_ = false;
}

// ------------------------------------------------------------------ per-iteration protocol
void Reducer::prepare_for_forward() {}

void Reducer::prepare_for_backward() {
  std::lock_guard<std::mutex> lk(mu_);
  expect_hooks_ = true;
  finalize_queued_ = false;
  next_bucket_ = 0;
  std::fill(ready_.begin(), ready_.end(), 0);
  for (auto& b : buckets_) {
    b.pending = static_cast<int64_t>(b.params.size());
    b.launched = false;
    b.work.reset();
  }
  if (record_order_) ready_order_.clear();
  backward_start_us_ = 0;
}

void Reducer::set_require_sync(bool v) {
  std::lock_guard<std::mutex> lk(mu_);
  require_sync_ = v;
}

void Reducer::autograd_hook(int64_t index) {
  std::lock_guard<std::mutex> lk(mu_);
  if (!expect_hooks_) return;
  if (backward_start_us_ == 0) backward_start_us_ = now_us();
  if (!finalize_queued_) {
    finalize_queued_ = true;
    torch::autograd::Engine::get_default_engine().queue_callback([this] { finalize_backward(); });
  }
  if (record_order_ && require_sync_) ready_order_.push_back(index);
  if (!require_sync_) return;  // no_sync(): gradients accumulate locally in their slots

  RINGDP_CHECK(!ready_[index],
               "Expected to mark a variable ready only once. Parameter index ", index,
               " was marked ready twice in one backward pass (reentrant backward, or a module "
               "reused in a way DDP cannot reduce).");
  ready_[index] = 1;
  at::Tensor& grad = params_[index].mutable_grad();
  at::Tensor& view = views_[index];
  if (grad.defined()) {
    const bool aliased = grad.data_ptr() == view.data_ptr() && grad.sizes() == view.sizes() &&
                         grad.strides() == view.strides();
    if (!aliased) {
      at::NoGradGuard ng;
      view.copy_(grad);
      grad = view;
    }
  } else {
    view.zero_();
    grad = view;
  }
  auto& b = buckets_[param_bucket_[index]];
  if (--b.pending == 0) {
    b.st.last_ready_us = static_cast<double>(now_us() - backward_start_us_);
    launch_ready_buckets();
  }
}

void Reducer::launch_ready_buckets() {
  while (next_bucket_ < static_cast<int64_t>(buckets_.size()) &&
         buckets_[next_bucket_].pending == 0) {
    launch_bucket(buckets_[next_bucket_], next_bucket_);
    ++next_bucket_;
  }
}

namespace {
// RINGDP_DDP_FORCE_COMM=1: issue the bucket collectives even on a one-rank group, so a single-GPU
// run exercises the whole communication path (side stream, events, RCCL inside a hipGraph).
bool force_comm() {
  const char* e = std::getenv("RINGDP_DDP_FORCE_COMM");  // read per bucket: tests toggle it
  return e != nullptr && e[0] != '\0' && e[0] != '0';
}
}  // namespace

void Reducer::launch_bucket(Bucket& b, int64_t index) {
  b.launched = true;
  if (trace::enabled()) {
    const std::string tag = "ringdp.bucket" + std::to_string(index) + ".launch";
    trace::mark(tag.c_str());
  }
  b.st.last_launch_us = static_cast<double>(now_us() - backward_start_us_);
  if ((pg_->size() == 1 && !force_comm()) || hook_ == CommHook::NONE) {
    b.work.reset();
    return;
  }
  const bool compress = hook_ == CommHook::BF16_COMPRESS || hook_ == CommHook::FP16_COMPRESS;
  if (split_ && (hook_ == CommHook::ALLREDUCE || compress)) {  // segmented capture
    split_this_iter_ = true;
    if (compress) {  // the wire copy rides in the segment that produced the gradients
      auto dt = hook_ == CommHook::BF16_COMPRESS ? at::kBFloat16 : at::kHalf;
      if (!b.wire.defined() || b.wire.numel() != b.flat.numel() || b.wire.scalar_type() != dt)
        b.wire = at::empty({b.flat.numel()}, b.flat.options().dtype(dt));
      ops::cast_copy(b.wire, b.flat);
    }
    if (split_(index)) {  // the replay issues the collective between segments
      b.work.reset();
      b.split_wire = compress;
      return;
    }
    std::vector<at::Tensor> v{compress ? b.wire : b.flat};  // inline: captured on the compute stream
    pg_->set_caller_stream_ops(true);
    try {
      b.work = pg_->allreduce(v, ReduceOp::AVG);
    } catch (...) {
      pg_->set_caller_stream_ops(false);
      throw;
    }
    pg_->set_caller_stream_ops(false);
    return;
  }
  switch (hook_) {
    case CommHook::ALLREDUCE: {
      std::vector<at::Tensor> v{b.flat};
      b.work = pg_->allreduce(v, ReduceOp::AVG);
      break;
    }
    case CommHook::BF16_COMPRESS:
    case CommHook::FP16_COMPRESS: {
      auto dt = hook_ == CommHook::BF16_COMPRESS ? at::kBFloat16 : at::kHalf;
      if (!b.wire.defined() || b.wire.numel() != b.flat.numel() || b.wire.scalar_type() != dt)
        b.wire = at::empty({b.flat.numel()}, b.flat.options().dtype(dt));
      ops::cast_copy(b.wire, b.flat);
      std::vector<at::Tensor> v{b.wire};
      b.work = pg_->allreduce(v, ReduceOp::AVG);
      break;
    }
    case CommHook::PYTHON: {
      RINGDP_CHECK(py_hook_, "python comm hook not set");
      b.work = py_hook_(index, b.flat);
      break;
    }
    case CommHook::NONE:
      break;
  }
}

void Reducer::finalize_backward() {
  std::lock_guard<std::mutex> lk(mu_);
  if (!expect_hooks_) return;
  expect_hooks_ = false;
  if (!require_sync_) {
    ++iteration_;
    return;
  }
  // Parameters that produced no gradient this iteration.
  std::vector<int64_t> missing;
  for (size_t i = 0; i < params_.size(); ++i)
    if (!ready_[i]) missing.push_back(static_cast<int64_t>(i));
  if (!missing.empty()) {
    if (!find_unused_) {
      std::string s;
      for (size_t k = 0; k < missing.size() && k < 32; ++k) s += std::to_string(missing[k]) + " ";
      // Put the reducer into a consistent state before raising.
      throw RingdpError(strcat_all(
          "[ringdp] DistributedDataParallel: parameters with indices [", s,
          "] did not receive gradients in this backward pass. Pass find_unused_parameters=True "
          "to DistributedDataParallel if some parameters are legitimately unused."));
    }
    at::NoGradGuard ng;
    for (auto i : missing) {
      ready_[i] = 1;
      at::Tensor& grad = params_[i].mutable_grad();
      if (grad.defined() && grad.data_ptr() != views_[i].data_ptr()) views_[i].copy_(grad);
      else if (!grad.defined()) views_[i].zero_();
      grad = views_[i];
      auto& b = buckets_[param_bucket_[i]];
      --b.pending;
    }
    launch_ready_buckets();
  }
  RINGDP_CHECK(next_bucket_ == static_cast<int64_t>(buckets_.size()),
               "reducer: not all buckets were launched");
  for (auto& b : buckets_) {
    if (b.work) {
      b.work->wait(false);
      double d = b.work->duration_us();
      if (d >= 0) {
        b.st.last_comm_us = d;
        b.st.total_comm_us += d;
        b.st.comm_samples += 1;
      }
      if (hook_ == CommHook::BF16_COMPRESS || hook_ == CommHook::FP16_COMPRESS) {
        ops::cast_copy(b.flat, b.wire);
      } else if (hook_ == CommHook::PYTHON) {
        auto& res = b.work->result();
        if (!res.empty() && res[0].defined() && res[0].data_ptr() != b.flat.data_ptr())
          b.flat.copy_(res[0].view({-1}));
      }
    }
  }
  if (split_this_iter_) {  // segmented capture: the join point before the optimizer
    split_this_iter_ = false;
    split_(-1);
    // compressed buckets whose collective runs between segments: decompress after the join
    for (auto& b : buckets_) {
      if (b.split_wire) {
        ops::cast_copy(b.flat, b.wire);
        b.split_wire = false;
      }
    }
  }
  ++iteration_;
}

std::shared_ptr<Work> Reducer::launch_collective(int64_t index) {
  RINGDP_CHECK(index >= 0 && index < static_cast<int64_t>(buckets_.size()), "reducer: bad bucket index ", index);
  const Bucket& b = buckets_[index];
  const bool compress = hook_ == CommHook::BF16_COMPRESS || hook_ == CommHook::FP16_COMPRESS;
  RINGDP_CHECK(!compress || b.wire.defined(), "reducer: bucket ", index, " has no wire buffer");
  std::vector<at::Tensor> v{compress ? b.wire : b.flat};
  return pg_->allreduce(v, ReduceOp::AVG);
}

}  // namespace ringdp
