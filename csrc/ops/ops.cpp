// Tensor-level wrappers around ringdp's HIP kernels.
#include "ops.h"

#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>

#include <atomic>
#include <cstring>
#include <map>
#include <mutex>

#include "../common.h"
#include "../kernels/kernels.h"

namespace ringdp {
namespace ops {

namespace {

hipStream_t cur_stream(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.get_device()).stream();
}

void check_cuda(const at::Tensor& t, const char* name) {
  RINGDP_CHECK(t.defined(), name, ": undefined tensor");
  RINGDP_CHECK(t.is_cuda(), name, ": expected a GPU tensor (ringdp HIP kernel), got ", t.device());
  RINGDP_CHECK(t.is_contiguous(), name, ": expected a contiguous tensor");
}

void check_dtype(const at::Tensor& t, at::ScalarType d, const char* name) {
  RINGDP_CHECK(t.scalar_type() == d, name, ": expected dtype ", c10::toString(d), ", got ",
               c10::toString(t.scalar_type()));
}

void check_shape(const at::Tensor& t, at::IntArrayRef s, const char* name) {
  RINGDP_CHECK(t.sizes() == s, name, ": expected shape ", s, ", got ", t.sizes());
}

// Persistent, zero-initialised arrival counters for last-arriver reductions.  Each call takes
// the next slot; the kernel's last workgroup resets its slot to 0, so no per-call memset launch
// is needed (and the slot index is stable under hipGraph capture).
unsigned* next_counter(const at::Tensor& like) {
  constexpr int kSlots = 4096;
  static std::mutex mu;
  static std::map<int, std::pair<at::Tensor, int>> pools;
  std::lock_guard<std::mutex> lk(mu);
  auto& e = pools[like.get_device()];
  if (!e.first.defined()) {
    e.first = at::zeros({kSlots}, like.options().dtype(at::kInt));
    e.second = 0;
  }
  unsigned* p = reinterpret_cast<unsigned*>(e.first.data_ptr<int>()) + e.second;
  e.second = (e.second + 16) % kSlots;  // 64-byte spacing between live counters
  return p;
}

bool aligned16(const at::Tensor& t) {
  return (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0;
}

kern::SgdArgs make_args(const SgdHyper& h, bool first, const c10::optional<at::Tensor>& lr_t,
                        const c10::optional<at::Tensor>& scale_t) {
  kern::SgdArgs a{};
  a.lr = static_cast<float>(h.lr);
  a.momentum = static_cast<float>(h.momentum);
  a.dampening = static_cast<float>(h.dampening);
  a.weight_decay = static_cast<float>(h.weight_decay);
  a.nesterov = h.nesterov;
  a.maximize = h.maximize;
  a.first_step = first;
  a.lr_ptr = nullptr;
  a.grad_scale_ptr = nullptr;
  if (lr_t && lr_t->defined()) {
    check_cuda(*lr_t, "lr tensor");
    check_dtype(*lr_t, at::kFloat, "lr tensor");
    a.lr_ptr = lr_t->data_ptr<float>();
  }
  if (scale_t && scale_t->defined()) {
    check_cuda(*scale_t, "grad_scale tensor");
    check_dtype(*scale_t, at::kFloat, "grad_scale tensor");
    a.grad_scale_ptr = scale_t->data_ptr<float>();
  }
  return a;
}

}  // namespace

// ------------------------------------------------------------------ casts
std::vector<at::Tensor> cast_bf16_multi(const std::vector<at::Tensor>& srcs) {
  std::vector<at::Tensor> out;
  kern::CastTable t{};
  for (const at::Tensor& x : srcs) {
    check_cuda(x, "cast_bf16_multi src");
    RINGDP_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous(), "cast_bf16_multi: contiguous fp32 tensors");
    RINGDP_CHECK(x.numel() % 4 == 0, "cast_bf16_multi: sizes must be multiples of 4");
    at::Tensor y = at::empty(x.sizes(), x.options().dtype(at::kBFloat16));
    out.push_back(y);
    if (t.n == kern::kCastMax) {
      kern::cast_f32_to_bf16_multi(t, cur_stream(x));
      t = kern::CastTable{};
    }
    kern::CastEntry& e = t.e[t.n++];
    e.src = x.data_ptr<float>();
    e.dst = y.data_ptr();
    e.start4 = t.total4;
    t.total4 += x.numel() / 4;
  }
  if (t.n > 0) kern::cast_f32_to_bf16_multi(t, cur_stream(srcs[0]));
  return out;
}

std::vector<at::Tensor> cast_bf16_t_multi(const std::vector<at::Tensor>& srcs) {
  std::vector<at::Tensor> out;
  kern::CastTTable t{};
  for (const at::Tensor& x : srcs) {
    check_cuda(x, "cast_bf16_t_multi src");
    RINGDP_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 2,
                 "cast_bf16_t_multi: contiguous fp32 matrices");
    const int64_t R = x.size(0), Cc = x.size(1);
    at::Tensor y = at::empty({R, Cc}, x.options().dtype(at::kBFloat16));
    at::Tensor yt = at::empty({Cc, R}, x.options().dtype(at::kBFloat16));
    out.push_back(y);
    out.push_back(yt);
    if (t.n == kern::kCastTMax) {
      kern::cast_t_multi(t, cur_stream(x));
      t = kern::CastTTable{};
    }
    kern::CastTEntry& e = t.e[t.n++];
    e.src = x.data_ptr<float>();
    e.dst = y.data_ptr();
    e.dst_t = yt.data_ptr();
    e.R = (int)R;
    e.C = (int)Cc;
    e.start_tile = t.total_tiles;
    t.total_tiles += (int)(((R + 63) / 64) * ((Cc + 63) / 64));
  }
  if (t.n > 0) kern::cast_t_multi(t, cur_stream(srcs[0]));
  return out;
}

void cast_copy(at::Tensor dst, const at::Tensor& src) {
  RINGDP_CHECK(dst.numel() == src.numel(), "cast_copy: numel mismatch");
  if (!dst.is_cuda()) {
    dst.copy_(src.view(dst.sizes()));
    return;
  }
  check_cuda(dst, "cast_copy dst");
  check_cuda(src, "cast_copy src");
  const int64_t n = src.numel();
  hipStream_t s = cur_stream(dst);
  auto sd = src.scalar_type(), dd = dst.scalar_type();
  const bool vec = aligned16(src) && aligned16(dst);
  if (sd == at::kFloat && dd == at::kBFloat16 && vec) {
    kern::cast_f32_to_bf16(src.data_ptr<float>(), dst.data_ptr(), n, s);
  } else if (sd == at::kBFloat16 && dd == at::kFloat && vec) {
    kern::cast_bf16_to_f32(src.data_ptr(), dst.data_ptr<float>(), n, s);
  } else if (sd == at::kFloat && dd == at::kHalf) {
    kern::cast_f32_to_f16(src.data_ptr<float>(), dst.data_ptr(), n, s);
  } else if (sd == at::kHalf && dd == at::kFloat) {
    kern::cast_f16_to_f32(src.data_ptr(), dst.data_ptr<float>(), n, s);
  } else if (sd == dd) {
    dst.copy_(src.view(dst.sizes()));
  } else {
    RINGDP_CHECK(false, "cast_copy: unsupported conversion ", c10::toString(sd), " -> ",
                 c10::toString(dd), vec ? "" : " (unaligned)");
  }
}

// ------------------------------------------------------------------ SGD
void sgd_flat(at::Tensor param, const at::Tensor& grad, const c10::optional<at::Tensor>& buf_opt, const SgdHyper& h,
              bool first_step, const c10::optional<at::Tensor>& lr_t,
              const c10::optional<at::Tensor>& scale_t, const c10::optional<at::Tensor>& packed,
              const std::vector<int64_t>& pack_offsets) {
  check_cuda(param, "sgd param");
  check_cuda(grad, "sgd grad");
  check_dtype(param, at::kFloat, "sgd param");
  check_dtype(grad, at::kFloat, "sgd grad");
  RINGDP_CHECK(param.numel() == grad.numel(), "sgd_flat: param/grad numel mismatch");
  float* m = nullptr;
  at::Tensor buf = buf_opt.has_value() ? *buf_opt : at::Tensor();
  if (h.momentum != 0.0) {
    check_cuda(buf, "sgd momentum buffer");
    RINGDP_CHECK(buf.numel() == param.numel(), "sgd_flat: momentum buffer numel mismatch");
    m = buf.data_ptr<float>();
  }
  RINGDP_CHECK(aligned16(param) && aligned16(grad) && (!m || aligned16(buf)),
               "sgd_flat: buffers must be 16-byte aligned");
  if (packed.has_value() && packed->defined()) {
    // the ConvNet's packed bf16 fragments, written as the weights are updated
    check_cuda(*packed, "packed convnet weights");
    check_dtype(*packed, at::kBFloat16, "packed convnet weights");
    RINGDP_CHECK(packed->numel() == kern::cn_packed_elems(), "packed convnet weights: wrong size");
    RINGDP_CHECK(pack_offsets.size() == 4, "sgd_flat: pack_offsets needs the 4 ConvNet weight offsets");
    const int64_t lens[4] = {32 * 25, 64 * 32 * 9, 128 * 64 * 9, 10 * 2048};
    for (int i = 0; i < 4; ++i)
      RINGDP_CHECK(pack_offsets[i] >= 0 && pack_offsets[i] + lens[i] <= param.numel(),
                   "sgd_flat: pack offset ", i, " outside the flat parameter range");
    kern::cn_sgd_flat_pack(param.data_ptr<float>(), grad.data_ptr<float>(), m, param.numel(),
                           make_args(h, first_step, lr_t, scale_t), pack_offsets.data(), packed->data_ptr(),
                           cur_stream(param));
    return;
  }
  kern::sgd_flat(param.data_ptr<float>(), grad.data_ptr<float>(), m, param.numel(),
                 make_args(h, first_step, lr_t, scale_t), cur_stream(param));
}

namespace {
constexpr int64_t kSgdChunk = 65536;
}

std::tuple<at::Tensor, int64_t, int64_t> sgd_multi_build(std::vector<at::Tensor> params,
                                                         std::vector<at::Tensor> grads,
                                                         std::vector<at::Tensor> bufs,
                                                         bool mom) {
  RINGDP_CHECK(params.size() == grads.size() && !params.empty(), "sgd_multi: bad tensor lists");
  if (mom) RINGDP_CHECK(bufs.size() == params.size(), "sgd_multi: need one buffer per param");
  std::vector<kern::SgdTensor> table(params.size());
  std::vector<int64_t> chunks;
  for (size_t i = 0; i < params.size(); ++i) {
    check_cuda(params[i], "sgd param");
    check_cuda(grads[i], "sgd grad");
    check_dtype(params[i], at::kFloat, "sgd param");
    check_dtype(grads[i], at::kFloat, "sgd grad");
    RINGDP_CHECK(params[i].numel() == grads[i].numel(), "sgd_multi: numel mismatch at ", i);
    if (mom) check_cuda(bufs[i], "sgd momentum buffer");
    table[i] = {params[i].data_ptr<float>(), grads[i].data_ptr<float>(),
                mom ? bufs[i].data_ptr<float>() : nullptr, params[i].numel()};
    for (int64_t s = 0; s < params[i].numel(); s += kSgdChunk) {
      chunks.push_back(static_cast<int64_t>(i));
      chunks.push_back(s);
    }
  }
  const int64_t tbytes = static_cast<int64_t>(table.size() * sizeof(kern::SgdTensor));
  const int64_t cbytes = static_cast<int64_t>(chunks.size() * sizeof(int64_t));
  at::Tensor host = at::empty({tbytes + cbytes}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(host.data_ptr(), table.data(), tbytes);
  std::memcpy(static_cast<char*>(host.data_ptr()) + tbytes, chunks.data(), cbytes);
  at::Tensor dev = host.to(params[0].device());  // synchronous: safe to cache and reuse
  return {dev, static_cast<int64_t>(chunks.size() / 2), tbytes};
}

void sgd_multi_run(const at::Tensor& dev, int64_t nchunks, int64_t tbytes, const SgdHyper& h,
                   bool first_step, const c10::optional<at::Tensor>& lr_t,
                   const c10::optional<at::Tensor>& scale_t) {
  check_cuda(dev, "sgd table");
  auto* dtable = reinterpret_cast<const kern::SgdTensor*>(dev.data_ptr());
  auto* dchunks = reinterpret_cast<const int64_t*>(static_cast<char*>(dev.data_ptr()) + tbytes);
  kern::sgd_multi(dtable, dchunks, nchunks, kSgdChunk, make_args(h, first_step, lr_t, scale_t),
                  cur_stream(dev));
}

void sgd_multi(std::vector<at::Tensor> params, std::vector<at::Tensor> grads,
               std::vector<at::Tensor> bufs, const SgdHyper& h, bool first_step,
               const c10::optional<at::Tensor>& lr_t, const c10::optional<at::Tensor>& scale_t) {
  if (params.empty()) return;
  auto t = sgd_multi_build(params, grads, bufs, h.momentum != 0.0);
  sgd_multi_run(std::get<0>(t), std::get<1>(t), std::get<2>(t), h, first_step, lr_t, scale_t);
}

// ------------------------------------------------------------------ cross entropy
std::tuple<at::Tensor, at::Tensor, at::Tensor> cross_entropy_fwd(const at::Tensor& logits,
                                                                 const at::Tensor& labels,
                                                                 int64_t ignore_index,
                                                                 double smoothing,
                                                                 int64_t reduction) {
  check_cuda(logits, "cross_entropy logits");
  check_cuda(labels, "cross_entropy labels");
  check_dtype(logits, at::kFloat, "cross_entropy logits");
  check_dtype(labels, at::kLong, "cross_entropy labels");
  RINGDP_CHECK(logits.dim() == 2 && labels.dim() == 1 && labels.size(0) == logits.size(0),
               "cross_entropy: expected logits [B, C] and labels [B]");
  RINGDP_CHECK(logits.is_contiguous() && labels.is_contiguous(), "cross_entropy: inputs must be contiguous");
  const int B = static_cast<int>(logits.size(0)), C = static_cast<int>(logits.size(1));
  const int nparts = kern::cross_entropy_parts(static_cast<int>(B), static_cast<int>(C));
  auto fo = logits.options();
  at::Tensor lse = at::empty({B}, fo);
  at::Tensor loss = reduction == 0 ? at::empty({B}, fo) : at::empty({}, fo);
  // ws: [2*nparts partials][denom][3 pad]
  at::Tensor ws = at::empty({2 * nparts + 4}, fo);
  unsigned* counter = next_counter(logits);
  kern::cross_entropy_fwd(logits.data_ptr<float>(), labels.data_ptr<int64_t>(), B, C,
                          static_cast<int>(ignore_index), static_cast<float>(smoothing),
                          static_cast<int>(reduction), lse.data_ptr<float>(),
                          loss.data_ptr<float>(), ws.data_ptr<float>(), counter, nparts,
                          cur_stream(logits));
  return {loss, lse, ws};
}

at::Tensor cross_entropy_bwd(const at::Tensor& logits, const at::Tensor& labels,
                             const at::Tensor& lse, const at::Tensor& ws,
                             const at::Tensor& grad_out, int64_t ignore_index, double smoothing,
                             int64_t reduction) {
  check_cuda(grad_out, "cross_entropy grad_out");
  at::Tensor g = grad_out.to(at::kFloat).contiguous();
  const int B = static_cast<int>(logits.size(0)), C = static_cast<int>(logits.size(1));
  const int nparts = static_cast<int>((ws.numel() - 4) / 2);
  at::Tensor d = at::empty_like(logits);
  kern::cross_entropy_bwd(logits.data_ptr<float>(), labels.data_ptr<int64_t>(),
                          lse.data_ptr<float>(), g.data_ptr<float>(),
                          ws.data_ptr<float>() + 2 * nparts, B, C, static_cast<int>(ignore_index),
                          static_cast<float>(smoothing), static_cast<int>(reduction),
                          d.data_ptr<float>(), cur_stream(logits));
  return d;
}

// ------------------------------------------------------------------ ConvNet
namespace {
void check_input(const at::Tensor& x, int64_t& B, bool& u8) {
  check_cuda(x, "convnet input");
  RINGDP_CHECK(x.dim() == 4 && x.size(1) == 1 && x.size(2) == 28 && x.size(3) == 28,
               "convnet input: expected [B, 1, 28, 28], got ", x.sizes());
  RINGDP_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kByte,
               "convnet input: expected float32 or uint8");
  B = x.size(0);
  u8 = x.scalar_type() == at::kByte;
}
}  // namespace

void check_f32_out(const at::Tensor& t, at::IntArrayRef shape, const char* name) {
  check_cuda(t, name);
  check_dtype(t, at::kFloat, name);
  check_shape(t, shape, name);
  RINGDP_CHECK(t.is_contiguous(), name, ": must be contiguous");
}

void check_act(const at::Tensor& t, at::IntArrayRef shape, at::ScalarType d, const char* name) {
  check_cuda(t, name);
  check_dtype(t, d, name);
  check_shape(t, shape, name);
  RINGDP_CHECK(t.is_contiguous(), name, ": must be contiguous");
}

void check_packed(const at::Tensor& p) {
  check_act(p, {kern::cn_packed_elems()}, at::kBFloat16, "packed convnet weights");
}

at::Tensor cn_pack_weights(const at::Tensor& w1, const at::Tensor& w2, const at::Tensor& w3,
                           const at::Tensor& wfc, const c10::optional<at::Tensor>& out_opt) {
  check_f32_out(w1, {32, 1, 5, 5}, "conv1 weight");
  check_f32_out(w2, {64, 32, 3, 3}, "conv2 weight");
  check_f32_out(w3, {128, 64, 3, 3}, "conv3 weight");
  check_f32_out(wfc, {10, 2048}, "fc1 weight");
  at::Tensor out;
  if (out_opt.has_value() && out_opt->defined()) {  // repack in place (a captured step reads this buffer)
    out = *out_opt;
    check_packed(out);
    RINGDP_CHECK(out.device() == w1.device(), "cn_pack_weights: out on another device");
  } else {
    out = at::empty({kern::cn_packed_elems()}, w1.options().dtype(at::kBFloat16));
  }
  kern::cn_pack_weights(w1.data_ptr<float>(), w2.data_ptr<float>(), w3.data_ptr<float>(),
                        wfc.data_ptr<float>(), out.data_ptr(), cur_stream(w1));
  return out;
}

std::tuple<at::Tensor, at::Tensor> cn_conv1_fwd(const at::Tensor& x, const at::Tensor& packed,
                                                const at::Tensor& b1, double mean, double std,
                                                double in_scale) {
  int64_t B;
  bool u8;
  check_input(x, B, u8);
  RINGDP_CHECK(x.is_contiguous(), "convnet input must be contiguous");
  check_packed(packed);
  check_f32_out(b1, {32}, "conv1 bias");
  auto opt = x.options();
  at::Tensor a1 = at::empty({B, 13, 13, 32}, opt.dtype(at::kBFloat16));
  // pool1 codes in window rows per channel pair [B][py][co/2][px (13 + 3 zero)][co&1] (see convnet.hip F1)
  at::Tensor idx = at::empty({B, 13, 16, 16}, opt.dtype(at::kByte));
  if (B == 0) return {a1, idx};
  kern::cn_conv1_fwd(x.data_ptr(), u8, packed.data_ptr(), b1.data_ptr<float>(), a1.data_ptr(),
                     idx.data_ptr<uint8_t>(), static_cast<int>(B), static_cast<float>(mean),
                     static_cast<float>(1.0 / std), static_cast<float>(in_scale), cur_stream(x));
  return {a1, idx};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> cn_conv1_fwd_pack(const at::Tensor& x, const at::Tensor& w1,
                                                                 const at::Tensor& w2, const at::Tensor& w3,
                                                                 const at::Tensor& wfc, const at::Tensor& b1,
                                                                 double mean, double std, double in_scale) {
  int64_t B;
  bool u8;
  check_input(x, B, u8);
  RINGDP_CHECK(x.is_contiguous(), "convnet input must be contiguous");
  check_f32_out(w1, {32, 1, 5, 5}, "conv1 weight");
  check_f32_out(w2, {64, 32, 3, 3}, "conv2 weight");
  check_f32_out(w3, {128, 64, 3, 3}, "conv3 weight");
  check_f32_out(wfc, {10, 2048}, "fc1 weight");
  check_f32_out(b1, {32}, "conv1 bias");
  auto opt = x.options();
  at::Tensor packed = at::empty({kern::cn_packed_elems()}, w1.options().dtype(at::kBFloat16));
  at::Tensor a1 = at::empty({B, 13, 13, 32}, opt.dtype(at::kBFloat16));
  at::Tensor idx = at::empty({B, 13, 16, 16}, opt.dtype(at::kByte));
  const float* pw[4] = {w1.data_ptr<float>(), w2.data_ptr<float>(), w3.data_ptr<float>(), wfc.data_ptr<float>()};
  if (B == 0) {
    kern::cn_pack_weights(pw[0], pw[1], pw[2], pw[3], packed.data_ptr(), cur_stream(w1));
    return {a1, idx, packed};
  }
  kern::cn_conv1_fwd(x.data_ptr(), u8, nullptr, b1.data_ptr<float>(), a1.data_ptr(), idx.data_ptr<uint8_t>(),
                     static_cast<int>(B), static_cast<float>(mean), static_cast<float>(1.0 / std),
                     static_cast<float>(in_scale), cur_stream(x), pw, packed.data_ptr());
  return {a1, idx, packed};
}

std::vector<at::Tensor> cn_forward_buffers(const at::Tensor& x) {
  int64_t B;
  bool u8;
  check_input(x, B, u8);
  auto bf = x.options().dtype(at::kBFloat16), u = x.options().dtype(at::kByte);
  return {at::empty({B, 13, 13, 32}, bf), at::empty({B, 13, 16, 16}, u), at::empty({B, 10, 10, 64}, bf),
          at::empty({B, 10, 10, 64}, u), at::empty({kern::cn_packed_elems()}, bf)};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> cn_forward_fused(
    const at::Tensor& x, const at::Tensor& w1, const at::Tensor& b1, const at::Tensor& w2, const at::Tensor& b2,
    const at::Tensor& w3, const at::Tensor& b3, const at::Tensor& wfc, const at::Tensor& bfc, double mean, double std,
    double in_scale, at::Tensor a1, at::Tensor idx1, at::Tensor a2, at::Tensor idx2, at::Tensor packed,
    bool do_pack) {
  int64_t B;
  bool u8;
  check_input(x, B, u8);
  RINGDP_CHECK(x.is_contiguous(), "convnet input must be contiguous");
  check_f32_out(w1, {32, 1, 5, 5}, "conv1 weight");
  check_f32_out(w2, {64, 32, 3, 3}, "conv2 weight");
  check_f32_out(w3, {128, 64, 3, 3}, "conv3 weight");
  check_f32_out(wfc, {10, 2048}, "fc1 weight");
  check_f32_out(b1, {32}, "conv1 bias");
  check_f32_out(b2, {64}, "conv2 bias");
  check_f32_out(b3, {128}, "conv3 bias");
  check_f32_out(bfc, {10}, "fc1 bias");
  check_act(a1, {B, 13, 13, 32}, at::kBFloat16, "a1 buffer");
  check_act(idx1, {B, 13, 16, 16}, at::kByte, "conv1 code buffer");
  check_act(a2, {B, 10, 10, 64}, at::kBFloat16, "a2 buffer");
  check_act(idx2, {B, 10, 10, 64}, at::kByte, "pool2 code buffer");
  check_packed(packed);
  auto opt = x.options();
  at::Tensor logits = at::empty({B, 10}, opt.dtype(at::kFloat));
  at::Tensor a3 = at::empty({B, 16, 128}, opt.dtype(at::kBFloat16));
  at::Tensor idx3 = at::empty({B, 16, 128}, opt.dtype(at::kByte));
  const float* pw[4] = {w1.data_ptr<float>(), w2.data_ptr<float>(), w3.data_ptr<float>(), wfc.data_ptr<float>()};
  if (B == 0) {
    kern::cn_pack_weights(pw[0], pw[1], pw[2], pw[3], packed.data_ptr(), cur_stream(x));
    return {logits, a3, idx3};
  }
  kern::cn_forward_fused(x.data_ptr(), u8, pw, b1.data_ptr<float>(), b2.data_ptr<float>(), b3.data_ptr<float>(),
                         bfc.data_ptr<float>(), packed.data_ptr(), a1.data_ptr(), idx1.data_ptr<uint8_t>(),
                         a2.data_ptr(), idx2.data_ptr<uint8_t>(), a3.data_ptr(), idx3.data_ptr<uint8_t>(),
                         logits.data_ptr<float>(), static_cast<int>(B), static_cast<float>(mean),
                         static_cast<float>(1.0 / std), static_cast<float>(in_scale), next_counter(x),
                         cur_stream(x), do_pack);
  return {logits, a3, idx3};
}

std::tuple<at::Tensor, at::Tensor> cn_conv2_fwd(const at::Tensor& a1, const at::Tensor& packed,
                                                const at::Tensor& b2) {
  const int64_t B = a1.size(0);
  check_act(a1, {B, 13, 13, 32}, at::kBFloat16, "conv2 input");
  check_packed(packed);
  check_f32_out(b2, {64}, "conv2 bias");
  at::Tensor a2 = at::empty({B, 10, 10, 64}, a1.options());
  at::Tensor idx2 = at::empty({B, 10, 10, 64}, a1.options().dtype(at::kByte));
  if (B == 0) return {a2, idx2};
  kern::cn_conv2_fwd(a1.data_ptr(), packed.data_ptr(), b2.data_ptr<float>(), a2.data_ptr(),
                     idx2.data_ptr<uint8_t>(), static_cast<int>(B), cur_stream(a1));
  return {a2, idx2};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> cn_conv3_fc_fwd(const at::Tensor& a2,
                                                               const at::Tensor& packed,
                                                               const at::Tensor& b3,
                                                               const at::Tensor& bfc) {
  const int64_t B = a2.size(0);
  check_act(a2, {B, 10, 10, 64}, at::kBFloat16, "pooled conv2 activation a2");
  check_packed(packed);
  check_f32_out(b3, {128}, "conv3 bias");
  check_f32_out(bfc, {10}, "fc1 bias");
  at::Tensor logits = at::empty({B, 10}, a2.options().dtype(at::kFloat));
  at::Tensor a3 = at::empty({B, 16, 128}, a2.options());
  at::Tensor idx3 = at::empty({B, 16, 128}, a2.options().dtype(at::kByte));
  if (B == 0) return {logits, a3, idx3};
  kern::cn_conv3_fc_fwd(a2.data_ptr(), packed.data_ptr(), b3.data_ptr<float>(), bfc.data_ptr<float>(),
                        logits.data_ptr<float>(), a3.data_ptr(), idx3.data_ptr<uint8_t>(),
                        static_cast<int>(B), cur_stream(a2));
  return {logits, a3, idx3};
}

namespace {
// A conv3 / fc1 weight-gradient reduction held back to ride along with the next conv12 backward's
// reduction launch (one launch instead of two).  Keyed by device; `keep` holds the slab tensors
// until the launch is queued (the caching allocator is stream-ordered, so releasing them right
// after the launch is safe).
struct PendingReduce {
  kern::ReduceList segs;
  std::vector<at::Tensor> keep;
  hipStream_t stream = nullptr;
};
std::mutex g_pend_mu;
std::map<int, PendingReduce> g_pend;
std::atomic<int64_t> g_merged{0};  // deferrals folded into a conv12 reduction launch (tests)

PendingReduce take_pending(int dev) {
  std::lock_guard<std::mutex> lk(g_pend_mu);
  PendingReduce p;
  auto it = g_pend.find(dev);
  if (it != g_pend.end()) {
    p = std::move(it->second);
    g_pend.erase(it);
  }
  return p;
}

void flush_pending(int dev) {
  PendingReduce p = take_pending(dev);
  if (!p.segs.empty()) kern::cn_launch_reduce(p.segs, p.stream);
}

at::Tensor conv3_fc_bwd_impl(const at::Tensor& a2, const at::Tensor& idx2, const at::Tensor& a3,
                             const at::Tensor& idx3, const at::Tensor& wfc, const at::Tensor* dlogits,
                             const kern::CeFuse* ce, const at::Tensor& packed, bool need_dz2, at::Tensor dw3,
                             at::Tensor db3, at::Tensor dwfc, at::Tensor dbfc, bool defer) {
  const int64_t B = a2.size(0);
  check_act(a2, {B, 10, 10, 64}, at::kBFloat16, "pooled conv2 activation a2");
  check_act(idx2, {B, 10, 10, 64}, at::kByte, "pool2 codes");
  check_act(a3, {B, 16, 128}, at::kBFloat16, "pooled conv3");
  check_act(idx3, {B, 16, 128}, at::kByte, "conv3 argmax");
  check_f32_out(wfc, {10, 2048}, "fc1 weight");
  check_packed(packed);
  check_f32_out(dw3, {128, 64, 3, 3}, "conv3 dw");
  check_f32_out(db3, {128}, "conv3 db");
  check_f32_out(dwfc, {10, 2048}, "fc1 dw");
  check_f32_out(dbfc, {10}, "fc1 db");
  at::Tensor dl;
  if (dlogits) {
    check_cuda(*dlogits, "logits grad");
    dl = dlogits->to(at::kFloat).contiguous();
    check_shape(dl, {B, 10}, "logits grad");
  }
  at::Tensor dz2;
  if (need_dz2) dz2 = at::empty({B, 11, 11, 64}, a2.options());
  const int dev = a2.get_device();
  flush_pending(dev);  // a stale deferral (its conv12 backward never ran) goes out first
  if (B == 0) {
    dw3.zero_();
    db3.zero_();
    dwfc.zero_();
    dbfc.zero_();
    return dz2;
  }
  const int bi = static_cast<int>(B);
  at::Tensor da3m = at::empty({B, 16, 128}, a2.options());
  at::Tensor fs = at::empty({kern::cn_fc_slab_floats(bi, need_dz2)}, dw3.options());
  at::Tensor cs = at::empty({kern::cn_conv3_slab_floats(bi, need_dz2)}, dw3.options());
  const hipStream_t st = cur_stream(a2);
  kern::ReduceList held;
  kern::cn_conv3_fc_bwd(a2.data_ptr(), idx2.data_ptr<uint8_t>(), a3.data_ptr(), idx3.data_ptr<uint8_t>(),
                        wfc.data_ptr<float>(), dl.defined() ? dl.data_ptr<float>() : nullptr, packed.data_ptr(),
                        da3m.data_ptr(), need_dz2 ? dz2.data_ptr() : nullptr, bi, fs.data_ptr<float>(),
                        cs.data_ptr<float>(), dw3.data_ptr<float>(), db3.data_ptr<float>(), dwfc.data_ptr<float>(),
                        dbfc.data_ptr<float>(), st, ce, defer ? &held : nullptr);
  if (defer) {
    std::lock_guard<std::mutex> lk(g_pend_mu);
    PendingReduce& p = g_pend[dev];
    p.segs = std::move(held);
    p.keep = {fs, cs};
    p.stream = st;
  }
  return dz2;
}
}  // namespace

at::Tensor cn_conv3_fc_bwd(const at::Tensor& a2, const at::Tensor& idx2, const at::Tensor& a3,
                           const at::Tensor& idx3, const at::Tensor& wfc, const at::Tensor& dlogits,
                           const at::Tensor& packed, bool need_dz2, at::Tensor dw3, at::Tensor db3,
                           at::Tensor dwfc, at::Tensor dbfc, bool defer_reduce) {
  return conv3_fc_bwd_impl(a2, idx2, a3, idx3, wfc, &dlogits, nullptr, packed, need_dz2, dw3, db3, dwfc, dbfc,
                           defer_reduce);
}

at::Tensor cn_conv3_fc_ce_bwd(const at::Tensor& a2, const at::Tensor& idx2, const at::Tensor& a3,
                              const at::Tensor& idx3, const at::Tensor& wfc, const at::Tensor& logits,
                              const at::Tensor& labels, const at::Tensor& lse, const at::Tensor& ws,
                              const at::Tensor& grad_out, int64_t ignore_index, double smoothing, int64_t reduction,
                              const at::Tensor& packed, bool need_dz2, at::Tensor dw3, at::Tensor db3,
                              at::Tensor dwfc, at::Tensor dbfc, bool defer_reduce) {
  const int64_t B = a2.size(0);
  check_cuda(logits, "cross_entropy logits");
  check_dtype(logits, at::kFloat, "cross_entropy logits");
  check_shape(logits, {B, 10}, "cross_entropy logits");
  check_cuda(labels, "cross_entropy labels");
  check_dtype(labels, at::kLong, "cross_entropy labels");
  check_shape(labels, {B}, "cross_entropy labels");
  check_cuda(lse, "cross_entropy lse");
  check_cuda(grad_out, "cross_entropy grad_out");
  RINGDP_CHECK(reduction >= 0 && reduction <= 2, "cross_entropy: bad reduction ", reduction);
  at::Tensor g = grad_out.to(at::kFloat).contiguous();
  RINGDP_CHECK(g.numel() == (reduction == 0 ? B : 1), "cross_entropy grad_out: expected ",
               reduction == 0 ? B : 1, " elements, got ", g.numel());
  const int nparts = static_cast<int>((ws.numel() - 4) / 2);
  const kern::CeFuse ce{logits.data_ptr<float>(), labels.data_ptr<int64_t>(), lse.data_ptr<float>(),
                        g.data_ptr<float>(), ws.data_ptr<float>() + 2 * nparts, static_cast<int>(ignore_index),
                        static_cast<float>(smoothing), static_cast<int>(reduction)};
  return conv3_fc_bwd_impl(a2, idx2, a3, idx3, wfc, nullptr, &ce, packed, need_dz2, dw3, db3, dwfc, dbfc,
                           defer_reduce);
}

void cn_flush_reduce(int64_t device) { flush_pending(static_cast<int>(device)); }

int64_t cn_merged_reductions() { return g_merged.load(); }

bool cn_reduce_pending(int64_t device) {
  std::lock_guard<std::mutex> lk(g_pend_mu);
  auto it = g_pend.find(static_cast<int>(device));
  return it != g_pend.end() && !it->second.segs.empty();
}

at::Tensor cn_conv2_bwd(const at::Tensor& a1, const at::Tensor& dz2, const at::Tensor& packed,
                        bool need_da1, at::Tensor dw2, at::Tensor db2) {
  const int64_t B = a1.size(0);
  check_act(a1, {B, 13, 13, 32}, at::kBFloat16, "conv2 input");
  check_act(dz2, {B, 11, 11, 64}, at::kBFloat16, "conv2 output grad");
  check_packed(packed);
  check_f32_out(dw2, {64, 32, 3, 3}, "conv2 dw");
  check_f32_out(db2, {64}, "conv2 db");
  at::Tensor da1;
  if (need_da1) da1 = at::empty_like(a1);
  if (B == 0) {
    dw2.zero_();
    db2.zero_();
    return da1;
  }
  const int bi = static_cast<int>(B);
  at::Tensor slabs = at::empty({kern::cn_conv2_slab_floats(bi, need_da1)}, dw2.options());
  kern::cn_conv2_bwd(a1.data_ptr(), dz2.data_ptr(), packed.data_ptr(), need_da1 ? da1.data_ptr() : nullptr,
                     bi, slabs.data_ptr<float>(), dw2.data_ptr<float>(), db2.data_ptr<float>(),
                     cur_stream(a1));
  return da1;
}

void cn_conv12_bwd(const at::Tensor& x, const at::Tensor& idx1, const at::Tensor& a1, const at::Tensor& dz2,
                   const at::Tensor& packed, at::Tensor dw2, at::Tensor db2, at::Tensor dw1, at::Tensor db1,
                   double mean, double std, double in_scale) {
  int64_t B;
  bool u8;
  check_input(x, B, u8);
  RINGDP_CHECK(x.is_contiguous(), "convnet input must be contiguous");
  check_act(idx1, {B, 13, 16, 16}, at::kByte, "conv1 argmax");
  check_act(a1, {B, 13, 13, 32}, at::kBFloat16, "conv2 input");
  check_act(dz2, {B, 11, 11, 64}, at::kBFloat16, "conv2 output grad");
  check_packed(packed);
  check_f32_out(dw2, {64, 32, 3, 3}, "conv2 dw");
  check_f32_out(db2, {64}, "conv2 db");
  check_f32_out(dw1, {32, 1, 5, 5}, "conv1 dw");
  check_f32_out(db1, {32}, "conv1 db");
  if (B == 0) {
    dw2.zero_();
    db2.zero_();
    dw1.zero_();
    db1.zero_();
    return;
  }
  const int bi = static_cast<int>(B);
  at::Tensor slabs = at::empty({kern::cn_conv12_slab_floats(bi)}, dw2.options());
  const hipStream_t st = cur_stream(x);
  PendingReduce pend = take_pending(x.get_device());
  if (!pend.segs.empty() && pend.stream != st) {  // deferred on another stream: it goes out there
    kern::cn_launch_reduce(pend.segs, pend.stream);
    pend.segs.clear();
  }
  if (!pend.segs.empty()) ++g_merged;
  kern::cn_conv12_bwd(x.data_ptr(), u8, idx1.data_ptr<uint8_t>(), a1.data_ptr(), dz2.data_ptr(), packed.data_ptr(),
                      bi, static_cast<float>(mean), static_cast<float>(1.0 / std), static_cast<float>(in_scale),
                      slabs.data_ptr<float>(), dw2.data_ptr<float>(), db2.data_ptr<float>(), dw1.data_ptr<float>(),
                      db1.data_ptr<float>(), st, pend.segs.empty() ? nullptr : &pend.segs);
}

void cn_conv1_wgrad(const at::Tensor& x, const at::Tensor& da1, const at::Tensor& idx1, at::Tensor dw1,
                    at::Tensor db1, double mean, double std, double in_scale) {
  int64_t B;
  bool u8;
  check_input(x, B, u8);
  RINGDP_CHECK(x.is_contiguous(), "convnet input must be contiguous");
  check_act(da1, {B, 13, 13, 32}, at::kBFloat16, "conv1 grad");
  check_act(idx1, {B, 13, 16, 16}, at::kByte, "conv1 argmax");
  check_f32_out(dw1, {32, 1, 5, 5}, "conv1 dw");
  check_f32_out(db1, {32}, "conv1 db");
  if (B == 0) {
    dw1.zero_();
    db1.zero_();
    return;
  }
  const int bi = static_cast<int>(B);
  at::Tensor slabs = at::empty({kern::cn_conv1_slab_floats(bi)}, dw1.options());
  kern::cn_conv1_wgrad(x.data_ptr(), u8, da1.data_ptr(), idx1.data_ptr<uint8_t>(), bi, static_cast<float>(mean),
                       static_cast<float>(1.0 / std), static_cast<float>(in_scale), slabs.data_ptr<float>(),
                       dw1.data_ptr<float>(), db1.data_ptr<float>(), cur_stream(x));
}

std::tuple<at::Tensor, at::Tensor> gather_augment(const at::Tensor& x, const c10::optional<at::Tensor>& labels,
                                                  const at::Tensor& idx, int64_t pad, bool flip,
                                                  std::vector<double> mean, std::vector<double> std,
                                                  int64_t seed, bool nhwc, at::ScalarType out_dtype) {
  check_cuda(x, "dataset images");
  check_dtype(x, at::kByte, "dataset images");
  RINGDP_CHECK(x.is_contiguous() && (x.dim() == 3 || x.dim() == 4),
               "dataset images: expected contiguous uint8 (N, H, W) or (N, H, W, C)");
  check_cuda(idx, "batch indices");
  check_dtype(idx, at::kLong, "batch indices");
  RINGDP_CHECK(idx.dim() == 1 && idx.is_contiguous(), "batch indices: expected 1-D contiguous int64");
  const int64_t H = x.size(1), W = x.size(2), Cc = x.dim() == 4 ? x.size(3) : 1, B = idx.size(0);
  RINGDP_CHECK(Cc <= 4, "gather_augment: at most 4 channels");
  RINGDP_CHECK(pad >= 0 && pad < H && pad < W, "gather_augment: bad padding");
  RINGDP_CHECK(out_dtype == at::kFloat || out_dtype == at::kBFloat16 || out_dtype == at::kByte,
               "gather_augment: out dtype must be float32, bfloat16 or uint8");
  kern::AugNorm nrm{};
  for (int c = 0; c < 4; ++c) {
    const double m = mean.empty() ? 0.0 : mean[std::min<size_t>(c, mean.size() - 1)];
    const double sd = std.empty() ? 1.0 : std[std::min<size_t>(c, std.size() - 1)];
    RINGDP_CHECK(sd != 0.0, "gather_augment: std must be non-zero");
    nrm.mean[c] = static_cast<float>(m);
    nrm.inv_std[c] = static_cast<float>(1.0 / sd);
  }
  auto opt = x.options().dtype(out_dtype);
  at::Tensor out = nhwc ? at::empty({B, H, W, Cc}, opt) : at::empty({B, Cc, H, W}, opt);
  at::Tensor y;
  const int64_t* lab = nullptr;
  if (labels.has_value() && labels->defined()) {
    check_cuda(*labels, "dataset labels");
    check_dtype(*labels, at::kLong, "dataset labels");
    RINGDP_CHECK(labels->is_contiguous() && labels->size(0) == x.size(0), "dataset labels: shape mismatch");
    y = at::empty({B}, labels->options());
    lab = labels->data_ptr<int64_t>();
  }
  if (B == 0) return {out, y};
  const int kind = out_dtype == at::kFloat ? 0 : (out_dtype == at::kBFloat16 ? 1 : 2);
  kern::gather_augment(x.data_ptr<uint8_t>(), lab, idx.data_ptr<int64_t>(), static_cast<int>(B),
                       static_cast<int>(H), static_cast<int>(W), static_cast<int>(Cc), static_cast<int>(pad), flip,
                       nrm, static_cast<uint64_t>(seed), nhwc, kind, out.data_ptr(),
                       lab ? y.data_ptr<int64_t>() : nullptr, cur_stream(x));
  return {out, y};
}

std::tuple<at::Tensor, at::Tensor> synth_u8_images(int64_t B, int64_t H, int64_t W,
                                                   int64_t num_classes, int64_t seed,
                                                   at::Device device) {
  RINGDP_CHECK(device.is_cuda(), "synth_u8_images: expected a GPU device");
  c10::DeviceGuard g(device);
  auto opt = at::TensorOptions().device(device);
  at::Tensor x = at::empty({B, 1, H, W}, opt.dtype(at::kByte));
  at::Tensor y = at::empty({B}, opt.dtype(at::kLong));
  kern::synth_u8_images(x.data_ptr<uint8_t>(), y.data_ptr<int64_t>(), static_cast<int>(B),
                        static_cast<int>(H * W), static_cast<int>(num_classes),
                        static_cast<uint64_t>(seed), cur_stream(x));
  return {x, y};
}

at::Tensor transpose_bf16(const at::Tensor& x) {
  check_cuda(x, "transpose_bf16");
  check_dtype(x, at::kBFloat16, "transpose_bf16");
  RINGDP_CHECK(x.dim() == 2, "transpose_bf16: 2-d input expected");
  at::Tensor out = at::empty({x.size(1), x.size(0)}, x.options());
  kern::transpose_bf16(x.data_ptr(), out.data_ptr(), x.size(0), x.size(1), cur_stream(x));
  return out;
}

}  // namespace ops
}  // namespace ringdp
