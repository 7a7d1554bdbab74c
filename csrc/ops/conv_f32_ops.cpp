// Tensor-level wrappers for the fp32 NCHW conv / pool kernels (csrc/kernels/conv_f32.hip): the
// ConvNet at the reference's fp32 precision (ringdp/ops/convnet_fp32.py).
#include <torch/extension.h>

#include "../kernels/kernels.h"
#include "ops.h"
#include "util.h"

namespace ringdp {
namespace ops {

namespace {

kern::ConvF32Geom geom(const at::Tensor& x, const at::Tensor& w, int64_t pad) {
  RINGDP_CHECK(x.dim() == 4 && w.dim() == 4, "conv_f32: expected 4-d input and weight");
  RINGDP_CHECK(w.size(2) == w.size(3), "conv_f32: square kernels only");
  RINGDP_CHECK(w.size(1) == x.size(1), "conv_f32: weight expects ", w.size(1), " input channels, input has ",
               x.size(1));
  kern::ConvF32Geom g;
  g.B = x.size(0);
  g.C = static_cast<int>(x.size(1));
  g.H = static_cast<int>(x.size(2));
  g.W = static_cast<int>(x.size(3));
  g.Kout = static_cast<int>(w.size(0));
  g.R = static_cast<int>(w.size(2));
  g.pad = static_cast<int>(pad);
  g.OH = g.H + 2 * g.pad - g.R + 1;
  g.OW = g.W + 2 * g.pad - g.R + 1;
  RINGDP_CHECK(g.OH > 0 && g.OW > 0, "conv_f32: empty output");
  return g;
}

void check_input(const at::Tensor& x) {
  util::gpu(x, "conv_f32 input");
  RINGDP_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kByte,
               "conv_f32 input: fp32 or raw uint8 pixels expected");
}

}  // namespace

at::Tensor f32_conv_fwd(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                        int64_t pad, double mean, double std) {
  check_input(x);
  util::f32_gpu(w, "conv_f32 weight");
  auto g = geom(x, w, pad);
  const float* b = nullptr;
  if (bias && bias->defined()) {
    util::f32_gpu(*bias, "conv_f32 bias");
    RINGDP_CHECK(bias->numel() == g.Kout, "conv_f32 bias: wrong size");
    b = bias->data_ptr<float>();
  }
  auto z = at::empty({g.B, g.Kout, g.OH, g.OW}, w.options());
  const bool u8 = x.scalar_type() == at::kByte;
  kern::conv_f32_fwd(g, u8 ? nullptr : x.data_ptr<float>(), u8 ? x.data_ptr<uint8_t>() : nullptr,
                     static_cast<float>(mean), static_cast<float>(1.0 / std), w.data_ptr<float>(), b,
                     z.data_ptr<float>(), util::stream_of(w));
  return z;
}

std::tuple<at::Tensor, at::Tensor> f32_conv_pool_fwd(const at::Tensor& x, const at::Tensor& w,
                                                     const c10::optional<at::Tensor>& bias, int64_t pad, double mean,
                                                     double std, int64_t stride) {
  check_input(x);
  util::f32_gpu(w, "conv_f32 weight");
  auto g = geom(x, w, pad);
  RINGDP_CHECK(stride == 1 || (g.OH % 2 == 0 && g.OW % 2 == 0),
               "conv_f32 + 2x2/s2 pool: the conv output must have even height and width");
  const float* b = nullptr;
  if (bias && bias->defined()) {
    util::f32_gpu(*bias, "conv_f32 bias");
    RINGDP_CHECK(bias->numel() == g.Kout, "conv_f32 bias: wrong size");
    b = bias->data_ptr<float>();
  }
  RINGDP_CHECK(stride == 1 || stride == 2, "conv_f32 + pool: 2x2 windows with stride 1 or 2");
  if (x.scalar_type() == at::kFloat) {  // small batches: split K, then sum + bias + ReLU + pool in one pass
    const int sl = kern::conv_f32_fwd_slices(g);
    if (sl > 1) {
      const int64_t PH = stride == 2 ? g.OH / 2 : g.OH - 1, PW = stride == 2 ? g.OW / 2 : g.OW - 1;
      auto a = at::empty({g.B, g.Kout, PH, PW}, w.options());
      auto code = at::empty({g.B, g.Kout, PH, PW}, w.options().dtype(at::kByte));
      auto slab = at::empty({static_cast<int64_t>(sl) * g.B * g.Kout * g.OH * g.OW}, w.options());
      kern::conv_f32_fwd_pool_split(g, x.data_ptr<float>(), w.data_ptr<float>(), b, slab.data_ptr<float>(), sl,
                                    static_cast<int>(stride), a.data_ptr<float>(), code.data_ptr<uint8_t>(),
                                    util::stream_of(w));
      return {a, code};
    }
  }
  if (stride == 1) {
    RINGDP_CHECK(x.scalar_type() == at::kFloat && g.OH * g.OW <= 128,
                 "conv_f32 + 2x2/s1 pool: fp32 input and at most 128 output pixels per image");
    auto a = at::empty({g.B, g.Kout, g.OH - 1, g.OW - 1}, w.options());
    auto code = at::empty({g.B, g.Kout, g.OH - 1, g.OW - 1}, w.options().dtype(at::kByte));
    kern::conv_f32_fwd_pool_s1(g, x.data_ptr<float>(), w.data_ptr<float>(), b, a.data_ptr<float>(),
                               code.data_ptr<uint8_t>(), util::stream_of(w));
    return {a, code};
  }
  RINGDP_CHECK(stride == 2, "conv_f32 + pool: 2x2 windows with stride 1 or 2");
  auto a = at::empty({g.B, g.Kout, g.OH / 2, g.OW / 2}, w.options());
  auto code = at::empty({g.B, g.Kout, g.OH / 2, g.OW / 2}, w.options().dtype(at::kByte));
  const bool u8 = x.scalar_type() == at::kByte;
  kern::conv_f32_fwd_pool(g, u8 ? nullptr : x.data_ptr<float>(), u8 ? x.data_ptr<uint8_t>() : nullptr,
                          static_cast<float>(mean), static_cast<float>(1.0 / std), w.data_ptr<float>(), b,
                          a.data_ptr<float>(), code.data_ptr<uint8_t>(), util::stream_of(w));
  return {a, code};
}

namespace {
void check_conv1(const at::Tensor& x, const at::Tensor& w1) {
  check_input(x);
  util::f32_gpu(w1, "conv1 weight");
  RINGDP_CHECK(x.dim() == 4 && x.size(1) == 1 && x.size(2) == 28 && x.size(3) == 28,
               "f32 conv1: [B, 1, 28, 28] input expected, got ", x.sizes());
  RINGDP_CHECK(w1.sizes() == at::IntArrayRef({32, 1, 5, 5}), "f32 conv1: [32, 1, 5, 5] weight expected");
  RINGDP_CHECK(x.size(0) * 32 * 169 < (int64_t{1} << 31), "f32 conv1: batch too large for 32-bit offsets");
}
}  // namespace

std::tuple<at::Tensor, at::Tensor> f32_conv1_pool_fwd(const at::Tensor& x, const at::Tensor& w1, const at::Tensor& b1,
                                                      double mean, double std) {
  check_conv1(x, w1);
  util::f32_gpu(b1, "conv1 bias");
  const int64_t B = x.size(0);
  auto a1 = at::empty({B, 32, 13, 13}, w1.options());
  auto code1 = at::empty({B, 32, 13, 13}, w1.options().dtype(at::kByte));
  const bool u8 = x.scalar_type() == at::kByte;
  auto xc = x.contiguous();
  kern::conv1_pool_f32_fwd(u8 ? nullptr : xc.data_ptr<float>(), u8 ? xc.data_ptr<uint8_t>() : nullptr, B,
                           static_cast<float>(mean), static_cast<float>(1.0 / std), w1.data_ptr<float>(),
                           b1.data_ptr<float>(), a1.data_ptr<float>(), code1.data_ptr<uint8_t>(), util::stream_of(w1));
  return {a1, code1};
}

void f32_conv1_wgrad(const at::Tensor& x, const at::Tensor& da1, const at::Tensor& code1, double mean, double std,
                     at::Tensor& dw1, at::Tensor& db1) {
  check_conv1(x, dw1);
  util::f32_gpu(da1, "conv1 pooled grad");
  util::f32_gpu(db1, "conv1 db");
  const int64_t B = x.size(0);
  RINGDP_CHECK(da1.sizes() == at::IntArrayRef({B, 32, 13, 13}) && code1.sizes() == da1.sizes() &&
                   code1.scalar_type() == at::kByte,
               "f32 conv1 wgrad: pooled grad / code must be [B, 32, 13, 13]");
  const int blocks = kern::conv1_f32_wgrad_blocks(B);
  auto slab = at::empty({static_cast<int64_t>(kern::f32_slab_capacity(blocks)) * 32 * 26}, da1.options());
  const bool u8 = x.scalar_type() == at::kByte;
  auto xc = x.contiguous();
  auto dac = da1.contiguous();
  auto st = util::stream_of(da1);
  kern::conv1_wgrad_f32(u8 ? nullptr : xc.data_ptr<float>(), u8 ? xc.data_ptr<uint8_t>() : nullptr, B,
                        static_cast<float>(mean), static_cast<float>(1.0 / std), dac.data_ptr<float>(),
                        code1.data_ptr<uint8_t>(), slab.data_ptr<float>(), st);
  kern::f32_slab_reduce(slab.data_ptr<float>(), blocks, 32, 25, 26, dw1.data_ptr<float>(), db1.data_ptr<float>(), st);
}

at::Tensor f32_conv_dgrad(const at::Tensor& dz, const at::Tensor& w, int64_t H, int64_t W, int64_t pad) {
  util::f32_gpu(dz, "conv_f32 dz");
  util::f32_gpu(w, "conv_f32 weight");
  kern::ConvF32Geom g;
  g.B = dz.size(0);
  g.Kout = static_cast<int>(w.size(0));
  g.C = static_cast<int>(w.size(1));
  g.R = static_cast<int>(w.size(2));
  g.H = static_cast<int>(H);
  g.W = static_cast<int>(W);
  g.pad = static_cast<int>(pad);
  g.OH = g.H + 2 * g.pad - g.R + 1;
  g.OW = g.W + 2 * g.pad - g.R + 1;
  RINGDP_CHECK(dz.dim() == 4 && dz.size(1) == g.Kout && dz.size(2) == g.OH && dz.size(3) == g.OW,
               "conv_f32 dgrad: dz has shape ", dz.sizes());
  auto dx = at::empty({g.B, g.C, g.H, g.W}, dz.options());
  if (kern::conv_dgrad_f32_scatter_ok(g) && dz.is_contiguous() && w.is_contiguous()) {
    at::Tensor wp = at::empty({kern::conv_dgrad_f32_scratch()}, w.options());
    kern::conv_dgrad_f32_scatter(g, dz.data_ptr<float>(), w.data_ptr<float>(), dx.data_ptr<float>(),
                                  wp.data_ptr<float>(), util::stream_of(dz));
    return dx;
  }
  const int slices = kern::conv_f32_dgrad_slices(g);
  at::Tensor slab;
  if (slices > 1) slab = at::empty({static_cast<int64_t>(slices) * dx.numel()}, dz.options());
  kern::conv_f32_dgrad(g, dz.data_ptr<float>(), w.data_ptr<float>(), dx.data_ptr<float>(),
                       slices > 1 ? slab.data_ptr<float>() : nullptr, slices, util::stream_of(dz));
  return dx;
}

void f32_conv_wgrad(const at::Tensor& dz, const at::Tensor& x, int64_t pad, double mean, double std,
                    at::Tensor& dw, const c10::optional<at::Tensor>& db) {
  check_input(x);
  util::f32_gpu(dz, "conv_f32 dz");
  util::f32_gpu(dw, "conv_f32 dw");
  auto g = geom(x, dw, pad);
  RINGDP_CHECK(dz.dim() == 4 && dz.size(0) == g.B && dz.size(1) == g.Kout && dz.size(2) == g.OH &&
                   dz.size(3) == g.OW,
               "conv_f32 wgrad: dz has shape ", dz.sizes());
  float* dbp = nullptr;
  if (db && db->defined()) {
    util::f32_gpu(*db, "conv_f32 db");
    RINGDP_CHECK(db->numel() == g.Kout, "conv_f32 db: wrong size");
    dbp = db->data_ptr<float>();
  }
  const int slices = kern::conv_f32_wgrad_slices(g);
  auto slab = at::empty({static_cast<int64_t>(slices) * g.Kout * (g.C * g.R * g.R + 1)}, dz.options());
  const bool u8 = x.scalar_type() == at::kByte;
  kern::conv_f32_wgrad(g, dz.data_ptr<float>(), u8 ? nullptr : x.data_ptr<float>(),
                       u8 ? x.data_ptr<uint8_t>() : nullptr, static_cast<float>(mean),
                       static_cast<float>(1.0 / std), slab.data_ptr<float>(), slices, dw.data_ptr<float>(), dbp,
                       util::stream_of(dz));
}

// Deferred weight gradients (the whole-network fp32 cross-entropy node, ringdp/ops/convnet_fp32.py): the GEMM /
// kernel runs now, its fixed-order slab reduction is returned as (slab, [slices, Kout, Nw, ncol]) and launched
// later by f32_slab_reduce_multi together with the other layers' (one launch per backward).
// conv3's data gradient + pool2's (2x2/s1) backward at small batches: dz2 [B, C, 11, 11] from dz3, with the split-K
// planes summed inside the pool backward (falls back to the two ops where that form does not apply)
at::Tensor f32_conv_dgrad_pool2s1_bwd(const at::Tensor& dz, const at::Tensor& w, const at::Tensor& code) {
  util::f32_gpu(dz, "conv_f32 dz");
  util::f32_gpu(w, "conv_f32 weight");
  kern::ConvF32Geom g;
  g.B = dz.size(0);
  g.Kout = static_cast<int>(w.size(0));
  g.C = static_cast<int>(w.size(1));
  g.R = static_cast<int>(w.size(2));
  g.pad = 0;
  g.OH = static_cast<int>(dz.size(2));
  g.OW = static_cast<int>(dz.size(3));
  g.H = g.OH + g.R - 1;
  g.W = g.OW + g.R - 1;
  RINGDP_CHECK(dz.dim() == 4 && dz.size(1) == g.Kout && dz.is_contiguous() && w.is_contiguous(),
               "conv_f32 dgrad + pool: dz has shape ", dz.sizes());
  RINGDP_CHECK(code.scalar_type() == at::kByte && code.dim() == 4 && code.size(0) == g.B && code.size(1) == g.C &&
                   code.size(2) == g.H && code.size(3) == g.W && code.is_contiguous(),
               "conv_f32 dgrad + pool: code must be [B, C, H, W] of the pooled map");
  if (!kern::conv_f32_dgrad_pool2s1_ok(g)) {
    at::Tensor dx = f32_conv_dgrad(dz, w, g.H, g.W, 0);
    return f32_pool_relu_bwd(dx, code, g.H + 1, g.W + 1, 2, 1);
  }
  const int slices = kern::conv_f32_dgrad_slices(g);
  at::Tensor slab = at::empty({static_cast<int64_t>(slices) * g.B * g.C * g.H * g.W}, dz.options());
  at::Tensor dzp = at::empty({g.B, g.C, g.H + 1, g.W + 1}, dz.options());
  kern::conv_f32_dgrad_pool2s1_bwd(g, dz.data_ptr<float>(), w.data_ptr<float>(), slab.data_ptr<float>(), slices,
                                   code.data_ptr<uint8_t>(), dzp.data_ptr<float>(), util::stream_of(dz));
  return dzp;
}

std::tuple<at::Tensor, std::vector<int64_t>> f32_conv_wgrad_slab(const at::Tensor& dz, const at::Tensor& x,
                                                                 int64_t pad, double mean, double std,
                                                                 const at::Tensor& dw, bool with_bias) {
  check_input(x);
  util::f32_gpu(dz, "conv_f32 dz");
  util::f32_gpu(dw, "conv_f32 dw");
  auto g = geom(x, dw, pad);
  RINGDP_CHECK(dz.dim() == 4 && dz.size(0) == g.B && dz.size(1) == g.Kout && dz.size(2) == g.OH &&
                   dz.size(3) == g.OW,
               "conv_f32 wgrad: dz has shape ", dz.sizes());
  const int slices = kern::conv_f32_wgrad_slices(g);
  auto slab = at::empty({static_cast<int64_t>(slices) * g.Kout * (g.C * g.R * g.R + 1)}, dz.options());
  const bool u8 = x.scalar_type() == at::kByte;
  kern::F32RedList segs;
  // dw / db pointers are not used by a deferred call (f32_slab_reduce_multi gets them from the caller)
  float dummy_db = 0.f;
  kern::conv_f32_wgrad(g, dz.data_ptr<float>(), u8 ? nullptr : x.data_ptr<float>(),
                       u8 ? x.data_ptr<uint8_t>() : nullptr, static_cast<float>(mean), static_cast<float>(1.0 / std),
                       slab.data_ptr<float>(), slices, nullptr, with_bias ? &dummy_db : nullptr, util::stream_of(dz),
                       &segs);
  RINGDP_CHECK(segs.size() == 1, "conv_f32 wgrad: expected one deferred reduction");
  const auto& q = segs[0];
  return {slab, {q.slices, q.Kout, q.Nw, q.ncol}};
}

std::tuple<at::Tensor, std::vector<int64_t>> f32_conv1_wgrad_slab(const at::Tensor& x, const at::Tensor& da1,
                                                                  const at::Tensor& code1, double mean, double std) {
  check_input(x);
  RINGDP_CHECK(x.dim() == 4 && x.size(1) == 1 && x.size(2) == 28 && x.size(3) == 28,
               "f32 conv1: [B, 1, 28, 28] input expected, got ", x.sizes());
  util::f32_gpu(da1, "conv1 pooled grad");
  const int64_t B = x.size(0);
  RINGDP_CHECK(da1.sizes() == at::IntArrayRef({B, 32, 13, 13}) && code1.sizes() == da1.sizes() &&
                   code1.scalar_type() == at::kByte,
               "f32 conv1 wgrad: pooled grad / code must be [B, 32, 13, 13]");
  const int blocks = kern::conv1_f32_wgrad_blocks(B);
  auto slab = at::empty({static_cast<int64_t>(kern::f32_slab_capacity(blocks)) * 32 * 26}, da1.options());
  const bool u8 = x.scalar_type() == at::kByte;
  auto xc = x.contiguous();
  auto dac = da1.contiguous();
  kern::conv1_wgrad_f32(u8 ? nullptr : xc.data_ptr<float>(), u8 ? xc.data_ptr<uint8_t>() : nullptr, B,
                        static_cast<float>(mean), static_cast<float>(1.0 / std), dac.data_ptr<float>(),
                        code1.data_ptr<uint8_t>(), slab.data_ptr<float>(), util::stream_of(da1));
  return {slab, {blocks, 32, 25, 26}};
}

std::tuple<at::Tensor, at::Tensor> f32_fc_ce_pool3_bwd(const at::Tensor& logits, const at::Tensor& labels,
                                                       const at::Tensor& lse, const at::Tensor& ws,
                                                       const at::Tensor& grad_out, int64_t ignore_index, double eps,
                                                       int64_t reduction, const at::Tensor& wfc,
                                                       const at::Tensor& code3) {
  util::f32_gpu(logits, "logits");
  util::f32_gpu(wfc, "fc1 weight");
  const int64_t B = logits.size(0);
  RINGDP_CHECK(logits.dim() == 2 && logits.size(1) == 10 && labels.numel() == B && lse.numel() == B &&
                   wfc.numel() == 10 * 2048 && wfc.is_contiguous() && logits.is_contiguous(),
               "fc_ce_pool3_bwd: the ConvNet head (10 classes, 2048 features) expected");
  RINGDP_CHECK(code3.scalar_type() == at::kByte && code3.numel() == B * 2048 && code3.is_contiguous(),
               "fc_ce_pool3_bwd: code3 must be [B, 128, 4, 4] uint8");
  RINGDP_CHECK(labels.scalar_type() == at::kLong && labels.is_contiguous(), "fc_ce_pool3_bwd: int64 labels");
  at::Tensor g = grad_out.to(at::kFloat).contiguous();
  const int64_t nparts = (ws.numel() - 4) / 2;
  at::Tensor dl = at::empty({B, 10}, logits.options());
  at::Tensor dz3 = at::empty({B, 128, 8, 8}, logits.options());
  kern::fc_ce_pool3_bwd_f32(logits.data_ptr<float>(), labels.data_ptr<int64_t>(), lse.data_ptr<float>(),
                            g.data_ptr<float>(), ws.data_ptr<float>() + 2 * nparts, static_cast<int>(ignore_index),
                            static_cast<float>(eps), static_cast<int>(reduction), wfc.data_ptr<float>(),
                            code3.data_ptr<uint8_t>(), static_cast<int>(B), dl.data_ptr<float>(), dz3.data_ptr<float>(),
                            util::stream_of(logits));
  return {dl, dz3};
}

void f32_slab_reduce_multi(const std::vector<at::Tensor>& slabs, const std::vector<std::vector<int64_t>>& meta,
                           const std::vector<at::Tensor>& dws, const std::vector<c10::optional<at::Tensor>>& dbs) {
  RINGDP_CHECK(slabs.size() == meta.size() && slabs.size() == dws.size() && slabs.size() == dbs.size(),
               "f32_slab_reduce_multi: one slab, meta, dw and db per segment");
  if (slabs.empty()) return;
  kern::F32RedList segs;
  for (size_t i = 0; i < slabs.size(); ++i) {
    const auto& m = meta[i];
    RINGDP_CHECK(m.size() == 4, "f32_slab_reduce_multi: meta is [slices, Kout, Nw, ncol]");
    util::f32_gpu(slabs[i], "slab");
    util::f32_gpu(dws[i], "dw");
    RINGDP_CHECK(dws[i].numel() == m[1] * m[2] && slabs[i].numel() >= m[0] * m[1] * m[3],
                 "f32_slab_reduce_multi: segment ", i, " does not match its slab / dw");
    float* db = nullptr;
    if (m[3] > m[2]) {
      RINGDP_CHECK(dbs[i].has_value() && dbs[i]->defined() && dbs[i]->numel() == m[1],
                   "f32_slab_reduce_multi: segment ", i, " has a bias column but no db");
      util::f32_gpu(*dbs[i], "db");
      db = dbs[i]->data_ptr<float>();
    }
    segs.push_back(kern::F32RedSeg{slabs[i].data_ptr<float>(), static_cast<int>(m[0]), static_cast<int>(m[1]),
                                   static_cast<int>(m[2]), static_cast<int>(m[3]), dws[i].data_ptr<float>(), db});
  }
  kern::f32_slab_reduce_multi(segs, util::stream_of(slabs[0]));
}

std::tuple<at::Tensor, at::Tensor> f32_pool_relu_fwd(const at::Tensor& z, int64_t k, int64_t stride) {
  util::f32_gpu(z, "pool_relu_f32 input");
  RINGDP_CHECK(z.dim() == 4, "pool_relu_f32: 4-d input expected");
  const int64_t H = z.size(2), W = z.size(3);
  const int64_t PH = (H - k) / stride + 1, PW = (W - k) / stride + 1;
  RINGDP_CHECK(k >= 1 && k * k <= 254 && PH > 0 && PW > 0, "pool_relu_f32: bad window");
  auto a = at::empty({z.size(0), z.size(1), PH, PW}, z.options());
  auto code = at::empty({z.size(0), z.size(1), PH, PW}, z.options().dtype(at::kByte));
  kern::pool_relu_f32_fwd(z.data_ptr<float>(), a.data_ptr<float>(), code.data_ptr<uint8_t>(),
                          z.size(0) * z.size(1), static_cast<int>(H), static_cast<int>(W), static_cast<int>(k),
                          static_cast<int>(stride), util::stream_of(z));
  return {a, code};
}

at::Tensor f32_pool_relu_bwd(const at::Tensor& da, const at::Tensor& code, int64_t H, int64_t W, int64_t k,
                             int64_t stride) {
  util::f32_gpu(da, "pool_relu_f32 grad");
  util::gpu(code, "pool_relu_f32 code");
  RINGDP_CHECK(code.sizes() == da.sizes(), "pool_relu_f32 bwd: code/grad shape mismatch");
  auto dz = at::empty({da.size(0), da.size(1), H, W}, da.options());
  kern::pool_relu_f32_bwd(da.data_ptr<float>(), code.data_ptr<uint8_t>(), dz.data_ptr<float>(),
                          da.size(0) * da.size(1), static_cast<int>(H), static_cast<int>(W), static_cast<int>(k),
                          static_cast<int>(stride), util::stream_of(da));
  return dz;
}

}  // namespace ops
}  // namespace ringdp
