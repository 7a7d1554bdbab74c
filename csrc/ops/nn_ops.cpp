// Tensor-level wrappers for the generic GEMM / implicit-GEMM conv / NHWC layer kernels
// (csrc/kernels/gemm.hip, nn.hip).  Activations are NHWC bf16; weights stay fp32 masters in
// PyTorch layout and are packed to bf16 per forward.
#include "nn_ops.h"

#include "../kernels/kernels.h"
#include "util.h"

namespace ringdp {
namespace ops {

using namespace util;

namespace {

kern::GemmEpilogue make_epi(void* C, int64_t ldc, int64_t cb, bool out_bf16) {
  kern::GemmEpilogue e{};
  e.mode = kern::GemmEpilogue::kStore;
  e.C = C;
  e.ldc = ldc;
  e.c_bstride = cb;
  e.out_bf16 = out_bf16;
  e.alpha = 1.f;
  return e;
}

kern::ConvGeom geom(const at::Tensor& x, int64_t K, int64_t R, int64_t S, int64_t stride, int64_t pad,
                    int64_t dil) {
  RINGDP_CHECK(x.dim() == 4, "conv input: expected NHWC [N, H, W, C]");
  kern::ConvGeom g{};
  g.N = (int)x.size(0);
  g.H = (int)x.size(1);
  g.W = (int)x.size(2);
  g.C = (int)x.size(3);
  g.K = (int)K;
  g.R = (int)R;
  g.S = (int)S;
  g.stride = (int)stride;
  g.pad = (int)pad;
  g.dil = (int)dil;
  g.P = (g.H + 2 * g.pad - g.dil * (g.R - 1) - 1) / g.stride + 1;
  g.Q = (g.W + 2 * g.pad - g.dil * (g.S - 1) - 1) / g.stride + 1;
  RINGDP_CHECK(g.C % 8 == 0 && g.K % 8 == 0, "conv: channels must be multiples of 8 (pad the input), got C=",
               g.C, " K=", g.K);
  RINGDP_CHECK(g.P > 0 && g.Q > 0, "conv: empty output");
  return g;
}

}  // namespace

at::Tensor gemm(const at::Tensor& a, const at::Tensor& b, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                bool a_row, bool b_row, int64_t batch, int64_t a_bstride, int64_t b_bstride, bool out_bf16,
                const c10::optional<at::Tensor>& bias, int64_t act, const c10::optional<at::Tensor>& residual,
                const c10::optional<at::Tensor>& preact, double alpha, const c10::optional<at::Tensor>& out) {
  bf16_gpu(a, "gemm A");
  bf16_gpu(b, "gemm B");
  RINGDP_CHECK(K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0, "gemm: K and leading dims must be multiples of 8");
  RINGDP_CHECK(!a_row || M % 8 == 0, "gemm: a row-contiguous A needs M % 8 == 0");
  RINGDP_CHECK(!b_row || N % 8 == 0, "gemm: a row-contiguous B needs N % 8 == 0");
  // bounds: the last element each operand touches must be inside its storage
  const int64_t a_need = (batch - 1) * a_bstride + (a_row ? (K - 1) * lda + M : (M - 1) * lda + K);
  const int64_t b_need = (batch - 1) * b_bstride + (b_row ? (K - 1) * ldb + N : (N - 1) * ldb + K);
  RINGDP_CHECK(a.numel() >= a_need && b.numel() >= b_need, "gemm: operand smaller than its described shape");
  at::Tensor c;
  if (out.has_value() && out->defined()) {
    c = *out;
    gpu(c, "gemm out");
    dtype(c, out_bf16 ? at::kBFloat16 : at::kFloat, "gemm out");
    RINGDP_CHECK(c.numel() >= batch * M * N, "gemm out too small");
  } else {
    c = at::empty({batch, M, N}, a.options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat));
  }
  auto e = make_epi(c.data_ptr(), N, M * N, out_bf16);
  e.alpha = static_cast<float>(alpha);
  e.act = static_cast<int>(act);
  if (bias.has_value() && bias->defined()) {
    f32_gpu(*bias, "gemm bias");
    RINGDP_CHECK(bias->numel() == N, "gemm bias: expected N elements");
    e.bias = bias->data_ptr<float>();
  }
  if (residual.has_value() && residual->defined()) {
    bf16_gpu(*residual, "gemm residual");
    RINGDP_CHECK(residual->numel() >= batch * M * N, "gemm residual too small");
    e.residual = residual->data_ptr();
  }
  if (preact.has_value() && preact->defined()) {
    bf16_gpu(*preact, "gemm preact");
    RINGDP_CHECK(preact->numel() >= batch * M * N, "gemm preact too small");
    e.preact = preact->data_ptr();
  }
  if (M == 0 || N == 0) return c;
  kern::GemmOperand A{a.data_ptr(), lda, a_bstride, a_row};
  kern::GemmOperand B{b.data_ptr(), ldb, b_bstride, b_row};
  kern::gemm_bf16(A, B, (int)batch, (int)M, (int)N, (int)K, e, 1, stream_of(a));
  return c;
}

at::Tensor gemm_splitk_f32(const at::Tensor& a, const at::Tensor& b, int64_t M, int64_t N, int64_t K, int64_t lda,
                           int64_t ldb, bool a_row, bool b_row, int64_t splits, const at::Tensor& out) {
  bf16_gpu(a, "gemm A");
  bf16_gpu(b, "gemm B");
  f32_gpu(out, "gemm out");
  RINGDP_CHECK(out.numel() == M * N, "gemm_splitk_f32: out must have M*N elements");
  RINGDP_CHECK(K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0, "gemm: K and leading dims must be multiples of 8");
  RINGDP_CHECK((!a_row || M % 8 == 0) && (!b_row || N % 8 == 0), "gemm: row-contiguous operand needs 8-multiple");
  splits = std::max<int64_t>(1, std::min<int64_t>(splits, std::max<int64_t>(1, K / 64)));
  at::Tensor part = at::empty({splits, M, N}, out.options());
  kern::GemmEpilogue e{};
  e.mode = kern::GemmEpilogue::kSplitK;
  e.partial = part.data_ptr<float>();
  kern::GemmOperand A{a.data_ptr(), lda, 0, a_row};
  kern::GemmOperand B{b.data_ptr(), ldb, 0, b_row};
  kern::gemm_bf16(A, B, 1, (int)M, (int)N, (int)K, e, (int)splits, stream_of(a));
  // the launcher may round the split count down: sum only what was written
  const int64_t kps = ((K + splits - 1) / splits + 63) / 64 * 64;
  const int64_t used = (K + kps - 1) / kps;
  kern::splitk_sum(part.data_ptr<float>(), (int)used, M * N, out.data_ptr<float>(), stream_of(a));
  return out;
}

std::tuple<at::Tensor, at::Tensor> pack_conv_weight(const at::Tensor& w, int64_t cpad) {
  f32_gpu(w, "conv weight");
  RINGDP_CHECK(w.dim() == 4, "conv weight: expected [K, C, R, S]");
  const int64_t K = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3);
  RINGDP_CHECK(cpad >= C && cpad % 8 == 0, "conv weight: padded channels must be >= C and a multiple of 8");
  auto opt = w.options().dtype(at::kBFloat16);
  at::Tensor krsc = at::empty({K, R, S, cpad}, opt), crsk = at::empty({cpad, R, S, K}, opt);
  kern::pack_conv_weight(w.data_ptr<float>(), (int)K, (int)C, (int)R, (int)S, (int)cpad, krsc.data_ptr(),
                         crsk.data_ptr(), stream_of(w));
  return {krsc, crsk};
}

std::tuple<at::Tensor, at::Tensor> conv2d_fwd(const at::Tensor& x, const at::Tensor& w_krsc, int64_t stride,
                                              int64_t pad, int64_t dil, bool want_stats) {
  bf16_gpu(x, "conv input");
  bf16_gpu(w_krsc, "conv packed weight");
  const auto g = geom(x, w_krsc.size(0), w_krsc.size(1), w_krsc.size(2), stride, pad, dil);
  RINGDP_CHECK(w_krsc.size(3) == g.C, "conv: packed weight channels ", w_krsc.size(3), " != input channels ", g.C);
  at::Tensor z = at::empty({g.N, g.P, g.Q, g.K}, x.options());
  at::Tensor sums;
  const int M = g.N * g.P * g.Q;
  auto e = make_epi(z.data_ptr(), g.K, 0, true);
  at::Tensor part;
  if (want_stats) {
    const int tiles = kern::gemm_tiles_m(M);
    part = at::empty({tiles, 2, g.K}, x.options().dtype(at::kFloat));
    e.stats = part.data_ptr<float>();
    sums = at::empty({2, g.K}, part.options());
  }
  kern::conv_fwd_bf16(x.data_ptr(), w_krsc.data_ptr(), g, e, stream_of(x));
  if (want_stats) {
    const int tiles = kern::gemm_tiles_m(M);
    at::Tensor scratch = at::empty({kern::reduce_parts_scratch_floats(tiles, g.K)}, part.options());
    kern::reduce_parts(part.data_ptr<float>(), tiles, g.K, scratch.data_ptr<float>(), sums.data_ptr<float>(),
                       sums.data_ptr<float>() + g.K, stream_of(x));
  }
  return {z, sums};
}

at::Tensor conv2d_dgrad(const at::Tensor& dz, const at::Tensor& w_crsk, int64_t H, int64_t W, int64_t stride,
                        int64_t pad, int64_t dil) {
  bf16_gpu(dz, "conv output grad");
  bf16_gpu(w_crsk, "conv packed weight (CRSK)");
  const int64_t Cp = w_crsk.size(0), R = w_crsk.size(1), S = w_crsk.size(2), K = w_crsk.size(3);
  at::Tensor dx = at::empty({dz.size(0), H, W, Cp}, dz.options());
  auto g = geom(dx, K, R, S, stride, pad, dil);
  RINGDP_CHECK(g.P == dz.size(1) && g.Q == dz.size(2) && dz.size(3) == K, "conv dgrad: output grad shape mismatch");
  auto e = make_epi(dx.data_ptr(), g.C, 0, true);
  kern::conv_dgrad_bf16(dz.data_ptr(), w_crsk.data_ptr(), g, e, stream_of(dz));
  return dx;
}

void conv2d_wgrad(const at::Tensor& dz, const at::Tensor& x, at::Tensor dw, int64_t stride, int64_t pad,
                  int64_t dil) {
  bf16_gpu(dz, "conv output grad");
  bf16_gpu(x, "conv input");
  f32_gpu(dw, "conv weight grad");
  RINGDP_CHECK(dw.dim() == 4, "conv weight grad: expected [K, C, R, S]");
  const int64_t K = dw.size(0), C = dw.size(1), R = dw.size(2), S = dw.size(3);
  auto g = geom(x, K, R, S, stride, pad, dil);
  RINGDP_CHECK(dz.size(0) == g.N && dz.size(1) == g.P && dz.size(2) == g.Q && dz.size(3) == K,
               "conv wgrad: output grad shape mismatch");
  // the GEMM runs over the padded channels; drop the padding when C < Cp
  at::Tensor target = dw;
  if (C != g.C) target = at::empty({K, (int64_t)g.C, R, S}, dw.options());
  const int splits = kern::conv_wgrad_splits(g, num_cus(x));
  at::Tensor part = at::empty({splits, K, (int64_t)g.R * g.S * g.C}, dw.options());
  kern::conv_wgrad_bf16(dz.data_ptr(), x.data_ptr(), g, splits, part.data_ptr<float>(), target.data_ptr<float>(),
                        stream_of(x));
  if (C != g.C) dw.copy_(target.narrow(1, 0, C));
}

at::Tensor nchw_to_nhwc(const at::Tensor& x, int64_t cpad) {
  gpu(x, "image batch");
  RINGDP_CHECK(x.dim() == 4, "image batch: expected NCHW");
  RINGDP_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "image batch: float or bf16");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  RINGDP_CHECK(cpad >= C && cpad % 8 == 0, "nchw_to_nhwc: bad channel padding");
  at::Tensor y = at::empty({N, H, W, cpad}, x.options().dtype(at::kBFloat16));
  kern::nchw_to_nhwc_pad(x.data_ptr(), x.scalar_type() == at::kBFloat16, (int)N, (int)C, (int)H, (int)W, (int)cpad,
                         y.data_ptr(), stream_of(x));
  return y;
}

std::tuple<at::Tensor, at::Tensor> bn_fwd_train(const at::Tensor& z, const at::Tensor& sums, const at::Tensor& gamma,
                                                const at::Tensor& beta, const c10::optional<at::Tensor>& running_mean,
                                                const c10::optional<at::Tensor>& running_var, double eps,
                                                double momentum, const c10::optional<at::Tensor>& residual,
                                                bool relu) {
  bf16_gpu(z, "bn input");
  const int64_t C = z.size(-1), M = z.numel() / C;
  RINGDP_CHECK(C % 8 == 0, "bn: channels must be a multiple of 8");
  f32_gpu(sums, "bn sums");
  f32_gpu(gamma, "bn weight");
  f32_gpu(beta, "bn bias");
  float* rm = nullptr;
  float* rv = nullptr;
  if (running_mean.has_value() && running_mean->defined()) {
    f32_gpu(*running_mean, "bn running_mean");
    f32_gpu(*running_var, "bn running_var");
    rm = running_mean->data_ptr<float>();
    rv = running_var->data_ptr<float>();
  }
  const void* res = nullptr;
  if (residual.has_value() && residual->defined()) {
    bf16_gpu(*residual, "bn residual");
    RINGDP_CHECK(residual->sizes() == z.sizes(), "bn residual: shape mismatch");
    res = residual->data_ptr();
  }
  at::Tensor ss = at::empty({2, C}, gamma.options());
  at::Tensor save = at::empty({2, C}, gamma.options());
  kern::bn_prepare(sums.data_ptr<float>(), M, (int)C, gamma.data_ptr<float>(), beta.data_ptr<float>(), (float)eps,
                   (float)momentum, rm, rv, ss.data_ptr<float>(), save.data_ptr<float>(), stream_of(z));
  at::Tensor y = at::empty_like(z);
  kern::bn_act_fwd(z.data_ptr(), ss.data_ptr<float>(), res, relu, M, (int)C, y.data_ptr(), stream_of(z));
  return {y, save};
}

at::Tensor bn_fwd_eval(const at::Tensor& z, const at::Tensor& scale_shift, const c10::optional<at::Tensor>& residual,
                       bool relu) {
  bf16_gpu(z, "bn input");
  f32_gpu(scale_shift, "bn scale/shift");
  const int64_t C = z.size(-1), M = z.numel() / C;
  const void* res = nullptr;
  if (residual.has_value() && residual->defined()) {
    bf16_gpu(*residual, "bn residual");
    res = residual->data_ptr();
  }
  at::Tensor y = at::empty_like(z);
  kern::bn_act_fwd(z.data_ptr(), scale_shift.data_ptr<float>(), res, relu, M, (int)C, y.data_ptr(), stream_of(z));
  return y;
}

std::tuple<at::Tensor, at::Tensor> bn_bwd(const at::Tensor& dy, const at::Tensor& y, const at::Tensor& z,
                                          const at::Tensor& save, const at::Tensor& gamma, bool relu,
                                          at::Tensor dgamma, at::Tensor dbeta) {
  bf16_gpu(dy, "bn output grad");
  bf16_gpu(z, "bn input");
  if (relu) bf16_gpu(y, "bn output");
  const int64_t C = z.size(-1), M = z.numel() / C;
  RINGDP_CHECK(C % 8 == 0 && C <= 2048, "bn backward: channels must be a multiple of 8 and <= 2048");
  f32_gpu(dgamma, "bn dweight");
  f32_gpu(dbeta, "bn dbias");
  const int nparts = kern::bn_bwd_parts(M);
  at::Tensor part = at::empty({nparts, 2, C}, gamma.options());
  at::Tensor g = at::empty_like(z);  // dL/d(pre-activation) = the residual branch's gradient
  kern::bn_bwd_reduce(dy.data_ptr(), relu ? y.data_ptr() : nullptr, z.data_ptr(), save.data_ptr<float>(), relu, M,
                      (int)C, part.data_ptr<float>(), g.data_ptr(), stream_of(z));
  at::Tensor dz = at::empty_like(z);
  at::Tensor scratch = at::empty({kern::reduce_parts_scratch_floats(nparts, (int)C)}, part.options());
  kern::bn_bwd_apply(part.data_ptr<float>(), nparts, scratch.data_ptr<float>(), g.data_ptr(), z.data_ptr(),
                     save.data_ptr<float>(),
                     gamma.data_ptr<float>(), M, (int)C, dgamma.data_ptr<float>(), dbeta.data_ptr<float>(),
                     dz.data_ptr(), stream_of(z));
  return {dz, g};
}

std::tuple<at::Tensor, at::Tensor> maxpool2d_fwd(const at::Tensor& x, int64_t k, int64_t stride, int64_t pad) {
  bf16_gpu(x, "maxpool input");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  RINGDP_CHECK(C % 8 == 0 && k * k <= 255, "maxpool: channels must be a multiple of 8");
  const int64_t P = (H + 2 * pad - k) / stride + 1, Q = (W + 2 * pad - k) / stride + 1;
  at::Tensor y = at::empty({N, P, Q, C}, x.options());
  at::Tensor arg = at::empty({N, P, Q, C}, x.options().dtype(at::kByte));
  kern::maxpool_fwd(x.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)k, (int)stride, (int)pad, (int)P, (int)Q,
                    y.data_ptr(), arg.data_ptr<uint8_t>(), stream_of(x));
  return {y, arg};
}

at::Tensor maxpool2d_bwd(const at::Tensor& dy, const at::Tensor& arg, int64_t H, int64_t W, int64_t k,
                         int64_t stride, int64_t pad) {
  bf16_gpu(dy, "maxpool output grad");
  const int64_t N = dy.size(0), P = dy.size(1), Q = dy.size(2), C = dy.size(3);
  at::Tensor dx = at::empty({N, H, W, C}, dy.options());
  kern::maxpool_bwd(dy.data_ptr(), arg.data_ptr<uint8_t>(), (int)N, (int)H, (int)W, (int)C, (int)k, (int)stride,
                    (int)pad, (int)P, (int)Q, dx.data_ptr(), stream_of(dy));
  return dx;
}

at::Tensor avgpool_fwd(const at::Tensor& x) {
  bf16_gpu(x, "avgpool input");
  const int64_t N = x.size(0), C = x.size(-1), HW = x.numel() / (N * C);
  at::Tensor y = at::empty({N, C}, x.options());
  kern::avgpool_fwd(x.data_ptr(), (int)N, (int)HW, (int)C, y.data_ptr(), stream_of(x));
  return y;
}

at::Tensor avgpool_bwd(const at::Tensor& dy, int64_t H, int64_t W) {
  bf16_gpu(dy, "avgpool output grad");
  const int64_t N = dy.size(0), C = dy.size(1);
  at::Tensor dx = at::empty({N, H, W, C}, dy.options());
  kern::avgpool_bwd(dy.data_ptr(), (int)N, (int)(H * W), (int)C, dx.data_ptr(), stream_of(dy));
  return dx;
}

at::Tensor add_bf16(const at::Tensor& a, const at::Tensor& b) {
  bf16_gpu(a, "add lhs");
  bf16_gpu(b, "add rhs");
  RINGDP_CHECK(a.sizes() == b.sizes() && a.numel() % 8 == 0, "add_bf16: same shape, numel % 8 == 0");
  at::Tensor y = at::empty_like(a);
  kern::add_bf16(a.data_ptr(), b.data_ptr(), a.numel(), y.data_ptr(), stream_of(a));
  return y;
}

}  // namespace ops
}  // namespace ringdp
