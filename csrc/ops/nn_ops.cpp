// Tensor-level wrappers for the generic GEMM / implicit-GEMM conv / NHWC layer kernels
// (csrc/kernels/gemm.hip, nn.hip).  Activations are NHWC bf16; weights stay fp32 masters in
// PyTorch layout and are packed to bf16 per forward.
#include "nn_ops.h"

#include <cstdlib>
#include <cstring>


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
                const c10::optional<at::Tensor>& preact, double alpha, const c10::optional<at::Tensor>& out,
                const c10::optional<at::Tensor>& colsum) {
  bf16_gpu(a, "gemm A");
  bf16_gpu(b, "gemm B");
  // 16-B vectors run along K for K-contiguous operands and along the rows otherwise
  RINGDP_CHECK(lda % 8 == 0 && ldb % 8 == 0, "gemm: leading dims must be multiples of 8");
  RINGDP_CHECK((a_row && b_row) || K % 8 == 0, "gemm: K must be a multiple of 8 for a K-contiguous operand");
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
  // act 3: the GELU backward, C = (A B^T) * GELU'(preact) with preact an INPUT (the forward's pre-activation)
  RINGDP_CHECK(act != 3 || (e.preact && !e.residual && !e.bias), "gemm act 3 (GELU backward) needs preact only");
  if (M == 0 || N == 0) return c;
  kern::GemmOperand A{a.data_ptr(), lda, a_bstride, a_row};
  kern::GemmOperand B{b.data_ptr(), ldb, b_bstride, b_row};
  if (colsum.has_value() && colsum->defined()) {  // out[n] = sum_m C[m][n] of the stored bf16 C (a bias gradient)
    f32_gpu(*colsum, "gemm colsum");
    RINGDP_CHECK(batch == 1 && out_bf16 && colsum->numel() == N && colsum->is_contiguous(),
                 "gemm colsum: [N] floats, single bf16 GEMM");
    at::Tensor part = at::empty({(M + 255) / 256 * 2, N}, a.options().dtype(at::kFloat));
    e.colsum_part = part.data_ptr<float>();
    if (kern::gemm_bf16_256(A, B, 1, (int)M, (int)N, (int)K, e, 1, stream_of(a))) {  // sums from the epilogue
      kern::rowsum_f32(part.data_ptr<float>(), (int)part.size(0), N, colsum->data_ptr<float>(), stream_of(a));
      return c;
    }
    e.colsum_part = nullptr;  // shape the phased kernel does not take: a separate column-sum pass
    kern::gemm_bf16(A, B, 1, (int)M, (int)N, (int)K, e, 1, stream_of(a));
    colsum_f32(c.view({M, N}), *colsum);
    return c;
  }
  kern::gemm_bf16(A, B, (int)batch, (int)M, (int)N, (int)K, e, 1, stream_of(a));
  return c;
}

at::Tensor gemm_splitk_f32(const at::Tensor& a, const at::Tensor& b, int64_t M, int64_t N, int64_t K, int64_t lda,
                           int64_t ldb, bool a_row, bool b_row, int64_t splits, const at::Tensor& out) {
  bf16_gpu(a, "gemm A");
  bf16_gpu(b, "gemm B");
  f32_gpu(out, "gemm out");
  RINGDP_CHECK(out.numel() == M * N, "gemm_splitk_f32: out must have M*N elements");
  RINGDP_CHECK(lda % 8 == 0 && ldb % 8 == 0, "gemm: leading dims must be multiples of 8");
  RINGDP_CHECK((a_row && b_row) || K % 8 == 0, "gemm: K must be a multiple of 8 for a K-contiguous operand");
  RINGDP_CHECK((!a_row || M % 8 == 0) && (!b_row || N % 8 == 0), "gemm: row-contiguous operand needs 8-multiple");
  splits = std::max<int64_t>(1, std::min<int64_t>(splits, std::max<int64_t>(1, K / 64)));
  splits = kern::gemm_bf16_pick_splits((int)M, (int)N, (int)K, (int)splits);
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

std::vector<at::Tensor> pack_conv_weights(const std::vector<at::Tensor>& ws, const std::vector<int64_t>& cpads) {
  RINGDP_CHECK(ws.size() == cpads.size(), "pack_conv_weights: one channel padding per weight");
  std::vector<at::Tensor> out;
  kern::PackTable t{};
  auto flush = [&](hipStream_t st) {
    kern::pack_conv_weights(t, st);
    t = kern::PackTable{};
  };
  for (size_t i = 0; i < ws.size(); ++i) {
    const at::Tensor& w = ws[i];
    const int64_t cpad = cpads[i];
    f32_gpu(w, "conv weight");
    RINGDP_CHECK(w.dim() == 4, "conv weight: expected [K, C, R, S]");
    const int64_t K = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3);
    RINGDP_CHECK(cpad >= C && cpad % 8 == 0, "conv weight: padded channels must be >= C and a multiple of 8");
    auto opt = w.options().dtype(at::kBFloat16);
    const int64_t kd = R * S * cpad;
    const int64_t ldk = (cpad == 8 && kd % 64 != 0) ? (kd + 63) / 64 * 64 : kd;  // as pack_conv_weight
    at::Tensor store = at::empty({K, ldk}, opt);
    at::Tensor crsk = at::empty({cpad, R, S, K}, opt);
    out.push_back(store.as_strided({K, R, S, cpad}, {ldk, S * cpad, cpad, 1}));
    out.push_back(crsk);
    if (t.n == kern::kPackMax) flush(stream_of(w));
    kern::PackEntry& e = t.e[t.n++];
    e.w = w.data_ptr<float>();
    e.krsc = store.data_ptr();
    e.crsk = crsk.data_ptr();
    e.start = t.total;
    e.start_tile = t.total_tiles;
    e.K = (int)K;
    e.C = (int)C;
    e.R = (int)R;
    e.S = (int)S;
    e.Cp = (int)cpad;
    e.ldk = (int)ldk;
    t.total += K * ldk;
    t.total_tiles += ((cpad * R * S + 63) / 64) * ((K + 63) / 64);
    e.start_tile2 = t.total_tiles2;
    t.total_tiles2 += kern::pack_tiles2((int)K, (int)cpad);
  }
  if (t.n > 0) flush(stream_of(ws[0]));
  return out;
}

std::tuple<at::Tensor, at::Tensor> pack_conv_weight(const at::Tensor& w, int64_t cpad) {
  f32_gpu(w, "conv weight");
  RINGDP_CHECK(w.dim() == 4, "conv weight: expected [K, C, R, S]");
  const int64_t K = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3);
  RINGDP_CHECK(cpad >= C && cpad % 8 == 0, "conv weight: padded channels must be >= C and a multiple of 8");
  auto opt = w.options().dtype(at::kBFloat16);
  // C = 8 (stem) with a ragged k-range: KRSC rows padded to whole 64-wide k-tiles with zeros (a strided
  // [K, R, S, 8] view of [K, ldk] storage) for conv_fwd's aligned C = 8 path
  const int64_t kd = R * S * cpad;
  const int64_t ldk = (cpad == 8 && kd % 64 != 0) ? (kd + 63) / 64 * 64 : kd;
  at::Tensor store = at::empty({K, ldk}, opt);
  at::Tensor krsc = store.as_strided({K, R, S, cpad}, {ldk, S * cpad, cpad, 1});
  at::Tensor crsk = at::empty({cpad, R, S, K}, opt);
  kern::pack_conv_weight(w.data_ptr<float>(), (int)K, (int)C, (int)R, (int)S, (int)cpad, (int)ldk, store.data_ptr(),
                         crsk.data_ptr(), stream_of(w));
  return {krsc, crsk};
}

std::tuple<at::Tensor, at::Tensor> conv2d_fwd(const at::Tensor& x, const at::Tensor& w_krsc, int64_t stride,
                                              int64_t pad, int64_t dil, bool want_stats) {
  bf16_gpu(x, "conv input");
  // rows may be padded (strided view, see pack_conv_weight): no contiguity check, the strides are
  // checked below
  RINGDP_CHECK(w_krsc.defined() && w_krsc.is_cuda(), "conv packed weight: expected a GPU tensor");
  dtype(w_krsc, at::kBFloat16, "conv packed weight");
  const auto g = geom(x, w_krsc.size(0), w_krsc.size(1), w_krsc.size(2), stride, pad, dil);
  RINGDP_CHECK(w_krsc.size(3) == g.C, "conv: packed weight channels ", w_krsc.size(3), " != input channels ", g.C);
  RINGDP_CHECK(w_krsc.stride(3) == 1 && w_krsc.stride(2) == g.C && w_krsc.stride(1) == g.S * g.C &&
                   w_krsc.stride(0) >= (int64_t)g.R * g.S * g.C,
               "conv: packed weight must be KRSC with contiguous rows");
  at::Tensor z = at::empty({g.N, g.P, g.Q, g.K}, x.options());
  at::Tensor sums;
  const int M = g.N * g.P * g.Q;
  const int Kd = g.R * g.S * g.C;
  auto e = make_epi(z.data_ptr(), g.K, 0, true);
  // few output tiles (small spatial maps): split the k-range, then one pass sums the partials, stores z
  // and produces the statistics groups (aligned loaders only)
  const bool pointwise = g.R == 1 && g.S == 1 && g.stride == 1 && g.pad == 0;
  const int splits = (Kd % 64 == 0 && (pointwise || g.C % 64 == 0)) ? kern::conv_gemm_splits(M, g.K, Kd) : 1;
  if (splits > 1) {
    at::Tensor part = at::empty({splits, M, g.K}, x.options().dtype(at::kFloat));
    e.mode = kern::GemmEpilogue::kSplitK;
    e.partial = part.data_ptr<float>();
    kern::conv_fwd_bf16(x.data_ptr(), w_krsc.data_ptr(), w_krsc.stride(0), g, e, stream_of(x), splits);
    float* mid = nullptr;
    if (want_stats) {
      sums = at::empty({kern::splitk_finish_groups(M), 2, g.K}, part.options());
      mid = sums.data_ptr<float>();
    }
    kern::splitk_finish(part.data_ptr<float>(), splits, M, g.K, z.data_ptr(), g.K, nullptr, mid, stream_of(x));
    return {z, sums};
  }
  at::Tensor part;
  if (want_stats) {
    const int tiles = kern::gemm_tiles_m(M);
    part = at::empty({tiles, 2, g.K}, x.options().dtype(at::kFloat));
    e.stats = part.data_ptr<float>();
  }
  kern::conv_fwd_bf16(x.data_ptr(), w_krsc.data_ptr(), w_krsc.stride(0), g, e, stream_of(x));
  if (want_stats) {  // first level of the fixed-order reduction; bn_fwd_train's prepare sums the G groups
    const int tiles = kern::gemm_tiles_m(M);
    if (tiles <= 64) {
      sums = part;  // few tiles: the prepare kernel sums the per-tile partials directly (one launch fewer)
    } else {
      sums = at::empty({kern::reduce_parts_groups(tiles), 2, g.K}, part.options());
      kern::reduce_parts_l1(part.data_ptr<float>(), tiles, g.K, sums.data_ptr<float>(), stream_of(x));
    }
  }
  return {z, sums};
}

at::Tensor conv2d_dgrad(const at::Tensor& dz, const at::Tensor& w_crsk, int64_t H, int64_t W, int64_t stride,
                        int64_t pad, int64_t dil, const c10::optional<at::Tensor>& residual) {
  bf16_gpu(dz, "conv output grad");
  bf16_gpu(w_crsk, "conv packed weight (CRSK)");
  const int64_t Cp = w_crsk.size(0), R = w_crsk.size(1), S = w_crsk.size(2), K = w_crsk.size(3);
  at::Tensor dx = at::empty({dz.size(0), H, W, Cp}, dz.options());
  auto g = geom(dx, K, R, S, stride, pad, dil);
  RINGDP_CHECK(g.P == dz.size(1) && g.Q == dz.size(2) && dz.size(3) == K, "conv dgrad: output grad shape mismatch");
  auto e = make_epi(dx.data_ptr(), g.C, 0, true);
  const void* res = nullptr;
  if (residual.has_value() && residual->defined()) {
    // the input's other gradient (a residual/shortcut branch) summed in the epilogue instead of by
    // autograd's separate add pass
    bf16_gpu(*residual, "conv dgrad residual");
    RINGDP_CHECK(residual->sizes() == dx.sizes(), "conv dgrad residual: shape mismatch");
    res = residual->data_ptr();
  }
  const int M = g.N * g.H * g.W, Kd = g.R * g.S * g.K;
  const bool pointwise = g.R == 1 && g.S == 1 && g.stride == 1 && g.pad == 0;
  // stride 2 takes the parity-class path; few output tiles otherwise: split the k-range
  const int splits = (g.stride != 2 && Kd % 64 == 0 && (pointwise || g.K % 64 == 0))
                         ? kern::conv_gemm_splits(M, g.C, Kd) : 1;
  if (splits > 1) {
    at::Tensor part = at::empty({splits, M, g.C}, dz.options().dtype(at::kFloat));
    e.mode = kern::GemmEpilogue::kSplitK;
    e.partial = part.data_ptr<float>();
    kern::conv_dgrad_bf16(dz.data_ptr(), w_crsk.data_ptr(), g, e, stream_of(dz), splits);
    kern::splitk_finish(part.data_ptr<float>(), splits, M, g.C, dx.data_ptr(), g.C, res, nullptr, stream_of(dz));
    return dx;
  }
  e.residual = res;
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
                                                bool relu, const c10::optional<at::Tensor>& num_batches_tracked) {
  bf16_gpu(z, "bn input");
  const int64_t C = z.size(-1), M = z.numel() / C;
  RINGDP_CHECK(C % 8 == 0, "bn: channels must be a multiple of 8");
  f32_gpu(sums, "bn sums");
  // [2, C] totals or [G, 2, C] group partials (conv2d_fwd's statistics)
  RINGDP_CHECK((sums.dim() == 2 && sums.size(0) == 2 && sums.size(1) == C) ||
                   (sums.dim() == 3 && sums.size(1) == 2 && sums.size(2) == C),
               "bn sums: expected [2, C] or [G, 2, C]");
  const int G = sums.dim() == 3 ? (int)sums.size(0) : 1;
  int64_t* nbt = nullptr;
  if (num_batches_tracked.has_value() && num_batches_tracked->defined()) {
    gpu(*num_batches_tracked, "bn num_batches_tracked");
    dtype(*num_batches_tracked, at::kLong, "bn num_batches_tracked");
    nbt = num_batches_tracked->data_ptr<int64_t>();
  }
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
  at::Tensor save = at::empty({2, C}, gamma.options());
  // RINGDP_BN_FOLD=1: one launch, every workgroup forms the scale / shift itself.  Opt-in: the redundant
  // per-workgroup statistics cost more than the launch they save (ResNet-18 B=256 1.913 -> 1.934 ms, ResNet-50
  // 34.05 -> 34.43 ms; profiles/r06/rejected/bn_fold.md)
  static const bool fold = [] { const char* v = std::getenv("RINGDP_BN_FOLD"); return v && std::atoi(v) != 0; }();
  if (fold && kern::bn_fold_ok(G, (int)C)) {
    at::Tensor y = at::empty_like(z);
    kern::bn_fold_act_fwd(sums.data_ptr<float>(), G, M, (int)C, gamma.data_ptr<float>(), beta.data_ptr<float>(),
                          (float)eps, (float)momentum, rm, rv, save.data_ptr<float>(), nbt, z.data_ptr(), res, relu,
                          y.data_ptr(), stream_of(z));
    return {y, save};
  }
  // save4 = [mean, inv_std, scale, shift]: the backward of a BN + ReLU without a residual re-derives the ReLU mask
  // from z and the scale / shift (bn_bwd need_g = false) instead of reading y
  at::Tensor save4 = at::empty({4, C}, gamma.options());
  float* ss = save4.data_ptr<float>() + 2 * C;
  kern::bn_prepare(sums.data_ptr<float>(), G, M, (int)C, gamma.data_ptr<float>(), beta.data_ptr<float>(), (float)eps,
                   (float)momentum, rm, rv, ss, save4.data_ptr<float>(), nbt, stream_of(z));
  at::Tensor y = at::empty_like(z);
  kern::bn_act_fwd(z.data_ptr(), ss, res, relu, M, (int)C, y.data_ptr(), stream_of(z));
  return {y, save4};
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
                                          at::Tensor dgamma, at::Tensor dbeta, bool need_g) {
  bf16_gpu(dy, "bn output grad");
  bf16_gpu(z, "bn input");
  const int64_t C = z.size(-1), M = z.numel() / C;
  RINGDP_CHECK(C % 8 == 0 && C <= 2048, "bn backward: channels must be a multiple of 8 and <= 2048");
  f32_gpu(dgamma, "bn dweight");
  f32_gpu(dbeta, "bn dbias");
  f32_gpu(save, "bn save");
  // need_g = false (no residual consumes the pre-activation gradient): nothing stores it.  Without ReLU the apply
  // pass reads dy itself; with ReLU and bn_fwd_train's [4, C] save the mask comes from z and the forward's
  // scale / shift (bit-identical to y > 0), so y is not read either.
  const bool zmask = !need_g && relu && save.dim() == 2 && save.size(0) == 4 && kern::bn_bwd_zmask_ok((int)C);
  const bool store_g = need_g || (relu && !zmask);
  if (relu && !zmask) bf16_gpu(y, "bn output");
  const float* ss = zmask ? save.data_ptr<float>() + 2 * C : nullptr;
  const int nparts = kern::bn_bwd_parts(M, (int)C);
  at::Tensor part = at::empty({nparts, 2, C}, gamma.options());
  at::Tensor g = store_g ? at::empty_like(z) : at::Tensor();  // dL/d(pre-activation): the residual's gradient
  kern::bn_bwd_reduce(dy.data_ptr(), (relu && !zmask) ? y.data_ptr() : nullptr, z.data_ptr(), save.data_ptr<float>(),
                      ss, relu, M, (int)C, part.data_ptr<float>(), store_g ? g.data_ptr() : nullptr, stream_of(z));
  at::Tensor dz = at::empty_like(z);
  at::Tensor scratch = at::empty({kern::reduce_parts_scratch_floats(nparts, (int)C)}, part.options());
  kern::bn_bwd_apply(part.data_ptr<float>(), nparts, scratch.data_ptr<float>(), store_g ? g.data_ptr() : dy.data_ptr(),
                     z.data_ptr(), save.data_ptr<float>(), ss, gamma.data_ptr<float>(), M, (int)C,
                     dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), dz.data_ptr(), stream_of(z));
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

std::tuple<at::Tensor, at::Tensor> head_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b) {
  bf16_gpu(x, "head input");
  f32_gpu(w, "head weight");
  f32_gpu(b, "head bias");
  const int64_t N = x.size(0), C = x.size(-1), HW = x.numel() / (N * C), J = w.size(0);
  RINGDP_CHECK(kern::head_ok((int)C, (int)J) && w.dim() == 2 && w.size(1) == C && b.numel() == J,
               "head: unsupported shape (C ", C, ", classes ", J, ")");
  at::Tensor logits = at::empty({N, J}, w.options());
  at::Tensor pooled = at::empty({N, C}, w.options());
  kern::head_fwd(x.data_ptr(), (int)N, (int)HW, (int)C, (int)J, w.data_ptr<float>(), b.data_ptr<float>(),
                 pooled.data_ptr<float>(), logits.data_ptr<float>(), stream_of(x));
  return {logits, pooled};
}

at::Tensor head_bwd(const c10::optional<at::Tensor>& dl, const c10::optional<at::Tensor>& logits,
                    const c10::optional<at::Tensor>& labels, const c10::optional<at::Tensor>& lse,
                    const c10::optional<at::Tensor>& ws, const c10::optional<at::Tensor>& grad_out,
                    int64_t ignore_index, double eps, int64_t reduction, const at::Tensor& pooled,
                    const at::Tensor& w, int64_t H, int64_t W, at::Tensor dw, at::Tensor db) {
  f32_gpu(pooled, "head pooled");
  f32_gpu(w, "head weight");
  f32_gpu(dw, "head dweight");
  f32_gpu(db, "head dbias");
  const int64_t N = pooled.size(0), C = pooled.size(1), J = w.size(0);
  RINGDP_CHECK(kern::head_ok((int)C, (int)J) && dw.sizes() == w.sizes() && db.numel() == J,
               "head backward: unsupported shape");
  const float* dlp = nullptr;
  kern::CeFuse ce{};
  at::Tensor g;
  if (dl.has_value() && dl->defined()) {
    f32_gpu(*dl, "head logits grad");
    RINGDP_CHECK(dl->dim() == 2 && dl->size(0) == N && dl->size(1) == J, "head backward: dl must be [N, J]");
    dlp = dl->data_ptr<float>();
  } else {
    RINGDP_CHECK(logits && labels && lse && ws && grad_out, "head backward: dl or the cross-entropy tensors");
    f32_gpu(*logits, "head logits");
    RINGDP_CHECK(logits->size(0) == N && logits->size(1) == J && labels->numel() == N, "head backward: CE shapes");
    g = grad_out->to(at::kFloat).contiguous();
    const int64_t nparts = (ws->numel() - 4) / 2;
    ce = kern::CeFuse{logits->data_ptr<float>(), labels->data_ptr<int64_t>(), lse->data_ptr<float>(),
                      g.data_ptr<float>(), ws->data_ptr<float>() + 2 * nparts, (int)ignore_index, (float)eps,
                      (int)reduction};
  }
  at::Tensor dx = at::empty({N, H, W, C}, w.options().dtype(at::kBFloat16));
  kern::head_bwd(dlp, dlp ? nullptr : &ce, pooled.data_ptr<float>(), w.data_ptr<float>(), (int)N, (int)(H * W),
                 (int)C, (int)J, dx.data_ptr(), dw.data_ptr<float>(), db.data_ptr<float>(), stream_of(pooled));
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

// ------------------------------------------------------------------ transformer layers
std::tuple<at::Tensor, at::Tensor> layernorm_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b,
                                                 double eps) {
  bf16_gpu(x, "layernorm input");
  f32_gpu(w, "layernorm weight");
  f32_gpu(b, "layernorm bias");
  const int64_t D = x.size(-1), rows = x.numel() / D;
  RINGDP_CHECK(D % 8 == 0 && D <= 2048 && w.numel() == D && b.numel() == D, "layernorm: bad shapes");
  at::Tensor y = at::empty_like(x);
  at::Tensor stats = at::empty({rows, 2}, w.options());
  kern::layernorm_fwd(x.data_ptr(), w.data_ptr<float>(), b.data_ptr<float>(), rows, (int)D, (float)eps, y.data_ptr(),
                      stats.data_ptr<float>(), stream_of(x));
  return {y, stats};
}

std::vector<at::Tensor> layernorm_fwd_q8(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b, double eps,
                                         at::Tensor hist) {
  bf16_gpu(x, "layernorm input");
  f32_gpu(w, "layernorm weight");
  f32_gpu(b, "layernorm bias");
  f32_gpu(hist, "fp8 amax history");
  const int64_t D = x.size(-1), rows = x.numel() / D;
  RINGDP_CHECK(D % 8 == 0 && D <= 2048 && w.numel() == D && b.numel() == D && rows % 16 == 0 && x.is_contiguous(),
               "layernorm_fwd_q8: bad shapes");
  RINGDP_CHECK(hist.is_contiguous() && hist.numel() == 1 + kern::layernorm_q8_blocks(rows),
               "layernorm_fwd_q8: history must hold 1 + ceil(rows / 64) floats");
  at::Tensor stats = at::empty({rows, 2}, w.options());
  at::Tensor q = at::empty({rows, D}, x.options().dtype(at::kByte)), qt = at::empty({D, rows}, x.options().dtype(at::kByte));
  at::Tensor scale = at::empty({1}, w.options());
  kern::layernorm_fwd_q8(x.data_ptr(), w.data_ptr<float>(), b.data_ptr<float>(), rows, (int)D, (float)eps,
                         stats.data_ptr<float>(), hist.data_ptr<float>(), q.data_ptr(), qt.data_ptr(),
                         scale.data_ptr<float>(), hist.data_ptr<float>() + 1, stream_of(x));
  return {stats, q, qt, scale};
}

int64_t layernorm_q8_slots(int64_t rows) { return kern::layernorm_q8_blocks(rows); }

std::vector<at::Tensor> layernorm_bwd_colsum(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& stats,
                                             const at::Tensor& w, const c10::optional<at::Tensor>& dres, at::Tensor dw,
                                             at::Tensor db) {
  bf16_gpu(dy, "layernorm output grad");
  bf16_gpu(x, "layernorm input");
  f32_gpu(stats, "layernorm stats");
  f32_gpu(dw, "layernorm dweight");
  f32_gpu(db, "layernorm dbias");
  const int64_t D = x.size(-1), rows = x.numel() / D;
  RINGDP_CHECK(dy.sizes() == x.sizes() && D % 4 == 0, "layernorm backward: shape mismatch");
  const void* dr = nullptr;
  if (dres.has_value() && dres->defined()) {
    bf16_gpu(*dres, "layernorm residual grad");
    RINGDP_CHECK(dres->sizes() == x.sizes(), "layernorm residual grad: shape mismatch");
    dr = dres->data_ptr();
  }
  at::Tensor dx = at::empty_like(x);
  at::Tensor scratch = at::empty({kern::layernorm_bwd_scratch_floats(rows, (int)D)}, w.options());
  at::Tensor cs = at::empty({kern::layernorm_bwd_blocks(rows), D}, w.options());
  kern::layernorm_bwd(dy.data_ptr(), x.data_ptr(), stats.data_ptr<float>(), w.data_ptr<float>(), dr, rows, (int)D,
                      dx.data_ptr(), scratch.data_ptr<float>(), dw.data_ptr<float>(), db.data_ptr<float>(),
                      stream_of(x), cs.data_ptr<float>());
  return {dx, cs};
}

at::Tensor layernorm_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& stats, const at::Tensor& w,
                         const c10::optional<at::Tensor>& dres, at::Tensor dw, at::Tensor db) {
  bf16_gpu(dy, "layernorm output grad");
  bf16_gpu(x, "layernorm input");
  f32_gpu(stats, "layernorm stats");
  f32_gpu(dw, "layernorm dweight");
  f32_gpu(db, "layernorm dbias");
  const int64_t D = x.size(-1), rows = x.numel() / D;
  RINGDP_CHECK(dy.sizes() == x.sizes(), "layernorm backward: shape mismatch");
  const void* dr = nullptr;
  if (dres.has_value() && dres->defined()) {
    bf16_gpu(*dres, "layernorm residual grad");
    RINGDP_CHECK(dres->sizes() == x.sizes(), "layernorm residual grad: shape mismatch");
    dr = dres->data_ptr();
  }
  at::Tensor dx = at::empty_like(x);
  at::Tensor scratch = at::empty({kern::layernorm_bwd_scratch_floats(rows, (int)D)}, w.options());
  kern::layernorm_bwd(dy.data_ptr(), x.data_ptr(), stats.data_ptr<float>(), w.data_ptr<float>(), dr, rows, (int)D,
                      dx.data_ptr(), scratch.data_ptr<float>(), dw.data_ptr<float>(), db.data_ptr<float>(),
                      stream_of(x));
  return dx;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> qkv_split(const at::Tensor& qkv, int64_t B, int64_t T, int64_t H,
                                                         int64_t Tp) {
  bf16_gpu(qkv, "qkv");
  const int64_t D3 = qkv.size(-1), Dh = D3 / 3 / H;
  RINGDP_CHECK(qkv.numel() == B * T * D3 && Dh * 3 * H == D3 && Dh % 8 == 0 && Tp >= T, "qkv_split: bad shapes");
  auto opt = qkv.options();
  at::Tensor q = at::empty({B * H, Tp, Dh}, opt), k = at::empty({B * H, Tp, Dh}, opt), v = at::empty({B * H, Tp, Dh}, opt);
  kern::qkv_split(qkv.data_ptr(), (int)B, (int)T, (int)H, (int)Dh, (int)Tp, q.data_ptr(), k.data_ptr(), v.data_ptr(),
                  stream_of(qkv));
  return {q, k, v};
}

at::Tensor qkv_merge(const at::Tensor& dq, const at::Tensor& dk, const at::Tensor& dv, int64_t B, int64_t T) {
  bf16_gpu(dq, "dq");
  bf16_gpu(dk, "dk");
  bf16_gpu(dv, "dv");
  const int64_t BH = dq.size(0), Tp = dq.size(1), Dh = dq.size(2), H = BH / B;
  at::Tensor out = at::empty({B * T, 3 * H * Dh}, dq.options());
  kern::qkv_merge(dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), (int)B, (int)T, (int)H, (int)Dh, (int)Tp,
                  out.data_ptr(), stream_of(dq));
  return out;
}

at::Tensor heads_to_rows(const at::Tensor& o, int64_t B, int64_t T) {
  bf16_gpu(o, "attention output");
  const int64_t BH = o.size(0), Tp = o.size(1), Dh = o.size(2), H = BH / B;
  at::Tensor out = at::empty({B * T, H * Dh}, o.options());
  kern::heads_to_rows(o.data_ptr(), (int)B, (int)T, (int)H, (int)Dh, (int)Tp, out.data_ptr(), stream_of(o));
  return out;
}

at::Tensor rows_to_heads(const at::Tensor& rows, int64_t B, int64_t T, int64_t H, int64_t Tp) {
  bf16_gpu(rows, "token rows");
  const int64_t D = rows.size(-1), Dh = D / H;
  at::Tensor out = at::empty({B * H, Tp, Dh}, rows.options());
  kern::rows_to_heads(rows.data_ptr(), (int)B, (int)T, (int)H, (int)Dh, (int)Tp, out.data_ptr(), stream_of(rows));
  return out;
}

at::Tensor softmax_fwd(const at::Tensor& scores, int64_t T, double scale) {
  f32_gpu(scores, "attention scores");
  const int64_t Tp = scores.size(-1), rows = scores.numel() / Tp;
  at::Tensor p = at::empty(scores.sizes(), scores.options().dtype(at::kBFloat16));
  kern::softmax_fwd(scores.data_ptr<float>(), rows, (int)T, (int)Tp, (float)scale, p.data_ptr(), stream_of(scores));
  return p;
}

std::vector<at::Tensor> attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, int64_t T,
                                 double scale) {
  bf16_gpu(q, "attention q");
  bf16_gpu(k, "attention k");
  bf16_gpu(v, "attention v");
  RINGDP_CHECK(q.dim() == 3 && q.sizes() == k.sizes() && q.sizes() == v.sizes() && q.is_contiguous() &&
                   k.is_contiguous() && v.is_contiguous(),
               "attn_fwd: q, k, v must be contiguous [BH, Tp, Dh]");
  const int64_t BH = q.size(0), Tp = q.size(1), Dh = q.size(2);
  at::Tensor p = at::empty({BH, Tp, Tp}, q.options());
  at::Tensor o = at::empty({BH, Tp, Dh}, q.options());
  const bool ok = kern::attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), (int)BH, (int)T, (int)Tp, (int)Dh,
                                 (float)scale, p.data_ptr(), o.data_ptr(), stream_of(q));
  RINGDP_CHECK(ok, "attn_fwd: unsupported shape (needs head dim 64, Tp % 16 == 0, Tp <= 256)");
  return {p, o};
}

at::Tensor attn_bwd_ds(const at::Tensor& dout, const at::Tensor& v, const at::Tensor& p, double scale) {
  bf16_gpu(dout, "attention dO");
  bf16_gpu(v, "attention v");
  bf16_gpu(p, "attention probs");
  RINGDP_CHECK(dout.dim() == 3 && dout.sizes() == v.sizes() && p.dim() == 3 && p.size(0) == v.size(0) &&
                   p.size(1) == v.size(1) && p.size(2) == v.size(1) && dout.is_contiguous() && v.is_contiguous() &&
                   p.is_contiguous(),
               "attn_bwd_ds: expected contiguous dO, V [BH, Tp, Dh] and P [BH, Tp, Tp]");
  at::Tensor ds = at::empty_like(p);
  const bool ok = kern::attn_bwd_ds(dout.data_ptr(), v.data_ptr(), p.data_ptr(), (int)v.size(0), (int)v.size(1),
                                    (int)v.size(2), (float)scale, ds.data_ptr(), stream_of(p));
  RINGDP_CHECK(ok, "attn_bwd_ds: unsupported shape (needs head dim 64, Tp % 16 == 0, Tp <= 256)");
  return ds;
}

at::Tensor attn_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                    const at::Tensor& p, int64_t B, int64_t T, int64_t H, double scale) {
  for (const at::Tensor* t : {&dout, &q, &k, &v}) {
    bf16_gpu(*t, "attention operand");
    RINGDP_CHECK(t->dim() == 3 && t->sizes() == q.sizes(), "attn_bwd: dO, Q, K, V must be [BH, Tp, Dh]");
  }
  bf16_gpu(p, "attention probs");
  const int64_t BH = q.size(0), Tp = q.size(1), Dh = q.size(2);
  RINGDP_CHECK(BH == B * H && p.dim() == 3 && p.size(0) == BH && p.size(1) == Tp && p.size(2) == Tp && T <= Tp,
               "attn_bwd: shape mismatch");
  at::Tensor dqkv = at::empty({B * T, 3 * H * Dh}, q.options());
  at::Tensor dsum = at::empty({BH, Tp}, q.options().dtype(at::kFloat));
  const bool ok = kern::attn_bwd(dout.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), p.data_ptr(), (int)B,
                                 (int)T, (int)H, (int)Tp, (int)Dh, (float)scale, dsum.data_ptr<float>(),
                                 dqkv.data_ptr(), stream_of(q));
  RINGDP_CHECK(ok, "attn_bwd: unsupported shape (needs head dim 64, Tp % 16 == 0, Tp <= 256)");
  return dqkv;
}

std::vector<at::Tensor> attn_fwd_rows(const at::Tensor& qkv, int64_t B, int64_t T, int64_t H, double scale,
                                      bool recompute) {
  bf16_gpu(qkv, "attention qkv rows");
  RINGDP_CHECK(qkv.dim() == 2 && qkv.size(0) == B * T && qkv.size(1) % (3 * H) == 0, "attn_fwd_rows: qkv [B*T, 3*H*Dh]");
  const int64_t Dh = qkv.size(1) / (3 * H), Tp = (T + 15) / 16 * 16;
  at::Tensor out = at::empty({B * T, H * Dh}, qkv.options());
  if (recompute) {  // saved for the backward: per-query log-sum-exp [B*H][Tp] fp32 instead of P
    at::Tensor lse = at::empty({B * H, Tp}, qkv.options().dtype(at::kFloat));
    const bool ok = kern::attn_fwd_rows_lse(qkv.data_ptr(), (int)B, (int)T, (int)H, (int)Tp, (int)Dh, (float)scale,
                                            lse.data_ptr<float>(), out.data_ptr(), stream_of(qkv));
    RINGDP_CHECK(ok, "attn_fwd_rows: unsupported shape (needs head dim 64, T <= 256)");
    return {lse, out};
  }
  at::Tensor p = at::empty({B * H, Tp, Tp}, qkv.options());
  const bool ok = kern::attn_fwd_rows(qkv.data_ptr(), (int)B, (int)T, (int)H, (int)Tp, (int)Dh, (float)scale,
                                      p.data_ptr(), out.data_ptr(), stream_of(qkv));
  RINGDP_CHECK(ok, "attn_fwd_rows: unsupported shape (needs head dim 64, T <= 256)");
  return {p, out};
}

at::Tensor attn_bwd_rows(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& p, int64_t B, int64_t T,
                         int64_t H, double scale, const c10::optional<at::Tensor>& colsum_part) {
  bf16_gpu(dout, "attention output grad rows");
  bf16_gpu(qkv, "attention qkv rows");
  const int64_t Dh = qkv.size(1) / (3 * H), Tp = (T + 15) / 16 * 16;
  if (p.scalar_type() == at::kFloat) {  // the forward saved the log-sum-exp: P is recomputed
    f32_gpu(p, "attention log-sum-exp");
    RINGDP_CHECK(qkv.dim() == 2 && qkv.size(0) == B * T && dout.dim() == 2 && dout.size(0) == B * T &&
                     dout.size(1) == H * Dh && p.dim() == 2 && p.size(0) == B * H && p.size(1) == Tp,
                 "attn_bwd_rows: shape mismatch");
    at::Tensor dqkv = at::empty_like(qkv);
    at::Tensor dsum = at::empty({B * H, Tp}, qkv.options().dtype(at::kFloat));
    float* csp = nullptr;
    if (colsum_part.has_value() && colsum_part->defined()) {  // every entry is written by one workgroup
      f32_gpu(*colsum_part, "attention dqkv column-sum partials");
      RINGDP_CHECK(colsum_part->numel() == B * qkv.size(1) && colsum_part->is_contiguous(),
                   "attn_bwd_rows: colsum_part must be [B, 3*H*Dh] floats");
      csp = colsum_part->data_ptr<float>();
    }
    const bool ok = kern::attn_bwd_rows_lse(dout.data_ptr(), qkv.data_ptr(), p.data_ptr<float>(), (int)B, (int)T, (int)H,
                                            (int)Tp, (int)Dh, (float)scale, dsum.data_ptr<float>(), dqkv.data_ptr(),
                                            stream_of(qkv), csp);
    RINGDP_CHECK(ok, "attn_bwd_rows: unsupported shape (needs head dim 64, T <= 256)");
    return dqkv;
  }
  RINGDP_CHECK(!(colsum_part.has_value() && colsum_part->defined()),
               "attn_bwd_rows: column sums need the recompute (log-sum-exp) path");
  bf16_gpu(p, "attention probs");
  RINGDP_CHECK(qkv.dim() == 2 && qkv.size(0) == B * T && dout.dim() == 2 && dout.size(0) == B * T &&
                   dout.size(1) == H * Dh && p.dim() == 3 && p.size(0) == B * H && p.size(1) == Tp && p.size(2) == Tp,
               "attn_bwd_rows: shape mismatch");
  at::Tensor dqkv = at::empty_like(qkv);
  at::Tensor dsum = at::empty({B * H, Tp}, qkv.options().dtype(at::kFloat));
  const bool ok = kern::attn_bwd_rows(dout.data_ptr(), qkv.data_ptr(), p.data_ptr(), (int)B, (int)T, (int)H, (int)Tp,
                                      (int)Dh, (float)scale, dsum.data_ptr<float>(), dqkv.data_ptr(), stream_of(qkv));
  RINGDP_CHECK(ok, "attn_bwd_rows: unsupported shape (needs head dim 64, T <= 256)");
  return dqkv;
}

at::Tensor softmax_bwd(const at::Tensor& p, const at::Tensor& dp, int64_t T, double scale) {
  bf16_gpu(p, "attention probs");
  f32_gpu(dp, "attention probs grad");
  const int64_t Tp = p.size(-1), rows = p.numel() / Tp;
  at::Tensor ds = at::empty_like(p);
  kern::softmax_bwd(p.data_ptr(), dp.data_ptr<float>(), rows, (int)T, (int)Tp, (float)scale, ds.data_ptr(),
                    stream_of(p));
  return ds;
}

at::Tensor gelu_bwd(const at::Tensor& dy, const at::Tensor& pre) {
  bf16_gpu(dy, "gelu output grad");
  bf16_gpu(pre, "gelu input");
  RINGDP_CHECK(dy.numel() == pre.numel() && dy.numel() % 8 == 0, "gelu_bwd: shape mismatch");
  at::Tensor dx = at::empty_like(pre);
  kern::gelu_bwd(dy.data_ptr(), pre.data_ptr(), dy.numel(), dx.data_ptr(), stream_of(dy));
  return dx;
}

at::Tensor assemble_tokens(const at::Tensor& patches, const at::Tensor& cls, const at::Tensor& pos) {
  bf16_gpu(patches, "patch embeddings");
  f32_gpu(cls, "class token");
  f32_gpu(pos, "position embedding");
  const int64_t B = patches.size(0), D = patches.size(-1), NP = patches.numel() / (B * D);
  RINGDP_CHECK(pos.numel() == (NP + 1) * D && cls.numel() == D, "assemble_tokens: bad shapes");
  at::Tensor out = at::empty({B, NP + 1, D}, patches.options());
  kern::assemble_tokens(patches.data_ptr(), cls.data_ptr<float>(), pos.data_ptr<float>(), (int)B, (int)NP, (int)D,
                        out.data_ptr(), stream_of(patches));
  return out;
}

at::Tensor assemble_tokens_bwd(const at::Tensor& dout, at::Tensor dpos, at::Tensor dcls) {
  bf16_gpu(dout, "token grad");
  f32_gpu(dpos, "position grad");
  f32_gpu(dcls, "class token grad");
  const int64_t B = dout.size(0), T = dout.size(1), D = dout.size(2);
  at::Tensor dp = at::empty({B, T - 1, D}, dout.options());
  kern::assemble_tokens_bwd(dout.data_ptr(), (int)B, (int)(T - 1), (int)D, dp.data_ptr(), dpos.data_ptr<float>(),
                            dcls.data_ptr<float>(), stream_of(dout));
  return dp;
}

at::Tensor cls_rows(const at::Tensor& x, int64_t B, int64_t T, bool reverse) {
  bf16_gpu(x, "token rows");
  const int64_t D = x.size(-1);
  at::Tensor y = reverse ? at::zeros({B, T, D}, x.options()) : at::empty({B, D}, x.options());
  kern::cls_rows(x.data_ptr(), (int)B, (int)T, (int)D, y.data_ptr(), reverse, stream_of(x));
  return y;
}

// ------------------------------------------------------------------ fp8 (e4m3) GEMM path
std::tuple<at::Tensor, at::Tensor> fp8_quantize(const at::Tensor& x, bool transpose) {
  bf16_gpu(x, "fp8 quantize input");
  RINGDP_CHECK(x.dim() == 2, "fp8_quantize: expected a 2-D tensor");
  const int64_t R = x.size(0), Cc = x.size(1);
  RINGDP_CHECK(Cc % 16 == 0 && (!transpose || R % 16 == 0), "fp8_quantize: dims must be multiples of 16");
  auto f = x.options().dtype(at::kFloat);
  at::Tensor amax = at::empty({1}, f), scale = at::empty({1}, f);
  at::Tensor q = transpose ? at::empty({Cc, R}, x.options().dtype(at::kByte)) : at::empty({R, Cc}, x.options().dtype(at::kByte));
  kern::fp8_amax(x.data_ptr(), x.numel(), amax.data_ptr<float>(), stream_of(x));
  kern::fp8_quantize(x.data_ptr(), R, Cc, transpose, amax.data_ptr<float>(), q.data_ptr(), scale.data_ptr<float>(),
                     stream_of(x));
  return {q, scale};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> fp8_quantize_both(const at::Tensor& x) {
  bf16_gpu(x, "fp8 quantize input");
  RINGDP_CHECK(x.dim() == 2 && x.size(0) % 16 == 0 && x.size(1) % 16 == 0,
               "fp8_quantize_both: expected a 2-D tensor with dims % 16 == 0");
  const int64_t R = x.size(0), Cc = x.size(1);
  auto f = x.options().dtype(at::kFloat);
  at::Tensor amax = at::empty({1}, f), scale = at::empty({1}, f);
  at::Tensor q = at::empty({R, Cc}, x.options().dtype(at::kByte)), qt = at::empty({Cc, R}, x.options().dtype(at::kByte));
  kern::fp8_amax(x.data_ptr(), x.numel(), amax.data_ptr<float>(), stream_of(x));
  kern::fp8_quantize(x.data_ptr(), R, Cc, true, amax.data_ptr<float>(), qt.data_ptr(), scale.data_ptr<float>(),
                     stream_of(x), q.data_ptr());
  return {q, qt, scale};
}

int64_t fp8_delayed_slots(int64_t rows, int64_t cols) { return kern::fp8_quant_tiles(rows, cols); }

std::tuple<at::Tensor, at::Tensor, at::Tensor> fp8_quantize_both_delayed(const at::Tensor& x, at::Tensor hist,
                                                                        bool init,
                                                                        const c10::optional<at::Tensor>& colsum,
                                                                        const c10::optional<at::Tensor>& gelu_pre,
                                                                        bool roll) {
  bf16_gpu(x, "fp8 quantize input");
  RINGDP_CHECK(x.dim() == 2 && x.size(0) % 16 == 0 && x.size(1) % 16 == 0,
               "fp8_quantize_both_delayed: expected a 2-D tensor with dims % 16 == 0");
  f32_gpu(hist, "fp8 amax history");
  const int64_t R = x.size(0), Cc = x.size(1);
  RINGDP_CHECK(hist.is_contiguous() && hist.numel() == 1 + fp8_delayed_slots(R, Cc),
               "fp8 amax history: expected 1 + fp8_delayed_slots(rows, cols) contiguous floats");
  at::Tensor scale = at::empty({1}, x.options().dtype(at::kFloat));
  at::Tensor q = at::empty({R, Cc}, x.options().dtype(at::kByte)), qt = at::empty({Cc, R}, x.options().dtype(at::kByte));
  at::Tensor part;
  if (colsum.has_value() && colsum->defined()) {  // column sums of x (a bias gradient) from the same pass
    f32_gpu(*colsum, "fp8 quantize colsum");
    RINGDP_CHECK(colsum->numel() == Cc && colsum->is_contiguous(), "fp8 quantize colsum: expected [cols] floats");
    part = at::empty({kern::fp8_quant_row_tiles(R), Cc}, x.options().dtype(at::kFloat));
  }
  // gelu_pre: quantise x * GELU'(gelu_pre) (an fp8 linear's GELU backward folded into the pass over its gradient)
  const void* pre = nullptr;
  at::Tensor src = x;
  if (gelu_pre.has_value() && gelu_pre->defined()) {
    bf16_gpu(*gelu_pre, "fp8 quantize gelu pre-activation");
    RINGDP_CHECK(gelu_pre->sizes() == x.sizes() && gelu_pre->is_contiguous() && x.is_contiguous(),
                 "fp8 quantize gelu pre-activation: expected a contiguous tensor of x's shape");
    if (init) {  // the site's first amax is measured on the finished gradient: materialise it once
      src = at::empty_like(x);
      kern::gelu_bwd(x.data_ptr(), gelu_pre->data_ptr(), x.numel(), src.data_ptr(), stream_of(x));
    } else {
      pre = gelu_pre->data_ptr();
    }
  }
  kern::fp8_quantize_delayed(src.data_ptr(), R, Cc, hist.data_ptr<float>(), init, qt.data_ptr(), scale.data_ptr<float>(),
                             q.data_ptr(), stream_of(x), part.defined() ? part.data_ptr<float>() : nullptr, pre, roll);
  if (part.defined())
    kern::rowsum_f32(part.data_ptr<float>(), (int)part.size(0), Cc, colsum->data_ptr<float>(), stream_of(x));
  return {q, qt, scale};
}

void fp8_roll_many(const at::Tensor& hists, const at::Tensor& ns) {
  RINGDP_CHECK(hists.is_cuda() && ns.is_cuda() && hists.scalar_type() == at::kLong && ns.scalar_type() == at::kInt &&
                   hists.dim() == 1 && hists.sizes() == ns.sizes() && hists.is_contiguous() && ns.is_contiguous(),
               "fp8_roll_many: expected int64 pointer and int32 count vectors of one length on the GPU");
  kern::fp8_roll_many(reinterpret_cast<float* const*>(hists.data_ptr<int64_t>()), ns.data_ptr<int>(),
                      (int)hists.numel(), stream_of(hists));
}

void rowsum_f32(const at::Tensor& part, at::Tensor out) {
  f32_gpu(part, "rowsum input");
  f32_gpu(out, "rowsum output");
  RINGDP_CHECK(part.dim() == 2 && part.is_contiguous() && part.size(1) % 4 == 0 && out.numel() == part.size(1) &&
                   out.is_contiguous(),
               "rowsum_f32: expected contiguous fp32 [rows, cols % 4 == 0] and fp32 [cols]");
  kern::rowsum_f32(part.data_ptr<float>(), (int)part.size(0), part.size(1), out.data_ptr<float>(), stream_of(part));
}

void colsum_f32(const at::Tensor& x, at::Tensor out) {
  bf16_gpu(x, "colsum input");
  f32_gpu(out, "colsum output");
  RINGDP_CHECK(x.dim() == 2 && x.is_contiguous() && x.size(1) % 8 == 0 && out.numel() == x.size(1) &&
                   out.is_contiguous(),
               "colsum_f32: expected contiguous bf16 [rows, cols % 8 == 0] and fp32 [cols]");
  const int64_t R = x.size(0), Cc = x.size(1);
  at::Tensor part = at::empty({kern::colsum_parts(R), Cc}, out.options());
  kern::colsum_bf16(x.data_ptr(), R, Cc, part.data_ptr<float>(), stream_of(x));
  kern::rowsum_f32(part.data_ptr<float>(), (int)part.size(0), Cc, out.data_ptr<float>(), stream_of(x));
}

at::Tensor gemm_fp8(const at::Tensor& a, const at::Tensor& b, const at::Tensor& scale_a, const at::Tensor& scale_b,
                    int64_t M, int64_t N, int64_t K, bool out_bf16, const c10::optional<at::Tensor>& bias, int64_t act,
                    const c10::optional<at::Tensor>& residual, const c10::optional<at::Tensor>& preact) {
  gpu(a, "fp8 A");
  gpu(b, "fp8 B");
  dtype(a, at::kByte, "fp8 A");
  dtype(b, at::kByte, "fp8 B");
  f32_gpu(scale_a, "fp8 scale A");
  f32_gpu(scale_b, "fp8 scale B");
  RINGDP_CHECK(K % 16 == 0, "gemm_fp8: K must be a multiple of 16");
  RINGDP_CHECK(a.numel() >= M * K && b.numel() >= N * K, "gemm_fp8: operand smaller than described");
  at::Tensor c = at::empty({M, N}, a.options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat));
  auto e = make_epi(c.data_ptr(), N, 0, out_bf16);
  e.act = static_cast<int>(act);
  e.scale_a = scale_a.data_ptr<float>();
  e.scale_b = scale_b.data_ptr<float>();
  if (bias.has_value() && bias->defined()) {
    f32_gpu(*bias, "gemm bias");
    e.bias = bias->data_ptr<float>();
  }
  if (residual.has_value() && residual->defined()) {
    bf16_gpu(*residual, "gemm residual");
    e.residual = residual->data_ptr();
  }
  if (preact.has_value() && preact->defined()) {
    bf16_gpu(*preact, "gemm preact");
    e.preact = preact->data_ptr();
  }
  kern::GemmOperand A{a.data_ptr(), K, 0, false}, B{b.data_ptr(), K, 0, false};
  kern::gemm_fp8(A, B, 1, (int)M, (int)N, (int)K, e, 1, stream_of(a));
  return c;
}

void fp8_roll(at::Tensor hist) {
  f32_gpu(hist, "fp8 amax history");
  RINGDP_CHECK(hist.is_contiguous() && hist.numel() >= 1, "fp8_roll: expected a contiguous history");
  kern::fp8_roll(hist.data_ptr<float>(), (int)(hist.numel() - 1), stream_of(hist));
}

std::vector<at::Tensor> fp8_quantize_weights(const std::vector<at::Tensor>& ws, const std::vector<at::Tensor>& hists) {
  RINGDP_CHECK(ws.size() == hists.size() && !ws.empty(), "fp8_quantize_weights: one history per weight");
  std::vector<at::Tensor> out;
  kern::QuantTTable t{};
  auto flush = [&](hipStream_t st) {
    if (t.n > 0) kern::fp8_quantize_multi(t, st);
    t = kern::QuantTTable{};
  };
  for (size_t i = 0; i < ws.size(); ++i) {
    const at::Tensor& w = ws[i];
    const at::Tensor& h = hists[i];
    f32_gpu(w, "fp8 weight");
    f32_gpu(h, "fp8 amax history");
    RINGDP_CHECK(w.dim() == 2 && w.is_contiguous() && w.size(0) % 16 == 0 && w.size(1) % 16 == 0,
                 "fp8_quantize_weights: contiguous fp32 [rows, cols] with dims % 16 == 0");
    const int64_t R = w.size(0), Cc = w.size(1);
    RINGDP_CHECK(h.is_contiguous() && h.numel() == 1 + fp8_delayed_slots(R, Cc), "fp8_quantize_weights: history size");
    at::Tensor q = at::empty({R, Cc}, w.options().dtype(at::kByte)), qt = at::empty({Cc, R}, w.options().dtype(at::kByte));
    at::Tensor scale = at::empty({1}, w.options());
    out.push_back(q);
    out.push_back(qt);
    out.push_back(scale);
    if (t.n == kern::kQuantTMax) flush(stream_of(w));
    kern::QuantTEntry& e = t.e[t.n++];
    e.src = w.data_ptr<float>();
    e.rows = R;
    e.cols = Cc;
    e.hist = h.data_ptr<float>();
    e.q = static_cast<uint8_t*>(q.data_ptr());
    e.qt = static_cast<uint8_t*>(qt.data_ptr());
    e.scale = scale.data_ptr<float>();
    e.tile0 = t.total_tiles;
    t.total_tiles += (int)kern::fp8_quant_tiles(R, Cc);
  }
  flush(stream_of(ws[0]));
  return out;
}

int64_t gemm_fp8_q8_slots(int64_t M, int64_t N) { return kern::gemm_fp8_q8_slots((int)M, (int)N); }

std::tuple<at::Tensor, at::Tensor, at::Tensor> gemm_fp8_quant_out(
    const at::Tensor& a, const at::Tensor& b, const at::Tensor& scale_a, const at::Tensor& scale_b, int64_t M,
    int64_t N, int64_t K, const c10::optional<at::Tensor>& bias, int64_t act, const c10::optional<at::Tensor>& preact,
    at::Tensor hist, const c10::optional<at::Tensor>& colsum) {
  gpu(a, "fp8 A");
  gpu(b, "fp8 B");
  dtype(a, at::kByte, "fp8 A");
  dtype(b, at::kByte, "fp8 B");
  f32_gpu(scale_a, "fp8 scale A");
  f32_gpu(scale_b, "fp8 scale B");
  f32_gpu(hist, "fp8 amax history");
  RINGDP_CHECK(M % 16 == 0 && N % 16 == 0 && K % 128 == 0, "gemm_fp8_quant_out: M, N % 16 and K % 128 must be 0");
  RINGDP_CHECK(a.numel() >= M * K && b.numel() >= N * K, "gemm_fp8_quant_out: operand smaller than described");
  RINGDP_CHECK(act == 0 || act == 2 || act == 3, "gemm_fp8_quant_out: act must be 0, 2 (GELU) or 3 (GELU backward)");
  RINGDP_CHECK(hist.is_contiguous() && hist.numel() == 1 + kern::gemm_fp8_q8_slots((int)M, (int)N),
               "gemm_fp8_quant_out: history must hold 1 + gemm_fp8_q8_slots(M, N) floats");
  auto e = make_epi(nullptr, N, 0, true);
  e.act = static_cast<int>(act);
  e.scale_a = scale_a.data_ptr<float>();
  e.scale_b = scale_b.data_ptr<float>();
  if (bias.has_value() && bias->defined()) {
    f32_gpu(*bias, "gemm bias");
    RINGDP_CHECK(bias->numel() == N && reinterpret_cast<uintptr_t>(bias->data_ptr()) % 16 == 0, "gemm bias: [N], 16-B aligned");
    e.bias = bias->data_ptr<float>();
  }
  if (act == 2 || act == 3) {
    RINGDP_CHECK(preact.has_value() && preact->defined(), "gemm_fp8_quant_out: act 2 / 3 need the pre-activation");
    bf16_gpu(*preact, "gemm preact");
    RINGDP_CHECK(preact->numel() == M * N && preact->is_contiguous(), "gemm preact: [M][N] contiguous");
    e.preact = preact->data_ptr();
  }
  at::Tensor q = at::empty({M, N}, a.options()), qt = at::empty({N, M}, a.options());
  at::Tensor scale = at::empty({1}, a.options().dtype(at::kFloat));
  at::Tensor part;
  if (colsum.has_value() && colsum->defined()) {
    f32_gpu(*colsum, "gemm colsum");
    RINGDP_CHECK(colsum->numel() == N && colsum->is_contiguous(), "gemm colsum: [N] floats");
    part = at::empty({kern::gemm_fp8_colsum_part_rows((int)M), N}, a.options().dtype(at::kFloat));
    e.colsum_part = part.data_ptr<float>();
  }
  e.q8 = static_cast<uint8_t*>(q.data_ptr());
  e.q8t = static_cast<uint8_t*>(qt.data_ptr());
  e.q8_amax = hist.data_ptr<float>();
  e.q8_scale = scale.data_ptr<float>();
  e.q8_tmax = hist.data_ptr<float>() + 1;
  kern::GemmOperand A{a.data_ptr(), K, 0, false}, B{b.data_ptr(), K, 0, false};
  kern::gemm_fp8(A, B, 1, (int)M, (int)N, (int)K, e, 1, stream_of(a));
  if (part.defined())
    kern::rowsum_f32(part.data_ptr<float>(), (int)part.size(0), N, colsum->data_ptr<float>(), stream_of(a));
  return {q, qt, scale};
}

void set_fp8_tile_mode(int64_t mode) { kern::set_fp8_tile_mode((int)mode); }
void set_bf16_tile_mode(int64_t mode) { kern::set_bf16_tile_mode((int)mode); }

void gemm_fp8_splitk_f32(const at::Tensor& a, const at::Tensor& b, const at::Tensor& scale_a,
                         const at::Tensor& scale_b, int64_t M, int64_t N, int64_t K, int64_t splits, at::Tensor out) {
  gpu(a, "fp8 A");
  gpu(b, "fp8 B");
  f32_gpu(out, "fp8 gemm out");
  RINGDP_CHECK(K % 16 == 0 && out.numel() == M * N, "gemm_fp8_splitk_f32: bad shapes");
  splits = std::max<int64_t>(1, std::min<int64_t>(splits, std::max<int64_t>(1, K / 128)));
  splits = kern::gemm_fp8_pick_splits((int)M, (int)N, (int)K, (int)splits);
  at::Tensor part = at::empty({splits, M, N}, out.options());
  kern::GemmEpilogue e{};
  e.mode = kern::GemmEpilogue::kSplitK;
  e.partial = part.data_ptr<float>();
  e.scale_a = scale_a.data_ptr<float>();
  e.scale_b = scale_b.data_ptr<float>();
  kern::GemmOperand A{a.data_ptr(), K, 0, false}, B{b.data_ptr(), K, 0, false};
  kern::gemm_fp8(A, B, 1, (int)M, (int)N, (int)K, e, (int)splits, stream_of(a));
  // split boundaries are in 64-slot (128-byte) units; sum only the planes that were written
  const int64_t kslots = K / 2;
  const int64_t kps = ((kslots + splits - 1) / splits + 63) / 64 * 64;
  const int64_t used = (kslots + kps - 1) / kps;
  kern::splitk_sum(part.data_ptr<float>(), (int)used, M * N, out.data_ptr<float>(), stream_of(a));
}

at::Tensor patchify(const at::Tensor& x, int64_t P) {
  gpu(x, "images");
  RINGDP_CHECK(x.dim() == 4 && (x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16),
               "patchify: expected NCHW float/bf16 images");
  const int64_t B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  RINGDP_CHECK(H % P == 0 && W % P == 0 && (C * P * P) % 8 == 0, "patchify: bad patch size");
  at::Tensor out = at::empty({B * (H / P) * (W / P), C * P * P}, x.options().dtype(at::kBFloat16));
  kern::patchify(x.data_ptr(), x.scalar_type() == at::kBFloat16, (int)B, (int)C, (int)H, (int)W, (int)P,
                 out.data_ptr(), stream_of(x));
  return out;
}

}  // namespace ops
}  // namespace ringdp
