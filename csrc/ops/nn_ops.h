// Tensor-level wrappers: generic GEMM, implicit-GEMM conv, NHWC layers (see nn_ops.cpp).
#pragma once

#include <ATen/ATen.h>

#include <tuple>

namespace ringdp {
namespace ops {

at::Tensor gemm(const at::Tensor& a, const at::Tensor& b, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                bool a_row, bool b_row, int64_t batch, int64_t a_bstride, int64_t b_bstride, bool out_bf16,
                const c10::optional<at::Tensor>& bias, int64_t act, const c10::optional<at::Tensor>& residual,
                const c10::optional<at::Tensor>& preact, double alpha, const c10::optional<at::Tensor>& out,
                const c10::optional<at::Tensor>& colsum = c10::nullopt);
at::Tensor gemm_splitk_f32(const at::Tensor& a, const at::Tensor& b, int64_t M, int64_t N, int64_t K, int64_t lda,
                           int64_t ldb, bool a_row, bool b_row, int64_t splits, const at::Tensor& out);
std::tuple<at::Tensor, at::Tensor> pack_conv_weight(const at::Tensor& w, int64_t cpad);
// several weights in one launch: returns [krsc0, crsk0, krsc1, crsk1, ...]
std::vector<at::Tensor> pack_conv_weights(const std::vector<at::Tensor>& ws, const std::vector<int64_t>& cpads);
std::tuple<at::Tensor, at::Tensor> conv2d_fwd(const at::Tensor& x, const at::Tensor& w_krsc, int64_t stride,
                                              int64_t pad, int64_t dil, bool want_stats);
at::Tensor conv2d_dgrad(const at::Tensor& dz, const at::Tensor& w_crsk, int64_t H, int64_t W, int64_t stride,
                        int64_t pad, int64_t dil, const c10::optional<at::Tensor>& residual);
void conv2d_wgrad(const at::Tensor& dz, const at::Tensor& x, at::Tensor dw, int64_t stride, int64_t pad, int64_t dil);
at::Tensor nchw_to_nhwc(const at::Tensor& x, int64_t cpad);
std::tuple<at::Tensor, at::Tensor> bn_fwd_train(const at::Tensor& z, const at::Tensor& sums, const at::Tensor& gamma,
                                                const at::Tensor& beta, const c10::optional<at::Tensor>& running_mean,
                                                const c10::optional<at::Tensor>& running_var, double eps,
                                                double momentum, const c10::optional<at::Tensor>& residual,
                                                bool relu, const c10::optional<at::Tensor>& num_batches_tracked);
at::Tensor bn_fwd_eval(const at::Tensor& z, const at::Tensor& scale_shift, const c10::optional<at::Tensor>& residual,
                       bool relu);
std::tuple<at::Tensor, at::Tensor> bn_bwd(const at::Tensor& dy, const at::Tensor& y, const at::Tensor& z,
                                          const at::Tensor& save, const at::Tensor& gamma, bool relu,
                                          at::Tensor dgamma, at::Tensor dbeta, bool need_g);
std::tuple<at::Tensor, at::Tensor> maxpool2d_fwd(const at::Tensor& x, int64_t k, int64_t stride, int64_t pad);
at::Tensor maxpool2d_bwd(const at::Tensor& dy, const at::Tensor& arg, int64_t H, int64_t W, int64_t k,
                         int64_t stride, int64_t pad);
at::Tensor avgpool_fwd(const at::Tensor& x);
at::Tensor avgpool_bwd(const at::Tensor& dy, int64_t H, int64_t W);
// classifier head at few classes (kern::head_ok): (logits fp32 [N, J], pooled fp32 [N, C])
std::tuple<at::Tensor, at::Tensor> head_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b);
// backward from dl [N, J], or (dl undefined) from the cross-entropy forward's (logits, labels, lse, ws, grad_out);
// returns dx [N, H, W, C] bf16, writes dw / db
at::Tensor head_bwd(const c10::optional<at::Tensor>& dl, const c10::optional<at::Tensor>& logits,
                    const c10::optional<at::Tensor>& labels, const c10::optional<at::Tensor>& lse,
                    const c10::optional<at::Tensor>& ws, const c10::optional<at::Tensor>& grad_out,
                    int64_t ignore_index, double eps, int64_t reduction, const at::Tensor& pooled,
                    const at::Tensor& w, int64_t H, int64_t W, at::Tensor dw, at::Tensor db);
at::Tensor add_bf16(const at::Tensor& a, const at::Tensor& b);

std::tuple<at::Tensor, at::Tensor> layernorm_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b,
                                                 double eps);
// LayerNorm forward writing e4m3 (delayed scaling, hist = [amax, per-64-row-block maxima]): [stats, q, qt, scale]
std::vector<at::Tensor> layernorm_fwd_q8(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b, double eps,
                                         at::Tensor hist);
int64_t layernorm_q8_slots(int64_t rows);
// layernorm_bwd plus per-block column sums of dx: returns [dx, colsum partials [blocks][D]]
std::vector<at::Tensor> layernorm_bwd_colsum(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& stats,
                                             const at::Tensor& w, const c10::optional<at::Tensor>& dres, at::Tensor dw,
                                             at::Tensor db);
at::Tensor layernorm_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& stats, const at::Tensor& w,
                         const c10::optional<at::Tensor>& dres, at::Tensor dw, at::Tensor db);
std::tuple<at::Tensor, at::Tensor, at::Tensor> qkv_split(const at::Tensor& qkv, int64_t B, int64_t T, int64_t H,
                                                         int64_t Tp);
at::Tensor qkv_merge(const at::Tensor& dq, const at::Tensor& dk, const at::Tensor& dv, int64_t B, int64_t T);
at::Tensor heads_to_rows(const at::Tensor& o, int64_t B, int64_t T);
at::Tensor rows_to_heads(const at::Tensor& rows, int64_t B, int64_t T, int64_t H, int64_t Tp);
at::Tensor softmax_fwd(const at::Tensor& scores, int64_t T, double scale);
at::Tensor attn_bwd_ds(const at::Tensor& dout, const at::Tensor& v, const at::Tensor& p, double scale);
at::Tensor attn_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                    const at::Tensor& p, int64_t B, int64_t T, int64_t H, double scale);
std::vector<at::Tensor> attn_fwd_rows(const at::Tensor& qkv, int64_t B, int64_t T, int64_t H, double scale,
                                      bool recompute = false);
at::Tensor attn_bwd_rows(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& p, int64_t B, int64_t T,
                         int64_t H, double scale,
                         const c10::optional<at::Tensor>& colsum_part = c10::nullopt);
std::vector<at::Tensor> attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, int64_t T,
                                 double scale);
at::Tensor softmax_bwd(const at::Tensor& p, const at::Tensor& dp, int64_t T, double scale);
at::Tensor gelu_bwd(const at::Tensor& dy, const at::Tensor& pre);
at::Tensor assemble_tokens(const at::Tensor& patches, const at::Tensor& cls, const at::Tensor& pos);
at::Tensor assemble_tokens_bwd(const at::Tensor& dout, at::Tensor dpos, at::Tensor dcls);
at::Tensor cls_rows(const at::Tensor& x, int64_t B, int64_t T, bool reverse);
at::Tensor patchify(const at::Tensor& x, int64_t P);
std::tuple<at::Tensor, at::Tensor> fp8_quantize(const at::Tensor& x, bool transpose);
std::tuple<at::Tensor, at::Tensor, at::Tensor> fp8_quantize_both(const at::Tensor& x);
int64_t fp8_delayed_slots(int64_t rows, int64_t cols);
std::tuple<at::Tensor, at::Tensor, at::Tensor> fp8_quantize_both_delayed(const at::Tensor& x, at::Tensor hist,
                                                                        bool init,
                                                                        const c10::optional<at::Tensor>& colsum,
                                                                        const c10::optional<at::Tensor>& gelu_pre,
                                                                        bool roll = true);
// hists: int64 [count] device pointers to the sites' history tensors, ns: int32 [count] their tile counts
void fp8_roll_many(const at::Tensor& hists, const at::Tensor& ns);
// fp8 GEMM whose epilogue writes e4m3 (row-major and transposed) with delayed scaling instead of bf16 C:
// hist = {amax to scale by, the launch's per-(tile, wave) maxima}; act 2 stores the pre-activation into
// preact, act 3 reads it (GELU backward); colsum (nullable) <- column sums of the quantised-from values
int64_t gemm_fp8_q8_slots(int64_t M, int64_t N);
void fp8_roll(at::Tensor hist);
// every weight's delayed-scaling e4m3 copy (row-major, transposed, scale) in one launch: returns [q, qt, scale] * n
std::vector<at::Tensor> fp8_quantize_weights(const std::vector<at::Tensor>& ws, const std::vector<at::Tensor>& hists);
std::tuple<at::Tensor, at::Tensor, at::Tensor> gemm_fp8_quant_out(
    const at::Tensor& a, const at::Tensor& b, const at::Tensor& scale_a, const at::Tensor& scale_b, int64_t M,
    int64_t N, int64_t K, const c10::optional<at::Tensor>& bias, int64_t act, const c10::optional<at::Tensor>& preact,
    at::Tensor hist, const c10::optional<at::Tensor>& colsum);
void colsum_f32(const at::Tensor& x, at::Tensor out);
void rowsum_f32(const at::Tensor& part, at::Tensor out);  // out[c] = sum_r part[r][c] (fixed order)
at::Tensor gemm_fp8(const at::Tensor& a, const at::Tensor& b, const at::Tensor& scale_a, const at::Tensor& scale_b,
                    int64_t M, int64_t N, int64_t K, bool out_bf16, const c10::optional<at::Tensor>& bias, int64_t act,
                    const c10::optional<at::Tensor>& residual, const c10::optional<at::Tensor>& preact);
void set_bf16_tile_mode(int64_t mode);
void set_fp8_tile_mode(int64_t mode);
void gemm_fp8_splitk_f32(const at::Tensor& a, const at::Tensor& b, const at::Tensor& scale_a,
                         const at::Tensor& scale_b, int64_t M, int64_t N, int64_t K, int64_t splits, at::Tensor out);

}  // namespace ops
}  // namespace ringdp
