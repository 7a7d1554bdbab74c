// Tensor-level wrappers around ringdp's HIP kernels (shape/dtype/device checks + launch on the
// caller's current HIP stream).  Every op fails loudly on bad input instead of falling back.
#pragma once

#include <ATen/ATen.h>

#include <tuple>
#include <vector>

namespace ringdp {
namespace ops {

// dst = src converted (fp32 <-> bf16 / fp16).  GPU: ringdp cast kernel; CPU: ATen copy.
void cast_copy(at::Tensor dst, const at::Tensor& src);
// fp32 -> bf16 copies of many tensors in one launch
std::vector<at::Tensor> cast_bf16_multi(const std::vector<at::Tensor>& srcs);
// fp32 matrices -> [bf16 W, bf16 W^T] pairs in one launch
std::vector<at::Tensor> cast_bf16_t_multi(const std::vector<at::Tensor>& srcs);

struct SgdHyper {
  double lr = 0.01;
  double momentum = 0.0;
  double dampening = 0.0;
  double weight_decay = 0.0;
  bool nesterov = false;
  bool maximize = false;
};
// One fused SGD step over flat fp32 buffers (momentum_buf may be undefined when momentum == 0).
void sgd_flat(at::Tensor param, const at::Tensor& grad, const c10::optional<at::Tensor>& momentum_buf,
              const SgdHyper& h, bool first_step, const c10::optional<at::Tensor>& lr_tensor,
              const c10::optional<at::Tensor>& grad_scale,
              const c10::optional<at::Tensor>& packed, const std::vector<int64_t>& pack_offsets);
// Multi-tensor SGD: one launch for lists of (possibly non-adjacent) fp32 tensors.
void sgd_multi(std::vector<at::Tensor> params, std::vector<at::Tensor> grads,
               std::vector<at::Tensor> bufs, const SgdHyper& h, bool first_step,
               const c10::optional<at::Tensor>& lr_tensor,
               const c10::optional<at::Tensor>& grad_scale);

// Cached multi-tensor table (graph-capture safe: build once outside capture, run many times).
std::tuple<at::Tensor, int64_t, int64_t> sgd_multi_build(std::vector<at::Tensor> params,
                                                         std::vector<at::Tensor> grads,
                                                         std::vector<at::Tensor> bufs,
                                                         bool with_momentum);
void sgd_multi_run(const at::Tensor& table, int64_t nchunks, int64_t table_bytes,
                   const SgdHyper& h, bool first_step, const c10::optional<at::Tensor>& lr_tensor,
                   const c10::optional<at::Tensor>& grad_scale);

// Cross entropy: returns (loss, lse, workspace); workspace holds the denominator for backward.
std::tuple<at::Tensor, at::Tensor, at::Tensor> cross_entropy_fwd(const at::Tensor& logits,
                                                                 const at::Tensor& labels,
                                                                 int64_t ignore_index,
                                                                 double label_smoothing,
                                                                 int64_t reduction);
at::Tensor cross_entropy_bwd(const at::Tensor& logits, const at::Tensor& labels,
                             const at::Tensor& lse, const at::Tensor& ws,
                             const at::Tensor& grad_out, int64_t ignore_index,
                             double label_smoothing, int64_t reduction);

// MNIST ConvNet blocks (see csrc/kernels/convnet.hip for the F1/F2/F3 split).
at::Tensor cn_pack_weights(const at::Tensor& w1, const at::Tensor& w2, const at::Tensor& w3,
                           const at::Tensor& wfc, const c10::optional<at::Tensor>& out);
std::tuple<at::Tensor, at::Tensor> cn_conv1_fwd(const at::Tensor& x, const at::Tensor& packed,
                                                const at::Tensor& b1, double mean, double std,
                                                double in_scale);
std::tuple<at::Tensor, at::Tensor> cn_conv2_fwd(const at::Tensor& a1, const at::Tensor& packed,
                                                const at::Tensor& b2);
// conv1 forward that also packs every layer's weights in the same launch: (a1, idx1, packed)
// Whole ConvNet forward in one launch: writes a1 / idx1 / a2 / idx2 / packed (cn_forward_buffers) and
// returns logits, a3, idx3.
std::vector<at::Tensor> cn_forward_buffers(const at::Tensor& x);
std::tuple<at::Tensor, at::Tensor, at::Tensor> cn_forward_fused(
    const at::Tensor& x, const at::Tensor& w1, const at::Tensor& b1, const at::Tensor& w2, const at::Tensor& b2,
    const at::Tensor& w3, const at::Tensor& b3, const at::Tensor& wfc, const at::Tensor& bfc, double mean, double std,
    double in_scale, at::Tensor a1, at::Tensor idx1, at::Tensor a2, at::Tensor idx2, at::Tensor packed,
    bool do_pack);
std::tuple<at::Tensor, at::Tensor, at::Tensor> cn_conv1_fwd_pack(const at::Tensor& x, const at::Tensor& w1,
                                                                 const at::Tensor& w2, const at::Tensor& w3,
                                                                 const at::Tensor& wfc, const at::Tensor& b1,
                                                                 double mean, double std, double in_scale);
std::tuple<at::Tensor, at::Tensor, at::Tensor> cn_conv3_fc_fwd(const at::Tensor& a2,
                                                               const at::Tensor& packed,
                                                               const at::Tensor& b3,
                                                               const at::Tensor& bfc);
at::Tensor cn_conv3_fc_bwd(const at::Tensor& a2, const at::Tensor& idx2, const at::Tensor& a3,
                           const at::Tensor& idx3, const at::Tensor& wfc, const at::Tensor& dlogits,
                           const at::Tensor& packed, bool need_dz2, at::Tensor dw3, at::Tensor db3,
                           at::Tensor dwfc, at::Tensor dbfc, bool defer_reduce);
// Same with the cross entropy backward fused into the fc1 backward (logits / lse / ws from
// cross_entropy_fwd).  defer_reduce: the weight-gradient reduction is held back and launched
// together with the next cn_conv12_bwd's on this device (or by cn_flush_reduce).
at::Tensor cn_conv3_fc_ce_bwd(const at::Tensor& a2, const at::Tensor& idx2, const at::Tensor& a3,
                              const at::Tensor& idx3, const at::Tensor& wfc, const at::Tensor& logits,
                              const at::Tensor& labels, const at::Tensor& lse, const at::Tensor& ws,
                              const at::Tensor& grad_out, int64_t ignore_index, double smoothing, int64_t reduction,
                              const at::Tensor& packed, bool need_dz2, at::Tensor dw3, at::Tensor db3,
                              at::Tensor dwfc, at::Tensor dbfc, bool defer_reduce);
void cn_flush_reduce(int64_t device);
bool cn_reduce_pending(int64_t device);
int64_t cn_merged_reductions();
at::Tensor cn_conv2_bwd(const at::Tensor& a1, const at::Tensor& dz2, const at::Tensor& packed,
                        bool need_da1, at::Tensor dw2, at::Tensor db2);
void cn_conv12_bwd(const at::Tensor& x, const at::Tensor& idx1, const at::Tensor& a1, const at::Tensor& dz2,
                   const at::Tensor& packed, at::Tensor dw2, at::Tensor db2, at::Tensor dw1, at::Tensor db1,
                   double mean, double std, double in_scale);
void cn_conv1_wgrad(const at::Tensor& x, const at::Tensor& da1, const at::Tensor& idx1, at::Tensor dw1,
                    at::Tensor db1, double mean, double std, double in_scale);

// Device input pipeline: gather + random crop/flip + ToTensor/Normalize in one launch.
std::tuple<at::Tensor, at::Tensor> gather_augment(const at::Tensor& x, const c10::optional<at::Tensor>& labels,
                                                  const at::Tensor& idx, int64_t pad, bool flip,
                                                  std::vector<double> mean, std::vector<double> std,
                                                  int64_t seed, bool nhwc, at::ScalarType out_dtype);

std::tuple<at::Tensor, at::Tensor> synth_u8_images(int64_t B, int64_t H, int64_t W,
                                                   int64_t num_classes, int64_t seed,
                                                   at::Device device);

// fp32 NCHW conv / pool (conv_f32_ops.cpp)
at::Tensor f32_conv_fwd(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                        int64_t pad, double mean, double std);
std::tuple<at::Tensor, at::Tensor> f32_conv_pool_fwd(const at::Tensor& x, const at::Tensor& w,
                                                     const c10::optional<at::Tensor>& bias, int64_t pad, double mean,
                                                     double std, int64_t stride);
std::tuple<at::Tensor, at::Tensor> f32_conv1_pool_fwd(const at::Tensor& x, const at::Tensor& w1, const at::Tensor& b1,
                                                      double mean, double std);
void f32_conv1_wgrad(const at::Tensor& x, const at::Tensor& da1, const at::Tensor& code1, double mean, double std,
                     at::Tensor& dw1, at::Tensor& db1);
at::Tensor f32_conv_dgrad(const at::Tensor& dz, const at::Tensor& w, int64_t H, int64_t W, int64_t pad);
void f32_conv_wgrad(const at::Tensor& dz, const at::Tensor& x, int64_t pad, double mean, double std,
                    at::Tensor& dw, const c10::optional<at::Tensor>& db);
at::Tensor f32_conv_dgrad_pool2s1_bwd(const at::Tensor& dz, const at::Tensor& w, const at::Tensor& code);
std::tuple<at::Tensor, std::vector<int64_t>> f32_conv_wgrad_slab(const at::Tensor& dz, const at::Tensor& x,
                                                                 int64_t pad, double mean, double std,
                                                                 const at::Tensor& dw, bool with_bias);
std::tuple<at::Tensor, std::vector<int64_t>> f32_conv1_wgrad_slab(const at::Tensor& x, const at::Tensor& da1,
                                                                  const at::Tensor& code1, double mean, double std);
std::tuple<at::Tensor, at::Tensor> f32_fc_ce_pool3_bwd(const at::Tensor& logits, const at::Tensor& labels,
                                                       const at::Tensor& lse, const at::Tensor& ws,
                                                       const at::Tensor& grad_out, int64_t ignore_index, double eps,
                                                       int64_t reduction, const at::Tensor& wfc,
                                                       const at::Tensor& code3);
void f32_slab_reduce_multi(const std::vector<at::Tensor>& slabs, const std::vector<std::vector<int64_t>>& meta,
                           const std::vector<at::Tensor>& dws, const std::vector<c10::optional<at::Tensor>>& dbs);
std::tuple<at::Tensor, at::Tensor> f32_pool_relu_fwd(const at::Tensor& z, int64_t k, int64_t stride);
at::Tensor f32_pool_relu_bwd(const at::Tensor& da, const at::Tensor& code, int64_t H, int64_t W, int64_t k,
                             int64_t stride);

at::Tensor transpose_bf16(const at::Tensor& x);
}  // namespace ops
}  // namespace ringdp
