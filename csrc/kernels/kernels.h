// Host-callable launchers for ringdp's CDNA4 HIP kernels (no torch types here: raw pointers +
// hipStream_t, so the .hip translation units stay free of PyTorch headers).
#pragma once

#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace ringdp {
namespace kern {

// ---------------------------------------------------------------- elementwise / optimizer
void cast_f32_to_bf16(const float* src, void* dst, int64_t n, hipStream_t s);
void cast_bf16_to_f32(const void* src, float* dst, int64_t n, hipStream_t s);
void cast_f32_to_f16(const float* src, void* dst, int64_t n, hipStream_t s);
void cast_f16_to_f32(const void* src, float* dst, int64_t n, hipStream_t s);

struct SgdArgs {
  float lr;
  float momentum;
  float dampening;
  float weight_decay;
  bool nesterov;
  bool maximize;
  bool first_step;        // momentum buffer := grad
  const float* lr_ptr;    // optional device-resident lr (overrides `lr`; graph-capture friendly)
  const float* grad_scale_ptr;  // optional device scalar: grad *= 1/(*grad_scale_ptr)
};
// One kernel over a flat fp32 range (params / grads / momentum laid out identically).
void sgd_flat(float* p, const float* g, float* m, int64_t n, const SgdArgs& a, hipStream_t s);
// Multi-tensor: device table of {p, g, m, n} + chunk list {tensor, start}; one launch.
struct SgdTensor {
  float* p;
  const float* g;
  float* m;
  int64_t n;
};
void sgd_multi(const SgdTensor* table, const int64_t* chunks, int64_t nchunks, int64_t chunk_elems,
               const SgdArgs& a, hipStream_t s);

// Deterministic split-K reduction: out[i] = sum_s slabs[s * n + i] (fixed order).
void splitk_reduce(const float* slabs, int nslices, int64_t n, float* out, hipStream_t s);

// ---------------------------------------------------------------- cross entropy
// logits [B, C] fp32; labels int64 [B]; writes lse [B], loss scalar (or per-row for
// reduction none), denom (number of non-ignored rows) in ws.
// reduction: 0 none, 1 mean, 2 sum.
void cross_entropy_fwd(const float* logits, const int64_t* labels, int B, int C, int ignore_index,
                       float label_smoothing, int reduction, float* lse, float* loss,
                       float* partials, unsigned* counter, int nparts, hipStream_t s);
void cross_entropy_bwd(const float* logits, const int64_t* labels, const float* lse,
                       const float* grad_out, const float* denom, int B, int C, int ignore_index,
                       float label_smoothing, int reduction, float* dlogits, hipStream_t s);

// ---------------------------------------------------------------- MNIST ConvNet
// Activations are NHWC bf16; weights are PyTorch-layout fp32 master weights.
// conv1 (1->32, k5, pad1) + ReLU + MaxPool(2,2): x [B,28,28] (u8 or f32) -> a1 [B,13,13,32].
void convnet_conv1_fwd(const void* x, bool x_is_u8, const float* w, const float* b, void* a1,
                       uint8_t* idx1, int B, float mean, float inv_std, float in_scale,
                       hipStream_t s);
// conv1 weight/bias grad from d(a1) (unpool + relu mask via idx1/a1).
int64_t convnet_conv1_wgrad_slab_floats(int B, int* nslices);
void convnet_conv1_wgrad(const void* x, bool x_is_u8, const void* da1, const uint8_t* idx1,
                         const void* a1, int B, float mean, float inv_std, float in_scale,
                         float* slabs, int nslices, float* dw, float* db, hipStream_t s);

// layer: 2 -> conv2 (32->64 @13x13, pool k2 s1 -> 10x10), 3 -> conv3 (64->128 @10x10, pool k2 s2
// -> 4x4).
void convnet_conv_fwd(int layer, const void* in, const float* w, const float* b, void* out,
                      uint8_t* idx, int B, hipStream_t s);
int64_t convnet_conv_wgrad_slab_floats(int layer, int B, int* nslices);
// Backward of conv+relu+pool: dout = d(pooled output).  Writes din (may be null to skip the
// data gradient), and dw/db via slabs + reduction.
void convnet_conv_bwd(int layer, const void* in, const float* w, const void* dout,
                      const uint8_t* idx, const void* out, void* din, int B, float* slabs,
                      int nslices, float* dw, float* db, hipStream_t s);

// fc (2048 -> 10) over the NHWC [B,4,4,128] activation; W is PyTorch [10, 2048] (CHW order).
void convnet_fc_fwd(const void* a3, const float* w, const float* b, float* logits, int B,
                    hipStream_t s);
int64_t convnet_fc_slab_floats(int B, int* nslices);
void convnet_fc_bwd(const void* a3, const float* w, const float* dlogits, void* da3, int B,
                    float* slabs, int nslices, float* dw, float* db, hipStream_t s);

// ---------------------------------------------------------------- data
// Synthetic MNIST-shaped batch (u8 images + labels) from a counter-based hash (deterministic).
void synth_u8_images(uint8_t* x, int64_t* labels, int B, int HW, int num_classes, uint64_t seed,
                     hipStream_t s);

}  // namespace kern
}  // namespace ringdp
