// Shared checks for the tensor-level op wrappers.
#pragma once

#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "../common.h"

namespace ringdp {
namespace ops {
namespace util {

inline hipStream_t stream_of(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.get_device()).stream();
}

inline void gpu(const at::Tensor& t, const char* name) {
  RINGDP_CHECK(t.defined(), name, ": undefined tensor");
  RINGDP_CHECK(t.is_cuda(), name, ": expected a GPU tensor (ringdp HIP kernel), got ", t.device());
  RINGDP_CHECK(t.is_contiguous(), name, ": expected a contiguous tensor");
}

inline void dtype(const at::Tensor& t, at::ScalarType d, const char* name) {
  RINGDP_CHECK(t.scalar_type() == d, name, ": expected dtype ", c10::toString(d), ", got ",
               c10::toString(t.scalar_type()));
}

inline void bf16_gpu(const at::Tensor& t, const char* name) {
  gpu(t, name);
  dtype(t, at::kBFloat16, name);
}

inline void f32_gpu(const at::Tensor& t, const char* name) {
  gpu(t, name);
  dtype(t, at::kFloat, name);
}

inline int num_cus(const at::Tensor& t) {
  static int cus = [&] {
    hipDeviceProp_t p;
    return hipGetDeviceProperties(&p, t.get_device()) == hipSuccess ? p.multiProcessorCount : 256;
  }();
  return cus;
}

}  // namespace util
}  // namespace ops
}  // namespace ringdp
