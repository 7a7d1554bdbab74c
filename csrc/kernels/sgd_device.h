// SGD element math shared by the optimizer kernels (elementwise.hip: flat / multi-tensor; convnet.hip: the
// flat step that also writes the ConvNet's packed bf16 weights).  Parity: torch/optim/sgd.py:343-380.
#pragma once

#include <hip/hip_runtime.h>

#include "kernels.h"

namespace ringdp {
namespace kern {

struct SgdDev {
  float lr, momentum, dampening, weight_decay, inv_scale;
  bool nesterov, maximize, first;
};

__device__ __forceinline__ SgdDev load_sgd(const SgdArgs& a) {
  SgdDev d;
  d.lr = a.lr_ptr ? *a.lr_ptr : a.lr;
  d.inv_scale = a.grad_scale_ptr ? 1.0f / *a.grad_scale_ptr : 1.0f;
  d.momentum = a.momentum;
  d.dampening = a.dampening;
  d.weight_decay = a.weight_decay;
  d.nesterov = a.nesterov;
  d.maximize = a.maximize;
  d.first = a.first_step;
  return d;
}

template <bool MOM>
__device__ __forceinline__ void sgd_elem(float& p, float g, float& m, const SgdDev& d) {
  g *= d.inv_scale;
  if (d.maximize) g = -g;
  if (d.weight_decay != 0.f) g = fmaf(d.weight_decay, p, g);
  if (MOM) {
    m = d.first ? g : fmaf(d.momentum, m, (1.f - d.dampening) * g);
    g = d.nesterov ? fmaf(d.momentum, m, g) : m;
  }
  p = fmaf(-d.lr, g, p);
}

}  // namespace kern
}  // namespace ringdp
