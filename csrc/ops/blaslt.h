// hipBLASLt backend for plain dense GEMMs (see blaslt.cpp).  RINGDP_GEMM_BACKEND=ringdp keeps every
// GEMM on ringdp's own MFMA kernels.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace ringdp {
namespace blaslt {

struct Problem {
  // row-major C[b][m][n] (ldc, c_bstride) = alpha * sum_k A(m,k) B(n,k) (+bias[n]) (+residual) -> act
  const void* A;
  const void* B;
  void* C;
  int M, N, K, batch = 1;
  int64_t lda, ldb, ldc;
  int64_t a_bstride = 0, b_bstride = 0, c_bstride = 0;
  bool a_row = false, b_row = false;  // false: K-contiguous; true: row-contiguous
  bool allow_row = false;             // row-contiguous operands at batch 1 (else only RINGDP_BLASLT_ROW=1)
  bool out_bf16 = true;
  float alpha = 1.f;
  const float* bias = nullptr;
  int act = 0;                 // 0 none, 2 GELU
  void* preact = nullptr;      // bf16 pre-activation (GELU aux)
  const void* residual = nullptr;
  // fp8 (OCP e4m3) operands, both K-contiguous, with per-tensor dequantisation scales (device fp32):
  // C = scale_a * scale_b * (A . B^T) ...
  bool fp8 = false;
  const float* scale_a = nullptr;
  const float* scale_b = nullptr;
};

bool enabled();
void set_enabled(bool on);  // tests / A-B runs
// Runs the GEMM on hipBLASLt when the problem maps onto it; false -> caller uses ringdp's kernels.
bool matmul(const Problem& p, hipStream_t stream);

}  // namespace blaslt
}  // namespace ringdp
