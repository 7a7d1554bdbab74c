// Epilogue shared by the 256x256 GEMM kernels (gemm_bf16_256.hip, gemm_fp8_256.hip): a lane holds
// 8 x 4 accumulator tiles of 16 x 16, each giving it C[m][n .. n+3] (the C^T MFMA orientation).
//
// Every global load the epilogue needs (bias, residual or the GELU-backward pre-activation) is issued
// before the first use: a load-wait-store chain per tile costs one L2/HBM round trip per tile, 32 in
// a row, which measured ~2x the whole 12-k-tile main loop on the ViT shapes (K = 768).
#pragma once

#include "device_common.h"
#include "kernels.h"

namespace ringdp {
namespace kern {

// QUAD: the phased kernel's tile order (acc[qm*4 + mt][qn*2 + nt], quadrants of 64 rows x 32 cols);
// otherwise acc[i][j] covers rows mrow + 16 i, columns ncol + 16 j.
template <bool QUAD>
__device__ __forceinline__ void gemm256_store(const dev::f32x4 (&acc)[8][4], const GemmEpilogue& ep, int M, int N,
                                              int zid, int bidx, int mrow, int ncol, float scale) {
  using namespace ringdp::dev;
  auto mof = [&](int i) { return QUAD ? mrow + (i >> 2) * 64 + 16 * (i & 3) : mrow + 16 * i; };
  auto nof = [&](int j) { return QUAD ? ncol + (j >> 1) * 32 + 16 * (j & 1) : ncol + 16 * j; };
  if (ep.mode == GemmEpilogue::kSplitK) {
    float* out = ep.partial + (int64_t)zid * M * N;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = mof(i);
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = nof(j);  // N % 4 == 0 (checked by the launchers)
        if (n < N) *reinterpret_cast<f32x4*>(out + (int64_t)m * N + n) = acc[i][j] * scale;
      }
    }
    return;
  }
  const int64_t cb = (int64_t)bidx * ep.c_bstride;
  // ---- all loads first
  f32x4 bias[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = nof(j);
    bias[j] = (ep.bias && n < N) ? *reinterpret_cast<const f32x4*>(ep.bias + n) : zero_f32x4();
  }
  const bf16* side = static_cast<const bf16*>(ep.residual ? ep.residual : (ep.act == 3 ? ep.preact : nullptr));
  bf16x4 sv[8][4];
  if (side) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = mof(i), n = nof(j);
        if (m < M && n < N) sv[i][j] = *reinterpret_cast<const bf16x4*>(side + cb + (int64_t)m * ep.ldc + n);
      }
  }
  // ---- compute + stores
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = mof(i);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = nof(j);
      if (n >= N) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] * scale * ep.alpha + bias[j][e];
      const int64_t off = cb + (int64_t)m * ep.ldc + n;
      if (ep.act == 3) {  // GELU backward: times GELU'(pre-activation)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x = (float)sv[i][j][e];
          v[e] *= 0.5f * (1.f + erff(x * 0.70710678118654752f)) + x * 0.3989422804014327f * __expf(-0.5f * x * x);
        }
      } else if (ep.preact) {
        *reinterpret_cast<bf16x4*>(static_cast<bf16*>(ep.preact) + off) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      }
      if (ep.residual) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += (float)sv[i][j][e];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (ep.act == 1) v[e] = fmaxf(v[e], 0.f);
        else if (ep.act == 2) v[e] = 0.5f * v[e] * (1.f + erff(v[e] * 0.70710678118654752f));
      }
      if (ep.out_bf16)
        *reinterpret_cast<bf16x4*>(static_cast<bf16*>(ep.C) + off) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      else
        *reinterpret_cast<f32x4*>(static_cast<float*>(ep.C) + off) = f32x4{v[0], v[1], v[2], v[3]};
    }
  }
}

}  // namespace kern
}  // namespace ringdp
