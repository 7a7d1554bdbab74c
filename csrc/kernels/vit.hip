// Transformer (ViT-B/16) layer kernels around the generic MFMA GEMM (BASELINE.json config 5).
//
// Token activations are row-major bf16 [rows][D].  Attention is computed on head-major tensors
// padded to a multiple-of-16 sequence (Tp >= T; padded keys are masked, padded queries are zero)
// so every attention matmul is one batched GEMM of the generic core (QK^T, PV and the four
// backward products), and the softmax lives in its own row kernel with the 1/sqrt(d) scale and
// the key mask fused.  LayerNorm keeps fp32 statistics; its backward fuses the residual-stream
// gradient add.
#include <algorithm>

#include "device_common.h"
#include "kernels.h"

namespace ringdp {
namespace kern {

using namespace ringdp::dev;

namespace {

inline int grid_for(int64_t n, int per_block = 256, int cap = 8192) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + per_block - 1) / per_block, cap));
}

// ---------------------------------------------------------------- LayerNorm (one wave per row)
// D <= 64 * 8 * 4 = 2048, D % 8 == 0
template <int VPL>  // 8-element vectors per lane
__global__ __launch_bounds__(256) void layernorm_fwd_kernel(const bf16* __restrict__ x, const float* __restrict__ w,
                                                            const float* __restrict__ b, int64_t rows, int D,
                                                            float eps, bf16* __restrict__ y,
                                                            float* __restrict__ stats) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nv = D / 8;
  const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + row * D);
  float v[VPL][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int vi = lane + 64 * i;
    if (vi < nv) {
      const bf16x8 t = xr[vi];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[i][j] = (float)t[j];
        s += v[i][j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    }
  }
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i)
    if (lane + 64 * i < nv)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[i][j] - mean;
        q += d * d;
      }
  const float rstd = rsqrtf(wave_sum(q) / (float)D + eps);
  bf16x8* yr = reinterpret_cast<bf16x8*>(y + row * D);
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int vi = lane + 64 * i;
    if (vi < nv) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = vi * 8 + j;
        o[j] = (bf16)((v[i][j] - mean) * rstd * w[c] + b[c]);
      }
      yr[vi] = o;
    }
  }
  if (lane == 0) {
    stats[2 * row] = mean;
    stats[2 * row + 1] = rstd;
  }
}

// LayerNorm forward that writes its output as e4m3 for the next fp8 linear instead of bf16: the normalised row
// (the exact values layernorm_fwd_kernel would store, rounded to bf16) is quantised with the delayed scale
// amax[0] / 448 (clamped to +-448) into q [rows][D] (8-B stores straight from the lanes) and, through an LDS
// tile of the block's 64 rows (193-dword rows: conflict-free), transposed into qt [D][rows] (8 lanes of a column
// group write 64 contiguous bytes).  tmax[block] <- the block's |y|max (the next roll); scale[0] <- the scale.
// rows % 16 == 0 (8-row groups are wholly inside), D % 8 == 0, dynamic LDS 64 * (D + 4) bytes.
constexpr int kLnQ8Rows = 64, kLnQ8Threads = 1024;  // 16 waves x 4 rows: the rows of a block in parallel
__device__ __forceinline__ uint32_t ln_pack_e4m3(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}
template <int VPL>
__global__ __launch_bounds__(kLnQ8Threads) void layernorm_fwd_q8_kernel(const bf16* __restrict__ x, const float* __restrict__ w,
                                                               const float* __restrict__ b, int64_t rows, int D,
                                                               float eps, float* __restrict__ stats,
                                                               const float* __restrict__ amax, uint8_t* __restrict__ q,
                                                               uint8_t* __restrict__ qt, float* __restrict__ scale,
                                                               float* __restrict__ tmax) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lnq_tile[];
  __shared__ float red[kLnQ8Threads / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nv = D / 8, ld = D + 4;
  const float qs = fmaxf(amax[0], 1e-12f) / 448.f, inv = 1.f / qs;
  if (blockIdx.x == 0 && threadIdx.x == 0) scale[0] = qs;
  const int64_t r0 = (int64_t)blockIdx.x * kLnQ8Rows;
  float vmax = 0.f;
  for (int rl = wave; rl < kLnQ8Rows; rl += kLnQ8Threads / 64) {
    const int64_t row = r0 + rl;
    if (row >= rows) break;
    const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + row * D);
    float v[VPL][8];
    float sm = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int vi = lane + 64 * i;
      if (vi < nv) {
        const bf16x8 t = xr[vi];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[i][j] = (float)t[j];
          sm += v[i][j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
      }
    }
    const float mean = wave_sum(sm) / (float)D;
    float qq = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i)
      if (lane + 64 * i < nv)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = v[i][j] - mean;
          qq += d * d;
        }
    const float rstd = rsqrtf(wave_sum(qq) / (float)D + eps);
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int vi = lane + 64 * i;
      if (vi < nv) {
        float e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int c = vi * 8 + j;
          const float y = (float)(bf16)((v[i][j] - mean) * rstd * w[c] + b[c]);  // layernorm_fwd_kernel's value
          vmax = fmaxf(vmax, fabsf(y));
          e[j] = fminf(fmaxf(y * inv, -448.f), 448.f);
        }
        const uint32_t lo = ln_pack_e4m3(e[0], e[1], e[2], e[3]), hi = ln_pack_e4m3(e[4], e[5], e[6], e[7]);
        *reinterpret_cast<uint2*>(q + row * D + vi * 8) = make_uint2(lo, hi);
        uint32_t* tw = reinterpret_cast<uint32_t*>(lnq_tile + rl * ld + vi * 8);
        tw[0] = lo;
        tw[1] = hi;
      }
    }
    if (lane == 0) {
      stats[2 * row] = mean;
      stats[2 * row + 1] = rstd;
    }
  }
  vmax = wave_max(vmax);
  if (lane == 0) red[wave] = vmax;
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = 0.f;
    for (int i = 0; i < kLnQ8Threads / 64; ++i) m = fmaxf(m, red[i]);
    tmax[blockIdx.x] = m;
  }
  // transposed: item = (8-row group rg, 4-column group cg)
  const int ncg = D / 4;
  for (int it = threadIdx.x; it < 8 * ncg; it += kLnQ8Threads) {
    const int rg = it & 7, c = 4 * (it >> 3);
    const int64_t m = r0 + 8 * rg;
    if (m >= rows) continue;
    uint32_t d[8];
#pragma unroll
    for (int ii = 0; ii < 8; ++ii) d[ii] = *reinterpret_cast<const uint32_t*>(lnq_tile + (8 * rg + ii) * ld + c);
    uint32_t col[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t a0 = d[4 * h], a1 = d[4 * h + 1], a2 = d[4 * h + 2], a3 = d[4 * h + 3];
      const uint32_t ab_lo = __builtin_amdgcn_perm(a1, a0, 0x05010400u), ab_hi = __builtin_amdgcn_perm(a1, a0, 0x07030602u);
      const uint32_t ce_lo = __builtin_amdgcn_perm(a3, a2, 0x05010400u), ce_hi = __builtin_amdgcn_perm(a3, a2, 0x07030602u);
      col[h][0] = __builtin_amdgcn_perm(ce_lo, ab_lo, 0x05040100u);
      col[h][1] = __builtin_amdgcn_perm(ce_lo, ab_lo, 0x07060302u);
      col[h][2] = __builtin_amdgcn_perm(ce_hi, ab_hi, 0x05040100u);
      col[h][3] = __builtin_amdgcn_perm(ce_hi, ab_hi, 0x07060302u);
    }
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
      *reinterpret_cast<uint2*>(qt + (int64_t)(c + jj) * rows + m) = make_uint2(col[0][jj], col[1][jj]);
  }
}

// dx = rstd * (w*dy - mean(w*dy) - xhat * mean(w*dy*xhat)) (+ dres);  dw/db partials per block
template <int VPL, bool CS>  // CS: also the column sums of dx into cs_part (compiled out otherwise)
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                            const float* __restrict__ stats,
                                                            const float* __restrict__ w, const bf16* __restrict__ dres,
                                                            int64_t rows, int D, int rows_per_block,
                                                            bf16* __restrict__ dx, float* __restrict__ part,
                                                            float* __restrict__ cs_part) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nv = D / 8;
  float dw[VPL][8], db[VPL][8], cs[VPL][8];  // cs (cs_part != null): column sums of the stored dx
#pragma unroll
  for (int i = 0; i < VPL; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) dw[i][j] = db[i][j] = cs[i][j] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = std::min<int64_t>(rows, r0 + rows_per_block);
  for (int64_t row = r0 + wave; row < r1; row += 4) {
    const float mean = stats[2 * row], rstd = stats[2 * row + 1];
    const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + row * D);
    const bf16x8* gr = reinterpret_cast<const bf16x8*>(dy + row * D);
    float xh[VPL][8], gw[VPL][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int vi = lane + 64 * i;
      if (vi < nv) {
        const bf16x8 xv = xr[vi], gv = gr[vi];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int c = vi * 8 + j;
          xh[i][j] = ((float)xv[j] - mean) * rstd;
          const float g = (float)gv[j];
          gw[i][j] = g * w[c];
          s1 += gw[i][j];
          s2 += gw[i][j] * xh[i][j];
          dw[i][j] += g * xh[i][j];
          db[i][j] += g;
        }
      }
    }
    const float m1 = wave_sum(s1) / (float)D, m2 = wave_sum(s2) / (float)D;
    bf16x8* dxr = reinterpret_cast<bf16x8*>(dx + row * D);
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int vi = lane + 64 * i;
      if (vi < nv) {
        bf16x8 rv = zero_bf16x8();
        if (dres) rv = reinterpret_cast<const bf16x8*>(dres + row * D)[vi];
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          o[j] = (bf16)(rstd * (gw[i][j] - m1 - xh[i][j] * m2) + (float)rv[j]);
          if constexpr (CS) cs[i][j] += (float)o[j];
        }
        dxr[vi] = o;
      }
    }
  }
  // combine the 4 waves (fixed order) and write this block's partial dw/db
  __shared__ float red[4][2048];
  constexpr int passes = CS ? 3 : 2;
  for (int pass = 0; pass < passes; ++pass) {
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int vi = lane + 64 * i;
      if (vi < nv)
#pragma unroll
        for (int j = 0; j < 8; ++j) red[wave][vi * 8 + j] = pass == 0 ? dw[i][j] : (pass == 1 ? db[i][j] : cs[i][j]);
    }
    __syncthreads();
    float* dst = pass < 2 ? part + ((int64_t)blockIdx.x * 2 + pass) * D : cs_part + (int64_t)blockIdx.x * D;
    for (int c = threadIdx.x; c < D; c += 256) dst[c] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
    __syncthreads();
  }
}

// ---------------------------------------------------------------- attention layout
// qkv [B*T][3*H*Dh] (Linear output) -> q/k/v [B*H][Tp][Dh] (rows >= T zero)
__global__ __launch_bounds__(256) void qkv_split_kernel(const bf16* __restrict__ qkv, int B, int T, int H, int Dh,
                                                        int Tp, bf16* __restrict__ q, bf16* __restrict__ k,
                                                        bf16* __restrict__ v) {
  const int dv = Dh / 8;
  const int64_t total = (int64_t)3 * B * H * Tp * dv;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int d8 = (int)(e % dv);
    int64_t r = e / dv;
    const int t = (int)(r % Tp);
    r /= Tp;
    const int h = (int)(r % H);
    r /= H;
    const int b = (int)(r % B);
    const int which = (int)(r / B);
    bf16x8 val = zero_bf16x8();
    if (t < T)
      val = *reinterpret_cast<const bf16x8*>(qkv + ((int64_t)b * T + t) * 3 * H * Dh + which * H * Dh + h * Dh + d8 * 8);
    bf16* dst = which == 0 ? q : (which == 1 ? k : v);
    *reinterpret_cast<bf16x8*>(dst + (((int64_t)b * H + h) * Tp + t) * Dh + d8 * 8) = val;
  }
}

// inverse: q/k/v grads [B*H][Tp][Dh] -> dqkv [B*T][3*H*Dh]
__global__ __launch_bounds__(256) void qkv_merge_kernel(const bf16* __restrict__ dq, const bf16* __restrict__ dk,
                                                        const bf16* __restrict__ dv_, int B, int T, int H, int Dh,
                                                        int Tp, bf16* __restrict__ dqkv) {
  const int dv = Dh / 8;
  const int64_t total = (int64_t)B * T * 3 * H * dv;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int d8 = (int)(e % dv);
    int64_t r = e / dv;
    const int h = (int)(r % H);
    r /= H;
    const int which = (int)(r % 3);
    r /= 3;
    const int t = (int)(r % T);
    const int b = (int)(r / T);
    const bf16* src = which == 0 ? dq : (which == 1 ? dk : dv_);
    *reinterpret_cast<bf16x8*>(dqkv + ((int64_t)b * T + t) * 3 * H * Dh + which * H * Dh + h * Dh + d8 * 8) =
        *reinterpret_cast<const bf16x8*>(src + (((int64_t)b * H + h) * Tp + t) * Dh + d8 * 8);
  }
}

// o [B*H][Tp][Dh] -> [B*T][H*Dh]   (and the reverse for the gradient)
template <bool TO_HEADS>
__global__ __launch_bounds__(256) void heads_kernel(const bf16* __restrict__ src, int B, int T, int H, int Dh, int Tp,
                                                    bf16* __restrict__ dst) {
  const int dv = Dh / 8;
  const int64_t total = TO_HEADS ? (int64_t)B * H * Tp * dv : (int64_t)B * T * H * dv;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int d8 = (int)(e % dv);
    int64_t r = e / dv;
    if (TO_HEADS) {  // dst [B*H][Tp][Dh] from src [B*T][H*Dh]
      const int t = (int)(r % Tp);
      r /= Tp;
      const int h = (int)(r % H);
      const int b = (int)(r / H);
      bf16x8 val = zero_bf16x8();
      if (t < T) val = *reinterpret_cast<const bf16x8*>(src + ((int64_t)b * T + t) * H * Dh + h * Dh + d8 * 8);
      *reinterpret_cast<bf16x8*>(dst + (((int64_t)b * H + h) * Tp + t) * Dh + d8 * 8) = val;
    } else {  // dst [B*T][H*Dh] from src [B*H][Tp][Dh]
      const int h = (int)(r % H);
      r /= H;
      const int t = (int)(r % T);
      const int b = (int)(r / T);
      *reinterpret_cast<bf16x8*>(dst + ((int64_t)b * T + t) * H * Dh + h * Dh + d8 * 8) =
          *reinterpret_cast<const bf16x8*>(src + (((int64_t)b * H + h) * Tp + t) * Dh + d8 * 8);
    }
  }
}

// ---------------------------------------------------------------- softmax over keys (one wave per row)
// s [rows][Tp] fp32 scores (unscaled) -> p bf16 = softmax(scale * s) over the first T keys; padded
// keys get 0.  Rows t >= T (padded queries) are written as zeros.
__global__ __launch_bounds__(256) void softmax_fwd_kernel(const float* __restrict__ s, int64_t rows, int T, int Tp,
                                                          float scale, bf16* __restrict__ p) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bool qpad = (int)(row % Tp) >= T;
  const float* sr = s + row * Tp;
  bf16* pr = p + row * Tp;
  if (qpad) {
    for (int c = lane; c < Tp; c += 64) pr[c] = (bf16)0.f;
    return;
  }
  float mx = -INFINITY;
  for (int c = lane; c < T; c += 64) mx = fmaxf(mx, sr[c] * scale);
  mx = wave_max(mx);
  float sum = 0.f;
  for (int c = lane; c < T; c += 64) sum += __expf(sr[c] * scale - mx);
  const float inv = 1.f / wave_sum(sum);
  for (int c = lane; c < Tp; c += 64) pr[c] = (bf16)(c < T ? __expf(sr[c] * scale - mx) * inv : 0.f);
}

// Register-resident variant for Tp <= 256 (ViT-B/16: Tp = 208): lane l owns columns 4l..4l+3, loaded once
// as a float4 and written once as 4 bf16 (the scalar kernel above streams each row 3 times).
__global__ __launch_bounds__(256) void softmax_fwd_vec_kernel(const float* __restrict__ s, int64_t rows, int T,
                                                              int Tp, float scale, bf16* __restrict__ p) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int c0 = 4 * lane;
  const bool live = c0 < Tp;
  uint2* out = reinterpret_cast<uint2*>(p + row * Tp + c0);
  if ((int)(row % Tp) >= T) {  // padded query row
    if (live) *out = make_uint2(0u, 0u);
    return;
  }
  float4 v = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
  if (live) v = *reinterpret_cast<const float4*>(s + row * Tp + c0);
  float x[4] = {v.x * scale, v.y * scale, v.z * scale, v.w * scale};
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (c0 + j >= T) x[j] = -INFINITY;
  const float mx = wave_max(fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3])));
  float e[4], sum = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    e[j] = c0 + j < T ? __expf(x[j] - mx) : 0.f;
    sum += e[j];
  }
  const float inv = 1.f / wave_sum(sum);
  if (live) {
    const bf16x4 o = bf16x4{(bf16)(e[0] * inv), (bf16)(e[1] * inv), (bf16)(e[2] * inv), (bf16)(e[3] * inv)};
    *out = __builtin_bit_cast(uint2, o);
  }
}

// ds = scale * p * (dp - sum_j dp_j p_j)  (bf16 out; padded keys / queries -> 0)
__global__ __launch_bounds__(256) void softmax_bwd_kernel(const bf16* __restrict__ p, const float* __restrict__ dp,
                                                          int64_t rows, int T, int Tp, float scale,
                                                          bf16* __restrict__ ds) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bf16* pr = p + row * Tp;
  const float* dr = dp + row * Tp;
  bf16* o = ds + row * Tp;
  float dot = 0.f;
  for (int c = lane; c < T; c += 64) dot += (float)pr[c] * dr[c];
  dot = wave_sum(dot);
  for (int c = lane; c < Tp; c += 64) o[c] = (bf16)(c < T ? scale * (float)pr[c] * (dr[c] - dot) : 0.f);
}

__global__ __launch_bounds__(256) void softmax_bwd_vec_kernel(const bf16* __restrict__ p,
                                                              const float* __restrict__ dp, int64_t rows, int T,
                                                              int Tp, float scale, bf16* __restrict__ ds) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int c0 = 4 * lane;
  const bool live = c0 < Tp;
  float pv[4] = {0.f, 0.f, 0.f, 0.f}, dv[4] = {0.f, 0.f, 0.f, 0.f};
  if (live) {
    const bf16x4 pb = __builtin_bit_cast(bf16x4, *reinterpret_cast<const uint2*>(p + row * Tp + c0));
    const float4 d = *reinterpret_cast<const float4*>(dp + row * Tp + c0);
    pv[0] = (float)pb[0];
    pv[1] = (float)pb[1];
    pv[2] = (float)pb[2];
    pv[3] = (float)pb[3];
    dv[0] = d.x;
    dv[1] = d.y;
    dv[2] = d.z;
    dv[3] = d.w;
  }
  float dot = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (c0 + j < T) dot += pv[j] * dv[j];
  dot = wave_sum(dot);
  if (live) {
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = c0 + j < T ? scale * pv[j] * (dv[j] - dot) : 0.f;
    *reinterpret_cast<uint2*>(ds + row * Tp + c0) =
        __builtin_bit_cast(uint2, bf16x4{(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]});
  }
}

// ---------------------------------------------------------------- misc
__global__ __launch_bounds__(256) void gelu_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ pre,
                                                       int64_t nvec, bf16* __restrict__ dx) {
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    const bf16x8 g = reinterpret_cast<const bf16x8*>(dy)[v], z = reinterpret_cast<const bf16x8*>(pre)[v];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = (float)z[j];
      const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
      const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
      o[j] = (bf16)((float)g[j] * (cdf + x * pdf));
    }
    reinterpret_cast<bf16x8*>(dx)[v] = o;
  }
}

// y = gelu_erf(x); the second half of a GEMM whose fused GELU-aux epilogue hipBLASLt has no algorithm for
__global__ __launch_bounds__(256) void gelu_fwd_kernel(const bf16* __restrict__ x, int64_t nvec, bf16* __restrict__ y) {
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    const bf16x8 z = reinterpret_cast<const bf16x8*>(x)[v];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float t = (float)z[j];
      o[j] = (bf16)(0.5f * t * (1.f + erff(t * 0.70710678118654752f)));
    }
    reinterpret_cast<bf16x8*>(y)[v] = o;
  }
}

// tokens [B][1+NP][D] = concat(cls, patches [B][NP][D]) + pos [1+NP][D]
__global__ __launch_bounds__(256) void assemble_tokens_kernel(const bf16* __restrict__ patches,
                                                              const float* __restrict__ cls,
                                                              const float* __restrict__ pos, int B, int NP, int D,
                                                              bf16* __restrict__ out) {
  const int T = NP + 1;
  const int64_t total = (int64_t)B * T * D;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int d = (int)(e % D);
    const int64_t r = e / D;
    const int t = (int)(r % T);
    const int64_t b = r / T;
    const float base = t == 0 ? cls[d] : (float)patches[(b * NP + t - 1) * D + d];
    out[e] = (bf16)(base + pos[(int64_t)t * D + d]);
  }
}

// gradients of assemble_tokens: dpatches (bf16) and per-block partial sums for dcls / dpos
__global__ __launch_bounds__(256) void assemble_tokens_bwd_kernel(const bf16* __restrict__ dout, int B, int NP, int D,
                                                                  bf16* __restrict__ dpatches,
                                                                  float* __restrict__ dpos, float* __restrict__ dcls) {
  const int T = NP + 1;
  // one thread per (t, d): sum over the batch in a fixed order
  const int64_t total = (int64_t)T * D;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int d = (int)(e % D);
    const int t = (int)(e / D);
    float acc = 0.f;
    for (int b = 0; b < B; ++b) {
      const float g = (float)dout[((int64_t)b * T + t) * D + d];
      acc += g;
      if (t > 0) dpatches[((int64_t)b * NP + t - 1) * D + d] = (bf16)g;
    }
    dpos[e] = acc;
    if (t == 0) dcls[d] = acc;
  }
}

// rows [B][T][D] -> the class-token rows [B][D] (and the reverse scatter for the gradient)
__global__ __launch_bounds__(256) void cls_rows_kernel(const bf16* __restrict__ x, int B, int T, int D,
                                                       bf16* __restrict__ y, int reverse) {
  const int64_t total = (int64_t)B * D;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t b = e / D;
    const int d = (int)(e % D);
    if (!reverse)
      y[e] = x[b * T * D + d];
    else
      y[b * T * D + d] = x[e];
  }
}

// NCHW fp32/bf16 images -> non-overlapping patch rows [B*NP][C*P*P] bf16 (column order c, kh, kw:
// the flattened conv_proj weight), i.e. the im2col of a stride-P PxP convolution.
template <bool BF>
__global__ __launch_bounds__(256) void patchify_kernel(const void* __restrict__ x, int B, int Cc, int H, int W,
                                                       int P, bf16* __restrict__ out) {
  const int gh = H / P, gw = W / P, K = Cc * P * P;
  const int64_t total = (int64_t)B * gh * gw * K;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int k = (int)(e % K);
    const int64_t r = e / K;
    const int pw = (int)(r % gw);
    const int ph = (int)((r / gw) % gh);
    const int64_t b = r / ((int64_t)gw * gh);
    const int c = k / (P * P), kh = (k / P) % P, kw = k % P;
    const int64_t src = ((b * Cc + c) * H + ph * P + kh) * W + pw * P + kw;
    out[e] = BF ? static_cast<const bf16*>(x)[src] : (bf16)static_cast<const float*>(x)[src];
  }
}

}  // namespace

void patchify(const void* x, bool x_bf16, int B, int C, int H, int W, int P, void* out, hipStream_t s) {
  const int64_t total = (int64_t)B * (H / P) * (W / P) * C * P * P;
  if (x_bf16)
    patchify_kernel<true><<<grid_for(total), 256, 0, s>>>(x, B, C, H, W, P, static_cast<bf16*>(out));
  else
    patchify_kernel<false><<<grid_for(total), 256, 0, s>>>(x, B, C, H, W, P, static_cast<bf16*>(out));
}

int layernorm_bwd_blocks(int64_t rows) { return (int)std::min<int64_t>(1024, std::max<int64_t>(1, (rows + 15) / 16)); }

void layernorm_fwd(const void* x, const float* w, const float* b, int64_t rows, int D, float eps, void* y,
                   float* stats, hipStream_t s) {
  const int nv = D / 8;
  const int grid = (int)((rows + 3) / 4);
  if (nv <= 64)
    layernorm_fwd_kernel<1><<<grid, 256, 0, s>>>(static_cast<const bf16*>(x), w, b, rows, D, eps, static_cast<bf16*>(y), stats);
  else if (nv <= 128)
    layernorm_fwd_kernel<2><<<grid, 256, 0, s>>>(static_cast<const bf16*>(x), w, b, rows, D, eps, static_cast<bf16*>(y), stats);
  else
    layernorm_fwd_kernel<4><<<grid, 256, 0, s>>>(static_cast<const bf16*>(x), w, b, rows, D, eps, static_cast<bf16*>(y), stats);
}

int64_t layernorm_q8_blocks(int64_t rows) { return (rows + kLnQ8Rows - 1) / kLnQ8Rows; }

void layernorm_fwd_q8(const void* x, const float* w, const float* b, int64_t rows, int D, float eps, float* stats,
                      const float* amax, void* q, void* qt, float* scale, float* tmax, hipStream_t s) {
  const int nb = (int)layernorm_q8_blocks(rows), nv = D / 8;
  const size_t lds = (size_t)kLnQ8Rows * (D + 4);
  auto go = [&](auto kern) {
    kern<<<nb, kLnQ8Threads, lds, s>>>(static_cast<const bf16*>(x), w, b, rows, D, eps, stats, amax, static_cast<uint8_t*>(q),
                              static_cast<uint8_t*>(qt), scale, tmax);
  };
  if (nv <= 64)
    go(layernorm_fwd_q8_kernel<1>);
  else if (nv <= 128)
    go(layernorm_fwd_q8_kernel<2>);
  else
    go(layernorm_fwd_q8_kernel<4>);
}

void layernorm_bwd(const void* dy, const void* x, const float* stats, const float* w, const void* dres, int64_t rows,
                   int D, void* dx, float* part, float* dw, float* db, hipStream_t s, float* cs_part) {
  const int nb = layernorm_bwd_blocks(rows);
  const int rpb = (int)((rows + nb - 1) / nb);
  const int nv = D / 8;
  auto args = [&](auto kern) {
    kern<<<nb, 256, 0, s>>>(static_cast<const bf16*>(dy), static_cast<const bf16*>(x), stats, w,
                            static_cast<const bf16*>(dres), rows, D, rpb, static_cast<bf16*>(dx), part, cs_part);
  };
  if (cs_part) {
    if (nv <= 64) args(layernorm_bwd_kernel<1, true>);
    else if (nv <= 128) args(layernorm_bwd_kernel<2, true>);
    else args(layernorm_bwd_kernel<4, true>);
  } else {
    if (nv <= 64) args(layernorm_bwd_kernel<1, false>);
    else if (nv <= 128) args(layernorm_bwd_kernel<2, false>);
    else args(layernorm_bwd_kernel<4, false>);
  }
  // part [nb][2][D] -> dw = sum part[.][0], db = sum part[.][1]
  reduce_parts(part, nb, D, part + (int64_t)nb * 2 * D, dw, db, s);
}

int layernorm_bwd_scratch_floats(int64_t rows, int D) {
  const int nb = layernorm_bwd_blocks(rows);
  return nb * 2 * D + reduce_parts_scratch_floats(nb, D);
}

void qkv_split(const void* qkv, int B, int T, int H, int Dh, int Tp, void* q, void* k, void* v, hipStream_t s) {
  qkv_split_kernel<<<grid_for((int64_t)3 * B * H * Tp * Dh / 8), 256, 0, s>>>(
      static_cast<const bf16*>(qkv), B, T, H, Dh, Tp, static_cast<bf16*>(q), static_cast<bf16*>(k), static_cast<bf16*>(v));
}

void qkv_merge(const void* dq, const void* dk, const void* dv, int B, int T, int H, int Dh, int Tp, void* dqkv,
               hipStream_t s) {
  qkv_merge_kernel<<<grid_for((int64_t)B * T * 3 * H * Dh / 8), 256, 0, s>>>(
      static_cast<const bf16*>(dq), static_cast<const bf16*>(dk), static_cast<const bf16*>(dv), B, T, H, Dh, Tp,
      static_cast<bf16*>(dqkv));
}

void heads_to_rows(const void* o, int B, int T, int H, int Dh, int Tp, void* rows, hipStream_t s) {
  heads_kernel<false><<<grid_for((int64_t)B * T * H * Dh / 8), 256, 0, s>>>(static_cast<const bf16*>(o), B, T, H, Dh, Tp,
                                                                            static_cast<bf16*>(rows));
}

void rows_to_heads(const void* rows, int B, int T, int H, int Dh, int Tp, void* o, hipStream_t s) {
  heads_kernel<true><<<grid_for((int64_t)B * H * Tp * Dh / 8), 256, 0, s>>>(static_cast<const bf16*>(rows), B, T, H, Dh,
                                                                            Tp, static_cast<bf16*>(o));
}

void softmax_fwd(const float* scores, int64_t rows, int T, int Tp, float scale, void* p, hipStream_t s) {
  if (Tp <= 256 && Tp % 4 == 0)
    softmax_fwd_vec_kernel<<<(int)((rows + 3) / 4), 256, 0, s>>>(scores, rows, T, Tp, scale, static_cast<bf16*>(p));
  else
    softmax_fwd_kernel<<<(int)((rows + 3) / 4), 256, 0, s>>>(scores, rows, T, Tp, scale, static_cast<bf16*>(p));
}

namespace {

// Fused attention forward for head dim 64 and Tp <= 256 (ViT-B/16: Tp = 208): per (batch, head) one
// 256-thread workgroup holds K and V in LDS (2 x Tp x 128 B, XOR-swizzled) and each wave walks 16-query
// tiles.  S^T = K Q^T is computed tile by tile (v_mfma_f32_16x16x32_bf16, keys as rows), so lane (g, q)
// holds keys 16t + 4g .. +3 of query q = lane & 15 in every key tile: the softmax over a query's keys is an
// in-lane reduction plus two xor-shuffles, and the same registers, as bf16, ARE the B operand of
// O^T = V^T P^T when the MFMA's k index is permuted to (tile pair, 4g + j) - the V^T fragment reads that
// same key order with ds_read_b64_tr_b16.  S never leaves registers (the unfused path wrote it as fp32:
// 2 x Tp^2 x 4 B per head of HBM traffic plus a softmax pass); P is still stored (bf16) for the backward.
// Semantics match softmax_fwd + the P V GEMM: keys >= T get probability 0, padded query rows are 0.
constexpr int ATT_D = 64;
// Strided view of one attention operand: element (b, h, t, d) at base + b*sb + h*sh + t*st + d - either
// head-major [B*H][Tp][64] (sb = Tp*64, sh = 0 with H = 1 per "batch" bh) or the token rows of the qkv
// projection [B*T][3*H*64] (sb = T*st, sh = 64, st = 3*H*64), which the kernels then read directly
// (no split/merge passes).  Rows t >= T read as zero.
struct AttnIn {
  const bf16* base;
  int64_t sb, sh, st;
  __device__ __forceinline__ const bf16* row(int bh, int H, int t) const {
    return base + (int64_t)(bh / H) * sb + (int64_t)(bh % H) * sh + (int64_t)t * st;
  }
  __device__ __forceinline__ bf16x8 load8(int bh, int H, int t, int T, int d) const {
    return t < T ? *reinterpret_cast<const bf16x8*>(row(bh, H, t) + d) : zero_bf16x8();
  }
};
struct AttnOut {
  bf16* base;
  int64_t sb, sh, st;
  int rows;  // rows t < rows are written (T for token rows, Tp for head-major)
  __device__ __forceinline__ bf16* row(int bh, int H, int t) const {
    return base + (int64_t)(bh / H) * sb + (int64_t)(bh % H) * sh + (int64_t)t * st;
  }
};
__device__ __forceinline__ int att_ksw(int r, int d) { return r * ATT_D + ((((d >> 3) ^ (r & 7))) << 3) + (d & 7); }
__device__ __forceinline__ int att_vsw(int r, int d) {
  return r * ATT_D + ((((d >> 4) ^ ((r >> 1) & 3))) << 4) + (d & 15);
}

// LSE: instead of P, store each query's log-sum-exp (lse[bh][Tp], +inf for padded queries) - the backward
// kernels recompute P = exp(scale S - lse) from Q and K (flash-attention style): P is 2 x Tp^2 bytes per head
// written here and read twice in the backward, the largest HBM stream of the attention (ViT-B/16: 133 MB per
// layer per pass, against 5.5 MFLOP of MFMA work per head to recompute it)
template <int NT, bool LSE>  // key tiles of 16 (Tp = 16 * NT)
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnIn q, AttnIn k, AttnIn v, int T, int H, float scale,
                                                       bf16* __restrict__ p, AttnOut o, float* __restrict__ lse) {
  constexpr int Tp = 16 * NT;
  __shared__ __attribute__((aligned(16))) bf16 Ks[Tp * ATT_D];
  __shared__ __attribute__((aligned(16))) bf16 Vs[Tp * ATT_D];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bh = blockIdx.x;
  for (int c = tid; c < Tp * 8; c += 256) {  // 16-B chunks: row c >> 3, columns 8 (c & 7) ..; rows >= T zero
    const int r = c >> 3, d = (c & 7) * 8;
    *reinterpret_cast<bf16x8*>(Ks + att_ksw(r, d)) = k.load8(bh, H, r, T, d);
    *reinterpret_cast<bf16x8*>(Vs + att_vsw(r, d)) = v.load8(bh, H, r, T, d);
  }
  __syncthreads();
  const int g = lane >> 4, qi = lane & 15;
  for (int qt = wave; qt < NT; qt += 4) {
    const int qrow = qt * 16 + qi;
    const bf16x8 qf0 = q.load8(bh, H, qrow, T, 8 * g);
    const bf16x8 qf1 = q.load8(bh, H, qrow, T, 32 + 8 * g);
    f32x4 st[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int kr = 16 * t + qi;
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(Ks + att_ksw(kr, 8 * g));
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(Ks + att_ksw(kr, 32 + 8 * g));
      st[t] = mfma16x16x32(a1, qf1, mfma16x16x32(a0, qf0, zero_f32x4()));
    }
    // softmax over keys for query qrow: lane holds keys 16t + 4g + i.  Only tiles that reach past T are masked
    // (a scalar test per tile; ViT-B/16: the last one): masking every score kept 52 lane masks live at once,
    // which the compiler spilled through v_writelane / v_readlane (248 extra VALU per query tile).
    // exp(s*scale - m) = exp2(s*c - m*c) with c = scale * log2(e): one fma + v_exp per score, and a masked
    // -inf score gives exp2(-inf) = 0.
#pragma unroll
    for (int t = 0; t < NT; ++t)
      if (16 * t + 16 > T)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (!(16 * t + 4 * g + i < T)) st[t][i] = -INFINITY;
    float mx = -INFINITY;  // of the raw scores (scale > 0)
#pragma unroll
    for (int t = 0; t < NT; ++t) mx = fmaxf(mx, fmaxf(fmaxf(st[t][0], st[t][1]), fmaxf(st[t][2], st[t][3])));
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float c2 = scale * 1.4426950408889634f, mc = mx * c2;
    float sum = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float e = __builtin_amdgcn_exp2f(fmaf(st[t][i], c2, -mc));
        st[t][i] = e;
        sum += e;
      }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    mx *= scale;  // the scaled maximum (the log-sum-exp below)
    const float inv = qrow < T ? 1.f / sum : 0.f;  // padded query rows: P = 0
    bf16x4 pb[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
      pb[t] = bf16x4{(bf16)(st[t][0] * inv), (bf16)(st[t][1] * inv), (bf16)(st[t][2] * inv), (bf16)(st[t][3] * inv)};
    if constexpr (LSE) {
      if (g == 0) lse[(int64_t)bh * Tp + qrow] = qrow < T ? mx + __logf(sum) : INFINITY;
    } else {  // tile pairs (t, t+1): lanes with g even store 8 keys of tile t, g odd 8 keys of tile t+1 (one xor-16
       // exchange of 8 B): 16-B stores, 64 contiguous bytes of each of 16 rows per store instruction
      bf16* prow = p + ((int64_t)bh * Tp + qrow) * Tp;
      const bool godd = g & 1;
#pragma unroll
      for (int t = 0; t + 1 < NT; t += 2) {
        const uint2 sv = __builtin_bit_cast(uint2, godd ? pb[t] : pb[t + 1]);
        const uint2 rv = make_uint2(__shfl_xor(sv.x, 16, 64), __shfl_xor(sv.y, 16, 64));
        const bf16x4 rcv = __builtin_bit_cast(bf16x4, rv);
        const bf16x4 lo = godd ? rcv : pb[t], hi = godd ? pb[t + 1] : rcv;
        const int col = godd ? 16 * (t + 1) + 4 * (g - 1) : 16 * t + 4 * g;
        *reinterpret_cast<bf16x8*>(prow + col) = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      if (NT & 1) *reinterpret_cast<bf16x4*>(prow + 16 * (NT - 1) + 4 * g) = pb[NT - 1];
    }
    // O^T[d][q] = sum over key pairs (t0, t1) of V^T (keys 16t + 4g + j) x P^T
    f32x4 ot[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) ot[dt] = zero_f32x4();
    const int q4 = qi >> 2, p4 = qi & 3;  // tr16 lane roles inside the 16-lane group
#pragma unroll
    for (int ks = 0; ks < (NT + 1) / 2; ++ks) {
      const int t0 = 2 * ks, t1 = 2 * ks + 1 < NT ? 2 * ks + 1 : t0;  // odd NT: the missing tile has P = 0
      const bf16x4 p1 = 2 * ks + 1 < NT ? pb[2 * ks + 1] : bf16x4{(bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
      const bf16x8 bfr = bf16x8{pb[t0][0], pb[t0][1], pb[t0][2], pb[t0][3], p1[0], p1[1], p1[2], p1[3]};
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x4 lo = lds_read_tr16(Vs + att_vsw(16 * t0 + 4 * g + q4, 16 * dt + 4 * p4));
        const bf16x4 hi = lds_read_tr16(Vs + att_vsw(16 * t1 + 4 * g + q4, 16 * dt + 4 * p4));
        const bf16x8 afr = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        ot[dt] = mfma16x16x32(afr, bfr, ot[dt]);
      }
    }
    if (qrow < o.rows) {
      bf16* orow = o.row(bh, H, qrow) + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        *reinterpret_cast<bf16x4*>(orow + 16 * dt) =
            bf16x4{(bf16)ot[dt][0], (bf16)ot[dt][1], (bf16)ot[dt][2], (bf16)ot[dt][3]};
    }
  }
}

// Fused attention backward front half: dS = scale * P * (dP - rowsum(dP * P)) with dP = dO V^T computed
// per 16-query tile as dP^T = V dO^T in registers (same lane layout as the forward's S^T: lane (g, q) holds
// keys 16t + 4g .. +3 of query q), so the fp32 dP never goes to memory (the unfused path wrote and re-read
// 2 x Tp^2 x 4 B per head).  Same semantics as softmax_bwd: padded keys / queries get dS = 0.
template <int NT>
__global__ __launch_bounds__(256) void attn_bwd_ds_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ v,
                                                          const bf16* __restrict__ p, float scale,
                                                          bf16* __restrict__ ds) {
  constexpr int Tp = 16 * NT;
  __shared__ __attribute__((aligned(16))) bf16 Vs[Tp * ATT_D];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t bh = blockIdx.x;
  const bf16* vb = v + bh * Tp * ATT_D;
  for (int c = tid; c < Tp * 8; c += 256) {
    const int r = c >> 3, d = (c & 7) * 8;
    *reinterpret_cast<bf16x8*>(Vs + att_ksw(r, d)) = reinterpret_cast<const bf16x8*>(vb)[c];
  }
  __syncthreads();
  const int g = lane >> 4, qi = lane & 15;
  for (int qt = wave; qt < NT; qt += 4) {
    const int qrow = qt * 16 + qi;
    const bf16* dp_ = dout + (bh * Tp + qrow) * ATT_D + 8 * g;
    const bf16x8 of0 = *reinterpret_cast<const bf16x8*>(dp_);
    const bf16x8 of1 = *reinterpret_cast<const bf16x8*>(dp_ + 32);
    const bf16* prow = p + (bh * Tp + qrow) * Tp + 4 * g;
    bf16x4 pv[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) pv[t] = *reinterpret_cast<const bf16x4*>(prow + 16 * t);
    f32x4 dpt[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int vr = 16 * t + qi;
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(Vs + att_ksw(vr, 8 * g));
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(Vs + att_ksw(vr, 32 + 8 * g));
      dpt[t] = mfma16x16x32(a1, of1, mfma16x16x32(a0, of0, zero_f32x4()));
    }
    float dot = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) dot = fmaf(dpt[t][i], (float)pv[t][i], dot);
    dot += __shfl_xor(dot, 16, 64);
    dot += __shfl_xor(dot, 32, 64);
    bf16* drow = ds + (bh * Tp + qrow) * Tp + 4 * g;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      bf16x4 r;
#pragma unroll
      for (int i = 0; i < 4; ++i) r[i] = (bf16)(scale * (float)pv[t][i] * (dpt[t][i] - dot));
      *reinterpret_cast<bf16x4*>(drow + 16 * t) = r;
    }
  }
}

// Fused attention backward, query side: dS (as attn_bwd_ds, in registers) and dQ = dS K in the same
// pass - dQ^T = K^T dS^T with the dS registers as the MFMA B operand and K^T read from LDS with
// ds_read_b64_tr_b16 (the forward's O^T = V^T P^T trick).  dQ rows go straight into the dqkv gradient
// rows [B*T][3*H*Dh]; D = rowsum(dP * P) per query is stored for the key-side kernel.
// Column sums of a kernel's 64-wide output block (a bias gradient's partial): lane (g, i) holds sums for columns
// 16 dt + 4g + e; reduced over the 16 lanes of each g, then over the 4 waves through `scratch` (>= 1 KiB of the
// kernel's LDS, free once its main loop is done - the caller has passed a barrier), and stored as 64 floats.
__device__ __forceinline__ void attn_colsum_store(float (&cs)[4][4], float* scratch, float* __restrict__ out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float t = cs[dt][e];
      t += __shfl_xor(t, 1, 64);
      t += __shfl_xor(t, 2, 64);
      t += __shfl_xor(t, 4, 64);
      t += __shfl_xor(t, 8, 64);
      cs[dt][e] = t;
    }
  if ((lane & 15) == 0) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int e = 0; e < 4; ++e) scratch[wave * 64 + 16 * dt + 4 * g + e] = cs[dt][e];
  }
  __syncthreads();
  if (threadIdx.x < 64)
    out[threadIdx.x] = (scratch[threadIdx.x] + scratch[64 + threadIdx.x]) + (scratch[128 + threadIdx.x] + scratch[192 + threadIdx.x]);
}

template <int NT, bool LSE>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(AttnIn dout, AttnIn k, AttnIn v,
                                                          const bf16* __restrict__ p, float scale, int T, int H,
                                                          float* __restrict__ dsum, AttnOut dq, AttnIn q,
                                                          const float* __restrict__ lse, float* __restrict__ cs_out) {
  constexpr int Tp = 16 * NT;
  __shared__ __attribute__((aligned(16))) bf16 Vs[Tp * ATT_D];
  __shared__ __attribute__((aligned(16))) bf16 Ks[Tp * ATT_D];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bh = blockIdx.x;
  for (int c = tid; c < Tp * 8; c += 256) {
    const int r = c >> 3, d = (c & 7) * 8;
    *reinterpret_cast<bf16x8*>(Vs + att_ksw(r, d)) = v.load8(bh, H, r, T, d);
    *reinterpret_cast<bf16x8*>(Ks + att_vsw(r, d)) = k.load8(bh, H, r, T, d);
  }
  __syncthreads();
  const int g = lane >> 4, qi = lane & 15;
  const int q4 = qi >> 2, p4 = qi & 3;
  float csum[4][4] = {};  // cs_out: column sums of the stored dQ rows (the qkv bias gradient's q part)
  for (int qt = wave; qt < NT; qt += 4) {
    const int qrow = qt * 16 + qi;
    const bf16x8 of0 = dout.load8(bh, H, qrow, T, 8 * g);
    const bf16x8 of1 = dout.load8(bh, H, qrow, T, 32 + 8 * g);
    bf16x4 pv[NT];
    if constexpr (LSE) {  // P recomputed: S^T tile by tile exactly as the forward (lane (g, q): keys 16t + 4g + i)
      const bf16x8 qf0 = q.load8(bh, H, qrow, T, 8 * g);
      const bf16x8 qf1 = q.load8(bh, H, qrow, T, 32 + 8 * g);
      const float lq = lse[(int64_t)bh * Tp + qrow];  // +inf for padded queries: P = 0
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int kr = 16 * t + qi;
        const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(Ks + att_vsw(kr, 8 * g));
        const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(Ks + att_vsw(kr, 32 + 8 * g));
        const f32x4 sv = mfma16x16x32(a1, qf1, mfma16x16x32(a0, qf0, zero_f32x4()));
#pragma unroll
        for (int i = 0; i < 4; ++i) pv[t][i] = (bf16)(16 * t + 4 * g + i < T ? __expf(sv[i] * scale - lq) : 0.f);
      }
    } else {
      const bf16* prow = p + ((int64_t)bh * Tp + qrow) * Tp + 4 * g;
#pragma unroll
      for (int t = 0; t < NT; ++t) pv[t] = *reinterpret_cast<const bf16x4*>(prow + 16 * t);
    }
    // dP = dO V^T tile by tile, recomputed in the second pass instead of held: the NT x 4 fp32 dP
    // registers had pushed the kernel to 232 VGPRs (one wave per SIMD)
    auto dp_tile = [&](int t) {
      const int vr = 16 * t + qi;
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(Vs + att_ksw(vr, 8 * g));
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(Vs + att_ksw(vr, 32 + 8 * g));
      return mfma16x16x32(a1, of1, mfma16x16x32(a0, of0, zero_f32x4()));
    };
    float dot = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const f32x4 dpt = dp_tile(t);
#pragma unroll
      for (int i = 0; i < 4; ++i) dot = fmaf(dpt[i], (float)pv[t][i], dot);
    }
    dot += __shfl_xor(dot, 16, 64);
    dot += __shfl_xor(dot, 32, 64);
    if (g == 0) dsum[(int64_t)bh * Tp + qrow] = dot;
    asm volatile("" ::: "memory");  // pass 2 re-reads V from LDS: no CSE of the pass-1 dP registers
    auto ds_tile = [&](int t) {
      const f32x4 dpt = dp_tile(t);
      bf16x4 r;
#pragma unroll
      for (int i = 0; i < 4; ++i) r[i] = (bf16)(scale * (float)pv[t][i] * (dpt[i] - dot));
      return r;
    };
    // dQ^T[d][q] = sum over key pairs (t0, t1) of K^T (keys 16t + 4g + j) x dS^T
    f32x4 qt4[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) qt4[dt] = zero_f32x4();
#pragma unroll
    for (int ks = 0; ks < (NT + 1) / 2; ++ks) {
      const int t0 = 2 * ks, t1 = 2 * ks + 1 < NT ? 2 * ks + 1 : t0;
      const bf16x4 d0 = ds_tile(t0);
      const bf16x4 d1 = 2 * ks + 1 < NT ? ds_tile(2 * ks + 1) : bf16x4{(bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
      const bf16x8 bfr = bf16x8{d0[0], d0[1], d0[2], d0[3], d1[0], d1[1], d1[2], d1[3]};
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x4 lo = lds_read_tr16(Ks + att_vsw(16 * t0 + 4 * g + q4, 16 * dt + 4 * p4));
        const bf16x4 hi = lds_read_tr16(Ks + att_vsw(16 * t1 + 4 * g + q4, 16 * dt + 4 * p4));
        const bf16x8 afr = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        qt4[dt] = mfma16x16x32(afr, bfr, qt4[dt]);
      }
    }
    if (qrow < dq.rows) {
      bf16* drow = dq.row(bh, H, qrow) + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x4 o = bf16x4{(bf16)qt4[dt][0], (bf16)qt4[dt][1], (bf16)qt4[dt][2], (bf16)qt4[dt][3]};
        *reinterpret_cast<bf16x4*>(drow + 16 * dt) = o;
#pragma unroll
        for (int e = 0; e < 4; ++e) csum[dt][e] += (float)o[e];
      }
    }
  }
  if (cs_out) {  // [B][3*H*64] partial row of batch bh / H, columns of head bh % H (q part)
    __syncthreads();  // every wave is done with Vs
    attn_colsum_store(csum, reinterpret_cast<float*>(Vs), cs_out + (int64_t)(bh / H) * 3 * H * ATT_D + (bh % H) * ATT_D);
  }
}

// Fused attention backward, key side: each wave owns key tiles kt = wave, wave + 4, .. and walks all query
// tiles in pairs, recomputing dP = dO V^T for its keys (rows = queries: lane (g, key) holds queries
// 16qt + 4g + r), reading P and the stored D, forming dS = scale P (dP - D), and accumulating
//   dV^T[d][key] += dO^T P     and     dK^T[d][key] += Q^T dS
// with those registers as the MFMA B operand (reduction over the query pair, permuted like the forward's
// key pairs) and dO^T / Q^T read from LDS with ds_read_b64_tr_b16.  dK, dV rows go straight into dqkv.
template <int NT, bool LSE>
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(AttnIn dout, AttnIn q, AttnIn v,
                                                            const bf16* __restrict__ p, const float* __restrict__ dsum,
                                                            float scale, int T, int H, AttnOut dk, AttnOut dv,
                                                            AttnIn k, const float* __restrict__ lse,
                                                            float* __restrict__ cs_out) {
  constexpr int Tp = 16 * NT;
  __shared__ __attribute__((aligned(16))) bf16 Qs[Tp * ATT_D];
  __shared__ __attribute__((aligned(16))) bf16 Os[Tp * ATT_D];  // dO
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bh = blockIdx.x;
  for (int c = tid; c < Tp * 8; c += 256) {
    const int r = c >> 3, d = (c & 7) * 8;
    *reinterpret_cast<bf16x8*>(Qs + att_vsw(r, d)) = q.load8(bh, H, r, T, d);
    *reinterpret_cast<bf16x8*>(Os + att_vsw(r, d)) = dout.load8(bh, H, r, T, d);
  }
  __syncthreads();
  const int g = lane >> 4, ki = lane & 15;
  const int q4 = ki >> 2, p4 = ki & 3;
  // per-query D = rowsum(dP * P) and log-sum-exp: a lane's 4 queries 16 qp + 4g + r are one 16-B load each
  const float* db = dsum + (int64_t)bh * Tp;
  const float* lq = LSE ? lse + (int64_t)bh * Tp : nullptr;
  float csk[4][4] = {}, csv[4][4] = {};  // cs_out: column sums of the stored dK / dV rows
  for (int kt = wave; kt < NT; kt += 4) {
    const int key = kt * 16 + ki;
    const bf16x8 vf0 = v.load8(bh, H, key, T, 8 * g);
    const bf16x8 vf1 = v.load8(bh, H, key, T, 32 + 8 * g);
    bf16x8 kf0 = zero_bf16x8(), kf1 = zero_bf16x8();
    if constexpr (LSE) {
      kf0 = k.load8(bh, H, key, T, 8 * g);
      kf1 = k.load8(bh, H, key, T, 32 + 8 * g);
    }
    const bf16* pcol = p + (int64_t)bh * Tp * Tp + key;
    f32x4 dva[4], dka[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dva[dt] = dka[dt] = zero_f32x4();
#pragma unroll 1  // (unrolled, the hoisted per-pair loads take the kernel to 256 VGPRs)
    for (int ks = 0; ks < (NT + 1) / 2; ++ks) {
      const int qp[2] = {2 * ks, 2 * ks + 1 < NT ? 2 * ks + 1 : 2 * ks};
      const bool has1 = 2 * ks + 1 < NT;
      bf16x4 pb[2], sb[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        // dP[q][key] for queries 16 qp + 4g + r: A = dO rows (from the LDS image), B = V rows (registers)
        const int orow = 16 * qp[u] + ki;
        const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(Os + att_vsw(orow, 8 * g));
        const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(Os + att_vsw(orow, 32 + 8 * g));
        const f32x4 dpv = mfma16x16x32(a1, vf1, mfma16x16x32(a0, vf0, zero_f32x4()));
        f32x4 spv = zero_f32x4();
        if constexpr (LSE) {  // S[q][key] for the same queries: A = Q rows (LDS image), B = K rows (registers)
          const bf16x8 c0 = *reinterpret_cast<const bf16x8*>(Qs + att_vsw(orow, 8 * g));
          const bf16x8 c1 = *reinterpret_cast<const bf16x8*>(Qs + att_vsw(orow, 32 + 8 * g));
          spv = mfma16x16x32(c1, kf1, mfma16x16x32(c0, kf0, zero_f32x4()));
        }
        const f32x4 dq4 = *reinterpret_cast<const f32x4*>(db + 16 * qp[u] + 4 * g);
        f32x4 lq4 = zero_f32x4();
        if constexpr (LSE) lq4 = *reinterpret_cast<const f32x4*>(lq + 16 * qp[u] + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qq = 16 * qp[u] + 4 * g + r;
          float pr;
          if constexpr (LSE)  // the bf16 value the forward would have stored
            pr = (u == 0 || has1) && key < T ? (float)(bf16)__expf(spv[r] * scale - lq4[r]) : 0.f;
          else
            pr = (u == 0 || has1) ? (float)pcol[(int64_t)qq * Tp] : 0.f;
          pb[u][r] = (bf16)pr;
          sb[u][r] = (bf16)(scale * pr * (dpv[r] - dq4[r]));
        }
      }
      const bf16x8 pfr = bf16x8{pb[0][0], pb[0][1], pb[0][2], pb[0][3], pb[1][0], pb[1][1], pb[1][2], pb[1][3]};
      const bf16x8 sfr = bf16x8{sb[0][0], sb[0][1], sb[0][2], sb[0][3], sb[1][0], sb[1][1], sb[1][2], sb[1][3]};
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x4 olo = lds_read_tr16(Os + att_vsw(16 * qp[0] + 4 * g + q4, 16 * dt + 4 * p4));
        const bf16x4 ohi = lds_read_tr16(Os + att_vsw(16 * qp[1] + 4 * g + q4, 16 * dt + 4 * p4));
        dva[dt] = mfma16x16x32(bf16x8{olo[0], olo[1], olo[2], olo[3], ohi[0], ohi[1], ohi[2], ohi[3]}, pfr, dva[dt]);
        const bf16x4 qlo = lds_read_tr16(Qs + att_vsw(16 * qp[0] + 4 * g + q4, 16 * dt + 4 * p4));
        const bf16x4 qhi = lds_read_tr16(Qs + att_vsw(16 * qp[1] + 4 * g + q4, 16 * dt + 4 * p4));
        dka[dt] = mfma16x16x32(bf16x8{qlo[0], qlo[1], qlo[2], qlo[3], qhi[0], qhi[1], qhi[2], qhi[3]}, sfr, dka[dt]);
      }
    }
    if (key < dk.rows) {
      bf16* krow = dk.row(bh, H, key) + 4 * g;
      bf16* vrow = dv.row(bh, H, key) + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x4 ko = bf16x4{(bf16)dka[dt][0], (bf16)dka[dt][1], (bf16)dka[dt][2], (bf16)dka[dt][3]};
        const bf16x4 vo = bf16x4{(bf16)dva[dt][0], (bf16)dva[dt][1], (bf16)dva[dt][2], (bf16)dva[dt][3]};
        *reinterpret_cast<bf16x4*>(krow + 16 * dt) = ko;
        *reinterpret_cast<bf16x4*>(vrow + 16 * dt) = vo;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          csk[dt][e] += (float)ko[e];
          csv[dt][e] += (float)vo[e];
        }
      }
    }
  }
  if (cs_out) {  // k part, then v part of the [B][3*H*64] partial row
    float* row = cs_out + (int64_t)(bh / H) * 3 * H * ATT_D + (bh % H) * ATT_D;
    __syncthreads();  // every wave is done with Qs / Os
    attn_colsum_store(csk, reinterpret_cast<float*>(Qs), row + H * ATT_D);
    attn_colsum_store(csv, reinterpret_cast<float*>(Os), row + 2 * H * ATT_D);
  }
}

template <int NT>
void attn_bwd_launch(AttnIn dout, AttnIn q, AttnIn k, AttnIn v, const void* p, int BH, int T, int H, float scale,
                     float* dsum, AttnOut dq, AttnOut dk, AttnOut dv, hipStream_t s, const float* lse = nullptr,
                     float* cs = nullptr) {
  if (lse) {
    attn_bwd_dq_kernel<NT, true><<<BH, 256, 0, s>>>(dout, k, v, nullptr, scale, T, H, dsum, dq, q, lse, cs);
    attn_bwd_dkdv_kernel<NT, true><<<BH, 256, 0, s>>>(dout, q, v, nullptr, dsum, scale, T, H, dk, dv, k, lse, cs);
    return;
  }
  attn_bwd_dq_kernel<NT, false><<<BH, 256, 0, s>>>(dout, k, v, static_cast<const bf16*>(p), scale, T, H, dsum, dq, q,
                                                   nullptr, cs);
  attn_bwd_dkdv_kernel<NT, false><<<BH, 256, 0, s>>>(dout, q, v, static_cast<const bf16*>(p), dsum, scale, T, H, dk, dv,
                                                     k, nullptr, cs);
}

template <int NT>
void attn_bwd_ds_launch(const void* dout, const void* v, const void* p, int BH, float scale, void* ds,
                        hipStream_t s) {
  attn_bwd_ds_kernel<NT><<<BH, 256, 0, s>>>(static_cast<const bf16*>(dout), static_cast<const bf16*>(v),
                                            static_cast<const bf16*>(p), scale, static_cast<bf16*>(ds));
}

template <int NT>
void attn_fwd_launch(AttnIn q, AttnIn k, AttnIn v, int BH, int T, int H, float scale, void* p, AttnOut o,
                     hipStream_t s, float* lse = nullptr) {
  if (lse)
    attn_fwd_kernel<NT, true><<<BH, 256, 0, s>>>(q, k, v, T, H, scale, nullptr, o, lse);
  else
    attn_fwd_kernel<NT, false><<<BH, 256, 0, s>>>(q, k, v, T, H, scale, static_cast<bf16*>(p), o, nullptr);
}

}  // namespace

// head-major [BH][Tp][64] views (H = 1: bh is the batch index) and token-row views of a [B*T][width]
// matrix at column offset col0
static AttnIn head_major(const void* base, int Tp) {
  return AttnIn{static_cast<const bf16*>(base), (int64_t)Tp * ATT_D, 0, ATT_D};
}
static AttnOut head_major_out(void* base, int Tp) { return AttnOut{static_cast<bf16*>(base), (int64_t)Tp * ATT_D, 0, ATT_D, Tp}; }
static AttnIn token_rows(const void* base, int T, int64_t width, int64_t col0) {
  return AttnIn{static_cast<const bf16*>(base) + col0, (int64_t)T * width, ATT_D, width};
}
static AttnOut token_rows_out(void* base, int T, int64_t width, int64_t col0) {
  return AttnOut{static_cast<bf16*>(base) + col0, (int64_t)T * width, ATT_D, width, T};
}

#define RINGDP_ATT_SWITCH(CALL)                                                                          \
  switch (Tp / 16) {                                                                                     \
    case 1: { constexpr int n = 1; CALL; return true; }   case 2: { constexpr int n = 2; CALL; return true; }   \
    case 3: { constexpr int n = 3; CALL; return true; }   case 4: { constexpr int n = 4; CALL; return true; }   \
    case 5: { constexpr int n = 5; CALL; return true; }   case 6: { constexpr int n = 6; CALL; return true; }   \
    case 7: { constexpr int n = 7; CALL; return true; }   case 8: { constexpr int n = 8; CALL; return true; }   \
    case 9: { constexpr int n = 9; CALL; return true; }   case 10: { constexpr int n = 10; CALL; return true; } \
    case 11: { constexpr int n = 11; CALL; return true; } case 12: { constexpr int n = 12; CALL; return true; } \
    case 13: { constexpr int n = 13; CALL; return true; } case 14: { constexpr int n = 14; CALL; return true; } \
    case 15: { constexpr int n = 15; CALL; return true; } case 16: { constexpr int n = 16; CALL; return true; } \
  }

bool attn_fwd(const void* q, const void* k, const void* v, int BH, int T, int Tp, int Dh, float scale, void* p,
              void* o, hipStream_t s) {
  if (Dh != ATT_D || Tp % 16 != 0 || Tp > 256 || Tp < 16 || T > Tp) return false;
  RINGDP_ATT_SWITCH((attn_fwd_launch<n>(head_major(q, Tp), head_major(k, Tp), head_major(v, Tp), BH, T, 1, scale, p,
                                        head_major_out(o, Tp), s)))
  return false;
}

bool attn_fwd_rows(const void* qkv, int B, int T, int H, int Tp, int Dh, float scale, void* p, void* out,
                   hipStream_t s) {
  if (Dh != ATT_D || Tp % 16 != 0 || Tp > 256 || Tp < 16 || T > Tp) return false;
  const int64_t w3 = (int64_t)3 * H * ATT_D, w1 = (int64_t)H * ATT_D;
  RINGDP_ATT_SWITCH((attn_fwd_launch<n>(token_rows(qkv, T, w3, 0), token_rows(qkv, T, w3, w1),
                                        token_rows(qkv, T, w3, 2 * w1), B * H, T, H, scale, p,
                                        token_rows_out(out, T, w1, 0), s)))
  return false;
}

bool attn_fwd_rows_lse(const void* qkv, int B, int T, int H, int Tp, int Dh, float scale, float* lse, void* out,
                       hipStream_t s) {
  if (Dh != ATT_D || Tp % 16 != 0 || Tp > 256 || Tp < 16 || T > Tp) return false;
  const int64_t w3 = (int64_t)3 * H * ATT_D, w1 = (int64_t)H * ATT_D;
  RINGDP_ATT_SWITCH((attn_fwd_launch<n>(token_rows(qkv, T, w3, 0), token_rows(qkv, T, w3, w1),
                                        token_rows(qkv, T, w3, 2 * w1), B * H, T, H, scale, nullptr,
                                        token_rows_out(out, T, w1, 0), s, lse)))
  return false;
}

bool attn_bwd_ds(const void* dout, const void* v, const void* p, int BH, int Tp, int Dh, float scale, void* ds,
                 hipStream_t s) {
  if (Dh != ATT_D || Tp % 16 != 0 || Tp > 256 || Tp < 16) return false;
  switch (Tp / 16) {
#define RINGDP_ATT_CASE(n) \
  case n:                 \
    attn_bwd_ds_launch<n>(dout, v, p, BH, scale, ds, s); \
    return true;
    RINGDP_ATT_CASE(1) RINGDP_ATT_CASE(2) RINGDP_ATT_CASE(3) RINGDP_ATT_CASE(4) RINGDP_ATT_CASE(5)
    RINGDP_ATT_CASE(6) RINGDP_ATT_CASE(7) RINGDP_ATT_CASE(8) RINGDP_ATT_CASE(9) RINGDP_ATT_CASE(10)
    RINGDP_ATT_CASE(11) RINGDP_ATT_CASE(12) RINGDP_ATT_CASE(13) RINGDP_ATT_CASE(14) RINGDP_ATT_CASE(15)
    RINGDP_ATT_CASE(16)
#undef RINGDP_ATT_CASE
  }
  return false;
}

bool attn_bwd(const void* dout, const void* q, const void* k, const void* v, const void* p, int B, int T, int H,
              int Tp, int Dh, float scale, float* dsum, void* dqkv, hipStream_t s) {
  if (Dh != ATT_D || Tp % 16 != 0 || Tp > 256 || Tp < 16 || T > Tp) return false;
  // head-major operands of batch bh = b*H + h: element (bh, t) at bh*Tp*64 + t*64 = b*(H*Tp*64) + h*(Tp*64) + ..
  const int64_t hm = (int64_t)Tp * ATT_D;
  auto hmv = [&](const void* base) { return AttnIn{static_cast<const bf16*>(base), H * hm, hm, ATT_D}; };
  const int64_t w3 = (int64_t)3 * H * ATT_D, w1 = (int64_t)H * ATT_D;
  RINGDP_ATT_SWITCH((attn_bwd_launch<n>(hmv(dout), hmv(q), hmv(k), hmv(v), p, B * H, T, H, scale, dsum,
                                        token_rows_out(dqkv, T, w3, 0), token_rows_out(dqkv, T, w3, w1),
                                        token_rows_out(dqkv, T, w3, 2 * w1), s)))
  return false;
}

bool attn_bwd_rows(const void* dout_rows, const void* qkv, const void* p, int B, int T, int H, int Tp, int Dh,
                   float scale, float* dsum, void* dqkv, hipStream_t s) {
  if (Dh != ATT_D || Tp % 16 != 0 || Tp > 256 || Tp < 16 || T > Tp) return false;
  const int64_t w3 = (int64_t)3 * H * ATT_D, w1 = (int64_t)H * ATT_D;
  RINGDP_ATT_SWITCH((attn_bwd_launch<n>(token_rows(dout_rows, T, w1, 0), token_rows(qkv, T, w3, 0),
                                        token_rows(qkv, T, w3, w1), token_rows(qkv, T, w3, 2 * w1), p, B * H, T, H,
                                        scale, dsum, token_rows_out(dqkv, T, w3, 0), token_rows_out(dqkv, T, w3, w1),
                                        token_rows_out(dqkv, T, w3, 2 * w1), s)))
  return false;
}

bool attn_bwd_rows_lse(const void* dout_rows, const void* qkv, const float* lse, int B, int T, int H, int Tp, int Dh,
                       float scale, float* dsum, void* dqkv, hipStream_t s, float* colsum_part) {
  if (Dh != ATT_D || Tp % 16 != 0 || Tp > 256 || Tp < 16 || T > Tp) return false;
  const int64_t w3 = (int64_t)3 * H * ATT_D, w1 = (int64_t)H * ATT_D;
  RINGDP_ATT_SWITCH((attn_bwd_launch<n>(token_rows(dout_rows, T, w1, 0), token_rows(qkv, T, w3, 0),
                                        token_rows(qkv, T, w3, w1), token_rows(qkv, T, w3, 2 * w1), nullptr, B * H, T,
                                        H, scale, dsum, token_rows_out(dqkv, T, w3, 0), token_rows_out(dqkv, T, w3, w1),
                                        token_rows_out(dqkv, T, w3, 2 * w1), s, lse, colsum_part)))
  return false;
}

void softmax_bwd(const void* p, const float* dp, int64_t rows, int T, int Tp, float scale, void* ds, hipStream_t s) {
  if (Tp <= 256 && Tp % 4 == 0)
    softmax_bwd_vec_kernel<<<(int)((rows + 3) / 4), 256, 0, s>>>(static_cast<const bf16*>(p), dp, rows, T, Tp, scale,
                                                             static_cast<bf16*>(ds));
  else
    softmax_bwd_kernel<<<(int)((rows + 3) / 4), 256, 0, s>>>(static_cast<const bf16*>(p), dp, rows, T, Tp, scale,
                                                           static_cast<bf16*>(ds));
}

void gelu_fwd(const void* x, int64_t n, void* y, hipStream_t s) {
  gelu_fwd_kernel<<<grid_for(n / 8), 256, 0, s>>>(static_cast<const bf16*>(x), n / 8, static_cast<bf16*>(y));
}

void gelu_bwd(const void* dy, const void* pre, int64_t n, void* dx, hipStream_t s) {
  gelu_bwd_kernel<<<grid_for(n / 8), 256, 0, s>>>(static_cast<const bf16*>(dy), static_cast<const bf16*>(pre), n / 8,
                                                  static_cast<bf16*>(dx));
}

void assemble_tokens(const void* patches, const float* cls, const float* pos, int B, int NP, int D, void* out,
                     hipStream_t s) {
  assemble_tokens_kernel<<<grid_for((int64_t)B * (NP + 1) * D), 256, 0, s>>>(static_cast<const bf16*>(patches), cls, pos,
                                                                             B, NP, D, static_cast<bf16*>(out));
}

void assemble_tokens_bwd(const void* dout, int B, int NP, int D, void* dpatches, float* dpos, float* dcls,
                         hipStream_t s) {
  assemble_tokens_bwd_kernel<<<grid_for((int64_t)(NP + 1) * D), 256, 0, s>>>(static_cast<const bf16*>(dout), B, NP, D,
                                                                             static_cast<bf16*>(dpatches), dpos, dcls);
}

void cls_rows(const void* x, int B, int T, int D, void* y, bool reverse, hipStream_t s) {
  cls_rows_kernel<<<grid_for((int64_t)B * D), 256, 0, s>>>(static_cast<const bf16*>(x), B, T, D, static_cast<bf16*>(y),
                                                           reverse ? 1 : 0);
}

}  // namespace kern
}  // namespace ringdp
