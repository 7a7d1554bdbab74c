// NHWC bf16 network layers around the implicit-GEMM convolutions (ResNet family; SURVEY.md §2.4
// "U14 ATen BN, add, avgpool (W2)"; ref/example_mp.py:50 resnet18).
//
// Batch norm is split MI355X-first: the per-channel sum / sum-of-squares come out of the producing
// conv's GEMM epilogue (gemm.hip, deterministic per-tile partials), so BN forward is ONE
// elementwise pass that also fuses the residual add and the ReLU; BN backward is one reduction pass
// (ReLU mask + the two channel sums) and one apply pass that also emits the residual branch's grad.
// Every kernel moves 16-B vectors of 8 channels.
#include <algorithm>
#include <cstdlib>

#include "device_common.h"
#include "kernels.h"

namespace ringdp {
namespace kern {

using namespace ringdp::dev;

namespace {

inline int grid_for(int64_t n, int per_block = 256, int cap = 4096) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + per_block - 1) / per_block, cap));
}

// KRSC rows are ldk >= R*S*Cp elements long (zero tail: the stem's k-range padded to whole 64-wide
// k-tiles, see ConvFwdA8 in gemm.hip)
__global__ __launch_bounds__(256) void pack_conv_weight_kernel(const float* __restrict__ w, int K, int C, int R,
                                                               int S, int Cp, int ldk, bf16* __restrict__ krsc,
                                                               bf16* __restrict__ crsk) {
  const int64_t total = (int64_t)K * ldk;
  const int kd = R * S * Cp;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int k = (int)(e / ldk), j = (int)(e - (int64_t)k * ldk);
    if (j >= kd) {
      krsc[e] = (bf16)0.f;
      continue;
    }
    // j indexes RSC(padded): j = (r*S + s)*Cp + c
    const int c = j % Cp, rs = j / Cp, sx = rs % S, r = rs / S;
    const float v = c < C ? w[(((int64_t)k * C + c) * R + r) * S + sx] : 0.f;
    krsc[e] = (bf16)v;
    crsk[(((int64_t)c * R + r) * S + sx) * K + k] = (bf16)v;
  }
}

// Many conv weights in one launch (a ResNet packs 21-53 of them per forward): the table travels as a
// kernel argument; each thread finds its weight by a scan of the prefix offsets (uniform per wave
// except at boundaries).
__device__ __forceinline__ void pack_table_to_lds(const PackTable& t, PackEntry* se) {
  // compile-time indices: indexing the by-value argument with a run-time index would copy it to
  // scratch memory per thread
#pragma unroll
  for (int i = 0; i < kPackMax; ++i)
    if (threadIdx.x == i && i < t.n) se[i] = t.e[i];
  __syncthreads();
}

// KRSC rows (row-padded): element j of row k = w[k][c][r][s], j = (r*S + s)*Cp + c; the source row is
// contiguous, so its strided gather stays in L1/L2
__global__ __launch_bounds__(256) void pack_krsc_multi_kernel(PackTable t) {
  __shared__ PackEntry se[kPackMax];
  pack_table_to_lds(t, se);
  int i = 0;  // f only grows: the table scan resumes where it stopped
  for (int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x; f < t.total; f += (int64_t)gridDim.x * 256) {
    while (i + 1 < t.n && f >= se[i + 1].start) ++i;
    const PackEntry d = se[i];
    const int64_t le = f - d.start;
    const int k = (int)(le / d.ldk), j = (int)(le - (int64_t)k * d.ldk);
    float v = 0.f;
    if (j < d.R * d.S * d.Cp) {
      const int c = j % d.Cp, rs = j / d.Cp;
      if (c < d.C) v = d.w[((int64_t)k * d.C + c) * d.R * d.S + rs];
    }
    static_cast<bf16*>(d.krsc)[le] = (bf16)v;
  }
}

// CRSK = the transpose of w viewed as [K][C*R*S] (same (c, r, s) order), plus zero rows for the padded
// channels: 64x64 tiles through LDS, both sides coalesced.  blockIdx.x = a tile of some entry
// (start_tile prefix over the entries).
__global__ __launch_bounds__(256) void pack_crsk_multi_kernel(PackTable t) {
  __shared__ PackEntry se[kPackMax];
  __shared__ float tile[64][65];
  pack_table_to_lds(t, se);
  const int b = blockIdx.x;
  int i = 0;
  while (i + 1 < t.n && b >= se[i + 1].start_tile) ++i;
  const PackEntry d = se[i];
  const int crs_real = d.C * d.R * d.S, crs_all = d.Cp * d.R * d.S;
  const int tiles_k = (d.K + 63) / 64;
  const int tb = b - (int)d.start_tile;
  const int crs0 = (tb / tiles_k) * 64, k0 = (tb % tiles_k) * 64;
  for (int idx = threadIdx.x; idx < 64 * 64; idx += 256) {
    const int kk = idx >> 6, cc = idx & 63;
    const int k = k0 + kk, crs = crs0 + cc;
    tile[kk][cc] = (k < d.K && crs < crs_real) ? d.w[(int64_t)k * crs_real + crs] : 0.f;
  }
  __syncthreads();
  bf16* out = static_cast<bf16*>(d.crsk);
  for (int idx = threadIdx.x; idx < 64 * 64; idx += 256) {
    const int cc = idx >> 6, kk = idx & 63;
    const int k = k0 + kk, crs = crs0 + cc;
    if (k < d.K && crs < crs_all) out[(int64_t)crs * d.K + k] = (bf16)tile[kk][cc];
  }
}

// Both bf16 layouts from ONE read of each fp32 weight (the two kernels above read it twice, the KRSC one with
// a strided gather): a tile of 32 output channels x ct input channels x all R*S taps - a contiguous run of each
// source row - is staged in LDS, then written as KRSC rows (runs of ct channels) and CRSK rows (runs of 32
// output channels).  Padded channels (c >= C) and the stem's row tail (ldk > R*S*Cp) are written as zeros.
constexpr int kPackTileFloats = 32 * 8 * 49;  // the largest tile: the 7x7 stem, Cp = 8 (3x3: 32 x 32 x 9)
__device__ __forceinline__ int pack_ct_dev(int Cp) { return Cp < 32 ? Cp : 32; }  // = kern::pack_ct
__global__ __launch_bounds__(256) void pack_both_multi_kernel(PackTable t) {
  __shared__ PackEntry se[kPackMax];
  __shared__ float tile[kPackTileFloats];
  pack_table_to_lds(t, se);
  const int b = blockIdx.x;
  int i = 0;
  while (i + 1 < t.n && b >= se[i + 1].start_tile2) ++i;
  const PackEntry d = se[i];
  const int RS = d.R * d.S, ct = pack_ct_dev(d.Cp), nct = (d.Cp + ct - 1) / ct;
  const int tb = b - d.start_tile2;
  const int k0 = (tb / nct) * 32, c0 = (tb % nct) * ct;
  const int run = ct * RS;  // floats of one source row in this tile
  // load: tile[kk][cc * RS + rs] = w[k0 + kk][c0 + cc][rs] (contiguous in the source)
  for (int idx = threadIdx.x; idx < 32 * run; idx += 256) {
    const int kk = idx / run, r = idx - kk * run, c = c0 + r / RS, k = k0 + kk;
    tile[idx] = (k < d.K && c < d.C) ? d.w[(int64_t)k * d.C * RS + (int64_t)c0 * RS + r] : 0.f;
  }
  __syncthreads();
  bf16* krsc = static_cast<bf16*>(d.krsc);
  bf16* crsk = static_cast<bf16*>(d.crsk);
  // KRSC: row k, element rs * Cp + c (runs of ct consecutive channels), 8 channels (one 16-B store) per thread;
  // ct, Cp and ldk are multiples of 8
  const int cv = ct >> 3;
  for (int idx = threadIdx.x; idx < 32 * RS * cv; idx += 256) {
    const int kk = idx / (RS * cv), r = idx - kk * RS * cv, rs = r / cv, cc = (r - rs * cv) * 8, k = k0 + kk;
    if (k >= d.K || c0 + cc >= d.Cp) continue;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (bf16)tile[kk * run + (cc + j) * RS + rs];
    *reinterpret_cast<bf16x8*>(krsc + (int64_t)k * d.ldk + rs * d.Cp + c0 + cc) = v;
  }
  // CRSK: row (c, rs), element k (runs of 32 output channels): 8 per thread when K % 8 == 0
  if ((d.K & 7) == 0) {
    for (int idx = threadIdx.x; idx < 4 * run; idx += 256) {
      const int crs = idx >> 2, kk = (idx & 3) * 8, cc = crs / RS, rs = crs - cc * RS, k = k0 + kk;
      if (k >= d.K || c0 + cc >= d.Cp) continue;
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (bf16)tile[(kk + j) * run + cc * RS + rs];
      *reinterpret_cast<bf16x8*>(crsk + ((int64_t)(c0 + cc) * RS + rs) * d.K + k) = v;
    }
  } else {
    for (int idx = threadIdx.x; idx < 32 * run; idx += 256) {
      const int crs = idx >> 5, kk = idx & 31, cc = crs / RS, rs = crs - cc * RS, k = k0 + kk;
      if (k < d.K && c0 + cc < d.Cp)
        crsk[((int64_t)(c0 + cc) * RS + rs) * d.K + k] = (bf16)tile[kk * run + cc * RS + rs];
    }
  }
  // the zero tail of KRSC rows padded to whole 64-wide k-tiles (the stem)
  const int kd = RS * d.Cp;
  if (c0 == 0 && d.ldk > kd) {
    const int tail = d.ldk - kd;
    for (int idx = threadIdx.x; idx < 32 * tail; idx += 256) {
      const int kk = idx / tail, j = kd + idx - kk * tail, k = k0 + kk;
      if (k < d.K) krsc[(int64_t)k * d.ldk + j] = (bf16)0.f;
    }
  }
}

template <bool BF>
__global__ __launch_bounds__(256) void nchw_to_nhwc_kernel(const void* __restrict__ x, int N, int C, int H, int W,
                                                           int Cp, bf16* __restrict__ y) {
  const int64_t total = (int64_t)N * H * W * Cp;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int c = (int)(e % Cp);
    const int64_t pix = e / Cp;  // n*H*W + h*W + w
    const int64_t n = pix / ((int64_t)H * W), hw = pix - n * H * W;
    float v = 0.f;
    if (c < C) {
      const int64_t src = (n * C + c) * H * W + hw;
      v = BF ? (float)static_cast<const bf16*>(x)[src] : static_cast<const float*>(x)[src];
    }
    y[e] = (bf16)v;
  }
}

// sums = G group partials [G][2][C] of the conv epilogue's per-tile statistics (first level of
// reduce_parts); the second level is summed here in the same fixed order (one launch fewer per BN).
// 64 channels [c0, c0 + 64) per call, 256 threads: wave w sums groups w, w+4, .. and the 4 wave totals
// combine in a fixed order; wave 0 then forms the per-channel scale / shift (-> sc_out / sh_out, either
// may be LDS) and, if write_stats, save / running statistics.  red: [4][2][64] floats.
__device__ __forceinline__ void bn_stats64(const float* __restrict__ sums, int G, int64_t M, int C, int c0,
                                           const float* __restrict__ gamma, const float* __restrict__ beta,
                                           float eps, float momentum, float* __restrict__ running_mean,
                                           float* __restrict__ running_var, float* sc_out, float* sh_out,
                                           float* __restrict__ save, bool write_stats, float (*red)[2][64]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = c0 + lane;
  // 4 independent partial chains per wave (loads of 4 groups in flight): the serial chain over G/4 groups
  // was latency-bound (10 us at G = 64 for a ResNet-18 layer-2 conv); combined in a fixed order
  float a4[4] = {0.f, 0.f, 0.f, 0.f}, q4[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    int g = wave;
    for (; g + 12 < G; g += 16) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a4[u] += sums[(int64_t)(g + 4 * u) * 2 * C + c];
        q4[u] += sums[(int64_t)(g + 4 * u) * 2 * C + C + c];
      }
    }
    for (; g < G; g += 4) {
      a4[0] += sums[(int64_t)g * 2 * C + c];
      q4[0] += sums[(int64_t)g * 2 * C + C + c];
    }
  }
  red[wave][0][lane] = (a4[0] + a4[1]) + (a4[2] + a4[3]);
  red[wave][1][lane] = (q4[0] + q4[1]) + (q4[2] + q4[3]);
  __syncthreads();
  if (wave == 0 && c < C) {
    const float s1 = (red[0][0][lane] + red[1][0][lane]) + (red[2][0][lane] + red[3][0][lane]);
    const float s2 = (red[0][1][lane] + red[1][1][lane]) + (red[2][1][lane] + red[3][1][lane]);
    const double inv = 1.0 / (double)M;
    const double mean = s1 * inv;
    const double var = fmax(s2 * inv - mean * mean, 0.0);  // biased (normalisation)
    const float invstd = (float)(1.0 / sqrt(var + eps));
    const float sc = gamma[c] * invstd;
    sc_out[c] = sc;
    sh_out[c] = beta[c] - (float)mean * sc;
    if (write_stats) {
      save[c] = (float)mean;
      save[C + c] = invstd;
      if (running_mean) {
        const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
        running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
        running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unbiased;
      }
    }
  }
  __syncthreads();  // red reusable
}

// nbt: BatchNorm.num_batches_tracked, incremented on device (one launch fewer again).
__global__ __launch_bounds__(256) void bn_prepare_kernel(const float* __restrict__ sums, int G, int64_t M, int C,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float eps, float momentum,
                                                         float* __restrict__ running_mean,
                                                         float* __restrict__ running_var, float* __restrict__ ss,
                                                         float* __restrict__ save, int64_t* __restrict__ nbt) {
  __shared__ float red[4][2][64];
  if (nbt && blockIdx.x == 0 && threadIdx.x == 0) nbt[0] += 1;
  bn_stats64(sums, G, M, C, blockIdx.x * 64, gamma, beta, eps, momentum, running_mean, running_var, ss, ss + C, save,
             true, red);
}

__global__ __launch_bounds__(256) void bn_act_fwd_kernel(const bf16* __restrict__ z, const float* __restrict__ ss,
                                                         const bf16* __restrict__ res, int relu, int64_t nvec, int C,
                                                         bf16* __restrict__ y) {
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    const int c0 = (int)((v * 8) % C);
    const bf16x8 zv = reinterpret_cast<const bf16x8*>(z)[v];
    bf16x8 rv = zero_bf16x8();
    if (res) rv = reinterpret_cast<const bf16x8*>(res)[v];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float f = (float)zv[j] * ss[c0 + j] + ss[C + c0 + j];
      if (res) f += (float)rv[j];
      if (relu) f = fmaxf(f, 0.f);
      o[j] = (bf16)f;
    }
    reinterpret_cast<bf16x8*>(y)[v] = o;
  }
}

// Column-stationary variants (C/8 divides 256: every ResNet width 64..2048): thread t owns the 8-channel
// column t % (C/8) for its whole life, so the per-channel coefficients are loaded once into registers
// (the grid-stride kernels above recompute a 64-bit modulo and reload 16-24 scalars per vector), and
// each thread keeps 4 rows of 16-B loads in flight.
constexpr int kBnUnroll = 4;

__device__ __forceinline__ void load8(const float* p, float (&o)[8]) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

template <bool kRes, bool kRelu>
__global__ __launch_bounds__(256) void bn_act_fwd_col_kernel(const bf16* __restrict__ z, const float* __restrict__ ss,
                                                             const bf16* __restrict__ res, int64_t M, int C,
                                                             bf16* __restrict__ y) {
  const int cv = C >> 3, rpb = 256 / cv;
  const int col = threadIdx.x % cv, rsub = threadIdx.x / cv;
  float sc[8], sh[8];
  load8(ss + col * 8, sc);
  load8(ss + C + col * 8, sh);
  const int64_t rstride = (int64_t)gridDim.x * rpb;
  for (int64_t r = (int64_t)blockIdx.x * rpb + rsub; r < M; r += kBnUnroll * rstride) {
    bf16x8 zv[kBnUnroll], rv[kBnUnroll];
#pragma unroll
    for (int u = 0; u < kBnUnroll; ++u) {
      const int64_t rr = r + u * rstride;
      if (rr < M) {
        zv[u] = reinterpret_cast<const bf16x8*>(z)[rr * cv + col];
        if (kRes) rv[u] = reinterpret_cast<const bf16x8*>(res)[rr * cv + col];
      }
    }
#pragma unroll
    for (int u = 0; u < kBnUnroll; ++u) {
      const int64_t rr = r + u * rstride;
      if (rr < M) {
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float f = fmaf((float)zv[u][j], sc[j], sh[j]);
          if (kRes) f += (float)rv[u][j];
          if (kRelu) f = fmaxf(f, 0.f);
          o[j] = (bf16)f;
        }
        reinterpret_cast<bf16x8*>(y)[rr * cv + col] = o;
      }
    }
  }
}

// BN forward with the statistics step folded in (few groups: kBnFoldMax): every workgroup forms the
// scale / shift of all C channels from the G group partials itself (bn_stats64, the prepare kernel's fixed
// order, so bit-identical to the two-launch path) into LDS; workgroup 0 also writes save / running
// statistics / num_batches_tracked.  One launch per BN instead of two.
struct BnFold {
  const float* sums;
  int G;
  const float* gamma;
  const float* beta;
  float eps, momentum;
  float* running_mean;
  float* running_var;
  float* save;
  int64_t* nbt;
};
constexpr int kBnFoldMax = 8192;  // G * C at most (the partials every workgroup re-reads from L2)

template <bool kRes, bool kRelu>
__global__ __launch_bounds__(256) void bn_fold_act_fwd_kernel(const bf16* __restrict__ z, BnFold f,
                                                              const bf16* __restrict__ res, int64_t M, int C,
                                                              bf16* __restrict__ y) {
  __shared__ float red[4][2][64];
  __shared__ __attribute__((aligned(16))) float sss[2][2048];
  const bool w0 = blockIdx.x == 0;
  if (f.nbt && w0 && threadIdx.x == 0) f.nbt[0] += 1;
  for (int c0 = 0; c0 < C; c0 += 64)
    bn_stats64(f.sums, f.G, M, C, c0, f.gamma, f.beta, f.eps, f.momentum, f.running_mean, f.running_var, sss[0],
               sss[1], f.save, w0, red);
  const int cv = C >> 3, rpb = 256 / cv;
  const int col = threadIdx.x % cv, rsub = threadIdx.x / cv;
  float sc[8], sh[8];
  load8(sss[0] + col * 8, sc);
  load8(sss[1] + col * 8, sh);
  const int64_t rstride = (int64_t)gridDim.x * rpb;
  for (int64_t r = (int64_t)blockIdx.x * rpb + rsub; r < M; r += kBnUnroll * rstride) {
    bf16x8 zv[kBnUnroll], rv[kBnUnroll];
#pragma unroll
    for (int u = 0; u < kBnUnroll; ++u) {
      const int64_t rr = r + u * rstride;
      if (rr < M) {
        zv[u] = reinterpret_cast<const bf16x8*>(z)[rr * cv + col];
        if (kRes) rv[u] = reinterpret_cast<const bf16x8*>(res)[rr * cv + col];
      }
    }
#pragma unroll
    for (int u = 0; u < kBnUnroll; ++u) {
      const int64_t rr = r + u * rstride;
      if (rr < M) {
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float v = fmaf((float)zv[u][j], sc[j], sh[j]);
          if (kRes) v += (float)rv[u][j];
          if (kRelu) v = fmaxf(v, 0.f);
          o[j] = (bf16)v;
        }
        reinterpret_cast<bf16x8*>(y)[rr * cv + col] = o;
      }
    }
  }
}

// dz = A*g + Bz*z + Cc per channel (A = gamma*invstd, Bz = -A*invstd*dgamma/M,
// Cc = -A*dbeta/M - Bz*mean): the coefficients are formed once per thread in registers.
// part != null (few partial rows, see kBnFewParts): every workgroup sums the [nparts][2][C] partials of
// its channels itself in a fixed order and workgroup 0 stores dgamma / dbeta - two launches fewer than
// the two-level reduction; otherwise dgamma / dbeta are inputs.
// kZMask: g is the unmasked dy and the ReLU mask is re-derived from z and ss (see bn_bwd_reduce_kernel)
template <bool kZMask>
__global__ __launch_bounds__(256) void bn_bwd_apply_col_kernel(const bf16* __restrict__ g, const bf16* __restrict__ z,
                                                               const float* __restrict__ save,
                                                               const float* __restrict__ ss,
                                                               const float* __restrict__ gamma,
                                                               float* __restrict__ dgamma,
                                                               float* __restrict__ dbeta, const float* __restrict__ part,
                                                               int nparts, int64_t M, int C, bf16* __restrict__ dz) {
  const int cv = C >> 3, rpb = 256 / cv;
  const int col = threadIdx.x % cv, rsub = threadIdx.x / cv;
  const float invM = 1.f / (float)M;
  float mean[8], inv[8], ga[8], dg[8], db[8], A[8], Bz[8], Cc[8], sc[8], sh[8];
  load8(save + col * 8, mean);
  load8(save + C + col * 8, inv);
  load8(gamma + col * 8, ga);
  if constexpr (kZMask) {
    load8(ss + col * 8, sc);
    load8(ss + C + col * 8, sh);
  }
  if (part) {
#pragma unroll
    for (int j = 0; j < 8; ++j) dg[j] = db[j] = 0.f;
    // two partial rows per step with separate accumulators (independent loads in flight; the one-row
    // serial chain took 12 us at 32 partials), combined in a fixed order
    float db2[8], dg2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) dg2[j] = db2[j] = 0.f;
    int p = 0;
#pragma unroll 2
    for (; p + 1 < nparts; p += 2) {
      float a[8], q[8], a2[8], q2[8];
      load8(part + (int64_t)p * 2 * C + col * 8, a);            // sum of g
      load8(part + (int64_t)p * 2 * C + C + col * 8, q);        // sum of g * zhat
      load8(part + (int64_t)(p + 1) * 2 * C + col * 8, a2);
      load8(part + (int64_t)(p + 1) * 2 * C + C + col * 8, q2);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        db[j] += a[j];
        dg[j] += q[j];
        db2[j] += a2[j];
        dg2[j] += q2[j];
      }
    }
    if (p < nparts) {
      float a[8], q[8];
      load8(part + (int64_t)p * 2 * C + col * 8, a);
      load8(part + (int64_t)p * 2 * C + C + col * 8, q);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        db[j] += a[j];
        dg[j] += q[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      db[j] += db2[j];
      dg[j] += dg2[j];
    }
    if (blockIdx.x == 0 && rsub == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        dbeta[col * 8 + j] = db[j];
        dgamma[col * 8 + j] = dg[j];
      }
    }
  } else {
    load8(dgamma + col * 8, dg);
    load8(dbeta + col * 8, db);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    A[j] = ga[j] * inv[j];
    Bz[j] = -A[j] * inv[j] * dg[j] * invM;
    Cc[j] = -A[j] * db[j] * invM - Bz[j] * mean[j];
  }
  const int64_t rstride = (int64_t)gridDim.x * rpb;
  for (int64_t r = (int64_t)blockIdx.x * rpb + rsub; r < M; r += kBnUnroll * rstride) {
    bf16x8 gv[kBnUnroll], zv[kBnUnroll];
#pragma unroll
    for (int u = 0; u < kBnUnroll; ++u) {
      const int64_t rr = r + u * rstride;
      if (rr < M) {
        gv[u] = reinterpret_cast<const bf16x8*>(g)[rr * cv + col];
        zv[u] = reinterpret_cast<const bf16x8*>(z)[rr * cv + col];
      }
    }
#pragma unroll
    for (int u = 0; u < kBnUnroll; ++u) {
      const int64_t rr = r + u * rstride;
      if (rr < M) {
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float gj = (float)gv[u][j];
          if constexpr (kZMask) {
            const bf16 yv = (bf16)fmaxf(fmaf((float)zv[u][j], sc[j], sh[j]), 0.f);
            if (!((float)yv > 0.f)) gj = 0.f;
          }
          o[j] = (bf16)fmaf(A[j], gj, fmaf(Bz[j], (float)zv[u][j], Cc[j]));
        }
        reinterpret_cast<bf16x8*>(dz)[rr * cv + col] = o;
      }
    }
  }
}

// Rows are split over workgroups; each thread owns one 8-channel vector column (C/8 columns, C <= 2048)
// and walks rows with a stride, accumulating in fp32; partials [part][2][C] (deterministic).
// Small tensors (ResNet-18 at CIFAR shape, layers 2-4: M*C <= 512K elements): at most kBnFewParts partial rows, which
// the apply kernel sums itself (no separate two-level reduction launches).  Larger ones keep up to 1024
// row slices so the reduction spreads over the whole chip (16 slices of a 50k x 1024 tensor took 7 ms per
// ResNet-50 step more).
constexpr int kBnFewParts = 32;
// RINGDP_BN_MAX_PARTS / RINGDP_BN_MIN_ROWS: partial-row count and rows per part of the large tensors (sweeps)
inline int64_t bn_rows_per_part(int64_t M, int C) {
  static const int64_t max_parts = [] { const char* v = getenv("RINGDP_BN_MAX_PARTS"); return v && *v ? std::max(1, atoi(v)) : 1024; }();
  static const int64_t min_rows = [] { const char* v = getenv("RINGDP_BN_MIN_ROWS"); return v && *v ? std::max(1, atoi(v)) : 64; }();
  if (M * C <= (int64_t)1 << 19) return std::max<int64_t>(32, (M + kBnFewParts - 1) / kBnFewParts);
  return std::max<int64_t>(min_rows, (M + max_parts - 1) / max_parts);
}

// kZMask: the ReLU mask re-derived from z and the forward's scale / shift (ss: the same fmaf and bf16 rounding
// as bn_act_fwd_col_kernel, so bit-identical to reading y) - a BN + ReLU without a residual add reads dy and z only.
// g_out == nullptr: the masked gradient is not stored (nobody but the apply pass needs it, and that pass re-masks).
template <bool kZMask>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ y,
                                                            const bf16* __restrict__ z, const float* __restrict__ save,
                                                            const float* __restrict__ ss,
                                                            int relu, int64_t M, int C, int64_t rows_per_part,
                                                            float* __restrict__ part, bf16* __restrict__ g_out) {
  const int cv = C / 8;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_part;
  const int64_t r1 = std::min<int64_t>(M, r0 + rows_per_part);
  const int lanes_per_row = cv;
  const int rows_in_flight = max(1, 256 / lanes_per_row);
  const int col = threadIdx.x % lanes_per_row, rsub = threadIdx.x / lanes_per_row;
  __shared__ __attribute__((aligned(16))) float red[2][256][8];  // [statistic][thread][channel of its 8]
  float sg[8], sgz[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sg[j] = sgz[j] = 0.f;
  if (rsub < rows_in_flight && col < lanes_per_row) {
    float mean[8], inv[8], sc[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mean[j] = save[col * 8 + j];
      inv[j] = save[C + col * 8 + j];
      sc[j] = kZMask ? ss[col * 8 + j] : 0.f;
      sh[j] = kZMask ? ss[C + col * 8 + j] : 0.f;
    }
    // kBnUnroll rows per step: 12 16-B loads in flight per thread (rows accumulate in a fixed order)
    for (int64_t r = r0 + rsub; r < r1; r += kBnUnroll * rows_in_flight) {
      bf16x8 d[kBnUnroll], zz[kBnUnroll], yy[kBnUnroll];
#pragma unroll
      for (int u = 0; u < kBnUnroll; ++u) {
        const int64_t rr = r + u * rows_in_flight;
        if (rr < r1) {
          const int64_t v = rr * cv + col;
          d[u] = reinterpret_cast<const bf16x8*>(dy)[v];
          zz[u] = reinterpret_cast<const bf16x8*>(z)[v];
          yy[u] = (relu && !kZMask) ? reinterpret_cast<const bf16x8*>(y)[v] : zero_bf16x8();
        }
      }
#pragma unroll
      for (int u = 0; u < kBnUnroll; ++u) {
        const int64_t rr = r + u * rows_in_flight;
        if (rr < r1) {
          bf16x8 go;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            bool off;
            if constexpr (kZMask) {
              const bf16 yv = (bf16)fmaxf(fmaf((float)zz[u][j], sc[j], sh[j]), 0.f);
              off = !((float)yv > 0.f);
            } else {
              off = relu && !((float)yy[u][j] > 0.f);
            }
            const float g = off ? 0.f : (float)d[u][j];
            go[j] = (bf16)g;
            const float gq = (float)go[j];
            sg[j] += gq;
            sgz[j] += gq * ((float)zz[u][j] - mean[j]) * inv[j];
          }
          if (g_out) reinterpret_cast<bf16x8*>(g_out)[rr * cv + col] = go;
        }
      }
    }
  }
  // combine the rows_in_flight partial rows for each column (fixed order): every thread parks its 16 sums
  // in LDS once, then each output (statistic, channel) is summed by its own thread - one barrier instead of
  // 16, and no thread walks 8 channels x rows_in_flight serial LDS reads (the old tail was most of the
  // kernel's time on small ResNet-18 layers)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][threadIdx.x][j] = sg[j];
    red[1][threadIdx.x][j] = sgz[j];
  }
  __syncthreads();
  for (int o = threadIdx.x; o < 2 * C; o += 256) {
    const int st = o / C, c = o - st * C, cl = c >> 3, j = c & 7;
    float a = 0.f;
    for (int k = 0; k < rows_in_flight; ++k) a += red[st][k * lanes_per_row + cl][j];
    part[((int64_t)blockIdx.x * 2 + st) * C + c] = a;
  }
}

__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const bf16* __restrict__ g, const bf16* __restrict__ z,
                                                           const float* __restrict__ save,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ dgamma,
                                                           const float* __restrict__ dbeta, int64_t M, int C,
                                                           int64_t nvec, bf16* __restrict__ dz) {
  const float invM = 1.f / (float)M;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    const int c0 = (int)((v * 8) % C);
    const bf16x8 gv = reinterpret_cast<const bf16x8*>(g)[v];
    const bf16x8 zv = reinterpret_cast<const bf16x8*>(z)[v];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      const float inv = save[C + c];
      const float zh = ((float)zv[j] - save[c]) * inv;
      const float d = gamma[c] * inv * ((float)gv[j] - dbeta[c] * invM - zh * dgamma[c] * invM);
      o[j] = (bf16)d;
    }
    reinterpret_cast<bf16x8*>(dz)[v] = o;
  }
}

// max pooling (ResNet stem 3x3 s2 p1), NHWC, 8 channels per thread; arg = window offset (dy*k + dx)
// of the first max, one byte per channel
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const bf16* __restrict__ x, int N, int H, int W, int C,
                                                          int k, int stride, int pad, int P, int Q,
                                                          bf16* __restrict__ y, uint8_t* __restrict__ arg) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * P * Q * cv;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int c8 = (int)(e % cv);
    int64_t t = e / cv;
    const int q = (int)(t % Q);
    t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    float best[8];
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) best[j] = -INFINITY;
    for (int dy = 0; dy < k; ++dy) {
      const int h = p * stride - pad + dy;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int dx = 0; dx < k; ++dx) {
        const int w = q * stride - pad + dx;
        if ((unsigned)w >= (unsigned)W) continue;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + (((int64_t)n * H + h) * W + w) * C + c8 * 8);
        const uint32_t a = (uint32_t)(dy * k + dx);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = (float)v[j];
          if (f > best[j]) {
            best[j] = f;
            if (j < 4)
              lo = (lo & ~(0xffu << (8 * j))) | (a << (8 * j));
            else
              hi = (hi & ~(0xffu << (8 * (j - 4)))) | (a << (8 * (j - 4)));
          }
        }
      }
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)best[j];
    reinterpret_cast<bf16x8*>(y)[e] = o;
    reinterpret_cast<uint2*>(arg)[e] = make_uint2(lo, hi);
  }
}

__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const bf16* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                          int N, int H, int W, int C, int k, int stride, int pad,
                                                          int P, int Q, bf16* __restrict__ dx) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * H * W * cv;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int c8 = (int)(e % cv);
    int64_t t = e / cv;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    float g[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = 0.f;
    // windows p with p*stride - pad <= h <= p*stride - pad + k - 1 (gather: deterministic)
    const int p_lo = max(0, (h + pad - k + stride) / stride), p_hi = min(P - 1, (h + pad) / stride);
    const int q_lo = max(0, (w + pad - k + stride) / stride), q_hi = min(Q - 1, (w + pad) / stride);
    for (int p = p_lo; p <= p_hi; ++p)
      for (int q = q_lo; q <= q_hi; ++q) {
        const int dyy = h - (p * stride - pad), dxx = w - (q * stride - pad);
        if (dyy < 0 || dyy >= k || dxx < 0 || dxx >= k) continue;
        const int want = dyy * k + dxx;
        const int64_t o = (((int64_t)n * P + p) * Q + q) * cv + c8;
        const uint2 am = reinterpret_cast<const uint2*>(arg)[o];
        const bf16x8 d = reinterpret_cast<const bf16x8*>(dy)[o];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int aj = (int)(((j < 4 ? am.x : am.y) >> (8 * (j & 3))) & 0xff);
          if (aj == want) g[j] += (float)d[j];
        }
      }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)g[j];
    reinterpret_cast<bf16x8*>(dx)[e] = o;
  }
}

// global average pool NHWC [N][HW][C] -> [N][C] (fp32 accumulation); one thread per (n, c)
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(const bf16* __restrict__ x, int N, int HW, int C,
                                                          bf16* __restrict__ y) {
  const int64_t total = (int64_t)N * C;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t n = e / C;
    const int c = (int)(e % C);
    float a = 0.f;
    for (int i = 0; i < HW; ++i) a += (float)x[(n * HW + i) * C + c];
    y[e] = (bf16)(a / (float)HW);
  }
}

__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const bf16* __restrict__ dy, int N, int HW, int C,
                                                          bf16* __restrict__ dx) {
  const int64_t total = (int64_t)N * HW * C;
  const float s = 1.f / (float)HW;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int c = (int)(e % C);
    const int64_t n = e / ((int64_t)HW * C);
    dx[e] = (bf16)((float)dy[n * C + c] * s);
  }
}

// ---------------------------------------------------------------- classifier head (avgpool + fc, J <= 16)
// ResNet's head at few classes (CIFAR: 10) as one launch each way instead of the ~19 launches of
// avgpool -> bf16 weight copy / row padding -> MFMA GEMM -> slice, and their backward (ref/example_mp.py:50:
// torchvision resnet18(num_classes=10)).  The work is tiny (N x C x J MACs); what costs is launches.
// Thread layout: 8 channels per thread, C/8 threads per image, 256/(C/8) images per pass.
constexpr int kHeadMaxJ = 16;
// JT: the class count at compile time (10: CIFAR), 0: run-time J <= kHeadMaxJ (per-class guards become branches)
template <int JT>
__global__ __launch_bounds__(256) void head_fwd_kernel(const bf16* __restrict__ x, int N, int HW, int C, int Jr,
                                                       const float* __restrict__ w, const float* __restrict__ b,
                                                       float* __restrict__ pooled, float* __restrict__ logits) {
  __shared__ float part[256][kHeadMaxJ + 1];
  constexpr int JM = JT > 0 ? JT : kHeadMaxJ;
  const int J = JT > 0 ? JT : Jr;
  const int cv = C >> 3, ipp = 256 / cv;
  const int col = threadIdx.x % cv, sub = threadIdx.x / cv;
  const int n = blockIdx.x * ipp + sub;
  const bool live = sub < ipp && n < N;
  float acc[JM];
#pragma unroll
  for (int j = 0; j < JM; ++j) acc[j] = 0.f;
  if (live) {
    float s[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] = 0.f;
    const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + (int64_t)n * HW * C) + col;
    for (int i = 0; i < HW; ++i) {  // fixed order over the window
      const bf16x8 v = xr[(int64_t)i * cv];
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += (float)v[k];
    }
    const float inv = 1.f / (float)HW;
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] *= inv;
    float4* pr = reinterpret_cast<float4*>(pooled + (int64_t)n * C + col * 8);
    pr[0] = make_float4(s[0], s[1], s[2], s[3]);
    pr[1] = make_float4(s[4], s[5], s[6], s[7]);
#pragma unroll
    for (int j = 0; j < JM; ++j) {
      if (JT > 0 || j < J) {
        float wv[8];
        load8(w + (int64_t)j * C + col * 8, wv);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[j] = fmaf(s[k], wv[k], acc[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < JM; ++j) part[threadIdx.x][j] = acc[j];
  __syncthreads();
  // one thread per (image, class): the image's cv partials in column order (fixed)
  for (int o = threadIdx.x; o < ipp * J; o += 256) {
    const int si = o / J, j = o - si * J, nn = blockIdx.x * ipp + si;
    if (nn >= N) continue;
    float a = 0.f;
    for (int c = 0; c < cv; ++c) a += part[si * cv + c][j];
    logits[(int64_t)nn * J + j] = a + b[j];
  }
}

// logits gradient of row r, class j: from a materialised dl (kCE false), or formed from the cross-entropy forward
// (ce, the expression of ce_bwd_kernel).  Branch-free: every load is unconditional (the reduction picks an index,
// not a path), so a call's loads issue together - conditional loads had made each call several dependent L2
// round trips.  sc: 1 (reduction none) or 1 / denom.
template <bool kCE>
__device__ __forceinline__ float head_dl(const float* __restrict__ dl, const CeFuse& ce, float sc, int J, int r, int j) {
  if (!kCE) return dl[(int64_t)r * J + j];
  const int64_t y = ce.labels[r];
  const float x = ce.logits[(int64_t)r * J + j], l = ce.lse[r];
  const float go = ce.grad_out[ce.reduction == 0 ? r : 0] * sc;
  const float p = __expf(x - l);
  const float q = (j == y ? (1.f - ce.eps) : 0.f) + ce.eps / (float)J;
  return y == ce.ignore_index ? 0.f : (p - q) * go;
}

// Backward: workgroups [0, nb_dx) form dx (d(pooled) = dl W / HW, broadcast over the window), the
// C/16 workgroups after them dW (16 channels each, the batch summed by 16 row groups combined in a fixed
// order) and, in the first of those, db.  No partial sums cross workgroups: one launch, deterministic.
constexpr int kHeadRows = 256;  // logits-gradient rows staged in LDS per chunk (dW role)
template <bool kCE, int JT>
__global__ __launch_bounds__(256) void head_bwd_kernel(const float* __restrict__ dl, CeFuse ce,
                                                       const float* __restrict__ pooled, const float* __restrict__ w,
                                                       int N, int HW, int C, int Jr, int nb_dx, bf16* __restrict__ dx,
                                                       float* __restrict__ dw, float* __restrict__ db) {
  constexpr int JM = JT > 0 ? JT : kHeadMaxJ;
  const int J = JT > 0 ? JT : Jr;
  __shared__ float g[kHeadRows][kHeadMaxJ];
  const float sc = kCE ? (ce.reduction == 0 ? 1.f : 1.f / ce.denom[0]) : 1.f;
  if ((int)blockIdx.x < nb_dx) {
    const int cv = C >> 3, ipp = 256 / cv;
    const int col = threadIdx.x % cv, sub = threadIdx.x / cv;
    const int n0 = blockIdx.x * ipp, n = n0 + sub;
    // this workgroup's ipp x J logits gradients first (independent loads in flight), then W from L2
    for (int o = threadIdx.x; o < ipp * J; o += 256) {
      const int si = o / J, j = o - si * J;
      if (n0 + si < N) g[si][j] = head_dl<kCE>(dl, ce, sc, J, n0 + si, j);
    }
    __syncthreads();
    if (sub >= ipp || n >= N) return;
    float d[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = 0.f;
#pragma unroll
    for (int j = 0; j < JM; ++j) {
      if (JT > 0 || j < J) {
        const float gj = g[sub][j];
        float wv[8];
        load8(w + (int64_t)j * C + col * 8, wv);
#pragma unroll
        for (int k = 0; k < 8; ++k) d[k] = fmaf(gj, wv[k], d[k]);
      }
    }
    const float inv = 1.f / (float)HW;
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = (bf16)(d[k] * inv);
    bf16x8* xr = reinterpret_cast<bf16x8*>(dx + (int64_t)n * HW * C) + col;
    for (int i = 0; i < HW; ++i) xr[(int64_t)i * cv] = o;
    return;
  }
  // dW role: 16 channels per workgroup; thread (cl = t & 15, rq = t >> 4) sums rows r = rq, rq + 16, .. of
  // its channel for every class (independent row loads in flight), then the 16 row-group partials of each
  // (class, channel) are combined in a fixed order through LDS
  float (*red)[16][kHeadMaxJ] = reinterpret_cast<float (*)[16][kHeadMaxJ]>(&g[0][0]);  // [16 rq][16 cl][J]
  const int c0 = ((int)blockIdx.x - nb_dx) * 16, cl = threadIdx.x & 15, rq = threadIdx.x >> 4;
  const int c = c0 + cl;
  float a[JM], bsum = 0.f;
#pragma unroll
  for (int j = 0; j < JM; ++j) a[j] = 0.f;
  for (int r0 = 0; r0 < N; r0 += kHeadRows) {
    const int rows = min(kHeadRows, N - r0);
    __syncthreads();  // the previous chunk's readers are done
    // four elements per thread at a time, all their loads before any LDS store (the stores would otherwise
    // order each element's L2 round trips after the previous one's: ~2 us per element)
    for (int e0 = threadIdx.x; e0 < rows * J; e0 += 4 * 256) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + 256 * u, r = e / J, j = e - r * J;
        v[u] = e < rows * J ? head_dl<kCE>(dl, ce, sc, J, r0 + r, j) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + 256 * u, r = e / J, j = e - r * J;
        if (e < rows * J) g[r][j] = v[u];
      }
    }
    __syncthreads();
    if (c < C) {
#pragma unroll 4
      for (int r = rq; r < rows; r += 16) {
        const float p = pooled[(int64_t)(r0 + r) * C + c];
#pragma unroll
        for (int j = 0; j < JM; ++j)
          if (JT > 0 || j < J) a[j] = fmaf(g[r][j], p, a[j]);
      }
    }
    if (blockIdx.x == nb_dx && threadIdx.x < J)
      for (int r = 0; r < rows; ++r) bsum += g[r][threadIdx.x];
  }
  __syncthreads();  // g is reused as red
#pragma unroll
  for (int j = 0; j < JM; ++j)
    if (JT > 0 || j < J) red[rq][cl][j] = a[j];
  __syncthreads();
  for (int o = threadIdx.x; o < 16 * J; o += 256) {
    const int j = o >> 4, cc = o & 15;
    if (c0 + cc >= C) continue;
    float v = 0.f;
    for (int q = 0; q < 16; ++q) v += red[q][cc][j];
    dw[(int64_t)j * C + c0 + cc] = v;
  }
  if (blockIdx.x == nb_dx && threadIdx.x < J) db[threadIdx.x] = bsum;
}

__global__ __launch_bounds__(256) void add_bf16_kernel(const bf16* __restrict__ a, const bf16* __restrict__ b,
                                                       int64_t nvec, bf16* __restrict__ y) {
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    const bf16x8 x = reinterpret_cast<const bf16x8*>(a)[v], z = reinterpret_cast<const bf16x8*>(b)[v];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)((float)x[j] + (float)z[j]);
    reinterpret_cast<bf16x8*>(y)[v] = o;
  }
}


// Per-channel sum / sum of squares of a stored bf16 conv output z [M][C] (the BN statistics of a conv
// whose GEMM ran on hipBLASLt, which has no statistics epilogue): partials [part][2][C] in the layout of
// the GEMM epilogue's per-tile statistics, rows split over workgroups as in bn_bwd_reduce.
__global__ __launch_bounds__(256) void bn_col_stats_kernel(const bf16* __restrict__ z, int64_t M, int C,
                                                           int64_t rows_per_part, float* __restrict__ part) {
  const int cv = C / 8;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_part;
  const int64_t r1 = std::min<int64_t>(M, r0 + rows_per_part);
  const int rows_in_flight = max(1, 256 / cv);
  const int col = threadIdx.x % cv, rsub = threadIdx.x / cv;
  __shared__ float red[2][256];
  float sa[8], sq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sa[j] = sq[j] = 0.f;
  if (rsub < rows_in_flight && col < cv) {
    for (int64_t r = r0 + rsub; r < r1; r += kBnUnroll * rows_in_flight) {
      bf16x8 zz[kBnUnroll];
#pragma unroll
      for (int u = 0; u < kBnUnroll; ++u) {
        const int64_t rr = r + u * rows_in_flight;
        zz[u] = rr < r1 ? reinterpret_cast<const bf16x8*>(z)[rr * cv + col] : zero_bf16x8();
      }
#pragma unroll
      for (int u = 0; u < kBnUnroll; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = (float)zz[u][j];
          sa[j] += v;
          sq[j] += v * v;
        }
    }
  }
  __syncthreads();
  for (int j = 0; j < 8; ++j) {
    red[0][threadIdx.x] = sa[j];
    red[1][threadIdx.x] = sq[j];
    __syncthreads();
    if (threadIdx.x < cv) {
      float a = 0.f, q = 0.f;
      for (int k = 0; k < rows_in_flight; ++k) {
        a += red[0][k * cv + threadIdx.x];
        q += red[1][k * cv + threadIdx.x];
      }
      part[((int64_t)blockIdx.x * 2) * C + threadIdx.x * 8 + j] = a;
      part[((int64_t)blockIdx.x * 2 + 1) * C + threadIdx.x * 8 + j] = q;
    }
    __syncthreads();
  }
}

}  // namespace

void pack_conv_weight(const float* w, int K, int C, int R, int S, int Cp, int ldk, void* krsc, void* crsk,
                      hipStream_t s) {
  const int64_t total = (int64_t)K * ldk;
  pack_conv_weight_kernel<<<grid_for(total), 256, 0, s>>>(w, K, C, R, S, Cp, ldk, static_cast<bf16*>(krsc),
                                                          static_cast<bf16*>(crsk));
}

void pack_conv_weights(const PackTable& t, hipStream_t s) {
  if (t.total <= 0) return;
  // RINGDP_PACK_SPLIT=1: the two-launch form (A/B)
  static const bool split = [] { const char* v = std::getenv("RINGDP_PACK_SPLIT"); return v && std::atoi(v) != 0; }();
  bool fits = true;  // every entry's tile must fit the LDS stage
  for (int i = 0; i < t.n; ++i) fits = fits && 32 * pack_ct(t.e[i].Cp) * t.e[i].R * t.e[i].S <= kPackTileFloats;
  if (!split && fits) {
    pack_both_multi_kernel<<<t.total_tiles2, 256, 0, s>>>(t);
    return;
  }
  pack_krsc_multi_kernel<<<grid_for(t.total), 256, 0, s>>>(t);
  pack_crsk_multi_kernel<<<(int)t.total_tiles, 256, 0, s>>>(t);
}

void nchw_to_nhwc_pad(const void* x, bool x_bf16, int N, int C, int H, int W, int Cp, void* y, hipStream_t s) {
  const int64_t total = (int64_t)N * H * W * Cp;
  if (x_bf16)
    nchw_to_nhwc_kernel<true><<<grid_for(total), 256, 0, s>>>(x, N, C, H, W, Cp, static_cast<bf16*>(y));
  else
    nchw_to_nhwc_kernel<false><<<grid_for(total), 256, 0, s>>>(x, N, C, H, W, Cp, static_cast<bf16*>(y));
}

void bn_prepare(const float* sums, int G, int64_t M, int C, const float* gamma, const float* beta, float eps,
                float momentum, float* running_mean, float* running_var, float* scale_shift, float* save,
                int64_t* num_batches_tracked, hipStream_t s) {
  bn_prepare_kernel<<<(C + 63) / 64, 256, 0, s>>>(sums, G, M, C, gamma, beta, eps, momentum, running_mean,
                                                    running_var, scale_shift, save, num_batches_tracked);
}

bool bn_fold_ok(int G, int C) {
  return C % 8 == 0 && C <= 2048 && 256 % (C / 8) == 0 && (int64_t)G * C <= kBnFoldMax;
}

void bn_fold_act_fwd(const float* sums, int G, int64_t M, int C, const float* gamma, const float* beta, float eps,
                     float momentum, float* running_mean, float* running_var, float* save,
                     int64_t* num_batches_tracked, const void* z, const void* res, bool relu, void* y, hipStream_t s) {
  const BnFold f{sums, G, gamma, beta, eps, momentum, running_mean, running_var, save, num_batches_tracked};
  const int rpb = 256 / (C / 8);
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((M + rpb * kBnUnroll - 1) / (rpb * kBnUnroll), 2048));
  const bf16* zb = static_cast<const bf16*>(z);
  const bf16* rb = static_cast<const bf16*>(res);
  bf16* yb = static_cast<bf16*>(y);
  if (res && relu) bn_fold_act_fwd_kernel<true, true><<<grid, 256, 0, s>>>(zb, f, rb, M, C, yb);
  else if (res) bn_fold_act_fwd_kernel<true, false><<<grid, 256, 0, s>>>(zb, f, rb, M, C, yb);
  else if (relu) bn_fold_act_fwd_kernel<false, true><<<grid, 256, 0, s>>>(zb, f, rb, M, C, yb);
  else bn_fold_act_fwd_kernel<false, false><<<grid, 256, 0, s>>>(zb, f, rb, M, C, yb);
}

void bn_act_fwd(const void* z, const float* ss, const void* res, bool relu, int64_t M, int C, void* y,
                hipStream_t s) {
  const int64_t nvec = M * C / 8;
  if (C % 8 == 0 && C <= 2048 && 256 % (C / 8) == 0) {
    const int rpb = 256 / (C / 8);
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((M + rpb * kBnUnroll - 1) / (rpb * kBnUnroll), 2048));
    const bf16* zb = static_cast<const bf16*>(z);
    const bf16* rb = static_cast<const bf16*>(res);
    bf16* yb = static_cast<bf16*>(y);
    if (res && relu) bn_act_fwd_col_kernel<true, true><<<grid, 256, 0, s>>>(zb, ss, rb, M, C, yb);
    else if (res) bn_act_fwd_col_kernel<true, false><<<grid, 256, 0, s>>>(zb, ss, rb, M, C, yb);
    else if (relu) bn_act_fwd_col_kernel<false, true><<<grid, 256, 0, s>>>(zb, ss, rb, M, C, yb);
    else bn_act_fwd_col_kernel<false, false><<<grid, 256, 0, s>>>(zb, ss, rb, M, C, yb);
    return;
  }
  bn_act_fwd_kernel<<<grid_for(nvec), 256, 0, s>>>(static_cast<const bf16*>(z), ss, static_cast<const bf16*>(res),
                                                   relu ? 1 : 0, nvec, C, static_cast<bf16*>(y));
}

int bn_bwd_parts(int64_t M, int C) {
  const int64_t rpp = bn_rows_per_part(M, C);
  return (int)((M + rpp - 1) / rpp);
}

int bn_col_stats(const void* z, int64_t M, int C, float* part, hipStream_t s) {
  const int nparts = bn_bwd_parts(M, C);
  bn_col_stats_kernel<<<nparts, 256, 0, s>>>(static_cast<const bf16*>(z), M, C, bn_rows_per_part(M, C), part);
  return nparts;
}

void bn_bwd_reduce(const void* dy, const void* y, const void* z, const float* save, const float* ss, bool relu,
                   int64_t M, int C, float* part, void* g_out, hipStream_t s) {
  if (ss)
    bn_bwd_reduce_kernel<true><<<bn_bwd_parts(M, C), 256, 0, s>>>(
        static_cast<const bf16*>(dy), nullptr, static_cast<const bf16*>(z), save, ss, 1, M, C, bn_rows_per_part(M, C),
        part, static_cast<bf16*>(g_out));
  else
    bn_bwd_reduce_kernel<false><<<bn_bwd_parts(M, C), 256, 0, s>>>(
        static_cast<const bf16*>(dy), static_cast<const bf16*>(y), static_cast<const bf16*>(z), save, nullptr,
        relu ? 1 : 0, M, C, bn_rows_per_part(M, C), part, static_cast<bf16*>(g_out));
}

bool bn_bwd_zmask_ok(int C) { return C % 8 == 0 && C <= 2048 && 256 % (C / 8) == 0; }

void bn_bwd_apply(const float* part, int nparts, float* scratch, const void* g, const void* z, const float* save,
                  const float* ss, const float* gamma, int64_t M, int C, float* dgamma, float* dbeta, void* dz,
                  hipStream_t s) {
  const int64_t nvec = M * C / 8;
  if (bn_bwd_zmask_ok(C)) {
    const bool few = nparts <= kBnFewParts;  // the apply kernel sums the partials itself
    if (!few) reduce_parts(part, nparts, C, scratch, dbeta, dgamma, s);  // part[p][0] = sum g, [1] = sum g*zhat
    const int rpb = 256 / (C / 8);
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((M + rpb * kBnUnroll - 1) / (rpb * kBnUnroll), 2048));
    if (ss)
      bn_bwd_apply_col_kernel<true><<<grid, 256, 0, s>>>(static_cast<const bf16*>(g), static_cast<const bf16*>(z), save,
                                                         ss, gamma, dgamma, dbeta, few ? part : nullptr, nparts, M, C,
                                                         static_cast<bf16*>(dz));
    else
      bn_bwd_apply_col_kernel<false><<<grid, 256, 0, s>>>(static_cast<const bf16*>(g), static_cast<const bf16*>(z),
                                                          save, nullptr, gamma, dgamma, dbeta, few ? part : nullptr,
                                                          nparts, M, C, static_cast<bf16*>(dz));
    return;
  }
  // (ss is only passed when bn_bwd_zmask_ok(C): this fallback never sees the z-mask form)
  reduce_parts(part, nparts, C, scratch, dbeta, dgamma, s);
  bn_bwd_apply_kernel<<<grid_for(nvec), 256, 0, s>>>(static_cast<const bf16*>(g), static_cast<const bf16*>(z), save,
                                                     gamma, dgamma, dbeta, M, C, nvec, static_cast<bf16*>(dz));
}

void maxpool_fwd(const void* x, int N, int H, int W, int C, int k, int stride, int pad, int P, int Q, void* y,
                 uint8_t* arg, hipStream_t s) {
  const int64_t total = (int64_t)N * P * Q * C / 8;
  maxpool_fwd_kernel<<<grid_for(total), 256, 0, s>>>(static_cast<const bf16*>(x), N, H, W, C, k, stride, pad, P, Q,
                                                     static_cast<bf16*>(y), arg);
}

void maxpool_bwd(const void* dy, const uint8_t* arg, int N, int H, int W, int C, int k, int stride, int pad, int P,
                 int Q, void* dx, hipStream_t s) {
  const int64_t total = (int64_t)N * H * W * C / 8;
  maxpool_bwd_kernel<<<grid_for(total), 256, 0, s>>>(static_cast<const bf16*>(dy), arg, N, H, W, C, k, stride, pad,
                                                     P, Q, static_cast<bf16*>(dx));
}

void avgpool_fwd(const void* x, int N, int HW, int C, void* y, hipStream_t s) {
  avgpool_fwd_kernel<<<grid_for((int64_t)N * C), 256, 0, s>>>(static_cast<const bf16*>(x), N, HW, C,
                                                              static_cast<bf16*>(y));
}

void avgpool_bwd(const void* dy, int N, int HW, int C, void* dx, hipStream_t s) {
  avgpool_bwd_kernel<<<grid_for((int64_t)N * HW * C), 256, 0, s>>>(static_cast<const bf16*>(dy), N, HW, C,
                                                                   static_cast<bf16*>(dx));
}

bool head_ok(int C, int J) { return J >= 1 && J <= kHeadMaxJ && C % 8 == 0 && C >= 8 && C <= 2048 && 256 % (C / 8) == 0; }

void head_fwd(const void* x, int N, int HW, int C, int J, const float* w, const float* b, float* pooled,
              float* logits, hipStream_t s) {
  const int ipp = 256 / (C / 8);
  const bf16* xb = static_cast<const bf16*>(x);
  if (J == 10)
    head_fwd_kernel<10><<<(N + ipp - 1) / ipp, 256, 0, s>>>(xb, N, HW, C, J, w, b, pooled, logits);
  else
    head_fwd_kernel<0><<<(N + ipp - 1) / ipp, 256, 0, s>>>(xb, N, HW, C, J, w, b, pooled, logits);
}

void head_bwd(const float* dl, const CeFuse* ce, const float* pooled, const float* w, int N, int HW, int C, int J,
              void* dx, float* dw, float* db, hipStream_t s) {
  const int ipp = 256 / (C / 8), nb_dx = (N + ipp - 1) / ipp;
  const CeFuse c = ce ? *ce : CeFuse{};
  const int grid = nb_dx + (C + 15) / 16;
  bf16* dxb = static_cast<bf16*>(dx);
  if (ce && J == 10)
    head_bwd_kernel<true, 10><<<grid, 256, 0, s>>>(nullptr, c, pooled, w, N, HW, C, J, nb_dx, dxb, dw, db);
  else if (ce)
    head_bwd_kernel<true, 0><<<grid, 256, 0, s>>>(nullptr, c, pooled, w, N, HW, C, J, nb_dx, dxb, dw, db);
  else if (J == 10)
    head_bwd_kernel<false, 10><<<grid, 256, 0, s>>>(dl, c, pooled, w, N, HW, C, J, nb_dx, dxb, dw, db);
  else
    head_bwd_kernel<false, 0><<<grid, 256, 0, s>>>(dl, c, pooled, w, N, HW, C, J, nb_dx, dxb, dw, db);
}

void add_bf16(const void* a, const void* b, int64_t n, void* y, hipStream_t s) {
  add_bf16_kernel<<<grid_for(n / 8), 256, 0, s>>>(static_cast<const bf16*>(a), static_cast<const bf16*>(b), n / 8,
                                                  static_cast<bf16*>(y));
}

}  // namespace kern
}  // namespace ringdp
