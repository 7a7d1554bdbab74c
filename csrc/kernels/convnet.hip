// MNIST ConvNet hot path for CDNA4 (gfx950): hand-written HIP, bf16 MFMA + LDS tiling.
//
// Model (ref/launch_dist.py:9-41):
//   conv1 1->32 k5 p1 (28->26) -> ReLU -> MaxPool(2,2) (13)
//   conv2 32->64 k3 (13->11)  -> ReLU -> MaxPool(2,1) (10)   [overlapping windows]
//   conv3 64->128 k3 (10->8)  -> ReLU -> MaxPool(2,2) (4)  -> view(-1, 2048) -> fc1 2048->10
//
// Kernel blocks (one autograd Function each, see ringdp/ops/convnet.py):
//   F1  conv1 + ReLU + pool1                       -> a1 [B,13,13,32] bf16 + argmax
//   F2  conv2 + ReLU                               -> r2 [B,11,11,64] bf16
//   F3  pool2 + conv3 + ReLU + pool3 + fc1         -> logits [B,10] fp32 (+ a3, argmax)
// The overlapping k2/s1 pool lives at the START of F3: its argmax is recomputed from r2 when
// needed, so no argmax tensor is stored for it and conv2's backward sees a plain ReLU mask.
//
// MI355X-first design:
//   * weight-stationary: weights are packed once per forward (cn_pack_weights) into bf16 MFMA
//     B-fragment order; every workgroup keeps its fragments in VGPRs for all the images it
//     processes; images stream through LDS with one-image-ahead register prefetch;
//   * window-ordered M: the GEMM rows of a conv followed by a 2x2/s2 pool are ordered
//     (pool window, position-in-window), so each lane's 4 accumulator registers of a
//     v_mfma_f32_16x16x32_bf16 tile are exactly one pool window -> bias + max + argmax + ReLU are
//     done in registers (conv1, conv3), no LDS round trip;
//   * fc1 is fused into the conv3 epilogue (partial logits reduced across lanes and waves);
//   * backward: dgrad is a weight-stationary full correlation over a zero-ringed LDS image; wgrad is
//     a TN GEMM whose operands are read with ds_read_b64_tr_b16 (the transposed read also does the
//     im2col gather), split over images into fp32 slabs reduced in a fixed order (deterministic);
//   * one multi-segment reduction launch per layer backward.
#include <vector>

#include "device_common.h"
#include "kernels.h"

namespace ringdp {
namespace kern {

using namespace ringdp::dev;

namespace {

__host__ __device__ constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }

// ------------------------------------------------------------------ packed weight layout
// bf16 element offsets inside the packed buffer.  Fragment order: [n-tile][k-step][lane][8].
constexpr int P1_OFF = 0, P1_N = 2 * 64 * 8;                    // conv1 fwd   (K = 25 -> 32)
constexpr int P2F_OFF = P1_OFF + P1_N, P2F_N = 4 * 9 * 512;     // conv2 fwd   (N 64, K 288)
constexpr int P3F_OFF = P2F_OFF + P2F_N, P3F_N = 8 * 18 * 512;  // conv3 fwd   (N 128, K 576)
constexpr int P2D_OFF = P3F_OFF + P3F_N, P2D_N = 2 * 18 * 512;  // conv2 dgrad (N 32, K 576)
constexpr int P3D_OFF = P2D_OFF + P2D_N, P3D_N = 4 * 36 * 512;  // conv3 dgrad (N 64, K 1152)
constexpr int PFC_OFF = P3D_OFF + P3D_N, PFC_N = 16 * 128 * 10; // fc1 [window][co][n]
constexpr int PACK_TOTAL = PFC_OFF + PFC_N;

__global__ __launch_bounds__(256) void pack_weights_kernel(const float* __restrict__ w1,
                                                           const float* __restrict__ w2,
                                                           const float* __restrict__ w3,
                                                           const float* __restrict__ wfc,
                                                           bf16* __restrict__ out) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= PACK_TOTAL) return;
  float v = 0.f;
  if (e < P2F_OFF) {
    const int j = e & 7, lane = (e >> 3) & 63, nt = e >> 9;
    const int co = nt * 16 + (lane & 15), t = 8 * (lane >> 4) + j;
    v = t < 25 ? w1[co * 25 + t] : 0.f;
  } else if (e < P2D_OFF) {  // forward fragments of conv2 / conv3: B[k = tap*CIN + ci][n = co]
    const bool l2 = e < P3F_OFF;
    const int r = e - (l2 ? P2F_OFF : P3F_OFF);
    const int CIN = l2 ? 32 : 64, KS = l2 ? 9 : 18;
    const float* w = l2 ? w2 : w3;
    const int j = r & 7, lane = (r >> 3) & 63, ks = (r >> 9) % KS, nt = (r >> 9) / KS;
    const int co = nt * 16 + (lane & 15), k = ks * 32 + 8 * (lane >> 4) + j;
    v = w[(co * CIN + k % CIN) * 9 + k / CIN];
  } else if (e < PFC_OFF) {  // dgrad fragments: B[k = tap'*COUT + co][n = ci] = W[co][ci][8 - tap']
    const bool l2 = e < P3D_OFF;
    const int r = e - (l2 ? P2D_OFF : P3D_OFF);
    const int CIN = l2 ? 32 : 64, COUT = l2 ? 64 : 128, KS = l2 ? 18 : 36;
    const float* w = l2 ? w2 : w3;
    const int j = r & 7, lane = (r >> 3) & 63, ks = (r >> 9) % KS, nt = (r >> 9) / KS;
    const int ci = nt * 16 + (lane & 15), k = ks * 32 + 8 * (lane >> 4) + j;
    v = w[((k % COUT) * CIN + ci) * 9 + (8 - k / COUT)];
  } else {
    const int r = e - PFC_OFF;
    const int n = r % 10, co = (r / 10) % 128, wd = r / 1280;
    v = wfc[n * 2048 + co * 16 + wd];
  }
  out[e] = (bf16)v;
}

__device__ __forceinline__ bf16x8 bmax8(const bf16x8& a, const bf16x8& b) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (float)a[j] >= (float)b[j] ? a[j] : b[j];
  return r;
}

// max over a 2x2 window of an LDS image with row stride rs (in bf16) and width w
__device__ __forceinline__ bf16x8 window_max8(const bf16* r0, int rs, int w) {
  return bmax8(bmax8(*reinterpret_cast<const bf16x8*>(r0), *reinterpret_cast<const bf16x8*>(r0 + rs)),
               bmax8(*reinterpret_cast<const bf16x8*>(r0 + w * rs),
                     *reinterpret_cast<const bf16x8*>(r0 + (w + 1) * rs)));
}

// First-max argmax over the 4 registers of a window + bias + ReLU (torch max_pool2d semantics:
// strict '>' keeps the first maximum in (0,0),(0,1),(1,0),(1,1) order).
__device__ __forceinline__ float pool4(const f32x4& c, float bias, int& arg) {
  float bm = c[0];
  arg = 0;
#pragma unroll
  for (int r = 1; r < 4; ++r)
    if (c[r] > bm) {
      bm = c[r];
      arg = r;
    }
  return fmaxf(bm + bias, 0.f);
}

__device__ __forceinline__ int byte_of(const uint2& v, int j) {
  return (int)(((j < 4 ? v.x : v.y) >> (8 * (j & 3))) & 0xff);
}

// window-ordered GEMM row r = 4*window + i of a pooled (2x2/s2) 8x8 map -> spatial y*pw + x
__device__ __forceinline__ int win_pos(int r, int pw) {
  const int w = r >> 2, i = r & 3;
  return (2 * (w >> 2) + (i >> 1)) * pw + 2 * (w & 3) + (i & 1);
}

__device__ __forceinline__ void stage_rows(const bf16* __restrict__ src, bf16* dst, int nchunks,
                                           int chunks_per_row, int rs, int tid, int nthreads) {
  for (int c = tid; c < nchunks; c += nthreads)
    *reinterpret_cast<bf16x8*>(dst + (c / chunks_per_row) * rs + (c % chunks_per_row) * 8) =
        reinterpret_cast<const bf16x8*>(src)[c];
}

// Async global -> LDS copy of 16 B per lane (global_load_lds_dwordx4): the LDS destination is the
// wave-uniform base + lane * 16, so the image it fills is lane-linear (no padding inside a wave's 1 KiB).
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// ================================================================== F1: conv1 (MFMA, K 25 -> 32)
constexpr int C1_XS = 30 * 30 + 12;  // zero-ringed 30x30 bf16 image (+pad)

template <bool U8>
__device__ __forceinline__ void c1_load(const void* xin, int b, int tid, uint32_t& u, float4& f) {
  if (tid < 196) {
    if (U8)
      u = reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(xin) + (int64_t)b * 784)[tid];
    else
      f = reinterpret_cast<const float4*>(static_cast<const float*>(xin) + (int64_t)b * 784)[tid];
  }
}

template <bool U8>
__device__ __forceinline__ void c1_store(bf16* xs, int tid, uint32_t u, float4 f, float mean,
                                         float inv_std, float in_scale) {
  if (tid < 196) {
    float v[4];
    if (U8) {
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = (float)((u >> (8 * k)) & 0xff) * in_scale;
    } else {
      v[0] = f.x;
      v[1] = f.y;
      v[2] = f.z;
      v[3] = f.w;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int p = 4 * tid + k, r = p / 28, c = p % 28;
      xs[(r + 1) * 30 + c + 1] = (bf16)((v[k] - mean) * inv_std);
    }
  }
}

template <bool U8>
__global__ __launch_bounds__(256) void conv1_fwd_kernel(const void* __restrict__ xin,
                                                        const bf16* __restrict__ packed,
                                                        const float* __restrict__ bias,
                                                        bf16* __restrict__ a1,
                                                        uint8_t* __restrict__ idx1, int B,
                                                        float mean, float inv_std, float in_scale) {
  __shared__ __attribute__((aligned(16))) bf16 xs[2][C1_XS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bf16x8* pk = reinterpret_cast<const bf16x8*>(packed + P1_OFF);
  const bf16x8 bw0 = pk[lane], bw1 = pk[64 + lane];
  const float bias0 = bias[lane & 15], bias1 = bias[16 + (lane & 15)];
  int toff[8];
  bool tval[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int t = 8 * (lane >> 4) + j;
    tval[j] = t < 25;
    toff[j] = tval[j] ? (t / 5) * 30 + t % 5 : 0;
  }
  for (int i = tid; i < 2 * C1_XS; i += 256) (&xs[0][0])[i] = (bf16)0.f;
  __syncthreads();
  uint32_t pu = 0;
  float4 pf = make_float4(0.f, 0.f, 0.f, 0.f);
  int b = blockIdx.x;
  if (b < B) {
    c1_load<U8>(xin, b, tid, pu, pf);
    c1_store<U8>(xs[0], tid, pu, pf, mean, inv_std, in_scale);
  }
  __syncthreads();
  int cur = 0;
  for (; b < B; b += gridDim.x) {
    const int nb = b + gridDim.x;
    if (nb < B) c1_load<U8>(xin, nb, tid, pu, pf);
    const bf16* x = xs[cur];
    for (int mt = wave; mt < 43; mt += 4) {
      const int r16 = lane & 15;
      const int w = 4 * mt + (r16 >> 2), i = r16 & 3;
      bf16x8 a = zero_bf16x8();
      if (w < 169) {
        const int base = (2 * (w / 13) + (i >> 1)) * 30 + 2 * (w % 13) + (i & 1);
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = tval[j] ? x[base + toff[j]] : (bf16)0.f;
      }
      const f32x4 c0 = mfma16x16x32(a, bw0, zero_f32x4());
      const f32x4 c1 = mfma16x16x32(a, bw1, zero_f32x4());
      const int wc = 4 * mt + (lane >> 4);
      if (wc < 169) {
        int g0, g1;
        const float v0 = pool4(c0, bias0, g0), v1 = pool4(c1, bias1, g1);
        const int64_t o = ((int64_t)b * 169 + wc) * 32 + (lane & 15);
        a1[o] = (bf16)v0;
        a1[o + 16] = (bf16)v1;
        idx1[o] = (uint8_t)g0;
        idx1[o + 16] = (uint8_t)g1;
      }
    }
    if (nb < B) c1_store<U8>(xs[cur ^ 1], tid, pu, pf, mean, inv_std, in_scale);
    __syncthreads();
    cur ^= 1;
  }
}

// ================================================================== F2: conv2 + ReLU
// 256 threads; wave (wm, wn) owns n-tiles {2wn, 2wn+1} x m-tiles {4wm..4wm+3} (121 rows -> 128).
constexpr int C2_XRS = 40;  // bf16 per LDS row of the a1 image (32 + 8 pad)
constexpr int C2_CRS = 72;  // bf16 per LDS row of the output staging tile (64 + 8)

__global__ __launch_bounds__(256, 2) void conv2_fwd_kernel(const bf16* __restrict__ a1,
                                                           const bf16* __restrict__ packed,
                                                           const float* __restrict__ bias,
                                                           bf16* __restrict__ r2, int B) {
  __shared__ __attribute__((aligned(16))) bf16 X[2][169 * C2_XRS];
  __shared__ __attribute__((aligned(16))) bf16 Cs[121 * C2_CRS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int r16 = lane & 15, q8 = (lane >> 4) * 8;
  const bf16x8* pk = reinterpret_cast<const bf16x8*>(packed + P2F_OFF);
  bf16x8 bw[2][9];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int ks = 0; ks < 9; ++ks) bw[t][ks] = pk[((2 * wn + t) * 9 + ks) * 64 + lane];
  float bv[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) bv[t] = bias[(2 * wn + t) * 16 + r16];
  int base[4];
  bool valid[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const int m = (4 * wm + mt) * 16 + r16;
    valid[mt] = m < 121;
    const int mm = valid[mt] ? m : 0;
    base[mt] = (mm / 11) * 13 + mm % 11;
  }
  bf16x8 pre[3];
  auto load = [&](int bb) {
    const bf16x8* src = reinterpret_cast<const bf16x8*>(a1 + (int64_t)bb * 169 * 32);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int c = tid + 256 * k;
      if (c < 676) pre[k] = src[c];
    }
  };
  auto store = [&](bf16* dst) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int c = tid + 256 * k;
      if (c < 676) *reinterpret_cast<bf16x8*>(dst + (c >> 2) * C2_XRS + (c & 3) * 8) = pre[k];
    }
  };
  int b = blockIdx.x;
  if (b < B) {
    load(b);
    store(X[0]);
  }
  __syncthreads();
  int cur = 0;
  for (; b < B; b += gridDim.x) {
    const int nb = b + gridDim.x;
    if (nb < B) load(nb);
    const bf16* x = X[cur];
    f32x4 acc[4][2];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[mt][0] = acc[mt][1] = zero_f32x4();
#pragma unroll
    for (int ks = 0; ks < 9; ++ks) {
      const int shift = (ks / 3) * 13 + ks % 3;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        bf16x8 a = zero_bf16x8();
        if (valid[mt]) a = *reinterpret_cast<const bf16x8*>(x + (base[mt] + shift) * C2_XRS + q8);
        acc[mt][0] = mfma16x16x32(a, bw[0][ks], acc[mt][0]);
        acc[mt][1] = mfma16x16x32(a, bw[1][ks], acc[mt][1]);
      }
    }
    __syncthreads();  // previous image's copy-out of Cs is complete
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = (4 * wm + mt) * 16 + (lane >> 4) * 4 + i;
          if (m < 121) Cs[m * C2_CRS + (2 * wn + t) * 16 + r16] = (bf16)fmaxf(acc[mt][t][i] + bv[t], 0.f);
        }
    if (nb < B) store(X[cur ^ 1]);
    __syncthreads();
    bf16x8* dst = reinterpret_cast<bf16x8*>(r2 + (int64_t)b * 121 * 64);
    for (int c = tid; c < 968; c += 256)
      dst[c] = *reinterpret_cast<const bf16x8*>(Cs + (c >> 3) * C2_CRS + (c & 7) * 8);
    cur ^= 1;
  }
}

// ================================================================== F3: pool2 + conv3 + ReLU + pool3 + fc1
// 256 threads; wave w owns output channels 32w..32w+31 (n-tiles 2w, 2w+1) for all 16 pool windows.
constexpr int C3_RRS = 64;  // bf16 per LDS row, r2 image (unpadded: filled by glds)
constexpr int C3_XRS = 72;  // bf16 per LDS row, pooled conv3 input (64 + 8)

__device__ __forceinline__ void pool2_into(const bf16* R, bf16* X, int tid, int nthreads) {
  for (int it = tid; it < 800; it += nthreads) {
    const int p = it >> 3, c = (it & 7) * 8;
    const int py = p / 10, px = p % 10;
    *reinterpret_cast<bf16x8*>(X + p * C3_XRS + c) = window_max8(R + (py * 11 + px) * C3_RRS + c, C3_RRS, 11);
  }
}

__global__ __launch_bounds__(256, 2) void conv3_fc_fwd_kernel(const bf16* __restrict__ r2,
                                                              const bf16* __restrict__ packed,
                                                              const float* __restrict__ bias,
                                                              const float* __restrict__ bfc,
                                                              float* __restrict__ logits,
                                                              bf16* __restrict__ a3,
                                                              uint8_t* __restrict__ idx3, int B) {
  __shared__ __attribute__((aligned(16))) bf16 R[121 * C3_RRS];
  __shared__ __attribute__((aligned(16))) bf16 X[100 * C3_XRS];
  __shared__ __attribute__((aligned(16))) bf16 Fc[PFC_N];
  __shared__ float red[4][10];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, q8 = (lane >> 4) * 8;
  const bf16x8* pk = reinterpret_cast<const bf16x8*>(packed + P3F_OFF);
  bf16x8 bw[2][18];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) bw[t][ks] = pk[((2 * wave + t) * 18 + ks) * 64 + lane];
  float bv[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) bv[t] = bias[32 * wave + 16 * t + r16];
  int base[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) base[mt] = win_pos(4 * (4 * mt + (r16 >> 2)) + (r16 & 3), 10);
  {
    const bf16x8* src = reinterpret_cast<const bf16x8*>(packed + PFC_OFF);
    for (int c = tid; c < PFC_N / 8; c += 256) reinterpret_cast<bf16x8*>(Fc)[c] = src[c];
  }
  // r2 image -> R: 968 16-B chunks = 16 wave-instructions (4 per wave), lane-linear
  auto stage = [&](int bb) {
    const bf16x8* src = reinterpret_cast<const bf16x8*>(r2 + (int64_t)bb * 121 * 64);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int inst = k * 4 + wave, c = inst * 64 + lane;
      if (c < 968) glds16(src + c, R + inst * 64 * 8);
    }
  };
  int b = blockIdx.x;
  if (b < B) stage(b);
  __syncthreads();
  for (; b < B; b += gridDim.x) {
    pool2_into(R, X, tid, 256);
    __syncthreads();  // X complete, R free
    const int nb = b + gridDim.x;
    if (nb < B) stage(nb);  // lands while the MFMAs below run
    f32x4 acc[4][2];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[mt][0] = acc[mt][1] = zero_f32x4();
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) {
      const int tap = ks >> 1, c0 = (ks & 1) * 32;
      const int shift = (tap / 3) * 10 + tap % 3;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(X + (base[mt] + shift) * C3_XRS + c0 + q8);
        acc[mt][0] = mfma16x16x32(a, bw[0][ks], acc[mt][0]);
        acc[mt][1] = mfma16x16x32(a, bw[1][ks], acc[mt][1]);
      }
    }
    float s[10];
#pragma unroll
    for (int n = 0; n < 10; ++n) s[n] = 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int wc = 4 * mt + (lane >> 4), co = 32 * wave + 16 * t + r16;
        int g;
        const bf16 pb = (bf16)pool4(acc[mt][t], bv[t], g);
        const int64_t o = ((int64_t)b * 16 + wc) * 128 + co;
        a3[o] = pb;
        idx3[o] = (uint8_t)g;
        const float pf = (float)pb;
        const uint32_t* fw = reinterpret_cast<const uint32_t*>(Fc + (wc * 128 + co) * 10);
#pragma unroll
        for (int h = 0; h < 5; ++h) {
          const uint32_t u = fw[h];
          s[2 * h] = fmaf(pf, __uint_as_float(u << 16), s[2 * h]);
          s[2 * h + 1] = fmaf(pf, __uint_as_float(u & 0xffff0000u), s[2 * h + 1]);
        }
      }
#pragma unroll
    for (int n = 0; n < 10; ++n) s[n] = wave_sum(s[n]);
    if (lane == 0) {
#pragma unroll
      for (int n = 0; n < 10; ++n) red[wave][n] = s[n];
    }
    __syncthreads();
    if (tid < 10)
      logits[(int64_t)b * 10 + tid] = ((red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid])) + bfc[tid];
  }
}

// ================================================================== F3 backward
// (1) fc1 backward: da3 = dl . Wfc, scattered to window-ordered d(conv3) rows D3[b][4w + i][co]
//     (one non-zero per window: the argmax, if the pooled value is > 0) + fc weight-grad slabs.
constexpr int FC_SLAB = 10 * 2048 + 10;

__global__ __launch_bounds__(256) void fc_bwd_kernel(const bf16* __restrict__ a3,
                                                     const uint8_t* __restrict__ idx3,
                                                     const float* __restrict__ wfc,
                                                     const float* __restrict__ dl,
                                                     bf16* __restrict__ d3, float* __restrict__ slabs,
                                                     int nslices, int B) {
  const int t = threadIdx.x;
  const int wd = t >> 4, co0 = (t & 15) * 8;  // this thread's 8 activations: window wd, channels co0..
  float wr[10][8];
#pragma unroll
  for (int n = 0; n < 10; ++n)
#pragma unroll
    for (int j = 0; j < 8; ++j) wr[n][j] = wfc[n * 2048 + (co0 + j) * 16 + wd];
  float acc[10][8];
#pragma unroll
  for (int n = 0; n < 10; ++n)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[n][j] = 0.f;
  float bacc = 0.f;
  const int per = cdiv(B, nslices);
  const int b_lo = blockIdx.x * per, b_hi = min(B, b_lo + per);
  for (int b = b_lo; b < b_hi; ++b) {
    float g[10];
#pragma unroll
    for (int n = 0; n < 10; ++n) g[n] = dl[(int64_t)b * 10 + n];
    const int64_t o = (int64_t)b * 2048 + wd * 128 + co0;
    const bf16x8 av = *reinterpret_cast<const bf16x8*>(a3 + o);
    const uint2 iv = *reinterpret_cast<const uint2*>(idx3 + o);
    float da[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s = 0.f;
      const float aj = (float)av[j];
#pragma unroll
      for (int n = 0; n < 10; ++n) {
        s = fmaf(g[n], wr[n][j], s);
        acc[n][j] = fmaf(g[n], aj, acc[n][j]);
      }
      da[j] = aj > 0.f ? s : 0.f;
    }
    bf16* drow = d3 + ((int64_t)b * 64 + 4 * wd) * 128 + co0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (bf16)(byte_of(iv, j) == i ? da[j] : 0.f);
      *reinterpret_cast<bf16x8*>(drow + i * 128) = v;
    }
    if (t < 10) bacc += dl[(int64_t)b * 10 + t];
  }
  float* slab = slabs + (int64_t)blockIdx.x * FC_SLAB;
#pragma unroll
  for (int n = 0; n < 10; ++n)
#pragma unroll
    for (int j = 0; j < 8; ++j) slab[n * 2048 + (co0 + j) * 16 + wd] = acc[n][j];
  if (t < 10) slab[20480 + t] = bacc;
}

// (2) conv3 backward, two roles in one 512-thread launch:
//   dgrad: da2 = full-corr(D3 image, flipped W3) -> pool2 backward (argmax recomputed from r2)
//          -> dr2 [B,11,11,64];
//   wgrad: dW3t[n = tap*64 + ci][co] = sum_k D3[k][co] * a2[pos(k) + tap][ci], a2 = pool2(r2).
constexpr int C3_PW = 12;    // padded d(conv3) image width (8 + 2*2)
constexpr int C3_PRS = 136;  // bf16 per padded-image row (128 + 8)
constexpr int C3_DARS = 68;  // floats per da2 row (64 + 4)
constexpr int C3_DRS = 136;  // bf16 per D3 row in LDS
constexpr int C3B_P_BYTES = C3_PW * C3_PW * C3_PRS * 2;  // 39168
constexpr int C3B_R_BYTES = 121 * C3_RRS * 2;            // 15488
constexpr int C3B_AM_BYTES = 100 * 64;                   // 6400
constexpr int C3B_DG_LDS = C3B_P_BYTES + C3B_R_BYTES + C3B_AM_BYTES;
constexpr int C3B_D_BYTES = 64 * C3_DRS * 2;   // 17408
constexpr int C3B_X_BYTES = 100 * C3_XRS * 2;  // 14400
constexpr int C3B_WG_LDS = C3B_D_BYTES + C3B_X_BYTES + C3B_R_BYTES;
constexpr int C3B_LDS = C3B_DG_LDS > C3B_WG_LDS ? C3B_DG_LDS : C3B_WG_LDS;
constexpr int C3_WSLAB = 576 * 128 + 128;  // dW3t + db3
static_assert(100 * C3_DARS * 4 <= C3B_P_BYTES, "da2 must fit in the padded-image region");

__device__ void conv3_dgrad_role(char* smem, const bf16* __restrict__ r2, const bf16* __restrict__ d3,
                                 const bf16* __restrict__ packed, bf16* __restrict__ dr2, int B,
                                 int block, int nblocks) {
  bf16* P = reinterpret_cast<bf16*>(smem);
  float* DA = reinterpret_cast<float*>(smem);  // aliases P after the MFMA phase
  bf16* R = reinterpret_cast<bf16*>(smem + C3B_P_BYTES);
  uint8_t* AM = reinterpret_cast<uint8_t*>(smem + C3B_P_BYTES + C3B_R_BYTES);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nt = wave & 3, mh = wave >> 2;  // n-tile (16 input channels), m-tile parity
  const int r16 = lane & 15, q8 = (lane >> 4) * 8;
  const bf16x8* pk = reinterpret_cast<const bf16x8*>(packed + P3D_OFF);
  bf16x8 bw[36];
#pragma unroll
  for (int ks = 0; ks < 36; ++ks) bw[ks] = pk[(nt * 36 + ks) * 64 + lane];
  int base[4];
  bool valid[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int mt = mh + 2 * k;
    const int m = mt * 16 + r16;
    valid[k] = mt < 7 && m < 100;
    const int mm = valid[k] ? m : 0;
    base[k] = (mm / 10) * C3_PW + mm % 10;
  }
  const int nk = mh ? 3 : 4;
  for (int b = block; b < B; b += nblocks) {
    __syncthreads();
    // zero the whole padded image (its ring was overwritten by DA), stage r2
    for (int c = tid; c < C3_PW * C3_PW * C3_PRS / 8; c += 512) reinterpret_cast<bf16x8*>(P)[c] = zero_bf16x8();
    stage_rows(r2 + (int64_t)b * 121 * 64, R, 968, 8, C3_RRS, tid, 512);
    __syncthreads();
    {
      const bf16x8* src = reinterpret_cast<const bf16x8*>(d3 + (int64_t)b * 64 * 128);
      for (int c = tid; c < 1024; c += 512) {
        const int r = c >> 4, cc = (c & 15) * 8;
        *reinterpret_cast<bf16x8*>(P + (win_pos(r, C3_PW) + 2 * C3_PW + 2) * C3_PRS + cc) = src[c];
      }
    }
    // pool2 argmax per window (first max), from the r2 image
    for (int it = tid; it < 800; it += 512) {
      const int p = it >> 3, c = (it & 7) * 8;
      const int py = p / 10, px = p % 10;
      const bf16* r0 = R + (py * 11 + px) * C3_RRS + c;
      const bf16x8 v0 = *reinterpret_cast<const bf16x8*>(r0);
      const bf16x8 v1 = *reinterpret_cast<const bf16x8*>(r0 + C3_RRS);
      const bf16x8 v2 = *reinterpret_cast<const bf16x8*>(r0 + 11 * C3_RRS);
      const bf16x8 v3 = *reinterpret_cast<const bf16x8*>(r0 + 12 * C3_RRS);
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float bm = (float)v0[j];
        uint32_t g = 0;
        if ((float)v1[j] > bm) {
          bm = (float)v1[j];
          g = 1;
        }
        if ((float)v2[j] > bm) {
          bm = (float)v2[j];
          g = 2;
        }
        if ((float)v3[j] > bm) g = 3;
        if (j < 4)
          lo |= g << (8 * j);
        else
          hi |= g << (8 * (j - 4));
      }
      *reinterpret_cast<uint2*>(AM + p * 64 + c) = make_uint2(lo, hi);
    }
    __syncthreads();
    f32x4 acc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = zero_f32x4();
#pragma unroll 4
    for (int ks = 0; ks < 36; ++ks) {
      const int tapp = ks >> 2, c0 = (ks & 3) * 32;
      const int shift = (tapp / 3) * C3_PW + tapp % 3;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (k < nk) {
          bf16x8 a = zero_bf16x8();
          if (valid[k]) a = *reinterpret_cast<const bf16x8*>(P + (base[k] + shift) * C3_PRS + c0 + q8);
          acc[k] = mfma16x16x32(a, bw[ks], acc[k]);
        }
      }
    }
    __syncthreads();  // P dead -> DA
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int mt = mh + 2 * k;
      if (k < nk) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = mt * 16 + (lane >> 4) * 4 + i;
          if (m < 100) DA[m * C3_DARS + nt * 16 + r16] = acc[k][i];
        }
      }
    }
    __syncthreads();
    // pool2 backward (gather): dr2[y][x] = sum of da2 over the windows whose argmax is (y, x)
    bf16x8* dst = reinterpret_cast<bf16x8*>(dr2 + (int64_t)b * 121 * 64);
    for (int it = tid; it < 968; it += 512) {
      const int pos = it >> 3, c = (it & 7) * 8;
      const int y = pos / 11, x = pos % 11;
      float g[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = 0.f;
      for (int py = max(0, y - 1); py <= min(9, y); ++py)
        for (int px = max(0, x - 1); px <= min(9, x); ++px) {
          const int want = (y - py) * 2 + (x - px);
          const int p = py * 10 + px;
          const uint2 am = *reinterpret_cast<const uint2*>(AM + p * 64 + c);
          const float4 d0 = *reinterpret_cast<const float4*>(DA + p * C3_DARS + c);
          const float4 d1 = *reinterpret_cast<const float4*>(DA + p * C3_DARS + c + 4);
          const float dv[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (byte_of(am, j) == want) g[j] += dv[j];
        }
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (bf16)g[j];
      dst[it] = v;
    }
  }
}

__device__ void conv3_wgrad_role(char* smem, const bf16* __restrict__ r2, const bf16* __restrict__ d3,
                                 float* __restrict__ slabs, int B, int nslices, int slice) {
  bf16* D = reinterpret_cast<bf16*>(smem);
  bf16* X = reinterpret_cast<bf16*>(smem + C3B_D_BYTES);
  bf16* R = reinterpret_cast<bf16*>(smem + C3B_D_BYTES + C3B_X_BYTES);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;  // m-tiles 4wm..4wm+3 (co), n-tiles 9wn..9wn+8
  const int g16 = lane & 15, grp = lane >> 4, q = g16 >> 2, p = g16 & 3;
  f32x4 acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = zero_f32x4();
  float bacc = 0.f;
  const int per = cdiv(B, nslices);
  const int b_lo = slice * per, b_hi = min(B, b_lo + per);
  for (int b = b_lo; b < b_hi; ++b) {
    __syncthreads();
    stage_rows(d3 + (int64_t)b * 64 * 128, D, 1024, 16, C3_DRS, tid, 512);
    stage_rows(r2 + (int64_t)b * 121 * 64, R, 968, 8, C3_RRS, tid, 512);
    __syncthreads();
    pool2_into(R, X, tid, 512);
    if (tid < 128) {
      float s = 0.f;
      for (int r = 0; r < 64; ++r) s += (float)D[r * C3_DRS + tid];
      bacc += s;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int kb = ks * 32 + grp * 8;
      bf16x8 af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m0 = (4 * wm + i) * 16;
        const bf16x4 lo = lds_read_tr16(D + (kb + q) * C3_DRS + m0 + 4 * p);
        const bf16x4 hi = lds_read_tr16(D + (kb + 4 + q) * C3_DRS + m0 + 4 * p);
        af[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      const int x0 = win_pos(kb + q, 10), x1 = win_pos(kb + 4 + q, 10);
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const int n0 = (9 * wn + j) * 16;  // n = tap*64 + ci
        const int tap = n0 >> 6, c0 = n0 & 63;
        const int shift = (tap / 3) * 10 + tap % 3;
        const bf16x4 lo = lds_read_tr16(X + (x0 + shift) * C3_XRS + c0 + 4 * p);
        const bf16x4 hi = lds_read_tr16(X + (x1 + shift) * C3_XRS + c0 + 4 * p);
        const bf16x8 bf = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][j] = mfma16x16x32(af[i], bf, acc[i][j]);
      }
    }
  }
  float* slab = slabs + (int64_t)slice * C3_WSLAB;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int co = (4 * wm + i) * 16 + grp * 4;
      const int n = (9 * wn + j) * 16 + g16;
      *reinterpret_cast<f32x4*>(slab + (int64_t)n * 128 + co) = acc[i][j];
    }
  if (tid < 128) slab[576 * 128 + tid] = bacc;
}

__global__ __launch_bounds__(512) void conv3_bwd_kernel(const bf16* __restrict__ r2,
                                                        const bf16* __restrict__ d3,
                                                        const bf16* __restrict__ packed,
                                                        bf16* __restrict__ dr2, int B,
                                                        float* __restrict__ slabs, int nslices,
                                                        int n_dgrad) {
  __shared__ __attribute__((aligned(16))) char smem[C3B_LDS];
  if ((int)blockIdx.x < n_dgrad)
    conv3_dgrad_role(smem, r2, d3, packed, dr2, B, blockIdx.x, n_dgrad);
  else
    conv3_wgrad_role(smem, r2, d3, slabs, B, nslices, blockIdx.x - n_dgrad);
}

// ================================================================== F2 backward
// dconv2 = dr2 * (r2 > 0) (ReLU mask); roles:
//   dgrad: da1 = full-corr(dconv2 image, flipped W2)  [13x13x32]
//   wgrad: dW2t[n = tap*32 + ci][co] = sum_pos dconv2[pos][co] * a1[pos + tap][ci]
constexpr int C2_PW = 15, C2_PRS = 72, C2_ORS = 40, C2_DRS = 72;
constexpr int C2B_P_BYTES = C2_PW * C2_PW * C2_PRS * 2;  // 32400
constexpr int C2B_O_BYTES = 169 * C2_ORS * 2;            // 13520
constexpr int C2B_D_BYTES = 128 * C2_DRS * 2;            // 18432
constexpr int C2B_X_BYTES = 169 * C2_XRS * 2;            // 13520
constexpr int C2B_LDS = (C2B_P_BYTES + C2B_O_BYTES) > (C2B_D_BYTES + C2B_X_BYTES)
                            ? (C2B_P_BYTES + C2B_O_BYTES)
                            : (C2B_D_BYTES + C2B_X_BYTES);
constexpr int C2_WSLAB = 288 * 64 + 64;

__device__ __forceinline__ bf16x8 relu_mask8(const bf16x8& g, const bf16x8& r) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)r[j] > 0.f ? g[j] : (bf16)0.f;
  return v;
}

__device__ void conv2_dgrad_role(char* smem, const bf16* __restrict__ r2, const bf16* __restrict__ dr2,
                                 const bf16* __restrict__ packed, bf16* __restrict__ da1, int B,
                                 int block, int nblocks) {
  bf16* P = reinterpret_cast<bf16*>(smem);
  bf16* O = reinterpret_cast<bf16*>(smem + C2B_P_BYTES);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nt = wave & 1, mg = wave >> 1;  // n-tile (16 input channels), m-tiles mg, mg+4, mg+8
  const int r16 = lane & 15, q8 = (lane >> 4) * 8;
  const bf16x8* pk = reinterpret_cast<const bf16x8*>(packed + P2D_OFF);
  bf16x8 bw[18];
#pragma unroll
  for (int ks = 0; ks < 18; ++ks) bw[ks] = pk[(nt * 18 + ks) * 64 + lane];
  int base[3];
  bool valid[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int mt = mg + 4 * k;
    const int m = mt * 16 + r16;
    valid[k] = mt < 11 && m < 169;
    const int mm = valid[k] ? m : 0;
    base[k] = (mm / 13) * C2_PW + mm % 13;
  }
  const int nk = mg == 3 ? 2 : 3;
  for (int c = tid; c < C2_PW * C2_PW * C2_PRS / 8; c += 512) reinterpret_cast<bf16x8*>(P)[c] = zero_bf16x8();
  for (int b = block; b < B; b += nblocks) {
    __syncthreads();
    {
      const bf16x8* g = reinterpret_cast<const bf16x8*>(dr2 + (int64_t)b * 121 * 64);
      const bf16x8* r = reinterpret_cast<const bf16x8*>(r2 + (int64_t)b * 121 * 64);
      for (int c = tid; c < 968; c += 512) {
        const int pos = c >> 3, cc = (c & 7) * 8;
        const int y = pos / 11, x = pos % 11;
        *reinterpret_cast<bf16x8*>(P + ((y + 2) * C2_PW + x + 2) * C2_PRS + cc) = relu_mask8(g[c], r[c]);
      }
    }
    __syncthreads();
    f32x4 acc[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) acc[k] = zero_f32x4();
#pragma unroll 2
    for (int ks = 0; ks < 18; ++ks) {
      const int tapp = ks >> 1, c0 = (ks & 1) * 32;
      const int shift = (tapp / 3) * C2_PW + tapp % 3;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        if (k < nk) {
          bf16x8 a = zero_bf16x8();
          if (valid[k]) a = *reinterpret_cast<const bf16x8*>(P + (base[k] + shift) * C2_PRS + c0 + q8);
          acc[k] = mfma16x16x32(a, bw[ks], acc[k]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int mt = mg + 4 * k;
      if (k < nk) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = mt * 16 + (lane >> 4) * 4 + i;
          if (m < 169) O[m * C2_ORS + nt * 16 + r16] = (bf16)acc[k][i];
        }
      }
    }
    __syncthreads();
    bf16x8* dst = reinterpret_cast<bf16x8*>(da1 + (int64_t)b * 169 * 32);
    for (int c = tid; c < 676; c += 512) dst[c] = *reinterpret_cast<const bf16x8*>(O + (c >> 2) * C2_ORS + (c & 3) * 8);
  }
}

__device__ void conv2_wgrad_role(char* smem, const bf16* __restrict__ a1, const bf16* __restrict__ r2,
                                 const bf16* __restrict__ dr2, float* __restrict__ slabs, int B,
                                 int nslices, int slice) {
  bf16* D = reinterpret_cast<bf16*>(smem);
  bf16* X = reinterpret_cast<bf16*>(smem + C2B_D_BYTES);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;  // m-tile wm (co 16wm..), n-tiles 9wn..9wn+8
  const int g16 = lane & 15, grp = lane >> 4, q = g16 >> 2, p = g16 & 3;
  f32x4 acc[9];
#pragma unroll
  for (int j = 0; j < 9; ++j) acc[j] = zero_f32x4();
  float bacc = 0.f;
  for (int c = tid; c < 128 * C2_DRS / 8; c += 512) reinterpret_cast<bf16x8*>(D)[c] = zero_bf16x8();
  const int per = cdiv(B, nslices);
  const int b_lo = slice * per, b_hi = min(B, b_lo + per);
  for (int b = b_lo; b < b_hi; ++b) {
    __syncthreads();
    {
      const bf16x8* g = reinterpret_cast<const bf16x8*>(dr2 + (int64_t)b * 121 * 64);
      const bf16x8* r = reinterpret_cast<const bf16x8*>(r2 + (int64_t)b * 121 * 64);
      for (int c = tid; c < 968; c += 512)
        *reinterpret_cast<bf16x8*>(D + (c >> 3) * C2_DRS + (c & 7) * 8) = relu_mask8(g[c], r[c]);
    }
    stage_rows(a1 + (int64_t)b * 169 * 32, X, 676, 4, C2_XRS, tid, 512);
    __syncthreads();
    if (tid < 64) {
      float s = 0.f;
      for (int r = 0; r < 121; ++r) s += (float)D[r * C2_DRS + tid];
      bacc += s;
    }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int kb = ks * 32 + grp * 8;
      const int m0 = wm * 16;
      const bf16x4 alo = lds_read_tr16(D + (kb + q) * C2_DRS + m0 + 4 * p);
      const bf16x4 ahi = lds_read_tr16(D + (kb + 4 + q) * C2_DRS + m0 + 4 * p);
      const bf16x8 af = bf16x8{alo[0], alo[1], alo[2], alo[3], ahi[0], ahi[1], ahi[2], ahi[3]};
      const int k0 = min(kb + q, 120), k1 = min(kb + 4 + q, 120);  // rows >= 121 of D are zero
      const int x0 = (k0 / 11) * 13 + k0 % 11, x1 = (k1 / 11) * 13 + k1 % 11;
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const int n0 = (9 * wn + j) * 16;  // n = tap*32 + ci
        const int tap = n0 >> 5, c0 = n0 & 31;
        const int shift = (tap / 3) * 13 + tap % 3;
        const bf16x4 lo = lds_read_tr16(X + (x0 + shift) * C2_XRS + c0 + 4 * p);
        const bf16x4 hi = lds_read_tr16(X + (x1 + shift) * C2_XRS + c0 + 4 * p);
        const bf16x8 bf = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        acc[j] = mfma16x16x32(af, bf, acc[j]);
      }
    }
  }
  float* slab = slabs + (int64_t)slice * C2_WSLAB;
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int co = wm * 16 + grp * 4;
    const int n = (9 * wn + j) * 16 + g16;
    *reinterpret_cast<f32x4*>(slab + (int64_t)n * 64 + co) = acc[j];
  }
  if (tid < 64) slab[288 * 64 + tid] = bacc;
}

__global__ __launch_bounds__(512) void conv2_bwd_kernel(const bf16* __restrict__ a1,
                                                        const bf16* __restrict__ r2,
                                                        const bf16* __restrict__ dr2,
                                                        const bf16* __restrict__ packed,
                                                        bf16* __restrict__ da1, int B,
                                                        float* __restrict__ slabs, int nslices,
                                                        int n_dgrad) {
  __shared__ __attribute__((aligned(16))) char smem[C2B_LDS];
  if ((int)blockIdx.x < n_dgrad)
    conv2_dgrad_role(smem, r2, dr2, packed, da1, B, blockIdx.x, n_dgrad);
  else
    conv2_wgrad_role(smem, a1, r2, dr2, slabs, B, nslices, blockIdx.x - n_dgrad);
}

// ================================================================== F1 backward (conv1 wgrad)
// dW1[co][t] = sum_{b, k} Dc[b][k][co] * xpad[b][pos(k) + (kh, kw)], K rows in window order
// (k = 4w + i: one non-zero row per window and channel - the argmax, if the pooled value > 0).
constexpr int C1W_K = 704;          // 676 rows padded to 22 k-steps
constexpr int C1W_DRS = C1W_K + 8;  // bf16 per co row of the transposed d(conv1)
constexpr int C1_WSLAB = 32 * 25 + 32;

template <bool U8>
__global__ __launch_bounds__(256) void conv1_wgrad_kernel(const void* __restrict__ xin,
                                                          const bf16* __restrict__ da1,
                                                          const uint8_t* __restrict__ idx1,
                                                          const bf16* __restrict__ a1, int B,
                                                          float mean, float inv_std, float in_scale,
                                                          float* __restrict__ slabs, int nslices) {
  __shared__ __attribute__((aligned(16))) bf16 Dt[32 * C1W_DRS];
  __shared__ __attribute__((aligned(16))) bf16 xs[C1_XS];
  __shared__ float bred[32][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int mt = wave >> 1, nt = wave & 1;
  const int r16 = lane & 15, q = lane >> 4;
  const int t = nt * 16 + r16;
  const bool tvalid = t < 25;
  const int toff = tvalid ? (t / 5) * 30 + t % 5 : 0;
  f32x4 acc = zero_f32x4();
  float bpart[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bpart[j] = 0.f;
  for (int i = tid; i < 32 * C1W_DRS / 8; i += 256) reinterpret_cast<bf16x8*>(Dt)[i] = zero_bf16x8();
  for (int i = tid; i < C1_XS; i += 256) xs[i] = (bf16)0.f;
  const int per = cdiv(B, nslices);
  const int b_lo = blockIdx.x * per, b_hi = min(B, b_lo + per);
  const int c0 = (tid & 3) * 8;  // fixed channel chunk of this thread in the staging loop
  for (int b = b_lo; b < b_hi; ++b) {
    __syncthreads();
    uint32_t u = 0;
    float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
    c1_load<U8>(xin, b, tid, u, f);
    c1_store<U8>(xs, tid, u, f, mean, inv_std, in_scale);
    for (int it = tid; it < 676; it += 256) {
      const int w = it >> 2;
      const int64_t o = ((int64_t)b * 169 + w) * 32 + c0;
      const bf16x8 g = *reinterpret_cast<const bf16x8*>(da1 + o);
      const bf16x8 pv = *reinterpret_cast<const bf16x8*>(a1 + o);
      const uint2 iv = *reinterpret_cast<const uint2*>(idx1 + o);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bf16 gb = (float)pv[j] > 0.f ? g[j] : (bf16)0.f;
        bpart[j] += (float)gb;
        const int ij = byte_of(iv, j);
        bf16x4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = i == ij ? gb : (bf16)0.f;
        *reinterpret_cast<bf16x4*>(Dt + (c0 + j) * C1W_DRS + 4 * w) = v;
      }
    }
    __syncthreads();
#pragma unroll 2
    for (int ks = 0; ks < 22; ++ks) {
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(Dt + (mt * 16 + r16) * C1W_DRS + ks * 32 + q * 8);
      bf16x8 bf = zero_bf16x8();
      if (tvalid) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = min(ks * 32 + q * 8 + j, 675);  // Dt columns >= 676 are zero
          const int w = k >> 2, i = k & 3;
          bf[j] = xs[(2 * (w / 13) + (i >> 1)) * 30 + 2 * (w % 13) + (i & 1) + toff];
        }
      }
      acc = mfma16x16x32(af, bf, acc);
    }
  }
  // bias: the 16 lanes of a wave with the same channel chunk (lane & 3) reduce by shuffles,
  // then the 4 waves through LDS (fixed order)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float v = bpart[j];
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64);
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (lane < 4) bred[c0 + j][wave] = v;
  }
  __syncthreads();
  float* slab = slabs + (int64_t)blockIdx.x * C1_WSLAB;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int co = mt * 16 + q * 4 + i;
    if (tvalid) slab[co * 25 + t] = acc[i];
  }
  if (tid < 32) slab[800 + tid] = (bred[tid][0] + bred[tid][1]) + (bred[tid][2] + bred[tid][3]);
}

// ================================================================== fixed-order slab reductions
struct ReduceSeg {
  const float* slabs;
  int64_t stride;  // floats between consecutive slices
  int64_t off;     // first float of this segment inside a slice
  int64_t n;       // outputs
  int nslices;
  float* out;
  int mode;  // 0: out[i] = sum; 1: conv transpose dWt[n = tap*cin + ci][co] -> W[co][ci][tap]
  int cin, cout;
  int blocks;
};
struct ReduceSegs {
  ReduceSeg seg[4];
  int count;
};

// Each workgroup owns 64 outputs of one segment and sums its slices with 4 waves (lane = output,
// coalesced rows) combined in a fixed order.
__global__ __launch_bounds__(256) void slab_reduce_kernel(ReduceSegs segs) {
  __shared__ float part[4][64];
  int blk = blockIdx.x, sidx = 0;
  while (sidx < segs.count - 1 && blk >= segs.seg[sidx].blocks) {
    blk -= segs.seg[sidx].blocks;
    ++sidx;
  }
  const ReduceSeg& sg = segs.seg[sidx];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t i = (int64_t)blk * 64 + lane;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (i < sg.n) {
    const float* pp = sg.slabs + sg.off + i;
    int s = wave;
    for (; s + 12 < sg.nslices; s += 16) {
      a0 += pp[(int64_t)s * sg.stride];
      a1 += pp[(int64_t)(s + 4) * sg.stride];
      a2 += pp[(int64_t)(s + 8) * sg.stride];
      a3 += pp[(int64_t)(s + 12) * sg.stride];
    }
    for (; s < sg.nslices; s += 4) a0 += pp[(int64_t)s * sg.stride];
  }
  part[wave][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (wave != 0 || i >= sg.n) return;
  const float v = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
  if (sg.mode == 0) {
    sg.out[i] = v;
  } else {
    const int n = (int)(i / sg.cout), co = (int)(i % sg.cout);
    sg.out[((int64_t)co * sg.cin + n % sg.cin) * 9 + n / sg.cin] = v;
  }
}

ReduceSeg seg(const float* slabs, int64_t stride, int64_t off, int64_t n, int nslices, float* out,
              int mode = 0, int cin = 0, int cout = 0) {
  return ReduceSeg{slabs, stride, off, n, nslices, out, mode, cin, cout, (int)((n + 63) / 64)};
}

void launch_reduce(const std::vector<ReduceSeg>& v, hipStream_t s) {
  ReduceSegs segs{};
  int total = 0;
  segs.count = (int)v.size();
  for (size_t k = 0; k < v.size(); ++k) {
    segs.seg[k] = v[k];
    total += v[k].blocks;
  }
  slab_reduce_kernel<<<total, 256, 0, s>>>(segs);
}

int num_cus() {
  static int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
      hipDeviceProp_t p;
      if (hipGetDeviceProperties(&p, dev) == hipSuccess) n = p.multiProcessorCount;
    }
    return n;
  }();
  return cus;
}

inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

}  // namespace

// ================================================================== launchers
int64_t cn_packed_elems() { return PACK_TOTAL; }

void cn_pack_weights(const float* w1, const float* w2, const float* w3, const float* wfc, void* out,
                     hipStream_t s) {
  pack_weights_kernel<<<cdiv(PACK_TOTAL, 256), 256, 0, s>>>(w1, w2, w3, wfc, static_cast<bf16*>(out));
}

void cn_conv1_fwd(const void* x, bool u8, const void* packed, const float* b1, void* a1, uint8_t* idx1,
                  int B, float mean, float inv_std, float in_scale, hipStream_t s) {
  const int grid = clampi(B, 1, 4 * num_cus());
  const bf16* pk = static_cast<const bf16*>(packed);
  if (u8)
    conv1_fwd_kernel<true><<<grid, 256, 0, s>>>(x, pk, b1, static_cast<bf16*>(a1), idx1, B, mean, inv_std, in_scale);
  else
    conv1_fwd_kernel<false><<<grid, 256, 0, s>>>(x, pk, b1, static_cast<bf16*>(a1), idx1, B, mean, inv_std, in_scale);
}

void cn_conv2_fwd(const void* a1, const void* packed, const float* b2, void* r2, int B, hipStream_t s) {
  const int grid = clampi(B, 1, 2 * num_cus());
  conv2_fwd_kernel<<<grid, 256, 0, s>>>(static_cast<const bf16*>(a1), static_cast<const bf16*>(packed), b2,
                                        static_cast<bf16*>(r2), B);
}

void cn_conv3_fc_fwd(const void* r2, const void* packed, const float* b3, const float* bfc, float* logits,
                     void* a3, uint8_t* idx3, int B, hipStream_t s) {
  const int grid = clampi(B, 1, 2 * num_cus());
  conv3_fc_fwd_kernel<<<grid, 256, 0, s>>>(static_cast<const bf16*>(r2), static_cast<const bf16*>(packed), b3,
                                           bfc, logits, static_cast<bf16*>(a3), idx3, B);
}

static int fc_slices(int B) { return clampi(cdiv(B, 4), 1, 128); }
static int conv3_wslices(int B) { return clampi(cdiv(B, 8), 1, num_cus()); }
static int conv2_wslices(int B) { return clampi(cdiv(B, 8), 1, num_cus()); }
static int conv1_wslices(int B) { return clampi(cdiv(B, 4), 1, 2 * num_cus()); }
int64_t cn_fc_slab_floats(int B) { return (int64_t)fc_slices(B) * FC_SLAB; }
int64_t cn_conv3_slab_floats(int B) { return (int64_t)conv3_wslices(B) * C3_WSLAB; }
int64_t cn_conv2_slab_floats(int B) { return (int64_t)conv2_wslices(B) * C2_WSLAB; }
int64_t cn_conv1_slab_floats(int B) { return (int64_t)conv1_wslices(B) * C1_WSLAB; }

void cn_conv3_fc_bwd(const void* r2, const void* a3, const uint8_t* idx3, const float* wfc, const float* dl,
                     const void* packed, void* d3, void* dr2, int B, float* fc_slabs, float* c3_slabs,
                     float* dw3, float* db3, float* dwfc, float* dbfc, hipStream_t s) {
  const int fs = fc_slices(B);
  fc_bwd_kernel<<<fs, 256, 0, s>>>(static_cast<const bf16*>(a3), idx3, wfc, dl, static_cast<bf16*>(d3),
                                   fc_slabs, fs, B);
  const int ws = conv3_wslices(B);
  const int nd = dr2 ? clampi(B, 1, num_cus()) : 0;
  conv3_bwd_kernel<<<nd + ws, 512, 0, s>>>(static_cast<const bf16*>(r2), static_cast<const bf16*>(d3),
                                           static_cast<const bf16*>(packed), static_cast<bf16*>(dr2), B,
                                           c3_slabs, ws, nd);
  launch_reduce({seg(c3_slabs, C3_WSLAB, 0, 576 * 128, ws, dw3, 1, 64, 128),
                 seg(c3_slabs, C3_WSLAB, 576 * 128, 128, ws, db3), seg(fc_slabs, FC_SLAB, 0, 20480, fs, dwfc),
                 seg(fc_slabs, FC_SLAB, 20480, 10, fs, dbfc)},
                s);
}

void cn_conv2_bwd(const void* a1, const void* r2, const void* dr2, const void* packed, void* da1, int B,
                  float* slabs, float* dw2, float* db2, hipStream_t s) {
  const int ws = conv2_wslices(B);
  const int nd = da1 ? clampi(B, 1, num_cus()) : 0;
  conv2_bwd_kernel<<<nd + ws, 512, 0, s>>>(static_cast<const bf16*>(a1), static_cast<const bf16*>(r2),
                                           static_cast<const bf16*>(dr2), static_cast<const bf16*>(packed),
                                           static_cast<bf16*>(da1), B, slabs, ws, nd);
  launch_reduce({seg(slabs, C2_WSLAB, 0, 288 * 64, ws, dw2, 1, 32, 64), seg(slabs, C2_WSLAB, 288 * 64, 64, ws, db2)},
                s);
}

void cn_conv1_wgrad(const void* x, bool u8, const void* da1, const uint8_t* idx1, const void* a1, int B,
                    float mean, float inv_std, float in_scale, float* slabs, float* dw1, float* db1,
                    hipStream_t s) {
  const int ws = conv1_wslices(B);
  if (u8)
    conv1_wgrad_kernel<true><<<ws, 256, 0, s>>>(x, static_cast<const bf16*>(da1), idx1,
                                                static_cast<const bf16*>(a1), B, mean, inv_std, in_scale,
                                                slabs, ws);
  else
    conv1_wgrad_kernel<false><<<ws, 256, 0, s>>>(x, static_cast<const bf16*>(da1), idx1,
                                                 static_cast<const bf16*>(a1), B, mean, inv_std, in_scale,
                                                 slabs, ws);
  launch_reduce({seg(slabs, C1_WSLAB, 0, 800, ws, dw1), seg(slabs, C1_WSLAB, 800, 32, ws, db1)}, s);
}

}  // namespace kern
}  // namespace ringdp
