// The ConvNet's first layer at fp32 (ref/launch_dist.py:35-41: conv1 1->32, 5x5, pad 1 on 28x28, ReLU,
// 2x2/s2 max-pool), as two dedicated kernels instead of implicit GEMMs (csrc/kernels/conv_f32.hip).
//
// With one input channel the implicit GEMM's operand gathers cost far more than its 25-deep
// products (PMC: the generic kernel ran at ~22 TF/s, the pool1 passes another 3 ms per step at
// B = 65536).  Here each wave owns one image at a time, normalised into a zero-bordered 30x30 LDS
// copy, so every im2col element is one LDS read at a lane-constant tap offset:
//   * forward: D[n][m] = w1[n][k] x img[m + tap k] on v_mfma_f32_16x16x4_f32 (7 k-steps of 4 taps,
//     weights held in registers), pixels in window-major order so the 4 pixels of a pooling window
//     are 4 adjacent lanes; bias + ReLU + max-pool + 1-byte argmax code in the epilogue; the
//     26x26x32 pre-activation is never written;
//   * weight gradient: D[n][tap] = sum_p dz1[n][p] x img[p + tap] over the wave's images, with
//     dz1 decoded on the fly from the pooled gradient and the code (the pool1 backward pass is
//     gone), column 25 of the B operand = 1 so the bias gradient is the same MFMA; per-workgroup
//     partials in a fixed order into a slab that the conv_f32 slab reduction sums.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "device_common.h"
#include "kernels.h"

namespace ringdp {
namespace kern {
namespace {

using dev::f32x4;

constexpr int IMG = 28, PADW = 30, OUTW = 26, PW1 = 13, NWIN = PW1 * PW1, C1 = 32, TAPS = 25;
constexpr int LDS_IMG = PADW * PADW + 4;
constexpr int WAVES = 4;

// Normalised image b into the wave's LDS copy (interior only: the zero border is written once).
// All 13 loads of a lane are issued before the first store: one memory round trip per image.
template <bool U8>
__device__ __forceinline__ void stage_image(float* im, const void* x, int b, float mean, float inv_std, int lane) {
  constexpr int PER = (IMG * IMG + 63) / 64;
  float v[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int i = min(lane + 64 * q, IMG * IMG - 1);
    if constexpr (U8) v[q] = static_cast<float>(static_cast<const unsigned char*>(x)[b * IMG * IMG + i]);
    else v[q] = static_cast<const float*>(x)[b * IMG * IMG + i];
  }
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int i = lane + 64 * q;
    if (i < IMG * IMG) {
      const int y = i / IMG, xx = i - y * IMG;
      im[(y + 1) * PADW + xx + 1] = U8 ? (v[q] * (1.0f / 255.0f) - mean) * inv_std : v[q];
    }
  }
}

// lane exchange inside a quad (DPP, full-rate VALU, no LDS round trip): xor 1 / xor 2
template <int X>
__device__ __forceinline__ int quad_xor(int v) {
  return __builtin_amdgcn_update_dpp(0, v, X == 1 ? 0xB1 : 0x4E, 0xF, 0xF, false);
}
template <int X>
__device__ __forceinline__ float quad_xor(float v) {
  return __builtin_bit_cast(float, quad_xor<X>(__builtin_bit_cast(int, v)));
}

// padded-image offset of window-major output pixel m (m < 676): window m >> 2 = (py, px), tap-in-
// window m & 3 = (wy, wx)
__device__ __forceinline__ int pix_base(int m) {
  const int w = m >> 2, t = m & 3, py = w / PW1, px = w - py * PW1;
  return (2 * py + (t >> 1)) * PADW + 2 * px + (t & 1);
}

// Small batches: one image per workgroup (its 4 waves split the image) instead of one per wave, so a
// B=100 step runs 100 workgroups x 4 waves, not 25 x 4 waves each walking a whole image (71 us).
__host__ __device__ inline bool split_mode(int64_t B) { return B < 2048; }

template <bool U8>
__global__ __launch_bounds__(256) void conv1_pool_f32_kernel(const void* __restrict__ x, const float* __restrict__ w1,
                                                             const float* __restrict__ b1, float* __restrict__ a1,
                                                             unsigned char* __restrict__ code1, int B, float mean,
                                                             float inv_std) {
  __shared__ float img[WAVES][LDS_IMG];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, lr = lane & 15, lk = lane >> 4;
  float* im = img[wave];
  for (int i = lane; i < LDS_IMG; i += 64) im[i] = 0.f;
  // A operand (row = pixel m): img[pix(m) + tap(4 s + lk)]; B operand (col = n): w1[16 j + lr][4 s + lk].
  // D[m][n] then leaves the 4 pixels of a pooling window (window-major m) in one lane's 4 accumulator
  // registers: the pool is a register reduction, no cross-lane exchange (the DPP quad form spent ~70 VALU
  // per lane and m-tile)
  float wreg[7][2];
  int tapoff[7];
#pragma unroll
  for (int s = 0; s < 7; ++s) {
    const int k = 4 * s + lk;
    tapoff[s] = k < TAPS ? (k / 5) * PADW + k % 5 : 0;  // weight 0 past tap 24
#pragma unroll
    for (int j = 0; j < 2; ++j) wreg[s][j] = k < TAPS ? w1[(16 * j + lr) * TAPS + k] : 0.f;
  }
  const float bias[2] = {b1[lr], b1[16 + lr]};

  // small batches (split_mode): the 4 waves share one image per round, each taking every 4th pixel group
  const bool split = split_mode(B);
  const int ipr = split ? 1 : WAVES;  // images per workgroup round
  const int rounds = (B + ipr * gridDim.x - 1) / (ipr * gridDim.x);
  for (int round = 0; round < rounds; ++round) {
    const int b = split ? round * gridDim.x + blockIdx.x : (round * gridDim.x + blockIdx.x) * WAVES + wave;
    __syncthreads();  // the previous image's reads are done (uniform trip count: every wave gets here)
    if (b < B) stage_image<U8>(im, x, b, mean, inv_std, lane);
    __syncthreads();
    if (b >= B) continue;
    float* ab = a1 + static_cast<int64_t>(b) * C1 * NWIN;
    unsigned char* cb = code1 + static_cast<int64_t>(b) * C1 * NWIN;
    // split mode with gridDim.y > 1 parts: workgroup (b, part) takes pixel groups part * WAVES + wave, step
    // WAVES * parts (every part stages the whole image: 784 B)
    const int gstep = split ? WAVES * static_cast<int>(gridDim.y) : 1;
    for (int g = split ? static_cast<int>(blockIdx.y) * WAVES + wave : 0; g < (4 * NWIN + 15) / 16; g += gstep) {
      const int m = 16 * g + lr;
      const int base = m < 4 * NWIN ? pix_base(m) : 0;
      f32x4 acc[2] = {{bias[0], bias[0], bias[0], bias[0]}, {bias[1], bias[1], bias[1], bias[1]}};
#pragma unroll
      for (int s = 0; s < 7; ++s) {
        const float p = im[base + tapoff[s]];
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(p, wreg[s][0], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(p, wreg[s][1], acc[1], 0, 0, 0);
      }
      // lane holds D[m = 16 g + 4 lk + r][n = 16 j + lr]: window 4 g + lk, its tap r
      const int win = 4 * g + lk;
      if (win < NWIN) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const f32x4 v = acc[j];
          const float best = fmaxf(fmaxf(fmaxf(v[0], v[1]), v[2]), v[3]);  // v_max3 + v_max
          // first maximum in window order wins, as max_pool2d
          const int bt = v[0] == best ? 0 : v[1] == best ? 1 : v[2] == best ? 2 : 3;
          const bool live = best > 0.f;
          const int n = 16 * j + lr;
          ab[n * NWIN + win] = live ? best : 0.f;
          cb[n * NWIN + win] = live ? static_cast<unsigned char>(bt) : 255;
        }
      }
    }
  }
}

// slab[blockIdx.x][n][c], c < 25: dW1 partial, c = 25: db1 partial
template <bool U8>
__global__ __launch_bounds__(256) void conv1_wgrad_f32_kernel(const void* __restrict__ x, const float* __restrict__ da1,
                                                              const unsigned char* __restrict__ code1,
                                                              float* __restrict__ slab, int B, float mean,
                                                              float inv_std) {
  __shared__ float img[WAVES][LDS_IMG];
  __shared__ f32x4 red[WAVES - 1][4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, lr = lane & 15, lk = lane >> 4;
  float* im = img[wave];
  for (int i = lane; i < LDS_IMG; i += 64) im[i] = 0.f;
  // B operand (col = tap column c = 16 jt + lr): img[pixel + tap offset], column 25 = 1, past it 0
  int tapoff[2];
  float tapmul[2], tapone[2];
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    const int c = 16 * jt + lr;
    tapoff[jt] = c < TAPS ? (c / 5) * PADW + c % 5 : 0;
    tapmul[jt] = c < TAPS ? 1.f : 0.f;
    tapone[jt] = c == TAPS ? 1.f : 0.f;
  }
  // k index = pixel p = 4 s + lk (window s, tap-in-window lk)
  const int woff = (lk >> 1) * PADW + (lk & 1);
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = dev::zero_f32x4();

  const bool split = split_mode(B);
  const int ipr = split ? 1 : WAVES;
  const int rounds = (B + ipr * gridDim.x - 1) / (ipr * gridDim.x);
  for (int round = 0; round < rounds; ++round) {
    const int b = split ? round * gridDim.x + blockIdx.x : (round * gridDim.x + blockIdx.x) * WAVES + wave;
    __syncthreads();
    if (b < B) stage_image<U8>(im, x, b, mean, inv_std, lane);
    __syncthreads();
    if (b >= B) continue;
    const float* db = da1 + static_cast<int64_t>(b) * C1 * NWIN;
    const unsigned char* cbp = code1 + static_cast<int64_t>(b) * C1 * NWIN;
    // one pooled row (13 windows) at a time: its 52 gradient / code loads are issued together
    // split mode with gridDim.y parts: workgroup (b, part) takes pooled rows part * WAVES + wave, step WAVES * parts
    const int rstep = split ? WAVES * static_cast<int>(gridDim.y) : 1;
    for (int py = split ? static_cast<int>(blockIdx.y) * WAVES + wave : 0; py < PW1; py += rstep) {
      float dv[PW1][2];
      int cv[PW1][2];
#pragma unroll
      for (int px = 0; px < PW1; ++px)
#pragma unroll
        for (int jn = 0; jn < 2; ++jn) {
          const int o = (16 * jn + lr) * NWIN + py * PW1 + px;
          cv[px][jn] = cbp[o];
          dv[px][jn] = db[o];
        }
#pragma unroll
      for (int px = 0; px < PW1; ++px) {
        // A operand (row = n = 16 jn + lr): dz1[n][p] = da1[n][window] where the code points at tap lk
        float av[2];
#pragma unroll
        for (int jn = 0; jn < 2; ++jn) av[jn] = cv[px][jn] == lk ? dv[px][jn] : 0.f;
        const int pb = 2 * py * PADW + 2 * px + woff;
        float bv[2];
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) bv[jt] = im[pb + tapoff[jt]] * tapmul[jt] + tapone[jt];
#pragma unroll
        for (int jn = 0; jn < 2; ++jn)
#pragma unroll
          for (int jt = 0; jt < 2; ++jt)
            acc[jn][jt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[jn], bv[jt], acc[jn][jt], 0, 0, 0);
      }
    }
  }
  // fixed-order sum over the 4 waves, then D[n][c]: lane holds n = 16 jn + 4 lk + r, c = 16 jt + lr
  if (wave > 0)
#pragma unroll
    for (int q = 0; q < 4; ++q) red[wave - 1][q][lane] = acc[q >> 1][q & 1];
  __syncthreads();
  if (wave > 0) return;
#pragma unroll
  for (int w = 0; w < WAVES - 1; ++w)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q >> 1][q & 1] += red[w][q][lane];
  float* out = slab + (static_cast<int64_t>(blockIdx.y) * gridDim.x + blockIdx.x) * C1 * (TAPS + 1);
#pragma unroll
  for (int jn = 0; jn < 2; ++jn)
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 16 * jn + 4 * lk + r, c = 16 * jt + lr;
        if (c <= TAPS) out[n * (TAPS + 1) + c] = acc[jn][jt][r];
      }
}

int conv1_blocks(int64_t B) {
  // 4 images per workgroup round (1 in split mode); ~4 workgroups per CU, at least a few rounds each
  const int64_t want = split_mode(B) ? B : (B + WAVES - 1) / WAVES;
  return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(want, 1024)));
}

}  // namespace

// workgroups per image in split mode (RINGDP_F32_CONV1_PARTS / _WPARTS override the forward's / the weight
// gradient's): B=100 -> 4 (400 workgroups; forward 22.5 -> 11.9 us)
static int conv1_parts(int64_t B, const char* env) {
  if (!split_mode(B)) return 1;
  if (const char* e = std::getenv(env)) {
    const int v = std::atoi(e);
    if (v > 0) return std::min(v, 11);
  }
  return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(4, 512 / std::max<int64_t>(B, 1))));
}
static int conv1_wparts(int64_t B) { return std::min(conv1_parts(B, "RINGDP_F32_CONV1_WPARTS"), 4); }

// weight-gradient partials (slab rows): one per workgroup, part-major
int conv1_f32_wgrad_blocks(int64_t B) { return conv1_blocks(B) * conv1_wparts(B); }

void conv1_pool_f32_fwd(const float* x, const unsigned char* xu8, int64_t B, float mean, float inv_std,
                        const float* w1, const float* b1, float* a1, unsigned char* code1, hipStream_t s) {
  const int nb = conv1_blocks(B);
  const dim3 grid(nb, conv1_parts(B, "RINGDP_F32_CONV1_PARTS"));
  if (xu8)
    hipLaunchKernelGGL(conv1_pool_f32_kernel<true>, grid, dim3(256), 0, s, xu8, w1, b1, a1, code1,
                       static_cast<int>(B), mean, inv_std);
  else
    hipLaunchKernelGGL(conv1_pool_f32_kernel<false>, grid, dim3(256), 0, s, x, w1, b1, a1, code1,
                       static_cast<int>(B), mean, inv_std);
}

void conv1_wgrad_f32(const float* x, const unsigned char* xu8, int64_t B, float mean, float inv_std, const float* da1,
                     const unsigned char* code1, float* slab, hipStream_t s) {
  const int nb = conv1_blocks(B);
  const dim3 grid(nb, conv1_wparts(B));  // conv1_f32_wgrad_blocks(B) = nb * parts slab rows
  if (xu8)
    hipLaunchKernelGGL(conv1_wgrad_f32_kernel<true>, grid, dim3(256), 0, s, xu8, da1, code1, slab,
                       static_cast<int>(B), mean, inv_std);
  else
    hipLaunchKernelGGL(conv1_wgrad_f32_kernel<false>, grid, dim3(256), 0, s, x, da1, code1, slab,
                       static_cast<int>(B), mean, inv_std);
}

}  // namespace kern
}  // namespace ringdp
