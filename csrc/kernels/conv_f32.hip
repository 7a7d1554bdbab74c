// fp32 NCHW convolution / linear / max-pool kernels: the MNIST ConvNet at the reference's
// precision (ref/launch_dist.py:50-59 trains in fp32).
//
// Every conv product (forward, data gradient, weight gradient; fc1 is a 1x1 conv over a 1x1
// image) is one implicit GEMM on the exact-f32 matrix cores (v_mfma_f32_16x16x4_f32, f32 in /
// f32 accumulate - the same arithmetic as an fmaf chain, so results track ATen fp32 to
// reduction-order rounding).  Operands are gathered straight from the NCHW tensors by small
// loader functors (im2col never materialised) into a 64x64x16 LDS tile; 4 waves each own a 32x32
// quadrant = 2x2 MFMA blocks.  The next k-tile is fetched into registers while the current one
// is multiplied.  Weight gradients reduce over B*OH*OW, so they run split-K into per-slice slabs
// that a fixed-order reduction sums (deterministic).  Max-pool forward fuses the ReLU and stores
// a 1-byte argmax code; its backward is a gather (each input position sums the windows whose code
// points at it), so the overlapping 2x2/s1 pool needs no atomics.
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "kernels.h"

namespace ringdp {
namespace kern {
namespace {

using dev::f32x4;

constexpr int BM = 64, BN = 64, BK = 16, TPB = 256;
constexpr int LDA = BM + 4, LDB = BN + 4;

// ---------------------------------------------------------------- loaders / epilogues
// GEMM C[M][N] = sum_k A(m, k) * B(k, n).  kContig tells the tile loader which index is
// contiguous in memory for that operand (so consecutive lanes walk it).

struct FwdA {  // A(m = (b, oy, ox), k = (c, ky, kx)) = x[b, c, oy + ky - pad, ox + kx - pad]
  static constexpr bool kContigM = true;
  const float* x;
  const unsigned char* xu8;
  float mean, inv_std;
  int C, H, W, R, pad, OH, OW, K;
  __device__ float operator()(int64_t m, int k) const {
    if (k >= K) return 0.f;
    const int ohw = OH * OW;
    const int64_t b = m / ohw;
    const int r = static_cast<int>(m - b * ohw);
    const int oy = r / OW, ox = r - (r / OW) * OW;
    const int rr = R * R;
    const int c = k / rr, t = k - c * rr;
    const int iy = oy + t / R - pad, ix = ox + t % R - pad;
    if (iy < 0 || iy >= H || ix < 0 || ix >= W) return 0.f;  // zero padding after Normalize
    const int64_t off = ((b * C + c) * H + iy) * W + ix;
    if (xu8) return (static_cast<float>(xu8[off]) * (1.0f / 255.0f) - mean) * inv_std;
    return x[off];
  }
};

struct WeightB {  // B(k = (c, ky, kx), n) = w[n][c][ky][kx]
  static constexpr bool kContigM = false;  // contiguous along k
  const float* w;
  int K;  // C*R*R
  __device__ float operator()(int k, int n) const { return k < K ? w[static_cast<int64_t>(n) * K + k] : 0.f; }
};

struct DgradA {  // A(m = (b, iy, ix), k = (n, ky, kx)) = dz[b, n, iy + pad - ky, ix + pad - kx]
  static constexpr bool kContigM = true;
  const float* dz;
  int Kout, H, W, R, pad, OH, OW, K;
  __device__ float operator()(int64_t m, int k) const {
    if (k >= K) return 0.f;
    const int hw = H * W;
    const int64_t b = m / hw;
    const int r = static_cast<int>(m - b * hw);
    const int iy = r / W, ix = r - (r / W) * W;
    const int rr = R * R;
    const int n = k / rr, t = k - n * rr;
    const int oy = iy + pad - t / R, ox = ix + pad - t % R;
    if (oy < 0 || oy >= OH || ox < 0 || ox >= OW) return 0.f;
    return dz[((b * Kout + n) * OH + oy) * OW + ox];
  }
};

struct DgradB {  // B(k = (n, ky, kx), c) = w[n][c][ky][kx]
  static constexpr bool kContigM = false;
  const float* w;
  int C, R, K;
  __device__ float operator()(int k, int c) const {
    if (k >= K) return 0.f;
    const int rr = R * R;
    const int n = k / rr, t = k - n * rr;
    return w[(static_cast<int64_t>(n) * C + c) * rr + t];
  }
};

struct WgradA {  // A(m = n, k = (b, oy, ox)) = dz[b, n, oy, ox]     (k runs over the batch)
  static constexpr bool kContigM = false;
  const float* dz;
  int Kout, OH, OW;
  int64_t K;
  __device__ float operator()(int n, int64_t k) const {
    if (k >= K) return 0.f;
    const int ohw = OH * OW;
    const int64_t b = k / ohw;
    const int r = static_cast<int>(k - b * ohw);
    return dz[(b * Kout + n) * ohw + r];
  }
};

struct WgradB {  // B(k = (b, oy, ox), j = (c, ky, kx)) = x[b, c, oy + ky - pad, ox + kx - pad];
                 // column j == Nw is all ones: the bias gradient comes out as one more GEMM column
  static constexpr bool kContigM = false;
  const float* x;
  const unsigned char* xu8;
  float mean, inv_std;
  int C, H, W, R, pad, OH, OW, Nw;
  int64_t K;
  __device__ float operator()(int64_t k, int j) const {
    if (k >= K) return 0.f;
    if (j == Nw) return 1.f;
    const int ohw = OH * OW;
    const int64_t b = k / ohw;
    const int r = static_cast<int>(k - b * ohw);
    const int oy = r / OW, ox = r - (r / OW) * OW;
    const int rr = R * R;
    const int c = j / rr, t = j - c * rr;
    const int iy = oy + t / R - pad, ix = ox + t % R - pad;
    if (iy < 0 || iy >= H || ix < 0 || ix >= W) return 0.f;
    const int64_t off = ((b * C + c) * H + iy) * W + ix;
    if (xu8) return (static_cast<float>(xu8[off]) * (1.0f / 255.0f) - mean) * inv_std;
    return x[off];
  }
};

struct NCHWOut {  // C[m = (b, y, x)][n] (+ bias[n]) -> out[b, n, y, x]
  float* out;
  const float* bias;
  int N, HW;
  __device__ void operator()(int64_t m, int n, float v) const {
    const int64_t b = m / HW;
    const int r = static_cast<int>(m - b * HW);
    out[(b * N + n) * HW + r] = v + (bias ? bias[n] : 0.f);
  }
};

struct SlabOut {  // split-K slice: slab[z][m][n]
  float* slab;
  int N;
  int64_t MN;
  __device__ void operator()(int64_t m, int n, float v, int z) const {
    slab[z * MN + m * N + n] = v;
  }
};

// ---------------------------------------------------------------- the GEMM core
// grid: x = m tiles (can be ~10^6 for a conv over a large batch), y = n tiles, z = k slices
// (each slice covers k_per_slice of K).
template <class LA, class LB, class Epi, bool kSplit>
__global__ __launch_bounds__(TPB) void gemm_f32_kernel(int64_t M, int N, int64_t K, int64_t k_per_slice,
                                                       LA la, LB lb, Epi epi) {
  __shared__ float As[BK][LDA];
  __shared__ float Bs[BK][LDB];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int64_t m0 = static_cast<int64_t>(blockIdx.x) * BM;
  const int n0 = blockIdx.y * BN;
  const int64_t kbeg = static_cast<int64_t>(blockIdx.z) * k_per_slice;
  const int64_t kend = kbeg + k_per_slice < K ? kbeg + k_per_slice : K;

  // tile-load assignment: 4 elements per thread per operand
  float ra[4], rb[4];
  auto fetch = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + i * TPB;  // 0..1023
      int mi, ki;
      if (LA::kContigM) { mi = e % BM; ki = e / BM; } else { ki = e % BK; mi = e / BK; }
      const int64_t m = m0 + mi;
      const int64_t k = k0 + ki;
      ra[i] = (m < M && k < kend) ? la(m, k) : 0.f;
      int ni, kj;
      if (LB::kContigM) { ni = e % BN; kj = e / BN; } else { kj = e % BK; ni = e / BK; }
      const int n = n0 + ni;
      const int64_t kb = k0 + kj;
      rb[i] = (n < N && kb < kend) ? lb(kb, n) : 0.f;
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + i * TPB;
      if (LA::kContigM) As[e / BM][e % BM] = ra[i]; else As[e % BK][e / BK] = ra[i];
      if (LB::kContigM) Bs[e / BN][e % BN] = rb[i]; else Bs[e % BK][e / BK] = rb[i];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = dev::zero_f32x4();

  const int lr = lane & 15, lk = lane >> 4;
  if (kbeg < kend) fetch(kbeg);
  for (int64_t k0 = kbeg; k0 < kend; k0 += BK) {
    __syncthreads();
    stash();
    __syncthreads();
    if (k0 + BK < kend) fetch(k0 + BK);  // next tile in flight during the MFMAs
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      const float a0 = As[kk + lk][wm + lr], a1 = As[kk + lk][wm + 16 + lr];
      const float b0 = Bs[kk + lk][wn + lr], b1 = Bs[kk + lk][wn + 16 + lr];
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
    }
  }
  // D: lane l, reg r -> row 4*(l >> 4) + r, col l & 15 of each 16x16 block
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm + i * 16 + 4 * lk + r;
        const int n = n0 + wn + j * 16 + lr;
        if (m < M && n < N) {
          if constexpr (kSplit) epi(m, n, acc[i][j][r], static_cast<int>(blockIdx.z));
          else epi(m, n, acc[i][j][r]);
        }
      }
}

template <class LA, class LB, class Epi>
void launch_gemm(int64_t M, int N, int64_t K, const LA& la, const LB& lb, const Epi& epi, hipStream_t s) {
  dim3 grid(static_cast<unsigned>((M + BM - 1) / BM), (N + BN - 1) / BN, 1);
  hipLaunchKernelGGL((gemm_f32_kernel<LA, LB, Epi, false>), grid, dim3(TPB), 0, s, M, N, K, K, la, lb, epi);
}

template <class LA, class LB>
void launch_gemm_splitk(int64_t M, int N, int64_t K, int slices, const LA& la, const LB& lb, float* slab,
                        hipStream_t s) {
  int64_t per = (K + slices - 1) / slices;
  per = (per + BK - 1) / BK * BK;
  dim3 grid(static_cast<unsigned>((M + BM - 1) / BM), (N + BN - 1) / BN, slices);
  SlabOut epi{slab, N, M * N};
  hipLaunchKernelGGL((gemm_f32_kernel<LA, LB, SlabOut, true>), grid, dim3(TPB), 0, s, M, N, K, per, la, lb, epi);
}

// ---------------------------------------------------------------- pooling (+ReLU)
// a[b,c,py,px] = relu(max over the k x k window at (py*st, px*st)); code = argmax offset
// (first maximum in row-major order, as max_pool2d); code 255 where the result is 0 (no gradient).
__global__ __launch_bounds__(256) void pool_relu_fwd_kernel(const float* __restrict__ z, float* __restrict__ a,
                                                            unsigned char* __restrict__ code, int64_t BC,
                                                            int H, int W, int PH, int PW, int k, int st) {
  const int64_t total = BC * PH * PW;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t bc = i / (PH * PW);
    const int r = static_cast<int>(i - bc * PH * PW);
    const int py = r / PW, px = r % PW;
    const float* zp = z + bc * H * W + (py * st) * W + px * st;
    float best = zp[0];
    int arg = 0;
    for (int dy = 0; dy < k; ++dy)
      for (int dx = 0; dx < k; ++dx) {
        const float v = zp[dy * W + dx];
        if (v > best) { best = v; arg = dy * k + dx; }
      }
    const bool live = best > 0.f;
    a[i] = live ? best : 0.f;
    code[i] = live ? static_cast<unsigned char>(arg) : 255;
  }
}

// dz[b,c,y,x] = sum over windows (py,px) covering (y,x) whose code points at (y,x) of da[b,c,py,px]
__global__ __launch_bounds__(256) void pool_relu_bwd_kernel(const float* __restrict__ da,
                                                            const unsigned char* __restrict__ code,
                                                            float* __restrict__ dz, int64_t BC, int H, int W,
                                                            int PH, int PW, int k, int st) {
  const int64_t total = BC * H * W;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t bc = i / (H * W);
    const int r = static_cast<int>(i - bc * H * W);
    const int y = r / W, x = r % W;
    float g = 0.f;
    for (int dy = 0; dy < k; ++dy) {
      const int ty = y - dy;
      if (ty < 0 || ty % st) continue;
      const int py = ty / st;
      if (py >= PH) continue;
      for (int dx = 0; dx < k; ++dx) {
        const int tx = x - dx;
        if (tx < 0 || tx % st) continue;
        const int px = tx / st;
        if (px >= PW) continue;
        const int64_t o = bc * PH * PW + py * PW + px;
        if (code[o] == dy * k + dx) g += da[o];
      }
    }
    dz[i] = g;
  }
}

// Fixed-order sum of the split-K slabs [slices][Kout][Nw + has_bias] into dw [Kout][Nw] and db [Kout].
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ slab, int slices, int Kout,
                                                           int Nw, int ncol, float* __restrict__ dw,
                                                           float* __restrict__ db) {
  const int64_t total = static_cast<int64_t>(Kout) * ncol;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    float acc = slab[i];
    for (int z = 1; z < slices; ++z) acc += slab[z * total + i];
    const int m = static_cast<int>(i / ncol), n = static_cast<int>(i - static_cast<int64_t>(m) * ncol);
    if (n < Nw) dw[static_cast<int64_t>(m) * Nw + n] = acc;
    else db[m] = acc;
  }
}

int grid_1d(int64_t n) {
  const int64_t g = (n + 255) / 256;
  return static_cast<int>(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}

int wgrad_slices(int64_t M, int N, int64_t K) {
  // enough slices to put >= ~1024 workgroups on the 256 CUs, each slice >= 512 deep
  const int64_t tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int64_t s = (1024 + tiles - 1) / tiles;
  const int64_t cap = (K + 511) / 512;
  if (s > cap) s = cap;
  return static_cast<int>(s < 1 ? 1 : (s > 512 ? 512 : s));
}

}  // namespace

int conv_f32_wgrad_slices(const ConvF32Geom& g) {
  return wgrad_slices(g.Kout, g.C * g.R * g.R + 1, g.B * static_cast<int64_t>(g.OH) * g.OW);
}

void conv_f32_fwd(const ConvF32Geom& g, const float* x, const unsigned char* xu8, float mean, float inv_std,
                  const float* w, const float* bias, float* z, hipStream_t s) {
  const int K = g.C * g.R * g.R;
  FwdA la{x, xu8, mean, inv_std, g.C, g.H, g.W, g.R, g.pad, g.OH, g.OW, K};
  WeightB lb{w, K};
  NCHWOut epi{z, bias, g.Kout, g.OH * g.OW};
  launch_gemm(g.B * static_cast<int64_t>(g.OH) * g.OW, g.Kout, K, la, lb, epi, s);
}

void conv_f32_dgrad(const ConvF32Geom& g, const float* dz, const float* w, float* dx, hipStream_t s) {
  const int K = g.Kout * g.R * g.R;
  DgradA la{dz, g.Kout, g.H, g.W, g.R, g.pad, g.OH, g.OW, K};
  DgradB lb{w, g.C, g.R, K};
  NCHWOut epi{dx, nullptr, g.C, g.H * g.W};
  launch_gemm(g.B * static_cast<int64_t>(g.H) * g.W, g.C, K, la, lb, epi, s);
}

void conv_f32_wgrad(const ConvF32Geom& g, const float* dz, const float* x, const unsigned char* xu8, float mean,
                    float inv_std, float* slab, int slices, float* dw, float* db, hipStream_t s) {
  const int64_t K = g.B * static_cast<int64_t>(g.OH) * g.OW;
  const int Nw = g.C * g.R * g.R;
  const int ncol = Nw + (db ? 1 : 0);
  WgradA la{dz, g.Kout, g.OH, g.OW, K};
  WgradB lb{x, xu8, mean, inv_std, g.C, g.H, g.W, g.R, g.pad, g.OH, g.OW, Nw, K};
  launch_gemm_splitk(g.Kout, ncol, K, slices, la, lb, slab, s);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(grid_1d(static_cast<int64_t>(g.Kout) * ncol)), dim3(256), 0, s,
                     slab, slices, g.Kout, Nw, ncol, dw, db);
}

void pool_relu_f32_fwd(const float* z, float* a, unsigned char* code, int64_t BC, int H, int W, int k, int st,
                       hipStream_t s) {
  const int PH = (H - k) / st + 1, PW = (W - k) / st + 1;
  hipLaunchKernelGGL(pool_relu_fwd_kernel, dim3(grid_1d(BC * PH * PW)), dim3(256), 0, s, z, a, code, BC, H, W,
                     PH, PW, k, st);
}

void pool_relu_f32_bwd(const float* da, const unsigned char* code, float* dz, int64_t BC, int H, int W, int k,
                       int st, hipStream_t s) {
  const int PH = (H - k) / st + 1, PW = (W - k) / st + 1;
  hipLaunchKernelGGL(pool_relu_bwd_kernel, dim3(grid_1d(BC * H * W)), dim3(256), 0, s, da, code, dz, BC, H, W,
                     PH, PW, k, st);
}

}  // namespace kern
}  // namespace ringdp
