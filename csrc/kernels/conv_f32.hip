// fp32 NCHW convolution / linear / max-pool kernels: the MNIST ConvNet at the reference's
// precision (ref/launch_dist.py:50-59 trains in fp32).
//
// Every conv product (forward, data gradient, weight gradient; fc1 is a 1x1 conv over a 1x1
// image) is one implicit GEMM on the exact-f32 matrix cores (v_mfma_f32_16x16x4_f32, f32 in /
// f32 accumulate - the same arithmetic as an fmaf chain, so results track ATen fp32 to
// reduction-order rounding).  Operands are gathered straight from the NCHW tensors (im2col never
// materialised) into double-buffered LDS k-tiles of 16; 4 waves each own a 32x32 block of the
// output (2x2 MFMA tiles), the workgroup tile is 64x64, 128x32 or 32x128 by the GEMM's shape.
//
// The f32 MFMA issues one 16x16x4 product per 32 cycles, so the operand gathers have to cost
// well under that per element.  The round-2 kernel spent ~10x the MFMA time in 64-bit divides in
// the loaders; here every index is 32-bit and the divides are gone from the k-loop:
//   * the thread-fixed index of an operand (its GEMM row for m-contiguous operands, its column
//     for k-contiguous ones) is decomposed once per tile;
//   * for m-contiguous operands the k decomposition (channel, ky, kx) -> (offset, dy, dx) is a
//     per-workgroup LDS table built at kernel start;
//   * for k-contiguous operands (the weight gradients, k = batch x pixel) every lane of a row of
//     the tile shares one k per k-tile, decomposed with multiply-high divisions (FastDiv).
// MFMAs take the B fragment as their row operand, so a lane's results run along m - the NCHW
// pixel index - and each store instruction writes 64-B runs of the output plane.
// Tensors whose element count reaches 2^31 are processed in batch chunks by the host launchers.
// Weight gradients reduce over B*OH*OW, so they run split-K into per-slice slabs that a
// fixed-order reduction sums (deterministic).  Max-pool forward fuses the ReLU and stores a 1-byte
// argmax code; its backward is a gather (each input position sums the windows whose code points
// at it), so the overlapping 2x2/s1 pool needs no atomics.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "device_common.h"
#include "kernels.h"

namespace ringdp {
namespace kern {
namespace {

using dev::f32x4;

constexpr int BK = 16, TPB = 256;

// n / d for 0 <= n < 2^31 without a divide: q = (mulhi(n, mul) + n) >> shift.
struct FastDiv {
  uint32_t d, mul, shift;
};
FastDiv make_fdiv(uint32_t d) {
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  const uint64_t m = ((1ull << 32) * ((1ull << s) - d)) / d + 1;
  return FastDiv{d, static_cast<uint32_t>(m), s};
}
__device__ __forceinline__ int fdiv(int n, const FastDiv& f) {
  return static_cast<int>((__umulhi(static_cast<uint32_t>(n), f.mul) + static_cast<uint32_t>(n)) >> f.shift);
}

// (dy, dx) packed as two int16 halves; "never in bounds" marker for padding rows / columns
__device__ __forceinline__ int pack_dyx(int dy, int dx) { return (dy & 0xffff) | (dx << 16); }
__device__ __forceinline__ int unpack_dy(int v) { return static_cast<int>(static_cast<short>(v & 0xffff)); }
__device__ __forceinline__ int unpack_dx(int v) { return v >> 16; }
constexpr int kOut = -0x2000;  // added to a coordinate <= 1024 it can never land in [0, H)

__device__ __forceinline__ float ld_x(const float* x, const unsigned char* xu8, float mean, float inv_std, int off) {
  if (xu8) return (static_cast<float>(xu8[off]) * (1.0f / 255.0f) - mean) * inv_std;
  return x[off];
}

// ---------------------------------------------------------------- operand loaders
// GEMM C[M][N] = sum_k A(m, k) * B(k, n).  kMC: the operand's thread-fixed index is contiguous in
// memory (lanes walk m), with a per-workgroup k table; otherwise lanes walk k.

struct FwdA {  // A(m = (b, oy, ox), k = (c, ky, kx)) = x[b, c, oy + ky - pad, ox + kx - pad]
  static constexpr bool kMC = true;
  const float* x;
  const unsigned char* xu8;
  float mean, inv_std;
  int C, H, W, R, pad, OW, K, M;
  FastDiv ohw, ow;
  struct O {
    int base, y, x;
  };
  __device__ O outer(int m) const {
    if (m >= M) return O{0, kOut, kOut};
    const int b = fdiv(m, ohw), r = m - b * static_cast<int>(ohw.d);
    const int oy = fdiv(r, ow), ox = r - oy * OW;
    return O{b * C * H * W + (oy - pad) * W + (ox - pad), oy - pad, ox - pad};
  }
  __device__ int2 ktab(int k) const {  // (offset, dy|dx)
    if (k >= K) return int2{0, pack_dyx(kOut, kOut)};
    const int rr = R * R, c = k / rr, t = k - c * rr, ky = t / R, kx = t - ky * R;
    return int2{c * H * W + ky * W + kx, pack_dyx(ky, kx)};
  }
  __device__ float load(const O& o, int2 kt) const {
    const int iy = o.y + unpack_dy(kt.y), ix = o.x + unpack_dx(kt.y);
    if (static_cast<unsigned>(iy) >= static_cast<unsigned>(H) || static_cast<unsigned>(ix) >= static_cast<unsigned>(W))
      return 0.f;  // zero padding after Normalize
    return ld_x(x, xu8, mean, inv_std, o.base + kt.x);
  }
};

struct DgradA {  // A(m = (b, iy, ix), k = (n, ky, kx)) = dz[b, n, iy + pad - ky, ix + pad - kx]
  static constexpr bool kMC = true;
  const float* dz;
  int Kout, W, R, OH, OW, pad, K, M;
  FastDiv hw, w;
  struct O {
    int base, y, x;
  };
  __device__ O outer(int m) const {
    if (m >= M) return O{0, kOut, kOut};
    const int b = fdiv(m, hw), r = m - b * static_cast<int>(hw.d);
    const int iy = fdiv(r, w), ix = r - iy * W;
    return O{b * Kout * OH * OW + (iy + pad) * OW + (ix + pad), iy + pad, ix + pad};
  }
  __device__ int2 ktab(int k) const {
    if (k >= K) return int2{0, pack_dyx(kOut, kOut)};
    const int rr = R * R, n = k / rr, t = k - n * rr, ky = t / R, kx = t - ky * R;
    return int2{n * OH * OW - ky * OW - kx, pack_dyx(-ky, -kx)};
  }
  __device__ float load(const O& o, int2 kt) const {
    const int oy = o.y + unpack_dy(kt.y), ox = o.x + unpack_dx(kt.y);
    if (static_cast<unsigned>(oy) >= static_cast<unsigned>(OH) || static_cast<unsigned>(ox) >= static_cast<unsigned>(OW))
      return 0.f;
    return dz[o.base + kt.x];
  }
};

struct WeightB {  // B(k = (c, ky, kx), n) = w[n][c][ky][kx]; lanes walk k
  static constexpr bool kMC = false;
  const float* w;
  int K, N;
  typedef int O;
  typedef int KS;
  __device__ O outer(int n) const { return n < N ? n * K : -1; }
  __device__ KS kstate(int k, int kend) const { return k < kend ? k : -1; }
  __device__ float load(O o, KS k) const { return (o >= 0 && k >= 0) ? w[o + k] : 0.f; }
};

struct DgradB {  // B(k = (n, ky, kx), c) = w[n][c][ky][kx]; lanes walk k
  static constexpr bool kMC = false;
  const float* w;
  int C, rr, K;
  FastDiv frr;
  typedef int O;
  typedef int KS;
  __device__ O outer(int c) const { return c < C ? c * rr : -1; }
  __device__ KS kstate(int k, int kend) const {
    if (k >= kend) return -1;
    const int n = fdiv(k, frr);
    return n * C * rr + (k - n * rr);
  }
  __device__ float load(O o, KS k) const { return (o >= 0 && k >= 0) ? w[o + k] : 0.f; }
};

struct WgradA {  // A(m = n, k = (b, r)) = dz[b, n, r]     (k runs over batch x output pixels)
  static constexpr bool kMC = false;
  const float* dz;
  int Kout, ohwi;
  FastDiv ohw;
  typedef int O;
  typedef int KS;
  __device__ O outer(int n) const { return n < Kout ? n * ohwi : -1; }
  __device__ KS kstate(int k, int kend) const {
    if (k >= kend) return -1;
    const int b = fdiv(k, ohw);
    return b * Kout * ohwi + (k - b * ohwi);
  }
  __device__ float load(O o, KS k) const { return (o >= 0 && k >= 0) ? dz[o + k] : 0.f; }
};

struct WgradB {  // B(k = (b, oy, ox), j = (c, ky, kx)) = x[b, c, oy + ky - pad, ox + kx - pad];
                 // column j == Nw is all ones: the bias gradient comes out as one more GEMM column
  static constexpr bool kMC = false;
  const float* x;
  const unsigned char* xu8;
  float mean, inv_std;
  int C, H, W, R, pad, OW, Nw;
  FastDiv ohw, ow;
  struct O {
    int off, dyx, kind;  // kind 0: pixel, 1: ones (bias column), 2: zero (past the last column)
  };
  struct KS {
    int base, y, x;  // y = oy - pad, x = ox - pad; y = kOut when k is past the slice
  };
  __device__ O outer(int j) const {
    if (j > Nw) return O{0, 0, 2};
    if (j == Nw) return O{0, 0, 1};
    const int rr = R * R, c = j / rr, t = j - c * rr, ky = t / R, kx = t - ky * R;
    return O{c * H * W + ky * W + kx, pack_dyx(ky, kx), 0};
  }
  __device__ KS kstate(int k, int kend) const {
    if (k >= kend) return KS{0, kOut, kOut};
    const int b = fdiv(k, ohw), r = k - b * static_cast<int>(ohw.d);
    const int oy = fdiv(r, ow), ox = r - oy * OW;
    return KS{b * C * H * W + (oy - pad) * W + (ox - pad), oy - pad, ox - pad};
  }
  __device__ float load(const O& o, const KS& k) const {
    if (o.kind == 2) return 0.f;
    if (o.kind == 1) return k.y == kOut ? 0.f : 1.f;
    const int iy = k.y + unpack_dy(o.dyx), ix = k.x + unpack_dx(o.dyx);
    if (static_cast<unsigned>(iy) >= static_cast<unsigned>(H) || static_cast<unsigned>(ix) >= static_cast<unsigned>(W))
      return 0.f;
    return ld_x(x, xu8, mean, inv_std, k.base + o.off);
  }
};

// ---------------------------------------------------------------- epilogues
struct NCHWOut {  // C[m = (b, p)][n] (+ bias[n]) -> out[b, n, p]
  float* out;
  const float* bias;
  int N, M;
  FastDiv hw;
  __device__ int row(int m) const {  // offset of out[b, 0, p]
    const int b = fdiv(m, hw);
    return b * N * static_cast<int>(hw.d) + (m - b * static_cast<int>(hw.d));
  }
  __device__ void store(int rowoff, int n, float v) const {
    out[rowoff + n * static_cast<int>(hw.d)] = v + (bias ? bias[n] : 0.f);
  }
};

struct SlabOut {  // split-K slice z: slab[z][m][n]
  float* slab;
  int N, M;
  __device__ int row(int m) const { return static_cast<int>(blockIdx.z) * M * N + m * N; }
  __device__ void store(int rowoff, int n, float v) const { slab[rowoff + n] = v; }
};

// ---------------------------------------------------------------- the GEMM core
// grid: x = m tiles, y = n tiles, z = k slices (each covers k_per_slice of K).  WM x WN waves of
// 32x32; with WM * WN < 4 the remaining waves split each k-tile's MFMA steps between them and the
// partial accumulators are summed in a fixed wave order at the end (the 32x32 tile of the small
// conv1 weight gradient).  ktab_n > 0: the A operand's k table (K rounded up to 16) in dynamic LDS.
template <int WM, int WN, class LA, class LB, class Epi>
__global__ __launch_bounds__(TPB) void gemm_f32_kernel(int M, int N, int K, int k_per_slice, int ktab_n, LA la,
                                                       LB lb, Epi epi) {
  constexpr int BM = 32 * WM, BN = 32 * WN, KSPLIT = 4 / (WM * WN);
  static_assert(KSPLIT * WM * WN == 4 && BK / 4 >= KSPLIT, "4 waves");
  constexpr int LDA = BM + 16, LDB = BN + 16;  // row stride: 16 banks apart, conflict-free reads
  constexpr int EA = BM * BK / TPB, EB = BN * BK / TPB;
  __shared__ float As[2][BK][LDA];
  __shared__ float Bs[2][BK][LDB];
  extern __shared__ int2 ktab[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wk = wave / (WM * WN), wmn = wave % (WM * WN);
  const int wm = (wmn / WN) * 32, wn = (wmn % WN) * 32;
  const int m0 = static_cast<int>(blockIdx.x) * BM;
  const int n0 = static_cast<int>(blockIdx.y) * BN;
  const int kbeg = static_cast<int>(blockIdx.z) * k_per_slice;
  const int kend = min(kbeg + k_per_slice, K);

  if constexpr (LA::kMC) {
    for (int k = tid; k < ktab_n; k += TPB) ktab[k] = la.ktab(k);
  }

  // thread-fixed operand state.  kMC: index o = tid % BO, k rows tid / BO + (TPB / BO) * i.
  // otherwise: k = tid % BK (one per k-tile), index rows tid / BK + (TPB / BK) * i.
  typename LA::O oa[LA::kMC ? 1 : EA];
  typename LB::O ob[LB::kMC ? 1 : EB];
  if constexpr (LA::kMC) oa[0] = la.outer(m0 + tid % BM);
  else
#pragma unroll
    for (int i = 0; i < EA; ++i) oa[i] = la.outer(m0 + tid / BK + (TPB / BK) * i);
  if constexpr (LB::kMC) ob[0] = lb.outer(n0 + tid % BN);
  else
#pragma unroll
    for (int i = 0; i < EB; ++i) ob[i] = lb.outer(n0 + tid / BK + (TPB / BK) * i);
  if constexpr (LA::kMC) __syncthreads();  // k table visible

  float ra[EA], rb[EB];
  auto fetch = [&](int k0) {
    if constexpr (LA::kMC) {
#pragma unroll
      for (int i = 0; i < EA; ++i) {
        const int k = k0 + tid / BM + (TPB / BM) * i;
        ra[i] = la.load(oa[0], ktab[k]);
      }
    } else {
      const auto ks = la.kstate(k0 + tid % BK, kend);
#pragma unroll
      for (int i = 0; i < EA; ++i) ra[i] = la.load(oa[i], ks);
    }
    if constexpr (LB::kMC) {
#pragma unroll
      for (int i = 0; i < EB; ++i) rb[i] = lb.load(ob[0], ktab[k0 + tid / BN + (TPB / BN) * i]);
    } else {
      const auto ks = lb.kstate(k0 + tid % BK, kend);
#pragma unroll
      for (int i = 0; i < EB; ++i) rb[i] = lb.load(ob[i], ks);
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int i = 0; i < EA; ++i) {
      if constexpr (LA::kMC) As[buf][tid / BM + (TPB / BM) * i][tid % BM] = ra[i];
      else As[buf][tid % BK][tid / BK + (TPB / BK) * i] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < EB; ++i) {
      if constexpr (LB::kMC) Bs[buf][tid / BN + (TPB / BN) * i][tid % BN] = rb[i];
      else Bs[buf][tid % BK][tid / BK + (TPB / BK) * i] = rb[i];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = dev::zero_f32x4();

  const int lr = lane & 15, lk = lane >> 4;
  if (kbeg < kend) {
    fetch(kbeg);
    stash(0);
  }
  __syncthreads();
  int buf = 0;
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    const bool more = k0 + BK < kend;
    if (more) fetch(k0 + BK);  // next tile in flight during the MFMAs
#pragma unroll
    for (int kk = 4 * wk; kk < BK; kk += 4 * KSPLIT) {
      const float a0 = As[buf][kk + lk][wm + lr], a1 = As[buf][kk + lk][wm + 16 + lr];
      const float b0 = Bs[buf][kk + lk][wn + lr], b1 = Bs[buf][kk + lk][wn + 16 + lr];
      // B as the row operand: D[n][m], lane l holds n = 4 (l >> 4) + r, m = l & 15
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(b0, a0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(b1, a0, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(b0, a1, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(b1, a1, acc[1][1], 0, 0, 0);
    }
    if (more) stash(buf ^ 1);  // the other buffer's last readers passed the previous barrier
    __syncthreads();
    buf ^= 1;
  }
  if constexpr (KSPLIT > 1) {
    __shared__ f32x4 red[KSPLIT > 1 ? (KSPLIT - 1) * 4 * 64 : 1];
    if (wk > 0)
#pragma unroll
      for (int q = 0; q < 4; ++q) red[((wk - 1) * 4 + q) * 64 + lane] = acc[q >> 1][q & 1];
    __syncthreads();
    if (wk > 0) return;
#pragma unroll
    for (int w = 0; w < KSPLIT - 1; ++w)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q >> 1][q & 1] += red[(w * 4 + q) * 64 + lane];
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + wm + i * 16 + lr;
    if (m >= M) continue;
    const int rowoff = epi.row(m);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn + j * 16 + 4 * lk + r;
        if (n < N) epi.store(rowoff, n, acc[i][j][r]);
      }
  }
}

// wave layout by GEMM shape: 64x64 by default, 128x32 for N <= 32, 32x128 for M <= 32, 32x32 with
// the k-tile split over the 4 waves when both are
int pick_layout(int M, int N) {
  if (M <= 32 && N <= 32) return 11;
  if (N <= 32 && M > 32) return 41;
  if (M <= 32 && N > 32) return 14;
  return 22;
}

template <int WM, int WN, class LA, class LB, class Epi>
void launch_layout(int M, int N, int K, int per, int slices, const LA& la, const LB& lb, const Epi& epi,
                   hipStream_t s) {
  constexpr int BM = 32 * WM, BN = 32 * WN;
  dim3 grid(static_cast<unsigned>((M + BM - 1) / BM), static_cast<unsigned>((N + BN - 1) / BN),
            static_cast<unsigned>(slices));
  const int ktab_n = LA::kMC ? (K + BK - 1) / BK * BK : 0;
  hipLaunchKernelGGL((gemm_f32_kernel<WM, WN, LA, LB, Epi>), grid, dim3(TPB), ktab_n * sizeof(int2), s, M, N, K,
                     per, ktab_n, la, lb, epi);
}

template <class LA, class LB, class Epi>
void launch_gemm(int M, int N, int K, int per, int slices, const LA& la, const LB& lb, const Epi& epi,
                 hipStream_t s) {
  switch (pick_layout(M, N)) {
    case 41: launch_layout<4, 1>(M, N, K, per, slices, la, lb, epi, s); break;
    case 14: launch_layout<1, 4>(M, N, K, per, slices, la, lb, epi, s); break;
    case 11: launch_layout<1, 1>(M, N, K, per, slices, la, lb, epi, s); break;
    default: launch_layout<2, 2>(M, N, K, per, slices, la, lb, epi, s); break;
  }
}

// ---------------------------------------------------------------- pooling (+ReLU)
// a[bc, py, px] = relu(max over the k x k window at (py*st, px*st)); code = argmax offset
// (first maximum in row-major order, as max_pool2d); code 255 where the result is 0 (no gradient).
__global__ __launch_bounds__(256) void pool_relu_fwd_kernel(const float* __restrict__ z, float* __restrict__ a,
                                                            unsigned char* __restrict__ code, int total, int H,
                                                            int W, FastDiv fphw, FastDiv fpw, int k, int st) {
  for (int i = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x); i < total;
       i += static_cast<int>(gridDim.x * blockDim.x)) {
    const int bc = fdiv(i, fphw), r = i - bc * static_cast<int>(fphw.d);
    const int py = fdiv(r, fpw), px = r - py * static_cast<int>(fpw.d);
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

// dz[bc, y, x] = sum over windows (py, px) covering (y, x) whose code points at (y, x) of da[bc, py, px]
__global__ __launch_bounds__(256) void pool_relu_bwd_kernel(const float* __restrict__ da,
                                                            const unsigned char* __restrict__ code,
                                                            float* __restrict__ dz, int total, FastDiv fhw,
                                                            FastDiv fw, int PH, int PW, int k, int st) {
  for (int i = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x); i < total;
       i += static_cast<int>(gridDim.x * blockDim.x)) {
    const int bc = fdiv(i, fhw), r = i - bc * static_cast<int>(fhw.d);
    const int y = fdiv(r, fw), x = r - y * static_cast<int>(fw.d);
    float g = 0.f;
    for (int dy = 0; dy < k; ++dy) {
      const int ty = y - dy;
      if (ty < 0) break;
      const int py = ty / st;
      if (py * st != ty || py >= PH) continue;
      for (int dx = 0; dx < k; ++dx) {
        const int tx = x - dx;
        if (tx < 0) break;
        const int px = tx / st;
        if (px * st != tx || px >= PW) continue;
        const int o = bc * PH * PW + py * PW + px;
        if (code[o] == dy * k + dx) g += da[o];
      }
    }
    dz[i] = g;
  }
}

// Non-overlapping 2x2/s2 windows: one thread per window writes its 2x2 block (the gradient at the
// coded position, zeros elsewhere); a trailing odd row / column (no window covers it) is zeroed by
// the last window of the row / column.
__global__ __launch_bounds__(256) void pool2s2_bwd_kernel(const float* __restrict__ da,
                                                          const unsigned char* __restrict__ code,
                                                          float* __restrict__ dz, int total, FastDiv fphw,
                                                          FastDiv fpw, int H, int W) {
  const int PH = H / 2, PW = W / 2;
  for (int i = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x); i < total;
       i += static_cast<int>(gridDim.x * blockDim.x)) {
    const int bc = fdiv(i, fphw), r = i - bc * static_cast<int>(fphw.d);
    const int py = fdiv(r, fpw), px = r - py * PW;
    const int c = code[i];
    const float g = da[i];
    float* o = dz + bc * H * W + 2 * py * W + 2 * px;
    const float2 top = make_float2(c == 0 ? g : 0.f, c == 1 ? g : 0.f);
    const float2 bot = make_float2(c == 2 ? g : 0.f, c == 3 ? g : 0.f);
    if ((W & 1) == 0) {
      *reinterpret_cast<float2*>(o) = top;
      *reinterpret_cast<float2*>(o + W) = bot;
    } else {
      o[0] = top.x; o[1] = top.y; o[W] = bot.x; o[W + 1] = bot.y;
      if (px == PW - 1) { o[2] = 0.f; o[W + 2] = 0.f; }
    }
    if ((H & 1) && py == PH - 1) {
      o[2 * W] = 0.f;
      o[2 * W + 1] = 0.f;
      if ((W & 1) && px == PW - 1) o[2 * W + 2] = 0.f;
    }
  }
}

// Overlapping 2x2/s1 windows: one thread per input position gathers the (up to) 4 windows covering it.
__global__ __launch_bounds__(256) void pool2s1_bwd_kernel(const float* __restrict__ da,
                                                          const unsigned char* __restrict__ code,
                                                          float* __restrict__ dz, int total, FastDiv fhw,
                                                          FastDiv fw, int PH, int PW) {
  for (int i = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x); i < total;
       i += static_cast<int>(gridDim.x * blockDim.x)) {
    const int bc = fdiv(i, fhw), r = i - bc * static_cast<int>(fhw.d);
    const int y = fdiv(r, fw), x = r - y * static_cast<int>(fw.d);
    const int base = bc * PH * PW;
    float g = 0.f;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int py = y - dy, px = x - dx;
        if (static_cast<unsigned>(py) < static_cast<unsigned>(PH) && static_cast<unsigned>(px) < static_cast<unsigned>(PW)) {
          const int o = base + py * PW + px;
          if (code[o] == dy * 2 + dx) g += da[o];
        }
      }
    dz[i] = g;
  }
}

// Fixed-order sum of the split-K slabs [slices][Kout][Nw + has_bias] into dw [Kout][Nw] and db [Kout].
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ slab, int slices, int Kout,
                                                           int Nw, int ncol, float* __restrict__ dw,
                                                           float* __restrict__ db) {
  const int total = Kout * ncol;
  for (int i = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x); i < total;
       i += static_cast<int>(gridDim.x * blockDim.x)) {
    float acc = slab[i];
    for (int z = 1; z < slices; ++z) acc += slab[static_cast<int64_t>(z) * total + i];
    const int m = i / ncol, n = i - m * ncol;
    if (n < Nw) dw[m * Nw + n] = acc;
    else db[m] = acc;
  }
}

int grid_1d(int64_t n) {
  const int64_t g = (n + 255) / 256;
  return static_cast<int>(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

// Largest batch chunk whose per-chunk element counts (each listed per-image size) stay < 2^31
// (RINGDP_F32_CHUNK_LIMIT lowers the bound: the tests run the chunked path at small batches).
int64_t batch_chunk(int64_t B, std::initializer_list<int64_t> per_image) {
  int64_t worst = 1;
  for (int64_t v : per_image) worst = std::max(worst, v);
  int64_t limit = (int64_t{1} << 31) - 1;
  if (const char* e = std::getenv("RINGDP_F32_CHUNK_LIMIT")) limit = std::max<int64_t>(1, std::min<int64_t>(limit, std::atoll(e)));
  const int64_t cap = limit / worst;
  return std::max<int64_t>(1, std::min(B, cap));
}

int wgrad_slices(int M, int N, int64_t K) {
  // enough slices to put >= ~2048 workgroups on the 256 CUs, each slice >= 1024 deep
  const int l = pick_layout(M, N);
  const int bm = 32 * (l / 10), bn = 32 * (l % 10);
  const int64_t tiles = static_cast<int64_t>((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  int64_t s = (2048 + tiles - 1) / tiles;
  const int64_t cap = (K + 1023) / 1024;
  if (s > cap) s = cap;
  return static_cast<int>(s < 1 ? 1 : (s > 1024 ? 1024 : s));
}

int64_t wgrad_chunk(const ConvF32Geom& g) {
  return batch_chunk(g.B, {static_cast<int64_t>(g.C) * g.H * g.W, static_cast<int64_t>(g.Kout) * g.OH * g.OW});
}

}  // namespace

int conv_f32_wgrad_slices(const ConvF32Geom& g) {
  const int64_t chunk = wgrad_chunk(g);
  const int64_t nchunks = (g.B + chunk - 1) / chunk;
  return static_cast<int>(nchunks) *
         wgrad_slices(g.Kout, g.C * g.R * g.R + 1, chunk * static_cast<int64_t>(g.OH) * g.OW);
}

void conv_f32_fwd(const ConvF32Geom& g, const float* x, const unsigned char* xu8, float mean, float inv_std,
                  const float* w, const float* bias, float* z, hipStream_t s) {
  const int K = g.C * g.R * g.R;
  const int64_t xin = static_cast<int64_t>(g.C) * g.H * g.W, zout = static_cast<int64_t>(g.Kout) * g.OH * g.OW;
  const int64_t chunk = batch_chunk(g.B, {xin, zout});
  for (int64_t b0 = 0; b0 < g.B; b0 += chunk) {
    const int nb = static_cast<int>(std::min(chunk, g.B - b0));
    const int M = nb * g.OH * g.OW;
    FwdA la{x ? x + b0 * xin : nullptr, xu8 ? xu8 + b0 * xin : nullptr, mean, inv_std, g.C, g.H, g.W, g.R, g.pad,
            g.OW, K, M, make_fdiv(g.OH * g.OW), make_fdiv(g.OW)};
    WeightB lb{w, K, g.Kout};
    NCHWOut epi{z + b0 * zout, bias, g.Kout, M, make_fdiv(g.OH * g.OW)};
    launch_gemm(M, g.Kout, K, K, 1, la, lb, epi, s);
  }
}

void conv_f32_dgrad(const ConvF32Geom& g, const float* dz, const float* w, float* dx, hipStream_t s) {
  const int K = g.Kout * g.R * g.R;
  const int64_t zin = static_cast<int64_t>(g.Kout) * g.OH * g.OW, xout = static_cast<int64_t>(g.C) * g.H * g.W;
  const int64_t chunk = batch_chunk(g.B, {zin, xout});
  for (int64_t b0 = 0; b0 < g.B; b0 += chunk) {
    const int nb = static_cast<int>(std::min(chunk, g.B - b0));
    const int M = nb * g.H * g.W;
    DgradA la{dz + b0 * zin, g.Kout, g.W, g.R, g.OH, g.OW, g.pad, K, M, make_fdiv(g.H * g.W), make_fdiv(g.W)};
    DgradB lb{w, g.C, g.R * g.R, K, make_fdiv(g.R * g.R)};
    NCHWOut epi{dx + b0 * xout, nullptr, g.C, M, make_fdiv(g.H * g.W)};
    launch_gemm(M, g.C, K, K, 1, la, lb, epi, s);
  }
}

void conv_f32_wgrad(const ConvF32Geom& g, const float* dz, const float* x, const unsigned char* xu8, float mean,
                    float inv_std, float* slab, int slices, float* dw, float* db, hipStream_t s) {
  const int Nw = g.C * g.R * g.R;
  const int ncol = Nw + (db ? 1 : 0);
  const int64_t xin = static_cast<int64_t>(g.C) * g.H * g.W, zin = static_cast<int64_t>(g.Kout) * g.OH * g.OW;
  const int64_t chunk = wgrad_chunk(g);
  const int ohw = g.OH * g.OW;
  int used = 0;
  for (int64_t b0 = 0; b0 < g.B; b0 += chunk) {
    const int nb = static_cast<int>(std::min(chunk, g.B - b0));
    const int K = nb * ohw;
    const int sl = wgrad_slices(g.Kout, Nw + 1, static_cast<int64_t>(chunk) * ohw);
    int per = (K + sl - 1) / sl;
    per = (per + BK - 1) / BK * BK;
    const int used_sl = (K + per - 1) / per;
    WgradA la{dz + b0 * zin, g.Kout, ohw, make_fdiv(ohw)};
    WgradB lb{x ? x + b0 * xin : nullptr, xu8 ? xu8 + b0 * xin : nullptr, mean, inv_std, g.C, g.H, g.W, g.R,
              g.pad, g.OW, Nw, make_fdiv(ohw), make_fdiv(g.OW)};
    SlabOut epi{slab + static_cast<int64_t>(used) * g.Kout * ncol, ncol, g.Kout};
    launch_gemm(g.Kout, ncol, K, per, used_sl, la, lb, epi, s);
    used += used_sl;
  }
  (void)slices;  // the slab holds conv_f32_wgrad_slices(g) >= used slices
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(grid_1d(static_cast<int64_t>(g.Kout) * ncol)), dim3(256), 0, s,
                     slab, used, g.Kout, Nw, ncol, dw, db);
}

void pool_relu_f32_fwd(const float* z, float* a, unsigned char* code, int64_t BC, int H, int W, int k, int st,
                       hipStream_t s) {
  const int PH = (H - k) / st + 1, PW = (W - k) / st + 1;
  const int64_t chunk = batch_chunk(BC, {static_cast<int64_t>(H) * W});
  for (int64_t c0 = 0; c0 < BC; c0 += chunk) {
    const int64_t nbc = std::min(chunk, BC - c0);
    const int total = static_cast<int>(nbc * PH * PW);
    hipLaunchKernelGGL(pool_relu_fwd_kernel, dim3(grid_1d(total)), dim3(256), 0, s, z + c0 * H * W,
                       a + c0 * PH * PW, code + c0 * PH * PW, total, H, W, make_fdiv(PH * PW), make_fdiv(PW), k, st);
  }
}

void pool_relu_f32_bwd(const float* da, const unsigned char* code, float* dz, int64_t BC, int H, int W, int k,
                       int st, hipStream_t s) {
  const int PH = (H - k) / st + 1, PW = (W - k) / st + 1;
  const int64_t chunk = batch_chunk(BC, {static_cast<int64_t>(H) * W});
  for (int64_t c0 = 0; c0 < BC; c0 += chunk) {
    const int64_t nbc = std::min(chunk, BC - c0);
    const int total = static_cast<int>(nbc * H * W);
    if (k == 2 && st == 2) {
      const int wins = static_cast<int>(nbc * PH * PW);
      hipLaunchKernelGGL(pool2s2_bwd_kernel, dim3(grid_1d(wins)), dim3(256), 0, s, da + c0 * PH * PW,
                         code + c0 * PH * PW, dz + c0 * H * W, wins, make_fdiv(PH * PW), make_fdiv(PW), H, W);
      continue;
    }
    if (k == 2 && st == 1) {
      hipLaunchKernelGGL(pool2s1_bwd_kernel, dim3(grid_1d(total)), dim3(256), 0, s, da + c0 * PH * PW,
                         code + c0 * PH * PW, dz + c0 * H * W, total, make_fdiv(H * W), make_fdiv(W), PH, PW);
      continue;
    }
    hipLaunchKernelGGL(pool_relu_bwd_kernel, dim3(grid_1d(total)), dim3(256), 0, s, da + c0 * PH * PW,
                       code + c0 * PH * PW, dz + c0 * H * W, total, make_fdiv(H * W), make_fdiv(W), PH, PW, k, st);
  }
}

}  // namespace kern
}  // namespace ringdp
