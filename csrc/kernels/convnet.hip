// MNIST ConvNet hot path for CDNA4 (gfx950): hand-written HIP, bf16 MFMA + LDS tiling.
//
// Model (ref/launch_dist.py:9-41):
//   conv1 1->32 k5 p1 (28->26) -> ReLU -> MaxPool(2,2) (13)
//   conv2 32->64 k3 (13->11)  -> ReLU -> MaxPool(2,1) (10)   [overlapping windows]
//   conv3 64->128 k3 (10->8)  -> ReLU -> MaxPool(2,2) (4)  -> view(-1, 2048) -> fc1 2048->10
//
// Design (MI355X-first, not a translation of cuDNN calls):
//   * activations stay NHWC bf16 and only the POOLED outputs are stored (+ a 1-byte argmax per
//     pooled element); ReLU/MaxPool are fused into the conv epilogue (K02/K03/K05/K06/K08/K09);
//   * conv2/conv3 forward = implicit GEMM on v_mfma_f32_16x16x32_bf16, whole input image staged
//     in LDS, weights converted fp32->bf16 while staged (no shadow weight copies), workgroups
//     loop over images so weights are staged once per workgroup;
//   * backward never materialises d(conv) in HBM: each kernel re-creates it while staging from
//     d(pooled) + argmax + pooled>0 (unpool+ReLU-mask, deterministic gather form even for the
//     overlapping k2/s1 pool, K17);
//   * dgrad = "full" correlation with flipped weights from a zero-ringed LDS image (MFMA);
//   * wgrad = TN GEMM over (image, position) with operands read by ds_read_b64_tr_b16 straight
//     from the NHWC LDS images (the transposed read also does the im2col gather), split over
//     images into fp32 slabs reduced in a fixed order (deterministic);
//   * conv1 (C_in = 1) forward is fp32 VALU direct convolution; its wgrad is an MFMA GEMM over a
//     row-padded unpooled grid with per-kw shifted copies of the input to keep reads aligned.
#include "device_common.h"
#include "kernels.h"

namespace ringdp {
namespace kern {

using namespace ringdp::dev;

namespace {

constexpr int kThreads = 256;

// ------------------------------------------------------------------ geometry
template <int L>
struct Geo;
template <>
struct Geo<2> {
  static constexpr int CIN = 32, COUT = 64, IH = 13, PS = 1, OH = 11, PH = 10;
};
template <>
struct Geo<3> {
  static constexpr int CIN = 64, COUT = 128, IH = 10, PS = 2, OH = 8, PH = 4;
};

__host__ __device__ constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }
__host__ __device__ constexpr int align16(int bytes) { return (bytes + 15) / 16 * 16; }

// 8 channels of d(conv output) at (y, x) from d(pooled), argmax and pooled > 0 (ReLU mask).
// Gather form: sums over every pooling window that covers (y, x) and selected it.
template <int OH, int PH, int PS, int C>
__device__ __forceinline__ void unpool_grad8(const bf16* __restrict__ dout, const uint8_t* __restrict__ idx,
                                             const bf16* __restrict__ pooled, int y, int x, int c0,
                                             float (&g)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) g[j] = 0.f;
  const int py_lo = y >= 1 ? (y - 1 + PS - 1) / PS : 0;
  const int py_hi = min(PH - 1, y / PS);
  const int px_lo = x >= 1 ? (x - 1 + PS - 1) / PS : 0;
  const int px_hi = min(PH - 1, x / PS);
  for (int py = py_lo; py <= py_hi; ++py) {
    for (int px = px_lo; px <= px_hi; ++px) {
      const int e = (py * PH + px) * C + c0;
      const int want = (y - py * PS) * 2 + (x - px * PS);
      const bf16x8 dv = *reinterpret_cast<const bf16x8*>(dout + e);
      const bf16x8 pv = *reinterpret_cast<const bf16x8*>(pooled + e);
      const uint2 iv = *reinterpret_cast<const uint2*>(idx + e);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t word = j < 4 ? iv.x : iv.y;
        const int ij = (word >> (8 * (j & 3))) & 0xff;
        if (ij == want && (float)pv[j] > 0.f) g[j] += (float)dv[j];
      }
    }
  }
}

// ------------------------------------------------------------------ conv1 forward (VALU fp32)
// One workgroup loops over images; per image: 30x30 zero-ringed normalised input in LDS.
// Work item = (channel group of 8, pooled position): 8 ch x 4 conv outputs x 25 taps.
template <bool U8>
__global__ __launch_bounds__(kThreads) void conv1_fwd_kernel(const void* __restrict__ xin,
                                                             const float* __restrict__ w,
                                                             const float* __restrict__ bias,
                                                             bf16* __restrict__ a1,
                                                             uint8_t* __restrict__ idx1, int B,
                                                             float mean, float inv_std, float in_scale) {
  __shared__ float xs[30 * 30];
  __shared__ float ws[32 * 25];
  __shared__ float bs[32];
  for (int i = threadIdx.x; i < 800; i += kThreads) ws[i] = w[i];
  if (threadIdx.x < 32) bs[threadIdx.x] = bias[threadIdx.x];
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    __syncthreads();
    for (int i = threadIdx.x; i < 900; i += kThreads) {
      const int r = i / 30 - 1, c = i % 30 - 1;
      float v = 0.f;
      if (r >= 0 && r < 28 && c >= 0 && c < 28) {
        const int64_t o = (int64_t)b * 784 + r * 28 + c;
        const float raw = U8 ? (float)static_cast<const uint8_t*>(xin)[o] * in_scale
                             : static_cast<const float*>(xin)[o];
        v = (raw - mean) * inv_std;
      }
      xs[i] = v;
    }
    __syncthreads();
    for (int item = threadIdx.x; item < 4 * 169; item += kThreads) {
      const int cg = item / 169, pp = item % 169;
      const int ph = pp / 13, pw = pp % 13;
      float patch[6][6];
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = 0; c < 6; ++c) patch[r][c] = xs[(2 * ph + r) * 30 + 2 * pw + c];
      bf16x8 outv;
      uint32_t iw0 = 0, iw1 = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int co = cg * 8 + j;
        float acc[4];
        const float bv = bs[co];
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = bv;
#pragma unroll
        for (int kh = 0; kh < 5; ++kh)
#pragma unroll
          for (int kw = 0; kw < 5; ++kw) {
            const float wv = ws[co * 25 + kh * 5 + kw];
            acc[0] = fmaf(wv, patch[kh][kw], acc[0]);
            acc[1] = fmaf(wv, patch[kh][kw + 1], acc[1]);
            acc[2] = fmaf(wv, patch[kh + 1][kw], acc[2]);
            acc[3] = fmaf(wv, patch[kh + 1][kw + 1], acc[3]);
          }
        int bi = 0;
        float bm = acc[0];
#pragma unroll
        for (int q = 1; q < 4; ++q)
          if (acc[q] > bm) {
            bm = acc[q];
            bi = q;
          }
        outv[j] = (bf16)fmaxf(bm, 0.f);
        if (j < 4)
          iw0 |= (uint32_t)bi << (8 * j);
        else
          iw1 |= (uint32_t)bi << (8 * (j - 4));
      }
      const int64_t o = ((int64_t)b * 169 + pp) * 32 + cg * 8;
      *reinterpret_cast<bf16x8*>(a1 + o) = outv;
      *reinterpret_cast<uint2*>(idx1 + o) = make_uint2(iw0, iw1);
    }
  }
}

// ------------------------------------------------------------------ conv3x3 fwd + ReLU + pool
// Implicit GEMM: M = OH*OH output positions, N = CN output channels (slice `ns` of NSPLIT),
// K = 9 taps x CIN.  A[m][k] = in[oh+kh][ow+kw][ci] read from the LDS image; B[n][k] = the
// slice's weights (bf16, k-contiguous rows).  Epilogue: bias -> fp32 LDS tile -> max-pool with
// argmax -> ReLU -> bf16 pooled output.
template <int L, int NSPLIT>
struct FwdCfg {
  using G = Geo<L>;
  static constexpr int CN = G::COUT / NSPLIT;
  static constexpr int K = 9 * G::CIN;
  static constexpr int KS = K / 32;
  static constexpr int M = G::OH * G::OH;
  static constexpr int MT = cdiv(M, 16);
  static constexpr int NT = CN / 16;
  static constexpr int A_RS = G::CIN + 8;  // bf16 elements per LDS image row (position)
  static constexpr int B_RS = K + 8;       // bf16 elements per LDS weight row
  static constexpr int C_RS = CN + 1;      // floats per epilogue row
  static constexpr int A_BYTES = align16(G::IH * G::IH * A_RS * 2);
  static constexpr int B_BYTES = align16(CN * B_RS * 2);
  static constexpr int C_BYTES = align16(M * C_RS * 4);
  static constexpr int LDS = B_BYTES + (A_BYTES > C_BYTES ? A_BYTES : C_BYTES);
  static constexpr int TILES = MT * NT;
  static constexpr int TPW = cdiv(TILES, 4);  // tiles per wave
};

template <int L, int NSPLIT>
__global__ __launch_bounds__(kThreads) void conv_fwd_kernel(const bf16* __restrict__ in,
                                                            const float* __restrict__ w,
                                                            const float* __restrict__ bias,
                                                            bf16* __restrict__ out,
                                                            uint8_t* __restrict__ idx, int B) {
  using G = Geo<L>;
  using F = FwdCfg<L, NSPLIT>;
  __shared__ __attribute__((aligned(16))) char smem[F::LDS];
  bf16* Bs = reinterpret_cast<bf16*>(smem);
  bf16* As = reinterpret_cast<bf16*>(smem + F::B_BYTES);
  float* Cs = reinterpret_cast<float*>(smem + F::B_BYTES);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ns = blockIdx.x % NSPLIT;
  const int co0 = ns * F::CN;
  const int groups = gridDim.x / NSPLIT;

  // Stage this slice's weights once: natural [co][ci][tap] order reads, [co][tap*CIN+ci] writes.
  for (int e = tid; e < F::CN * G::CIN * 9; e += kThreads) {
    const int co = e / (G::CIN * 9), r = e % (G::CIN * 9), ci = r / 9, tap = r % 9;
    Bs[co * F::B_RS + tap * G::CIN + ci] = (bf16)w[(int64_t)co0 * G::CIN * 9 + e];
  }

  for (int b = blockIdx.x / NSPLIT; b < B; b += groups) {
    __syncthreads();  // previous image's epilogue done with Cs (aliases As)
    // Stage the input image (NHWC) with padded rows.
    constexpr int CH8 = G::CIN / 8;
    const bf16* src = in + (int64_t)b * G::IH * G::IH * G::CIN;
    for (int e = tid; e < G::IH * G::IH * CH8; e += kThreads) {
      const int pos = e / CH8, q = e % CH8;
      *reinterpret_cast<bf16x8*>(As + pos * F::A_RS + q * 8) =
          *reinterpret_cast<const bf16x8*>(src + pos * G::CIN + q * 8);
    }
    __syncthreads();

    f32x4 acc[F::TPW];
#pragma unroll
    for (int t = 0; t < F::TPW; ++t) acc[t] = zero_f32x4();
    const int r16 = lane & 15, q8 = (lane >> 4) * 8;
    // Per-tile A-row base (position) for this lane.
    int arow[F::TPW];
    bool avalid[F::TPW];
#pragma unroll
    for (int t = 0; t < F::TPW; ++t) {
      const int tile = wave + 4 * t;
      const int mt = tile % F::MT;
      const int m = mt * 16 + r16;
      avalid[t] = tile < F::TILES && m < F::M;
      const int mm = avalid[t] ? m : 0;
      arow[t] = (mm / G::OH) * G::IH + (mm % G::OH);
    }
#pragma unroll 2
    for (int ks = 0; ks < F::KS; ++ks) {
      const int k0 = ks * 32;
      const int tap = k0 / G::CIN, ci0 = k0 % G::CIN;
      const int kh = tap / 3, kw = tap % 3;
      const int shift = kh * G::IH + kw;
#pragma unroll
      for (int t = 0; t < F::TPW; ++t) {
        const int tile = wave + 4 * t;
        if (tile >= F::TILES) continue;
        const int nt = tile / F::MT;
        const bf16x8 bfrag =
            *reinterpret_cast<const bf16x8*>(Bs + (nt * 16 + r16) * F::B_RS + k0 + q8);
        bf16x8 afrag = zero_bf16x8();
        if (avalid[t])
          afrag = *reinterpret_cast<const bf16x8*>(As + (arow[t] + shift) * F::A_RS + ci0 + q8);
        acc[t] = mfma16x16x32(afrag, bfrag, acc[t]);
      }
    }
    __syncthreads();  // all waves done reading As before Cs (alias) is written
#pragma unroll
    for (int t = 0; t < F::TPW; ++t) {
      const int tile = wave + 4 * t;
      if (tile >= F::TILES) continue;
      const int mt = tile % F::MT, nt = tile / F::MT;
      const int c = nt * 16 + r16;
      const float bv = bias[co0 + c];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = mt * 16 + (lane >> 4) * 4 + i;
        if (m < F::M) Cs[m * F::C_RS + c] = acc[t][i] + bv;
      }
    }
    __syncthreads();
    // Max-pool (k2, stride PS) with first-max argmax, then ReLU; 8 channels per item.
    constexpr int CG = F::CN / 8;
    bf16* ob = out + (int64_t)b * G::PH * G::PH * G::COUT;
    uint8_t* ib = idx + (int64_t)b * G::PH * G::PH * G::COUT;
    for (int e = tid; e < G::PH * G::PH * CG; e += kThreads) {
      const int pp = e / CG, cg = e % CG;
      const int ph = pp / G::PH, pw = pp % G::PH;
      const int m00 = (ph * G::PS) * G::OH + pw * G::PS;
      bf16x8 ov;
      uint32_t w0 = 0, w1 = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = cg * 8 + j;
        const float v0 = Cs[m00 * F::C_RS + c];
        const float v1 = Cs[(m00 + 1) * F::C_RS + c];
        const float v2 = Cs[(m00 + G::OH) * F::C_RS + c];
        const float v3 = Cs[(m00 + G::OH + 1) * F::C_RS + c];
        int bi = 0;
        float bm = v0;
        if (v1 > bm) { bm = v1; bi = 1; }
        if (v2 > bm) { bm = v2; bi = 2; }
        if (v3 > bm) { bm = v3; bi = 3; }
        ov[j] = (bf16)fmaxf(bm, 0.f);
        if (j < 4) w0 |= (uint32_t)bi << (8 * j);
        else w1 |= (uint32_t)bi << (8 * (j - 4));
      }
      const int o = pp * G::COUT + co0 + cg * 8;
      *reinterpret_cast<bf16x8*>(ob + o) = ov;
      *reinterpret_cast<uint2*>(ib + o) = make_uint2(w0, w1);
    }
  }
}

// ------------------------------------------------------------------ conv3x3 dgrad
// din[ih][iw][ci] = sum_{kh',kw',co} P[ih+kh'][iw+kw'][co] * W[co][ci][2-kh'][2-kw'], with P the
// d(conv) image (re-created from d(pooled)) inside a zero ring of width 2.
template <int L, int NSPLIT>
struct DgradCfg {
  using G = Geo<L>;
  static constexpr int CN = G::CIN / NSPLIT;   // input channels produced per workgroup
  static constexpr int K = 9 * G::COUT;
  static constexpr int KS = K / 32;
  static constexpr int PW = G::OH + 4;         // padded d(conv) width (= IH + 2)
  static constexpr int M = G::IH * G::IH;
  static constexpr int MT = cdiv(M, 16);
  static constexpr int NT = CN / 16;
  static constexpr int P_RS = G::COUT + 8;
  static constexpr int B_RS = K + 8;
  static constexpr int C_RS = CN + 1;
  static constexpr int P_BYTES = align16(PW * PW * P_RS * 2);
  static constexpr int B_BYTES = align16(CN * B_RS * 2);
  static constexpr int C_BYTES = align16(M * C_RS * 4);
  static constexpr int LDS = B_BYTES + (P_BYTES > C_BYTES ? P_BYTES : C_BYTES);
  static constexpr int TILES = MT * NT;
  static constexpr int TPW = cdiv(TILES, 4);
};

template <int L, int NSPLIT>
__device__ __forceinline__ void dgrad_body(char* smem, const float* __restrict__ w,
                                           const bf16* __restrict__ dout,
                                           const uint8_t* __restrict__ idx,
                                           const bf16* __restrict__ pooled, bf16* __restrict__ din,
                                           int B, int block, int nblocks) {
  using G = Geo<L>;
  using D = DgradCfg<L, NSPLIT>;
  bf16* Bs = reinterpret_cast<bf16*>(smem);
  bf16* Ps = reinterpret_cast<bf16*>(smem + D::B_BYTES);
  float* Cs = reinterpret_cast<float*>(smem + D::B_BYTES);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ns = block % NSPLIT;
  const int ci0 = ns * D::CN;
  const int groups = nblocks / NSPLIT;

  // Flipped, transposed weight slice: Bs[ci][tap'*COUT + co] = W[co][ci0+ci][8 - tap'].
  for (int e = tid; e < G::COUT * D::CN * 9; e += kThreads) {
    const int co = e / (D::CN * 9), r = e % (D::CN * 9), ci = r / 9, tap = r % 9;
    Bs[ci * D::B_RS + (8 - tap) * G::COUT + co] =
        (bf16)w[(int64_t)co * G::CIN * 9 + (int64_t)(ci0 + ci) * 9 + tap];
  }

  for (int b = block / NSPLIT; b < B; b += groups) {
    __syncthreads();
    // Zero ring + interior re-created from the pooled gradient.
    constexpr int CG = G::COUT / 8;
    const int64_t pbase = (int64_t)b * G::PH * G::PH * G::COUT;
    for (int e = tid; e < D::PW * D::PW * CG; e += kThreads) {
      const int pos = e / CG, cg = e % CG;
      const int y = pos / D::PW - 2, x = pos % D::PW - 2;
      bf16x8 v = zero_bf16x8();
      if (y >= 0 && y < G::OH && x >= 0 && x < G::OH) {
        float g[8];
        unpool_grad8<G::OH, G::PH, G::PS, G::COUT>(dout + pbase, idx + pbase, pooled + pbase, y,
                                                   x, cg * 8, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (bf16)g[j];
      }
      *reinterpret_cast<bf16x8*>(Ps + pos * D::P_RS + cg * 8) = v;
    }
    __syncthreads();

    f32x4 acc[D::TPW];
#pragma unroll
    for (int t = 0; t < D::TPW; ++t) acc[t] = zero_f32x4();
    const int r16 = lane & 15, q8 = (lane >> 4) * 8;
    int prow[D::TPW];
    bool valid[D::TPW];
#pragma unroll
    for (int t = 0; t < D::TPW; ++t) {
      const int tile = wave + 4 * t;
      const int m = (tile % D::MT) * 16 + r16;
      valid[t] = tile < D::TILES && m < D::M;
      const int mm = valid[t] ? m : 0;
      prow[t] = (mm / G::IH) * D::PW + (mm % G::IH);
    }
#pragma unroll 2
    for (int ks = 0; ks < D::KS; ++ks) {
      const int k0 = ks * 32;
      const int tap = k0 / G::COUT, c0 = k0 % G::COUT;
      const int shift = (tap / 3) * D::PW + (tap % 3);
#pragma unroll
      for (int t = 0; t < D::TPW; ++t) {
        const int tile = wave + 4 * t;
        if (tile >= D::TILES) continue;
        const int nt = tile / D::MT;
        const bf16x8 bfrag =
            *reinterpret_cast<const bf16x8*>(Bs + (nt * 16 + r16) * D::B_RS + k0 + q8);
        bf16x8 afrag = zero_bf16x8();
        if (valid[t])
          afrag = *reinterpret_cast<const bf16x8*>(Ps + (prow[t] + shift) * D::P_RS + c0 + q8);
        acc[t] = mfma16x16x32(afrag, bfrag, acc[t]);
      }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < D::TPW; ++t) {
      const int tile = wave + 4 * t;
      if (tile >= D::TILES) continue;
      const int mt = tile % D::MT, nt = tile / D::MT;
      const int c = nt * 16 + r16;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = mt * 16 + (lane >> 4) * 4 + i;
        if (m < D::M) Cs[m * D::C_RS + c] = acc[t][i];
      }
    }
    __syncthreads();
    constexpr int OG = D::CN / 8;
    bf16* db = din + (int64_t)b * D::M * G::CIN;
    for (int e = tid; e < D::M * OG; e += kThreads) {
      const int m = e / OG, cg = e % OG;
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (bf16)Cs[m * D::C_RS + cg * 8 + j];
      *reinterpret_cast<bf16x8*>(db + m * G::CIN + ci0 + cg * 8) = v;
    }
  }
}

// ------------------------------------------------------------------ conv3x3 wgrad (split-K)
// dWt[n = tap*CIN + ci][co] = sum_{b, pos} Dc[b][pos][co] * X[b][pos shifted by tap][ci].
// Wave grid WM x WN over (co tiles) x (n tiles of this tap group).
template <int L>
struct WgradCfg;
template <>
struct WgradCfg<2> {
  static constexpr int TG = 9, WM = 2, WN = 2;
};
template <>
struct WgradCfg<3> {
  static constexpr int TG = 3, WM = 1, WN = 4;
};

template <int L>
struct WgradGeo {
  using G = Geo<L>;
  using C = WgradCfg<L>;
  static constexpr int NPOS = G::OH * G::OH;
  static constexpr int KP = cdiv(NPOS, 32) * 32;       // K rows per image (zero padded)
  static constexpr int KS = KP / 32;
  static constexpr int NGROUPS = 9 / C::TG;
  static constexpr int NCH = C::TG * G::CIN;           // n columns per workgroup
  static constexpr int MTW = (G::COUT / 16) / C::WM;   // m tiles per wave
  static constexpr int NTW = (NCH / 16) / C::WN;       // n tiles per wave
  static constexpr int D_RS = G::COUT + 8;
  static constexpr int X_RS = G::CIN + 8;
  static constexpr int D_BYTES = align16(KP * D_RS * 2);
  static constexpr int X_BYTES = align16(G::IH * G::IH * X_RS * 2);
  static constexpr int LDS = D_BYTES + X_BYTES;
  static constexpr int NOUT = 9 * G::CIN * G::COUT;    // floats per slab (weights)
  static_assert((G::COUT / 16) % C::WM == 0, "bad WM");
  static_assert((NCH / 16) % C::WN == 0, "bad WN");
};

// Slab layout per slice s: [NOUT weights in dWt order (n-major, co fastest)] [COUT bias].
template <int L>
__device__ __forceinline__ void wgrad_body(char* smem, const bf16* __restrict__ x,
                                           const bf16* __restrict__ dout,
                                           const uint8_t* __restrict__ idx,
                                           const bf16* __restrict__ pooled,
                                           float* __restrict__ slabs, int B, int nslices,
                                           int block) {
  using G = Geo<L>;
  using C = WgradCfg<L>;
  using W = WgradGeo<L>;
  bf16* Ds = reinterpret_cast<bf16*>(smem);
  bf16* Xs = reinterpret_cast<bf16*>(smem + W::D_BYTES);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int slice = block / W::NGROUPS, tg = block % W::NGROUPS;
  const int wm = wave / C::WN, wn = wave % C::WN;
  const int per = cdiv(B, nslices);
  const int b_lo = slice * per, b_hi = min(B, b_lo + per);

  f32x4 acc[W::MTW][W::NTW];
#pragma unroll
  for (int i = 0; i < W::MTW; ++i)
#pragma unroll
    for (int j = 0; j < W::NTW; ++j) acc[i][j] = zero_f32x4();
  float bias_acc = 0.f;  // thread tid < COUT owns channel tid (tap group 0 only)

  const int g16 = lane & 15, grp = lane >> 4;
  const int q = g16 >> 2, p = g16 & 3;

  for (int b = b_lo; b < b_hi; ++b) {
    __syncthreads();
    constexpr int CG = G::COUT / 8;
    const int64_t pbase = (int64_t)b * G::PH * G::PH * G::COUT;
    for (int e = tid; e < W::KP * CG; e += kThreads) {
      const int pos = e / CG, cg = e % CG;
      bf16x8 v = zero_bf16x8();
      if (pos < W::NPOS) {
        float g[8];
        unpool_grad8<G::OH, G::PH, G::PS, G::COUT>(dout + pbase, idx + pbase, pooled + pbase,
                                                   pos / G::OH, pos % G::OH, cg * 8, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (bf16)g[j];
      }
      *reinterpret_cast<bf16x8*>(Ds + pos * W::D_RS + cg * 8) = v;
    }
    constexpr int XG = G::CIN / 8;
    const bf16* xb = x + (int64_t)b * G::IH * G::IH * G::CIN;
    for (int e = tid; e < G::IH * G::IH * XG; e += kThreads) {
      const int pos = e / XG, cg = e % XG;
      *reinterpret_cast<bf16x8*>(Xs + pos * W::X_RS + cg * 8) =
          *reinterpret_cast<const bf16x8*>(xb + pos * G::CIN + cg * 8);
    }
    __syncthreads();
    if (tg == 0 && tid < G::COUT) {
      float s = 0.f;
      for (int pos = 0; pos < W::NPOS; ++pos) s += (float)Ds[pos * W::D_RS + tid];
      bias_acc += s;
    }
    for (int ks = 0; ks < W::KS; ++ks) {
      const int kb = ks * 32 + grp * 8;  // this lane group's first k row
      // A fragments (d(conv)^T): rows k, columns co -> transposed reads.
      bf16x8 af[W::MTW];
#pragma unroll
      for (int i = 0; i < W::MTW; ++i) {
        const int m0 = (wm * W::MTW + i) * 16;
        const bf16x4 lo = lds_read_tr16(Ds + (kb + q) * W::D_RS + m0 + 4 * p);
        const bf16x4 hi = lds_read_tr16(Ds + (kb + 4 + q) * W::D_RS + m0 + 4 * p);
        af[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      // B rows: the X positions of k rows kb+q and kb+4+q (clamped; D is zero there).
      const int kr0 = min(kb + q, W::NPOS - 1), kr1 = min(kb + 4 + q, W::NPOS - 1);
      const int xr0 = (kr0 / G::OH) * G::IH + kr0 % G::OH;
      const int xr1 = (kr1 / G::OH) * G::IH + kr1 % G::OH;
#pragma unroll
      for (int j = 0; j < W::NTW; ++j) {
        const int n0 = (wn * W::NTW + j) * 16;           // column within this tap group
        const int tap = tg * C::TG + n0 / G::CIN, c0 = n0 % G::CIN;
        const int shift = (tap / 3) * G::IH + (tap % 3);
        const bf16x4 lo = lds_read_tr16(Xs + (xr0 + shift) * W::X_RS + c0 + 4 * p);
        const bf16x4 hi = lds_read_tr16(Xs + (xr1 + shift) * W::X_RS + c0 + 4 * p);
        const bf16x8 bf = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int i = 0; i < W::MTW; ++i) acc[i][j] = mfma16x16x32(af[i], bf, acc[i][j]);
      }
    }
  }
  // Write this slice's partial: slab[n][co] (co fastest) for n in this tap group.
  float* slab = slabs + (int64_t)slice * (W::NOUT + G::COUT);
#pragma unroll
  for (int i = 0; i < W::MTW; ++i) {
#pragma unroll
    for (int j = 0; j < W::NTW; ++j) {
      const int co = (wm * W::MTW + i) * 16 + (lane >> 4) * 4;
      const int n = tg * W::NCH + (wn * W::NTW + j) * 16 + g16;
      *reinterpret_cast<f32x4*>(slab + (int64_t)n * G::COUT + co) = acc[i][j];
    }
  }
  if (tg == 0 && tid < G::COUT) slab[W::NOUT + tid] = bias_acc;
}

// Fused backward launch: blocks [0, n_dgrad) compute the data gradient, the rest the weight
// gradient slabs (horizontal fusion: one launch, both read the same d(pooled)).
template <int L, int NSPLIT>
__global__ __launch_bounds__(kThreads) void conv_bwd_kernel(const bf16* __restrict__ in,
                                                            const float* __restrict__ w,
                                                            const bf16* __restrict__ dout,
                                                            const uint8_t* __restrict__ idx,
                                                            const bf16* __restrict__ pooled,
                                                            bf16* __restrict__ din, int B,
                                                            float* __restrict__ slabs,
                                                            int nslices, int n_dgrad) {
  constexpr int L1 = DgradCfg<L, NSPLIT>::LDS, L2 = WgradGeo<L>::LDS;
  __shared__ __attribute__((aligned(16))) char smem[L1 > L2 ? L1 : L2];
  if ((int)blockIdx.x < n_dgrad) {
    dgrad_body<L, NSPLIT>(smem, w, dout, idx, pooled, din, B, blockIdx.x, n_dgrad);
  } else {
    wgrad_body<L>(smem, in, dout, idx, pooled, slabs, B, nslices, blockIdx.x - n_dgrad);
  }
}

// Reduce slabs over slices (4 waves x quarter of the slices, fixed combine order) and scatter to
// the PyTorch weight layout [co][ci][kh][kw] + bias.
template <int L>
__global__ __launch_bounds__(kThreads) void conv_wgrad_reduce_kernel(const float* __restrict__ slabs,
                                                                     int nslices,
                                                                     float* __restrict__ dw,
                                                                     float* __restrict__ db) {
  using G = Geo<L>;
  using W = WgradGeo<L>;
  constexpr int SL = W::NOUT + G::COUT;
  __shared__ float part[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  float a0 = 0.f, a1 = 0.f;
  if (i < SL) {
    const float* p = slabs + i;
    int k = wave;
    for (; k + 4 < nslices; k += 8) {
      a0 += p[(int64_t)k * SL];
      a1 += p[(int64_t)(k + 4) * SL];
    }
    for (; k < nslices; k += 4) a0 += p[(int64_t)k * SL];
  }
  part[wave][lane] = a0 + a1;
  __syncthreads();
  if (wave != 0 || i >= SL) return;
  const float s = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
  if (i < W::NOUT) {
    const int n = i / G::COUT, co = i % G::COUT;
    const int tap = n / G::CIN, ci = n % G::CIN;
    dw[(co * G::CIN + ci) * 9 + tap] = s;
  } else {
    db[i - W::NOUT] = s;
  }
}

// ------------------------------------------------------------------ conv1 wgrad (MFMA)
// dW1[co][t] = sum_{b, y, x} Dc[b][y][x][co] * xpad[b][y + kh][x + kw], t = kh*5 + kw.
// K rows = (y, x) with x padded to 32 per row (26 valid); A = Dc^T staged [co][y*32+x];
// B[k][n=t] read from per-kw shifted copies of the input rows (aligned 16-byte reads).
constexpr int C1_KROW = 32;
constexpr int C1_K = 26 * C1_KROW;       // 832 = 26 k-steps
constexpr int C1_DT_RS = C1_K + 8;       // bf16 per co row
constexpr int C1_XS_RS = 40;             // bf16 per shifted input row (>= 32 + 8)
constexpr int C1_DT_BYTES = align16(32 * C1_DT_RS * 2);
constexpr int C1_XS_BYTES = align16(5 * 30 * C1_XS_RS * 2);
constexpr int C1_NOUT = 32 * 25;
constexpr int C1_SL = C1_NOUT + 32;

template <bool U8>
__global__ __launch_bounds__(kThreads) void conv1_wgrad_kernel(const void* __restrict__ xin,
                                                               const bf16* __restrict__ da1,
                                                               const uint8_t* __restrict__ idx1,
                                                               const bf16* __restrict__ a1, int B,
                                                               float mean, float inv_std,
                                                               float in_scale,
                                                               float* __restrict__ slabs,
                                                               int nslices) {
  __shared__ __attribute__((aligned(16))) char smem[C1_DT_BYTES + C1_XS_BYTES];
  bf16* Dt = reinterpret_cast<bf16*>(smem);
  bf16* Xs = reinterpret_cast<bf16*>(smem + C1_DT_BYTES);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int per = cdiv(B, nslices);
  const int b_lo = blockIdx.x * per, b_hi = min(B, b_lo + per);
  // Wave (mt, nt): co tile mt (0..1), tap tile nt (0..1: taps 0-15, 16-31 with 25.. = 0).
  const int mt = wave >> 1, nt = wave & 1;
  f32x4 acc = zero_f32x4();
  float bias_acc = 0.f;
  const int r16 = lane & 15, q8 = (lane >> 4) * 8;
  const int t = nt * 16 + r16;  // this lane's B column (tap)
  const bool tvalid = t < 25;
  const int kh = tvalid ? t / 5 : 0, kw = tvalid ? t % 5 : 0;

  for (int b = b_lo; b < b_hi; ++b) {
    __syncthreads();
    // Zero the transposed d(conv) image, then scatter the pooled gradients.
    for (int e = tid; e < 32 * C1_DT_RS / 8; e += kThreads)
      reinterpret_cast<bf16x8*>(Dt)[e] = zero_bf16x8();
    // Shifted input copies: Xs[kw][r][c] = xpad[r][c + kw], xpad = normalised input, ring of 1.
    for (int e = tid; e < 5 * 30 * 32; e += kThreads) {
      const int s = e / (30 * 32), rc = e % (30 * 32), r = rc / 32, c = rc % 32;
      const int yy = r - 1, xx = c + s - 1;
      float v = 0.f;
      if (yy >= 0 && yy < 28 && xx >= 0 && xx < 28) {
        const int64_t o = (int64_t)b * 784 + yy * 28 + xx;
        const float raw = U8 ? (float)static_cast<const uint8_t*>(xin)[o] * in_scale
                             : static_cast<const float*>(xin)[o];
        v = (raw - mean) * inv_std;
      }
      Xs[(s * 30 + r) * C1_XS_RS + c] = (bf16)v;
    }
    __syncthreads();
    for (int e = tid; e < 169 * 32; e += kThreads) {
      const int pp = e / 32, co = e % 32;
      const int64_t o = ((int64_t)b * 169 + pp) * 32 + co;
      const float pv = (float)a1[o];
      const float g = pv > 0.f ? (float)da1[o] : 0.f;
      const int i = idx1[o];
      const int y = (pp / 13) * 2 + (i >> 1), x = (pp % 13) * 2 + (i & 1);
      Dt[co * C1_DT_RS + y * C1_KROW + x] = (bf16)g;
    }
    __syncthreads();
    if (tid < 32) {
      float s = 0.f;
      for (int k = 0; k < C1_K; ++k) s += (float)Dt[tid * C1_DT_RS + k];
      bias_acc += s;
    }
    for (int ks = 0; ks < 26; ++ks) {
      const int y = ks;  // one padded row of 32 positions per k-step
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(Dt + (mt * 16 + r16) * C1_DT_RS + ks * 32 + q8);
      bf16x8 bf = zero_bf16x8();
      if (tvalid) bf = *reinterpret_cast<const bf16x8*>(Xs + (kw * 30 + y + kh) * C1_XS_RS + q8);
      acc = mfma16x16x32(af, bf, acc);
    }
  }
  float* slab = slabs + (int64_t)blockIdx.x * C1_SL;
  // C layout: col = tap (lane & 15), rows = co (lane >> 4)*4 + i.
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int co = mt * 16 + (lane >> 4) * 4 + i;
    if (tvalid) slab[co * 25 + t] = acc[i];
  }
  if (tid < 32) slab[C1_NOUT + tid] = bias_acc;
}

// ------------------------------------------------------------------ fc (2048 -> 10)
// Activation k' = pos*128 + c (NHWC), weight column k = c*16 + pos (PyTorch CHW flatten).
constexpr int FC_K = 2048, FC_N = 10;
__device__ __forceinline__ int fc_wcol(int kp) { return (kp & 127) * 16 + (kp >> 7); }

// One wave per image; W staged once per workgroup in LDS (fp32, activation order).
__global__ __launch_bounds__(kThreads) void fc_fwd_kernel(const bf16* __restrict__ a3,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ bias,
                                                          float* __restrict__ logits, int B) {
  __shared__ __attribute__((aligned(16))) float Ws[FC_N * FC_K];
  for (int e = threadIdx.x; e < FC_N * FC_K; e += kThreads) {
    const int n = e / FC_K, kp = e % FC_K;
    Ws[e] = w[n * FC_K + fc_wcol(kp)];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int b = blockIdx.x * 4 + wave; b < B; b += gridDim.x * 4) {
    float s[FC_N];
#pragma unroll
    for (int n = 0; n < FC_N; ++n) s[n] = 0.f;
    const bf16* xb = a3 + (int64_t)b * FC_K;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kp = j * 512 + lane * 8;
      const bf16x8 xv = *reinterpret_cast<const bf16x8*>(xb + kp);
#pragma unroll
      for (int n = 0; n < FC_N; ++n) {
        const float4 w0 = *reinterpret_cast<const float4*>(Ws + n * FC_K + kp);
        const float4 w1 = *reinterpret_cast<const float4*>(Ws + n * FC_K + kp + 4);
        s[n] += (float)xv[0] * w0.x + (float)xv[1] * w0.y + (float)xv[2] * w0.z +
                (float)xv[3] * w0.w + (float)xv[4] * w1.x + (float)xv[5] * w1.y +
                (float)xv[6] * w1.z + (float)xv[7] * w1.w;
      }
    }
#pragma unroll
    for (int n = 0; n < FC_N; ++n) s[n] = wave_sum(s[n]);
    if (lane < FC_N) {
      float v = 0.f;
#pragma unroll
      for (int n = 0; n < FC_N; ++n)
        if (n == lane) v = s[n];
      logits[(int64_t)b * FC_N + lane] = v + bias[lane];
    }
  }
}

// Each thread owns 8 activation columns: da3 for those columns per image, and dW partials
// (80 accumulators) over this slice's images.  Slab: [N*K in PyTorch order][N bias].
__global__ __launch_bounds__(kThreads) void fc_bwd_kernel(const bf16* __restrict__ a3,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ dlogits,
                                                          bf16* __restrict__ da3, int B,
                                                          float* __restrict__ slabs, int nslices) {
  const int kp0 = threadIdx.x * 8;
  float wr[FC_N][8];
#pragma unroll
  for (int n = 0; n < FC_N; ++n)
#pragma unroll
    for (int j = 0; j < 8; ++j) wr[n][j] = w[n * FC_K + fc_wcol(kp0 + j)];
  float acc[FC_N][8];
#pragma unroll
  for (int n = 0; n < FC_N; ++n)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[n][j] = 0.f;
  float bacc = 0.f;
  const int per = cdiv(B, nslices);
  const int b_lo = blockIdx.x * per, b_hi = min(B, b_lo + per);
  for (int b = b_lo; b < b_hi; ++b) {
    float dl[FC_N];
#pragma unroll
    for (int n = 0; n < FC_N; ++n) dl[n] = dlogits[(int64_t)b * FC_N + n];
    const bf16x8 xv = *reinterpret_cast<const bf16x8*>(a3 + (int64_t)b * FC_K + kp0);
    bf16x8 dv;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s = 0.f;
#pragma unroll
      for (int n = 0; n < FC_N; ++n) {
        s = fmaf(dl[n], wr[n][j], s);
        acc[n][j] = fmaf(dl[n], (float)xv[j], acc[n][j]);
      }
      dv[j] = (bf16)s;
    }
    *reinterpret_cast<bf16x8*>(da3 + (int64_t)b * FC_K + kp0) = dv;
    if (threadIdx.x < FC_N) bacc += dl[threadIdx.x];
  }
  float* slab = slabs + (int64_t)blockIdx.x * (FC_N * FC_K + FC_N);
#pragma unroll
  for (int n = 0; n < FC_N; ++n)
#pragma unroll
    for (int j = 0; j < 8; ++j) slab[n * FC_K + fc_wcol(kp0 + j)] = acc[n][j];
  if (threadIdx.x < FC_N) slab[FC_N * FC_K + threadIdx.x] = bacc;
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

// Number of weight-gradient slices (images split across workgroups).
inline int wgrad_slices(int B, int images_per_slice_min, int cap) {
  return clampi(cdiv(B, images_per_slice_min), 1, cap);
}

}  // namespace

namespace {
// Deterministic split-K reduction, parallel over slices: a workgroup owns 64 consecutive outputs;
// its 4 waves each sum a quarter of the slices (lane = output, fully coalesced 256-B rows), 4-way
// unrolled for memory-level parallelism; the 4 partials are combined in a fixed order in LDS.
// out[i] = sum_s slabs[s * stride + off + i],  i < n.
__global__ __launch_bounds__(kThreads) void strided_reduce_kernel(const float* __restrict__ slabs,
                                                                  int S, int64_t stride,
                                                                  int64_t off, int64_t n,
                                                                  float* __restrict__ out) {
  __shared__ float part[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + lane;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (i < n) {
    const float* p = slabs + off + i;
    int s = wave;
    for (; s + 12 < S; s += 16) {
      a0 += p[(int64_t)s * stride];
      a1 += p[(int64_t)(s + 4) * stride];
      a2 += p[(int64_t)(s + 8) * stride];
      a3 += p[(int64_t)(s + 12) * stride];
    }
    for (; s < S; s += 4) a0 += p[(int64_t)s * stride];
  }
  part[wave][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (wave == 0 && i < n) out[i] = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
}
}  // namespace

void strided_reduce(const float* slabs, int S, int64_t stride, int64_t off, int64_t n, float* out,
                    hipStream_t s) {
  const int grid = (int)((n + 63) / 64);
  strided_reduce_kernel<<<grid, kThreads, 0, s>>>(slabs, S, stride, off, n, out);
}

// ================================================================== launchers
void convnet_conv1_fwd(const void* x, bool x_is_u8, const float* w, const float* b, void* a1,
                       uint8_t* idx1, int B, float mean, float inv_std, float in_scale,
                       hipStream_t s) {
  const int grid = clampi(B, 1, 8 * num_cus());
  if (x_is_u8)
    conv1_fwd_kernel<true><<<grid, kThreads, 0, s>>>(x, w, b, static_cast<bf16*>(a1), idx1, B, mean,
                                                     inv_std, in_scale);
  else
    conv1_fwd_kernel<false><<<grid, kThreads, 0, s>>>(x, w, b, static_cast<bf16*>(a1), idx1, B, mean,
                                                      inv_std, in_scale);
}

int64_t convnet_conv1_wgrad_slab_floats(int B, int* nslices) {
  const int S = wgrad_slices(B, 4, 2 * num_cus());
  if (nslices) *nslices = S;
  return (int64_t)S * C1_SL;
}

void convnet_conv1_wgrad(const void* x, bool x_is_u8, const void* da1, const uint8_t* idx1,
                         const void* a1, int B, float mean, float inv_std, float in_scale,
                         float* slabs, int nslices, float* dw, float* db, hipStream_t s) {
  if (x_is_u8)
    conv1_wgrad_kernel<true><<<nslices, kThreads, 0, s>>>(x, static_cast<const bf16*>(da1), idx1,
                                                          static_cast<const bf16*>(a1), B, mean,
                                                          inv_std, in_scale, slabs, nslices);
  else
    conv1_wgrad_kernel<false><<<nslices, kThreads, 0, s>>>(x, static_cast<const bf16*>(da1), idx1,
                                                           static_cast<const bf16*>(a1), B, mean,
                                                           inv_std, in_scale, slabs, nslices);
  // Slab order == PyTorch [co][1][kh][kw], bias follows: two strided fixed-order reductions.
  strided_reduce(slabs, nslices, C1_SL, 0, C1_NOUT, dw, s);
  strided_reduce(slabs, nslices, C1_SL, C1_NOUT, 32, db, s);
}

namespace {
template <int L>
inline int fwd_nsplit(int B) {
  if (L == 2) return B >= 2048 ? 1 : (B >= 512 ? 2 : 4);
  return B >= 1024 ? 2 : 4;
}
template <int L, int NS>
void launch_fwd(const void* in, const float* w, const float* b, void* out, uint8_t* idx, int B,
                hipStream_t s) {
  const int groups = clampi(B, 1, cdiv(4 * num_cus(), NS));
  conv_fwd_kernel<L, NS><<<groups * NS, kThreads, 0, s>>>(static_cast<const bf16*>(in), w, b,
                                                          static_cast<bf16*>(out), idx, B);
}
template <int L>
constexpr int bwd_nsplit() {
  return L == 2 ? 2 : 4;
}
}  // namespace

void convnet_conv_fwd(int layer, const void* in, const float* w, const float* b, void* out,
                      uint8_t* idx, int B, hipStream_t s) {
  if (layer == 2) {
    const int ns = fwd_nsplit<2>(B);
    if (ns == 1) launch_fwd<2, 1>(in, w, b, out, idx, B, s);
    else if (ns == 2) launch_fwd<2, 2>(in, w, b, out, idx, B, s);
    else launch_fwd<2, 4>(in, w, b, out, idx, B, s);
  } else {
    const int ns = fwd_nsplit<3>(B);
    if (ns == 2) launch_fwd<3, 2>(in, w, b, out, idx, B, s);
    else launch_fwd<3, 4>(in, w, b, out, idx, B, s);
  }
}

int64_t convnet_conv_wgrad_slab_floats(int layer, int B, int* nslices) {
  int S;
  int64_t per;
  if (layer == 2) {
    S = wgrad_slices(B, 2, 2 * num_cus());
    per = WgradGeo<2>::NOUT + Geo<2>::COUT;
  } else {
    S = wgrad_slices(B, 4, (2 * num_cus()) / WgradGeo<3>::NGROUPS);
    per = WgradGeo<3>::NOUT + Geo<3>::COUT;
  }
  if (nslices) *nslices = S;
  return (int64_t)S * per;
}

void convnet_conv_bwd(int layer, const void* in, const float* w, const void* dout,
                      const uint8_t* idx, const void* out, void* din, int B, float* slabs,
                      int nslices, float* dw, float* db, hipStream_t s) {
  const bf16* inb = static_cast<const bf16*>(in);
  const bf16* doutb = static_cast<const bf16*>(dout);
  const bf16* outb = static_cast<const bf16*>(out);
  bf16* dinb = static_cast<bf16*>(din);
  if (layer == 2) {
    constexpr int NS = bwd_nsplit<2>();
    const int n_dgrad = din ? clampi(B, 1, cdiv(4 * num_cus(), NS)) * NS : 0;
    const int n_w = nslices * WgradGeo<2>::NGROUPS;
    conv_bwd_kernel<2, NS><<<n_dgrad + n_w, kThreads, 0, s>>>(inb, w, doutb, idx, outb, dinb, B,
                                                             slabs, nslices, n_dgrad);
    constexpr int SL = WgradGeo<2>::NOUT + Geo<2>::COUT;
    conv_wgrad_reduce_kernel<2><<<cdiv(SL, 64), kThreads, 0, s>>>(slabs, nslices, dw, db);
  } else {
    constexpr int NS = bwd_nsplit<3>();
    const int n_dgrad = din ? clampi(B, 1, cdiv(4 * num_cus(), NS)) * NS : 0;
    const int n_w = nslices * WgradGeo<3>::NGROUPS;
    conv_bwd_kernel<3, NS><<<n_dgrad + n_w, kThreads, 0, s>>>(inb, w, doutb, idx, outb, dinb, B,
                                                             slabs, nslices, n_dgrad);
    constexpr int SL = WgradGeo<3>::NOUT + Geo<3>::COUT;
    conv_wgrad_reduce_kernel<3><<<cdiv(SL, 64), kThreads, 0, s>>>(slabs, nslices, dw, db);
  }
}

void convnet_fc_fwd(const void* a3, const float* w, const float* b, float* logits, int B,
                    hipStream_t s) {
  const int grid = clampi(cdiv(B, 4), 1, num_cus());
  fc_fwd_kernel<<<grid, kThreads, 0, s>>>(static_cast<const bf16*>(a3), w, b, logits, B);
}

int64_t convnet_fc_slab_floats(int B, int* nslices) {
  const int S = wgrad_slices(B, 8, 128);
  if (nslices) *nslices = S;
  return (int64_t)S * (FC_N * FC_K + FC_N);
}

void convnet_fc_bwd(const void* a3, const float* w, const float* dlogits, void* da3, int B,
                    float* slabs, int nslices, float* dw, float* db, hipStream_t s) {
  fc_bwd_kernel<<<nslices, kThreads, 0, s>>>(static_cast<const bf16*>(a3), w, dlogits,
                                             static_cast<bf16*>(da3), B, slabs, nslices);
  constexpr int SL = FC_N * FC_K + FC_N;
  strided_reduce(slabs, nslices, SL, 0, FC_N * FC_K, dw, s);
  strided_reduce(slabs, nslices, SL, FC_N * FC_K, FC_N, db, s);
}

}  // namespace kern
}  // namespace ringdp
