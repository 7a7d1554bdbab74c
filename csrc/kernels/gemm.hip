// Generic bf16 MFMA GEMM core for CDNA4 (gfx950) with gather loaders and fused epilogues.
//
// Serves the deep-model families of BASELINE.json (ResNet-18/50 convolutions as implicit GEMM,
// ViT-B/16 linear layers and attention batches; SURVEY.md §2.4 U14 "cuDNN conv / cuBLAS addmm").
//
//   C[b][m][n] = epilogue( sum_k A(b, m, k) * B(b, n, k) )
//
// * Operands are described by LOADERS.  A loader is either K-contiguous (8 consecutive k of one
//   row per 16-B vector: dense row-major, NHWC im2col, transposed-conv gather) or ROW-contiguous
//   (8 consecutive rows of one k: dense column-major, the dY^T / im2col^T operands of a weight
//   gradient).  K-contiguous tiles are staged [row][k] and read with ds_read_b128; row-contiguous
//   tiles are staged [k][row] and read with ds_read_b64_tr_b16 - the transposed LDS read replaces
//   any explicit transpose pass.
// * 128x128 block tile, BK = 64, 256 threads = 2x2 waves of 64x64 (4x4 v_mfma_f32_16x16x32_bf16
//   tiles each), LDS double buffer with register-staged prefetch of the next k-tile (one barrier
//   per k-tile), XCD-aware block->tile mapping (blocks of one XCD walk the same A row-panel).
// * The MFMA is issued as C^T = B * A^T so every lane ends with 4 CONSECUTIVE n of one m: the
//   epilogue stores 8-byte (bf16) / 16-byte (fp32) runs, applies bias / ReLU / GELU / residual,
//   optionally keeps the pre-activation, and emits deterministic per-channel sum / sum-of-squares
//   partials (batch-norm statistics) or split-K fp32 partials.
#include <algorithm>
#include <cstdio>
#include <type_traits>

#include "device_common.h"
#include "gemm256_epilogue.h"
#include "kernels.h"

namespace ringdp {
namespace kern {

using namespace ringdp::dev;

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
// Stage images are unpadded and XOR-swizzled (modelled with tools/lds_bank_model.py; the previous
// 8-element row padding cost 2x on both fragment reads and needed 9 KiB more LDS; measured +3-5 %):
//  * K-contiguous [128 rows][64 k]: 16-B chunk c of row r lives at chunk c ^ (r & 7), so the 16 rows of a
//    ds_read_b128 lane group cover 16 distinct bank slots (8 -> 4 LDS cycles per read);
//  * row-contiguous [64 k][128 rows]: 32-B slot s of k-row R lives at slot s ^ f(R), f(R) = (R & 3) |
//    ((R >> 1) & 4), so the 8 k-rows of a ds_read_b64_tr_b16 32-lane half (R..R+3, R+8..R+11) cover the
//    8 slots of a 256-B bank row once (4 -> 2 cycles).
// (A 2-tile-deep register prefetch was tried on top: +32 VGPRs, no measurable gain - the loop is not
// waiting on global latency at 2 workgroups per CU.)
constexpr int KROW = BK;     // K-contiguous stage row (bf16)
constexpr int RROW = 128;    // row-contiguous stage row (bf16)
constexpr int STAGE_ELEMS = 128 * KROW;
static_assert(STAGE_ELEMS == BK * RROW, "stage size");
__device__ __forceinline__ int ksw(int r, int chunk) { return r * KROW + 8 * (chunk ^ (r & 7)); }
__device__ __forceinline__ int rsw(int kr, int col) {  // col: element column (multiple of 4)
  const int f = (kr & 3) | ((kr >> 1) & 4);
  return kr * RROW + (((col >> 4) ^ f) << 4) + (col & 15);
}

// GELU (erf form) and its derivative on the branch-free erf of gemm256_epilogue.h
__device__ __forceinline__ float gelu_erf(float x) { return gemm_gelu(x); }
__device__ __forceinline__ float gelu_grad(float x) { return gemm_gelu_grad(x); }  // d/dx of x * Phi(x)

// ------------------------------------------------------------------ loaders
struct DenseLoader {  // element (b, r, k): K-contig p[b*bs + r*ld + k]; row-contig p[b*bs + k*ld + r]
  const bf16* p;
  int64_t ld, bs;
  int R, K;
};

template <bool kRowContig>
struct Dense {
  static constexpr bool kRow = kRowContig;
  DenseLoader d;
  struct Row {
    const bf16* base;
    int r;
  };
  __device__ __forceinline__ Row row(int b, int r) const { return Row{d.p + (int64_t)b * d.bs, r}; }
  __device__ __forceinline__ bf16x8 load(const Row& rw, int k) const {
    if (rw.r >= d.R || k >= d.K) return zero_bf16x8();
    if (kRowContig) return *reinterpret_cast<const bf16x8*>(rw.base + (int64_t)k * d.ld + rw.r);
    return *reinterpret_cast<const bf16x8*>(rw.base + (int64_t)rw.r * d.ld + k);
  }
};

// Dense operand whose reduction length is a multiple of BK (every k-tile full): no per-vector bounds
// checks.  Out-of-range rows are clamped to the last row - their products only reach output rows /
// columns the epilogue drops.  The stager keeps one pointer per staged vector and steps it by a
// uniform offset per k-tile (the checked loader cost ~12 VALU per 16-B load: 2.8 VALU per MFMA at 4096^3).
template <bool kRowContig>
struct DenseAligned {
  static constexpr bool kRow = kRowContig;
  static constexpr int kKind = 1;
  DenseLoader d;
};

// im2col of an NHWC input for the forward conv: row m = (n, p, q), k = (r, s, c) - K-contiguous
struct ConvFwdA {
  static constexpr bool kRow = false;
  const bf16* x;
  ConvGeom g;
  int M, Kd;
  struct Row {
    const bf16* base;
    int h0, w0;
    bool ok;
  };
  __device__ __forceinline__ Row row(int, int m) const {
    if (m >= M) return Row{x, 0, 0, false};
    const int pq = g.P * g.Q;
    const int n = m / pq, rem = m - n * pq, p = rem / g.Q, q = rem - p * g.Q;
    return Row{x + (int64_t)n * g.H * g.W * g.C, p * g.stride - g.pad, q * g.stride - g.pad, true};
  }
  __device__ __forceinline__ bf16x8 load(const Row& rw, int k) const {
    if (!rw.ok || k >= Kd) return zero_bf16x8();
    const int rs = k / g.C, c = k - rs * g.C, r = rs / g.S, s = rs - r * g.S;
    const int h = rw.h0 + r * g.dil, w = rw.w0 + s * g.dil;
    if ((unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W) return zero_bf16x8();
    return *reinterpret_cast<const bf16x8*>(rw.base + ((int64_t)h * g.W + w) * g.C + c);
  }
};

// transposed-conv gather of dY for the data gradient: row m = (n, h, w) of the INPUT,
// k = (r, s, kout): dY[n][(h + pad - r*dil)/stride][(w + pad - s*dil)/stride][kout..] when exact
struct ConvDgradA {
  static constexpr bool kRow = false;
  const bf16* dy;
  ConvGeom g;
  int M, Kd;
  struct Row {
    const bf16* base;
    int hp, wp;
    bool ok;
  };
  __device__ __forceinline__ Row row(int, int m) const {
    if (m >= M) return Row{dy, 0, 0, false};
    const int hw = g.H * g.W;
    const int n = m / hw, rem = m - n * hw, h = rem / g.W, w = rem - h * g.W;
    return Row{dy + (int64_t)n * g.P * g.Q * g.K, h + g.pad, w + g.pad, true};
  }
  __device__ __forceinline__ bf16x8 load(const Row& rw, int k) const {
    if (!rw.ok || k >= Kd) return zero_bf16x8();
    const int rs = k / g.K, ko = k - rs * g.K, r = rs / g.S, s = rs - r * g.S;
    const int ph = rw.hp - r * g.dil, pw = rw.wp - s * g.dil;
    if (ph < 0 || pw < 0) return zero_bf16x8();
    const int p = ph / g.stride, q = pw / g.stride;
    if (p * g.stride != ph || q * g.stride != pw || p >= g.P || q >= g.Q) return zero_bf16x8();
    return *reinterpret_cast<const bf16x8*>(rw.base + ((int64_t)p * g.Q + q) * g.K + ko);
  }
};

// weight-gradient B operand: rows = filter taps kk = (r, s, c), k = output position m = (n, p, q):
// element = x[n][p*stride - pad + r*dil][q*stride - pad + s*dil][c]; 8 consecutive kk = 8 channels
struct ConvWgradB {
  static constexpr bool kRow = true;
  const bf16* x;
  ConvGeom g;
  int Mpos, Kd;  // Mpos = N*P*Q (the GEMM's K), Kd = R*S*C (rows)
  struct Row {
    int roff, soff, c;
    bool ok;
  };
  __device__ __forceinline__ Row row(int, int kk) const {
    if (kk >= Kd) return Row{0, 0, 0, false};
    const int rs = kk / g.C, c = kk - rs * g.C, r = rs / g.S, s = rs - r * g.S;
    return Row{r * g.dil - g.pad, s * g.dil - g.pad, c, true};
  }
  __device__ __forceinline__ bf16x8 load(const Row& rw, int m) const {
    if (!rw.ok || m >= Mpos) return zero_bf16x8();
    const int pq = g.P * g.Q;
    const int n = m / pq, rem = m - n * pq, p = rem / g.Q, q = rem - p * g.Q;
    const int h = p * g.stride + rw.roff, w = q * g.stride + rw.soff;
    if ((unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W) return zero_bf16x8();
    return *reinterpret_cast<const bf16x8*>(x + (((int64_t)n * g.H + h) * g.W + w) * g.C + rw.c);
  }
};

// ------------------------------------------------------------------ stage helpers
// K-contiguous operand: tile [128 rows][64 k] = 1024 vectors; thread t owns rows (t>>3) + 32i and
// the k-vector (t & 7).  Row-contiguous: tile [64 k][128 rows]; thread t owns the row-vector (t & 15)
// and k = (t >> 4) + 16i.
template <class L, class = void>
struct loader_kind : std::integral_constant<int, 0> {};
template <class L>
struct loader_kind<L, std::void_t<decltype(L::kKind)>> : std::integral_constant<int, L::kKind> {};

template <class L, class = void>
struct StagerRows {  // checked loaders: row descriptors
  typename L::Row rows[4];
  __device__ __forceinline__ void init(const L& ld, int b, int tile_r0, int tid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (L::kRow)
        rows[i] = ld.row(b, tile_r0 + 8 * (tid & 15));
      else
        rows[i] = ld.row(b, tile_r0 + (tid >> 3) + 32 * i);
    }
  }
  __device__ __forceinline__ bf16x8 get(const L& ld, int i, int k0, int tid) const {
    if (L::kRow) return ld.load(rows[0], k0 + (tid >> 4) + 16 * i);
    return ld.load(rows[i], k0 + 8 * (tid & 7));
  }
};
template <class L>
struct StagerRows<L, std::enable_if_t<loader_kind<L>::value == 1>> {  // aligned dense: per-vector pointers
  const bf16* ptr[4];
  int64_t kstep;  // elements per unit of k
  __device__ __forceinline__ void init(const L& ld, int b, int tile_r0, int tid) {
    const bf16* base = ld.d.p + (int64_t)b * ld.d.bs;
    if (L::kRow) {
      const int r = min(tile_r0 + 8 * (tid & 15), ld.d.R - 8);
#pragma unroll
      for (int i = 0; i < 4; ++i) ptr[i] = base + (int64_t)((tid >> 4) + 16 * i) * ld.d.ld + r;
      kstep = ld.d.ld;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = min(tile_r0 + (tid >> 3) + 32 * i, ld.d.R - 1);
        ptr[i] = base + (int64_t)r * ld.d.ld + 8 * (tid & 7);
      }
      kstep = 1;
    }
  }
  __device__ __forceinline__ bf16x8 get(const L&, int i, int k0, int) const {
    return *reinterpret_cast<const bf16x8*>(ptr[i] + (int64_t)k0 * kstep);
  }
};

// Implicit-GEMM conv forward with C % 64 == 0: a 64-wide k-tile lies inside one filter tap, so the tap
// (r, s) and channel base are computed once per k-tile from the uniform k0 (scalar ALU) instead of two
// integer divisions per 16-B load; each staged row keeps its image pointer and input origin.
struct ConvFwdA64 {
  static constexpr bool kRow = false;
  static constexpr int kKind = 2;
  const bf16* x;
  ConvGeom g;
  int M, Kd;
};
template <class L>
struct StagerRows<L, std::enable_if_t<loader_kind<L>::value == 2>> {
  const bf16* base[4];
  int h0[4], w0[4];
  __device__ __forceinline__ void init(const L& ld, int, int tile_r0, int tid) {
    const ConvGeom& g = ld.g;
    const int pq = g.P * g.Q;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = tile_r0 + (tid >> 3) + 32 * i;
      if (m < ld.M) {
        const int n = m / pq, rem = m - n * pq, p = rem / g.Q, q = rem - p * g.Q;
        base[i] = ld.x + (int64_t)n * g.H * g.W * g.C + 8 * (tid & 7);
        h0[i] = p * g.stride - g.pad;
        w0[i] = q * g.stride - g.pad;
      } else {
        base[i] = ld.x;
        h0[i] = -(1 << 20);  // always out of bounds -> zero
        w0[i] = 0;
      }
    }
  }
  __device__ __forceinline__ bf16x8 get(const L& ld, int i, int k0, int) const {
    const ConvGeom& g = ld.g;
    const int rs = k0 / g.C, c0 = k0 - rs * g.C, r = rs / g.S, sx = rs - r * g.S;  // uniform
    const int h = h0[i] + r * g.dil, w = w0[i] + sx * g.dil;
    if ((unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W) return zero_bf16x8();
    return *reinterpret_cast<const bf16x8*>(base[i] + ((int64_t)h * g.W + w) * g.C + c0);
  }
};

// Implicit-GEMM conv forward with C == 8 (the ResNet stem: RGB padded to 8 channels): one 16-B vector is
// one whole filter tap, so a 64-wide k-tile holds 8 taps; the k-range R*S*8 is padded to whole k-tiles
// (taps >= R*S read zeros, the packed weight rows carry a zero tail, ldw % 64 == 0).  The checked ConvFwdA
// path ran the 7x7 stem at 30 TFLOP/s (two integer divisions and bounds checks per vector, no aligned B).
struct ConvFwdA8 {
  static constexpr bool kRow = false;
  static constexpr int kKind = 4;
  const bf16* x;
  ConvGeom g;
  int M, Kd;
};
template <class L>
struct StagerRows<L, std::enable_if_t<loader_kind<L>::value == 4>> {
  const bf16* base[4];
  int h0[4], w0[4];
  __device__ __forceinline__ void init(const L& ld, int, int tile_r0, int tid) {
    const ConvGeom& g = ld.g;
    const int pq = g.P * g.Q;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = tile_r0 + (tid >> 3) + 32 * i;
      if (m < ld.M) {
        const int n = m / pq, rem = m - n * pq, p = rem / g.Q, q = rem - p * g.Q;
        base[i] = ld.x + (int64_t)n * g.H * g.W * 8;
        h0[i] = p * g.stride - g.pad;
        w0[i] = q * g.stride - g.pad;
      } else {
        base[i] = ld.x;
        h0[i] = -(1 << 20);
        w0[i] = 0;
      }
    }
  }
  __device__ __forceinline__ bf16x8 get(const L& ld, int i, int k0, int tid) const {
    const ConvGeom& g = ld.g;
    const int t = (k0 >> 3) + (tid & 7);  // this vector's tap
    const int r = t / g.S, sx = t - r * g.S;
    const int h = h0[i] + r * g.dil, w = w0[i] + sx * g.dil;
    if (t >= g.R * g.S || (unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W) return zero_bf16x8();
    return *reinterpret_cast<const bf16x8*>(base[i] + ((int64_t)h * g.W + w) * 8);
  }
};

// Transposed-conv gather of dY (data gradient) with K % 64 == 0: tap and output-channel base per k-tile.
struct ConvDgradA64 {
  static constexpr bool kRow = false;
  static constexpr int kKind = 3;
  const bf16* dy;
  ConvGeom g;
  int M, Kd;
};
template <class L>
struct StagerRows<L, std::enable_if_t<loader_kind<L>::value == 3>> {
  const bf16* base[4];
  int hp[4], wp[4];
  __device__ __forceinline__ void init(const L& ld, int, int tile_r0, int tid) {
    const ConvGeom& g = ld.g;
    const int hw = g.H * g.W;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = tile_r0 + (tid >> 3) + 32 * i;
      if (m < ld.M) {
        const int n = m / hw, rem = m - n * hw, h = rem / g.W, w = rem - h * g.W;
        base[i] = ld.dy + (int64_t)n * g.P * g.Q * g.K + 8 * (tid & 7);
        hp[i] = h + g.pad;
        wp[i] = w + g.pad;
      } else {
        base[i] = ld.dy;
        hp[i] = -(1 << 20);
        wp[i] = 0;
      }
    }
  }
  __device__ __forceinline__ bf16x8 get(const L& ld, int i, int k0, int) const {
    const ConvGeom& g = ld.g;
    const int rs = k0 / g.K, ko = k0 - rs * g.K, r = rs / g.S, sx = rs - r * g.S;  // uniform
    const int ph = hp[i] - r * g.dil, pw = wp[i] - sx * g.dil;
    if (ph < 0 || pw < 0) return zero_bf16x8();
    const int p = ph / g.stride, q = pw / g.stride;
    if (p * g.stride != ph || q * g.stride != pw || p >= g.P || q >= g.Q) return zero_bf16x8();
    return *reinterpret_cast<const bf16x8*>(base[i] + ((int64_t)p * g.Q + q) * g.K + ko);
  }
};

// Stride-2 data gradient by input-pixel parity class (batch index b = 2*(h&1) + (w&1)): a class's input
// pixels receive gradient only from the taps r = r0 + 2t (r0 = (ph + pad) & 1) and likewise s, so each
// class is a dense GEMM over its own taps - 1/4 of the gather form's MFMA work, which multiplies zeros
// for 3 of every 4 (pixel, tap) pairs.  K % 64 == 0 (a k-tile is inside one tap); rows of a class are
// (n, i, j) with h = 2i + ph, w = 2j + pw, written back to dX through out_row().
struct S2Class {
  int r0, s0, nr, ns, dh, dw, Hc, Wc;
};
__device__ __forceinline__ S2Class s2_class(const ConvGeom& g, int b) {
  S2Class c;
  const int ph = b >> 1, pw = b & 1;
  c.r0 = (ph + g.pad) & 1;
  c.s0 = (pw + g.pad) & 1;
  c.nr = max(0, (g.R - c.r0 + 1) / 2);
  c.ns = max(0, (g.S - c.s0 + 1) / 2);
  c.dh = (ph + g.pad - c.r0) / 2;
  c.dw = (pw + g.pad - c.s0) / 2;
  c.Hc = (g.H - ph + 1) / 2;
  c.Wc = (g.W - pw + 1) / 2;
  return c;
}
struct ConvDgradS2A {
  static constexpr bool kRow = false;
  static constexpr int kKind = 5;
  const bf16* dy;
  ConvGeom g;
  __device__ __forceinline__ int kext(int b) const {
    const S2Class c = s2_class(g, b);
    return c.nr * c.ns * g.K;
  }
  __device__ __forceinline__ int mext(int b) const {
    const S2Class c = s2_class(g, b);
    return g.N * c.Hc * c.Wc;
  }
  __device__ __forceinline__ int64_t out_row(int b, int m) const {  // dX row (n, h, w) of class row m
    const S2Class c = s2_class(g, b);
    const int hw = c.Hc * c.Wc;
    const int n = m / hw, rem = m - n * hw, i = rem / c.Wc, j = rem - i * c.Wc;
    return ((int64_t)n * g.H + 2 * i + (b >> 1)) * g.W + 2 * j + (b & 1);
  }
};
template <class L>
struct StagerRows<L, std::enable_if_t<loader_kind<L>::value == 5>> {
  const bf16* base[4];
  int pi[4], qj[4];
  int ns;
  __device__ __forceinline__ void init(const L& ld, int b, int tile_r0, int tid) {
    const ConvGeom& g = ld.g;
    const S2Class c = s2_class(g, b);
    ns = max(1, c.ns);
    const int hw = c.Hc * c.Wc, mc = g.N * hw;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = tile_r0 + (tid >> 3) + 32 * i;
      if (m < mc) {
        const int n = m / hw, rem = m - n * hw, ii = rem / c.Wc, jj = rem - ii * c.Wc;
        base[i] = ld.dy + (int64_t)n * g.P * g.Q * g.K + 8 * (tid & 7);
        pi[i] = ii + c.dh;
        qj[i] = jj + c.dw;
      } else {
        base[i] = ld.dy;
        pi[i] = -(1 << 20);
        qj[i] = 0;
      }
    }
  }
  __device__ __forceinline__ bf16x8 get(const L& ld, int i, int k0, int) const {
    const ConvGeom& g = ld.g;
    const int t = k0 / g.K, ko = k0 - t * g.K, tr = t / ns, ts = t - tr * ns;  // uniform
    const int p = pi[i] - tr, q = qj[i] - ts;
    if ((unsigned)p >= (unsigned)g.P || (unsigned)q >= (unsigned)g.Q) return zero_bf16x8();
    return *reinterpret_cast<const bf16x8*>(base[i] + ((int64_t)p * g.Q + q) * g.K + ko);
  }
};
// B of the parity-class dgrad: W as CRSK, row c, class k = (tr, ts, ko) -> tap (r0 + 2 tr, s0 + 2 ts)
struct ConvDgradS2B {
  static constexpr bool kRow = false;
  static constexpr int kKind = 6;
  const bf16* w_crsk;
  ConvGeom g;
};
template <class L>
struct StagerRows<L, std::enable_if_t<loader_kind<L>::value == 6>> {
  const bf16* ptr[4];
  int r0, s0, ns;
  __device__ __forceinline__ void init(const L& ld, int b, int tile_r0, int tid) {
    const ConvGeom& g = ld.g;
    const S2Class c = s2_class(g, b);
    r0 = c.r0;
    s0 = c.s0;
    ns = max(1, c.ns);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = min(tile_r0 + (tid >> 3) + 32 * i, g.C - 1);  // rows past C: dropped columns
      ptr[i] = ld.w_crsk + (int64_t)r * g.R * g.S * g.K + 8 * (tid & 7);
    }
  }
  __device__ __forceinline__ bf16x8 get(const L& ld, int i, int k0, int) const {
    const ConvGeom& g = ld.g;
    const int t = k0 / g.K, ko = k0 - t * g.K, tr = t / ns, ts = t - tr * ns;  // uniform
    const int tap = (r0 + 2 * tr) * g.S + s0 + 2 * ts;
    return *reinterpret_cast<const bf16x8*>(ptr[i] + (int64_t)tap * g.K + ko);
  }
};
// per-batch reduction length / row count / output row (parity-class dgrad; identity otherwise)
template <class L>
__device__ __forceinline__ int k_extent(const L& l, int b, int K) {
  if constexpr (loader_kind<L>::value == 5) return min(K, l.kext(b));
  else return K;
}
template <class L>
__device__ __forceinline__ int m_extent(const L& l, int b, int M) {
  if constexpr (loader_kind<L>::value == 5) return min(M, l.mext(b));
  else return M;
}

template <class L>
struct Stager {
  StagerRows<L> rs;
  bf16x8 v[4];
  __device__ __forceinline__ void init(const L& ld, int b, int tile_r0, int tid) { rs.init(ld, b, tile_r0, tid); }
  __device__ __forceinline__ void load(const L& ld, int k0, int tid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = rs.get(ld, i, k0, tid);
  }
  __device__ __forceinline__ void store(bf16* s, int tid) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (L::kRow)
        *reinterpret_cast<bf16x8*>(s + rsw((tid >> 4) + 16 * i, 8 * (tid & 15))) = v[i];
      else
        *reinterpret_cast<bf16x8*>(s + ksw((tid >> 3) + 32 * i, tid & 7)) = v[i];
    }
  }
};

// MFMA operand fragment for rows r0..r0+15 at k-step kk (32-wide) from a staged tile.
template <bool kRow>
__device__ __forceinline__ bf16x8 frag(const bf16* s, int r0, int kk, int lane) {
  if (!kRow) return *reinterpret_cast<const bf16x8*>(s + ksw(r0 + (lane & 15), kk * 4 + (lane >> 4)));
  const int q = (lane & 15) >> 2, p = lane & 3, kb = kk * 32 + 8 * (lane >> 4);
  const bf16x4 lo = lds_read_tr16(s + rsw(kb + q, r0 + 4 * p));
  const bf16x4 hi = lds_read_tr16(s + rsw(kb + 4 + q, r0 + 4 * p));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// ------------------------------------------------------------------ the kernel
typedef int i32x8 __attribute__((ext_vector_type(8)));

// fp8 (e4m3, OCP) operand fragment for v_mfma_scale_f32_16x16x128_f8f6f4: lane l holds row l&15,
// k = 32*(l>>4) + j (j < 32) = 32 bytes = two 16-B reads of a K-contiguous stage.  In the stage,
// one bf16 "slot" is 2 fp8 bytes, so a 64-slot stage row is 128 fp8 values = one MFMA k-step.
__device__ __forceinline__ i32x8 frag_fp8(const bf16* s, int r0, int lane) {
  const int row = r0 + (lane & 15);
  const bf16x8 lo = *reinterpret_cast<const bf16x8*>(s + ksw(row, 2 * (lane >> 4)));
  const bf16x8 hi = *reinterpret_cast<const bf16x8*>(s + ksw(row, 2 * (lane >> 4) + 1));
  i32x8 r;
  const int* a = reinterpret_cast<const int*>(&lo);
  const int* b = reinterpret_cast<const int*>(&hi);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    r[i] = a[i];
    r[4 + i] = b[i];
  }
  return r;
}

template <class LA, class LB, bool kFp8 = false>
__global__ __launch_bounds__(256, 2) void gemm_kernel(LA la, LB lb, GemmEpilogue ep, int M, int N, int K,
                                                      int tiles_m, int tiles_n, int splits, int k_per_split) {
  __shared__ __attribute__((aligned(16))) bf16 smem[2][2][STAGE_ELEMS];  // [stage][A|B]
  __shared__ float red[2][2][BN];                                      // BN-stat cross-wave reduction
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // block -> (batch*split, tile_m, tile_n); tiles of one XCD walk one A row-panel
  const int per_z = tiles_m * tiles_n;
  const int zid = blockIdx.y;
  const int t = xcd_remap(blockIdx.x, per_z);
  const int tm = t / tiles_n, tn = t - tm * tiles_n;
  const int b = zid / splits, split = zid - b * splits;
  const int m0 = tm * BM, n0 = tn * BN;
  const int Kb = k_extent(la, b, K), Mb = m_extent(la, b, M);
  const int kbeg = split * k_per_split, kend = min(Kb, kbeg + k_per_split);
  const int nkt = max(0, (kend - kbeg + BK - 1) / BK);

  Stager<LA> sa;
  Stager<LB> sb;
  sa.init(la, b, m0, tid);
  sb.init(lb, b, n0, tid);
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = zero_f32x4();
  if (nkt > 0) {
    sa.load(la, kbeg, tid);
    sb.load(lb, kbeg, tid);
    sa.store(smem[0][0], tid);
    sb.store(smem[0][1], tid);
  }
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nkt;
    if (more) {
      sa.load(la, kbeg + (kt + 1) * BK, tid);
      sb.load(lb, kbeg + (kt + 1) * BK, tid);
    }
    const bf16* As = smem[cur][0];
    const bf16* Bs = smem[cur][1];
    if constexpr (kFp8) {
      static_assert(!LA::kRow && !LB::kRow, "fp8 GEMM: K-contiguous operands only");
      i32x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag_fp8(As, wm * 64 + 16 * i, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag_fp8(Bs, wn * 64 + 16 * j, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)  // e4m3 x e4m3, unit block scales (2^0 = e8m0 127): per-tensor scales in the epilogue
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fb[j], fa[i], acc[i][j], 0, 0, 0, 127, 0, 127);
    } else {
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        bf16x8 fa[4], fb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = frag<LA::kRow>(As, wm * 64 + 16 * i, kk, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[j] = frag<LB::kRow>(Bs, wn * 64 + 16 * j, kk, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma16x16x32(fb[j], fa[i], acc[i][j]);  // C^T tile
      }
    }
    if (more) {
      sa.store(smem[cur ^ 1][0], tid);
      sb.store(smem[cur ^ 1][1], tid);
    }
    __syncthreads();
  }

  // ---------------- epilogue: lane holds C[m][n..n+3], m = m0 + wm*64 + 16i + (lane&15),
  //                  n = n0 + wn*64 + 16j + 4*(lane>>4)
  const int mrow = m0 + wm * 64 + (lane & 15);
  const int ncol = n0 + wn * 64 + 4 * (lane >> 4);
  const float dscale = (ep.scale_a ? ep.scale_a[0] : 1.f) * (ep.scale_b ? ep.scale_b[0] : 1.f);
  if (dscale != 1.f) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] *= dscale;
  }
  if (ep.mode == GemmEpilogue::kSplitK) {
    float* out = ep.partial + ((int64_t)zid) * M * N;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = mrow + 16 * i;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = ncol + 16 * j;
        if (n + 3 < N) {
          *reinterpret_cast<f32x4*>(out + (int64_t)m * N + n) = acc[i][j];
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n + e < N) out[(int64_t)m * N + n + e] = acc[i][j][e];
        }
      }
    }
    return;
  }
  // epilogue kind as wave-uniform values (scalar branches: a branch on a VGPR copy of a kernel argument
  // would exec-mask every path of every element, the GELU included)
  const int act = __builtin_amdgcn_readfirstlane(ep.act);
  const bool has_bias = __builtin_amdgcn_readfirstlane(ep.bias != nullptr ? 1 : 0) != 0;
  const bool has_res = __builtin_amdgcn_readfirstlane(ep.residual != nullptr ? 1 : 0) != 0;
  const bool has_pre = __builtin_amdgcn_readfirstlane(ep.preact != nullptr ? 1 : 0) != 0;
  const bool has_stats = __builtin_amdgcn_readfirstlane(ep.stats != nullptr ? 1 : 0) != 0;
  const bool out_bf16 = __builtin_amdgcn_readfirstlane(ep.out_bf16 ? 1 : 0) != 0;
  float ssum[4][4], ssq[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) ssum[j][e] = ssq[j][e] = 0.f;
  const int64_t cb = (int64_t)b * ep.c_bstride;
  // Every load of the epilogue is issued before the first use (bias, and the residual or GELU-backward
  // pre-activation of every full tile): a load-wait-store chain per tile is one memory round trip per
  // tile, 16 in a row.
  int64_t row_offs[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mrow + 16 * i;
    if constexpr (loader_kind<LA>::value == 5)
      row_offs[i] = m < Mb ? la.out_row(b, m) * ep.ldc : 0;
    else
      row_offs[i] = cb + (int64_t)m * ep.ldc;
  }
  float bias[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[j][e] = (has_bias && ncol + 16 * j + e < N) ? ep.bias[ncol + 16 * j + e] : 0.f;
  const bf16* side = static_cast<const bf16*>(has_res ? ep.residual : (act == 3 ? ep.preact : nullptr));
  bf16x4 sv[4][4];
  if (side) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (mrow + 16 * i < Mb && ncol + 16 * j + 3 < N)
          sv[i][j] = *reinterpret_cast<const bf16x4*>(side + row_offs[i] + ncol + 16 * j);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mrow + 16 * i;
    const bool mok = m < Mb;
    const int64_t row_off = row_offs[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = ncol + 16 * j;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] * ep.alpha + bias[j][e];
      const int64_t off = row_off + n;
      const bool full = mok && n + 3 < N;
      if (act == 3 && mok) {  // GELU backward: the incoming gradient times GELU'(pre-activation)
        const bf16* pa = static_cast<const bf16*>(ep.preact) + off;
        float z[4];
        if (full) {
          const bf16x4 r = sv[i][j];
#pragma unroll
          for (int e = 0; e < 4; ++e) z[e] = (float)r[e];
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) z[e] = n + e < N ? (float)pa[e] : 0.f;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] *= gelu_grad(z[e]);
      } else if (has_pre && mok) {
        bf16* pa = static_cast<bf16*>(ep.preact) + off;
        if (full) {
          *reinterpret_cast<bf16x4*>(pa) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n + e < N) pa[e] = (bf16)v[e];
        }
      }
      if (has_res && mok) {  // one 8-byte load per lane (4 scalar 2-byte loads cost +30 % on ResNet dgrads)
        const bf16* ra = static_cast<const bf16*>(ep.residual) + off;
        if (full) {
          const bf16x4 r = sv[i][j];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)r[e];
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n + e < N) v[e] += (float)ra[e];
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (act == 1) v[e] = fmaxf(v[e], 0.f);
        else if (act == 2) v[e] = gelu_erf(v[e]);
      }
      if (mok) {
        if (out_bf16) {
          bf16* c = static_cast<bf16*>(ep.C) + off;
          if (full) {
            *reinterpret_cast<bf16x4*>(c) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (n + e < N) c[e] = (bf16)v[e];
          }
          // statistics of what was stored (bf16-rounded), like a norm layer reading it back
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = (float)(bf16)v[e];
        } else {
          float* c = static_cast<float*>(ep.C) + off;
          if (full) {
            *reinterpret_cast<f32x4*>(c) = f32x4{v[0], v[1], v[2], v[3]};
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (n + e < N) c[e] = v[e];
          }
        }
        if (has_stats) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            ssum[j][e] += v[e];
            ssq[j][e] += v[e] * v[e];
          }
        }
      }
    }
  }
  if (!has_stats) return;
  // per-channel partials of this block's 128 rows: reduce over the 16 m-lanes, then the 2 m-waves
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        ssum[j][e] += __shfl_xor(ssum[j][e], o, 64);
        ssq[j][e] += __shfl_xor(ssq[j][e], o, 64);
      }
    }
  if ((lane & 15) == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int nl = wn * 64 + 16 * j + 4 * (lane >> 4) + e;
        red[wm][0][nl] = ssum[j][e];
        red[wm][1][nl] = ssq[j][e];
      }
  }
  __syncthreads();
  if (tid < BN) {
    const int n = n0 + tid;
    if (n < N) {
      float* st = ep.stats + ((int64_t)b * tiles_m + tm) * 2 * N;
      st[n] = red[0][0][tid] + red[1][0][tid];
      st[N + n] = red[0][1][tid] + red[1][1][tid];
    }
  }
}

template <class LA, class LB, bool kFp8 = false>
void launch(const LA& la, const LB& lb, const GemmEpilogue& ep, int batch, int M, int N, int K, int splits,
            hipStream_t s) {
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  splits = std::max(1, splits);
  int kps = (K + splits - 1) / splits;
  kps = (kps + BK - 1) / BK * BK;
  splits = (K + kps - 1) / kps;
  dim3 grid(tiles_m * tiles_n, batch * splits);
  gemm_kernel<LA, LB, kFp8><<<grid, 256, 0, s>>>(la, lb, ep, M, N, K, tiles_m, tiles_n, splits, kps);
}

// ------------------------------------------------------------------ reductions
// out[i] = sum_s part[s][i] (fixed order); optional KRSC -> KCRS permutation for conv weights.
__global__ __launch_bounds__(256) void splitk_sum_kernel(const float* __restrict__ part, int S, int64_t n,
                                                         float* __restrict__ out, int perm_k, int perm_c,
                                                         int perm_rs) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  // 8 interleaved partial sums keep 8 loads in flight (the sum is latency-bound: S/8 dependent rounds);
  // combined in a fixed order (deterministic)
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int s = 0;
  for (; s + 8 <= S; s += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] += part[(int64_t)(s + u) * n + i];
  }
  for (; s < S; ++s) acc[0] += part[(int64_t)s * n + i];
  const float a = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  if (perm_rs > 0) {  // i = ko*(RS*C) + rs*C + c  ->  ko*(C*RS) + c*RS + rs
    const int64_t per = (int64_t)perm_rs * perm_c;
    const int64_t ko = i / per, rem = i - ko * per, rs = rem / perm_c, c = rem - rs * perm_c;
    out[ko * per + c * perm_rs + rs] = a;
  } else {
    out[i] = a;
  }
  (void)perm_k;
}

// Two-level fixed-order reduction of per-tile channel partials part[tile][2][N] -> out0/out1[N]:
// level 1: block (64 channels, tile group) - lane = channel, 4 waves stride the group's tiles;
// level 2: one thread per channel sums the G group results in order.
constexpr int PR_GROUPS = 128;

__global__ __launch_bounds__(256) void reduce_parts_l1_kernel(const float* __restrict__ part, int nparts, int N,
                                                              int per_group, float* __restrict__ mid) {
  __shared__ float red[4][2][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane, g = blockIdx.y;
  const int t0 = g * per_group, t1 = min(nparts, t0 + per_group);
  float a = 0.f, q = 0.f;
  if (c < N)
    for (int t = t0 + wave; t < t1; t += 4) {
      a += part[(int64_t)t * 2 * N + c];
      q += part[(int64_t)t * 2 * N + N + c];
    }
  red[wave][0][lane] = a;
  red[wave][1][lane] = q;
  __syncthreads();
  if (wave == 0 && c < N) {
    mid[(int64_t)g * 2 * N + c] = (red[0][0][lane] + red[1][0][lane]) + (red[2][0][lane] + red[3][0][lane]);
    mid[(int64_t)g * 2 * N + N + c] = (red[0][1][lane] + red[1][1][lane]) + (red[2][1][lane] + red[3][1][lane]);
  }
}

// level 2: block = 64 channels, wave w sums groups w, w+4, .., the 4 wave totals combine in a fixed order
// (one thread per channel serialised G dependent adds over a handful of workgroups: 7-10 us per call)
__global__ __launch_bounds__(256) void reduce_parts_l2_kernel(const float* __restrict__ mid, int G, int N,
                                                              float* __restrict__ out0, float* __restrict__ out1) {
  __shared__ float red[4][2][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float a = 0.f, q = 0.f;
  if (c < N)
    for (int g = wave; g < G; g += 4) {
      a += mid[(int64_t)g * 2 * N + c];
      q += mid[(int64_t)g * 2 * N + N + c];
    }
  red[wave][0][lane] = a;
  red[wave][1][lane] = q;
  __syncthreads();
  if (wave == 0 && c < N) {
    out0[c] = (red[0][0][lane] + red[1][0][lane]) + (red[2][0][lane] + red[3][0][lane]);
    out1[c] = (red[0][1][lane] + red[1][1][lane]) + (red[2][1][lane] + red[3][1][lane]);
  }
}

// Split-K conv epilogue: out[r][c] = bf16(sum_s part[s][r][c] (+ residual)), plus (mid != null) the
// per-channel sum / sum of squares of the stored values per row group g -> mid[g][2][N] (the layout
// bn_prepare reads).  Block = 64 channels x one row group, wave w takes rows w, w+4, ..; fixed order.
__global__ __launch_bounds__(256) void splitk_finish_kernel(const float* __restrict__ part, int S, int M, int N,
                                                            bf16* __restrict__ out, int64_t ldc,
                                                            const bf16* __restrict__ residual,
                                                            float* __restrict__ mid, int rows_per_group) {
  __shared__ float red[4][2][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane, g = blockIdx.y;
  const int r0 = g * rows_per_group, r1 = min(M, r0 + rows_per_group);
  float a = 0.f, q = 0.f;
  if (c < N)
    for (int r = r0 + wave; r < r1; r += 4) {
      // 8 interleaved partial sums (independent loads in flight), combined in a fixed order
      const float* pr = part + (int64_t)r * N + c;
      const int64_t ps = (int64_t)M * N;
      float vv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      int sp = 0;
      for (; sp + 8 <= S; sp += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) vv[u] += pr[(sp + u) * ps];
      }
      for (; sp < S; ++sp) vv[0] += pr[sp * ps];
      float v = ((vv[0] + vv[1]) + (vv[2] + vv[3])) + ((vv[4] + vv[5]) + (vv[6] + vv[7]));
      if (residual) v += (float)residual[(int64_t)r * ldc + c];
      const bf16 o = (bf16)v;
      out[(int64_t)r * ldc + c] = o;
      const float f = (float)o;
      a += f;
      q += f * f;
    }
  if (!mid) return;
  red[wave][0][lane] = a;
  red[wave][1][lane] = q;
  __syncthreads();
  if (wave == 0 && c < N) {
    mid[(int64_t)g * 2 * N + c] = (red[0][0][lane] + red[1][0][lane]) + (red[2][0][lane] + red[3][0][lane]);
    mid[(int64_t)g * 2 * N + N + c] = (red[0][1][lane] + red[1][1][lane]) + (red[2][1][lane] + red[3][1][lane]);
  }
}

}  // namespace

// ================================================================== launchers
// 256x256 bf16 kernel (gemm_bf16_256.hip), K- or row-contiguous A and B: one workgroup per CU, so it pays
// when the tile count fills whole rounds of the 256 CUs.  RINGDP_BF16_TILE=128 / 256 forces a path.
static int g_bf16_tile = -1;
static int bf16_tile_mode() {
  if (g_bf16_tile < 0) {
    const char* v = getenv("RINGDP_BF16_TILE");
    g_bf16_tile = v ? atoi(v) : 0;
  }
  return g_bf16_tile;
}
void set_bf16_tile_mode(int mode) { g_bf16_tile = mode; }
// Minimum round fill for the 256x256 kernel (RINGDP_BF16_256_FILL).  ViT-B/16's N = 768 GEMMs (297 tiles:
// 2 rounds at 58 %) measured faster there than on the 128 core in 4 of 5 shapes (-1.5 % step,
// profiles/r03/gemm_routing.md).
static double bf16_256_fill() {
  static double f = -1.0;
  if (f < 0) {
    const char* v = getenv("RINGDP_BF16_256_FILL");
    f = v ? atof(v) : 0.55;
  }
  return f;
}
static bool bf16_use_256(int M, int N, int K, int batch, int splits) {
  const int mode = bf16_tile_mode();
  if (mode == 128) return false;
  if (mode == 256) return true;
  const int64_t tiles = (int64_t)((M + 255) / 256) * ((N + 255) / 256) * batch * std::max(1, splits);
  const int64_t rounds = (tiles + 255) / 256;
  const double fill = rounds > 0 ? (double)tiles / (256.0 * rounds) : 0.0;
  return tiles >= 192 && fill >= bf16_256_fill() && K / std::max(1, splits) >= 512;
}

// Split count that fills whole rounds of the 256 CUs with 256x256 tiles (>= 4 k-tiles per split), for
// the long-K weight gradients (K = tokens); `requested` (the 128-core choice) when none fills >= 75 %.
int gemm_bf16_pick_splits(int M, int N, int K, int requested) {
  if (requested <= 1 || bf16_tile_mode() == 128) return std::max(1, requested);
  const int64_t tiles = (int64_t)((M + 255) / 256) * ((N + 255) / 256);
  const int maxs = std::max(1, std::min(32, K / 256));
  int best = 0;
  double best_fill = 0.0;
  for (int sp = 1; sp <= maxs; ++sp) {
    const int64_t t = tiles * sp;
    if (t < 192) continue;
    const int64_t rounds = (t + 255) / 256;
    const double f = (double)t / (256.0 * rounds) - 0.002 * sp;  // fewer fp32 partial planes on a tie
    if (f > best_fill) {
      best_fill = f;
      best = sp;
    }
  }
  return best > 0 && bf16_use_256(M, N, K, 1, best) ? best : requested;
}

void gemm_bf16(const GemmOperand& A, const GemmOperand& B, int batch, int M, int N, int K, const GemmEpilogue& ep,
               int splits, hipStream_t s) {
  if (bf16_use_256(M, N, K, batch, splits) &&
      gemm_bf16_256(A, B, batch, M, N, K, ep, splits, s))
    return;
  const DenseLoader da{static_cast<const bf16*>(A.p), A.ld, A.bstride, M, K};
  const DenseLoader db{static_cast<const bf16*>(B.p), B.ld, B.bstride, N, K};
  // aligned fast path: every k-tile of every split full, row-contiguous operands in whole 8-row vectors
  // (M/N >= 8 and % 8), split-K slices in whole k-tiles
  const bool aligned = K % BK == 0 && (!A.row_contig || (M % 8 == 0 && M >= 8)) &&
                       (!B.row_contig || (N % 8 == 0 && N >= 8)) && M > 0 && N > 0;
  if (aligned) {
    if (!A.row_contig && !B.row_contig)
      launch(DenseAligned<false>{da}, DenseAligned<false>{db}, ep, batch, M, N, K, splits, s);
    else if (!A.row_contig && B.row_contig)
      launch(DenseAligned<false>{da}, DenseAligned<true>{db}, ep, batch, M, N, K, splits, s);
    else if (A.row_contig && !B.row_contig)
      launch(DenseAligned<true>{da}, DenseAligned<false>{db}, ep, batch, M, N, K, splits, s);
    else
      launch(DenseAligned<true>{da}, DenseAligned<true>{db}, ep, batch, M, N, K, splits, s);
    return;
  }
  if (!A.row_contig && !B.row_contig)
    launch(Dense<false>{da}, Dense<false>{db}, ep, batch, M, N, K, splits, s);
  else if (!A.row_contig && B.row_contig)
    launch(Dense<false>{da}, Dense<true>{db}, ep, batch, M, N, K, splits, s);
  else if (A.row_contig && !B.row_contig)
    launch(Dense<true>{da}, Dense<false>{db}, ep, batch, M, N, K, splits, s);
  else
    launch(Dense<true>{da}, Dense<true>{db}, ep, batch, M, N, K, splits, s);
}

// 256x256 fp8 kernel (gemm_fp8_256.hip): one workgroup per CU, so it pays when the tile count fills
// whole rounds of the 256 CUs; RINGDP_FP8_TILE=128 / 256 forces a path (A/B measurements).
static int g_fp8_tile = -1;  // -1: not read yet; 0 auto; 128 / 256 forced
static int fp8_tile_mode() {
  if (g_fp8_tile < 0) {
    const char* v = getenv("RINGDP_FP8_TILE");
    g_fp8_tile = v ? atoi(v) : 0;
  }
  return g_fp8_tile;
}
void set_fp8_tile_mode(int mode) { g_fp8_tile = mode; }
static double fp8_256_fill(int64_t tiles) {
  const int64_t rounds = (tiles + 255) / 256;
  return rounds > 0 ? (double)tiles / (256.0 * rounds) : 0.0;
}
// Measured (tools/gemm_bench.py --vit-fp8, ViT-B/16 shapes): the 256 kernel wins on the long-K split-K
// weight gradients (K = 25216 tokens: 74-86 us vs 95-118 us at >= 27 output tiles) and on K >= 4096
// (8192^3: 1.95 vs 1.67 PF/s).  It lost on short-K single-pass GEMMs only while its epilogue branched on
// VGPR copies of the epilogue flags; since those are scalar it wins there too at >= 75 % round fill.
static bool fp8_use_256(int M, int N, int Kbytes, int batch, int splits) {
  const int mode = fp8_tile_mode();
  if (mode == 128) return false;
  if (mode == 256) return true;
  const int64_t out_tiles = (int64_t)((M + 255) / 256) * ((N + 255) / 256) * batch;
  const int64_t tiles = out_tiles * std::max(1, splits);
  // round fill for the 256 kernel (RINGDP_FP8_256_FILL): ViT-B/16 fp8 5203-5231 img/s at 0.75, 5274-5284 at
  // 0.55, 5276-5293 at 0.45 (two boxes; profiles/r04/README.md)
  static const double min_fill = [] {
    const char* v = getenv("RINGDP_FP8_256_FILL");
    const double f = v ? atof(v) : 0.55;
    return f > 0.0 && f <= 1.0 ? f : 0.55;
  }();
  if (tiles < 192 || fp8_256_fill(tiles) < min_fill) return false;
  // (single-pass GEMMs of any K: with the scalar-branch epilogue the 256 kernel wins at >= 75 % round fill,
  // e.g. 25216 x 3072 x 768 104 vs 126 us, x 2304 87 vs 98 us; profiles/r03/gemm_tiles.jsonl)
  return splits > 1 ? out_tiles >= 16 : true;
}

int gemm_fp8_pick_splits(int M, int N, int Kbytes, int requested) {
  if (requested <= 1 || fp8_tile_mode() == 128) return std::max(1, requested);
  const int64_t tiles = (int64_t)((M + 255) / 256) * ((N + 255) / 256);
  const int maxs = std::max(1, std::min(32, Kbytes / 256));  // >= 2 k-steps per split
  int best = 0;
  double best_fill = 0.0;
  for (int sp = 1; sp <= maxs; ++sp) {
    const int64_t t = tiles * sp;
    if (t < 192) continue;
    const double f = fp8_256_fill(t) - 0.002 * sp;  // prefer fewer fp32 partial planes on a tie
    if (f > best_fill) {
      best_fill = f;
      best = sp;
    }
  }
  return best > 0 && fp8_use_256(M, N, Kbytes, 1, best) ? best : requested;
}

void gemm_fp8(const GemmOperand& A, const GemmOperand& B, int batch, int M, int N, int Kbytes, const GemmEpilogue& ep,
              int splits, hipStream_t s) {
  if (ep.q8) {  // e4m3 outputs exist only in the 256x256 kernel's epilogue (the op layer checked the shape)
    if (!gemm_fp8_256(A, B, batch, M, N, Kbytes, ep, splits, s)) {
      fprintf(stderr, "gemm_fp8: e4m3-output GEMM %d x %d x %d not supported by the 256x256 kernel\n", M, N, Kbytes);
      abort();
    }
    return;
  }
  if (fp8_use_256(M, N, Kbytes, batch, splits) && gemm_fp8_256(A, B, batch, M, N, Kbytes, ep, splits, s)) return;
  // K-contiguous e4m3 operands viewed as bf16 "slots" of 2 bytes for the 16-B stagers
  const DenseLoader da{static_cast<const bf16*>(A.p), A.ld / 2, A.bstride / 2, M, Kbytes / 2};
  const DenseLoader db{static_cast<const bf16*>(B.p), B.ld / 2, B.bstride / 2, N, Kbytes / 2};
  if ((Kbytes / 2) % BK == 0 && M > 0 && N > 0)
    launch<DenseAligned<false>, DenseAligned<false>, true>(DenseAligned<false>{da}, DenseAligned<false>{db}, ep, batch,
                                                           M, N, Kbytes / 2, splits, s);
  else
    launch<Dense<false>, Dense<false>, true>(Dense<false>{da}, Dense<false>{db}, ep, batch, M, N, Kbytes / 2, splits, s);
}

static bool is_pointwise(const ConvGeom& g) {
  return g.R == 1 && g.S == 1 && g.stride == 1 && g.pad == 0 && g.P == g.H && g.Q == g.W;
}

// Split count for a conv GEMM with few output tiles (ResNet-18 CIFAR layers 2-4 run 8-32 tiles of 128x128
// on 256 CUs with 18-72 serial k-tiles each): enough splits to give ~2 workgroups per CU, >= 4 k-tiles per
// split.  Returns the count the launcher will actually use (its rounding of the k-range per split).
// RINGDP_CONV_SPLIT_WGS / RINGDP_CONV_SPLIT_MINKT / RINGDP_WGRAD_SPLIT_WGS / RINGDP_WGRAD_SPLIT_MINKT override the
// workgroup targets and minimum k-tiles per split of the two split counts below (sweeps).
static int split_knob(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? std::max(1, atoi(v)) : dflt;
}

int conv_gemm_splits(int M, int N, int K) {
  static const int wgs = split_knob("RINGDP_CONV_SPLIT_WGS", 512), minkt = split_knob("RINGDP_CONV_SPLIT_MINKT", 4);
  const int64_t tiles = (int64_t)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int nkt = K / BK;
  if (tiles >= 128 || nkt < 2 * minkt) return 1;
  int S = (int)std::min<int64_t>(nkt / minkt, (wgs + tiles - 1) / tiles);
  S = std::max(1, std::min(S, 32));
  int kps = (K + S - 1) / S;
  kps = (kps + BK - 1) / BK * BK;
  return (K + kps - 1) / kps;
}

int splitk_finish_groups(int M) {
  const int rpg = std::max(16, (M + 127) / 128);
  return (M + rpg - 1) / rpg;
}

void splitk_finish(const float* part, int S, int M, int N, void* out, int64_t ldc, const void* residual, float* mid,
                   hipStream_t s) {
  const int rpg = std::max(16, (M + 127) / 128);
  const int G = (M + rpg - 1) / rpg;
  splitk_finish_kernel<<<dim3((N + 63) / 64, G), 256, 0, s>>>(part, S, M, N, static_cast<bf16*>(out), ldc,
                                                              static_cast<const bf16*>(residual), mid, rpg);
}

void conv_fwd_bf16(const void* x, const void* w_krsc, int64_t ldw, const ConvGeom& g, const GemmEpilogue& ep,
                   hipStream_t s, int splits) {
  const int M = g.N * g.P * g.Q, Kd = g.R * g.S * g.C;
  const ConvFwdA la{static_cast<const bf16*>(x), g, M, Kd};
  const DenseLoader db{static_cast<const bf16*>(w_krsc), ldw, 0, g.K, Kd};
  const int Kpad = (Kd + BK - 1) / BK * BK;
  if (Kd % BK != 0 && g.C == 8 && ldw % BK == 0 && ldw >= Kpad) {
    const DenseLoader dbp{static_cast<const bf16*>(w_krsc), ldw, 0, g.K, Kpad};
    launch(ConvFwdA8{static_cast<const bf16*>(x), g, M, Kpad}, DenseAligned<false>{dbp}, ep, 1, M, g.K, Kpad, 1, s);
    return;
  }
  if (Kd % BK == 0) {
    if (is_pointwise(g)) {  // 1x1 / stride 1 / pad 0: the im2col IS the NHWC activation matrix
      const DenseLoader da{static_cast<const bf16*>(x), g.C, 0, M, Kd};
      launch(DenseAligned<false>{da}, DenseAligned<false>{db}, ep, 1, M, g.K, Kd, splits, s);
    } else if (g.C % BK == 0) {
      launch(ConvFwdA64{static_cast<const bf16*>(x), g, M, Kd}, DenseAligned<false>{db}, ep, 1, M, g.K, Kd, splits,
             s);
    } else {
      launch(la, DenseAligned<false>{db}, ep, 1, M, g.K, Kd, 1, s);
    }
    return;
  }
  launch(la, Dense<false>{db}, ep, 1, M, g.K, Kd, 1, s);
}

static int g_s2_dgrad = -1;  // RINGDP_S2_DGRAD=0: gather form for stride-2 data gradients (A/B runs)
void conv_dgrad_bf16(const void* dy, const void* w_crsk, const ConvGeom& g, const GemmEpilogue& ep, hipStream_t s,
                     int splits) {
  const int M = g.N * g.H * g.W, Kd = g.R * g.S * g.K;
  if (g_s2_dgrad < 0) {
    const char* v = getenv("RINGDP_S2_DGRAD");
    g_s2_dgrad = v ? atoi(v) : 1;
  }
  if (g_s2_dgrad && g.stride == 2 && g.dil == 1 && g.K % BK == 0 && !ep.stats && ep.c_bstride == 0 &&
      ep.mode != GemmEpilogue::kSplitK) {
    // 4 parity classes as the batch; rows / k-range of the largest class (ph = pw = 0 for even pads)
    const int Mc = g.N * ((g.H + 1) / 2) * ((g.W + 1) / 2);
    const int Kc = ((g.R + 1) / 2) * ((g.S + 1) / 2) * g.K;
    launch(ConvDgradS2A{static_cast<const bf16*>(dy), g}, ConvDgradS2B{static_cast<const bf16*>(w_crsk), g}, ep, 4,
           Mc, g.C, Kc, 1, s);
    return;
  }
  const ConvDgradA la{static_cast<const bf16*>(dy), g, M, Kd};
  const DenseLoader db{static_cast<const bf16*>(w_crsk), Kd, 0, g.C, Kd};
  if (Kd % BK == 0) {
    if (is_pointwise(g)) {  // dX = dY W: dY is the dense [N*H*W][K] matrix
      const DenseLoader da{static_cast<const bf16*>(dy), g.K, 0, M, Kd};
      launch(DenseAligned<false>{da}, DenseAligned<false>{db}, ep, 1, M, g.C, Kd, splits, s);
    } else if (g.K % BK == 0) {
      launch(ConvDgradA64{static_cast<const bf16*>(dy), g, M, Kd}, DenseAligned<false>{db}, ep, 1, M, g.C, Kd, splits,
             s);
    } else {
      launch(la, DenseAligned<false>{db}, ep, 1, M, g.C, Kd, 1, s);
    }
    return;
  }
  launch(la, Dense<false>{db}, ep, 1, M, g.C, Kd, 1, s);
}

void conv_wgrad_bf16(const void* dy, const void* x, const ConvGeom& g, int splits, float* partial, float* dw_kcrs,
                     hipStream_t s) {
  const int Mpos = g.N * g.P * g.Q, Kd = g.R * g.S * g.C;
  // C[ko][kk] = sum_m dY[m][ko] * X(m, kk):  A = dY^T (row-contiguous, ld = K), B = im2col^T
  const DenseLoader da{static_cast<const bf16*>(dy), g.K, 0, g.K, Mpos};
  const ConvWgradB lb{static_cast<const bf16*>(x), g, Mpos, Kd};
  GemmEpilogue ep{};
  ep.mode = GemmEpilogue::kSplitK;
  ep.partial = partial;
  const int tiles_m = (g.K + BM - 1) / BM, tiles_n = (Kd + BN - 1) / BN;
  (void)tiles_m;
  (void)tiles_n;
  int kps = (Mpos + splits - 1) / splits;
  kps = (kps + BK - 1) / BK * BK;
  const int S = (Mpos + kps - 1) / kps;
  if (Mpos % BK == 0 && g.K % 8 == 0) {
    if (is_pointwise(g) && Kd % 8 == 0) {  // B = X^T: row-contiguous view of the NHWC activation
      const DenseLoader db{static_cast<const bf16*>(x), g.C, 0, Kd, Mpos};
      launch(DenseAligned<true>{da}, DenseAligned<true>{db}, ep, 1, g.K, Kd, Mpos, S, s);
    } else {
      launch(DenseAligned<true>{da}, lb, ep, 1, g.K, Kd, Mpos, S, s);
    }
  } else {
    launch(Dense<true>{da}, lb, ep, 1, g.K, Kd, Mpos, S, s);
  }
  const int64_t n = (int64_t)g.K * Kd;
  splitk_sum_kernel<<<(int)((n + 255) / 256), 256, 0, s>>>(partial, S, n, dw_kcrs, g.K, g.C, g.R * g.S);
}

int conv_wgrad_splits(const ConvGeom& g, int cus) {
  const int Mpos = g.N * g.P * g.Q, Kd = g.R * g.S * g.C;
  static const int wgs = split_knob("RINGDP_WGRAD_SPLIT_WGS", 0), minkt = split_knob("RINGDP_WGRAD_SPLIT_MINKT", 4);
  const int target = wgs > 0 ? wgs : 2 * cus;
  const int tiles = ((g.K + BM - 1) / BM) * ((Kd + BN - 1) / BN);
  const int want = std::max(1, (target + tiles - 1) / tiles);
  const int max_split = std::max(1, Mpos / (minkt * BK));
  return std::min(want, max_split);
}

void splitk_sum(const float* part, int S, int64_t n, float* out, hipStream_t s) {
  splitk_sum_kernel<<<(int)((n + 255) / 256), 256, 0, s>>>(part, S, n, out, 0, 0, 0);
}

int reduce_parts_scratch_floats(int nparts, int N) {
  const int G = std::min(PR_GROUPS, std::max(1, (nparts + 31) / 32));
  return 2 * N * G;
}

int reduce_parts_groups(int nparts) { return std::min(PR_GROUPS, std::max(1, (nparts + 31) / 32)); }

int reduce_parts_l1(const float* part, int nparts, int N, float* mid, hipStream_t s) {
  const int G = reduce_parts_groups(nparts);
  const int per = (nparts + G - 1) / G;
  reduce_parts_l1_kernel<<<dim3((N + 63) / 64, G), 256, 0, s>>>(part, nparts, N, per, mid);
  return G;
}

void reduce_parts(const float* part, int nparts, int N, float* scratch, float* out0, float* out1, hipStream_t s) {
  const int G = std::min(PR_GROUPS, std::max(1, (nparts + 31) / 32));
  const int per = (nparts + G - 1) / G;
  reduce_parts_l1_kernel<<<dim3((N + 63) / 64, G), 256, 0, s>>>(part, nparts, N, per, scratch);
  reduce_parts_l2_kernel<<<(N + 63) / 64, 256, 0, s>>>(scratch, G, N, out0, out1);
}

int gemm_tiles_m(int M) { return (M + BM - 1) / BM; }

}  // namespace kern
}  // namespace ringdp
