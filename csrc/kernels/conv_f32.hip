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
#include <type_traits>

#include "device_common.h"
#include "kernels.h"

namespace ringdp {
namespace kern {
namespace {

using dev::f32x4;

#ifndef RINGDP_F32_BK
#define RINGDP_F32_BK 16
#endif
constexpr int BK = RINGDP_F32_BK, TPB = 256;

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

// ---------------------------------------------------------------- operand loaders
// GEMM C[M][N] = sum_k A(m, k) * B(k, n).  kMC: the operand's thread-fixed index is contiguous in
// memory (lanes walk m), with a per-workgroup k table; otherwise lanes walk k.
// A loader resolves an element to a Ref: an element offset into its source and a valid flag.  The
// kernel reads every element with a raw buffer load (SGPR resource + 32-bit VGPR offset): invalid
// elements (zero padding, past an edge) get an offset beyond the resource's range and the hardware
// returns 0, so the loads are branch-free, their count is static and they need no 64-bit address
// arithmetic.  u8 pixels are normalised at the stash, where their padding (0 AFTER normalisation)
// needs the valid flag.
constexpr int kBadOff = 0x20000000;  // x 4 bytes = 2^31: past every source (chunks stay < 2^31 bytes)
struct Ref {
  int off, ok;
};
__device__ __forceinline__ Ref ref_if(bool ok, int off) { return Ref{ok ? off : kBadOff, ok ? 1 : 0}; }
__device__ __forceinline__ bool in2(int y, int x, int H, int W) {
  return static_cast<unsigned>(y) < static_cast<unsigned>(H) && static_cast<unsigned>(x) < static_cast<unsigned>(W);
}

template <bool U8>
struct Src {  // fp32 tensor, or raw uint8 pixels normalised as (v / 255 - mean) * inv_std
  typedef typename std::conditional<U8, unsigned char, float>::type T;
  static constexpr bool kU8 = U8;
  const T* p;
  int bytes;  // buffer-resource range
  float mean, inv_std;
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(p), 0, bytes, 0x00020000);
  }
  __device__ __forceinline__ T load(__amdgpu_buffer_rsrc_t r, int off) const {
    if constexpr (U8) return __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
    else return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off * 4, 0, 0));
  }
  __device__ __forceinline__ float cvt(T v) const {
    if constexpr (U8) return (static_cast<float>(v) * (1.0f / 255.0f) - mean) * inv_std;
    else return v;
  }
};

// PAD = false (a valid conv over an fp32 input): every (m, k) is in bounds, so rows past M and
// k past K are clamped onto real elements instead of checked - the rows are never stored and the
// weights past K are zero.
// WIN: window-major output pixels, m = (b, py, px, wy, wx) with (oy, ox) = (2 py + wy, 2 px + wx), so
// the 4 pixels of a 2x2/s2 pooling window are 4 consecutive m (the PoolOut epilogue); `ow` then
// divides by the pooled width.
// MODE 2: one image per 128-row m tile, m = (b, p < 128), p >= OH*OW clamped onto the last pixel
// (those rows are never stored) - the PoolS1Out epilogue pools a whole image from LDS.
template <bool U8, bool PAD, int MODE = 0>
struct FwdA {  // A(m = (b, oy, ox), k = (c, ky, kx)) = x[b, c, oy + ky - pad, ox + kx - pad]
  static constexpr bool kMC = true;
  Src<U8> src;
  int C, H, W, R, pad, OW, K, M;
  FastDiv ohw, ow;
  struct O {
    int base, y, x;
  };
  __device__ O outer(int m) const {
    if constexpr (!PAD) m = min(m, M - 1);
    else if (m >= M) return O{0, kOut, kOut};
    int b, r;
    if constexpr (MODE == 2) {
      b = m >> 7;
      r = min(m & 127, static_cast<int>(ohw.d) - 1);
    } else {
      b = fdiv(m, ohw);
      r = m - b * static_cast<int>(ohw.d);
    }
    int oy, ox;
    if constexpr (MODE == 1) {
      const int w = r >> 2, py = fdiv(w, ow);
      oy = 2 * py + ((r >> 1) & 1);
      ox = 2 * (w - py * static_cast<int>(ow.d)) + (r & 1);
    } else {
      oy = fdiv(r, ow);
      ox = r - oy * OW;
    }
    return O{b * C * H * W + (oy - pad) * W + (ox - pad), oy - pad, ox - pad};
  }
  __device__ int2 ktab(int k) const {  // (offset, dy|dx)
    if constexpr (!PAD) k = min(k, K - 1);
    else if (k >= K) return int2{0, pack_dyx(kOut, kOut)};
    const int rr = R * R, c = k / rr, t = k - c * rr, ky = t / R, kx = t - ky * R;
    return int2{c * H * W + ky * W + kx, pack_dyx(ky, kx)};
  }
  __device__ Ref ref(const O& o, int2 kt) const {  // zero padding after Normalize
    if constexpr (!PAD) return Ref{o.base + kt.x, 1};
    else return ref_if(in2(o.y + unpack_dy(kt.y), o.x + unpack_dx(kt.y), H, W), o.base + kt.x);
  }
};

struct DgradA {  // A(m = (b, iy, ix), k = (n, ky, kx)) = dz[b, n, iy + pad - ky, ix + pad - kx]
  static constexpr bool kMC = true;
  Src<false> src;
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
  __device__ Ref ref(const O& o, int2 kt) const {
    return ref_if(in2(o.y + unpack_dy(kt.y), o.x + unpack_dx(kt.y), OH, OW), o.base + kt.x);
  }
};

struct WeightB {  // B(k = (c, ky, kx), n) = w[n][c][ky][kx]; lanes walk k
  static constexpr bool kMC = false;
  Src<false> src;
  int K, N;
  typedef int O;
  typedef int KS;
  __device__ O outer(int n) const { return n < N ? n * K : -1; }
  __device__ KS kstate(int k, int kend) const { return k < kend ? k : -1; }
  __device__ Ref ref(O o, KS k) const { return ref_if((o | k) >= 0, o + k); }
};

struct DgradB {  // B(k = (n, ky, kx), c) = w[n][c][ky][kx]; lanes walk k
  static constexpr bool kMC = false;
  Src<false> src;
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
  __device__ Ref ref(O o, KS k) const { return ref_if((o | k) >= 0, o + k); }
};

struct WgradA {  // A(m = n, k = (b, r)) = dz[b, n, r]     (k runs over batch x output pixels)
  static constexpr bool kMC = false;
  Src<false> src;
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
  __device__ Ref ref(O o, KS k) const { return ref_if((o | k) >= 0, o + k); }
};

// PAD = false: as FwdA - columns past Nw and k past the slice are clamped onto real elements (the
// columns are never stored, A is zero past the slice).
template <bool U8, bool PAD>
struct WgradB {  // B(k = (b, oy, ox), j = (c, ky, kx)) = x[b, c, oy + ky - pad, ox + kx - pad]
  static constexpr bool kMC = false;
  Src<U8> src;
  int C, H, W, R, pad, OW, Nw;
  FastDiv ohw, ow;
  struct O {
    int off, dyx;  // dyx never in bounds past the last column
  };
  struct KS {
    int base, y, x;  // y = oy - pad, x = ox - pad; y = kOut when k is past the slice
  };
  __device__ O outer(int j) const {
    if constexpr (!PAD) j = min(j, Nw - 1);
    else if (j >= Nw) return O{0, pack_dyx(kOut, kOut)};
    const int rr = R * R, c = j / rr, t = j - c * rr, ky = t / R, kx = t - ky * R;
    return O{c * H * W + ky * W + kx, pack_dyx(ky, kx)};
  }
  __device__ KS kstate(int k, int kend) const {
    if constexpr (!PAD) k = min(k, kend - 1);
    else if (k >= kend) return KS{0, kOut, kOut};
    const int b = fdiv(k, ohw), r = k - b * static_cast<int>(ohw.d);
    const int oy = fdiv(r, ow), ox = r - oy * OW;
    return KS{b * C * H * W + (oy - pad) * W + (ox - pad), oy - pad, ox - pad};
  }
  __device__ Ref ref(const O& o, const KS& k) const {
    if constexpr (!PAD) return Ref{k.base + o.off, 1};
    return ref_if(in2(k.y + unpack_dy(o.dyx), k.x + unpack_dx(o.dyx), H, W), k.base + o.off);
  }
};

// ---------------------------------------------------------------- epilogues
struct NCHWOut {  // C[m = (b, p)][n] (+ bias[n]) -> out[b, n, p]
  static constexpr bool kPool = false, kPoolS1 = false;
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

// split-K data gradient (small batches): slice z stores its partial dx, NCHW, into slab plane z
struct NCHWSlabOut {
  static constexpr bool kPool = false, kPoolS1 = false;
  float* out;
  int N, M, plane;  // plane = M * N elements
  FastDiv hw;
  __device__ int row(int m) const {
    const int b = fdiv(m, hw);
    return static_cast<int>(blockIdx.z) * plane + b * N * static_cast<int>(hw.d) + (m - b * static_cast<int>(hw.d));
  }
  __device__ void store(int rowoff, int n, float v) const { out[rowoff + n * static_cast<int>(hw.d)] = v; }
};

struct SlabOut {  // split-K slice z: slab[z][m][n]
  static constexpr bool kPool = false, kPoolS1 = false;
  float* slab;
  int N, M;
  __device__ int row(int m) const { return static_cast<int>(blockIdx.z) * M * N + m * N; }
  __device__ void store(int rowoff, int n, float v) const { slab[rowoff + n] = v; }
};

// Fused ReLU + 2x2/s2 max-pool over window-major m (FwdA<.., WIN>): the 4 pixels of a window are
// the 4 lanes 4q..4q+3 of a 16-lane MFMA row group, reduced with two lane exchanges.
// a[b, n, w] = relu(max_t (C[m][n] + bias[n])), code[b, n, w] = first argmax t (255: not live); the
// pre-activation is never written.
struct PoolOut {
  static constexpr bool kPool = true, kPoolS1 = false;
  float* a;
  unsigned char* code;
  const float* bias;
  int N, M, phw;  // phw = pooled pixels per plane
  FastDiv hw;     // conv output pixels per plane
  __device__ int row(int m) const {  // offset of a[b, 0, w]
    const int b = fdiv(m, hw);
    return b * N * phw + ((m - b * static_cast<int>(hw.d)) >> 2);
  }
};

// Fused ReLU + 2x2/s1 (overlapping) max-pool over one image per 128-row tile (FwdA<.., 2>): the tile's
// C + bias goes to LDS and the workgroup pools the whole image from there.
struct PoolS1Out {
  static constexpr bool kPool = false, kPoolS1 = true;
  float* a;
  unsigned char* code;
  const float* bias;
  int N, OW, PW, phw;  // conv output width, pooled width, pooled pixels per plane
  FastDiv fphw, fpw;
};

template <int CTL>
__device__ __forceinline__ void pool_quad_step(float& best, int& bt) {
  const float ov = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, best), CTL, 0xF,
                                                                         0xF, false));
  const int ot = __builtin_amdgcn_update_dpp(0, bt, CTL, 0xF, 0xF, false);
  if (ov > best || (ov == best && ot < bt)) {
    best = ov;
    bt = ot;
  }
}

// ---------------------------------------------------------------- the GEMM core
// grid: x = m tiles, y = n tiles, z = k slices (each covers k_per_slice of K).  WM x WN waves, each
// owning a (16 TM) x (16 TN) block of the output (TM x TN MFMA tiles).  On gfx950 the f32 MFMA runs
// at the f32 VALU rate and the loaders' VALU work competes with it (PMC: MFMA busy 48 % with 5.7
// VALU instructions per MFMA on 32x32 wave blocks), so the wave blocks are as large as the GEMM's
// narrow side allows: elements gathered per MFMA per lane = 16 / BN (A) + 16 / BM (B).
// With WM * WN < 4 the remaining waves split each k-tile's MFMA steps between them and the partial
// accumulators are summed in a fixed wave order at the end (the 32x32 tile of conv1's weight
// gradient).  ktab_n > 0: the A operand's k table (K rounded up to BK) in dynamic LDS.
template <int WM, int WN, int TM, int TN, class LA, class LB, class Epi>
__global__ __launch_bounds__(TPB) void gemm_f32_kernel(int M, int N, int K, int k_per_slice, int ktab_n, int bias_col,
                                                       LA la, LB lb, Epi epi) {
  constexpr int BM = 16 * TM * WM, BN = 16 * TN * WN, KSPLIT = 4 / (WM * WN);
  static_assert(KSPLIT * WM * WN == 4 && BK / 4 >= KSPLIT, "4 waves");
  constexpr int LDA = BM + 16, LDB = BN + 16;  // row stride = 16 banks mod 64: conflict-free MFMA reads
  constexpr int EA = BM * BK / TPB, EB = BN * BK / TPB;
  constexpr int LDT = BM + 4;  // PoolS1Out staging row stride
  constexpr int SM_AB = 2 * BK * (LDA + LDB), SM = (Epi::kPoolS1 && BN * LDT > SM_AB) ? BN * LDT : SM_AB;
  __shared__ float smem[SM];
  auto As = reinterpret_cast<float(*)[BK][LDA]>(smem);
  auto Bs = reinterpret_cast<float(*)[BK][LDB]>(smem + 2 * BK * LDA);
  extern __shared__ int2 ktab[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wk = wave / (WM * WN), wmn = wave % (WM * WN);
  const int wm = (wmn / WN) * 16 * TM, wn = (wmn % WN) * 16 * TN;
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

  // the next k-tile's raw elements (loaded branch-free while the current tile is multiplied); u8
  // sources also keep a valid bit per element, applied when the tile is stashed
  const auto rsa = la.src.rsrc();
  const auto rsb = lb.src.rsrc();
  constexpr bool UA = decltype(la.src)::kU8, UB = decltype(lb.src)::kU8;
  typename decltype(la.src)::T ra[EA];
  typename decltype(lb.src)::T rb[EB];
  uint32_t va = 0, vb = 0;
  static_assert(EA <= 32 && EB <= 32, "valid bits");
  auto fetch = [&](int k0) {
    va = 0;
    vb = 0;
#pragma unroll
    for (int i = 0; i < EA; ++i) {
      Ref r;
      if constexpr (LA::kMC) r = la.ref(oa[0], ktab[k0 + tid / BM + (TPB / BM) * i]);
      else r = la.ref(oa[i], la.kstate(k0 + tid % BK, kend));
      ra[i] = la.src.load(rsa, r.off);
      if constexpr (UA) va |= static_cast<uint32_t>(r.ok) << i;
    }
#pragma unroll
    for (int i = 0; i < EB; ++i) {
      Ref r;
      if constexpr (LB::kMC) r = lb.ref(ob[0], ktab[k0 + tid / BN + (TPB / BN) * i]);
      else r = lb.ref(ob[i], lb.kstate(k0 + tid % BK, kend));
      rb[i] = lb.src.load(rsb, r.off);
      if constexpr (UB) vb |= static_cast<uint32_t>(r.ok) << i;
    }
  };
  // bias gradient (weight-gradient GEMMs, bias_col >= 0): row sums of A, accumulated by the n-tile 0
  // workgroups as they stash A (a k-contiguous dz tile) and reduced over the 16 k lanes at the end
  const bool bias_rows = !LA::kMC && bias_col >= 0 && blockIdx.y == 0;
  float bsum[LA::kMC ? 1 : EA];
#pragma unroll
  for (int i = 0; i < (LA::kMC ? 1 : EA); ++i) bsum[i] = 0.f;
  auto stash = [&](int buf) {
#pragma unroll
    for (int i = 0; i < EA; ++i) {
      float v;
      if constexpr (UA) v = ((va >> i) & 1) ? la.src.cvt(ra[i]) : 0.f;
      else v = ra[i];
      if constexpr (!LA::kMC) {
        if (bias_rows) bsum[i] += v;
      }
      if constexpr (LA::kMC) As[buf][tid / BM + (TPB / BM) * i][tid % BM] = v;
      else As[buf][tid % BK][tid / BK + (TPB / BK) * i] = v;
    }
#pragma unroll
    for (int i = 0; i < EB; ++i) {
      float v;
      if constexpr (UB) v = ((vb >> i) & 1) ? lb.src.cvt(rb[i]) : 0.f;
      else v = rb[i];
      if constexpr (LB::kMC) Bs[buf][tid / BN + (TPB / BN) * i][tid % BN] = v;
      else Bs[buf][tid % BK][tid / BK + (TPB / BK) * i] = v;
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = dev::zero_f32x4();

  const int lr = lane & 15, lk = lane >> 4;
  // this wave's k steps of a tile: all of them, or with KSPLIT waves per block every KSPLIT-th one
  // (wave-uniform start)
  constexpr int NKK = BK / 4 / KSPLIT;
  const int kk0 = 4 * __builtin_amdgcn_readfirstlane(wk);
  auto mfma_tile = [&](int buf) {
#pragma unroll
    for (int t = 0; t < NKK; ++t) {
      const int kk = (KSPLIT == 1 ? 4 * t : kk0 + 4 * KSPLIT * t) + lk;
      float a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = As[buf][kk][wm + 16 * i + lr];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = Bs[buf][kk][wn + 16 * j + lr];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)  // B as the row operand: D[n][m], lane l holds n = 4 (l >> 4) + r, m = l & 15
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[j], a[i], acc[i][j], 0, 0, 0);
    }
  };
  if (kbeg < kend) {
    fetch(kbeg);
    stash(0);
  }
  __syncthreads();
  int buf = 0;
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    const bool more = k0 + BK < kend;
    if (more) fetch(k0 + BK);  // next tile in flight during the MFMAs
    mfma_tile(buf);
    if (more) stash(buf ^ 1);  // the other buffer's last readers passed the previous barrier
    __syncthreads();
    buf ^= 1;
  }
  if constexpr (!LA::kMC) {
    if (bias_rows) {
      static_assert(BK == 16, "bias rows: one 16-lane group per A row");
#pragma unroll
      for (int i = 0; i < EA; ++i) {
        float v = bsum[i];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
        const int m = m0 + tid / BK + (TPB / BK) * i;
        if ((tid % BK) == 0 && m < M) epi.store(epi.row(m), bias_col, v);
      }
    }
  }
  if constexpr (KSPLIT > 1) {
    __shared__ f32x4 red[KSPLIT > 1 ? (KSPLIT - 1) * TM * TN * 64 : 1];
    if (wk > 0)
#pragma unroll
      for (int q = 0; q < TM * TN; ++q) red[((wk - 1) * TM * TN + q) * 64 + lane] = acc[q / TN][q % TN];
    __syncthreads();
    if (wk > 0) return;
#pragma unroll
    for (int w = 0; w < KSPLIT - 1; ++w)
#pragma unroll
      for (int q = 0; q < TM * TN; ++q) acc[q / TN][q % TN] += red[(w * TM * TN + q) * 64 + lane];
  }
  if constexpr (Epi::kPoolS1) {
    static_assert(BM == 128, "one image per 128-row tile");
    float* T = smem;  // [BN][LDT]; the k-loop ended with a barrier, As / Bs are dead
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int nl = wn + j * 16 + 4 * lk + r, n = n0 + nl;
          T[nl * LDT + wm + i * 16 + lr] = acc[i][j][r] + (epi.bias && n < N ? epi.bias[n] : 0.f);
        }
    __syncthreads();
    const int b = m0 >> 7;
    for (int idx = tid; idx < BN * epi.phw; idx += TPB) {
      const int nl = fdiv(idx, epi.fphw), q = idx - nl * epi.phw;
      if (n0 + nl >= N) break;
      const int py = fdiv(q, epi.fpw), px = q - py * epi.PW;
      const float* t = T + nl * LDT + py * epi.OW + px;
      const float v[4] = {t[0], t[1], t[epi.OW], t[epi.OW + 1]};
      float best = v[0];
      int bt = 0;
#pragma unroll
      for (int u = 1; u < 4; ++u)
        if (v[u] > best) { best = v[u]; bt = u; }
      const bool live = best > 0.f;
      const int64_t o = (static_cast<int64_t>(b) * N + n0 + nl) * epi.phw + q;
      epi.a[o] = live ? best : 0.f;
      epi.code[o] = live ? static_cast<unsigned char>(bt) : 255;
    }
  } else if constexpr (Epi::kPool) {
    const int tap = lr & 3;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm + i * 16 + lr;  // M is a multiple of 4: a window is all in or all out
      const int rowoff = epi.row(min(m, M - 1));
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n0 + wn + j * 16 + 4 * lk + r;
          // bias before the max, exactly as conv-then-pool (argmax ties included)
          float best = acc[i][j][r] + (epi.bias && n < N ? epi.bias[n] : 0.f);
          int bt = tap;
          // first maximum in window order wins, as max_pool2d; quad lane exchanges by DPP
          pool_quad_step<0xB1>(best, bt);  // xor 1: quad_perm [1,0,3,2]
          pool_quad_step<0x4E>(best, bt);  // xor 2: quad_perm [2,3,0,1]
          if (tap == 0 && m < M && n < N) {
            const bool live = best > 0.f;
            epi.a[rowoff + n * epi.phw] = live ? best : 0.f;
            epi.code[rowoff + n * epi.phw] = live ? static_cast<unsigned char>(bt) : 255;
          }
        }
    }
  } else {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm + i * 16 + lr;
      if (m >= M) continue;
      const int rowoff = epi.row(m);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n0 + wn + j * 16 + 4 * lk + r;
          if (n < N) epi.store(rowoff, n, acc[i][j][r]);
        }
    }
  }
}

// Workgroup tile layouts (WM, WN waves of TM x TN MFMA tiles), chosen per GEMM by its narrow side.
enum Layout { L32x32K4, L256x32, L128x64, L64x128, L32x128 };

constexpr int layout_bm(Layout l) { return l == L256x32 ? 256 : l == L128x64 ? 128 : l == L64x128 ? 64 : 32; }
constexpr int layout_bn(Layout l) { return l == L256x32 ? 32 : l == L128x64 ? 64 : l == L32x32K4 ? 32 : 128; }

// Forward / data-gradient GEMMs: m = pixels (huge), n = channels.  Weight gradients: m = output
// channels, n = input channels x taps (+ bias column), k = batch x pixels.
int f32_num_cus() {
  static const int n = [] {
    int dev = 0, v = 256;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      v = 256;
    return v;
  }();
  return n;
}

Layout pick_layout(int M, int N, int slices) {
  if (M <= 32 && N <= 32) return L32x32K4;
  if (M <= 32) return L32x128;
  Layout l = L64x128;
  if (N <= 32) l = L256x32;
  else if (N <= 64 || M >= 128) l = L128x64;
  // Small batches (the reference's 100 images per rank): the big tiles leave most CUs idle with one
  // long K loop each (conv3's data gradient at B=100: 79 workgroups, 97 us); 32x32 tiles with the
  // k-range split over the 4 waves fill the chip instead.
  const int bm = l == L256x32 ? 256 : (l == L128x64 ? 128 : 64), bn = l == L256x32 ? 32 : (l == L128x64 ? 64 : 128);
  const long blocks = (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  if (blocks * slices < f32_num_cus()) return L32x32K4;
  return l;
}

template <int WM, int WN, int TM, int TN, class LA, class LB, class Epi>
void launch_layout(int M, int N, int K, int per, int slices, int bias_col, const LA& la, const LB& lb,
                   const Epi& epi, hipStream_t s) {
  constexpr int BM = 16 * TM * WM, BN = 16 * TN * WN;
  dim3 grid(static_cast<unsigned>((M + BM - 1) / BM), static_cast<unsigned>((N + BN - 1) / BN),
            static_cast<unsigned>(slices));
  const int ktab_n = LA::kMC ? (K + BK - 1) / BK * BK : 0;
  hipLaunchKernelGGL((gemm_f32_kernel<WM, WN, TM, TN, LA, LB, Epi>), grid, dim3(TPB), ktab_n * sizeof(int2), s, M,
                     N, K, per, ktab_n, bias_col, la, lb, epi);
}

template <class LA, class LB, class Epi>
void launch_gemm(int M, int N, int K, int per, int slices, int bias_col, const LA& la, const LB& lb,
                 const Epi& epi, hipStream_t s) {
  switch (pick_layout(M, N, slices)) {
    case L32x32K4: launch_layout<1, 1, 2, 2>(M, N, K, per, slices, bias_col, la, lb, epi, s); break;
    case L256x32: launch_layout<4, 1, 4, 2>(M, N, K, per, slices, bias_col, la, lb, epi, s); break;
    case L128x64: launch_layout<4, 1, 2, 4>(M, N, K, per, slices, bias_col, la, lb, epi, s); break;
    case L64x128: launch_layout<2, 2, 2, 4>(M, N, K, per, slices, bias_col, la, lb, epi, s); break;
    case L32x128: launch_layout<1, 4, 2, 2>(M, N, K, per, slices, bias_col, la, lb, epi, s); break;
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

// 2x2/s2 windows with an even input width: two 8-B row loads per window.
__global__ __launch_bounds__(256) void pool2s2_fwd_kernel(const float* __restrict__ z, float* __restrict__ a,
                                                          unsigned char* __restrict__ code, int total, int H,
                                                          int W, FastDiv fphw, FastDiv fpw) {
  const int i = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= total) return;
  const int bc = fdiv(i, fphw), r = i - bc * static_cast<int>(fphw.d);
  const int py = fdiv(r, fpw), px = r - py * static_cast<int>(fpw.d);
  const float* zp = z + bc * H * W + (2 * py) * W + 2 * px;
  const float2 t = *reinterpret_cast<const float2*>(zp), b = *reinterpret_cast<const float2*>(zp + W);
  float best = t.x;
  int arg = 0;
  if (t.y > best) { best = t.y; arg = 1; }
  if (b.x > best) { best = b.x; arg = 2; }
  if (b.y > best) { best = b.y; arg = 3; }
  const bool live = best > 0.f;
  a[i] = live ? best : 0.f;
  code[i] = live ? static_cast<unsigned char>(arg) : 255;
}

// 2x2/s1 windows: the four loads issued together.
__global__ __launch_bounds__(256) void pool2s1_fwd_kernel(const float* __restrict__ z, float* __restrict__ a,
                                                          unsigned char* __restrict__ code, int total, int H,
                                                          int W, FastDiv fphw, FastDiv fpw) {
  const int i = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= total) return;
  const int bc = fdiv(i, fphw), r = i - bc * static_cast<int>(fphw.d);
  const int py = fdiv(r, fpw), px = r - py * static_cast<int>(fpw.d);
  const float* zp = z + bc * H * W + py * W + px;
  const float v0 = zp[0], v1 = zp[1], v2 = zp[W], v3 = zp[W + 1];
  float best = v0;
  int arg = 0;
  if (v1 > best) { best = v1; arg = 1; }
  if (v2 > best) { best = v2; arg = 2; }
  if (v3 > best) { best = v3; arg = 3; }
  const bool live = best > 0.f;
  a[i] = live ? best : 0.f;
  code[i] = live ? static_cast<unsigned char>(arg) : 255;
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
    // all 8 loads issued together (clamped in-plane addresses), then masked: one memory round trip
    int o[4];
    bool in[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int py = y - (q >> 1), px = x - (q & 1);
      in[q] = static_cast<unsigned>(py) < static_cast<unsigned>(PH) && static_cast<unsigned>(px) < static_cast<unsigned>(PW);
      o[q] = base + min(max(py, 0), PH - 1) * PW + min(max(px, 0), PW - 1);
    }
    int c[4];
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      c[q] = code[o[q]];
      v[q] = da[o[q]];
    }
    float g = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (in[q] && c[q] == q) g += v[q];
    dz[i] = g;
  }
}

// The same over tiles of 16 planes staged in LDS (16-B loads of da and the codes, coalesced stores of dz): the
// per-element form issues 8 scalar loads per output and ran at ~2.6 TB/s (conv2's pool2 backward at B=65536:
// 1.58 ms).  Needs PH * PW <= 128, PH * PW % 4 == 0 and a multiple of 16 planes.
constexpr int kP2Tile = 16;
// CPH / CPW > 0: compile-time window grid (the ConvNet's 10 x 10: the output index divisions become multiplies)
template <int CPH, int CPW>
// slices > 1: da is the data-gradient GEMM's split-K planes (slices x plane floats), summed in slice order while the
// tile is staged - the same sums as slab_sum_kernel, without its launch and the da round trip
__global__ __launch_bounds__(256) void pool2s1_bwd_tile_kernel(const float* __restrict__ da,
                                                               const unsigned char* __restrict__ code,
                                                               float* __restrict__ dz, int ntiles, int PH_, int PW_,
                                                               int slices, int64_t plane) {
  const int PH = CPH > 0 ? CPH : PH_, PW = CPW > 0 ? CPW : PW_;
  __shared__ __attribute__((aligned(16))) float D[kP2Tile * 128];
  __shared__ __attribute__((aligned(16))) unsigned char Cd[kP2Tile * 128];
  const int tid = threadIdx.x, W = PW + 1, hw = (PH + 1) * W, phw = PH * PW;
  const int n4 = kP2Tile * phw / 4, n16 = kP2Tile * phw / 16, nout = kP2Tile * hw;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t p0 = (int64_t)t * kP2Tile;
    const float4* src = reinterpret_cast<const float4*>(da + p0 * phw);
    for (int e = tid; e < n4; e += 256) {
      float4 acc = src[e];
      for (int z = 1; z < slices; ++z) {
        const float4 v = reinterpret_cast<const float4*>(da + z * plane + p0 * phw)[e];
        acc.x += v.x;
        acc.y += v.y;
        acc.z += v.z;
        acc.w += v.w;
      }
      reinterpret_cast<float4*>(D)[e] = acc;
    }
    const uint4* cs = reinterpret_cast<const uint4*>(code + p0 * phw);
    for (int e = tid; e < n16; e += 256) reinterpret_cast<uint4*>(Cd)[e] = cs[e];
    __syncthreads();
    float* out = dz + p0 * hw;
    for (int o = tid; o < nout; o += 256) {
      const int pl = o / hw, r = o - pl * hw, y = r / W, x = r - y * W;
      float g = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int py = y - (q >> 1), px = x - (q & 1);
        if (static_cast<unsigned>(py) < static_cast<unsigned>(PH) && static_cast<unsigned>(px) < static_cast<unsigned>(PW)) {
          const int i = pl * phw + py * PW + px;
          if (Cd[i] == q) g += D[i];
        }
      }
      out[o] = g;
    }
    __syncthreads();  // the tile is consumed before the next one is staged
  }
}

// Fixed-order sums of the split-K slabs [slices][Kout][Nw + has_bias]: stage 1 sums groups of
// kSlabGroup consecutive slices into part[group] (grid.y = groups), stage 2 sums the groups into
// dw [Kout][Nw] and db [Kout].  Two stages keep each thread's serial chain short.
constexpr int kSlabGroup = 32;
__global__ __launch_bounds__(256) void slab_group_kernel(const float* __restrict__ slab, int slices, int total,
                                                         float* __restrict__ part) {
  const int i = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= total) return;
  const int z0 = static_cast<int>(blockIdx.y) * kSlabGroup, z1 = min(z0 + kSlabGroup, slices);
  float acc = 0.f;
  for (int z = z0; z < z1; ++z) acc += slab[static_cast<int64_t>(z) * total + i];
  part[static_cast<int64_t>(blockIdx.y) * total + i] = acc;
}

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

// f32_slab_reduce of up to kF32RedMax segments in one launch: element e of a segment is the sum of its slices in
// the two-stage order of slab_group_kernel + wgrad_reduce_kernel (groups of kSlabGroup slices summed from 0.f,
// then the group sums in order; one group: the slices in order) - the same bits, done by one thread.
struct F32RedArgs {
  F32RedSeg seg[kF32RedMax];
  int bstart[kF32RedMax];  // first workgroup of each segment
  int n;
};
// Two kinds of workgroup, chosen per segment on the host: a segment of at most kSlabGroup slices (one group) gets
// 256 elements per workgroup, one thread each summing the slices in order (unconditional loads, all in flight);
// a segment with more slices gets 32 elements x 8 group lanes: lane q sums groups q, q + 8, .. into LDS and lane 0
// adds the group sums in order.  Both are the two-stage arithmetic of slab_group_kernel + wgrad_reduce_kernel.
// (One 32-element workgroup kind for every segment was 3553 workgroups at B=100 and ~20 us of dispatch; the
// serial one-thread form before it spent 20 us in conv1's 400-slice chain.)
constexpr int kRedLanes = 8, kRedElems = 256 / kRedLanes, kRedMaxGroups = 64;

__device__ __forceinline__ float red_group(const F32RedSeg& sg, int total, int e, int z0) {
  // unconditional loads (index clamped into the group) from a global-address-space pointer: a guarded load is a
  // branch the compiler will not hoist past, and the slab pointer read back from LDS would be a flat access
  const int nz = min(kSlabGroup, sg.slices - z0);
  const __attribute__((address_space(1))) float* src =
      (const __attribute__((address_space(1))) float*)(sg.slab + static_cast<int64_t>(z0) * total + e);
  float v[kSlabGroup];
#pragma unroll
  for (int z = 0; z < kSlabGroup; ++z) v[z] = src[static_cast<int64_t>(min(z, nz - 1)) * total];
  float p = 0.f;
#pragma unroll
  for (int z = 0; z < kSlabGroup; ++z)
    if (z < nz) p += v[z];
  return p;
}

__device__ __forceinline__ void red_store_f32(const F32RedSeg& sg, int e, float t) {
  const int m = e / sg.ncol, n = e - m * sg.ncol;
  if (n < sg.Nw) sg.dw[m * sg.Nw + n] = t;
  else sg.db[m] = t;
}

__global__ __launch_bounds__(256) void f32_reduce_multi_kernel(F32RedArgs a) {
  __shared__ float part[kRedMaxGroups][kRedElems];
  // the segment of this workgroup: compile-time indices into the by-value argument (a run-time index would copy
  // it to scratch per thread)
  int k = 0;
#pragma unroll
  for (int i = 1; i < kF32RedMax; ++i)
    if (i < a.n && (int)blockIdx.x >= a.bstart[i]) k = i;
  F32RedSeg sg = a.seg[0];
  int b0 = a.bstart[0];
#pragma unroll
  for (int i = 1; i < kF32RedMax; ++i)
    if (i == k) {
      sg = a.seg[i];
      b0 = a.bstart[i];
    }
  const int total = sg.Kout * sg.ncol, blk = (int)blockIdx.x - b0;
  const int ngroups = (sg.slices + kSlabGroup - 1) / kSlabGroup;
  if (ngroups == 1) {  // 256 elements, one thread each
    const int e = blk * 256 + (int)threadIdx.x;
    if (e < total) red_store_f32(sg, e, red_group(sg, total, e, 0));
    return;
  }
  const int el = threadIdx.x % kRedElems, q = threadIdx.x / kRedElems;
  const int e = blk * kRedElems + el;
  const bool live = e < total;
  const bool staged = ngroups <= kRedMaxGroups;
  for (int g = q; live && staged && g < ngroups; g += kRedLanes) part[g][el] = red_group(sg, total, e, g * kSlabGroup);
  __syncthreads();
  if (q != 0 || !live) return;
  float t;
  if (staged) {
    t = part[0][el];
    for (int g = 1; g < ngroups; ++g) t += part[g][el];
  } else {  // more slices than the LDS stage holds: every group in order by this thread
    t = red_group(sg, total, e, 0);
    for (int g = 1; g < ngroups; ++g) t += red_group(sg, total, e, g * kSlabGroup);
  }
  red_store_f32(sg, e, t);
}

// dx = sum over the split-K planes of NCHWSlabOut, in plane order (deterministic); n4 = plane / 4
__global__ __launch_bounds__(256) void slab_sum_kernel(const float4* __restrict__ slab, int slices, int n4,
                                                       float4* __restrict__ out) {
  for (int i = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x); i < n4;
       i += static_cast<int>(gridDim.x * blockDim.x)) {
    float4 acc = slab[i];
    for (int z = 1; z < slices; ++z) {
      const float4 v = slab[static_cast<int64_t>(z) * n4 + i];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    out[i] = acc;
  }
}

// ReLU + 2x2 max-pool (stride st) over the split-K planes of a plain NCHW conv output: each window value is
// the in-order sum of its slices plus the bias (bias before the max, as PoolOut / PoolS1Out), the first maximum
// in window order wins, code 255 where the result is 0.  One thread per pooled output.
// SC: the slice count at compile time (all 4 x SC loads of a window issued together), 0: run-time slices
template <int SC>
__global__ __launch_bounds__(256) void pool_slab_fwd_kernel(const float* __restrict__ slab, int slices_rt, int plane,
                                                            const float* __restrict__ bias, int C, int OH, int OW,
                                                            int st, int PH, int PW, int total, float* __restrict__ a,
                                                            unsigned char* __restrict__ code) {
  const int o = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
  if (o >= total) return;
  const int px = o % PW;
  int t = o / PW;
  const int py = t % PH;
  t /= PH;
  const int n = t % C;
  const int base = t * OH * OW + py * st * OW + px * st;  // t = b * C + n
  const float bn = bias ? bias[n] : 0.f;
  const int slices = SC > 0 ? SC : slices_rt;
  float best = 0.f;
  int bt = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = base + (u >> 1) * OW + (u & 1);
    float v = slab[i];
#pragma unroll
    for (int z = 1; z < (SC > 0 ? SC : 1); ++z) v += slab[static_cast<int64_t>(z) * plane + i];
    if (SC == 0)
      for (int z = 1; z < slices; ++z) v += slab[static_cast<int64_t>(z) * plane + i];
    v += bn;
    if (u == 0 || v > best) {
      best = v;
      bt = u;
    }
  }
  const bool live = best > 0.f;
  a[o] = live ? best : 0.f;
  code[o] = live ? static_cast<unsigned char>(bt) : 255;
}

int grid_1d(int64_t n) {
  const int64_t g = (n + 255) / 256;
  return static_cast<int>(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

// One element per thread for the pool kernels: their per-element loads are dependent (code, then
// gradient), so a grid-stride loop over a capped grid runs at one load round trip per iteration.
int grid_elems(int64_t n) { return static_cast<int>(std::max<int64_t>(1, (n + 255) / 256)); }

// Largest batch chunk whose per-chunk element counts (each listed per-image size) stay < 2^29, so
// every fp32 operand chunk is < 2^31 bytes: 32-bit buffer offsets, and kBadOff is out of range
// (RINGDP_F32_CHUNK_LIMIT lowers the bound: the tests run the chunked path at small batches).
int64_t batch_chunk(int64_t B, std::initializer_list<int64_t> per_image) {
  int64_t worst = 1;
  for (int64_t v : per_image) worst = std::max(worst, v);
  int64_t limit = (int64_t{1} << 29) - 1;
  if (const char* e = std::getenv("RINGDP_F32_CHUNK_LIMIT")) limit = std::max<int64_t>(1, std::min<int64_t>(limit, std::atoll(e)));
  const int64_t cap = limit / worst;
  return std::max<int64_t>(1, std::min(B, cap));
}

// RINGDP_F32_WGRAD_MIN_K: shallowest k slice of a weight gradient.  512 (was 1024): B=100 step 318 -> 296 us
// (256: 297, 128: 306); B=65536 unchanged (profiles/r05/fp32/).  320 on the round-6 step (every slab reduced by
// one launch, so more slices cost little): 216 -> 209 us (192: 217, 256: 211, 384: 212, 1024: 241;
// profiles/r06/fp32/b100_wgrad_depth_sweep.txt).
int wgrad_min_depth() {
  static const int d = [] {
    const char* e = std::getenv("RINGDP_F32_WGRAD_MIN_K");
    return e && *e ? std::max(BK, std::atoi(e)) : 320;
  }();
  return d;
}

int wgrad_slices(int M, int N, int64_t K) {
  // enough slices to put >= ~2048 workgroups on the 256 CUs, each slice >= wgrad_min_depth() deep
  const Layout l = pick_layout(M, N, 1 << 20);  // the big-tile layout (the launch may still pick 32x32)
  const int bm = layout_bm(l), bn = layout_bn(l);
  const int64_t tiles = static_cast<int64_t>((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  int64_t s = (2048 + tiles - 1) / tiles;
  // K below one minimum-depth slice on a grid of < 64 tiles (fc1 at B=100: 16 tiles, K = 100): 2-k-tile slices
  const int depth = (K < wgrad_min_depth() && tiles < 64) ? 2 * BK : wgrad_min_depth();
  const int64_t cap = (K + depth - 1) / depth;
  if (s > cap) s = cap;
  return static_cast<int>(s < 1 ? 1 : (s > 1024 ? 1024 : s));
}

int64_t wgrad_chunk(const ConvF32Geom& g) {
  return batch_chunk(g.B, {static_cast<int64_t>(g.C) * g.H * g.W, static_cast<int64_t>(g.Kout) * g.OH * g.OW});
}

// Linear layer with few outputs (the ConvNet's fc1: N = 10, K = 2048) at small batches: the GEMM core's
// single 128-row tile ran K serially in one workgroup (163 us at B=100).  One wave per input row: lane l
// accumulates k = l, l+64, ... for every output, then a fixed butterfly sums the lanes (deterministic).
template <int N>
__global__ __launch_bounds__(256) void linear_skinny_f32_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                              const float* __restrict__ bias, float* __restrict__ z,
                                                              int M, int K) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float* xr = x + (int64_t)row * K;
  float acc[N];
#pragma unroll
  for (int n = 0; n < N; ++n) acc[n] = 0.f;
  for (int k = lane; k < K; k += 64) {
    const float v = xr[k];
#pragma unroll
    for (int n = 0; n < N; ++n) acc[n] = fmaf(v, w[(int64_t)n * K + k], acc[n]);
  }
#pragma unroll
  for (int n = 0; n < N; ++n) {
    float v = acc[n];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    acc[n] = v;
  }
  if (lane < N) {
    float v = 0.f;
#pragma unroll
    for (int n = 0; n < N; ++n) v = lane == n ? acc[n] : v;
    z[(int64_t)row * N + lane] = v + (bias ? bias[lane] : 0.f);
  }
}

// The same with one 256-thread workgroup per row and 16-B loads (K % 4 == 0, 16-B aligned rows): each
// thread's chain is K / 1024 float4 steps instead of K / 64 scalar ones (B=100 fc1: 14.8 us -> see
// profiles/r05/fp32/); per-wave sums, then the 4 waves in order (deterministic).
template <int N>
__global__ __launch_bounds__(256) void linear_row_f32_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                             const float* __restrict__ bias, float* __restrict__ z,
                                                             int K) {
  __shared__ float red[4][N];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = blockIdx.x;
  const float4* xr = reinterpret_cast<const float4*>(x + (int64_t)row * K);
  const int K4 = K >> 2;
  float acc[N];
#pragma unroll
  for (int n = 0; n < N; ++n) acc[n] = 0.f;
  for (int k = tid; k < K4; k += 256) {
    const float4 v = xr[k];
#pragma unroll
    for (int n = 0; n < N; ++n) {
      const float4 q = reinterpret_cast<const float4*>(w + (int64_t)n * K)[k];
      acc[n] = fmaf(v.x, q.x, fmaf(v.y, q.y, fmaf(v.z, q.z, fmaf(v.w, q.w, acc[n]))));
    }
  }
#pragma unroll
  for (int n = 0; n < N; ++n) {
    float v = acc[n];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[wave][n] = v;
  }
  __syncthreads();
  if (tid < N) z[(int64_t)row * N + tid] = ((red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid])) + (bias ? bias[tid] : 0.f);
}

}  // namespace

bool conv3_wgrad_f32_ok(const ConvF32Geom& g);  // (below, with their kernels)
bool conv2_wgrad_f32_ok(const ConvF32Geom& g);
constexpr int W3_SLICES = 128;                    // its image slices (slab rows): 512 workgroups, 2 per CU
constexpr int W2_SLICES = 256;                    // conv2's (2 channel tiles): 512 workgroups

int conv_f32_wgrad_slices(const ConvF32Geom& g) {
  if (conv3_wgrad_f32_ok(g)) return W3_SLICES + (W3_SLICES + kSlabGroup - 1) / kSlabGroup;
  if (conv2_wgrad_f32_ok(g)) return W2_SLICES + (W2_SLICES + kSlabGroup - 1) / kSlabGroup;
  const int64_t chunk = wgrad_chunk(g);
  const int64_t nchunks = (g.B + chunk - 1) / chunk;
  const int slices = static_cast<int>(nchunks) *
                     wgrad_slices(g.Kout, g.C * g.R * g.R, chunk * static_cast<int64_t>(g.OH) * g.OW);
  return slices + (slices + kSlabGroup - 1) / kSlabGroup;  // + room for the stage-1 group sums
}

void conv_f32_fwd(const ConvF32Geom& g, const float* x, const unsigned char* xu8, float mean, float inv_std,
                  const float* w, const float* bias, float* z, hipStream_t s) {
  const int K = g.C * g.R * g.R;
  if (!xu8 && g.R == 1 && g.H == 1 && g.W == 1 && g.Kout == 10 && g.B <= 8192) {  // fc1 at small batches
    if (K % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(w) & 15) == 0)
      linear_row_f32_kernel<10><<<static_cast<unsigned>(g.B), 256, 0, s>>>(x, w, bias, z, K);
    else
      linear_skinny_f32_kernel<10><<<static_cast<unsigned>((g.B + 3) / 4), 256, 0, s>>>(x, w, bias, z,
                                                                                       static_cast<int>(g.B), K);
    return;
  }
  const int64_t xin = static_cast<int64_t>(g.C) * g.H * g.W, zout = static_cast<int64_t>(g.Kout) * g.OH * g.OW;
  const int64_t chunk = batch_chunk(g.B, {xin, zout});
  for (int64_t b0 = 0; b0 < g.B; b0 += chunk) {
    const int nb = static_cast<int>(std::min(chunk, g.B - b0));
    const int M = nb * g.OH * g.OW;
    const int xbytes = static_cast<int>(nb * xin);
    WeightB lb{{w, K * g.Kout * 4, 0.f, 1.f}, K, g.Kout};
    NCHWOut epi{z + b0 * zout, bias, g.Kout, M, make_fdiv(g.OH * g.OW)};
    if (xu8) {
      FwdA<true, true> la{{xu8 + b0 * xin, xbytes, mean, inv_std}, g.C, g.H, g.W, g.R, g.pad, g.OW, K, M,
                          make_fdiv(g.OH * g.OW), make_fdiv(g.OW)};
      launch_gemm(M, g.Kout, K, K, 1, -1, la, lb, epi, s);
    } else if (g.pad) {
      FwdA<false, true> la{{x + b0 * xin, xbytes * 4, 0.f, 1.f}, g.C, g.H, g.W, g.R, g.pad, g.OW, K, M,
                           make_fdiv(g.OH * g.OW), make_fdiv(g.OW)};
      launch_gemm(M, g.Kout, K, K, 1, -1, la, lb, epi, s);
    } else {
      FwdA<false, false> la{{x + b0 * xin, xbytes * 4, 0.f, 1.f}, g.C, g.H, g.W, g.R, g.pad, g.OW, K, M,
                            make_fdiv(g.OH * g.OW), make_fdiv(g.OW)};
      launch_gemm(M, g.Kout, K, K, 1, -1, la, lb, epi, s);
    }
  }
}

// ---------------------------------------------------------------- conv3 + ReLU + pool3 forward (fp32)
// The ConvNet's conv3 (64 -> 128 channels, 3x3 valid, 10x10 -> 8x8) with bias, ReLU and the 2x2/s2 max-pool
// (-> 4x4, + the argmax code of pool_relu / PoolOut) as one persistent 512-thread workgroup per CU.  Its
// 128 x 576 weights (295 KB) do not fit in LDS but do fit in the 8 waves' registers: wave w owns output
// channels [16 w, +16) and holds their whole K (144 k-steps of 4, tap-major: k = 64 tap + ci) as B operands,
// 144 VGPRs per lane, loaded once per launch.  Per image the waves share one LDS copy of the input (64
// channels x 10 x 10, row stride 112 floats = 16 banks apart, so the two channel rows of a b32 read never
// collide) and each runs 4 m-tiles x 144 k-steps with 4 independent accumulators.  The m-tile rows are
// window-major (row r of tile t: window 4 (r / 4) + t, tap r % 4), so a lane's 4 accumulator registers of
// tile t are the 4 pixels of window 4 lk + t: the pool is a register reduction and a lane's 4 tiles give 4
// consecutive pooled outputs of one channel (one float4 + one dword of codes per lane and image).
// The next image's input is loaded into registers during the k loop and stored to the other LDS buffer.
namespace {
constexpr int C3P_S = 112;  // floats per input channel row in LDS (100 + 12; 112 = 16 mod 32)

__global__ __launch_bounds__(512, 1) void conv3_pool_f32_kernel(const float* __restrict__ x,
                                                                const float* __restrict__ w,
                                                                const float* __restrict__ bias,
                                                                float* __restrict__ a,
                                                                unsigned char* __restrict__ code, int B) {
  __shared__ __attribute__((aligned(16))) float XI[2][64 * C3P_S];  // 2 x 28 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const int co = 16 * wave + lr;
  // B[k = 4 ks + lk][n = lr] = w[co][ci = 4 (ks & 15) + lk][tap = ks >> 4]
  float wr[144];
  {
    const float* wc = w + co * 576;
#pragma unroll
    for (int ks = 0; ks < 144; ++ks) wr[ks] = wc[(4 * (ks & 15) + lk) * 9 + (ks >> 4)];
  }
  const float bv = bias[co];
  // A: row lr of m-tile t = pixel (2 (lr >> 2) + ((lr >> 1) & 1), 2 t + (lr & 1)) of channel 4 (ks & 15) + lk
  int abase[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) abase[t] = lk * C3P_S + (2 * (lr >> 2) + ((lr >> 1) & 1)) * 10 + 2 * t + (lr & 1);
  auto koff = [](int ks) { const int tap = ks >> 4; return 4 * (ks & 15) * C3P_S + (tap / 3) * 10 + tap % 3; };
  // staging: an image is 1600 float4 (channel e / 25, column 4 (e % 25)); threads take 3 or 4 (named
  // registers: an array of them was left on the scratch stack)
  float4 st0, st1, st2, st3;
  auto load = [&](int b) {
    const float4* src = reinterpret_cast<const float4*>(x + (int64_t)b * 6400) + tid;
    st0 = src[0];
    st1 = src[512];
    st2 = src[1024];
    st3 = src[tid < 64 ? 1536 : 0];
  };
  auto put = [&](float* buf, int e, const float4& v) {
    const int c = e / 25, q = 4 * (e - 25 * c);
    *reinterpret_cast<float4*>(buf + c * C3P_S + q) = v;
  };
  auto stash = [&](float* buf) {
    put(buf, tid, st0);
    put(buf, tid + 512, st1);
    put(buf, tid + 1024, st2);
    if (tid < 64) put(buf, tid + 1536, st3);
  };
  int b = blockIdx.x;
  if (b < B) {
    load(b);
    stash(XI[0]);
  }
  __syncthreads();
  int cur = 0;
  for (; b < B; b += gridDim.x) {
    const int nb = b + gridDim.x;
    if (nb < B) load(nb);  // lands during the k loop
    const float* X = XI[cur];
    f32x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = f32x4{bv, bv, bv, bv};
    // k-step-major: the next k-step's 4 A reads issued ahead of this one's 4 MFMAs
    float av[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) av[t] = X[abase[t] + koff(0)];
#pragma unroll
    for (int ks = 0; ks < 144; ++ks) {
      float an[4];
      if (ks + 1 < 144) {
#pragma unroll
        for (int t = 0; t < 4; ++t) an[t] = X[abase[t] + koff(ks + 1)];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t], wr[ks], acc[t], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (ks + 1 < 144) {
#pragma unroll
        for (int t = 0; t < 4; ++t) av[t] = an[t];
      }
    }
    // lane: D[row 4 lk + r][co] of tile t = window 4 lk + t, tap r (row-major in the window)
    float o[4];
    uint32_t cw = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const f32x4 v = acc[t];
      const float best = fmaxf(fmaxf(fmaxf(v[0], v[1]), v[2]), v[3]);
      const uint32_t arg = v[0] == best ? 0u : v[1] == best ? 1u : v[2] == best ? 2u : 3u;  // first maximum
      const bool live = best > 0.f;
      o[t] = live ? best : 0.f;
      cw |= (live ? arg : 255u) << (8 * t);
    }
    reinterpret_cast<float4*>(a + (int64_t)b * 2048 + co * 16)[lk] = make_float4(o[0], o[1], o[2], o[3]);
    reinterpret_cast<uint32_t*>(code + (int64_t)b * 2048 + co * 16)[lk] = cw;
    if (nb < B) stash(XI[cur ^ 1]);
    __syncthreads();  // the next image staged; this one's reads done before it is overwritten next round
    cur ^= 1;
  }
}
}  // namespace

// smallest batch that takes the dedicated conv2 / conv3 forward kernels (one image per workgroup at a time)
// instead of split K + pool_slab_fwd (RINGDP_F32_FWD_MIN_B overrides; default 4 images per CU)
static int f32_fwd_dedicated_min_b() {
  static const int v = [] {
    const char* e = std::getenv("RINGDP_F32_FWD_MIN_B");
    return e && *e ? std::atoi(e) : 4 * f32_num_cus();
  }();
  return v;
}

bool conv3_pool_f32_ok(const ConvF32Geom& g) {
  static const bool on = [] {
    const char* v = std::getenv("RINGDP_F32_CONV3_FWD");
    return !(v && v[0] == '0');
  }();
  return on && g.Kout == 128 && g.C == 64 && g.R == 3 && g.pad == 0 && g.H == 10 && g.W == 10 &&
         g.B >= f32_fwd_dedicated_min_b() && g.B * 6400 < (int64_t{1} << 31);
}

void conv_f32_fwd_pool(const ConvF32Geom& g, const float* x, const unsigned char* xu8, float mean, float inv_std,
                       const float* w, const float* bias, float* a, unsigned char* code, hipStream_t s) {
  const int K = g.C * g.R * g.R;
  if (bias && !xu8 && conv3_pool_f32_ok(g)) {  // the ConvNet's conv3 at large batches: the dedicated kernel
    const int grid = static_cast<int>(std::min<int64_t>(g.B, f32_num_cus()));
    hipLaunchKernelGGL(conv3_pool_f32_kernel, dim3(grid), dim3(512), 0, s, x, w, bias, a, code, static_cast<int>(g.B));
    return;
  }
  const int phw = (g.OH / 2) * (g.OW / 2);
  const int64_t xin = static_cast<int64_t>(g.C) * g.H * g.W, aout = static_cast<int64_t>(g.Kout) * phw;
  const int64_t chunk = batch_chunk(g.B, {xin, static_cast<int64_t>(g.Kout) * g.OH * g.OW});
  for (int64_t b0 = 0; b0 < g.B; b0 += chunk) {
    const int nb = static_cast<int>(std::min(chunk, g.B - b0));
    const int M = nb * g.OH * g.OW;
    const int xbytes = static_cast<int>(nb * xin);
    WeightB lb{{w, K * g.Kout * 4, 0.f, 1.f}, K, g.Kout};
    PoolOut epi{a + b0 * aout, code + b0 * aout, bias, g.Kout, M, phw, make_fdiv(g.OH * g.OW)};
    const FastDiv fpw = make_fdiv(g.OW / 2);
    if (xu8) {
      FwdA<true, true, true> la{{xu8 + b0 * xin, xbytes, mean, inv_std}, g.C, g.H, g.W, g.R, g.pad, g.OW, K, M,
                                make_fdiv(g.OH * g.OW), fpw};
      launch_gemm(M, g.Kout, K, K, 1, -1, la, lb, epi, s);
    } else if (g.pad) {
      FwdA<false, true, true> la{{x + b0 * xin, xbytes * 4, 0.f, 1.f}, g.C, g.H, g.W, g.R, g.pad, g.OW, K, M,
                                 make_fdiv(g.OH * g.OW), fpw};
      launch_gemm(M, g.Kout, K, K, 1, -1, la, lb, epi, s);
    } else {
      FwdA<false, false, true> la{{x + b0 * xin, xbytes * 4, 0.f, 1.f}, g.C, g.H, g.W, g.R, g.pad, g.OW, K, M,
                                  make_fdiv(g.OH * g.OW), fpw};
      launch_gemm(M, g.Kout, K, K, 1, -1, la, lb, epi, s);
    }
  }
}

// ---------------------------------------------------------------- conv2 + ReLU + pool2 forward (fp32)
// The ConvNet's conv2 (32 -> 64 channels, 3x3 valid, 13x13 -> 11x11) with bias, ReLU and the overlapping 2x2/s1
// max-pool (+ its argmax code, pool2s1_fwd_kernel semantics) as one persistent kernel, two 256-thread
// workgroups per CU.  Wave w owns output channels [16 w, +16) with its 16 x 288 weights resident in registers
// (72 per lane); K runs tap-major (k = 32 tap + ci), so an A fragment - 16 positions x 4 input channels of one
// tap - is one b32 read of the LDS image at a per-lane base + a compile-time offset (no index math in the
// loop).  The 121 positions are 8 tiles of 16 (the last 7 rows read the image's tail and are never stored).
// Epilogue: conv + bias to an LDS tile, then pool + ReLU + code, 4 outputs (float4 / 4 code bytes) per thread.
namespace {
constexpr int C2F_ZS = 121 + 3;  // floats per channel row of the conv output tile

__global__ __launch_bounds__(256, 2) void conv2_pool_f32_kernel(const float* __restrict__ x,
                                                                 const float* __restrict__ w,
                                                                 const float* __restrict__ bias,
                                                                 float* __restrict__ a,
                                                                 unsigned char* __restrict__ code, int B) {
  __shared__ __attribute__((aligned(16))) float XI[5408 + 128];     // 22.1 KB: the input image (+ tail)
  __shared__ __attribute__((aligned(16))) float Z[64 * C2F_ZS];     // 31.7 KB: conv + bias
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  // weights: lane holds B[k = 4 ks + lk][co = 16 wave + lr] = w[co][ci = (4 ks + lk) & 31][tap = ks >> 3]
  float wr[72];
  {
    const float* wc = w + (16 * wave + lr) * 288;
#pragma unroll
    for (int ks = 0; ks < 72; ++ks) wr[ks] = wc[((4 * ks + lk) & 31) * 9 + (ks >> 3)];
  }
  const float bv = bias[16 * wave + lr];
  // A base per position tile: lane row p = 16 i + lr -> (oy, ox); + the input channel lk
  int pbase[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int p = min(16 * i + lr, 120);  // rows past 120: a real pixel, product never stored
    pbase[i] = lk * 169 + (p / 11) * 13 + p % 11;
  }
  // staging: the image is 5408 floats = 1352 float4, 5 or 6 per thread, loaded into named registers one image
  // ahead (in flight during the k loop) and stored after the pool phase
  float4 s0, s1, s2, s3, s4, s5;
  auto load = [&](int b) {
    const float4* src = reinterpret_cast<const float4*>(x + (int64_t)b * 5408) + tid;
    s0 = src[0];
    s1 = src[256];
    s2 = src[512];
    s3 = src[768];
    s4 = src[1024];
    s5 = src[tid < 72 ? 1280 : 0];
  };
  auto stash = [&]() {
    float4* d = reinterpret_cast<float4*>(XI) + tid;
    d[0] = s0;
    d[256] = s1;
    d[512] = s2;
    d[768] = s3;
    d[1024] = s4;
    if (tid < 72) d[1280] = s5;
  };
  if (blockIdx.x < B) {
    load(blockIdx.x);
    stash();
  }
  __syncthreads();
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    const int nb = b + gridDim.x;
    if (nb < B) load(nb);
    f32x4 acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = dev::zero_f32x4();
    // k-step-major with the next k-step's 8 A reads issued ahead of this one's 8 MFMAs (independent
    // accumulators back to back; left to itself the scheduler ran one position tile's 72 dependent MFMAs
    // in a row: 4.27 ms at B=65536)
    auto koff = [](int ks) { const int tap = ks >> 3; return 4 * (ks & 7) * 169 + (tap / 3) * 13 + tap % 3; };
    float av[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) av[i] = XI[pbase[i] + koff(0)];
#pragma unroll
    for (int ks = 0; ks < 72; ++ks) {
      float an[8];
      if (ks + 1 < 72) {
#pragma unroll
        for (int i = 0; i < 8; ++i) an[i] = XI[pbase[i] + koff(ks + 1)];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], wr[ks], acc[i], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (ks + 1 < 72) {
#pragma unroll
        for (int i = 0; i < 8; ++i) av[i] = an[i];
      }
    }
    // lane holds D[p = 16 i + 4 lk + r][co = 16 wave + lr]
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * i + 4 * lk + r;
        if (p < 121) Z[(16 * wave + lr) * C2F_ZS + p] = acc[i][r] + bv;
      }
    __syncthreads();
    // pool: quads of 4 consecutive outputs of one channel (100 per channel: never crossing a channel)
    float4* ao = reinterpret_cast<float4*>(a + (int64_t)b * 6400);
    uint32_t* co = reinterpret_cast<uint32_t*>(code + (int64_t)b * 6400);
    for (int qd = tid; qd < 1600; qd += 256) {
      const int ch = qd / 25, q0 = 4 * (qd - 25 * ch);
      float o[4];
      uint32_t cw = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = q0 + j, py = q / 10, px = q - 10 * py;
        const float* t = Z + ch * C2F_ZS + py * 11 + px;
        const float v0 = t[0], v1 = t[1], v2 = t[11], v3 = t[12];
        float best = v0;
        uint32_t arg = 0;
        if (v1 > best) { best = v1; arg = 1; }
        if (v2 > best) { best = v2; arg = 2; }
        if (v3 > best) { best = v3; arg = 3; }
        const bool live = best > 0.f;
        o[j] = live ? best : 0.f;
        cw |= (live ? arg : 255u) << (8 * j);
      }
      ao[qd] = make_float4(o[0], o[1], o[2], o[3]);
      co[qd] = cw;
    }
    if (nb < B) stash();  // XI was last read by the k loop, before the barrier above
    __syncthreads();  // Z free, the next image staged
  }
}
}  // namespace

bool conv2_pool_f32_ok(const ConvF32Geom& g) {
  static const bool on = [] {
    const char* v = std::getenv("RINGDP_F32_CONV2_FWD");
    return !(v && v[0] == '0');
  }();
  return on && g.Kout == 64 && g.C == 32 && g.R == 3 && g.pad == 0 && g.H == 13 && g.W == 13 &&
         g.B >= f32_fwd_dedicated_min_b() && g.B * 6400 < (int64_t{1} << 31);
}

void conv2_pool_f32(const ConvF32Geom& g, const float* x, const float* w, const float* bias, float* a,
                    unsigned char* code, hipStream_t s) {
  const int grid = static_cast<int>(std::min<int64_t>(g.B, 2 * f32_num_cus()));
  hipLaunchKernelGGL(conv2_pool_f32_kernel, dim3(grid), dim3(256), 0, s, x, w, bias, a, code, static_cast<int>(g.B));
}

void conv_f32_fwd_pool_s1(const ConvF32Geom& g, const float* x, const float* w, const float* bias, float* a,
                          unsigned char* code, hipStream_t s) {
  if (bias && conv2_pool_f32_ok(g)) {  // the ConvNet's conv2 at large batches: the dedicated kernel
    conv2_pool_f32(g, x, w, bias, a, code, s);
    return;
  }
  const int K = g.C * g.R * g.R;
  const int PH = g.OH - 1, PW = g.OW - 1, phw = PH * PW;
  const int64_t xin = static_cast<int64_t>(g.C) * g.H * g.W, aout = static_cast<int64_t>(g.Kout) * phw;
  const int64_t chunk = batch_chunk(g.B, {xin, int64_t{128} * g.Kout});
  for (int64_t b0 = 0; b0 < g.B; b0 += chunk) {
    const int nb = static_cast<int>(std::min(chunk, g.B - b0));
    const int M = nb * 128;
    WeightB lb{{w, K * g.Kout * 4, 0.f, 1.f}, K, g.Kout};
    PoolS1Out epi{a + b0 * aout, code + b0 * aout, bias, g.Kout, g.OW, PW, phw, make_fdiv(phw), make_fdiv(PW)};
    if (g.pad) {
      FwdA<false, true, 2> la{{x + b0 * xin, static_cast<int>(nb * xin * 4), 0.f, 1.f}, g.C, g.H, g.W, g.R, g.pad,
                              g.OW, K, M, make_fdiv(g.OH * g.OW), make_fdiv(g.OW)};
      launch_layout<4, 1, 2, 4>(M, g.Kout, K, K, 1, -1, la, lb, epi, s);
    } else {
      FwdA<false, false, 2> la{{x + b0 * xin, static_cast<int>(nb * xin * 4), 0.f, 1.f}, g.C, g.H, g.W, g.R, g.pad,
                               g.OW, K, M, make_fdiv(g.OH * g.OW), make_fdiv(g.OW)};
      launch_layout<4, 1, 2, 4>(M, g.Kout, K, K, 1, -1, la, lb, epi, s);
    }
  }
}

// Small batches, valid convs with a fused pool (the ConvNet's conv2 / conv3 at B=100: 100 one-image tiles x 18
// k-tiles, 800 32x32 tiles x 36 k-tiles, ~30 us each): the same k split as the data gradient below, into planes
// of the plain conv output, then pool_slab_fwd_kernel sums, adds the bias and pools.  RINGDP_F32_FWD_SLICES=n
// forces n (1: the one-launch fused kernels).
int conv_f32_fwd_slices(const ConvF32Geom& g) {
  if (g.pad != 0 || conv2_pool_f32_ok(g) || conv3_pool_f32_ok(g)) return 1;
  const int K = g.C * g.R * g.R;
  const int64_t xin = static_cast<int64_t>(g.C) * g.H * g.W, zout = static_cast<int64_t>(g.Kout) * g.OH * g.OW;
  if (batch_chunk(g.B, {xin, zout}) < g.B) return 1;
  const int64_t M = g.B * g.OH * g.OW, plane = M * g.Kout;
  const int64_t tiles32 = ((M + 31) / 32) * ((g.Kout + 31) / 32);
  int s = tiles32 >= 8 * f32_num_cus() ? 1 : std::min(8, (K + 8 * BK - 1) / (8 * BK));
  if (const char* e = std::getenv("RINGDP_F32_FWD_SLICES")) {
    const int v = std::atoi(e);
    if (v > 0) s = v;
  }
  s = std::max(1, std::min(s, std::min(16, (K + BK - 1) / BK)));
  if (static_cast<int64_t>(s) * plane >= (int64_t{1} << 29)) return 1;
  return s;
}

void conv_f32_fwd_pool_split(const ConvF32Geom& g, const float* x, const float* w, const float* bias, float* slab,
                             int slices, int st, float* a, unsigned char* code, hipStream_t s) {
  const int K = g.C * g.R * g.R;
  const int M = static_cast<int>(g.B * g.OH * g.OW);
  const int plane = M * g.Kout;
  int per = (K + slices - 1) / slices;
  per = (per + BK - 1) / BK * BK;
  const int used = (K + per - 1) / per;
  const int64_t xin = static_cast<int64_t>(g.C) * g.H * g.W;
  WeightB lb{{w, K * g.Kout * 4, 0.f, 1.f}, K, g.Kout};
  FwdA<false, false> la{{x, static_cast<int>(g.B * xin * 4), 0.f, 1.f}, g.C, g.H, g.W, g.R, g.pad, g.OW, K, M,
                        make_fdiv(g.OH * g.OW), make_fdiv(g.OW)};
  NCHWSlabOut epi{slab, g.Kout, M, plane, make_fdiv(g.OH * g.OW)};
  launch_gemm(M, g.Kout, K, per, used, -1, la, lb, epi, s);
  const int PH = st == 2 ? g.OH / 2 : g.OH - 1, PW = st == 2 ? g.OW / 2 : g.OW - 1;
  const int total = static_cast<int>(g.B) * g.Kout * PH * PW;
  const dim3 grid((total + 255) / 256);
#define RINGDP_POOL_SLAB(SCV)                                                                                         \
  hipLaunchKernelGGL(pool_slab_fwd_kernel<SCV>, grid, dim3(256), 0, s, slab, used, plane, bias, g.Kout, g.OH, g.OW, st, \
                     PH, PW, total, a, code)
  switch (used) {
    case 2: RINGDP_POOL_SLAB(2); break;
    case 3: RINGDP_POOL_SLAB(3); break;
    case 4: RINGDP_POOL_SLAB(4); break;
    case 5: RINGDP_POOL_SLAB(5); break;
    case 6: RINGDP_POOL_SLAB(6); break;
    case 8: RINGDP_POOL_SLAB(8); break;
    default: RINGDP_POOL_SLAB(0); break;
  }
#undef RINGDP_POOL_SLAB
}

// Small batches (the reference's 100 images): the data-gradient GEMM has few workgroups, each with one long k
// loop that is latency-bound (B=100 conv3: 626 workgroups of 32x32 x 72 k-tiles, 63 us).  Split K into slices
// of ~8 k-tiles (at most 8 slices): the grid then takes the big-tile layouts again (fewer gathers per MFMA)
// and the slices' partial dx planes are summed in order by slab_sum_kernel.  B=100 step, forced counts
// (profiles/r05/fp32/): 1 slice 353 us, 2: 353, 3: 342, 4: 329, 6: 313, 8: 312, 12: 317.  At least 6 slices on the
// round-6 step (conv2's 18 k-tiles had 3): 209 -> 207 us (forced 4: 220, 10: 207;
// profiles/r06/fp32/b100_slices_sweep.txt).  Big batches (>= 8 32x32 tiles per CU) and chunked batches keep one
// slice.  RINGDP_F32_DGRAD_SLICES=n forces n (1: off).
int conv_f32_dgrad_slices(const ConvF32Geom& g) {
  const int K = g.Kout * g.R * g.R;
  const int64_t zin = static_cast<int64_t>(g.Kout) * g.OH * g.OW, xout = static_cast<int64_t>(g.C) * g.H * g.W;
  if (batch_chunk(g.B, {zin, xout}) < g.B) return 1;
  const int64_t M = g.B * g.H * g.W, plane = M * g.C;
  if (plane % 4 != 0) return 1;
  const int64_t tiles32 = ((M + 31) / 32) * ((g.C + 31) / 32);
  int s = tiles32 >= 8 * f32_num_cus() ? 1 : std::min(8, std::max(6, (K + 8 * BK - 1) / (8 * BK)));
  if (const char* e = std::getenv("RINGDP_F32_DGRAD_SLICES")) {
    const int v = std::atoi(e);
    if (v > 0) s = v;
  }
  s = std::max(1, std::min(s, std::min(16, (K + BK - 1) / BK)));
  if (static_cast<int64_t>(s) * plane >= (int64_t{1} << 29)) return 1;
  return s;
}

// ---------------------------------------------------------------- conv3 data gradient, scatter form
// The ConvNet's conv3 (64 -> 128 channels, 3x3 valid, 10x10 -> 8x8) data gradient as one GEMM per kernel tap
// over the LIVE positions only: P_t[p][ci] = sum_co dz[co][p] * w[co][ci][t] (p over the 8x8 dz positions),
// scattered into dx[ci][p + (kh, kw)].  The implicit-GEMM path correlates the zero-padded 12x12 dz against
// the 10x10 output, and 36 % of its MACs multiply padding (profiles/r05/fp32/).
// One 256-thread workgroup per CU, persistent over images; wave w owns the 16 input channels
// [16 w, 16 w + 16) for all 9 taps and all 64 positions, so every A fragment (4 co x 16 positions) read from
// LDS feeds 9 MFMAs and no two waves write the same dx element.  The weights stay in L2: a lane streams its
// 9 tap values per k-step (3 x 16 B, repacked once per call into [wave][k-step][lane][12]) two k-steps ahead.
// col2im: tap by tap (fixed order: deterministic) into a wave-private fp32 LDS image, then stored
// coalesced - the wave's 16 x 100 outputs are one contiguous NCHW run.  The next image's dz (32 KB) is loaded
// into registers while this one multiplies and stashed to the other LDS buffer behind the same barrier (loads
// are counted in order, so the first weight wait also waits for that HBM round trip; issued after the k-loop
// instead, the stash waited for it: 5.9 -> 6.6 ms at B=65536).
// Exact fp32 MFMA (v_mfma_f32_16x16x4_f32): results differ from the GEMM path only by summation order.
constexpr int D3_AS = 80;   // floats per co row of the staged dz image (64 + 16: the 2 k rows of a b32 read
                            // land 16 banks apart)
constexpr int D3_XS = 101;  // floats per channel row of a wave's dx image (odd: the 16 channel rows of a
                            // b32 RMW hit 16 distinct banks)
constexpr int D3_WP = 4 * 32 * 9 * 64;  // repacked weights (floats): [wave][k-step][tap][lane]

__global__ __launch_bounds__(256) void d3_repack_kernel(const float* __restrict__ w, float* __restrict__ wp) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= D3_WP) return;
  const int lane = i & 63, t = (i >> 6) % 9, ks = (i / 576) & 31, ct = i / 18432;
  const int co = ks * 4 + (lane >> 4), ci = ct * 16 + (lane & 15);
  wp[i] = w[(co * 64 + ci) * 9 + t];
}

__global__ __launch_bounds__(256, 2) void conv3_dgrad_f32_kernel(const float* __restrict__ dz,
                                                                  const float* __restrict__ wp,
                                                                  float* __restrict__ dx, int B) {
  __shared__ __attribute__((aligned(16))) float A[1][128 * D3_AS];   // 40 KB (two workgroups per CU)
  __shared__ __attribute__((aligned(16))) float X[4][16 * D3_XS];   // 25.9 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const float* wl = wp + wave * 32 * 576 + lane;  // + (k-step * 9 + tap) * 64
  float* xw = X[wave];
  // an image's dz into the staging buffer: this thread's 8 float4 (2048 float4: co = e / 16, column 4 (e % 16)),
  // all loads issued before the first store
  auto copy_img = [&](int b, float* buf) {
    const float4* src = reinterpret_cast<const float4*>(dz + (int64_t)b * 8192) + tid;
    // named registers, not an array: the array form was left on the scratch stack
    const float4 r0 = src[0], r1 = src[256], r2 = src[512], r3 = src[768], r4 = src[1024], r5 = src[1280],
                 r6 = src[1536], r7 = src[1792];
    float* d = buf + (tid >> 4) * D3_AS + (tid & 15) * 4;  // + 16 co rows per 256 float4
    *reinterpret_cast<float4*>(d + 0 * 16 * D3_AS) = r0;
    *reinterpret_cast<float4*>(d + 1 * 16 * D3_AS) = r1;
    *reinterpret_cast<float4*>(d + 2 * 16 * D3_AS) = r2;
    *reinterpret_cast<float4*>(d + 3 * 16 * D3_AS) = r3;
    *reinterpret_cast<float4*>(d + 4 * 16 * D3_AS) = r4;
    *reinterpret_cast<float4*>(d + 5 * 16 * D3_AS) = r5;
    *reinterpret_cast<float4*>(d + 6 * 16 * D3_AS) = r6;
    *reinterpret_cast<float4*>(d + 7 * 16 * D3_AS) = r7;
  };
  int b = blockIdx.x;
  if (b < B) copy_img(b, A[0]);
  __syncthreads();
  for (; b < B; b += gridDim.x) {
    const int nb = b + gridDim.x;
    const float* a_img = A[0];
    f32x4 acc[9][4];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[t][i] = dev::zero_f32x4();
    // weights: two register sets, each reloaded right after its MFMAs were issued, for the k-step two ahead
    // (one coalesced 256-B dword load per tap, straight into the registers the MFMAs read).  The reloads are
    // unconditional (the last two read past this wave's k-steps: the next wave's, or the buffer's pad) and
    // pinned behind their k-step's MFMAs (sched_barrier), so each wait covers only the set about to be used
    // and every load has a whole k-step (36 MFMAs, ~1150 cycles) to arrive.
    float wa[9], wb[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      wa[t] = wl[t * 64];
      wb[t] = wl[(9 + t) * 64];
    }
    auto kstep = [&](int ks, const float (&wt)[9]) {
      float a[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = a_img[(ks * 4 + lk) * D3_AS + 16 * i + lr];
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i)  // rows: positions 16 i + (lane & 15); columns: channels
          acc[t][i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], wt[t], acc[t][i], 0, 0, 0);
    };
#pragma unroll 1
    for (int ks = 0; ks < 32; ks += 2) {
      kstep(ks, wa);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < 9; ++t) wa[t] = wl[((ks + 2) * 9 + t) * 64];
      __builtin_amdgcn_sched_barrier(0);
      kstep(ks + 1, wb);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < 9; ++t) wb[t] = wl[((ks + 3) * 9 + t) * 64];
      __builtin_amdgcn_sched_barrier(0);
    }
    // col2im into the wave's dx image: lane holds P_t[p = 16 i + 4 lk + r][ci = lr].  Lanes share
    // destinations across taps (the x = 4, 5 columns of lanes with lk even and odd), which the compiler's
    // per-thread alias analysis cannot see: a memory clobber between the phases keeps the wave's LDS
    // operations in program order (one wave's LDS operations then complete in order).
    for (int e = lane; e < 16 * D3_XS; e += 64) xw[e] = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      asm volatile("" ::: "memory");
      const int kh = t / 3, kw = t % 3;
      float v[16];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int p = 16 * i + 4 * lk + r;
          v[4 * i + r] = xw[lr * D3_XS + ((p >> 3) + kh) * 10 + (p & 7) + kw];
        }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int p = 16 * i + 4 * lk + r;
          xw[lr * D3_XS + ((p >> 3) + kh) * 10 + (p & 7) + kw] = v[4 * i + r] + acc[t][i][r];
        }
    }
    asm volatile("" ::: "memory");
    // the wave's 16 channels x 100 positions: one contiguous run of dx
    float* out = dx + (int64_t)b * 6400 + wave * 1600;
    for (int e = lane; e < 1600; e += 64) {
      const int c = e / 100;
      out[e] = xw[c * D3_XS + (e - 100 * c)];
    }
    asm volatile("" ::: "memory");
    __syncthreads();  // every wave's k loop has read this image
    // the next image's dz straight through registers into the single buffer: the round trip is exposed to
    // this workgroup only; the CU's other workgroup keeps the matrix cores busy meanwhile
    if (nb < B) copy_img(nb, A[0]);
    __syncthreads();
  }
}

// conv2 (32 -> 64 channels, 3x3 valid, 13x13 -> 11x11): its data gradient in the same scatter form.  dz2 has
// 121 positions (8 tiles of 16, the last 7 rows padding: never scattered); wave w owns input channels
// [16 (w & 1), +16) for positions [64 (w >> 1), +64), so the two waves of a channel tile write overlapping
// output rows: each scatters into its own LDS image and the pair is summed in a fixed order on the way out.
constexpr int D2_XS = 171;                  // floats per channel row of a wave's 13x13 image (odd)
constexpr int D2_WP = 2 * 16 * 9 * 64;      // repacked weights: [ci tile][k-step][tap][lane]

__global__ __launch_bounds__(256) void d2_repack_kernel(const float* __restrict__ w, float* __restrict__ wp) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= D2_WP) return;
  const int lane = i & 63, t = (i >> 6) % 9, ks = (i / 576) & 15, ct = i / 9216;
  const int co = ks * 4 + (lane >> 4), ci = ct * 16 + (lane & 15);
  wp[i] = w[(co * 32 + ci) * 9 + t];
}

__global__ __launch_bounds__(256, 2) void conv2_dgrad_f32_kernel(const float* __restrict__ dz,
                                                                  const float* __restrict__ wp,
                                                                  float* __restrict__ dx, int B) {
  __shared__ __attribute__((aligned(16))) float A[1][64 * 121 + 128];  // 31 KB (+ readable padding rows)
  __shared__ __attribute__((aligned(16))) float X[4][16 * D2_XS + 32];  // 44.3 KB (+ a dump row per wave)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4, ct = wave & 1, half = wave >> 1;
  const float* wl = wp + ct * 16 * 576 + lane;  // + (k-step * 9 + tap) * 64
  float* xw = X[wave];
  // per (tile i, row r) of this lane: the image offset (channel row included) of its dz position
  // p = 64 half + 16 i + 4 lk + r; past the 121 real positions the wave's dump row (branch-free col2im)
  int dst[16];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int p = 64 * half + 16 * i + 4 * lk + r;
      dst[4 * i + r] = p < 121 ? lr * D2_XS + (p / 11) * 13 + p % 11 : 16 * D2_XS;
    }
  // an image of dz is 7744 contiguous floats = 1936 float4: threads take 7 or 8 of them (the loads are
  // unconditional, clamped to the image, so they all issue before the first store)
  auto copy_img = [&](int b, float* buf) {
    const float4* src = reinterpret_cast<const float4*>(dz + (int64_t)b * 7744) + tid;
    float4* d = reinterpret_cast<float4*>(buf) + tid;
    // named registers (an array was left on the scratch stack); the last one exists for tid < 144
    const float4 r0 = src[0], r1 = src[256], r2 = src[512], r3 = src[768], r4 = src[1024], r5 = src[1280],
                 r6 = src[1536], r7 = src[tid < 144 ? 1792 : 0];
    d[0] = r0;
    d[256] = r1;
    d[512] = r2;
    d[768] = r3;
    d[1024] = r4;
    d[1280] = r5;
    d[1536] = r6;
    if (tid < 144) d[1792] = r7;
  };
  int b = blockIdx.x;
  if (b < B) copy_img(b, A[0]);
  __syncthreads();
  for (; b < B; b += gridDim.x) {
    const int nb = b + gridDim.x;
    const float* a_img = A[0] + 64 * half;
    f32x4 acc[9][4];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[t][i] = dev::zero_f32x4();
    float wa[9], wb[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      wa[t] = wl[t * 64];
      wb[t] = wl[(9 + t) * 64];
    }
    // rows of dz: co = 4 ks + lk at 121 floats; positions 16 i + lr of this half (rows 121.. of the last
    // tile read padding / the next channel: their products are never scattered)
    auto kstep = [&](int ks, const float (&wt)[9]) {
      float a[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = a_img[(ks * 4 + lk) * 121 + 16 * i + lr];
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[t][i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], wt[t], acc[t][i], 0, 0, 0);
    };
#pragma unroll 1
    for (int ks = 0; ks < 16; ks += 2) {  // as conv3_dgrad_f32_kernel: pinned, unconditional weight reloads
      kstep(ks, wa);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < 9; ++t) wa[t] = wl[((ks + 2) * 9 + t) * 64];
      __builtin_amdgcn_sched_barrier(0);
      kstep(ks + 1, wb);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < 9; ++t) wb[t] = wl[((ks + 3) * 9 + t) * 64];
      __builtin_amdgcn_sched_barrier(0);
    }
    // col2im into this wave's image (cross-lane shared destinations: keep program order, see conv3)
    for (int e = lane; e < 16 * D2_XS; e += 64) xw[e] = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      asm volatile("" ::: "memory");
      const int off = (t / 3) * 13 + t % 3;
      float v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = xw[dst[q] + off];
#pragma unroll
      for (int q = 0; q < 16; ++q) xw[dst[q] + off] = v[q] + acc[t][q >> 2][q & 3];
    }
    __syncthreads();  // both halves of every channel tile scattered
    {
      // channel tile ct, elements [1352 half, +1352) of its 16 x 169 run: half 0's image + half 1's, in order
      const float* x0 = X[ct];
      const float* x1 = X[ct + 2];
      float* out = dx + (int64_t)b * 5408 + ct * 2704;
      for (int e = 1352 * half + lane; e < 1352 * (half + 1); e += 64) {
        const int c = e / 169, q = e - 169 * c;
        out[e] = x0[c * D2_XS + q] + x1[c * D2_XS + q];
      }
    }
    if (nb < B) copy_img(nb, A[0]);  // every k loop finished before the barrier above (see conv3)
    __syncthreads();  // images read out, next dz staged
  }
}

// ---------------------------------------------------------------- conv3 weight gradient
// dW3[co][ci][t] = sum over images b and the 8x8 positions p of dz3[b][co][p] * a2[b][ci][p + t] (+ the bias
// gradient db3[co] = sum dz3): a dedicated kernel instead of the implicit GEMM's per-element gathers.  Workgroup
// (ct, slice) owns input channels [16 ct, +16) and images [B slice / S, B (slice + 1) / S); wave w owns output
// channels [32 w, +32) x 16 channels x 9 taps (18 MFMA tiles).  Per image both operands come from LDS with
// compile-time offsets: dz3 in its natural [co][p] order with a row stride of 2 mod 32 banks (the A fragment,
// 16 co x 4 positions, is a conflict-free b32 read; the transposed layout it replaces made every staging
// store a 16-way bank conflict) and the 16-channel a2 tile (the tap shift is an immediate).  The bias sums
// ride in the staging (ct = 0 workgroups, VALU).  The next image's operands are loaded into registers during
// the k loop.  Each workgroup writes its slice's partial dW into slab[slice][co][ci 9 + t] (+ the bias
// column), reduced by the same fixed-order f32_slab_reduce as the GEMM path: deterministic.
constexpr int W3_DS = 66;   // floats per co row of the dz3 tile (64 positions + 2; 66 = 2 mod 32)
constexpr int W3_AS = 101;  // floats per channel row of the a2 tile (odd)

__global__ __launch_bounds__(256, 2) void conv3_wgrad_f32_kernel(const float* __restrict__ dz,
                                                                  const float* __restrict__ a2,
                                                                  float* __restrict__ slab, int B) {
  // single-buffered (40.3 KB): two workgroups per CU, so one stages while the other multiplies
  __shared__ __attribute__((aligned(16))) float DZ[128 * W3_DS];  // 33.8 KB
  __shared__ __attribute__((aligned(16))) float AX[16 * W3_AS];   // 6.5 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const int ct = blockIdx.x & 3, slice = blockIdx.x >> 2;
  const int b0 = static_cast<int>((int64_t)B * slice / W3_SLICES), b1 = static_cast<int>((int64_t)B * (slice + 1) / W3_SLICES);
  const bool bias = ct == 0;
  // staging: dz3 = 2048 float4 (co = e >> 4, positions 4 (e & 15) ..), 8 per thread; the a2 tile = 400 float4
  // (channel 4 e / 100, never crossing a row), 1-2 per thread
  float4 rz[8], ra[2];
  auto load = [&](int b) {
    const float4* z4 = reinterpret_cast<const float4*>(dz + (int64_t)b * 8192);
#pragma unroll
    for (int u = 0; u < 8; ++u) rz[u] = z4[tid + 256 * u];
    const float4* a4 = reinterpret_cast<const float4*>(a2 + (int64_t)b * 6400 + ct * 1600);
    ra[0] = a4[tid];
    ra[1] = a4[tid < 144 ? 256 + tid : tid];
  };
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // bias partials of co (tid >> 4) + 16 u
  auto stash = [&]() {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + 256 * u, co = e >> 4, p = (e & 15) * 4;
      float2* d = reinterpret_cast<float2*>(DZ + co * W3_DS + p);  // 8-B aligned (W3_DS even)
      d[0] = make_float2(rz[u].x, rz[u].y);
      d[1] = make_float2(rz[u].z, rz[u].w);
      if (bias) bsum[u] += (rz[u].x + rz[u].y) + (rz[u].z + rz[u].w);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = tid + 256 * u;
      if (u == 0 || tid < 144) {
        const int c = (4 * e) / 100, q = 4 * e - 100 * c;
        AX[c * W3_AS + q + 0] = ra[u].x;
        AX[c * W3_AS + q + 1] = ra[u].y;
        AX[c * W3_AS + q + 2] = ra[u].z;
        AX[c * W3_AS + q + 3] = ra[u].w;
      }
    }
  };
  f32x4 acc[2][9];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[j][t] = dev::zero_f32x4();
  const int abase = (32 * wave + lr) * W3_DS + lk;  // A: output channel 32 w + 16 j + lr, position 4 ks + lk
  const int xbase = lr * W3_AS + lk;                // B: channel lr, position (ks >> 1, 4 (ks & 1) + lk) + tap
  if (b0 < b1) load(b0);
  for (int b = b0; b < b1; ++b) {
    stash();
    __syncthreads();
    if (b + 1 < b1) load(b + 1);  // in flight during the k loop
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      float a[2], w[9];
#pragma unroll
      for (int j = 0; j < 2; ++j) a[j] = DZ[abase + 4 * ks + 16 * j * W3_DS];
#pragma unroll
      for (int t = 0; t < 9; ++t) w[t] = AX[xbase + ((ks >> 1) + t / 3) * 10 + 4 * (ks & 1) + t % 3];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], w[t], acc[j][t], 0, 0, 0);
    }
    __syncthreads();  // the tile is read out before the next image's stash
  }
  // partial dW of this slice: lane holds D[co = 32 w + 16 j + 4 lk + r][ci = 16 ct + lr] per tap
  constexpr int NCOL = 64 * 9 + 1;
  float* out = slab + (int64_t)slice * 128 * NCOL;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = 32 * wave + 16 * j + 4 * lk + r;
#pragma unroll
      for (int t = 0; t < 9; ++t) out[co * NCOL + (16 * ct + lr) * 9 + t] = acc[j][t][r];
    }
  if (bias) {  // the 16 threads sharing co (tid >> 4) + 16 u hold the 4-position partials of all 64 positions
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      float v = bsum[u];
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 16);
      if ((tid & 15) == 0) out[((tid >> 4) + 16 * u) * NCOL + 576] = v;
    }
  }
}

// conv2's weight gradient (64 <- 32 channels, 13x13 -> 11x11) the same way: workgroup (ct of 2, slice) owns
// input channels [16 ct, +16), wave w output channels [16 w, +16) x 16 x 9 taps.  The 121 positions are 31
// k-steps of 4 (positions 121..123 of the dz2 tile are zero); a position's 13x13 offset is a per-lane table
// (the 11-wide rows do not split on k-step boundaries).  dz2 stays in its natural [co][p] order with a row
// stride of 2 mod 32 banks, so the A fragment (16 co x 4 positions) is a conflict-free read and the staging
// writes run along rows.  256 slices (512 workgroups, 2 per CU) and the next image's loads in flight during
// the k loop: with 256 workgroups and no prefetch the staging was exposed (4.49 ms vs the GEMM's 4.19).
constexpr int W2_S = 130;   // floats per output-channel row of the dz2 tile (121 + 9; 130 = 2 mod 32)
constexpr int W2_AS = 171;  // floats per channel row of the a1 tile (odd)

__global__ __launch_bounds__(256, 2) void conv2_wgrad_f32_kernel(const float* __restrict__ dz,
                                                                  const float* __restrict__ a1,
                                                                  float* __restrict__ slab, int B) {
  __shared__ __attribute__((aligned(16))) float DZ[64 * W2_S];   // 33.3 KB
  __shared__ __attribute__((aligned(16))) float AX[16 * W2_AS];  // 10.9 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const int ct = blockIdx.x & 1, slice = blockIdx.x >> 1;
  const int b0 = static_cast<int>((int64_t)B * slice / W2_SLICES), b1 = static_cast<int>((int64_t)B * (slice + 1) / W2_SLICES);
  const bool bias = ct == 0;
  // padding positions 121..123 of every row: zero once (never written by the staging)
  for (int e = tid; e < 64 * 3; e += 256) DZ[(e / 3) * W2_S + 121 + e % 3] = 0.f;
  int xoff[31];  // per k-step: the 13x13 offset of this lane's position 4 ks + lk (clamped past 120)
#pragma unroll
  for (int ks = 0; ks < 31; ++ks) {
    const int p = min(4 * ks + lk, 120);
    xoff[ks] = (p / 11) * 13 + p % 11;
  }
  f32x4 acc[9], accb = dev::zero_f32x4();  // accb: the bias sums (ct = 0), one MFMA against ones per k-step
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = dev::zero_f32x4();
  // staging registers: dz2 image = 7744 floats = 1936 float4 (8 per thread), a1 tile 16 x 169 = 676 float4 (3)
  float4 rz[8], ra[3];
  auto load = [&](int b) {
    const float4* z4 = reinterpret_cast<const float4*>(dz + (int64_t)b * 7744);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (tid + 256 * u < 1936) rz[u] = z4[tid + 256 * u];
    const float4* a4 = reinterpret_cast<const float4*>(a1 + (int64_t)b * 5408 + ct * 2704);
#pragma unroll
    for (int u = 0; u < 3; ++u)
      if (tid + 256 * u < 676) ra[u] = a4[tid + 256 * u];
  };
  auto stash = [&]() {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + 256 * u;
      if (e < 1936) {
        const float vv[4] = {rz[u].x, rz[u].y, rz[u].z, rz[u].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int f = 4 * e + j, co = f / 121, p = f - 121 * co;
          DZ[co * W2_S + p] = vv[j];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int e = tid + 256 * u;
      if (e < 676) {
        const float vv[4] = {ra[u].x, ra[u].y, ra[u].z, ra[u].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int f = 4 * e + j, c = f / 169, q = f - 169 * c;
          AX[c * W2_AS + q] = vv[j];
        }
      }
    }
  };
  const int abase = (16 * wave + lr) * W2_S + lk;  // A: output channel 16 w + lr, position 4 ks + lk
  const int xbase = lr * W2_AS;                    // B: channel lr, position offset xoff[ks] + tap
  if (b0 < b1) load(b0);
  for (int b = b0; b < b1; ++b) {
    stash();
    __syncthreads();
    if (b + 1 < b1) load(b + 1);  // in flight during the k loop
    // one straight k-loop per workgroup kind (a uniform branch outside it, not one per k-step)
    auto kloop = [&](auto with_bias) {
#pragma unroll
      for (int ks = 0; ks < 31; ++ks) {
        const float a = DZ[abase + 4 * ks];
        float w[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) w[t] = AX[xbase + xoff[ks] + (t / 3) * 13 + t % 3];
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w[t], acc[t], 0, 0, 0);
        if constexpr (decltype(with_bias)::value) accb = __builtin_amdgcn_mfma_f32_16x16x4f32(a, 1.f, accb, 0, 0, 0);
      }
    };
    if (bias)
      kloop(std::true_type{});
    else
      kloop(std::false_type{});
    __syncthreads();
  }
  constexpr int NCOL = 32 * 9 + 1;
  float* out = slab + (int64_t)slice * 64 * NCOL;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int co = 16 * wave + 4 * lk + r;
#pragma unroll
    for (int t = 0; t < 9; ++t) out[co * NCOL + (16 * ct + lr) * 9 + t] = acc[t][r];
  }
  if (bias && lr == 0) {  // every column of accb holds the row sums
#pragma unroll
    for (int r = 0; r < 4; ++r) out[(16 * wave + 4 * lk + r) * NCOL + 288] = accb[r];
  }
}

static bool wgrad_dedicated_on() {
  static const bool on = [] {
    const char* v = std::getenv("RINGDP_F32_WGRAD_DEDICATED");
    return !(v && v[0] == '0');
  }();
  return on;
}

bool conv3_wgrad_f32_ok(const ConvF32Geom& g) {
  return wgrad_dedicated_on() && g.Kout == 128 && g.C == 64 && g.R == 3 && g.pad == 0 && g.H == 10 &&
         g.W == 10 && g.B >= 8 * W3_SLICES && g.B * 8192 < (int64_t{1} << 31);
}

bool conv2_wgrad_f32_ok(const ConvF32Geom& g) {
  return wgrad_dedicated_on() && g.Kout == 64 && g.C == 32 && g.R == 3 && g.pad == 0 && g.H == 13 &&
         g.W == 13 && g.B >= 4 * W2_SLICES && g.B * 7744 < (int64_t{1} << 31);
}

static bool is_conv3_dgrad(const ConvF32Geom& g) {
  return g.Kout == 128 && g.C == 64 && g.R == 3 && g.pad == 0 && g.H == 10 && g.W == 10;
}
static bool is_conv2_dgrad(const ConvF32Geom& g) {
  return g.Kout == 64 && g.C == 32 && g.R == 3 && g.pad == 0 && g.H == 13 && g.W == 13;
}

bool conv_dgrad_f32_scatter_ok(const ConvF32Geom& g) {
  static const bool on = [] {
    const char* v = std::getenv("RINGDP_F32_DGRAD_SCATTER");
    return !(v && v[0] == '0');
  }();
  // the persistent one-image-per-workgroup form needs images for every CU; small batches keep split K
  return on && (is_conv3_dgrad(g) || is_conv2_dgrad(g)) && g.B >= 2 * f32_num_cus() &&
         g.B * 8192 < (int64_t{1} << 31);
}

void conv_dgrad_f32_scatter(const ConvF32Geom& g, const float* dz, const float* w, float* dx, float* wp,
                            hipStream_t s) {
  // two persistent workgroups per CU (single-buffered dz): one's col2im runs beside the other's MFMAs
  const int grid = static_cast<int>(std::min<int64_t>(g.B, 2 * f32_num_cus()));
  if (is_conv3_dgrad(g)) {
    hipLaunchKernelGGL(d3_repack_kernel, dim3((D3_WP + 255) / 256), dim3(256), 0, s, w, wp);
    hipLaunchKernelGGL(conv3_dgrad_f32_kernel, dim3(grid), dim3(256), 0, s, dz, wp, dx, static_cast<int>(g.B));
  } else {
    hipLaunchKernelGGL(d2_repack_kernel, dim3((D2_WP + 255) / 256), dim3(256), 0, s, w, wp);
    hipLaunchKernelGGL(conv2_dgrad_f32_kernel, dim3(grid), dim3(256), 0, s, dz, wp, dx, static_cast<int>(g.B));
  }
}

int conv_dgrad_f32_scratch() { return D3_WP + 2 * 576; }  // the larger repack + the prefetch pad

void conv_f32_dgrad(const ConvF32Geom& g, const float* dz, const float* w, float* dx, float* slab, int slices,
                    hipStream_t s) {
  const int K = g.Kout * g.R * g.R;
  const int64_t zin = static_cast<int64_t>(g.Kout) * g.OH * g.OW, xout = static_cast<int64_t>(g.C) * g.H * g.W;
  if (slab && slices > 1) {  // conv_f32_dgrad_slices(g) > 1: one chunk, plane % 4 == 0
    const int M = static_cast<int>(g.B * g.H * g.W);
    const int plane = M * g.C;
    int per = (K + slices - 1) / slices;
    per = (per + BK - 1) / BK * BK;
    const int used = (K + per - 1) / per;
    DgradA la{{dz, static_cast<int>(g.B * zin * 4), 0.f, 1.f}, g.Kout, g.W, g.R, g.OH, g.OW, g.pad, K, M,
              make_fdiv(g.H * g.W), make_fdiv(g.W)};
    DgradB lb{{w, K * g.C * 4, 0.f, 1.f}, g.C, g.R * g.R, K, make_fdiv(g.R * g.R)};
    NCHWSlabOut epi{slab, g.C, M, plane, make_fdiv(g.H * g.W)};
    launch_gemm(M, g.C, K, per, used, -1, la, lb, epi, s);
    hipLaunchKernelGGL(slab_sum_kernel, dim3(grid_1d(plane / 4)), dim3(256), 0, s, reinterpret_cast<const float4*>(slab),
                       used, plane / 4, reinterpret_cast<float4*>(dx));
    return;
  }
  const int64_t chunk = batch_chunk(g.B, {zin, xout});
  for (int64_t b0 = 0; b0 < g.B; b0 += chunk) {
    const int nb = static_cast<int>(std::min(chunk, g.B - b0));
    const int M = nb * g.H * g.W;
    DgradA la{{dz + b0 * zin, static_cast<int>(nb * zin * 4), 0.f, 1.f}, g.Kout, g.W, g.R, g.OH, g.OW, g.pad, K,
              M, make_fdiv(g.H * g.W), make_fdiv(g.W)};
    DgradB lb{{w, K * g.C * 4, 0.f, 1.f}, g.C, g.R * g.R, K, make_fdiv(g.R * g.R)};
    NCHWOut epi{dx + b0 * xout, nullptr, g.C, M, make_fdiv(g.H * g.W)};
    launch_gemm(M, g.C, K, K, 1, -1, la, lb, epi, s);
  }
}

void conv_f32_wgrad(const ConvF32Geom& g, const float* dz, const float* x, const unsigned char* xu8, float mean,
                    float inv_std, float* slab, int slices, float* dw, float* db, hipStream_t s, F32RedList* defer) {
  auto reduce = [&](int n, int Kout, int Nw, int ncol) {
    if (defer)
      defer->push_back(F32RedSeg{slab, n, Kout, Nw, ncol, dw, db});
    else
      f32_slab_reduce(slab, n, Kout, Nw, ncol, dw, db, s);
  };
  const int Nw = g.C * g.R * g.R;
  const int ncol = Nw + (db ? 1 : 0);
  if (!xu8 && db && conv3_wgrad_f32_ok(g)) {  // the ConvNet's conv3 / conv2 at large batches: dedicated kernels
    hipLaunchKernelGGL(conv3_wgrad_f32_kernel, dim3(4 * W3_SLICES), dim3(256), 0, s, dz, x, slab,
                       static_cast<int>(g.B));
    reduce(W3_SLICES, g.Kout, Nw, ncol);
    return;
  }
  if (!xu8 && db && conv2_wgrad_f32_ok(g)) {
    hipLaunchKernelGGL(conv2_wgrad_f32_kernel, dim3(2 * W2_SLICES), dim3(256), 0, s, dz, x, slab,
                       static_cast<int>(g.B));
    reduce(W2_SLICES, g.Kout, Nw, ncol);
    return;
  }
  const int64_t xin = static_cast<int64_t>(g.C) * g.H * g.W, zin = static_cast<int64_t>(g.Kout) * g.OH * g.OW;
  const int64_t chunk = wgrad_chunk(g);
  const int ohw = g.OH * g.OW;
  int used = 0;
  for (int64_t b0 = 0; b0 < g.B; b0 += chunk) {
    const int nb = static_cast<int>(std::min(chunk, g.B - b0));
    const int K = nb * ohw;
    const int sl = wgrad_slices(g.Kout, Nw, static_cast<int64_t>(chunk) * ohw);
    int per = (K + sl - 1) / sl;
    per = (per + BK - 1) / BK * BK;
    const int used_sl = (K + per - 1) / per;
    // GEMM columns = the Nw weights; the bias column (ncol - 1) comes from the dz row sums
    WgradA la{{dz + b0 * zin, static_cast<int>(nb * zin * 4), 0.f, 1.f}, g.Kout, ohw, make_fdiv(ohw)};
    SlabOut epi{slab + static_cast<int64_t>(used) * g.Kout * ncol, ncol, g.Kout};
    const int bias_col = db ? Nw : -1;
    const int xbytes = static_cast<int>(nb * xin);
    if (xu8) {
      WgradB<true, true> lb{{xu8 + b0 * xin, xbytes, mean, inv_std}, g.C, g.H, g.W, g.R, g.pad, g.OW, Nw,
                            make_fdiv(ohw), make_fdiv(g.OW)};
      launch_gemm(g.Kout, Nw, K, per, used_sl, bias_col, la, lb, epi, s);
    } else if (g.pad) {
      WgradB<false, true> lb{{x + b0 * xin, xbytes * 4, 0.f, 1.f}, g.C, g.H, g.W, g.R, g.pad, g.OW, Nw,
                             make_fdiv(ohw), make_fdiv(g.OW)};
      launch_gemm(g.Kout, Nw, K, per, used_sl, bias_col, la, lb, epi, s);
    } else {
      WgradB<false, false> lb{{x + b0 * xin, xbytes * 4, 0.f, 1.f}, g.C, g.H, g.W, g.R, g.pad, g.OW, Nw,
                              make_fdiv(ohw), make_fdiv(g.OW)};
      launch_gemm(g.Kout, Nw, K, per, used_sl, bias_col, la, lb, epi, s);
    }
    used += used_sl;
  }
  // the slab holds conv_f32_wgrad_slices(g) = (slices of all chunks) + their group count >= used + groups
  (void)slices;
  reduce(used, g.Kout, Nw, ncol);
}

int f32_slab_capacity(int slices) { return slices + (slices + kSlabGroup - 1) / kSlabGroup; }

void f32_slab_reduce(float* slab, int slices, int Kout, int Nw, int ncol, float* dw, float* db, hipStream_t s) {
  const int total = Kout * ncol;
  const float* src = slab;
  int nsum = slices;
  if (slices > kSlabGroup) {
    float* part = slab + static_cast<int64_t>(slices) * total;
    nsum = (slices + kSlabGroup - 1) / kSlabGroup;
    hipLaunchKernelGGL(slab_group_kernel, dim3((total + 255) / 256, nsum), dim3(256), 0, s, slab, slices, total,
                       part);
    src = part;
  }
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(grid_1d(total)), dim3(256), 0, s, src, nsum, Kout, Nw, ncol, dw, db);
}

void f32_slab_reduce_multi(const F32RedList& segs, hipStream_t s) {
  if (segs.empty()) return;
  if ((int)segs.size() > kF32RedMax) {
    for (const auto& g : segs)
      f32_slab_reduce(const_cast<float*>(g.slab), g.slices, g.Kout, g.Nw, g.ncol, g.dw, g.db, s);
    return;
  }
  F32RedArgs a{};
  a.n = static_cast<int>(segs.size());
  int blocks = 0;
  for (int i = 0; i < a.n; ++i) {
    a.seg[i] = segs[i];
    a.bstart[i] = blocks;
    const int total = segs[i].Kout * segs[i].ncol;
    const int per = segs[i].slices <= kSlabGroup ? 256 : kRedElems;  // the kernel's two workgroup kinds
    blocks += (total + per - 1) / per;
  }
  for (int i = a.n; i < kF32RedMax; ++i) a.bstart[i] = blocks;
  const int grid = blocks;
  hipLaunchKernelGGL(f32_reduce_multi_kernel, dim3(grid), dim3(256), 0, s, a);
}

void pool_relu_f32_fwd(const float* z, float* a, unsigned char* code, int64_t BC, int H, int W, int k, int st,
                       hipStream_t s) {
  const int PH = (H - k) / st + 1, PW = (W - k) / st + 1;
  const int64_t chunk = batch_chunk(BC, {static_cast<int64_t>(H) * W});
  for (int64_t c0 = 0; c0 < BC; c0 += chunk) {
    const int64_t nbc = std::min(chunk, BC - c0);
    const int total = static_cast<int>(nbc * PH * PW);
    if (k == 2 && st == 2 && (W & 1) == 0) {
      hipLaunchKernelGGL(pool2s2_fwd_kernel, dim3(grid_elems(total)), dim3(256), 0, s, z + c0 * H * W,
                         a + c0 * PH * PW, code + c0 * PH * PW, total, H, W, make_fdiv(PH * PW), make_fdiv(PW));
      continue;
    }
    if (k == 2 && st == 1) {
      hipLaunchKernelGGL(pool2s1_fwd_kernel, dim3(grid_elems(total)), dim3(256), 0, s, z + c0 * H * W,
                         a + c0 * PH * PW, code + c0 * PH * PW, total, H, W, make_fdiv(PH * PW), make_fdiv(PW));
      continue;
    }
    hipLaunchKernelGGL(pool_relu_fwd_kernel, dim3(grid_elems(total)), dim3(256), 0, s, z + c0 * H * W,
                       a + c0 * PH * PW, code + c0 * PH * PW, total, H, W, make_fdiv(PH * PW), make_fdiv(PW), k, st);
  }
}

// The fp32 ConvNet head backward at small batches (the whole-network cross-entropy node): the logits gradient
// (ce_bwd_kernel's expression, same bits) -> dl for fc1's weight gradient, fc1's data gradient
// da3[f] = sum_j dl[j] W[j][f] (an fmaf chain in j order) and pool3's backward (2x2/s2, code = dy*2+dx, 255 =
// no gradient) straight into dz3 [128][8][8] - one launch for the cross-entropy backward, fc1 data gradient and
// pool3 backward launches.  Workgroup = 256 features of one image; 8 per image.
__global__ __launch_bounds__(256) void fc_ce_pool3_bwd_f32_kernel(const float* __restrict__ logits,
                                                                  const int64_t* __restrict__ labels,
                                                                  const float* __restrict__ lse,
                                                                  const float* __restrict__ grad_out,
                                                                  const float* __restrict__ denom, int ignore_index,
                                                                  float eps, int reduction,
                                                                  const float* __restrict__ wfc,
                                                                  const unsigned char* __restrict__ code3,
                                                                  float* __restrict__ dl, float* __restrict__ dz3) {
  __shared__ float g[10];
  const int n = blockIdx.x >> 3, f = (blockIdx.x & 7) * 256 + threadIdx.x;
  if (threadIdx.x < 10) {
    const int c = threadIdx.x;
    const int64_t y = labels[n];
    float v = 0.f;
    if (y != ignore_index) {
      const float p = __expf(logits[n * 10 + c] - lse[n]);
      const float q = (c == y ? (1.f - eps) : 0.f) + eps / 10.f;
      v = (p - q) * (reduction == 0 ? grad_out[n] : grad_out[0] / denom[0]);
    }
    g[c] = v;
    if ((blockIdx.x & 7) == 0) dl[n * 10 + c] = v;
  }
  __syncthreads();
  float a = 0.f;
#pragma unroll
  for (int j = 0; j < 10; ++j) a = fmaf(g[j], wfc[j * 2048 + f], a);
  const int code = code3[n * 2048 + f];
  const int c = f >> 4, py = (f >> 2) & 3, px = f & 3;
  float* o = dz3 + (int64_t)n * 8192 + c * 64 + 2 * py * 8 + 2 * px;
  *reinterpret_cast<float2*>(o) = make_float2(code == 0 ? a : 0.f, code == 1 ? a : 0.f);
  *reinterpret_cast<float2*>(o + 8) = make_float2(code == 2 ? a : 0.f, code == 3 ? a : 0.f);
}

void fc_ce_pool3_bwd_f32(const float* logits, const int64_t* labels, const float* lse, const float* grad_out,
                         const float* denom, int ignore_index, float eps, int reduction, const float* wfc,
                         const unsigned char* code3, int B, float* dl, float* dz3, hipStream_t s) {
  if (B <= 0) return;
  hipLaunchKernelGGL(fc_ce_pool3_bwd_f32_kernel, dim3(8 * B), dim3(256), 0, s, logits, labels, lse, grad_out, denom,
                     ignore_index, eps, reduction, wfc, code3, dl, dz3);
}

bool conv_f32_dgrad_pool2s1_ok(const ConvF32Geom& g) {
  const int64_t BC = g.B * g.C;
  return conv_f32_dgrad_slices(g) > 1 && !conv_dgrad_f32_scatter_ok(g) && g.H == 10 && g.W == 10 && BC % kP2Tile == 0;
}

void conv_f32_dgrad_pool2s1_bwd(const ConvF32Geom& g, const float* dz, const float* w, float* slab, int slices,
                                const unsigned char* code, float* dzp, hipStream_t s) {
  // conv_f32_dgrad's split-K GEMM into slab (its planes are the pool's da), then the tiled 2x2/s1 pool backward
  // summing the planes as it stages them: one launch fewer than dgrad + slab_sum + pool backward
  const int K = g.Kout * g.R * g.R;
  const int64_t zin = static_cast<int64_t>(g.Kout) * g.OH * g.OW;
  const int M = static_cast<int>(g.B * g.H * g.W);
  const int plane = M * g.C;
  int per = (K + slices - 1) / slices;
  per = (per + BK - 1) / BK * BK;
  const int used = (K + per - 1) / per;
  DgradA la{{dz, static_cast<int>(g.B * zin * 4), 0.f, 1.f}, g.Kout, g.W, g.R, g.OH, g.OW, g.pad, K, M,
            make_fdiv(g.H * g.W), make_fdiv(g.W)};
  DgradB lb{{w, K * g.C * 4, 0.f, 1.f}, g.C, g.R * g.R, K, make_fdiv(g.R * g.R)};
  NCHWSlabOut epi{slab, g.C, M, plane, make_fdiv(g.H * g.W)};
  launch_gemm(M, g.C, K, per, used, -1, la, lb, epi, s);
  const int ntiles = static_cast<int>(g.B * g.C / kP2Tile);
  const dim3 grid(std::min(ntiles, 8 * f32_num_cus()));
  hipLaunchKernelGGL((pool2s1_bwd_tile_kernel<10, 10>), grid, dim3(256), 0, s, slab, code, dzp, ntiles, 10, 10, used,
                     static_cast<int64_t>(plane));
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
      hipLaunchKernelGGL(pool2s2_bwd_kernel, dim3(grid_elems(wins)), dim3(256), 0, s, da + c0 * PH * PW,
                         code + c0 * PH * PW, dz + c0 * H * W, wins, make_fdiv(PH * PW), make_fdiv(PW), H, W);
      continue;
    }
    if (k == 2 && st == 1 && PH * PW <= 128 && (PH * PW) % 4 == 0 && nbc % kP2Tile == 0 &&
        !(std::getenv("RINGDP_F32_P2BWD_TILE") && std::getenv("RINGDP_F32_P2BWD_TILE")[0] == '0')) {
      const int ntiles = static_cast<int>(nbc / kP2Tile);
      const dim3 grid(std::min(ntiles, 8 * f32_num_cus()));
      if (PH == 10 && PW == 10)
        hipLaunchKernelGGL((pool2s1_bwd_tile_kernel<10, 10>), grid, dim3(256), 0, s, da + c0 * PH * PW,
                           code + c0 * PH * PW, dz + c0 * H * W, ntiles, PH, PW, 1, int64_t{0});
      else
        hipLaunchKernelGGL((pool2s1_bwd_tile_kernel<0, 0>), grid, dim3(256), 0, s, da + c0 * PH * PW,
                           code + c0 * PH * PW, dz + c0 * H * W, ntiles, PH, PW, 1, int64_t{0});
      continue;
    }
    if (k == 2 && st == 1) {
      hipLaunchKernelGGL(pool2s1_bwd_kernel, dim3(grid_elems(total)), dim3(256), 0, s, da + c0 * PH * PW,
                         code + c0 * PH * PW, dz + c0 * H * W, total, make_fdiv(H * W), make_fdiv(W), PH, PW);
      continue;
    }
    hipLaunchKernelGGL(pool_relu_bwd_kernel, dim3(grid_elems(total)), dim3(256), 0, s, da + c0 * PH * PW,
                       code + c0 * PH * PW, dz + c0 * H * W, total, make_fdiv(H * W), make_fdiv(W), PH, PW, k, st);
  }
}

}  // namespace kern
}  // namespace ringdp
