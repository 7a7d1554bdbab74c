// MNIST ConvNet hot path for CDNA4 (gfx950): hand-written HIP, bf16 MFMA + LDS tiling.
//
// Model (ref/launch_dist.py:9-41):
//   conv1 1->32 k5 p1 (28->26) -> ReLU -> MaxPool(2,2) (13)
//   conv2 32->64 k3 (13->11)  -> ReLU -> MaxPool(2,1) (10)   [overlapping windows]
//   conv3 64->128 k3 (10->8)  -> ReLU -> MaxPool(2,2) (4)  -> view(-1, 2048) -> fc1 2048->10
//
// Kernel blocks (one autograd Function each, see ringdp/ops/convnet.py):
//   F1  conv1 + ReLU + pool1                       -> a1 [B,13,13,32] bf16 + argmax|relu byte
//   F2  conv2 + ReLU + pool2 (2x2/s1)              -> a2 [B,10,10,64] bf16 + pool2 code byte
//   F3  conv3 + ReLU + pool3, then fc1 (MFMA GEMM)  -> logits [B,10] fp32 (+ a3, argmax)
// conv2's pre-activation z2 is never materialised: F2 keeps only what F3 and the backward need
// (a2 = relu(pool2(z2)) and, per pooled value, the first-max position or "no gradient"), and F3's
// backward scatters d(a2) through those codes into dz2, a plain linear-layer gradient for conv2.
//
// MI355X-first design:
//   * weight-stationary: weights are packed once per forward (cn_pack_weights) into bf16 MFMA
//     B-fragment order; every workgroup keeps its fragments in VGPRs for all the images it
//     processes; images stream through LDS with one-image-ahead register prefetch;
//   * window-ordered M: the GEMM rows of a conv followed by a 2x2/s2 pool are ordered
//     (pool window, position-in-window), so each lane's 4 accumulator registers of a
//     v_mfma_f32_16x16x32_bf16 tile are exactly one pool window -> bias + max + argmax + ReLU are
//     done in registers (conv1, conv3), no LDS round trip;
//   * fc1 runs as a small MFMA GEMM over a3 (cheaper than reducing 10 logits across a workgroup);
//   * backward: dgrad is a weight-stationary full correlation over a zero-ringed LDS image; wgrad is
//     a TN GEMM whose operands are read with ds_read_b64_tr_b16 (the transposed read also does the
//     im2col gather), split over images into fp32 slabs reduced in a fixed order (deterministic);
//   * one multi-segment reduction launch per layer backward.
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include <cstdio>
#include <cstdlib>

#include "device_common.h"
#include "kernels.h"
#include "sgd_device.h"

namespace ringdp {
namespace kern {

using namespace ringdp::dev;

namespace {

__host__ __device__ constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }

// ------------------------------------------------------------------ packed weight layout
// bf16 element offsets inside the packed buffer.  Fragment order: [n-tile][k-step][lane][8].
constexpr int P1_OFF = 0, P1_N = 2 * 2 * 512;                   // conv1 fwd   (K = kh*8 + kw, 2 k-steps)
constexpr int P2F_OFF = P1_OFF + P1_N, P2F_N = 4 * 9 * 512;     // conv2 fwd   (N 64, K 288)
constexpr int P3F_OFF = P2F_OFF + P2F_N, P3F_N = 8 * 18 * 512;  // conv3 fwd   (N 128, K 576)
constexpr int P2D_OFF = P3F_OFF + P3F_N, P2D_N = 2 * 18 * 512;  // conv2 dgrad (N 32, K 576)
constexpr int P3D_OFF = P2D_OFF + P2D_N, P3D_N = 4 * 36 * 512;  // conv3 dgrad (N 64, K 1152)
constexpr int PFC_OFF = P3D_OFF + P3D_N, PFC_N = 16 * 128 * 10; // fc1 [window][co][n] (backward)
constexpr int PFF_OFF = PFC_OFF + PFC_N, PFF_N = 64 * 64 * 8;    // fc1 fwd B fragments, k = w*128 + co
constexpr int PACK_TOTAL = PFF_OFF + PFF_N;

struct PackSrc {
  const float* w1;
  const float* w2;
  const float* w3;
  const float* wfc;
};

// fp32 master weight of packed element e
__device__ __forceinline__ float pack_value(int e, const PackSrc& ws) {
  const float* __restrict__ w1 = ws.w1;
  const float* __restrict__ w2 = ws.w2;
  const float* __restrict__ w3 = ws.w3;
  const float* __restrict__ wfc = ws.wfc;
  float v = 0.f;
  if (e < P2F_OFF) {  // [nt][ks][lane][8]: k = ks*32 + 8*(lane>>4) + j -> kh = ks*4 + (lane>>4), kw = j
    // n-tile nt, column c = channel 2c + nt: a lane's two accumulator tiles are a channel pair
    const int j = e & 7, lane = (e >> 3) & 63, ks = (e >> 9) & 1, nt = e >> 10;
    const int co = 2 * (lane & 15) + nt, kh = ks * 4 + (lane >> 4), kw = j;
    v = (kh < 5 && kw < 5) ? w1[co * 25 + kh * 5 + kw] : 0.f;
  } else if (e < P2D_OFF) {  // forward fragments of conv2 / conv3: B[k = tap*CIN + ci][n = co]
    const bool l2 = e < P3F_OFF;
    const int r = e - (l2 ? P2F_OFF : P3F_OFF);
    const int CIN = l2 ? 32 : 64, KS = l2 ? 9 : 18;
    const float* w = l2 ? w2 : w3;
    const int j = r & 7, lane = (r >> 3) & 63, ks = (r >> 9) % KS, nt = (r >> 9) / KS;
    const int co = nt * 16 + (lane & 15), k = ks * 32 + 8 * (lane >> 4) + j;
    v = w[(co * CIN + k % CIN) * 9 + k / CIN];
  } else if (e >= P3D_OFF && e < PFC_OFF) {
    // conv3 dgrad, scatter form: A[row = ci][k = co] of tap t = W3[co][ci][t]; [ci tile][tap][kstep][lane][8]
    const int r = e - P3D_OFF;
    const int j = r & 7, lane = (r >> 3) & 63, ks = (r >> 9) % 36, nt = (r >> 9) / 36;
    const int ci = nt * 16 + (lane & 15), tap = ks >> 2, co = (ks & 3) * 32 + 8 * (lane >> 4) + j;
    v = w3[(co * 64 + ci) * 9 + tap];
  } else if (e < PFC_OFF) {  // dgrad fragments: B[k = tap'*COUT + co][n = ci] = W[co][ci][8 - tap']
    const bool l2 = e < P3D_OFF;
    const int r = e - (l2 ? P2D_OFF : P3D_OFF);
    const int CIN = l2 ? 32 : 64, COUT = l2 ? 64 : 128, KS = l2 ? 18 : 36;
    const float* w = l2 ? w2 : w3;
    const int j = r & 7, lane = (r >> 3) & 63, ks = (r >> 9) % KS, nt = (r >> 9) / KS;
    const int ci = nt * 16 + (lane & 15), k = ks * 32 + 8 * (lane >> 4) + j;
    v = w[((k % COUT) * CIN + ci) * 9 + (8 - k / COUT)];
  } else if (e < PFF_OFF) {
    const int r = e - PFC_OFF;
    const int n = r % 10, co = (r / 10) % 128, wd = r / 1280;
    v = wfc[n * 2048 + co * 16 + wd];
  } else {  // [ks][lane][8]: B[k = ks*32 + 8*(lane>>4) + j][n = lane & 15], k = window*128 + co
    const int r = e - PFF_OFF;
    const int j = r & 7, lane = (r >> 3) & 63, ks = r >> 9;
    const int n = lane & 15, k = ks * 32 + 8 * (lane >> 4) + j;
    v = n < 10 ? wfc[n * 2048 + (k & 127) * 16 + (k >> 7)] : 0.f;
  }
  return v;
}

// packs elements [first, PACK_TOTAL) with `nblocks` workgroups (this one is `blk`), 4 per thread
__device__ __forceinline__ void pack_range(const PackSrc& ws, bf16* __restrict__ out, int first, int blk, int nblocks) {
  for (int e0 = first + 4 * (blk * 256 + (int)threadIdx.x); e0 < PACK_TOTAL; e0 += 4 * 256 * nblocks) {
    bf16x4 q;
#pragma unroll
    for (int j = 0; j < 4; ++j) q[j] = (bf16)pack_value(e0 + j, ws);  // PACK_TOTAL % 4 == 0
    *reinterpret_cast<bf16x4*>(out + e0) = q;
  }
}
static_assert(PACK_TOTAL % 4 == 0 && P2F_OFF % 4 == 0, "packed regions in whole 8-B runs");

__global__ __launch_bounds__(256) void pack_weights_kernel(PackSrc ws, bf16* __restrict__ out) {
  pack_range(ws, out, 0, blockIdx.x, gridDim.x);
}

// The inverse of pack_value: the packed slots of one master weight element (conv1: 1, conv2 / conv3 / fc1: the
// forward and the backward copy), so the optimizer can write next step's fragments as it updates the fp32
// masters (no pack launch per forward).  `which`: 0 conv1 [32][1][5][5], 1 conv2 [64][32][3][3],
// 2 conv3 [128][64][3][3], 3 fc1 [10][2048]; l: the element's index in its tensor.  Padding slots (conv1
// taps past 5x5, fc1 columns past 10) never change: the first pack zeroed them.
__device__ __forceinline__ int frag_slot(int ks, int lane, int j, int nt, int KS) { return ((nt * KS + ks) * 64 + lane) * 8 + j; }
__device__ __forceinline__ void pack_scatter(int which, int l, bf16 v, bf16* __restrict__ out) {
  if (which == 0) {
    const int co = l / 25, r = l - co * 25, kh = r / 5, kw = r - kh * 5;
    out[P1_OFF + frag_slot(kh >> 2, ((kh & 3) << 4) | (co >> 1), kw, co & 1, 2)] = v;
  } else if (which == 1) {  // forward: k = tap*32 + ci; data gradient: k = (8 - tap)*64 + co, n = ci
    const int co = l / 288, ci = (l / 9) & 31, t = l % 9;
    const int kf = t * 32 + ci, kd = (8 - t) * 64 + co;
    out[P2F_OFF + frag_slot(kf >> 5, (((kf >> 3) & 3) << 4) | (co & 15), kf & 7, co >> 4, 9)] = v;
    out[P2D_OFF + frag_slot(kd >> 5, (((kd >> 3) & 3) << 4) | (ci & 15), kd & 7, ci >> 4, 18)] = v;
  } else if (which == 2) {  // forward: k = tap*64 + ci; data gradient (scatter form): ks = tap*4 + co/32
    const int co = l / 576, ci = (l / 9) & 63, t = l % 9;
    const int kf = t * 64 + ci;
    out[P3F_OFF + frag_slot(kf >> 5, (((kf >> 3) & 3) << 4) | (co & 15), kf & 7, co >> 4, 18)] = v;
    out[P3D_OFF + frag_slot(t * 4 + (co >> 5), (((co >> 3) & 3) << 4) | (ci & 15), co & 7, ci >> 4, 36)] = v;
  } else {  // fc1 column c = co*16 + window: backward [window][co][n], forward B fragments k = window*128 + co
    const int n = l >> 11, c = l & 2047, co = c >> 4, wd = c & 15;
    out[PFC_OFF + wd * 1280 + co * 10 + n] = v;
    const int k = wd * 128 + co;
    out[PFF_OFF + frag_slot(k >> 5, (((k >> 3) & 3) << 4) | n, k & 7, 0, 0)] = v;
  }
}

struct PackDst {
  bf16* out;
  int64_t off[4];  // each weight's first element in the flat parameter range
};
constexpr int kPackLen[4] = {32 * 25, 64 * 32 * 9, 128 * 64 * 9, 10 * 2048};

// SGD over a flat fp32 range (params / grads / momentum laid out identically, as elementwise.hip's
// sgd_flat_kernel) that also stores every updated ConvNet weight into its packed bf16 slots.
template <bool MOM>
__global__ __launch_bounds__(256) void cn_sgd_pack_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                          float* __restrict__ m, int64_t n, SgdArgs a, PackDst d) {
  const SgdDev sd = load_sgd(a);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = reinterpret_cast<float4*>(p)[i];
    const float4 gv = reinterpret_cast<const float4*>(g)[i];
    float4 mv = MOM ? reinterpret_cast<float4*>(m)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    sgd_elem<MOM>(pv.x, gv.x, mv.x, sd);
    sgd_elem<MOM>(pv.y, gv.y, mv.y, sd);
    sgd_elem<MOM>(pv.z, gv.z, mv.z, sd);
    sgd_elem<MOM>(pv.w, gv.w, mv.w, sd);
    reinterpret_cast<float4*>(p)[i] = pv;
    if (MOM) reinterpret_cast<float4*>(m)[i] = mv;
    const float v[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int64_t l0 = 4 * i - d.off[w];
      if (l0 + 3 < 0 || l0 >= kPackLen[w]) continue;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (l0 + k >= 0 && l0 + k < kPackLen[w]) pack_scatter(w, (int)(l0 + k), (bf16)v[k], d.out);
    }
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float pv = p[i], mv = MOM ? m[i] : 0.f;
    sgd_elem<MOM>(pv, g[i], mv, sd);
    p[i] = pv;
    if (MOM) m[i] = mv;
#pragma unroll
    for (int w = 0; w < 4; ++w)
      if (i >= d.off[w] && i - d.off[w] < kPackLen[w]) pack_scatter(w, (int)(i - d.off[w]), (bf16)pv, d.out);
  }
}

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned char u8x8 __attribute__((ext_vector_type(8)));

// Packed 16-bit VALU ops (two channels per instruction).  The constant 1 of min(m - v, 1) is made opaque
// to the optimiser (an empty asm that "defines" it): with a visible constant, LLVM turns the min into a
// per-element compare + select and scalarises the whole chain (the pool2 loop of the fused forward was
// 130 VALU + 40 SALU per 8 channels; this form is ~66 v_pk_* VALU).  (Every op as inline asm instead
// compiles to the same VALU count plus an s_nop between dependent asm statements.)
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 opaque_u16x2(uint32_t v) {
  asm volatile("" : "+v"(v));
  return __builtin_bit_cast(u16x2, v);
}

// relu(max over a 2x2 window) of 8 bf16 channels, plus the pool2 code byte per channel: one-hot bit
// dy*2+dx of the first maximum in (0,0),(0,1),(1,0),(1,1) order (torch max_pool2d semantics), 0 = the
// pooled value is 0 (no gradient flows).  Done on the raw bf16 bit patterns with packed int16
// ops (2 channels per instruction): for values >= 0 the integer order is the float order and any
// negative value is a negative int16, so max(v0..v3, 0) over int16 IS relu(max).  Per channel pair:
// k_i = min(m - v_i, 1) is 0 iff v_i == m (u16 difference; a negative v_i wraps to non-zero), the first
// index with v_i == m is k0 + k0 k1 + k0 k1 k2 = k0 + (k0 k1)(1 + k2), and the code is (1 << idx) * min(m, 1).
__device__ __forceinline__ void pool2_code8(const bf16* r0, int rs, int w, bf16x8& out, uint2& code) {
  const uint4 v0 = *reinterpret_cast<const uint4*>(r0);
  const uint4 v1 = *reinterpret_cast<const uint4*>(r0 + rs);
  const uint4 v2 = *reinterpret_cast<const uint4*>(r0 + w * rs);
  const uint4 v3 = *reinterpret_cast<const uint4*>(r0 + (w + 1) * rs);
  const u16x2 one = opaque_u16x2(0x00010001u);
  const uint32_t a[4] = {v0.x, v0.y, v0.z, v0.w}, b[4] = {v1.x, v1.y, v1.z, v1.w},
                 c[4] = {v2.x, v2.y, v2.z, v2.w}, d[4] = {v3.x, v3.y, v3.z, v3.w};
  // stage-major over the 4 channel pairs: dependent packed ops are never adjacent (gfx950 pads a packed
  // 16-bit result read by the next instruction with an s_nop, 4 cycles each)
  s16x2 sa[4], sb[4], sc[4], x0[4], x1[4], sm[4];
  u16x2 k0[4], k1[4], k2[4], t1[4], idx[4];
  uint32_t m[4], cd[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    sa[j] = __builtin_bit_cast(s16x2, a[j]);
    sb[j] = __builtin_bit_cast(s16x2, b[j]);
    sc[j] = __builtin_bit_cast(s16x2, c[j]);
    x0[j] = __builtin_elementwise_max(sa[j], sb[j]);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) x1[j] = __builtin_elementwise_max(sc[j], __builtin_bit_cast(s16x2, d[j]));
#pragma unroll
  for (int j = 0; j < 4; ++j) sm[j] = __builtin_elementwise_max(x0[j], x1[j]);
#pragma unroll
  for (int j = 0; j < 4; ++j) sm[j] = __builtin_elementwise_max(sm[j], (s16x2)0);
#pragma unroll
  for (int j = 0; j < 4; ++j) k0[j] = __builtin_bit_cast(u16x2, sm[j]) - __builtin_bit_cast(u16x2, sa[j]);
#pragma unroll
  for (int j = 0; j < 4; ++j) k1[j] = __builtin_bit_cast(u16x2, sm[j]) - __builtin_bit_cast(u16x2, sb[j]);
#pragma unroll
  for (int j = 0; j < 4; ++j) k2[j] = __builtin_bit_cast(u16x2, sm[j]) - __builtin_bit_cast(u16x2, sc[j]);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    k0[j] = __builtin_elementwise_min(k0[j], one);
    k1[j] = __builtin_elementwise_min(k1[j], one);
    k2[j] = __builtin_elementwise_min(k2[j], one);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) t1[j] = k0[j] * k1[j];
#pragma unroll
  for (int j = 0; j < 4; ++j) k2[j] = k2[j] + one;
#pragma unroll
  for (int j = 0; j < 4; ++j) idx[j] = t1[j] * k2[j] + k0[j];
#pragma unroll
  for (int j = 0; j < 4; ++j) t1[j] = __builtin_elementwise_min(__builtin_bit_cast(u16x2, sm[j]), one);
#pragma unroll
  for (int j = 0; j < 4; ++j) idx[j] = one << idx[j];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    m[j] = __builtin_bit_cast(uint32_t, sm[j]);
    cd[j] = __builtin_bit_cast(uint32_t, idx[j] * t1[j]);
  }
  out = __builtin_bit_cast(bf16x8, make_uint4(m[0], m[1], m[2], m[3]));
  // codes (one per 16-bit half, < 16) -> 8 bytes: v_perm_b32 picks bytes 0 / 2 of two registers each
  code = make_uint2(__builtin_amdgcn_perm(cd[1], cd[0], 0x06040200u), __builtin_amdgcn_perm(cd[3], cd[2], 0x06040200u));
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

// Async global -> LDS copy of 16 B per lane (global_load_lds_dwordx4): the LDS destination is the
// wave-uniform base + lane * 16, so the image it fills is lane-linear (no padding inside a wave's 1 KiB).
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// The same copy issued from inline asm.  With the builtin, the compiler sees an LDS write on the VM counter
// and drains it (s_waitcnt vmcnt(0)) before the next LDS read, however unrelated - the prefetch then never
// overlaps the compute it was issued ahead of (seen in the ISA of conv1_wgrad / conv3_fwd).  Here the copy
// is invisible to the compiler: the consumer must `s_waitcnt vmcnt(0)` itself before the barrier that
// publishes the buffer (c_dma_wait).  M0 is set inside the asm; no kernel using this sets M0 otherwise
// (the ISA of these kernels has no other M0 writer: checked when this was introduced).
__device__ __forceinline__ void glds16_async(const void* gsrc, void* lds_wave_base) {
  const unsigned base = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)((__attribute__((address_space(3))) char*)(lds_wave_base)));
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(base), "v"(gsrc) : "memory");
}
__device__ __forceinline__ void c_dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// The same copy from a wave-uniform base (SGPR pair) plus a 32-bit per-lane byte offset: the per-lane part of
// an image's copy is the same for every image, so it is computed once and no 64-bit address math runs per copy.
__device__ __forceinline__ void glds16_sv(const void* sbase, uint32_t voff, void* lds_wave_base) {
  const unsigned base = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)((__attribute__((address_space(3))) char*)(lds_wave_base)));
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(base), "v"(voff), "s"(sbase)
               : "memory");
}

// ================================================================== F1: conv1 (MFMA)
// The zero-ringed 30x30 input is staged as 8 copies shifted by s = 0..7 columns (rows of 32):
// copy s holds xpad[r][c + s].  Eight consecutive pixels xpad[r][ow .. ow+7] are then ONE aligned
// ds_read_b128 at copy (ow & 7), column (ow & ~7) - this is the im2col of a 5-wide filter row, so
// the GEMM K is laid out as k = kh*8 + kw (kw < 5 valid): 2 k-steps of 32, no per-element gather.
constexpr int XC_W = 32, XC_SZ = 30 * XC_W;  // one shifted copy (bf16)

template <bool U8>
__device__ __forceinline__ void c1_load(const void* xin, int b, int tid, uint32_t& u, float4& f) {
  if (tid < 196) {
    if (U8)
      u = reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(xin) + (int64_t)b * 784)[tid];
    else
      f = reinterpret_cast<const float4*>(static_cast<const float*>(xin) + (int64_t)b * 784)[tid];
  }
}

// Normalise this thread's 4 pixels (one row segment: columns pc0 .. pc0+3, pc0 = 4*(tid%7) + 1) and
// write them into copies 0..NC-1.  pc0 = 1 (mod 4), so each copy's alignment is known at compile time:
// one ds_write_b64 (s = 1 mod 4), two b32 (s = 3 mod 4) or b16 + b32 + b16 - instead of 4 b16 per copy.
// A segment starting at pc0 = 1 writes columns 1-s .. < 0 of copy s "before" its row, i.e. into columns
// 33-s+k of the previous row: those are only ever read as filter columns kw >= 5 (zero weights in the
// forward, zero dC rows >= 26 in wgrad), so the spill is harmless and the zero ring (copy column 29-s,
// column 0 of copy 0, rows 0/29) is never written.
template <bool U8, int NC, int RS = XC_W, int CS = XC_SZ>
__device__ __forceinline__ void c1_store(bf16* xc, int tid, uint32_t u, float4 f, float mean, float inv_std,
                                         float in_scale) {
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
    bf16 xv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) xv[k] = (bf16)((v[k] - mean) * inv_std);
    const uint32_t lo16 = __builtin_bit_cast(uint16_t, xv[0]), m1 = __builtin_bit_cast(uint16_t, xv[1]),
                   m2 = __builtin_bit_cast(uint16_t, xv[2]), hi16 = __builtin_bit_cast(uint16_t, xv[3]);
    const uint32_t p01 = lo16 | (m1 << 16), p23 = m2 | (hi16 << 16), p12 = m1 | (m2 << 16);
    const int pr = tid / 7 + 1, pc0 = 4 * (tid % 7) + 1;
#pragma unroll
    for (int s = 0; s < NC; ++s) {
      bf16* d = xc + s * CS + pr * RS + pc0 - s;  // may point before the row (see above)
      if ((s & 3) == 1) {
        *reinterpret_cast<uint2*>(d) = make_uint2(p01, p23);
      } else if ((s & 3) == 3) {
        reinterpret_cast<uint32_t*>(d)[0] = p01;
        reinterpret_cast<uint32_t*>(d)[1] = p23;
      } else {
        d[0] = xv[0];
        *reinterpret_cast<uint32_t*>(d + 1) = p12;
        d[3] = xv[3];
      }
    }
  }
}

// conv1 pool/ReLU codes for the backward: [B][py 13][co/2 16][px 16] bytes (px 13..15 zero), one nibble per
// channel (low: even co, high: odd co), each 1 << argmax (dy*2+dx) if the pooled value is > 0, else 0 (the
// gradient's destination, one-hot).  Window rows per channel pair let conv1 wgrad read the codes of 4
// neighbouring windows of one channel as one 4-byte load.  (Nibbles, not bytes: conv1 forward is bound by
// its HBM writes, 17.4 -> 14.1 KB per image.)
constexpr int C1I_IMG = 13 * 256;      // 3328 bytes per image
constexpr int C1A_IMG = 169 * 32;      // a1 elements per image

// relu(max) + argmax of a 2x2 window (the 4 accumulator registers of a window-ordered m-tile, bias
// included), as one signed-integer max over keys (bits(c_i) with the low 2 bits replaced by 3 - i): for
// positive values the int order is the float order, ties keep the first index (torch semantics), and a
// window whose maximum is <= 0 has no gradient, so its argmax is irrelevant.  Returns the pooled value's
// bits (<= 2 ulp of fp32 below the exact value) and the code byte (one-hot argmax, 0 if the ReLU is off).
__device__ __forceinline__ uint32_t pool4_key(const f32x4& c, uint32_t& code) {
  // v_bitop3_b32 0xBA = (S0 & ~S1) | S2: one instruction per key
  const int k0 = (int)__builtin_amdgcn_bitop3_b32(__float_as_uint(c[0]), 3u, 3u, 0xBA);
  const int k1 = (int)__builtin_amdgcn_bitop3_b32(__float_as_uint(c[1]), 3u, 2u, 0xBA);
  const int k2 = (int)__builtin_amdgcn_bitop3_b32(__float_as_uint(c[2]), 3u, 1u, 0xBA);
  const int k3 = (int)(__float_as_uint(c[3]) & ~3u);
  const int km = max(max(max(k0, k1), k2), max(k3, 0));  // two v_max3_i32
  code = km > 0 ? 1u << (~(uint32_t)km & 3u) : 0u;  // one-hot: bit dy*2+dx = where the gradient goes
  return (uint32_t)km;
}

// F1: 4 waves; per image 43 m-tiles of 16 window-ordered rows (169 windows), 2 n-tiles (channel pairs),
// K = 2 k-steps (filter rows 0-3 | 4).  Wave w owns m-tiles w, w+4, ..: their LDS offsets are
// computed once per workgroup and kept in registers.  Pooled outputs (one dword = 2 channels) and codes
// (2 bytes) are collected in LDS and written with 16-B stores; the next image's pixels are loaded into
// registers while this one computes.
constexpr int C1F_MT = 11;  // m-tiles per wave (wave 3: 10)
// copy stride padded 960 -> 1048 elements: the 16 A-row reads of a ds_read_b128 lane group then hit
// 2x fewer conflicting bank slots (modelled: 11.9 -> 8.2 LDS cycles per read, ideal 4)
constexpr int C1F_CS = 1048;
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
// PACK: this launch also packs every layer's weights (cn_pack_weights) for the kernels after it: workgroups
// >= conv_blocks do only that, and the conv1 workgroups build their own fragments from the fp32 masters
// (one launch per step fewer; at the reference batch every launch is ~5 us of a ~100 us step).
template <bool U8, bool PACK>
__global__ __launch_bounds__(256) void conv1_fwd_kernel(const void* __restrict__ xin,
                                                        const bf16* __restrict__ packed,
                                                        const float* __restrict__ bias,
                                                        bf16* __restrict__ a1,
                                                        uint8_t* __restrict__ idx1, int B,
                                                        float mean, float inv_std, float in_scale,
                                                        PackSrc ws, bf16* __restrict__ pack_out,
                                                        int conv_blocks) {
  if (PACK && (int)blockIdx.x >= conv_blocks) {
    pack_range(ws, pack_out, 0, blockIdx.x - conv_blocks, gridDim.x - conv_blocks);
    return;
  }
  __shared__ __attribute__((aligned(16))) bf16 xs[2][8 * C1F_CS];
  __shared__ __attribute__((aligned(16))) uint32_t ot[172 * 16];      // rows >= 169: dropped tiles
  __shared__ __attribute__((aligned(16))) uint8_t ct[C1I_IMG + 64];   // + a dump row for them
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, gq = lane >> 4;
  const bf16x8* pk = reinterpret_cast<const bf16x8*>(packed + P1_OFF);
  bf16x8 bw[2][2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (PACK) {
#pragma unroll
        for (int j = 0; j < 8; ++j) bw[nt][ks][j] = (bf16)pack_value(P1_OFF + ((nt * 2 + ks) * 64 + lane) * 8 + j, ws);
      } else {
        bw[nt][ks] = pk[(nt * 2 + ks) * 64 + lane];
      }
    }
  const float bias0 = bias[2 * r16], bias1 = bias[2 * r16 + 1];
  const f32x4 bias0v = {bias0, bias0, bias0, bias0}, bias1v = {bias1, bias1, bias1, bias1};
  // per m-tile: A-row offset inside a copy buffer (elements; kh row added per k-step) and code offset
  int aoff[C1F_MT], coff[C1F_MT];
#pragma unroll
  for (int j = 0; j < C1F_MT; ++j) {
    const int mt = wave + 4 * j;
    const int w = min(4 * mt + (r16 >> 2), 168), i = r16 & 3;  // rows >= 676: clamped, dropped
    const int oh = 2 * (w / 13) + (i >> 1), ow = 2 * (w % 13) + (i & 1);
    aoff[j] = (ow & 7) * C1F_CS + oh * XC_W + (ow & ~7) + gq * XC_W;
    const int wc = 4 * mt + gq;
    coff[j] = wc < 169 ? (wc / 13) * 256 + r16 * 16 + wc % 13 : C1I_IMG + lane;
  }
  for (int i = tid; i < 2 * 8 * C1F_CS / 8; i += 256) reinterpret_cast<bf16x8*>(&xs[0][0])[i] = zero_bf16x8();
  for (int i = tid; i < C1I_IMG / 16; i += 256) reinterpret_cast<uint4*>(ct)[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  uint32_t pu = 0;
  float4 pf = make_float4(0.f, 0.f, 0.f, 0.f);
  int b = blockIdx.x;
  if (b < B) {
    c1_load<U8>(xin, b, tid, pu, pf);
    c1_store<U8, 8, XC_W, C1F_CS>(xs[0], tid, pu, pf, mean, inv_std, in_scale);
  }
  __syncthreads();
  int cur = 0;
  const int nblk = PACK ? conv_blocks : (int)gridDim.x;
  for (; b < B; b += nblk) {
    const int nb = b + nblk;
    if (nb < B) c1_load<U8>(xin, nb, tid, pu, pf);
    const bf16* x = xs[cur];
    // software-pipelined: the MFMAs of tile j are issued before the epilogue of tile j-1
    auto epilogue = [&](int j, const f32x4& c0, const f32x4& c1) {
      uint32_t g0, g1;
      const uint32_t v0 = pool4_key(c0, g0), v1 = pool4_key(c1, g1);
      const bf16x2v pv = __builtin_convertvector(f32x2v{__uint_as_float(v0), __uint_as_float(v1)}, bf16x2v);
      ot[(4 * (wave + 4 * j) + gq) * 16 + r16] = __builtin_bit_cast(uint32_t, pv);  // v_cvt_pk_bf16_f32
      ct[coff[j]] = (uint8_t)(g0 | (g1 << 4));
    };
    f32x4 p0 = zero_f32x4(), p1 = zero_f32x4();
#pragma unroll
    for (int j = 0; j < C1F_MT; ++j) {
      f32x4 c0 = bias0v, c1 = bias1v;  // the bias rides in the accumulator (one channel per lane)
      const bool live = j < C1F_MT - 1 || wave < 3;  // wave-uniform
      if (live) {
        const bf16* xr = x + aoff[j];
        const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(xr);
        const bf16x8 a1v = *reinterpret_cast<const bf16x8*>(xr + (4 - gq) * XC_W);  // filter row 4
        c0 = mfma16x16x32(a0, bw[0][0], c0);
        c1 = mfma16x16x32(a0, bw[1][0], c1);
        c0 = mfma16x16x32(a1v, bw[0][1], c0);
        c1 = mfma16x16x32(a1v, bw[1][1], c1);
      }
      if (j > 0) epilogue(j - 1, p0, p1);
      if (live && j == C1F_MT - 1) epilogue(j, c0, c1);
      p0 = c0;
      p1 = c1;
    }
    if (nb < B) c1_store<U8, 8, XC_W, C1F_CS>(xs[cur ^ 1], tid, pu, pf, mean, inv_std, in_scale);
    __syncthreads();  // output tile complete; next image's copies written
    const uint4* os = reinterpret_cast<const uint4*>(ot);
    uint4* og = reinterpret_cast<uint4*>(a1 + (int64_t)b * C1A_IMG);
    for (int c = tid; c < C1A_IMG / 8; c += 256) og[c] = os[c];
    const uint4* cs = reinterpret_cast<const uint4*>(ct);
    uint4* cg = reinterpret_cast<uint4*>(idx1 + (int64_t)b * C1I_IMG);
    for (int c = tid; c < C1I_IMG / 16; c += 256) cg[c] = cs[c];
    __syncthreads();  // output tile read out before the next image overwrites it
    cur ^= 1;
  }
}

// ================================================================== F2: conv2 + ReLU + pool2
// 256 threads; wave (wm, wn) owns n-tiles {2wn, 2wn+1} x m-tiles {4wm..4wm+3} (121 rows -> 128).
constexpr int C2_XRS = 48;  // bf16 per LDS row of the a1 image (32 + 16 pad): 96-B rows, see c2f_tile_pos
// forward m-tile -> output position map (255 = padding row): every full tile holds two positions of
// each residue (y*13 + x) mod 8, one among lanes {0-3,12-15} and one among {4-11}, so with 96-B rows
// the 16 rows of a ds_read_b128 lane group land on 16 distinct 16-B bank slots (modelled 10.5 -> 4
// LDS cycles per operand read; generator: tools/lds_bank_model.py)
__constant__ uint8_t c2f_tile_pos[128] = {0,3,6,1,8,17,12,9,18,13,10,11,4,7,2,5,14,23,20,15,28,31,26,29,32,27,22,25,24,21,16,19,34,37,40,35,42,51,46,43,44,41,36,45,38,33,30,39,48,57,54,49,62,65,60,55,58,61,56,59,52,47,50,53,68,71,66,63,76,77,74,69,78,75,70,79,72,67,64,73,82,85,80,83,88,91,94,89,92,95,90,93,86,81,84,87,96,105,100,97,102,111,108,103,112,109,104,107,106,101,98,99,116,119,114,117,255,255,255,255,255,255,118,255,120,115,110,113};
constexpr int C2_CRS = 72;  // bf16 per LDS row of the output staging tile (64 + 8)

__global__ __launch_bounds__(256, 3) void conv2_fwd_kernel(const bf16* __restrict__ a1,
                                                           const bf16* __restrict__ packed,
                                                           const float* __restrict__ bias,
                                                           bf16* __restrict__ a2, uint8_t* __restrict__ idx2,
                                                           int B) {
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
  // operands swapped (weights = A): a lane's 4 accumulators are 4 consecutive channels of one
  // position, staged with one 8-byte LDS store
  const int c4 = (lane >> 4) * 4;
  f32x4 bv[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[t][i] = bias[(2 * wn + t) * 16 + c4 + i];
  int base[4], opos[4];  // padding rows read a valid address; their outputs are dropped
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    opos[mt] = c2f_tile_pos[(4 * wm + mt) * 16 + r16];
    const int mm = opos[mt] == 255 ? 0 : opos[mt];
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
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(x + (base[mt] + shift) * C2_XRS + q8);
        acc[mt][0] = mfma16x16x32(bw[0][ks], a, acc[mt][0]);
        acc[mt][1] = mfma16x16x32(bw[1][ks], a, acc[mt][1]);
      }
    }
    __syncthreads();  // previous image's pooling reads of Cs are complete
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int m = opos[mt];
      if (m < 121) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const f32x4 v = acc[mt][t] + bv[t];
          *reinterpret_cast<bf16x4*>(Cs + m * C2_CRS + (2 * wn + t) * 16 + c4) =
              bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
        }
      }
    }
    if (nb < B) store(X[cur ^ 1]);
    __syncthreads();
    // relu + overlapping 2x2/s1 pool of the staged z2 tile -> a2 and the pool2 codes
    bf16x8* da = reinterpret_cast<bf16x8*>(a2 + (int64_t)b * 6400);
    uint2* di = reinterpret_cast<uint2*>(idx2 + (int64_t)b * 6400);
    for (int it = tid; it < 800; it += 256) {
      const int p = it >> 3, c = (it & 7) * 8;
      bf16x8 v;
      uint2 code;
      pool2_code8(Cs + ((p / 10) * 11 + p % 10) * C2_CRS + c, C2_CRS, 11, v, code);
      da[it] = v;
      di[it] = code;
    }
    cur ^= 1;
  }
}

// ================================================================== F3: conv3 + ReLU + pool3 + fc1
// 256 threads; wave w owns output channels 32w..32w+31 (n-tiles 2w, 2w+1) for all 16 pool windows.
constexpr int C3_XRS = 72;  // bf16 per padded LDS row of a2 (backward wgrad role)

// a2 image -> LDS staging buffer R (lane-linear 16-B chunks, LDS-DMA: no VGPRs, lands while the
// previous image computes); nthreads threads issue the 13 wave-instructions (the last half full).
__device__ __forceinline__ void a2_glds(const bf16* __restrict__ a2, int b, bf16* R, int wave, int lane,
                                        int nwaves) {
  const bf16* src = a2 + (int64_t)b * 6400;
  for (int k = wave; k < 13; k += nwaves) {
    const int slot = k * 64 + lane;
    if (slot < 800) glds16_async(src + slot * 8, R + k * 512);
  }
}

// staging buffer -> padded MFMA rows (RS elements per row, C3_XRS by default): the padding keeps the 16
// rows of a fragment read on distinct banks, which a lane-linear DMA image cannot have
template <int RS = C3_XRS>
__device__ __forceinline__ void a2_relayout(const bf16* R, bf16* X, int tid, int nthreads) {
  for (int c = tid; c < 800; c += nthreads)
    *reinterpret_cast<bf16x8*>(X + (c >> 3) * RS + (c & 7) * 8) = reinterpret_cast<const bf16x8*>(R)[c];
}

// conv3 forward A-operand image: 160-B rows and this pool-window order of the m-tiles make every
// ds_read_b128 fragment read conflict-free (modelled with the b128 lane groups of MI355X_MICROARCH.md:
// 1.0 LDS cycles per read, was 2.0 with 144-B rows and the natural window order; the measured
// SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS was 3.0).  Entry 4*mt + j = the pool window (row-major
// in the 4x4 window grid) whose 4 positions are rows 4j..4j+3 of m-tile mt.
constexpr int C3F_XRS = 80;
__constant__ uint8_t c3f_win[16] = {1, 9, 13, 11, 10, 3, 15, 8, 7, 12, 0, 5, 4, 6, 2, 14};

// FC (small batches): fc1 runs in this launch too.  Each lane multiplies its 8 pooled values by their
// 10 fc1 weights (the [window][co][n] pack, staged in LDS once per workgroup) and the 256 lanes' partial
// logits are summed through LDS in a fixed order.  At B <= a few thousand the separate fc1 launch (and
// its ~1.5 us kernel boundary) cost more than this; at large B the MFMA fc1 pass over a3 is cheaper.
constexpr int C3F_FCW = 16 * 128 * 10;  // bf16 fc1 weights in LDS
template <bool FC>
__global__ __launch_bounds__(256, 2) void conv3_fwd_kernel(const bf16* __restrict__ a2,
                                                           const bf16* __restrict__ packed,
                                                           const float* __restrict__ bias,
                                                           bf16* __restrict__ a3,
                                                           uint8_t* __restrict__ idx3, int B,
                                                           const float* __restrict__ bfc,
                                                           float* __restrict__ logits) {
  __shared__ __attribute__((aligned(16))) bf16 R[100 * 64];
  __shared__ __attribute__((aligned(16))) bf16 X[100 * C3F_XRS];
  __shared__ __attribute__((aligned(16))) char fcs[FC ? C3F_FCW * 2 + 10 * 256 * 4 : 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  bf16* fw = reinterpret_cast<bf16*>(fcs);                      // [window][co][n]
  float* fred = reinterpret_cast<float*>(fcs + C3F_FCW * 2);    // [n][256 lanes]
  if (FC) {
    const uint4* src = reinterpret_cast<const uint4*>(packed + PFC_OFF);
    for (int c = tid; c < C3F_FCW / 8; c += 256) reinterpret_cast<uint4*>(fw)[c] = src[c];
  }
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
  int base[4], wcol[4];  // A row of this lane per m-tile; pool window of this lane's accumulators
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    base[mt] = win_pos(4 * c3f_win[4 * mt + (r16 >> 2)] + (r16 & 3), 10);
    wcol[mt] = c3f_win[4 * mt + (lane >> 4)];
  }
  int b = blockIdx.x;
  if (b < B) a2_glds(a2, b, R, wave, lane, 4);
  for (; b < B; b += gridDim.x) {
    c_dma_wait();
    __syncthreads();  // R has landed; the previous image's X reads are done
    a2_relayout<C3F_XRS>(R, X, tid, 256);
    __syncthreads();  // X complete, R free
    const int nb = b + gridDim.x;
    if (nb < B) a2_glds(a2, nb, R, wave, lane, 4);  // lands while the MFMAs below run
    f32x4 acc[4][2];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[mt][0] = acc[mt][1] = zero_f32x4();
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) {
      const int tap = ks >> 1, c0 = (ks & 1) * 32;
      const int shift = (tap / 3) * 10 + tap % 3;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(X + (base[mt] + shift) * C3F_XRS + c0 + q8);
        acc[mt][0] = mfma16x16x32(a, bw[0][ks], acc[mt][0]);
        acc[mt][1] = mfma16x16x32(a, bw[1][ks], acc[mt][1]);
      }
    }
    float part[10];
#pragma unroll
    for (int n = 0; n < 10; ++n) part[n] = 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int wc = wcol[mt], co = 32 * wave + 16 * t + r16;
        int g;
        const bf16 pb = (bf16)pool4(acc[mt][t], bv[t], g);
        const int64_t o = ((int64_t)b * 16 + wc) * 128 + co;
        a3[o] = pb;
        idx3[o] = (uint8_t)g;
        if (FC) {
          const float pv = (float)pb;
          const uint32_t* wp = reinterpret_cast<const uint32_t*>(fw + (wc * 128 + co) * 10);  // 4-B aligned
#pragma unroll
          for (int h = 0; h < 5; ++h) {
            const uint32_t u = wp[h];
            part[2 * h] = fmaf(pv, __uint_as_float(u << 16), part[2 * h]);
            part[2 * h + 1] = fmaf(pv, __uint_as_float(u & 0xffff0000u), part[2 * h + 1]);
          }
        }
      }
    if (FC) {
#pragma unroll
      for (int n = 0; n < 10; ++n) fred[n * 256 + tid] = part[n];
      __syncthreads();
      // 160 threads: logit n = t >> 4 sums lanes c + 16 i (i < 16), then 16 lanes combine by shuffles
      if (tid < 160) {
        const int n = tid >> 4, c = tid & 15;
        float v = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) v += fred[n * 256 + c + 16 * i];
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if (c == 0) logits[(int64_t)b * 10 + n] = v + bfc[n];
      }
      // the next image's top barrier orders these reads before fred is rewritten
    }
  }
}

// fc1 as its own MFMA GEMM: logits[b][n] = sum_k a3[b][k] * Wfc'[k][n] + bfc[n], k = window*128 + co.
// One wave per 16 images; A fragments stream straight from global (16 B per lane, no LDS), the
// 64 B-fragments (N = 10 padded to 16) sit in LDS.  Unfused from conv3 because reducing 10 logits
// across 256 lanes per image cost the conv3 kernel more than this whole pass over a3.
constexpr int FC1_G = 8;  // 16-image groups per workgroup
__global__ __launch_bounds__(256) void fc1_fwd_kernel(const bf16* __restrict__ a3,
                                                      const bf16* __restrict__ packed,
                                                      const float* __restrict__ bfc,
                                                      float* __restrict__ logits, int B) {
  // The 4 waves split K (512 each) and hold their 16 B-fragments in VGPRs, loaded once from the
  // L2-resident pack.  A bandwidth-bound pass over a3 (4 KB per image): group g+1's A fragments are
  // loaded while group g's MFMAs and cross-wave sum run (two register sets; one set in flight had run at
  // ~2.9 TB/s).  Partials are summed in a fixed order.
  __shared__ f32x4 red[2][3][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bf16x8* src = reinterpret_cast<const bf16x8*>(packed + PFF_OFF);
  bf16x8 w[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = src[(wave * 16 + j) * 64 + lane];
  const int g0 = blockIdx.x * FC1_G;
  const int ng = min(FC1_G, cdiv(B, 16) - g0);
  auto load = [&](int g, bf16x8 (&av)[16]) {
    const int row = min((g0 + g) * 16 + (lane & 15), B - 1);
    const bf16x8* ap = reinterpret_cast<const bf16x8*>(a3 + (int64_t)row * 2048) + (lane >> 4) + wave * 64;
#pragma unroll
    for (int j = 0; j < 16; ++j) av[j] = ap[j * 4];
  };
  auto group = [&](int g, const bf16x8 (&av)[16]) {
    const int b0 = (g0 + g) * 16;
    f32x4 acc0 = zero_f32x4(), acc1 = zero_f32x4();
#pragma unroll
    for (int j = 0; j < 16; j += 2) {
      acc0 = mfma16x16x32(av[j], w[j], acc0);
      acc1 = mfma16x16x32(av[j + 1], w[j + 1], acc1);
    }
    const f32x4 acc = acc0 + acc1;
    if (wave > 0) red[g & 1][wave - 1][lane] = acc;  // two slots: one barrier per group
    __syncthreads();
    if (wave == 0) {
      const f32x4 t = acc + red[g & 1][0][lane] + red[g & 1][1][lane] + red[g & 1][2][lane];
      const int nn = lane & 15;
      if (nn < 10) {
        const float bn = bfc[nn];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int bb = b0 + (lane >> 4) * 4 + i;
          if (bb < B) logits[(int64_t)bb * 10 + nn] = t[i] + bn;
        }
      }
    }
  };
  bf16x8 va[16], vb[16];
  if (ng > 0) load(0, va);
  for (int g = 0; g < ng; g += 2) {  // unrolled by 2: register sets are not indexable
    if (g + 1 < ng) load(g + 1, vb);
    group(g, va);
    if (g + 1 < ng) {
      if (g + 2 < ng) load(g + 2, va);
      group(g + 1, vb);
    }
  }
}

// ================================================================== F1+F2+F3: fused forward
// The whole forward of one image in one 512-thread workgroup, a1 / a2 never re-read from HBM (the
// three separate launches move 64 KB per image, this one 40 KB: the forward is HBM- as much as
// MFMA-bound).  Waves 0-3 are the PRODUCER (conv1 + pool1, conv2 + pool2 of image s), waves 4-7 the
// CONSUMER (conv3 + pool3 + fc1 of image s-1, one step behind).  A step is three barrier-separated
// phases, the same barriers for both halves:
//   phase 1  producer: conv1 MFMAs on the staged input -> pooled a1 straight into conv2's operand
//                      rows (X2) + codes (CT)               consumer: conv3 k-steps 0-8 of image s-1
//   phase 2  producer: next input -> XS; a1 / idx1 -> HBM; conv2 MFMAs -> Cs
//                                                           consumer: conv3 k-steps 9-17
//   phase 3  producer: pool2 of Cs -> a2 / idx2 (HBM) and conv3's operand rows X3
//                                                           consumer: pool3 -> a3 / idx3, fc1 partials
// Each LDS buffer has one writer phase and its readers in other phases, so every buffer is single.
// The layouts are the separate kernels' (conv1_fwd_kernel / conv2_fwd_kernel / conv3_fwd_kernel<true>).
// PACK: weight fragments built from the fp32 masters (pack_value) by each workgroup, and the extra
// workgroups >= conv_blocks write the packed buffer for the backward.
constexpr int FF_XS = 8 * C1F_CS * 2;      // 16768: conv1 input, 8 shifted copies
constexpr int FF_X2 = 172 * C2_XRS * 2;    // 16512: a1 in conv2 operand rows (+3 dump rows)
constexpr int FF_CT = C1I_IMG + 64;        // 3392: conv1 codes (+ dump row)
constexpr int FF_CS = 121 * C2_CRS * 2;    // 17424: conv2 output tile
constexpr int FF_X3H = 100 * C3F_XRS;      // bf16 per a2 image in conv3 operand rows (16000 B)
constexpr int FF_X3 = 2 * FF_X3H * 2;      // double-buffered: the consumer reads image s-1 while image s lands
constexpr int FF_FW = C3F_FCW * 2;         // 40960: fc1 weights [window][co][n]
constexpr int FF_FR = 10 * 256 * 4;        // 10240: fc1 partial logits [n][256]
constexpr int FF_OFF_X2 = FF_XS, FF_OFF_CT = FF_OFF_X2 + FF_X2, FF_OFF_CS = FF_OFF_CT + FF_CT,
              FF_OFF_X3 = FF_OFF_CS + FF_CS, FF_OFF_FW = FF_OFF_X3 + FF_X3, FF_OFF_FR = FF_OFF_FW + FF_FW;
constexpr int FF_LDS = FF_OFF_FR + FF_FR;  // 137296
static_assert(FF_OFF_X2 % 16 == 0 && FF_OFF_CT % 16 == 0 && FF_OFF_CS % 16 == 0 && FF_OFF_X3 % 16 == 0 &&
                  FF_OFF_FW % 16 == 0 && FF_LDS <= 160 * 1024,
              "fused forward LDS");

// RINGDP_FF_STAMPS (diagnostic builds only, tools/build_variant.py): lane 0 of every wave records s_memtime at
// the 7 phase points of steps [FF_ST_S0, FF_ST_S0 + 8) into LDS past FF_LDS; workgroup FF_ST_BLK prints them
// at the end (per-phase time of the producer and consumer roles)
#ifdef RINGDP_FF_STAMPS
constexpr int FF_ST_S0 = 100, FF_ST_BLK = 5, FF_ST_BYTES = 8 * 8 * 8 * 8;
#define FF_ST(k)                                                                                           \
  do {                                                                                                     \
    if (s >= FF_ST_S0 && s < FF_ST_S0 + 8 && (threadIdx.x & 63) == 0)                                      \
      reinterpret_cast<unsigned long long*>(smem + FF_LDS)[((threadIdx.x >> 6) * 8 + (s - FF_ST_S0)) * 8 + (k)] = \
          __builtin_amdgcn_s_memtime();                                                                    \
  } while (0)
#else
constexpr int FF_ST_BYTES = 0;
#define FF_ST(k) \
  do {           \
  } while (0)
#endif

template <bool PACK>
__device__ __forceinline__ bf16x8 ff_frag(const bf16* __restrict__ packed, const PackSrc& ws, int off, int lane) {
  bf16x8 v;
  if (PACK) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (bf16)pack_value(off + lane * 8 + j, ws);
  } else {
    v = reinterpret_cast<const bf16x8*>(packed + off)[lane];
  }
  return v;
}

// In-launch weight packing (PACK): workgroups >= conv_blocks write the packed fragments and count
// themselves done in sync[0]; a conv wave waits for all of them before its first fragment read (lane 0
// polls with an agent-scope acquire, s_sleep between polls, bounded: the pack workgroups depend on
// nothing, so they finish).  The last conv workgroup to finish resets both words for the next launch
// (graph-replay safe: the counters live in a persistent pool, ops.cpp next_counter).
__device__ __forceinline__ void ff_wait_packed(unsigned* sync, int npack) {
  if ((threadIdx.x & 63) == 0) {
    for (int it = 0; it < (1 << 24); ++it) {
      if (__hip_atomic_load(sync, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)npack) break;
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// pool2 + ReLU of items [lo, hi) (item = position p, 8-channel chunk) of the staged conv2 tile -> a2 /
// idx2 in HBM and the conv3 operand rows of buffer X3b.  Phase 3 splits the items between the producer
// and the consumer (the producer is the long pole: 1103 vs 808 us alone at B=65536).
// items [0, p2split) are the producer's (kernel argument; RINGDP_FF_P2, default 800 of 800 since the packed
// pool2: phase 3 is consumer-bound (profiles/r06/fwd_stamps.md), and step times of 560 / 704 / 800 were
// 3.335 / 3.333 / 3.325 ms, two runs each, profiles/r06/fwd_pool2/p2_resweep.txt)
__device__ __forceinline__ void ff_pool2(const bf16* Cs, bf16* X3b, bf16* __restrict__ a2, uint8_t* __restrict__ idx2,
                                         int b, int t, int lo, int hi) {
  // uniform per-image bases, 32-bit per-item offsets (no 64-bit address math per item); at most 3 items
  // per thread (hi - lo <= 800, 256 threads per role)
  bf16x8* da = reinterpret_cast<bf16x8*>(a2 + (int64_t)b * 6400);
  uint2* di = reinterpret_cast<uint2*>(idx2 + (int64_t)b * 6400);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int it = lo + t + 256 * k;
    if (it >= hi) break;
    const int p = it >> 3, c = (it & 7) * 8;
    const int y = (p * 205) >> 11;  // p / 10 for p < 100
    bf16x8 v;
    uint2 code;
    pool2_code8(Cs + (p + y) * C2_CRS + c, C2_CRS, 11, v, code);  // row y * 11 + (p - 10 y) = p + y
    da[it] = v;
    di[it] = code;
    *reinterpret_cast<bf16x8*>(X3b + p * C3F_XRS + c) = v;
  }
}

// software-pipelined A-fragment reads in the conv2 (producer) / conv3 (consumer) k-step loops (A/B build macros)
// RINGDP_FF_P2_ALL (default): the producer pools all 800 pool2 items and the consumer's phase 3 holds no pool2
// code at all (fewer live registers beside conv3's 144 weight registers); 0: the split is the run-time
// p2split argument (RINGDP_FF_P2)
#ifndef RINGDP_FF_P2_ALL
#define RINGDP_FF_P2_ALL 1
#endif
#ifndef RINGDP_FF_KPIPE
#define RINGDP_FF_KPIPE 0
#endif
// issue priority between the two waves of a SIMD (scheduling A/B through RINGDP_FF_ABLATE, results unchanged):
// by default age decides (the older producer wave wins); bit 4: the consumer at priority 1 in phase 3; bit 5:
// the producer at priority 1 in phases 1-2
#ifndef RINGDP_FF_PPIPE
#define RINGDP_FF_PPIPE 0
#endif
template <bool U8, bool PACK>
__device__ __forceinline__ void ff_producer(char* smem, const void* __restrict__ xin, const bf16* __restrict__ packed,
                            const PackSrc& ws, const float* __restrict__ b1, const float* __restrict__ b2,
                            bf16* __restrict__ a1, uint8_t* __restrict__ idx1, bf16* __restrict__ a2,
                            uint8_t* __restrict__ idx2, int B, int b0, int bstep, int nsteps, float mean,
                            float inv_std, float in_scale, unsigned* sync, int npack, int p2split, int prio) {
  bf16* XS = reinterpret_cast<bf16*>(smem);
  bf16* X2 = reinterpret_cast<bf16*>(smem + FF_OFF_X2);
  uint32_t* X2u = reinterpret_cast<uint32_t*>(X2);
  uint8_t* CT = reinterpret_cast<uint8_t*>(smem + FF_OFF_CT);
  bf16* Cs = reinterpret_cast<bf16*>(smem + FF_OFF_CS);
  bf16* X3 = reinterpret_cast<bf16*>(smem + FF_OFF_X3);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;  // tid < 256
  const int r16 = lane & 15, gq = lane >> 4;
  // ---- conv1 setup (conv1_fwd_kernel)
  bf16x8 bw1[2][2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) bw1[nt][ks] = ff_frag<PACK>(packed, ws, P1_OFF + (nt * 2 + ks) * 512, lane);
  if (PACK) ff_wait_packed(sync, npack);  // conv1's 32 values per lane came from the masters directly
  const float c1b0 = b1[2 * r16], c1b1 = b1[2 * r16 + 1];
  const f32x4 bias0v = {c1b0, c1b0, c1b0, c1b0}, bias1v = {c1b1, c1b1, c1b1, c1b1};
  int aoff[C1F_MT], coff[C1F_MT];
#pragma unroll
  for (int j = 0; j < C1F_MT; ++j) {
    const int mt = wave + 4 * j;
    const int w = min(4 * mt + (r16 >> 2), 168), i = r16 & 3;
    const int oh = 2 * (w / 13) + (i >> 1), ow = 2 * (w % 13) + (i & 1);
    aoff[j] = (ow & 7) * C1F_CS + oh * XC_W + (ow & ~7) + gq * XC_W;
    const int wc = 4 * mt + gq;
    coff[j] = wc < 169 ? (wc / 13) * 256 + r16 * 16 + wc % 13 : C1I_IMG + lane;
  }
  // ---- conv2 setup (conv2_fwd_kernel)
  const int wm = wave >> 1, wn = wave & 1, q8 = (lane >> 4) * 8, c4 = (lane >> 4) * 4;
  bf16x8 bw2[2][9];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int ks = 0; ks < 9; ++ks) bw2[t][ks] = ff_frag<false>(packed, ws, P2F_OFF + ((2 * wn + t) * 9 + ks) * 512, lane);
  f32x4 bv2[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) bv2[t][i] = b2[(2 * wn + t) * 16 + c4 + i];
  int base2[4], opos2[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    opos2[mt] = c2f_tile_pos[(4 * wm + mt) * 16 + r16];
    const int mm = opos2[mt] == 255 ? 0 : opos2[mt];
    base2[mt] = (mm / 11) * 13 + mm % 11;
  }
  // zero ring of the input copies and the never-written code columns (px 13..15), once
  for (int i = tid; i < FF_XS / 16; i += 256) reinterpret_cast<bf16x8*>(XS)[i] = zero_bf16x8();
  for (int i = tid; i < C1I_IMG / 16; i += 256) reinterpret_cast<uint4*>(CT)[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();  // [S0a] zeroing before the first input store
  uint32_t pu = 0;
  float4 pf = make_float4(0.f, 0.f, 0.f, 0.f);
  if (b0 < B) {
    c1_load<U8>(xin, b0, tid, pu, pf);
    c1_store<U8, 8, XC_W, C1F_CS>(XS, tid, pu, pf, mean, inv_std, in_scale);
  }
  __syncthreads();  // [S0b] first input staged
  for (int s = 0; s < nsteps; ++s) {
    const int b = b0 + s * bstep;
    const bool live = b < B;
    const int nb = b + bstep;
    FF_ST(0);
    if (prio & 2) __builtin_amdgcn_s_setprio(1);
    // ---------------- phase 1: conv1 -> X2 / CT
    if (live) {
      if (nb < B) c1_load<U8>(xin, nb, tid, pu, pf);
      auto epilogue = [&](int j, const f32x4& c0, const f32x4& c1) {
        uint32_t g0, g1;
        const uint32_t v0 = pool4_key(c0, g0), v1 = pool4_key(c1, g1);
        const bf16x2v pv = __builtin_convertvector(f32x2v{__uint_as_float(v0), __uint_as_float(v1)}, bf16x2v);
        X2u[(4 * (wave + 4 * j) + gq) * (C2_XRS / 2) + r16] = __builtin_bit_cast(uint32_t, pv);
        CT[coff[j]] = (uint8_t)(g0 | (g1 << 4));
      };
      f32x4 p0 = zero_f32x4(), p1 = zero_f32x4();
#pragma unroll
      for (int j = 0; j < C1F_MT; ++j) {
        f32x4 c0 = bias0v, c1 = bias1v;
        const bool lv = j < C1F_MT - 1 || wave < 3;
        if (lv) {
          const bf16* xr = XS + aoff[j];
          const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(xr);
          const bf16x8 a1v = *reinterpret_cast<const bf16x8*>(xr + (4 - gq) * XC_W);
          c0 = mfma16x16x32(a0, bw1[0][0], c0);
          c1 = mfma16x16x32(a0, bw1[1][0], c1);
          c0 = mfma16x16x32(a1v, bw1[0][1], c0);
          c1 = mfma16x16x32(a1v, bw1[1][1], c1);
        }
        if (j > 0) epilogue(j - 1, p0, p1);
        if (lv && j == C1F_MT - 1) epilogue(j, c0, c1);
        p0 = c0;
        p1 = c1;
      }
    }
    FF_ST(1);
    __syncthreads();  // [S1] X2 / CT complete, XS free
    FF_ST(2);
    // ---------------- phase 2: next input; a1 / idx1 out; conv2 -> Cs
    f32x4 acc[4][2];
    if (live) {
      if (nb < B) c1_store<U8, 8, XC_W, C1F_CS>(XS, tid, pu, pf, mean, inv_std, in_scale);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[mt][0] = acc[mt][1] = zero_f32x4();
#if RINGDP_FF_PPIPE
      // software-pipelined as the consumer's conv3 k-steps (RINGDP_FF_KPIPE)
      {
        auto a2_of = [&](int ks, int mt) {
          const int shift = (ks / 3) * 13 + ks % 3;
          return *reinterpret_cast<const bf16x8*>(X2 + (base2[mt] + shift) * C2_XRS + q8);
        };
        bf16x8 cur[4], nxt[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) cur[mt] = a2_of(0, mt);
#pragma unroll
        for (int ks = 0; ks < 9; ++ks) {
          if (ks + 1 < 9) {
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) nxt[mt] = a2_of(ks + 1, mt);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) {
            acc[mt][0] = mfma16x16x32(bw2[0][ks], cur[mt], acc[mt][0]);
            acc[mt][1] = mfma16x16x32(bw2[1][ks], cur[mt], acc[mt][1]);
          }
          __builtin_amdgcn_sched_barrier(0);
          if (ks + 1 < 9) {
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) cur[mt] = nxt[mt];
          }
        }
      }
#else
#pragma unroll
      for (int ks = 0; ks < 9; ++ks) {
        const int shift = (ks / 3) * 13 + ks % 3;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(X2 + (base2[mt] + shift) * C2_XRS + q8);
          acc[mt][0] = mfma16x16x32(bw2[0][ks], a, acc[mt][0]);
          acc[mt][1] = mfma16x16x32(bw2[1][ks], a, acc[mt][1]);
        }
      }
#endif
      // a1 / idx1 to HBM while the MFMAs drain
      uint4* og = reinterpret_cast<uint4*>(a1 + (int64_t)b * C1A_IMG);
      for (int c = tid; c < C1A_IMG / 8; c += 256)
        og[c] = *reinterpret_cast<const uint4*>(X2 + (c >> 2) * C2_XRS + (c & 3) * 8);
      const uint4* cs = reinterpret_cast<const uint4*>(CT);
      uint4* cg = reinterpret_cast<uint4*>(idx1 + (int64_t)b * C1I_IMG);
      for (int c = tid; c < C1I_IMG / 16; c += 256) cg[c] = cs[c];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int m = opos2[mt];
        if (m < 121) {
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const f32x4 v = acc[mt][t] + bv2[t];
            *reinterpret_cast<bf16x4*>(Cs + m * C2_CRS + (2 * wn + t) * 16 + c4) =
                bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
          }
        }
      }
    }
    FF_ST(3);
    __syncthreads();  // [S2] Cs complete
    FF_ST(4);
    if (prio & 2) __builtin_amdgcn_s_setprio(0);
    // ---------------- phase 3: pool2 -> a2 / idx2 (HBM) + X3 (items [0, FF_P2_PROD); the consumer pools the rest)
#if RINGDP_FF_P2_ALL
    if (live) ff_pool2(Cs, X3 + (s & 1) * FF_X3H, a2, idx2, b, tid, 0, 800);
#else
    if (live) ff_pool2(Cs, X3 + (s & 1) * FF_X3H, a2, idx2, b, tid, 0, p2split);
#endif
    FF_ST(5);
    __syncthreads();  // [S3] X3 complete; Cs, X2, CT free
    FF_ST(6);
  }
}

// the consumer's conv3 k-steps per phase: [0, KA) beside conv1, [KA, KB) beside conv2, [KB, 18) beside pool2
#ifndef RINGDP_FF_KA
#define RINGDP_FF_KA 4
#endif
#ifndef RINGDP_FF_KB
#define RINGDP_FF_KB 11
#endif
template <bool PACK>
__device__ __forceinline__ void ff_consumer(char* smem, const bf16* __restrict__ packed, const PackSrc& ws,
                            const float* __restrict__ b3, const float* __restrict__ bfc, bf16* __restrict__ a3,
                            uint8_t* __restrict__ idx3, float* __restrict__ logits, bf16* __restrict__ a2,
                            uint8_t* __restrict__ idx2, int Bp, int B, int b0, int bstep, int nsteps,
                            unsigned* sync, int npack, int p2split, int prio) {
  bf16* X3 = reinterpret_cast<bf16*>(smem + FF_OFF_X3);
  const bf16* Cs = reinterpret_cast<const bf16*>(smem + FF_OFF_CS);
  bf16* fw = reinterpret_cast<bf16*>(smem + FF_OFF_FW);
  float* fred = reinterpret_cast<float*>(smem + FF_OFF_FR);
  const int tid = threadIdx.x - 256, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, q8 = (lane >> 4) * 8;
  if (PACK) ff_wait_packed(sync, npack);
  // fc1 in this launch unless logits == nullptr (large batches: fc1_fwd_kernel, an MFMA pass over a3, takes
  // its ~200 VALU per lane and image out of phase 1, where the producer's conv1 epilogue is VALU-bound too)
  const bool fc = logits != nullptr;
  if (fc) {
    const uint4* src = reinterpret_cast<const uint4*>(packed + PFC_OFF);
    for (int c = tid; c < C3F_FCW / 8; c += 256) reinterpret_cast<uint4*>(fw)[c] = src[c];
  }
  bf16x8 bw[2][18];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) bw[t][ks] = ff_frag<false>(packed, ws, P3F_OFF + ((2 * wave + t) * 18 + ks) * 512, lane);
  float bv[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) bv[t] = b3[32 * wave + 16 * t + r16];
  const float bn = tid < 160 ? bfc[tid >> 4] : 0.f;
  int base[4], wcol[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    base[mt] = win_pos(4 * c3f_win[4 * mt + (r16 >> 2)] + (r16 & 3), 10);
    wcol[mt] = c3f_win[4 * mt + (lane >> 4)];
  }
  __syncthreads();  // [S0a]
  __syncthreads();  // [S0b]  (fw is complete past these)
  auto fc_reduce = [&](int bb) {  // after a barrier that follows the fred writes of image bb
    if (tid < 160) {
      const int n = tid >> 4, c = tid & 15;
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) v += fred[n * 256 + c + 16 * i];
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if (c == 0) logits[(int64_t)bb * 10 + n] = v + bn;
    }
  };
  f32x4 acc[4][2];
  // conv3 k-steps [k0, k1) of the image in buffer xb
#if RINGDP_FF_KPIPE
  // software-pipelined: the next k-step's 4 A fragments are read before this k-step's 8 MFMAs (sched_barrier
  // pins the order), so each LDS read has 8 MFMAs (128 cycles) to land instead of being waited on at once
  auto a_of = [&](const bf16* xb, int ks, int mt) {
    const int tap = ks >> 1, c0 = (ks & 1) * 32;
    const int shift = (tap / 3) * 10 + tap % 3;
    return *reinterpret_cast<const bf16x8*>(xb + (base[mt] + shift) * C3F_XRS + c0 + q8);
  };
  auto mfma_ks = [&](const bf16* xb, auto k0c, auto k1c) {
    constexpr int k0 = decltype(k0c)::value, k1 = decltype(k1c)::value;
    bf16x8 cur[4], nxt[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) cur[mt] = a_of(xb, k0, mt);
#pragma unroll
    for (int ks = k0; ks < k1; ++ks) {
      if (ks + 1 < k1) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) nxt[mt] = a_of(xb, ks + 1, mt);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        acc[mt][0] = mfma16x16x32(cur[mt], bw[0][ks], acc[mt][0]);
        acc[mt][1] = mfma16x16x32(cur[mt], bw[1][ks], acc[mt][1]);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (ks + 1 < k1) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) cur[mt] = nxt[mt];
      }
    }
  };
#else
  auto mfma_ks = [&](const bf16* xb, auto k0c, auto k1c) {
#pragma unroll
    for (int ks = decltype(k0c)::value; ks < decltype(k1c)::value; ++ks) {
      const int tap = ks >> 1, c0 = (ks & 1) * 32;
      const int shift = (tap / 3) * 10 + tap % 3;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(xb + (base[mt] + shift) * C3F_XRS + c0 + q8);
        acc[mt][0] = mfma16x16x32(a, bw[0][ks], acc[mt][0]);
        acc[mt][1] = mfma16x16x32(a, bw[1][ks], acc[mt][1]);
      }
    }
  };
#endif
  // Step s: pool3 / fc1-partials epilogue of image s-2 and the first 4 k-steps of image s-1 (phase 1,
  // beside the producer's MFMA-light conv1), fc1 reduction of s-2 + k-steps 4-10 (phase 2), k-steps
  // 11-17 (phase 3, beside the producer's VALU-only pool2): the MFMA pipe has work in every phase.
  for (int s = 0; s < nsteps; ++s) {
    const int bm = b0 + (s - 1) * bstep, be = bm - bstep;
    const bool live_m = s >= 1 && bm < B, live_e = s >= 2 && be < B;
    const bf16* xb = X3 + ((s - 1) & 1) * FF_X3H;
    FF_ST(0);
    // ---------------- phase 1
    if (live_e) {
      float part[10];
#pragma unroll
      for (int n = 0; n < 10; ++n) part[n] = 0.f;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int wc = wcol[mt], co = 32 * wave + 16 * t + r16;
          int g;
          const bf16 pb = (bf16)pool4(acc[mt][t], bv[t], g);
          const int64_t o = ((int64_t)be * 16 + wc) * 128 + co;
          a3[o] = pb;
          idx3[o] = (uint8_t)g;
          if (!fc) continue;
          const float pv = (float)pb;
          const uint32_t* wp = reinterpret_cast<const uint32_t*>(fw + (wc * 128 + co) * 10);
#pragma unroll
          for (int h = 0; h < 5; ++h) {
            const uint32_t u = wp[h];
            part[2 * h] = fmaf(pv, __uint_as_float(u << 16), part[2 * h]);
            part[2 * h + 1] = fmaf(pv, __uint_as_float(u & 0xffff0000u), part[2 * h + 1]);
          }
        }
      if (fc) {
#pragma unroll
        for (int n = 0; n < 10; ++n) fred[n * 256 + tid] = part[n];
      }
    }
    if (live_m) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[mt][0] = acc[mt][1] = zero_f32x4();
      mfma_ks(xb, std::integral_constant<int, 0>{}, std::integral_constant<int, RINGDP_FF_KA>{});
    }
    FF_ST(1);
    __syncthreads();  // [S1]
    FF_ST(2);
    // ---------------- phase 2
    if (live_e && fc) fc_reduce(be);
    if (live_m) mfma_ks(xb, std::integral_constant<int, RINGDP_FF_KA>{}, std::integral_constant<int, RINGDP_FF_KB>{});
    FF_ST(3);
    __syncthreads();  // [S2]
    FF_ST(4);
    // ---------------- phase 3: the rest of the producer's pool2 (image s), k-steps 11-17
    // phase 3 is the consumer's (fwd_stamps.md): win the SIMD's issue arbitration against the older producer wave
    if (prio & 1) __builtin_amdgcn_s_setprio(1);
#if !RINGDP_FF_P2_ALL
    {
      const int bpr = b0 + s * bstep;
      if (bpr < Bp) ff_pool2(Cs, X3 + (s & 1) * FF_X3H, a2, idx2, bpr, tid, p2split, 800);
    }
#endif
    if (live_m) mfma_ks(xb, std::integral_constant<int, RINGDP_FF_KB>{}, std::integral_constant<int, 18>{});
    FF_ST(5);
    __syncthreads();  // [S3]
    FF_ST(6);
    if (prio & 1) __builtin_amdgcn_s_setprio(0);
  }
}

template <bool U8, bool PACK>
__global__ __launch_bounds__(512, 1) void fused_fwd_kernel(const void* __restrict__ xin,
                                                          const bf16* __restrict__ packed, PackSrc ws,
                                                          bf16* __restrict__ pack_out, int conv_blocks,
                                                          const float* __restrict__ b1, const float* __restrict__ b2,
                                                          const float* __restrict__ b3, const float* __restrict__ bfc,
                                                          bf16* __restrict__ a1, uint8_t* __restrict__ idx1,
                                                          bf16* __restrict__ a2, uint8_t* __restrict__ idx2,
                                                          bf16* __restrict__ a3, uint8_t* __restrict__ idx3,
                                                          float* __restrict__ logits, int B, float mean,
                                                          float inv_std, float in_scale, int ablate,
                                                          unsigned* sync, int p2split) {
  const int npack = (int)gridDim.x - conv_blocks;
  if (PACK && (int)blockIdx.x >= conv_blocks) {
    if (threadIdx.x < 256) pack_range(ws, pack_out, 0, blockIdx.x - conv_blocks, npack);
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(sync, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  __shared__ __attribute__((aligned(16))) char ff_smem[FF_LDS + FF_ST_BYTES];
  const int b0 = blockIdx.x, bstep = conv_blocks;
  const int nimg = b0 < B ? (B - b0 + bstep - 1) / bstep : 0;
  const int nsteps = nimg + 2;  // the consumer's MFMAs trail by one step, its epilogue by two
  // wave-uniform role split (an SGPR condition: the two roles are separate code paths, not one
  // exec-masked sequence whose live ranges the register allocator would have to overlap)
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) < 4)
    ff_producer<U8, PACK>(ff_smem, xin, PACK ? pack_out : packed, ws, b1, b2, a1, idx1, a2, idx2,
                          (ablate & 1) ? 0 : B, b0, bstep, nsteps, mean, inv_std, in_scale, sync, npack, p2split,
                          __builtin_amdgcn_readfirstlane(ablate >> 4));
  else
    ff_consumer<PACK>(ff_smem, PACK ? pack_out : packed, ws, b3, bfc, a3, idx3, logits, a2, idx2,
                      (ablate & 1) ? 0 : B, (ablate & 2) ? 0 : B, b0, bstep, nsteps, sync, npack, p2split,
                      __builtin_amdgcn_readfirstlane(ablate >> 4));
#ifdef RINGDP_FF_STAMPS
  __syncthreads();
  if (blockIdx.x == FF_ST_BLK && threadIdx.x == 0 && nsteps > FF_ST_S0 + 8) {
    const unsigned long long* st = reinterpret_cast<const unsigned long long*>(ff_smem + FF_LDS);
    for (int w = 0; w < 8; ++w)
      for (int k = 0; k < 8; ++k) {
        const unsigned long long* r = st + (w * 8 + k) * 8;
        const unsigned long long t0 = st[k * 8];  // wave 0's step start
        printf("FFST w%d s%d %lld %lld %lld %lld %lld %lld %lld\n", w, k, (long long)(r[0] - t0),
               (long long)(r[1] - t0), (long long)(r[2] - t0), (long long)(r[3] - t0), (long long)(r[4] - t0),
               (long long)(r[5] - t0), (long long)(r[6] - t0));
      }
  }
#endif
  if (PACK) {  // the last conv workgroup out re-arms the counters
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned t = __hip_atomic_fetch_add(sync + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (t == (unsigned)conv_blocks - 1) {
        __hip_atomic_store(sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(sync + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// ================================================================== F3 backward
// (1) fc1 backward, one pass over a3: compact data gradient
//       da3m[b][w][co] = (a3 > 0) * sum_n dl[b][n] * Wfc[n][co*16 + w]     (bf16, Wfc from the pack)
//     and the fc1 weight/bias gradient of this block's images as an fp32 slab.  The conv3 backward
//     roles expand da3m to window-ordered rows (row 4w + argmax) in LDS.
// images per workgroup: enough workgroups to fill the chip at small batches (B=100: 25 of 4 images,
// was 4 of 32 and latency-bound at 21 us), fewer fp32 slabs at large ones (B=32768: 512 of 64 images,
// halving the 84 MB of slab traffic)
__host__ __device__ inline int fc_imgs(int B) { return B <= 1024 ? 4 : (B >= 65536 ? 128 : (B >= 32768 ? 64 : 32)); }
constexpr int FC_SLAB = 10 * 2048 + 10 + 128 + 2;  // dWfc + dbfc + db3 (the conv3 bias gradient is the sum
                                                    // of d(a3) over windows: no MFMA tile needed for it),
                                                    // padded to a 16-B multiple (vector slab reduction)

// kCE: the logits gradient is formed here from the cross-entropy forward's logits / log-sum-exp
// (same expression as ce_bwd_kernel, elementwise.hip) - 80 threads per group of 8 images into LDS -
// instead of read from a [B,10] tensor: the separate ce_bwd launch disappears.
// The body runs as its own launch (fc_bwd_kernel) or as the first workgroups of the conv3 backward launch at
// small batches (conv3_bwd_kernel<true>, blk = that workgroup's fc index; da3m == nullptr: the conv3
// roles form their own compact gradient, C3Pre::load).
template <bool kCE>
__device__ __forceinline__ void fc_bwd_body(const bf16* __restrict__ a3, const bf16* __restrict__ packed,
                                            const float* __restrict__ dl, bf16* __restrict__ da3m,
                                            float* __restrict__ slabs, int B, int imgs, const CeFuse& ce, int blk) {
  const int t = threadIdx.x;
  const int wd = t >> 4, co0 = (t & 15) * 8;  // this thread's 8 activations: window wd, channels co0..
  float wr[8][10];
  {
    // Pfc is [w][co][n]: this thread's 80 weights are contiguous (10 x 16 B)
    const bf16x8* src = reinterpret_cast<const bf16x8*>(packed + PFC_OFF + (wd * 128 + co0) * 10);
#pragma unroll
    for (int h = 0; h < 10; ++h) {
      const bf16x8 v = src[h];
#pragma unroll
      for (int e = 0; e < 8; ++e) wr[(8 * h + e) / 10][(8 * h + e) % 10] = (float)v[e];
    }
  }
  float acc[8][10];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int n = 0; n < 10; ++n) acc[j][n] = 0.f;
  float bacc = 0.f, dsum[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) dsum[j] = 0.f;
  const int b0 = blk * imgs, nimg = min(imgs, B - b0);
  // kCE: the logits gradient of all this block's images (<= 128 x 10) formed once into LDS, one barrier
  __shared__ float gl[128 * 10];
  if constexpr (kCE) {
    const float ce_scale = ce.reduction == 0 ? 1.f : ce.grad_out[0] / ce.denom[0];
    for (int e = t; e < nimg * 10; e += 256) {
      const int k = e / 10, n = e - 10 * k, b = b0 + k;
      float g = 0.f;
      const int64_t y = ce.labels[b];
      if (y != ce.ignore_index) {
        const float p = __expf(ce.logits[(int64_t)b * 10 + n] - ce.lse[b]);
        const float q = (n == y ? (1.f - ce.eps) : 0.f) + ce.eps / 10.f;
        g = (p - q) * (ce.reduction == 0 ? ce.grad_out[b] : ce_scale);
      }
      gl[e] = g;
    }
    __syncthreads();
  }
  for (int k0 = 0; k0 < nimg; k0 += 8) {
    bf16x8 av[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (k0 + k < nimg) av[k] = *reinterpret_cast<const bf16x8*>(a3 + (int64_t)(b0 + k0 + k) * 2048 + wd * 128 + co0);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k0 + k < nimg) {
        const int b = b0 + k0 + k;
        float g[10];
#pragma unroll
        for (int n = 0; n < 10; ++n) g[n] = kCE ? gl[(k0 + k) * 10 + n] : dl[(int64_t)b * 10 + n];
        bf16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float aj = (float)av[k][j];
          float s = 0.f;
#pragma unroll
          for (int n = 0; n < 10; ++n) {
            s = fmaf(g[n], wr[j][n], s);
            acc[j][n] = fmaf(g[n], aj, acc[j][n]);
          }
          const float m = aj > 0.f ? s : 0.f;
          dsum[j] += m;
          v[j] = (bf16)m;
        }
        if (da3m) *reinterpret_cast<bf16x8*>(da3m + (int64_t)b * 2048 + wd * 128 + co0) = v;
        if (t < 10) bacc += kCE ? gl[(k0 + k) * 10 + t] : dl[(int64_t)b * 10 + t];
      }
    }
  }
  // slab in thread order (coalesced): element (n*8 + j)*256 + t; the reduction (mode 2) maps it back
  // to dWfc[n][co*16 + w]
  float* slab = slabs + (int64_t)blk * FC_SLAB;
#pragma unroll
  for (int n = 0; n < 10; ++n)
#pragma unroll
    for (int j = 0; j < 8; ++j) slab[(n * 8 + j) * 256 + t] = acc[j][n];
  if (t < 10) slab[20480 + t] = bacc;
  // db3 partial: sum the 16 windows (4 per wave via lane shuffles, then the 4 waves) per channel
  __shared__ float red[4][128];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float v = dsum[j];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    dsum[j] = v;
  }
  if ((t & 63) < 16) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[t >> 6][co0 + j] = dsum[j];
  }
  __syncthreads();
  if (t < 128) slab[20490 + t] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
}

template <bool kCE>
__global__ __launch_bounds__(256) void fc_bwd_kernel(const bf16* __restrict__ a3, const bf16* __restrict__ packed,
                                                     const float* __restrict__ dl, bf16* __restrict__ da3m,
                                                     float* __restrict__ slabs, int B, int imgs, CeFuse ce) {
  fc_bwd_body<kCE>(a3, packed, dl, da3m, slabs, B, imgs, ce, blockIdx.x);
}

// (2) conv3 backward, two roles in one launch of 256-thread workgroups, two per CU (a CU usually
//     hosts one of each, so one role's barrier-separated phases overlap the other's MFMA stream):
//   dgrad: da2 = full-corr(d(conv3) image, flipped W3), then pool2 + ReLU backward: each da2 value goes
//          to the z2 position its pool2 code names (F2 forward) -> dz2 [B,11,11,64];
//   wgrad: dW3t[n = tap*64 + ci][co] = sum_k D3[k][co] * a2[pos(k) + tap][ci], a workgroup pair per
//          image slice (one half of the 576 n columns each).  db3 comes from fc1's backward.
// d(conv3) image in LDS with two zero rows above and below (12 rows x 8 columns): position (Y, X) at
// Y*C3_PY + X*C3_PX bf16.  288-B positions and unpadded 2304-B rows make every B-fragment read of the
// dgrad GEMM (lanes = 2 rows x 8 columns of one 16-B channel chunk) conflict-free: 4 LDS cycles per
// ds_read_b128 (tools/lds_bank_model.py; the 12x12 ring layout with 3648-B rows read these in 8).
constexpr int C3_PX = 144;   // bf16 per position (128 + 16)
constexpr int C3_PY = 1152;  // bf16 per row of positions (8 * 144)
constexpr int C3_DARS = 68;  // floats per da2 row (64 + 4)
constexpr int C3_DRS = 136;  // bf16 per D3 row in LDS
constexpr int C3D_P = 12 * C3_PY * 2;                       // 27648
constexpr int C3D_AM = 100 * 64;                            // 6400: pool2 codes of the current image
constexpr int C3D_DA = 100 * C3_DARS * 4;                   // 27200
constexpr int C3D_LDS = C3D_P + C3D_AM + C3D_DA;
static_assert(C3D_P % 16 == 0 && C3D_LDS <= 81920, "two conv3 backward workgroups per CU");
constexpr int C3W_D = 64 * C3_DRS * 2;   // 17408
constexpr int C3W_X = 100 * C3_XRS * 2;  // 14400
constexpr int C3W_R = 100 * 64 * 2;      // 12800: DMA staging of the next a2 image
constexpr int C3W_LDS = C3W_D + C3W_X + C3W_R;
constexpr int C3B_LDS = C3D_LDS > C3W_LDS ? C3D_LDS : C3W_LDS;
constexpr int C3_WSLAB = 576 * 128;  // dW3t

// The compact F3-backward input of one image, held in registers while the previous image is
// computed on: d(a3) chunk + its pool3 argmax bytes (threads < 256).
// Where the conv3 backward roles get an image's compact d(a3): the fc1 backward launch's da3m, or (small
// batches, fc1 backward inside this launch) computed in place from a3, the logits gradient and the packed
// fc1 weights - the same expression and order as fc_bwd_body, so the values are bit-identical.
struct C3Src {
  const bf16* da3m;  // null: compute
  const bf16* a3;
  const bf16* packed;
  const float* dl;   // logits gradient, or null with ce
  CeFuse ce;
};

struct C3Pre {
  bf16x8 da;
  uint2 id;
  template <bool kFC>
  __device__ __forceinline__ void load(const C3Src& src, const uint8_t* __restrict__ idx3, int b, int tid) {
    if (tid < 256) {
      id = reinterpret_cast<const uint2*>(idx3 + (int64_t)b * 2048)[tid];
      if (!kFC) {
        da = reinterpret_cast<const bf16x8*>(src.da3m + (int64_t)b * 2048)[tid];
        return;
      }
      const int wd = tid >> 4, co0 = (tid & 15) * 8;
      const bf16x8 av = reinterpret_cast<const bf16x8*>(src.a3 + (int64_t)b * 2048)[tid];
      float g[10];
      if (src.dl) {
#pragma unroll
        for (int n = 0; n < 10; ++n) g[n] = src.dl[(int64_t)b * 10 + n];
      } else {
        const CeFuse& ce = src.ce;
        const int64_t y = ce.labels[b];
        const float sc = ce.reduction == 0 ? ce.grad_out[b] : ce.grad_out[0] / ce.denom[0];
        const float lse = ce.lse[b];
#pragma unroll
        for (int n = 0; n < 10; ++n) {
          float gv = 0.f;
          if (y != ce.ignore_index) {
            const float p = __expf(ce.logits[(int64_t)b * 10 + n] - lse);
            const float q = (n == y ? (1.f - ce.eps) : 0.f) + ce.eps / 10.f;
            gv = (p - q) * sc;
          }
          g[n] = gv;
        }
      }
      const bf16x8* wsrc = reinterpret_cast<const bf16x8*>(src.packed + PFC_OFF + (wd * 128 + co0) * 10);
      bf16x8 wv[10];
#pragma unroll
      for (int h = 0; h < 10; ++h) wv[h] = wsrc[h];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float s = 0.f;
#pragma unroll
        for (int n = 0; n < 10; ++n) s = fmaf(g[n], (float)wv[(10 * j + n) / 8][(10 * j + n) % 8], s);
        da[j] = (bf16)((float)av[j] > 0.f ? s : 0.f);
      }
    }
  }
};

// Rows 0..3 of one channel pair: d = bf16 pair (channel 2k low, 2k+1 high), t = their pool3 argmax
// (0..3) in bits 0-1 of each halfword; row i keeps a channel iff its argmax == i.  The argmax bit planes
// become halfword sign masks (two packed shifts each) and every row is one v_bitop3 - 9 VALU per 8
// outputs instead of a compare + select per output.
typedef short s16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void c3_rows(uint32_t d, uint32_t t, uint32_t& r0, uint32_t& r1, uint32_t& r2,
                                        uint32_t& r3) {
  const s16x2v ts = __builtin_bit_cast(s16x2v, t);
  const uint32_t a0 = __builtin_bit_cast(uint32_t, (s16x2v)(ts << 15) >> 15);  // halfword = -(argmax bit 0)
  const uint32_t a1 = __builtin_bit_cast(uint32_t, (s16x2v)(ts << 14) >> 15);  // halfword = -(argmax bit 1)
  // v_bitop3 truth-table index = (S0 << 2) | (S1 << 1) | S2 with S0 = d, S1 = a0, S2 = a1
  r0 = __builtin_amdgcn_bitop3_b32(d, a0, a1, 0x10);  // d & ~a0 & ~a1
  r1 = __builtin_amdgcn_bitop3_b32(d, a0, a1, 0x40);  // d &  a0 & ~a1
  r2 = __builtin_amdgcn_bitop3_b32(d, a0, a1, 0x20);  // d & ~a0 &  a1
  r3 = __builtin_amdgcn_bitop3_b32(d, a0, a1, 0x80);  // d &  a0 &  a1
}

// Expand compact item tid (window w = tid >> 4, channels cc..cc+7) to the 4 window-ordered rows.
template <typename RowPtr>
__device__ __forceinline__ void c3_expand(const C3Pre& p, int tid, RowPtr row_ptr) {
  if (tid < 256) {
    const int w = tid >> 4, cc = (tid & 15) * 8;
    const uint4 dv = __builtin_bit_cast(uint4, p.da);
    const uint32_t dw[4] = {dv.x, dv.y, dv.z, dv.w};
    uint32_t r[4][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      // argmax bytes 2k, 2k+1 -> the low bytes of the two halfwords
      const uint32_t id4 = k < 2 ? p.id.x : p.id.y;
      const uint32_t t = __builtin_amdgcn_perm(id4, id4, (k & 1) ? 0x0c030c02u : 0x0c010c00u);
      c3_rows(dw[k], t, r[0][k], r[1][k], r[2][k], r[3][k]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *reinterpret_cast<uint4*>(row_ptr(4 * w + i) + cc) = make_uint4(r[i][0], r[i][1], r[i][2], r[i][3]);
  }
}

// pool2 codes of one image (6400 B = 400 x 16 B) -> LDS by DMA (4 waves, 7 wave-instructions)
__device__ __forceinline__ void codes_glds(const uint8_t* __restrict__ idx2, int b, uint8_t* AM, int wave,
                                           int lane) {
  const uint8_t* src = idx2 + (int64_t)b * 6400;
  for (int k = wave; k < 7; k += 4) {
    const int slot = k * 64 + lane;
    if (slot < 400) glds16_async(src + slot * 16, AM + k * 1024);
  }
}

// dgrad per image, gathered over kernel rows and scattered over kernel columns:
//   da2[y'][x + kx][ci] += sum_{ky, co} W3[co][ci][ky][kx] * dz3[y' - ky][x][co]
// over the 8 dz3 columns x and the 10 da2 rows y', K = 128 output channels (the full correlation over
// the 10x10 a2 image with the 3x3 flipped kernel needed 252 MFMAs per wave: 900 (position, tap) pairs
// of which only 576 are non-zero; the pure scatter form 144 plus a col2im read-add-write per tap).
// Operands are swapped so a lane's 4 results are 4 consecutive input channels of one position: wave w
// owns input channels 16w..16w+15, so its col2im into the fp32 da2 image never meets another wave's.
// The kx taps of an m-tile hit the same da2 words from different lanes, so a compiler barrier keeps
// each read behind the previous write (LDS executes one wave's instructions in order).  Fixed order:
// deterministic.
template <bool kFC>
__device__ __forceinline__ void conv3_dgrad_role(char* smem, const C3Src& src, const uint8_t* __restrict__ idx3,
                                 const uint8_t* __restrict__ idx2, const bf16* __restrict__ packed,
                                 bf16* __restrict__ dz2, int b_first, int b_end, int b_step) {
  bf16* P = reinterpret_cast<bf16*>(smem);
  uint8_t* AM = reinterpret_cast<uint8_t*>(smem + C3D_P);
  float* DA = reinterpret_cast<float*>(smem + C3D_P + C3D_AM);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, q8 = (lane >> 4) * 8, c4 = (lane >> 4) * 4;
  const bf16x8* pk = reinterpret_cast<const bf16x8*>(packed + P3D_OFF);
  bf16x8 aw[36];  // [tap][kstep] weight fragments of this wave's 16 input channels
#pragma unroll
  for (int j = 0; j < 36; ++j) aw[j] = pk[(wave * 36 + j) * 64 + lane];
  // lane r16 of m-tile mt: da2 row 2 mt + (r16 >> 3), dz3 column r16 & 7 (its kx = 0 da2 column)
  const int pbase = ((r16 >> 3) + 2) * C3_PY + (r16 & 7) * C3_PX + q8;
  const int dbase = ((r16 >> 3) * 10 + (r16 & 7)) * C3_DARS + 16 * wave + c4;
  // the zero rows of the image stay zero; only the 8x8 interior is rewritten per image
  for (int c = tid; c < C3D_P / 16; c += 256) reinterpret_cast<bf16x8*>(P)[c] = zero_bf16x8();
  // Gather over the kernel row ky, scatter over the kernel column kx.  Output m-tile mt = da2 rows
  // 2mt, 2mt+1 at the 8 dz3 columns x: for each ky the B fragments are the dz3 rows y' - ky (a row
  // offset into the zero-ringed image), and the three kx taps accumulate in three register tiles that
  // land on da2 columns x, x+1, x+2.  13 (mt, ky) pairs hold a non-zero row (mt 0 has no ky 2, mt 4
  // no ky 0): 156 MFMAs per wave (pure scatter: 144), but the fp32 col2im is one store + two
  // read-add-writes per m-tile (15 + 10 per wave) instead of a read-add-write per tap (72 + 72): the
  // 13-cycle ds_write_b128 traffic of that col2im had been as long as the MFMA stream itself.
  const int xcol = r16 & 7;
  auto mfma_phase = [&]() {
#pragma unroll
    for (int mt = 0; mt < 5; ++mt) {
      f32x4 acc[3] = {zero_f32x4(), zero_f32x4(), zero_f32x4()};
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        if ((mt == 0 && ky == 2) || (mt == 4 && ky == 0)) continue;  // both rows in the zero ring
        bf16x8 bfr[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          bfr[ks] = *reinterpret_cast<const bf16x8*>(P + pbase + (2 * mt - ky) * C3_PY + ks * 32);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) acc[kx] = mfma16x16x32(aw[(3 * ky + kx) * 4 + ks], bfr[ks], acc[kx]);
      }
      // da2 column x + kx; the lanes of column 7 open columns 8 (kx 1) and 9 (kx 2), which no earlier
      // tap of this image wrote: they add to zero instead of the previous image's value
      f32x4* d = reinterpret_cast<f32x4*>(DA + dbase + 20 * mt * C3_DARS);
      *d = acc[0];
#pragma unroll
      for (int kx = 1; kx < 3; ++kx) {
        asm volatile("" ::: "memory");  // the read below stays behind the other lanes' write above
        f32x4 old = d[kx * (C3_DARS / 4)];
        if (xcol == 7) old = zero_f32x4();
        d[kx * (C3_DARS / 4)] = old + acc[kx];
      }
    }
  };
  // pool2 + ReLU backward, one item per (output row y, channel quad), sliding along x: window (py, px)
  // covers outputs (py..py+1, px..px+1) and its one-hot code bit dy*2+dx names the one that receives
  // its gradient, so output (y, x) sums, in a fixed order, the windows (y, x), (y, x-1), (y-1, x),
  // (y-1, x-1) masked by code bits 0, 1, 2, 3.  Each window of a row is loaded once per item and used
  // for x and x+1; a missing window row (y = 0 or 10) reads a valid one under a mask of bit 4 (never set).
  const int gy = tid >> 4, gq = (tid & 15) * 4;
  const int rowA = min(gy, 9), rowB = max(gy - 1, 0);  // dy = 0 and dy = 1 window rows
  const int sA = gy <= 9 ? 0 : 4, sB = gy >= 1 ? 2 : 4;
  auto masked_add = [](f32x4& g, uint32_t cw, int sh, const f32x4& d) {
    const uint32_t m = (cw >> sh) & 0x01010101u;  // byte j = 1 iff channel j's window picked this output
#pragma unroll
    for (int j = 0; j < 4; ++j) g[j] = fmaf(d[j], (float)((m >> (8 * j)) & 0xffu), g[j]);
  };
  C3Pre pre;
  int b = b_first;
  if (b < b_end) pre.template load<kFC>(src, idx3, b, tid);
  for (; b < b_end; b += b_step) {
    __syncthreads();  // previous image fully consumed (P, DA, AM)
    c3_expand(pre, tid, [&](int r) {
      const int w = r >> 2, i = r & 3;
      return P + (2 * (w >> 2) + (i >> 1) + 2) * C3_PY + (2 * (w & 3) + (i & 1)) * C3_PX;
    });
    codes_glds(idx2, b, AM, wave, lane);  // this image's codes land during the MFMA phase
    const int nb = b + b_step;
    if (nb < b_end) pre.template load<kFC>(src, idx3, nb, tid);
    __syncthreads();
    mfma_phase();
    c_dma_wait();
    __syncthreads();
    if (tid < 176) {
      const uint32_t* cA = reinterpret_cast<const uint32_t*>(AM + rowA * 640 + gq);
      const uint32_t* cB = reinterpret_cast<const uint32_t*>(AM + rowB * 640 + gq);
      const f32x4* dA = reinterpret_cast<const f32x4*>(DA + rowA * 10 * C3_DARS + gq);
      const f32x4* dB = reinterpret_cast<const f32x4*>(DA + rowB * 10 * C3_DARS + gq);
      bf16x4* dst = reinterpret_cast<bf16x4*>(dz2 + ((int64_t)b * 121 + gy * 11) * 64 + gq);
      uint32_t pa = 0, pb = 0;  // window (., x-1)
      f32x4 qa = zero_f32x4(), qb = zero_f32x4();
#pragma unroll
      for (int x = 0; x < 11; ++x) {
        uint32_t na = 0, nb2 = 0;
        f32x4 ea = zero_f32x4(), eb = zero_f32x4();
        if (x < 10) {
          na = cA[x * 16];
          nb2 = cB[x * 16];
          ea = dA[x * (C3_DARS / 4)];
          eb = dB[x * (C3_DARS / 4)];
        }
        f32x4 g = zero_f32x4();
        if (x < 10) masked_add(g, na, sA, ea);
        if (x > 0) masked_add(g, pa, sA + 1, qa);
        if (x < 10) masked_add(g, nb2, sB, eb);
        if (x > 0) masked_add(g, pb, sB + 1, qb);
        dst[x * 16] = bf16x4{(bf16)g[0], (bf16)g[1], (bf16)g[2], (bf16)g[3]};
        pa = na;
        pb = nb2;
        qa = ea;
        qb = eb;
      }
    }
  }
}

// wgrad: workgroup half h of an image slice covers n-tiles 18h..18h+17 of dW3t [576][128];
// wave (wm, wn) owns m-tiles (co) 4wm..4wm+3 x n-tiles 18h + 9wn .. +8.
template <bool kFC>
__device__ __forceinline__ void conv3_wgrad_role(char* smem, const bf16* __restrict__ a2, const C3Src& src,
                                 const uint8_t* __restrict__ idx3, float* __restrict__ slabs, int B,
                                 int nslices, int slice, int h) {
  bf16* D = reinterpret_cast<bf16*>(smem);
  bf16* X = reinterpret_cast<bf16*>(smem + C3W_D);
  bf16* R = reinterpret_cast<bf16*>(smem + C3W_D + C3W_X);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int nt0 = 18 * h + 9 * wn;
  const int g16 = lane & 15, grp = lane >> 4, q = g16 >> 2, p = g16 & 3;
  f32x4 acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = zero_f32x4();
  const int per = cdiv(B, nslices);
  const int b_lo = slice * per, b_hi = min(B, b_lo + per);
  C3Pre pre;
  if (b_lo < b_hi) {
    pre.template load<kFC>(src, idx3, b_lo, tid);
    a2_glds(a2, b_lo, R, wave, lane, 4);
  }
  for (int b = b_lo; b < b_hi; ++b) {
    c_dma_wait();
    __syncthreads();  // R has landed; the previous image's D / X reads are done
    c3_expand(pre, tid, [&](int r) { return D + r * C3_DRS; });
    a2_relayout(R, X, tid, 256);
    __syncthreads();  // D, X complete; R free
    if (b + 1 < b_hi) {  // lands during the MFMAs
      pre.template load<kFC>(src, idx3, b + 1, tid);
      a2_glds(a2, b + 1, R, wave, lane, 4);
    }
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
        const int n0 = (nt0 + j) * 16;  // n = tap*64 + ci
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
  for (int i = 0; i < 4; ++i) {
    const int co = (4 * wm + i) * 16 + grp * 4;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int n = (nt0 + j) * 16 + g16;
      *reinterpret_cast<f32x4*>(slab + (int64_t)n * 128 + co) = acc[i][j];
    }
  }
}

// kFC (small batches): workgroups [0, n_fc) run the fc1 backward (weight / bias gradient slabs only) and the
// conv3 roles form each image's compact gradient themselves (C3Src without da3m): the fc1 backward launch
// disappears.  One workgroup per CU then (the compact-gradient load holds the fc1 weights in registers).
template <bool kFC>
__global__ __launch_bounds__(256, kFC ? 1 : 2) void conv3_bwd_kernel(const bf16* __restrict__ a2,
                                                                     const uint8_t* __restrict__ idx2, C3Src src,
                                                                     const uint8_t* __restrict__ idx3,
                                                                     const bf16* __restrict__ packed,
                                                                     bf16* __restrict__ dz2, int B,
                                                                     float* __restrict__ slabs, int n_wgrad,
                                                                     int n_dgrad, int b_dgrad, int n_fc,
                                                                     float* __restrict__ fc_slabs, int fc_n_imgs) {
  __shared__ __attribute__((aligned(16))) char smem[C3B_LDS];
  int blk = blockIdx.x;
  if (kFC) {
    if (blk < n_fc) {
      if (src.dl)
        fc_bwd_body<false>(src.a3, packed, src.dl, nullptr, fc_slabs, B, fc_n_imgs, src.ce, blk);
      else
        fc_bwd_body<true>(src.a3, packed, nullptr, nullptr, fc_slabs, B, fc_n_imgs, src.ce, blk);
      return;
    }
    blk -= n_fc;
  }
  int b_first = blk, b_end = b_dgrad, b_step = n_dgrad;
  if (blk >= n_dgrad) {
    const int w = blk - n_dgrad;
    conv3_wgrad_role<kFC>(smem, a2, src, idx3, slabs, B, n_wgrad, w >> 1, w & 1);
    // images [b_dgrad, B) of the data gradient go to the wgrad workgroups once their slice is done: a
    // dgrad workgroup is slower per image than its wgrad neighbour (pool2 backward, barrier phases), so
    // with one of each per CU the wgrad half would otherwise idle (static split: deterministic)
    if (dz2 == nullptr || b_dgrad >= B) return;
    __syncthreads();  // LDS changes role
    b_first = b_dgrad + w;
    b_end = B;
    b_step = 2 * n_wgrad;
  }
  conv3_dgrad_role<kFC>(smem, src, idx3, idx2, packed, dz2, b_first, b_end, b_step);  // one call site: inlined
}

// ---- conv3 backward with 8-wave workgroups (batches above fc_in_c3_max_batch: the fc1 backward launch
// leaves the compact gradient da3m).  One 512-thread workgroup per CU, in one of two roles:
//   dgrad, wave-specialised: waves 0-3 hold the conv3 weights and only run image s's dgrad MFMAs and
//     col2im (P[s&1] -> DA[s&1]); beside them waves 4-7 run the pool2 + ReLU backward of image s-1
//     (DA, codes -> dz2), expand image s+1's compact gradient (stage -> P) and issue the LDS-DMA of
//     later images.  One barrier per image: every buffer is written in one step and read in the next,
//     so P, DA, the codes and the compact stage are double-buffered.  The 4-wave role above ran these
//     phases one after the other, each behind a barrier of all four waves.
//   wgrad: 8 waves cover the whole 128 x 576 dW3t of their image slice (36 tiles each, 2 x 4 waves), so
//     an image is staged once (the 4-wave role needs a workgroup pair, each staging every image); image
//     i+1's operands (compact gradient -> D, a2 -> X by LDS-DMA straight into the padded rows) are staged
//     while image i's MFMAs run.
// All global -> LDS traffic is LDS-DMA from inline asm (invisible to the compiler's vmcnt bookkeeping),
// waited for explicitly before the barrier; the dz2 stores stay in flight across it.
// LDS layouts (every fragment read, col2im access and pool2 read modelled conflict-free with the lane
// groups of MI355X_MICROARCH.md; the 4-wave kernel's layouts measured 30-46 % bank-conflict cycles):
//   da2 (fp32): 256-B position rows, the 16-B chunk k of position (y, x) at slot k ^ 2(x & 7);
//   D (wgrad): rows of 144 bf16 in blocks of 8 rows, 1216 bf16 per block (tr16 reads of rows k..k+3 and
//     k+8..k+11 then cover the 64 banks once);  X (wgrad): a2 rows of 80 bf16 (10 16-B chunks).
constexpr int C3S_B = 2048 * 2 + 2048;  // compact stage of one image: da3m row (bf16) + pool3 argmax bytes
constexpr int C3V_DA = 100 * 64 * 4;    // 25600
constexpr int C3V_D = 8 * 1216 * 2;     // 19456
constexpr int C3V_XRS = 80;
constexpr int C3V_X = 100 * C3V_XRS * 2;  // 16000
constexpr int C3V_DG = 2 * (C3D_P + C3V_DA + C3D_AM + C3S_B);  // 131584
constexpr int C3V_WG = 3 * (C3V_D + C3V_X) + 2 * C3S_B;        // 118656
constexpr int C3V_LDS = C3V_DG > C3V_WG ? C3V_DG : C3V_WG;
static_assert(C3V_LDS <= 160 * 1024 && C3V_D % 16 == 0 && C3V_X % 16 == 0, "conv3 backward (8-wave) LDS");
__device__ __forceinline__ int c3v_drow(int r) { return (r >> 3) * 1216 + (r & 7) * 144; }
// float offset of 16-B chunk k (channels 4k..4k+3) of da2 position p = y * 10 + x
__device__ __forceinline__ int c3v_da(int p, int x, int k) { return p * 64 + ((k ^ (2 * (x & 7))) << 2); }
// exact 0.0 / 1.0 of byte J of v (one v_cvt_f32_ubyteJ; the compiler's form of (v >> 8J) & 0xff was a shift,
// an and and v_cvt_f32_ubyte0 per byte)
template <int J>
__device__ __forceinline__ float ubyte_f32(uint32_t v) {
  float r;
  if constexpr (J == 0) asm("v_cvt_f32_ubyte0 %0, %1" : "=v"(r) : "v"(v));
  else if constexpr (J == 1) asm("v_cvt_f32_ubyte1 %0, %1" : "=v"(r) : "v"(v));
  else if constexpr (J == 2) asm("v_cvt_f32_ubyte2 %0, %1" : "=v"(r) : "v"(v));
  else asm("v_cvt_f32_ubyte3 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

// v shifted right by N lanes inside each 16-lane DPP row (0 into the row's first N lanes)
template <int N>
__device__ __forceinline__ float dpp_row_shr(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x110 + N, 0xf, 0xf, true));
}

// barrier for LDS hand-offs: this wave's LDS operations drained, global stores left in flight (the release
// fence of __syncthreads() would also wait for those)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// wave-instruction k (0..5) of the compact stage of image b: da3m row (4 KiB), then the argmax bytes (2 KiB)
__device__ __forceinline__ void c3s_glds(const bf16* __restrict__ da3m, const uint8_t* __restrict__ idx3, int b,
                                         char* S, int k, int lane) {
  const uint32_t voff = ((k & 3) * 64 + lane) * 16;
  if (k < 4)
    glds16_sv(da3m + (int64_t)b * 2048, voff, S + k * 1024);
  else
    glds16_sv(idx3 + (int64_t)b * 2048, voff, S + k * 1024);
}

__device__ __forceinline__ void c3s_pre(const char* S, int tid, C3Pre& p) {
  if (tid < 256) {
    p.da = reinterpret_cast<const bf16x8*>(S)[tid];
    p.id = reinterpret_cast<const uint2*>(S + 4096)[tid];
  }
}

// a2 image -> C3V_XRS rows by LDS-DMA: wave-instruction k (0..15) covers LDS chunks 64k..64k+63, 10 16-B
// chunks per row, chunks 8, 9 of a row its padding (re-reading the row's first chunks); a2_rows_off is a lane's
// byte offset in the image (or ~0u past the 100 rows), a2_glds_rows issues the copy of image b
__device__ __forceinline__ uint32_t a2_rows_off(int k, int lane) {
  const int c = k * 64 + lane;
  if (c >= 1000) return ~0u;
  const int row = c / 10, sub = c - 10 * row;
  return (row * 64 + (sub & 7) * 8) * 2;
}
__device__ __forceinline__ void a2_glds_rows(const bf16* __restrict__ a2, int b, bf16* X, int k, uint32_t voff) {
  if (voff != ~0u) glds16_sv(a2 + (int64_t)b * 6400, voff, X + k * 512);
}

// pool2 + ReLU backward of one image (threads t < 176: output row t >> 4, channel quad t & 15), as in
// conv3_dgrad_role, from the swizzled da2 image
__device__ __forceinline__ void c3_pool2_bwd(const float* DA, const uint8_t* AM, bf16* __restrict__ dz2, int b,
                                             int t) {
  const int gy = t >> 4, k = t & 15, gq = k * 4;
  const int rowA = min(gy, 9), rowB = max(gy - 1, 0);
  const int sA = gy <= 9 ? 0 : 4, sB = gy >= 1 ? 2 : 4;
  auto masked_add = [](f32x4& g, uint32_t cw, int sh, const f32x4& d) {
    const uint32_t m = (cw >> sh) & 0x01010101u;
    g[0] = fmaf(d[0], ubyte_f32<0>(m), g[0]);
    g[1] = fmaf(d[1], ubyte_f32<1>(m), g[1]);
    g[2] = fmaf(d[2], ubyte_f32<2>(m), g[2]);
    g[3] = fmaf(d[3], ubyte_f32<3>(m), g[3]);
  };
  const uint32_t* cA = reinterpret_cast<const uint32_t*>(AM + rowA * 640 + gq);
  const uint32_t* cB = reinterpret_cast<const uint32_t*>(AM + rowB * 640 + gq);
  bf16x4* dst = reinterpret_cast<bf16x4*>(dz2 + ((int64_t)b * 121 + gy * 11) * 64 + gq);
  uint32_t pa = 0, pb = 0;
  f32x4 qa = zero_f32x4(), qb = zero_f32x4();
#pragma unroll
  for (int x = 0; x < 11; ++x) {
    uint32_t na = 0, nb2 = 0;
    f32x4 ea = zero_f32x4(), eb = zero_f32x4();
    if (x < 10) {
      na = cA[x * 16];
      nb2 = cB[x * 16];
      ea = *reinterpret_cast<const f32x4*>(DA + c3v_da(rowA * 10 + x, x, k));
      eb = *reinterpret_cast<const f32x4*>(DA + c3v_da(rowB * 10 + x, x, k));
    }
    f32x4 g = zero_f32x4();
    if (x < 10) masked_add(g, na, sA, ea);
    if (x > 0) masked_add(g, pa, sA + 1, qa);
    if (x < 10) masked_add(g, nb2, sB, eb);
    if (x > 0) masked_add(g, pb, sB + 1, qb);
    dst[x * 16] = bf16x4{(bf16)g[0], (bf16)g[1], (bf16)g[2], (bf16)g[3]};
    pa = na;
    pb = nb2;
    qa = ea;
    qb = eb;
  }
}

__device__ __forceinline__ void conv3_dgrad8_role(char* smem, const bf16* __restrict__ da3m,
                                                  const uint8_t* __restrict__ idx3, const uint8_t* __restrict__ idx2,
                                                  const bf16* __restrict__ packed, bf16* __restrict__ dz2, int b_first,
                                                  int b_end, int b_step, int ablate) {
  auto Pb = [&](int k) { return reinterpret_cast<bf16*>(smem + k * C3D_P); };
  auto DAb = [&](int k) { return reinterpret_cast<float*>(smem + 2 * C3D_P + k * C3V_DA); };
  // pool2 codes of image j in AM[j & 1], issued in step j (pool2 of image j runs in step j+1)
  auto AMb = [&](int k) { return reinterpret_cast<uint8_t*>(smem + 2 * (C3D_P + C3V_DA) + k * C3D_AM); };
  auto Sb = [&](int k) { return smem + 2 * (C3D_P + C3V_DA + C3D_AM) + k * C3S_B; };
  auto codes_dma = [&](int j, int lane) {
    const uint8_t* src = idx2 + (int64_t)(b_first + j * b_step) * 6400;
    uint8_t* AM = AMb(j & 1);
#pragma unroll
    for (int k = 0; k < 7; ++k)
      if (k * 64 + lane < 400) glds16_sv(src, (k * 64 + lane) * 16, AM + k * 1024);
  };
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = b_first < b_end ? (b_end - b_first + b_step - 1) / b_step : 0;
  // the zero rows of both dz3 images stay zero; the interiors are rewritten per image
  for (int c = tid; c < 2 * C3D_P / 16; c += 512) reinterpret_cast<bf16x8*>(smem)[c] = zero_bf16x8();
  // RINGDP_C3_ABLATE / RINGDP_C12_ABLATE bit 3 (a scheduling A/B, results unchanged): the younger (VALU / DMA)
  // half at issue priority 1 (MI355X_MICROARCH: two waves per SIMD, static priority)
  if ((ablate & 8) && wave >= 4) __builtin_amdgcn_s_setprio(1);
  if (wave < 4) {
    // ---- MFMA waves: wave w owns input channels 16w..16w+15 (as conv3_dgrad_role)
    const int r16 = lane & 15, q8 = (lane >> 4) * 8, c4 = (lane >> 4) * 4;
    const bf16x8* pk = reinterpret_cast<const bf16x8*>(packed + P3D_OFF);
    bf16x8 aw[36];
#pragma unroll
    for (int j = 0; j < 36; ++j) aw[j] = pk[(wave * 36 + j) * 64 + lane];
    const int pbase = ((r16 >> 3) + 2) * C3_PY + (r16 & 7) * C3_PX + q8;
    const int xcol = r16 & 7, chunk = 4 * wave + (c4 >> 2);
    // da2 targets of m-tile 0: (row r16 >> 3, column xcol); lanes of column 7 also columns 8 and 9
    const int dcol = c3v_da((r16 >> 3) * 10 + xcol, xcol, chunk);
    const int dc8 = c3v_da((r16 >> 3) * 10 + 8, 8, chunk), dc9 = c3v_da((r16 >> 3) * 10 + 9, 9, chunk);
    lds_barrier();  // [B0] zero rows
    lds_barrier();  // [B1] image 0 expanded
    for (int s = 0; s <= n; ++s) {
      if (s < n && !(ablate & 2)) {
        const bf16* P = Pb(s & 1);
        float* DA = DAb(s & 1);
        // the 13 (m-tile, ky) groups with a non-zero dz3 row, in order; group g+1's 4 B fragments are read
        // while group g's 12 MFMAs run (the reads issued right before their MFMAs had exposed ~100 cycles per
        // group)
        constexpr int NG = 13;
        auto gmt = [](int g) { return g < 2 ? 0 : (g < 11 ? (g - 2) / 3 + 1 : 4); };
        auto gky = [](int g) { return g < 2 ? g : (g < 11 ? (g - 2) % 3 : g - 10); };
        auto readB = [&](int g, bf16x8 (&b)[4]) {
#pragma unroll
          for (int ks = 0; ks < 4; ++ks)
            b[ks] = *reinterpret_cast<const bf16x8*>(P + pbase + (2 * gmt(g) - gky(g)) * C3_PY + ks * 32);
        };
        bf16x8 bfa[4], bfb[4];
        readB(0, bfa);
        f32x4 acc[3];
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          const int mt = gmt(g), ky = gky(g);
          bf16x8(&bcur)[4] = (g & 1) ? bfb : bfa;
          bf16x8(&bnxt)[4] = (g & 1) ? bfa : bfb;
          if (g + 1 < NG) readB(g + 1, bnxt);
          if (g == 0 || gmt(g - 1) != mt) acc[0] = acc[1] = acc[2] = zero_f32x4();
#pragma unroll
          for (int ks = 0; ks < 4; ++ks)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) acc[kx] = mfma16x16x32(aw[(3 * ky + kx) * 4 + ks], bcur[ks], acc[kx]);
          if (g + 1 < NG && gmt(g + 1) == mt) continue;
          // col2im along the row in registers: da2(x) = acc0(x) + acc1(x-1) + acc2(x-2), the shifted terms
          // by DPP row shifts inside each 16-lane group (= 2 dz3 rows x 8 columns; a term that would cross
          // into the next row is zeroed at its source lane); column 8 = acc1(7) + acc2(6), column 9 =
          // acc2(7) go out from the column-7 lanes.  One plain store per target, no read-add-write.
          f32x4 out, e8;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float a1 = xcol == 7 ? 0.f : acc[1][j], a2 = xcol >= 6 ? 0.f : acc[2][j];
            out[j] = (acc[0][j] + dpp_row_shr<1>(a1)) + dpp_row_shr<2>(a2);
            e8[j] = acc[1][j] + dpp_row_shr<1>(acc[2][j]);
          }
          *reinterpret_cast<f32x4*>(DA + dcol + 20 * mt * 64) = out;
          if (xcol == 7) {
            *reinterpret_cast<f32x4*>(DA + dc8 + 20 * mt * 64) = e8;
            *reinterpret_cast<f32x4*>(DA + dc9 + 20 * mt * 64) = acc[2];
          }
        }
      }
      lds_barrier();
    }
  } else {
    // ---- VALU waves: thread vt of 256; wave 7 issues every LDS-DMA (it has no pool2 items, so its
    // vmcnt covers exactly its DMAs)
    const int vt = tid - 256;
    const bool dma = wave == 7;
    auto row_ptr = [&](bf16* P) {
      return [P](int r) {
        const int w = r >> 2, i = r & 3;
        return P + (2 * (w >> 2) + (i >> 1) + 2) * C3_PY + (2 * (w & 3) + (i & 1)) * C3_PX;
      };
    };
    if (dma && n > 0) {
#pragma unroll
      for (int k = 0; k < 6; ++k) c3s_glds(da3m, idx3, b_first, Sb(0), k, lane);
      if (n > 1) {
#pragma unroll
        for (int k = 0; k < 6; ++k) c3s_glds(da3m, idx3, b_first + b_step, Sb(1), k, lane);
      }
      c_dma_wait();
    }
    lds_barrier();  // [B0]
    if (n > 0) {
      C3Pre pre;
      c3s_pre(Sb(0), vt, pre);
      c3_expand(pre, vt, row_ptr(Pb(0)));
    }
    lds_barrier();  // [B1]
    for (int s = 0; s <= n; ++s) {
      if (dma) {
        if (s + 2 < n) {
#pragma unroll
          for (int k = 0; k < 6; ++k) c3s_glds(da3m, idx3, b_first + (s + 2) * b_step, Sb(s & 1), k, lane);
        }
        if (s < n) codes_dma(s, lane);
      }
      if (s + 1 < n) {
        C3Pre pre;
        c3s_pre(Sb((s + 1) & 1), vt, pre);
        c3_expand(pre, vt, row_ptr(Pb((s + 1) & 1)));
      }
      if (s >= 1 && vt < 176 && !(ablate & 1)) c3_pool2_bwd(DAb((s - 1) & 1), AMb((s - 1) & 1), dz2, b_first + (s - 1) * b_step, vt);
      // (issuing image s+1's codes a step earlier and leaving them in flight measured slower)
      if (dma) c_dma_wait();
      lds_barrier();
    }
  }
}

__device__ __forceinline__ void conv3_wgrad8_role(char* smem, const bf16* __restrict__ a2, const bf16* __restrict__ da3m,
                                                  const uint8_t* __restrict__ idx3, float* __restrict__ slabs, int B,
                                                  int nslices, int slice) {
  // three D / X image buffers: image i computes from buffer i % 3 while image i+2 is staged into (i+2) % 3,
  // so image i+1's first fragments can be read before the barrier that ends image i
  auto Db = [&](int k) { return reinterpret_cast<bf16*>(smem + k * C3V_D); };
  auto Xb = [&](int k) { return reinterpret_cast<bf16*>(smem + 3 * C3V_D + k * C3V_X); };
  auto Sb = [&](int k) { return smem + 3 * (C3V_D + C3V_X) + k * C3S_B; };
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // wave (wm, wn): m-tiles (co) 4wm..4wm+3 x n-tiles 4j + wn (j < 9), n = tap*64 + ci, i.e. tap j and channels
  // 16wn..16wn+15: the tap part of every X address is then an immediate offset
  const int wm = wave & 1, wn = wave >> 1;
  const int g16 = lane & 15, grp = lane >> 4, q = g16 >> 2, p = g16 & 3;
  f32x4 acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = zero_f32x4();
  // images slice, slice + nslices, ...: the dgrad workgroups stride the batch the same way, so with both counts
  // multiples of 8 an image's two readers of the compact gradient run on one XCD at about the same time
  const int n = slice < B ? (B - slice + nslices - 1) / nslices : 0;
  auto img = [&](int i) { return slice + i * nslices; };
  // this wave's a2 DMA instructions: k = wave, wave + 8
  const uint32_t xo0 = a2_rows_off(wave, lane), xo1 = a2_rows_off(wave + 8, lane);
  auto dma_x = [&](int b, bf16* X) {
    a2_glds_rows(a2, b, X, wave, xo0);
    a2_glds_rows(a2, b, X, wave + 8, xo1);
  };
  auto expand = [&](const char* S, bf16* D) {
    C3Pre pre;
    c3s_pre(S, tid, pre);
    c3_expand(pre, tid, [&](int r) { return D + c3v_drow(r); });
  };
  auto readA = [&](int buf, int ks, bf16x8 (&af)[4]) {
    const bf16* D = Db(buf) + 64 * wm + 4 * p;
    const int kb = ks * 32 + grp * 8;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const bf16x4 lo = lds_read_tr16(D + c3v_drow(kb + q) + mi * 16);
      const bf16x4 hi = lds_read_tr16(D + c3v_drow(kb + 4 + q) + mi * 16);
      af[mi] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  };
  if (n > 0) {  // prologue: images 0 and 1 staged, image 2's compact gradient in S0
    if (wave < 6) {
      c3s_glds(da3m, idx3, img(0), Sb(0), wave, lane);
      if (n > 1) c3s_glds(da3m, idx3, img(1), Sb(1), wave, lane);
    }
    dma_x(img(0), Xb(0));
    if (n > 1) dma_x(img(1), Xb(1));
    c_dma_wait();
    lds_barrier();
    expand(Sb(0), Db(0));
    if (n > 1) expand(Sb(1), Db(1));
    lds_barrier();  // S0, S1 free
    if (n > 2 && wave < 6) c3s_glds(da3m, idx3, img(2), Sb(0), wave, lane);
    c_dma_wait();
  }
  lds_barrier();
  bf16x8 af[4], afn[4];
  if (n > 0) readA(0, 0, af);
  for (int i = 0; i < n; ++i) {
    const int cur = i % 3;
    const int st = (i + 2) % 3;  // staging buffer of image i+2
    if (i + 2 < n) dma_x(img(i + 2), Xb(st));
    if (i + 3 < n && wave < 6) c3s_glds(da3m, idx3, img(i + 3), Sb((i + 1) & 1), wave, lane);
    const int xb = (int)(Xb(cur) - reinterpret_cast<const bf16*>(smem)) + 16 * wn + 4 * p;  // element offset
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int kb = ks * 32 + grp * 8;
      int x0 = xb + win_pos(kb + q, 10) * C3V_XRS, x1 = xb + win_pos(kb + 4 + q, 10) * C3V_XRS;
      // the whole per-lane part of the address opaque to the optimiser: otherwise it folds the tap offset into
      // a per-tap SGPR or VGPR and pays one VALU add per fragment read instead of the immediate offset
      asm("" : "+v"(x0), "+v"(x1));
      const bf16* S0 = reinterpret_cast<const bf16*>(smem);
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const int shift = ((j / 3) * 10 + j % 3) * C3V_XRS;  // tap j
        const bf16x4 lo = lds_read_tr16(S0 + x0 + shift);
        const bf16x4 hi = lds_read_tr16(S0 + x1 + shift);
        const bf16x8 bf = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        if (j == 4) {  // next k-step's A fragments (image i+1's first, when ks = 1: its buffer is complete)
          if (ks == 0)
            readA(cur, 1, afn);
          else if (i + 1 < n)
            readA((i + 1) % 3, 0, af);
        }
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) acc[mi][j] = mfma16x16x32(ks == 0 ? af[mi] : afn[mi], bf, acc[mi][j]);
      }
      if (ks == 0 && i + 2 < n) expand(Sb(i & 1), Db(st));  // image i+2's D, under the second k-step
    }
    // (letting image i+2's a2 copies stay in flight across the barrier measured 50 us slower)
    c_dma_wait();
    lds_barrier();
  }
  float* slab = slabs + (int64_t)slice * C3_WSLAB;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int co = (4 * wm + mi) * 16 + grp * 4;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int nn = (4 * j + wn) * 16 + g16;
      *reinterpret_cast<f32x4*>(slab + (int64_t)nn * 128 + co) = acc[mi][j];
    }
  }
}

// blocks [0, n_dgrad): dgrad of images [0, b_dgrad) (strided); then n_wgrad wgrad slices, whose workgroups
// go on to the dgrad of images [b_dgrad, B) (static split: deterministic)
__global__ __launch_bounds__(512, 1) void conv3_bwd8_kernel(const bf16* __restrict__ a2, const uint8_t* __restrict__ idx2,
                                                           const bf16* __restrict__ da3m, const uint8_t* __restrict__ idx3,
                                                           const bf16* __restrict__ packed, bf16* __restrict__ dz2,
                                                           int B, float* __restrict__ slabs, int n_wgrad, int n_dgrad,
                                                           int b_dgrad, int ablate) {
  __shared__ __attribute__((aligned(16))) char smem[C3V_LDS];
  const int blk = blockIdx.x;
  if (blk < n_dgrad) {
    conv3_dgrad8_role(smem, da3m, idx3, idx2, packed, dz2, blk, b_dgrad, n_dgrad, ablate);
    return;
  }
  const int w = blk - n_dgrad;
  if (!(ablate & 4)) conv3_wgrad8_role(smem, a2, da3m, idx3, slabs, B, n_wgrad, w);
  if (dz2 == nullptr || b_dgrad >= B) return;
  __syncthreads();  // LDS changes role
  conv3_dgrad8_role(smem, da3m, idx3, idx2, packed, dz2, b_dgrad + w, B, n_wgrad, ablate);
}

__device__ __forceinline__ bf16x8 ones_column_frag(int lane) {
  const bf16 one = (bf16)((lane & 15) == 0 ? 1.f : 0.f);
  return bf16x8{one, one, one, one, one, one, one, one};
}

// ================================================================== F2 backward
// conv2's ReLU and pool2 are undone by F3's backward, so dz2 is the conv output gradient directly:
//   dgrad: da1 = full-corr(dz2 image, flipped W2)  [13x13x32]
//   wgrad: dW2t[n = tap*32 + ci][co] = sum_pos dz2[pos][co] * a1[pos + tap][ci]; db2 via a ones tile
constexpr int C2_PW = 15, C2_PRS = 80, C2_ORS = 40, C2_DRS = 72;
// dgrad m-tile -> output position map (255 = padding row).  Each full tile holds two positions of every
// residue (y*15 + x) mod 8, one among lanes {0-3,12-15} and one among lanes {4-11}: with 160-B rows
// (C2_PRS 80) the 16 rows of every ds_read_b128 lane group then land on 16 distinct 16-B bank slots
// (modelled 11.3 -> 4.7 LDS cycles per A-fragment read, ideal 4; generator: tools/lds_bank_model.py).
__constant__ uint8_t c2d_tile_pos[176] = {0,1,2,3,8,9,10,11,12,19,20,13,4,5,6,7,14,15,16,17,22,23,24,25,32,39,34,27,18,33,26,21,28,29,30,31,36,37,38,45,52,53,48,41,46,47,40,35,42,43,44,59,50,51,58,65,66,67,62,55,60,61,54,49,56,57,72,73,64,71,78,79,80,81,76,69,74,75,68,63,70,85,86,87,84,91,92,93,94,95,90,83,88,89,82,77,98,99,100,101,104,105,106,107,108,109,110,111,102,103,96,97,112,113,114,115,118,119,120,121,122,137,130,125,116,123,124,117,126,127,128,129,132,133,134,135,150,151,144,139,136,143,138,131,140,141,142,149,146,147,148,163,164,165,158,153,156,157,152,145,154,155,162,168,160,161,255,255,255,255,255,167,255,255,166,159};
constexpr int C2D_P = C2_PW * C2_PW * C2_PRS * 2;  // 32400
constexpr int C2D_O = 169 * C2_ORS * 2;            // 13520 (x2: double-buffered output tile)
// wgrad dz2 tile: rows k in blocks of 8 (80-element rows, 704-element blocks): the 8 rows of a tr16
// 32-lane group (k, k+1, k+2, k+3, k+8, ..) then cover the 8 32-B bank slots once (modelled 4 -> 2)
__device__ __forceinline__ int c2_drow(int r) { return (r >> 3) * 704 + (r & 7) * 80; }
constexpr int C2W_D = 16 * 704 * 2;                // 22528
constexpr int C2W_X = 169 * C2_XRS * 2;            // 13520
constexpr int C2B_LDS = (C2D_P + 2 * C2D_O) > (C2W_D + C2W_X) ? (C2D_P + 2 * C2D_O) : (C2W_D + C2W_X);
constexpr int C2_WSLAB = 288 * 64 + 64;

__device__ __forceinline__ void conv2_dgrad_role(char* smem, const bf16* __restrict__ dz2, const bf16* __restrict__ packed,
                                 bf16* __restrict__ da1, int B, int block, int nblocks) {
  bf16* P = reinterpret_cast<bf16*>(smem);
  bf16* O = reinterpret_cast<bf16*>(smem + C2D_P);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nt = wave & 1, mg = wave >> 1;  // n-tile (16 input channels), m-tiles mg, mg+4, mg+8
  const int r16 = lane & 15, q8 = (lane >> 4) * 8;
  const bf16x8* pk = reinterpret_cast<const bf16x8*>(packed + P2D_OFF);
  bf16x8 bw[18];
#pragma unroll
  for (int ks = 0; ks < 18; ++ks) bw[ks] = pk[(nt * 18 + ks) * 64 + lane];
  int base[3];  // padding rows read a valid address; their outputs are dropped
  int opos[3][4];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int mt = min(mg + 4 * k, 10);
    const int mm = c2d_tile_pos[mt * 16 + r16] == 255 ? 0 : c2d_tile_pos[mt * 16 + r16];
    base[k] = (mm / 13) * C2_PW + mm % 13;
#pragma unroll
    for (int i = 0; i < 4; ++i) opos[k][i] = c2d_tile_pos[mt * 16 + (lane >> 4) * 4 + i];
  }
  for (int c = tid; c < C2D_P / 16; c += 512) reinterpret_cast<bf16x8*>(P)[c] = zero_bf16x8();
  auto copy_out = [&](int bb, const bf16* src) {
    bf16x8* dst = reinterpret_cast<bf16x8*>(da1 + (int64_t)bb * 169 * 32);
    for (int c = tid; c < 676; c += 512) dst[c] = *reinterpret_cast<const bf16x8*>(src + (c >> 2) * C2_ORS + (c & 3) * 8);
  };
  bf16x8 pz[2];
  auto load = [&](int bb) {
    const bf16x8* src = reinterpret_cast<const bf16x8*>(dz2 + (int64_t)bb * 121 * 64);
    pz[0] = src[tid];
    if (tid + 512 < 968) pz[1] = src[tid + 512];
  };
  // m-tiles mg, mg+4, mg+8 < 11: 3 for waves with mg < 3, 2 for mg == 3 (compile-time trip counts)
  auto mfma_phase = [&](auto nk_c, bf16* Oc) {
    constexpr int NK = decltype(nk_c)::value;
    f32x4 acc[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) acc[k] = zero_f32x4();
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) {
      const int tapp = ks >> 1, c0 = (ks & 1) * 32;
      const int shift = (tapp / 3) * C2_PW + tapp % 3;
#pragma unroll
      for (int k = 0; k < NK; ++k)
        acc[k] = mfma16x16x32(*reinterpret_cast<const bf16x8*>(P + (base[k] + shift) * C2_PRS + c0 + q8), bw[ks],
                              acc[k]);
    }
#pragma unroll
    for (int k = 0; k < NK; ++k) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = opos[k][i];
        if (m < 169) Oc[m * C2_ORS + nt * 16 + r16] = (bf16)acc[k][i];
      }
    }
  };
  int b = block, prev = -1, cur = 0;
  if (b < B) load(b);
  for (; b < B; b += nblocks) {
    __syncthreads();
    if (prev >= 0) copy_out(prev, O + (cur ^ 1) * 169 * C2_ORS);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int c = tid + 512 * k;
      if (c < 968) {
        const int pos = c >> 3, cc = (c & 7) * 8;
        *reinterpret_cast<bf16x8*>(P + ((pos / 11 + 2) * C2_PW + pos % 11 + 2) * C2_PRS + cc) = pz[k];
      }
    }
    const int nb = b + nblocks;
    if (nb < B) load(nb);
    __syncthreads();
    bf16* Oc = O + cur * 169 * C2_ORS;
    if (mg < 3)
      mfma_phase(std::integral_constant<int, 3>{}, Oc);
    else
      mfma_phase(std::integral_constant<int, 2>{}, Oc);
    prev = b;
    cur ^= 1;
  }
  __syncthreads();
  if (prev >= 0) copy_out(prev, O + (cur ^ 1) * 169 * C2_ORS);
}

__device__ __forceinline__ void conv2_wgrad_role(char* smem, const bf16* __restrict__ a1, const bf16* __restrict__ dz2,
                                 float* __restrict__ slabs, int B, int nslices, int slice) {
  bf16* D = reinterpret_cast<bf16*>(smem);
  bf16* X = reinterpret_cast<bf16*>(smem + C2W_D);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;  // m-tile wm (co 16wm..), n-tiles 9wn..9wn+8
  const int g16 = lane & 15, grp = lane >> 4, q = g16 >> 2, p = g16 & 3;
  const bf16x8 onesf = ones_column_frag(lane);
  f32x4 acc[9], accb = zero_f32x4();
#pragma unroll
  for (int j = 0; j < 9; ++j) acc[j] = zero_f32x4();
  for (int c = tid; c < C2W_D / 16; c += 512) reinterpret_cast<bf16x8*>(D)[c] = zero_bf16x8();  // rows >= 121 stay 0
  const int per = cdiv(B, nslices);
  const int b_lo = slice * per, b_hi = min(B, b_lo + per);
  bf16x8 pz[2], pa[2];
  auto load = [&](int bb) {
    const bf16x8* zs = reinterpret_cast<const bf16x8*>(dz2 + (int64_t)bb * 121 * 64);
    const bf16x8* as = reinterpret_cast<const bf16x8*>(a1 + (int64_t)bb * 169 * 32);
    pz[0] = zs[tid];
    if (tid + 512 < 968) pz[1] = zs[tid + 512];
    pa[0] = as[tid];
    if (tid + 512 < 676) pa[1] = as[tid + 512];
  };
  if (b_lo < b_hi) load(b_lo);
  for (int b = b_lo; b < b_hi; ++b) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int c = tid + 512 * k;
      if (c < 968) *reinterpret_cast<bf16x8*>(D + c2_drow(c >> 3) + (c & 7) * 8) = pz[k];
      if (c < 676) *reinterpret_cast<bf16x8*>(X + (c >> 2) * C2_XRS + (c & 3) * 8) = pa[k];
    }
    if (b + 1 < b_hi) load(b + 1);
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int kb = ks * 32 + grp * 8;
      const int m0 = wm * 16;
      const bf16x4 alo = lds_read_tr16(D + c2_drow(kb + q) + m0 + 4 * p);
      const bf16x4 ahi = lds_read_tr16(D + c2_drow(kb + 4 + q) + m0 + 4 * p);
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
      if (wn == 0) accb = mfma16x16x32(af, onesf, accb);
    }
  }
  float* slab = slabs + (int64_t)slice * C2_WSLAB;
  const int co = wm * 16 + grp * 4;
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int n = (9 * wn + j) * 16 + g16;
    *reinterpret_cast<f32x4*>(slab + (int64_t)n * 64 + co) = acc[j];
  }
  if (wn == 0 && g16 == 0) *reinterpret_cast<f32x4*>(slab + 288 * 64 + co) = accb;
}

__global__ __launch_bounds__(512) void conv2_bwd_kernel(const bf16* __restrict__ a1,
                                                        const bf16* __restrict__ dz2,
                                                        const bf16* __restrict__ packed,
                                                        bf16* __restrict__ da1, int B,
                                                        float* __restrict__ slabs, int nslices,
                                                        int n_dgrad) {
  __shared__ __attribute__((aligned(16))) char smem[C2B_LDS];
  if ((int)blockIdx.x < n_dgrad)
    conv2_dgrad_role(smem, dz2, packed, da1, B, blockIdx.x, n_dgrad);
  else
    conv2_wgrad_role(smem, a1, dz2, slabs, B, nslices, blockIdx.x - n_dgrad);
}

// ================================================================== F1 backward (conv1 wgrad)
// dW1[co][t] = sum_{b, oh, ow} dC[b][oh][ow][co] * xpad[b][oh + kh][ow + kw]  as a TN GEMM with
// K = spatial positions in rows of 32 (k = oh*32 + ow, ow >= 26 zero): the X operand for tap
// (kh, kw) and 8 consecutive ow is one aligned ds_read_b128 of shifted copy kw.  dC = unpool(da1) *
// relu-mask is never materialised: the A fragment of lane (co, 8 positions ow..ow+7 of row oh) covers 4
// pool windows px..px+3 of window row oh/2, so it is built in registers from ONE ds_read_b64_tr_b16 of
// the compact da1 image (4 windows x 16 channels) and ONE 8-byte read of the code rows: element
// (window k, dx) = da1 if bit (oh&1)*2 + dx of the window's one-hot code is set, else 0.  Tap column t = 25 of the padded N is a ones
// column -> db1 for free.  The 4 waves split K (rows oh = wave mod 4) and cover all 2x2 output tiles,
// so every A and B fragment feeds 2 MFMAs; da1 and the codes of the next image land by LDS-DMA while
// the current one computes.
constexpr int C1_WSLAB = 32 * 25 + 32;
constexpr int C1W_RS = 48, C1W_CS = 1520;          // padded copies: B-operand reads 16 -> 6 LDS cycles
constexpr int C1W_XS = 0;                          // 5 shifted copies of the input image (bf16)
constexpr int C1W_D = 5 * C1W_CS * 2;              // 15200: da1 image [169 (+3 zero) windows][32] bf16, x2
constexpr int C1W_DSZ = 172 * 32 * 2;              // 11008
constexpr int C1W_C = C1W_D + 2 * C1W_DSZ;         // 37216: code rows [13][16][16][2] bytes, x2
constexpr int C1W_LDS = C1W_C + 2 * C1I_IMG;       // 43872 -> 3 workgroups per CU

template <bool U8>
__global__ __launch_bounds__(256) void conv1_wgrad_kernel(const void* __restrict__ xin,
                                                          const bf16* __restrict__ da1,
                                                          const uint8_t* __restrict__ idx1, int B,
                                                          float mean, float inv_std, float in_scale,
                                                          float* __restrict__ slabs, int nslices) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[C1W_LDS];  // one array: keeps the DMA in flight
  bf16* xs = reinterpret_cast<bf16*>(lds + C1W_XS);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i16 = lane & 15, g = lane >> 4, q = i16 >> 2, p = i16 & 3;
  // B operand (x) per n-tile: lane column t = 16 nt + i16; t = 25 is the ones column, t > 25 zero
  const int t1 = 16 + i16;
  const int xoff0 = (i16 % 5) * C1W_CS + (i16 / 5) * C1W_RS + 8 * g;
  const int xoff1 = t1 < 25 ? (t1 % 5) * C1W_CS + (t1 / 5) * C1W_RS + 8 * g : 0;
  const uint32_t b1fill = t1 == 25 ? 0x3f803f80u : 0u;  // bf16 1.0 pairs
  for (int i = tid; i < C1W_C / 16; i += 256) reinterpret_cast<uint4*>(lds)[i] = make_uint4(0, 0, 0, 0);
  const int per = cdiv(B, nslices);
  const int b_lo = min(B, blockIdx.x * per), b_hi = min(B, b_lo + per);
  auto dma = [&](int bb, int k) {
    const bf16* src = da1 + (int64_t)bb * C1A_IMG;
    uint8_t* dd = lds + C1W_D + k * C1W_DSZ;
    for (int i = wave; i < 11; i += 4) {
      const int c = i * 64 + lane;
      if (c < C1A_IMG / 8) glds16_async(src + c * 8, dd + i * 1024);
    }
    const uint8_t* cs = idx1 + (int64_t)bb * C1I_IMG;
    uint8_t* cd = lds + C1W_C + k * C1I_IMG;
    for (int i = wave; i < 7; i += 4) {
      const int c = i * 64 + lane;
      if (c < C1I_IMG / 16) glds16_async(cs + c * 16, cd + i * 1024);
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m) acc[m][0] = acc[m][1] = zero_f32x4();
  uint32_t xu = 0;
  float4 xf = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();  // zero fill done before any DMA / copy write lands
  if (b_lo < b_hi) {
    c1_load<U8>(xin, b_lo, tid, xu, xf);
    dma(b_lo, 0);
    c1_store<U8, 5, C1W_RS, C1W_CS>(xs, tid, xu, xf, mean, inv_std, in_scale);
  }
  int cur = 0;
  for (int b = b_lo; b < b_hi; ++b) {
    c_dma_wait();
    __syncthreads();  // copies of image b written, its da1 / codes landed
    if (b + 1 < b_hi) {
      c1_load<U8>(xin, b + 1, tid, xu, xf);
      dma(b + 1, cur ^ 1);
    }
    const bf16* D = reinterpret_cast<const bf16*>(lds + C1W_D + cur * C1W_DSZ);
    const uint8_t* CB = lds + C1W_C + cur * C1I_IMG;
    const int dy = wave & 1;  // ks = wave (mod 4): every k-step of a wave is the same window row half
    for (int ks = wave; ks < 26; ks += 4) {
      const int py = ks >> 1;
      bf16x8 A[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        // (bit-cast the whole vector: __builtin_bit_cast of a single vector element miscompiles to element 0)
        const uint2 d = __builtin_bit_cast(uint2, lds_read_tr16(D + (py * 13 + 4 * g + q) * 32 + m * 16 + 4 * p));
        const int co = m * 16 + i16;
        const uint32_t cu = *reinterpret_cast<const uint32_t*>(CB + py * 256 + (co >> 1) * 16 + 4 * g);
        const int csh = 4 * (co & 1) + 2 * dy;
        uint32_t pr[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t dv = k & 1 ? (k < 2 ? d.x : d.y) >> 16 : (k < 2 ? d.x : d.y) & 0xffffu;
          // the two one-hot bits of window row dy: 1 -> dx = 0, 2 -> dx = 1, 0 -> no gradient
          const uint32_t sel = __builtin_amdgcn_ubfe(cu, 8 * k + csh, 2);
          pr[k] = dv * ((sel * 0x8001u) & 0x10001u);  // dv, dv << 16 or 0
        }
        A[m] = __builtin_bit_cast(bf16x8, make_uint4(pr[0], pr[1], pr[2], pr[3]));
      }
      const bf16x8 B0 = *reinterpret_cast<const bf16x8*>(xs + xoff0 + ks * C1W_RS);
      bf16x8 B1 = *reinterpret_cast<const bf16x8*>(xs + xoff1 + ks * C1W_RS);
      if (t1 >= 25) B1 = __builtin_bit_cast(bf16x8, make_uint4(b1fill, b1fill, b1fill, b1fill));
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        acc[m][0] = mfma16x16x32(A[m], B0, acc[m][0]);
        acc[m][1] = mfma16x16x32(A[m], B1, acc[m][1]);
      }
    }
    if (b + 1 < b_hi) {
      __syncthreads();  // every wave is done reading the copies of image b
      c1_store<U8, 5, C1W_RS, C1W_CS>(xs, tid, xu, xf, mean, inv_std, in_scale);
    }
    cur ^= 1;
  }
  // combine the 4 K-groups in a fixed order (deterministic) and write this workgroup's slab
  __syncthreads();
  float* red = reinterpret_cast<float*>(lds);  // [wave][tile][lane][4]: 16 KiB
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
      *reinterpret_cast<f32x4*>(red + ((wave * 4 + m * 2 + n) * 64 + lane) * 4) = acc[m][n];
  __syncthreads();
  const int tile = tid >> 6;
  f32x4 sum = *reinterpret_cast<const f32x4*>(red + (tile * 64 + lane) * 4);
#pragma unroll
  for (int w = 1; w < 4; ++w) sum += *reinterpret_cast<const f32x4*>(red + ((w * 4 + tile) * 64 + lane) * 4);
  float* slab = slabs + (int64_t)blockIdx.x * C1_WSLAB;
  const int tap = (tile & 1) * 16 + i16;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int co = (tile >> 1) * 16 + g * 4 + r;
    if (tap < 25) slab[co * 25 + tap] = sum[r];
    if (tap == 25) slab[800 + co] = sum[r];
  }
}

// ================================================================== F2 backward + F1 wgrad, fused
// The conv2 data gradient of an image (da1, 13x13x32) has exactly one consumer: conv1's weight gradient.
// The dgrad workgroups therefore keep da1 in LDS and run conv1 wgrad on it right away (the input image
// and its pool1 codes arrive by register load / LDS-DMA while conv2 dgrad computes): da1 never goes to
// HBM (2 x 354 MB per step at B=32768), and conv1 wgrad + its reduction are no longer launches of their
// own.  Each dgrad workgroup leaves one conv1 slab (C1_WSLAB), reduced with conv2's slabs in one launch.
// conv1 part: the 8 waves split K (rows oh = wave mod 8; dy = wave & 1 stays fixed per wave) and cover
// all 2x2 output tiles, as conv1_wgrad_kernel does with 4 waves.
constexpr int C12_O = 172 * C2_ORS * 2;             // 13760: da1 [169 + 3 zero windows][32 (+8 pad)] bf16
constexpr int C12_XS = 5 * C1W_CS * 2;              // 15200: 5 shifted copies of the input image
// P | O[2] | xs[2] | codes[2]: image i uses buffer set i & 1, so conv1 wgrad of image i-1 runs interleaved
// with conv2 dgrad of image i (2 waves per SIMD: the MFMA stream of one hides the LDS/VALU of the other)
constexpr int C12_OFF_O = C2D_P, C12_OFF_X = C12_OFF_O + 2 * C12_O, C12_OFF_C = C12_OFF_X + 2 * C12_XS;
constexpr int C12_LDS = C12_OFF_C + 2 * C1I_IMG;    // 96976
constexpr int C12B_LDS = C12_LDS > (C2W_D + C2W_X) ? C12_LDS : (C2W_D + C2W_X);
static_assert(C2D_P % 16 == 0 && C12_O % 16 == 0 && C12_XS % 16 == 0, "16-B aligned LDS buffers");
static_assert(8 * 4 * 64 * 4 * 4 <= C12_OFF_X, "conv1 cross-wave reduction fits in P + O");

template <bool U8>
__device__ __forceinline__ void conv12_dgrad_role(char* smem, const void* __restrict__ xin, const uint8_t* __restrict__ idx1,
                                  const bf16* __restrict__ dz2, const bf16* __restrict__ packed, int B, int block,
                                  int nblocks, float mean, float inv_std, float in_scale,
                                  float* __restrict__ slabs1) {
  bf16* P = reinterpret_cast<bf16*>(smem);
  auto Obuf = [&](int k) { return reinterpret_cast<bf16*>(smem + C12_OFF_O + k * C12_O); };
  auto Xbuf = [&](int k) { return reinterpret_cast<bf16*>(smem + C12_OFF_X + k * C12_XS); };
  auto Cbuf = [&](int k) { return reinterpret_cast<uint8_t*>(smem + C12_OFF_C + k * C1I_IMG); };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // ---- conv2 dgrad operands (as conv2_dgrad_role)
  const int nt = wave & 1, mg = wave >> 1;
  const int r16 = lane & 15, q8 = (lane >> 4) * 8;
  const bf16x8* pk = reinterpret_cast<const bf16x8*>(packed + P2D_OFF);
  bf16x8 bw[18];
#pragma unroll
  for (int ks = 0; ks < 18; ++ks) bw[ks] = pk[(nt * 18 + ks) * 64 + lane];
  int base[3];
  int opos[3][4];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int mt = min(mg + 4 * k, 10);
    const int mm = c2d_tile_pos[mt * 16 + r16] == 255 ? 0 : c2d_tile_pos[mt * 16 + r16];
    base[k] = (mm / 13) * C2_PW + mm % 13;
#pragma unroll
    for (int i = 0; i < 4; ++i) opos[k][i] = c2d_tile_pos[mt * 16 + (lane >> 4) * 4 + i];
  }
  // ---- conv1 wgrad operands (as conv1_wgrad_kernel)
  const int i16 = lane & 15, g = lane >> 4, q = i16 >> 2, p = i16 & 3;
  const int t1 = 16 + i16;
  const int xoff0 = (i16 % 5) * C1W_CS + (i16 / 5) * C1W_RS + 8 * g;
  const int xoff1 = t1 < 25 ? (t1 % 5) * C1W_CS + (t1 / 5) * C1W_RS + 8 * g : 0;
  const uint32_t b1fill = t1 == 25 ? 0x3f803f80u : 0u;
  const int dy = wave & 1;
  f32x4 acc1[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m) acc1[m][0] = acc1[m][1] = zero_f32x4();
  // zero P (its ring stays zero), both O (windows 169..171 stay zero) and both copy sets (ring stays zero)
  for (int c = tid; c < C12_OFF_C / 16; c += 512) reinterpret_cast<bf16x8*>(smem)[c] = zero_bf16x8();
  // next image, staged in registers: dz2 rows, input pixels, pool1 code rows
  bf16x8 pz[2];
  uint4 pc = make_uint4(0, 0, 0, 0);
  uint32_t xu = 0;
  float4 xf = make_float4(0.f, 0.f, 0.f, 0.f);
  auto load = [&](int bb) {
    const bf16x8* src = reinterpret_cast<const bf16x8*>(dz2 + (int64_t)bb * 121 * 64);
    pz[0] = src[tid];
    if (tid + 512 < 968) pz[1] = src[tid + 512];
    if (tid < C1I_IMG / 16) pc = reinterpret_cast<const uint4*>(idx1 + (int64_t)bb * C1I_IMG)[tid];
    c1_load<U8>(xin, bb, tid, xu, xf);
  };
  auto stage = [&](int k) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = tid + 512 * j;
      if (c < 968) {
        const int pos = c >> 3, cc = (c & 7) * 8;
        *reinterpret_cast<bf16x8*>(P + ((pos / 11 + 2) * C2_PW + pos % 11 + 2) * C2_PRS + cc) = pz[j];
      }
    }
    if (tid < C1I_IMG / 16) reinterpret_cast<uint4*>(Cbuf(k))[tid] = pc;
    c1_store<U8, 5, C1W_RS, C1W_CS>(Xbuf(k), tid, xu, xf, mean, inv_std, in_scale);
  };
  // conv1 wgrad k-step j (rows oh = wave + 8j; j = 3 only for waves 0, 1) of the image in buffer set k
  auto c1_step = [&](int j, int k) {
    const int ks0 = wave + 8 * j;
    const bool ok = ks0 < 26;  // wave-uniform
    const int ks = ok ? ks0 : 0;
    const int py = ks >> 1;
    const bf16* O = Obuf(k);
    const bf16* xs = Xbuf(k);
    const uint8_t* CB = Cbuf(k);
    bf16x8 A[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const uint2 d = __builtin_bit_cast(uint2, lds_read_tr16(O + (py * 13 + 4 * g + q) * C2_ORS + m * 16 + 4 * p));
      const int co = m * 16 + i16;
      const uint32_t cu = *reinterpret_cast<const uint32_t*>(CB + py * 256 + (co >> 1) * 16 + 4 * g);
      const int csh = 4 * (co & 1) + 2 * dy;
      uint32_t pr[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t dv = e & 1 ? (e < 2 ? d.x : d.y) >> 16 : (e < 2 ? d.x : d.y) & 0xffffu;
        const uint32_t sel = __builtin_amdgcn_ubfe(cu, 8 * e + csh, 2);
        pr[e] = ok ? dv * ((sel * 0x8001u) & 0x10001u) : 0u;
      }
      A[m] = __builtin_bit_cast(bf16x8, make_uint4(pr[0], pr[1], pr[2], pr[3]));
    }
    const bf16x8 B0 = *reinterpret_cast<const bf16x8*>(xs + xoff0 + ks * C1W_RS);
    bf16x8 B1 = *reinterpret_cast<const bf16x8*>(xs + xoff1 + ks * C1W_RS);
    if (t1 >= 25) B1 = __builtin_bit_cast(bf16x8, make_uint4(b1fill, b1fill, b1fill, b1fill));
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      acc1[m][0] = mfma16x16x32(A[m], B0, acc1[m][0]);
      acc1[m][1] = mfma16x16x32(A[m], B1, acc1[m][1]);
    }
  };
  // conv2 dgrad of the image staged in P -> O[k]; with C1 set, conv1 k-steps of buffer set k ^ 1 are
  // issued between its k-steps (after dgrad k-steps 3, 7, 11, 15)
  auto phase = [&](auto nk_c, auto c1_c, int k) {
    constexpr int NK = decltype(nk_c)::value;
    constexpr bool C1 = decltype(c1_c)::value;
    f32x4 acc[NK];
#pragma unroll
    for (int m = 0; m < NK; ++m) acc[m] = zero_f32x4();
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) {
      const int tapp = ks >> 1, c0 = (ks & 1) * 32;
      const int shift = (tapp / 3) * C2_PW + tapp % 3;
#pragma unroll
      for (int m = 0; m < NK; ++m)
        acc[m] = mfma16x16x32(*reinterpret_cast<const bf16x8*>(P + (base[m] + shift) * C2_PRS + c0 + q8), bw[ks],
                              acc[m]);
      if (C1 && (ks & 3) == 3 && ks < 16) c1_step(ks >> 2, k ^ 1);
    }
    bf16* O = Obuf(k);
#pragma unroll
    for (int m = 0; m < NK; ++m) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pos = opos[m][i];
        if (pos < 169) O[pos * C2_ORS + nt * 16 + r16] = (bf16)acc[m][i];
      }
    }
  };
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using T = std::true_type;
  using Fa = std::false_type;
  __syncthreads();  // zero fill done
  int b = block, k = 0;
  if (b < B) load(b);
  for (int i = 0; b < B; ++i, b += nblocks, k ^= 1) {
    __syncthreads();  // readers of P and of buffer set k (image i-2) are done
    stage(k);
    const int nb = b + nblocks;
    if (nb < B) load(nb);
    __syncthreads();  // image i staged; O[k ^ 1] (image i-1's da1) complete
    if (i == 0) {
      if (mg < 3) phase(I3{}, Fa{}, k);
      else phase(I2{}, Fa{}, k);
    } else {
      if (mg < 3) phase(I3{}, T{}, k);
      else phase(I2{}, T{}, k);
    }
  }
  __syncthreads();
  if (b != block) {  // at least one image: conv1 wgrad of the last one (buffer set k ^ 1)
#pragma unroll
    for (int j = 0; j < 4; ++j) c1_step(j, k ^ 1);
  }
  // combine the 8 K-groups in a fixed order (deterministic) and write this workgroup's conv1 slab
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // [wave][tile][lane][4]: 32 KiB over P + O
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
      *reinterpret_cast<f32x4*>(red + ((wave * 4 + m * 2 + n) * 64 + lane) * 4) = acc1[m][n];
  __syncthreads();
  if (tid >= 256) return;
  const int tile = tid >> 6;
  f32x4 sum = *reinterpret_cast<const f32x4*>(red + (tile * 64 + lane) * 4);
#pragma unroll
  for (int w = 1; w < 8; ++w) sum += *reinterpret_cast<const f32x4*>(red + ((w * 4 + tile) * 64 + lane) * 4);
  float* slab = slabs1 + (int64_t)block * C1_WSLAB;
  const int tap = (tile & 1) * 16 + i16;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int co = (tile >> 1) * 16 + g * 4 + r;
    if (tap < 25) slab[co * 25 + tap] = sum[r];
    if (tap == 25) slab[800 + co] = sum[r];
  }
}

template <bool U8>
__global__ __launch_bounds__(512) void conv12_bwd_kernel(const void* __restrict__ xin,
                                                         const uint8_t* __restrict__ idx1,
                                                         const bf16* __restrict__ a1,
                                                         const bf16* __restrict__ dz2,
                                                         const bf16* __restrict__ packed, int B,
                                                         float mean, float inv_std, float in_scale,
                                                         float* __restrict__ slabs2, int nslices,
                                                         float* __restrict__ slabs1, int n_dgrad) {
  __shared__ __attribute__((aligned(16))) char smem[C12B_LDS];
  if ((int)blockIdx.x < n_dgrad)
    conv12_dgrad_role<U8>(smem, xin, idx1, dz2, packed, B, blockIdx.x, n_dgrad, mean, inv_std, in_scale, slabs1);
  else
    conv2_wgrad_role(smem, a1, dz2, slabs2, B, nslices, blockIdx.x - n_dgrad);
}

// ---- conv2 backward + conv1 wgrad with wave-specialised / pipelined 8-wave workgroups (the conv3 bwd8
// scheme; batches above fc_in_c3_max_batch).  One 512-thread workgroup per CU:
//   dgrad: waves 0-3 run conv2's data gradient of image s (both 16-channel n-tiles per wave, so every
//     A-fragment read feeds 2 MFMAs: half the LDS reads of conv12_dgrad_role) into da1 O[s&1]; beside them
//     waves 4-7 run conv1's weight gradient of image s-1 (from O[(s-1)&1]) and stage image s+1 (dz2 ->
//     P, input copies, pool1 codes; registers loaded one step ahead).  One barrier per image.  The
//     input copies and codes of image s-1 are still read while image s+1 is staged: three of those.
//   wgrad: conv2's weight gradient, 8 waves each 2 co tiles x 4-5 n-tiles (14 tr16 reads per 10 MFMAs per
//     k-step instead of 20 per 9), image i+1 staged from registers while image i's MFMAs run.
constexpr int C12V_DG = 2 * (C2D_P + C12_O) + 3 * (C12_XS + C1I_IMG);  // 155104
constexpr int C12V_WG = 3 * (C2W_D + C2W_X);                           // 108144
constexpr int C12V_LDS = C12V_DG > C12V_WG ? C12V_DG : C12V_WG;
static_assert(C12V_LDS <= 160 * 1024 && C1I_IMG % 16 == 0, "conv12 backward (8-wave) LDS");

template <bool U8>
__device__ __forceinline__ void conv12_dgrad8_role(char* smem, const void* __restrict__ xin,
                                                   const uint8_t* __restrict__ idx1, const bf16* __restrict__ dz2,
                                                   const bf16* __restrict__ packed, int B, int block, int nblocks,
                                                   float mean, float inv_std, float in_scale,
                                                   float* __restrict__ slabs1, int ablate) {
  auto Pb = [&](int k) { return reinterpret_cast<bf16*>(smem + k * C2D_P); };
  auto Ob = [&](int k) { return reinterpret_cast<bf16*>(smem + 2 * C2D_P + k * C12_O); };
  auto Xb = [&](int k) { return reinterpret_cast<bf16*>(smem + 2 * (C2D_P + C12_O) + k * C12_XS); };
  auto Cb = [&](int k) { return reinterpret_cast<uint8_t*>(smem + 2 * (C2D_P + C12_O) + 3 * C12_XS + k * C1I_IMG); };
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = block < B ? (B - block + nblocks - 1) / nblocks : 0;
  // zero rings of both dz2 images, the zero windows 169..171 of both da1 images, the rings of the copies
  for (int c = tid; c < (2 * (C2D_P + C12_O) + 3 * C12_XS) / 16; c += 512)
    reinterpret_cast<bf16x8*>(smem)[c] = zero_bf16x8();
  __syncthreads();
  // RINGDP_C3_ABLATE / RINGDP_C12_ABLATE bit 3 (a scheduling A/B, results unchanged): the younger (VALU / DMA)
  // half at issue priority 1 (MI355X_MICROARCH: two waves per SIMD, static priority)
  if ((ablate & 8) && wave >= 4) __builtin_amdgcn_s_setprio(1);
  if (wave < 4) {
    // ---- MFMA waves: m-tiles wave, wave + 4, wave + 8 (< 11), both n-tiles.  Weights are the A operand
    // (the B-fragment pack read as A: the same lane -> (channel, k) map), so a lane's 4 results are 4
    // consecutive input channels of one position: one 8-byte store each.
    const int r16 = lane & 15, q8 = (lane >> 4) * 8, c4 = (lane >> 4) * 4;
    const bf16x8* pk = reinterpret_cast<const bf16x8*>(packed + P2D_OFF);
    bf16x8 bw[2][18];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int ks = 0; ks < 18; ++ks) bw[nt][ks] = pk[(nt * 18 + ks) * 64 + lane];
    int base[3], opos[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int mt = min(wave + 4 * k, 10);
      const int mm = c2d_tile_pos[mt * 16 + r16];
      opos[k] = mm;
      base[k] = mm == 255 ? 0 : (mm / 13) * C2_PW + mm % 13;
    }
    auto phase = [&](auto nk_c, const bf16* P, bf16* O) {
      constexpr int NK = decltype(nk_c)::value;
      f32x4 acc[NK][2];
#pragma unroll
      for (int k = 0; k < NK; ++k) acc[k][0] = acc[k][1] = zero_f32x4();
#pragma unroll
      for (int ks = 0; ks < 18; ++ks) {
        const int tapp = ks >> 1, c0 = (ks & 1) * 32;
        const int shift = (tapp / 3) * C2_PW + tapp % 3;
#pragma unroll
        for (int k = 0; k < NK; ++k) {
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(P + (base[k] + shift) * C2_PRS + c0 + q8);
          acc[k][0] = mfma16x16x32(bw[0][ks], a, acc[k][0]);
          acc[k][1] = mfma16x16x32(bw[1][ks], a, acc[k][1]);
        }
      }
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        if (opos[k] < 169) {
#pragma unroll
          for (int nt = 0; nt < 2; ++nt)
            *reinterpret_cast<bf16x4*>(O + opos[k] * C2_ORS + nt * 16 + c4) =
                bf16x4{(bf16)acc[k][nt][0], (bf16)acc[k][nt][1], (bf16)acc[k][nt][2], (bf16)acc[k][nt][3]};
        }
      }
    };
    lds_barrier();  // [B1] image 0 staged
    for (int s = 0; s <= n; ++s) {
      if (s < n && !(ablate & 2)) {
        if (wave < 3)
          phase(std::integral_constant<int, 3>{}, Pb(s & 1), Ob(s & 1));
        else
          phase(std::integral_constant<int, 2>{}, Pb(s & 1), Ob(s & 1));
      }
      lds_barrier();
    }
    __syncthreads();  // [R0] the V waves' conv1 reduction reuses P
    __syncthreads();  // [R1]
  } else {
    // ---- conv1-wgrad / staging waves: thread vt of 256
    const int vt = tid - 256, vw = wave - 4;
    const int i16 = lane & 15, g = lane >> 4, q = i16 >> 2, p = i16 & 3;
    const int t1 = 16 + i16;
    const int xoff0 = (i16 % 5) * C1W_CS + (i16 / 5) * C1W_RS + 8 * g;
    const int xoff1 = t1 < 25 ? (t1 % 5) * C1W_CS + (t1 / 5) * C1W_RS + 8 * g : 0;
    const uint32_t b1fill = t1 == 25 ? 0x3f803f80u : 0u;
    const int dy = vw & 1;  // k-steps vw, vw + 4, ...: one window-row half per wave
    f32x4 acc1[2][2];
#pragma unroll
    for (int m = 0; m < 2; ++m) acc1[m][0] = acc1[m][1] = zero_f32x4();
    // the next images' inputs in registers, two sets: image j's set is j & 1, loaded two steps before it is
    // staged (one step of latency hiding was not enough: staging alone ran at the per-CU latency bound)
    // the next images' inputs in registers, two sets: image j's set is j & 1, loaded two steps before it is
    // staged (one step of latency hiding was not enough: staging alone ran at the per-CU latency bound).
    // (Staging dz2 from the MFMA waves instead measured 935 -> 1024 us: they are the critical path.)
    struct Regs {
      bf16x8 pz[4];
      uint4 pc;
      uint32_t xu;
      float4 xf;
    };
    Regs r0, r1;
    auto load = [&](Regs& r, int bb) {
      const bf16x8* src = reinterpret_cast<const bf16x8*>(dz2 + (int64_t)bb * 121 * 64);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (vt + 256 * j < 968) r.pz[j] = src[vt + 256 * j];
      if (vt < C1I_IMG / 16) r.pc = reinterpret_cast<const uint4*>(idx1 + (int64_t)bb * C1I_IMG)[vt];
      c1_load<U8>(xin, bb, vt, r.xu, r.xf);
    };
    auto stage = [&](const Regs& r, int k2, int k3) {
      bf16* P = Pb(k2);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = vt + 256 * j;
        if (c < 968) {
          const int pos = c >> 3, cc = (c & 7) * 8;
          *reinterpret_cast<bf16x8*>(P + ((pos / 11 + 2) * C2_PW + pos % 11 + 2) * C2_PRS + cc) = r.pz[j];
        }
      }
      if (vt < C1I_IMG / 16) reinterpret_cast<uint4*>(Cb(k3))[vt] = r.pc;
      c1_store<U8, 5, C1W_RS, C1W_CS>(Xb(k3), vt, r.xu, r.xf, mean, inv_std, in_scale);
    };
    auto c1_step = [&](int ks, const bf16* O, const bf16* xs, const uint8_t* CB) {
      const int py = ks >> 1;
      bf16x8 A[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const uint2 d = __builtin_bit_cast(uint2, lds_read_tr16(O + (py * 13 + 4 * g + q) * C2_ORS + m * 16 + 4 * p));
        const int co = m * 16 + i16;
        const uint32_t cu = *reinterpret_cast<const uint32_t*>(CB + py * 256 + (co >> 1) * 16 + 4 * g);
        const int csh = 4 * (co & 1) + 2 * dy;
        uint32_t pr[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t dv = e & 1 ? (e < 2 ? d.x : d.y) >> 16 : (e < 2 ? d.x : d.y) & 0xffffu;
          const uint32_t sel = __builtin_amdgcn_ubfe(cu, 8 * e + csh, 2);
          pr[e] = dv * ((sel * 0x8001u) & 0x10001u);
        }
        A[m] = __builtin_bit_cast(bf16x8, make_uint4(pr[0], pr[1], pr[2], pr[3]));
      }
      const bf16x8 B0 = *reinterpret_cast<const bf16x8*>(xs + xoff0 + ks * C1W_RS);
      bf16x8 B1 = *reinterpret_cast<const bf16x8*>(xs + xoff1 + ks * C1W_RS);
      if (t1 >= 25) B1 = __builtin_bit_cast(bf16x8, make_uint4(b1fill, b1fill, b1fill, b1fill));
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        acc1[m][0] = mfma16x16x32(A[m], B0, acc1[m][0]);
        acc1[m][1] = mfma16x16x32(A[m], B1, acc1[m][1]);
      }
    };
    if (n > 0) {
      load(r0, block);
      stage(r0, 0, 0);
      if (n > 1) load(r1, block + nblocks);
      if (n > 2) load(r0, block + 2 * nblocks);
    }
    lds_barrier();  // [B1]
    // step s: stage image s+1 (its set (s+1) & 1), refill that set with image s+3, conv1 wgrad of image s-1
    auto step = [&](int s, Regs& rs) {
      if (s + 1 < n) {
        stage(rs, (s + 1) & 1, (s + 1) % 3);
        if (s + 3 < n) load(rs, block + (s + 3) * nblocks);
      }
      if (s >= 1 && !(ablate & 1)) {
        const bf16* O = Ob((s - 1) & 1);
        const bf16* xs = Xb((s - 1) % 3);
        const uint8_t* CB = Cb((s - 1) % 3);
        for (int ks = vw; ks < 26; ks += 4) c1_step(ks, O, xs, CB);
      }
      lds_barrier();
    };
    for (int s = 0; s <= n; s += 2) {  // unrolled by 2: register sets are not indexable
      step(s, r1);
      if (s + 1 <= n) step(s + 1, r0);
    }
    // combine the 4 K-groups in a fixed order (deterministic) and write this workgroup's conv1 slab
    __syncthreads();  // [R0]
    float* red = reinterpret_cast<float*>(smem);  // [vw][tile][lane][4]: 16 KiB over P
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int nn = 0; nn < 2; ++nn)
        *reinterpret_cast<f32x4*>(red + ((vw * 4 + m * 2 + nn) * 64 + lane) * 4) = acc1[m][nn];
    __syncthreads();  // [R1]
    const int tile = vw;
    f32x4 sum = *reinterpret_cast<const f32x4*>(red + (tile * 64 + lane) * 4);
#pragma unroll
    for (int w = 1; w < 4; ++w) sum += *reinterpret_cast<const f32x4*>(red + ((w * 4 + tile) * 64 + lane) * 4);
    float* slab = slabs1 + (int64_t)block * C1_WSLAB;
    const int tap = (tile & 1) * 16 + i16;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = (tile >> 1) * 16 + g * 4 + r;
      if (tap < 25) slab[co * 25 + tap] = sum[r];
      if (tap == 25) slab[800 + co] = sum[r];
    }
  }
}

// conv2 wgrad, 8 waves: wave (wm2 = wave & 1, wn = wave >> 1) owns co tiles 2wm2, 2wm2+1 x the n-tiles
// (tap, half) of dW2t [288][64] with half = wn & 1 (input channels 16 half ..) and taps h, h+2, .. (h = wn >> 1:
// 5 taps for h = 0, 4 for h = 1); the tap part of every X address is an immediate offset (body<H>).  The
// wn = 0 waves also form the bias column sums.  Three D / X image buffers, as conv3_wgrad8_role: image i+1's
// first A fragments are read before the barrier that ends image i.  The inputs are staged from registers
// loaded one image ahead (an LDS-DMA form with per-lane sources - 37 wave-instructions per image into the
// padded layouts - measured 1044 vs 782 us for this role at B=65536).
__device__ __forceinline__ void conv2_wgrad8_role(char* smem, const bf16* __restrict__ a1, const bf16* __restrict__ dz2,
                                                  float* __restrict__ slabs, int B, int nslices, int slice) {
  auto Db = [&](int k) { return reinterpret_cast<bf16*>(smem + k * C2W_D); };
  auto Xb = [&](int k) { return reinterpret_cast<bf16*>(smem + 3 * C2W_D + k * C2W_X); };
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm2 = wave & 1, wn = wave >> 1, half = wn & 1, h = wn >> 1;
  const int g16 = lane & 15, grp = lane >> 4, q = g16 >> 2, p = g16 & 3;
  const bf16x8 onesf = ones_column_frag(lane);
  f32x4 acc[2][5], accb[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    accb[m] = zero_f32x4();
#pragma unroll
    for (int j = 0; j < 5; ++j) acc[m][j] = zero_f32x4();
  }
  // rows >= 121 of the three D images stay zero
  for (int c = tid; c < 3 * C2W_D / 16; c += 512) reinterpret_cast<bf16x8*>(smem)[c] = zero_bf16x8();
  // images slice, slice + nslices, ... (as the dgrad workgroups)
  const int n = slice < B ? (B - slice + nslices - 1) / nslices : 0;
  auto img = [&](int i) { return slice + i * nslices; };
  // inputs of later images in registers, two sets (image j: set j & 1, loaded two images before it is staged)
  struct Regs {
    bf16x8 pz[2], pa[2];
  };
  Regs r0, r1;
  auto load = [&](Regs& r, int bb) {
    const bf16x8* zs = reinterpret_cast<const bf16x8*>(dz2 + (int64_t)bb * 121 * 64);
    const bf16x8* as = reinterpret_cast<const bf16x8*>(a1 + (int64_t)bb * 169 * 32);
    r.pz[0] = zs[tid];
    if (tid + 512 < 968) r.pz[1] = zs[tid + 512];
    r.pa[0] = as[tid];
    if (tid + 512 < 676) r.pa[1] = as[tid + 512];
  };
  auto stage = [&](const Regs& r, int k) {
    bf16* D = Db(k);
    bf16* X = Xb(k);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = tid + 512 * j;
      if (c < 968) *reinterpret_cast<bf16x8*>(D + c2_drow(c >> 3) + (c & 7) * 8) = r.pz[j];
      if (c < 676) *reinterpret_cast<bf16x8*>(X + (c >> 2) * C2_XRS + (c & 3) * 8) = r.pa[j];
    }
  };
  auto readA = [&](int buf, int ks, bf16x8 (&af)[2]) {
    const bf16* D = Db(buf) + 32 * wm2 + 4 * p;
    const int kb = ks * 32 + grp * 8;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const bf16x4 alo = lds_read_tr16(D + c2_drow(kb + q) + m * 16);
      const bf16x4 ahi = lds_read_tr16(D + c2_drow(kb + 4 + q) + m * 16);
      af[m] = bf16x8{alo[0], alo[1], alo[2], alo[3], ahi[0], ahi[1], ahi[2], ahi[3]};
    }
  };
  __syncthreads();  // zero fill before the first stage
  if (n > 0) {
    load(r0, img(0));
    stage(r0, 0);
    if (n > 1) {
      load(r1, img(1));
      stage(r1, 1);
    }
    if (n > 2) load(r0, img(2));
    if (n > 3) load(r1, img(3));
  }
  lds_barrier();
  bf16x8 af[2], afn[2];
  if (n > 0) readA(0, 0, af);
  auto body = [&](auto h_c) {
    constexpr int H = decltype(h_c)::value;
    constexpr int NJ = H == 0 ? 5 : 4;
    auto image = [&](int i, Regs& rs) {
      const int cur = i % 3;
      if (i + 2 < n) {  // image i+2 (set rs) into the buffers image i-1 used; rs refilled with image i+4
        stage(rs, (i + 2) % 3);
        if (i + 4 < n) load(rs, img(i + 4));
      }
      const int xb = (int)(Xb(cur) - reinterpret_cast<const bf16*>(smem)) + 16 * half + 4 * p;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int kb = ks * 32 + grp * 8;
        const int k0 = min(kb + q, 120), k1 = min(kb + 4 + q, 120);  // rows >= 121 of D are zero
        int x0 = xb + ((k0 / 11) * 13 + k0 % 11) * C2_XRS, x1 = xb + ((k1 / 11) * 13 + k1 % 11) * C2_XRS;
        asm("" : "+v"(x0), "+v"(x1));  // as conv3_wgrad8_role: one VGPR base + immediate tap offsets
        const bf16* S0 = reinterpret_cast<const bf16*>(smem);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int tap = 2 * j + H;
          const int shift = ((tap / 3) * 13 + tap % 3) * C2_XRS;
          const bf16x4 lo = lds_read_tr16(S0 + x0 + shift);
          const bf16x4 hi = lds_read_tr16(S0 + x1 + shift);
          const bf16x8 bf = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          if (j == 2) {  // next k-step's A fragments (image i+1's first after the last k-step); af and afn
                         // alternate by k-step parity, so nothing is copied
            if (ks < 3) {
              if (ks & 1)
                readA(cur, ks + 1, af);
              else
                readA(cur, ks + 1, afn);
            } else if (i + 1 < n) {
              readA((i + 1) % 3, 0, af);
            }
          }
#pragma unroll
          for (int m = 0; m < 2; ++m) acc[m][j] = mfma16x16x32((ks & 1) ? afn[m] : af[m], bf, acc[m][j]);
        }
        if (wn == 0) {
#pragma unroll
          for (int m = 0; m < 2; ++m) accb[m] = mfma16x16x32((ks & 1) ? afn[m] : af[m], onesf, accb[m]);
        }
      }
      lds_barrier();
    };
    for (int i = 0; i < n; i += 2) {  // unrolled by 2: register sets are not indexable
      image(i, r0);
      if (i + 1 < n) image(i + 1, r1);
    }
  };
  if (h == 0)
    body(std::integral_constant<int, 0>{});
  else
    body(std::integral_constant<int, 1>{});
  float* slab = slabs + (int64_t)slice * C2_WSLAB;
  const int nj = h == 0 ? 5 : 4;
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int co = (2 * wm2 + m) * 16 + grp * 4;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      if (j < nj) {
        const int nn = ((2 * j + h) * 2 + half) * 16 + g16;  // n-tile (tap, half)
        *reinterpret_cast<f32x4*>(slab + (int64_t)nn * 64 + co) = acc[m][j];
      }
    }
    if (wn == 0 && g16 == 0) *reinterpret_cast<f32x4*>(slab + 288 * 64 + co) = accb[m];
  }
}

template <bool U8>
__global__ __launch_bounds__(512, 1) void conv12_bwd8_kernel(const void* __restrict__ xin,
                                                            const uint8_t* __restrict__ idx1,
                                                            const bf16* __restrict__ a1,
                                                            const bf16* __restrict__ dz2,
                                                            const bf16* __restrict__ packed, int B, float mean,
                                                            float inv_std, float in_scale,
                                                            float* __restrict__ slabs2, int nslices,
                                                            float* __restrict__ slabs1, int n_dgrad, int ablate) {
  __shared__ __attribute__((aligned(16))) char smem[C12V_LDS];
  if ((int)blockIdx.x < n_dgrad)
    conv12_dgrad8_role<U8>(smem, xin, idx1, dz2, packed, B, blockIdx.x, n_dgrad, mean, inv_std, in_scale, slabs1,
                           ablate);
  else if (!(ablate & 4))
    conv2_wgrad8_role(smem, a1, dz2, slabs2, B, nslices, blockIdx.x - n_dgrad);
}

// ================================================================== fixed-order slab reductions
// ReduceSeg: kernels.h
constexpr int kMaxRedSegs = 8;
struct ReduceSegs {
  ReduceSeg seg[kMaxRedSegs];
  int count;
};

// Each workgroup owns 64 x vec outputs of one segment (vec = 4: one 16-B load per slice per lane) and sums
// its slices with 8 waves (coalesced rows, 4 loads in flight per wave), combined in a fixed order.  Several
// waves per output group because the conv1 / fc1 segments have few outputs and hundreds of slices; 4
// outputs per lane and 8 (was 16) waves cut the B=100 merged reduction's wave count 8x.
constexpr int kRedWaves = 8;
__device__ __forceinline__ void red_store(const ReduceSeg& sg, int64_t i, float v) {
  if (sg.mode == 0) {
    sg.out[i] = v;
  } else if (sg.mode == 2) {
    const int t = (int)(i & 255), nj = (int)(i >> 8), n = nj >> 3, j = nj & 7;
    sg.out[n * 2048 + ((t & 15) * 8 + j) * 16 + (t >> 4)] = v;
  } else {
    const int n = (int)(i / sg.cout), co = (int)(i % sg.cout);
    sg.out[((int64_t)co * sg.cin + n % sg.cin) * 9 + n / sg.cin] = v;
  }
}

__global__ __launch_bounds__(64 * kRedWaves) void slab_reduce_kernel(ReduceSegs segs) {
  __shared__ f32x4 part[kRedWaves][64];
  int blk = blockIdx.x, sidx = 0;
  while (sidx < segs.count - 1 && blk >= segs.seg[sidx].blocks) {
    blk -= segs.seg[sidx].blocks;
    ++sidx;
  }
  const ReduceSeg& sg = segs.seg[sidx];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int V = sg.vec;
  const int64_t i0 = ((int64_t)blk * 64 + lane) * V;
  f32x4 a0 = zero_f32x4(), a1 = zero_f32x4(), a2 = zero_f32x4(), a3 = zero_f32x4();
  if (i0 < sg.n) {
    const float* pp = sg.slabs + sg.off + i0;
    int s = wave;
    if (V == 4) {
      for (; s + 3 * kRedWaves < sg.nslices; s += 4 * kRedWaves) {
        a0 += *reinterpret_cast<const f32x4*>(pp + (int64_t)s * sg.stride);
        a1 += *reinterpret_cast<const f32x4*>(pp + (int64_t)(s + kRedWaves) * sg.stride);
        a2 += *reinterpret_cast<const f32x4*>(pp + (int64_t)(s + 2 * kRedWaves) * sg.stride);
        a3 += *reinterpret_cast<const f32x4*>(pp + (int64_t)(s + 3 * kRedWaves) * sg.stride);
      }
      for (; s < sg.nslices; s += kRedWaves) a0 += *reinterpret_cast<const f32x4*>(pp + (int64_t)s * sg.stride);
    } else {
      for (; s + 3 * kRedWaves < sg.nslices; s += 4 * kRedWaves) {
        a0[0] += pp[(int64_t)s * sg.stride];
        a1[0] += pp[(int64_t)(s + kRedWaves) * sg.stride];
        a2[0] += pp[(int64_t)(s + 2 * kRedWaves) * sg.stride];
        a3[0] += pp[(int64_t)(s + 3 * kRedWaves) * sg.stride];
      }
      for (; s < sg.nslices; s += kRedWaves) a0[0] += pp[(int64_t)s * sg.stride];
    }
  }
  part[wave][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (wave != 0 || i0 >= sg.n) return;
  f32x4 v = zero_f32x4();
#pragma unroll
  for (int w = 0; w < kRedWaves; ++w) v += part[w][lane];
  for (int k = 0; k < V; ++k) red_store(sg, i0 + k, v[k]);
}

ReduceSeg seg(const float* slabs, int64_t stride, int64_t off, int64_t n, int nslices, float* out,
              int mode = 0, int cin = 0, int cout = 0) {
  const int vec = ((off | stride | n) & 3) == 0 ? 4 : 1;
  return ReduceSeg{slabs, stride, off, n, nslices, out, mode, cin, cout, (int)((n + 64 * vec - 1) / (64 * vec)), vec};
}

void launch_reduce(const std::vector<ReduceSeg>& v, hipStream_t s) {
  if (v.empty()) return;
  if (v.size() > (size_t)kMaxRedSegs) {  // more than one launch holds: split
    launch_reduce(std::vector<ReduceSeg>(v.begin(), v.begin() + kMaxRedSegs), s);
    launch_reduce(std::vector<ReduceSeg>(v.begin() + kMaxRedSegs, v.end()), s);
    return;
  }
  ReduceSegs segs{};
  int total = 0;
  segs.count = (int)v.size();
  for (size_t k = 0; k < v.size(); ++k) {
    segs.seg[k] = v[k];
    total += v[k].blocks;
  }
  slab_reduce_kernel<<<total, 64 * kRedWaves, 0, s>>>(segs);
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

// largest batch whose fc1 backward runs inside the conv3 backward launch (RINGDP_CN_FC_IN_C3_MAX overrides)
int fc_in_c3_max_batch() {
  static const int v = [] {
    const char* e = std::getenv("RINGDP_CN_FC_IN_C3_MAX");
    return e ? std::atoi(e) : 2048;
  }();
  return v;
}

// largest batch whose fc1 runs inside the conv3 forward launch (RINGDP_CN_FC_FUSED_MAX overrides)
int fc_fused_max_batch() {
  static const int v = [] {
    const char* e = std::getenv("RINGDP_CN_FC_FUSED_MAX");
    return e ? std::atoi(e) : 4096;
  }();
  return v;
}

// workgroups per CU of a persistent forward kernel; RINGDP_CN_WPC_<name> overrides (A/B runs)
int wpc(const char* name, int dflt) {
  char key[64];
  std::snprintf(key, sizeof(key), "RINGDP_CN_WPC_%s", name);
  const char* v = std::getenv(key);
  return v ? std::max(1, std::atoi(v)) : dflt;
}

}  // namespace

// ================================================================== launchers
int64_t cn_packed_elems() { return PACK_TOTAL; }

void cn_pack_weights(const float* w1, const float* w2, const float* w3, const float* wfc, void* out,
                     hipStream_t s) {
  pack_weights_kernel<<<cdiv(PACK_TOTAL, 1024), 256, 0, s>>>(PackSrc{w1, w2, w3, wfc}, static_cast<bf16*>(out));
}

void cn_conv1_fwd(const void* x, bool u8, const void* packed, const float* b1, void* a1, uint8_t* idx1,
                  int B, float mean, float inv_std, float in_scale, hipStream_t s, const float* const* pack_w,
                  void* pack_out) {
  const int grid = clampi(B, 1, wpc("C1F", 3) * num_cus());  // 51 KiB LDS: 3 workgroups per CU
  const bf16* pk = static_cast<const bf16*>(packed);
  bf16* a1b = static_cast<bf16*>(a1);
  if (pack_w) {
    // + the pack workgroups (4 elements per thread): PACK_TOTAL / 1024 of them
    const PackSrc ws{pack_w[0], pack_w[1], pack_w[2], pack_w[3]};
    const int g = grid + cdiv(PACK_TOTAL, 1024);
    bf16* po = static_cast<bf16*>(pack_out);
    if (u8)
      conv1_fwd_kernel<true, true><<<g, 256, 0, s>>>(x, pk, b1, a1b, idx1, B, mean, inv_std, in_scale, ws, po, grid);
    else
      conv1_fwd_kernel<false, true><<<g, 256, 0, s>>>(x, pk, b1, a1b, idx1, B, mean, inv_std, in_scale, ws, po, grid);
    return;
  }
  const PackSrc none{nullptr, nullptr, nullptr, nullptr};
  if (u8)
    conv1_fwd_kernel<true, false><<<grid, 256, 0, s>>>(x, pk, b1, a1b, idx1, B, mean, inv_std, in_scale, none, nullptr, grid);
  else
    conv1_fwd_kernel<false, false><<<grid, 256, 0, s>>>(x, pk, b1, a1b, idx1, B, mean, inv_std, in_scale, none, nullptr, grid);
}

void cn_sgd_flat_pack(float* p, const float* g, float* m, int64_t n, const SgdArgs& a, const int64_t* offsets,
                      void* packed, hipStream_t s) {
  if (n <= 0) return;
  PackDst d{static_cast<bf16*>(packed), {offsets[0], offsets[1], offsets[2], offsets[3]}};
  const int grid = std::max<int64_t>(1, std::min<int64_t>((n / 4 + 256) / 256, 2048));
  if (m && a.momentum != 0.f)
    cn_sgd_pack_kernel<true><<<grid, 256, 0, s>>>(p, g, m, n, a, d);
  else
    cn_sgd_pack_kernel<false><<<grid, 256, 0, s>>>(p, g, m, n, a, d);
}

void cn_forward_fused(const void* x, bool u8, const float* const* w, const float* b1, const float* b2,
                      const float* b3, const float* bfc, void* packed, void* a1, uint8_t* idx1, void* a2,
                      uint8_t* idx2, void* a3, uint8_t* idx3, float* logits, int B, float mean, float inv_std,
                      float in_scale, unsigned* sync, hipStream_t s, bool do_pack) {
  const int conv = clampi(B, 1, wpc("FF", 1) * num_cus());  // 121 KiB LDS: one 512-thread workgroup per CU
  const PackSrc ws{w[0], w[1], w[2], w[3]};
  bf16* pk = static_cast<bf16*>(packed);
  bf16 *a1b = static_cast<bf16*>(a1), *a2b = static_cast<bf16*>(a2), *a3b = static_cast<bf16*>(a3);
  static const int ablate = [] { const char* v = getenv("RINGDP_FF_ABLATE"); return v ? atoi(v) : 0; }();
  static const int p2split = [] { const char* v = getenv("RINGDP_FF_P2"); const int n = v ? atoi(v) : 800;
                                  return n >= 0 && n <= 800 ? n : 800; }();
  // In-launch packing (RINGDP_FF_INPACK=1) is correct but slow on MI355X: the pack workgroups' agent-scope
  // release has to write their XCD's L2 back before the other XCDs may read the fragments (measured
  // B=100: 114 us against 23 us with the separate pack launch), so it is off by default.
  static const bool inpack = [] { const char* v = getenv("RINGDP_FF_INPACK"); return v && atoi(v) != 0; }();
  // Pack workgroups in this launch, the conv workgroups waiting for them, only while whole CUs stay
  // free for the pack workgroups: a conv workgroup takes a CU's entire register file (2 x 256 VGPRs per
  // SIMD), so with a conv workgroup on every CU the pack workgroups could never start.
  if (inpack && sync && conv <= num_cus() - 32) {
    const int grid = conv + cdiv(PACK_TOTAL, 1024);
    if (u8)
      fused_fwd_kernel<true, true><<<grid, 512, 0, s>>>(x, nullptr, ws, pk, conv, b1, b2, b3, bfc, a1b, idx1, a2b,
                                                        idx2, a3b, idx3, logits, B, mean, inv_std, in_scale, ablate,
                                                        sync, p2split);
    else
      fused_fwd_kernel<false, true><<<grid, 512, 0, s>>>(x, nullptr, ws, pk, conv, b1, b2, b3, bfc, a1b, idx1, a2b,
                                                         idx2, a3b, idx3, logits, B, mean, inv_std, in_scale, ablate,
                                                         sync, p2split);
    return;
  }
  // (do_pack false: the optimizer wrote these fragments when it last updated the weights)
  if (do_pack) pack_weights_kernel<<<cdiv(PACK_TOTAL, 1024), 256, 0, s>>>(ws, pk);
  const bool fc_in = B <= fc_fused_max_batch();  // else fc1 as its own MFMA pass over a3
  float* lg = fc_in ? logits : nullptr;
  if (u8)
    fused_fwd_kernel<true, false><<<conv, 512, 0, s>>>(x, pk, ws, nullptr, conv, b1, b2, b3, bfc, a1b, idx1, a2b,
                                                       idx2, a3b, idx3, lg, B, mean, inv_std, in_scale, ablate,
                                                       nullptr, p2split);
  else
    fused_fwd_kernel<false, false><<<conv, 512, 0, s>>>(x, pk, ws, nullptr, conv, b1, b2, b3, bfc, a1b, idx1, a2b,
                                                        idx2, a3b, idx3, lg, B, mean, inv_std, in_scale, ablate,
                                                        nullptr, p2split);
  if (!fc_in) fc1_fwd_kernel<<<cdiv(B, 16 * FC1_G), 256, 0, s>>>(a3b, pk, bfc, logits, B);
}

void cn_conv2_fwd(const void* a1, const void* packed, const float* b2, void* a2, uint8_t* idx2, int B,
                  hipStream_t s) {
  const int grid = clampi(B, 1, wpc("C2F", 3) * num_cus());  // 49 KiB LDS, 157 VGPRs: 3 per CU (303 -> 260 us)
  conv2_fwd_kernel<<<grid, 256, 0, s>>>(static_cast<const bf16*>(a1), static_cast<const bf16*>(packed), b2,
                                        static_cast<bf16*>(a2), idx2, B);
}

void cn_conv3_fc_fwd(const void* a2, const void* packed, const float* b3, const float* bfc, float* logits,
                     void* a3, uint8_t* idx3, int B, hipStream_t s) {
  const int grid = clampi(B, 1, wpc("C3F", 2) * num_cus());
  const bf16* a2b = static_cast<const bf16*>(a2);
  const bf16* pk = static_cast<const bf16*>(packed);
  if (B <= fc_fused_max_batch()) {
    conv3_fwd_kernel<true><<<grid, 256, 0, s>>>(a2b, pk, b3, static_cast<bf16*>(a3), idx3, B, bfc, logits);
    return;
  }
  conv3_fwd_kernel<false><<<grid, 256, 0, s>>>(a2b, pk, b3, static_cast<bf16*>(a3), idx3, B, nullptr, nullptr);
  fc1_fwd_kernel<<<cdiv(B, 16 * FC1_G), 256, 0, s>>>(static_cast<const bf16*>(a3), pk, bfc, logits, B);
}

// Work split of the role-fused backward launches.  All blocks of a launch are co-resident (one
// 512-thread block per CU), so dgrad and wgrad blocks are sized to finish together: dgrad does
// ~2x (conv3) / ~1.25x (conv2) the MFMA work of wgrad per image.
// Fraction of the CUs given to the dgrad role (RINGDP_C3_DGRAD_FRAC / RINGDP_C2_DGRAD_FRAC override
// the measured defaults; used for tuning sweeps).
static double split_frac(const char* env, double dflt) {
  const char* v = getenv(env);
  if (!v) return dflt;
  const double f = atof(v);
  return f > 0.05 && f < 0.95 ? f : dflt;
}

// fewest images per weight-gradient slab (small batches: more slabs = more reduction traffic)
static int min_slab_images(const char* env, int dflt) {
  const char* v = getenv(env);
  const int n = v ? atoi(v) : dflt;
  return n >= 1 && n <= 64 ? n : dflt;
}

// 8-wave conv3 backward (conv3_bwd8_kernel): batches above fc_in_c3_max_batch, RINGDP_C3_V3=0 keeps the
// 4-wave kernel (A/B)
static bool c3_v3(int B) {
  static const bool on = [] {
    const char* v = getenv("RINGDP_C3_V3");
    return !(v && v[0] == '0');
  }();
  return on && B > fc_in_c3_max_batch();
}

// timing-only ablations of the 8-wave conv3 backward (wrong results): bit 0 skips the pool2 backward,
// bit 1 the dgrad MFMA phase, bit 2 the weight gradient (RINGDP_C3_ABLATE)
static int c3_ablate() {
  static const int v = [] {
    const char* e = getenv("RINGDP_C3_ABLATE");
    return e ? atoi(e) : 0;
  }();
  return v;
}

// dgrad and wgrad do about the same MFMA work per image (624 / 576 MFMAs); measured best split 0.5-0.6 of
// the workgroup slots (B=32768).
static void c3_split(int B, bool dgrad, int& nd, int& ws) {
  if (c3_v3(B)) {  // one 512-thread workgroup per CU; ws = wgrad slices, one workgroup each
    const int cus = num_cus();
    if (!dgrad) {
      nd = 0;
      ws = clampi(cdiv(B, 8), 1, cus);
      return;
    }
    static const double frac = split_frac("RINGDP_C3_DGRAD_FRAC", 0.55);
    nd = clampi(((int)(frac * cus) + 4) / 8 * 8, 8, cus - 8);  // multiples of 8: see conv3_wgrad8_role
    ws = clampi(cdiv(B, 8), 1, cus - nd);
    return;
  }
  // 256-thread workgroups, two per CU; ws = image slices, each served by a pair of workgroups
  const int slots = 2 * num_cus();
  if (!dgrad) {
    nd = 0;
    ws = clampi(cdiv(B, 8), 1, slots / 2);
    return;
  }
  static const double frac = split_frac("RINGDP_C3_DGRAD_FRAC", 0.5);
  static const int wmin = min_slab_images("RINGDP_C3_WMIN", 2);
  nd = clampi(B, 1, (int)(frac * slots));
  const int per = cdiv(B, nd);
  ws = clampi(cdiv(B, std::max(per, wmin)), 1, std::max(1, (slots - nd) / 2));  // >= wmin images per slab
}

// Images [0, result) of the conv3 data gradient run on the dgrad workgroups, the rest on the wgrad
// workgroups after their weight-gradient slice (RINGDP_C3_STEAL = that share; large batches only, where
// each dgrad workgroup has many images).  0.07 (was 0.1): B=65536 step 3.304-3.315 -> 3.259-3.292 ms, three
// passes each of 0.06 / 0.07 / 0.08 all ahead of 0.1, 0.0 behind it (profiles/r06/c3_steal_sweep.txt).
static int c3_dgrad_images(int B, int nd) {
  static const double steal = [] {
    const char* v = getenv("RINGDP_C3_STEAL");
    const double f = v ? atof(v) : 0.07;
    return f >= 0.0 && f < 0.9 ? f : 0.07;
  }();
  if (nd <= 0 || B < 32 * nd) return B;
  return B - (int)(steal * B);
}

static void c2_split(int B, bool dgrad, int& nd, int& ws) {
  const int cus = num_cus();
  if (!dgrad) {
    nd = 0;
    ws = clampi(cdiv(B, 8), 1, cus);
    return;
  }
  static const double frac = split_frac("RINGDP_C2_DGRAD_FRAC", 0.55);
  nd = clampi(B, 1, (int)(frac * cus));
  const int per = cdiv(B, nd);
  ws = clampi(cdiv(B, std::max(per, 2)), 1, std::max(1, cus - nd));  // >= 2 images per slab
}

// fused conv2 backward + conv1 wgrad: the dgrad role also does conv1 wgrad (104 MFMAs per image on top
// of conv2 dgrad's 396; conv2 wgrad: 304)
// 8-wave conv2 backward + conv1 wgrad (conv12_bwd8_kernel): the conv3 bwd8 batches; RINGDP_C12_V3=0 keeps the
// 8-wave unpipelined kernel (A/B)
static bool c12_v3(int B) {
  static const bool on = [] {
    const char* v = getenv("RINGDP_C12_V3");
    return !(v && v[0] == '0');
  }();
  return on && B > fc_in_c3_max_batch();
}

// timing-only ablations of the 8-wave conv12 backward (wrong results): bit 0 skips conv1 wgrad, bit 1 the
// conv2 dgrad MFMAs, bit 2 the conv2 weight gradient (RINGDP_C12_ABLATE)
static int c12_ablate() {
  static const int v = [] {
    const char* e = getenv("RINGDP_C12_ABLATE");
    return e ? atoi(e) : 0;
  }();
  return v;
}

static void c12_split(int B, int& nd, int& ws) {
  const int cus = num_cus();
  if (c12_v3(B)) {
    static const double frac3 = split_frac("RINGDP_C12_DGRAD_FRAC", 0.65);
    nd = clampi(((int)(frac3 * cus) + 4) / 8 * 8, 8, cus - 8);  // multiples of 8: see conv2_wgrad8_role
    ws = clampi(cdiv(B, 8), 1, cus - nd);
    return;
  }
  static const double frac = split_frac("RINGDP_C12_DGRAD_FRAC", 0.64);
  static const int wmin = min_slab_images("RINGDP_C12_WMIN", 2);
  nd = clampi(B, 1, (int)(frac * cus));
  const int per = cdiv(B, nd);
  ws = clampi(cdiv(B, std::max(per, wmin)), 1, std::max(1, cus - nd));
}

static int conv1_wslices(int B) { return clampi(cdiv(B, 4), 1, 3 * num_cus()); }

// images per fc1-backward workgroup (RINGDP_CN_FC_IMGS overrides the table for A/B runs)
static int fc_imgs_host(int B) {
  static const int forced = [] {
    const char* v = getenv("RINGDP_CN_FC_IMGS");
    return v && *v ? atoi(v) : 0;
  }();
  return forced > 0 ? std::min(forced, 128) : fc_imgs(B);  // <= 128: the CE logits-gradient LDS block
}
int64_t cn_fc_slab_floats(int B, bool) { return (int64_t)cdiv(B, fc_imgs_host(B)) * FC_SLAB; }
int64_t cn_conv3_slab_floats(int B, bool dgrad) {
  int nd, ws;
  c3_split(B, dgrad, nd, ws);
  return (int64_t)ws * C3_WSLAB;
}
int64_t cn_conv2_slab_floats(int B, bool dgrad) {
  int nd, ws;
  c2_split(B, dgrad, nd, ws);
  return (int64_t)ws * C2_WSLAB;
}
int64_t cn_conv12_slab_floats(int B) {
  int nd, ws;
  c12_split(B, nd, ws);
  return (int64_t)ws * C2_WSLAB + (int64_t)nd * C1_WSLAB;
}
int64_t cn_conv1_slab_floats(int B) { return (int64_t)conv1_wslices(B) * C1_WSLAB; }

void cn_conv3_fc_bwd(const void* a2, const uint8_t* idx2, const void* a3, const uint8_t* idx3, const float* wfc,
                     const float* dl, const void* packed, void* da3m, void* dz2, int B, float* fc_slabs,
                     float* c3_slabs, float* dw3, float* db3, float* dwfc, float* dbfc, hipStream_t s,
                     const CeFuse* ce, ReduceList* defer) {
  (void)wfc;  // the data gradient uses the packed bf16 copy, like every other dgrad
  int nd, ws;
  c3_split(B, dz2 != nullptr, nd, ws);
  const int fs = cdiv(B, fc_imgs_host(B));
  const bf16* a3b = static_cast<const bf16*>(a3);
  const bf16* pk = static_cast<const bf16*>(packed);
  const CeFuse cef = ce ? *ce : CeFuse{};
  if (B <= fc_in_c3_max_batch()) {  // fc1 backward inside the conv3 backward launch
    const C3Src src{nullptr, a3b, pk, ce ? nullptr : dl, cef};
    conv3_bwd_kernel<true><<<fs + nd + 2 * ws, 256, 0, s>>>(static_cast<const bf16*>(a2), idx2, src, idx3, pk,
                                                             static_cast<bf16*>(dz2), B, c3_slabs, ws, nd,
                                                             c3_dgrad_images(B, nd), fs, fc_slabs, fc_imgs_host(B));
  } else {
    if (ce)
      fc_bwd_kernel<true><<<fs, 256, 0, s>>>(a3b, pk, nullptr, static_cast<bf16*>(da3m), fc_slabs, B, fc_imgs_host(B), cef);
    else
      fc_bwd_kernel<false><<<fs, 256, 0, s>>>(a3b, pk, dl, static_cast<bf16*>(da3m), fc_slabs, B, fc_imgs_host(B), cef);
    if (c3_v3(B)) {
      conv3_bwd8_kernel<<<nd + ws, 512, 0, s>>>(static_cast<const bf16*>(a2), idx2, static_cast<const bf16*>(da3m), idx3,
                                               pk, static_cast<bf16*>(dz2), B, c3_slabs, ws, nd, c3_dgrad_images(B, nd),
                                               c3_ablate());
    } else {
      const C3Src src{static_cast<const bf16*>(da3m), a3b, pk, dl, cef};
      conv3_bwd_kernel<false><<<nd + 2 * ws, 256, 0, s>>>(static_cast<const bf16*>(a2), idx2, src, idx3, pk,
                                                         static_cast<bf16*>(dz2), B, c3_slabs, ws, nd,
                                                         c3_dgrad_images(B, nd), 0, nullptr, 0);
    }
  }
  ReduceList r{seg(c3_slabs, C3_WSLAB, 0, 576 * 128, ws, dw3, 1, 64, 128),
               seg(fc_slabs, FC_SLAB, 20490, 128, fs, db3), seg(fc_slabs, FC_SLAB, 0, 20480, fs, dwfc, 2),
               seg(fc_slabs, FC_SLAB, 20480, 10, fs, dbfc)};
  if (defer)
    defer->insert(defer->end(), r.begin(), r.end());
  else
    launch_reduce(r, s);
}

void cn_launch_reduce(const ReduceList& segs, hipStream_t s) { launch_reduce(segs, s); }

void cn_conv2_bwd(const void* a1, const void* dz2, const void* packed, void* da1, int B, float* slabs,
                  float* dw2, float* db2, hipStream_t s) {
  int nd, ws;
  c2_split(B, da1 != nullptr, nd, ws);
  conv2_bwd_kernel<<<nd + ws, 512, 0, s>>>(static_cast<const bf16*>(a1), static_cast<const bf16*>(dz2),
                                           static_cast<const bf16*>(packed), static_cast<bf16*>(da1), B, slabs,
                                           ws, nd);
  launch_reduce({seg(slabs, C2_WSLAB, 0, 288 * 64, ws, dw2, 1, 32, 64), seg(slabs, C2_WSLAB, 288 * 64, 64, ws, db2)},
                s);
}

void cn_conv12_bwd(const void* x, bool u8, const uint8_t* idx1, const void* a1, const void* dz2,
                   const void* packed, int B, float mean, float inv_std, float in_scale, float* slabs, float* dw2,
                   float* db2, float* dw1, float* db1, hipStream_t s, const ReduceList* extra) {
  int nd, ws;
  c12_split(B, nd, ws);
  float* slabs2 = slabs;
  float* slabs1 = slabs + (int64_t)ws * C2_WSLAB;
  const bf16* a1b = static_cast<const bf16*>(a1);
  const bf16* dzb = static_cast<const bf16*>(dz2);
  const bf16* pk = static_cast<const bf16*>(packed);
  if (c12_v3(B)) {
    if (u8)
      conv12_bwd8_kernel<true><<<nd + ws, 512, 0, s>>>(x, idx1, a1b, dzb, pk, B, mean, inv_std, in_scale, slabs2, ws,
                                                       slabs1, nd, c12_ablate());
    else
      conv12_bwd8_kernel<false><<<nd + ws, 512, 0, s>>>(x, idx1, a1b, dzb, pk, B, mean, inv_std, in_scale, slabs2, ws,
                                                        slabs1, nd, c12_ablate());
  } else if (u8)
    conv12_bwd_kernel<true><<<nd + ws, 512, 0, s>>>(x, idx1, a1b, dzb, pk, B, mean, inv_std, in_scale, slabs2, ws,
                                                    slabs1, nd);
  else
    conv12_bwd_kernel<false><<<nd + ws, 512, 0, s>>>(x, idx1, a1b, dzb, pk, B, mean, inv_std, in_scale, slabs2, ws,
                                                     slabs1, nd);
  ReduceList r = extra ? *extra : ReduceList{};  // a deferred conv3 / fc1 reduction rides along
  for (const ReduceSeg& g : {seg(slabs2, C2_WSLAB, 0, 288 * 64, ws, dw2, 1, 32, 64),
                             seg(slabs2, C2_WSLAB, 288 * 64, 64, ws, db2), seg(slabs1, C1_WSLAB, 0, 800, nd, dw1),
                             seg(slabs1, C1_WSLAB, 800, 32, nd, db1)})
    r.push_back(g);
  launch_reduce(r, s);
}

void cn_conv1_wgrad(const void* x, bool u8, const void* da1, const uint8_t* idx1, int B, float mean,
                    float inv_std, float in_scale, float* slabs, float* dw1, float* db1, hipStream_t s) {
  const int ws = conv1_wslices(B);
  if (u8)
    conv1_wgrad_kernel<true><<<ws, 256, 0, s>>>(x, static_cast<const bf16*>(da1), idx1, B, mean, inv_std, in_scale,
                                                slabs, ws);
  else
    conv1_wgrad_kernel<false><<<ws, 256, 0, s>>>(x, static_cast<const bf16*>(da1), idx1, B, mean, inv_std, in_scale,
                                                 slabs, ws);
  launch_reduce({seg(slabs, C1_WSLAB, 0, 800, ws, dw1), seg(slabs, C1_WSLAB, 800, 32, ws, db1)}, s);
}

}  // namespace kern
}  // namespace ringdp
