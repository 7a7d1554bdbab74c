// Epilogue shared by the 256x256 GEMM kernels (gemm_bf16_256.hip, gemm_fp8_256.hip): a lane holds
// 8 x 4 accumulator tiles of 16 x 16, each giving it C[m][n .. n+3] (the C^T MFMA orientation).
//
// Every global load the epilogue needs (bias, residual or the GELU-backward pre-activation) is issued
// before the first use: a load-wait-store chain per tile costs one L2/HBM round trip per tile, 32 in
// a row, which measured ~2x the whole 12-k-tile main loop on the ViT shapes (K = 768).
#pragma once

#include "device_common.h"
#include "kernels.h"

namespace ringdp {
namespace kern {


typedef unsigned int gemm_u32x4 __attribute__((ext_vector_type(4)));

// One 16-B output store in the cache flavour ep.store_cache: 0 plain (the line stays in the XCD's L2),
// 1 nontemporal (`nt`), 2 write-through `sc1` (the line leaves L2: the output does not evict the operand
// panels the next tiles read).  Asm stores end with s_nop 1 (their data VGPRs are read after issue).
__device__ __forceinline__ void gemm_st16(void* p, uint4 v, int flavour) {
  const gemm_u32x4 w = {v.x, v.y, v.z, v.w};
  if (flavour == 2) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
  } else if (flavour == 1) {
    __builtin_nontemporal_store(w, reinterpret_cast<gemm_u32x4*>(p));
  } else {
    *reinterpret_cast<uint4*>(p) = v;
  }
}

// 16-B output stores need whole 8-column runs, 16-B aligned rows and base
__device__ __forceinline__ bool wide_ok(const GemmEpilogue& ep, int N) {
  return N % 8 == 0 && ep.ldc % 8 == 0 && (reinterpret_cast<uintptr_t>(ep.C) & 15) == 0 && (ep.c_bstride % 8) == 0;
}

// erf to ~3e-7 absolute without branches (Abramowitz-Stegun 7.1.26 + hardware rcp / exp): ocml's erff
// takes two divergent polynomial paths on |x| < 1, which exec-masks both in every wave of an epilogue.
__device__ __forceinline__ float gemm_erf(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  return copysignf(1.f - p * t * __expf(-ax * ax), x);
}
__device__ __forceinline__ float gemm_gelu(float x) { return 0.5f * x * (1.f + gemm_erf(x * 0.70710678118654752f)); }
// GELU'(x) = Phi(x) + x phi(x): erf's exp(-(x/sqrt2)^2) IS exp(-x^2/2), so one exp serves both terms
// (one transcendental and 3 VALU fewer per element of the GELU-backward GEMM epilogue)
__device__ __forceinline__ float gemm_gelu_grad(float x) {
  const float e = __expf(-0.5f * x * x);
  const float ax = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float erf_abs = 1.f - p * t * e;  // erf(|x| / sqrt2)
  return 0.5f * (1.f + copysignf(erf_abs, x)) + x * 0.3989422804014327f * e;
}

// Epilogue flags as wave-uniform values: read through readfirstlane, so every branch on them is a scalar
// branch (kernel-argument structs can end up in VGPRs, and a branch on a VGPR value is exec-masked:
// every wave then runs every path of every element, the GELU's erf included).
struct EpiFlags {
  int act, mode;
  bool bias, res, pre, st_pre, q8;
};
__device__ __forceinline__ EpiFlags epi_flags(const GemmEpilogue& ep) {
  EpiFlags f;
  f.act = __builtin_amdgcn_readfirstlane(ep.act);
  f.mode = __builtin_amdgcn_readfirstlane(ep.store_mode);
  f.bias = __builtin_amdgcn_readfirstlane(ep.bias != nullptr ? 1 : 0) != 0;
  f.res = __builtin_amdgcn_readfirstlane(ep.residual != nullptr ? 1 : 0) != 0;
  f.pre = __builtin_amdgcn_readfirstlane(ep.preact != nullptr ? 1 : 0) != 0;
  f.st_pre = f.pre && f.act != 3;
  f.q8 = __builtin_amdgcn_readfirstlane(ep.q8 != nullptr ? 1 : 0) != 0;
  return f;
}

// value of one accumulator quad after scale, bias, [GELU backward], [pre-activation copy], residual, activation
template <int ACT>
__device__ __forceinline__ void epi_values(const dev::f32x4& a, float sa, const dev::f32x4& bias, const dev::bf16x4& side,
                                           bool has_res, float (&v)[4]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = fmaf(a[e], sa, bias[e]);
    if (ACT == 3) v[e] *= gemm_gelu_grad((float)side[e]);
  }
}
template <int ACT>
__device__ __forceinline__ void epi_finish(float (&v)[4], const dev::bf16x4& side, bool has_res) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (has_res) v[e] += (float)side[e];
    if (ACT == 1) v[e] = fmaxf(v[e], 0.f);
    else if (ACT == 2) v[e] = gemm_gelu(v[e]);
  }
}

__device__ __forceinline__ uint32_t gemm_pack_e4m3(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}

// e4m3 outputs (GemmEpilogue::q8).  The wave's 128 x 64 e4m3 tile goes to LDS as [128 rows][64 B] (16-B chunk
// c of row r at c ^ ((r >> 3) & 3)), from which it is stored row-major as 16-B row pieces and transposed as in
// quant_t_kernel (fp8.hip): a lane gathers 8 rows x 4 columns (b32 reads), 16 v_perm_b32 make 4 columns x 8
// rows, and the 16 lanes of one column group write 128 contiguous bytes of an output row.  M % 16 == 0 and
// N % 16 == 0 (checked by the launcher), so 16-B pieces and 8-row groups are wholly inside or outside.
template <bool QUAD, int ACT>
__device__ __forceinline__ void gemm256_store_q8(const dev::f32x4 (&acc)[8][4], const GemmEpilogue& ep,
                                                 const EpiFlags& fl, int M, int N, int mrow, int ncol, float sa,
                                                 char* lds_wave) {
  using namespace ringdp::dev;
  auto mof = [&](int i) { return QUAD ? mrow + (i >> 2) * 64 + 16 * (i & 3) : mrow + 16 * i; };
  auto nof = [&](int j) { return QUAD ? ncol + (j >> 1) * 32 + 16 * (j & 1) : ncol + 16 * j; };
  const int lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4;
  const float qs = fmaxf(ep.q8_amax[0], 1e-12f) / 448.f;  // the scale quant_t_kernel would use
  const float inv = 1.f / qs;
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) ep.q8_scale[0] = qs;
  const bool want_cs = __builtin_amdgcn_readfirstlane(ep.colsum_part != nullptr ? 1 : 0) != 0;
  f32x4 bias[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = nof(j);
    bias[j] = (fl.bias && n < N) ? *reinterpret_cast<const f32x4*>(ep.bias + n) : zero_f32x4();
  }
  const bool has_side = fl.res || ACT == 3;
  const bf16* side = static_cast<const bf16*>(fl.res ? ep.residual : ep.preact);
  float vmax = 0.f;
  float cs[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) cs[j][e] = 0.f;
  // side inputs (residual / GELU pre-activation) preloaded half a wave tile at a time: all 32 quads at once
  // next to the 128 accumulator registers spills
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    bf16x4 sv[4][4];
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sv[ii][j] = bf16x4{(bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
        if (has_side) {
          const int m = min(mof(4 * half + ii), M - 1), n = min(nof(j), N - 4);
          sv[ii][j] = *reinterpret_cast<const bf16x4*>(side + (int64_t)m * ep.ldc + n);
        }
      }
#pragma unroll
  for (int ii = 0; ii < 4; ++ii) {
    const int i = 4 * half + ii;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = mof(i), n = nof(j);
      const bool ok = m < M && n < N;
      float v[4];
      epi_values<ACT>(acc[i][j], sa, bias[j], sv[ii][j], fl.res, v);
      if (fl.st_pre && ok)
        *reinterpret_cast<bf16x4*>(static_cast<bf16*>(ep.preact) + (int64_t)m * ep.ldc + n) =
            bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      epi_finish<ACT>(v, sv[ii][j], fl.res);
      float q[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float vb = ok ? (float)(bf16)v[e] : 0.f;  // rows past M hold clamped-row garbage
        vmax = fmaxf(vmax, fabsf(vb));
        cs[j][e] += vb;
        q[e] = fminf(fmaxf(vb * inv, -448.f), 448.f);
      }
      // opaque running reductions: without these the unrolled max / sum chains are re-associated into trees
      // over all 128 values, which keeps every value (and its accumulator) live at once and spills
      asm volatile("" : "+v"(vmax), "+v"(cs[j][0]), "+v"(cs[j][1]), "+v"(cs[j][2]), "+v"(cs[j][3]));
      const int r = (QUAD ? (i >> 2) * 64 + 16 * (i & 3) : 16 * i) + fr;
      const int c = QUAD ? (j >> 1) * 32 + 16 * (j & 1) + 4 * fq : 16 * j + 4 * fq;  // byte column
      *reinterpret_cast<uint32_t*>(lds_wave + r * 64 + (((c >> 4) ^ ((r >> 3) & 3)) << 4) + (c & 15)) =
          gemm_pack_e4m3(q[0], q[1], q[2], q[3]);
    }
  }
  }
  const int m_base = mrow - fr, n_base = ncol - 4 * fq;  // the wave tile's first row / column
  // (each wave reads back only what it wrote: LDS executes one wave's operations in order)
#pragma unroll
  for (int k = 0; k < 8; ++k) {  // row-major: lane -> row 16k + lane / 4, 16-B piece lane & 3
    const int r = 16 * k + (lane >> 2), ch = lane & 3;
    const uint4 w = *reinterpret_cast<const uint4*>(lds_wave + r * 64 + ((ch ^ ((r >> 3) & 3)) << 4));
    const int m = m_base + r, n = n_base + 16 * ch;
    if (m < M && n < N) *reinterpret_cast<uint4*>(ep.q8 + (int64_t)m * N + n) = w;
  }
  {  // transposed: lane -> rows 8 rg .. 8 rg + 7, columns 16 p + 4 (lane >> 4) + 0..3
    const int rg = lane & 15;
    const int m = m_base + 8 * rg;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int oc = 16 * p + 4 * fq;
      uint32_t d[8];
#pragma unroll
      for (int ii = 0; ii < 8; ++ii) {
        const int r = 8 * rg + ii;
        d[ii] = *reinterpret_cast<const uint32_t*>(lds_wave + r * 64 + (((oc >> 4) ^ (rg & 3)) << 4) + (oc & 15));
      }
      uint32_t col[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t a = d[4 * h], b = d[4 * h + 1], c = d[4 * h + 2], e = d[4 * h + 3];
        const uint32_t ab_lo = __builtin_amdgcn_perm(b, a, 0x05010400u), ab_hi = __builtin_amdgcn_perm(b, a, 0x07030602u);
        const uint32_t ce_lo = __builtin_amdgcn_perm(e, c, 0x05010400u), ce_hi = __builtin_amdgcn_perm(e, c, 0x07030602u);
        col[h][0] = __builtin_amdgcn_perm(ce_lo, ab_lo, 0x05040100u);
        col[h][1] = __builtin_amdgcn_perm(ce_lo, ab_lo, 0x07060302u);
        col[h][2] = __builtin_amdgcn_perm(ce_hi, ab_hi, 0x05040100u);
        col[h][3] = __builtin_amdgcn_perm(ce_hi, ab_hi, 0x07060302u);
      }
      if (m < M) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int n = n_base + oc + jj;
          if (n < N) *reinterpret_cast<uint2*>(ep.q8t + (int64_t)n * M + m) = make_uint2(col[0][jj], col[1][jj]);
        }
      }
    }
  }
  vmax = wave_max(vmax);
  if (lane == 0) ep.q8_tmax[(int64_t)blockIdx.x * 8 + (threadIdx.x >> 6)] = vmax;
  if (want_cs) {  // the 16 lanes of one fq hold the same columns: xor 1 / 2 / 4 / 8 sums their rows
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = cs[j][e];
        t += __shfl_xor(t, 1, 64);
        t += __shfl_xor(t, 2, 64);
        t += __shfl_xor(t, 4, 64);
        t += __shfl_xor(t, 8, 64);
        cs[j][e] = t;
      }
    if (fr == 0) {
      float* row = ep.colsum_part + (int64_t)(m_base >> 7) * N;  // one partial row per 128-row wave tile
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = nof(j);
        if (n < N) *reinterpret_cast<f32x4*>(row + n) = f32x4{cs[j][0], cs[j][1], cs[j][2], cs[j][3]};
      }
    }
  }
}

// QUAD: the phased kernel's tile order (acc[qm*4 + mt][qn*2 + nt], quadrants of 64 rows x 32 cols);
// otherwise acc[i][j] covers rows mrow + 16 i, columns ncol + 16 j.
// lds_wave: this wave's 16 KiB of the kernel's LDS (free once the main loop's last barrier has passed):
// store mode 2 writes the wave's 128 x 64 bf16 tile there and stores it back as whole 128-B rows.
template <bool QUAD, int ACT, bool Q8, bool CS>
__device__ __forceinline__ void gemm256_store_impl(const dev::f32x4 (&acc)[8][4], const GemmEpilogue& ep,
                                                   const EpiFlags& fl, int M, int N, int bidx, int mrow, int ncol,
                                                   float scale, char* lds_wave) {
  using namespace ringdp::dev;
  auto mof = [&](int i) { return QUAD ? mrow + (i >> 2) * 64 + 16 * (i & 3) : mrow + 16 * i; };
  auto nof = [&](int j) { return QUAD ? ncol + (j >> 1) * 32 + 16 * (j & 1) : ncol + 16 * j; };
  const int64_t cb = (int64_t)bidx * ep.c_bstride;
  const float sa = scale * ep.alpha;
  if constexpr (Q8) {  // (the bf16 kernels compile without this path: it costs them registers)
    if (fl.q8) {  // before the full-tile preloads below: its own loads are staged by halves
      gemm256_store_q8<QUAD, ACT>(acc, ep, fl, M, N, mrow, ncol, sa, lds_wave);
      return;
    }
  }
  // ---- all loads first
  f32x4 bias[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = nof(j);
    bias[j] = (fl.bias && n < N) ? *reinterpret_cast<const f32x4*>(ep.bias + n) : zero_f32x4();
  }
  const bool has_side = fl.res || ACT == 3;
  const bf16* side = static_cast<const bf16*>(fl.res ? ep.residual : ep.preact);
  bf16x4 sv[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) sv[i][j] = bf16x4{(bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
  if (has_side) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = min(mof(i), M - 1), n = min(nof(j), N - 4);
        sv[i][j] = *reinterpret_cast<const bf16x4*>(side + cb + (int64_t)m * ep.ldc + n);
      }
  }
  if (ep.out_bf16 && fl.mode == 3) {  // probe: compute but never store
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  const int lane = threadIdx.x & 63;
  if (ep.out_bf16 && (fl.mode == 2 || fl.mode == 4) && wide_ok(ep, N)) {
    // final values -> bf16 -> LDS image [128 rows][64 cols] (128-B rows, 16-B chunk c of row r at c ^ (r & 7)),
    // then 8 lanes per row store whole 128-B rows
    const int fr = lane & 15, fq = lane >> 4;
    float cs[4][4];  // CS: column sums of the stored values over this lane's rows
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) cs[j][e] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = mof(i), n = nof(j);
        float v[4];
        epi_values<ACT>(acc[i][j], sa, bias[j], sv[i][j], fl.res, v);
        if (fl.st_pre && m < M && n < N)
          *reinterpret_cast<bf16x4*>(static_cast<bf16*>(ep.preact) + cb + (int64_t)m * ep.ldc + n) =
              bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
        epi_finish<ACT>(v, sv[i][j], fl.res);
        if constexpr (CS) {
          const bool ok = m < M && n < N;
#pragma unroll
          for (int e = 0; e < 4; ++e) cs[j][e] += ok ? (float)(bf16)v[e] : 0.f;
          asm volatile("" : "+v"(cs[j][0]), "+v"(cs[j][1]), "+v"(cs[j][2]), "+v"(cs[j][3]));  // (see the q8 path)
        }
        const int r = (QUAD ? (i >> 2) * 64 + 16 * (i & 3) : 16 * i) + fr;    // row in the wave tile
        const int c = QUAD ? (j >> 1) * 32 + 16 * (j & 1) + 4 * fq : 16 * j + 4 * fq;  // column
        *reinterpret_cast<bf16x4*>(lds_wave + r * 128 + ((((c >> 3) ^ (r & 7)) << 4) | ((c & 7) << 1))) =
            bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      }
    }
    // each wave reads back only what it wrote (LDS executes one wave's operations in order)
    const int m_base = mrow - fr, n_base = ncol - 4 * fq;  // the wave tile's first row / column
    // Row order rotated per wave tile: in lockstep, every wave of every block would write the same row
    // offset at the same moment, i.e. addresses a multiple of 128 rows apart - on a few memory channels.
    const int rot = ep.store_rot ? (((m_base >> 7) * 5 + (n_base >> 6) * 3) & 15) : 0;
    bf16* cbase = static_cast<bf16*>(ep.C) + cb;
#pragma unroll
    for (int k0 = 0; k0 < 16; ++k0) {
      const int k = (k0 + rot) & 15;
      const int r = 8 * k + (lane >> 3), ch = lane & 7;
      const uint4 w = *reinterpret_cast<const uint4*>(lds_wave + r * 128 + ((ch ^ (r & 7)) << 4));
      const int m = m_base + r, n = n_base + 8 * ch;
      if (m < M && n < N) {
        // probe mode 4: the whole epilogue, but every store goes to one 16-B sink (no HBM write traffic)
        void* dst = fl.mode == 4 ? ep.sink : static_cast<void*>(cbase + (int64_t)m * ep.ldc + n);
        gemm_st16(dst, w, ep.store_cache);
      }
    }
    if constexpr (CS) {  // the 16 lanes of one fq hold the same columns: xor 1 / 2 / 4 / 8 sums their rows
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float t = cs[j][e];
          t += __shfl_xor(t, 1, 64);
          t += __shfl_xor(t, 2, 64);
          t += __shfl_xor(t, 4, 64);
          t += __shfl_xor(t, 8, 64);
          cs[j][e] = t;
        }
      if (fr == 0) {
        float* row = ep.colsum_part + (int64_t)(m_base >> 7) * N;  // one partial row per 128-row wave tile
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = nof(j);
          if (n < N) *reinterpret_cast<f32x4*>(row + n) = f32x4{cs[j][0], cs[j][1], cs[j][2], cs[j][3]};
        }
      }
    }
    return;
  }
  if (ep.out_bf16 && fl.mode == 1 && wide_ok(ep, N)) {
    // lanes l and l ^ 16 (same row, adjacent 4-column groups) exchange one of their two vertically adjacent
    // tiles, so each stores 8 consecutive bf16 (16 B) instead of 4 (8 B)
    const bool upper = (lane >> 4) & 1;  // odd 4-column group: keeps the lower tile of the pair
#pragma unroll
    for (int i2 = 0; i2 < 8; i2 += 2) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = nof(j);
        unsigned pk[2][2];  // [tile of the pair][2 x packed bf16 pair]
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int i = i2 + t;
          const int m = mof(i);
          float v[4];
          epi_values<ACT>(acc[i][j], sa, bias[j], sv[i][j], fl.res, v);
          if (fl.st_pre && m < M && n < N)
            *reinterpret_cast<bf16x4*>(static_cast<bf16*>(ep.preact) + cb + (int64_t)m * ep.ldc + n) =
                bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
          epi_finish<ACT>(v, sv[i][j], fl.res);
          const bf16x4 q = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
          const unsigned* qu = reinterpret_cast<const unsigned*>(&q);
          pk[t][0] = qu[0];
          pk[t][1] = qu[1];
        }
        // the lower lane sends its upper tile, the upper lane its lower tile
        const unsigned s0 = upper ? pk[0][0] : pk[1][0], s1 = upper ? pk[0][1] : pk[1][1];
        const unsigned r0 = __shfl_xor(s0, 16, 64), r1 = __shfl_xor(s1, 16, 64);
        const int i = upper ? i2 + 1 : i2;
        const int m = mof(i);
        const int nc = upper ? n - 4 : n;  // first of the 8 columns this lane stores
        if (m < M && nc < N) {
          uint4 w;
          if (upper) w = make_uint4(r0, r1, pk[1][0], pk[1][1]);
          else w = make_uint4(pk[0][0], pk[0][1], r0, r1);
          gemm_st16(static_cast<bf16*>(ep.C) + cb + (int64_t)m * ep.ldc + nc, w, ep.store_cache);
        }
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = mof(i);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = nof(j);
      if (n >= N) continue;
      float v[4];
      epi_values<ACT>(acc[i][j], sa, bias[j], sv[i][j], fl.res, v);
      const int64_t off = cb + (int64_t)m * ep.ldc + n;
      if (fl.st_pre)
        *reinterpret_cast<bf16x4*>(static_cast<bf16*>(ep.preact) + off) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      epi_finish<ACT>(v, sv[i][j], fl.res);
      if (ep.out_bf16)
        *reinterpret_cast<bf16x4*>(static_cast<bf16*>(ep.C) + off) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      else
        *reinterpret_cast<f32x4*>(static_cast<float*>(ep.C) + off) = f32x4{v[0], v[1], v[2], v[3]};
    }
  }
}

// Q8: the e4m3-output path (GemmEpilogue::q8) is compiled in (the fp8 kernel); CS: the bf16 LDS-row store path
// also writes column-sum partials (ep.colsum_part; the launcher forces store mode 2)
template <bool QUAD, bool Q8 = false, bool CS = false>
__device__ __forceinline__ void gemm256_store(const dev::f32x4 (&acc)[8][4], const GemmEpilogue& ep, int M, int N,
                                              int zid, int bidx, int mrow, int ncol, float scale, char* lds_wave) {
  using namespace ringdp::dev;
  if (__builtin_amdgcn_readfirstlane(ep.mode) == GemmEpilogue::kSplitK) {
    auto mof = [&](int i) { return QUAD ? mrow + (i >> 2) * 64 + 16 * (i & 3) : mrow + 16 * i; };
    auto nof = [&](int j) { return QUAD ? ncol + (j >> 1) * 32 + 16 * (j & 1) : ncol + 16 * j; };
    float* out = ep.partial + (int64_t)zid * M * N;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = mof(i);
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = nof(j);  // N % 4 == 0 (checked by the launchers)
        if (n < N) *reinterpret_cast<f32x4*>(out + (int64_t)m * N + n) = acc[i][j] * scale;
      }
    }
    return;
  }
  const EpiFlags fl = epi_flags(ep);
  // one specialised body per activation: the per-element code holds no branch on the epilogue kind
  switch (fl.act) {
    case 1: gemm256_store_impl<QUAD, 1, Q8, CS>(acc, ep, fl, M, N, bidx, mrow, ncol, scale, lds_wave); break;
    case 2: gemm256_store_impl<QUAD, 2, Q8, CS>(acc, ep, fl, M, N, bidx, mrow, ncol, scale, lds_wave); break;
    case 3: gemm256_store_impl<QUAD, 3, Q8, CS>(acc, ep, fl, M, N, bidx, mrow, ncol, scale, lds_wave); break;
    default: gemm256_store_impl<QUAD, 0, Q8, CS>(acc, ep, fl, M, N, bidx, mrow, ncol, scale, lds_wave); break;
  }
}

// ------------------------------------------------------------------------------------------------
// Epilogue of the persistent kernels (gemm_bf16_256q): no LDS (the next tile's first k-tile is already
// landing there) and an EXACT number of store instructions per lane, gemm256_q_stores(ep): stores past the
// M / N edge go to ep.sink instead of being skipped, so the kernel can count them in its vmcnt waits.
// bf16 outputs need wide_ok (checked by the launcher).
__device__ __forceinline__ int gemm256_q_stores(const GemmEpilogue& ep) {
  if (ep.mode == GemmEpilogue::kSplitK || !ep.out_bf16) return 32;
  return (ep.preact && ep.act != 3) ? 48 : 16;
}

template <bool QUAD>
__device__ __forceinline__ void gemm256_store_q(const dev::f32x4 (&acc)[8][4], const GemmEpilogue& ep, int M, int N,
                                                int zid, int bidx, int mrow, int ncol, float scale) {
  using namespace ringdp::dev;
  auto mof = [&](int i) { return QUAD ? mrow + (i >> 2) * 64 + 16 * (i & 3) : mrow + 16 * i; };
  auto nof = [&](int j) { return QUAD ? ncol + (j >> 1) * 32 + 16 * (j & 1) : ncol + 16 * j; };
  char* sink = static_cast<char*>(ep.sink);
  if (ep.mode == GemmEpilogue::kSplitK || !ep.out_bf16) {
    float* out = ep.mode == GemmEpilogue::kSplitK ? ep.partial + (int64_t)zid * M * N
                                                   : static_cast<float*>(ep.C) + (int64_t)bidx * ep.c_bstride;
    const int64_t ld = ep.mode == GemmEpilogue::kSplitK ? N : ep.ldc;
    const bool plain = ep.mode == GemmEpilogue::kSplitK;
    f32x4 bias[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = nof(j);
      bias[j] = (!plain && ep.bias && n < N) ? *reinterpret_cast<const f32x4*>(ep.bias + n) : zero_f32x4();
    }
    const bf16* res = plain ? nullptr : static_cast<const bf16*>(ep.residual);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = mof(i);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = nof(j);
        const bool ok = m < M && n < N;
        f32x4 v = acc[i][j] * scale;
        if (!plain) {
          v = v * ep.alpha + bias[j];
          if (res && ok) {
            const bf16x4 r = *reinterpret_cast<const bf16x4*>(res + (int64_t)bidx * ep.c_bstride + (int64_t)m * ep.ldc + n);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += (float)r[e];
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (ep.act == 1) v[e] = fmaxf(v[e], 0.f);
            else if (ep.act == 2) v[e] = gemm_gelu(v[e]);
          }
        }
        void* dst = ok ? static_cast<void*>(out + (int64_t)m * ld + n) : static_cast<void*>(sink);
        gemm_st16(dst, __builtin_bit_cast(uint4, v), ep.store_cache);
      }
    }
    return;
  }
  const int64_t cb = (int64_t)bidx * ep.c_bstride;
  f32x4 bias[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = nof(j);
    bias[j] = (ep.bias && n < N) ? *reinterpret_cast<const f32x4*>(ep.bias + n) : zero_f32x4();
  }
  const bf16* side = static_cast<const bf16*>(ep.residual ? ep.residual : (ep.act == 3 ? ep.preact : nullptr));
  bf16x4 sv[8][4];
  if (side) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = min(mof(i), M - 1), n = min(nof(j), N - 4);
        sv[i][j] = *reinterpret_cast<const bf16x4*>(side + cb + (int64_t)m * ep.ldc + n);
      }
  }
  const bool store_pre = ep.preact && ep.act != 3;
  const int lane = threadIdx.x & 63;
  const bool upper = (lane >> 4) & 1;  // odd 4-column group: keeps the lower tile of the pair
#pragma unroll
  for (int i2 = 0; i2 < 8; i2 += 2) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = nof(j);
      unsigned pk[2][2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int i = i2 + t;
        const int m = mof(i);
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] * scale * ep.alpha + bias[j][e];
        if (ep.act == 3) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] *= gemm_gelu_grad((float)sv[i][j][e]);
        } else if (store_pre) {
          const bool ok = m < M && n < N;
          bf16x4* pd = ok ? reinterpret_cast<bf16x4*>(static_cast<bf16*>(ep.preact) + cb + (int64_t)m * ep.ldc + n)
                          : reinterpret_cast<bf16x4*>(sink);
          *pd = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
        }
        if (ep.residual) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)sv[i][j][e];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (ep.act == 1) v[e] = fmaxf(v[e], 0.f);
          else if (ep.act == 2) v[e] = gemm_gelu(v[e]);
        }
        const bf16x4 q = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
        const unsigned* qu = reinterpret_cast<const unsigned*>(&q);
        pk[t][0] = qu[0];
        pk[t][1] = qu[1];
      }
      const unsigned s0 = upper ? pk[0][0] : pk[1][0], s1 = upper ? pk[0][1] : pk[1][1];
      const unsigned r0 = __shfl_xor(s0, 16, 64), r1 = __shfl_xor(s1, 16, 64);
      const int i = upper ? i2 + 1 : i2;
      const int m = mof(i);
      const int nc = upper ? n - 4 : n;  // first of the 8 columns this lane stores
      uint4 w;
      if (upper) w = make_uint4(r0, r1, pk[1][0], pk[1][1]);
      else w = make_uint4(pk[0][0], pk[0][1], r0, r1);
      const bool ok = m < M && nc < N;
      uint4* dst = ok ? reinterpret_cast<uint4*>(static_cast<bf16*>(ep.C) + cb + (int64_t)m * ep.ldc + nc)
                      : reinterpret_cast<uint4*>(sink);
      gemm_st16(dst, w, ep.store_cache);
    }
  }
}

}  // namespace kern
}  // namespace ringdp
