// Per-tensor e4m3 (OCP, gfx950-native) quantisation for the fp8 GEMM path (BASELINE.json config 5,
// "ViT-B/16 ... fp8: CDNA4 fp8 MFMA GEMM path").
//   amax  : |x|max over a bf16 tensor (atomicMax on the float bits of non-negative values:
//           order-independent, so deterministic)
//   quant : scale = max(amax, tiny) / 448 (written to device memory for the GEMM epilogue),
//           q = cvt_e4m3(x / scale); optional transpose through a 64x64 LDS tile so every GEMM
//           operand (x^T, w^T, dy^T) is K-contiguous.  No host synchronisation anywhere.
//   delayed: (the training path, ringdp/ops/transformer.py) scale from the previous call's amax, rolled
//           from the per-tile maxima that call recorded; values clamped to +-448.
#include <algorithm>

#include "device_common.h"
#include "kernels.h"

namespace ringdp {
namespace kern {

using namespace ringdp::dev;

namespace {

constexpr float kE4M3Max = 448.f;

// One atomic per workgroup (not per wave) and at most 2 workgroups per CU: thousands of atomics on one
// address serialise in the L2 atomic unit (measured 82 us per call at 8192 wave-atomics).  Two
// 16-B loads in flight per thread.
__global__ __launch_bounds__(256) void amax_kernel(const bf16* __restrict__ x, int64_t nvec,
                                                   unsigned* __restrict__ out) {
  __shared__ float red[4];
  float m0 = 0.f, m1 = 0.f;
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; v + stride < nvec; v += 2 * stride) {
    const bf16x8 t0 = reinterpret_cast<const bf16x8*>(x)[v];
    const bf16x8 t1 = reinterpret_cast<const bf16x8*>(x)[v + stride];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      m0 = fmaxf(m0, fabsf((float)t0[j]));
      m1 = fmaxf(m1, fabsf((float)t1[j]));
    }
  }
  if (v < nvec) {
    const bf16x8 t0 = reinterpret_cast<const bf16x8*>(x)[v];
#pragma unroll
    for (int j = 0; j < 8; ++j) m0 = fmaxf(m0, fabsf((float)t0[j]));
  }
  float m = wave_max(fmaxf(m0, m1));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(out, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}

__device__ __forceinline__ float qscale(const float* amax) { return fmaxf(amax[0], 1e-12f) / kE4M3Max; }

__device__ __forceinline__ uint32_t pack4(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}

__global__ __launch_bounds__(256) void quant_kernel(const bf16* __restrict__ x, int64_t nvec,
                                                    const float* __restrict__ amax, uint8_t* __restrict__ out,
                                                    float* __restrict__ scale) {
  const float inv = 1.f / qscale(amax);
  if (blockIdx.x == 0 && threadIdx.x == 0) scale[0] = qscale(amax);
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    const bf16x8 t = reinterpret_cast<const bf16x8*>(x)[v];
    uint2 o;
    o.x = pack4((float)t[0] * inv, (float)t[1] * inv, (float)t[2] * inv, (float)t[3] * inv);
    o.y = pack4((float)t[4] * inv, (float)t[5] * inv, (float)t[6] * inv, (float)t[7] * inv);
    reinterpret_cast<uint2*>(out)[v] = o;
  }
}

// x [rows][cols] bf16 -> out [cols][rows] e4m3 (and, when out_rm != null, the row-major copy too:
// one read of x for both GEMM orientations); 128-row x 64-column tiles (rows, cols % 16 == 0).
// Each thread has 4 rows of 16-B loads in flight and converts its values once: the e4m3 bytes go to the
// row-major output and to a byte tile in LDS (68-B rows), from which each thread gathers 8 rows x 4
// columns and transposes them with 16 v_perm_b32 into 4 x 8 bytes of transposed output (the 16 lanes of
// one column group write 128 contiguous bytes per output row in one store instruction).  (The 64x64 version kept
// fp32 in LDS, converted twice and wrote 64-B segments: 2.9 TB/s; ViT-B/16 fp8 runs 144 of these passes.)
// Delayed scaling (amax_next != null): the scale comes from a previous amax, so values are clamped to
// the e4m3 range before conversion, and each tile's |x|max is stored to amax_next[tile] for the next
// call's roll - no separate amax pass over x.
// colsum != null: also this tile's 64 column sums of x (fp32, over its 128 rows; a fixed-order tree) to
// colsum[blockIdx.y][cols] - the bias gradient of a linear layer rides on the quantisation of dz.
// gpre (nullable): the tensor quantised is x * GELU'(gpre) - the GELU backward of an fp8 linear fused into
// the quantisation of its output gradient (the bf16 dz never reaches memory)
constexpr int kQT_R = 128, kQT_C = 64, kQT_RS = 68;  // 17-dword rows

__device__ __forceinline__ bf16x8 load_bf16x8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ bf16x8 load_bf16x8(const float* p) {  // fp32 master weights: the bf16 copy's values
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  return bf16x8{(bf16)a.x, (bf16)a.y, (bf16)a.z, (bf16)a.w, (bf16)b.x, (bf16)b.y, (bf16)b.z, (bf16)b.w};
}

// One 128 x 64 tile (bx, by) of the quantise(+transpose) pass; X = bf16 or fp32 (rounded to bf16 on load).
template <typename X>
__device__ __forceinline__ void quant_t_tile(const X* __restrict__ x, int64_t rows, int64_t cols,
                                             const float* __restrict__ amax, uint8_t* __restrict__ out,
                                             float* __restrict__ scale, uint8_t* __restrict__ out_rm,
                                             unsigned* __restrict__ amax_next, float* __restrict__ colsum,
                                             const bf16* __restrict__ gpre, int bx, int by, int gx) {
  __shared__ __attribute__((aligned(16))) uint8_t tile[kQT_R * kQT_RS];
  __shared__ float red[4];
  __shared__ float csum[4][64];
  const float inv = 1.f / qscale(amax);
  const float lim = amax_next ? kE4M3Max : INFINITY;
  float bmax = 0.f;
  if (bx == 0 && by == 0 && threadIdx.x == 0) scale[0] = qscale(amax);
  const int64_t r0 = (int64_t)by * kQT_R, c0 = (int64_t)bx * kQT_C;
  const int t = threadIdx.x, cv = t & 7, rr = t >> 3;
  const int64_t gc = c0 + cv * 8;
  bf16x8 v[4], pz[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int64_t gr = r0 + rr + 32 * p;
    v[p] = zero_bf16x8();
    pz[p] = zero_bf16x8();
    if (gr < rows && gc < cols) {
      v[p] = load_bf16x8(x + gr * cols + gc);
      if (gpre) pz[p] = *reinterpret_cast<const bf16x8*>(gpre + gr * cols + gc);
    }
  }
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int r = rr + 32 * p;
    const int64_t gr = r0 + r;
    float q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float f = (float)v[p][j];
      if (gpre) {  // the bf16 dz the unfused path would have stored, then quantised
        const float z = (float)pz[p][j];
        f = (float)(bf16)(f * (0.5f * (1.f + erff(z * 0.70710678118654752f)) +
                               z * 0.3989422804014327f * __expf(-0.5f * z * z)));
      }
      bmax = fmaxf(bmax, fabsf(f));
      cs[j] += f;
      q[j] = fminf(fmaxf(f * inv, -lim), lim);
    }
    uint2 o;
    o.x = pack4(q[0], q[1], q[2], q[3]);
    o.y = pack4(q[4], q[5], q[6], q[7]);
    uint32_t* tw = reinterpret_cast<uint32_t*>(tile + r * kQT_RS + cv * 8);  // 4-B aligned rows: two b32
    tw[0] = o.x;
    tw[1] = o.y;
    if (out_rm && gr < rows && gc < cols) *reinterpret_cast<uint2*>(out_rm + gr * cols + gc) = o;
  }
  __syncthreads();
  {  // transposed store: columns oc..oc+3 of rows rg*8 .. rg*8+7; the 16 lanes of one oc write 128
     // contiguous bytes of each of its 4 output rows (b32 tile reads: 2-way bank conflicts with 17-dword rows)
    const int rg = t & 15, oc = (t >> 4) * 4;
    uint32_t d[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = *reinterpret_cast<const uint32_t*>(tile + (rg * 8 + i) * kQT_RS + oc);
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
    const int64_t orow = r0 + rg * 8;
    if (orow < rows) {  // rows % 16 == 0: an 8-row group is all in or all out
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t oc_g = c0 + oc + j;
        if (oc_g < cols) *reinterpret_cast<uint2*>(out + oc_g * rows + orow) = make_uint2(col[0][j], col[1][j]);
      }
    }
  }
  if (colsum) {  // lanes with equal t & 7 hold the same 8 columns: xor 8 / 16 / 32, then the 4 waves
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      cs[j] += __shfl_xor(cs[j], 8, 64);
      cs[j] += __shfl_xor(cs[j], 16, 64);
      cs[j] += __shfl_xor(cs[j], 32, 64);
    }
    if ((t & 63) < 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) csum[t >> 6][(t & 7) * 8 + j] = cs[j];
    }
    __syncthreads();
    if (t < 64 && c0 + t < cols)
      colsum[(int64_t)by * cols + c0 + t] = (csum[0][t] + csum[1][t]) + (csum[2][t] + csum[3][t]);
  }
  if (amax_next) {  // this tile's |x|max -> its own slot (thousands of same-address atomics serialise)
    bmax = wave_max(bmax);
    if ((t & 63) == 0) red[t >> 6] = bmax;
    __syncthreads();
    if (t == 0)
      amax_next[by * gx + bx] = __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
  }
}

__global__ __launch_bounds__(256) void quant_t_kernel(const bf16* __restrict__ x, int64_t rows, int64_t cols,
                                                      const float* __restrict__ amax, uint8_t* __restrict__ out,
                                                      float* __restrict__ scale, uint8_t* __restrict__ out_rm,
                                                      unsigned* __restrict__ amax_next, float* __restrict__ colsum,
                                                      const bf16* __restrict__ gpre) {
  quant_t_tile(x, rows, cols, amax, out, scale, out_rm, amax_next, colsum, gpre, blockIdx.x, blockIdx.y, gridDim.x);
}

// Many fp32 matrices (a model's weights, delayed scaling) in one launch: the table is a kernel argument copied
// to LDS with compile-time indices (run-time indexing of the argument goes to scratch); block b belongs to
// the last entry whose first tile <= b.
__global__ __launch_bounds__(256) void quant_t_multi_kernel(QuantTTable tab) {
  __shared__ QuantTEntry se[kQuantTMax];
#pragma unroll
  for (int i = 0; i < kQuantTMax; ++i)
    if (threadIdx.x == i && i < tab.n) se[i] = tab.e[i];
  __syncthreads();
  int i = 0;
  while (i + 1 < tab.n && (int)blockIdx.x >= se[i + 1].tile0) ++i;
  const QuantTEntry& e = se[i];
  const int gx = (int)((e.cols + kQT_C - 1) / kQT_C);
  const int l = (int)blockIdx.x - e.tile0, by = l / gx, bx = l - by * gx;
  quant_t_tile(e.src, e.rows, e.cols, e.hist, e.qt, e.scale, e.q, reinterpret_cast<unsigned*>(e.hist + 1), nullptr,
               nullptr, bx, by, gx);
}

// Delayed-scaling roll: hist[0] (the amax the next quantisation scales by) <- max of the per-tile maxima
// hist[1 .. 1+n) the previous call of this site wrote (kept if they are all zero).
__global__ __launch_bounds__(1024) void amax_roll_kernel(float* __restrict__ hist, int n) {
  __shared__ float red[16];
  float m0 = 0.f, m1 = 0.f;  // 1024 threads, two loads in flight each (n is up to ~20k tile maxima)
  int i = threadIdx.x;
  for (; i + 1024 < n; i += 2048) {
    m0 = fmaxf(m0, hist[1 + i]);
    m1 = fmaxf(m1, hist[1 + i + 1024]);
  }
  if (i < n) m0 = fmaxf(m0, hist[1 + i]);
  const float m = wave_max(fmaxf(m0, m1));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f;
    for (int w = 0; w < 16; ++w) a = fmaxf(a, red[w]);
    if (a > 0.f) hist[0] = a;
  }
}

// amax_roll_kernel for many sites: workgroup i rolls hists[i] (n = ns[i] tile maxima)
__global__ __launch_bounds__(256) void amax_roll_many_kernel(float* const* __restrict__ hists, const int* __restrict__ ns) {
  __shared__ float red[4];
  float* hist = hists[blockIdx.x];
  const int n = ns[blockIdx.x];
  float m0 = 0.f, m1 = 0.f;
  int i = threadIdx.x;
  for (; i + 256 < n; i += 512) {
    m0 = fmaxf(m0, hist[1 + i]);
    m1 = fmaxf(m1, hist[1 + i + 256]);
  }
  if (i < n) m0 = fmaxf(m0, hist[1 + i]);
  const float m = wave_max(fmaxf(m0, m1));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float a = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (a > 0.f) hist[0] = a;
  }
}

// part[blockIdx.y][c] = sum of x[r][c] over rows [blockIdx.y * rows_per, +rows_per): 64 columns per block,
// 32 row lanes x 8 columns per thread, a fixed-order tree at the end (deterministic).
__global__ __launch_bounds__(256) void colsum_part_kernel(const bf16* __restrict__ x, int64_t rows, int64_t cols,
                                                          int64_t rows_per, float* __restrict__ part) {
  __shared__ float csum[4][64];
  const int t = threadIdx.x, cv = t & 7;
  const int64_t c = (int64_t)blockIdx.x * 64 + cv * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per, r1 = min(rows, r0 + rows_per);
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < cols) {
    for (int64_t r = r0 + (t >> 3); r < r1; r += 32) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + r * cols + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) cs[j] += (float)v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    cs[j] += __shfl_xor(cs[j], 8, 64);
    cs[j] += __shfl_xor(cs[j], 16, 64);
    cs[j] += __shfl_xor(cs[j], 32, 64);
  }
  if ((t & 63) < 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) csum[t >> 6][cv * 8 + j] = cs[j];
  }
  __syncthreads();
  const int64_t cc = (int64_t)blockIdx.x * 64 + t;
  if (t < 64 && cc < cols) part[(int64_t)blockIdx.y * cols + cc] = (csum[0][t] + csum[1][t]) + (csum[2][t] + csum[3][t]);
}

// out[c] = sum over s < S of part[s][c]: 64 columns per block as 16 float4 lanes x 16 row lanes (many
// partial rows - splitk_sum walks them serially per column), then a fixed-order tree (deterministic).
__global__ __launch_bounds__(256) void rowsum_f32_kernel(const float* __restrict__ part, int S, int64_t n,
                                                         float* __restrict__ out) {
  __shared__ f32x4 red[16][16];
  const int t = threadIdx.x, cl = t & 15, rl = t >> 4;
  const int64_t c = (int64_t)blockIdx.x * 64 + cl * 4;
  f32x4 a0 = zero_f32x4(), a1 = zero_f32x4();
  if (c < n) {
    int s = rl;
    for (; s + 16 < S; s += 32) {
      a0 += *reinterpret_cast<const f32x4*>(part + (int64_t)s * n + c);
      a1 += *reinterpret_cast<const f32x4*>(part + (int64_t)(s + 16) * n + c);
    }
    if (s < S) a0 += *reinterpret_cast<const f32x4*>(part + (int64_t)s * n + c);
  }
  red[rl][cl] = a0 + a1;
  __syncthreads();
  if (t < 16 && (int64_t)blockIdx.x * 64 + t * 4 < n) {
    f32x4 v = red[0][t];
    for (int r = 1; r < 16; ++r) v += red[r][t];
    *reinterpret_cast<f32x4*>(out + (int64_t)blockIdx.x * 64 + t * 4) = v;
  }
}

}  // namespace

void rowsum_f32(const float* part, int S, int64_t n, float* out, hipStream_t s) {
  rowsum_f32_kernel<<<(unsigned)((n + 63) / 64), 256, 0, s>>>(part, S, n, out);
}

int64_t fp8_quant_tiles(int64_t rows, int64_t cols) {
  return ((rows + kQT_R - 1) / kQT_R) * ((cols + kQT_C - 1) / kQT_C);
}
int64_t fp8_quant_row_tiles(int64_t rows) { return (rows + kQT_R - 1) / kQT_R; }

int colsum_parts(int64_t rows) { return (int)std::max<int64_t>(1, std::min<int64_t>(64, (rows + 255) / 256)); }

void colsum_bf16(const void* x, int64_t rows, int64_t cols, float* part, hipStream_t s) {
  const int parts = colsum_parts(rows);
  const int64_t rows_per = (rows + parts - 1) / parts;
  dim3 grid((unsigned)((cols + 63) / 64), (unsigned)parts);
  colsum_part_kernel<<<grid, 256, 0, s>>>(static_cast<const bf16*>(x), rows, cols, rows_per, part);
}

void fp8_amax(const void* x, int64_t n, float* amax, hipStream_t s) {
  hipMemsetAsync(amax, 0, sizeof(float), s);
  const int64_t nvec = n / 8;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((nvec + 255) / 256, 512));
  amax_kernel<<<grid, 256, 0, s>>>(static_cast<const bf16*>(x), nvec, reinterpret_cast<unsigned*>(amax));
}

void fp8_quantize(const void* x, int64_t rows, int64_t cols, bool transpose, const float* amax, void* out,
                  float* scale, hipStream_t s, void* out_rowmajor) {
  if (!transpose) {
    const int64_t nvec = rows * cols / 8;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((nvec + 255) / 256, 8192));
    quant_kernel<<<grid, 256, 0, s>>>(static_cast<const bf16*>(x), nvec, amax, static_cast<uint8_t*>(out), scale);
  } else {
    dim3 grid((unsigned)((cols + kQT_C - 1) / kQT_C), (unsigned)((rows + kQT_R - 1) / kQT_R));
    quant_t_kernel<<<grid, 256, 0, s>>>(static_cast<const bf16*>(x), rows, cols, amax, static_cast<uint8_t*>(out),
                                        scale, static_cast<uint8_t*>(out_rowmajor), nullptr, nullptr, nullptr);
  }
}

void fp8_quantize_delayed(const void* x, int64_t rows, int64_t cols, float* hist, bool init, void* out_t,
                          float* scale, void* out_rowmajor, hipStream_t s, float* colsum_part, const void* gelu_pre,
                          bool roll) {
  dim3 grid((unsigned)((cols + kQT_C - 1) / kQT_C), (unsigned)((rows + kQT_R - 1) / kQT_R));
  if (init)
    fp8_amax(x, rows * cols, hist, s);  // first use of the site: the exact amax of this tensor
  else if (roll)
    amax_roll_kernel<<<1, 1024, 0, s>>>(hist, (int)(grid.x * grid.y));
  quant_t_kernel<<<grid, 256, 0, s>>>(static_cast<const bf16*>(x), rows, cols, hist, static_cast<uint8_t*>(out_t),
                                      scale, static_cast<uint8_t*>(out_rowmajor), reinterpret_cast<unsigned*>(hist + 1),
                                      colsum_part, static_cast<const bf16*>(gelu_pre));
}

void fp8_quantize_multi(const QuantTTable& t, hipStream_t s) {
  if (t.n > 0 && t.total_tiles > 0) quant_t_multi_kernel<<<t.total_tiles, 256, 0, s>>>(t);
}

void fp8_roll(float* hist, int n, hipStream_t s) { amax_roll_kernel<<<1, 1024, 0, s>>>(hist, n); }

void fp8_roll_many(float* const* hists, const int* ns, int count, hipStream_t s) {
  if (count > 0) amax_roll_many_kernel<<<count, 256, 0, s>>>(hists, ns);
}

}  // namespace kern
}  // namespace ringdp
