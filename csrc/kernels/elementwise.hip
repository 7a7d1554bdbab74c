// ringdp elementwise / optimizer / loss kernels for CDNA4 (gfx950).
//
//  * SGD: one fused, float4-vectorised kernel over the DDP flat parameter range (replaces the
//    ~5 _foreach_* launches of torch's multi-tensor SGD); the math is
//    torch/optim/sgd.py:343-380 (wd, momentum/dampening, nesterov, maximize).
//  * split-K reduction used by every weight-gradient kernel (deterministic slice order).
//  * cross entropy forward (lse + mean loss, last-arriving workgroup reduces the partials in a
//    fixed order) and backward (softmax - target).
#include "device_common.h"
#include "kernels.h"
#include "sgd_device.h"

namespace ringdp {
namespace kern {

using namespace ringdp::dev;

namespace {

inline int grid_for(int64_t work, int block, int cap = 4096) {
  int64_t g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return static_cast<int>(g);
}

// out[c][r] = in[r][c] for a bf16 [R][C] matrix, through a 64x64 LDS tile (+2 pad: conflict-free
// column reads); 16-bit elements, 256 threads.
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const unsigned short* __restrict__ in,
                                                             unsigned short* __restrict__ out, int64_t R,
                                                             int64_t C) {
  __shared__ unsigned short tile[64][66];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int64_t r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < R && c < C) ? in[r * C + c] : (unsigned short)0;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int64_t c = c0 + i, r = r0 + tx;
    if (c < C && r < R) out[c * R + r] = tile[tx][i];
  }
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ src, bf16* __restrict__ dst, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = reinterpret_cast<const float4*>(src)[i];
    bf16x4 o = {(bf16)v.x, (bf16)v.y, (bf16)v.z, (bf16)v.w};
    reinterpret_cast<bf16x4*>(dst)[i] = o;
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dst[i] = (bf16)src[i];
}

// Many fp32 -> bf16 casts in one launch (a model's weights per forward): the table is a kernel
// argument copied to LDS with compile-time indices (run-time indexing of the argument goes to scratch);
// 4-element vectors, every tensor's length a multiple of 4 (checked on the host).
__global__ __launch_bounds__(256) void cast_multi_kernel(CastTable t) {
  __shared__ CastEntry se[kCastMax];
#pragma unroll
  for (int i = 0; i < kCastMax; ++i)
    if (threadIdx.x == i && i < t.n) se[i] = t.e[i];
  __syncthreads();
  int i = 0;  // v only grows, so the table scan resumes where the previous vector's ended
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < t.total4; v += (int64_t)gridDim.x * 256) {
    while (i + 1 < t.n && v >= se[i + 1].start4) ++i;
    const int64_t l = v - se[i].start4;
    const float4 x = reinterpret_cast<const float4*>(se[i].src)[l];
    reinterpret_cast<bf16x4*>(se[i].dst)[l] = bf16x4{(bf16)x.x, (bf16)x.y, (bf16)x.z, (bf16)x.w};
  }
}

// fp32 [R][C] -> bf16 [R][C] and its transpose bf16 [C][R], many matrices in one launch: block = one 64x64
// tile of some matrix (start_tile prefix in the table), read once, both outputs written coalesced (the
// transpose through LDS).  A linear layer's forward uses W, its data gradient W^T.
__global__ __launch_bounds__(256) void cast_t_multi_kernel(CastTTable t) {
  __shared__ CastTEntry se[kCastTMax];
  __shared__ float tile[64][65];
#pragma unroll
  for (int i = 0; i < kCastTMax; ++i)
    if (threadIdx.x == i && i < t.n) se[i] = t.e[i];
  __syncthreads();
  const int b = blockIdx.x;
  int i = 0;
  while (i + 1 < t.n && b >= se[i + 1].start_tile) ++i;
  const CastTEntry d = se[i];
  const int tiles_c = (d.C + 63) / 64;
  const int tb = b - d.start_tile;
  const int r0 = (tb / tiles_c) * 64, c0 = (tb % tiles_c) * 64;
  bf16* w = static_cast<bf16*>(d.dst);
  bf16* wt = static_cast<bf16*>(d.dst_t);
  if (r0 + 64 <= d.R && c0 + 64 <= d.C && (d.R & 3) == 0 && (d.C & 3) == 0) {
    // whole tile: 16-B loads, 8-B stores on both sides (16 lanes = one 128-B row segment); the scalar form
    // below moved ~2.7 TB/s
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int idx = threadIdx.x + 256 * k, rr = idx >> 4, c4 = (idx & 15) * 4;
      const int64_t o = (int64_t)(r0 + rr) * d.C + c0 + c4;
      const float4 x = *reinterpret_cast<const float4*>(d.src + o);
      *reinterpret_cast<bf16x4*>(w + o) = bf16x4{(bf16)x.x, (bf16)x.y, (bf16)x.z, (bf16)x.w};
      tile[rr][c4] = x.x;
      tile[rr][c4 + 1] = x.y;
      tile[rr][c4 + 2] = x.z;
      tile[rr][c4 + 3] = x.w;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int idx = threadIdx.x + 256 * k, cc = idx >> 4, r4 = (idx & 15) * 4;
      *reinterpret_cast<bf16x4*>(wt + (int64_t)(c0 + cc) * d.R + r0 + r4) =
          bf16x4{(bf16)tile[r4][cc], (bf16)tile[r4 + 1][cc], (bf16)tile[r4 + 2][cc], (bf16)tile[r4 + 3][cc]};
    }
    return;
  }
  for (int idx = threadIdx.x; idx < 64 * 64; idx += 256) {
    const int rr = idx >> 6, cc = idx & 63;
    const int r = r0 + rr, c = c0 + cc;
    float x = 0.f;
    if (r < d.R && c < d.C) {
      x = d.src[(int64_t)r * d.C + c];
      w[(int64_t)r * d.C + c] = (bf16)x;
    }
    tile[rr][cc] = x;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < 64 * 64; idx += 256) {
    const int cc = idx >> 6, rr = idx & 63;
    const int r = r0 + rr, c = c0 + cc;
    if (r < d.R && c < d.C) wt[(int64_t)c * d.R + r] = (bf16)tile[rr][cc];
  }
}

__global__ void cast_bf16_f32_kernel(const bf16* __restrict__ src, float* __restrict__ dst, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    bf16x4 v = reinterpret_cast<const bf16x4*>(src)[i];
    reinterpret_cast<float4*>(dst)[i] = make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dst[i] = (float)src[i];
}

__global__ void cast_f32_f16_kernel(const float* __restrict__ src, _Float16* __restrict__ dst, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dst[i] = (_Float16)src[i];
}

__global__ void cast_f16_f32_kernel(const _Float16* __restrict__ src, float* __restrict__ dst, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dst[i] = (float)src[i];
}

template <bool MOM>
__global__ __launch_bounds__(256) void sgd_flat_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                       float* __restrict__ m, int64_t n, SgdArgs a) {
  const SgdDev d = load_sgd(a);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = n / 4;
  float4 dummy = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = reinterpret_cast<float4*>(p)[i];
    float4 gv = reinterpret_cast<const float4*>(g)[i];
    float4 mv = MOM ? reinterpret_cast<float4*>(m)[i] : dummy;
    sgd_elem<MOM>(pv.x, gv.x, mv.x, d);
    sgd_elem<MOM>(pv.y, gv.y, mv.y, d);
    sgd_elem<MOM>(pv.z, gv.z, mv.z, d);
    sgd_elem<MOM>(pv.w, gv.w, mv.w, d);
    reinterpret_cast<float4*>(p)[i] = pv;
    if (MOM) reinterpret_cast<float4*>(m)[i] = mv;
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float pv = p[i], mv = MOM ? m[i] : 0.f;
    sgd_elem<MOM>(pv, g[i], mv, d);
    p[i] = pv;
    if (MOM) m[i] = mv;
  }
}

template <bool MOM>
__global__ __launch_bounds__(256) void sgd_multi_kernel(const SgdTensor* __restrict__ table,
                                                        const int64_t* __restrict__ chunks,
                                                        int64_t chunk_elems, SgdArgs a) {
  const SgdDev d = load_sgd(a);
  const int64_t t = chunks[2 * blockIdx.x];
  const int64_t start = chunks[2 * blockIdx.x + 1];
  const SgdTensor T = table[t];
  const int64_t end = start + chunk_elems < T.n ? start + chunk_elems : T.n;
  for (int64_t i = start + threadIdx.x; i < end; i += blockDim.x) {
    float pv = T.p[i], mv = MOM ? T.m[i] : 0.f;
    sgd_elem<MOM>(pv, T.g[i], mv, d);
    T.p[i] = pv;
    if (MOM) T.m[i] = mv;
  }
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ slabs, int S,
                                                            int64_t n, float* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if ((n & 3) == 0) {
    const int64_t n4 = n / 4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
      float4 acc = reinterpret_cast<const float4*>(slabs)[i];
      for (int s = 1; s < S; ++s) {
        float4 v = reinterpret_cast<const float4*>(slabs + (int64_t)s * n)[i];
        acc.x += v.x;
        acc.y += v.y;
        acc.z += v.z;
        acc.w += v.w;
      }
      reinterpret_cast<float4*>(out)[i] = acc;
    }
  } else {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      float acc = slabs[i];
      for (int s = 1; s < S; ++s) acc += slabs[(int64_t)s * n + i];
      out[i] = acc;
    }
  }
}

// ---------------------------------------------------------------- cross entropy
// Row loss: one lane per row for small C (the MNIST head: C = 10, no cross-lane work at all), one
// wave per row otherwise.  Per-block partial sums + an agent-scope last-arriver reduction that runs
// in a fixed order (deterministic, graph-capturable: the counter re-arms itself).
__device__ __forceinline__ float ce_row_loss(float lse, float xy, float sx, int C, float eps) {
  return (1.f - eps) * (lse - xy) + eps * (lse - sx / (float)C);
}

template <bool kSmallC>
__global__ __launch_bounds__(256) void ce_fwd_kernel(const float* __restrict__ logits,
                                                     const int64_t* __restrict__ labels, int B, int C,
                                                     int ignore_index, float eps, int reduction,
                                                     float* __restrict__ lse_out, float* __restrict__ loss,
                                                     float* __restrict__ partials, unsigned* counter,
                                                     int nparts) {
  __shared__ float s_sum[256], s_cnt[256];
  __shared__ int s_last;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float tsum = 0.f, tcnt = 0.f;
  if (kSmallC) {
    for (int r = blockIdx.x * 256 + tid; r < B; r += nparts * 256) {
      const float* x = logits + (int64_t)r * C;
      const int64_t y = labels[r];
      float mx = -INFINITY, sx = 0.f, xy = 0.f;
      for (int c = 0; c < C; ++c) {
        const float v = x[c];
        mx = fmaxf(mx, v);
        sx += v;
        xy = (c == y) ? v : xy;
      }
      float se = 0.f;
      for (int c = 0; c < C; ++c) se += __expf(x[c] - mx);
      const float lse = mx + __logf(se);
      const bool valid = y != ignore_index;
      const float l = valid ? ce_row_loss(lse, xy, sx, C, eps) : 0.f;
      lse_out[r] = lse;
      if (reduction == 0) loss[r] = l;
      tsum += l;
      tcnt += valid ? 1.f : 0.f;
    }
  } else {
    for (int r = blockIdx.x * 4 + wave; r < B; r += nparts * 4) {
      const float* x = logits + (int64_t)r * C;
      float mx = -INFINITY;
      for (int c = lane; c < C; c += 64) mx = fmaxf(mx, x[c]);
      mx = wave_max(mx);
      float se = 0.f, sx = 0.f;
      for (int c = lane; c < C; c += 64) {
        se += __expf(x[c] - mx);
        sx += x[c];
      }
      se = wave_sum(se);
      sx = wave_sum(sx);
      const float lse = mx + __logf(se);
      const int64_t y = labels[r];
      const bool valid = y != ignore_index;
      const float l = valid ? ce_row_loss(lse, x[y], sx, C, eps) : 0.f;
      if (lane == 0) {
        lse_out[r] = lse;
        if (reduction == 0) loss[r] = l;
        tsum += l;
        tcnt += valid ? 1.f : 0.f;
      }
    }
  }
  if (reduction == 0) return;
  s_sum[tid] = tsum;
  s_cnt[tid] = tcnt;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {  // fixed-shape tree: deterministic
    if (tid < off) {
      s_sum[tid] += s_sum[tid + off];
      s_cnt[tid] += s_cnt[tid + off];
    }
    __syncthreads();
  }
  if (nparts == 1) {  // one block (B <= 256 rows for small C): no cross-block hand-off, no fences
    if (tid == 0) {
      const float denom = reduction == 1 ? s_cnt[0] : 1.f;
      partials[2 * nparts] = denom;
      loss[0] = reduction == 1 ? s_sum[0] / denom : s_sum[0];
    }
    return;
  }
  if (tid == 0) {
    partials[2 * blockIdx.x] = s_sum[0];
    partials[2 * blockIdx.x + 1] = s_cnt[0];
    // Publish the partial (agent-scope release), then take a ticket; the last arriver reduces.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == (unsigned)nparts - 1);
    if (s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!s_last) return;
  float a = 0.f, c = 0.f;
  for (int i = tid; i < nparts; i += 256) {  // fixed assignment + fixed tree below: deterministic
    a += __builtin_nontemporal_load(&partials[2 * i]);
    c += __builtin_nontemporal_load(&partials[2 * i + 1]);
  }
  s_sum[tid] = a;
  s_cnt[tid] = c;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (tid < off) {
      s_sum[tid] += s_sum[tid + off];
      s_cnt[tid] += s_cnt[tid + off];
    }
    __syncthreads();
  }
  if (tid == 0) {
    const float denom = reduction == 1 ? s_cnt[0] : 1.f;
    partials[2 * nparts] = denom;
    loss[0] = reduction == 1 ? s_sum[0] / denom : s_sum[0];
    __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ __launch_bounds__(256) void ce_bwd_kernel(const float* __restrict__ logits,
                                                     const int64_t* __restrict__ labels,
                                                     const float* __restrict__ lse,
                                                     const float* __restrict__ grad_out,
                                                     const float* __restrict__ denom, int B, int C,
                                                     int ignore_index, float eps, int reduction,
                                                     float* __restrict__ dlogits) {
  const int64_t n = (int64_t)B * C;
  const float scale_all = reduction == 0 ? 1.f : grad_out[0] / denom[0];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / C), c = (int)(i % C);
    const int64_t y = labels[r];
    float g = 0.f;
    if (y != ignore_index) {
      const float p = __expf(logits[i] - lse[r]);
      const float q = (c == y ? (1.f - eps) : 0.f) + eps / (float)C;
      g = (p - q) * (reduction == 0 ? grad_out[r] : scale_all);
    }
    dlogits[i] = g;
  }
}

// ---------------------------------------------------------------- synthetic data
__device__ __forceinline__ uint32_t hash32(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return (uint32_t)x;
}

__global__ void synth_u8_kernel(uint8_t* __restrict__ x, int64_t* __restrict__ labels, int B, int HW,
                                int num_classes, uint64_t seed) {
  const int64_t n = (int64_t)B * HW;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    x[i] = (uint8_t)(hash32(seed * 0x9E3779B97F4A7C15ULL + (uint64_t)i) & 0xff);
    if (i < B) labels[i] = (int64_t)(hash32(~seed + 0x1234567ULL * (uint64_t)(i + 1)) % num_classes);
  }
}

}  // namespace

void cast_f32_to_bf16(const float* src, void* dst, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  cast_f32_bf16_kernel<<<grid_for(n / 4 + 1, 256), 256, 0, s>>>(src, static_cast<bf16*>(dst), n);
}
void cast_t_multi(const CastTTable& t, hipStream_t s) {
  if (t.total_tiles > 0) cast_t_multi_kernel<<<t.total_tiles, 256, 0, s>>>(t);
}
void cast_f32_to_bf16_multi(const CastTable& t, hipStream_t s) {
  if (t.total4 > 0) cast_multi_kernel<<<grid_for(t.total4, 256), 256, 0, s>>>(t);
}
void cast_bf16_to_f32(const void* src, float* dst, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  cast_bf16_f32_kernel<<<grid_for(n / 4 + 1, 256), 256, 0, s>>>(static_cast<const bf16*>(src), dst, n);
}
void cast_f32_to_f16(const float* src, void* dst, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  cast_f32_f16_kernel<<<grid_for(n, 256), 256, 0, s>>>(src, static_cast<_Float16*>(dst), n);
}
void cast_f16_to_f32(const void* src, float* dst, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  cast_f16_f32_kernel<<<grid_for(n, 256), 256, 0, s>>>(static_cast<const _Float16*>(src), dst, n);
}

void sgd_flat(float* p, const float* g, float* m, int64_t n, const SgdArgs& a, hipStream_t s) {
  if (n <= 0) return;
  const int grid = grid_for(n / 4 + 1, 256, 2048);
  if (m && a.momentum != 0.f)
    sgd_flat_kernel<true><<<grid, 256, 0, s>>>(p, g, m, n, a);
  else
    sgd_flat_kernel<false><<<grid, 256, 0, s>>>(p, g, m, n, a);
}

void sgd_multi(const SgdTensor* table, const int64_t* chunks, int64_t nchunks, int64_t chunk_elems,
               const SgdArgs& a, hipStream_t s) {
  if (nchunks <= 0) return;
  if (a.momentum != 0.f)
    sgd_multi_kernel<true><<<(unsigned)nchunks, 256, 0, s>>>(table, chunks, chunk_elems, a);
  else
    sgd_multi_kernel<false><<<(unsigned)nchunks, 256, 0, s>>>(table, chunks, chunk_elems, a);
}

void transpose_bf16(const void* in, void* out, int64_t R, int64_t C, hipStream_t s) {
  if (R <= 0 || C <= 0) return;
  dim3 grid((unsigned)((C + 63) / 64), (unsigned)((R + 63) / 64));
  transpose_bf16_kernel<<<grid, 256, 0, s>>>(static_cast<const unsigned short*>(in), static_cast<unsigned short*>(out),
                                            R, C);
}

void splitk_reduce(const float* slabs, int nslices, int64_t n, float* out, hipStream_t s) {
  if (n <= 0) return;
  splitk_reduce_kernel<<<grid_for(n / 4 + 1, 256, 1024), 256, 0, s>>>(slabs, nslices, n, out);
}

void cross_entropy_fwd(const float* logits, const int64_t* labels, int B, int C, int ignore_index,
                       float label_smoothing, int reduction, float* lse, float* loss,
                       float* partials, unsigned* counter, int nparts, hipStream_t s) {
  if (C <= kCeSmallC)
    ce_fwd_kernel<true><<<nparts, 256, 0, s>>>(logits, labels, B, C, ignore_index, label_smoothing, reduction,
                                               lse, loss, partials, counter, nparts);
  else
    ce_fwd_kernel<false><<<nparts, 256, 0, s>>>(logits, labels, B, C, ignore_index, label_smoothing, reduction,
                                                lse, loss, partials, counter, nparts);
}

void cross_entropy_bwd(const float* logits, const int64_t* labels, const float* lse,
                       const float* grad_out, const float* denom, int B, int C, int ignore_index,
                       float label_smoothing, int reduction, float* dlogits, hipStream_t s) {
  const int64_t n = (int64_t)B * C;
  ce_bwd_kernel<<<grid_for(n, 256, 1024), 256, 0, s>>>(logits, labels, lse, grad_out, denom, B, C,
                                                       ignore_index, label_smoothing, reduction,
                                                       dlogits);
}

// Replay beacon: the last node of a captured step bumps a device counter and stores the new value
// (one vector store, system scope) into host-coherent memory, where the RCCL watchdog thread reads it
// without any HIP call.
__global__ void beacon_kernel(unsigned long long* __restrict__ dev_ctr, unsigned long long* host) {
  if (threadIdx.x != 0) return;
  const unsigned long long v = __hip_atomic_load(dev_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1ull;  // vector load
  __hip_atomic_store(dev_ctr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(host, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

void replay_beacon_mark(unsigned long long* dev_ctr, unsigned long long* host, hipStream_t s) {
  beacon_kernel<<<1, 64, 0, s>>>(dev_ctr, host);
}

void synth_u8_images(uint8_t* x, int64_t* labels, int B, int HW, int num_classes, uint64_t seed,
                     hipStream_t s) {
  const int64_t n = (int64_t)B * HW;
  synth_u8_kernel<<<grid_for(n, 256, 2048), 256, 0, s>>>(x, labels, B, HW, num_classes, seed);
}

}  // namespace kern
}  // namespace ringdp
