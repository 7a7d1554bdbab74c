// CDNA4 (gfx950) device helpers shared by ringdp HIP kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ringdp {
namespace dev {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWave = 64;

__device__ __forceinline__ f32x4 mfma16x16x32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses row q / columns 4p..4p+3 of a
// 4x16 block of 16-bit elements; lane i receives column i of the 4 rows.
__device__ __forceinline__ bf16x4 lds_read_tr16(const bf16* lds_ptr) {
  i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) i16x4*)(lds_ptr));
  return __builtin_bit_cast(bf16x4, v);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ bf16x8 zero_bf16x8() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (bf16)0.0f;
  return z;
}

__device__ __forceinline__ f32x4 zero_f32x4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// XCD-aware block remap (bijective for any grid): blocks that share an XCD (id % 8) get a
// contiguous range of logical ids, so neighbouring tiles share the XCD's L2.
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int q = nblocks / 8, r = nblocks % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// tile id -> (tm, tn) of a tiles_m x tiles_n grid, group_m tile rows at a time (bijective): the tiles one
// XCD runs at once (consecutive ids after xcd_remap) then share group_m A panels and a few B panels in
// its L2 instead of 1 A panel and up to 32 B panels (row-major order)
__device__ __forceinline__ void grouped_tile(int t, int tiles_m, int tiles_n, int group_m, int& tm, int& tn) {
  if (group_m <= 1) {
    tm = t / tiles_n;
    tn = t - tm * tiles_n;
    return;
  }
  const int gsz = group_m * tiles_n, g = t / gsz, first = g * group_m;
  const int gm = min(tiles_m - first, group_m), w = t - g * gsz;
  tm = first + w % gm;
  tn = w / gm;
}

}  // namespace dev
}  // namespace ringdp
