// Device-side input pipeline: gather a batch from an HBM-resident uint8 dataset by sampler index,
// apply the reference's augmentation (zero-pad + random crop, horizontal flip) and ToTensor +
// Normalize, and write the model's input layout/dtype - one launch per batch.
//
// Parity: torchvision RandomCrop(size, padding) -> RandomHorizontalFlip -> ToTensor -> Normalize
// (ref/example_mp.py:56-70; SURVEY.md §2.2 R12, §2.4 U15 "HIP gather/normalize/augment kernel").
// Per-sample randomness comes from a counter-based hash of (seed, sample position), so a batch is
// reproducible and independent of launch geometry.
#include <algorithm>

#include "device_common.h"
#include "kernels.h"

namespace ringdp {
namespace kern {

using namespace ringdp::dev;

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// out_kind: 0 = float32, 1 = bf16, 2 = uint8 (no normalisation; crop/flip only)
template <int KIND>
__global__ __launch_bounds__(256) void gather_augment_kernel(const uint8_t* __restrict__ x,
                                                             const int64_t* __restrict__ labels,
                                                             const int64_t* __restrict__ idx, int B, int H,
                                                             int W, int C, int pad, int flip, AugNorm nrm,
                                                             uint64_t seed, int nhwc, void* __restrict__ out,
                                                             int64_t* __restrict__ yout) {
  const int64_t total = (int64_t)B * C * H * W;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    int b, c, h, w;
    if (nhwc) {
      c = (int)(e % C);
      int64_t r = e / C;
      w = (int)(r % W);
      r /= W;
      h = (int)(r % H);
      b = (int)(r / H);
    } else {
      w = (int)(e % W);
      int64_t r = e / W;
      h = (int)(r % H);
      r /= H;
      c = (int)(r % C);
      b = (int)(r / C);
    }
    const uint64_t rnd = mix64(seed ^ mix64((uint64_t)b));
    const int span = 2 * pad + 1;
    const int oy = pad ? (int)(rnd % span) : 0;
    const int ox = pad ? (int)((rnd >> 16) % span) : 0;
    const bool fl = flip && ((rnd >> 40) & 1);
    const int wc = fl ? (W - 1 - w) : w;
    const int sy = h + oy - pad, sx = wc + ox - pad;
    const int64_t src = idx[b];
    uint8_t v = 0;
    if (sy >= 0 && sy < H && sx >= 0 && sx < W) v = x[((src * H + sy) * W + sx) * C + c];
    if (KIND == 2) {
      static_cast<uint8_t*>(out)[e] = v;
    } else {
      const float f = ((float)v * (1.f / 255.f) - nrm.mean[c]) * nrm.inv_std[c];
      if (KIND == 0)
        static_cast<float*>(out)[e] = f;
      else
        static_cast<bf16*>(out)[e] = (bf16)f;
    }
    if (labels && c == 0 && h == 0 && w == 0) yout[b] = labels[src];
  }
}

}  // namespace

void gather_augment(const uint8_t* x, const int64_t* labels, const int64_t* idx, int B, int H, int W, int C,
                    int pad, bool flip, const AugNorm& nrm, uint64_t seed, bool nhwc, int out_kind, void* out,
                    int64_t* yout, hipStream_t s) {
  const int64_t total = (int64_t)B * C * H * W;
  if (total <= 0) return;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 8192);
  switch (out_kind) {
    case 0:
      gather_augment_kernel<0><<<grid, 256, 0, s>>>(x, labels, idx, B, H, W, C, pad, flip, nrm, seed, nhwc, out, yout);
      break;
    case 1:
      gather_augment_kernel<1><<<grid, 256, 0, s>>>(x, labels, idx, B, H, W, C, pad, flip, nrm, seed, nhwc, out, yout);
      break;
    default:
      gather_augment_kernel<2><<<grid, 256, 0, s>>>(x, labels, idx, B, H, W, C, pad, flip, nrm, seed, nhwc, out, yout);
  }
}

}  // namespace kern
}  // namespace ringdp
