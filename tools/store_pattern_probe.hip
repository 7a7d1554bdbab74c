// Output-tile store patterns of a 256x256-tile bf16 GEMM epilogue, measured alone (no compute): M x N
// bf16 written by one 512-thread workgroup per 256x256 tile (8 waves as 2 x 4, each owning 128 x 64).
//   0 rows8    each wave instruction = 8 rows x 128 B (the wave's 64 columns), rows in order
//   1 rows8rot the same, the wave's 16 row groups rotated by a per-tile offset
//   2 full2    the workgroup writes whole 512-B tile rows: each instruction = 2 rows x 512 B
//   3 full2rot the same, rows rotated per tile
//   4 lane16   16-B pieces, lane = row (16 rows x 4 pieces per instruction: the MFMA-fragment order)
//   5 fill     contiguous 1 KiB per instruction over the whole matrix (a memset shape)
// Persistent grid (one workgroup per CU looping over tiles) or one workgroup per tile.
// hipcc --offload-arch=gfx950 -O3 tools/store_pattern_probe.hip -o store_pattern_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
      std::exit(1);                                                                            \
    }                                                                                          \
  } while (0)

template <bool BIGLDS>
__global__ __launch_bounds__(512) void store_tiles(uint4* __restrict__ C, int M, int N, int tiles_n, int ntiles,
                                                   int mode, int persistent, int spin) {
  // BIGLDS: 128 KiB of LDS per workgroup (one per CU, as the 256x256 GEMM), touched so it is kept
  __shared__ uint4 pad[BIGLDS ? 8192 : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (BIGLDS) pad[tid] = make_uint4(tid, 0, 0, 0);
  if (spin) {  // stand-in for a tile's compute: `spin` x ~1000 cycles of dependent VALU
    float x = (float)tid;
    for (int i = 0; i < spin * 250; ++i) x = x * 0.999f + 0.5f;
    if (x == 12345.f) C[0] = make_uint4(1, 1, 1, 1);
  }
  const int wr = wave >> 2, wc = wave & 3;
  const uint4 v = make_uint4(tid, blockIdx.x, 1, 2);
  const int step = persistent ? gridDim.x : ntiles;
  for (int t = blockIdx.x; t < ntiles; t += step) {
    const int m0 = (t / tiles_n) * 256, n0 = (t % tiles_n) * 256;
    const int rot = (t * 7) & 15;
    if (mode == 0 || mode == 1) {
      for (int k0 = 0; k0 < 16; ++k0) {
        const int k = mode == 1 ? (k0 + rot) & 15 : k0;
        const int r = m0 + wr * 128 + 8 * k + (lane >> 3);
        const int c = n0 + wc * 64 + 8 * (lane & 7);
        if (r < M && c < N) C[((size_t)r * N + c) / 8] = v;
      }
    } else if (mode == 2 || mode == 3) {
      // 128 row pairs over 8 waves: wave w writes pairs w, w + 8, ..
      for (int k0 = 0; k0 < 16; ++k0) {
        const int k = mode == 3 ? (k0 + rot) & 15 : k0;
        const int r = m0 + 2 * (wave + 8 * k) + (lane >> 5);
        const int c = n0 + 8 * (lane & 31);
        if (r < M && c < N) C[((size_t)r * N + c) / 8] = v;
      }
    } else if (mode == 4) {
      for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 2; ++j) {
          const int r = m0 + wr * 128 + 16 * i + (lane & 15);
          const int c = n0 + wc * 64 + 32 * j + 8 * (lane >> 4);
          if (r < M && c < N) C[((size_t)r * N + c) / 8] = v;
        }
    } else if (mode == 5) {
      const size_t base = (size_t)t * 256 * 256 / 8;  // 8 KiB-contiguous chunks of the matrix
      for (int k = 0; k < 16; ++k) {
        const size_t i = base + (size_t)k * 512 + tid;
        if (i < (size_t)M * N / 8) C[i] = v;
      }
    }
  }
}

int main() {
  const int M = 25216, N = 3072;
  const int tiles_n = N / 256, ntiles = ((M + 255) / 256) * tiles_n;
  uint4* C;
  CK(hipMalloc(&C, (size_t)M * N * 2));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int cfg = 0; cfg < 8; ++cfg) {
    // cfg: bit 0 big LDS (1 WG per CU), bit 1 spin (~20 us of "compute" per tile), bit 2 skip stores
    const bool big = cfg & 1;
    const int spin = (cfg & 2) ? 40 : 0;
    const int mode = (cfg & 4) ? 6 : 2;
    const int persistent = 0;
    {
      const int grid = ntiles;
      auto launch = [&]() {
        if (big) store_tiles<true><<<grid, 512>>>(C, M, N, tiles_n, ntiles, mode, persistent, spin);
        else store_tiles<false><<<grid, 512>>>(C, M, N, tiles_n, ntiles, mode, persistent, spin);
      };
      for (int i = 0; i < 3; ++i) launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a));
      for (int i = 0; i < 20; ++i) launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      const double us = ms * 1000.0 / 20;
      std::printf("{\"big_lds\": %d, \"spin\": %d, \"stores\": %d, \"us\": %.1f}\n", (int)big, spin, mode != 6, us);
    }
  }
  return 0;
}
