// 256x256-tile e4m3 GEMM for the ViT-B/16 fp8 linears (BASELINE.json config 5):
//   C[m][n] = epilogue( scale_a * scale_b * sum_k A[m][k] * B[n][k] ),  A, B K-contiguous bytes.
//
// One 512-thread workgroup per CU (8 waves as 2 (M) x 4 (N), 128x64 outputs each, 32 accumulator tiles).
// Operand tiles (256 rows x 128 k-bytes = one v_mfma_scale_f32_16x16x128_f8f6f4 k-step) arrive by LDS-DMA
// (global_load_lds_dwordx4 issued from inline asm) into two 64 KiB stages; each wave waits for its own
// copies with a COUNTED vmcnt and a raw s_barrier publishes the stage, so the copy of tile k+2 stays in
// flight across the barriers of tile k+1 (an LDS-DMA the compiler can see would be drained by the
// vmcnt(0) that __syncthreads() carries).  The stage image is lane-linear (8 rows x 128 B per wave
// instruction); the XOR swizzle of the 16-B chunks (applied to the per-lane GLOBAL source address) is
// chunk c of row r at c ^ f(r), f(r) = (r & 6) | ((r >> 3) & 1).  A ds_read_b128 is serviced in four
// 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32); a fragment read puts rows r = 0..15 and
// chunks c, c ^ 2 in each, and its bank quad is 8 * (r & 1) + (c ^ f(r)): with f = r & 7 (rounds 1-3)
// rows r and r + 8 of one group collide (2-way, PMC: 4 conflict cycles per read, 51 M per 8192^3
// GEMM); with bit 3 of r folded into bit 0 the 16 lanes hit 16 distinct quads.  MFMA issue is bracketed by
// s_setprio(1) so a wave holding the matrix core is not interleaved with another's LDS reads.
//
// The generic 128x128 core (gemm.hip) measured 0.75-1.36 PF/s on these shapes, at 2 workgroups per CU
// with register-staged loads; this kernel trades occupancy for a deeper DMA pipeline and half the
// operand re-reads per FLOP.
#include <algorithm>
#include <cstdlib>

#include "device_common.h"
#include "gemm256_epilogue.h"
#include "kernels.h"

namespace ringdp {
namespace kern {

using namespace ringdp::dev;

namespace {

constexpr int TM = 256, TN = 256, TK = 128;  // TK in bytes (= e4m3 values)
constexpr int STAGE = (TM + TN) * TK;        // 64 KiB: A rows then B rows, 128 B each
constexpr int DMA_PER_WAVE = (TM + TN) * TK / 1024 / 8;  // 8 wave-instructions of 1 KiB per stage

typedef int i32x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }

// 16 B per lane global -> LDS at (wave-uniform base + lane * 16); M0 is set inside the asm.
__device__ __forceinline__ void glds16(const void* gsrc, const void* lds_wave_base) {
  const unsigned base = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)((const __attribute__((address_space(3))) char*)(lds_wave_base)));
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(base), "v"(gsrc) : "memory");
}

// chunk swizzle of stage row r (see the header); swz = 0: the round-3 r & 7 (A/B knob RINGDP_FP8_SWZ)
__device__ __forceinline__ int chunk_swz(int r, int swz) { return swz ? ((r & 6) | ((r >> 3) & 1)) : (r & 7); }

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__global__ __launch_bounds__(512, 1) void gemm_fp8_256_kernel(const uint8_t* __restrict__ A, int64_t lda,
                                                             int64_t a_bs, const uint8_t* __restrict__ B,
                                                             int64_t ldb, int64_t b_bs, GemmEpilogue ep, int M,
                                                             int N, int K, int tiles_m, int tiles_n, int splits,
                                                             int k_per_split, int swz, int group_m) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int per_z = tiles_m * tiles_n;
  const int zid = blockIdx.y;
  const int t = xcd_remap(blockIdx.x, per_z);
  int tm, tn;
  grouped_tile(t, tiles_m, tiles_n, group_m, tm, tn);  // L2 reuse across the XCD's concurrent tiles
  const int b = zid / splits, split = zid - b * splits;
  const int m0 = tm * TM, n0 = tn * TN;
  const int kbeg = split * k_per_split, kend = min(K, kbeg + k_per_split);
  const int nkt = max(0, (kend - kbeg) / TK);

  // this lane's 8 DMA sources per stage: wave instruction i = 8*wave + j covers stage rows 8*i .. 8*i+7
  // (A rows for i < 32, then B rows); lane -> row 8*i + (lane >> 3), physical chunk lane & 7 holding
  // logical chunk (lane & 7) ^ f(row)
  const uint8_t* src[DMA_PER_WAVE];
#pragma unroll
  for (int j = 0; j < DMA_PER_WAVE; ++j) {
    const int i = DMA_PER_WAVE * wave + j;
    const int r = 8 * (i & 31) + (lane >> 3);
    const int lc = (lane & 7) ^ chunk_swz(r, swz);
    if (i < 32) {
      const int row = min(m0 + r, M - 1);  // rows past the edge re-read the last one; dropped on store
      src[j] = A + (int64_t)b * a_bs + (int64_t)row * lda + kbeg + lc * 16;
    } else {
      const int row = min(n0 + r, N - 1);
      src[j] = B + (int64_t)b * b_bs + (int64_t)row * ldb + kbeg + lc * 16;
    }
  }
  auto issue = [&](int kt, int s) {
    char* st = smem + s * STAGE + DMA_PER_WAVE * wave * 1024;
#pragma unroll
    for (int j = 0; j < DMA_PER_WAVE; ++j) glds16(src[j] + (int64_t)kt * TK, st + j * 1024);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = zero_f32x4();

  // fragment byte offsets inside a stage: row R = tile row + (lane & 15) (R & 15 == lane & 15), chunks
  // 2*(lane>>4) and +1 (32 k-bytes per lane)
  const int c0 = 2 * (lane >> 4), fr = chunk_swz(lane & 15, swz);
  const int sw0 = ((c0 ^ fr) << 4), sw1 = (((c0 + 1) ^ fr) << 4);
  const int a_off = (wm * 128 + (lane & 15)) * TK;
  const int b_off = TM * TK + (wn * 64 + (lane & 15)) * TK;

  if (nkt > 0) issue(0, 0);
  if (nkt > 1) issue(1, 1);
  for (int kt = 0; kt < nkt; ++kt) {
    const int s = kt & 1;
    if (kt + 1 < nkt)
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // tile kt has landed; kt + 1 may be in flight
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();  // every wave's copies of tile kt are in LDS
    const char* st = smem + s * STAGE;
    i32x8 fb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const char* p = st + b_off + j * 16 * TK;
      const int4 lo = *reinterpret_cast<const int4*>(p + sw0);
      const int4 hi = *reinterpret_cast<const int4*>(p + sw1);
      fb[j] = i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    }
#pragma unroll
    for (int mh = 0; mh < 2; ++mh) {
      i32x8 fa[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const char* p = st + a_off + (4 * mh + i) * 16 * TK;
        const int4 lo = *reinterpret_cast<const int4*>(p + sw0);
        const int4 hi = *reinterpret_cast<const int4*>(p + sw1);
        fa[i] = i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)  // C^T tile: lane ends with 4 consecutive n of one m; unit block scales
          acc[4 * mh + i][j] =
              __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fb[j], fa[i], acc[4 * mh + i][j], 0, 0, 0, 127, 0, 127);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's fragment reads of stage s retired
    raw_barrier();                   // every wave is done reading stage s
    if (kt + 2 < nkt) issue(kt + 2, s);  // lands while tile kt + 1 computes
  }

  // ---------------- epilogue: lane holds C[m][n..n+3], m = m0 + wm*128 + 16i + (lane&15),
  //                  n = n0 + wn*64 + 16j + 4*(lane>>4)
  const int mrow = m0 + wm * 128 + (lane & 15);
  const int ncol = n0 + wn * 64 + 4 * (lane >> 4);
  const float dscale = (ep.scale_a ? ep.scale_a[0] : 1.f) * (ep.scale_b ? ep.scale_b[0] : 1.f);
  gemm256_store<false, true>(acc, ep, M, N, zid, b, mrow, ncol, dscale, smem + wave * 16384);
}

}  // namespace

int64_t gemm_fp8_q8_slots(int M, int N) { return (int64_t)((M + TM - 1) / TM) * ((N + TN - 1) / TN) * 8; }
int64_t gemm_fp8_colsum_part_rows(int M) { return (int64_t)((M + TM - 1) / TM) * 2; }

static int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}

bool gemm_fp8_256(const GemmOperand& A, const GemmOperand& Bop, int batch, int M, int N, int Kbytes,
                  const GemmEpilogue& ep, int splits, hipStream_t s) {
  // K-contiguous operands with 16-B aligned rows, whole 128-byte k-steps, whole 4-column runs, no
  // statistics epilogue (BN layers never run in fp8)
  if (ep.q8 && (M % 16 != 0 || N % 16 != 0 || batch != 1 || splits > 1 || ep.mode != GemmEpilogue::kStore))
    return false;
  if (A.row_contig || Bop.row_contig || Kbytes % TK != 0 || N % 4 != 0 || M <= 0 || N <= 0 || ep.stats ||
      A.ld % 16 != 0 || Bop.ld % 16 != 0 || (ep.mode != GemmEpilogue::kSplitK && ep.ldc % 4 != 0) ||
      reinterpret_cast<uintptr_t>(ep.bias) % 16 != 0)
    return false;
  const int tiles_m = (M + TM - 1) / TM, tiles_n = (N + TN - 1) / TN;
  splits = std::max(1, splits);
  int kps = (Kbytes + splits - 1) / splits;
  kps = (kps + TK - 1) / TK * TK;
  splits = (Kbytes + kps - 1) / kps;
  dim3 grid(tiles_m * tiles_n, batch * splits);
  static const int swz = env_int("RINGDP_FP8_SWZ", 1), group_m = env_int("RINGDP_FP8_GROUP_M", 4);
  GemmEpilogue e2 = ep;
  // bf16 output: 16-B stores after a lane exchange (mode 1) measured +0.8 % on the ViT-B/16 fp8 step over the
  // LDS-staged rows the bf16 kernels use (5957 / 5973 vs 5910 / 5928 img/s, profiles/r04/fp8/env_sweep.txt)
  static const int wide = env_int("RINGDP_FP8_WIDE_STORE", 1);
  e2.store_mode = wide % 10;
  e2.store_rot = wide < 10;
  e2.store_cache = gemm_store_cache();
  gemm_fp8_256_kernel<<<grid, 512, 0, s>>>(static_cast<const uint8_t*>(A.p), A.ld, A.bstride,
                                           static_cast<const uint8_t*>(Bop.p), Bop.ld, Bop.bstride, e2, M, N, Kbytes,
                                           tiles_m, tiles_n, splits, kps, swz, group_m);
  return true;
}

}  // namespace kern
}  // namespace ringdp
