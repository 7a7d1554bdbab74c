// 256x256-tile bf16 GEMM (ViT linears forward, pointwise-conv forward, and the long-K weight gradients):
//   C[m][n] = epilogue( sum_k A[m][k] * B[n][k] ),  A, B bf16 with K contiguous or row-contiguous.
//
// The bf16 twin of gemm_fp8_256.hip (same pipeline, same byte geometry): one 512-thread workgroup
// per CU (8 waves as 2 (M) x 4 (N), 128x64 outputs each, 32 accumulator tiles); operand tiles of
// 256 rows x 64 k (128 B per row = two v_mfma_f32_16x16x32_bf16 k-steps) arrive by LDS-DMA
// (global_load_lds_dwordx4 from inline asm) into two 64 KiB stages; each wave waits for its own
// copies with a COUNTED vmcnt and a raw s_barrier publishes the stage, so the copy of tile k+2 stays
// in flight across the barriers of tile k+1.  16-B chunk c of stage row r sits at c ^ (r & 7) (the
// XOR swizzle is applied to the per-lane global source address, since the DMA image is lane-linear),
// which keeps the fragment reads conflict-free.  MFMA issue is bracketed by s_setprio(1).
//
// The generic 128x128 core (gemm.hip) runs these shapes at 0.62-0.87 PF/s with two register-staged
// workgroups per CU; this kernel trades occupancy for a deeper DMA pipeline and half the operand
// re-reads per FLOP.
#include <algorithm>

#include "device_common.h"
#include "gemm256_epilogue.h"
#include "kernels.h"

namespace ringdp {
namespace kern {

using namespace ringdp::dev;

namespace {

constexpr int TM = 256, TN = 256, TK = 128;  // TK in bytes (= 64 bf16 values, two k-steps of 32)
constexpr int TKE = TK / 2;                  // k elements per tile
constexpr int STAGE = (TM + TN) * TK;        // 64 KiB: A rows then B rows, 128 B each
constexpr int DMA_PER_WAVE = (TM + TN) * TK / 1024 / 8;  // 8 wave-instructions of 1 KiB per stage


// 16 B per lane global -> LDS at (wave-uniform base + lane * 16); M0 is set inside the asm.
__device__ __forceinline__ void glds16(const void* gsrc, const void* lds_wave_base) {
  const unsigned base = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)((const __attribute__((address_space(3))) char*)(lds_wave_base)));
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(base), "v"(gsrc) : "memory");
}

// the same copy from a wave-uniform 64-bit base (SGPRs) plus a per-lane 32-bit byte offset
__device__ __forceinline__ void glds16s(uint32_t voff, const void* sbase, const void* lds_wave_base) {
  const unsigned base = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)((const __attribute__((address_space(3))) char*)(lds_wave_base)));
  const uint64_t sb = (uint64_t)(uintptr_t)sbase;
  // (readfirstlane returns int: go through uint32_t, or a low half >= 2^31 would sign-extend into the high one)
  const uint64_t sbu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)(sb >> 32)) << 32) |
                       (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)sb);
  // s_nop 4: the base SGPRs were just written by v_readfirstlane (VALU SGPR write -> VMEM base read);
  // s_nop 0: SALU M0 write -> LDS-DMA M0 read
  asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(base), "v"(voff), "s"(sbu) : "memory");
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Row-contiguous operand X (element (r, k) at k * ld + r; weight gradients sum over the token index,
// which is the ROW of both activations): its stage part is [64 k-rows][256 cols] (512 B rows, the same
// 32 KiB), filled by DMA instructions of two k-rows each, and read back with ds_read_b64_tr_b16, which
// hands lane i of a 16-lane group column i of a 4-row block: two reads give the 8 consecutive k of
// the MFMA operand.  32-B unit u of k-row r sits at u ^ f(r), f(r) = (r & 3) | ((r >> 3) & 1) << 2:
// a 32-lane half of a transposed read touches rows 8g+4h+{0..3} and 8(g+1)+4h+{0..3}, whose eight
// f values are distinct, so the half covers all 64 banks once (conflict-free).
__device__ __forceinline__ int tr_swz(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

// fragment of the 16-row sub-tile `unit` (0..15) for k-step ks: row-contiguous image
__device__ __forceinline__ bf16x8 frag_tr(const char* part, int unit, int ks, int tr_off, int f) {
  const bf16x4 lo = lds_read_tr16(reinterpret_cast<const bf16*>(part + tr_off + (32 * ks) * 512 + ((unit ^ f) << 5)));
  const bf16x4 hi =
      lds_read_tr16(reinterpret_cast<const bf16*>(part + tr_off + (32 * ks + 4) * 512 + ((unit ^ f) << 5)));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// A/B as bytes: lda / ldb / a_bs / b_bs / K / k_per_split in BYTES (2 per bf16 element).  AROW / BROW:
// the operand is row-contiguous (k-major); then M (resp. N) % 8 == 0 and its ld % 8 == 0.
template <bool AROW, bool BROW>
__global__ __launch_bounds__(512, 1) void gemm_bf16_256_kernel(const uint8_t* __restrict__ A, int64_t lda,
                                                              int64_t a_bs, const uint8_t* __restrict__ B,
                                                              int64_t ldb, int64_t b_bs, GemmEpilogue ep, int M,
                                                              int N, int K, int tiles_m, int tiles_n, int splits,
                                                              int k_per_split, int group_m) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int per_z = tiles_m * tiles_n;
  const int zid = blockIdx.y;
  const int t = xcd_remap(blockIdx.x, per_z);
  int tm, tn;
  grouped_tile(t, tiles_m, tiles_n, group_m, tm, tn);
  const int b = zid / splits, split = zid - b * splits;
  const int m0 = tm * TM, n0 = tn * TN;
  const int kbeg = split * k_per_split, kend = min(K, kbeg + k_per_split);
  const int nkt = max(0, (kend - kbeg) / TK);

  // this lane's 8 DMA sources per stage: wave instruction i = 8*wave + j (A part for i < 32, then B).
  // K-contiguous part: rows 8*i .. 8*i+7, lane -> row 8*i + (lane >> 3), physical chunk lane & 7 holding
  // logical chunk (lane & 7) ^ (row & 7).  Row-contiguous part: k-rows 2*i, 2*i+1, lane -> k-row
  // 2*i + (lane >> 5), 16-B chunk lane & 31 of the 512-B row, in unit (chunk >> 1) ^ f(k-row).
  const uint8_t* src[DMA_PER_WAVE];
#pragma unroll
  for (int j = 0; j < DMA_PER_WAVE; ++j) {
    const int i = DMA_PER_WAVE * wave + j;
    const bool a_part = i < 32;
    const bool row = a_part ? AROW : BROW;
    const uint8_t* base = a_part ? A + (int64_t)b * a_bs : B + (int64_t)b * b_bs;
    const int64_t ld = a_part ? lda : ldb;
    const int lim = a_part ? M : N, r0 = a_part ? m0 : n0;
    if (row) {
      const int kr = 2 * (i & 31) + (lane >> 5), c = lane & 31;
      const int col = min(r0 + (((c >> 1) ^ tr_swz(kr)) << 4) + 8 * (c & 1), lim - 8);  // past the edge: dropped
      src[j] = base + (int64_t)(kbeg / 2 + kr) * ld + (int64_t)col * 2;
    } else {
      const int r = 8 * (i & 31) + (lane >> 3);
      const int lc = (lane & 7) ^ (r & 7);
      const int rr = min(r0 + r, lim - 1);  // rows past the edge re-read the last one; dropped on store
      src[j] = base + (int64_t)rr * ld + kbeg + lc * 16;
    }
  }
  // bytes one k-tile advances this wave's sources (wave-uniform: waves 0-3 copy A, 4-7 copy B)
  const int64_t kstep = wave < 4 ? (AROW ? 64 * lda : TK) : (BROW ? 64 * ldb : TK);
  auto issue = [&](int kt, int s) {
    char* st = smem + s * STAGE + DMA_PER_WAVE * wave * 1024;
#pragma unroll
    for (int j = 0; j < DMA_PER_WAVE; ++j) glds16(src[j] + (int64_t)kt * kstep, st + j * 1024);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = zero_f32x4();

  // fragment byte offsets inside a stage: row R = tile row + (lane & 15) (R & 7 == lane & 7); k-step s
  // reads logical chunk 4s + (lane >> 4) (8 bf16 = k 32s + 8*(lane>>4) .. +7)
  const int sw0 = ((((lane >> 4)) ^ (lane & 7)) << 4), sw1 = (((4 + (lane >> 4)) ^ (lane & 7)) << 4);
  const int a_off = (wm * 128 + (lane & 15)) * TK;
  const int b_off = TM * TK + (wn * 64 + (lane & 15)) * TK;
  // transposed reads: lane 4q+p of group g addresses k-row 8g + q (+32 ks, +4 for the upper half),
  // columns 4p .. 4p+3 of the sub-tile's 32-B unit; f(k-row) depends only on q and g & 1
  const int tr_g = lane >> 4, tr_q = (lane >> 2) & 3;
  const int tr_off = (8 * tr_g + tr_q) * 512 + 8 * (lane & 3);
  const int tr_f = tr_q | ((tr_g & 1) << 2);

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
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int sw = ks ? sw1 : sw0;
      bf16x8 fb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fb[j] = BROW ? frag_tr(st + TM * TK, wn * 4 + j, ks, tr_off, tr_f)
                     : *reinterpret_cast<const bf16x8*>(st + b_off + j * 16 * TK + sw);
#pragma unroll
      for (int mh = 0; mh < 2; ++mh) {
        bf16x8 fa[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          fa[i] = AROW ? frag_tr(st, wm * 8 + 4 * mh + i, ks, tr_off, tr_f)
                       : *reinterpret_cast<const bf16x8*>(st + a_off + (4 * mh + i) * 16 * TK + sw);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)  // C^T tile: lane ends with 4 consecutive n of one m
            acc[4 * mh + i][j] = mfma16x16x32(fb[j], fa[i], acc[4 * mh + i][j]);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's fragment reads of stage s retired
    raw_barrier();                   // every wave is done reading stage s
    if (kt + 2 < nkt) issue(kt + 2, s);  // lands while tile kt + 1 computes
  }

  // ---------------- epilogue: lane holds C[m][n..n+3], m = m0 + wm*128 + 16i + (lane&15),
  //                  n = n0 + wn*64 + 16j + 4*(lane>>4)
  gemm256_store<false>(acc, ep, M, N, zid, b, m0 + wm * 128 + (lane & 15), n0 + wn * 64 + 4 * (lane >> 4), 1.f,
                       smem + wave * 16384);
}

// ------------------------------------------------------------------------------------------------
// K-contiguous A and B: the phased pipeline.  Each 64-k tile is computed in 4 phases, one per
// (64-row x 32-col) quadrant of the wave's 128 x 64 outputs, in the order q00 q01 q11 q10.  The tile's
// operands live in four 16 KiB half-tiles, grouped by the phase that first reads them:
//   A-lo = tile rows {0-63, 128-191}     (quadrant row 0 of both wave rows: read in phase 0)
//   B-lo = tile cols {0-31, 64-95, ...}  (quadrant col 0 of the four wave columns: phase 0)
//   B-hi = the other 128 cols            (phase 1)
//   A-hi = tile rows {64-127, 192-255}   (phase 2)
// Phase p of tile t issues the half-tile of tile t+1 that phase p needs (2 LDS-DMA instructions per
// wave), so every half-tile is in flight for 3-4 phases of MFMA work before it is read; one counted
// vmcnt + one raw barrier per phase retire exactly the half-tile the next phase reads (never
// vmcnt(0) in the loop), and each buffer region is refilled >= 3 phases after its last read.
// Fragments are read once per tile: A of a quadrant row in phases 0 and 2, B-lo in phase 0 (kept in
// registers for phase 3), B-hi in phase 1.
constexpr int HT = 128 * TK;   // 16 KiB half-tile
constexpr int PBUF = 4 * HT;   // one k-tile: [A-lo | B-lo | B-hi | A-hi]

// tile row (A) / col (B) of slot row j of half-tile kind h (0 A-lo, 1 B-lo, 2 B-hi, 3 A-hi)
__device__ __forceinline__ int half_row(int h, int j) {
  switch (h) {
    case 0: return j < 64 ? j : j + 64;
    case 3: return j < 64 ? j + 64 : j + 128;
    case 1: return (j >> 5) * 64 + (j & 31);
    default: return (j >> 5) * 64 + 32 + (j & 31);
  }
}

template <bool CS>  // CS: the epilogue also writes column-sum partials (ep.colsum_part)
__global__ __launch_bounds__(512, 1) void gemm_bf16_256p_kernel(const uint8_t* __restrict__ A, int64_t lda,
                                                               int64_t a_bs, const uint8_t* __restrict__ B,
                                                               int64_t ldb, int64_t b_bs, GemmEpilogue ep, int M,
                                                               int N, int K, int tiles_m, int tiles_n, int splits,
                                                               int k_per_split, int group_m) {
  __shared__ __attribute__((aligned(16))) char smem[2 * PBUF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int per_z = tiles_m * tiles_n;
  const int zid = blockIdx.y;
  const int t = xcd_remap(blockIdx.x, per_z);
  int tm, tn;
  grouped_tile(t, tiles_m, tiles_n, group_m, tm, tn);
  const int b = zid / splits, split = zid - b * splits;
  const int m0 = tm * TM, n0 = tn * TN;
  const int kbeg = split * k_per_split, kend = min(K, kbeg + k_per_split);
  const int nkt = max(0, (kend - kbeg) / TK);

  // this lane's DMA source for instruction i (0, 1) of half-tile kind h: slot row 16*wave + 8i + lane/8,
  // physical 16-B chunk lane & 7 holding logical chunk (lane & 7) ^ (slot row & 7)
  const uint8_t* src[4][2];
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const bool is_a = h == 0 || h == 3;
    const uint8_t* base = is_a ? A + (int64_t)b * a_bs : B + (int64_t)b * b_bs;
    const int64_t ld = is_a ? lda : ldb;
    const int lim = is_a ? M : N, r0 = is_a ? m0 : n0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int j = 16 * wave + 8 * i + (lane >> 3);
      const int lc = (lane & 7) ^ (j & 7);
      const int rr = min(r0 + half_row(h, j), lim - 1);  // past the edge: re-read the last row, dropped on store
      src[h][i] = base + (int64_t)rr * ld + kbeg + lc * 16;
    }
  }
  auto issue = [&](int h, int kt) {
    char* dst = smem + (kt & 1) * PBUF + h * HT + 2 * wave * 1024;
    glds16(src[h][0] + (int64_t)kt * TK, dst);
    glds16(src[h][1] + (int64_t)kt * TK, dst + 1024);
  };

  f32x4 acc[8][4];  // [qm*4 + mt][qn*2 + nt]
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = zero_f32x4();

  // fragment offsets: slot row = (wr*64 | wc*32) + 16*tile + (lane & 15) == lane (mod 8), so the swizzled
  // chunk of k-step s is (4s + lane/16) ^ (lane & 7)
  const int sw0 = (((lane >> 4)) ^ (lane & 7)) << 4, sw1 = ((4 + (lane >> 4)) ^ (lane & 7)) << 4;
  const int a_row = (wr * 64 + (lane & 15)) * TK;
  const int b_row = (wc * 32 + (lane & 15)) * TK;

  if (nkt > 0) {
#pragma unroll
    for (int h = 0; h < 4; ++h) issue(h, 0);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // A-lo, B-lo of tile 0
    raw_barrier();
  }
  bf16x8 fa[4][2], fbl[2][2], fbh[2][2];
  for (int kt = 0; kt < nkt; ++kt) {
    const char* st = smem + (kt & 1) * PBUF;
    const bool next = kt + 1 < nkt;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      // fragments this phase reads first
      if (p == 0 || p == 2) {
        const char* ap = st + (p == 0 ? 0 : 3 * HT) + a_row;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          fa[mt][0] = *reinterpret_cast<const bf16x8*>(ap + mt * 16 * TK + sw0);
          fa[mt][1] = *reinterpret_cast<const bf16x8*>(ap + mt * 16 * TK + sw1);
        }
      }
      if (p == 0 || p == 1) {
        const char* bp = st + (p == 0 ? HT : 2 * HT) + b_row;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const bf16x8 x0 = *reinterpret_cast<const bf16x8*>(bp + nt * 16 * TK + sw0);
          const bf16x8 x1 = *reinterpret_cast<const bf16x8*>(bp + nt * 16 * TK + sw1);
          if (p == 0) {
            fbl[nt][0] = x0;
            fbl[nt][1] = x1;
          } else {
            fbh[nt][0] = x0;
            fbh[nt][1] = x1;
          }
        }
      }
      // next tile's half-tile for this phase: [A-lo, B-lo, B-hi, A-hi][p]
      if (next) issue(p, kt + 1);
      const int qm = (p == 2 || p == 3) ? 1 : 0;
      const bool qn1 = p == 1 || p == 2;
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt)  // C^T tile: lane ends with 4 consecutive n of one m
            acc[qm * 4 + mt][(qn1 ? 2 : 0) + nt] =
                mfma16x16x32(qn1 ? fbh[nt][ks] : fbl[nt][ks], fa[mt][ks], acc[qm * 4 + mt][(qn1 ? 2 : 0) + nt]);
      __builtin_amdgcn_s_setprio(0);
      // retire the half-tile the next phase reads first (one phase ahead of the read)
      if (p == 0) {
        if (next) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // B-hi(t)
        else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      } else if (p == 1) {
        if (next) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // A-hi(t)
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else if (p == 3) {
        if (next) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // A-lo(t+1), B-lo(t+1)
      }
      raw_barrier();
    }
  }

  // ---------------- epilogue: acc[qm*4+mt][qn*2+nt] holds C[m][n..n+3],
  //   m = m0 + wr*128 + qm*64 + 16 mt + (lane & 15),  n = n0 + wc*64 + qn*32 + 16 nt + 4 (lane >> 4)
  gemm256_store<true, false, CS>(acc, ep, M, N, zid, b, m0 + wr * 128 + (lane & 15), n0 + wc * 64 + 4 * (lane >> 4),
                                 1.f, smem + wave * 16384);
}

// ------------------------------------------------------------------------------------------------
// The phased pipeline as a PERSISTENT kernel: one workgroup per CU walks tiles w = blockIdx.x,
// blockIdx.x + gridDim.x, ... (XCD-remapped over the whole work list).  The last k-tile of a tile issues
// the half-tiles of the NEXT tile's first k-tile (same phase / buffer rules as any k-tile), so the next
// tile's operands land while this tile's epilogue runs; the epilogue uses no LDS and issues an exact
// number of stores (gemm256_store_q), which the first k-tile of the next tile adds to its two counted
// waits.  What this removes per tile: the cold prologue (a full DMA latency with no MFMA work) and the
// workgroup launch; the stores drain during the next tile's first phases.
// Counted waits (DMA instructions younger than the half-tile retired; e = the epilogue's stores):
//   steady k-tile              p0 B-hi: 4        p1 A-hi: 4        p3 next A-lo/B-lo: 4
//   last k-tile, no next tile  p0: 2             p1: 0
//   first k-tile, early issue  p0: 10 + e        p1: 8 + e         p3: 4 + e   (k-tile 1 issued before e)
//   second k-tile after early / first k-tile otherwise: p0 4 + e (2 + e), p1 4 + e (0), p3 4
__global__ __launch_bounds__(512, 1) void gemm_bf16_256q_kernel(const uint8_t* __restrict__ A, int64_t lda,
                                                               int64_t a_bs, const uint8_t* __restrict__ B,
                                                               int64_t ldb, int64_t b_bs, GemmEpilogue ep, int M,
                                                               int N, int K, int tiles_m, int tiles_n, int splits,
                                                               int k_per_split, int total, int group_m) {
  __shared__ __attribute__((aligned(16))) char smem[2 * PBUF];
  // wave index in an SGPR (readfirstlane): the per-wave terms of the DMA offsets and LDS addresses then cost
  // no VGPRs
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int per_z = tiles_m * tiles_n;
  const int nstores = gemm256_q_stores(ep);

  // per-lane 32-bit byte offsets of the 8 DMA sources (kind h, instruction i) from the tile's A / B base,
  // which live in SGPRs (global_load_lds_dwordx4 v_off, s[base]): 8 VGPRs instead of 16 for 64-bit pointers
  uint32_t off[4][2];
  const uint8_t* abase = A;
  const uint8_t* bbase = B;
  int m0 = 0, n0 = 0, zid = 0, bb = 0, nkt = 0;
  // work item -> tile coordinates, operand bases and this lane's DMA offsets (see gemm_bf16_256p_kernel)
  auto setup = [&](int w, int& tm0, int& tn0, int& z, int& b, int& nk) {
    const int t = xcd_remap(w, total);
    z = t / per_z;
    const int tt = t - z * per_z;
    int tm, tn;
    grouped_tile(tt, tiles_m, tiles_n, group_m, tm, tn);
    b = z / splits;
    const int split = z - b * splits;
    tm0 = tm * TM;
    tn0 = tn * TN;
    const int kbeg = split * k_per_split, kend = min(K, kbeg + k_per_split);
    nk = max(0, (kend - kbeg) / TK);
    abase = A + (int64_t)b * a_bs + kbeg;
    bbase = B + (int64_t)b * b_bs + kbeg;
    // the lane index through an opaque move: the per-lane row terms below are then recomputed here (a few
    // VALU ops per tile) instead of being hoisted out of the tile loop into registers the main loop needs
    int ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const bool is_a = h == 0 || h == 3;
      const int ld = is_a ? (int)lda : (int)ldb;
      const int lim = is_a ? M : N, r0 = is_a ? tm0 : tn0;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int j = 16 * wave + 8 * i + (ln >> 3);
        const int lc = (ln & 7) ^ (j & 7);
        const int rr = min(r0 + half_row(h, j), lim - 1);
        off[h][i] = (uint32_t)rr * (uint32_t)ld + (uint32_t)(lc * 16);
      }
    }
  };
  // half-tile h of k-tile kt (of the tile the offsets describe) into buffer `buf`
  auto issue = [&](int h, int kt, int buf) {
    const uint8_t* base = (h == 0 || h == 3) ? abase : bbase;
    char* dst = smem + buf * PBUF + h * HT + 2 * wave * 1024;
    glds16s(off[h][0] + (uint32_t)(kt * TK), base, dst);
    glds16s(off[h][1] + (uint32_t)(kt * TK), base, dst + 1024);
  };
  auto wait_vm = [&](int n) {  // s_waitcnt needs an immediate; n is even here (2 DMAs per half-tile)
    switch (n) {
      case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
      case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
      case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
      case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
      case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
      case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
      case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
      case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
      case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
      case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
      case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
      case 22: asm volatile("s_waitcnt vmcnt(22)" ::: "memory"); break;
      case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
      case 26: asm volatile("s_waitcnt vmcnt(26)" ::: "memory"); break;
      case 28: asm volatile("s_waitcnt vmcnt(28)" ::: "memory"); break;
      case 30: asm volatile("s_waitcnt vmcnt(30)" ::: "memory"); break;
      case 32: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
      case 34: asm volatile("s_waitcnt vmcnt(34)" ::: "memory"); break;
      case 36: asm volatile("s_waitcnt vmcnt(36)" ::: "memory"); break;
      case 38: asm volatile("s_waitcnt vmcnt(38)" ::: "memory"); break;
      case 40: asm volatile("s_waitcnt vmcnt(40)" ::: "memory"); break;
      case 42: asm volatile("s_waitcnt vmcnt(42)" ::: "memory"); break;
      case 44: asm volatile("s_waitcnt vmcnt(44)" ::: "memory"); break;
      case 46: asm volatile("s_waitcnt vmcnt(46)" ::: "memory"); break;
      case 48: asm volatile("s_waitcnt vmcnt(48)" ::: "memory"); break;
      case 50: asm volatile("s_waitcnt vmcnt(50)" ::: "memory"); break;
      case 52: asm volatile("s_waitcnt vmcnt(52)" ::: "memory"); break;
      case 54: asm volatile("s_waitcnt vmcnt(54)" ::: "memory"); break;
      case 56: asm volatile("s_waitcnt vmcnt(56)" ::: "memory"); break;
      case 58: asm volatile("s_waitcnt vmcnt(58)" ::: "memory"); break;
      case 60: asm volatile("s_waitcnt vmcnt(60)" ::: "memory"); break;
      case 62: asm volatile("s_waitcnt vmcnt(62)" ::: "memory"); break;
      default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
  };

  const int sw0 = (((lane >> 4)) ^ (lane & 7)) << 4, sw1 = ((4 + (lane >> 4)) ^ (lane & 7)) << 4;
  const int a_row = (wr * 64 + (lane & 15)) * TK;
  const int b_row = (wc * 32 + (lane & 15)) * TK;

  int w = blockIdx.x;
  if (w >= total) return;
  setup(w, m0, n0, zid, bb, nkt);
  int g = 0;  // running k-tile count of this workgroup: k-tile g lives in buffer g & 1
  if (nkt > 0) {
#pragma unroll
    for (int h = 0; h < 4; ++h) issue(h, 0, 0);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // A-lo, B-lo of the first k-tile
    raw_barrier();
  }
  int extra = 0;       // stores of the previous tile's epilogue still counted in vmcnt
  bool early = false;  // this tile's k-tile 1 was issued before the previous tile's epilogue
  bf16x8 fa[4][2], fb[2][2];
  for (;;) {
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = zero_f32x4();
    const int wn = w + gridDim.x;
    const bool has_next = wn < total;
    int nm0 = 0, nn0 = 0, nz = 0, nb = 0, nnkt = 0;
    for (int kt = 0; kt < nkt; ++kt, ++g) {
      const char* st = smem + (g & 1) * PBUF;
      const bool last = kt + 1 == nkt;
      if (last && has_next) {
        // the sources of this tile are no longer needed: switch to the next tile's (k-tile 0 of it is
        // issued by the phases below); an empty next tile (nnkt == 0) gets nothing issued
        setup(wn, nm0, nn0, nz, nb, nnkt);
      }
      const bool next = !last || (has_next && nnkt > 0);
      const int nkt_issue = last ? 0 : kt + 1;
      // counted waits, in DMA instructions younger than the half-tile each one retires (see the table in
      // the comment above the kernel); `e` = the previous epilogue's stores when they are among them
      const bool skip = early && kt == 0;  // k-tile 1 is already in flight
      const int e = (kt == 0 || (early && kt == 1)) ? extra : 0;
      const int w0 = skip ? 10 + e : (next ? 4 + e : 2 + e);
      const int w1 = skip ? 8 + e : (next ? 4 + e : 0);
      const int w3 = skip ? 4 + e : 4;
      const bool do3 = skip || next;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        if (p == 0 || p == 2) {
          const char* ap = st + (p == 0 ? 0 : 3 * HT) + a_row;
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) {
            fa[mt][0] = *reinterpret_cast<const bf16x8*>(ap + mt * 16 * TK + sw0);
            fa[mt][1] = *reinterpret_cast<const bf16x8*>(ap + mt * 16 * TK + sw1);
          }
        }
        if (p != 2) {  // B-lo in phases 0 and 3 (re-read: 16 VGPRs fewer than keeping it), B-hi in phase 1
          const char* bp = st + (p == 1 ? 2 * HT : HT) + b_row;
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) {
            fb[nt][0] = *reinterpret_cast<const bf16x8*>(bp + nt * 16 * TK + sw0);
            fb[nt][1] = *reinterpret_cast<const bf16x8*>(bp + nt * 16 * TK + sw1);
          }
        }
        if (next && !skip) issue(p, nkt_issue, (g + 1) & 1);
        const int qm = (p == 2 || p == 3) ? 1 : 0;
        const bool qn1 = p == 1 || p == 2;
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt)
              acc[qm * 4 + mt][(qn1 ? 2 : 0) + nt] = mfma16x16x32(fb[nt][ks], fa[mt][ks], acc[qm * 4 + mt][(qn1 ? 2 : 0) + nt]);
        __builtin_amdgcn_s_setprio(0);
        // retire the half-tile the next phase reads first; in the first k-tile of a tile the previous
        // epilogue's `e` stores sit between the waited-for copies and the newest ones
        if (p == 0) {
          wait_vm(w0);  // B-hi of this k-tile
        } else if (p == 1) {
          wait_vm(w1);  // A-hi of this k-tile
        } else if (p == 3) {
          if (do3) wait_vm(w3);  // A-lo, B-lo of the next k-tile
        }
        raw_barrier();
      }
    }
    bool cold = false;  // an empty tile (no k-tiles) issued nothing for the next one: start it cold
    if (has_next && nkt == 0) {
      setup(wn, nm0, nn0, nz, nb, nnkt);
      cold = true;
    }
    // the next tile's k-tile 1 goes into the buffer the last k-tile just finished with, BEFORE the epilogue:
    // the first waits of the next tile then retire copies that are all older than this epilogue's stores
    // and the stores get ~7 phases to drain before any wait covers them
    const bool early_next = has_next && nnkt >= 2 && !cold;
    if (early_next) {
#pragma unroll
      for (int h = 0; h < 4; ++h) issue(h, 1, (g + 1) & 1);
    }
    gemm256_store_q<true>(acc, ep, M, N, zid, bb, m0 + wr * 128 + (lane & 15), n0 + wc * 64 + 4 * (lane >> 4), 1.f);
    if (!has_next) break;
    early = early_next;
    if (cold && nnkt > 0) {
#pragma unroll
      for (int h = 0; h < 4; ++h) issue(h, 0, g & 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // A-lo, B-lo of its first k-tile (and every store)
      raw_barrier();
    }
    w = wn;
    m0 = nm0;
    n0 = nn0;
    zid = nz;
    bb = nb;
    nkt = nnkt;
    extra = cold ? 0 : nstores;
  }
}

// ------------------------------------------------------------------------------------------------
// Two workgroups per CU: 256x128 tiles, 4 waves (2 (M) x 2 (N), the same 128x64 wave tile and 32
// accumulator tiles as above), 32-k stages of 24 KiB (A 256 x 64 B, B 128 x 64 B), three of them: 72 KiB
// per workgroup, so two fit in the 160 KiB LDS and the CU holds the same 8 waves as the one-workgroup
// kernels.  What the second workgroup buys: one tile's cold prologue (the first DMA round trip) and its
// output drain (128 KiB of stores per 256x256 of output) run while the other workgroup's MFMAs issue - in
// the one-workgroup kernels both are exposed on every tile (profiles/r03/gemm_epilogue.md).
// Stage image: 64-B rows, physical 16-B chunk p of row r holds logical chunk p ^ f(r), f(r) = (r >> 2) & 2:
// a ds_read_b128 lane group ({0-3,12-15,20-27}, ...) reads rows {j, 12+j, 4+j, 8+j} at two chunks, and
// that f sends each group's 16 reads to 16 distinct 16-B bank slots (conflict-free).  One barrier per
// stage; stage kt+2 is issued right after it (into the buffer stage kt-1 was read from).
constexpr int N2_TN = 128, N2_TK = 64;  // N2_TK in bytes (32 bf16: one MFMA k-step)
constexpr int N2_STAGE = (TM + N2_TN) * N2_TK;  // 24 KiB
constexpr int N2_NBUF = 3;
__device__ __forceinline__ int n2_swz(int r) { return (r >> 2) & 2; }

template <bool CS>
__global__ __launch_bounds__(256, 2) void gemm_bf16_256n_kernel(const uint8_t* __restrict__ A, int64_t lda,
                                                               int64_t a_bs, const uint8_t* __restrict__ B,
                                                               int64_t ldb, int64_t b_bs, GemmEpilogue ep, int M,
                                                               int N, int K, int tiles_m, int tiles_n, int splits,
                                                               int k_per_split, int group_m) {
  __shared__ __attribute__((aligned(16))) char smem[N2_NBUF * N2_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int per_z = tiles_m * tiles_n;
  const int zid = blockIdx.y;
  const int t = xcd_remap(blockIdx.x, per_z);
  int tm, tn;
  grouped_tile(t, tiles_m, tiles_n, group_m, tm, tn);
  const int b = zid / splits, split = zid - b * splits;
  const int m0 = tm * TM, n0 = tn * N2_TN;
  const int kbeg = split * k_per_split, kend = min(K, kbeg + k_per_split);
  const int nkt = max(0, (kend - kbeg) / N2_TK);

  // this lane's 6 DMA sources per stage: 4 of A (stage rows 64 wave + 16 j + lane / 4), 2 of B (stage rows
  // 256 + 32 wave + 16 j + lane / 4); lane -> physical chunk lane & 3, logical chunk (lane & 3) ^ f(row)
  const uint8_t* src[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const bool a_part = j < 4;
    const int r = a_part ? 64 * wave + 16 * j + (lane >> 2) : 32 * wave + 16 * (j - 4) + (lane >> 2);
    const int lc = (lane & 3) ^ n2_swz(r);
    const uint8_t* base = a_part ? A + (int64_t)b * a_bs : B + (int64_t)b * b_bs;
    const int64_t ld = a_part ? lda : ldb;
    const int rr = min((a_part ? m0 : n0) + r, (a_part ? M : N) - 1);  // past the edge: re-read, dropped on store
    src[j] = base + (int64_t)rr * ld + kbeg + lc * 16;
  }
  auto issue = [&](int kt) {
    char* st = smem + (kt % N2_NBUF) * N2_STAGE;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      char* dst = j < 4 ? st + (64 * wave + 16 * j) * N2_TK : st + TM * N2_TK + (32 * wave + 16 * (j - 4)) * N2_TK;
      glds16(src[j] + (int64_t)kt * N2_TK, dst);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = zero_f32x4();

  // fragment reads: row R = 16 tile + (lane & 15) (so f(R) = f(lane & 15)), logical chunk lane >> 4
  const int fr = lane & 15;
  const int frag = fr * N2_TK + (((lane >> 4) ^ n2_swz(fr)) << 4);
  const int a_off = wm * 128 * N2_TK + frag;
  const int b_off = TM * N2_TK + wn * 64 * N2_TK + frag;

  // Fragments are register double-buffered: stage kt + 1 is read into the other set while stage kt's MFMAs
  // issue, so a buffer is free as soon as every wave has READ it (the barrier of the next stage), and the
  // DMA runs three stages ahead (stage kt + 3 goes into stage kt's buffer).
  struct Frags {
    bf16x8 a[8], b[4];
  };
  auto load = [&](Frags& f, int kt) {
    const char* st = smem + (kt % N2_NBUF) * N2_STAGE;
#pragma unroll
    for (int j = 0; j < 4; ++j) f.b[j] = *reinterpret_cast<const bf16x8*>(st + b_off + j * 16 * N2_TK);
#pragma unroll
    for (int i = 0; i < 8; ++i) f.a[i] = *reinterpret_cast<const bf16x8*>(st + a_off + i * 16 * N2_TK);
  };
  auto mfmas = [&](const Frags& f) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16x16x32(f.b[j], f.a[i], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
  };
  // stage kt: publish stage kt + 1 (its copies landed: only kt + 2 may still be in flight), refill the buffer
  // of stage kt (every wave's reads of it retired before the barrier), read kt + 1, multiply kt
  auto step = [&](int kt, const Frags& cur, Frags& nxt) {
    if (kt + 1 < nkt) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (kt + 2 < nkt)
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      raw_barrier();
      if (kt + 3 < nkt) issue(kt + 3);
      load(nxt, kt + 1);
    }
    mfmas(cur);
  };

  if (nkt > 0) issue(0);
  if (nkt > 1) issue(1);
  if (nkt > 2) issue(2);
  Frags f0, f1;
  if (nkt > 0) {
    if (nkt > 2)
      asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (nkt > 1)
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();
    load(f0, 0);
  }
  for (int kt = 0; kt < nkt; kt += 2) {
    step(kt, f0, f1);
    if (kt + 1 < nkt) step(kt + 1, f1, f0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();  // the epilogue reuses the stage buffers as per-wave scratch
  gemm256_store<false, false, CS>(acc, ep, M, N, zid, b, m0 + wm * 128 + (lane & 15), n0 + wn * 64 + 4 * (lane >> 4),
                                  1.f, smem + wave * 16384);
}

int g_phased = -1;
int phased_mode() {
  if (g_phased < 0) {
    const char* v = getenv("RINGDP_GEMM256_PHASED");  // 0: the single-stage-wait pipeline (A/B)
    g_phased = (v && v[0] == '0') ? 0 : 1;
  }
  return g_phased;
}

}  // namespace

void set_gemm256_phased(int on) { g_phased = on ? 1 : 0; }

// persistent phased kernel (gemm_bf16_256q), off by default: RINGDP_GEMM256_PERSIST=1 selects it.
// Measured (tools/gemm_epi_probe.py, profiles/r03/gemm_epilogue.md): 10-20 % SLOWER than one workgroup per
// tile on every shape tried - the output stores of a tile drain slowly under load, and the in-order vmcnt
// makes the next tile's first DMA wait behind them; with one workgroup per CU the drain is just as exposed
// at the workgroup's end, so neither form overlaps it.
static int g_persist = -1;
static int persist_mode() {
  if (g_persist < 0) {
    const char* v = getenv("RINGDP_GEMM256_PERSIST");
    g_persist = (v && v[0] == '1') ? 1 : 0;
  }
  return g_persist;
}
void set_gemm256_persist(int on) { g_persist = on ? 1 : 0; }

// 256 B of device memory per device that the persistent epilogue's edge stores land in (never read)
static void* store_sink() {
  static void* sinks[64] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (!sinks[dev]) {
    if (hipMalloc(&sinks[dev], 256) != hipSuccess) sinks[dev] = nullptr;
  }
  return sinks[dev];
}

static int cu_count() {
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

static int g_wide = -1;
int gemm_wide_store_mode() {
  if (g_wide < 0) {
    const char* v = getenv("RINGDP_GEMM_WIDE_STORE");
    g_wide = v && *v ? atoi(v) : 2;
  }
  return g_wide;
}
void set_gemm_wide_store(int mode) { g_wide = mode; }
static int g_store_cache = -1;
int gemm_store_cache() {
  if (g_store_cache < 0) {
    const char* v = getenv("RINGDP_GEMM_STORE_CACHE");
    g_store_cache = v && *v ? atoi(v) : 0;
  }
  return g_store_cache;
}
void set_gemm_store_cache(int flavour) { g_store_cache = flavour; }
// K-contiguous bf16 GEMMs on the two-workgroups-per-CU 256x128 kernel: 0 (default) never, 1 always, 2 when
// N <= 1024; its tile-order group (tile rows per group, RINGDP_GEMM_2WG_GROUP, default 4).  Measured
// (profiles/r05/two_wg/): 2-7 % faster than the 256x256 kernel on the N <= 1024 shapes back to back, 5-13 %
// slower on N >= 2048 and at 8192^3, and neutral in the ViT-B/16 and ResNet-50 steps, so it stays opt-in.
static int g_two_wg = -1, g_two_wg_group = -1;
static int two_wg_mode() {
  if (g_two_wg < 0) {
    const char* v = getenv("RINGDP_GEMM_2WG");
    g_two_wg = v && *v ? atoi(v) : 0;
  }
  return g_two_wg;
}
static int two_wg_group() {
  if (g_two_wg_group < 0) {
    const char* v = getenv("RINGDP_GEMM_2WG_GROUP");
    g_two_wg_group = v && *v ? std::max(1, atoi(v)) : 4;
  }
  return g_two_wg_group;
}
void set_gemm_two_wg(int mode, int group_m) {
  g_two_wg = mode;
  if (group_m > 0) g_two_wg_group = group_m;
}

static int bf16_group_m() {  // tile rows per group of the tile order (1 = row-major, rounds 1-3)
  static const int g = [] {
    const char* v = getenv("RINGDP_BF16_GROUP_M");
    return v && *v ? atoi(v) : 4;
  }();
  return g;
}

bool gemm_bf16_256(const GemmOperand& A, const GemmOperand& Bop, int batch, int M, int N, int K,
                   const GemmEpilogue& ep, int splits, hipStream_t s) {
  // 16-B aligned rows, whole 64-element k-tiles (k-rows of a row-contiguous operand), whole 4-column
  // runs, whole 8-column chunks of a row-contiguous operand, no statistics epilogue
  if (K % TKE != 0 || N % 4 != 0 || M <= 0 || N <= 0 || ep.stats || A.ld % 8 != 0 || Bop.ld % 8 != 0 ||
      (ep.mode != GemmEpilogue::kSplitK && ep.ldc % 4 != 0) || ep.scale_a || ep.scale_b ||
      reinterpret_cast<uintptr_t>(ep.bias) % 16 != 0 ||
      (A.row_contig && (M % 8 != 0 || A.bstride % 8 != 0)) || (Bop.row_contig && (N % 8 != 0 || Bop.bstride % 8 != 0)))
    return false;
  const int tiles_m = (M + TM - 1) / TM, tiles_n = (N + TN - 1) / TN;
  splits = std::max(1, splits);
  int kps = (K + splits - 1) / splits;
  kps = (kps + TKE - 1) / TKE * TKE;
  splits = (K + kps - 1) / kps;
  dim3 grid(tiles_m * tiles_n, batch * splits);
  const bool wide_bf16 = N % 8 == 0 && ep.ldc % 8 == 0 && (reinterpret_cast<uintptr_t>(ep.C) & 15) == 0 &&
                         ep.c_bstride % 8 == 0;
  const int twm = two_wg_mode();
  if (!A.row_contig && !Bop.row_contig && (twm == 1 || (twm == 2 && N <= 1024)) &&
      (!ep.colsum_part || (batch == 1 && splits == 1 && ep.out_bf16 && wide_bf16 && ep.mode == GemmEpilogue::kStore))) {
    const int tiles_n2 = (N + N2_TN - 1) / N2_TN;
    GemmEpilogue e3 = ep;
    e3.store_mode = ep.colsum_part ? 2 : gemm_wide_store_mode() % 10;
    e3.store_rot = gemm_wide_store_mode() < 10;
    e3.store_cache = gemm_store_cache();
    e3.sink = store_sink();
    dim3 grid2(tiles_m * tiles_n2, batch * splits);
    auto go2 = [&](auto kern) {
      kern<<<grid2, 256, 0, s>>>(static_cast<const uint8_t*>(A.p), A.ld * 2, A.bstride * 2,
                                 static_cast<const uint8_t*>(Bop.p), Bop.ld * 2, Bop.bstride * 2, e3, M, N, K * 2,
                                 tiles_m, tiles_n2, splits, kps * 2, two_wg_group());
    };
    if (ep.colsum_part) go2(gemm_bf16_256n_kernel<true>);
    else go2(gemm_bf16_256n_kernel<false>);
    return true;
  }
  if (ep.colsum_part) {  // column sums ride in the phased kernel's LDS-row bf16 stores only
    if (A.row_contig || Bop.row_contig || !phased_mode() || batch != 1 || splits != 1 || !ep.out_bf16 || !wide_bf16 ||
        ep.mode != GemmEpilogue::kStore)
      return false;
    GemmEpilogue e3 = ep;
    e3.store_mode = 2;
    e3.store_rot = gemm_wide_store_mode() < 10;
    e3.store_cache = gemm_store_cache();
    e3.sink = store_sink();
    gemm_bf16_256p_kernel<true><<<grid, 512, 0, s>>>(static_cast<const uint8_t*>(A.p), A.ld * 2, A.bstride * 2,
                                                      static_cast<const uint8_t*>(Bop.p), Bop.ld * 2, Bop.bstride * 2,
                                                      e3, M, N, K * 2, tiles_m, tiles_n, splits, kps * 2,
                                                      bf16_group_m());
    return true;
  }
  GemmEpilogue e2 = ep;
  e2.store_mode = gemm_wide_store_mode() % 10;
  e2.store_rot = gemm_wide_store_mode() < 10;
  e2.store_cache = gemm_store_cache();
  e2.sink = store_sink();
  const int group_m = bf16_group_m();
  auto go = [&](auto kern) {
    kern<<<grid, 512, 0, s>>>(static_cast<const uint8_t*>(A.p), A.ld * 2, A.bstride * 2,
                              static_cast<const uint8_t*>(Bop.p), Bop.ld * 2, Bop.bstride * 2, e2, M, N, K * 2,
                              tiles_m, tiles_n, splits, kps * 2, group_m);
  };
  const bool off32 = (int64_t)M * A.ld * 2 + (int64_t)K * 2 < (1ll << 32) &&
                     (int64_t)N * Bop.ld * 2 + (int64_t)K * 2 < (1ll << 32);
  if (!A.row_contig && !Bop.row_contig && phased_mode() && persist_mode() && off32 &&
      (ep.mode == GemmEpilogue::kSplitK || !ep.out_bf16 || wide_bf16)) {
    e2.sink = store_sink();
    if (e2.sink) {
      const int total = tiles_m * tiles_n * batch * splits;
      const int g = std::min(total, cu_count());
      gemm_bf16_256q_kernel<<<g, 512, 0, s>>>(static_cast<const uint8_t*>(A.p), A.ld * 2, A.bstride * 2,
                                             static_cast<const uint8_t*>(Bop.p), Bop.ld * 2, Bop.bstride * 2, e2, M,
                                             N, K * 2, tiles_m, tiles_n, splits, kps * 2, total, group_m);
      return true;
    }
  }
  if (!A.row_contig && !Bop.row_contig) {
    if (phased_mode()) go(gemm_bf16_256p_kernel<false>);
    else go(gemm_bf16_256_kernel<false, false>);
  }
  else if (A.row_contig && Bop.row_contig) go(gemm_bf16_256_kernel<true, true>);
  else if (A.row_contig) go(gemm_bf16_256_kernel<true, false>);
  else go(gemm_bf16_256_kernel<false, true>);
  return true;
}

}  // namespace kern
}  // namespace ringdp
