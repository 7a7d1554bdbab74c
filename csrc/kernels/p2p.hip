// One-shot peer-to-peer all-reduce over IPC-mapped buffers (xGMI on an 8x MI355X node).
//
// Why: a ring all-reduce of a small bucket is latency-bound - 2(N-1) dependent steps
// (the ConvNet's 455 KB bucket at N=8 is 14 ring steps of ~57 KB).  On a fully
// connected xGMI node every GPU can read every peer directly, so one hop suffices:
//   1. each rank copies its segment of the input into its own IPC-exported staging buffer;
//   2. it signals "epoch e written" to the same segment's flag on every peer (system scope);
//   3. once all N flags of that segment read e, it sums the N staged copies in RANK ORDER
//      (bit-identical result on every rank) and writes the output in place.
// Each GPU reads (N-1)/N of the data once from each of its 7 links in parallel instead of
// 2(N-1) serialized ring hops.
//
// Memory: staging buffers and flags are hipDeviceMallocUncached (fine-grained, uncached on
// every agent), so peer reads never see stale cache lines; order comes from the release fence
// before each flag store and the acquire after each poll.  Double buffering by epoch parity
// makes one signal per op enough: the next writer of a slot is op e+2, which cannot start
// before every peer has arrived at op e+1, i.e. finished reading op e (kernels on a stream are
// ordered).  Segments are fixed (block b always owns bytes [b*seg, (b+1)*seg)), so blocks never
// touch each other's staging bytes whatever the op size; per-block epoch counters live in
// device memory, so the kernel is hipGraph-replayable (no epoch argument frozen at capture).
// Every poll is bounded: past the deadline the block records an error word and exits, so a dead
// peer can never leave waves spinning forever.
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace ringdp {
namespace kern {
namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ unsigned poll_flag(unsigned* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ float4 ld4(const char* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(char* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

__device__ __forceinline__ void add_bf16x8(float (&acc)[8], float4 raw) {
  const unsigned* w = reinterpret_cast<const unsigned*>(&raw);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    acc[2 * k] += __uint_as_float(w[k] << 16);
    acc[2 * k + 1] += __uint_as_float(w[k] & 0xffff0000u);
  }
}

__device__ __forceinline__ unsigned bf16_bits(float x) {  // round to nearest even
  unsigned u = __float_as_uint(x);
  if ((u & 0x7f800000u) == 0x7f800000u) return (u >> 16) | ((u & 0xffffu) ? 0x40u : 0u);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

__global__ __launch_bounds__(kThreads) void p2p_allreduce_kernel(P2PArgs a) {
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t seg0 = static_cast<int64_t>(b) * a.seg_bytes;
  const int64_t len = min(static_cast<int64_t>(a.seg_bytes), a.nbytes - seg0);
  __shared__ unsigned s_epoch;
  __shared__ int s_fail;
  if (tid == 0) {
    s_epoch = a.epochs[b] + 1u;
    s_fail = 0;
  }
  __syncthreads();
  const unsigned e = s_epoch;
  const int64_t slot_off = static_cast<int64_t>(e & 1u) * a.slot_bytes + seg0;

  // 1. stage my segment (16 B per lane per pass)
  char* mine = a.bufs[a.rank] + slot_off;
  const char* in = reinterpret_cast<const char*>(a.data) + seg0;
  for (int64_t i = static_cast<int64_t>(tid) * 16; i < len; i += kThreads * 16) st4(mine + i, ld4(in + i));
  // every storing wave drains before the block signals (R1 of the visibility rules)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // 2. release + one flag per peer (lane p signals peer p)
  if (tid < a.world) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(a.flags[tid] + b * kP2PMaxRanks + a.rank, e, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }

  // 3. lane p polls peer p's arrival at this segment (bounded), then one acquire per wave
  if (tid < a.world) {
    unsigned* f = a.flags[a.rank] + b * kP2PMaxRanks + tid;
    const uint64_t t0 = wall_clock64();
    while (static_cast<int>(poll_flag(f) - e) < 0) {
      if (wall_clock64() - t0 > a.timeout_ticks) {
        s_fail = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (s_fail) {
    if (tid == 0) {
      __hip_atomic_store(a.error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      a.epochs[b] = e;  // keep the epoch sequence aligned with the peers that did arrive
    }
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");

  // 4. sum the N staged copies in rank order, write the result in place
  char* out = reinterpret_cast<char*>(a.data) + seg0;
  if (a.dtype == 0) {  // fp32
    for (int64_t i = static_cast<int64_t>(tid) * 16; i < len; i += kThreads * 16) {
      float4 acc = ld4(a.bufs[0] + slot_off + i);
      for (int p = 1; p < a.world; ++p) {
        const float4 v = ld4(a.bufs[p] + slot_off + i);
        acc.x += v.x;
        acc.y += v.y;
        acc.z += v.z;
        acc.w += v.w;
      }
      acc.x *= a.scale;
      acc.y *= a.scale;
      acc.z *= a.scale;
      acc.w *= a.scale;
      st4(out + i, acc);
    }
  } else {  // bf16: accumulate in fp32, round once
    for (int64_t i = static_cast<int64_t>(tid) * 16; i < len; i += kThreads * 16) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int p = 0; p < a.world; ++p) add_bf16x8(acc, ld4(a.bufs[p] + slot_off + i));
      unsigned w[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        w[k] = bf16_bits(acc[2 * k] * a.scale) | (bf16_bits(acc[2 * k + 1] * a.scale) << 16);
      st4(out + i, *reinterpret_cast<float4*>(w));
    }
  }
  if (tid == 0) a.epochs[b] = e;
}

}  // namespace

void p2p_allreduce(const P2PArgs& a, hipStream_t s) {
  const int blocks = static_cast<int>((a.nbytes + a.seg_bytes - 1) / a.seg_bytes);
  if (blocks <= 0) return;
  hipLaunchKernelGGL(p2p_allreduce_kernel, dim3(blocks), dim3(kThreads), 0, s, a);
}

}  // namespace kern
}  // namespace ringdp
