// Collectives over IPC-mapped peer memory: the "xgmi" process-group backend (host side:
// csrc/comm/xgmi_engine.cpp, csrc/comm/xgmi_pg.cpp).
//
// Topology it is written for: an 8x MI355X node is a fully connected xGMI graph (7 links per GPU).
// A ring all-reduce drives one outgoing link per GPU per step and pays 2(N-1) dependent hops; here
// every rank PUSHES its data straight into every peer's staging memory (remote stores are posted
// writes: all N-1 links carry traffic at once and nobody waits on a remote read round trip), then
// reduces what arrived from LOCAL memory:
//   * one-shot all-reduce (small buckets): push the whole message to every peer, one handshake,
//     every rank sums the N copies in rank order (bit-identical results on every rank);
//   * two-shot all-reduce (large buckets): push chunk j to rank j (reduce-scatter), rank j sums its
//     chunk in rank order and pushes the result to every peer (all-gather): 2(N-1)/N of the data per
//     rank, spread over all links, and 2 handshakes instead of 2(N-1) ring steps;
//   * reduce-scatter, all-gather, broadcast, barrier, and paired send/recv on the same machinery.
// Ranks may also share one GPU (IPC within one device): a one-GPU box runs the real multi-process
// protocol, which RCCL refuses.
//
// Protocol (per workgroup b of a fixed grid of G workgroups; every op launches exactly G):
//   - segment ownership is fixed: byte offset o of any message belongs to workgroup (o / 4 KiB) % G,
//     on the pushing and on the consuming rank alike;
//   - every op advances workgroup b's epoch e (device memory: hipGraph-replayable) and uses the slot
//     parity e & 1 of the staging regions;
//   - handshake: stores -> every storing wave `s_waitcnt vmcnt(0)` -> barrier -> one lane per peer:
//     system-scope release fence -> asm `vmcnt(0)` -> relaxed system-scope flag store of e into the
//     peer's flag word [b][me]; then one lane per peer polls its own word [b][peer] relaxed (bounded,
//     s_sleep), one system acquire, `vmcnt(0)`, barrier, plain loads (MI355X_MICROARCH.md visibility
//     rules, system scope because the producer is another process / another GPU);
//   - every collective op has every rank signal every peer, so when workgroup b writes a peer's
//     parity-(e&1) slot at epoch e it has already seen that peer's signal of epoch e-1, which the peer
//     sent only after its epoch e-2 kernel (the previous user of that slot) had completed;
//   - send/recv pairs use their own per-pair epochs and slots plus an ack word for slot reuse;
//   - every poll is bounded: past the deadline the workgroup sets the error word (host-mapped, read by
//     the watchdog) and exits, so a dead peer never leaves waves spinning.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace ringdp {
namespace kern {
namespace {

constexpr int kT = kXgThreads;
constexpr int kSeg = kXgSeg;

__device__ __forceinline__ unsigned ld_flag(const unsigned* f) {
  return __hip_atomic_load(const_cast<unsigned*>(f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_flag(unsigned* f, unsigned v) {
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint4 ld16(const char* p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ void st16(char* p, uint4 v) { *reinterpret_cast<uint4*>(p) = v; }
// the first n (< 16) bytes at p, zero-filled (a message's tail vector)
// (byte loops fully unrolled over register words: an addressable local would live in scratch)
__device__ __forceinline__ uint4 ld_part(const char* p, int n) {
  uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i < n) w[i >> 2] |= static_cast<uint32_t>(static_cast<uint8_t>(p[i])) << (8 * (i & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ void st_part(char* p, uint4 v, int n) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i < n) p[i] = static_cast<char>(w[i >> 2] >> (8 * (i & 3)));
}
__device__ __forceinline__ uint4 ld_n(const char* p, int n) { return n == 16 ? ld16(p) : ld_part(p, n); }
__device__ __forceinline__ void st_n(char* p, uint4 v, int n) {
  if (n == 16) st16(p, v);
  else st_part(p, v, n);
}

// ---------------------------------------------------------------- element traits (16 B vectors)
struct Bf16 { unsigned short x; };
struct F16 { unsigned short x; };

__device__ __forceinline__ unsigned short f32_to_bf16_rne(float f) {
  unsigned u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return static_cast<unsigned short>((u >> 16) | ((u & 0xffffu) ? 0x40u : 0u));
  return static_cast<unsigned short>((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

template <typename T> struct Tr;
template <> struct Tr<float> {
  static constexpr int N = 4;
  using A = float;
  __device__ static A up(float x) { return x; }
  __device__ static float down(A a) { return a; }
  static constexpr bool kFloat = true;
};
template <> struct Tr<double> {
  static constexpr int N = 2;
  using A = double;
  __device__ static A up(double x) { return x; }
  __device__ static double down(A a) { return a; }
  static constexpr bool kFloat = true;
};
template <> struct Tr<Bf16> {
  static constexpr int N = 8;
  using A = float;
  __device__ static A up(Bf16 x) { return __uint_as_float(static_cast<unsigned>(x.x) << 16); }
  __device__ static Bf16 down(A a) { return Bf16{f32_to_bf16_rne(a)}; }
  static constexpr bool kFloat = true;
};
template <> struct Tr<F16> {
  static constexpr int N = 8;
  using A = float;
  __device__ static A up(F16 x) { return static_cast<float>(__ushort_as_half(x.x)); }
  __device__ static F16 down(A a) { return F16{__half_as_ushort(__float2half_rn(a))}; }
  static constexpr bool kFloat = true;
};
template <> struct Tr<int32_t> {
  static constexpr int N = 4;
  using A = int32_t;
  __device__ static A up(int32_t x) { return x; }
  __device__ static int32_t down(A a) { return a; }
  static constexpr bool kFloat = false;
};
template <> struct Tr<int64_t> {
  static constexpr int N = 2;
  using A = int64_t;
  __device__ static A up(int64_t x) { return x; }
  __device__ static int64_t down(A a) { return a; }
  static constexpr bool kFloat = false;
};
template <> struct Tr<int8_t> {
  static constexpr int N = 16;
  using A = int32_t;
  __device__ static A up(int8_t x) { return x; }
  __device__ static int8_t down(A a) { return static_cast<int8_t>(a); }
  static constexpr bool kFloat = false;
};
template <> struct Tr<uint8_t> {
  static constexpr int N = 16;
  using A = int32_t;
  __device__ static A up(uint8_t x) { return x; }
  __device__ static uint8_t down(A a) { return static_cast<uint8_t>(a); }
  static constexpr bool kFloat = false;
};

template <int RED, typename A>
__device__ __forceinline__ A red_op(A x, A y) {
  if constexpr (RED == XG_SUM) return x + y;
  else if constexpr (RED == XG_PROD) return x * y;
  else if constexpr (RED == XG_MIN) return y < x ? y : x;
  else return y > x ? y : x;
}

// Sum (or product / min / max) of one 16-B vector over the sources, kept in the accumulation type
// (fp32 for 16-bit floats: rounded once at the end, as the rank-order fp32 reference does).
template <typename T, int RED>
struct VecAcc {
  typename Tr<T>::A v[Tr<T>::N];
  __device__ __forceinline__ void set(uint4 raw) {
    const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
    for (int i = 0; i < Tr<T>::N; ++i) v[i] = Tr<T>::up(e[i]);
  }
  __device__ __forceinline__ void add(uint4 raw) {
    const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
    for (int i = 0; i < Tr<T>::N; ++i) v[i] = red_op<RED>(v[i], Tr<T>::up(e[i]));
  }
  __device__ __forceinline__ uint4 get(const XgArgs& a) const {
    uint4 raw;
    T* e = reinterpret_cast<T*>(&raw);
#pragma unroll
    for (int i = 0; i < Tr<T>::N; ++i) {
      typename Tr<T>::A x = v[i];
      if (a.average) {
        if constexpr (Tr<T>::kFloat) x = x * static_cast<typename Tr<T>::A>(a.scale);
        else x = x / static_cast<typename Tr<T>::A>(a.world);
      }
      e[i] = Tr<T>::down(x);
    }
    return raw;
  }
};

// ---------------------------------------------------------------- staging / flag addressing
__device__ __forceinline__ char* reg_a(const XgArgs& a, int owner, int par, int src) {
  return a.stage_tab[owner] + a.off_a + (static_cast<int64_t>(par) * a.world + src) * a.slot;
}
__device__ __forceinline__ char* reg_b(const XgArgs& a, int owner, int par, int src) {
  return a.stage_tab[owner] + a.off_b + (static_cast<int64_t>(par) * a.world + src) * a.slot;
}
__device__ __forceinline__ char* reg_p(const XgArgs& a, int owner, int src, int par) {
  return a.stage_tab[owner] + a.off_p2p + (static_cast<int64_t>(src) * 2 + par) * a.p2p_slot;
}
// collective handshake words on `owner`: [channel][block][source rank]
__device__ __forceinline__ unsigned* flag_c(const XgArgs& a, int owner, int ch, int b, int src) {
  return a.flag_tab[owner] + (static_cast<int64_t>(ch) * a.nblocks + b) * kXgMaxRanks + src;
}
// send/recv: data-ready words on the receiver [src][block], ack words on the sender [dst][block]
__device__ __forceinline__ unsigned* flag_pd(const XgArgs& a, int owner, int src, int b) {
  return a.flag_tab[owner] + 2 * a.nblocks * kXgMaxRanks + src * a.nblocks + b;
}
__device__ __forceinline__ unsigned* flag_pa(const XgArgs& a, int owner, int dst, int b) {
  return a.flag_tab[owner] + 3 * a.nblocks * kXgMaxRanks + dst * a.nblocks + b;
}

// Bounded relaxed poll until (int)(*f - e) >= 0.  false: timed out.
__device__ __forceinline__ bool poll_ge(const unsigned* f, unsigned e, uint64_t timeout_ticks) {
  const uint64_t t0 = wall_clock64();
  while (static_cast<int>(ld_flag(f) - e) < 0) {
    if (wall_clock64() - t0 > timeout_ticks) return false;
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// All of this workgroup's stores are published to every peer (flag word [b][me] := e on each peer),
// then the workgroup waits until every peer has published epoch e to us.  Called by all threads.
__device__ __forceinline__ bool exchange(const XgArgs& a, int ch, int b, unsigned e, int* s_fail) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
  __syncthreads();
  const int tid = threadIdx.x;
  const bool lane_peer = tid < a.world && tid != a.rank;
  if (lane_peer) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the fence's own wait may be dropped (ROCm 7.2)
    st_flag(flag_c(a, tid, ch, b, a.rank), e);
    if (!poll_ge(flag_c(a, a.rank, ch, b, tid), e, a.timeout_ticks)) *s_fail = 1;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  return *s_fail == 0;
}

// Byte offsets of a message owned by this thread, workgroup b of G: o = (b + k G) * 4 KiB + 16 tid.
#define XG_FOR_OWNED(o, len)                                                                       \
  for (int64_t o = static_cast<int64_t>(b) * kSeg + 16 * tid; o < (len);                          \
       o += static_cast<int64_t>(a.nblocks) * kSeg)

__device__ __forceinline__ int vec_bytes(int64_t o, int64_t len) {
  return static_cast<int>(len - o < 16 ? len - o : 16);
}

// The same ownership, kU vectors per iteration (offsets o0 + u * G * 4 KiB): the loads of all kU are
// issued before any dependent store / add, so a thread has kU memory round trips in flight instead
// of one (a 26 MB two-shot is ~100 owned vectors per thread).
constexpr int kU = 4;
#define XG_FOR_OWNED_U(o0, len)                                                                    \
  for (int64_t o0 = static_cast<int64_t>(b) * kSeg + 16 * tid; o0 < (len);                        \
       o0 += static_cast<int64_t>(kU) * a.nblocks * kSeg)
#define XG_UOFF(o0, u) ((o0) + static_cast<int64_t>(u) * a.nblocks * kSeg)

template <typename T, int RED>
__device__ __forceinline__ void run_oneshot(const XgArgs& a, int b, unsigned e, int par, int* s_fail) {
  const int tid = threadIdx.x, me = a.rank, W = a.world;
  const int64_t S = a.nbytes;
  XG_FOR_OWNED_U(o0, S) {
    uint4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t o = XG_UOFF(o0, u);
      if (o < S) v[u] = ld_n(a.in + o, vec_bytes(o, S));
    }
    for (int p = 0; p < W; ++p) {
      if (p == me) continue;
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int64_t o = XG_UOFF(o0, u);
        if (o < S) st16(reg_a(a, p, par, me) + o, v[u]);
      }
    }
  }
  if (!exchange(a, 0, b, e, s_fail)) return;
  XG_FOR_OWNED_U(o0, S) {
    VecAcc<T, RED> acc[kU];
    for (int r = 0; r < W; ++r) {
      uint4 v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int64_t o = XG_UOFF(o0, u);
        if (o < S) v[u] = r == me ? ld_n(a.in + o, vec_bytes(o, S)) : ld16(reg_a(a, me, par, r) + o);
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (r == 0) acc[u].set(v[u]);
        else acc[u].add(v[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t o = XG_UOFF(o0, u);
      if (o < S) st_n(a.out + o, acc[u].get(a), vec_bytes(o, S));
    }
  }
}

// Chunk j of a two-shot all-reduce: bytes [j*C, min(S, (j+1)*C)).
__device__ __forceinline__ int64_t chunk_len(const XgArgs& a, int j) {
  const int64_t lo = j * a.chunk, hi = lo + a.chunk < a.nbytes ? lo + a.chunk : a.nbytes;
  return hi > lo ? hi - lo : 0;
}

template <typename T, int RED>
__device__ __forceinline__ void run_twoshot(const XgArgs& a, int b, unsigned e, int par, int* s_fail) {
  const int tid = threadIdx.x, me = a.rank, W = a.world;
  const int64_t C = a.chunk;
  // 1. reduce-scatter: my copy of chunk p goes to rank p
  XG_FOR_OWNED_U(o0, C) {
    for (int p = 0; p < W; ++p) {
      if (p == me) continue;
      const int64_t L = chunk_len(a, p);
      uint4 v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int64_t o = XG_UOFF(o0, u);
        if (o < L) v[u] = ld_n(a.in + p * C + o, vec_bytes(o, L));
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int64_t o = XG_UOFF(o0, u);
        if (o < L) st16(reg_a(a, p, par, me) + o, v[u]);
      }
    }
  }
  if (!exchange(a, 0, b, e, s_fail)) return;
  // 2. my chunk: rank-order sum, written locally and pushed to every peer
  const int64_t Lme = chunk_len(a, me);
  XG_FOR_OWNED_U(o0, Lme) {
    VecAcc<T, RED> acc[kU];
    for (int r = 0; r < W; ++r) {
      uint4 v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int64_t o = XG_UOFF(o0, u);
        if (o < Lme) v[u] = r == me ? ld_n(a.in + me * C + o, vec_bytes(o, Lme)) : ld16(reg_a(a, me, par, r) + o);
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (r == 0) acc[u].set(v[u]);
        else acc[u].add(v[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t o = XG_UOFF(o0, u);
      if (o >= Lme) continue;
      const uint4 res = acc[u].get(a);
      st_n(a.out + me * C + o, res, vec_bytes(o, Lme));
      for (int p = 0; p < W; ++p)
        if (p != me) st16(reg_b(a, p, par, me) + o, res);
    }
  }
  if (!exchange(a, 1, b, e, s_fail)) return;
  // 3. all-gather: every other chunk from the rank that reduced it
  XG_FOR_OWNED_U(o0, C) {
    for (int r = 0; r < W; ++r) {
      if (r == me) continue;
      const int64_t L = chunk_len(a, r);
      uint4 v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int64_t o = XG_UOFF(o0, u);
        if (o < L) v[u] = ld16(reg_b(a, me, par, r) + o);
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int64_t o = XG_UOFF(o0, u);
        if (o < L) st_n(a.out + r * C + o, v[u], vec_bytes(o, L));
      }
    }
  }
}

// in: W blocks of M bytes at stride a.stride; out: my M bytes.
template <typename T, int RED>
__device__ __forceinline__ void run_reduce_scatter(const XgArgs& a, int b, unsigned e, int par, int* s_fail) {
  const int tid = threadIdx.x, me = a.rank, W = a.world;
  const int64_t M = a.nbytes;
  XG_FOR_OWNED(o, M) {
    for (int p = 0; p < W; ++p)
      if (p != me) st16(reg_a(a, p, par, me) + o, ld_n(a.in + p * a.stride + o, vec_bytes(o, M)));
  }
  if (!exchange(a, 0, b, e, s_fail)) return;
  XG_FOR_OWNED(o, M) {
    const int n = vec_bytes(o, M);
    VecAcc<T, RED> acc;
    for (int r = 0; r < W; ++r) {
      const uint4 v = r == me ? ld_n(a.in + me * a.stride + o, n) : ld16(reg_a(a, me, par, r) + o);
      if (r == 0) acc.set(v);
      else acc.add(v);
    }
    st_n(a.out + o, acc.get(a), n);
  }
}

// in: my M bytes; out: W blocks of M bytes at stride a.stride.
__device__ __forceinline__ void run_allgather(const XgArgs& a, int b, unsigned e, int par, int* s_fail) {
  const int tid = threadIdx.x, me = a.rank, W = a.world;
  const int64_t M = a.nbytes;
  XG_FOR_OWNED(o, M) {
    const int n = vec_bytes(o, M);
    const uint4 v = ld_n(a.in + o, n);
    st_n(a.out + me * a.stride + o, v, n);
    for (int p = 0; p < W; ++p)
      if (p != me) st16(reg_a(a, p, par, me) + o, v);
  }
  if (!exchange(a, 0, b, e, s_fail)) return;
  XG_FOR_OWNED(o, M) {
    const int n = vec_bytes(o, M);
    for (int r = 0; r < W; ++r)
      if (r != me) st_n(a.out + r * a.stride + o, ld16(reg_a(a, me, par, r) + o), n);
  }
}

__device__ __forceinline__ void run_broadcast(const XgArgs& a, int b, unsigned e, int par, int* s_fail) {
  const int tid = threadIdx.x, me = a.rank, W = a.world, root = a.root;
  const int64_t S = a.nbytes;
  if (me == root) {
    XG_FOR_OWNED(o, S) {
      const int n = vec_bytes(o, S);
      const uint4 v = ld_n(a.in + o, n);
      for (int p = 0; p < W; ++p)
        if (p != me) st16(reg_a(a, p, par, root) + o, v);
      if (a.out != a.in) st_n(a.out + o, v, n);
    }
  }
  if (!exchange(a, 0, b, e, s_fail)) return;
  if (me != root) {
    XG_FOR_OWNED(o, S) st_n(a.out + o, ld16(reg_a(a, me, par, root) + o), vec_bytes(o, S));
  }
}

__device__ __forceinline__ void run_send(const XgArgs& a, int b, int* s_fail, unsigned* ep) {
  const int tid = threadIdx.x, me = a.rank, dst = a.peer;
  const unsigned e = *ep + 1u;
  const int par = e & 1;
  const int64_t S = a.nbytes;
  // slot parity e&1 was last filled at epoch e-2: the receiver must have acknowledged reading it
  if (tid == 0 && e > 2u) {
    if (!poll_ge(flag_pa(a, me, dst, b), e - 2u, a.timeout_ticks)) *s_fail = 1;
  }
  __syncthreads();
  if (*s_fail) return;
  XG_FOR_OWNED(o, S) st16(reg_p(a, dst, me, par) + o, ld_n(a.in + o, vec_bytes(o, S)));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st_flag(flag_pd(a, dst, me, b), e);
  }
  if (tid == 0) *ep = e;
}

__device__ __forceinline__ void run_recv(const XgArgs& a, int b, int* s_fail, unsigned* ep) {
  const int tid = threadIdx.x, me = a.rank, src = a.peer;
  const unsigned e = *ep + 1u;
  const int par = e & 1;
  const int64_t S = a.nbytes;
  if (tid == 0) {
    if (!poll_ge(flag_pd(a, me, src, b), e, a.timeout_ticks)) *s_fail = 1;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (*s_fail) return;
  XG_FOR_OWNED(o, S) st_n(a.out + o, ld16(reg_p(a, me, src, par) + o), vec_bytes(o, S));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every read of the slot has returned
  __syncthreads();
  if (tid == 0) {
    st_flag(flag_pa(a, src, me, b), e);
    *ep = e;
  }
}

template <typename T, int RED>
__global__ __launch_bounds__(kT) void xgmi_kernel(XgArgs a) {
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  __shared__ unsigned s_epoch;
  __shared__ int s_fail;
  if (a.kind == XG_SEND || a.kind == XG_RECV) {
    unsigned* ep = a.epochs + a.nblocks * (1 + (a.kind == XG_SEND ? 0 : kXgMaxRanks) + a.peer) + b;
    if (tid == 0) s_fail = 0;
    __syncthreads();
    if (a.kind == XG_SEND) run_send(a, b, &s_fail, ep);
    else run_recv(a, b, &s_fail, ep);
    if (tid == 0 && s_fail) {
      __hip_atomic_store(a.error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      *ep = *ep + 1u;  // stay aligned with the peer's count
    }
    return;
  }
  if (tid == 0) {
    s_epoch = a.epochs[b] + 1u;
    s_fail = 0;
  }
  __syncthreads();
  const unsigned e = s_epoch;
  const int par = e & 1;
  switch (a.kind) {
    case XG_BARRIER: exchange(a, 0, b, e, &s_fail); break;
    case XG_ONESHOT: run_oneshot<T, RED>(a, b, e, par, &s_fail); break;
    case XG_TWOSHOT: run_twoshot<T, RED>(a, b, e, par, &s_fail); break;
    case XG_REDUCE_SCATTER: run_reduce_scatter<T, RED>(a, b, e, par, &s_fail); break;
    case XG_ALLGATHER: run_allgather(a, b, e, par, &s_fail); break;
    case XG_BROADCAST: run_broadcast(a, b, e, par, &s_fail); break;
    default: break;
  }
  if (tid == 0) {
    if (s_fail) __hip_atomic_store(a.error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    a.epochs[b] = e;
  }
}

template <typename T>
void launch_t(const XgArgs& a, hipStream_t s) {
  const dim3 grid(a.nblocks), block(kT);
  switch (a.red) {
    case XG_SUM: hipLaunchKernelGGL((xgmi_kernel<T, XG_SUM>), grid, block, 0, s, a); break;
    case XG_PROD: hipLaunchKernelGGL((xgmi_kernel<T, XG_PROD>), grid, block, 0, s, a); break;
    case XG_MIN: hipLaunchKernelGGL((xgmi_kernel<T, XG_MIN>), grid, block, 0, s, a); break;
    default: hipLaunchKernelGGL((xgmi_kernel<T, XG_MAX>), grid, block, 0, s, a); break;
  }
}

}  // namespace

void xgmi_collective(const XgArgs& a, hipStream_t s) {
  const bool reduces = a.kind == XG_ONESHOT || a.kind == XG_TWOSHOT || a.kind == XG_REDUCE_SCATTER;
  if (!reduces) {  // data movement only: one instantiation serves every dtype
    hipLaunchKernelGGL((xgmi_kernel<uint8_t, XG_SUM>), dim3(a.nblocks), dim3(kT), 0, s, a);
    return;
  }
  switch (a.dtype) {
    case XG_F32: launch_t<float>(a, s); break;
    case XG_BF16: launch_t<Bf16>(a, s); break;
    case XG_F16: launch_t<F16>(a, s); break;
    case XG_F64: launch_t<double>(a, s); break;
    case XG_I32: launch_t<int32_t>(a, s); break;
    case XG_I64: launch_t<int64_t>(a, s); break;
    case XG_I8: launch_t<int8_t>(a, s); break;
    default: launch_t<uint8_t>(a, s); break;
  }
}

}  // namespace kern
}  // namespace ringdp
