// Host-callable launchers for ringdp's CDNA4 HIP kernels (no torch types here: raw pointers +
// hipStream_t, so the .hip translation units stay free of PyTorch headers).
#pragma once

#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <vector>

namespace ringdp {
namespace kern {

// ---------------------------------------------------------------- elementwise / optimizer
void cast_f32_to_bf16(const float* src, void* dst, int64_t n, hipStream_t s);
void cast_bf16_to_f32(const void* src, float* dst, int64_t n, hipStream_t s);
void cast_f32_to_f16(const float* src, void* dst, int64_t n, hipStream_t s);
void cast_f16_to_f32(const void* src, float* dst, int64_t n, hipStream_t s);
// out[c][r] = in[r][c], bf16 [R][C] -> [C][R]
void transpose_bf16(const void* in, void* out, int64_t R, int64_t C, hipStream_t s);

struct SgdArgs {
  float lr;
  float momentum;
  float dampening;
  float weight_decay;
  bool nesterov;
  bool maximize;
  bool first_step;        // momentum buffer := grad
  const float* lr_ptr;    // optional device-resident lr (overrides `lr`; graph-capture friendly)
  const float* grad_scale_ptr;  // optional device scalar: grad *= 1/(*grad_scale_ptr)
};
// Graph-replay beacon (RcclPG watchdog): ++*dev_ctr, then the new value -> *host (host-coherent).
void replay_beacon_mark(unsigned long long* dev_ctr, unsigned long long* host, hipStream_t s);
// One kernel over a flat fp32 range (params / grads / momentum laid out identically).
void sgd_flat(float* p, const float* g, float* m, int64_t n, const SgdArgs& a, hipStream_t s);
// Multi-tensor: device table of {p, g, m, n} + chunk list {tensor, start}; one launch.
struct SgdTensor {
  float* p;
  const float* g;
  float* m;
  int64_t n;
};
void sgd_multi(const SgdTensor* table, const int64_t* chunks, int64_t nchunks, int64_t chunk_elems,
               const SgdArgs& a, hipStream_t s);

// Deterministic split-K reduction: out[i] = sum_s slabs[s * n + i] (fixed order).
void splitk_reduce(const float* slabs, int nslices, int64_t n, float* out, hipStream_t s);

// ---------------------------------------------------------------- xGMI collectives (xgmi.hip)
// Collectives over IPC-mapped peer staging memory; host side csrc/comm/xgmi_engine.cpp.
constexpr int kXgMaxRanks = 16;
constexpr int kXgThreads = 256;
constexpr int kXgSeg = kXgThreads * 16;  // bytes one workgroup moves per pass
enum XgKind : int {
  XG_BARRIER = 0,
  XG_ONESHOT = 1,         // all-reduce: push everything to everyone, local rank-order reduce
  XG_TWOSHOT = 2,         // all-reduce: reduce-scatter by push + all-gather by push
  XG_REDUCE_SCATTER = 3,
  XG_ALLGATHER = 4,
  XG_BROADCAST = 5,
  XG_SEND = 6,
  XG_RECV = 7,
};
enum XgDtype : int { XG_F32 = 0, XG_BF16, XG_F16, XG_F64, XG_I32, XG_I64, XG_I8, XG_U8 };
enum XgRed : int { XG_SUM = 0, XG_PROD, XG_MIN, XG_MAX };
struct XgArgs {
  char* stage[kXgMaxRanks];      // staging buffer of every rank (IPC-mapped; [rank] = mine)
  unsigned* flags[kXgMaxRanks];  // flag block of every rank (IPC-mapped)
  char* const* stage_tab;        // the same two tables in device memory (what the kernels index)
  unsigned* const* flag_tab;
  unsigned* epochs;              // local: [G] collective, [16][G] send per peer, [16][G] recv per peer
  int* error;                    // device address of a host-mapped word: set when a peer never arrived
  uint64_t timeout_ticks;        // wall_clock64 ticks (100 MHz)
  int world;
  int rank;
  int nblocks;                   // G: fixed for the group (segment ownership must not change)
  int64_t slot;                  // bytes per (parity, source) slot of regions A and B
  int64_t p2p_slot;              // bytes per (source, parity) slot of the send/recv region
  int64_t off_a, off_b, off_p2p; // region offsets inside every staging buffer
  // the op
  int kind;
  int dtype;
  int red;
  int average;                   // divide by world (float: * scale)
  float scale;
  int root;                      // broadcast
  int peer;                      // send: destination, recv: source
  const char* in;
  char* out;
  int64_t nbytes;                // oneshot/twoshot/broadcast/send/recv: message; RS/AG: per-rank block
  int64_t chunk;                 // twoshot: per-rank chunk (multiple of 16)
  int64_t stride;                // RS: input block stride, AG: output block stride (bytes)
};
void xgmi_collective(const XgArgs& a, hipStream_t s);

// ---------------------------------------------------------------- fp32 NCHW conv / pool (conv_f32.hip)
// stride-1 conv, square kernel R, symmetric zero padding; fc layers are R=1 convs over 1x1 images
struct ConvF32Geom {
  int64_t B;
  int C, H, W;     // input
  int Kout, R, pad;
  int OH, OW;      // output
};
// z = conv(x) + bias.  Input either fp32 `x` or raw uint8 `xu8` normalised on load ((v/255-mean)*inv_std).
void conv_f32_fwd(const ConvF32Geom& g, const float* x, const unsigned char* xu8, float mean, float inv_std,
                  const float* w, const float* bias, float* z, hipStream_t s);
// Fused conv + bias + ReLU + 2x2/s2 max-pool (OH, OW even): a = relu(maxpool(conv(x) + bias)) with
// the 1-byte argmax code of pool_relu_f32_fwd; the conv output is never written.
void conv_f32_fwd_pool(const ConvF32Geom& g, const float* x, const unsigned char* xu8, float mean, float inv_std,
                       const float* w, const float* bias, float* a, unsigned char* code, hipStream_t s);
// Same with the overlapping 2x2/s1 pool (fp32 input, OH * OW <= 128): one image per 128-row tile.
void conv_f32_fwd_pool_s1(const ConvF32Geom& g, const float* x, const float* w, const float* bias, float* a,
                          unsigned char* code, hipStream_t s);
// small-batch valid conv + ReLU + 2x2 pool (stride st) by split K: slab = conv_f32_fwd_slices(g) x B*Kout*OH*OW floats
int conv_f32_fwd_slices(const ConvF32Geom& g);
void conv_f32_fwd_pool_split(const ConvF32Geom& g, const float* x, const float* w, const float* bias, float* slab,
                             int slices, int st, float* a, unsigned char* code, hipStream_t s);
// slab: conv_f32_dgrad_slices(g) x B*C*H*W floats of split-K partials when that count is > 1 (else unused)
int conv_f32_dgrad_slices(const ConvF32Geom& g);
// The ConvNet's conv3 (128 -> 64 channels, 8x8 -> 10x10) and conv2 (64 -> 32, 11x11 -> 13x13) data gradients
// over the live taps only (scatter form, conv_f32.hip); ok: one of these geometries and a batch of at least two
// images per CU; wp: conv_dgrad_f32_scratch() floats
bool conv_dgrad_f32_scatter_ok(const ConvF32Geom& g);
int conv_dgrad_f32_scratch();
void conv_dgrad_f32_scatter(const ConvF32Geom& g, const float* dz, const float* w, float* dx, float* wp,
                            hipStream_t s);
void conv_f32_dgrad(const ConvF32Geom& g, const float* dz, const float* w, float* dx, float* slab, int slices,
                    hipStream_t s);
// The data gradient of a conv whose input came from a 2x2/s1 max-pool of a 11x11 map (the ConvNet's conv3 at small
// batches: split K) with that pool's backward in the same pass over the split-K planes: dzp [B][C][11][11].
// ok: split K applies, H = W = 10 and B*C a multiple of the pool tile; slab: conv_f32_dgrad_slices(g) planes.
bool conv_f32_dgrad_pool2s1_ok(const ConvF32Geom& g);
void conv_f32_dgrad_pool2s1_bwd(const ConvF32Geom& g, const float* dz, const float* w, float* slab, int slices,
                                const unsigned char* code, float* dzp, hipStream_t s);
// split-K weight (+ bias, when db != nullptr) gradient; slab: slices * Kout * (C*R*R + 1) floats
int conv_f32_wgrad_slices(const ConvF32Geom& g);
// One fixed-order slab reduction (f32_slab_reduce) as a segment of a multi-segment launch
struct F32RedSeg {
  const float* slab;
  int slices, Kout, Nw, ncol;
  float* dw;
  float* db;
};
using F32RedList = std::vector<F32RedSeg>;
// defer != null: the reduction is appended to *defer instead of launched (f32_slab_reduce_multi later)
void conv_f32_wgrad(const ConvF32Geom& g, const float* dz, const float* x, const unsigned char* xu8, float mean,
                    float inv_std, float* slab, int slices, float* dw, float* db, hipStream_t s,
                    F32RedList* defer = nullptr);
// Fixed-order sum of split-K slabs [slices][Kout][ncol] into dw [Kout][Nw] and (column Nw) db;
// the slab must hold f32_slab_capacity(slices) slices (room for the stage-1 group sums).
int f32_slab_capacity(int slices);
void f32_slab_reduce(float* slab, int slices, int Kout, int Nw, int ncol, float* dw, float* db, hipStream_t s);
// every segment's f32_slab_reduce in ONE launch (at most kF32RedMax segments), bit-identical to the two-stage form
constexpr int kF32RedMax = 8;
void f32_slab_reduce_multi(const F32RedList& segs, hipStream_t s);
// The ConvNet's conv1 (1->32, 5x5, pad 1, 28x28) + bias + ReLU + 2x2/s2 max-pool at fp32
// (conv1_f32.hip): a1 [B][32][13][13] and its argmax code; and its weight + bias gradient from the
// pooled gradient da1 and the code (the pool backward is folded in): per-workgroup partials in slab
// [conv1_f32_wgrad_blocks(B)][32][26] (capacity f32_slab_capacity of that), reduced into dw1, db1.
int conv1_f32_wgrad_blocks(int64_t B);
void conv1_pool_f32_fwd(const float* x, const unsigned char* xu8, int64_t B, float mean, float inv_std,
                        const float* w1, const float* b1, float* a1, unsigned char* code1, hipStream_t s);
void conv1_wgrad_f32(const float* x, const unsigned char* xu8, int64_t B, float mean, float inv_std, const float* da1,
                     const unsigned char* code1, float* slab, hipStream_t s);
// The fp32 ConvNet's cross-entropy backward + fc1 data gradient + pool3 backward in one launch (10 classes, 2048
// features = [128][4][4]): dl [B][10] (for fc1's weight gradient) and dz3 [B][128][8][8]
void fc_ce_pool3_bwd_f32(const float* logits, const int64_t* labels, const float* lse, const float* grad_out,
                         const float* denom, int ignore_index, float eps, int reduction, const float* wfc,
                         const unsigned char* code3, int B, float* dl, float* dz3, hipStream_t s);
// a = relu(maxpool_k,st(z)) with a 1-byte argmax code (255: no gradient); backward is a gather
void pool_relu_f32_fwd(const float* z, float* a, unsigned char* code, int64_t BC, int H, int W, int k, int st,
                       hipStream_t s);
void pool_relu_f32_bwd(const float* da, const unsigned char* code, float* dz, int64_t BC, int H, int W, int k,
                       int st, hipStream_t s);

// ---------------------------------------------------------------- cross entropy
// logits [B, C] fp32; labels int64 [B]; writes lse [B], loss scalar (or per-row for
// reduction none), denom (number of non-ignored rows) in ws.
// reduction: 0 none, 1 mean, 2 sum.  nparts = cross_entropy_parts(B, C) workgroups.
constexpr int kCeSmallC = 32;  // up to this many classes: one lane per row
inline int cross_entropy_parts(int B, int C) {
  const int rows_per_block = C <= kCeSmallC ? 256 : 4;
  const int n = (B + rows_per_block - 1) / rows_per_block;
  return n < 1 ? 1 : (n > 1024 ? 1024 : n);
}
void cross_entropy_fwd(const float* logits, const int64_t* labels, int B, int C, int ignore_index,
                       float label_smoothing, int reduction, float* lse, float* loss,
                       float* partials, unsigned* counter, int nparts, hipStream_t s);
void cross_entropy_bwd(const float* logits, const int64_t* labels, const float* lse,
                       const float* grad_out, const float* denom, int B, int C, int ignore_index,
                       float label_smoothing, int reduction, float* dlogits, hipStream_t s);

// ---------------------------------------------------------------- MNIST ConvNet
// Activations are NHWC bf16 (a1 [B,13,13,32], a2 [B,10,10,64], a3 [B,16 windows,128]); weights are
// PyTorch-layout fp32 masters, packed once per forward into bf16 MFMA fragments.
int64_t cn_packed_elems();
void cn_pack_weights(const float* w1, const float* w2, const float* w3, const float* wfc, void* out,
                     hipStream_t s);
// F1: conv1 + ReLU + pool1 (x u8 or fp32 [B,28,28]; normalisation fused).
// pack_w = {w1, w2, w3, wfc}: the same launch also packs every layer's weights into pack_out (then
// `packed` is not read: conv1 builds its fragments from w1).
void cn_conv1_fwd(const void* x, bool u8, const void* packed, const float* b1, void* a1, uint8_t* idx1,
                  int B, float mean, float inv_std, float in_scale, hipStream_t s,
                  const float* const* pack_w = nullptr, void* pack_out = nullptr);
// F2: conv2 + bias + ReLU + pool2 (2x2/s1) -> a2 [B,10,10,64] + pool2 codes idx2 [B,10,10,64]
// (0..3 = first-max position in the window, bit 2 = pooled value 0 / no gradient).
void cn_conv2_fwd(const void* a1, const void* packed, const float* b2, void* a2, uint8_t* idx2, int B,
                  hipStream_t s);
// F3: conv3 + ReLU + pool3 + fc1 on a2 -> logits (+ a3 [B,16,128] / argmax for backward).
void cn_conv3_fc_fwd(const void* a2, const void* packed, const float* b3, const float* bfc, float* logits,
                     void* a3, uint8_t* idx3, int B, hipStream_t s);

// F1+F2+F3 in one launch (conv1 -> conv2 -> conv3 + fc1 per image, a1 / a2 kept in LDS between the
// layers; also packs the bf16 weight fragments into `packed` for the backward).  w = {w1, w2, w3, wfc}.
void cn_forward_fused(const void* x, bool u8, const float* const* w, const float* b1, const float* b2,
                      const float* b3, const float* bfc, void* packed, void* a1, uint8_t* idx1, void* a2,
                      uint8_t* idx2, void* a3, uint8_t* idx3, float* logits, int B, float mean, float inv_std,
                      float in_scale, unsigned* sync, hipStream_t s, bool do_pack = true);
// SGD over the flat parameter range that also writes the updated ConvNet weights into their packed bf16
// fragments (cn_pack_weights layout); offsets[4]: first flat element of conv1 / conv2 / conv3 / fc1 weight
void cn_sgd_flat_pack(float* p, const float* g, float* m, int64_t n, const SgdArgs& a, const int64_t* offsets,
                      void* packed, hipStream_t s);  // sync: 2 zeroed words, self re-arming

// Workspace sizes (floats) of the backward weight-gradient slabs.
int64_t cn_fc_slab_floats(int B, bool dgrad);
int64_t cn_conv3_slab_floats(int B, bool dgrad);
int64_t cn_conv2_slab_floats(int B, bool dgrad);
int64_t cn_conv1_slab_floats(int B);
// One output range of the fixed-order slab reduction (sum over slices, optional layout transform).
struct ReduceSeg {
  const float* slabs;
  int64_t stride;  // floats between consecutive slices
  int64_t off;     // first float of this segment inside a slice
  int64_t n;       // outputs
  int nslices;
  float* out;
  int mode;  // 0: out[i] = sum; 1: conv transpose dWt[n = tap*cin + ci][co] -> W[co][ci][tap];
             // 2: fc1 slab in fc_bwd thread order (n*8 + j)*256 + t -> dWfc[n][co*16 + w]
  int cin, cout;
  int blocks;
  int vec;  // outputs per thread: 4 when off, stride and n are multiples of 4 floats (16-B loads), else 1
};
using ReduceList = std::vector<ReduceSeg>;
void cn_launch_reduce(const ReduceList& segs, hipStream_t s);  // one launch, at most 8 segments

// Cross entropy fused into the fc1 backward: the kernel forms dlogits itself from the forward's
// logits / log-sum-exp (ce_fwd_kernel) instead of reading a materialised [B,10] gradient.
struct CeFuse {
  const float* logits;
  const int64_t* labels;
  const float* lse;
  const float* grad_out;  // scalar (mean / sum) or [B] (none)
  const float* denom;     // ce_fwd's valid-row count (mean) - device scalar
  int ignore_index;
  float eps;
  int reduction;  // 0 none, 1 mean, 2 sum
};

// F3 backward: da3m is a [B,16,128] bf16 workspace; dz2 [B,11,11,64] (the gradient of conv2's
// pre-activation, through pool2 + ReLU) may be null (skip the data gradient).  Either dl ([B,10]
// fp32 logits gradient) or ce (fused cross entropy) is given.  defer != null: the weight-gradient
// reduction is appended to *defer instead of launched (the caller folds it into a later launch).
void cn_conv3_fc_bwd(const void* a2, const uint8_t* idx2, const void* a3, const uint8_t* idx3, const float* wfc,
                     const float* dl, const void* packed, void* da3m, void* dz2, int B, float* fc_slabs,
                     float* c3_slabs, float* dw3, float* db3, float* dwfc, float* dbfc, hipStream_t s,
                     const CeFuse* ce = nullptr, ReduceList* defer = nullptr);
// F2 backward: da1 may be null.
void cn_conv2_bwd(const void* a1, const void* dz2, const void* packed, void* da1, int B, float* slabs,
                  float* dw2, float* db2, hipStream_t s);
// F1 backward (weights only: the input needs no gradient).  idx1 bytes carry argmax | relu<<2, laid
// out [B][13 py][16 co/2][16 px][co&1] (px 13..15 zero).
// conv2 backward (dgrad + wgrad) fused with conv1 wgrad: da1 stays in LDS; one reduction launch for
// dW2/db2/dW1/db1.  slabs: cn_conv12_slab_floats(B) floats.
int64_t cn_conv12_slab_floats(int B);
void cn_conv12_bwd(const void* x, bool u8, const uint8_t* idx1, const void* a1, const void* dz2,
                   const void* packed, int B, float mean, float inv_std, float in_scale, float* slabs, float* dw2,
                   float* db2, float* dw1, float* db1, hipStream_t s, const ReduceList* extra = nullptr);
void cn_conv1_wgrad(const void* x, bool u8, const void* da1, const uint8_t* idx1, int B, float mean,
                    float inv_std, float in_scale, float* slabs, float* dw1, float* db1, hipStream_t s);

// ---------------------------------------------------------------- generic GEMM / implicit-GEMM conv
// (csrc/kernels/gemm.hip)  C[b][m][n] = epilogue(sum_k A(b, m, k) * B(b, n, k)), bf16 in, fp32 acc.
struct GemmOperand {
  const void* p;     // bf16
  int64_t ld;        // row stride (K-contiguous) or k stride (row-contiguous)
  int64_t bstride;   // batch stride (elements)
  bool row_contig;   // false: element (r, k) at p[r*ld + k]; true: at p[k*ld + r]
};
struct GemmEpilogue {
  enum Mode : int { kStore = 0, kSplitK = 1 };
  int mode;
  void* C;            // fp32 or bf16 [b][m][ldc]
  int64_t ldc, c_bstride;
  bool out_bf16;
  float alpha;
  const float* bias;  // [N] or null
  int act;            // 0 none, 1 relu, 2 gelu (erf), 3 gelu backward: C *= GELU'(preact) (preact is an input)
  void* preact;       // bf16 copy of the value before residual/activation (same layout as C) or null;
                      // with act 3 it is read: the forward's pre-activation
  const void* residual;  // bf16, same layout as C, added before the activation
  float* stats;       // [b][tiles_m][2][N] per-channel sum / sumsq partials of the stored C, or null
  float* partial;     // split-K fp32 partials [b*splits][M][N]
  const float* scale_a;  // optional device per-tensor dequant scales (fp8 GEMM): C *= scale_a[0]*scale_b[0]
  const float* scale_b;
  int store_mode;     // set by the 256x256 launchers (bf16 output): 0 8-B stores, 1 16-B stores after a lane
                      // exchange, 2 staged through LDS into whole 128-B rows, 3 discard (probe only)
  bool store_rot;     // mode 2: rotate the row order per wave tile (spreads concurrent rows over channels)
  int store_cache;    // 256x256 kernels' 16-B output stores: 0 plain, 1 nontemporal, 2 write-through sc1
  void* sink;         // persistent 256x256 kernels: >= 16 B target of the stores past the M / N edge (set by
                      // the launcher)
  // e4m3 outputs instead of C (256x256 fp8 kernel only): the final value v (after bias / GELU / GELU backward,
  // rounded to bf16 as a stored C would be) is quantised with the delayed scale q8_amax[0] / 448 (clamped to
  // +-448) into q8 [M][N] and its transpose q8t [N][M]; q8_scale[0] <- that scale; q8_tmax[tile * 8 + wave]
  // <- |v|max of each wave's 128 x 64 outputs (the next roll).
  // colsum_part (nullable; the fp8 q8 path, and bf16 outputs of the 256x256 phased kernel) [tiles_m * 2][N] <- the
  // column sums of the stored (bf16-rounded) values over each wave's 128 rows (a bias gradient)
  uint8_t* q8;
  uint8_t* q8t;
  const float* q8_amax;
  float* q8_scale;
  float* q8_tmax;
  float* colsum_part;
};
struct ConvGeom {
  int N, H, W, C;   // input NHWC (C padded to a multiple of 8)
  int K, R, S;      // output channels, filter
  int P, Q;         // output spatial
  int stride, pad, dil;
};
void gemm_bf16(const GemmOperand& A, const GemmOperand& B, int batch, int M, int N, int K, const GemmEpilogue& ep,
               int splits, hipStream_t s);
// e4m3 x e4m3 (both K-contiguous; ld / bstride / K in BYTES, multiples of 16) on the block-scaled
// MFMA (v_mfma_scale_f32_16x16x128_f8f6f4, unit block scales; per-tensor scales via ep.scale_a/b).
void gemm_fp8(const GemmOperand& A, const GemmOperand& B, int batch, int M, int N, int Kbytes, const GemmEpilogue& ep,
              int splits, hipStream_t s);
// the 256x256 e4m3 kernel behind gemm_fp8 (false = shape not supported, nothing launched)
void set_bf16_tile_mode(int mode);  // 0 auto, 128 / 256 forced (A/B measurements)
// tile-maximum slots and colsum partial rows of a gemm_fp8 launch with e4m3 outputs (ep.q8)
int64_t gemm_fp8_q8_slots(int M, int N);
int64_t gemm_fp8_colsum_part_rows(int M);
// 256x256 bf16 kernel for K-contiguous A and B (gemm_bf16_256.hip); false when the shape/layout is not
// supported (the caller falls back to the 128x128 core).  K in elements.
bool gemm_bf16_256(const GemmOperand& A, const GemmOperand& B, int batch, int M, int N, int K,
                   const GemmEpilogue& ep, int splits, hipStream_t s);
void set_gemm256_persist(int on);  // A/B: 1 persistent phased kernel (default), 0 one workgroup per tile
void set_gemm256_phased(int on);  // A/B: 1 phased pipeline (default), 0 the single-stage-wait kernel
void set_gemm_wide_store(int mode);
void set_gemm_two_wg(int mode, int group_m);  // bf16 K-contiguous GEMMs on the 2-workgroup 256x128 kernel: 0 never (default), 1 always, 2 N <= 1024
void set_gemm_store_cache(int flavour);  // A/B: GemmEpilogue::store_cache of the 256x256 kernels  // A/B: epilogue store mode of the 256x256 kernels (GemmEpilogue::store_mode)
int gemm_wide_store_mode();         // RINGDP_GEMM_WIDE_STORE (default 2)
int gemm_store_cache();             // RINGDP_GEMM_STORE_CACHE (default 0)
bool gemm_fp8_256(const GemmOperand& A, const GemmOperand& B, int batch, int M, int N, int Kbytes,
                  const GemmEpilogue& ep, int splits, hipStream_t s);
// split-K count gemm_fp8 should be called with for an (M x N) fp32-partial GEMM (fills whole CU rounds)
int gemm_fp8_pick_splits(int M, int N, int Kbytes, int requested);
int gemm_bf16_pick_splits(int M, int N, int K, int requested);
void set_fp8_tile_mode(int mode);  // 0 auto, 128 / 256 force a kernel (tests, A/B runs)
// per-tensor fp8 quantisation (fp8.hip): amax -> scale = amax / 448 -> e4m3, optionally transposed
void fp8_amax(const void* x, int64_t n, float* amax, hipStream_t s);
void fp8_quantize(const void* x, int64_t rows, int64_t cols, bool transpose, const float* amax, void* out,
                  float* scale, hipStream_t s, void* out_rowmajor = nullptr);
// delayed scaling: hist = {amax to scale by, per-64x64-tile |x|max of the last call...}; hist[0] is
// rolled from the tile maxima (or, init = first call of a site, measured exactly), then x is quantised
// (q^T into out_t, q into out_rowmajor) while its tile maxima are written for the next call.
// tile counts of the quantise(+transpose) pass: per-tile amax slots and colsum partial rows
int64_t fp8_quant_tiles(int64_t rows, int64_t cols);
int64_t fp8_quant_row_tiles(int64_t rows);
void fp8_quantize_delayed(const void* x, int64_t rows, int64_t cols, float* hist, bool init, void* out_t,
                          float* scale, void* out_rowmajor, hipStream_t s, float* colsum_part = nullptr,
                          const void* gelu_pre = nullptr, bool roll = true);
// the rolls of many sites in one launch (one workgroup per site): hist_i[0] <- max hist_i[1 .. 1+n_i) when
// that is > 0.  A training step rolls every site once before its first quantisation (roll = false above)
void fp8_roll_many(float* const* hists, const int* ns, int count, hipStream_t s);
void fp8_roll(float* hist, int n, hipStream_t s);
// delayed-scaling quantise + transpose of many fp32 matrices (a model's weights) in one launch: entry i covers
// blocks [tile0, tile0 + its 128 x 64 tile count); hist as fp8_quantize_delayed's (already rolled)
struct QuantTEntry {
  const float* src;  // [rows][cols] fp32 (quantised from its bf16 rounding)
  int64_t rows, cols;
  float* hist;
  uint8_t* q;   // [rows][cols] e4m3
  uint8_t* qt;  // [cols][rows] e4m3
  float* scale;
  int tile0;
};
constexpr int kQuantTMax = 60;  // 60 x 64 B + header < the 4 KiB kernel-argument limit
struct QuantTTable {
  int n;
  int total_tiles;
  QuantTEntry e[kQuantTMax];
};
void fp8_quantize_multi(const QuantTTable& t, hipStream_t s);  // one site: hist[0] <- max hist[1 .. 1+n) when > 0
// column sums of a bf16 [rows][cols] matrix as colsum_parts(rows) fp32 partial rows (sum them with splitk_sum;
// fp8_quantize_delayed's colsum_part has one partial row per 64-row tile instead)
int colsum_parts(int64_t rows);
void colsum_bf16(const void* x, int64_t rows, int64_t cols, float* part, hipStream_t s);
// out[c] = sum_s part[s][c] for many partial rows (n % 4 == 0), fixed order
void rowsum_f32(const float* part, int S, int64_t n, float* out, hipStream_t s);
// w_krsc rows are ldw elements apart (>= R*S*C; a multiple of 64 enables the C = 8 stem path)
// splits > 1 (aligned C % 64 / pointwise paths only): ep must be kSplitK with a [splits][M][N] partial;
// finish with splitk_finish
void conv_fwd_bf16(const void* x, const void* w_krsc, int64_t ldw, const ConvGeom& g, const GemmEpilogue& ep,
                   hipStream_t s, int splits = 1);
void conv_dgrad_bf16(const void* dy, const void* w_crsk, const ConvGeom& g, const GemmEpilogue& ep, hipStream_t s,
                     int splits = 1);
int conv_gemm_splits(int M, int N, int K);
int splitk_finish_groups(int M);
// out (bf16, ldc) = sum of S fp32 partials [S][M][N] (+ residual); mid (nullable) = [groups][2][N] stats
void splitk_finish(const float* part, int S, int M, int N, void* out, int64_t ldc, const void* residual, float* mid,
                   hipStream_t s);
void conv_wgrad_bf16(const void* dy, const void* x, const ConvGeom& g, int splits, float* partial, float* dw_kcrs,
                     hipStream_t s);
int conv_wgrad_splits(const ConvGeom& g, int cus);
void splitk_sum(const float* part, int S, int64_t n, float* out, hipStream_t s);
// out0[c] = sum_t part[t][0][c], out1[c] = sum_t part[t][1][c]  (two-level, fixed order)
int reduce_parts_scratch_floats(int nparts, int N);
void reduce_parts(const float* part, int nparts, int N, float* scratch, float* out0, float* out1, hipStream_t s);
// first level only: part [nparts][2][N] -> mid [G][2][N]; returns G
int reduce_parts_groups(int nparts);
int reduce_parts_l1(const float* part, int nparts, int N, float* mid, hipStream_t s);
int gemm_tiles_m(int M);

// ---------------------------------------------------------------- NHWC network layers (nn.hip)
// w_krsc rows are ldk >= R*S*Cp elements (zero tail)
void pack_conv_weight(const float* w_kcrs, int K, int C, int R, int S, int Cp, int ldk, void* w_krsc, void* w_crsk,
                      hipStream_t s);
struct CastEntry {
  const float* src;
  void* dst;       // bf16
  int64_t start4;  // first 4-element vector of this tensor in the launch's index space
};
constexpr int kCastMax = 96;  // 96 x 24 B + header < the 4 KiB kernel-argument limit
struct CastTable {
  int n;
  int64_t total4;
  CastEntry e[kCastMax];
};
void cast_f32_to_bf16_multi(const CastTable& t, hipStream_t s);
struct CastTEntry {
  const float* src;  // [R][C] fp32
  void* dst;         // [R][C] bf16
  void* dst_t;       // [C][R] bf16
  int R, C;
  int start_tile;    // first 64x64 tile of this matrix in the launch
};
constexpr int kCastTMax = 96;  // 96 x 40 B + header < the 4 KiB kernel-argument limit
struct CastTTable {
  int n;
  int total_tiles;
  CastTEntry e[kCastTMax];
};
void cast_t_multi(const CastTTable& t, hipStream_t s);
struct PackEntry {
  const float* w;
  void* krsc;  // bf16
  void* crsk;  // bf16
  int64_t start;       // first KRSC element of this weight in the launch's flat index space
  int64_t start_tile;  // first 64x64 CRSK transpose tile
  int K, C, R, S, Cp, ldk;
  int start_tile2;     // first (32 k x kPackCt(Cp) c x R*S) tile of the one-launch pack (pack_both_multi_kernel)
};
// channels per tile of the one-launch pack: every channel of the stem (7x7, Cp = 8), 32 otherwise
inline int pack_ct(int Cp) { return Cp < 32 ? Cp : 32; }
inline int pack_tiles2(int K, int Cp) { return ((K + 31) / 32) * ((Cp + pack_ct(Cp) - 1) / pack_ct(Cp)); }
constexpr int kPackMax = 48;  // 48 x 72 B + header < the 4 KiB kernel-argument limit
struct PackTable {
  int n;
  int64_t total, total_tiles;
  int total_tiles2;
  PackEntry e[kPackMax];
};
void pack_conv_weights(const PackTable& t, hipStream_t s);
void nchw_to_nhwc_pad(const void* x, bool x_bf16, int N, int C, int H, int W, int Cp, void* y, hipStream_t s);
// batch norm (training): sums = [sum(C), sumsq(C)] over M rows -> scale/shift (+ saved mean/invstd,
// running-stat update), then y = act(z*scale + shift [+ res])
// sums: G group partials [G][2][C] (reduce_parts_l1); num_batches_tracked (nullable) is incremented
void bn_prepare(const float* sums, int G, int64_t M, int C, const float* gamma, const float* beta, float eps,
                float momentum, float* running_mean, float* running_var, float* scale_shift, float* save,
                int64_t* num_batches_tracked, hipStream_t s);
void bn_act_fwd(const void* z, const float* scale_shift, const void* res, bool relu, int64_t M, int C, void* y,
                hipStream_t s);
// bn_prepare + bn_act_fwd as one launch when the group partials are few (G * C <= 8192): every workgroup forms
// the scale / shift itself (same fixed order, same bits); save / running stats / nbt written once
bool bn_fold_ok(int G, int C);
void bn_fold_act_fwd(const float* sums, int G, int64_t M, int C, const float* gamma, const float* beta, float eps,
                     float momentum, float* running_mean, float* running_var, float* save,
                     int64_t* num_batches_tracked, const void* z, const void* res, bool relu, void* y, hipStream_t s);
// backward part 1: g = dy * (y > 0 if relu); partial sums of g and g*zhat per channel -> part
// BN statistics of a stored bf16 z [M][C] (C % 8 == 0, C <= 2048): partials [bn_bwd_parts(M, C)][2][C]
// (sum, sum of squares); returns the partial count.
int bn_col_stats(const void* z, int64_t M, int C, float* part, hipStream_t s);
int bn_bwd_parts(int64_t M, int C);
// ss != nullptr (bn_bwd_zmask_ok(C)): the ReLU mask from z and the forward's scale / shift instead of y; g_out may
// be nullptr (the masked gradient is not stored)
void bn_bwd_reduce(const void* dy, const void* y, const void* z, const float* save, const float* ss, bool relu,
                   int64_t M, int C, float* part, void* g_out, hipStream_t s);
bool bn_bwd_zmask_ok(int C);
// part 2: dgamma/dbeta and dz = scale*(g - mean(g) - zhat*mean(g*zhat))/..., plus d(residual) = g.  With ss, g is
// the unmasked dy and the mask is re-derived from z as in part 1.
void bn_bwd_apply(const float* part, int nparts, float* scratch, const void* g, const void* z, const float* save,
                  const float* ss, const float* gamma, int64_t M, int C, float* dgamma, float* dbeta, void* dz,
                  hipStream_t s);
void maxpool_fwd(const void* x, int N, int H, int W, int C, int k, int stride, int pad, int P, int Q, void* y,
                 uint8_t* arg, hipStream_t s);
void maxpool_bwd(const void* dy, const uint8_t* arg, int N, int H, int W, int C, int k, int stride, int pad, int P,
                 int Q, void* dx, hipStream_t s);
void avgpool_fwd(const void* x, int N, int HW, int C, void* y, hipStream_t s);
void avgpool_bwd(const void* dy, int N, int HW, int C, void* dx, hipStream_t s);
void add_bf16(const void* a, const void* b, int64_t n, void* y, hipStream_t s);
// classifier head, few classes (J <= 16, C % 8 == 0, C/8 divides 256): x [N][HW][C] bf16 -> pooled [N][C] fp32
// (window mean) and logits [N][J] fp32 = pooled W^T + b; backward from dl [N][J] or a fused cross entropy (ce):
// dx [N][HW][C] bf16, dw [J][C], db [J] (written, not accumulated)
bool head_ok(int C, int J);
void head_fwd(const void* x, int N, int HW, int C, int J, const float* w, const float* b, float* pooled,
              float* logits, hipStream_t s);
void head_bwd(const float* dl, const CeFuse* ce, const float* pooled, const float* w, int N, int HW, int C, int J,
              void* dx, float* dw, float* db, hipStream_t s);

// ---------------------------------------------------------------- transformer layers (vit.hip)
void layernorm_fwd(const void* x, const float* w, const float* b, int64_t rows, int D, float eps, void* y,
                   float* stats, hipStream_t s);
int layernorm_bwd_scratch_floats(int64_t rows, int D);
// LayerNorm forward with e4m3 outputs (q [rows][D], qt [D][rows]) at the delayed scale amax[0] / 448; tmax gets one
// |y|max per 64-row block (layernorm_q8_blocks); rows % 16 == 0, D % 8 == 0, D <= 2048
int64_t layernorm_q8_blocks(int64_t rows);
void layernorm_fwd_q8(const void* x, const float* w, const float* b, int64_t rows, int D, float eps, float* stats,
                      const float* amax, void* q, void* qt, float* scale, float* tmax, hipStream_t s);
// cs_part (nullable): [layernorm_bwd_blocks(rows)][D] per-block column sums of dx (the bias gradient of the
// linear whose output gradient dx is)
int layernorm_bwd_blocks(int64_t rows);
void layernorm_bwd(const void* dy, const void* x, const float* stats, const float* w, const void* dres, int64_t rows,
                   int D, void* dx, float* scratch, float* dw, float* db, hipStream_t s, float* cs_part = nullptr);
void qkv_split(const void* qkv, int B, int T, int H, int Dh, int Tp, void* q, void* k, void* v, hipStream_t s);
void qkv_merge(const void* dq, const void* dk, const void* dv, int B, int T, int H, int Dh, int Tp, void* dqkv,
               hipStream_t s);
void heads_to_rows(const void* o, int B, int T, int H, int Dh, int Tp, void* rows, hipStream_t s);
void rows_to_heads(const void* rows, int B, int T, int H, int Dh, int Tp, void* o, hipStream_t s);
void softmax_fwd(const float* scores, int64_t rows, int T, int Tp, float scale, void* p, hipStream_t s);
// fused attention forward (head dim 64, Tp % 16 == 0, Tp <= 256): P = softmax(scale Q K^T) over the T real
// keys (bf16 [BH][Tp][Tp], padded query rows 0) and O = P V (bf16 [BH][Tp][64]); false = unsupported shape
bool attn_fwd(const void* q, const void* k, const void* v, int BH, int T, int Tp, int Dh, float scale, void* p,
              void* o, hipStream_t s);
// fused dP = dO V^T + softmax backward: dS = scale * P * (dP - rowsum(dP * P)) (bf16 [BH][Tp][Tp])
bool attn_bwd_ds(const void* dout, const void* v, const void* p, int BH, int Tp, int Dh, float scale, void* ds,
                 hipStream_t s);
// fused attention backward (head dim 64, Tp <= 256): dQ, dK, dV straight into the dqkv rows [B*T][3*H*Dh];
// dsum = [B*H][Tp] fp32 scratch
bool attn_bwd(const void* dout, const void* q, const void* k, const void* v, const void* p, int B, int T, int H,
              int Tp, int Dh, float scale, float* dsum, void* dqkv, hipStream_t s);
// the same kernels reading the qkv projection rows [B*T][3*H*64] and writing the output rows [B*T][H*64]
// (forward) / taking dO rows [B*T][H*64] (backward): no head-major split, merge or transposes
bool attn_fwd_rows(const void* qkv, int B, int T, int H, int Tp, int Dh, float scale, void* p, void* out,
                   hipStream_t s);
// P-recompute variants: the forward stores the per-query log-sum-exp lse [B*H][Tp] instead of P
bool attn_fwd_rows_lse(const void* qkv, int B, int T, int H, int Tp, int Dh, float scale, float* lse, void* out,
                       hipStream_t s);
// colsum_part (nullable): [B][3*H*64] per-batch column sums of dqkv (the qkv bias gradient before the sum over B)
bool attn_bwd_rows_lse(const void* dout_rows, const void* qkv, const float* lse, int B, int T, int H, int Tp, int Dh,
                       float scale, float* dsum, void* dqkv, hipStream_t s, float* colsum_part = nullptr);
bool attn_bwd_rows(const void* dout_rows, const void* qkv, const void* p, int B, int T, int H, int Tp, int Dh,
                   float scale, float* dsum, void* dqkv, hipStream_t s);
void softmax_bwd(const void* p, const float* dp, int64_t rows, int T, int Tp, float scale, void* ds, hipStream_t s);
void gelu_bwd(const void* dy, const void* pre, int64_t n, void* dx, hipStream_t s);
void gelu_fwd(const void* x, int64_t n, void* y, hipStream_t s);  // n % 8 == 0
void assemble_tokens(const void* patches, const float* cls, const float* pos, int B, int NP, int D, void* out,
                     hipStream_t s);
void assemble_tokens_bwd(const void* dout, int B, int NP, int D, void* dpatches, float* dpos, float* dcls,
                         hipStream_t s);
void cls_rows(const void* x, int B, int T, int D, void* y, bool reverse, hipStream_t s);
void patchify(const void* x, bool x_bf16, int B, int C, int H, int W, int P, void* out, hipStream_t s);

// ---------------------------------------------------------------- data
// Gather B samples of a uint8 (N, H, W, C) dataset by index, random-crop (zero pad) + h-flip, then
// ToTensor + Normalize; out_kind 0 = fp32, 1 = bf16, 2 = uint8 (no normalisation).  Output NCHW
// (or NHWC when nhwc).  yout[b] = labels[idx[b]] when labels != nullptr.
struct AugNorm {
  float mean[4];
  float inv_std[4];
};
void gather_augment(const uint8_t* x, const int64_t* labels, const int64_t* idx, int B, int H, int W, int C,
                    int pad, bool flip, const AugNorm& nrm, uint64_t seed, bool nhwc, int out_kind, void* out,
                    int64_t* yout, hipStream_t s);
// Synthetic MNIST-shaped batch (u8 images + labels) from a counter-based hash (deterministic).
void synth_u8_images(uint8_t* x, int64_t* labels, int B, int HW, int num_classes, uint64_t seed,
                     hipStream_t s);

}  // namespace kern
}  // namespace ringdp
