// hipBLASLt backend for plain dense GEMMs (the ViT linears, fc layers): the library's tuned gfx950
// kernels beat ringdp's generic 128x128 / 256x256 MFMA cores by 1.5-3x on these shapes
// (tools/gemm256_ab.py), and plain library GEMMs are exactly what hipBLASLt is for.  Everything
// fused or gathered (implicit-GEMM convs with BN statistics, attention, the ConvNet blocks) stays on
// ringdp's own kernels.
//
// Mapping: ringdp computes row-major C[m][n] = sum_k A(m,k) B(n,k).  A row-major C is the column-major
// C^T (N x M, ld = ldc), so hipBLASLt computes D = op(Bs) * op(As) with the B side as its "A":
//   B K-contiguous (B(n,k) at n*ldb + k)  -> column-major K x N, op T;  row-contiguous -> N x K, op N
//   A K-contiguous (A(m,k) at m*lda + k)  -> column-major K x M, op N;  row-contiguous -> M x K, op T
// Bias (length N = rows of D), GELU-with-aux (pre-activation output) and the residual as C with
// beta = 1 map onto hipBLASLt epilogues.  Algorithms come from the library heuristic once per
// problem signature and are cached; the workspace is allocated once per device.  Calls are
// stream-ordered and hipGraph-capturable.
#include "blaslt.h"

#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>

#include "../common.h"
#include "../kernels/kernels.h"

namespace ringdp {
namespace blaslt {

namespace {

constexpr size_t kWorkspace = 64ull << 20;

#define LT_CHECK(expr)                                                                             \
  do {                                                                                             \
    hipblasStatus_t _s = (expr);                                                                   \
    if (_s != HIPBLAS_STATUS_SUCCESS)                                                              \
      throw RingdpError(strcat_all("[ringdp] hipBLASLt error ", static_cast<int>(_s), " at ",      \
                                   __FILE__, ":", __LINE__, " (", #expr, ")"));                    \
  } while (0)

struct DeviceState {
  hipblasLtHandle_t handle = nullptr;
  void* workspace = nullptr;
};

std::mutex g_mu;
std::map<int, DeviceState> g_dev;

using Key = std::tuple<int, int, int, int, int64_t, int64_t, int64_t, int, int, int, int, int, int, int64_t,
                       int64_t, int64_t, int>;
std::map<Key, hipblasLtMatmulAlgo_t> g_algos;
std::map<Key, bool> g_unsupported;

DeviceState& state(int dev) {
  auto& s = g_dev[dev];
  if (!s.handle) {
    LT_CHECK(hipblasLtCreate(&s.handle));
    RINGDP_CHECK(hipMalloc(&s.workspace, kWorkspace) == hipSuccess, "hipBLASLt workspace allocation failed");
  }
  return s;
}

}  // namespace

static int g_on = -1;  // -1: read RINGDP_GEMM_BACKEND on first use
bool enabled() {
  if (g_on < 0) {
    const char* v = std::getenv("RINGDP_GEMM_BACKEND");
    g_on = (v && std::strcmp(v, "ringdp") == 0) ? 0 : 1;
  }
  return g_on == 1;
}
void set_enabled(bool on) { g_on = on ? 1 : 0; }

static bool matmul_once(const Problem& p, hipStream_t stream);

bool matmul(const Problem& p, hipStream_t stream) {
  if (matmul_once(p, stream)) return true;
  // hipBLASLt has no GELU-aux algorithm for some large shapes (ViT-B/16 fc1 forward, 25216x3072x768):
  // bias epilogue into the pre-activation, then one GELU pass (2 bytes/elem in and out). Measured
  // faster than ringdp's fused 256x256 kernel there (tools/gpu_vit.sh).
  if (enabled() && p.act == 2 && p.preact && p.out_bf16 && !p.residual && p.ldc == p.N &&
      (p.batch == 1 || p.c_bstride == (int64_t)p.M * p.N) && ((int64_t)p.M * p.N * p.batch) % 8 == 0) {
    Problem q = p;
    q.act = 0;
    q.preact = nullptr;
    q.C = p.preact;
    if (!matmul_once(q, stream)) return false;
    kern::gelu_fwd(p.preact, (int64_t)p.M * p.N * p.batch, p.C, stream);
    return true;
  }
  // likewise no DGELU algorithm (same ViT shape): plain GEMM, then C *= GELU'(preact) in place - ringdp's
  // own fused epilogue runs this short-K shape 1.7x slower than the pair
  if (enabled() && p.act == 3 && p.preact && p.out_bf16 && !p.residual && !p.bias && p.ldc == p.N &&
      (p.batch == 1 || p.c_bstride == (int64_t)p.M * p.N) && ((int64_t)p.M * p.N * p.batch) % 8 == 0) {
    Problem q = p;
    q.act = 0;
    q.preact = nullptr;
    if (!matmul_once(q, stream)) return false;
    kern::gelu_bwd(p.C, p.preact, (int64_t)p.M * p.N * p.batch, p.C, stream);
    return true;
  }
  return false;
}

static bool matmul_once(const Problem& p, hipStream_t stream) {
  if (!enabled()) return false;
  if (p.M <= 0 || p.N <= 0 || p.K <= 0) return false;
  if (p.residual && p.act) return false;             // ringdp adds the residual after storing preact
  if (p.residual && !p.out_bf16) return false;       // C and D share a type
  if (p.preact && p.act != 2 && p.act != 3) return false;
  if (p.act == 3 && (!p.preact || p.bias || p.residual || !p.out_bf16)) return false;
  if (p.act == 1) return false;                      // ReLU layers are ringdp-fused (BN) anyway
  // Measured (tools/blaslt_check.py, ViT-B/16 shapes): the library wins on K-contiguous operands
  // (forward linears: 35-118 us vs 52-201 us with the bias epilogue) and loses on row-contiguous ones
  // (weight gradients 135-275 us vs 66-195 us): those stay on ringdp's kernels.
  static const int row_ok = [] {
    const char* v = std::getenv("RINGDP_BLASLT_ROW");
    return v ? std::atoi(v) : 2;  // batched row-contiguous (attention-shaped): 75 vs 91-97 us, attn_gemm_ab.py
  }();
  // batched attention-shaped problems (RINGDP_BLASLT_ROW=2) or everything (=1): A/B runs
  if ((p.a_row || p.b_row) && !(p.allow_row || row_ok == 1 || (row_ok == 2 && p.batch > 1))) return false;
  int dev = 0;
  hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceState& st = state(dev);

  const hipblasOperation_t opA = p.b_row ? HIPBLAS_OP_N : HIPBLAS_OP_T;  // hipBLASLt "A" = our B
  const hipblasOperation_t opB = p.a_row ? HIPBLAS_OP_T : HIPBLAS_OP_N;  // hipBLASLt "B" = our A
  // stored shapes (column-major rows x cols)
  const int64_t a_rows = p.b_row ? p.N : p.K, a_cols = p.b_row ? p.K : p.N;
  const int64_t b_rows = p.a_row ? p.M : p.K, b_cols = p.a_row ? p.K : p.M;
  const hipDataType dtD = p.out_bf16 ? HIP_R_16BF : HIP_R_32F;
  hipblasLtEpilogue_t epi = HIPBLASLT_EPILOGUE_DEFAULT;
  if (p.act == 2) epi = p.preact ? (p.bias ? HIPBLASLT_EPILOGUE_GELU_AUX_BIAS : HIPBLASLT_EPILOGUE_GELU_AUX)
                                 : (p.bias ? HIPBLASLT_EPILOGUE_GELU_BIAS : HIPBLASLT_EPILOGUE_GELU);
  else if (p.act == 3) epi = HIPBLASLT_EPILOGUE_DGELU;  // aux = the forward's pre-activation (input)
  else if (p.bias) epi = HIPBLASLT_EPILOGUE_BIAS;

  const Key key{p.M, p.N, p.K, p.batch, p.lda, p.ldb, p.ldc, p.a_row, p.b_row, p.out_bf16, (int)epi,
                p.residual != nullptr, dev, p.a_bstride, p.b_bstride, p.c_bstride, p.fp8 ? 1 : 0};
  const hipDataType dtIn = p.fp8 ? HIP_R_8F_E4M3 : HIP_R_16BF;
  if (g_unsupported.count(key)) return false;

  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr, ld = nullptr;
  hipblasLtMatmulPreference_t pref = nullptr;
  auto cleanup = [&] {
    if (pref) hipblasLtMatmulPreferenceDestroy(pref);
    if (la) hipblasLtMatrixLayoutDestroy(la);
    if (lb) hipblasLtMatrixLayoutDestroy(lb);
    if (lc) hipblasLtMatrixLayoutDestroy(lc);
    if (ld) hipblasLtMatrixLayoutDestroy(ld);
    if (desc) hipblasLtMatmulDescDestroy(desc);
  };
  try {
    LT_CHECK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opA, sizeof(opA)));
    LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opB, sizeof(opB)));
    LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
    if (p.fp8) {  // hipBLASLt "A" is our B
      if (p.scale_b)
        LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_A_SCALE_POINTER, &p.scale_b, sizeof(void*)));
      if (p.scale_a)
        LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_B_SCALE_POINTER, &p.scale_a, sizeof(void*)));
    }
    if (p.bias) {
      const hipDataType bt = HIP_R_32F;
      LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &p.bias, sizeof(void*)));
      LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
    }
    if (p.preact) {
      const int64_t aux_ld = p.ldc;
      const hipDataType at = HIP_R_16BF;
      LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &p.preact,
                                               sizeof(void*)));
      LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &aux_ld, sizeof(aux_ld)));
      LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at, sizeof(at)));
      if (p.batch > 1) {
        const int64_t abs = p.c_bstride;
        LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_BATCH_STRIDE, &abs,
                                                 sizeof(abs)));
      }
    }
    LT_CHECK(hipblasLtMatrixLayoutCreate(&la, dtIn, a_rows, a_cols, p.ldb));
    LT_CHECK(hipblasLtMatrixLayoutCreate(&lb, dtIn, b_rows, b_cols, p.lda));
    LT_CHECK(hipblasLtMatrixLayoutCreate(&lc, dtD, p.N, p.M, p.ldc));
    LT_CHECK(hipblasLtMatrixLayoutCreate(&ld, dtD, p.N, p.M, p.ldc));
    if (p.batch > 1) {
      const int32_t bc = p.batch;
      for (auto* l : {la, lb, lc, ld})
        LT_CHECK(hipblasLtMatrixLayoutSetAttribute(l, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc, sizeof(bc)));
      LT_CHECK(hipblasLtMatrixLayoutSetAttribute(la, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &p.b_bstride,
                                                 sizeof(int64_t)));
      LT_CHECK(hipblasLtMatrixLayoutSetAttribute(lb, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &p.a_bstride,
                                                 sizeof(int64_t)));
      LT_CHECK(hipblasLtMatrixLayoutSetAttribute(lc, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &p.c_bstride,
                                                 sizeof(int64_t)));
      LT_CHECK(hipblasLtMatrixLayoutSetAttribute(ld, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &p.c_bstride,
                                                 sizeof(int64_t)));
    }
    auto it = g_algos.find(key);
    if (it == g_algos.end()) {
      LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
      const uint64_t ws = kWorkspace;
      LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws)));
      hipblasLtMatmulHeuristicResult_t res{};
      int n = 0;
      if (hipblasLtMatmulAlgoGetHeuristic(st.handle, desc, la, lb, lc, ld, pref, 1, &res, &n) !=
              HIPBLAS_STATUS_SUCCESS ||
          n < 1) {
        if (std::getenv("RINGDP_BLASLT_DEBUG"))
          std::fprintf(stderr, "[ringdp] hipBLASLt: no algorithm for M=%d N=%d K=%d batch=%d epilogue=%d fp8=%d "
                               "residual=%d out_bf16=%d; using ringdp's kernel\n",
                       p.M, p.N, p.K, p.batch, (int)epi, (int)p.fp8, p.residual != nullptr, (int)p.out_bf16);
        g_unsupported[key] = true;
        cleanup();
        return false;
      }
      it = g_algos.emplace(key, res.algo).first;
    }
    const float alpha = p.alpha, beta = p.residual ? 1.f : 0.f;
    const void* cptr = p.residual ? p.residual : p.C;
    LT_CHECK(hipblasLtMatmul(st.handle, desc, &alpha, p.B, la, p.A, lb, &beta, cptr, lc, p.C, ld, &it->second,
                             st.workspace, kWorkspace, stream));
  } catch (...) {
    cleanup();
    throw;
  }
  cleanup();
  return true;
}

}  // namespace blaslt
}  // namespace ringdp
