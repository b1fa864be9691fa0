// Library GEMM path of tt_gemm: the plain bf16 input projection (C = A B^T + bias, both
// operands K-contiguous, bf16 out) through hipBLASLt. Host code only.
//
// Why: on the layer-1 input projection (M = B*T = 524288, N = 6H = 3072, K = 2H = 1024 per
// tower) hipBLASLt's stream-K 256x256 kernel runs 2.86 ms per tower against 3.5 ms for
// gemm_persist (tools/bench_blaslt.py, profiles/r05_blaslt_shapes.txt); at K 320 (layer 0),
// on the split-K weight gradients and on dX l1 the hand-written kernels are as fast or
// faster, so only this class goes to the library (option gemm_lt, include/tt_hip.h).
// The caller passes the workspace (tt_gemm_ws_size floats, TT_GEMM_LT_WS bytes for a
// one-split call): the library allocates no device memory of its own for it.
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "tt_api.h"

namespace tt {
namespace {
struct LtKey {
  int dev, m, n, k;
  long lda, ldb, ldc;
  bool bias;
  bool operator<(const LtKey& o) const {
    return std::tie(dev, m, n, k, lda, ldb, ldc, bias) < std::tie(o.dev, o.m, o.n, o.k, o.lda, o.ldb, o.ldc, o.bias);
  }
};
struct LtPlan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo{};
};
std::mutex g_lt_mu;
std::map<int, hipblasLtHandle_t> g_handles;
std::map<LtKey, LtPlan> g_plans;

int lt_fail(const char* what, hipblasStatus_t s) {
  set_error("tt_gemm (hipBLASLt): %s failed (status %d)", what, (int)s);
  return TT_EINVAL;
}
#define TT_LT(expr)                                      \
  do {                                                   \
    hipblasStatus_t s_ = (expr);                         \
    if (s_ != HIPBLAS_STATUS_SUCCESS) return lt_fail(#expr, s_); \
  } while (0)

// Column-major view of the row-major problem: D^T [n x m] = W [n x k] * X^T [k x m], i.e.
// hipBLASLt A = the weights (k x n, ld ldb, transposed), B = the activations (k x m, ld lda),
// D = n x m with ld ldc; the bias runs along D's rows (length n = our columns).
int lt_plan(hipblasLtHandle_t h, const LtKey& key, LtPlan** out) {
  auto it = g_plans.find(key);
  if (it != g_plans.end()) {
    *out = &it->second;
    return 0;
  }
  LtPlan p;
  TT_LT(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const int32_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  TT_LT(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  TT_LT(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  if (key.bias) {
    const uint32_t epi = HIPBLASLT_EPILOGUE_BIAS;
    const int32_t bt = HIP_R_32F;
    TT_LT(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
    TT_LT(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  TT_LT(hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, key.k, key.n, key.ldb));
  TT_LT(hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, key.k, key.m, key.lda));
  TT_LT(hipblasLtMatrixLayoutCreate(&p.lc, HIP_R_16BF, key.n, key.m, key.ldc));
  hipblasLtMatmulPreference_t pref;
  TT_LT(hipblasLtMatmulPreferenceCreate(&pref));
  const uint64_t wsb = TT_GEMM_LT_WS;
  TT_LT(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
  hipblasLtMatmulHeuristicResult_t res[1];
  int nres = 0;
  const hipblasStatus_t hs = hipblasLtMatmulAlgoGetHeuristic(h, p.desc, p.la, p.lb, p.lc, p.lc, pref, 1, res, &nres);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (hs != HIPBLAS_STATUS_SUCCESS || nres < 1) return lt_fail("hipblasLtMatmulAlgoGetHeuristic", hs);
  if (res[0].workspaceSize > TT_GEMM_LT_WS) {
    set_error("tt_gemm (hipBLASLt): algorithm wants %zu workspace bytes", (size_t)res[0].workspaceSize);
    return TT_EINVAL;
  }
  p.algo = res[0].algo;
  *out = &g_plans.emplace(key, p).first->second;
  return 0;
}
}  // namespace

// C_b = A_b B_b^T (+ bias_b) for bf16 A [m][lda], B [n][ldb], C [m][ldc]; ws holds TT_GEMM_LT_WS bytes.
int gemm_lt(int m, int n, int k, const void* const* a, const void* const* b, void* const* c,
            const float* const* bias, int nbatch, long lda, long ldb, long ldc, void* ws, hipStream_t st) {
  int dev = 0;
  TT_CHECK_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_lt_mu);
  auto hi = g_handles.find(dev);
  if (hi == g_handles.end()) {
    hipblasLtHandle_t h;
    TT_LT(hipblasLtCreate(&h));
    hi = g_handles.emplace(dev, h).first;
  }
  const hipblasLtHandle_t h = hi->second;
  const float one = 1.f, zero = 0.f;
  for (int i = 0; i < nbatch; ++i) {
    LtPlan* p = nullptr;
    TT_PROPAGATE(lt_plan(h, LtKey{dev, m, n, k, lda, ldb, ldc, bias[i] != nullptr}, &p));
    if (bias[i]) {
      const void* bp = bias[i];
      TT_LT(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp)));
    }
    TT_LT(hipblasLtMatmul(h, p->desc, &one, b[i], p->la, a[i], p->lb, &zero, c[i], p->lc, c[i], p->lc, &p->algo, ws,
                          TT_GEMM_LT_WS, st));
  }
  return 0;
}
}  // namespace tt
