// hipBLASLt algorithm search for one bf16 GEMM shape (measurement tool; nothing in the
// product path uses it). Row-major C[m][n] = op(A) op(B) as tt_gemm's layouts:
//   a_kouter 0: A [m][k]; 1: A [k][m].   b_kouter 0: B [n][k]; 1: B [k][n].
// Prints the time of each of the heuristic's top algorithms (hipEvents, 5 iterations).
// Build: hipcc --offload-arch=gfx950 -O2 tools/lt_search.cpp -o tools/lt_search -lhipblaslt
// Run:   tools/lt_search m n k a_kouter b_kouter out_f32 nbatch
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    auto e_ = (x);                                                          \
    if ((int)e_ != 0) {                                                     \
      fprintf(stderr, "%s failed: %d (line %d)\n", #x, (int)e_, __LINE__); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 8) {
    fprintf(stderr, "usage: m n k a_kouter b_kouter out_f32 nbatch\n");
    return 2;
  }
  const long m = atol(argv[1]), n = atol(argv[2]), k = atol(argv[3]);
  const int ako = atoi(argv[4]), bko = atoi(argv[5]), of32 = atoi(argv[6]), nb = atoi(argv[7]);
  // column-major view: D^T [n x m] = op(B') op(A'), A' = our B, B' = our A
  // our B [n][k] (bko 0) = col-major k x n (ld k) -> op T gives n x k; [k][n] (bko 1) = col-major n x k -> N
  // our A [m][k] (ako 0) = col-major k x m (ld k) -> N gives k x m; [k][m] (ako 1) = col-major m x k -> T
  const hipblasOperation_t ta = bko ? HIPBLAS_OP_N : HIPBLAS_OP_T, tb = ako ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  const long ra = bko ? n : k, ca = bko ? k : n, rb = ako ? m : k, cb = ako ? k : m;
  void *A, *B, *D, *ws;
  const size_t wsb = 64u << 20;
  CK(hipMalloc(&A, (size_t)m * k * 2));
  CK(hipMalloc(&B, (size_t)n * k * 2));
  CK(hipMalloc(&D, (size_t)m * n * (of32 ? 4 : 2)));
  CK(hipMalloc(&ws, wsb));
  CK(hipMemset(A, 0x3c, (size_t)m * k * 2));
  CK(hipMemset(B, 0x3c, (size_t)n * k * 2));
  hipblasLtHandle_t h;
  CK(hipblasLtCreate(&h));
  hipblasLtMatmulDesc_t desc;
  CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  int32_t o1 = ta, o2 = tb;
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &o1, sizeof(o1)));
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &o2, sizeof(o2)));
  hipblasLtMatrixLayout_t la, lb, ld;
  CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, ra, ca, ra));
  CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, rb, cb, rb));
  CK(hipblasLtMatrixLayoutCreate(&ld, of32 ? HIP_R_32F : HIP_R_16BF, n, m, n));
  hipblasLtMatmulPreference_t pref;
  CK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t w = wsb;
  CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &w, sizeof(w)));
  std::vector<hipblasLtMatmulHeuristicResult_t> res(32);
  int nres = 0;
  CK(hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, ld, ld, pref, 32, res.data(), &nres));
  const float one = 1.f, zero = 0.f;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < nres; ++i) {
    auto run = [&]() {
      for (int b = 0; b < nb; ++b)
        if (hipblasLtMatmul(h, desc, &one, B, la, A, lb, &zero, D, ld, D, ld, &res[i].algo, ws, wsb, 0) != 0) return false;
      return true;
    };
    if (!run()) {
      printf("algo %2d failed\n", i);
      continue;
    }
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int it = 0; it < 5; ++it) run();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 5;
    printf("algo %2d ws %8zu  %.3f ms  %.1f TFLOP/s\n", i, (size_t)res[i].workspaceSize, ms,
           2.0 * m * n * k * nb / (ms * 1e-3) / 1e12);
    fflush(stdout);
  }
  return 0;
}
