// Serving search (server/python-api/app.py:94-101): cosine scores of a few normalised
// queries against a resident, normalised document matrix, and the top-k per query,
// without materialising the score matrix for small query batches.
//
//   Q <= SCAN_QMAX: search_scan_kernel streams the document matrix once per 8 queries:
//     every lane scores whole document rows (16-byte loads; the query rows are uniform,
//     so they come through the scalar cache) and keeps a sorted per-lane top-k; each
//     wave merges its lanes and writes k candidates; topk_merge_kernel reduces the
//     candidates of all waves per query.
//   larger Q: cosine GEMM into a score block, then ttk::topk_split_kernel (many waves
//     per row, one column chunk each) and the same merge: the long rows of a large
//     document pool are scanned by many waves instead of one.
// Ordering everywhere: value descending, ties towards the lower document index.
#include <cfloat>
#include <climits>

#include "tt_api.h"
#include "tt_common.h"
#include "tt_topk.h"

namespace {

using ttk::SK_MAX;
using ttk::insert;
using ttk::wave_topk;
// queries per scan workgroup: QB sorted lists of KM entries live in registers
template <int KM> constexpr int scan_qb() { return KM <= 4 ? 8 : 2; }
constexpr int SCAN_QMAX = 64;     // above this the GEMM path re-reads the matrix less
constexpr int DOCS_PER_LANE = 4;  // 1024 documents per scan workgroup
constexpr int BLK_DOCS = 256 * DOCS_PER_LANE;

template <typename T, int KM, int SCAN_QB = scan_qb<KM>()>
__global__ __launch_bounds__(256) void search_scan_kernel(const float* __restrict__ qn, long Q,
                                                          const T* __restrict__ dn, long N, int h, int k,
                                                          float* __restrict__ cv, int* __restrict__ ci) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long q0 = (long)blockIdx.y * SCAN_QB;
  const int nq = (int)(Q - q0 < SCAN_QB ? Q - q0 : SCAN_QB);
  const long nslots = (long)gridDim.x * 4;
  const long slot = (long)blockIdx.x * 4 + wave;
  float lv[SCAN_QB][KM];
  int li[SCAN_QB][KM];
#pragma unroll
  for (int q = 0; q < SCAN_QB; ++q) ttk::init<KM>(lv[q], li[q]);
  const long dbase = (long)blockIdx.x * BLK_DOCS + wave * 64 * DOCS_PER_LANE + lane;
  for (int r = 0; r < DOCS_PER_LANE; ++r) {
    const long d = dbase + 64L * r;
    if (d < N) {
      const T* row = dn + d * h;
      float acc[SCAN_QB];
#pragma unroll
      for (int q = 0; q < SCAN_QB; ++q) acc[q] = 0.f;
      for (int c = 0; c < h; c += 8) {
        float x[8];
        ld8(row + c, x);
#pragma unroll
        for (int q = 0; q < SCAN_QB; ++q) {
          if (q < nq) {
            const float* qq = qn + (q0 + q) * h + c;  // uniform: scalar loads
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[q] = fmaf(x[e], qq[e], acc[q]);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < SCAN_QB; ++q)
        if (q < nq) insert<KM>(lv[q], li[q], k, acc[q], (int)d);
    }
  }
#pragma unroll
  for (int q = 0; q < SCAN_QB; ++q) {
    if (q < nq) {
      const long o = ((q0 + q) * nslots + slot) * k;
      wave_topk<KM>(lv[q], li[q], k, cv + o, ci + o);
    }
  }
}

struct SearchWs {
  long cv, ci, qd, S, total;
};

inline SearchWs search_ws(int dtype, long Q, long N, int h, int k) {
  auto al = [](long x) { return (x + 255) & ~255L; };
  SearchWs w{};
  long ncand, off = 0;
  if (Q <= SCAN_QMAX) {
    ncand = tt_ceil_div(N, BLK_DOCS) * 4 * k;
    w.qd = w.S = 0;
  } else {
    ncand = tt_ceil_div(N, ttk::split_chunk(Q, N)) * k;
  }
  w.cv = off; off = al(off + Q * ncand * 4);
  w.ci = off; off = al(off + Q * ncand * 4);
  if (Q > SCAN_QMAX) {
    const int esz = dtype == TT_DT_BF16 ? 2 : 4;
    w.qd = off; off = al(off + Q * h * esz);
    w.S = off;  off = al(off + Q * N * 4);
  }
  w.total = off;
  return w;
}

template <int KM>
int search_launch(int dtype, const float* qn, long Q, const void* dn, long N, int h, int k, int32_t* idx,
                  float* val, char* ws, hipStream_t st) {
  const SearchWs w = search_ws(dtype, Q, N, h, k);
  float* cv = reinterpret_cast<float*>(ws + w.cv);
  int* ci = reinterpret_cast<int*>(ws + w.ci);
  long ncand;
  if (Q <= SCAN_QMAX) {
    const long nblk = tt_ceil_div(N, BLK_DOCS);
    ncand = nblk * 4 * k;
    dim3 grid((unsigned)nblk, (unsigned)tt_ceil_div(Q, scan_qb<KM>()));
    if (dtype == TT_DT_BF16)
      hipLaunchKernelGGL((search_scan_kernel<bf16_t, KM>), grid, dim3(256), 0, st, qn, Q, (const bf16_t*)dn, N, h,
                         k, cv, ci);
    else
      hipLaunchKernelGGL((search_scan_kernel<float, KM>), grid, dim3(256), 0, st, qn, Q, (const float*)dn, N, h, k,
                         cv, ci);
    TT_CHECK_LAUNCH("search_scan_kernel");
  } else {
    void* qd = ws + w.qd;
    float* S = reinterpret_cast<float*>(ws + w.S);
    if (dtype == TT_DT_BF16) TT_PROPAGATE(tt_cast(TT_DT_BF16, qn, Q * h, qd, st));
    else TT_CHECK_HIP(hipMemcpyAsync(qd, qn, Q * h * 4, hipMemcpyDeviceToDevice, st));
    tt_gemm_batch g{};
    g.a[0] = qd; g.b[0] = dn; g.c[0] = S;
    TT_PROPAGATE(tt_gemm(dtype, TT_DT_F32, 0, 0, (int)Q, (int)N, h, &g, 1, h, h, N, 1.f, 0, 0, 0, 0, 0.f, 1, nullptr,
                         st));
    const long chunk = ttk::split_chunk(Q, N), nsp = tt_ceil_div(N, chunk);
    ncand = nsp * k;
    hipLaunchKernelGGL((ttk::topk_split_kernel<KM>), dim3((unsigned)tt_ceil_div(Q, 4), (unsigned)nsp), dim3(256), 0,
                       st, S, Q, N, chunk, -1L, k, cv, ci);
    TT_CHECK_LAUNCH("topk_split_kernel");
  }
  hipLaunchKernelGGL((ttk::topk_merge_kernel<KM>), dim3((unsigned)tt_ceil_div(Q, 4)), dim3(256), 0, st, cv, ci, Q, ncand,
                     k, idx, val);
  TT_CHECK_LAUNCH("topk_merge_kernel");
  return 0;
}

}  // namespace

extern "C" long tt_search_ws_size(int dtype, long Q, long N, int h, int k) {
  return search_ws(dtype, Q, N, h, k).total;
}

extern "C" int tt_search_topk(int dtype, const float* qn, long Q, const void* dn, long N, int h, int k, int32_t* idx,
                              float* val, void* ws, void* stream) {
  TT_CHECK_ARG(dtype == TT_DT_F32 || dtype == TT_DT_BF16, "tt_search_topk: bad dtype");
  TT_CHECK_ARG(k >= 1 && k <= SK_MAX && k <= N, "tt_search_topk: k=%d (N=%ld)", k, N);
  TT_CHECK_ARG(h > 0 && h % 8 == 0, "tt_search_topk: h=%d must be a multiple of 8", h);
  TT_CHECK_ARG(N <= INT_MAX && Q >= 0 && Q <= 65535L * 4, "tt_search_topk: N=%ld Q=%ld", N, Q);
  TT_CHECK_ARG(((uintptr_t)dn | (uintptr_t)qn) % 16 == 0, "tt_search_topk: operands must be 16-byte aligned");
  if (Q == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  char* ws_c = static_cast<char*>(ws);
  if (k <= 4) return search_launch<4>(dtype, qn, Q, dn, N, h, k, idx, val, ws_c, st);
  return search_launch<SK_MAX>(dtype, qn, Q, dn, N, h, k, idx, val, ws_c, st);
}
