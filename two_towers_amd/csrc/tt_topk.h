// Top-k building blocks shared by hard-negative mining (tt_loss.hip) and the serving
// search (tt_search.hip). Ordering: value descending, ties towards the lower index.
#pragma once
#include <cfloat>
#include <climits>

#include "tt_common.h"

namespace ttk {

constexpr int SK_MAX = 16;

TT_DEV bool better(float v, int i, float bv, int bi) { return v > bv || (v == bv && i < bi); }

// Insert (v, id) into the descending list (lv, li)[0..k).
template <int KM>
TT_DEV void insert(float (&lv)[KM], int (&li)[KM], int k, float v, int id) {
  if (!better(v, id, lv[k - 1], li[k - 1])) return;
  float cv = v;
  int ci = id;
#pragma unroll
  for (int q = 0; q < KM; ++q) {
    if (q < k && better(cv, ci, lv[q], li[q])) {
      const float tv = lv[q];
      const int ti = li[q];
      lv[q] = cv;
      li[q] = ci;
      cv = tv;
      ci = ti;
    }
  }
}

template <int KM>
TT_DEV void init(float (&lv)[KM], int (&li)[KM]) {
#pragma unroll
  for (int j = 0; j < KM; ++j) { lv[j] = -FLT_MAX; li[j] = INT_MAX; }
}

// k rounds of a wave arg-max over the lanes' sorted lists; lane 0 gets the result.
template <int KM>
TT_DEV void wave_topk(const float (&lv)[KM], const int (&li)[KM], int k, float* ov, int* oi) {
  const int lane = threadIdx.x & 63;
  int head = 0;
  for (int q = 0; q < k; ++q) {
    float hv = -FLT_MAX;
    int hi = INT_MAX;
#pragma unroll
    for (int p = 0; p < KM; ++p)
      if (p == head) { hv = lv[p]; hi = li[p]; }
    float bv = hv;
    int bi = hi;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float xv = __shfl_xor(bv, o, 64);
      const int xi = __shfl_xor(bi, o, 64);
      if (better(xv, xi, bv, bi)) { bv = xv; bi = xi; }
    }
    if (lane == 0) {
      ov[q] = bv;
      oi[q] = bi;
    }
    if (hi == bi && head < KM) ++head;
  }
}

// One wave per (row, column chunk) of a dense score block S [rows, cols]: k candidates
// per chunk into (cv, ci)[row][chunk][k]. Column label_off + row (if label_off >= 0)
// scores -1 (the positive of get_hard_negatives, enhanced_two_tower.py:130).
template <int KM>
__global__ __launch_bounds__(256) void topk_split_kernel(const float* __restrict__ S, long rows, long cols,
                                                         long chunk, long label_off, int k, float* __restrict__ cv,
                                                         int* __restrict__ ci) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  float lv[KM];
  int li[KM];
  init<KM>(lv, li);
  const long c0 = (long)blockIdx.y * chunk;
  const long c1 = c0 + chunk < cols ? c0 + chunk : cols;
  const long lab = label_off >= 0 ? label_off + row : -1;
  const float* sr = S + row * cols;
  for (long c = c0 + lane; c < c1; c += 64) insert<KM>(lv, li, k, c == lab ? -1.f : sr[c], (int)c);
  const long o = (row * gridDim.y + blockIdx.y) * k;
  wave_topk<KM>(lv, li, k, cv + o, ci + o);
}

// One wave per row: top-k of ncand candidates (cv, ci)[row][0..ncand).
template <int KM>
__global__ __launch_bounds__(256) void topk_merge_kernel(const float* __restrict__ cv, const int* __restrict__ ci,
                                                         long rows, long ncand, int k, int32_t* __restrict__ idx,
                                                         float* __restrict__ val) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  float lv[KM];
  int li[KM];
  init<KM>(lv, li);
  for (long c = lane; c < ncand; c += 64) insert<KM>(lv, li, k, cv[row * ncand + c], ci[row * ncand + c]);
  float ov[KM];
  int oi[KM];
  wave_topk<KM>(lv, li, k, ov, oi);
  if (lane == 0) {
    for (int q = 0; q < k; ++q) {
      idx[row * k + q] = oi[q];
      if (val) val[row * k + q] = ov[q];
    }
  }
}

// Column chunk per wave for a [rows, cols] block: enough waves to fill the chip.
inline long split_chunk(long rows, long cols) {
  long chunk = cols;
  while (chunk > 1024 && rows * ((cols + chunk - 1) / chunk) < 32768) chunk = (chunk + 1) / 2;
  return (chunk + 63) / 64 * 64;
}

}  // namespace ttk
