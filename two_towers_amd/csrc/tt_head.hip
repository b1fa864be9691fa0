// Projection heads built on tt_gemm plus fused LayerNorm+ReLU(+Dropout) kernels:
//   enhanced: Linear(4h->2h) -> LayerNorm(2h) -> ReLU -> Linear(2h->h)
//   margin:   Linear(2H->H) -> LayerNorm(H) -> ReLU -> Dropout(p), one set of weights
//             shared by both towers (query and doc rows stacked into one batch).
#include <algorithm>
#include <climits>

#include "tt_api.h"
#include "tt_common.h"

namespace {

constexpr int LN_MAXC = 16;  // columns per lane -> up to 1024 columns (h <= 512)

// One wave per row. u = relu((x - mean) * rstd * g + b)
// With drop_thresh != 0 the ReLU output is multiplied by the counter-based dropout
// mask keep(seed, row, col) / (1 - p) (tt_dropout_scale, recomputed by the backward).
template <typename T, typename TO>
__global__ __launch_bounds__(256) void ln_relu_fwd_kernel(const T* __restrict__ x, long rows, int C,
                                                          const float* __restrict__ gam,
                                                          const float* __restrict__ bet, float eps,
                                                          TO* __restrict__ u, float* __restrict__ mean,
                                                          float* __restrict__ rstd, uint32_t drop_seed,
                                                          uint32_t drop_thresh, float inv_keep) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const T* xr = x + row * C;
  float v[LN_MAXC];
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < LN_MAXC; ++q) {
    const int c = lane + 64 * q;
    v[q] = c < C ? Elt<T>::ld(xr + c) : 0.f;
    s += v[q];
  }
  const float mu = wave_sum(s) / C;
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < LN_MAXC; ++q) {
    const int c = lane + 64 * q;
    const float d = c < C ? v[q] - mu : 0.f;
    ss += d * d;
  }
  const float rs = rsqrtf(wave_sum(ss) / C + eps);
#pragma unroll
  for (int q = 0; q < LN_MAXC; ++q) {
    const int c = lane + 64 * q;
    if (c < C) {
      float o = fmaxf((v[q] - mu) * rs * gam[c] + bet[c], 0.f);
      if (drop_thresh) o *= tt_dropout_scale(drop_seed, (uint32_t)row, (uint32_t)c, drop_thresh, inv_keep);
      Elt<TO>::st(u + row * C + c, o);
    }
  }
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

// One wave per row; each block covers rows_per_block rows and writes one partial
// row [NP][C] of (dgamma, dbeta, dx-colsum [, column sum of dout2]) to part: the
// partial rows are then summed in a fixed order (tt_colsum), so every bias and affine
// gradient is bit-for-bit reproducible (no float atomics). dout2 [rows, C2] (NP = 4):
// the output gradient of the head's last Linear, whose column sum is that layer's bias
// gradient, read in the same pass.
template <typename T, int NP>
__global__ __launch_bounds__(256) void ln_relu_bwd_kernel(const float* __restrict__ du, const T* __restrict__ x,
                                                          const float* __restrict__ gam,
                                                          const float* __restrict__ bet,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ rstd, long rows, int C,
                                                          int rows_per_block, T* __restrict__ dx,
                                                          float* __restrict__ part, uint32_t drop_seed,
                                                          uint32_t drop_thresh, float inv_keep,
                                                          const float* __restrict__ dout2, int C2) {
  __shared__ float red[4][NP][LN_MAXC * 64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float pg[LN_MAXC], pb[LN_MAXC], pd[LN_MAXC], p2[LN_MAXC];
#pragma unroll
  for (int q = 0; q < LN_MAXC; ++q) pg[q] = pb[q] = pd[q] = p2[q] = 0.f;
  const long r0 = (long)blockIdx.x * rows_per_block;
  for (long row = r0 + wave; row < std::min(rows, r0 + rows_per_block); row += 4) {
    if constexpr (NP == 4) {
#pragma unroll
      for (int q = 0; q < LN_MAXC; ++q) {
        const int c = lane + 64 * q;
        if (c < C2) p2[q] += dout2[row * C2 + c];
      }
    }
    const float mu = mean[row], rs = rstd[row];
    float xh[LN_MAXC], da[LN_MAXC];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < LN_MAXC; ++q) {
      const int c = lane + 64 * q;
      xh[q] = 0.f;
      da[q] = 0.f;
      if (c < C) {
        xh[q] = (Elt<T>::ld(x + row * C + c) - mu) * rs;
        const float a = xh[q] * gam[c] + bet[c];
        da[q] = a > 0.f ? du[row * C + c] : 0.f;
        if (drop_thresh) da[q] *= tt_dropout_scale(drop_seed, (uint32_t)row, (uint32_t)c, drop_thresh, inv_keep);
        const float dxh = da[q] * gam[c];
        s1 += dxh;
        s2 += dxh * xh[q];
        pg[q] += da[q] * xh[q];
        pb[q] += da[q];
      }
    }
    s1 = wave_sum(s1) / C;
    s2 = wave_sum(s2) / C;
#pragma unroll
    for (int q = 0; q < LN_MAXC; ++q) {
      const int c = lane + 64 * q;
      if (c < C) {
        const float d = rs * (da[q] * gam[c] - s1 - xh[q] * s2);
        Elt<T>::st(dx + row * C + c, d);
        pd[q] += d;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < LN_MAXC; ++q) {
    red[wave][0][lane + 64 * q] = pg[q];
    red[wave][1][lane + 64 * q] = pb[q];
    red[wave][2][lane + 64 * q] = pd[q];
    if constexpr (NP == 4) red[wave][NP - 1][lane + 64 * q] = p2[q];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < NP * C; e += 256) {
    const int k = e / C, c = e % C;
    part[(long)blockIdx.x * NP * C + e] = red[0][k][c] + red[1][k][c] + red[2][k][c] + red[3][k][c];
  }
}

constexpr int LN_ROWS_PER_BLOCK = 16;  // 512 blocks at B 8192: fills the chip

inline long head_ws_layout(int dtype, int B, int h, long* o_dout, long* o_du, long* o_dp1, long* o_part,
                           long* o_sk) {
  const int esz = dtype == TT_DT_BF16 ? 2 : 4;
  auto al = [](long x) { return (x + 255) & ~255L; };
  long off = 0;
  *o_dout = off; off = al(off + (long)B * h * esz);
  *o_du = off;   off = al(off + (long)B * 2 * h * 4);
  *o_dp1 = off;  off = al(off + (long)B * 2 * h * esz);
  const long nblk = tt_ceil_div(B, LN_ROWS_PER_BLOCK);
  *o_part = off; off = al(off + nblk * 4L * 2 * h * 4);
  const int s2 = tt_gemm_pick_splits(h, 2 * h, B, 1);
  const int s1 = tt_gemm_pick_splits(2 * h, 4 * h, B, 1);
  const long sk = std::max(tt_gemm_ws_size(h, 2 * h, 1, s2), tt_gemm_ws_size(2 * h, 4 * h, 1, s1));
  *o_sk = off; off = al(off + sk * 4);
  return off;
}

}  // namespace

extern "C" long tt_proj_head_bwd_ws_size(int dtype, int B, int h) {
  long a, b, c, d, e;
  return head_ws_layout(dtype, B, h, &a, &b, &c, &d, &e);
}

extern "C" int tt_proj_head_fwd(int dtype, const tt_head_fwd_io* io, int ntower, int B, int h, float ln_eps,
                                void* stream) {
  TT_CHECK_ARG(ntower >= 1 && ntower <= 4, "tt_proj_head_fwd: ntower");
  TT_CHECK_ARG(2 * h <= 64 * LN_MAXC, "tt_proj_head_fwd: h=%d too large", h);
  hipStream_t st = (hipStream_t)stream;
  tt_gemm_batch g1{}, g2{};
  for (int i = 0; i < ntower; ++i) {
    g1.a[i] = io[i].x; g1.b[i] = io[i].w1; g1.c[i] = io[i].p1; g1.bias[i] = io[i].b1;
    g2.a[i] = io[i].u; g2.b[i] = io[i].w2; g2.c[i] = io[i].out; g2.bias[i] = io[i].b2;
  }
  // p1 = x w1^T + b1   [B, 2h]
  TT_PROPAGATE(tt_gemm(dtype, dtype, 0, 0, B, 2 * h, 4 * h, &g1, ntower, 4 * h, 4 * h, 2 * h, 1.f, 0, 0, 0, 0,
                       0.f, 1, nullptr, stream));
  for (int i = 0; i < ntower; ++i) {
    dim3 grid(tt_ceil_div(B, 4));
    if (dtype == TT_DT_BF16)
      hipLaunchKernelGGL((ln_relu_fwd_kernel<bf16_t, bf16_t>), grid, dim3(256), 0, st, (const bf16_t*)io[i].p1,
                         (long)B, 2 * h, io[i].ln_g, io[i].ln_b, ln_eps, (bf16_t*)io[i].u, io[i].mean, io[i].rstd,
                         0u, 0u, 1.f);
    else
      hipLaunchKernelGGL((ln_relu_fwd_kernel<float, float>), grid, dim3(256), 0, st, (const float*)io[i].p1,
                         (long)B, 2 * h, io[i].ln_g, io[i].ln_b, ln_eps, (float*)io[i].u, io[i].mean, io[i].rstd,
                         0u, 0u, 1.f);
    TT_CHECK_LAUNCH("ln_relu_fwd_kernel");
  }
  // out = u w2^T + b2  [B, h] fp32
  TT_PROPAGATE(tt_gemm(dtype, TT_DT_F32, 0, 0, B, h, 2 * h, &g2, ntower, 2 * h, 2 * h, h, 1.f, 0, 0, 0, 0, 0.f, 1,
                       nullptr, stream));
  return 0;
}

extern "C" int tt_proj_head_bwd(int dtype, const tt_head_bwd_io* io, int ntower, int B, int h, float ln_eps,
                                void* stream) {
  (void)ln_eps;
  TT_CHECK_ARG(ntower >= 1 && ntower <= 4, "tt_proj_head_bwd: ntower");
  TT_CHECK_ARG(2 * h <= 64 * LN_MAXC, "tt_proj_head_bwd: h=%d too large", h);
  hipStream_t st = (hipStream_t)stream;
  long o_dout, o_du, o_dp1, o_part, o_sk;
  head_ws_layout(dtype, B, h, &o_dout, &o_du, &o_dp1, &o_part, &o_sk);
  const int C = 2 * h;
  const long nblk = tt_ceil_div(B, LN_ROWS_PER_BLOCK);
  for (int i = 0; i < ntower; ++i) {
    const tt_head_bwd_io& q = io[i];
    char* ws = static_cast<char*>(q.ws);
    void* dout_t = ws + o_dout;
    float* du = reinterpret_cast<float*>(ws + o_du);
    void* dp1 = ws + o_dp1;
    float* part = reinterpret_cast<float*>(ws + o_part);
    float* sk = reinterpret_cast<float*>(ws + o_sk);
    TT_PROPAGATE(tt_cast(dtype, q.dout, (long)B * h, dout_t, stream));
    // dW2 = dout^T u   [h, 2h]
    {
      tt_gemm_batch g{};
      g.a[0] = dout_t; g.b[0] = q.u; g.c[0] = q.dw2;
      const int sp = tt_gemm_pick_splits(h, C, B, 1);
      TT_PROPAGATE(tt_gemm(dtype, TT_DT_F32, 1, 1, h, C, B, &g, 1, h, C, C, 1.f, 0, 0, 0, 0, 0.f, sp, sk, stream));
    }
    // du = dout w2   [B, 2h]
    {
      tt_gemm_batch g{};
      g.a[0] = dout_t; g.b[0] = q.w2; g.c[0] = du;
      TT_PROPAGATE(tt_gemm(dtype, TT_DT_F32, 0, 1, B, C, h, &g, 1, h, C, C, 1.f, 0, 0, 0, 0, 0.f, 1, nullptr, stream));
    }
    // LayerNorm + ReLU backward -> dp1, partial (dgamma, dbeta, db1, db2)
    if (dtype == TT_DT_BF16)
      hipLaunchKernelGGL((ln_relu_bwd_kernel<bf16_t, 4>), dim3(nblk), dim3(256), 0, st, du, (const bf16_t*)q.p1,
                         q.ln_g, q.ln_b, q.mean, q.rstd, (long)B, C, LN_ROWS_PER_BLOCK, (bf16_t*)dp1, part, 0u, 0u,
                         1.f, q.dout, h);
    else
      hipLaunchKernelGGL((ln_relu_bwd_kernel<float, 4>), dim3(nblk), dim3(256), 0, st, du, (const float*)q.p1,
                         q.ln_g, q.ln_b, q.mean, q.rstd, (long)B, C, LN_ROWS_PER_BLOCK, (float*)dp1, part, 0u, 0u,
                         1.f, q.dout, h);
    TT_CHECK_LAUNCH("ln_relu_bwd_kernel");
    TT_PROPAGATE(tt_colsum(part, nblk, C, 4L * C, q.dg, 0, stream));
    TT_PROPAGATE(tt_colsum(part + C, nblk, C, 4L * C, q.dbeta, 0, stream));
    TT_PROPAGATE(tt_colsum(part + 2 * C, nblk, C, 4L * C, q.db1, 0, stream));
    TT_PROPAGATE(tt_colsum(part + 3 * C, nblk, h, 4L * C, q.db2, 0, stream));
    // dW1 = dp1^T x   [2h, 4h]
    {
      tt_gemm_batch g{};
      g.a[0] = dp1; g.b[0] = q.x; g.c[0] = q.dw1;
      const int sp = tt_gemm_pick_splits(C, 2 * C, B, 1);
      TT_PROPAGATE(tt_gemm(dtype, TT_DT_F32, 1, 1, C, 2 * C, B, &g, 1, C, 2 * C, 2 * C, 1.f, 0, 0, 0, 0, 0.f, sp, sk,
                           stream));
    }
    // dx = dp1 w1   [B, 4h]
    {
      tt_gemm_batch g{};
      g.a[0] = dp1; g.b[0] = q.w1; g.c[0] = q.dx;
      TT_PROPAGATE(tt_gemm(dtype, TT_DT_F32, 0, 1, B, 2 * C, C, &g, 1, C, 2 * C, 2 * C, 1.f, 0, 0, 0, 0, 0.f, 1,
                           nullptr, stream));
    }
  }
  return 0;
}

// ------------------------------------------------------------------ margin head
namespace {

inline long head1_ws_layout(int dtype, long rows, int C, long* o_dp1, long* o_part, long* o_sk) {
  const int esz = dtype == TT_DT_BF16 ? 2 : 4;
  auto al = [](long x) { return (x + 255) & ~255L; };
  long off = 0;
  *o_dp1 = off;  off = al(off + rows * C * esz);
  const long nblk = tt_ceil_div(rows, LN_ROWS_PER_BLOCK);
  *o_part = off; off = al(off + nblk * 3L * C * 4);
  const int sp = tt_gemm_pick_splits(C, 2 * C, (int)rows, 1);
  *o_sk = off;   off = al(off + tt_gemm_ws_size(C, 2 * C, 1, sp) * 4);
  return off;
}

inline void drop_params(float p, uint32_t* thresh, float* inv_keep) {
  // keep iff (hash >> 8) >= thresh, i.e. P(drop) = thresh / 2^24 (tt_dropout_scale)
  *thresh = p > 0.f ? (uint32_t)(p * 16777216.0f + 0.5f) : 0u;
  *inv_keep = p > 0.f ? 1.f / (1.f - p) : 1.f;
}

}  // namespace

extern "C" long tt_proj_head1_bwd_ws_size(int dtype, long rows, int C) {
  long a, b, c;
  return head1_ws_layout(dtype, rows, C, &a, &b, &c);
}

extern "C" int tt_proj_head1_fwd(int dtype, const tt_head1_fwd_io* io, long rows, int C, float ln_eps,
                                 float drop_p, uint32_t drop_seed, void* stream) {
  TT_CHECK_ARG(C >= 1 && C <= 64 * LN_MAXC, "tt_proj_head1_fwd: C=%d out of range", C);
  TT_CHECK_ARG(rows >= 1 && rows <= INT_MAX, "tt_proj_head1_fwd: rows");
  TT_CHECK_ARG(drop_p >= 0.f && drop_p < 1.f, "tt_proj_head1_fwd: drop_p");
  hipStream_t st = (hipStream_t)stream;
  // p1 = x w1^T + b1   [rows, C]
  tt_gemm_batch g{};
  g.a[0] = io->x; g.b[0] = io->w1; g.c[0] = io->p1; g.bias[0] = io->b1;
  TT_PROPAGATE(tt_gemm(dtype, dtype, 0, 0, (int)rows, C, 2 * C, &g, 1, 2 * C, 2 * C, C, 1.f, 0, 0, 0, 0, 0.f, 1,
                       nullptr, stream));
  uint32_t thresh;
  float inv_keep;
  drop_params(drop_p, &thresh, &inv_keep);
  dim3 grid(tt_ceil_div(rows, 4));
  if (dtype == TT_DT_BF16)
    hipLaunchKernelGGL((ln_relu_fwd_kernel<bf16_t, float>), grid, dim3(256), 0, st, (const bf16_t*)io->p1, rows, C,
                       io->ln_g, io->ln_b, ln_eps, io->out, io->mean, io->rstd, drop_seed, thresh, inv_keep);
  else
    hipLaunchKernelGGL((ln_relu_fwd_kernel<float, float>), grid, dim3(256), 0, st, (const float*)io->p1, rows, C,
                       io->ln_g, io->ln_b, ln_eps, io->out, io->mean, io->rstd, drop_seed, thresh, inv_keep);
  TT_CHECK_LAUNCH("ln_relu_fwd_kernel");
  return 0;
}

extern "C" int tt_proj_head1_bwd(int dtype, const tt_head1_bwd_io* io, long rows, int C, float drop_p,
                                 uint32_t drop_seed, void* stream) {
  TT_CHECK_ARG(C >= 1 && C <= 64 * LN_MAXC, "tt_proj_head1_bwd: C=%d out of range", C);
  TT_CHECK_ARG(rows >= 1 && rows <= INT_MAX, "tt_proj_head1_bwd: rows");
  TT_CHECK_ARG(drop_p >= 0.f && drop_p < 1.f, "tt_proj_head1_bwd: drop_p");
  hipStream_t st = (hipStream_t)stream;
  long o_dp1, o_part, o_sk;
  head1_ws_layout(dtype, rows, C, &o_dp1, &o_part, &o_sk);
  char* ws = static_cast<char*>(io->ws);
  void* dp1 = ws + o_dp1;
  float* part = reinterpret_cast<float*>(ws + o_part);
  float* sk = reinterpret_cast<float*>(ws + o_sk);
  uint32_t thresh;
  float inv_keep;
  drop_params(drop_p, &thresh, &inv_keep);
  const long nblk = tt_ceil_div(rows, LN_ROWS_PER_BLOCK);
  // Dropout + ReLU + LayerNorm backward -> dp1, partial (dgamma, dbeta, db1)
  if (dtype == TT_DT_BF16)
    hipLaunchKernelGGL((ln_relu_bwd_kernel<bf16_t, 3>), dim3(nblk), dim3(256), 0, st, io->dout,
                       (const bf16_t*)io->p1, io->ln_g, io->ln_b, io->mean, io->rstd, rows, C, LN_ROWS_PER_BLOCK,
                       (bf16_t*)dp1, part, drop_seed, thresh, inv_keep, (const float*)nullptr, 0);
  else
    hipLaunchKernelGGL((ln_relu_bwd_kernel<float, 3>), dim3(nblk), dim3(256), 0, st, io->dout,
                       (const float*)io->p1, io->ln_g, io->ln_b, io->mean, io->rstd, rows, C, LN_ROWS_PER_BLOCK,
                       (float*)dp1, part, drop_seed, thresh, inv_keep, (const float*)nullptr, 0);
  TT_CHECK_LAUNCH("ln_relu_bwd_kernel");
  TT_PROPAGATE(tt_colsum(part, nblk, C, 3L * C, io->dg, 0, stream));
  TT_PROPAGATE(tt_colsum(part + C, nblk, C, 3L * C, io->dbeta, 0, stream));
  TT_PROPAGATE(tt_colsum(part + 2 * C, nblk, C, 3L * C, io->db1, 0, stream));
  // dW1 = dp1^T x   [C, 2C]: the sum over all rows is the sum over both towers
  {
    tt_gemm_batch g{};
    g.a[0] = dp1; g.b[0] = io->x; g.c[0] = io->dw1;
    const int sp = tt_gemm_pick_splits(C, 2 * C, (int)rows, 1);
    TT_PROPAGATE(tt_gemm(dtype, TT_DT_F32, 1, 1, C, 2 * C, (int)rows, &g, 1, C, 2 * C, 2 * C, 1.f, 0, 0, 0, 0, 0.f,
                         sp, sk, stream));
  }
  // dx = dp1 w1   [rows, 2C]
  {
    tt_gemm_batch g{};
    g.a[0] = dp1; g.b[0] = io->w1; g.c[0] = io->dx;
    TT_PROPAGATE(tt_gemm(dtype, TT_DT_F32, 0, 1, (int)rows, 2 * C, C, &g, 1, C, 2 * C, 2 * C, 1.f, 0, 0, 0, 0, 0.f, 1,
                         nullptr, stream));
  }
  return 0;
}
