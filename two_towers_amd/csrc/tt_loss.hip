// Contrastive losses on the tower outputs: L2 normalisation, the fused in-batch
// softmax cross-entropy (InfoNCE) over the B x N score matrix, hard-negative top-k
// mining and the hinge (margin) loss over mined negatives.
#include <algorithm>
#include <float.h>

#include "tt_api.h"
#include "tt_gemm_core.h"
#include "tt_topk.h"

namespace {

constexpr int MAXC = 16;  // features per lane (h <= 1024)

// ---------------------------------------------------------------- L2 normalise
template <typename T>
__global__ __launch_bounds__(256) void l2norm_fwd_kernel(const float* __restrict__ x, long rows, int C, float eps,
                                                         T* __restrict__ y, float* __restrict__ y32,
                                                         float* __restrict__ norm) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  float v[MAXC];
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < MAXC; ++q) {
    const int c = lane + 64 * q;
    v[q] = c < C ? x[row * C + c] : 0.f;
    ss += v[q] * v[q];
  }
  const float nrm = sqrtf(wave_sum(ss));
  const float inv = 1.f / fmaxf(nrm, eps);
#pragma unroll
  for (int q = 0; q < MAXC; ++q) {
    const int c = lane + 64 * q;
    if (c < C) {
      Elt<T>::st(y + row * C + c, v[q] * inv);
      if (y32) y32[row * C + c] = v[q] * inv;
    }
  }
  if (lane == 0) norm[row] = nrm;
}

__global__ __launch_bounds__(256) void l2norm_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                         const float* __restrict__ norm, long rows, int C, float eps,
                                                         float* __restrict__ dx, int accumulate) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float nrm = norm[row];
  float g[MAXC], yy[MAXC];
  float dot = 0.f;
#pragma unroll
  for (int q = 0; q < MAXC; ++q) {
    const int c = lane + 64 * q;
    g[q] = c < C ? dy[row * C + c] : 0.f;
    yy[q] = c < C ? y[row * C + c] : 0.f;
    dot += g[q] * yy[q];
  }
  dot = wave_sum(dot);
  const bool clamped = !(nrm > eps);
  const float inv = 1.f / fmaxf(nrm, eps);
#pragma unroll
  for (int q = 0; q < MAXC; ++q) {
    const int c = lane + 64 * q;
    if (c < C) {
      const float d = clamped ? g[q] * inv : (g[q] - yy[q] * dot) * inv;
      float* p = dx + row * C + c;
      *p = accumulate ? *p + d : d;
    }
  }
}

// ----------------------------------------------------------- fused InfoNCE fwd
// Grid (col_splits, row_blocks). Each workgroup sweeps its share of 128-column
// dn tiles for 128 q rows, keeping a per-lane running (max, sum-exp) per row, and
// writes one (max, sumexp) partial per row and split. S is never stored.
template <typename T>
__global__ __launch_bounds__(256) void infonce_fwd_kernel(const T* __restrict__ qn, long bq, const T* __restrict__ dn,
                                                          long nd, int h, float inv_tau, float offdiag,
                                                          long label_off, int ct_per_split, float* __restrict__ pm,
                                                          float* __restrict__ pl, float* __restrict__ diag) {
  using ML = ttg::MainLoop<T, false, false, 128, 128>;
  __shared__ __attribute__((aligned(16))) char lds[ML::LDS_BYTES];
  __shared__ float red_m[2][128], red_l[2][128];
  const int m0 = blockIdx.y * 128;
  const long nct = (nd + 127) / 128;
  const long ct0 = (long)blockIdx.x * ct_per_split;
  const long ct1 = std::min(nct, ct0 + ct_per_split);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int nk = (h * (int)sizeof(T) + ttg::KTB - 1) / ttg::KTB;
  float rm[4][4], rl[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) { rm[i][r] = -FLT_MAX; rl[i][r] = 0.f; }

  for (long ct = ct0; ct < ct1; ++ct) {
    const int n0 = (int)(ct * 128);
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    ML::run(ttg::KCPlain<T>{qn, h, m0, (int)bq}, ttg::KCPlain<T>{dn, h, n0, (int)nd}, h, 0, nk, lds, acc);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long row = m0 + wm + 16 * i + 4 * (lane >> 4) + r;
        float sv[4];
        float tmax = -FLT_MAX;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const long col = n0 + wn + 16 * j + (lane & 15);
          float s = acc[i][j][r] * inv_tau;
          const bool lab = (col == label_off + row);
          if (!lab) s -= offdiag;
          if (lab && row < bq) diag[row] = s;
          if (col >= nd) s = -FLT_MAX;
          sv[j] = s;
          tmax = fmaxf(tmax, s);
        }
        const float nm = fmaxf(rm[i][r], tmax);
        float l = rl[i][r] * __expf(rm[i][r] - nm);
#pragma unroll
        for (int j = 0; j < 4; ++j) l += (sv[j] > -FLT_MAX) ? __expf(sv[j] - nm) : 0.f;
        rm[i][r] = nm;
        rl[i][r] = l;
      }
  }
  // merge the 16 lanes sharing each row, then the two waves sharing it
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float M = max16(rm[i][r]);
      const float L = sum16(rl[i][r] * __expf(rm[i][r] - M));
      if ((lane & 15) == 0) {
        const int rr = wm + 16 * i + 4 * (lane >> 4) + r;
        red_m[wave & 1][rr] = M;
        red_l[wave & 1][rr] = L;
      }
    }
  __syncthreads();
  if (threadIdx.x < 128) {
    const long row = m0 + threadIdx.x;
    if (row < bq) {
      const float a = red_m[0][threadIdx.x], b = red_m[1][threadIdx.x];
      const float M = fmaxf(a, b);
      const float L = red_l[0][threadIdx.x] * __expf(a - M) + red_l[1][threadIdx.x] * __expf(b - M);
      pm[(long)blockIdx.x * bq + row] = M;
      pl[(long)blockIdx.x * bq + row] = L;
    }
  }
}

__global__ __launch_bounds__(256) void infonce_finalize_kernel(const float* __restrict__ pm,
                                                               const float* __restrict__ pl, int splits, long bq,
                                                               const float* __restrict__ diag, float* __restrict__ lse,
                                                               float* __restrict__ row_loss) {
  const long row = (long)blockIdx.x * 256 + threadIdx.x;
  if (row >= bq) return;
  float M = -FLT_MAX;
  for (int s = 0; s < splits; ++s) M = fmaxf(M, pm[(long)s * bq + row]);
  float L = 0.f;
  for (int s = 0; s < splits; ++s) L += pl[(long)s * bq + row] * __expf(pm[(long)s * bq + row] - M);
  const float v = M + __logf(L);
  lse[row] = v;
  row_loss[row] = v - diag[row];
}

// dS[i][j] = g * (softmax_ij - [j == label_i]) in dtype, full tiles; g = *gscale (the
// upstream gradient, read on the device: no host sync) or 1 when gscale is null.
template <typename T>
__global__ __launch_bounds__(256) void infonce_dscore_kernel(const T* __restrict__ qn, long bq,
                                                             const T* __restrict__ dn, long nd, int h, float inv_tau,
                                                             float offdiag, long label_off,
                                                             const float* __restrict__ lse,
                                                             const float* __restrict__ gscale, long ldds,
                                                             T* __restrict__ ds) {
  const float gs = gscale ? *gscale : 1.f;
  using ML = ttg::MainLoop<T, false, false, 128, 128>;
  __shared__ __attribute__((aligned(16))) char lds[ML::LDS_BYTES];
  const int m0 = blockIdx.y * 128, n0 = blockIdx.x * 128;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (h * (int)sizeof(T) + ttg::KTB - 1) / ttg::KTB;
  ML::run(ttg::KCPlain<T>{qn, h, m0, (int)bq}, ttg::KCPlain<T>{dn, h, n0, (int)nd}, h, 0, nk, lds, acc);
  ML::epilogue(acc, [&](int r, int c, float v) {
    const long row = m0 + r, col = n0 + c;
    if (row >= bq || col >= nd) return;
    const bool lab = (col == label_off + row);
    float s = v * inv_tau;
    if (!lab) s -= offdiag;
    const float p = __expf(s - lse[row]);
    Elt<T>::st(ds + row * ldds + col, gs * (p - (lab ? 1.f : 0.f)));
  });
}

// ---------------------------------------------- fused InfoNCE backward, bf16, no dS
// dS[i][j] = g * (softmax_ij - [j == label_i]) is recomputed tile by tile and consumed
// in LDS; nothing of size B x N is written. Two roles of one kernel:
//   OWNQ : a workgroup owns 128 query rows i and sweeps document tiles j:
//          dq_i  = inv_tau * sum_j dS_ij d_j
//   !OWNQ: a workgroup owns 128 document rows j and sweeps query tiles i:
//          dd_j  = inv_tau * sum_i dS_ij q_i
// Per 64-row tile of the swept operand X: S = O . X^T (MFMA over K = H, own rows and the
// tile staged in LDS as K-contig images), dS -> LDS as the bf16 A operand, then
// dO += dS . X with X's K-contig image read as the K-outer B operand by transposing
// reads (ds_read_b64_tr_b16), so each X tile is loaded once for both products. X tiles are
// LDS-DMA'd one tile ahead. A sweep may be split over workgroups (fp32 partial slabs,
// summed by infonce_slab_sum_kernel).
//   LDS (H = 256): own rows 64 KiB + two X tiles 2 x 32 KiB + dS 16 KiB = 144 KiB.
// 8 waves as 4 (own rows) x 2: product 1 wave tile 32 x 32, product 2 wave tile 32 x H/2.
template <int H>
struct FlashCfg {
  static constexpr int NKT = H / 64;            // K-tiles of 64 features
  static constexpr int OWN = 128 * 128 * NKT;   // own-row images (128 rows x 128 B each)
  static constexpr int XT = 64 * 128 * NKT;     // one X tile
  static constexpr int DS = 128 * 128;          // dS: 128 own rows x 64 tile rows (one K-tile)
  static constexpr int LDS = OWN + 2 * XT + DS;
  static constexpr int NO = H / 32;             // 16-column MFMA tiles per wave, product 2
};

// MFMA B fragment of X^T . (k = tile row, n = feature) from the K-contig X image of feature
// K-tile `img` (rows of 128 B, 16-B chunk c of row k at c ^ ((k >> 1) & 7)): the reads of
// frag<bf16, true>, addressed into this layout.
TT_DEV uint4 frag_kc_tr(const char* img, int n0, int ks) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i4 = lane & 15, q = i4 >> 2, p = i4 & 3;
  const int k0 = ks * 32 + 8 * g + q, k1 = k0 + 4;
  const int n = n0 + 4 * p;
  const int o0 = k0 * 128 + ((((n >> 3) & 7) ^ ((k0 >> 1) & 7)) << 4) + ((n >> 2) & 1) * 8;
  const int o1 = k1 * 128 + ((((n >> 3) & 7) ^ ((k1 >> 1) & 7)) << 4) + ((n >> 2) & 1) * 8;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + o0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + o1));
  uint4 v;
  v.x = (uint32_t)(uint16_t)lo[0] | ((uint32_t)(uint16_t)lo[1] << 16);
  v.y = (uint32_t)(uint16_t)lo[2] | ((uint32_t)(uint16_t)lo[3] << 16);
  v.z = (uint32_t)(uint16_t)hi[0] | ((uint32_t)(uint16_t)hi[1] << 16);
  v.w = (uint32_t)(uint16_t)hi[2] | ((uint32_t)(uint16_t)hi[3] << 16);
  return v;
}

// rows [r0, r0 + nrows_img) of a row-major bf16 [rows][H] matrix -> K-contig images (one
// per 64-feature K-tile, 128 B per row), by LDS-DMA; rows past `rows` read the zero page
template <int H>
TT_DEV void flash_stage(const bf16_t* src, long rows, long r0, int nrows_img, uint32_t img) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int pieces = nrows_img * 128 / 1024;  // 1 KiB pieces per K-tile image
  for (int kt = 0; kt < H / 64; ++kt)
    for (int pc = wave; pc < pieces; pc += 8) {
      const int p = pc * 64 + lane, row = p >> 3, c = (p & 7) ^ ((row >> 1) & 7);
      const long gr = r0 + row;
      const void* s = gr < rows ? static_cast<const void*>(src + gr * H + kt * 64 + c * 8)
                                : static_cast<const void*>(ttg::g_tt_zero_page);
      ttg::dma16(s, img + (uint32_t)(kt * nrows_img * 128 + pc * 1024));
    }
}

template <int H, bool OWNQ>
__global__ __launch_bounds__(512) void infonce_bwd_flash_kernel(const bf16_t* __restrict__ qn, long bq,
                                                                const bf16_t* __restrict__ dn, long nd, float inv_tau,
                                                                float offdiag, long label_off,
                                                                const float* __restrict__ lse,
                                                                const float* __restrict__ gscale, int tiles_per_split,
                                                                float* __restrict__ out) {
  using C = FlashCfg<H>;
  __shared__ __attribute__((aligned(16))) char lds[C::LDS];
  const float gs = gscale ? *gscale : 1.f;
  const bf16_t* O = OWNQ ? qn : dn;
  const bf16_t* X = OWNQ ? dn : qn;
  const long nown = OWNQ ? bq : nd, nx = OWNQ ? nd : bq;
  const long o0 = (long)blockIdx.y * 128;
  const long ntile = (nx + 63) / 64;
  const long t0 = (long)blockIdx.x * tiles_per_split, t1 = std::min(ntile, t0 + tiles_per_split);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;  // product 1: own rows x tile rows
  const int wf = (wave & 1) * (H / 2);                    // product 2: feature columns
  const uint32_t lb = __builtin_amdgcn_readfirstlane(ttg::lds_addr_of(lds));
  char* dsimg = lds + C::OWN + 2 * C::XT;
  f32x4 acc_o[2][C::NO];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < C::NO; ++j) acc_o[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // per own row (product-1 layout: rows wm + 16i + 4(lane>>4) + r): its lse when OWNQ
  float lown[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long row = o0 + wm + 16 * i + 4 * (lane >> 4) + r;
      lown[i][r] = (OWNQ && row < nown) ? lse[row] : 0.f;
    }
  if (t0 < t1) {
    flash_stage<H>(O, nown, o0, 128, lb);
    flash_stage<H>(X, nx, t0 * 64, 64, lb + C::OWN);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (long t = t0; t < t1; ++t) {
    const int cur = (int)((t - t0) & 1);
    const char* xi = lds + C::OWN + cur * C::XT;
    if (t + 1 < t1) flash_stage<H>(X, nx, (t + 1) * 64, 64, lb + C::OWN + (cur ^ 1) * C::XT);
    // product 1: S tile [128 own x 64 tile rows]
    f32x4 acc_s[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc_s[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < C::NKT; ++kt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        uint4 fa[2], fb[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) fa[i] = ttg::frag<bf16_t, false>(lds + kt * 128 * 128, wm + 16 * i, ks);
#pragma unroll
        for (int j = 0; j < 2; ++j) fb[j] = ttg::frag<bf16_t, false>(xi + kt * 64 * 128, wn + 16 * j, ks);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc_s[i][j] = ttg::mma<bf16_t>(fa[i], fb[j], acc_s[i][j]);
      }
    // dS (own row, tile row) -> bf16 K-contig image [128 own rows][64 tile rows]
    float lx[2] = {0.f, 0.f};
    if (!OWNQ) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const long xr = t * 64 + wn + 16 * j + (lane & 15);
        lx[j] = xr < nx ? lse[xr] : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int orl = wm + 16 * i + 4 * (lane >> 4) + r, xcl = wn + 16 * j + (lane & 15);
          const long orow = o0 + orl, xrow = t * 64 + xcl;
          const long qi = OWNQ ? orow : xrow, dj = OWNQ ? xrow : orow;
          const bool lab = dj == label_off + qi;
          float s = acc_s[i][j][r] * inv_tau;
          if (!lab) s -= offdiag;
          const float p = __expf(s - (OWNQ ? lown[i][r] : lx[j]));
          const float v = (orow < nown && xrow < nx) ? gs * (p - (lab ? 1.f : 0.f)) : 0.f;
          *reinterpret_cast<bf16_t*>(dsimg + orl * 128 + ((((xcl >> 3) ^ ((orl >> 1) & 7))) << 4) + (xcl & 7) * 2) =
              f2bf(v);
        }
    __syncthreads();
    // product 2: dO[128 own x H] += dS[128 x 64] . X[64 x H]
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 fa[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = ttg::frag<bf16_t, false>(dsimg, wm + 16 * i, ks);
#pragma unroll
      for (int j = 0; j < C::NO; ++j) {
        const int f = wf + 16 * j;
        const uint4 fb = frag_kc_tr(xi + (f >> 6) * 64 * 128, f & 63, ks);
#pragma unroll
        for (int i = 0; i < 2; ++i) acc_o[i][j] = ttg::mma<bf16_t>(fa[i], fb, acc_o[i][j]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of tile t+1
    __syncthreads();                                   // everyone's; dS and tile t are free
  }
  // out: [splits][nown][H] fp32 slab of this split (or the final array when unsplit)
  float* dst = out + (long)blockIdx.x * nown * H;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long row = o0 + wm + 16 * i + 4 * (lane >> 4) + r;
      if (row >= nown) continue;
#pragma unroll
      for (int j = 0; j < C::NO; ++j) dst[row * H + wf + 16 * j + (lane & 15)] = acc_o[i][j][r] * inv_tau;
    }
}

__global__ __launch_bounds__(256) void infonce_slab_sum_kernel(const float* __restrict__ slab, int splits, long n,
                                                               float* __restrict__ out) {
  const long i = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= n) return;
  float4 a = *reinterpret_cast<const float4*>(slab + i);
  for (int s = 1; s < splits; ++s) {
    const float4 b = *reinterpret_cast<const float4*>(slab + (long)s * n + i);
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  *reinterpret_cast<float4*>(out + i) = a;
}

// sweep splits per role: enough workgroups to cover the 256 CUs
inline int flash_splits(long nown, long nx) {
  const long blocks = (nown + 127) / 128, ntile = (nx + 63) / 64;
  return (int)std::max<long>(1, std::min<long>(ntile, 256 / std::max<long>(blocks, 1)));
}
inline bool flash_ok(int dtype, int h) { return dtype == TT_DT_BF16 && (h == 128 || h == 256); }

constexpr int TOPK_MAX = ttk::SK_MAX;

// ---------------------------------------------------------------- margin loss
__global__ __launch_bounds__(256) void margin_fwd_kernel(const float* __restrict__ qn, long bq,
                                                         const float* __restrict__ dn, int h, long label_off,
                                                         const int32_t* __restrict__ idx, int k, float margin,
                                                         float* __restrict__ row_loss) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= bq) return;
  const float* q = qn + row * h;
  const float* dp = dn + (label_off + row) * h;
  float pos = 0.f, neg = 0.f;
  for (int c = lane; c < h; c += 64) pos += q[c] * dp[c];
  for (int j = 0; j < k; ++j) {
    const float* dj = dn + (long)idx[row * k + j] * h;
    for (int c = lane; c < h; c += 64) neg += q[c] * dj[c];
  }
  pos = wave_sum(pos);
  neg = wave_sum(neg) / k;
  if (lane == 0) row_loss[row] = fmaxf(margin - pos + neg, 0.f);
}

// Backward in three launches, deterministic (the same inputs give the same bits in every
// run: no float atomics; the document gradient of every document is summed in a fixed
// order). Mined negatives repeat across rows (rows of one batch share their hardest
// documents), so the document sums go through groups of R rows:
//   margin_rows_kernel    : one wave per row (all rows in flight): dqn and the row's
//                           coefficients (positive -gscale, each negative gscale / k; 0
//                           when the hinge is inactive);
//   margin_group_kernel   : one workgroup per R rows (R (k + 1) <= 2048 entries): the
//                           group's (document, entry) keys sorted in LDS (bitonic), slots
//                           numbered in sorted order, one coefficient-weighted sum of q rows
//                           per distinct document in entry order -> partial row P[g][slot];
//                           slot map SM[document][g] = slot + 1 (0: the group has none);
//   margin_combine_kernel : one wave per document: the partials of the groups that hold
//                           it, in ascending group order, then ddn[document] += the sum.
constexpr int MB_ENT = 2048;

// rows per group: the largest power of two <= 32 with R (k + 1) <= MB_ENT (32: 256 groups at
// B 8192, one per CU; 64 measured 80 us for the group pass at configs[2])
inline int margin_group_rows(int k) {
  int r = 32;
  while (r > 1 && (long)r * (k + 1) > MB_ENT) r >>= 1;
  return r;
}

__global__ __launch_bounds__(256) void margin_rows_kernel(const float* __restrict__ qn, long bq,
                                                          const float* __restrict__ dn, int h, long label_off,
                                                          const int32_t* __restrict__ idx, int k, float margin,
                                                          const float* __restrict__ gscale, float* __restrict__ dqn,
                                                          float2* __restrict__ coef) {
  const float gs = gscale ? *gscale : 1.f;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= bq) return;
  const float* q = qn + row * h;
  const float* dp = dn + (label_off + row) * h;
  float pos = 0.f, neg = 0.f;
  for (int c = lane; c < h; c += 64) pos += q[c] * dp[c];
  for (int j = 0; j < k; ++j) {
    const float* dj = dn + (long)idx[row * k + j] * h;
    for (int c = lane; c < h; c += 64) neg += q[c] * dj[c];
  }
  pos = wave_sum(pos);
  neg = wave_sum(neg) / k;
  // torch.clamp(min=0) passes the gradient where the argument is >= 0
  const bool active = (margin - pos + neg) >= 0.f;
  const float gn = active ? gs / k : 0.f;
  const float gp = active ? -gs : 0.f;
  for (int c = lane; c < h; c += 64) {
    float d = gp * dp[c];
    for (int j = 0; j < k; ++j) d += gn * dn[(long)idx[row * k + j] * h + c];
    dqn[row * h + c] = d;
  }
  if (lane == 0) coef[row] = make_float2(gp, gn);
}

// q rows of a group staged in LDS for the partial sums when they fit (h <= 512 at R 64)
constexpr int MG_QS_BYTES = 64 * 512 * 4;

__global__ __launch_bounds__(256) void margin_group_kernel(const float* __restrict__ qn, long bq, int h,
                                                           long label_off, const int32_t* __restrict__ idx, int k,
                                                           const float2* __restrict__ coef, int R, int G,
                                                           float* __restrict__ P, int* __restrict__ SM) {
  __shared__ unsigned long long key[MB_ENT];  // document << 32 | entry; unused = all ones
  __shared__ int head[MB_ENT];                // sorted position of slot u's first entry
  __shared__ int wsum[256];
  __shared__ __attribute__((aligned(16))) float qs[MG_QS_BYTES / 4];
  const int g = blockIdx.x;
  const long r0 = (long)g * R;
  const int nr = (int)(bq - r0 < R ? bq - r0 : R);
  const int kp = k + 1;  // entry 0 of a row: its positive; 1..k: its negatives
  const int ne = nr * kp;
  __shared__ float2 cf[64];  // the rows' coefficients (R <= 64)
  const bool staged = (long)nr * h * 4 <= MG_QS_BYTES;
  if (staged)
    for (int e = threadIdx.x; e < nr * h; e += 256) qs[e] = qn[r0 * h + e];
  if (threadIdx.x < nr) cf[threadIdx.x] = coef[r0 + threadIdx.x];
  int n2 = 2;
  while (n2 < ne) n2 <<= 1;
  for (int e = threadIdx.x; e < n2; e += 256) {
    unsigned long long v = ~0ull;
    if (e < ne) {
      const int rl = e / kp, j = e - rl * kp;
      if (coef[r0 + rl].x != 0.f) {
        const long doc = j == 0 ? label_off + r0 + rl : (long)idx[(r0 + rl) * k + j - 1];
        v = ((unsigned long long)doc << 32) | (unsigned)e;
      }
    }
    key[e] = v;
  }
  __syncthreads();
  for (int size = 2; size <= n2; size <<= 1) {  // bitonic sort, ascending
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < n2 / 2; t += 256) {
        const int i = 2 * t - (t & (stride - 1));
        const int j = i + stride;
        const bool up = (i & size) == 0;
        const unsigned long long a = key[i], b = key[j];
        if ((a > b) == up) { key[i] = b; key[j] = a; }
      }
      __syncthreads();
    }
  }
  // slots in sorted order: thread t owns positions [t * per, (t + 1) * per)
  const int per = (n2 + 255) / 256;
  const int p0 = threadIdx.x * per;
  int cnt = 0;
  for (int i = p0; i < p0 + per && i < n2; ++i) {
    const unsigned long long v = key[i];
    cnt += v != ~0ull && (i == 0 || (key[i - 1] >> 32) != (v >> 32));
  }
  wsum[threadIdx.x] = cnt;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {  // inclusive scan of the per-thread counts
    const int add = threadIdx.x >= off ? wsum[threadIdx.x - off] : 0;
    __syncthreads();
    wsum[threadIdx.x] += add;
    __syncthreads();
  }
  int u = wsum[threadIdx.x] - cnt;
  __shared__ int s_nh, s_nv;  // slots; valid keys (they sort first)
  for (int i = p0; i < p0 + per && i < n2; ++i) {
    const unsigned long long v = key[i];
    if (v == ~0ull) continue;
    if (i == 0 || (key[i - 1] >> 32) != (v >> 32)) head[u++] = i;
    if (i + 1 == n2 || key[i + 1] == ~0ull) s_nv = i + 1;
  }
  if (threadIdx.x == 255) s_nh = wsum[255];
  if (threadIdx.x == 0 && key[0] == ~0ull) s_nv = 0;
  __syncthreads();
  const int nh = s_nh, nv = s_nv;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* Pg = P + (long)g * R * kp * h;
  // one wave per slot: the coefficient-weighted sum of the slot's q rows in entry order
  // (from LDS when staged), written as the group's partial row
  for (int sl = wave; sl < nh; sl += 4) {
    const int i0 = head[sl], i1 = sl + 1 < nh ? head[sl + 1] : nv;
    const unsigned doc = (unsigned)(key[i0] >> 32);
    for (int c0 = 0; c0 < h; c0 += 256) {
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      for (int i = i0; i < i1; ++i) {
        const int e = (int)(key[i] & 0xffffffffu);
        const int rl = e / kp;
        const float w = e - rl * kp == 0 ? cf[rl].x : cf[rl].y;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int c = c0 + lane + 64 * m;
          if (c < h) acc[m] += w * (staged ? qs[rl * h + c] : qn[(r0 + rl) * h + c]);
        }
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int c = c0 + lane + 64 * m;
        if (c < h) Pg[(long)sl * h + c] = acc[m];
      }
    }
    if (lane == 0) SM[(long)doc * G + g] = sl + 1;
  }
}

// One wave per document: the partials of the groups that hold it, added in ascending
// group order; their loads are issued eight at a time before the adds (independent
// rows), so a document's chain costs one load latency per eight groups.
__global__ __launch_bounds__(256) void margin_combine_kernel(const int* __restrict__ SM, int G,
                                                             const float* __restrict__ P, long gstride, int h,
                                                             long nd, float* __restrict__ ddn) {
  const long doc = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (doc >= nd) return;
  const int* sm = SM + doc * G;
  bool any = false;
  for (int g0 = 0; g0 < G; g0 += 64) any |= __builtin_amdgcn_ballot_w64(g0 + lane < G && sm[g0 + lane] != 0) != 0;
  if (!any) return;
  for (int c0 = 0; c0 < h; c0 += 256) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int g0 = 0; g0 < G; g0 += 64) {
      const int s = g0 + lane < G ? sm[g0 + lane] : 0;
      unsigned long long mask = __builtin_amdgcn_ballot_w64(s != 0);
      while (mask) {  // groups in ascending order, eight loads in flight
        constexpr int NB = 8;
        float v[NB][4];
        int n = 0;
#pragma unroll
        for (int u = 0; u < NB; ++u) {
          if (mask) {
            const int b = __builtin_ctzll(mask);
            mask &= mask - 1;
            const int slot = __builtin_amdgcn_readlane(s, b) - 1;
            const float* p = P + (long)(g0 + b) * gstride + (long)slot * h;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
              const int c = c0 + lane + 64 * m;
              v[u][m] = c < h ? p[c] : 0.f;
            }
            n = u + 1;
          }
        }
#pragma unroll
        for (int u = 0; u < NB; ++u)
          if (u < n)
#pragma unroll
            for (int m = 0; m < 4; ++m) acc[m] += v[u][m];
      }
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int c = c0 + lane + 64 * m;
      if (c < h) ddn[doc * h + c] += acc[m];
    }
  }
}

struct MarginWs {
  int R, G;
  long off_sm, off_p, bytes;
};
inline MarginWs margin_ws(long bq, long nd, int h, int k) {
  auto al = [](long x) { return (x + 255) & ~255L; };
  MarginWs w{};
  w.R = margin_group_rows(k);
  w.G = (int)((bq + w.R - 1) / w.R);
  w.off_sm = al(bq * 8);
  w.off_p = w.off_sm + al(nd * w.G * 4);
  w.bytes = w.off_p + al((long)w.G * w.R * (k + 1) * h * 4);
  return w;
}

inline int esize(int dtype) { return dtype == TT_DT_BF16 ? 2 : 4; }

struct InfoWs {
  long ds, sk;
};
inline long infonce_ws(int dtype, long bq, long nd, int h, InfoWs* w) {
  auto al = [](long x) { return (x + 255) & ~255L; };
  const int s1 = tt_gemm_pick_splits((int)bq, h, (int)nd, 1);
  const int s2 = tt_gemm_pick_splits((int)nd, h, (int)bq, 1);
  const long sk = std::max(tt_gemm_ws_size((int)bq, h, 1, s1), tt_gemm_ws_size((int)nd, h, 1, s2));
  w->ds = 0;
  w->sk = al(bq * ((nd + 7) / 8 * 8) * esize(dtype));
  return w->sk + al(sk * 4);
}

}  // namespace

extern "C" int tt_l2norm_fwd(int dtype, const float* x, long rows, int cols, float eps, void* y, float* y32,
                             float* norm, void* stream) {
  TT_CHECK_ARG(cols <= 64 * MAXC, "tt_l2norm_fwd: cols %d > %d", cols, 64 * MAXC);
  if (rows == 0) return 0;
  dim3 g((unsigned)tt_ceil_div(rows, 4));
  if (dtype == TT_DT_BF16)
    hipLaunchKernelGGL(l2norm_fwd_kernel<bf16_t>, g, dim3(256), 0, (hipStream_t)stream, x, rows, cols, eps,
                       (bf16_t*)y, y32, norm);
  else
    hipLaunchKernelGGL(l2norm_fwd_kernel<float>, g, dim3(256), 0, (hipStream_t)stream, x, rows, cols, eps,
                       (float*)y, y32, norm);
  TT_CHECK_LAUNCH("l2norm_fwd_kernel");
  return 0;
}

extern "C" int tt_l2norm_bwd(const float* dy, const float* y32, const float* norm, long rows, int cols, float eps,
                             float* dx, int accumulate, void* stream) {
  TT_CHECK_ARG(cols <= 64 * MAXC, "tt_l2norm_bwd: cols %d", cols);
  if (rows == 0) return 0;
  hipLaunchKernelGGL(l2norm_bwd_kernel, dim3((unsigned)tt_ceil_div(rows, 4)), dim3(256), 0, (hipStream_t)stream, dy,
                     y32, norm, rows, cols, eps, dx, accumulate);
  TT_CHECK_LAUNCH("l2norm_bwd_kernel");
  return 0;
}

extern "C" long tt_infonce_fwd_ws_size(long bq, long nd) {
  const int rb = tt_ceil_div(bq, 128);
  const long nct = (nd + 127) / 128;
  const long splits = std::max<long>(1, std::min<long>(nct, tt_ceil_div(1024, rb)));
  return (2L * splits * bq + bq) * (long)sizeof(float);
}

extern "C" int tt_infonce_fwd(int dtype, const void* qn, long bq, const void* dn, long nd, int h, float inv_tau,
                              float offdiag_sub, long label_offset, float* lse, float* row_loss, void* ws,
                              void* stream) {
  TT_CHECK_ARG(dtype == TT_DT_F32 || dtype == TT_DT_BF16, "tt_infonce_fwd: bad dtype");
  TT_CHECK_ARG(label_offset >= 0 && label_offset + bq <= nd, "tt_infonce_fwd: labels outside [0, nd)");
  TT_CHECK_ARG((h * esize(dtype)) % 16 == 0, "tt_infonce_fwd: h=%d misaligned", h);
  TT_CHECK_ARG(bq <= 65535L * 128 && nd < (1L << 31), "tt_infonce_fwd: too large");
  if (bq == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int rb = tt_ceil_div(bq, 128);
  const long nct = (nd + 127) / 128;
  int splits = (int)std::max<long>(1, std::min<long>(nct, tt_ceil_div(1024, rb)));
  const int per = tt_ceil_div(nct, splits);
  splits = tt_ceil_div(nct, per);
  TT_CHECK_ARG(ws != nullptr, "tt_infonce_fwd: null workspace");
  float* pool = static_cast<float*>(ws);
  float* pm = pool;
  float* pl = pool + (long)splits * bq;
  float* diag = pl + (long)splits * bq;
  dim3 grid(splits, rb);
  if (dtype == TT_DT_BF16)
    hipLaunchKernelGGL(infonce_fwd_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)qn, bq, (const bf16_t*)dn,
                       nd, h, inv_tau, offdiag_sub, label_offset, per, pm, pl, diag);
  else
    hipLaunchKernelGGL(infonce_fwd_kernel<float>, grid, dim3(256), 0, st, (const float*)qn, bq, (const float*)dn, nd,
                       h, inv_tau, offdiag_sub, label_offset, per, pm, pl, diag);
  TT_CHECK_LAUNCH("infonce_fwd_kernel");
  hipLaunchKernelGGL(infonce_finalize_kernel, dim3(tt_ceil_div(bq, 256)), dim3(256), 0, st, pm, pl, splits, bq, diag,
                     lse, row_loss);
  TT_CHECK_LAUNCH("infonce_finalize_kernel");
  return 0;
}

static bool use_flash(int dtype, int h) { return flash_ok(dtype, h) && tt::opt(tt::OPT_INFONCE_FLASH) != 0; }

extern "C" long tt_infonce_bwd_ws_size(int dtype, long bq, long nd, int h) {
  if (use_flash(dtype, h)) {  // fp32 partial slabs of split sweeps (none when unsplit)
    const int sq = flash_splits(bq, nd), sd = flash_splits(nd, bq);
    const long a = sq > 1 ? (long)sq * bq * h : 0, b = sd > 1 ? (long)sd * nd * h : 0;
    return std::max<long>(256, std::max(a, b) * (long)sizeof(float));
  }
  InfoWs w;
  return infonce_ws(dtype, bq, nd, h, &w);
}

// one role of the fused backward: out = dq (OWNQ) or dd, through slabs when split
template <int H, bool OWNQ>
static int flash_role(const bf16_t* qn, long bq, const bf16_t* dn, long nd, float inv_tau, float offdiag,
                      long label_off, const float* lse, const float* gscale, float* out, float* slab,
                      hipStream_t st) {
  const long nown = OWNQ ? bq : nd, nx = OWNQ ? nd : bq;
  const long ntile = (nx + 63) / 64;
  int splits = flash_splits(nown, nx);
  const int per = tt_ceil_div(ntile, splits);
  splits = tt_ceil_div(ntile, per);
  const dim3 grid((unsigned)splits, (unsigned)tt_ceil_div(nown, 128));
  hipLaunchKernelGGL((infonce_bwd_flash_kernel<H, OWNQ>), grid, dim3(512), 0, st, qn, bq, dn, nd, inv_tau, offdiag,
                     label_off, lse, gscale, per, splits > 1 ? slab : out);
  TT_CHECK_LAUNCH("infonce_bwd_flash_kernel");
  if (splits > 1) {
    const long n = nown * H;
    hipLaunchKernelGGL(infonce_slab_sum_kernel, dim3((unsigned)tt_ceil_div(n / 4, 256)), dim3(256), 0, st, slab,
                       splits, n, out);
    TT_CHECK_LAUNCH("infonce_slab_sum_kernel");
  }
  return 0;
}

extern "C" int tt_infonce_bwd(int dtype, const void* qn, long bq, const void* dn, long nd, int h, float inv_tau,
                              float offdiag_sub, long label_offset, const float* lse, const float* gscale, float* dqn,
                              float* ddn, void* ws, void* stream) {
  TT_CHECK_ARG(dtype == TT_DT_F32 || dtype == TT_DT_BF16, "tt_infonce_bwd: bad dtype");
  TT_CHECK_ARG(label_offset >= 0 && label_offset + bq <= nd, "tt_infonce_bwd: labels outside [0, nd)");
  if (bq == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (use_flash(dtype, h)) {
    TT_CHECK_ARG((((uintptr_t)qn | (uintptr_t)dn) & 15) == 0, "tt_infonce_bwd: bf16 rows must be 16-byte aligned");
    TT_CHECK_ARG(ws != nullptr && bq <= 65535L * 128 && nd <= 65535L * 128, "tt_infonce_bwd: workspace/size");
    const bf16_t* q = static_cast<const bf16_t*>(qn);
    const bf16_t* d = static_cast<const bf16_t*>(dn);
    float* slab = static_cast<float*>(ws);
    if (h == 256) {
      TT_PROPAGATE((flash_role<256, true>(q, bq, d, nd, inv_tau, offdiag_sub, label_offset, lse, gscale, dqn, slab, st)));
      TT_PROPAGATE((flash_role<256, false>(q, bq, d, nd, inv_tau, offdiag_sub, label_offset, lse, gscale, ddn, slab, st)));
    } else {
      TT_PROPAGATE((flash_role<128, true>(q, bq, d, nd, inv_tau, offdiag_sub, label_offset, lse, gscale, dqn, slab, st)));
      TT_PROPAGATE((flash_role<128, false>(q, bq, d, nd, inv_tau, offdiag_sub, label_offset, lse, gscale, ddn, slab, st)));
    }
    return 0;
  }
  InfoWs w;
  infonce_ws(dtype, bq, nd, h, &w);
  char* base = static_cast<char*>(ws);
  void* ds = base + w.ds;
  float* sk = reinterpret_cast<float*>(base + w.sk);
  const long ldds = (nd + 7) / 8 * 8;  // 16-byte aligned rows for the dS operand
  dim3 grid((unsigned)tt_ceil_div(nd, 128), (unsigned)tt_ceil_div(bq, 128));
  if (dtype == TT_DT_BF16)
    hipLaunchKernelGGL(infonce_dscore_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)qn, bq,
                       (const bf16_t*)dn, nd, h, inv_tau, offdiag_sub, label_offset, lse, gscale, ldds, (bf16_t*)ds);
  else
    hipLaunchKernelGGL(infonce_dscore_kernel<float>, grid, dim3(256), 0, st, (const float*)qn, bq, (const float*)dn,
                       nd, h, inv_tau, offdiag_sub, label_offset, lse, gscale, ldds, (float*)ds);
  TT_CHECK_LAUNCH("infonce_dscore_kernel");
  // dqn = inv_tau * dS dn   (NN)
  {
    tt_gemm_batch g{};
    g.a[0] = ds; g.b[0] = dn; g.c[0] = dqn;
    const int sp = tt_gemm_pick_splits((int)bq, h, (int)nd, 1);
    TT_PROPAGATE(tt_gemm(dtype, TT_DT_F32, 0, 1, (int)bq, h, (int)nd, &g, 1, ldds, h, h, inv_tau, 0, 0, 0, 0, 0.f, sp,
                         sk, stream));
  }
  // ddn = inv_tau * dS^T qn (TN)
  {
    tt_gemm_batch g{};
    g.a[0] = ds; g.b[0] = qn; g.c[0] = ddn;
    const int sp = tt_gemm_pick_splits((int)nd, h, (int)bq, 1);
    TT_PROPAGATE(tt_gemm(dtype, TT_DT_F32, 1, 1, (int)nd, h, (int)bq, &g, 1, ldds, h, h, inv_tau, 0, 0, 0, 0, 0.f, sp,
                         sk, stream));
  }
  return 0;
}

// ws: the score block S [bq, nd] fp32, then the per-chunk candidates (values, indices)
// bf16 operands with h in {128, 256}: the streamed scan of tt_score.hip (no score matrix)
long tt_hn_scan_ws_size(long bq, long nd, int k);
bool tt_hn_scan_supported(int dtype, int h);
int tt_hn_scan_topk(const void* qn, long bq, const void* dn, long nd, int h, long label_offset, int k, int32_t* idx,
                    float* val, void* ws, void* stream);

extern "C" long tt_hardneg_ws_size(int dtype, long bq, long nd, int h, int k) {
  if (tt_hn_scan_supported(dtype, h)) return tt_hn_scan_ws_size(bq, nd, k < 1 ? 1 : k);
  const long ncand = tt_ceil_div(nd, ttk::split_chunk(bq, nd)) * (long)TOPK_MAX;
  return ((bq * nd * 4 + 255) & ~255L) + 2 * ((bq * ncand * 4 + 255) & ~255L);
}

extern "C" int tt_hardneg_topk(int dtype, const void* qn, long bq, const void* dn, long nd, int h, long label_offset,
                               int k, int32_t* idx, float* val, void* ws, void* stream) {
  TT_CHECK_ARG(k >= 1 && k <= TOPK_MAX && k <= nd, "tt_hardneg_topk: k=%d (nd=%ld)", k, nd);
  TT_CHECK_ARG(label_offset < 0 || label_offset + bq <= nd, "tt_hardneg_topk: labels outside [0, nd)");
  if (bq == 0) return 0;
  if (tt_hn_scan_supported(dtype, h)) {
    TT_CHECK_ARG((((uintptr_t)qn | (uintptr_t)dn) & 15) == 0, "tt_hardneg_topk: bf16 rows must be 16-byte aligned");
    return tt_hn_scan_topk(qn, bq, dn, nd, h, label_offset, k, idx, val, ws, stream);
  }
  float* S = static_cast<float*>(ws);
  tt_gemm_batch g{};
  g.a[0] = qn; g.b[0] = dn; g.c[0] = S;
  TT_PROPAGATE(tt_gemm(dtype, TT_DT_F32, 0, 0, (int)bq, (int)nd, h, &g, 1, h, h, nd, 1.f, 0, 0, 0, 0, 0.f, 1,
                       nullptr, stream));
  // many waves per row (column chunks), then one wave per row merges the candidates
  const long chunk = ttk::split_chunk(bq, nd), nsp = tt_ceil_div(nd, chunk);
  const long ncand = nsp * k;
  char* cbase = static_cast<char*>(ws) + ((bq * nd * 4 + 255) & ~255L);
  float* cv = reinterpret_cast<float*>(cbase);
  int* ci = reinterpret_cast<int*>(cbase + ((bq * nsp * TOPK_MAX * 4 + 255) & ~255L));
  hipStream_t st = (hipStream_t)stream;
  const dim3 gs((unsigned)tt_ceil_div(bq, 4), (unsigned)nsp);
  if (k <= 4)
    hipLaunchKernelGGL((ttk::topk_split_kernel<4>), gs, dim3(256), 0, st, S, bq, nd, chunk, label_offset, k, cv, ci);
  else
    hipLaunchKernelGGL((ttk::topk_split_kernel<TOPK_MAX>), gs, dim3(256), 0, st, S, bq, nd, chunk, label_offset, k,
                       cv, ci);
  TT_CHECK_LAUNCH("topk_split_kernel");
  const dim3 gm((unsigned)tt_ceil_div(bq, 4));
  if (k <= 4)
    hipLaunchKernelGGL((ttk::topk_merge_kernel<4>), gm, dim3(256), 0, st, cv, ci, bq, ncand, k, idx, val);
  else
    hipLaunchKernelGGL((ttk::topk_merge_kernel<TOPK_MAX>), gm, dim3(256), 0, st, cv, ci, bq, ncand, k, idx, val);
  TT_CHECK_LAUNCH("topk_merge_kernel");
  return 0;
}

extern "C" int tt_margin_fwd(const float* qn, long bq, const float* dn, long nd, int h, long label_offset,
                             const int32_t* idx, int k, float margin, float* row_loss, void* stream) {
  TT_CHECK_ARG(label_offset >= 0 && label_offset + bq <= nd && k >= 1, "tt_margin_fwd: bad labels/k");
  if (bq == 0) return 0;
  hipLaunchKernelGGL(margin_fwd_kernel, dim3((unsigned)tt_ceil_div(bq, 4)), dim3(256), 0, (hipStream_t)stream, qn, bq,
                     dn, h, label_offset, idx, k, margin, row_loss);
  TT_CHECK_LAUNCH("margin_fwd_kernel");
  return 0;
}

extern "C" long tt_margin_bwd_ws_size(long bq, long nd, int h, int k) {
  if (bq <= 0 || k < 1) return 256;
  return margin_ws(bq, nd, h, k).bytes;
}

extern "C" int tt_margin_bwd(const float* qn, long bq, const float* dn, long nd, int h, long label_offset,
                             const int32_t* idx, int k, float margin, const float* gscale, float* dqn, float* ddn,
                             void* ws, void* stream) {
  TT_CHECK_ARG(label_offset >= 0 && label_offset + bq <= nd && k >= 1 && k < MB_ENT, "tt_margin_bwd: bad labels/k");
  TT_CHECK_ARG(nd < (1L << 31), "tt_margin_bwd: nd=%ld too large", nd);
  if (bq == 0) return 0;
  TT_CHECK_ARG(ws != nullptr, "tt_margin_bwd: null workspace (tt_margin_bwd_ws_size bytes)");
  const MarginWs w = margin_ws(bq, nd, h, k);
  char* base = static_cast<char*>(ws);
  float2* coef = reinterpret_cast<float2*>(base);
  int* SM = reinterpret_cast<int*>(base + w.off_sm);
  float* P = reinterpret_cast<float*>(base + w.off_p);
  hipStream_t st = (hipStream_t)stream;
  TT_CHECK_HIP(hipMemsetAsync(SM, 0, nd * w.G * 4, st));
  hipLaunchKernelGGL(margin_rows_kernel, dim3((unsigned)tt_ceil_div(bq, 4)), dim3(256), 0, st, qn, bq, dn, h,
                     label_offset, idx, k, margin, gscale, dqn, coef);
  TT_CHECK_LAUNCH("margin_rows_kernel");
  hipLaunchKernelGGL(margin_group_kernel, dim3((unsigned)w.G), dim3(256), 0, st, qn, bq, h, label_offset, idx, k,
                     coef, w.R, w.G, P, SM);
  TT_CHECK_LAUNCH("margin_group_kernel");
  hipLaunchKernelGGL(margin_combine_kernel, dim3((unsigned)tt_ceil_div(nd, 4)), dim3(256), 0, st, SM, w.G, P,
                     (long)w.R * (k + 1) * h, h, nd, ddn);
  TT_CHECK_LAUNCH("margin_combine_kernel");
  return 0;
}
