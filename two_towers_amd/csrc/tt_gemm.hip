// Generic batched MFMA GEMM (NT / NN / TN, optional split-K) and the C-ABI
// entry points tt_gemm / tt_gemm_ws_size / tt_gemm_pick_splits.
#include <stdarg.h>
#include <stdlib.h>

#include <type_traits>

#include "tt_api.h"
#include "tt_gemm_core.h"

namespace tt {
static thread_local char g_err[512];
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace tt

extern "C" const char* tt_version(void) { return "tt_hip 0.1.0 gfx950"; }
extern "C" const char* tt_last_error(void) { return tt::g_err; }

namespace {

struct GemmArgs {
  const void* a[4];
  const void* b[4];
  void* c[4];
  const float* bias[4];
  int bshift[4];
  long lda, ldb, ldc;
  int M, N, K;
  int splits, kt_per_split;
  float alpha;
  int beta, relu, seq_t;
  uint32_t drop_seed, drop_thresh;
  float drop_inv_keep;
  long part_stride;  // elements between split partials (fp32), 0 if no split
  int vec_ok;        // C rows 16-byte aligned: 8-column vector stores allowed
  int force_regstage;
};

constexpr int BM = 128, BN = 128;

// XCD-aware tile order: consecutive workgroup ids are dealt round-robin over the 8
// XCDs, so remap them (bijectively) to give every XCD a contiguous run of tiles in
// row-major order; the tiles of one A panel then share that XCD's L2.
__device__ __forceinline__ void tile_of(int& mt, int& nt) {
  const int ntn = gridDim.x, nwg = gridDim.x * gridDim.y;
  const int bid = blockIdx.y * ntn + blockIdx.x;
  const int xcd = bid & 7, loc = bid >> 3;
  const int q = nwg >> 3, r = nwg & 7;
  const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  mt = id / ntn;
  nt = id - mt * ntn;
}

template <typename T, bool AKO, bool BKO, bool SHIFT, typename TO, bool DMA>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs g) {
  using ML = std::conditional_t<DMA, ttg::MainLoopDMA<T, AKO, BKO, BM, BN>, ttg::MainLoop<T, AKO, BKO, BM, BN>>;
  __shared__ __attribute__((aligned(16))) char lds[ML::LDS_BYTES];
  const int z = blockIdx.z;
  const int bi = z / g.splits, s = z % g.splits;
  int mt, nt;
  tile_of(mt, nt);
  const int m0 = mt * BM, n0 = nt * BN;
  const T* A = static_cast<const T*>(g.a[bi]);
  const T* B = static_cast<const T*>(g.b[bi]);

  f32x4 acc[ML::TM][ML::TN];
#pragma unroll
  for (int i = 0; i < ML::TM; ++i)
#pragma unroll
    for (int j = 0; j < ML::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (g.K * (int)sizeof(T) + ttg::KTB - 1) / ttg::KTB;
  const int kt0 = s * g.kt_per_split;
  const int kt1 = min(nk, kt0 + g.kt_per_split);

  auto run = [&](const auto& la) {
    if constexpr (!BKO) {
      ttg::KCPlain<T> lb{B, g.ldb, n0, g.N};
      ML::run(la, lb, g.K, kt0, kt1, lds, acc);
    } else if constexpr (SHIFT) {
      ttg::KOShift<T> lb{B, g.ldb, n0, g.N - n0, g.seq_t, g.bshift[bi]};
      ML::run(la, lb, g.K, kt0, kt1, lds, acc);
    } else {
      ttg::KOPlain<T> lb{B, g.ldb, n0, g.N - n0};
      ML::run(la, lb, g.K, kt0, kt1, lds, acc);
    }
  };
  if constexpr (AKO) {
    run(ttg::KOPlain<T>{A, g.lda, m0, g.M - m0});
  } else {
    run(ttg::KCPlain<T>{A, g.lda, m0, g.M});
  }

  // ---- epilogue: stage each 64-row half of the fp32 tile in LDS, then every thread
  // finishes 8 consecutive columns of a row and writes them with 16-byte stores.
  const bool partial = g.splits > 1;
  TO* C = partial ? nullptr : static_cast<TO*>(g.c[bi]);
  float* P = partial ? static_cast<float*>(g.c[bi]) + (long)s * g.part_stride : nullptr;
  const long ldc = partial ? (long)g.N : g.ldc;
  const float* bias = partial ? nullptr : g.bias[bi];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, tid = threadIdx.x;
  constexpr int CLD = BN + 4;
  float* L = reinterpret_cast<float*>(lds);
  const int cg = (tid & 15) * 8;
  for (int hf = 0; hf < 2; ++hf) {
    if ((wave >> 1) == hf) {
      const int wn = (wave & 1) * (BN / 2);
#pragma unroll
      for (int i = 0; i < ML::TM; ++i)
#pragma unroll
        for (int j = 0; j < ML::TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            L[(16 * i + 4 * (lane >> 4) + r) * CLD + wn + 16 * j + (lane & 15)] = acc[i][j][r];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int rl = (tid >> 4) + 16 * k;
      const int gm = m0 + hf * 64 + rl, gn = n0 + cg;
      if (gm < g.M && gn < g.N) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = L[rl * CLD + cg + e];
        const bool full = gn + 8 <= g.N && g.vec_ok;
        if (partial) {
          float* dst = P + (long)gm * ldc + gn;
          if (full) st8(dst, v);
          else
            for (int e = 0; e < 8 && gn + e < g.N; ++e) dst[e] = v[e];
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float x = v[e] * g.alpha;
            if (bias && gn + e < g.N) x += bias[gn + e];
            if (g.relu) x = fmaxf(x, 0.f);
            if (g.drop_thresh) x *= tt_dropout_scale(g.drop_seed, gm, gn + e, g.drop_thresh, g.drop_inv_keep);
            v[e] = x;
          }
          TO* dst = C + (long)gm * ldc + gn;
          if (full) {
            if (g.beta) {
              float o[8];
              ld8(dst, o);
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] += o[e];
            }
            st8(dst, v);
          } else {
            for (int e = 0; e < 8 && gn + e < g.N; ++e) {
              float x = v[e];
              if (g.beta) x += Elt<TO>::ld(dst + e);
              Elt<TO>::st(dst + e, x);
            }
          }
        }
      }
    }
    __syncthreads();
  }
}

// out_b[m][n] = alpha * sum_s part_b[s][m][n] (+ bias[n]) (+ out_b)
template <typename TO>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* ws, long part_stride, int splits,
                                                            int M, int N, GemmArgs g) {
  const int bi = blockIdx.y;
  const float* P = ws + (long)bi * splits * part_stride;
  TO* C = static_cast<TO*>(g.c[bi]);
  const float* bias = g.bias[bi];
  const long total = (long)M * N;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    float v = 0.f;
    for (int s = 0; s < splits; ++s) v += P[(long)s * part_stride + e];
    const int m = (int)(e / N), n = (int)(e % N);
    v *= g.alpha;
    if (bias) v += bias[n];
    TO* p = C + (long)m * g.ldc + n;
    if (g.beta) v += Elt<TO>::ld(p);
    Elt<TO>::st(p, v);
  }
}

template <typename T, typename TO>
int launch_gemm(int akout, int bkout, bool shift, const GemmArgs& g, int nbatch, dim3 grid,
                hipStream_t st) {
  // LDS-DMA staging needs whole 16-byte chunks along K (K-contig) or along the
  // columns (K-outer); otherwise the register-staged loop masks element-wise.
  constexpr int EPC = 16 / (int)sizeof(T);
  const bool dma = (akout ? g.M % EPC == 0 : g.K % EPC == 0) && (bkout ? g.N % EPC == 0 : g.K % EPC == 0) &&
                   !g.force_regstage;
#define TT_L(AK, BK, SH)                                                                     \
  do {                                                                                       \
    if (dma) hipLaunchKernelGGL((gemm_kernel<T, AK, BK, SH, TO, true>), grid, dim3(256), 0, st, g);  \
    else hipLaunchKernelGGL((gemm_kernel<T, AK, BK, SH, TO, false>), grid, dim3(256), 0, st, g);     \
  } while (0)
  if (!akout && !bkout) TT_L(false, false, false);
  else if (!akout && bkout && !shift) TT_L(false, true, false);
  else if (!akout && bkout && shift) TT_L(false, true, true);
  else if (akout && !bkout) TT_L(true, false, false);
  else if (akout && bkout && !shift) TT_L(true, true, false);
  else TT_L(true, true, true);
#undef TT_L
  TT_CHECK_LAUNCH("gemm_kernel");
  return 0;
}

}  // namespace

extern "C" long tt_gemm_ws_size(int m, int n, int nbatch, int splits) {
  return splits > 1 ? (long)m * n * nbatch * splits : 0;
}

extern "C" int tt_gemm_pick_splits(int m, int n, int k, int nbatch) {
  const long tiles = (long)tt_ceil_div(m, BM) * tt_ceil_div(n, BN) * nbatch;
  if (tiles >= 512) return 1;
  const int nk = tt_ceil_div(k, 64);
  int s = (int)((1024 + tiles - 1) / tiles);
  s = s > nk / 8 ? nk / 8 : s;  // keep >= 8 K-tiles per split
  if (s > 64) s = 64;
  return s < 1 ? 1 : s;
}

extern "C" int tt_gemm(int dtype, int out_dtype, int a_kouter, int b_kouter, int m, int n, int k,
                       const tt_gemm_batch* batch, int nbatch, long lda, long ldb, long ldc,
                       float alpha, int beta_accum, int relu, int seq_t, uint32_t drop_seed,
                       float drop_p, int splits, float* splitk_ws, void* stream) {
  TT_CHECK_ARG(dtype == TT_DT_F32 || dtype == TT_DT_BF16, "tt_gemm: bad dtype %d", dtype);
  TT_CHECK_ARG(out_dtype == TT_DT_F32 || out_dtype == dtype, "tt_gemm: bad out_dtype %d", out_dtype);
  TT_CHECK_ARG(nbatch >= 1 && nbatch <= 4, "tt_gemm: nbatch %d not in [1,4]", nbatch);
  TT_CHECK_ARG(m >= 0 && n >= 0 && k >= 0, "tt_gemm: negative dims");
  if (m == 0 || n == 0) return 0;
  const int esz = dtype == TT_DT_BF16 ? 2 : 4;
  const int epc = 16 / esz;
  (void)epc;
  TT_CHECK_ARG((lda * esz) % 16 == 0 && (ldb * esz) % 16 == 0,
               "tt_gemm: leading dimensions must be 16-byte multiples (lda=%ld ldb=%ld)", lda, ldb);
  if (splits < 1) splits = 1;
  TT_CHECK_ARG(splits == 1 || (relu == 0 && drop_p == 0.f), "tt_gemm: split-K excludes relu/dropout");
  TT_CHECK_ARG(splits == 1 || splitk_ws != nullptr, "tt_gemm: split-K needs a workspace");
  TT_CHECK_ARG(drop_p >= 0.f && drop_p < 1.f, "tt_gemm: drop_p %f", drop_p);
  bool shift = false;
  GemmArgs g{};
  for (int b = 0; b < nbatch; ++b) {
    TT_CHECK_ARG(batch->a[b] && batch->b[b] && batch->c[b], "tt_gemm: null operand in batch %d", b);
    TT_CHECK_ARG(((uintptr_t)batch->a[b] | (uintptr_t)batch->b[b]) % 16 == 0,
                 "tt_gemm: operands must be 16-byte aligned (batch %d)", b);
    g.a[b] = batch->a[b];
    g.b[b] = batch->b[b];
    g.c[b] = batch->c[b];
    g.bias[b] = batch->bias[b];
    g.bshift[b] = batch->bshift[b];
    if (batch->bshift[b] != 0) shift = true;
  }
  TT_CHECK_ARG(!shift || (b_kouter && seq_t > 0), "tt_gemm: bshift needs b_kouter and seq_t");
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = m; g.N = n; g.K = k;
  g.alpha = alpha; g.beta = beta_accum; g.relu = relu; g.seq_t = seq_t;
  static const int force_reg = getenv("TT_GEMM_REGSTAGE") ? atoi(getenv("TT_GEMM_REGSTAGE")) : 0;
  g.force_regstage = force_reg;
  g.drop_seed = drop_seed;
  g.drop_thresh = drop_p > 0.f ? (uint32_t)(drop_p * 16777216.0f + 0.5f) : 0u;
  g.drop_inv_keep = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
  const int nk = tt_ceil_div((long)k * esz, 128);
  if (splits > nk) splits = nk > 0 ? nk : 1;
  g.kt_per_split = tt_ceil_div(nk, splits);
  splits = nk > 0 ? tt_ceil_div(nk, g.kt_per_split) : 1;
  g.splits = splits;
  hipStream_t st = static_cast<hipStream_t>(stream);
  dim3 grid(tt_ceil_div(n, BN), tt_ceil_div(m, BM), nbatch * splits);
  TT_CHECK_ARG(grid.y <= 65535, "tt_gemm: m=%d too large", m);

  {
    const int osz = out_dtype == TT_DT_BF16 ? 2 : 4;
    bool ok = (ldc * osz) % 16 == 0;
    for (int b = 0; b < nbatch; ++b) ok = ok && ((uintptr_t)batch->c[b] % 16 == 0);
    g.vec_ok = ok;
  }
  if (splits > 1) {
    GemmArgs gp = g;
    gp.part_stride = (long)m * n;
    gp.vec_ok = (n % 4 == 0);
    for (int b = 0; b < nbatch; ++b) gp.c[b] = splitk_ws + (long)b * splits * gp.part_stride;
    int rc = dtype == TT_DT_BF16 ? launch_gemm<bf16_t, float>(a_kouter, b_kouter, shift, gp, nbatch, grid, st)
                                 : launch_gemm<float, float>(a_kouter, b_kouter, shift, gp, nbatch, grid, st);
    if (rc) return rc;
    const long total = (long)m * n;
    dim3 rg((unsigned)std::min<long>(tt_ceil_div(total, 256), 2048), nbatch);
    if (out_dtype == TT_DT_F32)
      hipLaunchKernelGGL(splitk_reduce_kernel<float>, rg, dim3(256), 0, st, splitk_ws, gp.part_stride, splits, m, n, g);
    else
      hipLaunchKernelGGL(splitk_reduce_kernel<bf16_t>, rg, dim3(256), 0, st, splitk_ws, gp.part_stride, splits, m, n, g);
    TT_CHECK_LAUNCH("splitk_reduce_kernel");
    return 0;
  }
  if (dtype == TT_DT_BF16) {
    return out_dtype == TT_DT_BF16 ? launch_gemm<bf16_t, bf16_t>(a_kouter, b_kouter, shift, g, nbatch, grid, st)
                                   : launch_gemm<bf16_t, float>(a_kouter, b_kouter, shift, g, nbatch, grid, st);
  }
  return launch_gemm<float, float>(a_kouter, b_kouter, shift, g, nbatch, grid, st);
}
