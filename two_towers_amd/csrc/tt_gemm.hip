// Generic batched MFMA GEMM (NT / NN / TN, optional split-K) and the C-ABI
// entry points tt_gemm / tt_gemm_ws_size / tt_gemm_pick_splits.
#include <float.h>
#include <stdarg.h>
#include <stdlib.h>

#include <atomic>
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

namespace tt {
namespace {
struct OptDef {
  const char* name;
  const char* env;
  int dflt;
};
constexpr OptDef kOpts[OPT_N] = {
    {"gru_step", "TT_GRU_STEP", 0},               {"gru_depth", "TT_GRU_DEPTH", 4},
    {"gru_bwd_rows", "TT_GRU_BWD_ROWS", 0},     {"gru_bwd_big", "TT_GRU_BWD_BIG", 1},
    {"gru_bwd_streams", "TT_GRU_BWD_STREAMS", 2}, {"gemm_persist", "TT_GEMM_PERSIST", 1},
    {"gemm_a3", "TT_GEMM_A3", 1},                 {"gemm_regstage", "TT_GEMM_REGSTAGE", 0},
    {"gemm_stream_out", "TT_GEMM_STREAM_OUT", 1}, {"hn_gemm", "TT_HN_GEMM", 0},
    {"gru_bwd_persist", "TT_GRU_BWD_PERSIST", 1}, {"gru_fwd_step_rows", "TT_GRU_FWD_STEP_ROWS", 0},
    {"infonce_flash", "TT_INFONCE_FLASH", 1},     {"hn_map", "TT_HN_MAP", 2},
    {"gemm_skew", "TT_GEMM_SKEW", 0},             {"gemm_persist_maxk", "TT_GEMM_PERSIST_MAXK", 24},
    {"gru_fwd_xc", "TT_GRU_FWD_XC", 1},           {"gru_xc_skip", "TT_GRU_XC_SKIP", 0},
    {"gru_xc_spins", "TT_GRU_XC_SPINS", 22},      {"gru_bwd_skew", "TT_GRU_BWD_SKEW", 14},
    {"gru_fwd_skew", "TT_GRU_FWD_SKEW", 0},       {"gemm_bres", "TT_GEMM_BRES", 1},
    {"gru_xc_coop", "TT_GRU_XC_COOP", 0},         {"gemm_buf", "TT_GEMM_BUF", 1},
    {"gemm_order", "TT_GEMM_ORDER", 0},           {"gru_step_ring", "TT_GRU_STEP_RING", 4},
    {"gru_fwd_xs", "TT_GRU_FWD_XS", 1},           {"hn_scan_gemm", "TT_HN_SCAN_GEMM", 0},
    {"gemm_iepi", "TT_GEMM_IEPI", 1},             {"bres_rows", "TT_BRES_ROWS", 32},
    {"hn_scan_v", "TT_HN_SCAN_V", 5},             {"gemm_w4", "TT_GEMM_W4", 0},
};
struct OptTable {
  std::atomic<int> v[OPT_N];
  OptTable() {
    for (int i = 0; i < OPT_N; ++i) {
      const char* e = getenv(kOpts[i].env);
      v[i].store(e && *e ? atoi(e) : kOpts[i].dflt, std::memory_order_relaxed);
    }
  }
};
OptTable& opts() {
  static OptTable t;  // thread-safe one-time init
  return t;
}
int find_opt(const char* name) {
  for (int i = 0; name && i < OPT_N; ++i)
    if (strcmp(name, kOpts[i].name) == 0) return i;
  return -1;
}
}  // namespace
int opt(Opt o) { return opts().v[o].load(std::memory_order_relaxed); }
}  // namespace tt

extern "C" const char* tt_version(void) { return "tt_hip 0.2.0 gfx950"; }
extern "C" const char* tt_last_error(void) { return tt::g_err; }
extern "C" int tt_set_option(const char* name, int value) {
  const int i = tt::find_opt(name);
  TT_CHECK_ARG(i >= 0, "tt_set_option: unknown option '%s'", name ? name : "(null)");
  tt::opts().v[i].store(value, std::memory_order_relaxed);
  return 0;
}
extern "C" int tt_get_option(const char* name, int* value) {
  const int i = tt::find_opt(name);
  TT_CHECK_ARG(i >= 0 && value, "tt_get_option: unknown option '%s'", name ? name : "(null)");
  *value = tt::opt((tt::Opt)i);
  return 0;
}

namespace {

struct GemmArgs {
  const void* a[4];
  const void* b[4];
  void* c[4];
  const float* bias[4];
  int bshift[4];
  const void* a_hi[4];
  int a_split;
  long lda, ldb, ldc;
  int M, N, K;
  int splits, kt_per_split;
  float alpha;
  int beta, relu, seq_t;
  uint32_t drop_seed, drop_thresh, drop_row0;
  float drop_inv_keep;
  long part_stride;  // elements between split partials (fp32), 0 if no split
  int vec_ok;        // C rows 16-byte aligned: 8-column vector stores allowed
  int force_regstage;
  int skew;  // persistent GEMM start skew (OPT_GEMM_SKEW)
  int bias_vec_ok;  // every bias pointer 16-byte aligned
  int stream_out;   // write-through (sc1) output stores: big outputs
  int walk_g, walk_x;  // gemm_persist tile walk: column panels per group, workgroup sets (0: default)
  int nbatch;
  // gemm_persist<..., HN>: the hard-negative scan's epilogue (tt_score.hip): per (row, 64-column
  // chunk) only the maximum leaves, into cm[row * nch + chunk]; column label_off + row scores
  // -1 (the positive), columns >= N -inf
  float* cm;
  long nch, label_off;
};

constexpr int BM = 128, BN = 128;  // tile of the register-staged / small path

// 1-D grid in XCD-aware order (ttg::xcd_remap): ids enumerate (batch*split, m-tile,
// n-tile) with the n-tile fastest, so the tiles of one A panel, and all tiles of one
// split-K slice, share an XCD's L2.
#ifndef TT_TAIL_SKIP  // 0: tail tiles' idle wave rows run their MFMAs (traffic experiment only)
#define TT_TAIL_SKIP 1
#endif
using ttg::xcd_remap;
#ifndef PERSIST_IEPI  // 1: gemm_persist (A3) runs each tile's epilogue inside the next tile's first K-tile
#define PERSIST_IEPI 1
#endif
#ifndef PERSIST_BAL  // 1: gemm_persist (A3) reads its fragments in the balanced 12/4/8 order of Loop8::run3
#define PERSIST_BAL 1
#endif
#ifndef TT_EPI_PAIR  // 1: bf16 register-direct epilogues store whole 128-B lines (row_pair, tt_common.h)
#define TT_EPI_PAIR 1
#endif
#ifndef TT_GEMM_BAL
#define TT_GEMM_BAL true
#endif

template <typename T, bool AKO, bool BKO, bool SHIFT, typename TO, int TBM, int TBN, int WGM, int WGN, bool DMA,
          bool A3 = false, bool BUF = false>
__global__ __launch_bounds__(64 * WGM * WGN) void gemm_kernel(GemmArgs g) {
  using ML = std::conditional_t<
      DMA,
      std::conditional_t<TBM == 256 && TBN == 256 && WGM == 2 && WGN == 4,
                         ttg::Loop8<T, AKO, BKO, TT_GEMM_BAL, A3, false, BUF>,
                         ttg::DLoop<T, AKO, BKO, TBM, TBN, WGM, WGN>>,
      ttg::MainLoop<T, AKO, BKO, TBM, TBN>>;
  static_assert(DMA || (TBM == 128 && TBN == 128 && WGM == 2 && WGN == 2), "register path is 128x128");
  constexpr int NT = 64 * WGM * WGN;
  constexpr int LDSB = ML::LDS_BYTES > 64 * (TBN + 4) * 4 ? ML::LDS_BYTES : 64 * (TBN + 4) * 4;
  __shared__ __attribute__((aligned(16))) char lds[LDSB];
  const int ntn = (g.N + TBN - 1) / TBN, ntm = (g.M + TBM - 1) / TBM;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int bs = id / (ntm * ntn), tile = id - bs * (ntm * ntn);
  const int mt = tile / ntn, nt = tile - mt * ntn;
  const int bi = bs / g.splits, s = bs - bi * g.splits;
  const int m0 = mt * TBM, n0 = nt * TBN;
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

  // 8-phase loop: a wave row whose 128 tile rows all lie past M skips its MFMAs (tail tiles)
  constexpr bool L8T = DMA && TBM == 256 && TBN == 256 && WGM == 2 && WGN == 4;
  const bool mm = !L8T || !TT_TAIL_SKIP || __builtin_amdgcn_readfirstlane((int)(m0 + (int)(threadIdx.x >> 8) * 128 < g.M));
  auto lrun = [&](const auto& la, const auto& lb) {
    if constexpr (L8T) ML::run(la, lb, g.K, kt0, kt1, lds, acc, mm);
    else ML::run(la, lb, g.K, kt0, kt1, lds, acc);
  };
  auto run = [&](const auto& la) {
    if constexpr (!BKO) {
      lrun(la, ttg::KCPlain<T>{B, g.ldb, n0, g.N});
    } else if constexpr (SHIFT) {
      lrun(la, ttg::KOShift<T>{B, g.ldb, n0, g.N - n0, g.seq_t, g.bshift[bi]});
    } else {
      lrun(la, ttg::KOPlain<T>{B, g.ldb, n0, g.N - n0});
    }
  };
  if constexpr (AKO) {
    ttg::KOPlain<T> la{A, g.lda, m0, g.M - m0};
    if (g.a_split > 0) {
      la.base1 = static_cast<const T*>(g.a_hi[bi]);
      la.csplit = g.a_split;
    }
    run(la);
  } else {
    run(ttg::KCPlain<T>{A, g.lda, m0, g.M});
  }

#ifdef TT_DIAG
  if (g.force_regstage == 9) {  // diagnostic build only: main loop without epilogue
    float sum = 0.f;  // every accumulator chain stays live (no MFMA is dead code)
#pragma unroll
    for (int i = 0; i < ML::TM; ++i)
#pragma unroll
      for (int j = 0; j < ML::TN; ++j) sum += acc[i][j][0] + acc[i][j][3];
    if (sum == 12345.f) static_cast<float*>(g.c[bi])[0] = 1.f;
    return;
  }
#endif
  // ---- epilogue: stage 64-row slices of the fp32 tile in LDS, then every thread
  // finishes 8 consecutive columns of a row and writes them with 16-byte stores.
  const bool partial = g.splits > 1;
  TO* C = partial ? nullptr : static_cast<TO*>(g.c[bi]);
  float* P = partial ? static_cast<float*>(g.c[bi]) + (long)s * g.part_stride : nullptr;
  const long ldc = partial ? (long)g.N : g.ldc;
  const float* bias = partial ? nullptr : g.bias[bi];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, tid = threadIdx.x;
  constexpr int WTM = TBM / WGM, WTN = TBN / WGN;
  const int wm = wave / WGN * WTM, wn = wave % WGN * WTN;
  constexpr int CLD = TBN + 4;
  constexpr int TPR = TBN / 8;          // threads per row
  constexpr int RPP = NT / TPR;         // rows per pass per sweep
  float* L = reinterpret_cast<float*>(lds);
  const int cg = (tid % TPR) * 8;
  const __amdgpu_buffer_rsrc_t crs = tt_rsrc(partial ? (const void*)P : (const void*)(C + (long)m0 * ldc + n0));
  float bv[8];  // this thread's 8 bias values (its columns are fixed)
#pragma unroll
  for (int e = 0; e < 8; ++e) bv[e] = 0.f;
  if (bias) {
    if (n0 + cg + 8 <= g.N && g.bias_vec_ok) ld8(bias + n0 + cg, bv);
    else
      for (int e = 0; e < 8; ++e)
        if (n0 + cg + e < g.N) bv[e] = bias[n0 + cg + e];
  }
  for (int hf = 0; hf < TBM / 64; ++hf) {
    if (wm <= hf * 64 && hf * 64 < wm + WTM) {
      const int i0 = (hf * 64 - wm) / 16;
#pragma unroll
      for (int i = 0; i < ML::TM; ++i)
        if (i >= i0 && i < i0 + 4)
#pragma unroll
          for (int j = 0; j < ML::TN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              L[(16 * (i - i0) + 4 * (lane >> 4) + r) * CLD + wn + 16 * j + (lane & 15)] = acc[i][j][r];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 64 / RPP; ++k) {
      const int rl = tid / TPR + RPP * k;
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
            float x = v[e] * g.alpha + bv[e];
            if (g.relu) x = fmaxf(x, 0.f);
            if (g.drop_thresh) x *= tt_dropout_scale(g.drop_seed, g.drop_row0 + (uint32_t)gm, gn + e, g.drop_thresh, g.drop_inv_keep);
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
            if (g.stream_out)
              st8_sc1(crs, (int)(((long)(gm - m0) * ldc + (gn - n0)) * (long)sizeof(TO)), v, (TO*)nullptr);
            else
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

// ---- direct epilogue of a 256x256 tile accumulated transposed (Loop8 CT) ----------
// The wave's 128 x 64 block sits at (wm, wn) and acc[i][j][r] = C(wm + 16i + (lane & 15),
// wn + 16j + 4 (lane >> 4) + r), so no LDS staging is needed: alpha / bias / relu /
// dropout in fp32, then
//   bf16: pack pairs and exchange column tiles j, j+1 with one v_permlane16_swap per
//         dword: lane group q then holds columns 16 (j + (q & 1)) + 8 (q >> 1) .. +7 of its
//         row, one 16-byte store per (i, j pair) -> 16 stores per wave;
//   fp32: each lane's 4 columns are one 16-byte store -> 32 stores per wave.
// A wave of a full tile (every row and column in range, vector-aligned C) issues exactly
// EPI_STORES<TO> stores, which the persistent kernel's next counted wait allows for.
template <typename TO>
constexpr int EPI_STORES = sizeof(TO) == 2 ? 16 : 32;

// MI/NI (>= 0): only the accumulator quadrant rows 4 MI..4 MI+3, column pair NI (the Loop8
// quad), for the persistent kernel's interleaved epilogue (PERSIST_IEPI); -1: the whole block.
template <typename TO, int MI = -1, int NI = -1>
TT_DEV void epi_direct(const GemmArgs& g, const f32x4 (&acc)[8][4], TO* C, const float* bias, int m0, int n0,
                       int wm, int wn, bool full) {
  constexpr int I0 = MI < 0 ? 0 : 4 * MI, I1 = MI < 0 ? 8 : 4 * MI + 4;
  constexpr int JP0 = NI < 0 ? 0 : NI, JP1 = NI < 0 ? 2 : NI + 1;
  const int lane = threadIdx.x & 63, q = lane >> 4, lr = lane & 15;
  float bv[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[j][e] = 0.f;
  if (bias) {
#pragma unroll
    for (int j = 2 * JP0; j < 2 * JP1; ++j) {
      const int c = n0 + wn + 16 * j + 4 * q;
      if (full && g.bias_vec_ok) {
        const float4 b4 = *reinterpret_cast<const float4*>(bias + c);
        bv[j][0] = b4.x; bv[j][1] = b4.y; bv[j][2] = b4.z; bv[j][3] = b4.w;
      } else {
        for (int e = 0; e < 4; ++e)
          if (c + e < g.N) bv[j][e] = bias[c + e];
      }
    }
  }
#ifdef TT_DIAG
  if (g.force_regstage == 9) {  // diagnostic build only: no stores (every accumulator stays live)
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) sum += acc[i][j][0] + acc[i][j][3] + bv[j][0];
    if (sum == 12345.f) C[0] = (TO)0;
    return;
  }
#endif
  const __amdgpu_buffer_rsrc_t crs = tt_rsrc(C + (long)m0 * g.ldc + n0);
  auto fin = [&](float x, float b, int gm, int gn) {
    x = x * g.alpha + b;
    if (g.relu) x = fmaxf(x, 0.f);
    if (g.drop_thresh) x *= tt_dropout_scale(g.drop_seed, g.drop_row0 + (uint32_t)gm, gn, g.drop_thresh, g.drop_inv_keep);
    return x;
  };
  auto put = [&](int gm, int gn, uint4 v) {
#ifdef TT_DIAG
    if (g.force_regstage == 10) {  // diagnostic: same stores into a 64-row (L2-resident) window
      *reinterpret_cast<uint4*>(C + (long)(gm & 63) * g.ldc + gn) = v;
      return;
    }
#endif
    const int off = (int)(((long)(gm - m0) * g.ldc + (gn - n0)) * (long)sizeof(TO));
    if (g.stream_out == 2) st16_buf_aux<2>(crs, off, v);
    else if (g.stream_out == 3) st16_buf_aux<17>(crs, off, v);
    else if (g.stream_out) st16_sc1(crs, off, v);
    else *reinterpret_cast<uint4*>(C + (long)gm * g.ldc + gn) = v;
  };
#pragma unroll
  for (int i = I0; i < I1; ++i) {
    const int gm = m0 + wm + 16 * i + lr;
    if constexpr (sizeof(TO) == 2) {
#if TT_EPI_PAIR
      if (NI < 0 && full) {  // whole 128-B lines: 8 rows per store instruction (row_pair)
        uint4 v[2];
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          uint32_t w[2][2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int j = 2 * jp + h, c = n0 + wn + 16 * j + 4 * q;
            float x[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) x[e] = fin(acc[i][j][e], bv[j][e], gm, c + e);
            w[h][0] = (uint32_t)f2bf(x[0]) | ((uint32_t)f2bf(x[1]) << 16);
            w[h][1] = (uint32_t)f2bf(x[2]) | ((uint32_t)f2bf(x[3]) << 16);
          }
          const auto s0 = __builtin_amdgcn_permlane16_swap(w[0][0], w[1][0], false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(w[0][1], w[1][1], false, false);
          v[jp] = make_uint4(s0[0], s1[0], s0[1], s1[1]);
        }
        uint4 da, db;
        row_pair(v[0], v[1], da, db);
        const int ra = m0 + wm + 16 * i + (lr & 7);
        const int cs = n0 + wn + 16 * (q & 1) + 8 * (q >> 1) + (lr & 8 ? 32 : 0);
        put(ra, cs, da);
        put(ra + 8, cs, db);
        continue;
      }
#endif
#pragma unroll
      for (int jp = JP0; jp < JP1; ++jp) {
        uint32_t w[2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int j = 2 * jp + h, c = n0 + wn + 16 * j + 4 * q;
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fin(acc[i][j][e], bv[j][e], gm, c + e);
          w[h][0] = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
          w[h][1] = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        }
        const auto s0 = __builtin_amdgcn_permlane16_swap(w[0][0], w[1][0], false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(w[0][1], w[1][1], false, false);
        const uint4 v = make_uint4(s0[0], s1[0], s0[1], s1[1]);
        const int cs = n0 + wn + 16 * (2 * jp + (q & 1)) + 8 * (q >> 1);
        if (full) {
          put(gm, cs, v);
        } else if (gm < g.M) {
          if (cs + 8 <= g.N && g.vec_ok) {
            put(gm, cs, v);
          } else {
            const uint32_t u[4] = {v.x, v.y, v.z, v.w};
            for (int e = 0; e < 8 && cs + e < g.N; ++e)
              Elt<TO>::st(C + (long)gm * g.ldc + cs + e, __uint_as_float(e & 1 ? u[e >> 1] & 0xFFFF0000u : u[e >> 1] << 16));
          }
        }
      }
    } else {
#pragma unroll
      for (int j = 2 * JP0; j < 2 * JP1; ++j) {
        const int c = n0 + wn + 16 * j + 4 * q;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fin(acc[i][j][e], bv[j][e], gm, c + e);
        const uint4 u = make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                                   __float_as_uint(v[3]));
        if (full) {
          put(gm, c, u);
        } else if (gm < g.M) {
          if (c + 4 <= g.N && g.vec_ok) put(gm, c, u);
          else
            for (int e = 0; e < 4 && c + e < g.N; ++e) Elt<TO>::st(C + (long)gm * g.ldc + c + e, v[e]);
        }
      }
    }
  }
}

// Quadrant epilogue of gemm_persist IE (interleaved): a full tile, alpha 1, bias, no relu /
// dropout, bf16 out; rows 4 MI..4 MI+3 of the wave block, column pair NI: bias, bf16 pairs,
// one v_permlane16_swap per dword, one 16-byte store per row block (write-through when sc1).
template <int MI, int NI>
TT_DEV void epi_quad_simple(const GemmArgs& g, const f32x4 (&acc)[8][4], bf16_t* C, const float* bias, int m0, int n0,
                            int wm, int wn) {
  const int lane = threadIdx.x & 63, q = lane >> 4, lr = lane & 15;
  float bv[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float4 b4 = bias ? *reinterpret_cast<const float4*>(bias + n0 + wn + 16 * (2 * NI + h) + 4 * q)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
    bv[h][0] = b4.x; bv[h][1] = b4.y; bv[h][2] = b4.z; bv[h][3] = b4.w;
  }
  const __amdgpu_buffer_rsrc_t crs = tt_rsrc(C + (long)m0 * g.ldc + n0);
  const int cs = wn + 16 * (2 * NI + (q & 1)) + 8 * (q >> 1);
#pragma unroll
  for (int i = 4 * MI; i < 4 * MI + 4; ++i) {
    uint32_t w[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x4 a = acc[i][2 * NI + h];
      w[h][0] = (uint32_t)f2bf(a[0] + bv[h][0]) | ((uint32_t)f2bf(a[1] + bv[h][1]) << 16);
      w[h][1] = (uint32_t)f2bf(a[2] + bv[h][2]) | ((uint32_t)f2bf(a[3] + bv[h][3]) << 16);
    }
    const auto s0 = __builtin_amdgcn_permlane16_swap(w[0][0], w[1][0], false, false);
    const auto s1 = __builtin_amdgcn_permlane16_swap(w[0][1], w[1][1], false, false);
    const uint4 v = make_uint4(s0[0], s1[0], s0[1], s1[1]);
    const int off = (int)(((long)(wm + 16 * i + lr) * g.ldc + cs) * 2L);
    if (g.stream_out == 2) st16_buf_aux<2>(crs, off, v);
    else if (g.stream_out) st16_sc1(crs, off, v);
    else st16_buf(crs, (uint32_t)off, 0, v);
  }
}

// ---- chunk-max epilogue of the hard-negative scan (gemm_persist HN) --------------------
// The wave's 128 x 64 block (CT: acc[i][j][r] = C(wm + 16i + (lane & 15), wn + 16j + 4q + r))
// is exactly one 64-column chunk of 128 query rows: per row the 16 lane-local values, then
// the maximum over the four lane groups q (v_permlane16/32_swap), so every lane holds its
// row's chunk maximum; lane group q stores rows i = 2q, 2q + 1 (2 stores per wave). Masked
// form (a tile holding a positive column or columns past N): the positive scores -1, columns
// past N -inf -- get_hard_negatives's sims[positive_idx] = -1 (enhanced_two_tower.py:130).
TT_DEV float rowgroup_max4(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
TT_DEV void epi_chunkmax(const GemmArgs& g, const f32x4 (&acc)[8][4], int m0, int n0, int wm, int wn) {
  const int lane = threadIdx.x & 63, q = lane >> 4, lr = lane & 15;
  const int c0 = n0 + wn;  // the wave's chunk starts here
  const bool masked = (g.label_off >= 0 && g.label_off + m0 + wm < c0 + 64 && c0 < g.label_off + m0 + wm + 128) ||
                      c0 + 64 > g.N;
  float mx[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float v[16];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[4 * j + r] = acc[i][j][r];
    if (masked) {
      const long lab = g.label_off >= 0 ? g.label_off + m0 + wm + 16 * i + lr : -1;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int col = c0 + 16 * j + 4 * q + r;
          if (col == lab) v[4 * j + r] = -1.f;
          if (col >= g.N) v[4 * j + r] = -FLT_MAX;
        }
    }
    float m = fmaxf(fmaxf(v[0], v[1]), v[2]);
#pragma unroll
    for (int e = 3; e < 15; e += 2) m = fmaxf(fmaxf(m, v[e]), v[e + 1]);
    mx[i] = rowgroup_max4(fmaxf(m, v[15]));
  }
  const long chunk = c0 / 64;
  if (chunk >= g.nch) return;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = 2 * q + u;
    float m = mx[0];
#pragma unroll
    for (int e = 1; e < 8; ++e) m = i == e ? mx[e] : m;
    const long row = (long)m0 + wm + 16 * i + lr;
    if (row < g.M) g.cm[row * g.nch + chunk] = m;
  }
}

// ---- B-resident short-K GEMM (the GRU's layer-0 input projection) ----------------------
// C_b[m][n] = A_b[m][:K] . B_b[n][:K] + bias_b[n], bf16 in and out, fp32 accumulation,
// K <= 384 and a multiple of 32, N a multiple of 192 (input_proj_l0: M = B*T, N = 6H =
// 3072, K = Ep = 320). The persistent 256x256 GEMM spends most of such a tile outside
// the MFMAs -- 5 K-tiles of products, then an epilogue whose 128 KiB of stores do not
// overlap them -- because all 8 waves of a tile meet at every barrier.
// Here each workgroup keeps one 192-column panel of B (K x 192 bf16, <= 144 KiB) in LDS
// for the whole launch, and its 8 waves walk 32-row A tiles INDEPENDENTLY: A fragments
// come straight from global memory (16 bytes per lane, NKS/2 k-steps ahead, across tile
// boundaries), so the main loop has no barrier at all and one wave's epilogue stores run
// beside the other waves' MFMAs. The 8 XCD-local groups of workgroups (one per M range)
// cover all panels, so each A row is fetched into an XCD's L2 once and read by the 16
// (or 32) panels' workgroups. Same MFMA (16x16x32, B fragment first: the transposed
// accumulate of the persistent kernel), same k order from zero: bit-identical to it.
#ifndef BRES_DIAG  // timing-only diagnostic switches of gemm_bres (results wrong): 1 no output stores
#define BRES_DIAG 0
#endif
#ifndef BRES_STORE  // output store policy of gemm_bres: 0 plain, 1 write-through (sc1), 2 non-temporal
#define BRES_STORE 0
#endif
#ifndef BRES_PD  // gemm_bres A prefetch: 1 a whole tile ahead, 0 half a tile
#define BRES_PD 1
#endif
#ifndef BRES_STAG  // waves 4-7 start BRES_STAG x 64 cycles late (0: together)
#define BRES_STAG 0
#endif
constexpr int BR_COLS = 192;  // B panel columns per workgroup
// RB: 16-row blocks per wave tile. RB 2 (32-row tiles, 8 waves): every 16-byte B fragment
// read from LDS feeds 2 MFMAs, so the LDS read port (128 B/clk per CU) needs twice the
// matrix pipe's time -- with neither stores nor A loads the kernel still took 1.60 ms per
// step against 0.82 for its MFMAs alone (profiles/r05_bres_diag.txt). RB 4 (64-row tiles,
// 4 waves of up to 512 registers, option bres_rows 64): each fragment feeds 4 MFMAs. Same
// MFMAs per output element in the same k order either way: bit-identical.
template <int NKS, int RB = 2>  // k-steps of 32
__global__ __launch_bounds__(RB == 2 ? 512 : 256, 1) void gemm_bres(GemmArgs g, int npan, int nbatch) {
  static_assert(RB == 2 || RB == 4, "32- or 64-row wave tiles");
  constexpr int NW = RB == 2 ? 8 : 4;  // waves
  constexpr int NT = 64 * NW;
  constexpr int TR = 16 * RB;          // rows per wave tile
  constexpr int NKT = (NKS + 1) / 2;  // 64-deep K-tile images
  constexpr int IMG = BR_COLS * ttg::KTB;
  // A prefetch depth in k-steps (divides NKS); BRES_PD 1: a whole tile, so that the next
  // tile's fragments are all requested before this tile's stores (one in-order vmcnt)
  constexpr int PD = ((BRES_PD && NKS * RB <= 20) || NKS % 2 != 0) ? NKS : NKS / 2;  // (NKS 12: 20 spills)
  __shared__ __attribute__((aligned(16))) char lds[NKT * IMG + BR_COLS * 4];
  float* bias_s = reinterpret_cast<float*>(lds + NKT * IMG);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // workgroup -> (row group gi, batch entry bi, panel): consecutive ids (one XCD's run)
  // share a row group, so its A rows are read into that L2 once for all panels
  const int ptot = npan * nbatch;
  const int bid = ttg::xcd_remap(blockIdx.x, gridDim.x);
  const int ngrp = gridDim.x / ptot;
  const int gi = bid / ptot, p = bid % ptot;
  const int bi = p / npan, n0 = (p % npan) * BR_COLS;
  const bf16_t* A = static_cast<const bf16_t*>(g.a[bi]);
  const bf16_t* Bm = static_cast<const bf16_t*>(g.b[bi]);
  bf16_t* C = static_cast<bf16_t*>(g.c[bi]);
  const float* bias = g.bias[bi];
  // the panel of B -> K-tile images (rows of 128 B, kc_off swizzle), zero past K; bias -> LDS
  for (int id = tid; id < NKT * BR_COLS * 8; id += NT) {
    const int kt = id / (BR_COLS * 8), rem = id % (BR_COLS * 8), row = rem >> 3, c = rem & 7;
    const int k = kt * 64 + c * 8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (k < g.K) v = *reinterpret_cast<const uint4*>(Bm + (long)(n0 + row) * g.ldb + k);
    *reinterpret_cast<uint4*>(lds + kt * IMG + ttg::kc_off(row, c)) = v;
  }
  for (int c = tid; c < BR_COLS; c += NT) bias_s[c] = bias ? bias[n0 + c] : 0.f;
  __syncthreads();
  // this group's rows, in TR-row tiles dealt to the waves round-robin
  const int mg = ((g.M + ngrp - 1) / ngrp + TR - 1) / TR * TR;
  const int g0 = gi * mg;
  const int ntl = max(0, min(mg, g.M - g0) + TR - 1) / TR;
  const __amdgpu_buffer_rsrc_t ra = tt_rsrc_n(A + (long)g0 * g.lda, g0 < g.M);
  const int lr = lane & 15, q = lane >> 4;
  // A fragment of (tile t, k-step ks, row block rb): rows past M read zero (offset past the
  // resource's range)
  auto lda_frag = [&](int t, int ks, int rb) {
    const int row = t * TR + rb * 16 + lr;
    const uint32_t off = t < ntl && g0 + row < g.M ? (uint32_t)((row * (int)g.lda + ks * 32 + q * 8) * 2) : 0x80000000u;
    return ld16_buf(ra, off, 0);
  };
  if (BRES_STAG > 0 && wave >= NW / 2) __builtin_amdgcn_s_sleep(BRES_STAG);
  if (TT_PRIO_HALF && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  uint4 ar[PD][RB];
  int t = wave;
#pragma unroll
  for (int i = 0; i < PD; ++i)
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) ar[i][rb] = lda_frag(t, i, rb);
  for (; t < ntl; t += NW) {
    f32x4 acc[RB][BR_COLS / 16];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int j = 0; j < BR_COLS / 16; ++j) acc[rb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      uint4 a[RB];
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) a[rb] = ar[ks % PD][rb];
      // refill the slot: k-step ks + PD of this tile, or of the wave's next tile
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
        ar[ks % PD][rb] = ks + PD < NKS ? lda_frag(t, ks + PD, rb) : lda_frag(t + NW, ks + PD - NKS, rb);
      const char* img = lds + (ks >> 1) * IMG;
#pragma unroll
      for (int j = 0; j < BR_COLS / 16; ++j) {
        const uint4 fb = ttg::frag<bf16_t, false>(img, 16 * j, ks & 1);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb][j] = ttg::mma<bf16_t>(fb, a[rb], acc[rb][j]);
      }
      // one k-step per scheduling region: hipcc would otherwise hoist every B fragment
      // read of the tile ahead of the MFMAs (and spill)
      __builtin_amdgcn_sched_barrier(0);
    }
    // epilogue: acc[rb][j][e] = C(row TR t + 16rb + lr, col 16j + 4q + e); bias, bf16, pairs of
    // column tiles exchanged (v_permlane16_swap) into 16-byte row stores
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int row = t * TR + rb * 16 + lr;
      const bool ok = g0 + row < g.M;
#pragma unroll
      for (int jp = 0; jp < BR_COLS / 32; ++jp) {
        uint32_t w[2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int j = 2 * jp + h;
          const float4 b4 = *reinterpret_cast<const float4*>(bias_s + 16 * j + 4 * q);
          const float v0 = acc[rb][j][0] + b4.x, v1 = acc[rb][j][1] + b4.y;
          const float v2 = acc[rb][j][2] + b4.z, v3 = acc[rb][j][3] + b4.w;
          w[h][0] = (uint32_t)f2bf(v0) | ((uint32_t)f2bf(v1) << 16);
          w[h][1] = (uint32_t)f2bf(v2) | ((uint32_t)f2bf(v3) << 16);
        }
        const auto s0 = __builtin_amdgcn_permlane16_swap(w[0][0], w[1][0], false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(w[0][1], w[1][1], false, false);
        const int cs = n0 + 16 * (2 * jp + (q & 1)) + 8 * (q >> 1);
#if BRES_DIAG & 1  // timing only: no stores (the packed values stay live)
        asm volatile("" ::"v"(s0[0]), "v"(s1[0]), "v"(s0[1]), "v"(s1[1]), "v"(ok));
#else
        if (ok) {
          const uint4 v = make_uint4(s0[0], s1[0], s0[1], s1[1]);
          if constexpr (BRES_STORE == 0) {
            *reinterpret_cast<uint4*>(C + (long)(g0 + row) * g.ldc + cs) = v;
          } else {
            const __amdgpu_buffer_rsrc_t rc = tt_rsrc(C + (long)g0 * g.ldc);
            st16_buf_aux<BRES_STORE == 1 ? 16 : 2>(rc, (int)(((long)row * g.ldc + cs) * 2), v);
          }
        }
#endif
      }
    }
  }
}

// ---- persistent 256x256 GEMM: one workgroup per CU walks tiles w, w+nwg, ... and the
// 8-phase K-tile stream runs straight across tile boundaries: the last K-tiles of tile
// i prefetch the first K-tiles of tile i+nwg (their pieces re-resolved on the fly), so
// tile i's epilogue (32-row LDS passes, separate 32 KiB) runs while tile i+nwg's first
// half-tiles land. No split-K, no accumulate-into-C (those use gemm_kernel).
// A3 (default): A prefetched two K-tiles ahead through a 3-slot ring (Loop8 A3 layout,
// 160 KiB), the product accumulated transposed and stored by epi_direct straight from
// registers: no LDS and no barrier between tiles, so the K-tile stream never pauses; the
// first counted wait of the next tile lets the epilogue's stores stay in flight. Measured
// before this: the LDS-staged epilogue plus its barriers cost ~20k cycles per tile, more
// than the 5 K-tiles of MFMAs of input_proj_l0.
template <typename T, bool AKO, bool BKO, bool SHIFT, typename TO, bool A3, bool BUF = false, bool HN = false,
          bool IE = false>
__global__ __launch_bounds__(512) void gemm_persist(GemmArgs g, int ntiles) {
  static_assert(!HN || (A3 && !AKO && !BKO && !SHIFT), "the scan epilogue runs on the A3 direct-epilogue form");
  using L8 = ttg::Loop8<T, AKO, BKO, false, A3, A3, BUF>;  // A3: transposed accumulate, direct epilogue
  using Piece = typename L8::Piece;
  constexpr int STG = A3 ? 0 : 32 * 256 * 4;
  static_assert(!A3 || 2 * L8::HALF >= 32 * 256 * 4, "staging fits an A slot");
  __shared__ __attribute__((aligned(16))) char lds[L8::LDS_BYTES + STG];
  float* stg = reinterpret_cast<float*>(lds + L8::LDS_BYTES);  // !A3 only
  const int nwg = gridDim.x;
  const int w = xcd_remap(blockIdx.x, nwg);
  if (w >= ntiles) return;
  // Tile walk. Default: tile q = w, w + nwg, ... (n-tile fastest), so at any time an XCD's
  // 32 workgroups cover ~3 row panels x ALL column panels: every B panel is re-fetched from
  // the Infinity Cache once per row panel when B exceeds the XCD's L2 (input_proj_l1: W_ih
  // 6 MiB per tower). g.order (option gemm_order, when nwg = 256, 256 | ntiles and 4 | ntn):
  // tiles are grouped in units of 4 column panels x 1 row panel, units ordered column group
  // first, and XCD x walks its own contiguous eighth of them 32 at a time -- 8 row panels x
  // the same 4 column panels per round, so 4 B panels (2 MiB at K 1024) stay in its L2.
  // Both walks are one formula (host-set g.walk_g / g.walk_x; 0 = the default walk): tile
  // q = ((group * nbatch + bi) * ntm + mt) * G + j covers column panel group * G + j, and the
  // workgroups are split into X equal sets that walk consecutive spans of q.
  const int G = g.walk_g > 0 ? g.walk_g : (g.N + 255) / 256;
  const int X = g.walk_x > 0 ? g.walk_x : 1;
  const int P = nwg / X, span = ntiles / X;
  const int qbeg = (w / P) * span + w % P;
  const int qstep = P;
  const int qend = (w / P + 1) * span;
  // optional start skew: workgroups in four phases, so the tiles' output bursts (all CUs
  // finish a tile at about the same time otherwise) spread over the tile period
  for (int i = 0; i < (w & 3) * g.skew; ++i) __builtin_amdgcn_s_sleep(64);
  const int ntn = (g.N + 255) / 256, ntm = (g.M + 255) / 256;
  const int nk = (g.K * (int)sizeof(T) + ttg::KTB - 1) / ttg::KTB;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, tid = threadIdx.x;
  const int wr = wave >> 2, bh = (wave & 3) >> 1, bc = (wave & 1) * 64;
  const int wm = wr * 128, wn = (wave & 3) * 64;
  const uint32_t base = __builtin_amdgcn_readfirstlane(ttg::lds_addr_of(lds));

  struct TileId { int bi, m0, n0; };
  auto decode = [&](int q) {
    TileId t;
    const int u = q / G, per = g.nbatch * ntm;
    const int gr = u / per, rr = u - gr * per;
    t.bi = rr / ntm;
    t.m0 = (rr - t.bi * ntm) * 256;
    t.n0 = (gr * G + (q - u * G)) * 256;
    return t;
  };
  // A / B loaders of tile q (q >= ntiles: a loader whose pieces are all out of range)
  auto loader_a = [&](int q) {
    const TileId t = decode(q < qend ? q : 0);
    const T* A = static_cast<const T*>(g.a[t.bi]);
    if constexpr (AKO) {
      ttg::KOPlain<T> la{A, g.lda, t.m0, q < qend ? g.M - t.m0 : 0};
      if (g.a_split > 0) {
        la.base1 = static_cast<const T*>(g.a_hi[t.bi]);
        la.csplit = g.a_split;
      }
      return la;
    } else {
      return ttg::KCPlain<T>{A, g.lda, t.m0, q < qend ? g.M : t.m0};
    }
  };
  auto loader_b = [&](int q) {
    const TileId t = decode(q < qend ? q : 0);
    const T* B = static_cast<const T*>(g.b[t.bi]);
    if constexpr (!BKO) {
      return ttg::KCPlain<T>{B, g.ldb, t.n0, q < qend ? g.N : t.n0};
    } else if constexpr (SHIFT) {
      return ttg::KOShift<T>{B, g.ldb, t.n0, q < qend ? g.N - t.n0 : 0, g.seq_t, g.bshift[t.bi]};
    } else {
      return ttg::KOPlain<T>{B, g.ldb, t.n0, q < qend ? g.N - t.n0 : 0};
    }
  };
#ifdef TT_DIAG
  if constexpr (A3) {
    if (g.force_regstage == 11) {  // diagnostic build only: the epilogue stores alone, no K loop
      f32x4 acc[8][4];
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{(float)i, (float)j, 1.f, 2.f};
      for (int q = qbeg; q < qend; q += qstep) {
        const TileId t = decode(q);
        const bool full = t.m0 + 256 <= g.M && t.n0 + 256 <= g.N && g.vec_ok;
        epi_direct<TO>(g, acc, static_cast<TO*>(g.c[t.bi]), g.bias[t.bi], t.m0, t.n0, wm, wn, full);
      }
      return;
    }
  }
#endif
  auto la = loader_a(qbeg);
  auto lb = loader_b(qbeg);
  typename L8::template Half<AKO, decltype(la)> pa0, pa1;
  typename L8::template Half<BKO, decltype(lb)> pb0, pb1;
  pa0.init(la, 0, nk, g.K, 0);
  pa1.init(la, 0, nk, g.K, 128);
  pb0.init(lb, 0, nk, g.K, 0);
  pb1.init(lb, 0, nk, g.K, 128);
  if constexpr (A3) {
    pa0.issue(0, base);
    pa1.issue(0, base + L8::HALF);
    pb0.issue(0, base + L8::BOFF);
    pb1.issue(0, base + L8::BOFF + L8::HALF);
    pa0.issue(1, base + 2 * L8::HALF);
    pa1.issue(1, base + 3 * L8::HALF);
    pb0.issue(1, base + L8::BOFF + 2 * L8::HALF);
    pb1.issue(1, base + L8::BOFF + 3 * L8::HALF);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    pa0.issue(0, base);
    pa1.issue(0, base + L8::HALF);
    pb0.issue(0, base + 2 * L8::HALF);
    pb1.issue(0, base + 3 * L8::HALF);
    pb0.issue(1, base + L8::SLOT + 2 * L8::HALF);
    pb1.issue(1, base + L8::SLOT + 3 * L8::HALF);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  const bool late = __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256;  // wave row 1
  if (TT_PRIO_HALF && late) __builtin_amdgcn_s_setprio(1);
  if (late) __builtin_amdgcn_s_barrier();

  int git = 0;  // running K-tile index of the stream (slot parity)
  int as = 0;   // A3: A slot of the stream's current K-tile (git mod 3)
  int ra_off = 0, rb_off = 0;  // K-tile index of the A / B pieces' tile start in this tile's terms
  bool epi_full = false;       // A3: the previous tile's epilogue issued EPI_STORES<TO> stores per wave
  // IEPI: the epilogue of tile i runs inside the first K-tile of tile i + 1, each accumulator
  // quadrant just before the phase whose MFMAs first overwrite it (the quad order (0,0),
  // (0,1), (1,1), (1,0)), so one wave row's epilogue arithmetic and stores overlap the other
  // row's MFMAs instead of all 8 waves leaving the matrix pipe idle between tiles; the last
  // quadrant's stores follow K-tile 2's DMAs and may stay in flight into K-tile 1's wait
  constexpr bool IEPI = IE && A3 && !HN && PERSIST_BAL && std::is_same<TO, bf16_t>::value;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  TileId prev_t{0, 0, 0};
  bool have_prev = false;
  // the quadrant's epilogue of the previous tile, then its accumulators cleared
  auto iepi = [&](auto mi_c, auto ni_c) {
    constexpr int MI = decltype(mi_c)::value, NI = decltype(ni_c)::value;
    if constexpr (IEPI)
      epi_quad_simple<MI, NI>(g, acc, static_cast<bf16_t*>(g.c[prev_t.bi]), g.bias[prev_t.bi], prev_t.m0, prev_t.n0,
                              wm, wn);
#pragma unroll
    for (int i = 4 * MI; i < 4 * MI + 4; ++i)
#pragma unroll
      for (int j = 2 * NI; j < 2 * NI + 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  for (int q = qbeg; q < qend; q += qstep) {
    const int qn = q + qstep;
    const TileId cur_t = decode(q);
    if constexpr (!IEPI) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    uint4 fa[2][4], fb[2][4];
    if constexpr (A3) {
      for (int r = 0; r < nk; ++r, ++git) {
        const bool ep = IEPI && r == 0 && have_prev;  // wave-uniform
        const int an = as == 0 ? 2 : as - 1;  // slot of K-tile r+2 = slot of r-1
        const int bs = git & 1;
        const char* ia = lds + as * (2 * L8::HALF) + wr * L8::HALF;
        const char* ib = lds + L8::BOFF + bs * (2 * L8::HALF) + bh * L8::HALF;
        const uint32_t anx = base + (uint32_t)an * (2 * L8::HALF);
        const uint32_t bcur = base + L8::BOFF + (uint32_t)bs * (2 * L8::HALF);
        // the stream's A and B K-tile r+2 belong to tile qn once r + 2 == nk
        if (r + 2 == nk) {
          la = loader_a(qn);
          pa0.init(la, 0, nk, g.K, 0);
          pa1.init(la, 0, nk, g.K, 128);
          ra_off = nk;
        }
#if PERSIST_BAL
        // balanced fragment reads (the run3 schedule): P1 A rows 0-63 + B columns 0-31 (12
        // reads), P2 B columns 32-63 (4), P3 A rows 64-127 (8); B is last read in P2, so both
        // B halves of K-tile r+2 are restaged in P4, two phases later
        // (IEPI: each quadrant's epilogue before the phase's fragment reads, when the fewest
        // fragment registers are live)
        if constexpr (IEPI)
          if (ep) iepi(C0{}, C0{});
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
          for (int i = 0; i < 4; ++i) fa[ks][i] = ttg::frag2<T, AKO>(ia, 16 * i, ks);
#pragma unroll
          for (int j = 0; j < 2; ++j) fb[ks][j] = ttg::frag2<T, BKO>(ib, bc + 16 * j, ks);
        }
        pa0.issue(r + 2 - ra_off, anx);
        L8::quad(0, 0, fa, fb, acc);
        if constexpr (IEPI)
          if (ep) iepi(C0{}, C1{});
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int j = 2; j < 4; ++j) fb[ks][j] = ttg::frag2<T, BKO>(ib, bc + 16 * j, ks);
        pa1.issue(r + 2 - ra_off, anx + L8::HALF);
        L8::quad(0, 1, fa, fb, acc);
        if constexpr (IEPI)
          if (ep) iepi(C1{}, C1{});
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < 4; ++i) fa[ks][i] = ttg::frag2<T, AKO>(ia, 64 + 16 * i, ks);
        L8::quad(1, 1, fa, fb, acc);
        if (r + 2 == nk) {
          lb = loader_b(qn);
          pb0.init(lb, 0, nk, g.K, 0);
          pb1.init(lb, 0, nk, g.K, 128);
          rb_off = nk;
        }
        pb0.issue(r + 2 - rb_off, bcur);
        pb1.issue(r + 2 - rb_off, bcur + L8::HALF);
        if constexpr (IEPI)
          if (ep) iepi(C1{}, C0{});
#else
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
          for (int i = 0; i < 4; ++i) fa[ks][i] = ttg::frag2<T, AKO>(ia, 16 * i, ks);
#pragma unroll
          for (int j = 0; j < 4; ++j) fb[ks][j] = ttg::frag2<T, BKO>(ib, bc + 16 * j, ks);
        }
        pa0.issue(r + 2 - ra_off, anx);
        L8::quad(0, 0, fa, fb, acc);
        pa1.issue(r + 2 - ra_off, anx + L8::HALF);
        L8::quad(0, 1, fa, fb, acc);
        if (r + 2 == nk) {
          lb = loader_b(qn);
          pb0.init(lb, 0, nk, g.K, 0);
          pb1.init(lb, 0, nk, g.K, 128);
          rb_off = nk;
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < 4; ++i) fa[ks][i] = ttg::frag2<T, AKO>(ia, 64 + 16 * i, ks);
        pb0.issue(r + 2 - rb_off, bcur);
        L8::quad(1, 1, fa, fb, acc);
        pb1.issue(r + 2 - rb_off, bcur + L8::HALF);
#endif
        // K-tile r+1 landed; the 8 DMAs of r+2 stay in flight, and at r = 0 also the
        // previous tile's epilogue stores (issued after r+1's DMAs, before r+2's)
#ifdef TT_DIAG
        const bool loose = g.force_regstage == 12 && r < 3 && epi_full;  // timing only: stores never waited for
#else
        constexpr bool loose = false;
#endif
        if constexpr (HN) {
          // the scan's 2 chunk-max stores of the previous tile stay in flight at r = 0
          if (r == 0 && epi_full) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else if (IEPI) {
          // r = 0: the previous tile's stores (all quadrants, EPI_STORES) and K-tile 2's 8 DMAs
          // are younger than K-tile 1; r = 1: only quadrant (1,0)'s stores (a quarter) and
          // K-tile 3's DMAs are younger than K-tile 2. A partial previous tile issued fewer
          // stores: vmcnt(8) then waits for more than needed, never less
          if (r == 0 && epi_full) {
            if constexpr (EPI_STORES<TO> == 16) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
          } else if (r == 1 && epi_full) {
            if constexpr (EPI_STORES<TO> == 16) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
          } else {
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
          }
        } else if ((r == 0 && epi_full) || loose) {
          if constexpr (EPI_STORES<TO> == 16) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        }
        L8::quad(1, 0, fa, fb, acc);
        as = as == 2 ? 0 : as + 1;
      }
      ra_off -= nk;
      rb_off -= nk;
      // epilogue straight from the accumulators: no LDS, no barrier, so the K-tile stream
      // (and the two wave rows' one-barrier stagger) runs on into tile qn unchanged
      if constexpr (HN) {
        epi_chunkmax(g, acc, cur_t.m0, cur_t.n0, wm, wn);
        // 2 stores per wave unless the wave's chunk or rows lie wholly past the ends
        epi_full = __builtin_amdgcn_readfirstlane((int)(cur_t.m0 + 256 <= g.M && cur_t.n0 + 256 <= 64 * g.nch)) != 0;
        continue;
      }
      const bool full = cur_t.m0 + 256 <= g.M && cur_t.n0 + 256 <= g.N && g.vec_ok;
      if constexpr (IEPI) {  // the epilogue runs in the next tile's first K-tile (or after the loop)
        prev_t = cur_t;
        have_prev = true;
        epi_full = __builtin_amdgcn_readfirstlane((int)full) != 0;
        continue;
      }
      epi_direct<TO>(g, acc, static_cast<TO*>(g.c[cur_t.bi]), g.bias[cur_t.bi], cur_t.m0, cur_t.n0, wm, wn, full);
      epi_full = __builtin_amdgcn_readfirstlane((int)full) != 0;
      continue;
    }
    for (int r = 0; r < (A3 ? 0 : nk); ++r, ++git) {
      const int cs = git & 1;
      const uint32_t cur = base + cs * L8::SLOT, nxt = base + (cs ^ 1) * L8::SLOT;
      const char* ia = lds + cs * L8::SLOT + wr * L8::HALF;
      const char* ib = lds + cs * L8::SLOT + (2 + bh) * L8::HALF;
      // the stream's next A K-tile belongs to tile qn once r + 1 == nk
      if (r + 1 == nk) {
        la = loader_a(qn);
        pa0.init(la, 0, nk, g.K, 0);
        pa1.init(la, 0, nk, g.K, 128);
        ra_off = nk;
      }
      // P1
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[ks][i] = ttg::frag2<T, AKO>(ia, 16 * i, ks);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[ks][j] = ttg::frag2<T, BKO>(ib, bc + 16 * j, ks);
      }
      pa0.issue(r + 1 - ra_off, nxt);
      L8::quad(0, 0, fa, fb, acc);
      // P2
      pa1.issue(r + 1 - ra_off, nxt + L8::HALF);
      L8::quad(0, 1, fa, fb, acc);
      // P3: the stream's B K-tile r+2 belongs to tile qn once r + 2 == nk
      if (r + 2 == nk) {
        lb = loader_b(qn);
        pb0.init(lb, 0, nk, g.K, 0);
        pb1.init(lb, 0, nk, g.K, 128);
        rb_off = nk;
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[ks][i] = ttg::frag2<T, AKO>(ia, 64 + 16 * i, ks);
      pb0.issue(r + 2 - rb_off, cur + 2 * L8::HALF);
      L8::quad(1, 1, fa, fb, acc);
      // P4
      pb1.issue(r + 2 - rb_off, cur + 3 * L8::HALF);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      L8::quad(1, 0, fa, fb, acc);
    }
    ra_off -= nk;
    rb_off -= nk;
    if (!late) __builtin_amdgcn_s_barrier();  // re-align the two wave rows

    // ---- epilogue: 8 passes of 32 rows through the separate staging area
    TO* C = static_cast<TO*>(g.c[cur_t.bi]);
    const float* bias = g.bias[cur_t.bi];
    const int m0 = cur_t.m0, n0 = cur_t.n0;
    const int cg = (tid & 31) * 8, rlo = tid >> 5;  // 8 columns, rows rlo and rlo + 16
    float bv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[e] = 0.f;
    if (bias) {
      if (n0 + cg + 8 <= g.N && g.bias_vec_ok) ld8(bias + n0 + cg, bv);
      else
        for (int e = 0; e < 8; ++e)
          if (n0 + cg + e < g.N) bv[e] = bias[n0 + cg + e];
    }
    const __amdgpu_buffer_rsrc_t crs = tt_rsrc(C + (long)m0 * g.ldc + n0);
    for (int p = 0; p < 8; ++p) {
      const int i0 = (p * 32 - wm) / 16;  // this wave's accumulator rows in the pass
      if (p * 32 >= wm && p * 32 < wm + 128) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (i >= i0 && i < i0 + 2)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
              for (int rr = 0; rr < 4; ++rr)
                stg[(16 * (i - i0) + 4 * (lane >> 4) + rr) * 256 + wn + 16 * j + (lane & 15)] = acc[i][j][rr];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int rl = rlo + 16 * k;
        const int gm = m0 + p * 32 + rl, gn = n0 + cg;
        if (gm < g.M && gn < g.N) {
          float v[8];
          const float4 x0 = *reinterpret_cast<const float4*>(stg + rl * 256 + cg);
          const float4 x1 = *reinterpret_cast<const float4*>(stg + rl * 256 + cg + 4);
          v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w; v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float x = v[e] * g.alpha + bv[e];
            if (g.relu) x = fmaxf(x, 0.f);
            if (g.drop_thresh) x *= tt_dropout_scale(g.drop_seed, g.drop_row0 + (uint32_t)gm, gn + e, g.drop_thresh, g.drop_inv_keep);
            v[e] = x;
          }
          TO* dst = C + (long)gm * g.ldc + gn;
          if (gn + 8 <= g.N && g.vec_ok) {
            if (g.stream_out)
              st8_sc1(crs, (int)(((long)(gm - m0) * g.ldc + (gn - n0)) * (long)sizeof(TO)), v, (TO*)nullptr);
            else
              st8(dst, v);
          } else {
            for (int e = 0; e < 8 && gn + e < g.N; ++e) Elt<TO>::st(dst + e, v[e]);
          }
        }
      }
      __builtin_amdgcn_s_barrier();  // staging free for the next pass
    }
    if (late && qn < qend) __builtin_amdgcn_s_barrier();  // re-stagger for the next tile
  }
  if constexpr (IE && A3 && !HN && PERSIST_BAL && std::is_same<TO, bf16_t>::value) {  // the last tile's epilogue
    if (have_prev) {
      iepi(C0{}, C0{});
      iepi(C0{}, C1{});
      iepi(C1{}, C1{});
      iepi(C1{}, C0{});
    }
  }
  if constexpr (A3)
    if (!late) __builtin_amdgcn_s_barrier();  // the late row's extra prologue barrier
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // trailing zero-page DMAs land before exit
}

// out_b[m][n] = alpha * sum_s part_b[s][m][n] (+ bias[n]) (+ out_b); V consecutive elements
// of one row per thread (V 4: N % 4 == 0, 16-byte partial loads), the slices summed in order
// s = 0, 1, ... either way
template <typename TO, int V>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* ws, long part_stride, int splits,
                                                            int M, int N, GemmArgs g) {
  const int bi = blockIdx.y;
  const float* P = ws + (long)bi * splits * part_stride;
  TO* C = static_cast<TO*>(g.c[bi]);
  const float* bias = g.bias[bi];
  const long total = (long)M * N / V;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    float v[V];
    if constexpr (V == 4) {
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int s = 0; s < splits; ++s) {
        const float4 b = reinterpret_cast<const float4*>(P + (long)s * part_stride)[e];
        a.x += b.x;
        a.y += b.y;
        a.z += b.z;
        a.w += b.w;
      }
      v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w;
    } else {
      v[0] = 0.f;
      for (int s = 0; s < splits; ++s) v[0] += P[(long)s * part_stride + e];
    }
    const int m = (int)(e * V / N), n0 = (int)(e * V % N);
#pragma unroll
    for (int u = 0; u < V; ++u) {
      float x = v[u] * g.alpha;
      if (bias) x += bias[n0 + u];
      TO* p = C + (long)m * g.ldc + n0 + u;
      if (g.beta) x += Elt<TO>::ld(p);
      Elt<TO>::st(p, x);
    }
  }
}

template <typename T, typename TO, int TBM, int TBN, int WGM, int WGN, bool DMA, bool A3 = false, bool BUF = false>
int launch_t(int akout, int bkout, bool shift, const GemmArgs& g, long nwg, hipStream_t st) {
  dim3 grid((unsigned)nwg), blk(64 * WGM * WGN);
#define TT_L(AK, BK, SH) \
  hipLaunchKernelGGL((gemm_kernel<T, AK, BK, SH, TO, TBM, TBN, WGM, WGN, DMA, A3, BUF>), grid, blk, 0, st, g)
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

// 256x256 tiles (8 waves) for problems with enough tiles to fill the chip, else
// 128x128 (4 waves); register staging only when a chunk can straddle a boundary.
inline bool use_big(int m, int n, long tiles256) { return m >= 256 && n >= 256 && tiles256 >= 256; }

template <typename T, typename TO>
int launch_persist(int akout, int bkout, bool shift, const GemmArgs& g0, int ntiles, bool buf, hipStream_t st) {
  dim3 grid((unsigned)std::min(ntiles, 256)), blk(512);
  // option gemm_order: column groups of 4 panels per XCD (each XCD's 32 workgroups walk
  // their own eighth of the tiles: 8 row panels x the same 4 column panels per round, so
  // those B panels stay in the XCD's L2); needs 256 workgroups, 256 | tiles, 4 | column panels
  GemmArgs g = g0;
  g.walk_g = g.walk_x = 0;
  if (tt::opt(tt::OPT_GEMM_ORDER) && ntiles % 256 == 0 && ((g.N + 255) / 256) % 4 == 0) {
    g.walk_g = 4;
    g.walk_x = 8;
  }
#define TT_L(AK, BK, SH, A3, BUF) \
  hipLaunchKernelGGL((gemm_persist<T, AK, BK, SH, TO, A3, BUF>), grid, blk, 0, st, g, ntiles)
#define TT_L2(AK, BK, SH) \
  do {                     \
    if (a3 && buf) TT_L(AK, BK, SH, true, true); \
    else if (a3) TT_L(AK, BK, SH, true, false); \
    else TT_L(AK, BK, SH, false, false);   \
  } while (0)
  const bool a3 = tt::opt(tt::OPT_GEMM_A3) != 0;
  // interleaved epilogue (gemm_persist IE): NT, bf16 out, full tiles, alpha 1, bias only
  if constexpr (std::is_same<TO, bf16_t>::value) {
    if (PERSIST_IEPI && tt::opt(tt::OPT_GEMM_IEPI) && !akout && !bkout && !shift && a3 && buf && g.M % 256 == 0 &&
        g.N % 256 == 0 && g.vec_ok && g.bias_vec_ok && g.alpha == 1.f && !g.relu && !g.drop_thresh && !g.beta &&
        g.stream_out <= 2 && g.force_regstage == 0) {
      hipLaunchKernelGGL((gemm_persist<T, false, false, false, TO, true, true, false, true>), grid, blk, 0, st, g, ntiles);
      TT_CHECK_LAUNCH("gemm_persist");
      return 0;
    }
  }
  if (!akout && !bkout) TT_L2(false, false, false);
  else if (!akout && bkout && !shift) TT_L2(false, true, false);
  else if (!akout && bkout && shift) TT_L2(false, true, true);
  else if (akout && !bkout) TT_L2(true, false, false);
  else if (akout && bkout && !shift) TT_L2(true, true, false);
  else TT_L2(true, true, true);
#undef TT_L2
#undef TT_L
  TT_CHECK_LAUNCH("gemm_persist");
  return 0;
}

// ---- four-wave 256x256 NT GEMM (option gemm_w4; bf16 in / out, bias) ------------------
// The 8-wave loops above give each wave a 128x64 tile: per 32-deep K-slice the workgroup
// reads 96 KiB of fragments from LDS for 4.2 MFLOP, which with the DMA writes fills the
// LDS port for as long as the MFMAs run. Here 4 waves (one per SIMD, up to 512 registers)
// own 128x128 tiles (256 accumulator registers, in AGPRs): 64 KiB of fragment reads per
// K-slice, every fragment feeding 8 MFMAs. The K loop runs 32-deep K-tiles through a 4-slot
// LDS ring (A and B images of 256 rows x 64 B, 16-byte chunk c of row r at slot
// c ^ ((r >> 1) & 3)), three K-tiles of buffer LDS-DMAs in flight, one barrier per K-tile,
// and the fragments of K-tile kt+1 read from LDS between the MFMAs of kt (double-buffered in
// registers) so the one wave per SIMD always has MFMAs to issue. Same MFMA, operand order
// (transposed accumulate) and k order as gemm_persist: bit-identical to it.
#ifndef W4_LEAD  // gemm_w4 (LDS-DMA form): K-tiles in flight beyond the next (2; 3 = slot kt % 4 refilled
#define W4_LEAD 2    // with K-tile kt+4 as soon as every wave holds kt's fragments; measured no faster)
#endif
namespace w4 {
constexpr int SLOT = 32768;  // A image 16 KiB + B image 16 KiB
constexpr int NS = 4;
struct Frags {
  uint4 a[8], b[8];
};
TT_DEV uint4 frag(const char* img, int r0) {
  const int lane = threadIdx.x & 63;
  const int row = r0 + (lane & 15);
  return *reinterpret_cast<const uint4*>(img + row * 64 + (((lane >> 4) ^ ((row >> 1) & 3)) << 4));
}
}  // namespace w4

// RS (option gemm_w4 2): the operand K-tiles are staged through registers instead of
// LDS-DMA (one wave per SIMD pays each DMA piece's issue cost in its own MFMA stream):
// 16-byte buffer loads of K-tile kt+3 issued during K-tile kt, written to LDS with
// ds_write_b128 one step later, three LDS slots.
template <bool RS>
__global__ __launch_bounds__(256, 1) void gemm_w4(GemmArgs g, int ntm, int ntn) {
  constexpr int NSL = RS ? 3 : w4::NS;
  __shared__ __attribute__((aligned(16))) char lds[NSL * w4::SLOT];
  const int id = ttg::xcd_remap(blockIdx.x, gridDim.x);
  const int per = ntm * ntn;
  const int bi = id / per, tile = id - bi * per;
  const int mt = tile / ntn, nt = tile - mt * ntn;
  const int m0 = mt * 256, n0 = nt * 256;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wr = wave >> 1, wc = wave & 1;
  const bf16_t* A = static_cast<const bf16_t*>(g.a[bi]);
  const bf16_t* B = static_cast<const bf16_t*>(g.b[bi]);
  const uint32_t base = __builtin_amdgcn_readfirstlane(ttg::lds_addr_of(lds));
  // this wave's 8 DMA pieces per K-tile: pieces 8 wave .. 8 wave + 7 of 32 (0-15 A rows
  // 16p.., 16-31 B rows 16(p-16)..); lane -> (row, chunk slot) of the 1 KiB piece
  const bool isA = wave < 2;
  const long ld = isA ? g.lda : g.ldb;
  const long r0 = isA ? m0 : n0;
  const long rows_left = (isA ? g.M : g.N) - r0;
  const long nrec = rows_left * ld * 2;
  const uint32_t nrec32 = (uint32_t)(nrec > 0xFFFFFFFFL ? 0xFFFFFFFFL : nrec);
  const ttg::tt_rsrc4 rs = ttg::make_rsrc4((isA ? A : B) + r0 * ld, nrec32);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>((isA ? A : B) + r0 * ld), (short)0, (int)(nrec32 > 0x7fffffffu ? 0x7fffffffu : nrec32), 0x00020000);
  // piece j of this wave covers operand rows 16 ((wave & 1) 8 + j) + (lane >> 2); the chunk
  // swizzle (row >> 1) & 3 = (lane >> 3) & 3 does not depend on j, so one per-lane offset
  // serves every piece and the piece's row advance rides in the SGPR soffset with the K-tile's
  const int prow = 16 * (wave & 1) * 8 + (lane >> 2);
  const uint32_t voff = (uint32_t)(prow * ld * 2 + (((lane & 3) ^ ((lane >> 3) & 3)) << 4));
  const uint32_t pstep = (uint32_t)(16 * ld * 2);
  const uint32_t pbase = (uint32_t)wave * 8u * 1024u;  // this wave's first piece in a slot
  auto dma = [&](int kt, int j) {
    ttg::dma16_buf(rs, voff, (uint32_t)kt * 64u + (uint32_t)j * pstep,
                   base + (uint32_t)(kt % NSL) * w4::SLOT + pbase + (uint32_t)j * 1024u);
  };
  auto gload = [&](int kt, int j) { return ld16_buf(rsb, voff, (int)((uint32_t)kt * 64u + (uint32_t)j * pstep)); };
  auto lput = [&](int kt, int j, const uint4& v) {
    *reinterpret_cast<uint4*>(lds + (kt % NSL) * w4::SLOT + pbase + j * 1024 + lane * 16) = v;
  };
  const int nk = g.K / 32;
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (RS) {
    // K-tiles 0, 1 through registers into slots 0, 1; K-tile 2's loads in flight in S1
    uint4 S0[8], S1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) S0[j] = gload(0, j);
#pragma unroll
    for (int j = 0; j < 8; ++j) S1[j] = gload(1, j);
#pragma unroll
    for (int j = 0; j < 8; ++j) lput(0, j, S0[j]);
#pragma unroll
    for (int j = 0; j < 8; ++j) lput(1, j, S1[j]);
#pragma unroll
    for (int j = 0; j < 8; ++j) S0[j] = gload(2, j);
    __syncthreads();
    w4::Frags F0, F1;
    {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        F0.a[i] = w4::frag(lds, wr * 128 + 16 * i);
        F0.b[i] = w4::frag(lds + 16384, wc * 128 + 16 * i);
      }
    }
    // step kt: slot (kt+1) % 3 holds K-tile kt+1 (written during step kt-1); Sw holds K-tile
    // kt+2's global data (loaded during step kt-1), written now into slot (kt+2) % 3 -- last
    // read during step kt-2 (K-tile kt-1), so free after step kt-1's barrier; K-tile kt+3's
    // loads go into Sw as its values are written
    auto step = [&](const w4::Frags& Fc, w4::Frags& Fn, uint4 (&Sw)[8], int kt) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's writes of K-tile kt+1
      __builtin_amdgcn_s_barrier();
      const char* img = lds + ((kt + 1) % NSL) * w4::SLOT;
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        Fn.a[i] = w4::frag(img, wr * 128 + 16 * i);
        Fn.b[i] = w4::frag(img + 16384, wc * 128 + 16 * i);
        lput(kt + 2, i, Sw[i]);
        Sw[i] = gload(kt + 3, i);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = ttg::mma<bf16_t>(Fc.b[j], Fc.a[i], acc[i][j]);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    for (int kt = 0; kt < nk; kt += 2) {
      step(F0, F1, S0, kt);
      step(F1, F0, S0, kt + 1);
    }
    (void)S1;
  } else {
    // Every K-tile step issues the same work whether or not it is needed (K-tiles past the
    // end are read from the next rows / zeros into slots nothing reads, and the last step's
    // next-fragment reads are discarded), so the loop has no branches and the waits are
    // constant: younger than K-tile kt+1's pieces are only K-tile kt+2's, 8 per wave.
    // prologue: K-tiles 0..W4_LEAD in flight, wait for 0
#pragma unroll
    for (int kt = 0; kt <= W4_LEAD; ++kt)
#pragma unroll
      for (int j = 0; j < 8; ++j) dma(kt, j);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * W4_LEAD) : "memory");
    __builtin_amdgcn_s_barrier();
    w4::Frags F0, F1;
    {
      const char* img = lds;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        F0.a[i] = w4::frag(img, wr * 128 + 16 * i);
        F0.b[i] = w4::frag(img + 16384, wc * 128 + 16 * i);
      }
    }
    // one K-tile: its MFMAs from Fc, K-tile kt+1's fragments into Fn between them, and K-tile
    // kt+3's DMA pieces, one per row block
    auto step = [&](const w4::Frags& Fc, w4::Frags& Fn, int kt) {
      // K-tile kt+1 landed (this wave's pieces; younger: K-tiles kt+2 .. kt+W4_LEAD)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * (W4_LEAD - 1)) : "memory");
      // W4_LEAD 3 refills slot kt % 4, whose fragments (K-tile kt, read during step kt-1) must
      // have reached every wave's registers before the barrier
      if (W4_LEAD >= 3) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // ... everyone's; and every wave is done with slot (kt+W4_LEAD+1) % 4
      const char* img = lds + ((kt + 1) % w4::NS) * w4::SLOT;
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        Fn.a[i] = w4::frag(img, wr * 128 + 16 * i);
        Fn.b[i] = w4::frag(img + 16384, wc * 128 + 16 * i);
        dma(kt + W4_LEAD + 1, i);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = ttg::mma<bf16_t>(Fc.b[j], Fc.a[i], acc[i][j]);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    // nk even here (the host requires K % 64 == 0)
    for (int kt = 0; kt < nk; kt += 2) {
      step(F0, F1, kt);
      step(F1, F0, kt + 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing DMAs land before the LDS is released
  }
  // epilogue: acc[i][j][e] = C(row wr*128 + 16 i + (lane & 15), col wc*128 + 16 j + 4 (lane >> 4) + e)
  bf16_t* C = static_cast<bf16_t*>(g.c[bi]);
  const float* bias = g.bias[bi];
  const int q = lane >> 4, lr = lane & 15;
  const __amdgpu_buffer_rsrc_t crs = tt_rsrc(C + (long)m0 * g.ldc + n0);
#pragma unroll
  for (int jp = 0; jp < 4; ++jp) {
    float bv[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 b4 = bias ? *reinterpret_cast<const float4*>(bias + n0 + wc * 128 + 16 * (2 * jp + h) + 4 * q)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
      bv[h][0] = b4.x; bv[h][1] = b4.y; bv[h][2] = b4.z; bv[h][3] = b4.w;
    }
    const int cs = wc * 128 + 16 * (2 * jp + (q & 1)) + 8 * (q >> 1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint32_t w[2][2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 a = acc[i][2 * jp + h];
        w[h][0] = (uint32_t)f2bf(a[0] + bv[h][0]) | ((uint32_t)f2bf(a[1] + bv[h][1]) << 16);
        w[h][1] = (uint32_t)f2bf(a[2] + bv[h][2]) | ((uint32_t)f2bf(a[3] + bv[h][3]) << 16);
      }
      const auto s0 = __builtin_amdgcn_permlane16_swap(w[0][0], w[1][0], false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(w[0][1], w[1][1], false, false);
      const uint4 v = make_uint4(s0[0], s1[0], s0[1], s1[1]);
      const int off = (int)(((long)(wr * 128 + 16 * i + lr) * g.ldc + cs) * 2L);
      if (g.stream_out) st16_sc1(crs, off, v);
      else st16_buf(crs, (uint32_t)off, 0, v);
    }
  }
}

// gemm_bres where it applies (bf16 NT, bias only, N % 192 == 0, short K): returns true if launched
template <typename T, typename TO>
bool try_bres(int akout, int bkout, bool shift, const GemmArgs& g, int nbatch, hipStream_t st, int* rc) {
  *rc = 0;
  if constexpr (!std::is_same<T, bf16_t>::value || !std::is_same<TO, bf16_t>::value) {
    return false;
  } else {
    if (tt::opt(tt::OPT_GEMM_BRES) == 0 || akout || bkout || shift || g.splits != 1 || g.beta || g.relu ||
        g.drop_thresh || g.alpha != 1.f || g.force_regstage)
      return false;
    if (g.N % BR_COLS || g.K % 32 || g.K < 32 || g.K > 384 || !g.vec_ok || (g.lda * 2) % 16) return false;
    for (int b = 0; b < nbatch; ++b)
      if (g.bias[b] && (uintptr_t)g.bias[b] % 16) return false;
    const int npan = g.N / BR_COLS, ptot = npan * nbatch, nwg = 256;
    if (ptot > nwg || nwg % ptot) return false;
    if ((long)g.M < (long)(nwg / ptot) * 256 || (long)g.M * g.lda * 2 >= (1L << 31)) return false;
    const bool r64 = tt::opt(tt::OPT_BRES_ROWS) == 64;
    const dim3 grid(nwg), blk(r64 ? 256 : 512);
    switch (g.K / 32) {
#define TT_BR(n)                                                                   \
  case n:                                                                          \
    if (r64)                                                                       \
      hipLaunchKernelGGL((gemm_bres<n, 4>), grid, blk, 0, st, g, npan, nbatch);    \
    else                                                                           \
      hipLaunchKernelGGL((gemm_bres<n, 2>), grid, blk, 0, st, g, npan, nbatch);    \
    break;
      TT_BR(1) TT_BR(2) TT_BR(3) TT_BR(4) TT_BR(5) TT_BR(6) TT_BR(7) TT_BR(8) TT_BR(9) TT_BR(10) TT_BR(11) TT_BR(12)
#undef TT_BR
      default: return false;
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      tt::set_error("gemm_bres: %s", hipGetErrorString(e));
      *rc = (int)e;
    }
    return true;
  }
}

template <typename T, typename TO>
int launch_gemm(int akout, int bkout, bool shift, GemmArgs& g, int nbatch, hipStream_t st) {
  constexpr int EPC = 16 / (int)sizeof(T);
  {
    int rc = 0;
    if (try_bres<T, TO>(akout, bkout, shift, g, nbatch, st, &rc)) return rc;
  }
  const bool dma = (akout ? g.M % EPC == 0 : g.K % EPC == 0) && (bkout ? g.N % EPC == 0 : g.K % EPC == 0) &&
                   g.force_regstage != 1;
  const long t256 = (long)tt_ceil_div(g.M, 256) * tt_ceil_div(g.N, 256) * nbatch * g.splits;
  // persistent tiles with the epilogue under the next tile's first K-tiles: many tiles,
  // short K (the epilogue is a large share of a tile: measured faster up to 16 K-tiles,
  // slower at 48 and 128), no split-K, no accumulate (env TT_GEMM_PERSIST=0 disables)
  const bool persist_ok = tt::opt(tt::OPT_GEMM_PERSIST) != 0;
  const int nk = (g.K * (int)sizeof(T) + ttg::KTB - 1) / ttg::KTB;
  // operand DMAs through buffer resources (Loop8 BUF): whole K-tiles, every
  // K-outer operand's byte range from a split's first K-tile (two K-tiles of prefetch
  // past its end included) addressable by a 32-bit offset, and a split-column A operand
  // whose second block lies after the first in the same rows
  bool buf = tt::opt(tt::OPT_GEMM_BUF) != 0 && g.K % (ttg::KTB / (int)sizeof(T)) == 0;
  {
    const long span = (long)(g.kt_per_split + 2) * (ttg::KTB / (int)sizeof(T)) * (long)sizeof(T);
    if (akout && span * g.lda >= (1L << 32)) buf = false;
    if (bkout && span * g.ldb >= (1L << 32)) buf = false;
    // the shifted operand's buffer form (Loop8 SHalf) masks one k-row per sequence
    // boundary: it needs T to be a whole number of K-tiles
    if (shift && g.seq_t % (ttg::KTB / (int)sizeof(T)) != 0) buf = false;
    if (!akout && (long)256 * g.lda * (long)sizeof(T) >= (1L << 31)) buf = false;
    if (!bkout && (long)256 * g.ldb * (long)sizeof(T) >= (1L << 31)) buf = false;
    for (int b = 0; b < 4 && g.a_split > 0; ++b) {
      if (!g.a[b]) continue;
      const long d = (long)((const char*)g.a_hi[b] - (const char*)g.a[b]) / (long)sizeof(T);
      if (d < 0 || d + (g.M - g.a_split) > g.lda) buf = false;
    }
  }
  if constexpr (std::is_same<T, bf16_t>::value && std::is_same<TO, bf16_t>::value) {
    // gemm_w4 (opt-in): NT, whole 256x256 tiles, K a multiple of 64, bias only
    if (tt::opt(tt::OPT_GEMM_W4) && !akout && !bkout && !shift && g.splits == 1 && !g.beta && !g.relu &&
        !g.drop_thresh && g.alpha == 1.f && g.force_regstage == 0 && g.M % 256 == 0 && g.N % 256 == 0 && g.K % 64 == 0 &&
        g.K >= 32 && g.vec_ok && g.bias_vec_ok && (g.lda * 2) % 16 == 0 && (g.ldb * 2) % 16 == 0 &&
        256L * g.lda * 2 < (1L << 31) && 256L * g.ldb * 2 < (1L << 31) && 256L * g.ldc * 2 < (1L << 31)) {
      const int ntm = g.M / 256, ntn = g.N / 256;
      if (tt::opt(tt::OPT_GEMM_W4) == 2)
        hipLaunchKernelGGL(gemm_w4<true>, dim3((unsigned)(ntm * ntn * nbatch)), dim3(256), 0, st, g, ntm, ntn);
      else
        hipLaunchKernelGGL(gemm_w4<false>, dim3((unsigned)(ntm * ntn * nbatch)), dim3(256), 0, st, g, ntm, ntn);
      TT_CHECK_LAUNCH("gemm_w4");
      return 0;
    }
  }
  if (dma && persist_ok && !shift && (g.force_regstage == 0 || g.force_regstage >= 9) && g.splits == 1 && !g.beta && nk >= 2 && nk <= tt::opt(tt::OPT_GEMM_PERSIST_MAXK) && t256 >= 512 &&
      use_big(g.M, g.N, t256))
    return launch_persist<T, TO>(akout, bkout, shift, g, (int)t256, buf, st);
  if (dma && g.force_regstage != 2 && use_big(g.M, g.N, t256)) {
    if (tt::opt(tt::OPT_GEMM_A3) && buf)
      return launch_t<T, TO, 256, 256, 2, 4, true, true, true>(akout, bkout, shift, g, t256, st);
    if (tt::opt(tt::OPT_GEMM_A3)) return launch_t<T, TO, 256, 256, 2, 4, true, true>(akout, bkout, shift, g, t256, st);
    return launch_t<T, TO, 256, 256, 2, 4, true>(akout, bkout, shift, g, t256, st);
  }
  const long t128 = (long)tt_ceil_div(g.M, 128) * tt_ceil_div(g.N, 128) * nbatch * g.splits;
  if (dma) return launch_t<T, TO, 128, 128, 2, 2, true>(akout, bkout, shift, g, t128, st);
  return launch_t<T, TO, 128, 128, 2, 2, false>(akout, bkout, shift, g, t128, st);
}

}  // namespace

// Step 1 of the hard-negative top-k (tt_score.hip) on the persistent 256x256 GEMM:
// S = Q D^T (bf16, K = h a multiple of 64) accumulated transposed -- the hn_scan kernel's MFMA
// orientation, instruction and k order, so the chunk maxima are the values hn_rescore
// recomputes bit for bit -- with the chunk-max epilogue instead of C stores. Tiles in column
// groups per XCD (gemm_order's walk) when the shape allows.
int tt::tt_hn_scan_gemm(const void* q, long bq, const void* d, long nd, int h, long label_off, float* cm, long nch,
                    hipStream_t st) {
  TT_CHECK_ARG(h % 64 == 0 && h <= 1024 && bq > 0 && nd > 0 && bq < (1L << 31) && nd < (1L << 31),
               "tt_hn_scan_gemm: h %d, bq %ld, nd %ld", h, bq, nd);
  GemmArgs g{};
  g.a[0] = q;
  g.b[0] = d;
  g.lda = g.ldb = h;
  g.M = (int)bq;
  g.N = (int)nd;
  g.K = h;
  g.alpha = 1.f;
  g.splits = 1;
  g.kt_per_split = h / 64;
  g.nbatch = 1;
  g.cm = cm;
  g.nch = nch;
  g.label_off = label_off;
  const long ntm = (bq + 255) / 256, ntn = (nd + 255) / 256, ntiles = ntm * ntn;
  TT_CHECK_ARG(ntiles < (1L << 31), "tt_hn_scan_gemm: too many tiles");
  if (ntiles % 256 == 0 && ntn % 4 == 0) {
    g.walk_g = 4;
    g.walk_x = 8;
  }
  hipLaunchKernelGGL((gemm_persist<bf16_t, false, false, false, float, true, true, true>),
                     dim3((unsigned)std::min<long>(ntiles, 256)), dim3(512), 0, st, g, (int)ntiles);
  TT_CHECK_LAUNCH("gemm_persist (hard-negative scan)");
  return 0;
}

extern "C" long tt_gemm_ws_size(int m, int n, int nbatch, int splits) {
  (void)m;
  return splits > 1 ? (long)m * n * nbatch * splits : 0;
}

extern "C" int tt_gemm_pick_splits(int m, int n, int k, int nbatch) {
  // Enough workgroups for >= 2-3 rounds over the 256 CUs, with the last round as
  // full as possible; never fewer than 8 K-tiles (64 bf16) per split.
  const bool big = m >= 256 && n >= 256;
  const long tiles = big ? (long)tt_ceil_div(m, 256) * tt_ceil_div(n, 256) * nbatch
                         : (long)tt_ceil_div(m, BM) * tt_ceil_div(n, BN) * nbatch;
  const long target = big ? 512 : 1024;
  if (tiles >= target) return 1;
  const int smax = std::max(1, std::min(64, tt_ceil_div(k, 64) / 8));
  int best = 1;
  double best_eff = 0.0;
  const int s_lo = (int)std::min<long>(smax, std::max<long>(1, target / tiles));
  for (int s = s_lo; s <= std::min<long>(smax, 3 * target / tiles + 1); ++s) {
    const long w = tiles * s;
    const double eff = (double)w / (256.0 * (double)tt_ceil_div(w, 256));
    if (eff > best_eff + 1e-9) { best_eff = eff; best = s; }
  }
  return std::min(best, smax);
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
    g.a_hi[b] = batch->a_hi[b];
    if (batch->a_split > 0)
      TT_CHECK_ARG(batch->a_hi[b] && (uintptr_t)batch->a_hi[b] % 16 == 0, "tt_gemm: a_hi[%d] null or misaligned", b);
    if (batch->bshift[b] != 0) shift = true;
  }
  TT_CHECK_ARG(!shift || (b_kouter && seq_t > 0), "tt_gemm: bshift needs b_kouter and seq_t");
  TT_CHECK_ARG(batch->a_split >= 0 && (batch->a_split == 0 || (a_kouter && batch->a_split % (16 / esz) == 0)),
               "tt_gemm: a_split %d needs a_kouter and a 16-byte multiple", batch->a_split);
  g.a_split = batch->a_split;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = m; g.N = n; g.K = k;
  g.alpha = alpha; g.beta = beta_accum; g.relu = relu; g.seq_t = seq_t;
  g.force_regstage = tt::opt(tt::OPT_GEMM_REGSTAGE);
  g.nbatch = nbatch;
  g.skew = tt::opt(tt::OPT_GEMM_SKEW);
  g.drop_seed = drop_seed;
  g.drop_row0 = batch->drop_row0;
  g.drop_thresh = drop_p > 0.f ? (uint32_t)(drop_p * 16777216.0f + 0.5f) : 0u;
  g.drop_inv_keep = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
  const int nk = tt_ceil_div((long)k * esz, 128);
  if (splits > nk) splits = nk > 0 ? nk : 1;
  g.kt_per_split = nk > 0 ? tt_ceil_div(nk, splits) : 1;
  splits = nk > 0 ? tt_ceil_div(nk, g.kt_per_split) : 1;
  g.splits = splits;
  {
    const int osz = out_dtype == TT_DT_BF16 ? 2 : 4;
    bool ok = (ldc * osz) % 16 == 0;
    for (int b = 0; b < nbatch; ++b) ok = ok && ((uintptr_t)batch->c[b] % 16 == 0);
    g.vec_ok = ok;
    bool bok = true;
    for (int b = 0; b < nbatch; ++b) bok = bok && ((uintptr_t)batch->bias[b] % 16 == 0);
    g.bias_vec_ok = bok;
    // outputs far larger than the L2s are streamed past them (sc1); ld*rows must
    // stay addressable by a 32-bit per-tile byte offset
    g.stream_out = ok && (long)m * n * osz >= (64L << 20) && (long)256 * ldc * osz < (1L << 31);
    g.stream_out = g.stream_out ? tt::opt(tt::OPT_GEMM_STREAM_OUT) : 0;  // 1 sc1, 2 nt, 3 sc0 sc1 (persistent)
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  TT_CHECK_ARG((long)tt_ceil_div(m, 128) * tt_ceil_div(n, 128) * nbatch * splits < (1L << 31), "tt_gemm: too many tiles");

  if (splits > 1) {
    GemmArgs gp = g;
    gp.part_stride = (long)m * n;
    gp.vec_ok = (n % 4 == 0);
    for (int b = 0; b < nbatch; ++b) gp.c[b] = splitk_ws + (long)b * splits * gp.part_stride;
    int rc = dtype == TT_DT_BF16 ? launch_gemm<bf16_t, float>(a_kouter, b_kouter, shift, gp, nbatch, st)
                                 : launch_gemm<float, float>(a_kouter, b_kouter, shift, gp, nbatch, st);
    if (rc) return rc;
    const bool v4 = n % 4 == 0 && (uintptr_t)splitk_ws % 16 == 0;  // dense [m][n] partials, 16-byte rows
    const long total = (long)m * n / (v4 ? 4 : 1);
    dim3 rg((unsigned)std::min<long>(tt_ceil_div(total, 256), 2048), nbatch);
#define TT_RED(TO, V) hipLaunchKernelGGL((splitk_reduce_kernel<TO, V>), rg, dim3(256), 0, st, splitk_ws, gp.part_stride, splits, m, n, g)
    if (out_dtype == TT_DT_F32) {
      if (v4) TT_RED(float, 4); else TT_RED(float, 1);
    } else {
      if (v4) TT_RED(bf16_t, 4); else TT_RED(bf16_t, 1);
    }
#undef TT_RED
    TT_CHECK_LAUNCH("splitk_reduce_kernel");
    return 0;
  }
  if (dtype == TT_DT_BF16) {
    return out_dtype == TT_DT_BF16 ? launch_gemm<bf16_t, bf16_t>(a_kouter, b_kouter, shift, g, nbatch, st)
                                   : launch_gemm<bf16_t, float>(a_kouter, b_kouter, shift, g, nbatch, st);
  }
  return launch_gemm<float, float>(a_kouter, b_kouter, shift, g, nbatch, st);
}
