// Bidirectional GRU layer, forward and BPTT, as one fused kernel per time step.
//
// Batch rows are independent, so a step is a plain GEMM over the whole batch with
// the gate arithmetic fused into its epilogue:
//   fwd step s : gh = h_{s-1} Whh^T                (M=B, N=3H, K=H)   + r,z,n,h' epilogue
//                (saves the pre-activations of r, z, n and gh_n for the backward)
//   bwd step s : c  = dgh_{s+1} Whh                (M=B, N=H,  K=3H)  + dh, dgx, dgh epilogue
// Up to 4 recurrences (2 towers x 2 directions) share a launch via blockIdx.z.
// The forward tile is 128 batch rows x (3 gates x 64 hidden units): the B-tile rows
// are ordered [unit half][gate][32 units] so that every lane holds r, z and n for
// the same (b, j) in registers and the update needs no data exchange.
#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <type_traits>

#include "tt_api.h"
#include "tt_gemm_core.h"

namespace {

struct FwdRec {
  const void* g; const void* whh; const float* bhn; void* y; void* x1; void* save; float* hs;
  int dir; uint32_t seed; int col0;
  uint32_t row0;  // dropout row of local row 0 (data-parallel: rank * B * T)
};
struct FwdArgs {
  FwdRec r[4];
  int B, T, H;
  long ldg, ldy;
  int s;
  uint32_t drop_thresh;
  float inv_keep;
#ifdef TT_DIAG
  int dbg;  // diagnostic build only: 1 no stores, 2 no G loads
#endif
};

struct BwdRec {
  const void* save; const void* y; const void* dy; const float* dfinal; const void* whh;
  void* dgx; void* dgh; void* dh; float* dbias; int dir;
};
struct BwdArgs {
  BwdRec r[4];
  int B, T, H;
  long ldy, ldd, ldf;
  int s;
  int skew;  // gru_bwd_rows: odd workgroups of an XCD start skew x s_sleep(127) late (option gru_bwd_skew)
#ifdef TT_DIAG
  int dbg;  // diagnostic build only: 1 no GEMM, 2 no epilogue loads, 4 no stores
#endif
};


// The forward GRU cell (enhanced_two_tower.py:17-33 via nn.GRU) in one fixed operation
// order, shared by every forward kernel: FP contraction is off and the two fused
// multiply-adds are explicit, so no kernel's result depends on how hipcc contracted its
// own copy of the expression -- the per-step, persistent and wave-owned-rows forwards are
// bit-identical by construction. Returns h' and the saved pre-activations.
TT_DEV void gru_cell(float xr, float xz, float xn, float lr, float lz, float ln, float bn, float hp, float& y,
                     float& ar, float& az, float& an, float& ghn) {
#pragma clang fp contract(off)
  constexpr float L2E = 0x1.715476p+0f;
  ghn = ln + bn;
  ar = xr + lr;
  az = xz + lz;
  const float rg = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(L2E * -ar));
  const float zg = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(L2E * -az));
  an = __builtin_fmaf(rg, ghn, xn);
  const float ng = 1.0f - 2.0f * __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(L2E * (2.0f * an)) + 1.0f);
  y = __builtin_fmaf(zg, hp, (1.0f - zg) * ng);
}

// B-tile row r of the forward step -> row (gate*H + j) of Whh [3H, H].
template <typename T>
struct GateRows {
  static constexpr bool SHIFTED = false, KSPLIT = false;
  const T* w; int H, j0;
  TT_DEV const T* rowptr(int r) const {
    const int half = r / 96, rem = r - half * 96;
    const int g = rem >> 5, j = j0 + half * 32 + (rem & 31);
    return j < H ? w + (long)(g * H + j) * H : nullptr;
  }
  TT_DEV const T* at(int r, int k) const { const T* p = rowptr(r); return p ? p + k : nullptr; }
};

// BMR batch rows per tile: 128 (4 waves, two workgroups per CU) or 256 (8 waves as 4 x 2,
// half the W_hh traffic per FLOP and twice the MFMA work per K-tile barrier): at configs[4]
// (H 1024, B 8192) 48.0-48.6 vs 50.3-51.5 ms per layer. A 4-stage LDS ring with counted
// waits on 128-row tiles (one workgroup per CU) measured 85.7 ms.
template <typename T, int BMR, int NS = 2>  // NS: LDS stages of the product (DLoop)
__global__ __launch_bounds__(2 * BMR) void gru_fwd_step(FwdArgs a) {
  constexpr int NT = 2 * BMR;
  using ML = ttg::DLoop<T, false, false, BMR, 192, BMR / 64, 2, NS>;
  __shared__ __attribute__((aligned(16))) char lds[ML::LDS_BYTES];
  // 1-D grid, XCD-aware: the H/64 unit tiles of one batch tile are consecutive ids on one
  // XCD, so its h_{s-1} panel is fetched into that XCD's L2 once, not once per tile.
  const int ntj = (a.H + 63) / 64, ntm = (a.B + BMR - 1) / BMR;
  const int id = ttg::xcd_remap(blockIdx.x, gridDim.x);
  const int rz = id / (ntm * ntj), rem = id - rz * ntm * ntj;
  const FwdRec R = a.r[rz];
  const int H = a.H, T_ = a.T, s = a.s;
  const int m0 = (rem / ntj) * BMR, j0 = (rem % ntj) * 64;
  const int t = R.dir ? T_ - 1 - s : s;
  const int tp = R.dir ? t + 1 : t - 1;
  const T* Y = static_cast<const T*>(R.y);

  f32x4 acc[ML::TM][ML::TN];
#pragma unroll
  for (int i = 0; i < ML::TM; ++i)
#pragma unroll
    for (int j = 0; j < ML::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bool prod = s > 0, epi = true;
#ifdef TT_DIAG
  // diagnostic build, per-step forward (gru_fwd_step): 8 no product, 16 no epilogue
  if (a.dbg & 8) prod = false;
  if (a.dbg & 16) epi = false;
#endif
  const int tid = threadIdx.x;
  const int cur = s & 1, prv = cur ^ 1;
  const T* G = static_cast<const T*>(R.g);
  const float* hs_prv = R.hs + (long)prv * a.B * H;
  if (prod) {
    ttg::KCPlain<T> la{Y + (long)tp * a.ldy, (long)T_ * a.ldy, m0, a.B};
    GateRows<T> lb{static_cast<const T*>(R.whh), H, j0};
    const int nk = (H * (int)sizeof(T) + ttg::KTB - 1) / ttg::KTB;
    ML::run(la, lb, H, 0, nk, lds, acc);
  }
  if (!epi) {
    if (acc[0][0][0] == 1.2345f) static_cast<T*>(R.y)[0] = T(0);  // keep the product
    return;
  }

  // ---- epilogue, one 64-row half at a time: stage the fp32 gate tile in LDS, then
  // every thread updates 8 consecutive hidden units of a row with 16-byte accesses.
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* L = reinterpret_cast<float*>(lds);  // [3][64][FLD]
  constexpr int FLD = 68;                    // 64 units + 16 B pad
  T* Yw = static_cast<T*>(R.y);
  T* X1 = static_cast<T*>(R.x1);
  T* S = static_cast<T*>(R.save);
  float* hs_cur = R.hs + (long)cur * a.B * H;
  const __amdgpu_buffer_rsrc_t srs = tt_rsrc(S + ((long)m0 * T_ + t) * (4L * H));
  const __amdgpu_buffer_rsrc_t xrs = tt_rsrc(X1 ? X1 + ((long)m0 * T_ + t) * a.ldy : Yw);
  for (int hf = 0; hf < BMR / 64; ++hf) {
    if ((wave >> 1) == hf) {
      const int nb = (wave & 1) * 32;
#pragma unroll
      for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jh = 0; jh < 2; ++jh)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              L[(g * 64 + 16 * i + 4 * (lane >> 4) + r) * FLD + nb + 16 * jh + (lane & 15)] = acc[i][g * 2 + jh][r];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 512 / NT; ++k) {
      const int rl = (tid >> 3) + (NT / 8) * k, jg = (tid & 7) * 8;
      const int b = m0 + hf * 64 + rl, j = j0 + jg;
      if (b < a.B && j < H) {
        const long row = (long)b * T_ + t;
        float xr[8], xz[8], xn[8], hp[8], bn[8], y[8], sr[8], sz[8], sn[8], sg[8];
        ld8(G + row * a.ldg + j, xr);
        ld8(G + row * a.ldg + H + j, xz);
        ld8(G + row * a.ldg + 2 * H + j, xn);
        ld8(R.bhn + j, bn);
        if (s > 0) ld8(hs_prv + (long)b * H + j, hp);
        else {
#pragma unroll
          for (int e = 0; e < 8; ++e) hp[e] = 0.f;
        }
        const float* Lr = L + (0 * 64 + rl) * FLD + jg;
        const float* Lz = L + (1 * 64 + rl) * FLD + jg;
        const float* Ln = L + (2 * 64 + rl) * FLD + jg;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          // saved: pre-activations, not gate values: the backward recomputes sigma/tanh
          // in fp32, so 1-z and 1-n^2 keep full precision even with bf16 storage
          gru_cell(xr[e], xz[e], xn[e], Lr[e], Lz[e], Ln[e], bn[e], hp[e], y[e], sr[e], sz[e], sn[e], sg[e]);
        st8(hs_cur + (long)b * H + j, y);
        st8(Yw + row * a.ldy + j, y);
        // saved pre-activations and the dropout copy are only read by later kernels:
        // stream them past L2 (sc1) so Whh and the h_{s-1} rows stay resident
        const int so = (int)((((long)(b - m0) * T_) * 4L * H + j) * (long)sizeof(T));
        st8_sc1(srs, so, sr, (T*)nullptr);
        st8_sc1(srs, so + H * (int)sizeof(T), sz, (T*)nullptr);
        st8_sc1(srs, so + 2 * H * (int)sizeof(T), sn, (T*)nullptr);
        st8_sc1(srs, so + 3 * H * (int)sizeof(T), sg, (T*)nullptr);
        if (X1) {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            y[e] *= a.drop_thresh ? tt_dropout_scale(R.seed, R.row0 + (uint32_t)row, (uint32_t)(R.col0 + j + e),
                                                     a.drop_thresh, a.inv_keep)
                                  : 1.f;
          st8_sc1(xrs, (int)((((long)(b - m0) * T_) * a.ldy + j) * (long)sizeof(T)), y, (T*)nullptr);
        }
      }
    }
    __syncthreads();
  }
}

// BMR batch rows per tile: 128, or 64 (3 tiles per CU at NS 2); NS: LDS stages (DLoop)
template <typename T, int BMR, int NS = 2>
__global__ __launch_bounds__(256) void gru_bwd_step(BwdArgs a) {
  using ML = ttg::DLoop<T, false, true, BMR, 128, 2, 2, NS>;
  constexpr int LDSB = ML::LDS_BYTES > 64 * 132 * 4 ? ML::LDS_BYTES : 64 * 132 * 4;
  __shared__ __attribute__((aligned(16))) char lds[LDSB];
  const int ntj = (a.H + 127) / 128, ntm = (a.B + BMR - 1) / BMR;
  const int id = ttg::xcd_remap(blockIdx.x, gridDim.x);
  const int rz = id / (ntm * ntj), rem = id - rz * ntm * ntj;
  const int mt = rem / ntj;
  const BwdRec R = a.r[rz];
  const int H = a.H, T_ = a.T, s = a.s;
  const int m0 = mt * BMR, j0 = (rem % ntj) * 128;
  const int t = R.dir ? T_ - 1 - s : s;
  const int tn = R.dir ? t - 1 : t + 1;  // time of step s+1
  const int tp = R.dir ? t + 1 : t - 1;  // time of step s-1
  const bool last = (s == T_ - 1);
  const T* DGX = static_cast<const T*>(R.dgx);
  const T* DGH = static_cast<const T*>(R.dgh);

  f32x4 acc[ML::TM][ML::TN];
#pragma unroll
  for (int i = 0; i < ML::TM; ++i)
#pragma unroll
    for (int j = 0; j < ML::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (!last) {
    // dL/dgh_{s+1} = [dL/dar, dL/daz | dL/d(W_hn h)]: r|z from the dgx buffer, n from dgh
    ttg::KCSplit<T> la{DGX + (long)tn * a.ldd, DGH + (long)tn * a.ldd, (long)T_ * a.ldd, m0, a.B, 2 * H};
    ttg::KOPlain<T> lb{static_cast<const T*>(R.whh), H, j0, H - j0};
    const int K = 3 * H;
    const int nk = (K * (int)sizeof(T) + ttg::KTB - 1) / ttg::KTB;
    ML::run(la, lb, K, 0, nk, lds, acc);
  }

  // ---- epilogue, one 64-row half at a time through LDS; each thread owns 8
  // consecutive units of a row (16-byte accesses) for 4 rows per half.
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, tid = threadIdx.x;
  float* L = reinterpret_cast<float*>(lds);  // [64][BLD]
  constexpr int BLD = 132;                   // 128 units + 16 B pad
  const int cur = s & 1, nxt = cur ^ 1;
  const T* S = static_cast<const T*>(R.save);
  const T* Y = static_cast<const T*>(R.y);
  const T* DY = static_cast<const T*>(R.dy);
  T* DGXw = static_cast<T*>(R.dgx);
  T* DGHw = static_cast<T*>(R.dgh);
  // carry_s = dh_s * z_s, stored in the compute dtype: it feeds one step's dh exactly
  // like the bf16 GEMM operand dL/dgh_{s+1} does (same rounding), at half the bytes
  T* cr_cur = static_cast<T*>(R.dh) + (long)cur * a.B * H;
  const T* cr_nxt = static_cast<const T*>(R.dh) + (long)nxt * a.B * H;
  const long S4 = 4L * H;
  const int jg = (tid & 15) * 8;
  const int j = j0 + jg;
  const __amdgpu_buffer_rsrc_t grs = tt_rsrc(DGXw + ((long)m0 * T_ + t) * a.ldd);
  float bsum[4][8];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) bsum[q][e] = 0.f;
  for (int hf = 0; hf < BMR / 64; ++hf) {
    // waves whose accumulator rows fall in this 64-row slice stage them
    const int wrow = (wave >> 1) * (BMR / 2) - hf * 64;
    if (wrow >= 0 && wrow < 64) {
      const int wn = (wave & 1) * 64;
#pragma unroll
      for (int i = 0; i < ML::TM; ++i)
#pragma unroll
        for (int jt = 0; jt < 4; ++jt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            L[(wrow + 16 * i + 4 * (lane >> 4) + r) * BLD + wn + 16 * jt + (lane & 15)] = acc[i][jt][r];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int rl = (tid >> 4) + 16 * k;
      const int b = m0 + hf * 64 + rl;
      if (b < a.B && j < H) {
        const long row = (long)b * T_ + t;
        float cin[8], dy[8], ar[8], az[8], an[8], gh[8], hp[8];
        if (!last) ld8(cr_nxt + (long)b * H + j, cin);
        else if (R.dfinal) ld8(R.dfinal + (long)b * a.ldf + j, cin);
        else {
#pragma unroll
          for (int e = 0; e < 8; ++e) cin[e] = 0.f;
        }
        if (DY) ld8(DY + row * a.ldy + j, dy);
        else {
#pragma unroll
          for (int e = 0; e < 8; ++e) dy[e] = 0.f;
        }
        const T* sp = S + row * S4 + j;
        ld8(sp, ar);
        ld8(sp + H, az);
        ld8(sp + 2 * H, an);
        ld8(sp + 3 * H, gh);
        if (s > 0) ld8(Y + ((long)b * T_ + tp) * a.ldy + j, hp);
        else {
#pragma unroll
          for (int e = 0; e < 8; ++e) hp[e] = 0.f;
        }
        const float* Lc = L + rl * BLD + jg;
        float o_r[8], o_z[8], o_n[8], o_hn[8], cout[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float dht = Lc[e] + cin[e] + dy[e];
          float rg, omr, zg, omz, ng, sech2;
          tt_sigmoid_pair(ar[e], rg, omr);
          tt_sigmoid_pair(az[e], zg, omz);
          tt_tanh_sech2(an[e], ng, sech2);
          const float dnp = dht * omz * sech2;
          const float drp = dnp * gh[e] * rg * omr;
          const float dzp = dht * (hp[e] - ng) * zg * omz;
          o_r[e] = drp; o_z[e] = dzp; o_n[e] = dnp; o_hn[e] = dnp * rg;
          cout[e] = dht * zg;
          bsum[0][e] += drp; bsum[1][e] += dzp; bsum[2][e] += dnp; bsum[3][e] += dnp * rg;
        }
        st8(cr_cur + (long)b * H + j, cout);
        // dL/dar, dL/daz are shared by dL/dgx and dL/dgh and re-read by the next step's
        // GEMM: plain stores. dL/dan is next read by the weight-gradient GEMMs only:
        // stream it past L2. dL/d(W_hn h) goes to its own H-column block.
        T* xw = DGXw + row * a.ldd + j;
        st8(xw, o_r);
        st8(xw + H, o_z);
        const int go = (int)((((long)(b - m0) * T_) * a.ldd + j + 2 * H) * (long)sizeof(T));
        st8_sc1(grs, go, o_n, (T*)nullptr);
        st8(DGHw + row * a.ldd + j, o_hn);
      }
    }
    __syncthreads();
  }
  // bias partial sums of this 128-row tile: lanes l, l^16, l^32, l^48 share columns
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = bsum[q][e];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      bsum[q][e] = v;
    }
  float* red = L;  // [4 waves][4][128]
  if (lane < 16) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) red[(wave * 4 + q) * 128 + lane * 8 + e] = bsum[q][e];
  }
  __syncthreads();
  if (tid < 128 && j0 + tid < H) {
    float* pb = R.dbias + (long)mt * (4L * H) + j0 + tid;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      pb[q * H] += red[(0 * 4 + q) * 128 + tid] + red[(1 * 4 + q) * 128 + tid] + red[(2 * 4 + q) * 128 + tid] +
                   red[(3 * 4 + q) * 128 + tid];
  }
}

TT_DEV void unpack8(uint4 v, float (&f)[8]) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xFFFF0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xFFFF0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xFFFF0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xFFFF0000u);
}

#ifndef TT_BWD_BUF  // backward product DMAs through buffer resources (0: per-lane pointers)
#define TT_BWD_BUF 1
#endif
#ifndef TT_BWD_STAG  // gru_bwd_rows product: wave rows one barrier apart (1; measured 0.6% slower than lockstep)
#define TT_BWD_STAG 0
#endif
#ifndef TT_BWD_NB  // gru_bwd_rows: epilogue rows whose loads are in flight together
#define TT_BWD_NB 2
#endif
#ifndef TT_BWD_NT
#define TT_BWD_NT 3
#endif
#ifndef TT_BWD_PIPE  // gru_bwd_rows epilogue: 1 rows one ahead (loads before the previous row's stores); 0 batches of NB
#define TT_BWD_PIPE 1
#endif
#ifndef TT_BWD_CREG  // gru_bwd_rows: the BPTT carry in registers (0: bf16 ping-pong buffer in HBM)
#define TT_BWD_CREG 1
#endif
#ifndef TT_BWD_OUT_NT  // gru_bwd_rows: the dG_r / dG_z / dGh_n output stores non-temporal (1) or plain (0)
#define TT_BWD_OUT_NT 0
#endif
// 8 floats -> 8 bf16 in one 16-byte store, non-temporal when NT
template <bool NT>
TT_DEV void st8_pol(bf16_t* p, const float (&f)[8]) {
  if constexpr (NT) {
    tt_u32x4 w;
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
    __builtin_nontemporal_store(w, reinterpret_cast<tt_u32x4*>(p));
  } else {
    st8(p, f);
  }
}

// ---- backward step on 256x256 tiles (bf16): the recurrent GEMM on the 8-phase loop --
// One workgroup (8 waves) per 256 rows x 256 hidden units of a recurrence: at B 8192,
// H 512 the four recurrences are exactly 256 tiles, one per CU, so the GEMM runs at the
// 8-phase loop's rate (the 128x128 two-phase loop reached ~680 TFLOP/s here) and the
// epilogue (two 128-row passes staged in the freed DMA slots) streams the gate
// gradients. Bias partials land in partial row 2*mt (tt_gru_bias_rows() counts 128-row
// tiles; the odd rows stay zero).
__global__ __launch_bounds__(512) void gru_bwd_big(BwdArgs a) {
  using L8 = ttg::Loop8<bf16_t, false, true, false, false, false, TT_BWD_BUF != 0>;  // W_hh by buffer DMA
  static_assert(L8::LDS_BYTES >= 128 * 256 * 4 && L8::LDS_BYTES >= 8 * 4 * 256 * 4, "staging fits the slots");
  __shared__ __attribute__((aligned(16))) char lds[L8::LDS_BYTES];
  const int H = a.H, T_ = a.T, s = a.s;
  const int ntj = (H + 255) / 256, ntm = (a.B + 255) / 256;
  const int id = ttg::xcd_remap(blockIdx.x, gridDim.x);
  const int rz = id / (ntm * ntj), rem = id - rz * ntm * ntj;
  const int mt = rem / ntj;
  const BwdRec R = a.r[rz];
  const int m0 = mt * 256, j0 = (rem % ntj) * 256;
  const int t = R.dir ? T_ - 1 - s : s;
  const int tn = R.dir ? t - 1 : t + 1;
  const int tp = R.dir ? t + 1 : t - 1;
  const bool last = (s == T_ - 1);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, tid = threadIdx.x;
  const int wn = (wave & 3) * 64;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#ifdef TT_DIAG
  const int dbg = a.dbg;  // diagnostic build only: 1 no GEMM, 2 no epilogue loads, 4 no stores
#else
  constexpr int dbg = 0;
#endif
  if (!last && !(dbg & 1)) {
    const bf16_t* DGX = static_cast<const bf16_t*>(R.dgx);
    const bf16_t* DGH = static_cast<const bf16_t*>(R.dgh);
    ttg::KCSplit<bf16_t> la{DGX + (long)tn * a.ldd, DGH + (long)tn * a.ldd, (long)T_ * a.ldd, m0, a.B, 2 * H};
    ttg::KOPlain<bf16_t> lb{static_cast<const bf16_t*>(R.whh), H, j0, H - j0};
    L8::run(la, lb, 3 * H, 0, (3 * H + L8::KTE - 1) / L8::KTE, lds, acc);
  }

  // ---- epilogue in two passes: pass p stages rows 64p..64p+63 of both wave rows
  // (tile rows 64p.. and 128+64p..) as an fp32 [128][256] image over the freed slots, so
  // half of every wave's accumulators die before the gate arithmetic of the first pass.
  float* L = reinterpret_cast<float*>(lds);
  const int cur = s & 1, nxt = cur ^ 1;
  const bf16_t* S = static_cast<const bf16_t*>(R.save);
  const bf16_t* Y = static_cast<const bf16_t*>(R.y);
  const bf16_t* DY = static_cast<const bf16_t*>(R.dy);
  bf16_t* DGXw = static_cast<bf16_t*>(R.dgx);
  bf16_t* DGHw = static_cast<bf16_t*>(R.dgh);
  bf16_t* cr_cur = static_cast<bf16_t*>(R.dh) + (long)cur * a.B * H;
  const bf16_t* cr_nxt = static_cast<const bf16_t*>(R.dh) + (long)nxt * a.B * H;
  const long S4 = 4L * H;
  const int jg = (tid & 31) * 8;
  const int j = j0 + jg;
  const __amdgpu_buffer_rsrc_t grs = tt_rsrc(DGXw + ((long)m0 * T_ + t) * a.ldd);
  // epilogue operands as buffer resources based at the tile's first row (per-lane byte
  // offsets < 2 GiB, checked on the host); an absent operand gets num_records 0 and an
  // out-of-range row offset 0x80000000, so both read zeros without a branch
  const __amdgpu_buffer_rsrc_t rc = tt_rsrc_n(cr_nxt + (long)m0 * H, !last);
  const __amdgpu_buffer_rsrc_t rd = tt_rsrc_n(DY ? DY + ((long)m0 * T_ + t) * a.ldy : S, DY != nullptr);
  const __amdgpu_buffer_rsrc_t rsv = tt_rsrc_n(S + ((long)m0 * T_ + t) * S4, true);
  const __amdgpu_buffer_rsrc_t ry = tt_rsrc_n(s > 0 ? Y + ((long)m0 * T_ + tp) * a.ldy : S, s > 0);
  float bsum[4][8];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) bsum[q][e] = 0.f;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jt = 0; jt < 4; ++jt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          L[((wave >> 2) * 64 + 16 * i + 4 * (lane >> 4) + r) * 256 + wn + 16 * jt + (lane & 15)] = acc[4 * p + i][jt][r];
    __syncthreads();
    // Rows in batches of NB: the 7 operand loads of every row of a batch are issued back
    // to back (branch-free: an absent operand reads the zero page), one wait, then the
    // gate math and the stores. With loads and stores both pending hipcc waits vmcnt(0)
    // at the next use of a load (MI355X_MICROARCH.md: one in-order counter), so a per-row
    // load/compute/store loop paid the load and the store latency once per row.
    constexpr int NB = 2;
#pragma unroll
    for (int kb = 0; kb < 8; kb += NB) {
      uint4 vin[NB][7];
#pragma unroll
      for (int kk = 0; kk < NB; ++kk) {
        // tile row of image row (tid >> 5) + 16 k: wave row k >> 2, row in pass
        const int bl = (tid >> 5) + p * 64 + 16 * ((kb + kk) & 3) + 128 * ((kb + kk) >> 2);
        const bool ok = m0 + bl < a.B && !(dbg & 2);
        const uint32_t oc = ok ? (uint32_t)(bl * H + j) * 2u : 0x80000000u;
        const uint32_t oy = ok ? (uint32_t)(bl * T_ * (int)a.ldy + j) * 2u : 0x80000000u;
        const uint32_t os = ok ? (uint32_t)(bl * T_ * (int)S4 + j) * 2u : 0x80000000u;
        vin[kk][0] = ld16_buf(rc, oc, 0);
        // TT_BWD_NT: non-temporal loads of the once-read streams (1: S, 2: dy and h_{s-1}), so
        // that they do not displace the re-read gate gradients from the caches
        vin[kk][1] = ld16_buf<(TT_BWD_NT & 2) ? 2 : 0>(rd, oy, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) vin[kk][2 + q] = ld16_buf<(TT_BWD_NT & 1) ? 2 : 0>(rsv, os, q * 2 * H);
        vin[kk][6] = ld16_buf<(TT_BWD_NT & 2) ? 2 : 0>(ry, oy, 0);
      }
#pragma unroll
      for (int kk = 0; kk < NB; ++kk) {
        const int rl = (tid >> 5) + 16 * (kb + kk);
        const int b = m0 + (rl >> 6) * 128 + p * 64 + (rl & 63);
        if (b >= a.B) continue;
        const long row = (long)b * T_ + t;
        float cin[8], dy[8], ar[8], az[8], an[8], gh[8], hp[8];
        unpack8(vin[kk][0], cin);
        unpack8(vin[kk][1], dy);
        unpack8(vin[kk][2], ar);
        unpack8(vin[kk][3], az);
        unpack8(vin[kk][4], an);
        unpack8(vin[kk][5], gh);
        unpack8(vin[kk][6], hp);
        if (last && R.dfinal) ld8(R.dfinal + (long)b * a.ldf + j, cin);  // fp32 final-state gradient
        const float* Lc = L + rl * 256 + jg;
        float o_r[8], o_z[8], o_n[8], o_hn[8], cout[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float dht = Lc[e] + cin[e] + dy[e];
          float rg, omr, zg, omz, ng, sech2;
          tt_sigmoid_pair(ar[e], rg, omr);
          tt_sigmoid_pair(az[e], zg, omz);
          tt_tanh_sech2(an[e], ng, sech2);
          const float dnp = dht * omz * sech2;
          const float drp = dnp * gh[e] * rg * omr;
          const float dzp = dht * (hp[e] - ng) * zg * omz;
          o_r[e] = drp; o_z[e] = dzp; o_n[e] = dnp; o_hn[e] = dnp * rg;
          cout[e] = dht * zg;
          bsum[0][e] += drp; bsum[1][e] += dzp; bsum[2][e] += dnp; bsum[3][e] += dnp * rg;
        }
        if (dbg & 4) {
          if (o_r[0] == 12345.f) L[0] = o_z[1] + o_n[2] + o_hn[3] + cout[4];
          continue;
        }
        st8(cr_cur + (long)b * H + j, cout);
        bf16_t* xw = DGXw + row * a.ldd + j;
        st8(xw, o_r);
        st8(xw + H, o_z);
        const int go = (int)((((long)(b - m0) * T_) * a.ldd + j + 2 * H) * 2L);
        st8_sc1(grs, go, o_n, (bf16_t*)nullptr);
        st8(DGHw + row * a.ldd + j, o_hn);
      }
    }
    __syncthreads();
  }
  // bias partials of the 256-row tile (all into partial row 2*mt; row 2*mt+1 stays zero):
  // lanes l and l^32 share columns
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) bsum[q][e] += __shfl_xor(bsum[q][e], 32, 64);
  float* red = L;  // [8 waves][4][256]
  if (lane < 32) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) red[(wave * 4 + q) * 256 + lane * 8 + e] = bsum[q][e];
  }
  __syncthreads();
  if (tid < 256 && j0 + tid < H) {
    float* pb = R.dbias + (long)(mt * 2) * (4L * H) + j0 + tid;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) v += red[(w * 4 + q) * 256 + tid];
      pb[q * H] += v;
    }
  }
}

// ---- persistent ("row-owning") backward, bf16, H in {256, 512} --------------------
// One launch per layer. A workgroup (8 waves) owns 128 batch rows x ALL H units of one
// recurrence and walks every time step itself: batch rows never interact, so no step
// waits for another workgroup.
// Per step: acc[128 x H] = dL/dgh_{s+1}[128 x 3H] . W_hh[3H x H] on MFMA (A: the rows'
// own gradients of the previous iteration, K-contig, r|z from dgx and n from dgh; B: W_hh,
// K-outer, read from the XCD's L2), then the gate gradients with the accumulator tile
// staged once as a bf16 image through the freed LDS; the step's bias partials are added
// into the tile's partial row. The product runs on 32-deep K-tiles (A 128 rows x 64 B =
// 8 KiB, W_hh 32 k x H = H/128 sub-images of 8 KiB) in a 4-slot LDS ring with three
// K-tiles in flight and counted waits (vmcnt = this wave's DMAs of the younger tiles):
// 7.61 vs 7.81 ms per layer at configs[2] against 64-deep K-tiles in two slots.
//   A image: 64-byte rows, 16-byte chunk c of row r at c ^ ((r >> 1) & 3) (conflict-free
//   for the ds_read_b128 lane groups); W_hh: the K-outer bf16 image of the first 32 k-rows.
// H 1024 (configs[4], the reference's hidden 512): the accumulator of 128 rows x H units
// would be 256 registers per lane, so every step runs in NP = 2 column passes of HP = 512
// units (a pass = the product of the rows' whole dL/dgh_{s+1} with W_hh's columns of the
// pass, then the epilogue of those units); the A operand is streamed once per pass.
template <int H>
struct BwdRowsCfg {
  static constexpr int NP = H > 512 ? H / 512 : 1;  // column passes per step
  static constexpr int HP = H / NP;                 // units per pass
  static constexpr int NQ = HP / 128;
  static constexpr int SLOT = 8192 + NQ * 8192;  // 40 KiB at HP = 512
  static constexpr int NS = 4;
  static constexpr int LDS = NS * SLOT;
  static constexpr int P = SLOT / 1024 / 8;  // DMAs per wave per K-tile
  static constexpr int NCB = HP / 64;
  static constexpr int TPR = HP / 8;
  static constexpr int RPI = 512 / TPR;
  static constexpr int LDB = HP + 8;
  static_assert(SLOT % 8192 == 0 && 128 * LDB * 2 <= LDS && RPI * 4 * HP * 4 <= LDS, "ring layout");
};

TT_DEV uint4 frag_kc64(const char* img, int r0) {  // A fragment of a 32-deep, 64-byte-row image
  const int lane = threadIdx.x & 63;
  const int row = r0 + (lane & 15);
  return *reinterpret_cast<const uint4*>(img + row * 64 + (((lane >> 4) ^ ((row >> 1) & 3)) << 4));
}

template <int N, int P>
TT_DEV void wait_younger(int n) {  // s_waitcnt vmcnt(P * n), n in [0, N]
  if constexpr (N > 0) {
    if (n >= N) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P * N) : "memory");
      return;
    }
    wait_younger<N - 1, P>(n);
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

template <int H>
__global__ __launch_bounds__(512) void gru_bwd_rows(BwdArgs a) {
  using C = BwdRowsCfg<H>;
  __shared__ __attribute__((aligned(16))) char lds[C::LDS];
  const int T_ = a.T, ntm = (a.B + 127) / 128;
  const int id = ttg::xcd_remap(blockIdx.x, gridDim.x);
  const int rz = id / ntm, mt = id - rz * ntm;
  const BwdRec R = a.r[rz];
  const int m0 = mt * 128;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave >> 2, wc = wave & 3;
  const bf16_t* DGX = static_cast<const bf16_t*>(R.dgx);
  const bf16_t* DGH = static_cast<const bf16_t*>(R.dgh);
  bf16_t* DGXw = static_cast<bf16_t*>(R.dgx);
  bf16_t* DGHw = static_cast<bf16_t*>(R.dgh);
  const bf16_t* S = static_cast<const bf16_t*>(R.save);
  const bf16_t* Y = static_cast<const bf16_t*>(R.y);
  const bf16_t* DY = static_cast<const bf16_t*>(R.dy);
  const bf16_t* W = static_cast<const bf16_t*>(R.whh);
  const uint32_t lbase = __builtin_amdgcn_readfirstlane(ttg::lds_addr_of(lds));
  constexpr int NK = 3 * H / 32;  // 32-deep K-tiles per step
  // workgroups in lockstep put every CU in its product phase (L2-bound) at the same time and
  // then in its HBM-bound epilogue; a start skew for half of them interleaves the phases
  // (skew < 0: four phases, |skew| apart)
  if (a.skew != 0) {
    const int ph = a.skew > 0 ? (int)((blockIdx.x >> 3) & 1) : (int)((blockIdx.x >> 3) & 3);
    const int n = ph * (a.skew > 0 ? a.skew : -a.skew);
    for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(127);
  }
  const long ldr = (long)T_ * a.ldd;
  // DMA pieces of a slot, wave + 8j (j < P): piece 0..7 = the A image (row q >> 2, chunk
  // slot q & 3 of 16-byte unit q), then NQ x 8 pieces of W_hh sub-images (k-row q >> 4,
  // chunk slot q & 15)
  int prow[C::P], pcol[C::P];
#pragma unroll
  for (int j = 0; j < C::P; ++j) {
    const int pc = wave + 8 * j, q = (pc & 7) * 64 + lane;
    if (pc < 8) {
      const int row = q >> 2;
      prow[j] = row;
      pcol[j] = ((q & 3) ^ ((row >> 1) & 3)) * 8;
    } else {
      const int sub = (pc - 8) >> 3, kl = q >> 4;
      prow[j] = -1;
      pcol[j] = kl * H + sub * 128 + (((q & 15) ^ (ttg::ko_v(kl) << 1)) * 8);  // + the pass's first unit
    }
  }
  const int jg = (tid % C::TPR) * 8, rsub = tid / C::TPR;
  float* L = reinterpret_cast<float*>(lds);
  float* part = R.dbias + (long)mt * (4L * H);
  const char* zp = reinterpret_cast<const char*>(ttg::g_tt_zero_page);
#ifdef TT_DIAG
  const int dbg = a.dbg;  // diagnostic build only: 1 no GEMM, 2 no epilogue loads, 4 no stores
#else
  constexpr int dbg = 0;
#endif

  // CREG: the BPTT carry dh_s * z_s never leaves the chip. The epilogue writes it (bf16, the
  // rounding of the carry buffer it replaces) over the slot of the accumulator image it has
  // just read for the same (row, units), and the next step's product starts from it: each
  // lane loads its accumulator tile from that image before the first DMA of the step, so
  // the product sums onto the carry (dh = bf16(carry + dL/dgh W_hh) + dy, where the
  // buffer form adds the carry after rounding the product). Saves the carry's 4 of the
  // ~28 bytes per row, unit and step.
  constexpr bool CREG = TT_BWD_CREG != 0 && C::NP == 1;
  constexpr int NIT = 128 / C::RPI;  // epilogue row iterations per thread
  static_assert(!CREG || 128 * C::LDB * 2 + C::RPI * C::HP * 4 <= C::LDS, "carry image + one bias row of partials");
  static_assert(!CREG || C::HP <= 512, "one bias column per thread");
  // CREG: every thread's bias sums (4 gates x its 8 units) run over all its rows of all
  // steps in registers, and the workgroup reduces them across its 8 row groups once, at the
  // end (a per-step reduction cost 8 barriers and an LDS round trip per step)
  float bacc[4][8];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) bacc[q][e] = 0.f;
  for (int s = T_ - 1; s >= 0; --s) {
    const int t = R.dir ? T_ - 1 - s : s;
    const int tn = R.dir ? t - 1 : t + 1;
    const int tp = R.dir ? t + 1 : t - 1;
    const bool last = (s == T_ - 1);
    // one column pass: units [u0, u0 + HP)
    auto column_pass = [&](const int u0) {
    f32x4 acc[4][C::NCB];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < C::NCB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (CREG && !last) {
      // this lane's accumulator tile <- the carry image (C^T layout: 4 consecutive units of
      // one row), then every lane must be done reading before the first DMA overwrites it
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jc = 0; jc < C::NCB; ++jc) {
          const uint2 w = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(lds) +
                                                          (wr * 64 + 16 * i + (lane & 15)) * C::LDB + wc * (C::HP / 4) +
                                                          16 * jc + 4 * (lane >> 4));
          acc[i][jc] = f32x4{__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xFFFF0000u),
                             __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xFFFF0000u)};
        }
      __syncthreads();
    }
    if (!last && !(dbg & 1)) {
#if TT_BWD_BUF
      // the pieces through buffer resources (ttg::dma16_buf): A = the tile's rows at time tn,
      // r|z columns from dgx (k < 2H) or the n column block from dgh (k >= 2H, the resource
      // based 2H columns early so that k indexes it directly), rows past B read zero; W_hh
      // from the pass's first unit; the K-tile advance is the SGPR soffset
      const long abytes = (long)(a.B - m0) * ldr * 2;
      const uint32_t anrec = (uint32_t)(abytes > 0xFFFFFFFFL ? 0xFFFFFFFFL : abytes);
      const ttg::tt_rsrc4 rsx = ttg::make_rsrc4(DGX + (long)tn * a.ldd + (long)m0 * ldr, anrec);
      const ttg::tt_rsrc4 rsh = ttg::make_rsrc4(DGH + (long)tn * a.ldd + (long)m0 * ldr - 2 * H, anrec);
      const ttg::tt_rsrc4 rsw = ttg::make_rsrc4(W + u0, 0xFFFFFFFFu);
      uint32_t voff[C::P];
#pragma unroll
      for (int j = 0; j < C::P; ++j)
        voff[j] = prow[j] >= 0 ? (uint32_t)(((long)prow[j] * ldr + pcol[j]) * 2) : (uint32_t)(pcol[j] * 2);
      auto issue = [&](int r) {
        const uint32_t img = lbase + (uint32_t)(r % C::NS) * C::SLOT;
        const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const bool hi = r * 32 >= 2 * H;
#pragma unroll
        for (int j = 0; j < C::P; ++j) {
          const int pc = wv + 8 * j;
          if (pc < 8) ttg::dma16_buf(hi ? rsh : rsx, voff[j], (uint32_t)r * 64u, img + (uint32_t)pc * 1024u);
          else ttg::dma16_buf(rsw, voff[j], (uint32_t)r * (uint32_t)(64 * H), img + (uint32_t)pc * 1024u);
        }
      };
#else
      // A source of this lane's A pieces: dL/dgh_{s+1} of row m0 + prow, r|z from dgx, n from dgh
      const char* as0[C::P];
      const char* as1[C::P];
#pragma unroll
      for (int j = 0; j < C::P; ++j) {
        const int b = m0 + (prow[j] < 0 ? 0 : prow[j]);
        const bool ok = prow[j] >= 0 && b < a.B;
        as0[j] = ok ? reinterpret_cast<const char*>(DGX + (long)tn * a.ldd + (long)b * ldr + pcol[j]) : zp;
        as1[j] = ok ? reinterpret_cast<const char*>(DGH + (long)tn * a.ldd + (long)b * ldr + pcol[j] - 2 * H) : zp;
      }
      auto issue = [&](int r) {
        const uint32_t img = lbase + (uint32_t)(r % C::NS) * C::SLOT;
        const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const bool hi = r * 32 >= 2 * H;
#pragma unroll
        for (int j = 0; j < C::P; ++j) {
          const int pc = wv + 8 * j;
          const char* src;
          if (pc < 8) {
            src = hi ? as1[j] : as0[j];
            if (src != zp) src += (long)r * 64;  // 32 k of bf16
          } else {
            src = reinterpret_cast<const char*>(W + (long)r * 32 * H + u0 + pcol[j]);
          }
          ttg::dma16(src, img + (uint32_t)pc * 1024u);
        }
      };
#endif
      issue(0);
      issue(1);
      issue(2);
#if TT_BWD_STAG
      // The two wave rows run one barrier apart (wave row 1 late), two barriers per K-tile:
      // each wave reads ALL of K-tile r's fragments after the K-tile's start barrier and
      // retires them before its mid barrier, so one row's reads and DMA issue overlap the
      // other row's MFMAs. Slot (r + 3) % 4 = r - 1's is refilled after K-tile r's start
      // barrier: both rows retired their reads of r - 1 by then. Tile r + 1 must be waited
      // for (every wave, its own pieces) before absolute barrier 2r + 2: the early row's
      // next start barrier, the late row's mid barrier of r.
      const bool late = wr == 1;
      wait_younger<C::NS - 2, C::P>(NK - 1);  // tile 0 landed
      __builtin_amdgcn_s_barrier();
      if (late) __builtin_amdgcn_s_barrier();
#pragma unroll 1
      for (int r = 0; r < NK; ++r) {
        if (r > 0) __builtin_amdgcn_s_barrier();  // start of K-tile r
        if (r + 3 < NK) issue(r + 3);
        const char* sl = lds + (r % C::NS) * C::SLOT;
        uint4 fa[4], fb[C::NCB];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = frag_kc64(sl, wr * 64 + 16 * i);
        const char* ib = sl + 8192 + ((wc * (C::HP / 4)) >> 7) * 8192;
        const int cb = (wc * (C::HP / 4)) & 127;
#pragma unroll
        for (int j = 0; j < C::NCB; ++j) fb[j] = ttg::frag<bf16_t, true>(ib, cb + 16 * j, 0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int j = 0; j < C::NCB / 2; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i][j] = ttg::mma<bf16_t>(fb[j], fa[i], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every read of tile r retired
        __builtin_amdgcn_sched_barrier(0);
        if (late) wait_younger<C::NS - 2, C::P>(NK - 2 - r);  // tile r + 1 landed
        __builtin_amdgcn_s_barrier();                          // mid
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int j = C::NCB / 2; j < C::NCB; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i][j] = ttg::mma<bf16_t>(fb[j], fa[i], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
        if (!late) wait_younger<C::NS - 2, C::P>(NK - 2 - r);  // tile r + 1 landed
      }
      if (!late) __builtin_amdgcn_s_barrier();  // the late row's extra barrier
#else
#pragma unroll 1
      for (int r = 0; r < NK; ++r) {
        wait_younger<C::NS - 2, C::P>(NK - 1 - r);  // tile r landed (up to 2 younger in flight)
        __builtin_amdgcn_s_barrier();               // everyone's; slot (r + 3) % 4 = r - 1's is free
        if (r + 3 < NK) issue(r + 3);
        const char* sl = lds + (r % C::NS) * C::SLOT;
        uint4 fa[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = frag_kc64(sl, wr * 64 + 16 * i);
        const char* ib = sl + 8192 + ((wc * (C::HP / 4)) >> 7) * 8192;
        const int cb = (wc * (C::HP / 4)) & 127;
#pragma unroll
        for (int jp = 0; jp < C::NCB; jp += 2) {
          uint4 fb[2];
#pragma unroll
          for (int j = 0; j < 2; ++j) fb[j] = ttg::frag<bf16_t, true>(ib, cb + 16 * (jp + j), 0);
          __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)  // C^T accumulators: 4 consecutive units of one row per lane
              acc[i][jp + j] = ttg::mma<bf16_t>(fb[j], fa[i], acc[i][jp + j]);
          __builtin_amdgcn_s_setprio(0);
        }
      }
#endif
      __builtin_amdgcn_s_barrier();  // every wave done with the slots before the staging
    }
    // ---- epilogue: as gru_bwd_rows
    const long trow = (long)m0 * T_ + t;
    const __amdgpu_buffer_rsrc_t rc =
        tt_rsrc_n(static_cast<const bf16_t*>(R.dh) + (long)((s + 1) & 1) * a.B * H + (long)m0 * H, !last);
    bf16_t* cr_cur = static_cast<bf16_t*>(R.dh) + (long)(s & 1) * a.B * H + (long)m0 * H;
    const __amdgpu_buffer_rsrc_t rd = tt_rsrc_n(DY ? DY + trow * a.ldy : S, DY != nullptr);
    const __amdgpu_buffer_rsrc_t rsv = tt_rsrc_n(S + trow * 4L * H, true);
    const __amdgpu_buffer_rsrc_t ry = tt_rsrc_n(s > 0 ? Y + ((long)m0 * T_ + tp) * a.ldy : S, s > 0);
    const __amdgpu_buffer_rsrc_t grs = tt_rsrc(DGXw + trow * a.ldd);
    uint32_t* L16 = reinterpret_cast<uint32_t*>(lds);
    // the accumulator as a bf16 image: one 8-byte store of 4 units per (row block, column block)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jc = 0; jc < C::NCB; ++jc) {
        const uint32_t w0 = (uint32_t)f2bf(acc[i][jc][0]) | ((uint32_t)f2bf(acc[i][jc][1]) << 16);
        const uint32_t w1 = (uint32_t)f2bf(acc[i][jc][2]) | ((uint32_t)f2bf(acc[i][jc][3]) << 16);
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(lds) + (wr * 64 + 16 * i + (lane & 15)) * C::LDB +
                                  wc * (C::HP / 4) + 16 * jc + 4 * (lane >> 4)) = make_uint2(w0, w1);
      }
    __syncthreads();
    float bsum_own[4][8];
    auto& bsum = CREG ? bacc : bsum_own;
    if constexpr (!CREG) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e) bsum[q][e] = 0.f;
    }
    constexpr int NB = TT_BWD_NB;  // rows per batch of epilogue loads
    // one epilogue row of this thread (row rsub + RPI k of the tile): its 7 operand loads ...
    auto load_row = [&](const int k, uint4 (&v)[7]) {  // k >= NIT: out of range, reads zero
      const int bl = rsub + C::RPI * k;
      const bool ok = k < NIT && m0 + bl < a.B && !(dbg & 2);
      const uint32_t oc = ok ? (uint32_t)(bl * H + u0 + jg) * 2u : 0x80000000u;
      const uint32_t oy = ok ? (uint32_t)(bl * T_ * (int)a.ldy + u0 + jg) * 2u : 0x80000000u;
      const uint32_t os = ok ? (uint32_t)(bl * T_ * 4 * H + u0 + jg) * 2u : 0x80000000u;
      v[0] = CREG ? make_uint4(0, 0, 0, 0) : ld16_buf(rc, oc, 0);  // CREG: the carry is in gm
      // TT_BWD_NT: non-temporal loads of the once-read streams (1: S, 2: dy and h_{s-1}), so
      // that they do not displace the re-read gate gradients from the caches
      v[1] = ld16_buf<(TT_BWD_NT & 2) ? 2 : 0>(rd, oy, 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[2 + q] = ld16_buf<(TT_BWD_NT & 1) ? 2 : 0>(rsv, os, q * 2 * H);
      v[6] = ld16_buf<(TT_BWD_NT & 2) ? 2 : 0>(ry, oy, 0);
    };
    // ... and its gate math, carry and stores
    auto finish_row = [&](const int k, const uint4 (&v)[7]) {
      const int bl = rsub + C::RPI * k;
      const int b = m0 + bl;
      if (b >= a.B) return;
      float cin[8], dy[8], ar[8], az[8], an[8], gh[8], hp[8], gm[8];
      unpack8(v[0], cin);
      unpack8(v[1], dy);
      unpack8(v[2], ar);
      unpack8(v[3], az);
      unpack8(v[4], an);
      unpack8(v[5], gh);
      unpack8(v[6], hp);
      unpack8(*reinterpret_cast<const uint4*>(L16 + ((bl * C::LDB + jg) >> 1)), gm);
      if (last && R.dfinal) {
        // the fp32 final-state gradient (first step of the launch only), loaded and waited
        // for inside one asm block: a compiler-visible conditional load here would put a
        // vmcnt(0) on every row's path and drain the next row's loads (TT_BWD_PIPE)
        const float* pf = R.dfinal + (long)b * a.ldf + u0 + jg;
        tt_u32x4 d0, d1;
        asm volatile("global_load_dwordx4 %0, %2, off\n\tglobal_load_dwordx4 %1, %2, off offset:16\n\ts_waitcnt vmcnt(0)"
                     : "=&v"(d0), "=&v"(d1)
                     : "v"(pf)
                     : "memory");
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          cin[e] = __uint_as_float(d0[e]);
          cin[4 + e] = __uint_as_float(d1[e]);
        }
      }
      float o_r[8], o_z[8], o_n[8], o_hn[8], cout[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dht = gm[e] + cin[e] + dy[e];
        float rg, omr, zg, omz, ng, sech2;
        tt_sigmoid_pair(ar[e], rg, omr);
        tt_sigmoid_pair(az[e], zg, omz);
        tt_tanh_sech2(an[e], ng, sech2);
        const float dnp = dht * omz * sech2;
        const float drp = dnp * gh[e] * rg * omr;
        const float dzp = dht * (hp[e] - ng) * zg * omz;
        o_r[e] = drp; o_z[e] = dzp; o_n[e] = dnp; o_hn[e] = dnp * rg;
        cout[e] = dht * zg;
        bsum[0][e] += drp; bsum[1][e] += dzp; bsum[2][e] += dnp; bsum[3][e] += dnp * rg;
      }
      if constexpr (CREG)  // over the gm slot this thread just read: the next step's carry
        *reinterpret_cast<uint4*>(L16 + ((bl * C::LDB + jg) >> 1)) = pack8bf(cout);
      if (dbg & 4) {
        if (o_r[0] == 12345.f) L16[0] = __float_as_uint(o_z[1] + o_n[2] + o_hn[3] + cout[4]);
        return;
      }
      if constexpr (!CREG) st8(cr_cur + (long)bl * H + u0 + jg, cout);
      const long row = (long)b * T_ + t;
      bf16_t* xw = DGXw + row * a.ldd + u0 + jg;
      st8_pol<TT_BWD_OUT_NT != 0>(xw, o_r);
      st8_pol<TT_BWD_OUT_NT != 0>(xw + H, o_z);
      st8_sc1(grs, (int)(((long)bl * T_ * a.ldd + u0 + jg + 2 * H) * 2L), o_n, (bf16_t*)nullptr);
      st8_pol<TT_BWD_OUT_NT != 0>(DGHw + row * a.ldd + u0 + jg, o_hn);
    };
    auto batch = [&](const int kb) {
      uint4 vin[NB][7];
#pragma unroll
      for (int kk = 0; kk < NB; ++kk) load_row(kb + kk, vin[kk]);
#pragma unroll
      for (int kk = 0; kk < NB; ++kk) finish_row(kb + kk, vin[kk]);
    };
#if TT_BWD_PIPE
    // rows one ahead: row k+1's loads go out before row k's stores, so the wait for a row's
    // loads never covers the stores of the row before it (one in-order vmcnt)
    static_assert(NIT % 2 == 0, "rows in pairs");
    uint4 vr[2][7];
    load_row(0, vr[0]);
#pragma unroll 1
    for (int k = 0; k < NIT; k += 2) {
      load_row(k + 1, vr[1]);
      finish_row(k, vr[0]);
      load_row(k + 2, vr[0]);  // unconditional (the last pair's is out of range): no branch whose
      finish_row(k + 1, vr[1]);  // merge would make the next wait drain every load
    }
#else
#pragma unroll 1
    for (int kb = 0; kb < NIT; kb += NB) batch(kb);
#endif
    if constexpr (!CREG) {  // (CREG: the step-end barrier below orders the carry image)
      __syncthreads();
      float* red = L;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e) red[(rsub * 4 + q) * C::HP + jg + e] = bsum[q][e];
      __syncthreads();
      for (int c = tid; c < 4 * C::HP; c += 512) {
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < C::RPI; ++w) v += red[w * 4 * C::HP + c];
        part[(c / C::HP) * H + u0 + c % C::HP] += v;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    };
    if constexpr (C::NP == 1) {
      column_pass(0);
    } else {
#pragma unroll 1
      for (int pass = 0; pass < C::NP; ++pass) column_pass(pass * C::HP);
    }
  }
  if constexpr (CREG) {
    // the bias partials one gate row at a time (the LDS is free after the last step)
    float* red = reinterpret_cast<float*>(lds);
#pragma unroll 1
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int e = 0; e < 8; ++e) red[rsub * C::HP + jg + e] = bacc[q][e];
      __syncthreads();
      if (tid < C::HP) {
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < C::RPI; ++w) v += red[w * C::HP + tid];
        part[q * H + tid] = v;
      }
      __syncthreads();
    }
  }
}

// ---- persistent ("row-resident") forward, bf16 ---------------------------------
// Batch rows never interact, so one workgroup can own 64 rows of one recurrence for
// all T steps: h_{s-1} stays in LDS as the A operand (bf16 KC image, never re-read
// from HBM), the fp32 state h_s stays in registers, and only Whh (1.5 MiB per
// recurrence at H=512, L2-resident) is streamed per step. HBM traffic per (row, unit,
// step) drops to what the recurrence must read (G) and write (Y, saved
// pre-activations, dropout copy): 16-18 B instead of 28 B, in one launch instead of T.
//   LDS: Hb 64 KiB (64 rows x H<=512 bf16) | 2 x 24 KiB Whh K-tiles | 48 KiB fp32 gates
// Per step, per block of 64 hidden units: GEMM [64 x 192] += Hb[64 x H] Whh_blk^T
// (8 waves as 2 x 4, wave tile 32 x 48), gates staged through LDS, then every thread
// updates 8 consecutive units of one row with 16-byte global accesses.
constexpr int PR = 64, PH_MAX = 512, PNT = 512;
constexpr int P_HB = PR * PH_MAX * 2;      // 65536
constexpr int P_BST = 192 * ttg::KTB;      // 24576 per stage
constexpr int P_STG = PR * 192 * 4;        // 49152
constexpr int P_LDS = P_HB + 2 * P_BST + P_STG;
static_assert(P_LDS <= 163840, "persistent GRU LDS budget");

// fp32 gate tile [64 rows][48 chunks of 4]: chunk c of row r at c ^ (r & 15)
// (conflict-free for the MFMA-layout writes and the 8-float row reads below).

TT_DEV int stg_off(int row, int col) { return row * 192 + ((((col >> 2) ^ (row & 15))) << 2) + (col & 3); }

// Whh K-tile q = blk*(H/64) + kt of a step, B-tile row (g*64 + u) -> Whh row
// g*H + blk*64 + u; 3 chunks of 16 B per thread.
struct WTile {
  uint4 v0, v1, v2;
};
TT_DEV uint4 fwd_load_chunk(const bf16_t* W, int H, int blk, int kt, int i) {
  const int id = threadIdx.x + PNT * i, c = id & 7, row = id >> 3;
  const int g = row >> 6, u = row & 63;
  return *reinterpret_cast<const uint4*>(W + (long)(g * H + blk * 64 + u) * H + kt * 64 + c * 8);
}
TT_DEV void fwd_load_b(const bf16_t* W, int H, int q, WTile& r) {
  const int nkt = H >> 6, blk = q / nkt, kt = q - blk * nkt;
  r.v0 = fwd_load_chunk(W, H, blk, kt, 0);
  r.v1 = fwd_load_chunk(W, H, blk, kt, 1);
  r.v2 = fwd_load_chunk(W, H, blk, kt, 2);
}
TT_DEV void fwd_store_b(char* img, const WTile& r) {
  const int t = threadIdx.x;
  *reinterpret_cast<uint4*>(img + ttg::kc_off(t >> 3, t & 7)) = r.v0;
  *reinterpret_cast<uint4*>(img + ttg::kc_off((t + PNT) >> 3, t & 7)) = r.v1;
  *reinterpret_cast<uint4*>(img + ttg::kc_off((t + 2 * PNT) >> 3, t & 7)) = r.v2;
}
// One K-tile of the step GEMM: prefetch K-tile q+D into register set Y (wrapping into
// the next step; the very last prefetches are harmless reloads, unconditional so the
// sets stay in registers), MFMAs on LDS stage it&1, then K-tile q+1 (set X, loaded
// D-1 tiles ago) into the other stage.
#ifdef TT_DIAG
// diagnostic build only: per-phase s_memtime totals of wave 0 of every workgroup
__device__ unsigned long long g_fwd_prof[2048][8];
#define TT_STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define TT_ACC(i, d) (prf[i] += (d))
#define TT_PROF_PARAM , unsigned long long (&prf)[8], int dbg
#define TT_PROF_ARGS , prf, a.dbg
#else
#define TT_STAMP(v) do { } while (0)
#define TT_ACC(i, d) do { } while (0)
#define TT_PROF_PARAM
#define TT_PROF_ARGS
#endif
template <int D>
TT_DEV void fwd_kstep(const bf16_t* W, int H, int Q, int q, int kt, bool mm, const char* hb, char* bst, int& it,
                      int wm, int wn, f32x4 (&acc)[2][3], WTile& X, WTile& Y TT_PROF_PARAM) {
  TT_STAMP(t0);
#ifdef TT_DIAG
  if (!(dbg & 16)) fwd_load_b(W, H, (q + D) % Q, Y);  // 16: no W_hh loads
  if (dbg & 8) mm = false;                            // 8: no MFMAs
#else
  fwd_load_b(W, H, (q + D) % Q, Y);
#endif
  if (mm) {  // h_{-1} = 0: the first step has no recurrent term
    const char* ia = hb + kt * (PR * ttg::KTB);
    const char* ib = bst + (it & 1) * P_BST;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 fa[2], fb[3];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = ttg::frag<bf16_t, false>(ia, wm + 16 * i, ks);
#pragma unroll
      for (int j = 0; j < 3; ++j) fb[j] = ttg::frag<bf16_t, false>(ib, wn + 16 * j, ks);
      __builtin_amdgcn_s_setprio(1);  // ≈ 1 % (profiles/r02_gru_fwd_prio_ab.txt)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)  // operands swapped: acc holds C^T (4 gate columns of a row per lane)
          acc[i][j] = ttg::mma<bf16_t>(fb[j], fa[i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  TT_STAMP(t1);
  fwd_store_b(bst + ((it + 1) & 1) * P_BST, X);
  TT_STAMP(t2);
  __syncthreads();
  TT_STAMP(t3);
  TT_ACC(0, t1 - t0);  // W_hh load issue + fragment reads + MFMA
  TT_ACC(1, t2 - t1);  // wait for the ring set + its LDS store
  TT_ACC(2, t3 - t2);  // barrier
  ++it;
}

// Whh K-tiles in flight in registers: 1, 2 or 4 (D divides H/64); NKT = H/64 when known
// at compile time (0: runtime). A compile-time NKT unrolls the block's K loop, so hipcc's
// vmcnt bookkeeping at its first K-tiles counts the previous block's epilogue stores and
// the gate loads exactly instead of the loop-merged minimum: with one in-order counter
// that minimum made the first W_hh waits of every block also wait for those stores.
template <int D, int NKT>
__global__ __launch_bounds__(PNT) void gru_fwd_seq(FwdArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[P_LDS];
  char* hb = lds;
  char* bst = lds + P_HB;
  float* stg = reinterpret_cast<float*>(lds + P_HB + 2 * P_BST);
  const int ntm = (a.B + PR - 1) / PR;
  const int id = ttg::xcd_remap(blockIdx.x, gridDim.x);
  const int rz = id / ntm;
  const FwdRec R = a.r[rz];
  const int H = a.H, T_ = a.T;
  const int m0 = (id - rz * ntm) * PR;
  const int nblk = NKT ? NKT : H / 64, nkt = NKT ? NKT : H / 64, Q = nblk * nkt;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = (wave >> 2) * 32, wn = (wave & 3) * 48;
  const bf16_t* W = static_cast<const bf16_t*>(R.whh);
  const bf16_t* G = static_cast<const bf16_t*>(R.g);
  bf16_t* Yw = static_cast<bf16_t*>(R.y);
  bf16_t* X1 = static_cast<bf16_t*>(R.x1);
  bf16_t* S = static_cast<bf16_t*>(R.save);
  // epilogue ownership: row rl, units blk*64 + jg .. +8 of every block
  const int rl = tid >> 3, jg = (tid & 7) * 8;
  const int b = m0 + rl;
  const bool rowok = b < a.B;
  // gate inputs and outputs through buffer resources based at this workgroup's first
  // row: no branches around the memory instructions (a tail row's offset is out of
  // range, so it reads zeros and its stores are dropped; no X1 = num_records 0), so
  // every wave issues the same count and the waits above stay exact
  const long r0w = (long)m0 * T_;
  const __amdgpu_buffer_rsrc_t rG = tt_rsrc_n(G + r0w * a.ldg, true);
  const __amdgpu_buffer_rsrc_t rY = tt_rsrc_n(Yw + r0w * a.ldy, true);
  const __amdgpu_buffer_rsrc_t rX1 = tt_rsrc_n(X1 ? X1 + r0w * a.ldy : Yw, X1 != nullptr);
  const __amdgpu_buffer_rsrc_t rS = tt_rsrc_n(S + r0w * 4L * H, true);
#ifdef TT_DIAG
  const bool gok = rowok && !(a.dbg & 2), sok = rowok && !(a.dbg & 1);
#else
  const bool gok = rowok, sok = rowok;
#endif

  float hreg[PH_MAX / 64][8];
#pragma unroll
  for (int i = 0; i < PH_MAX / 64; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) hreg[i][e] = 0.f;

  WTile r0, r1, r2, r3;
  fwd_load_b(W, H, 0, r0);
  fwd_store_b(bst, r0);
  if (D >= 2) fwd_load_b(W, H, 1 % Q, r1);
  if (D >= 4) {
    fwd_load_b(W, H, 2 % Q, r2);
    fwd_load_b(W, H, 3 % Q, r3);
  }
  int it = 0;  // running K-tile counter: Whh stage = it & 1
#ifdef TT_DIAG
  unsigned long long prf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  TT_STAMP(k_start);
#endif
  __syncthreads();
  // six dropped stores (out-of-range offset) stand in for the epilogue's six, so every
  // path into a block's first K-tiles has the same pending count and hipcc's waits
  // there leave the stores in flight
#pragma unroll
  for (int q = 0; q < 6; ++q) st16_buf(rY, 0x80000000u + 16u * q, 0, make_uint4(0, 0, 0, 0));

  for (int s = 0; s < T_; ++s) {
    const int t = R.dir ? T_ - 1 - s : s;
    const long row = (long)b * T_ + t;
    const int lrow = rl * T_ + t;  // row within this workgroup's resources
#pragma unroll 1
    for (int blk = 0; blk < nblk; ++blk) {
      // gate inputs of this block's epilogue, issued before the GEMM so they land under it
      uint4 gx[3];
      const uint32_t og = gok ? (uint32_t)(lrow * (int)a.ldg + blk * 64 + jg) * 2u : 0x80000000u;
#pragma unroll
      for (int g = 0; g < 3; ++g) gx[g] = ld16_buf(rG, og, g * H * 2);
      // b_hn with them: a load issued after the K loop would make its wait drain the
      // W_hh ring prefetches too (one in-order vmcnt)
      const float4 bn0 = *reinterpret_cast<const float4*>(R.bhn + blk * 64 + jg);
      const float4 bn1 = *reinterpret_cast<const float4*>(R.bhn + blk * 64 + jg + 4);
      f32x4 acc[2][3];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      // ring of D register sets: iteration q reads set (q+1)%D, refills set q%D
#define TT_KS(j, X, Y) fwd_kstep<D>(W, H, Q, blk * nkt + kt + j, kt + j, s > 0, hb, bst, it, wm, wn, acc, X, Y TT_PROF_ARGS)
      if constexpr (D == 1) {
#pragma unroll
        for (int kt = 0; kt < nkt; ++kt) TT_KS(0, r0, r0);
      } else if constexpr (D == 2) {
#pragma unroll
        for (int kt = 0; kt < nkt; kt += 2) {
          TT_KS(0, r1, r0);
          TT_KS(1, r0, r1);
        }
      } else {
#pragma unroll
        for (int kt = 0; kt < nkt; kt += 4) {
          TT_KS(0, r1, r0);
          TT_KS(1, r2, r1);
          TT_KS(2, r3, r2);
          TT_KS(3, r0, r3);
        }
      }
#undef TT_KS
      TT_STAMP(e0);
      // gates -> LDS (fp32), then per-thread rows
      // (C^T accumulators: one 16-byte store per block instead of four 4-byte ones; ≈ 0.4 %,
      // bit-identical, profiles/r02_gru_fwd_ct_ab.txt)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
          *reinterpret_cast<f32x4*>(stg + stg_off(wm + 16 * i + (lane & 15), wn + 16 * j + 4 * (lane >> 4))) =
              acc[i][j];
      __syncthreads();
      TT_STAMP(e1);
      TT_ACC(3, e1 - e0);  // gate staging + barrier
      const int j = blk * 64 + jg;
      float xr[8], xz[8], xn[8], bn[8], lr[8], lz[8], ln[8], y[8], sr[8], sz[8], sn[8], sg[8];
      unpack8(gx[0], xr);
      unpack8(gx[1], xz);
      unpack8(gx[2], xn);
      bn[0] = bn0.x; bn[1] = bn0.y; bn[2] = bn0.z; bn[3] = bn0.w;
      bn[4] = bn1.x; bn[5] = bn1.y; bn[6] = bn1.z; bn[7] = bn1.w;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float4 v0 = *reinterpret_cast<const float4*>(stg + stg_off(rl, 0 * 64 + jg + 4 * h));
        const float4 v1 = *reinterpret_cast<const float4*>(stg + stg_off(rl, 1 * 64 + jg + 4 * h));
        const float4 v2 = *reinterpret_cast<const float4*>(stg + stg_off(rl, 2 * 64 + jg + 4 * h));
        lr[4 * h] = v0.x; lr[4 * h + 1] = v0.y; lr[4 * h + 2] = v0.z; lr[4 * h + 3] = v0.w;
        lz[4 * h] = v1.x; lz[4 * h + 1] = v1.y; lz[4 * h + 2] = v1.z; lz[4 * h + 3] = v1.w;
        ln[4 * h] = v2.x; ln[4 * h + 1] = v2.y; ln[4 * h + 2] = v2.z; ln[4 * h + 3] = v2.w;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
#ifdef TT_DIAG
        if (a.dbg & 4) {  // 4: no transcendentals (cheap stand-ins keep the data flow)
          sg[e] = ln[e] + bn[e];
          sr[e] = xr[e] + lr[e]; sz[e] = xz[e] + lz[e];
          const float rg = sr[e] * 0.25f + 0.5f, zg = sz[e] * 0.25f + 0.5f;
          sn[e] = xn[e] + rg * sg[e];
          y[e] = (1.f - zg) * sn[e] * 0.5f + zg * hreg[0][e];
          continue;
        }
#endif
        gru_cell(xr[e], xz[e], xn[e], lr[e], lz[e], ln[e], bn[e], hreg[0][e], y[e], sr[e], sz[e], sn[e], sg[e]);
      }
      float ynew[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) ynew[e] = y[e];
      {
        const uint32_t oy = sok ? (uint32_t)(lrow * (int)a.ldy + j) * 2u : 0x80000000u;
        const uint32_t os = sok ? (uint32_t)(lrow * 4 * H + j) * 2u : 0x80000000u;
        st16_buf(rY, oy, 0, pack8bf(y));
        st16_buf(rS, os, 0, pack8bf(sr));
        st16_buf(rS, os, 2 * H, pack8bf(sz));
        st16_buf(rS, os, 4 * H, pack8bf(sn));
        st16_buf(rS, os, 6 * H, pack8bf(sg));
        if (X1 && a.drop_thresh) {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            y[e] *= tt_dropout_scale(R.seed, R.row0 + (uint32_t)row, (uint32_t)(R.col0 + j + e), a.drop_thresh,
                                     a.inv_keep);
        }
        st16_buf(rX1, oy, 0, pack8bf(y));
      }
      TT_STAMP(e2);
      TT_ACC(4, e2 - e1);  // gate math + stores issued
      // stg is rewritten only after the next block's K loop (whose barriers order it)
      // the state of block blk moves to the back: hreg[0] is always the current block
#pragma unroll
      for (int i = 0; i < PH_MAX / 64 - 1; ++i)
#pragma unroll
        for (int e = 0; e < 8; ++e) hreg[i][e] = hreg[i + 1][e];
#pragma unroll
      for (int e = 0; e < 8; ++e) hreg[PH_MAX / 64 - 1][e] = ynew[e];
    }
    for (int r = nblk; r < PH_MAX / 64; ++r) {  // complete the rotation: hreg[b] = block b
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = hreg[0][e];
#pragma unroll
        for (int i = 0; i < PH_MAX / 64 - 1; ++i) hreg[i][e] = hreg[i + 1][e];
        hreg[PH_MAX / 64 - 1][e] = v;
      }
    }
    // h_s -> A operand of step s+1 (every wave finished reading h_{s-1}: the last
    // K-tile ended with a barrier)
#pragma unroll
    for (int i = 0; i < PH_MAX / 64; ++i) {
      if (i < nblk) {
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          w[k] = (uint32_t)f2bf(hreg[i][2 * k]) | ((uint32_t)f2bf(hreg[i][2 * k + 1]) << 16);
        *reinterpret_cast<uint4*>(hb + i * (PR * ttg::KTB) + ttg::kc_off(rl, tid & 7)) =
            make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
    __syncthreads();
  }
#ifdef TT_DIAG
  TT_STAMP(k_end);
  prf[7] = k_end - k_start;
  if (threadIdx.x == 0 && blockIdx.x < 2048)
    for (int i = 0; i < 8; ++i) g_fwd_prof[blockIdx.x][i] = prf[i];
#endif
}

// ---- column-split persistent forward (gru_fwd_xc, bf16, H 256 / 512) ----------------
// Every other forward here gives a workgroup a set of batch rows and all 3H gate columns,
// so each workgroup re-streams the whole W_hh (1.5 MiB at H 512) from L2 at every step:
// that stream, ~30 GB/s into a CU, is what bounds gru_fwd_seq. Here the
// split is the other way round. A group of M = H/64 workgroups (one per CU, all on one XCD
// under round-robin placement -- speed only, never correctness) shares a block of batch
// rows; member m owns hidden units [64m, 64m+64) and keeps its 192 W_hh rows (r, z, n of
// those units; 192 KiB at H 512) in the accumulator registers of its 4 waves for the whole
// launch. Per step the members exchange h instead: each writes its 64 units of h_s for the
// block's rows to a group image (16-byte write-through stores), drains, and bumps the
// group's arrival counter; before step s+1 every member waits for all M arrivals and reads
// the full h_s rows back (16-byte write-through loads, so no L1 line can be stale:
// cdna_hip_programming.md §6 Guideline 16 / MI355X_MICROARCH.md, hand-off table row 1).
// That is H*2 bytes of L2 traffic per row and step instead of the whole W_hh per 64 rows.
//   rows : the group's rows run in rounds of RR = 256 (fp32 state of a round in LDS), each
//          round in chunks of 32 rows: h chunk -> LDS (double-buffered) -> MFMA
//          (acc = C^T: 4 consecutive units of one row per lane) -> gates staged in LDS ->
//          every thread updates 8 consecutive units of one row with 16-byte G / Y / S / X1
//          accesses (full 128-byte lines per row and member)
//   order: the MFMAs of chunk c+1 are issued ahead of chunk c's gate arithmetic, so the
//          matrix pipe and the VALU run side by side in each wave
// Same MFMA sequence along k (K-steps of 32 in order, from zero) and the same gru_cell as
// the per-step kernel, so every output is bit-identical to it (tests/test_gpu_gru_persistent.py).
// Needs all groups resident at once: one workgroup per CU (the LDS use forbids two), grid =
// 8 * M * (CUs / 8M) <= CUs, checked against the occupancy query and launched cooperatively
// (the runtime rejects a grid that cannot be co-resident; tt_gru_fwd then runs the row-owning
// gru_fwd_seq). Every wait is bounded: a wait that gives up marks the launch (per-launch flag,
// so the rest of the launch drains quickly) and sets the caller's status word (sticky).
typedef __attribute__((address_space(1))) unsigned xc_gu32;
#ifndef XC_G_AUX  // cache policy of the column-split forward's G loads (2: non-temporal, measured 2% faster)
#define XC_G_AUX 2
#endif
#ifndef XC_OUT_AUX  // cache policy of the column-split forward's Y / S / X1 stores (2: non-temporal):
#define XC_OUT_AUX 2  // plain stores evicted the group's h images from L2 before the members read them
#endif                // (fetch 8.61 -> 6.52 GB per launch, 9.70 -> 9.65 ms per step; profiles/r06_xs_out_policy_ab.txt)
#ifndef XC_VALU_PER_MFMA
#define XC_VALU_PER_MFMA 3
#endif
namespace xc {
constexpr int NT = 256;                // 4 waves, one per SIMD
constexpr int CR = 32;                 // batch rows per chunk (8 epilogue threads per row)
constexpr int RR = 256;                // batch rows per round
constexpr int NCH = RR / CR;           // chunks per round
constexpr int SSTR = 68;               // LDS fp32 state row stride (64 units + 16 B pad)
constexpr int STG = CR * 192 * 4;      // gate staging [32 rows][192 columns] fp32
constexpr int CSTR = 64;               // per-group counter words (256 B): [0..2] counters, [8 + m] member XCDs (m < 32)
constexpr unsigned OOB = 0x80000000u;  // buffer offset past num_records: load 0 / store dropped
template <int H>
struct Cfg {
  static constexpr int M = H / 64;         // members per group
  static constexpr int NKT = H / 32;       // MFMA K-steps
  static constexpr int QPW = H / 64;       // 1-KiB h pieces per wave and chunk
  static constexpr int SLOT = CR * H * 2;  // h chunk image: [K-step][row block][16 B x 64 lanes]
  static constexpr int ST = RR * SSTR * 4;
  static constexpr int LDS = ST + 2 * SLOT + STG;
};
static_assert(Cfg<512>::LDS <= 163840 && Cfg<256>::LDS <= 163840, "gru_fwd_xc LDS budget");
}  // namespace xc

struct XcWs {
  bf16_t* xb;        // [groups][2][RR][H] h exchange images (parity = step index & 1)
  unsigned* cnt;     // [groups][CSTR] arrival counters, zeroed before every launch
  unsigned* err;     // this launch gave up a wait (zeroed with the counters)
  unsigned* status;  // the caller's status word: set on a timeout, never cleared here
  unsigned spins;    // polls before a wait gives up
  int skip;          // diagnostic: member skip-1 of group 0 never publishes (0: off)
  int xmap;          // members of a group are consecutive blocks (dealt over the XCDs)
  int qg;         // groups per XCD
  int nrec;       // recurrences (groups are dealt to them round-robin)
  int rpg;        // batch rows per group
  int nround;     // rounds of RR rows per group
  int fast_ok;    // the exchange may stay in the XCD's L2 where the group shares one
  int skew;       // odd groups start skew x s_sleep(127) late (option gru_fwd_skew; speed only)
};

TT_DEV void xc_wait(xc_gu32* cnt, unsigned target, const XcWs& ws) {
  xc_gu32* err = (xc_gu32*)(uintptr_t)ws.err;
  for (unsigned spins = 0;; ++spins) {
    if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return;
    if ((spins & 1023u) == 1023u) {
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
      if (spins > ws.spins) {  // 2^22 polls: several seconds, a member never arrived
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_or((xc_gu32*)(uintptr_t)ws.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Whether every member of a group runs on one XCD (HW_REG_XCC_ID), decided identically by
// all members at launch start: then the exchange images may be written with plain stores,
// which keep the lines in that XCD's L2 (the members' write-through loads bypass only their
// own L1, so they read the L2 copy); otherwise every image store is write-through (sc1) and
// the readers fetch from the Infinity Cache. Placement changes only the speed, never the
// result. Counter words: [0] step arrivals, [1] start arrivals, [8 + m] member m's XCD + 1.
TT_DEV bool xc_group_on_one_xcd(unsigned* cntw, int M, int mem, bool allowed, const XcWs& ws) {
  __shared__ int s_fast;
  if (threadIdx.x == 0) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xc_gu32* w = (xc_gu32*)(uintptr_t)cntw;
    __hip_atomic_store(w + 8 + mem, (xcc & 15u) + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(w + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    xc_wait(w + 1, (unsigned)M, ws);
    unsigned first = __hip_atomic_load(w + 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool same = allowed && first != 0u;
    for (int m = 1; m < M; ++m) same &= __hip_atomic_load(w + 8 + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == first;
    s_fast = same ? 1 : 0;
  }
  __syncthreads();
  return s_fast != 0;
}

// h rows [32c, 32c+32) of an exchange image -> registers (write-through loads): piece p of
// wave w is K-step kt, row block rb of the chunk image, one 16-byte MFMA fragment per lane
// (per-piece lane offsets ho[p] computed once; the chunk offset is a constant)
template <int H>
TT_DEV void xc_h_offsets(uint32_t (&ho)[xc::Cfg<H>::QPW]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int p = 0; p < xc::Cfg<H>::QPW; ++p) {
    const int q = w * xc::Cfg<H>::QPW + p, kt = q >> 1, rb = q & 1;
    ho[p] = (uint32_t)(((rb * 16 + (lane & 15)) * H + kt * 32 + (lane >> 4) * 8) * 2);
  }
}
template <int H>
TT_DEV void xc_load_h(__amdgpu_buffer_rsrc_t rx, const uint32_t (&ho)[xc::Cfg<H>::QPW], int c,
                      tt_u32x4 (&hv)[xc::Cfg<H>::QPW]) {
#pragma unroll
  for (int p = 0; p < xc::Cfg<H>::QPW; ++p)
    hv[p] = __builtin_amdgcn_raw_buffer_load_b128(rx, (int)ho[p], c * xc::CR * H * 2, 16);
}
template <int H>
TT_DEV void xc_put_h(char* slot, const tt_u32x4 (&hv)[xc::Cfg<H>::QPW]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int p = 0; p < xc::Cfg<H>::QPW; ++p)
    *reinterpret_cast<tt_u32x4*>(slot + (w * xc::Cfg<H>::QPW + p) * 1024 + lane * 16) = hv[p];
}
// gh^T of the chunk's 32 rows x this wave's 48 gate columns (16 units x r, z, n); the
// fragments of K-step kt+2 are requested before the MFMAs of kt (LDS latency off the chain)
template <int H>
TT_DEV void xc_mfma(const char* slot, const tt_u32x4 (&wa)[3][xc::Cfg<H>::NKT], f32x4 (&acc)[2][3]) {
  constexpr int NKT = xc::Cfg<H>::NKT;
  const int lane = threadIdx.x & 63;
  auto frag = [&](int kt, int rb) {
    return *reinterpret_cast<const tt_u32x4*>(slot + (kt * 2 + rb) * 1024 + lane * 16);
  };
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int g = 0; g < 3; ++g) acc[rb][g] = f32x4{0.f, 0.f, 0.f, 0.f};
  tt_u32x4 f[3][2];
  f[0][0] = frag(0, 0); f[0][1] = frag(0, 1);
  f[1][0] = frag(1, 0); f[1][1] = frag(1, 1);
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    if (kt + 2 < NKT) {
      f[(kt + 2) % 3][0] = frag(kt + 2, 0);
      f[(kt + 2) % 3][1] = frag(kt + 2, 1);
    }
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int g = 0; g < 3; ++g)
        acc[rb][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8v, wa[g][kt]),
                                                             __builtin_bit_cast(bf16x8v, f[kt % 3][rb]), acc[rb][g], 0, 0, 0);
  }
}
TT_DEV void xc_stage(float* stg, const f32x4 (&acc)[2][3]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int g = 0; g < 3; ++g)
      *reinterpret_cast<f32x4*>(stg + stg_off(rb * 16 + (lane & 15), g * 64 + 16 * w + 4 * (lane >> 4))) = acc[rb][g];
}


// gru_fwd_xcp: gru_fwd_xc with the step boundary pipelined away. The chunks of all steps
// form one stream: the h chunks three ahead are requested across the step boundary, the
// MFMAs of the next step's first chunk are woven into this step's last gate arithmetic, and
// the members publish each half step (chunks 0-3, 4-7) on its own counter, so a member
// waits for the first half of step s only while it computes the second half of step s-1
// of its own. Same arithmetic, same order, same outputs as gru_fwd_xc (bit-identical).
template <int H, bool DROP>
__global__ __launch_bounds__(xc::NT, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void gru_fwd_xcp(FwdArgs a, XcWs ws) {
  using C = xc::Cfg<H>;
  constexpr int M = C::M, NKT = C::NKT;
  __shared__ __attribute__((aligned(16))) char lds[C::LDS];
  float* stt = reinterpret_cast<float*>(lds);
  char* slots = lds + C::ST;
  float* stg = reinterpret_cast<float*>(lds + C::ST + 2 * C::SLOT);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  uint32_t ho[C::QPW];
  xc_h_offsets<H>(ho);
  // group / member: blocks b and b + 8 share an XCD under round-robin placement, so a
  // group's members are blocks x, x + 8, ... (xmap: consecutive blocks, one per XCD -- the
  // cross-XCD exchange, for tests)
  const int xcd = blockIdx.x & 7, jj = blockIdx.x >> 3;
  const int grp = ws.xmap ? (int)blockIdx.x / M : xcd * ws.qg + jj / M;
  const int mem = ws.xmap ? (int)blockIdx.x % M : jj % M;
  const int rz = grp % ws.nrec, gi = grp / ws.nrec;
  const FwdRec R = a.r[rz];
  const int T_ = a.T, B = a.B;
  const int gb0 = gi * ws.rpg;
  xc_gu32* cw = (xc_gu32*)(uintptr_t)(ws.cnt + grp * xc::CSTR);
  xc_gu32* cntA = cw;      // arrivals of half steps A (chunks 0-3)
  xc_gu32* cntB = cw + 2;  // and B (chunks 4-7)
  const bool publish = !(grp == 0 && mem == ws.skip - 1);  // diagnostic skip: never counted in
  bf16_t* xbg = ws.xb + (long)grp * 2 * xc::RR * H;
  const __amdgpu_buffer_rsrc_t rx[2] = {tt_rsrc(xbg), tt_rsrc(xbg + xc::RR * H)};
  tt_u32x4 wa[3][NKT];
  {
    const bf16_t* W = static_cast<const bf16_t*>(R.whh);
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
        wa[g][kt] = *reinterpret_cast<const tt_u32x4*>(
            W + (long)(g * H + 64 * mem + 16 * wave + (lane & 15)) * H + kt * 32 + (lane >> 4) * 8);
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) asm volatile("" : "+a"(wa[g][kt]));
  }
  const int cr = tid >> 3, u0 = (tid & 7) * 8, j = 64 * mem + u0;
  float bn[8];
  {
    const float4 b0 = *reinterpret_cast<const float4*>(R.bhn + j);
    const float4 b1 = *reinterpret_cast<const float4*>(R.bhn + j + 4);
    bn[0] = b0.x; bn[1] = b0.y; bn[2] = b0.z; bn[3] = b0.w;
    bn[4] = b1.x; bn[5] = b1.y; bn[6] = b1.z; bn[7] = b1.w;
  }
  const bf16_t* G = static_cast<const bf16_t*>(R.g);
  bf16_t* Yw = static_cast<bf16_t*>(R.y);
  bf16_t* X1 = static_cast<bf16_t*>(R.x1);
  bf16_t* S = static_cast<bf16_t*>(R.save);
  const bool fast = xc_group_on_one_xcd(ws.cnt + grp * xc::CSTR, M, mem, ws.fast_ok != 0, ws);
  // every member of a group is delayed alike (they wait for each other at every step)
  if (ws.skew > 0 && (grp & 1))
    for (int i = 0; i < ws.skew; ++i) __builtin_amdgcn_s_sleep(127);
  const int NS = ws.nround * T_;  // steps over all rounds
  // step idx -> its step in the round, time, first batch row, rows
  struct Step {
    int s, t, rb0, nrow;
  };
  auto step_of = [&](int idx) {
    Step q;
    const int r = idx / T_;
    q.s = idx - r * T_;
    q.t = R.dir ? T_ - 1 - q.s : q.s;
    q.rb0 = gb0 + r * xc::RR;
    q.nrow = min(min(ws.rpg - r * xc::RR, xc::RR), B - q.rb0);
    return q;
  };
  auto g_rsrc = [&](const Step& q) {
    return tt_rsrc_n(G + (long)(q.nrow > 0 ? q.rb0 : 0) * T_ * a.ldg, q.nrow > 0);
  };
  auto load_g = [&](const Step& q, __amdgpu_buffer_rsrc_t rG, int c, tt_u32x4 (&gx)[3]) {
    const uint32_t og = c * xc::CR + cr < q.nrow ? (uint32_t)(((c * xc::CR + cr) * T_ + q.t) * (int)a.ldg + j) * 2u
                                                  : xc::OOB;
#pragma unroll
    for (int g = 0; g < 3; ++g) gx[g] = __builtin_amdgcn_raw_buffer_load_b128(rG, (int)og, g * H * 2, XC_G_AUX);
  };
  // h chunk c of step q (from the image of step idx - 1), or zeros at a round's first step
  tt_u32x4 hv[C::QPW];
  auto load_h = [&](const Step& q, int qidx, int c) {
    if (q.s == 0) {
#pragma unroll
      for (int p = 0; p < C::QPW; ++p) hv[p] = tt_u32x4{0u, 0u, 0u, 0u};
    } else {
      xc_load_h<H>(rx[(qidx - 1) & 1], ho, c, hv);
    }
  };
  float lr[8], lz[8], ln[8], hp[8];
  auto read_gates = [&](int c, bool first) {  // first: h_{-1} = 0 (the round's state is stale)
    const int rr = c * xc::CR + cr;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 v0 = *reinterpret_cast<const float4*>(stg + stg_off(cr, 0 * 64 + u0 + 4 * h));
      const float4 v1 = *reinterpret_cast<const float4*>(stg + stg_off(cr, 1 * 64 + u0 + 4 * h));
      const float4 v2 = *reinterpret_cast<const float4*>(stg + stg_off(cr, 2 * 64 + u0 + 4 * h));
      const float4 p = *reinterpret_cast<const float4*>(stt + rr * xc::SSTR + u0 + 4 * h);
      lr[4 * h] = v0.x; lr[4 * h + 1] = v0.y; lr[4 * h + 2] = v0.z; lr[4 * h + 3] = v0.w;
      lz[4 * h] = v1.x; lz[4 * h + 1] = v1.y; lz[4 * h + 2] = v1.z; lz[4 * h + 3] = v1.w;
      ln[4 * h] = v2.x; ln[4 * h + 1] = v2.y; ln[4 * h + 2] = v2.z; ln[4 * h + 3] = v2.w;
      hp[4 * h] = first ? 0.f : p.x; hp[4 * h + 1] = first ? 0.f : p.y;
      hp[4 * h + 2] = first ? 0.f : p.z; hp[4 * h + 3] = first ? 0.f : p.w;
    }
  };
  f32x4 acc[2][3];
  // ---- prologue: step 0's chunks 0-2 are zero h (slots zeroed), its gate inputs 0
  for (int i = tid; i < 2 * C::SLOT / 16; i += xc::NT)
    reinterpret_cast<float4*>(slots)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  Step cur = step_of(0);
  __amdgpu_buffer_rsrc_t rGc = g_rsrc(cur);
  tt_u32x4 gq[2][3];
  load_g(cur, rGc, 0, gq[0]);
#pragma unroll
  for (int p = 0; p < C::QPW; ++p) hv[p] = tt_u32x4{0u, 0u, 0u, 0u};
  __syncthreads();
  xc_mfma<H>(slots, wa, acc);
  xc_stage(stg, acc);
  __syncthreads();
  read_gates(0, true);
  for (int idx = 0; idx < NS; ++idx) {
    const bool has_next = idx + 1 < NS;
    const Step nxt = step_of(has_next ? idx + 1 : idx);
    const __amdgpu_buffer_rsrc_t rGn = g_rsrc(nxt);
    const long r0w = (long)(cur.nrow > 0 ? cur.rb0 : 0) * T_;
    const bool on = cur.nrow > 0;
    const __amdgpu_buffer_rsrc_t rY = tt_rsrc_n(Yw + r0w * a.ldy, on);
    const __amdgpu_buffer_rsrc_t rX1 = tt_rsrc_n(X1 ? X1 + r0w * a.ldy : Yw, on && X1 != nullptr);
    const __amdgpu_buffer_rsrc_t rS = tt_rsrc_n(S + r0w * 4L * H, on);
    const __amdgpu_buffer_rsrc_t rdst_h = rx[idx & 1];
    const int t = cur.t;
#pragma unroll
    for (int c = 0; c < xc::NCH; ++c) {
      const bool more = c + 1 < xc::NCH || has_next;  // a chunk follows in the stream
      // gate inputs of the next chunk (one ahead, two sets)
      if (c + 1 < xc::NCH) load_g(cur, rGc, c + 1, gq[(c + 1) & 1]);
      else if (has_next) load_g(nxt, rGn, 0, gq[0]);
      {
        const int rr = c * xc::CR + cr;
        const bool ok = rr < cur.nrow;
        float xr[8], xz[8], xn[8], y[8], sr[8], sz[8], sn[8], sg[8], msk[8];
        const uint32_t grow = (uint32_t)(cur.rb0 + rr) * (uint32_t)T_ + (uint32_t)t;
        const tt_u32x4(&gcur)[3] = gq[c & 1];
        unpack8(make_uint4(gcur[0][0], gcur[0][1], gcur[0][2], gcur[0][3]), xr);
        unpack8(make_uint4(gcur[1][0], gcur[1][1], gcur[1][2], gcur[1][3]), xz);
        unpack8(make_uint4(gcur[2][0], gcur[2][1], gcur[2][2], gcur[2][3]), xn);
        if (more) {  // the next chunk's MFMAs woven with this chunk's cells
          const char* base = slots + ((c + 1) & 1) * C::SLOT + lane * 16;
          auto frag = [&](int kt, int rb) { return *reinterpret_cast<const tt_u32x4*>(base + (kt * 2 + rb) * 1024); };
#pragma unroll
          for (int rb = 0; rb < 2; ++rb)
#pragma unroll
            for (int g = 0; g < 3; ++g) acc[rb][g] = f32x4{0.f, 0.f, 0.f, 0.f};
          tt_u32x4 f[3][2];
          f[0][0] = frag(0, 0); f[0][1] = frag(0, 1);
          f[1][0] = frag(1, 0); f[1][1] = frag(1, 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int kt = 0; kt < NKT; ++kt) {
            if (kt + 2 < NKT) {
              f[(kt + 2) % 3][0] = frag(kt + 2, 0);
              f[(kt + 2) % 3][1] = frag(kt + 2, 1);
            }
#pragma unroll
            for (int rb = 0; rb < 2; ++rb)
#pragma unroll
              for (int g = 0; g < 3; ++g)
                acc[rb][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                    __builtin_bit_cast(bf16x8v, wa[g][kt]), __builtin_bit_cast(bf16x8v, f[kt % 3][rb]), acc[rb][g], 0, 0, 0);
            if constexpr (DROP) {
#pragma unroll
              for (int e = 0; e < 8; ++e)
                if (e * NKT / 8 == kt) {
                  msk[e] = tt_dropout_scale(R.seed, R.row0 + grow, (uint32_t)(R.col0 + j + e), a.drop_thresh, a.inv_keep);
                  asm volatile("" : "+v"(msk[e]));
                }
            }
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if ((e + 1) * NKT / 8 - 1 == kt) {
                asm volatile("" : "+v"(xr[e]), "+v"(xz[e]), "+v"(xn[e]), "+v"(lr[e]), "+v"(lz[e]), "+v"(ln[e]),
                             "+v"(hp[e]));
                gru_cell(xr[e], xz[e], xn[e], lr[e], lz[e], ln[e], bn[e], hp[e], y[e], sr[e], sz[e], sn[e], sg[e]);
                asm volatile("" : "+v"(y[e]), "+v"(sr[e]), "+v"(sz[e]), "+v"(sn[e]), "+v"(sg[e]));
              }
#pragma unroll
            for (int i = 0; i < 6; ++i) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x002, XC_VALU_PER_MFMA, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            gru_cell(xr[e], xz[e], xn[e], lr[e], lz[e], ln[e], bn[e], hp[e], y[e], sr[e], sz[e], sn[e], sg[e]);
            if constexpr (DROP)
              msk[e] = tt_dropout_scale(R.seed, R.row0 + grow, (uint32_t)(R.col0 + j + e), a.drop_thresh, a.inv_keep);
          }
        }
        *reinterpret_cast<float4*>(stt + rr * xc::SSTR + u0) = make_float4(y[0], y[1], y[2], y[3]);
        *reinterpret_cast<float4*>(stt + rr * xc::SSTR + u0 + 4) = make_float4(y[4], y[5], y[6], y[7]);
        const uint4 yb = pack8bf(y);
        if (fast) st16_buf(rdst_h, (uint32_t)(rr * H + j) * 2u, 0, yb);
        else st16_buf_sc1(rdst_h, (uint32_t)(rr * H + j) * 2u, 0, yb);
        asm volatile("" ::: "memory");  // exactly 6 stores follow (the publish below waits for the rest)
        const int lrow = rr * T_ + t;
        const uint32_t oy = ok ? (uint32_t)(lrow * (int)a.ldy + j) * 2u : xc::OOB;
        const uint32_t os = ok ? (uint32_t)(lrow * 4 * H + j) * 2u : xc::OOB;
        // outputs: read only by later kernels (cache policy XC_OUT_AUX; offsets folded into
        // the lane offset, soffset 0, as st16_buf does)
        st16_buf_aux<XC_OUT_AUX>(rY, (int)oy, yb);
        st16_buf_aux<XC_OUT_AUX>(rS, (int)os, pack8bf(sr));
        st16_buf_aux<XC_OUT_AUX>(rS, (int)(os + 2u * H), pack8bf(sz));
        st16_buf_aux<XC_OUT_AUX>(rS, (int)(os + 4u * H), pack8bf(sn));
        st16_buf_aux<XC_OUT_AUX>(rS, (int)(os + 6u * H), pack8bf(sg));
        if constexpr (DROP) {
#pragma unroll
          for (int e = 0; e < 8; ++e) y[e] *= msk[e];
          st16_buf_aux<XC_OUT_AUX>(rX1, (int)oy, pack8bf(y));
        } else {
          st16_buf_aux<XC_OUT_AUX>(rX1, (int)oy, yb);
        }
      }
      // end of a half step: every wave's exchange stores done (only the six output stores
      // after the last one may still be in flight); counted in after the barrier
      if (c == 3 || c == 7) asm volatile("s_nop 0\n\ts_waitcnt vmcnt(6)" ::: "memory");  // s_nop 0: marker (test_host)
      // h chunk two ahead into the slot this chunk's MFMAs used; request the one three ahead
      if (c + 2 < xc::NCH || has_next) xc_put_h<H>(slots + (c & 1) * C::SLOT, hv);
      if (c + 3 < xc::NCH) load_h(cur, idx, c + 3);
      else if (has_next) load_h(nxt, idx + 1, c + 3 - xc::NCH);
      // before the barrier: wait for the half step whose chunks are requested next
      // iteration (chunk 4 of this step, chunk 0 of the next), also the write-after-read
      // guard of the image half this member writes next
      if (tid == 0) {
        if (c == 0 && idx > 0) xc_wait(cntB, (unsigned)(M * idx), ws);
        if (c == 4 && has_next) xc_wait(cntA, (unsigned)(M * (idx + 1)), ws);
      }
      __syncthreads();
      if (tid == 0 && c == 3 && publish) __hip_atomic_fetch_add(cntA, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (tid == 0 && c == 7 && publish) __hip_atomic_fetch_add(cntB, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (more) {
        xc_stage(stg, acc);
        __syncthreads();
        if (c + 1 < xc::NCH) read_gates(c + 1, cur.s == 0);
        else read_gates(0, nxt.s == 0);
      }
    }
    cur = nxt;
    rGc = rGn;
  }
}

// gru_fwd_xs: the column-split forward with the two kinds of work on different waves.
// gru_fwd_xcp gives each SIMD ONE wave that issues both the chunk MFMAs (96 per 32-row
// chunk) and the gate arithmetic, stores and exchange traffic (~375 vector instructions
// per chunk): in-order issue exposes every dependency stall, ~4k cycles per chunk
// against ~2.5k of issue. Here 8 waves share the CU, two per SIMD:
//   matrix waves 0-3 hold the member's W_hh rows in their accumulator registers (as
//     gru_fwd_xcp's waves) and compute the gates of chunk i + 1 (h from the LDS slot,
//     result staged in gate buffer (i + 1) & 1);
//   vector waves 4-7 finish chunk i: gates from buffer i & 1, the fp32 state of the round
//     in their own registers (no LDS), gru_cell, the exchange and output stores, the G
//     prefetch, the h chunk two ahead into the slot chunk i's MFMAs used, the half-step
//     counters;
// so each SIMD's matrix pipe and vector issue are fed by different waves (MI355X_MICROARCH.md
// "Two waves per SIMD"), with ONE barrier per chunk. The MFMA sequence per chunk and the
// cell are gru_fwd_xcp's (same k order from zero, gru_cell): bit-identical outputs.
#ifndef XS_VPRIO  // gru_fwd_xs: 1 = the vector waves run at s_setprio 1 (static priority experiment)
#define XS_VPRIO 0
#endif
#ifndef XS_MPUB  // gru_fwd_xs: arrivals published by matrix wave 0 (0: by vector thread 0)
#define XS_MPUB 1
#endif
#ifndef XS_MPOLL  // gru_fwd_xs: the group counters polled by matrix wave 0 (0: by vector thread 0)
#define XS_MPOLL 1
#endif
#ifndef XS_GA  // gru_fwd_xs: chunks of gate inputs requested ahead
#define XS_GA 1
#endif
namespace xs {
constexpr int NT = 512;
template <int H>
struct Cfg {
  static constexpr int SLOT = xc::Cfg<H>::SLOT;
  static constexpr int LDS = 2 * SLOT + 2 * xc::STG;
};
static_assert(Cfg<512>::LDS <= 163840, "gru_fwd_xs LDS budget");
}  // namespace xs

template <int H, bool DROP>
__global__ __launch_bounds__(xs::NT, 1) __attribute__((amdgpu_waves_per_eu(2, 2))) void gru_fwd_xs(FwdArgs a, XcWs ws) {
  using C = xc::Cfg<H>;
  constexpr int M = C::M, NKT = C::NKT, QPW = C::QPW;
#ifdef TT_DIAG  // timing only (results wrong): 1 no output stores, 2 no G loads, 4 no exchange
  const int dbg = a.dbg;  // loads (h = 0), 8 no MFMAs, 16 no gate arithmetic, 32 no counter waits
#else
  constexpr int dbg = 0;
#endif
  __shared__ __attribute__((aligned(16))) char lds[xs::Cfg<H>::LDS];
  char* slots = lds;
  float* stgb = reinterpret_cast<float*>(lds + 2 * C::SLOT);  // [2][32 rows][192] fp32
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const bool mw = wave < 4;                 // matrix wave
  const int vw = wave - 4, vt = tid - 256;  // vector wave / thread index
  const int xcd = blockIdx.x & 7, jj = blockIdx.x >> 3;
  const int grp = ws.xmap ? (int)blockIdx.x / M : xcd * ws.qg + jj / M;
  const int mem = ws.xmap ? (int)blockIdx.x % M : jj % M;
  const int rz = grp % ws.nrec, gi = grp / ws.nrec;
  const FwdRec R = a.r[rz];
  const int T_ = a.T, B = a.B;
  const int gb0 = gi * ws.rpg;
  xc_gu32* cw = (xc_gu32*)(uintptr_t)(ws.cnt + grp * xc::CSTR);
  xc_gu32* cntA = cw;
  xc_gu32* cntB = cw + 2;
  const bool publish = !(grp == 0 && mem == ws.skip - 1);
  bf16_t* xbg = ws.xb + (long)grp * 2 * xc::RR * H;
  const __amdgpu_buffer_rsrc_t rx[2] = {tt_rsrc(xbg), tt_rsrc(xbg + xc::RR * H)};
  const bool fast = xc_group_on_one_xcd(ws.cnt + grp * xc::CSTR, M, mem, ws.fast_ok != 0, ws);
  if (ws.skew > 0 && (grp & 1))
    for (int i = 0; i < ws.skew; ++i) __builtin_amdgcn_s_sleep(127);
  const int NS = ws.nround * T_;
  struct Step {
    int s, t, rb0, nrow;
  };
  auto step_of = [&](int idx) {
    Step q;
    const int r = idx / T_;
    q.s = idx - r * T_;
    q.t = R.dir ? T_ - 1 - q.s : q.s;
    q.rb0 = gb0 + r * xc::RR;
    q.nrow = min(min(ws.rpg - r * xc::RR, xc::RR), B - q.rb0);
    return q;
  };
  // zero h for step 0's chunks 0 and 1 (every wave helps), then the roles split
  for (int i = tid; i < 2 * C::SLOT / 16; i += xs::NT) reinterpret_cast<float4*>(slots)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  if (mw) {
    // ---------------------------------------------------------------- matrix waves
    tt_u32x4 wa[3][NKT];
    {
      const bf16_t* W = static_cast<const bf16_t*>(R.whh);
#pragma unroll
      for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt)
          wa[g][kt] = *reinterpret_cast<const tt_u32x4*>(
              W + (long)(g * H + 64 * mem + 16 * wave + (lane & 15)) * H + kt * 32 + (lane >> 4) * 8);
#pragma unroll
      for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt) asm volatile("" : "+v"(wa[g][kt]));
    }
    // gates of one chunk from h slot `sl` into gate buffer `gb` (C^T: 4 units of a row per lane)
    auto chunk = [&](const char* sl, float* gb) {
      f32x4 acc[2][3];
      if (dbg & 8) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
          for (int g = 0; g < 3; ++g)
            *reinterpret_cast<f32x4*>(gb + stg_off(rb * 16 + (lane & 15), g * 64 + 16 * wave + 4 * (lane >> 4))) =
                f32x4{0.f, 0.f, 0.f, 0.f};
        return;
      }
      const char* base = sl + lane * 16;
      auto frag = [&](int kt, int rb) { return *reinterpret_cast<const tt_u32x4*>(base + (kt * 2 + rb) * 1024); };
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int g = 0; g < 3; ++g) acc[rb][g] = f32x4{0.f, 0.f, 0.f, 0.f};
      tt_u32x4 f[3][2];
      f[0][0] = frag(0, 0); f[0][1] = frag(0, 1);
      f[1][0] = frag(1, 0); f[1][1] = frag(1, 1);
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        if (kt + 2 < NKT) {
          f[(kt + 2) % 3][0] = frag(kt + 2, 0);
          f[(kt + 2) % 3][1] = frag(kt + 2, 1);
        }
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
          for (int g = 0; g < 3; ++g)
            acc[rb][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8v, wa[g][kt]), __builtin_bit_cast(bf16x8v, f[kt % 3][rb]), acc[rb][g], 0, 0, 0);
      }
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int g = 0; g < 3; ++g)
          *reinterpret_cast<f32x4*>(gb + stg_off(rb * 16 + (lane & 15), g * 64 + 16 * wave + 4 * (lane >> 4))) = acc[rb][g];
    };
    chunk(slots, stgb);  // step 0, chunk 0 (zero h)
    __syncthreads();
    for (int idx = 0; idx < NS; ++idx) {
      const bool has_next = idx + 1 < NS;
#pragma unroll
      for (int c = 0; c < xc::NCH; ++c) {
        if (c + 1 < xc::NCH || has_next) chunk(slots + ((c + 1) & 1) * C::SLOT, stgb + ((c + 1) & 1) * (xc::STG / 4));
#if XS_MPOLL
        // the group counters are polled by a matrix-wave lane (its memory queue is empty, so a
        // poll drains nothing; a vector-wave poll waited for that wave's stores)
        if (tid == 0 && !(dbg & 32)) {
          if (c == 0 && idx > 0) xc_wait(cntB, (unsigned)(M * idx), ws);
          if (c == 4 && has_next) xc_wait(cntA, (unsigned)(M * (idx + 1)), ws);
        }
#endif
        __syncthreads();
#if XS_MPUB
        // ... and the arrivals published by it too, after the barrier that follows every vector
        // wave's drain of its exchange stores (keeps the atomic out of a storing wave's queue)
        if (tid == 0 && c == 3 && publish) __hip_atomic_fetch_add(cntA, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (tid == 0 && c == 7 && publish) __hip_atomic_fetch_add(cntB, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
      }
    }
    return;
  }
  // ------------------------------------------------------------------ vector waves
  uint32_t ho[QPW];
#pragma unroll
  for (int p = 0; p < QPW; ++p) {
    const int q = vw * QPW + p, kt = q >> 1, rb = q & 1;
    ho[p] = (uint32_t)(((rb * 16 + (lane & 15)) * H + kt * 32 + (lane >> 4) * 8) * 2);
  }
  const int cr = vt >> 3, u0 = (vt & 7) * 8, j = 64 * mem + u0;
  float bn[8];
  {
    const float4 b0 = *reinterpret_cast<const float4*>(R.bhn + j);
    const float4 b1 = *reinterpret_cast<const float4*>(R.bhn + j + 4);
    bn[0] = b0.x; bn[1] = b0.y; bn[2] = b0.z; bn[3] = b0.w;
    bn[4] = b1.x; bn[5] = b1.y; bn[6] = b1.z; bn[7] = b1.w;
  }
  const bf16_t* G = static_cast<const bf16_t*>(R.g);
  bf16_t* Yw = static_cast<bf16_t*>(R.y);
  bf16_t* X1 = static_cast<bf16_t*>(R.x1);
  bf16_t* S = static_cast<bf16_t*>(R.save);
  auto g_rsrc = [&](const Step& q) { return tt_rsrc_n(G + (long)(q.nrow > 0 ? q.rb0 : 0) * T_ * a.ldg, q.nrow > 0); };
  auto load_g = [&](const Step& q, __amdgpu_buffer_rsrc_t rG, int c, tt_u32x4 (&gx)[3]) {
    const uint32_t og = c * xc::CR + cr < q.nrow ? (uint32_t)(((c * xc::CR + cr) * T_ + q.t) * (int)a.ldg + j) * 2u
                                                  : xc::OOB;
#pragma unroll
    for (int g = 0; g < 3; ++g)
      gx[g] = (dbg & 2) ? tt_u32x4{0u, 0u, 0u, 0u} : __builtin_amdgcn_raw_buffer_load_b128(rG, (int)og, g * H * 2, XC_G_AUX);
  };
  tt_u32x4 hv[QPW];
  auto load_h = [&](const Step& q, int qidx, int c) {
    if (q.s == 0 || (dbg & 4)) {
#pragma unroll
      for (int p = 0; p < QPW; ++p) hv[p] = tt_u32x4{0u, 0u, 0u, 0u};
    } else {
#pragma unroll
      for (int p = 0; p < QPW; ++p)
        hv[p] = __builtin_amdgcn_raw_buffer_load_b128(rx[(qidx - 1) & 1], (int)ho[p], c * xc::CR * H * 2, 16);
    }
  };
  float st[xc::NCH][8];  // fp32 state of this thread's (row, 8 units) in each chunk of the round
  Step cur = step_of(0);
  __amdgpu_buffer_rsrc_t rGc = g_rsrc(cur);
  // gate inputs XS_GA chunks ahead, in a ring of GR sets (a power of two > XS_GA, so that a
  // chunk's set is fixed at compile time: 8 chunks per step)
  constexpr int GR = XS_GA < 2 ? 2 : 4;
  static_assert(XS_GA >= 1 && XS_GA < GR && xc::NCH % GR == 0, "gate-input ring");
  tt_u32x4 gq[GR][3];
#pragma unroll
  for (int c = 0; c < XS_GA; ++c) load_g(cur, rGc, c, gq[c]);
#pragma unroll
  for (int p = 0; p < QPW; ++p) hv[p] = tt_u32x4{0u, 0u, 0u, 0u};  // step 0, chunk 2
  __syncthreads();  // the matrix waves' chunk 0
  if (XS_VPRIO) __builtin_amdgcn_s_setprio(1);  // the vector waves win VALU/issue arbitration
  for (int idx = 0; idx < NS; ++idx) {
    const bool has_next = idx + 1 < NS;
    const Step nxt = step_of(has_next ? idx + 1 : idx);
    const __amdgpu_buffer_rsrc_t rGn = g_rsrc(nxt);
    const long r0w = (long)(cur.nrow > 0 ? cur.rb0 : 0) * T_;
    const bool on = cur.nrow > 0;
    const __amdgpu_buffer_rsrc_t rY = tt_rsrc_n(Yw + r0w * a.ldy, on);
    const __amdgpu_buffer_rsrc_t rX1 = tt_rsrc_n(X1 ? X1 + r0w * a.ldy : Yw, on && X1 != nullptr);
    const __amdgpu_buffer_rsrc_t rS = tt_rsrc_n(S + r0w * 4L * H, on);
    const __amdgpu_buffer_rsrc_t rdst_h = rx[idx & 1];
    const int t = cur.t;
    const bool first = cur.s == 0;
#pragma unroll
    for (int c = 0; c < xc::NCH; ++c) {
      const int gslot = c % GR, gnext = (c + XS_GA) % GR;
      if (c + XS_GA < xc::NCH) load_g(cur, rGc, c + XS_GA, gq[gnext]);
      else if (has_next) load_g(nxt, rGn, c + XS_GA - xc::NCH, gq[gnext]);
      {
        const int rr = c * xc::CR + cr;
        const bool ok = rr < cur.nrow;
        const float* gb = stgb + (c & 1) * (xc::STG / 4);
        float xr[8], xz[8], xn[8], lr[8], lz[8], ln[8], y[8], sr[8], sz[8], sn[8], sg[8];
        const tt_u32x4(&gcur)[3] = gq[gslot];
        unpack8(make_uint4(gcur[0][0], gcur[0][1], gcur[0][2], gcur[0][3]), xr);
        unpack8(make_uint4(gcur[1][0], gcur[1][1], gcur[1][2], gcur[1][3]), xz);
        unpack8(make_uint4(gcur[2][0], gcur[2][1], gcur[2][2], gcur[2][3]), xn);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float4 v0 = *reinterpret_cast<const float4*>(gb + stg_off(cr, 0 * 64 + u0 + 4 * h));
          const float4 v1 = *reinterpret_cast<const float4*>(gb + stg_off(cr, 1 * 64 + u0 + 4 * h));
          const float4 v2 = *reinterpret_cast<const float4*>(gb + stg_off(cr, 2 * 64 + u0 + 4 * h));
          lr[4 * h] = v0.x; lr[4 * h + 1] = v0.y; lr[4 * h + 2] = v0.z; lr[4 * h + 3] = v0.w;
          lz[4 * h] = v1.x; lz[4 * h + 1] = v1.y; lz[4 * h + 2] = v1.z; lz[4 * h + 3] = v1.w;
          ln[4 * h] = v2.x; ln[4 * h + 1] = v2.y; ln[4 * h + 2] = v2.z; ln[4 * h + 3] = v2.w;
        }
        const uint32_t grow = (uint32_t)(cur.rb0 + rr) * (uint32_t)T_ + (uint32_t)t;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float hp = first ? 0.f : st[c][e];
          if (dbg & 16) {
            y[e] = xr[e] + lr[e] + hp; sr[e] = xz[e] + lz[e]; sz[e] = xn[e] + ln[e]; sn[e] = bn[e]; sg[e] = hp;
          } else {
            gru_cell(xr[e], xz[e], xn[e], lr[e], lz[e], ln[e], bn[e], hp, y[e], sr[e], sz[e], sn[e], sg[e]);
          }
          st[c][e] = y[e];
        }
        const uint4 yb = pack8bf(y);
        if (fast) st16_buf(rdst_h, (uint32_t)(rr * H + j) * 2u, 0, yb);
        else st16_buf_sc1(rdst_h, (uint32_t)(rr * H + j) * 2u, 0, yb);
        asm volatile("" ::: "memory");  // exactly 6 stores follow (the publish below waits for the rest)
        const int lrow = rr * T_ + t;
        const bool okd = ok && !(dbg & 1);
        const uint32_t oy = okd ? (uint32_t)(lrow * (int)a.ldy + j) * 2u : xc::OOB;
        const uint32_t os = okd ? (uint32_t)(lrow * 4 * H + j) * 2u : xc::OOB;
        st16_buf_aux<XC_OUT_AUX>(rY, (int)oy, yb);
        st16_buf_aux<XC_OUT_AUX>(rS, (int)os, pack8bf(sr));
        st16_buf_aux<XC_OUT_AUX>(rS, (int)(os + 2u * H), pack8bf(sz));
        st16_buf_aux<XC_OUT_AUX>(rS, (int)(os + 4u * H), pack8bf(sn));
        st16_buf_aux<XC_OUT_AUX>(rS, (int)(os + 6u * H), pack8bf(sg));
        if constexpr (DROP) {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            y[e] *= tt_dropout_scale(R.seed, R.row0 + grow, (uint32_t)(R.col0 + j + e), a.drop_thresh, a.inv_keep);
          st16_buf_aux<XC_OUT_AUX>(rX1, (int)oy, pack8bf(y));
        } else {
          st16_buf_aux<XC_OUT_AUX>(rX1, (int)oy, yb);
        }
      }
      if (c == 3 || c == 7) asm volatile("s_nop 0\n\ts_waitcnt vmcnt(6)" ::: "memory");  // s_nop 0: marker (test_host)
      // h chunk two ahead into the slot chunk c's MFMAs used (read before the last barrier);
      // request the one three ahead
      if (c + 2 < xc::NCH || has_next) {
#pragma unroll
        for (int p = 0; p < QPW; ++p)
          *reinterpret_cast<tt_u32x4*>(slots + (c & 1) * C::SLOT + (vw * QPW + p) * 1024 + lane * 16) = hv[p];
      }
      if (c + 3 < xc::NCH) load_h(cur, idx, c + 3);
      else if (has_next) load_h(nxt, idx + 1, c + 3 - xc::NCH);
      if (!XS_MPOLL && vt == 0 && !(dbg & 32)) {
        if (c == 0 && idx > 0) xc_wait(cntB, (unsigned)(M * idx), ws);
        if (c == 4 && has_next) xc_wait(cntA, (unsigned)(M * (idx + 1)), ws);
      }
      __syncthreads();
      if (!XS_MPUB && vt == 0 && c == 3 && publish) __hip_atomic_fetch_add(cntA, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!XS_MPUB && vt == 0 && c == 7 && publish) __hip_atomic_fetch_add(cntB, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    cur = nxt;
    rGc = rGn;
  }
}

#ifdef TT_DIAG
}  // namespace
extern "C" int tt_diag_fwd_prof(unsigned long long* out) {  // [2048][8] host buffer
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fwd_prof), sizeof(g_fwd_prof)) == hipSuccess ? 0 : 1;
}
namespace {
#endif
bool gru_fwd_persistent(int dtype, int H) {
  // Every bf16 width H % 64 == 0, H <= 512. Round 2 retired the runtime-NKT instances
  // (H 64: garbage in the saved gh_n of step 0, 33 of 150 probe runs); the cause was the
  // unprotected wide-store data hazard of SGPR-soffset buffer stores (tt_common.h
  // st16_buf), which the fixed-NKT bench instances had as well.
  if (dtype != TT_DT_BF16 || H % 64 != 0 || H > PH_MAX) return false;
  return tt::opt(tt::OPT_GRU_STEP) != 1;
}

}  // namespace

// batch rows per backward tile: 128, or 64 with option gru_bwd_rows = 64 (3 workgroups
// per CU; measured slower at B=8192, H=512: 13.6 vs 11.5 ms per layer)
// Per-step backward tile rows: option gru_bwd_rows 64 / 128, or 0 (auto): 64 where 128-row
// tiles would leave the grid under one workgroup per CU (configs[1]: B 1024, fp32, H 512 ->
// 128 workgroups; 64-row tiles: gru_bwd 26.1 -> 15.4 ms per step, profiles/r04_bench_c1_c.txt)
static int bwd_rows(int B, int H, int nrec) {
  const int o = tt::opt(tt::OPT_GRU_BWD_ROWS);
  if (o == 64 || o == 128) return o;
  // 64-row tiles up to one 128-row workgroup per CU (fp32 B 2048, H 512: 9.93 ms per layer
  // on 64-row tiles, two per CU, vs 12.48 on 128-row tiles with the product ring,
  // profiles/r04_gru_bwd_rows_b2048_aa.txt)
  return (long)tt_ceil_div(H, 128) * tt_ceil_div(B, 128) * nrec <= 256 ? 64 : 128;
}
// partial bias rows: one per backward row tile (the smallest tile: 64 rows; rows of a
// larger-tile launch past its tile count are zero-filled by tt_gru_bwd and add nothing)
extern "C" int tt_gru_bias_rows(int B) { return tt_ceil_div(B, 64); }

extern "C" int tt_gru_fwd_launches(int dtype, int T, int H) { return gru_fwd_persistent(dtype, H) ? 1 : T; }

// bf16 H 256 / 512 (and H 1024 in two column passes with option gru_bwd_persist = 2: measured
// slower than the per-step 256x256 kernel at configs[4], 97.0 vs 92.9 ms per step,
// profiles/r04_bench_c4_c.txt)
static bool gru_bwd_persistent(int dtype, int H) {
  const int o = tt::opt(tt::OPT_GRU_BWD_PERSIST);
  return dtype == TT_DT_BF16 && (H == 256 || H == 512 || (H == 1024 && o == 2)) &&
         tt::opt(tt::OPT_GRU_BWD_ROWS) != 64 && o != 0;
}
extern "C" int tt_gru_bwd_launches(int dtype, int T, int H) { return gru_bwd_persistent(dtype, H) ? 1 : T; }
extern "C" int tt_gru_bwd_carry_on_chip(int dtype, int T, int H) {
  (void)T;
  return TT_BWD_CREG != 0 && gru_bwd_persistent(dtype, H) && H <= 512 ? 1 : 0;
}

// Per-device side stream + fork/join events for tt_gru_bwd's second launch chain,
// created once per device under a mutex (host threads may call on distinct streams).
// The fork/join events are per device, so two host threads running the backward on the
// same device at once must not both take the two-chain path (one stream
// per thread; the default row-owning and 256-tile backwards never use it).
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};
static int side_stream(SideStream** out) {
  static SideStream ss[64];
  static std::mutex mu;
  int dev = 0;
  TT_CHECK_HIP(hipGetDevice(&dev));
  TT_CHECK_ARG(dev >= 0 && dev < 64, "tt_gru_bwd: device %d", dev);
  std::lock_guard<std::mutex> lock(mu);
  SideStream& x = ss[dev];
  if (!x.s) {
    SideStream n;
    TT_CHECK_HIP(hipStreamCreateWithFlags(&n.s, hipStreamNonBlocking));
    TT_CHECK_HIP(hipEventCreateWithFlags(&n.fork, hipEventDisableTiming));
    TT_CHECK_HIP(hipEventCreateWithFlags(&n.join, hipEventDisableTiming));
    x = n;
  }
  *out = &x;
  return 0;
}

// ---- column-split forward: geometry, caller-passed workspace, residency check ---------
// Workspace (tt_gru_fwd_ws_size bytes, caller-allocated, one per launch in flight):
//   [0, 256)            status word at 0: set by a launch whose member wait timed out, never
//                       cleared by the library (the caller zeroes it at allocation)
//   [256, 256 + CNT)    per-group arrival counters + the per-launch timeout flag, zeroed
//                       by tt_gru_fwd before every launch (stream-ordered)
//   [IMG, IMG + ...)    exchange images [groups][2][RR][H] bf16
constexpr int XC_MAX_GROUPS = 512;
constexpr long XC_HDR = 256;
struct XcGeo {
  XcWs w{};
  int grid = 0, ng = 0;
  long cnt_bytes = 0, img_off = 0, bytes = 0;
};

// per-device facts, read once: CU count and the co-residency of the column-split kernels
// (1 workgroup per CU each, from the occupancy query)
struct XcDev {
  int cus = 0;
  int occ[2][2] = {{0, 0}, {0, 0}};  // [H 256 / 512][DROP]
  int occ_xs[2] = {0, 0};            // gru_fwd_xs<512, DROP>
};
static std::mutex g_xc_mu;
static XcDev g_xc[64];

template <int H, bool DROP>
static const void* xc_kernel() {
  return reinterpret_cast<const void*>(&gru_fwd_xcp<H, DROP>);
}
template <bool DROP>
static const void* xs_kernel() {
  return reinterpret_cast<const void*>(&gru_fwd_xs<512, DROP>);
}
// the specialized-wave form (gru_fwd_xs) where it is selected and built (H 512)
static bool xs_on(int H) { return H == 512 && tt::opt(tt::OPT_GRU_FWD_XS) != 0; }

static int xc_device(XcDev** out) {
  int dev = 0;
  TT_CHECK_HIP(hipGetDevice(&dev));
  TT_CHECK_ARG(dev >= 0 && dev < 64, "tt_gru_fwd: device %d", dev);
  std::lock_guard<std::mutex> lock(g_xc_mu);
  XcDev& x = g_xc[dev];
  if (!x.cus) {
    int cus = 0;
    TT_CHECK_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const void* k[2][2] = {{xc_kernel<256, false>(), xc_kernel<256, true>()},
                           {xc_kernel<512, false>(), xc_kernel<512, true>()}};
    for (int h = 0; h < 2; ++h)
      for (int d = 0; d < 2; ++d) TT_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&x.occ[h][d], k[h][d], xc::NT, 0));
    const void* kx[2] = {xs_kernel<false>(), xs_kernel<true>()};
    for (int d = 0; d < 2; ++d) TT_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&x.occ_xs[d], kx[d], xs::NT, 0));
    x.cus = cus;
  }
  *out = &x;
  return 0;
}

// Launch geometry of the column-split forward, or false where it does not apply.
static bool xc_geometry(const XcDev& dev, int dtype, int H, int nrec, int B, int T, long ldg, long ldy, bool drop,
                        XcGeo& g) {
  const int v = tt::opt(tt::OPT_GRU_FWD_XC);
  if (v == 0 || dtype != TT_DT_BF16 || (H != 512 && H != 256) || tt::opt(tt::OPT_GRU_STEP) == 1) return false;
  const int M = H / 64;
  const int qg = dev.cus / (8 * M);
  const int ng = 8 * qg;
  if (qg < 1 || ng > XC_MAX_GROUPS || ng % nrec != 0) return false;
  // every member must be resident at once: one workgroup per CU, grid <= CUs
  const int occ = xs_on(H) ? dev.occ_xs[drop] : dev.occ[H == 512][drop];
  if (occ < 1 || ng * M > dev.cus * occ) return false;
  const int gpr = ng / nrec;
  // auto mode: only where every group gets at least half a round of rows
  if ((v & 3) == 1 && (long)B < (long)gpr * (xc::RR / 2)) return false;
  // per-round resources: byte offsets of RR rows x T steps stay below 2 GiB
  if ((long)xc::RR * T * std::max({4L * H, ldy, ldg}) * 2 >= (1L << 31)) return false;
  g.w.qg = qg;
  g.w.nrec = nrec;
  g.w.rpg = tt_ceil_div(B, gpr);
  g.w.nround = tt_ceil_div(g.w.rpg, xc::RR);
  g.w.fast_ok = (v & 4) ? 0 : 1;  // option bit 4: always write-through images
  g.w.xmap = (v & 16) ? 1 : 0;    // option bit 16: members dealt over the XCDs
  g.w.skip = tt::opt(tt::OPT_GRU_XC_SKIP);
  g.w.skew = tt::opt(tt::OPT_GRU_FWD_SKEW);
  const int sp = std::min(30, std::max(10, tt::opt(tt::OPT_GRU_XC_SPINS)));
  g.w.spins = 1u << sp;
  g.grid = ng * M;
  g.ng = ng;
  g.cnt_bytes = ((long)ng * xc::CSTR * 4 + 256 + 255) / 256 * 256;  // counters + the launch flag
  g.img_off = XC_HDR + g.cnt_bytes;
  g.bytes = g.img_off + (long)ng * 2 * xc::RR * H * 2;
  return true;
}

static int xc_plan(int dtype, int nrec, int B, int T, int H, long ldg, long ldy, bool drop, XcGeo& g, bool* ok) {
  *ok = false;
  if (dtype != TT_DT_BF16 || nrec < 1 || nrec > 4 || B <= 0 || T <= 0 || (H != 256 && H != 512) ||
      tt::opt(tt::OPT_GRU_FWD_XC) == 0)
    return 0;
  XcDev* x = nullptr;
  TT_PROPAGATE(xc_device(&x));
  *ok = xc_geometry(*x, dtype, H, nrec, B, T, ldg, ldy, drop, g);
  return 0;
}

extern "C" long tt_gru_fwd_ws_size(int dtype, int nrec, int B, int T, int H, long ldg, long ldy) {
  XcGeo g;
  bool ok = false;
  // the dropout and plain instances have the same geometry; take the larger occupancy
  // question (both are 1 per CU) as the dropout form's
  if (xc_plan(dtype, nrec, B, T, H, ldg, ldy, true, g, &ok) != 0 || !ok) return 0;
  return g.bytes;
}

// Launches the column-split forward when it applies and ws is large enough (*used = true);
// a grid the runtime will not make co-resident leaves *used false (row-owning fallback).
static int gru_fwd_xc_launch(const FwdArgs& a, int nrec, int B, int T, int H, long ldg, long ldy, void* ws,
                             long ws_bytes, hipStream_t st, bool* used) {
  *used = false;
  if (!ws) return 0;
  const bool drop = a.drop_thresh != 0 && a.r[0].x1 != nullptr;
  XcGeo g;
  bool ok = false;
  TT_PROPAGATE(xc_plan(TT_DT_BF16, nrec, B, T, H, ldg, ldy, drop, g, &ok));
  if (!ok || ws_bytes < g.bytes) return 0;
  TT_CHECK_ARG(((uintptr_t)ws & 255) == 0, "tt_gru_fwd: ws must be 256-byte aligned");
  char* base = static_cast<char*>(ws);
  g.w.status = reinterpret_cast<unsigned*>(base);
  g.w.cnt = reinterpret_cast<unsigned*>(base + XC_HDR);
  g.w.err = g.w.cnt + g.ng * xc::CSTR;
  g.w.xb = reinterpret_cast<bf16_t*>(base + g.img_off);
  TT_CHECK_HIP(hipMemsetAsync(base + XC_HDR, 0, g.cnt_bytes, st));
  FwdArgs ak = a;
  XcWs wk = g.w;
  void* args[] = {&ak, &wk};
  const bool xs = xs_on(H);
  const void* fn = xs ? (drop ? xs_kernel<true>() : xs_kernel<false>())
                 : H == 512 ? (drop ? xc_kernel<512, true>() : xc_kernel<512, false>())
                            : (drop ? xc_kernel<256, true>() : xc_kernel<256, false>());
  const int nt = xs ? xs::NT : xc::NT;
  // A plain launch by default: xc_plan has already checked the grid (<= one workgroup per
  // CU) against the occupancy query, which is all a cooperative launch checks on gfx950
  // (MI355X_MICROARCH.md "coop-launch": same residency, +15-19 us per launch), and the
  // member waits are bounded (status word -> GruTimeoutError, Adam step guard). Option
  // gru_xc_coop 1 restores hipLaunchCooperativeKernel; under rocprofv3 that form made the
  // profiled process fault in teardown after the profiler's finalisation
  // (profiles/r04_rocprof_crash_k.txt), the plain one does not.
  const hipError_t e = tt::opt(tt::OPT_GRU_XC_COOP)
                           ? hipLaunchCooperativeKernel(fn, dim3(g.grid), dim3(nt), args, 0, st)
                           : hipLaunchKernel(fn, dim3(g.grid), dim3(nt), args, 0, st);
  if (e == hipErrorCooperativeLaunchTooLarge) {
    (void)hipGetLastError();  // clear it: the row-owning kernel runs instead
    return 0;
  }
  TT_CHECK_HIP(e);
  TT_CHECK_LAUNCH("gru_fwd_xcp");
  *used = true;
  return 0;
}

extern "C" int tt_gru_fwd_launches_for(int dtype, int nrec, int B, int T, int H, long ldg, long ldy) {
  XcGeo g;
  bool ok = false;
  if (xc_plan(dtype, nrec, B, T, H, ldg, ldy, true, g, &ok) == 0 && ok) return 1;
  return tt_gru_fwd_launches(dtype, T, H);
}

extern "C" int tt_gru_fwd(int dtype, const tt_gru_fwd_rec* recs, int nrec, int B, int T, int H, long ldg,
                          long ldy, float drop_p, void* ws, long ws_bytes, void* stream) {
  TT_CHECK_ARG(dtype == TT_DT_F32 || dtype == TT_DT_BF16, "tt_gru_fwd: bad dtype");
  TT_CHECK_ARG(nrec >= 1 && nrec <= 4, "tt_gru_fwd: nrec %d", nrec);
  TT_CHECK_ARG(B > 0 && T > 0 && H > 0, "tt_gru_fwd: bad shape");
  TT_CHECK_ARG(ws_bytes >= 0 && (ws != nullptr || ws_bytes == 0), "tt_gru_fwd: ws / ws_bytes");
  const int esz = dtype == TT_DT_BF16 ? 2 : 4;
  // epilogues update 8 consecutive hidden units per thread
  TT_CHECK_ARG(H % 8 == 0 && (ldy * esz) % 16 == 0, "tt_gru_fwd: H=%d (multiple of 8)/ldy=%ld misaligned", H, ldy);
  TT_CHECK_ARG(drop_p >= 0.f && drop_p < 1.f, "tt_gru_fwd: drop_p");
  TT_CHECK_ARG(tt_ceil_div(B, 128) <= 65535, "tt_gru_fwd: B too large");
  TT_CHECK_ARG(128L * T * std::max({4L * H, ldy, ldg}) * esz < (1L << 31), "tt_gru_fwd: tile byte offsets exceed 2 GiB");
  FwdArgs a{};
  for (int i = 0; i < nrec; ++i) {
    const tt_gru_fwd_rec& r = recs[i];
    TT_CHECK_ARG(r.g && r.whh && r.bhn && r.y && r.save && r.hstate, "tt_gru_fwd: null pointer in rec %d", i);
    a.r[i] = FwdRec{r.g, r.whh, r.bhn, r.y, r.x1, r.save, r.hstate, r.dir, r.drop_seed, r.drop_col0, r.drop_row0};
  }
  a.B = B; a.T = T; a.H = H; a.ldg = ldg; a.ldy = ldy;
  a.drop_thresh = drop_p > 0.f ? (uint32_t)(drop_p * 16777216.0f + 0.5f) : 0u;
  a.inv_keep = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
#ifdef TT_DIAG
  if (const char* e = getenv("TT_GRU_DBG")) a.dbg = atoi(e);
#endif
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TT_DT_BF16) {
    bool used = false;
    TT_PROPAGATE(gru_fwd_xc_launch(a, nrec, B, T, H, ldg, ldy, ws, ws_bytes, st, &used));
    if (used) return 0;
  }
  if (gru_fwd_persistent(dtype, H)) {
    const dim3 grid(tt_ceil_div(B, PR) * nrec);
    int depth = (H / 64) % 4 == 0 ? 4 : (H / 64) % 2 == 0 ? 2 : 1;
    depth = std::min(depth, tt::opt(tt::OPT_GRU_DEPTH));
    if (depth >= 4 && H == 512) hipLaunchKernelGGL((gru_fwd_seq<4, 8>), grid, dim3(PNT), 0, st, a);
    else if (depth >= 4 && H == 256) hipLaunchKernelGGL((gru_fwd_seq<4, 4>), grid, dim3(PNT), 0, st, a);
    else if (depth >= 4) hipLaunchKernelGGL((gru_fwd_seq<4, 0>), grid, dim3(PNT), 0, st, a);
    else if (depth == 2 && H == 512) hipLaunchKernelGGL((gru_fwd_seq<2, 8>), grid, dim3(PNT), 0, st, a);
    else if (depth == 2 && H == 256) hipLaunchKernelGGL((gru_fwd_seq<2, 4>), grid, dim3(PNT), 0, st, a);
    else if (depth == 2) hipLaunchKernelGGL((gru_fwd_seq<2, 0>), grid, dim3(PNT), 0, st, a);
    else if (H == 512) hipLaunchKernelGGL((gru_fwd_seq<1, 8>), grid, dim3(PNT), 0, st, a);
    else if (H == 256) hipLaunchKernelGGL((gru_fwd_seq<1, 4>), grid, dim3(PNT), 0, st, a);
    else hipLaunchKernelGGL((gru_fwd_seq<1, 0>), grid, dim3(PNT), 0, st, a);
    TT_CHECK_LAUNCH("gru_fwd_seq");
    return 0;
  }
  // 256-row tiles where they still give >= 2 workgroups per CU (option gru_fwd_step_rows
  // 128 / 256 forces one)
  int bmr = tt::opt(tt::OPT_GRU_FWD_STEP_ROWS);
  if (bmr != 128 && bmr != 256)
    bmr = (long)tt_ceil_div(H, 64) * tt_ceil_div(B, 256) * nrec >= 512 ? 256 : 128;
  // the step kernel's S / X1 byte offsets are int relative to the tile's first row
  const long span = (long)T * std::max({4L * H, ldy, ldg}) * esz;
  if (bmr == 256 && 256L * span >= (1L << 31)) bmr = 128;
  TT_CHECK_ARG((long)bmr * span < (1L << 31), "tt_gru_fwd: tile byte offsets exceed 2 GiB (B tile %d)", bmr);
  dim3 grid(tt_ceil_div(H, 64) * tt_ceil_div(B, bmr) * nrec);
  // 128-row tiles: a 3-stage product ring when option gru_step_ring >= 3 and the grid is
  // one workgroup per CU at most (120 KiB of LDS: at two per CU the second workgroup's
  // overlap is worth more, configs[4] 49.7 vs 85.9 ms per layer, profiles/r04_gru_fwd_ring_c4_s.txt)
  XcDev* xd = nullptr;
  TT_PROPAGATE(xc_device(&xd));
  const bool ring = tt::opt(tt::OPT_GRU_STEP_RING) >= 3 && (long)grid.x <= xd->cus;
  for (int s = 0; s < T; ++s) {
    a.s = s;
    if (dtype == TT_DT_BF16) {
      if (bmr == 256) hipLaunchKernelGGL((gru_fwd_step<bf16_t, 256>), grid, dim3(512), 0, st, a);
      else if (ring) hipLaunchKernelGGL((gru_fwd_step<bf16_t, 128, 3>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((gru_fwd_step<bf16_t, 128>), grid, dim3(256), 0, st, a);
    } else {
      if (bmr == 256) hipLaunchKernelGGL((gru_fwd_step<float, 256>), grid, dim3(512), 0, st, a);
      else if (ring) hipLaunchKernelGGL((gru_fwd_step<float, 128, 3>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((gru_fwd_step<float, 128>), grid, dim3(256), 0, st, a);
    }
    TT_CHECK_LAUNCH("gru_fwd_step");
  }
  return 0;
}

// option gru_step_ring: LDS stages of the per-step backward's product (2: double buffer)
template <typename T, int BMR>
static void launch_bwd_step(int ring, dim3 grid, hipStream_t st, const BwdArgs& a) {
  if (ring >= 4) hipLaunchKernelGGL((gru_bwd_step<T, BMR, 4>), grid, dim3(256), 0, st, a);
  else if (ring == 3) hipLaunchKernelGGL((gru_bwd_step<T, BMR, 3>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((gru_bwd_step<T, BMR>), grid, dim3(256), 0, st, a);
}

extern "C" int tt_gru_bwd(int dtype, const tt_gru_bwd_rec* recs, int nrec, int B, int T, int H, long ldy,
                          long ldd, long ldf, void* stream) {
  TT_CHECK_ARG(dtype == TT_DT_F32 || dtype == TT_DT_BF16, "tt_gru_bwd: bad dtype");
  TT_CHECK_ARG(nrec >= 1 && nrec <= 4, "tt_gru_bwd: nrec %d", nrec);
  TT_CHECK_ARG(B > 0 && T > 0 && H > 0, "tt_gru_bwd: bad shape");
  const int esz = dtype == TT_DT_BF16 ? 2 : 4;
  TT_CHECK_ARG(H % 8 == 0 && (ldd * esz) % 16 == 0, "tt_gru_bwd: H=%d (multiple of 8)/ldd=%ld misaligned", H, ldd);
  TT_CHECK_ARG(256L * T * std::max({ldd, ldy, 4L * H}) * esz < (1L << 31), "tt_gru_bwd: tile byte offsets exceed 2 GiB");
  hipStream_t st = (hipStream_t)stream;
  BwdArgs a{};
  for (int i = 0; i < nrec; ++i) {
    const tt_gru_bwd_rec& r = recs[i];
    TT_CHECK_ARG(r.save && r.y && r.whh && r.dgx && r.dgh && r.dhstate && r.dbias_part,
                 "tt_gru_bwd: null pointer in rec %d", i);
    a.r[i] = BwdRec{r.save, r.y, r.dy, r.dfinal, r.whh, r.dgx, r.dgh, r.dhstate, r.dbias_part, r.dir};
    TT_CHECK_HIP(hipMemsetAsync(r.dbias_part, 0, sizeof(float) * 4L * H * tt_gru_bias_rows(B), st));
  }
  a.B = B; a.T = T; a.H = H; a.ldy = ldy; a.ldd = ldd; a.ldf = ldf;
  a.skew = tt::opt(tt::OPT_GRU_BWD_SKEW);
#ifdef TT_DIAG
  if (const char* e = getenv("TT_GRU_DBG")) a.dbg = atoi(e);
#endif
  const int bmr = bwd_rows(B, H, nrec);
  // bf16, H 256 / 512: one row-owning launch per layer (option gru_bwd_persist = 0: per-step
  // launches)
  if (gru_bwd_persistent(dtype, H)) {
    TT_CHECK_ARG(128L * T * std::max({ldd, ldy, 4L * H}) * esz < (1L << 31), "tt_gru_bwd: tile offsets exceed 2 GiB");
    const dim3 grid(tt_ceil_div(B, 128) * nrec);
    if (H == 1024) hipLaunchKernelGGL(gru_bwd_rows<1024>, grid, dim3(512), 0, st, a);
    else if (H == 512) hipLaunchKernelGGL(gru_bwd_rows<512>, grid, dim3(512), 0, st, a);
    else hipLaunchKernelGGL(gru_bwd_rows<256>, grid, dim3(512), 0, st, a);
    TT_CHECK_LAUNCH("gru_bwd_rows");
    return 0;
  }
  // bf16 with H a multiple of 256: 256x256 tiles on the 8-phase loop, one launch per step
  // (option gru_bwd_big = 0 selects the 128x128 step kernels)
  if (dtype == TT_DT_BF16 && H % 256 == 0 && bmr == 128 && tt::opt(tt::OPT_GRU_BWD_BIG) != 0) {
    const dim3 grid((H / 256) * tt_ceil_div(B, 256) * nrec);
    for (int s = T - 1; s >= 0; --s) {
      a.s = s;
      hipLaunchKernelGGL(gru_bwd_big, grid, dim3(512), 0, st, a);
      TT_CHECK_LAUNCH("gru_bwd_big");
    }
    return 0;
  }
  // Two independent chains of step launches (recurrences [0, nrec/2) on the caller's
  // stream, the rest on a side stream): each step kernel is GEMM-then-epilogue, so one
  // chain's HBM-bound epilogues overlap the other chain's MFMA main loops on the same CUs.
  const int ngrp = (nrec >= 2 && tt::opt(tt::OPT_GRU_BWD_STREAMS) != 1) ? 2 : 1;
  BwdArgs ga[2] = {a, a};
  int gn[2] = {nrec, 0};
  if (ngrp == 2) {
    gn[0] = nrec / 2;
    gn[1] = nrec - gn[0];
    for (int i = 0; i < gn[1]; ++i) ga[1].r[i] = a.r[gn[0] + i];
  }
  hipStream_t gs[2] = {st, st};
  SideStream* side = nullptr;
  if (ngrp == 2) {
    TT_PROPAGATE(side_stream(&side));
    gs[1] = side->s;
    TT_CHECK_HIP(hipEventRecord(side->fork, st));
    TT_CHECK_HIP(hipStreamWaitEvent(side->s, side->fork, 0));
  }
  // the product ring (option gru_step_ring) where every chain's workgroups fit one per CU
  // (96-128 KiB of LDS); otherwise two stages and up to two workgroups per CU
  XcDev* xd = nullptr;
  TT_PROPAGATE(xc_device(&xd));
  long wgs = 0;
  for (int g = 0; g < ngrp; ++g) wgs += (long)tt_ceil_div(H, 128) * tt_ceil_div(B, bmr) * gn[g];
  const int ring = wgs <= xd->cus ? tt::opt(tt::OPT_GRU_STEP_RING) : 2;
  for (int s = T - 1; s >= 0; --s) {
    for (int g = 0; g < ngrp; ++g) {
      ga[g].s = s;
      const dim3 grid(tt_ceil_div(H, 128) * tt_ceil_div(B, bmr) * gn[g]);
      if (dtype == TT_DT_BF16) {
        if (bmr == 64) launch_bwd_step<bf16_t, 64>(ring, grid, gs[g], ga[g]);
        else launch_bwd_step<bf16_t, 128>(ring, grid, gs[g], ga[g]);
      } else {
        if (bmr == 64) launch_bwd_step<float, 64>(ring, grid, gs[g], ga[g]);
        else launch_bwd_step<float, 128>(ring, grid, gs[g], ga[g]);
      }
      TT_CHECK_LAUNCH("gru_bwd_step");
    }
  }
  if (ngrp == 2) {
    TT_CHECK_HIP(hipEventRecord(side->join, side->s));
    TT_CHECK_HIP(hipStreamWaitEvent(st, side->join, 0));
  }
  return 0;
}
