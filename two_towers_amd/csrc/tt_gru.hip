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
  int stagger;  // persistent forward (compile-time NKT only): option gru_stagger
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
template <typename T, int BMR>
__global__ __launch_bounds__(2 * BMR) void gru_fwd_step(FwdArgs a) {
  constexpr int NT = 2 * BMR;
  using ML = ttg::DLoop<T, false, false, BMR, 192, BMR / 64, 2>;
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
  if (s > 0) {
    ttg::KCPlain<T> la{Y + (long)tp * a.ldy, (long)T_ * a.ldy, m0, a.B};
    GateRows<T> lb{static_cast<const T*>(R.whh), H, j0};
    const int nk = (H * (int)sizeof(T) + ttg::KTB - 1) / ttg::KTB;
    ML::run(la, lb, H, 0, nk, lds, acc);
  }

  // ---- epilogue, one 64-row half at a time: stage the fp32 gate tile in LDS, then
  // every thread updates 8 consecutive hidden units of a row with 16-byte accesses.
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, tid = threadIdx.x;
  float* L = reinterpret_cast<float*>(lds);  // [3][64][FLD]
  constexpr int FLD = 68;                    // 64 units + 16 B pad
  const int cur = s & 1, prv = cur ^ 1;
  const T* G = static_cast<const T*>(R.g);
  T* Yw = static_cast<T*>(R.y);
  T* X1 = static_cast<T*>(R.x1);
  T* S = static_cast<T*>(R.save);
  float* hs_cur = R.hs + (long)cur * a.B * H;
  const float* hs_prv = R.hs + (long)prv * a.B * H;
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

template <typename T, int BMR>  // BMR batch rows per tile: 128, or 64 (3 tiles per CU)
__global__ __launch_bounds__(256) void gru_bwd_step(BwdArgs a) {
  using ML = ttg::DLoop<T, false, true, BMR, 128, 2, 2>;
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

// ---- backward step on 256x256 tiles (bf16): the recurrent GEMM on the 8-phase loop --
// One workgroup (8 waves) per 256 rows x 256 hidden units of a recurrence: at B 8192,
// H 512 the four recurrences are exactly 256 tiles, one per CU, so the GEMM runs at the
// 8-phase loop's rate (the 128x128 two-phase loop reached ~680 TFLOP/s here) and the
// epilogue (two 128-row passes staged in the freed DMA slots) streams the gate
// gradients. Bias partials land in partial row 2*mt (tt_gru_bias_rows() counts 128-row
// tiles; the odd rows stay zero).
__global__ __launch_bounds__(512) void gru_bwd_big(BwdArgs a) {
  using L8 = ttg::Loop8<bf16_t, false, true>;
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
        vin[kk][1] = ld16_buf(rd, oy, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) vin[kk][2 + q] = ld16_buf(rsv, os, q * 2 * H);
        vin[kk][6] = ld16_buf(ry, oy, 0);
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
template <int H>
struct BwdRowsCfg {
  static constexpr int NQ = H / 128;
  static constexpr int SLOT = 8192 + NQ * 8192;  // 40 KiB at H = 512
  static constexpr int NS = 4;
  static constexpr int LDS = NS * SLOT;
  static constexpr int P = SLOT / 1024 / 8;  // DMAs per wave per K-tile
  static constexpr int NCB = H / 64;
  static constexpr int TPR = H / 8;
  static constexpr int RPI = 512 / TPR;
  static constexpr int LDB = H + 8;
  static_assert(SLOT % 8192 == 0 && 128 * LDB * 2 <= LDS && RPI * 4 * H * 4 <= LDS, "ring layout");
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
      pcol[j] = kl * H + sub * 128 + (((q & 15) ^ (ttg::ko_v(kl) << 1)) * 8);
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

  for (int s = T_ - 1; s >= 0; --s) {
    const int t = R.dir ? T_ - 1 - s : s;
    const int tn = R.dir ? t - 1 : t + 1;
    const int tp = R.dir ? t + 1 : t - 1;
    const bool last = (s == T_ - 1);
    f32x4 acc[4][C::NCB];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < C::NCB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (!last && !(dbg & 1)) {
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
            src = reinterpret_cast<const char*>(W + (long)r * 32 * H + pcol[j]);
          }
          ttg::dma16(src, img + (uint32_t)pc * 1024u);
        }
      };
      issue(0);
      issue(1);
      issue(2);
#pragma unroll 1
      for (int r = 0; r < NK; ++r) {
        wait_younger<C::NS - 2, C::P>(NK - 1 - r);  // tile r landed (up to 2 younger in flight)
        __builtin_amdgcn_s_barrier();               // everyone's; slot (r + 3) % 4 = r - 1's is free
        if (r + 3 < NK) issue(r + 3);
        const char* sl = lds + (r % C::NS) * C::SLOT;
        uint4 fa[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = frag_kc64(sl, wr * 64 + 16 * i);
        const char* ib = sl + 8192 + ((wc * (H / 4)) >> 7) * 8192;
        const int cb = (wc * (H / 4)) & 127;
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
                                  wc * (H / 4) + 16 * jc + 4 * (lane >> 4)) = make_uint2(w0, w1);
      }
    __syncthreads();
    float bsum[4][8];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) bsum[q][e] = 0.f;
    constexpr int NB = 2;
#pragma unroll 1
    for (int kb = 0; kb < 128 / C::RPI; kb += NB) {
      uint4 vin[NB][7];
#pragma unroll
      for (int kk = 0; kk < NB; ++kk) {
        const int bl = rsub + C::RPI * (kb + kk);
        const bool ok = m0 + bl < a.B && !(dbg & 2);
        const uint32_t oc = ok ? (uint32_t)(bl * H + jg) * 2u : 0x80000000u;
        const uint32_t oy = ok ? (uint32_t)(bl * T_ * (int)a.ldy + jg) * 2u : 0x80000000u;
        const uint32_t os = ok ? (uint32_t)(bl * T_ * 4 * H + jg) * 2u : 0x80000000u;
        vin[kk][0] = ld16_buf(rc, oc, 0);
        vin[kk][1] = ld16_buf(rd, oy, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) vin[kk][2 + q] = ld16_buf(rsv, os, q * 2 * H);
        vin[kk][6] = ld16_buf(ry, oy, 0);
      }
#pragma unroll
      for (int kk = 0; kk < NB; ++kk) {
        const int bl = rsub + C::RPI * (kb + kk);
        const int b = m0 + bl;
        if (b >= a.B) continue;
        float cin[8], dy[8], ar[8], az[8], an[8], gh[8], hp[8], gm[8];
        unpack8(vin[kk][0], cin);
        unpack8(vin[kk][1], dy);
        unpack8(vin[kk][2], ar);
        unpack8(vin[kk][3], az);
        unpack8(vin[kk][4], an);
        unpack8(vin[kk][5], gh);
        unpack8(vin[kk][6], hp);
        unpack8(*reinterpret_cast<const uint4*>(L16 + ((bl * C::LDB + jg) >> 1)), gm);
        if (last && R.dfinal) ld8(R.dfinal + (long)b * a.ldf + jg, cin);
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
        if (dbg & 4) {
          if (o_r[0] == 12345.f) L16[0] = __float_as_uint(o_z[1] + o_n[2] + o_hn[3] + cout[4]);
          continue;
        }
        st8(cr_cur + (long)bl * H + jg, cout);
        const long row = (long)b * T_ + t;
        bf16_t* xw = DGXw + row * a.ldd + jg;
        st8(xw, o_r);
        st8(xw + H, o_z);
        st8_sc1(grs, (int)(((long)bl * T_ * a.ldd + jg + 2 * H) * 2L), o_n, (bf16_t*)nullptr);
        st8(DGHw + row * a.ldd + jg, o_hn);
      }
    }
    __syncthreads();
    float* red = L;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) red[(rsub * 4 + q) * H + jg + e] = bsum[q][e];
    __syncthreads();
    for (int c = tid; c < 4 * H; c += 512) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < C::RPI; ++w) v += red[w * 4 * H + c];
      part[c] += v;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
}

// ---- row-owning backward, 64 rows per workgroup, two workgroups per CU ------------
// gru_bwd_rows runs one 512-thread workgroup per CU, so each CU alternates between its
// MFMA phase (the recurrent product) and its HBM phase (the gate-gradient epilogue) with
// nothing to fill the other unit. Here a workgroup owns 64 rows of one recurrence (256
// threads, 80 KiB of LDS), two are resident per CU, and the second half of the grid
// starts `phase` sleeps late, so the two run out of step: one's epilogue streams while
// the other's product runs.
//   Per step: acc[64 x H] = dL/dgh_{s+1}[64 x 3H] . W_hh[3H x H] in H/256 column passes
//   (a pass's accumulator stays in registers; 4 waves x 64 columns, acc[4][4] each), each
//   K-tile one LDS slot: A 64 rows x 128 B (8 KiB) + two 128-column W_hh sub-images
//   (32 KiB), by LDS-DMA one K-tile ahead. The epilogue stages the whole accumulator as a
//   bf16 [64][H+8] image and updates 8 units of one row per thread, as gru_bwd_rows.
template <int H>
struct BwdR64Cfg {
  static constexpr int NP = H / 256;             // column passes per step
  static constexpr int SLOT = 8192 + 2 * 16384;  // A + two B sub-images
  static constexpr int LDS = 2 * SLOT;           // 80 KiB
  static constexpr int TPR = H / 8;              // epilogue threads per row
  static constexpr int RPI = 256 / TPR;          // rows per epilogue iteration
  static constexpr int LDB = H + 8;              // staged bf16 row pitch
  static_assert(64 * LDB * 2 <= LDS && RPI * 4 * H * 4 <= LDS, "staging fits the slots");
};

template <int H>
__global__ __launch_bounds__(256, 2) void gru_bwd_r64(BwdArgs a, int phase) {
  using C = BwdR64Cfg<H>;
  __shared__ __attribute__((aligned(16))) char lds[C::LDS];
  const int T_ = a.T, ntm = (a.B + 63) / 64;
  const int id = ttg::xcd_remap(blockIdx.x, gridDim.x);
  const int rz = id / ntm, mt = id - rz * ntm;
  const BwdRec R = a.r[rz];
  const int m0 = mt * 64;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const bf16_t* DGX = static_cast<const bf16_t*>(R.dgx);
  const bf16_t* DGH = static_cast<const bf16_t*>(R.dgh);
  bf16_t* DGXw = static_cast<bf16_t*>(R.dgx);
  bf16_t* DGHw = static_cast<bf16_t*>(R.dgh);
  const bf16_t* S = static_cast<const bf16_t*>(R.save);
  const bf16_t* Y = static_cast<const bf16_t*>(R.y);
  const bf16_t* DY = static_cast<const bf16_t*>(R.dy);
  const bf16_t* W = static_cast<const bf16_t*>(R.whh);
  const uint32_t lbase = __builtin_amdgcn_readfirstlane(ttg::lds_addr_of(lds));
  constexpr int NK = 3 * H / 64;  // K-tiles per pass
  const long ldr = (long)T_ * a.ldd;  // elements between batch rows of dgx / dgh
  // DMA pieces (1 KiB per wave-instruction). A: pieces wave + 4j (j < 2) of the 8 KiB KC
  // image; per thread the row and the source chunk its LDS slot holds.
  int arow[2], acol[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int p = (wave + 4 * j) * 64 + lane, row = p >> 3;
    arow[j] = row;
    acol[j] = ((p & 7) ^ ((row >> 1) & 7)) * 8;
  }
  // B: pieces wave + 4j (j < 4) of each 16 KiB KO sub-image: k-row and source column
  int boff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int p = (wave + 4 * j) * 64 + lane, kl = p >> 4, q = p & 15;
    boff[j] = kl * H + (q ^ (ttg::ko_v(kl) << 1)) * 8;
  }
  const int jg = (tid % C::TPR) * 8, rsub = tid / C::TPR;
  float* L = reinterpret_cast<float*>(lds);
  float* part = R.dbias + (long)mt * (4L * H);  // this tile's partial row (zeroed by the host)

  if (blockIdx.x >= gridDim.x / 2)  // second resident workgroup of a CU: start out of step
    for (int i = 0; i < phase; ++i) __builtin_amdgcn_s_sleep(127);

  for (int s = T_ - 1; s >= 0; --s) {
    const int t = R.dir ? T_ - 1 - s : s;
    const int tn = R.dir ? t - 1 : t + 1;
    const int tp = R.dir ? t + 1 : t - 1;
    const bool last = (s == T_ - 1);
    f32x4 acc[C::NP][4][4];
#pragma unroll
    for (int p = 0; p < C::NP; ++p)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[p][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (!last) {
      // A rows: this workgroup's own dL/dgh_{s+1} (r|z columns from dgx, n from dgh)
      const char* asrc[2][2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int b = m0 + arow[j];
        const bool ok = b < a.B;
        asrc[j][0] = ok ? reinterpret_cast<const char*>(DGX + (long)tn * a.ldd + (long)b * ldr + acol[j])
                        : reinterpret_cast<const char*>(ttg::g_tt_zero_page);
        asrc[j][1] = ok ? reinterpret_cast<const char*>(DGH + (long)tn * a.ldd + (long)b * ldr + acol[j] - 2 * H)
                        : reinterpret_cast<const char*>(ttg::g_tt_zero_page);
      }
      // K-tile `it` (pass it / NK, K-tile it % NK) into slot image `img`
      auto issue = [&](int it, uint32_t img) {
        const int p = it / NK, r = it - p * NK;
        const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const bool hi = r * 64 >= 2 * H;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const char* src = asrc[j][hi ? 1 : 0];
          if (src != reinterpret_cast<const char*>(ttg::g_tt_zero_page)) src += (long)r * ttg::KTB;
          ttg::dma16(src, img + (uint32_t)(wv + 4 * j) * 1024u);
        }
        const bf16_t* wb = W + (long)r * 64 * H + p * 256;
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            ttg::dma16(wb + q * 128 + boff[j], img + 8192u + 16384u * q + (uint32_t)(wv + 4 * j) * 1024u);
      };
      constexpr int NIT = C::NP * NK;
      issue(0, lbase);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
#pragma unroll 1
      for (int it = 0; it < NIT; ++it) {
        const int cs = it & 1;
        const char* sl = lds + cs * C::SLOT;
        if (it + 1 < NIT) issue(it + 1, lbase + (cs ^ 1) * C::SLOT);
        const char* ib = sl + 8192 + (wave >> 1) * 16384;
        const int cb = (wave & 1) * 64;
        const int p = it / NK;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {  // one 32-deep half at a time: 32 fragment registers
          uint4 fa[4], fb[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) fa[i] = ttg::frag<bf16_t, false>(sl, 16 * i, ks);
#pragma unroll
          for (int j = 0; j < 4; ++j) fb[j] = ttg::frag<bf16_t, true>(ib, cb + 16 * j, ks);
          __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int pp = 0; pp < C::NP; ++pp) {
            if (pp != p) continue;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
              for (int j = 0; j < 4; ++j) acc[pp][i][j] = ttg::mma<bf16_t>(fa[i], fb[j], acc[pp][i][j]);
          }
          __builtin_amdgcn_s_setprio(0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of K-tile it+1
        __builtin_amdgcn_s_barrier();                      // everyone's; slot cs is free
      }
    }
    // ---- epilogue (as gru_bwd_rows): the accumulator as a bf16 [64][LDB] image
    const long trow = (long)m0 * T_ + t;
    const __amdgpu_buffer_rsrc_t rc =
        tt_rsrc_n(static_cast<const bf16_t*>(R.dh) + (long)((s + 1) & 1) * a.B * H + (long)m0 * H, !last);
    bf16_t* cr_cur = static_cast<bf16_t*>(R.dh) + (long)(s & 1) * a.B * H + (long)m0 * H;
    const __amdgpu_buffer_rsrc_t rd = tt_rsrc_n(DY ? DY + trow * a.ldy : S, DY != nullptr);
    const __amdgpu_buffer_rsrc_t rsv = tt_rsrc_n(S + trow * 4L * H, true);
    const __amdgpu_buffer_rsrc_t ry = tt_rsrc_n(s > 0 ? Y + ((long)m0 * T_ + tp) * a.ldy : S, s > 0);
    const __amdgpu_buffer_rsrc_t grs = tt_rsrc(DGXw + trow * a.ldd);
    uint32_t* L16 = reinterpret_cast<uint32_t*>(lds);
#pragma unroll
    for (int p = 0; p < C::NP; ++p)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            reinterpret_cast<bf16_t*>(lds)[(16 * i + 4 * (lane >> 4) + e) * C::LDB + p * 256 + wave * 64 + 16 * j +
                                           (lane & 15)] = f2bf(acc[p][i][j][e]);
    __syncthreads();
    float bsum[4][8];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) bsum[q][e] = 0.f;
    constexpr int NB = 2;
#pragma unroll 1
    for (int kb = 0; kb < 64 / C::RPI; kb += NB) {
      uint4 vin[NB][7];
#pragma unroll
      for (int kk = 0; kk < NB; ++kk) {
        const int bl = rsub + C::RPI * (kb + kk);
        const bool ok = m0 + bl < a.B;
        const uint32_t oc = ok ? (uint32_t)(bl * H + jg) * 2u : 0x80000000u;
        const uint32_t oy = ok ? (uint32_t)(bl * T_ * (int)a.ldy + jg) * 2u : 0x80000000u;
        const uint32_t os = ok ? (uint32_t)(bl * T_ * 4 * H + jg) * 2u : 0x80000000u;
        vin[kk][0] = ld16_buf(rc, oc, 0);
        vin[kk][1] = ld16_buf(rd, oy, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) vin[kk][2 + q] = ld16_buf(rsv, os, q * 2 * H);
        vin[kk][6] = ld16_buf(ry, oy, 0);
      }
#pragma unroll
      for (int kk = 0; kk < NB; ++kk) {
        const int bl = rsub + C::RPI * (kb + kk);
        const int b = m0 + bl;
        if (b >= a.B) continue;
        float cin[8], dy[8], ar[8], az[8], an[8], gh[8], hp[8], gm[8];
        unpack8(vin[kk][0], cin);
        unpack8(vin[kk][1], dy);
        unpack8(vin[kk][2], ar);
        unpack8(vin[kk][3], az);
        unpack8(vin[kk][4], an);
        unpack8(vin[kk][5], gh);
        unpack8(vin[kk][6], hp);
        unpack8(*reinterpret_cast<const uint4*>(L16 + ((bl * C::LDB + jg) >> 1)), gm);
        if (last && R.dfinal) ld8(R.dfinal + (long)b * a.ldf + jg, cin);
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
        st8(cr_cur + (long)bl * H + jg, cout);
        const long row = (long)b * T_ + t;
        bf16_t* xw = DGXw + row * a.ldd + jg;
        st8(xw, o_r);
        st8(xw + H, o_z);
        st8_sc1(grs, (int)(((long)bl * T_ * a.ldd + jg + 2 * H) * 2L), o_n, (bf16_t*)nullptr);
        st8(DGHw + row * a.ldd + jg, o_hn);
      }
    }
    __syncthreads();  // the image is rewritten by the bias reduction
    float* red = L;  // [RPI][4][H]
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) red[(rsub * 4 + q) * H + jg + e] = bsum[q][e];
    __syncthreads();
    for (int c = tid; c < 4 * H; c += 256) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < C::RPI; ++w) v += red[w * 4 * H + c];
      part[c] += v;
    }
    // this step's dL/dgh and carry feed the next iteration's DMA
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
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
template <int D, bool EW = false>
TT_DEV void fwd_kstep(const bf16_t* W, int H, int Q, int q, int kt, bool mm, const char* hb, char* bst, int& it,
                      int wm, int wn, f32x4 (&acc)[2][3], WTile& X, WTile& Y TT_PROF_PARAM) {
  if constexpr (EW) {
    // early-write order: both sub-steps' fragments requested at once with the ring set's
    // LDS store between them, so the second read latency and the store transfer run under
    // the first sub-step's MFMAs instead of after the last one
    fwd_load_b(W, H, (q + D) % Q, Y);
    const char* ia = hb + kt * (PR * ttg::KTB);
    const char* ib = bst + (it & 1) * P_BST;
    uint4 fa[2][2], fb[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i) fa[0][i] = ttg::frag<bf16_t, false>(ia, wm + 16 * i, 0);
#pragma unroll
    for (int j = 0; j < 3; ++j) fb[0][j] = ttg::frag<bf16_t, false>(ib, wn + 16 * j, 0);
    fwd_store_b(bst + ((it + 1) & 1) * P_BST, X);
#pragma unroll
    for (int i = 0; i < 2; ++i) fa[1][i] = ttg::frag<bf16_t, false>(ia, wm + 16 * i, 1);
#pragma unroll
    for (int j = 0; j < 3; ++j) fb[1][j] = ttg::frag<bf16_t, false>(ib, wn + 16 * j, 1);
    if (mm) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j) acc[i][j] = ttg::mma<bf16_t>(fb[ks][j], fa[ks][i], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    __syncthreads();
    ++it;
    return;
  }
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

// P2 form: two K-tiles per barrier through a 4-stage W_hh ring (the two extra stages are
// the gate staging area, free during the K loop): read K-tiles it, it+1 from stages
// it % 4, (it+1) % 4, store the register pair X (K-tiles it+2, it+3, loaded one interval
// ago) into the two other stages, load it+4, it+5 into the pair Y. The stages written
// here were last read in the previous interval, before its barrier.
TT_DEV char* fwd_stage(char* lds, int i) { return lds + P_HB + (i & 3) * P_BST; }
TT_DEV void fwd_kpair(const bf16_t* W, int H, int Q, int q, int kt, bool mm, const char* hb, char* lds, int& it,
                      int wm, int wn, f32x4 (&acc)[2][3], WTile& X0, WTile& X1, WTile& Y0, WTile& Y1) {
  fwd_load_b(W, H, (q + 4) % Q, Y0);
  fwd_load_b(W, H, (q + 5) % Q, Y1);
  if (mm) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const char* ia = hb + (kt + h) * (PR * ttg::KTB);
      const char* ib = fwd_stage(lds, it + h);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        uint4 fa[2], fb[3];
#pragma unroll
        for (int i = 0; i < 2; ++i) fa[i] = ttg::frag<bf16_t, false>(ia, wm + 16 * i, ks);
#pragma unroll
        for (int j = 0; j < 3; ++j) fb[j] = ttg::frag<bf16_t, false>(ib, wn + 16 * j, ks);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j) acc[i][j] = ttg::mma<bf16_t>(fb[j], fa[i], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
      }
    }
  }
  fwd_store_b(fwd_stage(lds, it + 2), X0);
  fwd_store_b(fwd_stage(lds, it + 3), X1);
  __syncthreads();
  it += 2;
}

// Whh K-tiles in flight in registers: 1, 2 or 4 (D divides H/64); NKT = H/64 when known
// at compile time (0: runtime). A compile-time NKT unrolls the block's K loop, so hipcc's
// vmcnt bookkeeping at its first K-tiles counts the previous block's epilogue stores and
// the gate loads exactly instead of the loop-merged minimum: with one in-order counter
// that minimum made the first W_hh waits of every block also wait for those stores.
// DS (deferred stores): a block's six 16-byte outputs per thread stay packed in registers
// and are issued one per K-tile during the next block's first six K-tiles (the last
// block's after the step loop), so the HBM writes run under the W_hh stream and the MFMAs
// instead of in a burst at every block's end; the first block's six slots are dropped
// stores (out-of-range offset), so every K-tile issues the same count.
template <int D, int NKT, bool P2 = false, bool EW = false, bool DS = false, bool TM = false>
__global__ __launch_bounds__(PNT) void gru_fwd_seq(FwdArgs a) {
  static_assert(!P2 || (D == 4 && NKT % 4 == 0 && NKT > 0), "paired K-tiles: 4 register sets, NKT % 4 == 0");
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
  // TM (time-major rows t*B + b, timing experiment): the resources are rebased every step
  const long r0w = (long)m0 * T_;
  __amdgpu_buffer_rsrc_t rG = tt_rsrc_n(G + r0w * a.ldg, true);
  __amdgpu_buffer_rsrc_t rY = tt_rsrc_n(Yw + r0w * a.ldy, true);
  __amdgpu_buffer_rsrc_t rX1 = tt_rsrc_n(X1 ? X1 + r0w * a.ldy : Yw, X1 != nullptr);
  __amdgpu_buffer_rsrc_t rS = tt_rsrc_n(S + r0w * 4L * H, true);
#ifdef TT_DIAG
  const bool gok = rowok && !(a.dbg & 2), sok = rowok && !(a.dbg & 1);
#else
  const bool gok = rowok, sok = rowok;
#endif
  // experimental: every step's block order starts at boff so the workgroups of one XCD
  // (blockIdx.x = x mod 8) stream different W_hh blocks at the same instant; hreg[i]
  // then holds block (boff + i) mod nblk. Compiled only into the fixed-NKT instances.
  const int boff = (NKT != 0 && a.stagger) ? (int)((blockIdx.x >> 3) % (unsigned)nblk) : 0;
  const int qoff = boff * nkt;

  float hreg[PH_MAX / 64][8];
#pragma unroll
  for (int i = 0; i < PH_MAX / 64; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) hreg[i][e] = 0.f;

  WTile r0, r1, r2, r3;
  if constexpr (P2) {  // K-tiles 0, 1 into stages 0, 1; 2, 3 in the register pair (r0, r1)
    fwd_load_b(W, H, qoff, r0);
    fwd_load_b(W, H, (qoff + 1) % Q, r1);
    fwd_store_b(fwd_stage(lds, 0), r0);
    fwd_store_b(fwd_stage(lds, 1), r1);
    fwd_load_b(W, H, (qoff + 2) % Q, r0);
    fwd_load_b(W, H, (qoff + 3) % Q, r1);
  } else {
    fwd_load_b(W, H, qoff, r0);
    fwd_store_b(bst, r0);
    if (D >= 2) fwd_load_b(W, H, (qoff + 1) % Q, r1);
    if (D >= 4) {
      fwd_load_b(W, H, (qoff + 2) % Q, r2);
      fwd_load_b(W, H, (qoff + 3) % Q, r3);
    }
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
  uint4 pend[6];  // DS: the previous block's packed outputs: Y, S r / z / n / gh_n, X1
  uint32_t poy = 0x80000000u, pos = 0x80000000u;
  if constexpr (DS) {
#pragma unroll
    for (int q = 0; q < 6; ++q) pend[q] = make_uint4(0, 0, 0, 0);
  } else {
#pragma unroll
    for (int q = 0; q < 6; ++q) st16_buf(rY, 0x80000000u + 16u * q, 0, make_uint4(0, 0, 0, 0));
  }
  auto flush = [&](int q) {  // DS: issue pending output q (q compile-time after unrolling)
    if (q == 0) st16_buf(rY, poy, 0, pend[0]);
    else if (q < 5) st16_buf(rS, pos, (q - 1) * 2 * H, pend[q]);
    else st16_buf(rX1, poy, 0, pend[5]);
  };

  for (int s = 0; s < T_; ++s) {
    const int t = R.dir ? T_ - 1 - s : s;
    const long row = (long)b * T_ + t;
    const int lrow = TM ? rl : rl * T_ + t;  // row within this workgroup's resources
    if constexpr (TM) {
      const long tr = (long)t * a.B + m0;
      rG = tt_rsrc_n(G + tr * a.ldg, true);
      rY = tt_rsrc_n(Yw + tr * a.ldy, true);
      rX1 = tt_rsrc_n(X1 ? X1 + tr * a.ldy : Yw, X1 != nullptr);
      rS = tt_rsrc_n(S + tr * 4L * H, true);
    }
#pragma unroll 1
    for (int blk0 = 0; blk0 < nblk; ++blk0) {
      const int blk = blk0 + boff < nblk ? blk0 + boff : blk0 + boff - nblk;
      {
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
#define TT_KS(j, X, Y) fwd_kstep<D, EW>(W, H, Q, blk * nkt + kt + j, kt + j, s > 0, hb, bst, it, wm, wn, acc, X, Y TT_PROF_ARGS)
        if constexpr (P2) {
#pragma unroll
          for (int kt = 0; kt < nkt; kt += 4) {
            fwd_kpair(W, H, Q, blk * nkt + kt, kt, s > 0, hb, lds, it, wm, wn, acc, r0, r1, r2, r3);
            fwd_kpair(W, H, Q, blk * nkt + kt + 2, kt + 2, s > 0, hb, lds, it, wm, wn, acc, r2, r3, r0, r1);
          }
        } else if constexpr (D == 1) {
#pragma unroll
          for (int kt = 0; kt < nkt; ++kt) TT_KS(0, r0, r0);
        } else if constexpr (D == 2) {
#pragma unroll
          for (int kt = 0; kt < nkt; kt += 2) {
            TT_KS(0, r1, r0);
            if constexpr (DS) { if (kt < 6) flush(kt); }
            TT_KS(1, r0, r1);
            if constexpr (DS) { if (kt + 1 < 6) flush(kt + 1); }
          }
        } else {
#pragma unroll
          for (int kt = 0; kt < nkt; kt += 4) {
            TT_KS(0, r1, r0);
            if constexpr (DS) { if (kt < 6) flush(kt); }
            TT_KS(1, r2, r1);
            if constexpr (DS) { if (kt + 1 < 6) flush(kt + 1); }
            TT_KS(2, r3, r2);
            if constexpr (DS) { if (kt + 2 < 6) flush(kt + 2); }
            TT_KS(3, r0, r3);
            if constexpr (DS) { if (kt + 3 < 6) flush(kt + 3); }
          }
        }
#undef TT_KS
        if constexpr (DS) {  // fewer than six K-tiles per block: the rest of the previous block's outputs
#pragma unroll
          for (int q = NKT; q < 6; ++q) flush(q);
        }
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
        if constexpr (P2) __syncthreads();  // stg = ring stages 2, 3: read before the next block restages them
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
          if constexpr (DS) {
            pend[0] = pack8bf(y);
            pend[1] = pack8bf(sr);
            pend[2] = pack8bf(sz);
            pend[3] = pack8bf(sn);
            pend[4] = pack8bf(sg);
            poy = oy;
            pos = os;
          } else {
            st16_buf(rY, oy, 0, pack8bf(y));
            st16_buf(rS, os, 0, pack8bf(sr));
            st16_buf(rS, os, 2 * H, pack8bf(sz));
            st16_buf(rS, os, 4 * H, pack8bf(sn));
            st16_buf(rS, os, 6 * H, pack8bf(sg));
          }
#ifdef TT_DIAG
          if (X1 && a.drop_thresh && !(a.dbg & 32)) {  // 32: X1 copy without the mask hash
#else
          if (X1 && a.drop_thresh) {
#endif
#pragma unroll
            for (int e = 0; e < 8; ++e)
              y[e] *= tt_dropout_scale(R.seed, R.row0 + (uint32_t)row, (uint32_t)(R.col0 + j + e), a.drop_thresh,
                                       a.inv_keep);
          }
          if constexpr (DS) pend[5] = pack8bf(y);
          else st16_buf(rX1, oy, 0, pack8bf(y));
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
        const int blk = i + boff < nblk ? i + boff : i + boff - nblk;
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          w[k] = (uint32_t)f2bf(hreg[i][2 * k]) | ((uint32_t)f2bf(hreg[i][2 * k + 1]) << 16);
        *reinterpret_cast<uint4*>(hb + blk * (PR * ttg::KTB) + ttg::kc_off(rl, tid & 7)) =
            make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
    __syncthreads();
  }
  if constexpr (DS) {
#pragma unroll
    for (int q = 0; q < 6; ++q) flush(q);  // the last block's outputs
  }
#ifdef TT_DIAG
  TT_STAMP(k_end);
  prf[7] = k_end - k_start;
  if (threadIdx.x == 0 && blockIdx.x < 2048)
    for (int i = 0; i < 8; ++i) g_fwd_prof[blockIdx.x][i] = prf[i];
#endif
}

// ---- row-resident forward with the gates in registers (R x H = 65536) -------------
// EXPERIMENT, off by default (option gru_fwd_rr 1 / 2 / 3); bit-identical to gru_fwd_seq
// and measured slower (profiles/r02_gru_fwd_rr_ab.txt).
// R = 128 rows per workgroup at H = 512: twice the rows per streamed W_hh byte of
// gru_fwd_seq. The bf16 h image (R x H x 2 = 128 KiB) and a 2-stage ring of 32-deep
// W_hh K-tiles (2 x 12 KiB) fill the LDS, so there is no room for fp32 gate staging: the
// B-image rows are ordered [slab of 16 units][gate][16 units] and the accumulators hold
// C^T, so a lane owns r, z and n of 4 consecutive units of MI rows per slab and updates
// them in registers with 8-byte G / Y / S accesses. Waves as WM (rows) x WN (slab
// groups); NT 256 = one wave per SIMD, NT 512 = two per SIMD. The fp32 state alone is 128
// registers per lane at NT 512, so the epilogue spills (46-136 registers by variant).
// Measured at configs[2] (4 recurrences, B 8192, T 64): 15.1-17.6 ms vs 7.25 for
// gru_fwd_seq; with the Y / S / X1 stores compiled out (-DRR_DBG=1) the 2 x 4 layout
// takes 6.50 ms, so the 8-byte stores (16 rows x 32 B per wave instruction, each 128-byte
// line completed by four waves) cost ~9.6 ms, not the W_hh stream. H 1024 at 64 rows
// measured W_hh-bound: 92 vs 48 ms per layer at configs[4] (6 MiB W_hh per recurrence
// does not stay in a 4 MiB L2), not instantiated.
#ifndef RR_DBG
#define RR_DBG 0
#endif
constexpr int RR_KTB = 64;                // bytes per W_hh row of a 32-deep K-tile
constexpr int RR_BST = 192 * RR_KTB;      // 12288 per stage
// W image rows of 64 B, chunk c at c ^ ((row >> 1) & 3): conflict-free for the 16-row
// ds_read_b128 fragment groups and the 8-lane ds_write_b128 groups
TT_DEV int rr_w_off(int row, int c) { return row * RR_KTB + ((c ^ ((row >> 1) & 3)) << 4); }

template <int H, int NT, int WN_ = NT / 128>
struct RRCfg {
  static constexpr int R = 65536 / H;     // batch rows per workgroup
  static constexpr int WN = WN_;          // wave columns
  static constexpr int WM = NT / 64 / WN; // wave rows
  static constexpr int MI = R / WM / 16;  // 16-row fragments per wave
  static constexpr int UG = 4 / WN;       // 16-unit slabs per wave
  static constexpr int NB = H / 64;       // 64-unit blocks per step
  static constexpr int NK = H / 32;       // 32-deep K-tiles per block
  static constexpr int Q = NB * NK;       // K-tiles per step
  static constexpr int HB = R * H * 2;    // h image bytes
  static constexpr int LDS = HB + 2 * RR_BST;
  static constexpr int NC = 768 / NT;     // 16-byte W chunks per thread and K-tile (1.5 -> 2)
  static_assert(LDS <= 163840, "row-resident GRU LDS budget");
};

template <int NT>
struct RRTile {
  uint4 v[NT == 256 ? 3 : 2];
};
// per-thread byte offset of chunk id within K-tile (0, 0); the K-tile's own offset
// (blk*64 rows, kt*32 columns) is wave-uniform and goes in soffset. NT 512: chunks t and
// t + 512 (threads < 256; the others' second offset is out of range and reads nothing)
template <int H>
TT_DEV uint32_t rr_w_byte(int id) {
  const int n = id >> 2, c = id & 3;
  const int slab = n / 48, rem = n - slab * 48, g = rem >> 4, u = rem & 15;
  return (uint32_t)(((g * H + slab * 16 + u) * H + c * 8) * 2);
}
template <int H, int NT>
TT_DEV void rr_load_b(__amdgpu_buffer_rsrc_t rW, const uint32_t (&w)[NT == 256 ? 3 : 2], int q, RRTile<NT>& r) {
  constexpr int NK = RRCfg<H, NT>::NK;
  const int blk = q / NK, kt = q - blk * NK;
  const int so = (blk * 64 * H + kt * 32) * 2;
#pragma unroll
  for (int c = 0; c < (NT == 256 ? 3 : 2); ++c) r.v[c] = ld16_buf(rW, w[c], so);
}
template <int NT>
TT_DEV void rr_store_b(char* img, const RRTile<NT>& r) {
  const int t = threadIdx.x;
#pragma unroll
  for (int c = 0; c < (NT == 256 ? 3 : 1); ++c) {
    const int id = t + NT * c;
    *reinterpret_cast<uint4*>(img + rr_w_off(id >> 2, id & 3)) = r.v[c];
  }
  if (NT == 512 && t < 256) *reinterpret_cast<uint4*>(img + rr_w_off((t + 512) >> 2, t & 3)) = r.v[1];
}
TT_DEV uint2 ld8_buf(__amdgpu_buffer_rsrc_t r, uint32_t voff, int soff) {
  typedef unsigned u32x2 __attribute__((vector_size(8)));
  const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, soff, 0);
  return make_uint2(v[0], v[1]);
}
TT_DEV void st8_buf(__amdgpu_buffer_rsrc_t r, uint32_t voff, int soff, uint2 v) {
  typedef unsigned u32x2 __attribute__((vector_size(8)));
  u32x2 w = {v.x, v.y};
  __builtin_amdgcn_raw_buffer_store_b64(w, r, (int)voff, soff, 0);
}
TT_DEV uint2 pack4bf(const float (&f)[4]) {
  return make_uint2((uint32_t)f2bf(f[0]) | ((uint32_t)f2bf(f[1]) << 16),
                    (uint32_t)f2bf(f[2]) | ((uint32_t)f2bf(f[3]) << 16));
}
TT_DEV void unpack4(uint2 v, float (&f)[4]) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xFFFF0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xFFFF0000u);
}

// One 32-deep K-tile: prefetch K-tile q+D into set Y, MFMAs on stage kt&1 (every block
// starts on an even K-tile count), store set X (K-tile q+1) into the other stage, barrier.
template <int H, int NT, int WN, int D>
TT_DEV void rr_kstep(__amdgpu_buffer_rsrc_t rW, const uint32_t (&w)[NT == 256 ? 3 : 2], int q, int kt, bool mm,
                     const char* hb, char* bst, int wm, int wn,
                     f32x4 (&acc)[RRCfg<H, NT, WN>::MI][3 * RRCfg<H, NT, WN>::UG], RRTile<NT>& X, RRTile<NT>& Y) {
  using C = RRCfg<H, NT, WN>;
  const int lane = threadIdx.x & 63;
  rr_load_b<H, NT>(rW, w, (q + D) % C::Q, Y);
  if (mm) {  // h_{-1} = 0: the first step has no recurrent term
    // the A tile offset is opaque to the compiler: folded into immediates it needs a
    // second set of base registers past 64 KiB, which it hoists and spills
    int aoff = (kt >> 1) * (C::R * ttg::KTB);
    asm volatile("" : "+s"(aoff));
    const char* ia = hb + aoff;
    const char* ib = bst + (kt & 1) * RR_BST;
    uint4 fb[3 * C::UG];
#pragma unroll
    for (int j = 0; j < 3 * C::UG; ++j)
      fb[j] = *reinterpret_cast<const uint4*>(ib + rr_w_off(wn + 16 * j + (lane & 15), lane >> 4));
#pragma unroll
    for (int i = 0; i < C::MI; ++i) {
      const uint4 fa = ttg::frag<bf16_t, false>(ia, wm + 16 * i, kt & 1);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < 3 * C::UG; ++j) acc[i][j] = ttg::mma<bf16_t>(fb[j], fa, acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  rr_store_b<NT>(bst + ((kt + 1) & 1) * RR_BST, X);
  __syncthreads();
}

template <int H, int NT, int WN, int D>
__global__ __launch_bounds__(NT) void gru_fwd_rr(FwdArgs a) {
  using C = RRCfg<H, NT, WN>;
  constexpr int R = C::R, MI = C::MI, NB = C::NB, NK = C::NK, UG = C::UG;
  constexpr int NW = NT == 256 ? 3 : 2;
  __shared__ __attribute__((aligned(16))) char lds[C::LDS];
  char* hb = lds;
  char* bst = lds + C::HB;
  const int ntm = (a.B + R - 1) / R;
  const int id = ttg::xcd_remap(blockIdx.x, gridDim.x);
  const int rz = id / ntm;
  const FwdRec Rc = a.r[rz];
  const int T_ = a.T;
  const int m0 = (id - rz * ntm) * R;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wc = wave % WN;
  const int wm = (wave / WN) * (R / C::WM), wn = wc * 48 * UG;
  // first of this lane's 4 units of slab ug within a block: (wc*UG + ug)*16 + 4*(lane>>4)
  const int ub = wc * UG * 16 + 4 * (lane >> 4);
  const bf16_t* G = static_cast<const bf16_t*>(Rc.g);
  bf16_t* Yw = static_cast<bf16_t*>(Rc.y);
  bf16_t* X1 = static_cast<bf16_t*>(Rc.x1);
  bf16_t* S = static_cast<bf16_t*>(Rc.save);
  // buffer resources based at this workgroup's first row (see gru_fwd_seq): a tail row's
  // offset is out of range, so its loads read zeros and its stores are dropped
  const long r0w = (long)m0 * T_;
  const __amdgpu_buffer_rsrc_t rW = tt_rsrc_n(Rc.whh, true);
  const __amdgpu_buffer_rsrc_t rG = tt_rsrc_n(G + r0w * a.ldg, true);
  const __amdgpu_buffer_rsrc_t rY = tt_rsrc_n(Yw + r0w * a.ldy, true);
  const __amdgpu_buffer_rsrc_t rX1 = tt_rsrc_n(X1 ? X1 + r0w * a.ldy : Yw, X1 != nullptr);
  const __amdgpu_buffer_rsrc_t rS = tt_rsrc_n(S + r0w * 4L * H, true);
  uint32_t w[NW];
#pragma unroll
  for (int c = 0; c < NW; ++c) w[c] = rr_w_byte<H>(tid + NT * c);
  if (NT == 512) w[1] = tid < 256 ? rr_w_byte<H>(tid + 512) : 0x80000000u;
  int rl[MI];
  bool ok[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    rl[i] = wm + 16 * i + (lane & 15);
    ok[i] = m0 + rl[i] < a.B;
  }

  // fp32 state: hreg[i][blk][ug][e] = h(row rl[i], unit blk*64 + ub + 16*ug + e); rotated
  // so that hreg[.][0] is always the block being updated
  float hreg[MI][NB][UG][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int k = 0; k < NB; ++k)
#pragma unroll
      for (int u = 0; u < UG; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) hreg[i][k][u][e] = 0.f;

  RRTile<NT> r0, r1, r2, r3;
  rr_load_b<H, NT>(rW, w, 0, r0);
  rr_store_b<NT>(bst, r0);
  if (D >= 2) rr_load_b<H, NT>(rW, w, 1, r1);
  if (D >= 4) {
    rr_load_b<H, NT>(rW, w, 2, r2);
    rr_load_b<H, NT>(rW, w, 3, r3);
  }
  __syncthreads();
  // dropped stores standing in for the epilogue's, so every path into a block's first
  // K-tiles has the same pending count (see gru_fwd_seq)
#pragma unroll
  for (int q = 0; q < 6 * MI * UG; ++q) st8_buf(rY, 0x80000000u + 8u * q, 0, make_uint2(0, 0));

  for (int s = 0; s < T_; ++s) {
    const int t = Rc.dir ? T_ - 1 - s : s;
#pragma unroll 1
    for (int blk = 0; blk < NB; ++blk) {
      uint2 gx[MI][UG][3];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const uint32_t og = ok[i] ? (uint32_t)((rl[i] * T_ + t) * (int)a.ldg + blk * 64 + ub) * 2u : 0x80000000u;
#pragma unroll
        for (int u = 0; u < UG; ++u)
#pragma unroll
          for (int g = 0; g < 3; ++g) gx[i][u][g] = ld8_buf(rG, og, (g * H + 16 * u) * 2);
      }
      float4 bn[UG];
#pragma unroll
      for (int u = 0; u < UG; ++u) bn[u] = *reinterpret_cast<const float4*>(Rc.bhn + blk * 64 + ub + 16 * u);
      f32x4 acc[MI][3 * UG];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 3 * UG; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#define TT_KS(j, X, Y) rr_kstep<H, NT, WN, D>(rW, w, blk * NK + kt + j, kt + j, s > 0, hb, bst, wm, wn, acc, X, Y)
      if constexpr (D == 2) {
#pragma unroll
        for (int kt = 0; kt < NK; kt += 2) { TT_KS(0, r1, r0); TT_KS(1, r0, r1); }
      } else {
#pragma unroll
        for (int kt = 0; kt < NK; kt += 4) { TT_KS(0, r1, r0); TT_KS(1, r2, r1); TT_KS(2, r3, r2); TT_KS(3, r0, r3); }
      }
#undef TT_KS
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int lrow = rl[i] * T_ + t;
        const uint32_t drow = Rc.row0 + (uint32_t)((long)(m0 + rl[i]) * T_ + t);
#pragma unroll
        for (int u = 0; u < UG; ++u) {
          const int j = blk * 64 + ub + 16 * u;
          float xr[4], xz[4], xn[4];
          unpack4(gx[i][u][0], xr);
          unpack4(gx[i][u][1], xz);
          unpack4(gx[i][u][2], xn);
          const float bnv[4] = {bn[u].x, bn[u].y, bn[u].z, bn[u].w};
          float y[4], sr[4], sz[4], sn[4], sg[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            gru_cell(xr[e], xz[e], xn[e], acc[i][3 * u][e], acc[i][3 * u + 1][e], acc[i][3 * u + 2][e], bnv[e],
                     hreg[i][0][u][e], y[e], sr[e], sz[e], sn[e], sg[e]);
          const uint32_t oy = ok[i] ? (uint32_t)(lrow * (int)a.ldy + j) * 2u : 0x80000000u;
          const uint32_t os = ok[i] ? (uint32_t)(lrow * 4 * H + j) * 2u : 0x80000000u;
#if RR_DBG & 1
          if (a.B < 0) {  // never: stores off, data kept live
#endif
          st8_buf(rY, oy, 0, pack4bf(y));
          st8_buf(rS, os, 0, pack4bf(sr));
          st8_buf(rS, os, 2 * H, pack4bf(sz));
          st8_buf(rS, os, 4 * H, pack4bf(sn));
          st8_buf(rS, os, 6 * H, pack4bf(sg));
          if (X1 && a.drop_thresh) {
            float yd[4];
#pragma unroll
            for (int e = 0; e < 4; ++e)
              yd[e] = y[e] * tt_dropout_scale(Rc.seed, drow, (uint32_t)(Rc.col0 + j + e), a.drop_thresh, a.inv_keep);
            st8_buf(rX1, oy, 0, pack4bf(yd));
          } else {
            st8_buf(rX1, oy, 0, pack4bf(y));
          }
#if RR_DBG & 1
          }
#endif
          // the state of block blk moves to the back: hreg[i][0] is always the current block
#pragma unroll
          for (int k = 0; k < NB - 1; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) hreg[i][k][u][e] = hreg[i][k + 1][u][e];
#pragma unroll
          for (int e = 0; e < 4; ++e) hreg[i][NB - 1][u][e] = y[e];
        }
      }
    }
    // h_s -> A operand of step s+1 (every wave finished reading h_{s-1}: the last K-tile
    // ended with a barrier); unit blk*64 + v is chunk v/8 of K-tile blk, half v&4
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int k = 0; k < NB; ++k)
#pragma unroll
        for (int u = 0; u < UG; ++u) {
          const int v = ub + 16 * u;
          *reinterpret_cast<uint2*>(hb + k * (R * ttg::KTB) + ttg::kc_off(rl[i], v >> 3) + (v & 4) * 2) =
              pack4bf(hreg[i][k][u]);
        }
    __syncthreads();
  }
}


// ---- persistent forward with 16 waves (four per SIMD), bf16, H 256 / 512 --------------
// gru_fwd_seq's row-resident scheme -- 64 rows of one recurrence per workgroup, h_{s-1} as
// the bf16 A image in LDS, W_hh streamed every step through a 2-stage LDS ring, the gates
// staged once through LDS -- with twice the waves: 1024 threads as 4 (rows) x 4 (gate
// columns), wave tile 16 x 48, every thread owning 4 units of one row (8-byte gate loads
// and output stores: 16 lanes write a row's whole 128-byte line). At <= 128 VGPRs a SIMD
// holds four waves instead of two, so one wave's fragment-read, W_hh-load and store
// latencies overlap the other waves' MFMAs and gate arithmetic; the price is that every
// B fragment is read by four waves (LDS reads per K-tile 128 KiB instead of 80). Same
// MFMA k order and gate arithmetic as the per-step kernel: bit-identical outputs.
namespace s16 {
constexpr int NT = 1024;
}
struct S16Set {  // one thread's share of a W_hh K-tile (threads < 512 store both chunks)
  uint4 v0, v1;
};
TT_DEV uint4 s16_chunk(const bf16_t* W, int H, int blk, int kt, int id) {
  const int c = id & 7, row = id >> 3, g = row >> 6, u = row & 63;
  return *reinterpret_cast<const uint4*>(W + (long)(g * H + blk * 64 + u) * H + kt * 64 + c * 8);
}
TT_DEV void s16_load_b(const bf16_t* W, int H, int q, int nkt, S16Set& r) {
  const int blk = q / nkt, kt = q - blk * nkt;
  const int t = threadIdx.x;
  r.v0 = s16_chunk(W, H, blk, kt, t);
  // 1536 16-byte chunks per K-tile: the second load of threads >= 512 repeats their first
  // chunk (unconditional, so the set stays in registers) and is not stored
  r.v1 = s16_chunk(W, H, blk, kt, t < 512 ? t + s16::NT : t);
}
TT_DEV void s16_store_b(char* img, const S16Set& r) {
  const int t = threadIdx.x;
  *reinterpret_cast<uint4*>(img + ttg::kc_off(t >> 3, t & 7)) = r.v0;
  if (t < 512) *reinterpret_cast<uint4*>(img + ttg::kc_off((t + s16::NT) >> 3, t & 7)) = r.v1;
}
TT_DEV void st8_bufv(__amdgpu_buffer_rsrc_t r, uint32_t voff, int soff, uint2 v) {  // soff folded
  typedef unsigned u32x2 __attribute__((vector_size(8)));
  u32x2 w = {v.x, v.y};
  __builtin_amdgcn_raw_buffer_store_b64(w, r, (int)(voff + (uint32_t)soff), 0, 0);
}
// one K-tile: refill register set Y with K-tile q+2, MFMAs on stage it&1, set X (K-tile
// q+1) into the other stage, barrier
TT_DEV void s16_kstep(const bf16_t* W, int H, int Q, int nkt, int q, int kt, bool mm, const char* hb, char* bst,
                      int& it, int wm, int wn, f32x4 (&acc)[3], S16Set& X, S16Set& Y) {
  s16_load_b(W, H, (q + 2) % Q, nkt, Y);
  if (mm) {
    const char* ia = hb + kt * (PR * ttg::KTB);
    const char* ib = bst + (it & 1) * P_BST;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const uint4 fa = ttg::frag<bf16_t, false>(ia, wm, ks);
      uint4 fb[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) fb[j] = ttg::frag<bf16_t, false>(ib, wn + 16 * j, ks);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[j] = ttg::mma<bf16_t>(fb[j], fa, acc[j]);  // C^T, as gru_fwd_seq
      __builtin_amdgcn_s_setprio(0);
    }
  }
  s16_store_b(bst + ((it + 1) & 1) * P_BST, X);
  __syncthreads();
  ++it;
}

template <int NKT>
__global__ __launch_bounds__(1024) void gru_fwd_seq16(FwdArgs a) {
  static_assert(NKT == 4 || NKT == 8, "H 256 / 512");
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
  constexpr int nkt = NKT, Q = NKT * NKT;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = (wave >> 2) * 16, wn = (wave & 3) * 48;
  const bf16_t* W = static_cast<const bf16_t*>(R.whh);
  const bf16_t* G = static_cast<const bf16_t*>(R.g);
  bf16_t* Yw = static_cast<bf16_t*>(R.y);
  bf16_t* X1 = static_cast<bf16_t*>(R.x1);
  bf16_t* S = static_cast<bf16_t*>(R.save);
  const int rl = tid >> 4, jg = (tid & 15) * 4;  // epilogue: row rl, units blk*64 + jg .. +4
  const int b = m0 + rl;
  const bool rowok = b < a.B;
  const long r0w = (long)m0 * T_;
  const __amdgpu_buffer_rsrc_t rG = tt_rsrc_n(G + r0w * a.ldg, true);
  const __amdgpu_buffer_rsrc_t rY = tt_rsrc_n(Yw + r0w * a.ldy, true);
  const __amdgpu_buffer_rsrc_t rX1 = tt_rsrc_n(X1 ? X1 + r0w * a.ldy : Yw, X1 != nullptr);
  const __amdgpu_buffer_rsrc_t rS = tt_rsrc_n(S + r0w * 4L * H, true);

  float hreg[NKT][4];  // fp32 state of this thread's units; hreg[0] = the block being updated
#pragma unroll
  for (int i = 0; i < NKT; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) hreg[i][e] = 0.f;
  S16Set r0, r1;
  s16_load_b(W, H, 0, nkt, r0);
  s16_store_b(bst, r0);
  s16_load_b(W, H, 1, nkt, r1);
  int it = 0;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 6; ++q) st8_bufv(rY, 0x80000000u + 8u * q, 0, make_uint2(0, 0));  // as gru_fwd_seq

  for (int s = 0; s < T_; ++s) {
    const int t = R.dir ? T_ - 1 - s : s;
    const long row = (long)b * T_ + t;
    const int lrow = rl * T_ + t;
#pragma unroll 1
    for (int blk = 0; blk < NKT; ++blk) {
      uint2 gx[3];
      const uint32_t og = rowok ? (uint32_t)(lrow * (int)a.ldg + blk * 64 + jg) * 2u : 0x80000000u;
#pragma unroll
      for (int g = 0; g < 3; ++g) gx[g] = ld8_buf(rG, og, g * H * 2);
      const float4 bn4 = *reinterpret_cast<const float4*>(R.bhn + blk * 64 + jg);
      f32x4 acc[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < nkt; kt += 2) {
        s16_kstep(W, H, Q, nkt, blk * nkt + kt, kt, s > 0, hb, bst, it, wm, wn, acc, r1, r0);
        s16_kstep(W, H, Q, nkt, blk * nkt + kt + 1, kt + 1, s > 0, hb, bst, it, wm, wn, acc, r0, r1);
      }
#pragma unroll
      for (int j = 0; j < 3; ++j)
        *reinterpret_cast<f32x4*>(stg + stg_off(wm + (lane & 15), wn + 16 * j + 4 * (lane >> 4))) = acc[j];
      __syncthreads();
      const float4 v0 = *reinterpret_cast<const float4*>(stg + stg_off(rl, 0 * 64 + jg));
      const float4 v1 = *reinterpret_cast<const float4*>(stg + stg_off(rl, 1 * 64 + jg));
      const float4 v2 = *reinterpret_cast<const float4*>(stg + stg_off(rl, 2 * 64 + jg));
      const float lr[4] = {v0.x, v0.y, v0.z, v0.w}, lz[4] = {v1.x, v1.y, v1.z, v1.w}, ln[4] = {v2.x, v2.y, v2.z, v2.w};
      const float bn[4] = {bn4.x, bn4.y, bn4.z, bn4.w};
      float xr[4], xz[4], xn[4], y[4], sr[4], sz[4], sn[4], sg[4];
      unpack4(gx[0], xr);
      unpack4(gx[1], xz);
      unpack4(gx[2], xn);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        gru_cell(xr[e], xz[e], xn[e], lr[e], lz[e], ln[e], bn[e], hreg[0][e], y[e], sr[e], sz[e], sn[e], sg[e]);
      const int j = blk * 64 + jg;
      const uint32_t oy = rowok ? (uint32_t)(lrow * (int)a.ldy + j) * 2u : 0x80000000u;
      const uint32_t os = rowok ? (uint32_t)(lrow * 4 * H + j) * 2u : 0x80000000u;
      st8_bufv(rY, oy, 0, pack4bf(y));
      st8_bufv(rS, os, 0, pack4bf(sr));
      st8_bufv(rS, os, 2 * H, pack4bf(sz));
      st8_bufv(rS, os, 4 * H, pack4bf(sn));
      st8_bufv(rS, os, 6 * H, pack4bf(sg));
      float yd[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        yd[e] = (X1 && a.drop_thresh) ? y[e] * tt_dropout_scale(R.seed, R.row0 + (uint32_t)row, (uint32_t)(R.col0 + j + e),
                                                                 a.drop_thresh, a.inv_keep)
                                      : y[e];
      st8_bufv(rX1, oy, 0, pack4bf(yd));
#pragma unroll
      for (int i = 0; i < NKT - 1; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) hreg[i][e] = hreg[i + 1][e];
#pragma unroll
      for (int e = 0; e < 4; ++e) hreg[NKT - 1][e] = y[e];
    }
    // h_s -> A operand of step s+1 (every wave finished reading h_{s-1}: the last K-tile
    // ended with a barrier); units jg .. +4 are half (jg & 4) of chunk jg >> 3
#pragma unroll
    for (int i = 0; i < NKT; ++i)
      *reinterpret_cast<uint2*>(hb + i * (PR * ttg::KTB) + ttg::kc_off(rl, jg >> 3) + (jg & 4) * 2) = pack4bf(hreg[i]);
    __syncthreads();
  }
}

// ---- wave-owned-rows persistent forward (gru_fwd_wr, bf16, H 256 / 512) ------------------
// Each of the 4 waves (one per SIMD) owns 16 batch rows of one recurrence for all T steps
// and keeps, in its own registers, h_{s-1} as the MFMA operand (bf16, k-step kk = units
// 32kk .. 32kk+31) and the fp32 state h (for the z * h term). So no hidden state touches LDS:
// the whole 160 KiB is a 6-slot ring of W_hh K-tiles (192 gate rows x 64 deep = 24 KiB)
// filled by LDS-DMA five K-tiles ahead, with counted vmcnt waits placed here (every global
// access of the kernel is inline asm, so hipcc inserts none) and one barrier per K-tile.
// The W_hh rows of a 64-unit block are permuted inside the K-tile image so that, with the
// MFMA operands swapped (acc = C^T), a lane's two accumulator fragments of one gate hold 8
// consecutive units of one batch row: exactly the lane's h operand fragment of k-step
// 2*blk + cg for the next step, its fp32 state, and one 16-byte G / Y / S / X1 access.
// Same MFMA sequence along k and the same gate arithmetic as gru_fwd_seq, so the outputs
// are bit-identical to it and to the per-step kernel.
// compile-time loop: f(std::integral_constant<int, I>) for I in [I0, N)
template <int I0, int N, class F>
TT_DEV void static_for(F&& f) {
  if constexpr (I0 < N) {
    f(std::integral_constant<int, I0>{});
    static_for<I0 + 1, N>(f);
  }
}

namespace wr {
constexpr int NT = 256, NW = 4, ROWS = 64;   // 4 waves x 16 batch rows
constexpr int TILE = 192 * ttg::KTB;          // W_hh K-tile image: 192 gate rows x 128 B
constexpr int NSLOT = 6, AHEAD = NSLOT - 1;   // ring slots; K-tiles DMA'd ahead
constexpr int PPW = TILE / 1024 / NW;         // 1 KiB DMA pieces per wave and K-tile (6)
constexpr int NGL = 6, NSTO = 12;             // G loads / stores per lane and block

// vmcnt for the wait that retires K-tile kt of a block in steady state: the number of
// this wave's VMEM operations issued after that K-tile's DMA. Per block, in order:
// K-tile 0: its DMA (of K-tile +AHEAD), the block's G loads; K-tiles 1..: their DMA;
// epilogue: the stores.
constexpr int steady_wait(int nkt, int kt) {
  // walk back from the current point (before K-tile kt's own DMA) to the DMA of
  // K-tile (kt - AHEAD), counting everything issued after it
  int n = 0, b = 0, k = kt;  // position: block offset b (0 = this block), K-tile k
  for (int back = 0; back < AHEAD; ++back) {
    // step to the previous K-tile, counting the ops between
    --k;
    if (k < 0) { k = nkt - 1; --b; n += NSTO; }  // crossed the previous block's epilogue
    if (back < AHEAD - 1) n += PPW;              // that K-tile's DMA is younger than ours
    if (k == 0 && back < AHEAD - 1) n += NGL;    // G loads follow K-tile 0's DMA
    if (k == 0 && back == AHEAD - 1) n += NGL;   // ... also when K-tile 0 issued our DMA
  }
  (void)b;
  return n;
}
}  // namespace wr

TT_DEV uint32_t wr_u32(const void* p, int sh) { return (uint32_t)(((uintptr_t)p) >> sh); }
// 16-byte buffer load / store from inline asm (invisible to hipcc's vmcnt bookkeeping; the
// kernel places every wait). The store ends in s_nop 1: a VALU write of its data VGPRs
// must be two wait states behind it, and hipcc does not see inside the asm.
TT_DEV tt_u32x4 wr_ld16(tt_u32x4 rs, uint32_t voff) {
  tt_u32x4 v;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(voff), "s"(rs) : "memory");
  return v;
}
TT_DEV void wr_st16(tt_u32x4 rs, uint32_t voff, uint4 d) {
  tt_u32x4 v = {d.x, d.y, d.z, d.w};
  asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen\n\ts_nop 1" ::"v"(v), "v"(voff), "s"(rs) : "memory");
}
// descriptor words as SGPRs (base, num_records 0x7fffffff or 0, default format)
TT_DEV tt_u32x4 wr_rsrc(const void* base, bool on) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  tt_u32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32) & 0xFFFFu);
  r[2] = on ? 0x7fffffffu : 0u;
  r[3] = 0x00020000u;
  return r;
}
template <int N>
TT_DEV void wr_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// 16 bytes per lane from buffer rs at voff + soff into LDS at lds_addr + 16 * lane (the
// buffer form of the LDS-DMA: one per-lane 32-bit offset, the per-K-tile offset in soff)
TT_DEV void wr_dma(tt_u32x4 rs, uint32_t voff, uint32_t soff, uint32_t lds_addr) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rs), "s"(lds_addr), "s"(soff)
               : "memory");
}

template <int H>
__global__ __launch_bounds__(wr::NT, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void gru_fwd_wr(FwdArgs a) {
  constexpr int KS = H / 32, NB = H / 64, NKT = H / 64;
  __shared__ __attribute__((aligned(16))) char lds[wr::NSLOT * wr::TILE + H * 4];
  float* bhn = reinterpret_cast<float*>(lds + wr::NSLOT * wr::TILE);
  const int ntm = (a.B + wr::ROWS - 1) / wr::ROWS;
  const int id = ttg::xcd_remap(blockIdx.x, gridDim.x);
  const int rz = id / ntm;
  const FwdRec R = a.r[rz];
  const int T_ = a.T;
  const int m0 = (id - rz * ntm) * wr::ROWS;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lg = lane >> 4;
  const int rl = wave * 16 + (lane & 15);  // this lane's batch row within the workgroup
  const bool rowok = m0 + rl < a.B;
  const long r0w = (long)m0 * T_;
  const tt_u32x4 rG = wr_rsrc(static_cast<const bf16_t*>(R.g) + r0w * a.ldg, true);
  const tt_u32x4 rY = wr_rsrc(static_cast<bf16_t*>(R.y) + r0w * a.ldy, true);
  const tt_u32x4 rX = wr_rsrc(R.x1 ? static_cast<bf16_t*>(R.x1) + r0w * a.ldy : R.y, R.x1 != nullptr);
  const tt_u32x4 rS = wr_rsrc(static_cast<bf16_t*>(R.save) + r0w * 4L * H, true);
  const bool drop = R.x1 != nullptr && a.drop_thresh != 0;
  for (int i = tid; i < H; i += wr::NT) bhn[i] = R.bhn[i];

  // this lane's DMA pieces: image row ir = 8 p + lane/8 (p = wave*PPW + j), 16-byte
  // position lane%8 holds chunk c = pos ^ swz(ir) of W_hh row g*H + 64 blk + unit(ir)
  uint32_t poff[wr::PPW];
#pragma unroll
  for (int j = 0; j < wr::PPW; ++j) {
    const int p = wave * wr::PPW + j, ir = 8 * p + (lane >> 3), pos = lane & 7;
    const int c = pos ^ ((ir >> 1) & 7);
    const int f = ir >> 4, rho = ir & 15;
    const int g = f >> 2, cg = (f >> 1) & 1, pp = f & 1;
    const int u = 32 * cg + 8 * (rho >> 2) + 4 * pp + (rho & 3);
    poff[j] = (uint32_t)(((g * H + u) * H + 8 * c) * 2);
  }
  tt_u32x4 rW = wr_rsrc(R.whh, true);
  rW[2] = (uint32_t)(3 * H * H * 2);  // exact size: offsets past it read zeros
  const uint32_t lbase = __builtin_amdgcn_readfirstlane(ttg::lds_addr_of(lds));
  // DMA of stream K-tile q (block qb = (q / NKT) % NB, K-tile qk = q % NKT) into its slot;
  // past the stream's end an out-of-range offset (zeros), so every wave always issues PPW
  const int QT = (T_ - 1) * NB * NKT;
  auto dma = [&](int q) __attribute__((always_inline)) {
    const int qk = q % NKT, qb = (q / NKT) % NB, slot = q % wr::NSLOT;
    const uint32_t so = q < QT ? (uint32_t)(qb * 64 * H * 2 + qk * ttg::KTB) : 0x40000000u;
    const uint32_t lb = lbase + (uint32_t)(slot * wr::TILE + wave * wr::PPW * 1024);
#pragma unroll
    for (int j = 0; j < wr::PPW; ++j) wr_dma(rW, poff[j], so, lb + (uint32_t)(j * 1024));
  };

  uint4 hA[KS];       // h_{s-1}, bf16, as the MFMA operand of k-step kk
  float st[KS][8];    // fp32 state: units 32 kk + 8 lg + e of row rl
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    hA[kk] = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int e = 0; e < 8; ++e) st[kk][e] = 0.f;
  }

  // G loads of block blk at time t (6 per lane: gates r, z, n of unit groups cg 0 / 1)
  auto load_g = [&](int blk, int t, tt_u32x4 (&gx)[2][3]) __attribute__((always_inline)) {
    const uint32_t og = rowok ? (uint32_t)((rl * T_ + t) * (int)a.ldg + 64 * blk + 8 * lg) * 2u : 0x80000000u;
#pragma unroll
    for (int cg = 0; cg < 2; ++cg)
#pragma unroll
      for (int g = 0; g < 3; ++g) gx[cg][g] = wr_ld16(rG, og + (uint32_t)((g * H + 32 * cg) * 2));
  };
  // epilogue of block blk at time t from the accumulators (C^T fragments f = 4g + 2cg + pp)
  auto epilogue = [&](int blk, int t, const f32x4 (&acc)[12], tt_u32x4 (&gx)[2][3]) __attribute__((always_inline)) {
    const uint32_t oy = rowok ? (uint32_t)((rl * T_ + t) * (int)a.ldy + 64 * blk + 8 * lg) * 2u : 0x80000000u;
    const uint32_t os = rowok ? (uint32_t)((rl * T_ + t) * 4 * H + 64 * blk + 8 * lg) * 2u : 0x80000000u;
    const uint32_t row = R.row0 + (uint32_t)((m0 + rl) * T_ + t);
#pragma unroll
    for (int cg = 0; cg < 2; ++cg) {
      const int kk = 2 * blk + cg;
      float xr[8], xz[8], xn[8], bn[8], y[8], sr[8], sz[8], sn[8], sg[8];
      unpack8(make_uint4(gx[cg][0][0], gx[cg][0][1], gx[cg][0][2], gx[cg][0][3]), xr);
      unpack8(make_uint4(gx[cg][1][0], gx[cg][1][1], gx[cg][1][2], gx[cg][1][3]), xz);
      unpack8(make_uint4(gx[cg][2][0], gx[cg][2][1], gx[cg][2][2], gx[cg][2][3]), xn);
      const float4 b0 = *reinterpret_cast<const float4*>(bhn + 64 * blk + 32 * cg + 8 * lg);
      const float4 b1 = *reinterpret_cast<const float4*>(bhn + 64 * blk + 32 * cg + 8 * lg + 4);
      bn[0] = b0.x; bn[1] = b0.y; bn[2] = b0.z; bn[3] = b0.w;
      bn[4] = b1.x; bn[5] = b1.y; bn[6] = b1.z; bn[7] = b1.w;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int pp = e >> 2, r = e & 3;
        gru_cell(xr[e], xz[e], xn[e], acc[2 * cg + pp][r], acc[4 + 2 * cg + pp][r], acc[8 + 2 * cg + pp][r], bn[e],
                 st[kk][e], y[e], sr[e], sz[e], sn[e], sg[e]);
        st[kk][e] = y[e];
      }
      const uint32_t dc = (uint32_t)(32 * cg * 2);
      wr_st16(rY, oy + dc, pack8bf(y));
      wr_st16(rS, os + dc, pack8bf(sr));
      wr_st16(rS, os + dc + 2 * H, pack8bf(sz));
      wr_st16(rS, os + dc + 4 * H, pack8bf(sn));
      wr_st16(rS, os + dc + 6 * H, pack8bf(sg));
      if (drop) {
        // the mask columns are loop-invariant: opaque here, or hipcc hoists all of them out
        // of the step loop and spills them
        uint32_t cb = (uint32_t)(R.col0 + 64 * blk + 32 * cg + 8 * lg);
        asm volatile("" : "+v"(cb));
#pragma unroll
        for (int e = 0; e < 8; ++e) y[e] *= tt_dropout_scale(R.seed, row, cb + e, a.drop_thresh, a.inv_keep);
      }
      wr_st16(rX, oy + dc, pack8bf(y));
    }
  };
  // one K-tile (64 deep = k-steps 2 kt, 2 kt + 1) of block blk from ring slot q % NSLOT
  auto ktile = [&](int q, int kt, f32x4 (&acc)[12]) __attribute__((always_inline)) {
    const char* img = lds + (q % wr::NSLOT) * wr::TILE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 fb[12];
#pragma unroll
      for (int f = 0; f < 12; ++f) fb[f] = ttg::frag<bf16_t, false>(img, 16 * f, ks);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int f = 0; f < 12; ++f) acc[f] = ttg::mma<bf16_t>(fb[f], hA[2 * kt + ks], acc[f]);
      __builtin_amdgcn_s_setprio(0);
    }
  };
  __syncthreads();  // bhn staged

  // step 0: h_{-1} = 0, gates from G alone
  {
    const int t = R.dir ? T_ - 1 : 0;
    f32x4 acc[12];
#pragma unroll
    for (int f = 0; f < 12; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
    static_for<0, NB>([&](auto bc) __attribute__((always_inline)) {
      constexpr int blk = decltype(bc)::value;
      tt_u32x4 gx[2][3];
      load_g(blk, t, gx);
      wr_wait<0>();
      asm volatile("" : "+v"(gx[0][0]), "+v"(gx[0][1]), "+v"(gx[0][2]), "+v"(gx[1][0]), "+v"(gx[1][1]), "+v"(gx[1][2]));
      epilogue(blk, t, acc, gx);
    });
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) hA[kk] = pack8bf(st[kk]);
  }
  if (T_ == 1) {
    wr_wait<0>();
    return;
  }
  // the stream: K-tiles of steps 1 .. T-1; prologue DMAs K-tiles 0 .. AHEAD-1
#pragma unroll
  for (int q = 0; q < wr::AHEAD; ++q) dma(q);
  int q = 0;
  for (int s = 1; s < T_; ++s) {
    const int t = R.dir ? T_ - 1 - s : s;
    const bool steady = s >= 2;  // step 1: conservative waits (the prologue's history differs)
    static_for<0, NB>([&](auto bc) __attribute__((always_inline)) {
      constexpr int blk = decltype(bc)::value;
      f32x4 acc[12];
#pragma unroll
      for (int f = 0; f < 12; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
      tt_u32x4 gx[2][3];
      static_for<0, NKT>([&](auto kc) __attribute__((always_inline)) {
        constexpr int kt = decltype(kc)::value;
        // K-tile q landed (this wave's pieces), then every wave's
        if (steady) wr_wait<wr::steady_wait(NKT, kt)>();
        else wr_wait<wr::PPW * (wr::AHEAD - 1)>();
        __builtin_amdgcn_s_barrier();
        dma(q + wr::AHEAD);
        if constexpr (kt == 0) load_g(blk, t, gx);
        ktile(q, kt, acc);
        ++q;
      });
      // G of this block: issued after K-tile 0's DMA, followed by NKT-1 K-tiles' DMAs
      wr_wait<wr::PPW * (NKT - 1)>();
      asm volatile("" : "+v"(gx[0][0]), "+v"(gx[0][1]), "+v"(gx[0][2]), "+v"(gx[1][0]), "+v"(gx[1][1]), "+v"(gx[1][2]));
      epilogue(blk, t, acc, gx);
    });
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) hA[kk] = pack8bf(st[kk]);
  }
  wr_wait<0>();  // trailing zero-page DMAs land before the workgroup exits
  __builtin_amdgcn_s_barrier();
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
// 8 * M * (CUs / 8M) <= CUs; every wait is bounded (timeout flag, tt_gru_fwd_xc_status).
typedef __attribute__((address_space(1))) unsigned xc_gu32;
#ifndef XC_OUT_AUX
#define XC_OUT_AUX 0
#endif
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
  bf16_t* xb;     // [groups][2][RR][H] h exchange images (parity = step index & 1)
  unsigned* cnt;  // [groups][CSTR] arrival counters, zeroed before every launch
  unsigned* err;  // set on a wait timeout
  int qg;         // groups per XCD
  int nrec;       // recurrences (groups are dealt to them round-robin)
  int rpg;        // batch rows per group
  int nround;     // rounds of RR rows per group
  int fast_ok;    // the exchange may stay in the XCD's L2 where the group shares one
};

TT_DEV void xc_wait(xc_gu32* cnt, unsigned target, xc_gu32* err) {
  for (unsigned spins = 0;; ++spins) {
    if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return;
    if ((spins & 1023u) == 1023u) {
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
      if (spins > (1u << 22)) {  // several seconds: a member never arrived
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
TT_DEV bool xc_group_on_one_xcd(unsigned* cntw, int M, int mem, bool allowed, xc_gu32* err) {
  __shared__ int s_fast;
  if (threadIdx.x == 0) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xc_gu32* w = (xc_gu32*)(uintptr_t)cntw;
    __hip_atomic_store(w + 8 + mem, (xcc & 15u) + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(w + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    xc_wait(w + 1, (unsigned)M, err);
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

template <int H, bool DROP>
__global__ __launch_bounds__(xc::NT, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void gru_fwd_xc(FwdArgs a, XcWs ws) {
  using C = xc::Cfg<H>;
  constexpr int M = C::M;
  __shared__ __attribute__((aligned(16))) char lds[C::LDS];
  float* stt = reinterpret_cast<float*>(lds);
  char* slots = lds + C::ST;
  float* stg = reinterpret_cast<float*>(lds + C::ST + 2 * C::SLOT);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  uint32_t ho[C::QPW];
  xc_h_offsets<H>(ho);
  // group / member: blocks b and b + 8 share an XCD under round-robin placement
  const int xcd = blockIdx.x & 7, jj = blockIdx.x >> 3;
  const int grp = xcd * ws.qg + jj / M, mem = jj % M;
  const int rz = grp % ws.nrec, gi = grp / ws.nrec;
  const FwdRec R = a.r[rz];
  const int T_ = a.T, B = a.B;
  const int gb0 = gi * ws.rpg;  // first batch row of the group
  xc_gu32* cnt = (xc_gu32*)(uintptr_t)(ws.cnt + grp * xc::CSTR);
  xc_gu32* err = (xc_gu32*)(uintptr_t)ws.err;
  bf16_t* xbg = ws.xb + (long)grp * 2 * xc::RR * H;
  const __amdgpu_buffer_rsrc_t rx[2] = {tt_rsrc(xbg), tt_rsrc(xbg + xc::RR * H)};

  // this wave's W_hh rows: A operand of gate g, K-step kt = rows g*H + 64 mem + 16 wave +
  // (lane & 15), k = 32 kt + 8 (lane >> 4) .. +7; kept in accumulator registers
  tt_u32x4 wa[3][C::NKT];
  {
    const bf16_t* W = static_cast<const bf16_t*>(R.whh);
    // all loads first (one wait), then the moves into the accumulator file
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
      for (int kt = 0; kt < C::NKT; ++kt)
        wa[g][kt] = *reinterpret_cast<const tt_u32x4*>(
            W + (long)(g * H + 64 * mem + 16 * wave + (lane & 15)) * H + kt * 32 + (lane >> 4) * 8);
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
      for (int kt = 0; kt < C::NKT; ++kt) asm volatile("" : "+a"(wa[g][kt]));
  }
  // epilogue ownership: chunk row cr, units j .. j+7 of this member's 64
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

  const bool fast = xc_group_on_one_xcd(ws.cnt + grp * xc::CSTR, M, mem, ws.fast_ok != 0, err);
#ifdef TT_DIAG
  unsigned long long prf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  TT_STAMP(k_start);
#endif
  int idx = 0;  // step counter over all rounds: parity of the exchange image, counter target
  for (int r = 0; r < ws.nround; ++r) {
    const int rb0 = gb0 + r * xc::RR;  // first batch row of the round
    const int nrow = min(min(ws.rpg - r * xc::RR, xc::RR), B - rb0);  // rows of this round (may be <= 0)
    const bool on = nrow > 0;
    const long r0w = (long)(on ? rb0 : 0) * T_;
    const __amdgpu_buffer_rsrc_t rG = tt_rsrc_n(G + r0w * a.ldg, on);
    const __amdgpu_buffer_rsrc_t rY = tt_rsrc_n(Yw + r0w * a.ldy, on);
    const __amdgpu_buffer_rsrc_t rX1 = tt_rsrc_n(X1 ? X1 + r0w * a.ldy : Yw, on && X1 != nullptr);
    const __amdgpu_buffer_rsrc_t rS = tt_rsrc_n(S + r0w * 4L * H, on);
    // a round starts from h_{-1} = 0: zero fp32 state and zero h images, so step 0 runs the
    // same MFMAs as every other step (0 * W = +0 exactly) and the chunk loop below is one
    // basic block (the matrix pipe and the gate arithmetic interleave)
    for (int i = tid; i < (C::ST + 2 * C::SLOT) / 16; i += xc::NT)
      reinterpret_cast<float4*>(lds)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    // gate inputs of chunk c at step s: 3 x 16 bytes per thread, issued a chunk ahead
    // (per-lane offset of row cr; the chunk and gate offsets are wave-uniform)
    const int cstep_g = xc::CR * T_ * (int)a.ldg * 2;
    auto load_g = [&](int s, int c, tt_u32x4 (&gx)[3]) {
      const int t = R.dir ? T_ - 1 - s : s;
      const uint32_t og = c * xc::CR + cr < nrow ? (uint32_t)((cr * T_ + t) * (int)a.ldg + j) * 2u : xc::OOB;
#pragma unroll
      for (int g = 0; g < 3; ++g) gx[g] = __builtin_amdgcn_raw_buffer_load_b128(rG, (int)og, c * cstep_g + g * H * 2, 0);
    };
    // a ring of three gate-input sets: chunk c's in gq[c % 3], requested two chunks ahead
    tt_u32x4 gq[3][3];
    load_g(0, 0, gq[0]);
    load_g(0, 1, gq[1]);
    for (int s = 0; s < T_; ++s, ++idx) {
      const int t = R.dir ? T_ - 1 - s : s;
#ifdef TT_DIAG
      const bool mm = s > 0 && !(a.dbg & 8);  // 8: no exchange loads (timing only)
#else
      const bool mm = s > 0;  // h_{-1} = 0: step 0 reads no exchange image (its slots are zero)
#endif
      TT_STAMP(p0);
      // all members finished step idx-1: its h is complete, and nobody still reads the
      // image this step overwrites (written two steps ago)
#ifdef TT_DIAG
      if (!(a.dbg & 1))
#endif
        if (idx > 0 && tid == 0) xc_wait(cnt, (unsigned)(M * idx), err);
      __syncthreads();
      TT_STAMP(p1);
      const __amdgpu_buffer_rsrc_t rsrc_h = rx[(idx - 1) & 1];
      const __amdgpu_buffer_rsrc_t rdst_h = rx[idx & 1];
      tt_u32x4 hv[C::QPW];
      f32x4 acc[2][3];
      if (mm) {
        xc_load_h<H>(rsrc_h, ho, 0, hv);
        xc_put_h<H>(slots, hv);
        xc_load_h<H>(rsrc_h, ho, 1, hv);
      }
      __syncthreads();
      xc_mfma<H>(slots, wa, acc);
      if (mm) {
        xc_put_h<H>(slots + C::SLOT, hv);
        xc_load_h<H>(rsrc_h, ho, 2, hv);
      }
      xc_stage(stg, acc);
      __syncthreads();
      // the gates and fp32 state of chunk c into registers, right after its staging barrier:
      // the arithmetic then depends on registers only and interleaves with the next MFMAs
      float lr[8], lz[8], ln[8], hp[8];
      auto read_gates = [&](int c) {
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
          hp[4 * h] = p.x; hp[4 * h + 1] = p.y; hp[4 * h + 2] = p.z; hp[4 * h + 3] = p.w;
        }
      };
      read_gates(0);
      TT_STAMP(p2);
#pragma unroll
      for (int c = 0; c < xc::NCH; ++c) {
        TT_STAMP(c0);
        if (c + 2 < xc::NCH) load_g(s, c + 2, gq[(c + 2) % 3]);
        // ---- gate arithmetic of chunk c, woven into the MFMAs of chunk c+1: one K-step
        // (six MFMAs) and a share of the cells per scheduling region, so the matrix pipe
        // and the VALU run side by side in each wave (one wave per SIMD)
        {
          const int rr = c * xc::CR + cr;
          const bool ok = rr < nrow;
          float xr[8], xz[8], xn[8], y[8], sr[8], sz[8], sn[8], sg[8], msk[8];
          const uint32_t grow = (uint32_t)(rb0 + rr) * (uint32_t)T_ + (uint32_t)t;
          const tt_u32x4(&gcur)[3] = gq[c % 3];
          unpack8(make_uint4(gcur[0][0], gcur[0][1], gcur[0][2], gcur[0][3]), xr);
          unpack8(make_uint4(gcur[1][0], gcur[1][1], gcur[1][2], gcur[1][3]), xz);
          unpack8(make_uint4(gcur[2][0], gcur[2][1], gcur[2][2], gcur[2][3]), xn);
          if (c + 1 < xc::NCH) {
            constexpr int NKT = C::NKT;
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
              if constexpr (DROP) {  // the dropout mask of element e (independent of the cell)
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
                  // opaque inputs and outputs pin the cell to this K-step's region
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
          // the exchange image (all rows): L2-resident where the group shares an XCD
          if (fast) st16_buf(rdst_h, (uint32_t)(rr * H + j) * 2u, 0, yb);
          else st16_buf_sc1(rdst_h, (uint32_t)(rr * H + j) * 2u, 0, yb);
          // exactly 6 stores follow (Y, S r/z/n/gh_n, X1): the publish waits
          // for the exchange store only, not for them
          asm volatile("" ::: "memory");
          const int lrow = rr * T_ + t;
          uint32_t oy = ok ? (uint32_t)(lrow * (int)a.ldy + j) * 2u : xc::OOB;
          uint32_t os = ok ? (uint32_t)(lrow * 4 * H + j) * 2u : xc::OOB;
#ifdef TT_DIAG
          if (a.dbg & 2) oy = os = xc::OOB;  // 2: no Y / S / X1 stores (dropped)
#endif
          st16_buf(rY, oy, 0, yb);
          st16_buf(rS, os, 0, pack8bf(sr));
          st16_buf(rS, os, 2 * H, pack8bf(sz));
          st16_buf(rS, os, 4 * H, pack8bf(sn));
          st16_buf(rS, os, 6 * H, pack8bf(sg));
          if constexpr (DROP) {
#pragma unroll
            for (int e = 0; e < 8; ++e) y[e] *= msk[e];
            st16_buf(rX1, oy, 0, pack8bf(y));
          } else {
            st16_buf(rX1, oy, 0, yb);  // dropped unless an eval X1 copy was asked for
          }
        }
        if (mm && c + 2 < xc::NCH) {
          xc_put_h<H>(slots + (c & 1) * C::SLOT, hv);  // chunk c+2 into the slot chunk c used
          if (c + 3 < xc::NCH) xc_load_h<H>(rsrc_h, ho, c + 3, hv);
        }
        TT_STAMP(c1);
        __syncthreads();
        if (c + 1 < xc::NCH) {
          xc_stage(stg, acc);
          __syncthreads();
          read_gates(c + 1);
        }
        TT_STAMP(c2);
        TT_ACC(2, c1 - c0);  // chunk: MFMAs + gate arithmetic + h restage issued
        TT_ACC(3, c2 - c1);  // chunk barriers + gate staging
      }
      TT_STAMP(p3);
      // publish h_s: every wave drains its stores (the exchange stores are write-through),
      // then one lane counts the workgroup in
#ifdef TT_DIAG
      if (!(a.dbg & 4))
#endif
        asm volatile("s_nop 0\n\ts_waitcnt vmcnt(6)" ::: "memory");  // all but the last chunk's 6 output stores (s_nop 0: a marker for tests/test_host.py)
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (s + 1 < T_) {
        load_g(s + 1, 0, gq[0]);
        load_g(s + 1, 1, gq[1]);
      }
      TT_STAMP(p4);
      TT_ACC(0, p1 - p0);  // wait for the group + barrier
      TT_ACC(1, p2 - p1);  // prologue: chunks 0-1 of h, MFMAs of chunk 0
      TT_ACC(4, p4 - p3);  // drain + publish
    }
  }
#ifdef TT_DIAG
  TT_STAMP(k_end);
  prf[7] = k_end - k_start;
  if (threadIdx.x == 0 && blockIdx.x < 2048)
    for (int i = 0; i < 8; ++i) g_fwd_prof[blockIdx.x][i] = prf[i];
#endif
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
  const int xcd = blockIdx.x & 7, jj = blockIdx.x >> 3;
  const int grp = xcd * ws.qg + jj / M, mem = jj % M;
  const int rz = grp % ws.nrec, gi = grp / ws.nrec;
  const FwdRec R = a.r[rz];
  const int T_ = a.T, B = a.B;
  const int gb0 = gi * ws.rpg;
  xc_gu32* cw = (xc_gu32*)(uintptr_t)(ws.cnt + grp * xc::CSTR);
  xc_gu32* cntA = cw;      // arrivals of half steps A (chunks 0-3)
  xc_gu32* cntB = cw + 2;  // and B (chunks 4-7)
  xc_gu32* err = (xc_gu32*)(uintptr_t)ws.err;
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
  const bool fast = xc_group_on_one_xcd(ws.cnt + grp * xc::CSTR, M, mem, ws.fast_ok != 0, err);
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
    for (int g = 0; g < 3; ++g) gx[g] = __builtin_amdgcn_raw_buffer_load_b128(rG, (int)og, g * H * 2, 0);
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
        if (c == 0 && idx > 0) xc_wait(cntB, (unsigned)(M * idx), err);
        if (c == 4 && has_next) xc_wait(cntA, (unsigned)(M * (idx + 1)), err);
      }
      __syncthreads();
      if (tid == 0 && c == 3) __hip_atomic_fetch_add(cntA, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (tid == 0 && c == 7) __hip_atomic_fetch_add(cntB, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

// ---- column-split forward for H 1024 (gru_fwd_xk, bf16; configs[4]'s hidden 512) -------
// At H 1024 a 64-unit member's W_hh rows (192 x 1024, 384 KiB) exceed the accumulator
// file, so a member owns 32 units (96 gate rows x 1024 = 192 KiB) and a group is 32
// workgroups: one XCD. The 96 gate columns are 6 MFMA tiles, so the 4 waves split K
// instead (256 each, 8 K-steps x 6 tiles = 192 AGPRs) and every LDS fragment is read by one
// wave only; the four partial products meet in LDS and are summed in a fixed order by the
// gate arithmetic (so results agree with the per-step kernel to rounding, not bitwise).
// Rows in rounds of 256, chunks of 32: ONE 64 KiB h chunk image in LDS (the next chunk
// waits in registers and is written in right after the MFMAs that read the image); every
// thread updates 4 units of one row (the member's 32 units of a row are 64 bytes).
// Exchange, counters, XCD check and the per-step wait as gru_fwd_xc.
namespace xk {
constexpr int NT = 256, CR = 32, RR = 256, NCH = RR / CR, NU = 32;
constexpr int PSTR = 100;  // partial-product row stride in floats (96 + 4: conflict-free rows)
constexpr int SSTR = 36;   // fp32 state row stride (32 units + 16 B)
template <int H>
struct Cfg {
  static constexpr int M = H / NU;
  static constexpr int NKW = H / 4 / 32;            // K-steps per wave
  static constexpr int QPW = CR * H * 2 / 16 / NT;  // 16-byte h loads per thread and chunk
  static constexpr int SLOT = CR * H * 2;           // [K-step][row block][16 B x 64 lanes]
  static constexpr int PST = 4 * CR * PSTR * 4;
  static constexpr int ST = RR * SSTR * 4;
  static constexpr int LDS = SLOT + PST + ST;
};
static_assert(Cfg<1024>::LDS <= 163840, "gru_fwd_xk LDS budget");
}  // namespace xk

template <int H, bool DROP>
__global__ __launch_bounds__(xk::NT, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void gru_fwd_xk(FwdArgs a, XcWs ws) {
  using C = xk::Cfg<H>;
  constexpr int M = C::M, NKW = C::NKW, QPW = C::QPW;
  __shared__ __attribute__((aligned(16))) char lds[C::LDS];
  char* slot = lds;
  float* pst = reinterpret_cast<float*>(lds + C::SLOT);
  float* stt = reinterpret_cast<float*>(lds + C::SLOT + C::PST);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int xcd = blockIdx.x & 7, jj = blockIdx.x >> 3;
  const int grp = xcd * ws.qg + jj / M, mem = jj % M;
  const int rz = grp % ws.nrec, gi = grp / ws.nrec;
  const FwdRec R = a.r[rz];
  const int T_ = a.T, B = a.B;
  const int gb0 = gi * ws.rpg;
  xc_gu32* cnt = (xc_gu32*)(uintptr_t)(ws.cnt + grp * xc::CSTR);
  xc_gu32* err = (xc_gu32*)(uintptr_t)ws.err;
  bf16_t* xbg = ws.xb + (long)grp * 2 * xk::RR * H;
  const __amdgpu_buffer_rsrc_t rx[2] = {tt_rsrc(xbg), tt_rsrc(xbg + xk::RR * H)};
  // W_hh tile mt of this wave's K quarter: gate mt >> 1, units 32 mem + 16 (mt & 1) + lane&15
  tt_u32x4 wa[6][NKW];
  {
    const bf16_t* W = static_cast<const bf16_t*>(R.whh);
#pragma unroll
    for (int mt = 0; mt < 6; ++mt)
#pragma unroll
      for (int ks = 0; ks < NKW; ++ks)
        wa[mt][ks] = *reinterpret_cast<const tt_u32x4*>(
            W + (long)((mt >> 1) * H + xk::NU * mem + 16 * (mt & 1) + (lane & 15)) * H + (wave * NKW + ks) * 32 +
            (lane >> 4) * 8);
#pragma unroll
    for (int mt = 0; mt < 6; ++mt)
#pragma unroll
      for (int ks = 0; ks < NKW; ++ks) asm volatile("" : "+a"(wa[mt][ks]));
  }
  // h loads: 16-byte unit q = p * 256 + tid of the chunk image = K-step q >> 7, row block
  // (q >> 6) & 1, kq (q >> 4) & 3, row q & 15: piece p is 2 K-steps (128 B) further along
  const uint32_t xo0 =
      (uint32_t)(((((tid >> 6) & 1) * 16 + (tid & 15)) * H + (tid >> 7) * 32 + ((tid >> 4) & 3) * 8) * 2);
  // epilogue ownership: row er, units u0 .. u0+3 of the member's 32
  const int er = tid >> 3, u0 = (tid & 7) * 4, j = xk::NU * mem + u0;
  float bn[4];
  {
    const float4 b4 = *reinterpret_cast<const float4*>(R.bhn + j);
    bn[0] = b4.x; bn[1] = b4.y; bn[2] = b4.z; bn[3] = b4.w;
  }
  const bf16_t* G = static_cast<const bf16_t*>(R.g);
  bf16_t* Yw = static_cast<bf16_t*>(R.y);
  bf16_t* X1 = static_cast<bf16_t*>(R.x1);
  bf16_t* S = static_cast<bf16_t*>(R.save);
  const bool fast = xc_group_on_one_xcd(ws.cnt + grp * xc::CSTR, M, mem, ws.fast_ok != 0, err);
  auto st8b = [](__amdgpu_buffer_rsrc_t r, uint32_t off, uint2 v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v), r,
                                          (int)off, 0, 0);
  };
  auto pk4 = [](const float (&f)[4]) {
    return make_uint2((uint32_t)f2bf(f[0]) | ((uint32_t)f2bf(f[1]) << 16),
                      (uint32_t)f2bf(f[2]) | ((uint32_t)f2bf(f[3]) << 16));
  };
  int idx = 0;
  for (int r = 0; r < ws.nround; ++r) {
    const int rb0 = gb0 + r * xk::RR;
    const int nrow = min(min(ws.rpg - r * xk::RR, xk::RR), B - rb0);
    const bool on = nrow > 0;
    const long r0w = (long)(on ? rb0 : 0) * T_;
    const __amdgpu_buffer_rsrc_t rG = tt_rsrc_n(G + r0w * a.ldg, on);
    const __amdgpu_buffer_rsrc_t rY = tt_rsrc_n(Yw + r0w * a.ldy, on);
    const __amdgpu_buffer_rsrc_t rX1 = tt_rsrc_n(X1 ? X1 + r0w * a.ldy : Yw, on && X1 != nullptr);
    const __amdgpu_buffer_rsrc_t rS = tt_rsrc_n(S + r0w * 4L * H, on);
    for (int i = tid; i < C::SLOT / 16; i += xk::NT)
      reinterpret_cast<float4*>(slot)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i = tid; i < C::ST / 16; i += xk::NT)
      reinterpret_cast<float4*>(stt)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = 0; s < T_; ++s, ++idx) {
      const int t = R.dir ? T_ - 1 - s : s;
      const bool mm = s > 0;
      if (idx > 0 && tid == 0) xc_wait(cnt, (unsigned)(M * idx), err);
      __syncthreads();
      const __amdgpu_buffer_rsrc_t rsrc = rx[(idx - 1) & 1];
      const __amdgpu_buffer_rsrc_t rdst = rx[idx & 1];
      tt_u32x4 hv[QPW];
      auto load_h = [&](int c) {
#pragma unroll
        for (int p = 0; p < QPW; ++p)
          hv[p] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(xo0 + p * 128), c * xk::CR * H * 2, 16);
      };
      auto put_h = [&]() {
#pragma unroll
        for (int p = 0; p < QPW; ++p) *reinterpret_cast<tt_u32x4*>(slot + tid * 16 + p * 4096) = hv[p];
      };
      f32x4 acc[2][6];
      auto mfma = [&]() {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
          for (int mt = 0; mt < 6; ++mt) acc[rb][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
        const char* base = slot + wave * NKW * 2048 + lane * 16;
        tt_u32x4 f[2][2];
        f[0][0] = *reinterpret_cast<const tt_u32x4*>(base);
        f[0][1] = *reinterpret_cast<const tt_u32x4*>(base + 1024);
#pragma unroll
        for (int ks = 0; ks < NKW; ++ks) {
          if (ks + 1 < NKW) {
            f[(ks + 1) & 1][0] = *reinterpret_cast<const tt_u32x4*>(base + (ks + 1) * 2048);
            f[(ks + 1) & 1][1] = *reinterpret_cast<const tt_u32x4*>(base + (ks + 1) * 2048 + 1024);
          }
#pragma unroll
          for (int rb = 0; rb < 2; ++rb)
#pragma unroll
            for (int mt = 0; mt < 6; ++mt)
              acc[rb][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  __builtin_bit_cast(bf16x8v, wa[mt][ks]), __builtin_bit_cast(bf16x8v, f[ks & 1][rb]), acc[rb][mt], 0, 0, 0);
        }
      };
      auto stage = [&]() {  // C^T: row 16 rb + (lane & 15), columns 16 mt + 4 (lane >> 4) .. +3
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
          for (int mt = 0; mt < 6; ++mt)
            *reinterpret_cast<f32x4*>(pst + (wave * xk::CR + 16 * rb + (lane & 15)) * xk::PSTR + 16 * mt +
                                      4 * (lane >> 4)) = acc[rb][mt];
      };
      float gh[3][4];
      auto read_part = [&]() {  // column of gate g, unit u = 32 g + u; K quarters summed in order
#pragma unroll
        for (int g = 0; g < 3; ++g) {
          float4 v = *reinterpret_cast<const float4*>(pst + (0 * xk::CR + er) * xk::PSTR + 32 * g + u0);
#pragma unroll
          for (int w = 1; w < 4; ++w) {
            const float4 q = *reinterpret_cast<const float4*>(pst + (w * xk::CR + er) * xk::PSTR + 32 * g + u0);
            v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w;
          }
          gh[g][0] = v.x; gh[g][1] = v.y; gh[g][2] = v.z; gh[g][3] = v.w;
        }
      };
      uint2 gx[3];
      auto load_g = [&](int c) {
        const int rr = c * xk::CR + er;
        const uint32_t og = rr < nrow ? (uint32_t)((rr * T_ + t) * (int)a.ldg + j) * 2u : xc::OOB;
#pragma unroll
        for (int g = 0; g < 3; ++g) {
          const auto w = __builtin_amdgcn_raw_buffer_load_b64(rG, (int)og, g * H * 2, 0);
          gx[g] = make_uint2(w[0], w[1]);
        }
      };
      // prologue: chunk 0 into the image, chunk 1 in registers; MFMAs of chunk 0
      if (mm) {
        load_h(0);
        put_h();
        load_h(1);
      }
      load_g(0);
      __syncthreads();
      mfma();
      __syncthreads();  // every wave done reading chunk 0's image
      stage();
      if (mm) {
        put_h();
        load_h(2);
      }
      __syncthreads();
      read_part();
#pragma unroll 1
      for (int c = 0; c < xk::NCH; ++c) {
        const uint2 gcur[3] = {gx[0], gx[1], gx[2]};
        const float gc[3][4] = {{gh[0][0], gh[0][1], gh[0][2], gh[0][3]},
                                {gh[1][0], gh[1][1], gh[1][2], gh[1][3]},
                                {gh[2][0], gh[2][1], gh[2][2], gh[2][3]}};
        if (c + 1 < xk::NCH) {
          load_g(c + 1);
          mfma();  // chunk c+1 from the image
        }
        {
          const int rr = c * xk::CR + er;
          const bool ok = rr < nrow;
          const float4 hp4 = *reinterpret_cast<const float4*>(stt + rr * xk::SSTR + u0);
          const float hp[4] = {hp4.x, hp4.y, hp4.z, hp4.w};
          float y[4], sr[4], sz[4], sn[4], sg[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const uint32_t w0 = e < 2 ? gcur[0].x : gcur[0].y, w1 = e < 2 ? gcur[1].x : gcur[1].y,
                           w2 = e < 2 ? gcur[2].x : gcur[2].y;
            const float xr = __uint_as_float((e & 1) ? w0 & 0xFFFF0000u : w0 << 16);
            const float xz = __uint_as_float((e & 1) ? w1 & 0xFFFF0000u : w1 << 16);
            const float xn = __uint_as_float((e & 1) ? w2 & 0xFFFF0000u : w2 << 16);
            gru_cell(xr, xz, xn, gc[0][e], gc[1][e], gc[2][e], bn[e], hp[e], y[e], sr[e], sz[e], sn[e], sg[e]);
          }
          *reinterpret_cast<float4*>(stt + rr * xk::SSTR + u0) = make_float4(y[0], y[1], y[2], y[3]);
          const uint2 yb = pk4(y);
          const uint32_t ox = (uint32_t)(rr * H + j) * 2u;
          if (fast) st8b(rdst, ox, yb);
          else __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, yb), rdst, (int)ox, 0, 16);
          const int lrow = rr * T_ + t;
          const uint32_t oy = ok ? (uint32_t)(lrow * (int)a.ldy + j) * 2u : xc::OOB;
          const uint32_t os = ok ? (uint32_t)(lrow * 4 * H + j) * 2u : xc::OOB;
          st8b(rY, oy, yb);
          st8b(rS, os, pk4(sr));
          st8b(rS, os + 2u * H, pk4(sz));
          st8b(rS, os + 4u * H, pk4(sn));
          st8b(rS, os + 6u * H, pk4(sg));
          if constexpr (DROP) {
            const uint32_t grow = (uint32_t)(rb0 + rr) * (uint32_t)T_ + (uint32_t)t;
#pragma unroll
            for (int e = 0; e < 4; ++e)
              y[e] *= tt_dropout_scale(R.seed, R.row0 + grow, (uint32_t)(R.col0 + j + e), a.drop_thresh, a.inv_keep);
            st8b(rX1, oy, pk4(y));
          } else {
            st8b(rX1, oy, yb);
          }
        }
        __syncthreads();  // chunk c+1's image and chunk c's partial products fully read
        if (c + 1 < xk::NCH) {
          stage();
          if (mm && c + 2 < xk::NCH) {
            put_h();  // chunk c+2 into the image
            if (c + 3 < xk::NCH) load_h(c + 3);
          }
          __syncthreads();
          read_part();
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---- column-split persistent backward (gru_bwd_xc, bf16, H 256 / 512) ---------------
// The BPTT of gru_fwd_xc's split (gru_bwd_rows' per-step math): member m of a group of
// M = H/64 workgroups owns hidden units [64m, 64m+64) of the group's rows and keeps
// W_hh[:, its units] (3H x 64, 192 KiB at H 512) in the accumulator registers. Per step
//   dh_t[rows, own units] = dL/dgh_{t+1}[rows, 3H] . W_hh[3H, own units]
// needs the gate gradients of ALL units (r | z | W_hn h blocks), so the members exchange
// those instead: each publishes its 3 x 64 columns of the step's dL/dgh through a group
// image (16-byte write-through stores, drain, arrival counter) and reads back the 3H
// columns of every row (write-through loads) -- 3H * 2 bytes per row and step of L2
// traffic instead of the whole W_hh per 128 rows. The 4 waves split K (3H/4 each, so every
// operand fragment is read from LDS once per chunk and feeds four MFMAs); the four partial
// products are summed in a fixed order by the gate arithmetic. Rows run in rounds of 256
// with the bf16 carry dh*z in LDS, in chunks of 16 rows. Same gate arithmetic and the same
// bf16 rounding points as gru_bwd_rows (the accumulator, the carry); the K summation order
// differs (four quarter sums), so results agree with it to bf16 rounding
// (tests/test_gpu_gru_persistent.py). Bias partials: one row per group (row gi of the
// recurrence's partial block), written once at the end.
namespace xb {
constexpr int NT = 256;
constexpr int CR = 16;                  // rows per chunk
constexpr int RR = 256;                 // rows per round
constexpr int NCH = RR / CR;
constexpr int PSTG = 4 * CR * 64 * 4;   // four partial products [16 rows][64 units] fp32
template <int H>
struct Cfg {
  static constexpr int M = H / 64;
  static constexpr int KW = 3 * H / 4;       // K per wave
  static constexpr int NKS = KW / 32;        // K-steps per wave
  static constexpr int QPT = 3 * H * CR * 2 / 16 / NT;  // 16-byte exchange loads per thread and chunk
  static constexpr int SLOT = CR * 3 * H * 2;          // gradient chunk image [K-step][kq][row] x 16 B
  static constexpr int CARRY = RR * 64 * 2;            // bf16 dh * z of the round's rows
  static constexpr int LDS = 2 * SLOT + PSTG + CARRY;
};
static_assert(Cfg<512>::LDS <= 163840 && Cfg<256>::LDS <= 163840, "gru_bwd_xc LDS budget");
TT_DEV int pstg_off(int w, int row, int u) {  // 16-byte chunk (u >> 2) of row at (u >> 2) ^ row
  return ((w * CR + row) * 16 + (((u >> 2) ^ row) & 15)) * 4 + (u & 3);
}
}  // namespace xb

struct XbWs {
  bf16_t* xb;     // [groups][2][RR][3H] exchange images of dL/dgh
  unsigned* cnt;
  unsigned* err;
  int qg, nrec, rpg, nround;
  int fast_ok;
};

template <int H>
__global__ __launch_bounds__(xb::NT, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void gru_bwd_xc(BwdArgs a, XbWs ws) {
  using C = xb::Cfg<H>;
  constexpr int M = C::M, NKS = C::NKS, QPT = C::QPT;
  __shared__ __attribute__((aligned(16))) char lds[C::LDS];
  char* slots = lds;
  float* pst = reinterpret_cast<float*>(lds + 2 * C::SLOT);
  bf16_t* carry = reinterpret_cast<bf16_t*>(lds + 2 * C::SLOT + xb::PSTG);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int xcd = blockIdx.x & 7, jj = blockIdx.x >> 3;
  const int grp = xcd * ws.qg + jj / M, mem = jj % M;
  const int rz = grp % ws.nrec, gi = grp / ws.nrec;
  const BwdRec R = a.r[rz];
  const int T_ = a.T, B = a.B;
  const int gb0 = gi * ws.rpg;
  xc_gu32* cnt = (xc_gu32*)(uintptr_t)(ws.cnt + grp * xc::CSTR);
  xc_gu32* err = (xc_gu32*)(uintptr_t)ws.err;
  bf16_t* xbg = ws.xb + (long)grp * 2 * xb::RR * 3 * H;
  const __amdgpu_buffer_rsrc_t rx[2] = {tt_rsrc(xbg), tt_rsrc(xbg + xb::RR * 3 * H)};

  // W_hh^T fragments (A operand of the C^T product): wave w covers k in [w KW, (w+1) KW);
  // K-step ks, unit tile nt: lane holds W_hh[k0 + 8 (lane >> 4) + i][64 mem + 16 nt + (lane & 15)]
  tt_u32x4 wa[NKS][4];
  {
    const bf16_t* W = static_cast<const bf16_t*>(R.whh);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int k0 = wave * C::KW + ks * 32 + (lane >> 4) * 8, u = 64 * mem + 16 * nt + (lane & 15);
        uint32_t w4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          w4[i] = (uint32_t)W[(long)(k0 + 2 * i) * H + u] | ((uint32_t)W[(long)(k0 + 2 * i + 1) * H + u] << 16);
        wa[ks][nt] = tt_u32x4{w4[0], w4[1], w4[2], w4[3]};
      }
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) asm volatile("" : "+a"(wa[ks][nt]));
  }
  // exchange loads: thread piece p of a chunk = 16 bytes (8 k) of one row; the chunk image
  // is [K-step][kq][row] x 16 B, so the MFMA fragment of K-step kt is 1 KiB contiguous
  // (16-byte unit q = p * 256 + tid of the image: K-step q >> 6, kq (q >> 4) & 3, row q & 15,
  // so piece p is 256 bytes further along the exchange row and 4 KiB further in LDS)
  const uint32_t xo0 = (uint32_t)(((tid & 15) * 3 * H + (tid >> 6) * 32 + ((tid >> 4) & 3) * 8) * 2);
  const uint32_t lo0 = (uint32_t)(tid * 16);
  // epilogue ownership: chunk row er, units u0 .. u0+3 of this member's 64
  const int er = tid >> 4, u0 = (tid & 15) * 4, j = 64 * mem + u0;
  const bf16_t* S = static_cast<const bf16_t*>(R.save);
  const bf16_t* Y = static_cast<const bf16_t*>(R.y);
  const bf16_t* DY = static_cast<const bf16_t*>(R.dy);
  bf16_t* DGX = static_cast<bf16_t*>(R.dgx);
  bf16_t* DGH = static_cast<bf16_t*>(R.dgh);
  float bsum[4][4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int e = 0; e < 4; ++e) bsum[q][e] = 0.f;

  const bool fast = xc_group_on_one_xcd(ws.cnt + grp * xc::CSTR, M, mem, ws.fast_ok != 0, err);
#ifdef TT_DIAG
  unsigned long long prf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  TT_STAMP(k_start);
  const int dbg = a.dbg;  // 1 no group wait, 2 no output stores, 4 no drain, 8 no MFMA, 16 no exchange loads
#else
  constexpr int dbg = 0;
#endif
  int idx = 0;
  for (int r = 0; r < ws.nround; ++r) {
    const int rb0 = gb0 + r * xb::RR;
    const int nrow = min(min(ws.rpg - r * xb::RR, xb::RR), B - rb0);
    const bool on = nrow > 0;
    const long r0w = (long)(on ? rb0 : 0) * T_;
    const __amdgpu_buffer_rsrc_t rS = tt_rsrc_n(S + r0w * 4L * H, on);
    const __amdgpu_buffer_rsrc_t rY = tt_rsrc_n(Y + r0w * a.ldy, on);
    const __amdgpu_buffer_rsrc_t rD = tt_rsrc_n(DY ? DY + r0w * a.ldy : Y, on && DY != nullptr);
    const __amdgpu_buffer_rsrc_t rGX = tt_rsrc_n(DGX + r0w * a.ldd, on);
    const __amdgpu_buffer_rsrc_t rGH = tt_rsrc_n(DGH + r0w * a.ldd, on);
    for (int i = tid; i < 2 * C::SLOT / 16; i += xb::NT)
      reinterpret_cast<float4*>(slots)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    // per-chunk inputs of the gate arithmetic: saved r | z | n | gh_n pre-activations, dY,
    // h_{t-1}: 8 bytes each (4 units), issued a chunk ahead
    auto load_in = [&](int s, int c, uint2 (&v)[6]) {
      const int t = R.dir ? T_ - 1 - s : s;
      const int tp = R.dir ? t + 1 : t - 1;
      const int rr = c * xb::CR + er;
      const bool ok = rr < nrow;
      const uint32_t os = ok ? (uint32_t)((rr * T_ + t) * 4 * H + j) * 2u : xc::OOB;
      const uint32_t od = ok ? (uint32_t)((rr * T_ + t) * (int)a.ldy + j) * 2u : xc::OOB;
      const uint32_t oh = ok && s > 0 ? (uint32_t)((rr * T_ + tp) * (int)a.ldy + j) * 2u : xc::OOB;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const auto w = __builtin_amdgcn_raw_buffer_load_b64(rS, (int)os, q * 2 * H, 0);
        v[q] = make_uint2(w[0], w[1]);
      }
      const auto wd = __builtin_amdgcn_raw_buffer_load_b64(rD, (int)od, 0, 0);
      const auto wh = __builtin_amdgcn_raw_buffer_load_b64(rY, (int)oh, 0, 0);
      v[4] = make_uint2(wd[0], wd[1]);
      v[5] = make_uint2(wh[0], wh[1]);
    };
    // gate-arithmetic inputs: a ring of four chunk sets (chunk c in vq[c % 4]), requested
    // three chunks ahead -- 16-row chunks are short next to HBM latency
    uint2 vq[4][6];
    load_in(T_ - 1, 0, vq[0]);
    load_in(T_ - 1, 1, vq[1]);
    load_in(T_ - 1, 2, vq[2]);
    for (int s = T_ - 1; s >= 0; --s, ++idx) {
      const int t = R.dir ? T_ - 1 - s : s;
      const bool last = s == T_ - 1;  // the first step processed: no recurrent gradient yet
      const bool mm = !last && !(dbg & 16);
      TT_STAMP(p0);
      if (idx > 0 && tid == 0 && !(dbg & 1)) xc_wait(cnt, (unsigned)(M * idx), err);
      __syncthreads();
      TT_STAMP(p1);
      const __amdgpu_buffer_rsrc_t rsrc = rx[(idx - 1) & 1];
      const __amdgpu_buffer_rsrc_t rdst = rx[idx & 1];
      tt_u32x4 hv[QPT];
      auto load_x = [&](int c) {
#pragma unroll
        for (int p = 0; p < QPT; ++p)
          hv[p] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(xo0 + p * 256), c * xb::CR * 3 * H * 2, 16);
      };
      auto put_x = [&](char* slot) {
#pragma unroll
        for (int p = 0; p < QPT; ++p) *reinterpret_cast<tt_u32x4*>(slot + lo0 + p * 4096) = hv[p];
      };
      // partial product of chunk c: wave's K quarter x 64 units (C^T: 4 units of a row per lane)
      f32x4 acc[4];
      auto mfma = [&](const char* slot) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (dbg & 8) return;
        const char* base = slot + wave * NKS * 1024 + lane * 16;
        tt_u32x4 f[3];
        f[0] = *reinterpret_cast<const tt_u32x4*>(base);
        f[1] = *reinterpret_cast<const tt_u32x4*>(base + 1024);
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          if (ks + 2 < NKS) f[(ks + 2) % 3] = *reinterpret_cast<const tt_u32x4*>(base + (ks + 2) * 1024);
#pragma unroll
          for (int nt = 0; nt < 4; ++nt)
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8v, wa[ks][nt]),
                                                              __builtin_bit_cast(bf16x8v, f[ks % 3]), acc[nt], 0, 0, 0);
        }
      };
      auto stage = [&]() {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          *reinterpret_cast<f32x4*>(pst + xb::pstg_off(wave, lane & 15, 16 * nt + 4 * (lane >> 4))) = acc[nt];
      };
      float gm[4], cin[4];
      auto read_part = [&](int c) {  // the four K quarters summed in order, rounded like gru_bwd_rows
        float4 p0 = *reinterpret_cast<const float4*>(pst + xb::pstg_off(0, er, u0));
        const float4 p1 = *reinterpret_cast<const float4*>(pst + xb::pstg_off(1, er, u0));
        const float4 p2 = *reinterpret_cast<const float4*>(pst + xb::pstg_off(2, er, u0));
        const float4 p3 = *reinterpret_cast<const float4*>(pst + xb::pstg_off(3, er, u0));
        gm[0] = bf2f(f2bf(((p0.x + p1.x) + p2.x) + p3.x));
        gm[1] = bf2f(f2bf(((p0.y + p1.y) + p2.y) + p3.y));
        gm[2] = bf2f(f2bf(((p0.z + p1.z) + p2.z) + p3.z));
        gm[3] = bf2f(f2bf(((p0.w + p1.w) + p2.w) + p3.w));
        const uint2 cv = *reinterpret_cast<const uint2*>(carry + (c * xb::CR + er) * 64 + u0);
        cin[0] = __uint_as_float(cv.x << 16); cin[1] = __uint_as_float(cv.x & 0xFFFF0000u);
        cin[2] = __uint_as_float(cv.y << 16); cin[3] = __uint_as_float(cv.y & 0xFFFF0000u);
        if (last) {
          const int b = rb0 + c * xb::CR + er;
#pragma unroll
          for (int e = 0; e < 4; ++e) cin[e] = 0.f;
          if (R.dfinal && c * xb::CR + er < nrow) {
            const float4 d = *reinterpret_cast<const float4*>(R.dfinal + (long)b * a.ldf + j);
            cin[0] = d.x; cin[1] = d.y; cin[2] = d.z; cin[3] = d.w;
          }
        }
      };
      if (mm) {
        load_x(0);
        put_x(slots);
        load_x(1);
      }
      __syncthreads();
      mfma(slots);
      if (mm) {
        put_x(slots + C::SLOT);
        load_x(2);
      }
      stage();
      __syncthreads();
      read_part(0);
      TT_STAMP(p2);
#pragma unroll 1
      for (int c4 = 0; c4 < xb::NCH; c4 += 4)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = c4 + k;
        const uint2(&vcur)[6] = vq[k];
        TT_STAMP(c0);
        if (c + 3 < xb::NCH) load_in(s, c + 3, vq[(k + 3) & 3]);
        if (c + 1 < xb::NCH) mfma(slots + ((k + 1) & 1) * C::SLOT);
        {
          const int rr = c * xb::CR + er;
          float ar[4], az[4], an[4], gh[4], dy[4], hp[4];
          auto un4 = [](uint2 v, float (&f)[4]) {
            f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xFFFF0000u);
            f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xFFFF0000u);
          };
          un4(vcur[0], ar); un4(vcur[1], az); un4(vcur[2], an); un4(vcur[3], gh);
          un4(vcur[4], dy); un4(vcur[5], hp);
          float o_r[4], o_z[4], o_n[4], o_hn[4], cout[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
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
          }
          auto pk4 = [](const float (&f)[4]) {
            return make_uint2((uint32_t)f2bf(f[0]) | ((uint32_t)f2bf(f[1]) << 16),
                              (uint32_t)f2bf(f[2]) | ((uint32_t)f2bf(f[3]) << 16));
          };
          const uint2 br = pk4(o_r), bz = pk4(o_z), bn_ = pk4(o_n), bh = pk4(o_hn);
          *reinterpret_cast<uint2*>(carry + rr * 64 + u0) = pk4(cout);
          const bool ok = rr < nrow;
          if (ok) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              bsum[0][e] += o_r[e]; bsum[1][e] += o_z[e]; bsum[2][e] += o_n[e]; bsum[3][e] += o_hn[e];
            }
          }
          // the exchange image: this member's r | z | W_hn h columns of the row
          const uint32_t ox = (uint32_t)(rr * 3 * H + j) * 2u;
          typedef __attribute__((ext_vector_type(2))) unsigned u2v;
          if (fast) {  // the image stays in the XCD's L2 (see gru_fwd_xc)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, br), rdst, (int)ox, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, bz), rdst, (int)(ox + 2u * H), 0, 0);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, bh), rdst, (int)(ox + 4u * H), 0, 0);
          } else {
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, br), rdst, (int)ox, 0, 16);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, bz), rdst, (int)(ox + 2u * H), 0, 16);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, bh), rdst, (int)(ox + 4u * H), 0, 16);
          }
          const uint32_t og = ok && !(dbg & 2) ? (uint32_t)((rr * T_ + t) * (int)a.ldd + j) * 2u : xc::OOB;
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, br), rGX, (int)og, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, bz), rGX, (int)(og + 2u * H), 0, 0);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, bn_), rGX, (int)(og + 4u * H), 0, 16);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, bh), rGH, (int)og, 0, 0);
        }
        if (mm && c + 2 < xb::NCH) {
          put_x(slots + (k & 1) * C::SLOT);
          if (c + 3 < xb::NCH) load_x(c + 3);
        }
        TT_STAMP(c1);
        __syncthreads();
        if (c + 1 < xb::NCH) {
          stage();
          __syncthreads();
          read_part(c + 1);
        }
        TT_STAMP(c2);
        TT_ACC(2, c1 - c0);
        TT_ACC(3, c2 - c1);
      }
      TT_STAMP(p3);
      if (!(dbg & 4)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (s > 0) {
        load_in(s - 1, 0, vq[0]);
        load_in(s - 1, 1, vq[1]);
        load_in(s - 1, 2, vq[2]);
      }
      TT_STAMP(p4);
      TT_ACC(0, p1 - p0);
      TT_ACC(1, p2 - p1);
      TT_ACC(4, p4 - p3);
    }
  }
  // bias partials: the 16 threads of a unit quad (one per chunk row) in a fixed order
  __syncthreads();
  float* red = pst;  // [16 rows][4 gates][64 units]
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int e = 0; e < 4; ++e) red[(er * 4 + q) * 64 + u0 + e] = bsum[q][e];
  __syncthreads();
  {
    const int q = tid >> 6, u = tid & 63;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < xb::CR; ++w) v += red[(w * 4 + q) * 64 + u];
    R.dbias[(long)gi * 4 * H + q * H + 64 * mem + u] = v;
  }
#ifdef TT_DIAG
  TT_STAMP(k_end);
  prf[7] = k_end - k_start;
  if (threadIdx.x == 0 && blockIdx.x < 2048)
    for (int i = 0; i < 8; ++i) g_fwd_prof[blockIdx.x][i] = prf[i];
#endif
}

#ifdef TT_DIAG
}  // namespace
extern "C" int tt_diag_fwd_prof(unsigned long long* out) {  // [2048][8] host buffer
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fwd_prof), sizeof(g_fwd_prof)) == hipSuccess ? 0 : 1;
}
namespace {
#endif
// gru_fwd_rr (experiment) where it applies: bf16, H 512, option gru_fwd_rr 1 (2 x 4 waves),
// 2 (8 x 1 waves) or 3 (256 threads, one wave per SIMD)
bool gru_fwd_rr_ok(int dtype, int H) {
  return dtype == TT_DT_BF16 && H == 512 && tt::opt(tt::OPT_GRU_STEP) != 1 &&
         tt::opt(tt::OPT_GRU_FWD_RR) != 0;
}
bool gru_fwd_wr_ok(int dtype, int H) {
  return dtype == TT_DT_BF16 && (H == 256 || H == 512) && tt::opt(tt::OPT_GRU_STEP) != 1 &&
         tt::opt(tt::OPT_GRU_FWD_WR) != 0 && tt::opt(tt::OPT_GRU_FWD_RR) == 0;
}
bool gru_fwd_persistent(int dtype, int H) {
  if (gru_fwd_rr_ok(dtype, H) || gru_fwd_wr_ok(dtype, H)) return true;
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
static int bwd_rows() { return tt::opt(tt::OPT_GRU_BWD_ROWS) == 64 ? 64 : 128; }
// partial bias rows: one per backward row tile (64 rows with gru_bwd_r64; extra rows of
// a smaller-tile count are zero-filled by tt_gru_bwd and add nothing)
extern "C" int tt_gru_bias_rows(int B) {
  // at least 64: the column-split backward writes one row per group of its recurrence
  return std::max(64, tt_ceil_div(B, tt::opt(tt::OPT_GRU_BWD_R64) ? 64 : bwd_rows()));
}

extern "C" int tt_gru_fwd_launches(int dtype, int T, int H) { return gru_fwd_persistent(dtype, H) ? 1 : T; }

static bool gru_bwd_persistent(int dtype, int H) {
  return dtype == TT_DT_BF16 && (H == 256 || H == 512) && bwd_rows() == 128 && tt::opt(tt::OPT_GRU_BWD_PERSIST) != 0;
}
extern "C" int tt_gru_bwd_launches(int dtype, int T, int H) { return gru_bwd_persistent(dtype, H) ? 1 : T; }

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

// gru_fwd_xc workspace per device: exchange images, arrival counters and the timeout flag,
// allocated on first use under a mutex (one column-split forward per device at a time: a
// second host thread on another stream would share the counters).
struct XcDev {
  int cus = 0;
  size_t xb_bytes = 0;
  bf16_t* xb = nullptr;
  unsigned* cnt = nullptr;  // [512 groups][CSTR] + the timeout flag after them
  size_t xg_bytes = 0;
  bf16_t* xg = nullptr;     // gru_bwd_xc exchange images
};
static std::mutex g_xc_mu;
static XcDev g_xc[64];
constexpr int XC_MAX_GROUPS = 512;

// Launch geometry of the column-split forward, or false where it does not apply.
static bool xc_geometry(int dtype, int H, int nrec, int B, int T, long ldg, long ldy, int cus, XcWs& w, int& grid) {
  const int v = tt::opt(tt::OPT_GRU_FWD_XC);
  if (v == 0 || dtype != TT_DT_BF16 || (H != 512 && H != 256)) return false;
  if (tt::opt(tt::OPT_GRU_STEP) == 1 || tt::opt(tt::OPT_GRU_FWD_RR) || tt::opt(tt::OPT_GRU_FWD_WR) ||
      tt::opt(tt::OPT_GRU_FWD_PAIR))
    return false;
  const int M = H / 64;
  const int qg = cus / (8 * M);
  const int ng = 8 * qg;
  if (qg < 1 || ng > XC_MAX_GROUPS || ng % nrec != 0) return false;
  const int gpr = ng / nrec;
  // auto mode: only where every group gets at least half a round of rows
  if ((v & 3) == 1 && (long)B < (long)gpr * (xc::RR / 2)) return false;
  // per-round resources: byte offsets of RR rows x T steps stay below 2 GiB
  if ((long)xc::RR * T * std::max({4L * H, ldy, ldg}) * 2 >= (1L << 31)) return false;
  w.qg = qg;
  w.nrec = nrec;
  w.rpg = tt_ceil_div(B, gpr);
  w.nround = tt_ceil_div(w.rpg, xc::RR);
  w.fast_ok = (v & 4) ? 0 : 1;  // option bit 4: always write-through images
  grid = ng * M;
  return true;
}

static int xc_device(XcDev** out) {
  int dev = 0;
  TT_CHECK_HIP(hipGetDevice(&dev));
  TT_CHECK_ARG(dev >= 0 && dev < 64, "tt_gru_fwd: device %d", dev);
  std::lock_guard<std::mutex> lock(g_xc_mu);
  XcDev& x = g_xc[dev];
  if (!x.cus) {
    TT_CHECK_HIP(hipDeviceGetAttribute(&x.cus, hipDeviceAttributeMultiprocessorCount, dev));
    TT_CHECK_HIP(hipMalloc(reinterpret_cast<void**>(&x.cnt), sizeof(unsigned) * (XC_MAX_GROUPS * xc::CSTR + 64)));
    TT_CHECK_HIP(hipMemset(x.cnt, 0, sizeof(unsigned) * (XC_MAX_GROUPS * xc::CSTR + 64)));
  }
  *out = &x;
  return 0;
}

// Timeout flag of the column-split forward on the current device (1 = a wait gave up: the
// outputs of that launch are invalid); clears it. Synchronises the device.
extern "C" int tt_gru_fwd_xc_status(int* timed_out) {
  TT_CHECK_ARG(timed_out, "tt_gru_fwd_xc_status: null");
  XcDev* x = nullptr;
  TT_PROPAGATE(xc_device(&x));
  TT_CHECK_HIP(hipDeviceSynchronize());
  unsigned* flag = x->cnt + XC_MAX_GROUPS * xc::CSTR;
  unsigned v = 0;
  TT_CHECK_HIP(hipMemcpy(&v, flag, sizeof(v), hipMemcpyDeviceToHost));
  TT_CHECK_HIP(hipMemset(flag, 0, sizeof(unsigned)));
  *timed_out = v != 0;
  return 0;
}

// H 1024: gru_fwd_xk, 32 units per member, one group per XCD
static bool xk_geometry(int H, int nrec, int B, int T, long ldg, long ldy, int cus, XcWs& w, int& grid) {
  // opt-in (option gru_fwd_xc = 2 / 6): measured slower than the per-step kernel at
  // configs[4] (63.3 vs 48.0 ms per layer; 16-row chunks)
  const int v = tt::opt(tt::OPT_GRU_FWD_XC);
  if ((v & 3) != 2 || H != 1024) return false;
  if (tt::opt(tt::OPT_GRU_STEP) == 1) return false;
  const int M = H / xk::NU;
  const int qg = cus / (8 * M);
  const int ng = 8 * qg;
  if (qg < 1 || ng > XC_MAX_GROUPS || ng % nrec != 0) return false;
  const int gpr = ng / nrec;
  if ((v & 3) == 1 && (long)B < (long)gpr * (xk::RR / 2)) return false;
  if ((long)xk::RR * T * std::max({4L * H, ldy, ldg}) * 2 >= (1L << 31)) return false;
  w.qg = qg;
  w.nrec = nrec;
  w.rpg = tt_ceil_div(B, gpr);
  w.nround = tt_ceil_div(w.rpg, xk::RR);
  w.fast_ok = (v & 4) ? 0 : 1;
  grid = ng * M;
  return true;
}

static int gru_fwd_xc_launch(const FwdArgs& a, int nrec, int B, int T, int H, long ldg, long ldy, hipStream_t st,
                             bool* used) {
  *used = false;
  if (tt::opt(tt::OPT_GRU_FWD_XC) == 0 || (H != 512 && H != 256 && H != 1024)) return 0;
  XcDev* x = nullptr;
  TT_PROPAGATE(xc_device(&x));
  XcWs w{};
  int grid = 0;
  const bool k1024 = H == 1024;
  if (k1024 ? !xk_geometry(H, nrec, B, T, ldg, ldy, x->cus, w, grid)
            : !xc_geometry(TT_DT_BF16, H, nrec, B, T, ldg, ldy, x->cus, w, grid))
    return 0;
  const int ng = grid / (k1024 ? H / xk::NU : H / 64);
  {
    std::lock_guard<std::mutex> lock(g_xc_mu);
    const size_t need = (size_t)ng * 2 * xc::RR * H * sizeof(bf16_t);
    if (x->xb_bytes < need) {
      if (x->xb) TT_CHECK_HIP(hipFree(x->xb));
      x->xb = nullptr;
      x->xb_bytes = 0;
      TT_CHECK_HIP(hipMalloc(reinterpret_cast<void**>(&x->xb), need));
      x->xb_bytes = need;
    }
  }
  w.xb = x->xb;
  w.cnt = x->cnt;
  w.err = x->cnt + XC_MAX_GROUPS * xc::CSTR;
  TT_CHECK_HIP(hipMemsetAsync(x->cnt, 0, sizeof(unsigned) * ng * xc::CSTR, st));
  const bool drop = a.drop_thresh != 0 && a.r[0].x1 != nullptr;
  if (k1024) {
    if (drop) hipLaunchKernelGGL((gru_fwd_xk<1024, true>), dim3(grid), dim3(xk::NT), 0, st, a, w);
    else hipLaunchKernelGGL((gru_fwd_xk<1024, false>), dim3(grid), dim3(xk::NT), 0, st, a, w);
  } else if (!(tt::opt(tt::OPT_GRU_FWD_XC) & 8)) {  // the step-pipelined form (option bit 8: per-step waits)
    if (H == 512 && drop) hipLaunchKernelGGL((gru_fwd_xcp<512, true>), dim3(grid), dim3(xc::NT), 0, st, a, w);
    else if (H == 512) hipLaunchKernelGGL((gru_fwd_xcp<512, false>), dim3(grid), dim3(xc::NT), 0, st, a, w);
    else if (drop) hipLaunchKernelGGL((gru_fwd_xcp<256, true>), dim3(grid), dim3(xc::NT), 0, st, a, w);
    else hipLaunchKernelGGL((gru_fwd_xcp<256, false>), dim3(grid), dim3(xc::NT), 0, st, a, w);
  } else if (H == 512 && drop) hipLaunchKernelGGL((gru_fwd_xc<512, true>), dim3(grid), dim3(xc::NT), 0, st, a, w);
  else if (H == 512) hipLaunchKernelGGL((gru_fwd_xc<512, false>), dim3(grid), dim3(xc::NT), 0, st, a, w);
  else if (drop) hipLaunchKernelGGL((gru_fwd_xc<256, true>), dim3(grid), dim3(xc::NT), 0, st, a, w);
  else hipLaunchKernelGGL((gru_fwd_xc<256, false>), dim3(grid), dim3(xc::NT), 0, st, a, w);
  TT_CHECK_LAUNCH("gru_fwd_xc");
  *used = true;
  return 0;
}

// Launch geometry of the column-split backward, or false where it does not apply (bias
// partial rows: one per group, so the recurrence's partial block must have that many).
static bool xb_geometry(int H, int nrec, int B, int T, long ldy, long ldd, int cus, XbWs& w, int& grid) {
  const int v = tt::opt(tt::OPT_GRU_BWD_XC);
  if (v == 0 || (H != 512 && H != 256) || tt::opt(tt::OPT_GRU_BWD_PERSIST) == 0 || tt::opt(tt::OPT_GRU_BWD_R64) ||
      bwd_rows() != 128)
    return false;
  const int M = H / 64;
  const int qg = cus / (8 * M);
  const int ng = 8 * qg;
  if (qg < 1 || ng > XC_MAX_GROUPS || ng % nrec != 0) return false;
  const int gpr = ng / nrec;
  if (tt_gru_bias_rows(B) < gpr) return false;
  if ((v & 3) == 1 && (long)B < (long)gpr * (xb::RR / 2)) return false;
  if ((long)xb::RR * T * std::max({4L * H, ldy, ldd}) * 2 >= (1L << 31)) return false;
  w.qg = qg;
  w.nrec = nrec;
  w.rpg = tt_ceil_div(B, gpr);
  w.nround = tt_ceil_div(w.rpg, xb::RR);
  w.fast_ok = (v & 4) ? 0 : 1;
  grid = ng * M;
  return true;
}

static int gru_bwd_xc_launch(const BwdArgs& a, int nrec, int B, int T, int H, long ldy, long ldd, hipStream_t st,
                             bool* used) {
  *used = false;
  if (tt::opt(tt::OPT_GRU_BWD_XC) == 0 || (H != 512 && H != 256)) return 0;
  XcDev* x = nullptr;
  TT_PROPAGATE(xc_device(&x));
  XbWs w{};
  int grid = 0;
  if (!xb_geometry(H, nrec, B, T, ldy, ldd, x->cus, w, grid)) return 0;
  const int ng = grid / (H / 64);
  {
    std::lock_guard<std::mutex> lock(g_xc_mu);
    const size_t need = (size_t)ng * 2 * xb::RR * 3 * H * sizeof(bf16_t);
    if (x->xg_bytes < need) {
      if (x->xg) TT_CHECK_HIP(hipFree(x->xg));
      x->xg = nullptr;
      x->xg_bytes = 0;
      TT_CHECK_HIP(hipMalloc(reinterpret_cast<void**>(&x->xg), need));
      x->xg_bytes = need;
    }
  }
  w.xb = x->xg;
  w.cnt = x->cnt;
  w.err = x->cnt + XC_MAX_GROUPS * xc::CSTR;
  TT_CHECK_HIP(hipMemsetAsync(x->cnt, 0, sizeof(unsigned) * ng * xc::CSTR, st));
  if (H == 512) hipLaunchKernelGGL(gru_bwd_xc<512>, dim3(grid), dim3(xb::NT), 0, st, a, w);
  else hipLaunchKernelGGL(gru_bwd_xc<256>, dim3(grid), dim3(xb::NT), 0, st, a, w);
  TT_CHECK_LAUNCH("gru_bwd_xc");
  *used = true;
  return 0;
}

extern "C" int tt_gru_fwd_launches_for(int dtype, int nrec, int B, int T, int H, long ldg, long ldy) {
  if (dtype == TT_DT_BF16 && nrec >= 1 && nrec <= 4 && B > 0 && T > 0) {
    XcDev* x = nullptr;
    if (xc_device(&x) == 0) {
      XcWs w{};
      int grid = 0;
      if (H == 1024 ? xk_geometry(H, nrec, B, T, ldg, ldy, x->cus, w, grid)
                    : xc_geometry(dtype, H, nrec, B, T, ldg, ldy, x->cus, w, grid))
        return 1;
    }
  }
  return tt_gru_fwd_launches(dtype, T, H);
}

extern "C" int tt_gru_fwd(int dtype, const tt_gru_fwd_rec* recs, int nrec, int B, int T, int H, long ldg,
                          long ldy, float drop_p, void* stream) {
  TT_CHECK_ARG(dtype == TT_DT_F32 || dtype == TT_DT_BF16, "tt_gru_fwd: bad dtype");
  TT_CHECK_ARG(nrec >= 1 && nrec <= 4, "tt_gru_fwd: nrec %d", nrec);
  TT_CHECK_ARG(B > 0 && T > 0 && H > 0, "tt_gru_fwd: bad shape");
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
  a.stagger = tt::opt(tt::OPT_GRU_STAGGER);
#ifdef TT_DIAG
  if (const char* e = getenv("TT_GRU_DBG")) a.dbg = atoi(e);
#endif
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TT_DT_BF16) {
    bool used = false;
    TT_PROPAGATE(gru_fwd_xc_launch(a, nrec, B, T, H, ldg, ldy, st, &used));
    if (used) return 0;
  }
  if (gru_fwd_rr_ok(dtype, H)) {
    const dim3 grid(tt_ceil_div(B, 65536 / H) * nrec);
    const int v = tt::opt(tt::OPT_GRU_FWD_RR);
    if (v == 1) hipLaunchKernelGGL((gru_fwd_rr<512, 512, 4, 2>), grid, dim3(512), 0, st, a);       // 2 x 4 waves
    else if (v == 2) hipLaunchKernelGGL((gru_fwd_rr<512, 512, 1, 2>), grid, dim3(512), 0, st, a);  // 8 x 1 waves
    else hipLaunchKernelGGL((gru_fwd_rr<512, 256, 2, 2>), grid, dim3(256), 0, st, a);              // one wave per SIMD
    TT_CHECK_LAUNCH("gru_fwd_rr");
    return 0;
  }
  if (gru_fwd_wr_ok(dtype, H)) {
    const dim3 grid(tt_ceil_div(B, wr::ROWS) * nrec);
    if (H == 512) hipLaunchKernelGGL(gru_fwd_wr<512>, grid, dim3(wr::NT), 0, st, a);
    else hipLaunchKernelGGL(gru_fwd_wr<256>, grid, dim3(wr::NT), 0, st, a);
    TT_CHECK_LAUNCH("gru_fwd_wr");
    return 0;
  }
  if (gru_fwd_persistent(dtype, H)) {
    const dim3 grid(tt_ceil_div(B, PR) * nrec);
    int depth = (H / 64) % 4 == 0 ? 4 : (H / 64) % 2 == 0 ? 2 : 1;
    depth = std::min(depth, tt::opt(tt::OPT_GRU_DEPTH));
    const bool pair = depth >= 4 && tt::opt(tt::OPT_GRU_FWD_PAIR) == 1;
    const bool ew = depth >= 4 && tt::opt(tt::OPT_GRU_FWD_PAIR) == 2;  // early-write K-tile order
    const int fo = tt::opt(tt::OPT_GRU_FWD_PAIR);
    if (fo == 6 && (H == 512 || H == 256)) {  // 16 waves per workgroup
      if (H == 512) hipLaunchKernelGGL(gru_fwd_seq16<8>, grid, dim3(s16::NT), 0, st, a);
      else hipLaunchKernelGGL(gru_fwd_seq16<4>, grid, dim3(s16::NT), 0, st, a);
      TT_CHECK_LAUNCH("gru_fwd_seq16");
      return 0;
    }
    if (fo == 5 && depth >= 4 && H == 512) {  // timing experiment only: time-major row addressing
      hipLaunchKernelGGL((gru_fwd_seq<4, 8, false, false, false, true>), grid, dim3(PNT), 0, st, a);
      TT_CHECK_LAUNCH("gru_fwd_seq");
      return 0;
    }
    if (fo == 3 && depth >= 4 && H == 512) hipLaunchKernelGGL((gru_fwd_seq<4, 8, false, false, true>), grid, dim3(PNT), 0, st, a);
    else if (fo == 3 && depth >= 4 && H == 256) hipLaunchKernelGGL((gru_fwd_seq<4, 4, false, false, true>), grid, dim3(PNT), 0, st, a);
    else if (fo == 4 && depth >= 2 && H == 512) hipLaunchKernelGGL((gru_fwd_seq<2, 8, false, false, true>), grid, dim3(PNT), 0, st, a);
    else if (fo == 4 && depth >= 2 && H == 256) hipLaunchKernelGGL((gru_fwd_seq<2, 4, false, false, true>), grid, dim3(PNT), 0, st, a);
    else if (ew && H == 512) hipLaunchKernelGGL((gru_fwd_seq<4, 8, false, true>), grid, dim3(PNT), 0, st, a);
    else if (ew && H == 256) hipLaunchKernelGGL((gru_fwd_seq<4, 4, false, true>), grid, dim3(PNT), 0, st, a);
    else if (pair && H == 512) hipLaunchKernelGGL((gru_fwd_seq<4, 8, true>), grid, dim3(PNT), 0, st, a);
    else if (pair && H == 256) hipLaunchKernelGGL((gru_fwd_seq<4, 4, true>), grid, dim3(PNT), 0, st, a);
    else if (depth >= 4 && H == 512) hipLaunchKernelGGL((gru_fwd_seq<4, 8>), grid, dim3(PNT), 0, st, a);
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
  for (int s = 0; s < T; ++s) {
    a.s = s;
    if (dtype == TT_DT_BF16) {
      if (bmr == 256) hipLaunchKernelGGL((gru_fwd_step<bf16_t, 256>), grid, dim3(512), 0, st, a);
      else hipLaunchKernelGGL((gru_fwd_step<bf16_t, 128>), grid, dim3(256), 0, st, a);
    } else {
      if (bmr == 256) hipLaunchKernelGGL((gru_fwd_step<float, 256>), grid, dim3(512), 0, st, a);
      else hipLaunchKernelGGL((gru_fwd_step<float, 128>), grid, dim3(256), 0, st, a);
    }
    TT_CHECK_LAUNCH("gru_fwd_step");
  }
  return 0;
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
#ifdef TT_DIAG
  if (const char* e = getenv("TT_GRU_DBG")) a.dbg = atoi(e);
#endif
  const int bmr = bwd_rows();
  // bf16, H 256 / 512: one row-owning launch per layer (option gru_bwd_persist = 0: per-step
  // launches)
  if (gru_bwd_persistent(dtype, H)) {
    bool used = false;
    TT_PROPAGATE(gru_bwd_xc_launch(a, nrec, B, T, H, ldy, ldd, st, &used));
    if (used) return 0;
    TT_CHECK_ARG(128L * T * std::max({ldd, ldy, 4L * H}) * esz < (1L << 31), "tt_gru_bwd: tile offsets exceed 2 GiB");
    if (tt::opt(tt::OPT_GRU_BWD_R64)) {
      const dim3 grid(tt_ceil_div(B, 64) * nrec);
      const int ph = std::max(0, tt::opt(tt::OPT_GRU_BWD_PHASE));
      if (H == 512) hipLaunchKernelGGL(gru_bwd_r64<512>, grid, dim3(256), 0, st, a, ph);
      else hipLaunchKernelGGL(gru_bwd_r64<256>, grid, dim3(256), 0, st, a, ph);
      TT_CHECK_LAUNCH("gru_bwd_r64");
      return 0;
    }
    const dim3 grid(tt_ceil_div(B, 128) * nrec);
    if (H == 512) hipLaunchKernelGGL(gru_bwd_rows<512>, grid, dim3(512), 0, st, a);
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
  for (int s = T - 1; s >= 0; --s) {
    for (int g = 0; g < ngrp; ++g) {
      ga[g].s = s;
      const dim3 grid(tt_ceil_div(H, 128) * tt_ceil_div(B, bmr) * gn[g]);
      if (dtype == TT_DT_BF16) {
        if (bmr == 64) hipLaunchKernelGGL((gru_bwd_step<bf16_t, 64>), grid, dim3(256), 0, gs[g], ga[g]);
        else hipLaunchKernelGGL((gru_bwd_step<bf16_t, 128>), grid, dim3(256), 0, gs[g], ga[g]);
      } else {
        if (bmr == 64) hipLaunchKernelGGL((gru_bwd_step<float, 64>), grid, dim3(256), 0, gs[g], ga[g]);
        else hipLaunchKernelGGL((gru_bwd_step<float, 128>), grid, dim3(256), 0, gs[g], ga[g]);
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
