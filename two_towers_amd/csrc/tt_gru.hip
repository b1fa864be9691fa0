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
#include "tt_api.h"
#include "tt_gemm_core.h"

namespace {

struct FwdRec {
  const void* g; const void* whh; const float* bhn; void* y; void* x1; void* save; float* hs;
  int dir; uint32_t seed; int col0;
};
struct FwdArgs {
  FwdRec r[4];
  int B, T, H;
  long ldg, ldy;
  int s;
  uint32_t drop_thresh;
  float inv_keep;
};

struct BwdRec {
  const void* save; const void* y; const void* dy; const float* dfinal; const void* whh;
  void* dgx; void* dgh; float* dh; float* dbias; int dir;
};
struct BwdArgs {
  BwdRec r[4];
  int B, T, H;
  long ldy, ldd, ldf;
  int s;
};

// B-tile row r of the forward step -> row (gate*H + j) of Whh [3H, H].
template <typename T>
struct GateRows {
  const T* w; int H, j0;
  TT_DEV const T* rowptr(int r) const {
    const int half = r / 96, rem = r - half * 96;
    const int g = rem >> 5, j = j0 + half * 32 + (rem & 31);
    return j < H ? w + (long)(g * H + j) * H : nullptr;
  }
};

template <typename T>
__global__ __launch_bounds__(256) void gru_fwd_step(FwdArgs a) {
  using ML = ttg::MainLoop<T, false, false, 128, 192>;
  __shared__ __attribute__((aligned(16))) char lds[ML::LDS_BYTES];
  const FwdRec R = a.r[blockIdx.z];
  const int H = a.H, T_ = a.T, s = a.s;
  const int m0 = blockIdx.y * 128, j0 = blockIdx.x * 64;
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

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = (wave >> 1) * 64, half = wave & 1;
  const int cur = s & 1, prv = cur ^ 1;
  const T* G = static_cast<const T*>(R.g);
  T* Yw = static_cast<T*>(R.y);
  T* X1 = static_cast<T*>(R.x1);
  T* S = static_cast<T*>(R.save);
  float* hs_cur = R.hs + (long)cur * a.B * H;
  const float* hs_prv = R.hs + (long)prv * a.B * H;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jh = 0; jh < 2; ++jh)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = m0 + wm + 16 * i + 4 * (lane >> 4) + r;
        const int j = j0 + half * 32 + 16 * jh + (lane & 15);
        if (b >= a.B || j >= H) continue;
        const long row = (long)b * T_ + t;
        const T* gp = G + row * a.ldg + j;
        const float xr = Elt<T>::ld(gp), xz = Elt<T>::ld(gp + H), xn = Elt<T>::ld(gp + 2 * H);
        const float ghn = acc[i][4 + jh][r] + R.bhn[j];
        const float ar = xr + acc[i][jh][r], az = xz + acc[i][2 + jh][r];
        const float rg = tt_sigmoid(ar);
        const float zg = tt_sigmoid(az);
        const float an = xn + rg * ghn;
        const float ng = tt_tanh(an);
        const float hp = s > 0 ? hs_prv[(long)b * H + j] : 0.f;
        const float hn = (1.f - zg) * ng + zg * hp;
        hs_cur[(long)b * H + j] = hn;
        Elt<T>::st(Yw + row * a.ldy + j, hn);
        T* sp = S + row * (4L * H) + j;
        // pre-activations, not gate values: the backward recomputes sigma/tanh in fp32,
        // so 1-z and 1-n^2 keep full precision even with bf16 storage
        Elt<T>::st(sp, ar);
        Elt<T>::st(sp + H, az);
        Elt<T>::st(sp + 2 * H, an);
        Elt<T>::st(sp + 3 * H, ghn);
        if (X1) {
          const float m = a.drop_thresh ? tt_dropout_scale(R.seed, (uint32_t)row, (uint32_t)(R.col0 + j),
                                                           a.drop_thresh, a.inv_keep)
                                        : 1.f;
          Elt<T>::st(X1 + row * a.ldy + j, hn * m);
        }
      }
}

template <typename T>
__global__ __launch_bounds__(256) void gru_bwd_step(BwdArgs a) {
  using ML = ttg::MainLoop<T, false, true, 128, 128>;
  __shared__ __attribute__((aligned(16))) char lds[ML::LDS_BYTES];
  const BwdRec R = a.r[blockIdx.z];
  const int H = a.H, T_ = a.T, s = a.s;
  const int m0 = blockIdx.y * 128, j0 = blockIdx.x * 128;
  const int t = R.dir ? T_ - 1 - s : s;
  const int tn = R.dir ? t - 1 : t + 1;  // time of step s+1
  const int tp = R.dir ? t + 1 : t - 1;  // time of step s-1
  const bool last = (s == T_ - 1);
  const T* DGH = static_cast<const T*>(R.dgh);

  f32x4 acc[ML::TM][ML::TN];
#pragma unroll
  for (int i = 0; i < ML::TM; ++i)
#pragma unroll
    for (int j = 0; j < ML::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (!last) {
    ttg::KCPlain<T> la{DGH + (long)tn * a.ldd, (long)T_ * a.ldd, m0, a.B};
    ttg::KOPlain<T> lb{static_cast<const T*>(R.whh), H, j0, H - j0};
    const int K = 3 * H;
    const int nk = (K * (int)sizeof(T) + ttg::KTB - 1) / ttg::KTB;
    ML::run(la, lb, K, 0, nk, lds, acc);
  }

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int cur = s & 1, nxt = cur ^ 1;
  const T* S = static_cast<const T*>(R.save);
  const T* Y = static_cast<const T*>(R.y);
  const T* DY = static_cast<const T*>(R.dy);
  T* DGX = static_cast<T*>(R.dgx);
  T* DGHw = static_cast<T*>(R.dgh);
  float* dh_cur = R.dh + (long)cur * a.B * H;
  const float* dh_nxt = R.dh + (long)nxt * a.B * H;
  const long S4 = 4L * H;

#pragma unroll
  for (int jt = 0; jt < 4; ++jt) {
    const int j = j0 + wn + 16 * jt + (lane & 15);
    float sr = 0.f, sz = 0.f, sn = 0.f, shn = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = m0 + wm + 16 * i + 4 * (lane >> 4) + r;
        if (b >= a.B || j >= H) continue;
        const long row = (long)b * T_ + t;
        float carry;
        if (!last) {
          carry = dh_nxt[(long)b * H + j] * tt_sigmoid(Elt<T>::ld(S + ((long)b * T_ + tn) * S4 + H + j));
        } else {
          carry = R.dfinal ? R.dfinal[(long)b * a.ldf + j] : 0.f;
        }
        float dht = acc[i][jt][r] + carry;
        if (DY) dht += Elt<T>::ld(DY + row * a.ldy + j);
        const T* sp = S + row * S4 + j;
        const float ar = Elt<T>::ld(sp), az = Elt<T>::ld(sp + H), an = Elt<T>::ld(sp + 2 * H),
                    ghn = Elt<T>::ld(sp + 3 * H);
        const float rg = tt_sigmoid(ar), omr = tt_sigmoid(-ar);
        const float zg = tt_sigmoid(az), omz = tt_sigmoid(-az);
        const float ng = tt_tanh(an);
        const float hp = s > 0 ? Elt<T>::ld(Y + ((long)b * T_ + tp) * a.ldy + j) : 0.f;
        const float dn = dht * omz;
        const float dz = dht * (hp - ng);
        const float dnp = dn * tt_sech2(an);
        const float drp = dnp * ghn * rg * omr;
        const float dzp = dz * zg * omz;
        const float dhn = dnp * rg;
        dh_cur[(long)b * H + j] = dht;
        T* gx = DGX + row * a.ldd + j;
        T* gh = DGHw + row * a.ldd + j;
        Elt<T>::st(gx, drp);
        Elt<T>::st(gx + H, dzp);
        Elt<T>::st(gx + 2 * H, dnp);
        Elt<T>::st(gh, drp);
        Elt<T>::st(gh + H, dzp);
        Elt<T>::st(gh + 2 * H, dhn);
        sr += drp; sz += dzp; sn += dnp; shn += dhn;
      }
    // bias partial sums: reduce the 4 row groups sharing this column
    sr += __shfl_xor(sr, 16, 64); sr += __shfl_xor(sr, 32, 64);
    sz += __shfl_xor(sz, 16, 64); sz += __shfl_xor(sz, 32, 64);
    sn += __shfl_xor(sn, 16, 64); sn += __shfl_xor(sn, 32, 64);
    shn += __shfl_xor(shn, 16, 64); shn += __shfl_xor(shn, 32, 64);
    if (lane < 16 && j < H) {
      float* pb = R.dbias + (long)(blockIdx.y * 2 + (wave >> 1)) * (4L * H) + j;
      pb[0] += sr;
      pb[H] += sz;
      pb[2 * H] += sn;
      pb[3 * H] += shn;
    }
  }
}

}  // namespace

extern "C" int tt_gru_bias_rows(int B) { return tt_ceil_div(B, 128) * 2; }

extern "C" int tt_gru_fwd(int dtype, const tt_gru_fwd_rec* recs, int nrec, int B, int T, int H, long ldg,
                          long ldy, float drop_p, void* stream) {
  TT_CHECK_ARG(dtype == TT_DT_F32 || dtype == TT_DT_BF16, "tt_gru_fwd: bad dtype");
  TT_CHECK_ARG(nrec >= 1 && nrec <= 4, "tt_gru_fwd: nrec %d", nrec);
  TT_CHECK_ARG(B > 0 && T > 0 && H > 0, "tt_gru_fwd: bad shape");
  const int esz = dtype == TT_DT_BF16 ? 2 : 4;
  TT_CHECK_ARG(H % (16 / esz) == 0 && (ldy * esz) % 16 == 0, "tt_gru_fwd: H=%d/ldy=%ld misaligned", H, ldy);
  TT_CHECK_ARG(drop_p >= 0.f && drop_p < 1.f, "tt_gru_fwd: drop_p");
  TT_CHECK_ARG(tt_ceil_div(B, 128) <= 65535, "tt_gru_fwd: B too large");
  FwdArgs a{};
  for (int i = 0; i < nrec; ++i) {
    const tt_gru_fwd_rec& r = recs[i];
    TT_CHECK_ARG(r.g && r.whh && r.bhn && r.y && r.save && r.hstate, "tt_gru_fwd: null pointer in rec %d", i);
    a.r[i] = FwdRec{r.g, r.whh, r.bhn, r.y, r.x1, r.save, r.hstate, r.dir, r.drop_seed, r.drop_col0};
  }
  a.B = B; a.T = T; a.H = H; a.ldg = ldg; a.ldy = ldy;
  a.drop_thresh = drop_p > 0.f ? (uint32_t)(drop_p * 16777216.0f + 0.5f) : 0u;
  a.inv_keep = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(tt_ceil_div(H, 64), tt_ceil_div(B, 128), nrec);
  for (int s = 0; s < T; ++s) {
    a.s = s;
    if (dtype == TT_DT_BF16) hipLaunchKernelGGL(gru_fwd_step<bf16_t>, grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(gru_fwd_step<float>, grid, dim3(256), 0, st, a);
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
  TT_CHECK_ARG(H % (16 / esz) == 0 && (ldd * esz) % 16 == 0, "tt_gru_bwd: H=%d/ldd=%ld misaligned", H, ldd);
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
  dim3 grid(tt_ceil_div(H, 128), tt_ceil_div(B, 128), nrec);
  for (int s = T - 1; s >= 0; --s) {
    a.s = s;
    if (dtype == TT_DT_BF16) hipLaunchKernelGGL(gru_bwd_step<bf16_t>, grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(gru_bwd_step<float>, grid, dim3(256), 0, st, a);
    TT_CHECK_LAUNCH("gru_bwd_step");
  }
  return 0;
}
