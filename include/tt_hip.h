/* tt_hip.h — C ABI of libtt_hip.so, the MI355X (gfx950) implementation of the
 * two-tower contrastive training step of mateomarin/two_towers.
 *
 * The reference has no native code and no FFI: its hot path is PyTorch module calls
 * (nn.GRU, nn.Linear, nn.LayerNorm, F.normalize, matmul, cross_entropy,
 * cosine_similarity, topk, optim.Adam). Each entry point below replaces one of those
 * call sites; the reference file:line it stands in for is given per function.
 * two_towers_amd/ (Python, ctypes) binds these entry points behind the reference's
 * own nn.Module surface (EnhancedTwoTowerModel, InfoNCELoss, MarginRankingLoss,
 * get_hard_negatives).
 *
 * Conventions
 *  - All pointers are device pointers (HBM) owned by the caller; nothing here
 *    allocates device memory. Scratch ("ws") is caller-provided.
 *  - dtype selects storage/arithmetic of the tensor operands: TT_DT_F32 (exact fp32
 *    MFMA) or TT_DT_BF16 (bf16 storage, fp32 accumulation). Tensors typed `float*`
 *    are always fp32.
 *  - Matrices are row-major with an explicit leading dimension in ELEMENTS.
 *  - stream is a hipStream_t (NULL = default stream); every call is stream-ordered
 *    and asynchronous. Thread-safe on distinct streams.
 *  - Return 0 on success, TT_EINVAL on a bad argument, else a hipError_t code;
 *    tt_last_error() returns a thread-local message for the last failure.
 */
#ifndef TT_HIP_H
#define TT_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TT_OK 0
#define TT_EINVAL 1000
#define TT_DT_F32 0
#define TT_DT_BF16 1

/* Library version string, e.g. "tt_hip 0.2.0 gfx950". */
const char* tt_version(void);
/* Message describing the last non-zero return on this thread ("" if none). */
const char* tt_last_error(void);
/* Kernel-variant switches (process-wide; initialised once from the environment variable
 * of the same name in upper case with a TT_ prefix, e.g. gru_step <- TT_GRU_STEP):
 * GRU: gru_step, gru_depth, gru_bwd_rows, gru_bwd_big, gru_bwd_streams, gru_bwd_persist,
 * gru_bwd_skew, gru_fwd_step_rows, gru_fwd_xc, gru_fwd_xs, gru_fwd_skew, gru_xc_coop,
 * gru_step_ring; GEMM: gemm_persist, gemm_persist_maxk, gemm_a3, gemm_buf, gemm_bres,
 * bres_rows, gemm_iepi, gemm_order, gemm_skew, gemm_regstage, gemm_stream_out; losses:
 * hn_gemm, hn_map, hn_scan_gemm, infonce_flash; diagnostics gru_xc_skip, gru_xc_spins. The authoritative list with
 * defaults is kOpts in two_towers_amd/csrc/tt_gemm.hip. Every variant computes the same
 * function; they exist for A/B measurement and for tests that compare variants.
 * Not synchronised with launches in flight: set them between steps. */
int tt_set_option(const char* name, int value);
int tt_get_option(const char* name, int* value);

/* ---------------------------------------------------------------- featurisation */
/* Word2Vec row gather: out[i, :] = table[ids[i], :] for ids[i] >= 0, zero row for
 * ids[i] < 0 (pad / all-OOV).  Replaces the per-word lookup + zero padding of
 * EnhancedDataset.text_to_embedding (enhanced_two_tower.py:144-166).
 * table [vocab, ep], out [n, ep]; ep * sizeof(dtype) must be a multiple of 16. */
int tt_embed_gather(int dtype, const void* table, long vocab, int ep, const int32_t* ids, long n,
                    void* out, void* stream);

/* Packs float rows [n, e] into dtype rows [n, ep] (zero columns e..ep-1): the
 * reference's float [B,T,E] encoder input (enhanced_two_tower.py:50,56) into the
 * padded layout the projections read. */
int tt_pack_rows(int dtype, const float* src, long n, int e, int ep, void* out, void* stream);
/* Weight packing in one launch: up to 16 jobs, each dst[r][c] = src[r][c] (+ src2[r][c]) for
 * c < cols and 0 for cols <= c < dcols, r < rows, written as bf16 (dst_bf16) or fp32. cols,
 * dcols, lds, ldd multiples of 4 and src / src2 / dst 16-byte aligned. Replaces the per-step
 * torch.cat / pad / cast of the GRU weights and the folded r|z biases (towers.py _Packed). */
typedef struct {
  const float* src;
  const float* src2; /* NULL or a second fp32 operand of the same layout, added */
  void* dst;
  int rows, cols, dcols;
  long lds, ldd;
  int dst_bf16;
} tt_pack_job;
int tt_pack_multi(const tt_pack_job* jobs, int njobs, void* stream);

/* y[i] = (dtype)x[i] (fp32 -> dtype) for n elements. */
int tt_cast(int dtype, const float* x, long n, void* y, void* stream);

/* out[c] (+)= sum_r x[r*ld + c] over r < rows (x fp32). Bias gradients: summed in a
 * fixed order (no atomics), so results are bit-for-bit reproducible. */
int tt_colsum(const float* x, long rows, int cols, long ld, float* out, int accumulate, void* stream);

/* ------------------------------------------------------------------------ GEMM */
/* Batched MFMA GEMM (up to 4 independent problems of one shape per launch):
 *     C_b[m][n] = alpha * sum_k A_b(m,k) B_b(n,k) (+ bias_b[n]) (relu) (*dropmask) (+ C_b)
 * a_kouter = 0: A stored [m][k] (lda);   1: A stored [k][m] (lda).
 * b_kouter = 0: B stored [n][k] (ldb);   1: B stored [k][n] (ldb).
 * With b_kouter = 1 and bshift[b] != 0, B row k is read from row k + shift when
 * (k mod seq_t) + shift lies in [0, seq_t), else treated as zero (GRU h_{t-1} operand).
 * drop_p > 0 multiplies element (m, n) by the counter-based dropout mask
 * keep(drop_seed, m, n) / (1 - drop_p) (see tt_gru_fwd).
 * splits > 1 splits K across workgroups: fp32 partials go to splitk_ws
 * (tt_gemm_ws_size floats) and are reduced into C; relu/dropout unsupported then.
 * out_dtype is TT_DT_F32 or dtype. Any m, n, k; operand base pointers and leading
 * dimensions must be 16-byte aligned (lda * sizeof(dtype) % 16 == 0).
 * Every problem runs on the hand-written MFMA kernels of this library (tt_gemm.hip,
 * tt_gemm_core.h); no vendor GEMM is linked. */
typedef struct {
  const void* a[4];
  const void* b[4];
  void* c[4];
  const float* bias[4];
  int bshift[4];
  /* a_kouter = 1 only: columns m >= a_split of A come from a_hi[b] + (m - a_split)
   * (same lda); a_split = 0 disables. Lets dW_hh read the GRU dL/dgh operand, whose
   * r|z columns live in the dL/dgx buffer, without a copy. */
  const void* a_hi[4];
  int a_split;
  /* dropout (drop_p > 0): the mask of element (m, n) is keep(drop_seed, drop_row0 + m, n) */
  uint32_t drop_row0;
} tt_gemm_batch;

int tt_gemm(int dtype, int out_dtype, int a_kouter, int b_kouter, int m, int n, int k,
            const tt_gemm_batch* batch, int nbatch, long lda, long ldb, long ldc, float alpha,
            int beta_accum, int relu, int seq_t, uint32_t drop_seed, float drop_p, int splits,
            float* splitk_ws, void* stream);
/* fp32 elements of splitk_ws: the split partials for splits > 1, else 0. */
long tt_gemm_ws_size(int m, int n, int nbatch, int splits);
/* Heuristic split count for a (m, n, k, nbatch) problem. */
int tt_gemm_pick_splits(int m, int n, int k, int nbatch);

/* ------------------------------------------------------------------------- GRU */
/* One bidirectional GRU layer, forward, all time steps (torch nn.GRU semantics:
 * r = s(Wir x + bir + Whr h + bhr), z = s(Wiz x + biz + Whz h + bhz),
 * n = tanh(Win x + bin + r*(Whn h + bhn)), h' = (1-z) n + z h, h0 = 0).
 * Replaces nn.GRU at enhanced_two_tower.py:51,57 (per layer, up to 4 recurrences =
 * {query,doc} x {fwd,rev} per launch). The input projection g = x Wih^T + bih
 * (+ [bhr, bhz, 0]) is a tt_gemm done by the caller. H must be a multiple of 8 (the
 * epilogues update 8 consecutive hidden units per thread; tt_gru_bwd likewise). */
typedef struct {
  const void* g;       /* [B*T, ldg]: gate pre-activations r|z|n (3H columns)        */
  const void* whh;     /* [3H, H]                                                    */
  const float* bhn;    /* [H]                                                        */
  void* y;             /* h_t: element (b,t,j) at y[(b*T+t)*ldy + j]                 */
  void* x1;            /* optional dropout(y) for the next layer (same layout) or NULL */
  void* save;          /* [B*T, 4H] saved pre-activations of r|z|n and gh_n (backward) */
  float* hstate;       /* fp32 scratch [2][B][H] (per-step kernel only)              */
  int dir;             /* 0: t = 0..T-1 ; 1: t = T-1..0                              */
  uint32_t drop_seed;  /* dropout stream of x1                                       */
  int drop_col0;       /* column of this recurrence inside the layer output (dir*H)  */
  uint32_t drop_row0;  /* mask row of local row 0: the mask of element (b, t, col) is
                          keep(drop_seed, drop_row0 + b*T + t, drop_col0 + col), so a
                          data-parallel rank passes rank * B * T and draws the masks the
                          single-process run of the global batch would               */
} tt_gru_fwd_rec;

int tt_gru_fwd(int dtype, const tt_gru_fwd_rec* recs, int nrec, int B, int T, int H, long ldg,
               long ldy, float drop_p, void* ws, long ws_bytes, void* stream);
/* Kernel launches tt_gru_fwd issues without a workspace: 1 for the persistent bf16 kernel
 * (H % 64 == 0, H <= 512; 64 batch rows per workgroup kept resident for all T steps, hstate
 * unused), T for the per-step kernel (fp32, other H, or option gru_step = 1). */
int tt_gru_fwd_launches(int dtype, int T, int H);
/* Device scratch (bytes, 0 = none used) that lets tt_gru_fwd run the column-split persistent
 * kernel for this call shape on the current device: bf16, H 256 / 512, a batch large enough
 * (or option gru_fwd_xc = 2), and every member workgroup co-resident (one per CU, checked
 * against the occupancy query; a plain launch by default, hipLaunchCooperativeKernel with
 * option gru_xc_coop = 1). The occupancy check covers an idle device only: kernels of other
 * streams may keep members from being co-resident, and then the bounded member waits give up
 * and set the STATUS word below (outputs invalid, reported -- never silently wrong); callers
 * that overlap other work with this launch should expect that. H/64 workgroups share a block of
 * batch rows, each keeps 64 units' W_hh rows in registers, and they exchange h every step
 * through ws: per-group arrival counters (zeroed by every call, stream-ordered) and exchange
 * images. ws: 256-byte aligned, one buffer per launch in flight (distinct streams need
 * distinct buffers). NULL, or ws_bytes below the size: the row-owning kernel runs instead.
 * The first 4 bytes of ws are a STATUS word: nonzero once a launch gave up waiting for a
 * member (that launch's outputs are invalid). The library sets it and never clears it; the
 * caller zeroes it when it allocates ws and reads it back (asynchronously) after the call. */
long tt_gru_fwd_ws_size(int dtype, int nrec, int B, int T, int H, long ldg, long ldy);
/* Launches tt_gru_fwd issues for this exact call shape given a tt_gru_fwd_ws_size workspace
 * (1 where a column-split or row-owning persistent kernel applies, T for the per-step
 * kernel); needs the device. */
int tt_gru_fwd_launches_for(int dtype, int nrec, int B, int T, int H, long ldg, long ldy);

/* Backward (BPTT) of tt_gru_fwd. Produces dL/dg (= dgx, feeds dWih, dbih and the
 * layer-input gradient) and dL/dgh (feeds dWhh), plus bias partial sums (one row per
 * 128-row batch tile: tt_gru_bias_rows(B) rows; columns r|z|n|ghn; reduce with tt_colsum:
 * dbih = [0:3H], dbhh = [0:2H] ++ [3H:4H]). */
typedef struct {
  const void* save;    /* [B*T, 4H] from tt_gru_fwd          */
  const void* y;       /* layer output (source of h_{s-1})   */
  const void* dy;      /* dL/dy (ldy) or NULL                */
  const float* dfinal; /* dL/dh_final [B, ldf] or NULL       */
  const void* whh;     /* [3H, H]                            */
  void* dgx;           /* [B*T, ldd]: dL/d(r|z|n pre-activation), 3H columns        */
  void* dgh;           /* [B*T, ldd]: dL/d(W_hn h + b_hn), H columns; dL/dgh (the
                          dW_hh operand) is [r|z columns of dgx, this block]        */
  void* dhstate;       /* scratch [2][B][H] of dtype (carry dh*z) */
  float* dbias_part;   /* fp32 [tt_gru_bias_rows(B)][4H]; zeroed by tt_gru_bwd */
  int dir;
} tt_gru_bwd_rec;

int tt_gru_bwd(int dtype, const tt_gru_bwd_rec* recs, int nrec, int B, int T, int H, long ldy,
               long ldd, long ldf, void* stream);
/* Kernel launches tt_gru_bwd issues: 1 for the row-owning bf16 kernel (H 256 or 512: one
 * workgroup per 128 batch rows x all H units walks every step), T otherwise. */
int tt_gru_bwd_launches(int dtype, int T, int H);
/* 1 when tt_gru_bwd keeps the BPTT carry on chip (the row-owning kernel at H <= 512: no
 * carry bytes in HBM), 0 when it round-trips a bf16 / fp32 carry buffer (dhstate). */
int tt_gru_bwd_carry_on_chip(int dtype, int T, int H);
int tt_gru_bias_rows(int B);

/* ------------------------------------------------------------ projection head */
/* Linear(4h->2h) -> LayerNorm(2h, eps) -> ReLU -> Linear(2h->h), fwd and bwd.
 * Replaces query_proj/doc_proj (enhanced_two_tower.py:36-48, applied :54,60).
 * Weights in dtype (w1 [2h,4h], w2 [h,2h]); biases/LN affine fp32. */
typedef struct {
  const void* w1; const float* b1; const float* ln_g; const float* ln_b;
  const void* w2; const float* b2;
  const void* x;   /* [B, 4h] dtype : cat(h_fwd_final, h_rev_final)            */
  void* p1;        /* [B, 2h] dtype : saved pre-LayerNorm activations           */
  float* mean;     /* [B]                                                       */
  float* rstd;     /* [B]                                                       */
  void* u;         /* [B, 2h] dtype : saved post-ReLU activations               */
  float* out;      /* [B, h]  fp32                                              */
} tt_head_fwd_io;

int tt_proj_head_fwd(int dtype, const tt_head_fwd_io* io, int ntower, int B, int h, float ln_eps,
                     void* stream);

typedef struct {
  const void* w1; const float* ln_g; const float* ln_b; const void* w2;
  const void* x; const void* p1; const float* mean; const float* rstd; const void* u;
  const float* dout;  /* [B, h] fp32 upstream gradient                              */
  float* dx;          /* [B, 4h] fp32 gradient wrt x                                */
  float* dw1; float* db1; float* dg; float* dbeta; float* dw2; float* db2;  /* fp32 grads (overwritten) */
  void* ws;           /* scratch, tt_proj_head_bwd_ws_size bytes                     */
} tt_head_bwd_io;

int tt_proj_head_bwd(int dtype, const tt_head_bwd_io* io, int ntower, int B, int h, float ln_eps,
                     void* stream);
long tt_proj_head_bwd_ws_size(int dtype, int B, int h);

/* Margin-model head Linear(2H->H) -> LayerNorm(H, eps) -> ReLU -> Dropout(drop_p), one
 * set of weights shared by both towers (margin_two_tower.py:30-35, applied in encode
 * :58-62). Query and doc rows are stacked into one [rows, 2H] batch, so the weight
 * gradients of the backward are already the sum over the two towers. C = H. The dropout
 * mask is the counter-based keep(drop_seed, row, col) of tt_gru_fwd, recomputed by the
 * backward. Weights in dtype (w1 [C, 2C]); biases/LN affine fp32. */
typedef struct {
  const void* x;   /* [rows, 2C] dtype : cat(h_fwd_final, h_rev_final)           */
  const void* w1; const float* b1; const float* ln_g; const float* ln_b;
  void* p1;        /* [rows, C] dtype : saved pre-LayerNorm activations          */
  float* mean;     /* [rows]                                                     */
  float* rstd;     /* [rows]                                                     */
  float* out;      /* [rows, C] fp32                                             */
} tt_head1_fwd_io;

int tt_proj_head1_fwd(int dtype, const tt_head1_fwd_io* io, long rows, int C, float ln_eps, float drop_p,
                      uint32_t drop_seed, void* stream);

typedef struct {
  const void* x; const void* w1; const float* ln_g; const float* ln_b;
  const void* p1; const float* mean; const float* rstd;
  const float* dout;  /* [rows, C] fp32 upstream gradient                          */
  float* dx;          /* [rows, 2C] fp32 gradient wrt x                            */
  float* dw1; float* db1; float* dg; float* dbeta;  /* fp32 grads (overwritten)    */
  void* ws;           /* scratch, tt_proj_head1_bwd_ws_size bytes                  */
} tt_head1_bwd_io;

int tt_proj_head1_bwd(int dtype, const tt_head1_bwd_io* io, long rows, int C, float drop_p, uint32_t drop_seed,
                      void* stream);
long tt_proj_head1_bwd_ws_size(int dtype, long rows, int C);

/* ---------------------------------------------------------------------- losses */
/* y = x / max(||x||_2, eps) row-wise (F.normalize, enhanced_two_tower.py:74-75; also
 * the normalisation inside F.cosine_similarity, :112-117,125-128). y in dtype, y32
 * optional fp32 copy, norm[rows] fp32 = ||x||. */
int tt_l2norm_fwd(int dtype, const float* x, long rows, int cols, float eps, void* y, float* y32,
                  float* norm, void* stream);
/* dx (+)= (dy - y (y.dy)) / max(||x||, eps)  (dy, y32 fp32). */
int tt_l2norm_bwd(const float* dy, const float* y32, const float* norm, long rows, int cols,
                  float eps, float* dx, int accumulate, void* stream);

/* InfoNCE / in-batch softmax cross-entropy over S = inv_tau * qn dn^T
 * (enhanced_two_tower.py:78-82). offdiag_sub is subtracted from every S_ij with
 * j != label_i: the in-batch branch of MarginRankingLoss (:92-101) uses
 * offdiag_sub = margin on un-normalised inputs.
 * Row i's label column is label_offset + i. The B x N score matrix is never written:
 * each workgroup streams dn tiles through one fused MFMA kernel with a running
 * log-sum-exp. Outputs lse[i] and row_loss[i] = lse[i] - S[i][label]. */
int tt_infonce_fwd(int dtype, const void* qn, long bq, const void* dn, long nd, int h,
                   float inv_tau, float offdiag_sub, long label_offset, float* lse,
                   float* row_loss, void* ws, void* stream);
long tt_infonce_fwd_ws_size(long bq, long nd);
/* Gradient of g * sum_i row_loss[i]: dqn [bq,h], ddn [nd,h] (fp32, overwritten).
 * gscale: DEVICE pointer to the fp32 upstream gradient g (autograd's grad_output, read
 * by the kernels so the backward never waits on the host), or NULL for g = 1.
 * ws: tt_infonce_bwd_ws_size bytes. */
int tt_infonce_bwd(int dtype, const void* qn, long bq, const void* dn, long nd, int h,
                   float inv_tau, float offdiag_sub, long label_offset, const float* lse,
                   const float* gscale, float* dqn, float* ddn, void* ws, void* stream);
long tt_infonce_bwd_ws_size(int dtype, long bq, long nd, int h);

/* Hard-negative mining, batched over rows (get_hard_negatives,
 * enhanced_two_tower.py:123-133): sims = qn dn^T (cosine for normalised inputs), the
 * positive column label_offset+i set to -1 (label_offset < 0: no column masked), top-k
 * (1 <= k <= min(16, nd)) indices per row sorted by descending similarity; ties broken
 * towards the lower column index. Also the scoring step of the serving /search
 * (server/python-api/app.py:94-101, label_offset < 0).
 * idx [bq, k] int32, val [bq, k] fp32 (optional). ws: tt_hardneg_ws_size bytes.
 * bf16 with h in {128, 256} (qn, dn 16-byte aligned, else TT_EINVAL) never stores the score matrix
 * (streamed MFMA scan + exact chunk selection + bit-identical rescoring, tt_score.hip). */
int tt_hardneg_topk(int dtype, const void* qn, long bq, const void* dn, long nd, int h,
                    long label_offset, int k, int32_t* idx, float* val, void* ws, void* stream);
long tt_hardneg_ws_size(int dtype, long bq, long nd, int h, int k);

/* Serving search (server/python-api/app.py:94-101: F.cosine_similarity of one encoded
 * query against every cached document row, then torch.topk): qn [Q, h] fp32 normalised
 * queries, dn [N, h] dtype normalised documents (resident), top-k (1 <= k <= min(16, N))
 * indices/scores per query, value descending, ties towards the lower document index.
 * Q <= 64: one fused pass over dn per 8 queries (per-lane top-k, no score matrix);
 * larger Q: cosine GEMM + column-split top-k. h % 8 == 0. ws: tt_search_ws_size bytes. */
int tt_search_topk(int dtype, const float* qn, long Q, const void* dn, long N, int h, int k,
                   int32_t* idx, float* val, void* ws, void* stream);
long tt_search_ws_size(int dtype, long Q, long N, int h, int k);

/* MarginRankingLoss with explicit negatives (enhanced_two_tower.py:102-121) on
 * normalised vectors: pos_i = qn_i.dn_{label_offset+i}, negm_i = mean_j qn_i.dn_{idx[i,j]},
 * row_loss_i = max(margin - pos_i + negm_i, 0). Negatives are rows of dn. */
int tt_margin_fwd(const float* qn, long bq, const float* dn, long nd, int h, long label_offset,
                  const int32_t* idx, int k, float margin, float* row_loss, void* stream);
/* Gradient of g * sum_i row_loss_i: dqn (overwritten), ddn (accumulated; the caller
 * zeroes it). gscale: device pointer to g (as tt_infonce_bwd) or NULL for 1.
 * ws: tt_margin_bwd_ws_size(bq, nd, h, k) bytes (required). Deterministic: no float
 * atomics; the rows are taken in groups of R (R (k + 1) <= 2048), each group sums the
 * q rows of each document it mined in entry order, and each document's group partials
 * are added in ascending group order (hard negatives are shared by many rows).
 * 1 <= k < 2048. */
int tt_margin_bwd(const float* qn, long bq, const float* dn, long nd, int h, long label_offset,
                  const int32_t* idx, int k, float margin, const float* gscale, float* dqn, float* ddn,
                  void* ws, void* stream);
long tt_margin_bwd_ws_size(long bq, long nd, int h, int k);

/* out[0] = scale * sum_i x[i]. */
int tt_sum(const float* x, long n, float scale, float* out, void* stream);

/* ------------------------------------------------------------------- optimiser */
/* torch.optim.Adam (train_enhanced.py:43,63) over up to 48 fp32 tensors per call,
 * bit-for-bit the update order of torch's single-tensor Adam:
 *   m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2 ;
 *   p -= lr/(1-b1^step) * m / (sqrt(v)/sqrt(1-b2^step) + eps)   (g += wd*p first).
 * skip: device int32 word or NULL; when it reads non-zero at launch time the kernel
 * changes nothing (p, m, v untouched). two_towers_amd.Adam passes the OR of the status
 * words of the column-split forwards since the last step (tt_gru_fwd ws), so a step whose
 * forward timed out cannot update the weights; no host synchronisation is involved. */
int tt_adam_multi(float* const* params, const float* const* grads, float* const* exp_avg,
                  float* const* exp_avg_sq, const long* sizes, int ntensors, float lr, float beta1,
                  float beta2, float eps, float weight_decay, int step, const int32_t* skip, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TT_HIP_H */
