// Host-side helpers for the C-ABI layer: error capture and launch checks.
#pragma once
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include "../../include/tt_hip.h"

namespace tt {
void set_error(const char* fmt, ...);

// Kernel-variant switches. Read once from the environment (TT_GRU_STEP, ...) when the
// library is first used, changed only through tt_set_option(): nothing on a launch
// path calls getenv.
enum Opt {
  OPT_GRU_STEP,         // 1: per-step GRU forward even where the persistent kernel applies
  OPT_GRU_DEPTH,        // persistent forward W_hh ring depth cap (1, 2, 4)
  OPT_GRU_BWD_ROWS,     // 128 or 64 batch rows per backward step tile (0: by grid size)
  OPT_GRU_BWD_BIG,      // 0: 128x128 backward step kernels instead of 256x256
  OPT_GRU_BWD_STREAMS,  // 1: one stream chain for the 128x128 backward
  OPT_GEMM_PERSIST,     // 0: no persistent short-K GEMM
  OPT_GEMM_A3,          // 1: 256x256 GEMM with A prefetched two K-tiles ahead (3-slot A ring)
  OPT_GEMM_REGSTAGE,    // 1/2: force register staging / 128-tiles (9: no epilogue, timing)
  OPT_GEMM_STREAM_OUT,  // 0: no write-through output stores
  OPT_HN_GEMM,          // 1: hard-negative top-k through GEMM + split top-k, no scan
  OPT_GRU_BWD_PERSIST,  // 0: per-step backward launches instead of the row-owning kernel; 2: also at H 1024
  OPT_GRU_FWD_STEP_ROWS, // per-step GRU forward batch rows per tile: 128, 256 (0: by size)
  OPT_INFONCE_FLASH,    // 0: InfoNCE backward through a materialised dS (bf16, h 128/256 default fused)
  OPT_HN_MAP,           // hn_scan block -> (row tile, split) map: 0 split per XCD, 1 row tile per XCD, 2 (default) row-tile half x split quarter per XCD
  OPT_GEMM_SKEW,        // persistent GEMM: start workgroup w after (w % 4) * skew * 4096 cycles
  OPT_GEMM_PERSIST_MAXK,  // persistent GEMM for problems of at most this many K-tiles
  OPT_GRU_FWD_XC,       // column-split persistent forward: 0 off, 1 where the batch fills it, 2 wherever it
                        // applies (+4: write-through exchange images; +16: members dealt across XCDs)
  OPT_GRU_XC_SKIP,      // diagnostic: member m-1 of group 0 never publishes (0: off); the others' waits time out
  OPT_GRU_XC_SPINS,     // column-split wait bound: log2 of the poll count before a wait gives up (default 22)
  OPT_GRU_BWD_SKEW,     // gru_bwd_rows: start delay (s_sleep 127 units) of half the workgroups of each XCD
                        // (default 14, about half a step at configs[2]: 7.05-7.09 vs 7.49-7.54 ms per launch)
  OPT_GRU_FWD_SKEW,     // gru_fwd_xcp: start delay (s_sleep 127 units) of the odd groups
  OPT_GEMM_BRES,        // 0: no B-resident short-K GEMM (layer-0 input projection)
  OPT_GRU_XC_COOP,      // 1: column-split forward by hipLaunchCooperativeKernel (default 0: a plain, occupancy-checked launch)
  OPT_GEMM_BUF,         // 0: 256x256 GEMM operand DMAs through per-lane pointers instead of buffer resources
  OPT_GEMM_ORDER,       // 1: persistent GEMM tiles in column groups per XCD
  OPT_GRU_STEP_RING,    // LDS stages of the per-step GRU kernels' product (2: double buffer; fwd uses <= 3)
  OPT_GRU_FWD_XS,       // 1: column-split forward with matrix and vector waves (gru_fwd_xs, H 512); 0: gru_fwd_xcp
  OPT_HN_SCAN_GEMM,     // 1: hard-negative scan on the persistent 256x256 GEMM with a chunk-max epilogue
                        // (bit-identical; measured slower: 44.8 vs 38.7 us at 8192^2 x 256); 0: hn_scan_kernel
  OPT_GEMM_IEPI,        // 1: the persistent GEMM's plain bf16 bias epilogue interleaved into the next tile's first K-tile
  OPT_BRES_ROWS,        // gemm_bres rows per wave tile: 32 (8 waves) or 64 (4 waves, each B fragment read feeds 4 MFMAs)
  OPT_HN_SCAN_V,        // h 256 hard-negative scan variant: 0 round-3 form, 4 64 queries per wave, 5 five-slot ring
  OPT_GEMM_W4,          // 1: bf16 NT GEMMs with bias on the four-wave 128x128-per-wave kernel (gemm_w4)
  OPT_N
};
int opt(Opt o);
// tt_gemm.hip: the hard-negative scan's chunk maxima (tt_score.hip step 1) on gemm_persist
int tt_hn_scan_gemm(const void* q, long bq, const void* d, long nd, int h, long label_off, float* cm, long nch,
                    hipStream_t st);
}  // namespace tt

#define TT_CHECK_ARG(cond, ...)            \
  do {                                     \
    if (!(cond)) {                         \
      tt::set_error(__VA_ARGS__);          \
      return TT_EINVAL;                    \
    }                                      \
  } while (0)

#define TT_CHECK_LAUNCH(what)                                                        \
  do {                                                                               \
    hipError_t e_ = hipGetLastError();                                               \
    if (e_ != hipSuccess) {                                                          \
      tt::set_error("%s: %s", what, hipGetErrorString(e_));                          \
      return (int)e_;                                                                \
    }                                                                                \
  } while (0)

#define TT_CHECK_HIP(expr)                                                           \
  do {                                                                               \
    hipError_t e_ = (expr);                                                          \
    if (e_ != hipSuccess) {                                                          \
      tt::set_error("%s: %s", #expr, hipGetErrorString(e_));                         \
      return (int)e_;                                                                \
    }                                                                                \
  } while (0)

#define TT_PROPAGATE(expr)     \
  do {                         \
    int rc_ = (expr);          \
    if (rc_ != 0) return rc_;  \
  } while (0)

static inline int tt_ceil_div(long a, long b) { return (int)((a + b - 1) / b); }
