// Score-matrix scans on MFMA that never store the B x N score matrix.
//
// Hard-negative mining (get_hard_negatives, enhanced_two_tower.py:123-133, batched over
// rows; the positive column scores -1, enhanced_two_tower.py:130) as an exact top-k in
// four launches:
//   1. hn_scan    : S = Q D^T on MFMA, streamed: one workgroup keeps 256 query rows in
//                   registers and sweeps 64-column document tiles through a 3-slot LDS
//                   ring (LDS-DMA, two tiles in flight). Per (row, 64-column chunk) it
//                   keeps only the chunk maximum.
//   2. hn_select  : per row, the k chunks ranked first by (chunk max desc, chunk asc).
//                   Every element of the row's top-k lies in them: the k-th chunk max
//                   theta is a value with >= k elements at or above it, so each top-k
//                   element is >= theta, and lives in a chunk whose max is > theta (all of
//                   those are selected) or == theta (the lowest-indexed of those are
//                   selected, and they hold the lowest-indexed elements equal to theta).
//   3. hn_rescore : per chunk, the rows that selected it (gathered 16 at a time) x the
//                   chunk's 64 columns recomputed with
//                   the SAME MFMA sequence as step 1 (same instruction, same k order, same
//                   fragment k layout), so each score is bit-identical to the one step 1
//                   ranked; k x 64 candidates per row.
//   4. hn_final   : per row, top-k of its candidates (value desc, column asc).
// Work: step 1 is the whole contraction (2 B N h FLOPs); steps 2-4 touch B k 64 h.
#include <float.h>
#include <stdlib.h>

#include "tt_api.h"
#include "tt_gemm_core.h"
#include "tt_topk.h"

namespace {

#ifndef HN_SPREAD  // 1: a tile's due DMAs spread over its k-steps (measured slower: 44.6 vs 38.2 us, the
#define HN_SPREAD 0  // last pieces then land one tile before their wait instead of two); 0: one burst
#endif
#ifndef HN_DSPLIT  // h 256: 1 = every wave takes all 64 documents of a tile for 32 queries (the
#define HN_DSPLIT 1  // round-3 form, 37.7 us); 2 = half the documents for 64 queries (41.9 us, r05_hn_scan_ab)
#endif
#ifndef HN_Q64_PF  // fragment prefetch distance (k-steps) of the 64-query scan: 0 keeps it spill-free
#define HN_Q64_PF 0
#endif
constexpr int SC_COLS = 64;     // document columns per tile (= per chunk)
constexpr int SC_TPS_MAX = 32;  // tiles per workgroup (chunk-max staging)

// Per width (h = 32 KS). h <= 256: 8 waves (two per SIMD, 256 query rows per workgroup)
// and a 4-slot LDS tile ring that travels in pairs. h 512: a tile is 64 KiB and the
// query fragments alone are 128 registers per lane, so 4 waves (one per SIMD, 512
// registers each, 128 query rows) and a 2-slot ring, one tile per barrier.
// DH (h 256): the waves split each tile's documents DH ways; a wave then holds RB = 2 DH
// query blocks (64 queries at DH 2, 128 registers of fragments) and reads only its 32
// documents' fragments, so every LDS fragment read feeds 4 MFMAs and the workgroup reads
// each tile from LDS 4 times instead of 8 -- the LDS reads, not the MFMAs, were the
// largest part of the scan (profiles/r04_hn_scan_diag.txt: 11 of 38 us). The two
// halves' chunk maxima meet in LDS (ds_max_f32; max is exact in any order).
// V: the variant (option hn_scan_v; h 256 only, 0 elsewhere).
// V 4: 8 waves of 64 queries (4 MFMA blocks) x all 64 documents of a tile, 512 query rows
// per workgroup: every LDS fragment read feeds 4 MFMAs (the workgroup reads a tile from
// LDS once per 64 queries instead of once per 32) and a workgroup's 512 x (8 tiles) block
// needs 512 KiB into the CU instead of 640; single accumulator set (the partner wave on the
// SIMD covers each wave's chunk-max epilogue), chunk maxima of at most 8 tiles staged.
// V 5: the round-3 body on a 5-slot ring retired ONE tile per barrier, four tiles (128 KiB)
// in flight instead of one pair (64 KiB): the chunk maxima leave the LDS (each wave stores
// its rows' maxima straight to CM, 16 lanes x 4 B per query block and tile) to make room,
// and every wait is counted (vmcnt = the DMAs of the 3 younger tiles + the 4 younger tiles'
// maxima stores; every tile issues the same DMA and store count, past-the-end tiles read
// the zero page or the next split's documents into a free slot).
template <int KS, int V = 0>
struct ScanCfg {
  static constexpr int WAVES = KS <= 8 ? 8 : 4;
  static constexpr int DH = KS == 8 && V == 0 ? HN_DSPLIT : 1;  // document splits per tile
  static constexpr int RB = V == 4 ? 4 : 2 * DH;                 // 16-query MFMA blocks per wave
  static constexpr int NDB = 4 / DH;                             // 16-document blocks per wave
  static constexpr int QW = WAVES / DH;                          // query groups
  static constexpr int ROWS = QW * RB * 16;
  static constexpr int SLOTS = V == 5 ? 5 : KS <= 8 ? 4 : 2;
  static constexpr bool SINGLE = DH > 1 || V == 4;  // one accumulator set, maxima after each tile
  static constexpr bool DIRECT = V == 5;            // maxima stored to CM from registers
  static constexpr int TPSM = V == 4 ? 8 : V == 5 ? 0 : SC_TPS_MAX;  // chunk-max staging (tiles)
  static constexpr long PLAN_TPS = V == 5 ? (1L << 30) : TPSM;       // tiles per workgroup cap
  static constexpr int PF = V == 4 ? HN_Q64_PF : 2;                  // fragment prefetch, k-steps ahead
};

// max over the four 16-lane rows of a wave (lanes l, l+16, l+32, l+48), result in all
TT_DEV float rowgroup_max4(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// LDS image of one 64-column document tile, h = 32 KS bf16 per document: document n
// holds CPR 16-byte chunks, chunk c stored at slot c ^ (n & 15) so that the fragment
// reads (16 documents x one chunk per lane group) are bank-conflict free.
template <int KS>
struct ScanTile {
  static constexpr int CPR = KS * 4;
  static constexpr int BYTES = SC_COLS * CPR * 16;
  static constexpr int DPW = BYTES / 1024 / ScanCfg<KS>::WAVES;  // 1 KiB DMA instructions per wave
  static_assert(DPW >= 1 && BYTES % (1024 * ScanCfg<KS>::WAVES) == 0, "tile/wave mismatch");
  TT_DEV static int off(int n, int c) { return (n * CPR + (c ^ (n & 15))) * 16; }
};

// One lane's share of a tile DMA, resolved once: element offset within the tile and the
// tile document it reads.
template <int KS, bool LAZY = false>  // LAZY: the lane's (document, offset) recomputed per piece (no registers held)
struct ScanDma {
  using TI = ScanTile<KS>;
  int doc[LAZY ? 1 : TI::DPW];
  int eoff[LAZY ? 1 : TI::DPW];
  TT_DEV static void at(int i, int& n, int& e) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int p = (wave * TI::DPW + i) * 64 + lane;
    n = p / TI::CPR;
    e = n * (32 * KS) + ((p % TI::CPR) ^ (n & 15)) * 8;
  }
  TT_DEV void init() {
    if constexpr (!LAZY) {
#pragma unroll
      for (int i = 0; i < TI::DPW; ++i) at(i, doc[i], eoff[i]);
    }
  }
  // piece i of the tile starting at document n0 into the slot at LDS address base
  TT_DEV void piece(const bf16_t* __restrict__ D, long nd, long n0, uint32_t base, int i) const {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int n, e;
    if constexpr (LAZY) {
      at(i, n, e);
    } else {
      n = doc[i];
      e = eoff[i];
    }
    const void* src = n0 + n < nd ? static_cast<const void*>(D + n0 * (32 * KS) + e) : ttg::g_tt_zero_page;
    ttg::dma16(src, __builtin_amdgcn_readfirstlane(base + (uint32_t)(wave * TI::DPW + i) * 1024u));
  }
  TT_DEV void issue(const bf16_t* __restrict__ D, long nd, long n0, uint32_t base) const {
#pragma unroll
    for (int i = 0; i < TI::DPW; ++i) piece(D, nd, n0, base, i);
  }
};

// Fragment of row `row` of a [nrows, 32 KS] bf16 matrix for k-step ks: lane holds
// elements k = 32 ks + 8 (lane >> 4) .. +8 (the 16x16x32 operand layout).
TT_DEV uint4 ld_frag(const bf16_t* __restrict__ base, long row, long nrows, int h, int ks) {
  const int lane = threadIdx.x & 63;
  if (row >= nrows) return make_uint4(0, 0, 0, 0);
  return *reinterpret_cast<const uint4*>(base + row * h + ks * 32 + 8 * (lane >> 4));
}

// Step 1. The MFMA runs transposed, C[doc][query] = sum_k D[doc][k] Q[query][k]: A = the
// LDS document fragments, B = the register-resident query fragments (both operands use
// the same 16-rows x 8-k per lane layout). So each lane holds 16 scores of ONE query per
// 64-document tile and the chunk maximum is 15 lane-local max + two permlane swaps.
// Grid: row tiles x column splits, 1-D: block b -> split b % S (a split's workgroups
// share one XCD label and its document slice stays in that L2), row tile b / S.
template <int KS, int V = 0>
__global__ __launch_bounds__(ScanCfg<KS>::WAVES * 64, 1) void hn_scan_kernel(const bf16_t* __restrict__ Q, long bq,
                                                                 const bf16_t* __restrict__ D, long nd,
                                                                 long label_off, int S, int tps, long nch,
                                                                 float* __restrict__ CM, int map) {
  using TI = ScanTile<KS>;
  using Cfg = ScanCfg<KS, V>;
  constexpr int SC_WAVES = Cfg::WAVES, SC_ROWS = Cfg::ROWS, SC_SLOTS = Cfg::SLOTS;
  constexpr int SC_RB = Cfg::RB, NDB = Cfg::NDB, DH = Cfg::DH, QW = Cfg::QW, TPSM = Cfg::TPSM;
  // tile ring + chunk maxima [tile][row]: 4 x 32 KiB + 32 KiB (h 256) or 2 x 64 KiB + 16
  // KiB (h 512), one workgroup per CU
  __shared__ __attribute__((aligned(16))) char lds[SC_SLOTS * TI::BYTES + TPSM * SC_ROWS * 4];
  float* cms = reinterpret_cast<float*>(lds + SC_SLOTS * TI::BYTES);
  // map 0: blocks round-robin over the XCDs, so split b % S stays on one XCD and its
  // document slice in that L2; map 1 (option hn_map): the S splits of a row tile share an
  // XCD (xcd_remap), so the tile's query rows are fetched into that L2 once
  // map 2: XCD x (= b % 8) owns row-tile half x & 1 and split quarter x >> 1, so each XCD
  // reads half of Q and a quarter of D (8 x 3 MB at 8192^2 x 256 instead of 8 x 4.5 MB);
  // needs RT % 2 == 0 and S % 4 == 0 (the host falls back to map 0 otherwise)
  int split, rt;
  if (map == 2) {
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3, sq = S >> 2;
    split = (x >> 1) * sq + j % sq;
    rt = (x & 1) * (int)(gridDim.x / S / 2) + j / sq;
  } else {
    const int bid = map ? ttg::xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    split = bid % S;
    rt = bid / S;
  }
  const long t0 = (long)split * tps;
  const int nt = (int)(nch - t0 < tps ? nch - t0 : tps);
  if (nt <= 0) return;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int qw = wave % QW, dh = wave / QW;  // query group, document part
  const int db0 = dh * NDB;                  // this wave's first 16-document block
  const long row0 = (long)rt * SC_ROWS + qw * (SC_RB * 16);
  if (DH > 1) {  // the halves' chunk maxima meet in LDS: start from -inf (ordered before
    // the first ds_max by tile 0's barrier)
    for (int e = threadIdx.x; e < TPSM * SC_ROWS; e += SC_WAVES * 64) cms[e] = -FLT_MAX;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  constexpr int h = 32 * KS;
  // The first two tiles are requested before the query rows, so their latency overlaps.
  ScanDma<KS, (V == 4)> dm;
  dm.init();
  const uint32_t lbase = __builtin_amdgcn_readfirstlane(ttg::lds_addr_of(lds));
  dm.issue(D, nd, t0 * SC_COLS, lbase);
  if (SC_SLOTS == 4 && nt > 1) dm.issue(D, nd, (t0 + 1) * SC_COLS, lbase + TI::BYTES);
  if constexpr (Cfg::DIRECT) {  // tiles 1-3 (unconditionally: uniform counts)
#pragma unroll
    for (int j = 1; j < 4; ++j) dm.issue(D, nd, (t0 + j) * SC_COLS, lbase + (uint32_t)j * TI::BYTES);
  }
  uint4 qa[SC_RB][KS];
#pragma unroll
  for (int qb = 0; qb < SC_RB; ++qb)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qa[qb][ks] = ld_frag(Q, row0 + qb * 16 + (lane & 15), bq, h, ks);
  // Retire the query loads here, so that hipcc does not place a vmcnt(0) inside the tile
  // loop (it cannot see the LDS-DMAs and would wait for the tiles in flight every tile).
#pragma unroll
  for (int qb = 0; qb < SC_RB; ++qb)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      asm volatile("" ::"v"(qa[qb][ks].x), "v"(qa[qb][ks].y), "v"(qa[qb][ks].z), "v"(qa[qb][ks].w));
  if constexpr (Cfg::DIRECT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tiles 0-3 landed
  // CM rows of this workgroup through a buffer range: rows past bq store nothing (an
  // offset past num_records), so every wave issues the same number of store instructions
  const __amdgpu_buffer_rsrc_t rcm = tt_rsrc(CM);

  // Tiles travel in pairs: at every even tile, one wait + barrier retires the pair (t, t+1)
  // for every wave and frees slots (t+2)%4, (t+3)%4 (last read before this barrier), into
  // which the next pair is requested; it lands while this pair is computed.
  // With two slots (h 512) every tile is retired alone and the next one requested into
  // the slot its predecessor freed.
  // The DMAs of the tiles that become due at tile t's barrier (t + 1 with two slots; t + 2
  // and t + 3 at the start of a pair) are issued at tile t's first k-step (HN_SPREAD 1:
  // spread over its k-steps, NPK per k-step -- slower, profiles/r05_hn_scan_ab_e.txt).
  constexpr int NPD = SC_SLOTS == 4 ? 2 * TI::DPW : TI::DPW;  // pieces due per DMA tile
  constexpr int NPK = HN_SPREAD ? (NPD + KS - 1) / KS : NPD;  // pieces per k-step (0: all at k-step 0)
  // 5-slot ring: tile t's DMAs were issued during tile t-4; younger than them: the DMAs of
  // tiles t+1..t+3 and the maxima stores of tiles t-5..t-2 (issued while processing tiles
  // t-4..t-1; tile 0 stores nothing during tile 0), SC_RB per tile
  constexpr int VM_FULL = 3 * TI::DPW + 4 * SC_RB, VM_T4 = 3 * TI::DPW + 3 * SC_RB;
  static_assert(!Cfg::DIRECT || VM_FULL < 64, "vmcnt range");
  auto sync = [&](int t) {
    if constexpr (Cfg::DIRECT) {
      if (t == 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_T4) : "memory");
      else if (t > 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_FULL) : "memory");
      __builtin_amdgcn_s_barrier();  // every wave done with tile t-1: its slot takes tile t+4
    } else if (SC_SLOTS == 2 || (t & 1) == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  };
  // issue the share of k-step ks of the pieces due at tile t (a tile with no pieces due:
  // the second of a pair)
  auto dma_k = [&](int t, int ks) {
#pragma unroll
    for (int u = 0; u < NPK; ++u) {
      const int i = ks * NPK + u;
      if (i >= NPD) break;
      if constexpr (Cfg::DIRECT) {
        const int tt = t + 4;  // always issued (see sync)
        dm.piece(D, nd, (t0 + tt) * SC_COLS, lbase + (uint32_t)(tt % 5) * TI::BYTES, i);
      } else if (SC_SLOTS == 2) {
        if (t + 1 < nt) dm.piece(D, nd, (t0 + t + 1) * SC_COLS, lbase + (uint32_t)((t + 1) % 2) * TI::BYTES, i);
      } else if ((t & 1) == 0) {
        const int tt = t + 2 + i / TI::DPW;
        if (tt < nt) dm.piece(D, nd, (t0 + tt) * SC_COLS, lbase + (uint32_t)(tt % SC_SLOTS) * TI::BYTES, i % TI::DPW);
      }
    }
  };
  // Chunk maxima of tile t (masked form: positive -> -1, documents past nd -> -inf).
  // the chunk maximum of (tile t, row) -> cms: stored, or max-ed with the other document
  // part's (ds_max_f32 on the -inf initialised slot)
  auto put_max = [&](int t, int qb, float m) {
    if (lane < 16) {
      if constexpr (Cfg::DIRECT) {
        const long row = row0 + qb * 16 + lane;
        const uint32_t off = row < bq ? (uint32_t)((row * nch + t0 + t) * 4) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(m), rcm, (int)off, 0, 0);
        return;
      }
      float* dst = cms + t * SC_ROWS + qw * SC_RB * 16 + qb * 16 + lane;
      if constexpr (DH == 1) {
        *dst = m;
      } else {
        const uint32_t a = ttg::lds_addr_of(dst);
        asm volatile("ds_max_f32 %0, %1" ::"v"(a), "v"(m) : "memory");
      }
    }
  };
  auto chunk_max = [&](const f32x4 (&a)[NDB][SC_RB], int t, bool masked) {
    const int n0 = (int)((t0 + t) * SC_COLS);
    const bool diag = label_off >= 0 && label_off + row0 < n0 + SC_COLS && n0 < label_off + row0 + SC_RB * 16;
#pragma unroll
    for (int qb = 0; qb < SC_RB; ++qb) {
      float v[4 * NDB];
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[db * 4 + r] = a[db][qb][r];
      if (masked) {
        // lane-relative: document (db0 + db) * 16 + 4 (lane >> 4) + r is the label iff
        // db * 16 + r == lab, past nd iff db * 16 + r >= lim (compile-time left sides, so no
        // per-element index registers are held across the tile loop)
        const int sh = db0 * 16 + 4 * (lane >> 4) + (int)n0;
        const int lab = (int)(label_off + row0) + qb * 16 + (lane & 15) - sh;
        const int lim = (int)(nd - sh);
#pragma unroll
        for (int db = 0; db < NDB; ++db)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (diag && db * 16 + r == lab) v[db * 4 + r] = -1.f;
            if (db * 16 + r >= lim) v[db * 4 + r] = -FLT_MAX;
          }
      }
      float m = fmaxf(fmaxf(v[0], v[1]), v[2]);
#pragma unroll
      for (int j = 3; j < 4 * NDB - 1; j += 2) m = fmaxf(fmaxf(m, v[j]), v[j + 1]);
      m = rowgroup_max4(fmaxf(m, v[4 * NDB - 1]));
      put_max(t, qb, m);
    }
  };
  // MFMAs of tile t into acc, with (EPI) the unmasked chunk maxima of tile t-1 (prev)
  // woven between its k-steps. Program order is pinned with sched_barrier: per k-step,
  // the fragment reads of k-step ks+2, the 8 MFMAs of ks, then one slice of the epilogue,
  // so the LDS reads run two k-steps ahead and the epilogue VALU fills MFMA issue gaps
  // (hipcc otherwise sinks every read to just before its MFMA and clusters the VALU).
  auto tile = [&](f32x4 (&acc)[NDB][SC_RB], const f32x4 (&prev)[NDB][SC_RB], int t, bool epi) {
    const char* img = lds + (t % SC_SLOTS) * TI::BYTES;
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int qb = 0; qb < SC_RB; ++qb) acc[db][qb] = f32x4{0.f, 0.f, 0.f, 0.f};
    // fragment ring: k-steps PF ahead
    constexpr int PF = Cfg::PF;
    uint4 fa[PF + 1][NDB];
#pragma unroll
    for (int ks = 0; ks < PF; ++ks)
#pragma unroll
      for (int db = 0; db < NDB; ++db)
        fa[ks][db] =
            *reinterpret_cast<const uint4*>(img + TI::off((db0 + db) * 16 + (lane & 15), ks * 4 + (lane >> 4)));
    // epilogue slice i: query block i / NSQ; NDB / 2 partial maxima over two document
    // blocks each, then the 4-row-group reduction and the store
    constexpr int NSQ = NDB / 2 + 1;  // slices per query block
    float m = 0.f;
    auto slice = [&](int i) {
      const int qb = i / NSQ, part = i % NSQ;
      if (qb >= SC_RB) return;
      if (part < NSQ - 1) {
        const f32x4 x = prev[2 * part][qb], y = prev[2 * part + 1][qb];
        const float hm =
            fmaxf(fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3])), fmaxf(fmaxf(y[0], y[1]), fmaxf(y[2], y[3])));
        m = part == 0 ? hm : fmaxf(m, hm);
      } else {
        m = rowgroup_max4(m);
        put_max(t - 1, qb, m);
      }
    };
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      dma_k(t, ks);
      if (ks + PF < KS) {
#pragma unroll
        for (int db = 0; db < NDB; ++db)
          fa[(ks + PF) % (PF + 1)][db] = *reinterpret_cast<const uint4*>(
              img + TI::off((db0 + db) * 16 + (lane & 15), (ks + PF) * 4 + (lane >> 4)));
      }
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int qb = 0; qb < SC_RB; ++qb)
          acc[db][qb] = ttg::mma<bf16_t>(fa[ks % (PF + 1)][db], qa[qb][ks], acc[db][qb]);
      if (epi) slice(ks);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (epi) {
#pragma unroll
      for (int i = KS; i < NSQ * SC_RB; ++i) slice(i);
    }
  };
  f32x4 accA[NDB][SC_RB], accB[NDB][SC_RB];
  // Tiles holding a positive (label) column or documents past nd take the masked form.
  auto special = [&](int t) {
    const long n0 = (t0 + t) * SC_COLS;
    return (label_off >= 0 && label_off + row0 < n0 + SC_COLS && n0 < label_off + row0 + SC_RB * 16) ||
           n0 + SC_COLS > nd;
  };
  auto step = [&](f32x4 (&cur)[NDB][SC_RB], const f32x4 (&prev)[NDB][SC_RB], int t) {  // t >= 1
    sync(t);
    if (special(t - 1)) {
      tile(cur, prev, t, false);
      chunk_max(prev, t - 1, true);
    } else {
      tile(cur, prev, t, true);
    }
  };
  if constexpr (Cfg::SINGLE) {
    // document-split and 64-query forms: the 64-query fragments leave no registers for a
    // second accumulator set, so each tile's maxima follow its own MFMAs (the partner wave
    // on the SIMD keeps the matrix pipe busy meanwhile)
    for (int t = 0; t < nt; ++t) {
      sync(t);
      tile(accA, accA, t, false);
      chunk_max(accA, t, special(t));
    }
  } else {
    sync(0);
    tile(accB, accA, 0, false);
    int t = 1;
    for (; t + 1 < nt; t += 2) {
      step(accA, accB, t);
      step(accB, accA, t + 1);
    }
    if (t < nt) {
      step(accA, accB, t);
      chunk_max(accA, t, special(t));
    } else {
      chunk_max(accB, t - 1, special(t - 1));
    }
  }
  if constexpr (Cfg::DIRECT) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing zero-page / next-split DMAs land before exit
    return;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's ds_max (inline asm: not counted by hipcc)
  __syncthreads();
  const long rbase = (long)rt * SC_ROWS;
  for (int e = threadIdx.x; e < SC_ROWS * nt; e += SC_WAVES * 64) {
    const int rl = e / nt, tt = e % nt;
    if (rbase + rl < bq) CM[(rbase + rl) * nch + t0 + tt] = cms[tt * SC_ROWS + rl];
  }
}

// Step 2: one wave per row: sel[row][0..nsel) = the chunks ranked first.
template <int KM>
__global__ __launch_bounds__(256) void hn_select_kernel(const float* __restrict__ CM, long bq, long nch, int k,
                                                        int32_t* __restrict__ sel) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= bq) return;
  float lv[KM];
  int li[KM];
  ttk::init<KM>(lv, li);
  const int nsel = (int)(nch < k ? nch : k);
  // four loads in flight per lane before the inserts (nch is 128 at 8192 documents)
  const float* cr = CM + row * nch;
  for (long c0 = lane; c0 < nch; c0 += 4 * 64) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = c0 + u * 64 < nch ? cr[c0 + u * 64] : -FLT_MAX;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (c0 + u * 64 < nch) ttk::insert<KM>(lv, li, nsel, v[u], (int)(c0 + u * 64));
  }
  float ov[KM];
  int oi[KM];
  ttk::wave_topk<KM>(lv, li, nsel, ov, oi);
  if (lane == 0)
    for (int q = 0; q < nsel; ++q) sel[row * k + q] = oi[q];
}

// Step 3: one workgroup per (chunk c, segment of RS_SEG rows). It collects the (row,
// slot) entries of its segment that selected c (a scan of sel; LDS list), then its waves
// rescore them 16 rows at a time with the MFMA orientation and k order of step 1: the
// chunk's documents as A (staged in LDS), the gathered query rows as B. The segments bound
// the work of one workgroup when every row selects the same chunks (correlated rows).
constexpr int RS_SEG = 1024;
constexpr int RS_THREADS = 512;

template <int KS>
__global__ __launch_bounds__(RS_THREADS) void hn_rescore_kernel(const bf16_t* __restrict__ Q, long bq,
                                                         const bf16_t* __restrict__ D, long nd, long label_off, int k,
                                                         int nsel, const int32_t* __restrict__ sel,
                                                         float* __restrict__ cand) {
  constexpr int h = 32 * KS;
  // the chunk's documents (64 x h bf16: 16 / 32 / 64 KiB) are staged in LDS, 16-byte
  // chunk c of document n at slot c ^ (n & 15) so the 16-document fragment reads are
  // conflict-free (held in registers instead, h 256 takes 207 registers per lane and
  // measured 29.7 us at 8192 x 8192 for the rescoring against 22.1 at h 512 from LDS)
  constexpr int CPD = 4 * KS;  // 16-byte chunks per document
  __shared__ int list[RS_SEG];  // a row selects a chunk at most once
  __shared__ int lcount;
  __shared__ uint4 dimg[SC_COLS * CPD];
  const int c = blockIdx.x;
  const long n0 = (long)c * SC_COLS;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long seg = (long)blockIdx.y * RS_SEG;
  const long seg1 = seg + RS_SEG < bq ? seg + RS_SEG : bq;
  if (threadIdx.x == 0) lcount = 0;
#pragma unroll
  for (int q = 0; q < SC_COLS * CPD / RS_THREADS; ++q) {
    const int i = threadIdx.x + q * RS_THREADS, n = i / CPD, cc = i % CPD;
    dimg[n * CPD + (cc ^ (n & 15))] =
        n0 + n < nd ? *reinterpret_cast<const uint4*>(D + (n0 + n) * h + cc * 8) : make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  // the segment's entries, 4 per 16-byte load (seg * k is a multiple of 4)
  // The list order depends on the LDS atomic's arbitration, but no output does: each
  // entry e's 64 scores go to cand[e] and are computed by lanes whose B fragment is that
  // entry's query row only (an MFMA output element C[doc][query] reads one A row and one
  // B row), so which wave or which lane group takes the entry changes nothing.
  const int total = (int)(seg1 - seg) * k;
  const int4* s4 = reinterpret_cast<const int4*>(sel + seg * k);
#pragma unroll 4
  for (int i = threadIdx.x; i < total / 4; i += RS_THREADS) {
    const int4 v = s4[i];
    const int w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (w[j] == c && (nsel == k || (4 * i + j) % k < nsel)) list[atomicAdd(&lcount, 1)] = 4 * i + j;
  }
  for (int e = total / 4 * 4 + threadIdx.x; e < total; e += RS_THREADS)
    if (sel[seg * k + e] == c && (nsel == k || e % k < nsel)) list[atomicAdd(&lcount, 1)] = e;
  __syncthreads();
  const int n = lcount;
  if (wave * 16 >= n) return;
  for (int g = wave; g * 16 < n; g += RS_THREADS / 64) {
    const int ei = g * 16 + (lane & 15);
    const long e = ei < n ? seg * k + list[ei] : -1;
    const long row = e >= 0 ? e / k : bq;  // bq -> zero fragment
    // keeps the LDS fragment reads inside the loop (hoisted, they would need 256 registers)
    asm volatile("" ::: "memory");
    f32x4 acc[4];
#pragma unroll
    for (int db = 0; db < 4; ++db) acc[db] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const uint4 qf = ld_frag(Q, row, bq, h, ks);
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const int dn = db * 16 + (lane & 15);
        const uint4 df = dimg[dn * CPD + ((ks * 4 + (lane >> 4)) ^ (dn & 15))];
        acc[db] = ttg::mma<bf16_t>(df, qf, acc[db]);
      }
    }
    if (e >= 0) {
      float* dst = cand + e * SC_COLS;  // e = row * k + slot
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long doc = n0 + db * 16 + 4 * (lane >> 4) + r;
          v[r] = acc[db][r];
          if (label_off >= 0 && doc == label_off + row) v[r] = -1.f;
          if (doc >= nd) v[r] = -FLT_MAX;
        }
        *reinterpret_cast<float4*>(dst + db * 16 + 4 * (lane >> 4)) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  }
}

// Step 4: one wave per row over its nsel x 64 candidates.
template <int KM>
__global__ __launch_bounds__(256) void hn_final_kernel(const float* __restrict__ cand, const int32_t* __restrict__ sel,
                                                       long bq, long nch, int k, int32_t* __restrict__ idx,
                                                       float* __restrict__ val) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= bq) return;
  const int nsel = (int)(nch < k ? nch : k);
  float lv[KM];
  int li[KM];
  ttk::init<KM>(lv, li);
  // every selected chunk's candidate and chunk id requested before the first insert
  float cv[KM];
  int cc[KM];
#pragma unroll
  for (int s = 0; s < KM; ++s) {
    cv[s] = s < nsel ? cand[(row * k + s) * SC_COLS + lane] : -FLT_MAX;
    cc[s] = s < nsel ? sel[row * k + s] : 0;
  }
#pragma unroll
  for (int s = 0; s < KM; ++s)
    if (s < nsel) ttk::insert<KM>(lv, li, k, cv[s], cc[s] * SC_COLS + lane);
  float ov[KM];
  int oi[KM];
  ttk::wave_topk<KM>(lv, li, k, ov, oi);
  if (lane == 0) {
    for (int q = 0; q < k; ++q) {
      idx[row * k + q] = oi[q];
      if (val) val[row * k + q] = ov[q];
    }
  }
}

struct HnPlan {
  long nch, RT, S, tps;
  long off_sel, off_cand, bytes;
};

long al256(long x) { return (x + 255) & ~255L; }

HnPlan hn_plan(long bq, long nd, int k, int rows, long tpsm = SC_TPS_MAX) {
  HnPlan p{};
  p.nch = (nd + SC_COLS - 1) / SC_COLS;
  p.RT = (bq + rows - 1) / rows;
  long S = (256 + p.RT - 1) / p.RT;
  const long smin = (p.nch + tpsm - 1) / tpsm;
  if (S < smin) S = smin;
  if (S > p.nch) S = p.nch;
  p.tps = (p.nch + S - 1) / S;
  p.S = (p.nch + p.tps - 1) / p.tps;
  p.off_sel = al256(bq * p.nch * 4);
  p.off_cand = p.off_sel + al256(bq * k * 4);
  p.bytes = p.off_cand + al256(bq * k * SC_COLS * 4);
  return p;
}

template <int KS, int V>
void hn_scan_launch(const bf16_t* qn, long bq, const bf16_t* dn, long nd, long label_offset, const HnPlan& p, float* CM,
                    hipStream_t st) {
  int map = tt::opt(tt::OPT_HN_MAP);
  if (map == 2 && (p.RT % 2 != 0 || p.S % 4 != 0)) map = 0;
  hipLaunchKernelGGL((hn_scan_kernel<KS, V>), dim3((unsigned)(p.RT * p.S)), dim3(ScanCfg<KS, V>::WAVES * 64), 0, st, qn,
                     bq, dn, nd, label_offset, (int)p.S, (int)p.tps, p.nch, CM, map);
}

template <int KS>
int hn_run(const bf16_t* qn, long bq, const bf16_t* dn, long nd, long label_offset, int k, int32_t* idx, float* val,
           char* ws, hipStream_t st) {
  int v = KS == 8 ? tt::opt(tt::OPT_HN_SCAN_V) : 0;
  if (v != 4 && v != 5) v = 0;
  if (v == 5 && bq * ((nd + SC_COLS - 1) / SC_COLS) * 4 >= (1L << 31)) v = 0;  // CM offsets in 32 bits
  const HnPlan p = v == 4   ? hn_plan(bq, nd, k, ScanCfg<KS, 4>::ROWS, ScanCfg<KS, 4>::PLAN_TPS)
                   : v == 5 ? hn_plan(bq, nd, k, ScanCfg<KS, 5>::ROWS, ScanCfg<KS, 5>::PLAN_TPS)
                            : hn_plan(bq, nd, k, ScanCfg<KS>::ROWS);
  float* CM = reinterpret_cast<float*>(ws);
  int32_t* sel = reinterpret_cast<int32_t*>(ws + p.off_sel);
  float* cand = reinterpret_cast<float*>(ws + p.off_cand);
  const int nsel = (int)(p.nch < k ? p.nch : k);
  if (tt::opt(tt::OPT_HN_SCAN_GEMM) && (32 * KS) % 64 == 0) {
    // the same chunk maxima from the persistent 256x256 GEMM (tt_gemm.hip gemm_persist HN):
    // same MFMA, operand orientation and k order as hn_scan_kernel, so hn_rescore below
    // still reproduces every ranked value bit for bit
    TT_PROPAGATE(tt::tt_hn_scan_gemm(qn, bq, dn, nd, 32 * KS, label_offset, CM, p.nch, st));
  } else {
    if constexpr (KS == 8) {
      if (v == 4)
        hn_scan_launch<KS, 4>(qn, bq, dn, nd, label_offset, p, CM, st);
      else if (v == 5)
        hn_scan_launch<KS, 5>(qn, bq, dn, nd, label_offset, p, CM, st);
      else
        hn_scan_launch<KS, 0>(qn, bq, dn, nd, label_offset, p, CM, st);
    } else {
      hn_scan_launch<KS, 0>(qn, bq, dn, nd, label_offset, p, CM, st);
    }
    TT_CHECK_LAUNCH("hn_scan_kernel");
  }
  const dim3 rows4((unsigned)tt_ceil_div(bq, 4));
  if (k <= 8)
    hipLaunchKernelGGL((hn_select_kernel<8>), rows4, dim3(256), 0, st, CM, bq, p.nch, k, sel);
  else
    hipLaunchKernelGGL((hn_select_kernel<16>), rows4, dim3(256), 0, st, CM, bq, p.nch, k, sel);
  TT_CHECK_LAUNCH("hn_select_kernel");
  hipLaunchKernelGGL((hn_rescore_kernel<KS>), dim3((unsigned)p.nch, (unsigned)tt_ceil_div(bq, RS_SEG)), dim3(RS_THREADS), 0, st, qn, bq, dn, nd, label_offset,
                     k, nsel, sel, cand);
  TT_CHECK_LAUNCH("hn_rescore_kernel");
  if (k <= 8)
    hipLaunchKernelGGL((hn_final_kernel<8>), rows4, dim3(256), 0, st, cand, sel, bq, p.nch, k, idx, val);
  else
    hipLaunchKernelGGL((hn_final_kernel<16>), rows4, dim3(256), 0, st, cand, sel, bq, p.nch, k, idx, val);
  TT_CHECK_LAUNCH("hn_final_kernel");
  return 0;
}

}  // namespace

// Used by tt_hardneg_topk (tt_loss.hip) for bf16 operands with h in {128, 256, 512}.
// The workspace does not depend on the rows per workgroup.
long tt_hn_scan_ws_size(long bq, long nd, int k) { return hn_plan(bq, nd, k, ScanCfg<8>::ROWS).bytes; }

// option hn_gemm = 1 forces the GEMM + split top-k path (tests compare the two bit-exactly:
// both produce every score with the same MFMA instruction and k order).
bool tt_hn_scan_supported(int dtype, int h) {
  const bool force_gemm = tt::opt(tt::OPT_HN_GEMM) == 1;
  return !force_gemm && dtype == TT_BF16 && (h == 128 || h == 256 || h == 512);
}

int tt_hn_scan_topk(const void* qn, long bq, const void* dn, long nd, int h, long label_offset, int k, int32_t* idx,
                    float* val, void* ws, void* stream) {
  const bf16_t* q = static_cast<const bf16_t*>(qn);
  const bf16_t* d = static_cast<const bf16_t*>(dn);
  char* w = static_cast<char*>(ws);
  hipStream_t st = (hipStream_t)stream;
  if (h == 512) return hn_run<16>(q, bq, d, nd, label_offset, k, idx, val, w, st);
  if (h == 256) return hn_run<8>(q, bq, d, nd, label_offset, k, idx, val, w, st);
  return hn_run<4>(q, bq, d, nd, label_offset, k, idx, val, w, st);
}
