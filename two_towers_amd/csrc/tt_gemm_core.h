// MFMA GEMM main loop shared by every contraction on the path (input projections,
// GRU step GEMMs, weight gradients, projection head).
//
// One 256-thread workgroup (4 waves as 2x2) computes a BM x BN fp32 tile of
//     C[m][n] = sum_k A(m,k) * B(n,k)
// Each operand is staged through LDS in one of two layouts:
//   K-contig ("KC"): element (r,k) at row r, k contiguous   -> LDS image [rows][128 B]
//   K-outer  ("KO"): element (r,k) at row k, r contiguous   -> LDS image [k][rows]
// so NT, NN and TN products all run on the same loop (no transposed copies).
//
// A K-tile is 128 bytes of K per row (64 bf16 or 32 fp32); it is consumed in two
// 64-byte sub-steps. One 16-byte LDS chunk of a KC row holds 8 bf16 / 4 fp32 k-values:
//   bf16: lane l reads 16 B at chunk (l>>4)+4*ks -> k = 8*(l>>4)+j, exactly the
//         v_mfma_f32_16x16x32_bf16 fragment.
//   fp32: the same 16 B are 4 k-values; four v_mfma_f32_16x16x4_f32 consume them
//         with k permuted identically on A and B, so the sum is unchanged.
// KO images are read with ds_read_b64_tr_b16 (bf16) or ds_read_b32 (fp32).
// All images are XOR-swizzled so that the fragment reads are bank-conflict free
// (verified against the gfx950 lane groups in tools/check_swizzle.py).
#pragma once
#include <type_traits>

#include "tt_common.h"

typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

#ifndef TT_PRIO_HALF  // 1: waves 4-7 of the 8-wave loops run at s_setprio 1 (the second-dispatched half)
#define TT_PRIO_HALF 0
#endif
#ifndef TT_SHIFT_BUF  // 0: the time-shifted operand keeps per-piece pointer DMAs (the round-4 form)
#define TT_SHIFT_BUF 1
#endif

namespace ttg {

constexpr int KTB = 128;  // K-tile bytes per row

// ---- LDS byte offsets --------------------------------------------------------
// KC image: rows of 128 B, 16-B chunk c stored at c ^ ((row>>1)&7).
TT_DEV int kc_off(int row, int c) { return row * KTB + ((c ^ ((row >> 1) & 7)) << 4); }
// KO bf16 image: k-rows of 256 B (128 columns), 16-B chunk c stored at c ^ 2v(k).
TT_DEV int ko_v(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }
TT_DEV int ko16_off(int k, int c) { return k * 256 + ((c ^ (ko_v(k) << 1)) << 4); }
// KO fp32 image: k-rows of 512 B (128 columns), column m stored at m ^ 16*((k>>2)&1).
TT_DEV int ko32_off_chunk(int k, int c) { return k * 512 + ((c ^ (((k >> 2) & 1) << 2)) << 4); }
TT_DEV int ko32_off_elem(int k, int m) { return k * 512 + ((m ^ (((k >> 2) & 1) << 4)) << 2); }

template <typename T, bool KO, int ROWS>
struct Img {
  // bytes of one stage of this operand's image
  static constexpr int BYTES = KO ? (KTB / (int)sizeof(T)) * ROWS * (int)sizeof(T) : ROWS * KTB;
  static constexpr int CHUNKS = BYTES / 16;
  static_assert(!KO || ROWS == 128, "K-outer images are 128 columns wide");
};

// ---- loaders -------------------------------------------------------------------
// A KC loader provides rowptr(r): pointer to element (r, k=0) of tile-row r, or nullptr.
// A KO loader provides at(k, col): pointer to element (k, tile column col), or nullptr,
// and ncols: number of valid tile columns (tail).

// First n (< elements per chunk) elements of a 16-byte chunk, zero-filled: the
// K (or column) tail of an operand whose extent is not a multiple of 16 bytes.
template <typename T>
TT_DEV uint4 load_partial(const T* p, int n) {
  union {
    uint4 v;
    T e[16 / sizeof(T)];
  } u;
  u.v = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int i = 0; i < (int)(16 / sizeof(T)); ++i)
    if (i < n) u.e[i] = p[i];
  return u.v;
}

template <typename T, bool KO, int ROWS, class L>
TT_DEV void stage_load(const L& ld, int kt, int K, uint4 (&r)[Img<T, KO, ROWS>::CHUNKS / 256]) {
  constexpr int N = Img<T, KO, ROWS>::CHUNKS / 256;
  constexpr int EPC = Elt<T>::EPC;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int id = tid + 256 * i;
    uint4 v = make_uint4(0, 0, 0, 0);
    if constexpr (!KO) {
      const int row = id >> 3, c = id & 7;
      const T* p = ld.rowptr(row);
      const int k = kt * (KTB / (int)sizeof(T)) + c * EPC;
      if (p != nullptr && k < K) v = (k + EPC <= K) ? *reinterpret_cast<const uint4*>(p + k) : load_partial(p + k, K - k);
    } else {
      constexpr int CPR = ROWS * (int)sizeof(T) / 16;  // chunks per k-row
      const int kl = id / CPR, c = id % CPR;
      const int k = kt * (KTB / (int)sizeof(T)) + kl;
      const int col = c * EPC;
      const T* p = (k < K && col < ld.ncols) ? ld.at(k, col) : nullptr;
      if (p != nullptr)
        v = (col + EPC <= ld.ncols) ? *reinterpret_cast<const uint4*>(p) : load_partial(p, ld.ncols - col);
    }
    r[i] = v;
  }
}

template <typename T, bool KO, int ROWS>
TT_DEV void stage_store(char* img, const uint4 (&r)[Img<T, KO, ROWS>::CHUNKS / 256]) {
  constexpr int N = Img<T, KO, ROWS>::CHUNKS / 256;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int id = tid + 256 * i;
    int off;
    if constexpr (!KO) {
      off = kc_off(id >> 3, id & 7);
    } else if constexpr (sizeof(T) == 2) {
      off = ko16_off(id >> 4, id & 15);
    } else {
      off = ko32_off_chunk(id >> 5, id & 31);
    }
    *reinterpret_cast<uint4*>(img + off) = r[i];
  }
}

// Fragment of a 16-row (or 16-column) slab starting at tile row r0, sub-step ks.
// Returned as 16 bytes: bf16x8 for bf16, f32x4 for fp32.
template <typename T, bool KO>
TT_DEV uint4 frag(const char* img, int r0, int ks) {
  const int lane = threadIdx.x & 63;
  if constexpr (!KO) {
    const int row = r0 + (lane & 15);
    const int c = (lane >> 4) + 4 * ks;
    return *reinterpret_cast<const uint4*>(img + kc_off(row, c));
  } else if constexpr (sizeof(T) == 2) {
    const int g = lane >> 4, i4 = lane & 15, q = i4 >> 2, p = i4 & 3;
    const int k0 = ks * 32 + 8 * g + q;
    const int cc = (r0 >> 2) + p;  // 8-byte chunk along the row
    const int k1 = k0 + 4;
    const int o0 = ko16_off(k0, cc >> 1) + ((cc & 1) << 3);
    const int o1 = ko16_off(k1, cc >> 1) + ((cc & 1) << 3);
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + o0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + o1));
    uint4 v;
    v.x = (uint32_t)(uint16_t)lo[0] | ((uint32_t)(uint16_t)lo[1] << 16);
    v.y = (uint32_t)(uint16_t)lo[2] | ((uint32_t)(uint16_t)lo[3] << 16);
    v.z = (uint32_t)(uint16_t)hi[0] | ((uint32_t)(uint16_t)hi[1] << 16);
    v.w = (uint32_t)(uint16_t)hi[2] | ((uint32_t)(uint16_t)hi[3] << 16);
    return v;
  } else {
    const int g = lane >> 4;
    const int m = r0 + (lane & 15);
    const int kb = ks * 16 + 4 * g;
    uint4 v;
    v.x = *reinterpret_cast<const uint32_t*>(img + ko32_off_elem(kb + 0, m));
    v.y = *reinterpret_cast<const uint32_t*>(img + ko32_off_elem(kb + 1, m));
    v.z = *reinterpret_cast<const uint32_t*>(img + ko32_off_elem(kb + 2, m));
    v.w = *reinterpret_cast<const uint32_t*>(img + ko32_off_elem(kb + 3, m));
    return v;
  }
}

template <typename T>
TT_DEV f32x4 mma(uint4 a, uint4 b, f32x4 c) {
  if constexpr (sizeof(T) == 2) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8v, a),
                                                   __builtin_bit_cast(bf16x8v, b), c, 0, 0, 0);
  } else {
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), c, 0, 0, 0);
    return c;
  }
}

template <typename T, bool AKO, bool BKO, int BM, int BN>
struct MainLoop {
  using IA = Img<T, AKO, BM>;
  using IB = Img<T, BKO, BN>;
  static constexpr int STAGE = IA::BYTES + IB::BYTES;
  static constexpr int LDS_BYTES = 2 * STAGE;
  static constexpr int TM = BM / 32, TN = BN / 32;  // MFMA tiles per wave (2x2 waves)
  static_assert(IA::CHUNKS % 256 == 0 && IB::CHUNKS % 256 == 0, "tile/thread mismatch");

  // Accumulates K-tiles [kt0, kt1) into acc. Caller zero-initialises acc.
  template <class LA, class LB>
  TT_DEV static void run(const LA& la, const LB& lb, int K, int kt0, int kt1, char* lds,
                         f32x4 (&acc)[TM][TN]) {
    if (kt0 >= kt1) return;
    const int wave = threadIdx.x >> 6;
    const int wm = (wave >> 1) * (BM / 2), wn = (wave & 1) * (BN / 2);
    uint4 ra[IA::CHUNKS / 256], rb[IB::CHUNKS / 256];
    stage_load<T, AKO, BM>(la, kt0, K, ra);
    stage_load<T, BKO, BN>(lb, kt0, K, rb);
    stage_store<T, AKO, BM>(lds, ra);
    stage_store<T, BKO, BN>(lds + IA::BYTES, rb);
    __syncthreads();
    for (int kt = kt0; kt < kt1; ++kt) {
      const int cur = (kt - kt0) & 1;
      const bool more = kt + 1 < kt1;
      if (more) {
        stage_load<T, AKO, BM>(la, kt + 1, K, ra);
        stage_load<T, BKO, BN>(lb, kt + 1, K, rb);
      }
      const char* ia = lds + cur * STAGE;
      const char* ib = ia + IA::BYTES;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        uint4 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = frag<T, AKO>(ia, wm + 16 * i, ks);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = frag<T, BKO>(ib, wn + 16 * j, ks);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mma<T>(fa[i], fb[j], acc[i][j]);
      }
      if (more) {
        char* nx = lds + (cur ^ 1) * STAGE;
        stage_store<T, AKO, BM>(nx, ra);
        stage_store<T, BKO, BN>(nx + IA::BYTES, rb);
      }
      __syncthreads();
    }
  }

  // Visit every accumulator element as (tile_row, tile_col, value).
  template <class F>
  TT_DEV static void epilogue(const f32x4 (&acc)[TM][TN], F&& f) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wm = (wave >> 1) * (BM / 2), wn = (wave & 1) * (BN / 2);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          f(wm + 16 * i + 4 * (lane >> 4) + r, wn + 16 * j + (lane & 15), acc[i][j][r]);
  }
};

// ---- LDS-DMA main loop ----------------------------------------------------------
// Same tile, images and fragment reads as MainLoop, but operands are staged with
// global_load_lds_dwordx4: each wave-instruction writes 1 KiB of LDS linearly
// (lane L -> base + 16 L), so the XOR swizzle is applied to the per-lane SOURCE
// address instead of the LDS destination. Out-of-range chunks read a zero page.
// Requires every 16-byte chunk to be entirely valid or entirely out of range:
// K * sizeof(T) % 16 == 0 for K-contig operands, ncols % (16/sizeof(T)) == 0 for
// K-outer ones. Double-buffered: the DMA of tile k+1 overlaps the MFMAs of tile k.
__device__ __attribute__((weak)) uint4 g_tt_zero_page[64];

typedef __attribute__((address_space(3))) void lds_void;

template <typename T, bool KO, int ROWS, class L>
TT_DEV void stage_dma(const L& ld, int kt, int K, char* img) {
  constexpr int CHUNKS = Img<T, KO, ROWS>::CHUNKS;
  constexpr int EPC = Elt<T>::EPC;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int i = wave; i < CHUNKS / 64; i += 4) {
    const int p = i * 64 + lane;  // image position of this lane's 16 bytes
    const void* src = g_tt_zero_page;
    if constexpr (!KO) {
      const int row = p >> 3;
      const int c = (p & 7) ^ ((row >> 1) & 7);
      const T* rp = ld.rowptr(row);
      const int k = kt * (KTB / (int)sizeof(T)) + c * EPC;
      if (rp != nullptr && k < K) src = rp + k;
    } else {
      constexpr int CPR = ROWS * (int)sizeof(T) / 16;
      const int kl = p / CPR, q = p % CPR;
      int c;
      if constexpr (sizeof(T) == 2) c = q ^ (ko_v(kl) << 1);
      else c = q ^ (((kl >> 2) & 1) << 2);
      const int k = kt * (KTB / (int)sizeof(T)) + kl;
      const T* kp = (k < K && c * EPC < ld.ncols) ? ld.at(k, c * EPC) : nullptr;
      if (kp != nullptr) src = kp;
    }
    __builtin_amdgcn_global_load_lds(src, (lds_void*)(img + i * 1024), 16, 0, 0);
  }
}

template <typename T, bool AKO, bool BKO, int BM, int BN>
struct MainLoopDMA {
  using Base = MainLoop<T, AKO, BKO, BM, BN>;
  using IA = typename Base::IA;
  using IB = typename Base::IB;
  static constexpr int STAGE = Base::STAGE;
  static constexpr int LDS_BYTES = Base::LDS_BYTES;
  static constexpr int TM = Base::TM, TN = Base::TN;

  template <class LA, class LB>
  TT_DEV static void run(const LA& la, const LB& lb, int K, int kt0, int kt1, char* lds, f32x4 (&acc)[TM][TN]) {
    if (kt0 >= kt1) return;
    const int wave = threadIdx.x >> 6;
    const int wm = (wave >> 1) * (BM / 2), wn = (wave & 1) * (BN / 2);
    stage_dma<T, AKO, BM>(la, kt0, K, lds);
    stage_dma<T, BKO, BN>(lb, kt0, K, lds + IA::BYTES);
    for (int kt = kt0; kt < kt1; ++kt) {
      const int cur = (kt - kt0) & 1;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of tile kt landed
      __builtin_amdgcn_s_barrier();                      // ...and every wave's; stage cur^1 is free
      const char* ia = lds + cur * STAGE;
      const char* ib = ia + IA::BYTES;
      // All of tile kt's fragments are read BEFORE the next DMA is issued: hipcc cannot
      // tell the two stages apart and would otherwise wait for that DMA (vmcnt(0))
      // ahead of the first ds_read, serialising the copy and the MFMAs.
      uint4 fa[2][TM], fb[2][TN];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[ks][i] = frag<T, AKO>(ia, wm + 16 * i, ks);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[ks][j] = frag<T, BKO>(ib, wn + 16 * j, ks);
      }
      if (kt + 1 < kt1) {
        char* nx = lds + (cur ^ 1) * STAGE;
        stage_dma<T, AKO, BM>(la, kt + 1, K, nx);
        stage_dma<T, BKO, BN>(lb, kt + 1, K, nx + IA::BYTES);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mma<T>(fa[ks][i], fb[ks][j], acc[i][j]);
    }
    __builtin_amdgcn_s_barrier();  // every wave done reading before the caller reuses LDS
  }
};

// ---- generic LDS-DMA loop (any wave grid; 256-wide tiles) ------------------------
// One LDS-DMA of 16 bytes per lane into LDS byte address lds_addr + 16*lane, issued
// from inline asm so that hipcc neither counts it nor waits for it: the loop below
// places every s_waitcnt vmcnt itself (recipe: cdna_hip_programming.md §5.7).
TT_DEV void dma16(const void* src, uint32_t lds_addr) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds_addr)
               : "memory");
}
TT_DEV uint32_t lds_addr_of(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
// The same 16-byte-per-lane LDS-DMA through a buffer resource: per-lane byte offset voff
// (fixed for a piece), wave-uniform soffset (the K-tile's byte advance, an SGPR), and
// out-of-range offsets (past num_records) read zero. A piece issue is then scalar work
// plus the load -- no per-lane select of the source and no 64-bit address add.
typedef unsigned tt_rsrc4 __attribute__((ext_vector_type(4)));
TT_DEV void dma16_buf(tt_rsrc4 rs, uint32_t voff, uint32_t soff, uint32_t lds_addr) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rs), "s"(soff), "s"(lds_addr)
      : "memory");
}
// raw buffer descriptor: 48-bit base, stride 0, num_records bytes, the flags of tt_rsrc
TT_DEV tt_rsrc4 make_rsrc4(const void* base, uint32_t nrec) {
  const uint64_t b = (uint64_t)(uintptr_t)base;
  tt_rsrc4 r;
  r.x = __builtin_amdgcn_readfirstlane((uint32_t)b);
  r.y = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32) & 0xFFFFu);
  r.z = __builtin_amdgcn_readfirstlane(nrec);
  r.w = 0x00020000u;
  return r;
}

// Image of one K-tile of an operand with ROWS tile rows: K-contig = ROWS x 128 B rows;
// K-outer = ROWS/128 sub-images of [KT k][128 columns] (16 KiB each).
template <typename T, bool KO, int ROWS>
struct Img2 {
  static constexpr int KOSUB = (KTB / (int)sizeof(T)) * 128 * (int)sizeof(T);
  static constexpr int BYTES = KO ? (ROWS / 128) * KOSUB : ROWS * KTB;
  static constexpr int CHUNKS = BYTES / 16;
  static_assert(!KO || ROWS % 128 == 0, "K-outer tiles are multiples of 128 columns");
};

template <typename T, bool KO, int ROWS, int NW, class L>
TT_DEV void stage_dma2(const L& ld, int kt, int K, char* img) {
  using I = Img2<T, KO, ROWS>;
  constexpr int EPC = Elt<T>::EPC;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr_of(img));
#pragma unroll
  for (int i = wave; i < I::CHUNKS / 64; i += NW) {
    const int p = i * 64 + lane;
    const void* src = g_tt_zero_page;
    if constexpr (!KO) {
      const int row = p >> 3;
      const int c = (p & 7) ^ ((row >> 1) & 7);
      const int k = kt * (KTB / (int)sizeof(T)) + c * EPC;
      const T* rp = k < K ? ld.at(row, k) : nullptr;
      if (rp != nullptr) src = rp;
    } else {
      const int sub = p >> 10, pp = p & 1023;
      constexpr int CPR = 128 * (int)sizeof(T) / 16;
      const int kl = pp / CPR, q = pp % CPR;
      int c;
      if constexpr (sizeof(T) == 2) c = q ^ (ko_v(kl) << 1);
      else c = q ^ (((kl >> 2) & 1) << 2);
      const int col = sub * 128 + c * EPC;
      const int k = kt * (KTB / (int)sizeof(T)) + kl;
      const T* kp = (k < K && col < ld.ncols) ? ld.at(k, col) : nullptr;
      if (kp != nullptr) src = kp;
    }
    dma16(src, base + (uint32_t)i * 1024u);
  }
}

template <typename T, bool KO>
TT_DEV uint4 frag2(const char* img, int r0, int ks) {
  if constexpr (!KO) return frag<T, false>(img, r0, ks);
  else return frag<T, true>(img + (r0 >> 7) * Img2<T, true, 128>::KOSUB, r0 & 127, ks);
}

// NS LDS stages: NS = 2 waits for each K-tile's DMAs with vmcnt(0) right before it is read
// (one K-tile in flight during the MFMAs); NS > 2 keeps NS - 1 K-tiles in flight with a
// counted wait (the DMAs of the younger K-tiles), for loops whose K-tile of MFMAs is short
// against the operand's load latency (the fp32 per-step GRU kernels at small batch).
template <typename T, bool AKO, bool BKO, int BM, int BN, int WGM, int WGN, int NS = 2>
struct DLoop {
  static constexpr int NW = WGM * WGN;
  static constexpr int NT = 64 * NW;
  using IA = Img2<T, AKO, BM>;
  using IB = Img2<T, BKO, BN>;
  static constexpr int STAGE = IA::BYTES + IB::BYTES;
  static constexpr int LDS_BYTES = NS * STAGE;
  // this wave's DMAs per K-tile (the fewest over the waves: a wave that issues more waits
  // for some of its younger DMAs too, which is safe)
  static constexpr int DPW = (IA::CHUNKS / 64) / NW + (IB::CHUNKS / 64) / NW;
  static_assert(NS >= 2 && NS <= 4 && (NS - 2) * DPW <= 63, "DLoop stages");
  static constexpr int WTM = BM / WGM, WTN = BN / WGN;  // wave tile
  static constexpr int TM = WTM / 16, TN = WTN / 16;
  static_assert(IA::CHUNKS % 64 == 0 && IB::CHUNKS % 64 == 0, "tile/wave mismatch");

  TT_DEV static int wave_m0() { return (int)(threadIdx.x >> 6) / WGN * WTM; }
  TT_DEV static int wave_n0() { return (int)(threadIdx.x >> 6) % WGN * WTN; }

  // Accumulates K-tiles [kt0, kt1) into acc (caller zeroes it); ends with a barrier.
  template <class LA, class LB>
  TT_DEV static void mma_tile(const char* ia, int wm, int wn, f32x4 (&acc)[TM][TN]) {
    const char* ib = ia + IA::BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = frag2<T, AKO>(ia, wm + 16 * i, ks);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = frag2<T, BKO>(ib, wn + 16 * j, ks);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mma<T>(fa[i], fb[j], acc[i][j]);
    }
  }
  template <class LA, class LB>
  TT_DEV static void run(const LA& la, const LB& lb, int K, int kt0, int kt1, char* lds, f32x4 (&acc)[TM][TN]) {
    if (kt0 >= kt1) return;
    const int wm = wave_m0(), wn = wave_n0();
    if constexpr (NS > 2) {
#pragma unroll
      for (int i = 0; i < NS - 1; ++i)
        if (kt0 + i < kt1) {
          stage_dma2<T, AKO, BM, NW>(la, kt0 + i, K, lds + i * STAGE);
          stage_dma2<T, BKO, BN, NW>(lb, kt0 + i, K, lds + i * STAGE + IA::BYTES);
        }
      int rd = 0, wr = NS - 1;  // slots of K-tile kt and of K-tile kt + NS - 1
      for (int kt = kt0; kt < kt1; ++kt) {
        // K-tiles younger than kt already issued: min(NS - 2, kt1 - 1 - kt)
        const int younger = kt1 - 1 - kt;
        if (younger >= NS - 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * DPW) : "memory");
        else if (NS == 4 && younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DPW) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave's DMAs of kt landed; slot wr was read at kt - 1
        if (kt + NS - 1 < kt1) {
          char* nx = lds + wr * STAGE;
          stage_dma2<T, AKO, BM, NW>(la, kt + NS - 1, K, nx);
          stage_dma2<T, BKO, BN, NW>(lb, kt + NS - 1, K, nx + IA::BYTES);
        }
        mma_tile<LA, LB>(lds + rd * STAGE, wm, wn, acc);
        rd = rd == NS - 1 ? 0 : rd + 1;
        wr = wr == NS - 1 ? 0 : wr + 1;
      }
      __builtin_amdgcn_s_barrier();
      return;
    }
    stage_dma2<T, AKO, BM, NW>(la, kt0, K, lds);
    stage_dma2<T, BKO, BN, NW>(lb, kt0, K, lds + IA::BYTES);
    for (int kt = kt0; kt < kt1; ++kt) {
      const int cur = (kt - kt0) & 1;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of tile kt landed
      __builtin_amdgcn_s_barrier();                      // every wave's; stage cur^1 is free
      if (kt + 1 < kt1) {                                // tile kt+1 flies during tile kt's MFMAs
        char* nx = lds + (cur ^ 1) * STAGE;
        stage_dma2<T, AKO, BM, NW>(la, kt + 1, K, nx);
        stage_dma2<T, BKO, BN, NW>(lb, kt + 1, K, nx + IA::BYTES);
      }
      const char* ia = lds + cur * STAGE;
      const char* ib = ia + IA::BYTES;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        uint4 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = frag2<T, AKO>(ia, wm + 16 * i, ks);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = frag2<T, BKO>(ib, wn + 16 * j, ks);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mma<T>(fa[i], fb[j], acc[i][j]);
      }
    }
    __builtin_amdgcn_s_barrier();
  }
};

// ---- 256x256 8-phase LDS-DMA loop (8 waves as 2M x 4N, wave tile 128 x 64) ----------
// The tile's A and B K-tiles are staged as four 16 KiB half-tiles (A rows 0-127 / 128-255,
// B columns 0-127 / 128-255) into two LDS slots (128 KiB). Each K-tile runs 4 phases, one
// 64x32 accumulator quadrant (16 MFMAs) each, with one half-tile DMA issued per phase:
//   P1: read A(rows 0-63 of the wave) + all B fragments; DMA A0 of K-tile t+1
//   P2: DMA A1 of t+1
//   P3: read A(rows 64-127); DMA B0 of t+2 into the current slot (B last read in P1)
//   P4: DMA B1 of t+2; s_waitcnt vmcnt(4) -> K-tile t+1 has landed
// The two wave rows (wr = 0, 1) run one barrier apart, so one group's fragment reads
// and DMA issue overlap the other group's MFMAs; every restage is >= 2 phases after the
// last read of its half-tile and every read >= 1 barrier after the wait that retired it,
// with the one extra barrier the stagger needs (recipe: cdna_hip_programming.md §5, the
// 256^2 8-phase template: counted vmcnt, raw s_barrier, all LDS in one array). Every wave
// issues 2 DMAs per half-tile, always (a K-tile past the slice end reads the zero page),
// so the counts are exact.
// A3: A gets a 3-slot ring (prefetched two K-tiles ahead, like B) in 160 KiB: A slots at
// 0, 32, 64 KiB, B slots at 96, 128 KiB. A of K-tile r+2 goes into the slot K-tile r-1
// used (both wave rows finished reading it one interval before this K-tile's P1); every
// K-tile then has 8 DMAs per wave in flight at its wait (vmcnt(8)).
// CT: accumulate the transposed product (B fragment as the MFMA's first operand), so that
// acc[i][j][r] is C(16i + (lane & 15), 16j + 4 (lane >> 4) + r): every lane holds 4
// consecutive output columns of one row, which an epilogue stores straight from registers.
template <typename T, bool AKO, bool BKO, bool BAL = false, bool A3 = false, bool CT = false, bool BUF = false>
struct Loop8 {
  static constexpr int HALF = 16384, SLOT = 4 * HALF, LDS_BYTES = A3 ? 10 * HALF : 2 * SLOT;
  static constexpr int BOFF = 6 * HALF;  // A3: first B slot
  static constexpr int TM = 8, TN = 4;
  static constexpr int KTE = KTB / (int)sizeof(T);  // K elements per K-tile

  // One thread's two 1 KiB pieces of a half-tile, resolved once per tile: the source
  // address at K-tile kt0 plus the number of K-tiles for which the piece is in range
  // (K tail, M/N tail and slice end folded together), so a DMA issue costs a 64-bit add,
  // a compare and a select instead of re-deriving the row/column address every K-tile.
  struct Piece {
    const char* p;  // source at K-tile kt0 (any valid address when lim == 0)
    int lim;        // in range for relative K-tiles [0, lim)
    int t0;         // KOShift: time index of the piece's k-row at kt0
  };
  template <bool KO, class L>
  TT_DEV static void init_half(const L& ld, int kt0, int ktl, int K, int roff, Piece (&pc)[2]) {
    constexpr int EPC = Elt<T>::EPC;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int p = (wave + 8 * j) * 64 + lane;
      pc[j].p = reinterpret_cast<const char*>(g_tt_zero_page);
      pc[j].lim = 0;
      pc[j].t0 = 0;
      if constexpr (!KO) {
        const int row = p >> 3;
        const int c = (p & 7) ^ ((row >> 1) & 7);
        const T* rp = ld.rowptr(roff + row);
        const int k0 = kt0 * KTE + c * EPC;
        if (rp != nullptr) {
          pc[j].p = reinterpret_cast<const char*>(rp + k0);
          pc[j].lim = min(ktl - kt0, (K - k0 + KTE - 1) / KTE);
        }
      } else {
        constexpr int CPR = 128 * (int)sizeof(T) / 16;
        const int kl = p / CPR, q = p % CPR;
        int c;
        if constexpr (sizeof(T) == 2) c = q ^ (ko_v(kl) << 1);
        else c = q ^ (((kl >> 2) & 1) << 2);
        const int col = roff + c * EPC;
        const int k0 = kt0 * KTE + kl;
        if (col < ld.ncols && k0 < K) {
          pc[j].p = reinterpret_cast<const char*>(ld.raw_at(k0, col));
          pc[j].lim = min(ktl - kt0, (K - k0 + KTE - 1) / KTE);
          if constexpr (L::SHIFTED) pc[j].t0 = k0 % ld.T_;
        }
      }
    }
  }
  // DMA relative K-tile r of a half-tile (delta = bytes between consecutive K-tiles).
  template <class L>
  TT_DEV static void issue_half(const L& ld, const Piece (&pc)[2], int r, long delta, uint32_t img) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#if defined(TT_L8_DIAG) && TT_L8_DIAG == 1  // timing only (results wrong): no DMA in the loop
    if (r > 1) return;
#elif defined(TT_L8_DIAG) && TT_L8_DIAG == 2  // timing only: every K-tile re-reads the piece's first address
    for (int j = 0; j < 2; ++j) dma16(pc[j].p, img + (uint32_t)(wave + 8 * j) * 1024u);
    return;
#endif
    int dt = 0;
    if constexpr (L::SHIFTED) {  // time advance of K-tile r: 32-bit, a mask when T is a power of two
      const unsigned rk = (unsigned)r * (unsigned)KTE, tu = (unsigned)ld.T_;
      dt = (int)((tu & (tu - 1u)) == 0u ? rk & (tu - 1u) : rk % tu);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bool ok = r < pc[j].lim;
      long off = (long)r * delta;
      if constexpr (L::SHIFTED) {
        int t = pc[j].t0 + dt;
        t -= t >= ld.T_ ? ld.T_ : 0;
        const int ts = t + ld.shift;
        ok = ok && ts >= 0 && ts < ld.T_;
        off += (long)ld.shift * ld.ld * (long)sizeof(T);
      }
      if constexpr (L::KSPLIT) {  // K-tiles past the split continue in the second base
        const int skt = ld.ksplit / KTE;
        if (r >= skt) off += (long)(ld.base1 - ld.base0) * (long)sizeof(T) - (long)skt * KTB;
      }
      const char* src = ok ? pc[j].p + off : reinterpret_cast<const char*>(g_tt_zero_page);
      dma16(src, img + (uint32_t)(wave + 8 * j) * 1024u);
    }
  }
  // BUF: the half-tile's two pieces through a buffer resource (dma16_buf): the resource
  // and the per-K-tile byte advance are wave-uniform, each lane keeps one 32-bit offset
  // per piece. Rows of a K-contig operand past its end and K-rows of a K-outer one past K
  // read zero through num_records; columns past a K-outer operand's end and K-tiles past a
  // split's end read whatever lies there, which only reaches output rows / columns that
  // are never stored, or K-tiles that are never consumed. Needs K % KTE == 0 and the
  // operand's byte range from the half's first K-tile below 2^32 (the host checks both).
  struct BufHalf {
    tt_rsrc4 rs;
    uint32_t delta;
    uint32_t voff[2];
  };
  template <bool KO, class L>
  TT_DEV static void init_buf(const L& ld, int kt0, int K, int roff, BufHalf& h) {
    constexpr int EPC = Elt<T>::EPC;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if constexpr (!KO) {
      const long r0 = (long)ld.r0 + roff;
      const long rows = (long)ld.rows - r0;
      long nrec = rows > 0 ? rows * ld.ld * (long)sizeof(T) - (long)kt0 * KTB : 0;
      nrec = nrec < 0 ? 0 : (nrec > 0xFFFFFFFFL ? 0xFFFFFFFFL : nrec);
      h.rs = make_rsrc4(ld.base + r0 * ld.ld + (long)kt0 * KTE, (uint32_t)nrec);
      h.delta = KTB;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int p = (wave + 8 * j) * 64 + lane;
        const int row = p >> 3, c = (p & 7) ^ ((row >> 1) & 7);
        h.voff[j] = (uint32_t)(((long)row * ld.ld + c * EPC) * (long)sizeof(T));
      }
    } else {
      const long k0 = (long)kt0 * KTE;
      long nrec = K > k0 ? ((long)K - k0) * ld.ld * (long)sizeof(T) : 0;
      nrec = nrec > 0xFFFFFFFFL ? 0xFFFFFFFFL : nrec;
      h.rs = make_rsrc4(ld.base + k0 * ld.ld, (uint32_t)nrec);
      h.delta = (uint32_t)((long)KTE * ld.ld * (long)sizeof(T));
      constexpr int CPR = 128 * (int)sizeof(T) / 16;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int p = (wave + 8 * j) * 64 + lane;
        const int kl = p / CPR, q = p % CPR;
        int c;
        if constexpr (sizeof(T) == 2) c = q ^ (ko_v(kl) << 1);
        else c = q ^ (((kl >> 2) & 1) << 2);
        h.voff[j] = (uint32_t)(((long)kl * ld.ld + ld.col_off(roff + c * EPC)) * (long)sizeof(T));
      }
    }
  }
  TT_DEV static void issue_buf(const BufHalf& h, int r, uint32_t img) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)r * h.delta);
#pragma unroll
    for (int j = 0; j < 2; ++j) dma16_buf(h.rs, h.voff[j], soff, img + (uint32_t)(wave + 8 * j) * 1024u);
  }
  // One half-tile source: Piece form (any loader) or buffer form (BUF, plain loaders).
  template <bool KO, class L>
  struct PHalf {
    L ld;
    Piece pc[2];
    long delta;
    TT_DEV void init(const L& l, int kt0, int ktl, int K, int roff) {
      ld = l;
      init_half<KO>(l, kt0, ktl, K, roff, pc);
      delta = KO ? (long)KTE * l.ld * (long)sizeof(T) : (long)KTB;
    }
    TT_DEV void issue(int r, uint32_t img) const { issue_half(ld, pc, r, delta, img); }
    TT_DEV void fix(int, uint32_t) const {}
  };
  template <bool KO, class L>
  struct BHalf {
    BufHalf h;
    TT_DEV void init(const L& l, int kt0, int ktl, int K, int roff) { init_buf<KO>(l, kt0, K, roff, h); }
    TT_DEV void issue(int r, uint32_t img) const { issue_buf(h, r, img); }
    TT_DEV void fix(int, uint32_t) const {}
  };
  // BUF form of the time-shifted K-outer operand (KOShift, dW_hh's h_{s-1}) for T a
  // multiple of the K-tile depth: every piece reads the K-tile's own k-rows moved by
  // `shift` rows, so the pieces keep fixed per-lane offsets and the K-tile advance stays an
  // SGPR (no per-piece time arithmetic or source select). The one k-row per masked K-tile
  // whose time index t has t + shift outside [0, T) (k-row 0 for shift -1 when t = 0,
  // k-row KTE-1 for shift +1 when t = T-1) then holds a neighbouring sequence's row; the
  // lanes that DMA'd it overwrite it with zeros in LDS after the wait that retires the
  // K-tile (fix), before the barrier that precedes its first fragment read. Every lane
  // stays in range (out-of-range lanes slow the whole DMA instruction down: DESIGN.md §3)
  // except the operand's very last K-tile under shift +1, whose row K reads zero through
  // num_records. Shift -1 at the operand's first K-tile would read row -1: that K-tile's
  // masked lanes read row 0 instead (voff0), which fix zeroes as well.
  template <bool KO, class L>
  struct SHalf {
    BufHalf h;
    uint32_t voff0[2];  // relative K-tile 0
    int kt0, tkt;       // first K-tile, K-tiles per sequence
    int klm;            // masked k-row: 0 (shift -1) or KTE-1 (shift +1)
    bool zl[2];         // this lane DMA'd the masked k-row in piece j
    bool zany;          // ... in either piece, for some lane of this wave (wave-uniform)
    TT_DEV void init(const L& l, int kt0_, int ktl, int K, int roff) {
      static_assert(KO, "time-shifted operands are K-outer");
      const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
      kt0 = kt0_;
      tkt = l.T_ / KTE;
      klm = l.shift < 0 ? 0 : KTE - 1;
      const long k0 = (long)kt0 * KTE;
      long nrec = ((long)K - k0 - l.shift) * l.ld * (long)sizeof(T);
      nrec = nrec < 0 ? 0 : (nrec > 0xFFFFFFFFL ? 0xFFFFFFFFL : nrec);
      h.rs = make_rsrc4(l.base + (k0 + l.shift) * l.ld, (uint32_t)nrec);
      h.delta = (uint32_t)((long)KTE * l.ld * (long)sizeof(T));
      constexpr int CPR = 128 * (int)sizeof(T) / 16;
      bool any = false;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int p = (wave + 8 * j) * 64 + lane;
        const int kl = p / CPR, q = p % CPR;
        int c;
        if constexpr (sizeof(T) == 2) c = q ^ (ko_v(kl) << 1);
        else c = q ^ (((kl >> 2) & 1) << 2);
        const long col = (long)l.c0 + roff + c * Elt<T>::EPC;
        h.voff[j] = (uint32_t)(((long)kl * l.ld + col) * (long)sizeof(T));
        zl[j] = kl == klm;
        any |= zl[j];
        // shift -1 from the operand's first K-tile: k-row 0 would be row -1
        voff0[j] = (zl[j] && kt0 == 0 && l.shift < 0) ? (uint32_t)((l.ld + col) * (long)sizeof(T)) : h.voff[j];
      }
      zany = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_ballot_w64(any) != 0 ? 1 : 0) != 0;
    }
    TT_DEV void issue(int r, uint32_t img) const {
      const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
      const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)r * h.delta);
#pragma unroll
      for (int j = 0; j < 2; ++j) dma16_buf(h.rs, r == 0 ? voff0[j] : h.voff[j], soff, img + (uint32_t)(wave + 8 * j) * 1024u);
    }
    // after this wave's wait that retired relative K-tile r (image img): zero the masked
    // k-row if K-tile r has one; ordered before the next barrier by lgkmcnt(0)
    TT_DEV void fix(int r, uint32_t img) const {
      const int kt = kt0 + r;
      const bool masked = (klm == 0 ? kt : kt + 1) % tkt == 0;
      if (!zany || !masked) return;
      const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if (zl[j]) {
          const uint32_t a = img + (uint32_t)(wave + 8 * j) * 1024u + (uint32_t)lane * 16u;
          const tt_rsrc4 z = {0u, 0u, 0u, 0u};
          asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(z) : "memory");
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  };
  template <bool KO, class L>
  using Half = std::conditional_t<BUF && !L::KSPLIT && (!L::SHIFTED || TT_SHIFT_BUF),
                                  std::conditional_t<L::SHIFTED, SHalf<KO, L>, BHalf<KO, L>>, PHalf<KO, L>>;

  // mm (wave-uniform): false for a wave whose 128 tile rows all lie past M (the second wave
  // row of a tail tile with <= 128 rows): it keeps its DMA share and barriers, skips its MFMAs
  TT_DEV static void quad(int mi, int ni, const uint4 (&fa)[2][4], const uint4 (&fb)[2][4], f32x4 (&acc)[TM][TN],
                          bool mm = true) {
    __builtin_amdgcn_s_barrier();
    if (mm) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[4 * mi + i][2 * ni + j] = CT ? mma<T>(fb[ks][2 * ni + j], fa[ks][i], acc[4 * mi + i][2 * ni + j])
                                             : mma<T>(fa[ks][i], fb[ks][2 * ni + j], acc[4 * mi + i][2 * ni + j]);
      __builtin_amdgcn_s_setprio(0);
    }
    __builtin_amdgcn_s_barrier();
  }

  template <class LA, class LB>
  TT_DEV static void run(const LA& la, const LB& lb, int K, int kt0, int kt1, char* lds, f32x4 (&acc)[TM][TN],
                         bool mm = true) {
    if (kt0 >= kt1) return;
    const int wave = threadIdx.x >> 6;
    const int wr = wave >> 2, bh = (wave & 3) >> 1, bc = (wave & 1) * 64;
    const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr_of(lds));
    Half<AKO, LA> pa0, pa1;
    Half<BKO, LB> pb0, pb1;
    pa0.init(la, kt0, kt1, K, 0);
    pa1.init(la, kt0, kt1, K, 128);
    pb0.init(lb, kt0, kt1, K, 0);
    pb1.init(lb, kt0, kt1, K, 128);
    if constexpr (A3) {
      if (mm) run3<true>(kt1 - kt0, lds, base, pa0, pa1, pb0, pb1, acc);
      else run3<false>(kt1 - kt0, lds, base, pa0, pa1, pb0, pb1, acc);
      return;
    }
    pa0.issue(0, base);
    pa1.issue(0, base + HALF);
    pb0.issue(0, base + 2 * HALF);
    pb1.issue(0, base + 3 * HALF);
    pb0.issue(1, base + SLOT + 2 * HALF);
    pb1.issue(1, base + SLOT + 3 * HALF);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    pb0.fix(0, base + 2 * HALF);
    pb1.fix(0, base + 3 * HALF);
    __builtin_amdgcn_s_barrier();
    const bool late = __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256;  // wave row 1
    if (TT_PRIO_HALF && late) __builtin_amdgcn_s_setprio(1);
    if (late) __builtin_amdgcn_s_barrier();
    uint4 fa[2][4], fb[2][4];
    for (int r = 0; r < kt1 - kt0; ++r) {
      const int cs = r & 1;
      const uint32_t cur = base + cs * SLOT, nxt = base + (cs ^ 1) * SLOT;
      const char* ia = lds + cs * SLOT + wr * HALF;
      const char* ib = lds + cs * SLOT + (2 + bh) * HALF;
      if constexpr (BAL) {
        // balanced reads: P1 A rows 0-63 + B columns 0-31 (12 reads), P2 B columns 32-63
        // (4), P3 A rows 64-127 (8); B is last read in P2, so both B halves of K-tile
        // r+2 are restaged in P4 (two phases later)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
          for (int i = 0; i < 4; ++i) fa[ks][i] = frag2<T, AKO>(ia, 16 * i, ks);
#pragma unroll
          for (int j = 0; j < 2; ++j) fb[ks][j] = frag2<T, BKO>(ib, bc + 16 * j, ks);
        }
        pa0.issue(r + 1, nxt);
        quad(0, 0, fa, fb, acc);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int j = 2; j < 4; ++j) fb[ks][j] = frag2<T, BKO>(ib, bc + 16 * j, ks);
        pa1.issue(r + 1, nxt + HALF);
        quad(0, 1, fa, fb, acc);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < 4; ++i) fa[ks][i] = frag2<T, AKO>(ia, 64 + 16 * i, ks);
        quad(1, 1, fa, fb, acc);
        pb0.issue(r + 2, cur + 2 * HALF);
        pb1.issue(r + 2, cur + 3 * HALF);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        pb0.fix(r + 1, nxt + 2 * HALF);
        pb1.fix(r + 1, nxt + 3 * HALF);
        quad(1, 0, fa, fb, acc);
        continue;
      }
      // P1
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[ks][i] = frag2<T, AKO>(ia, 16 * i, ks);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[ks][j] = frag2<T, BKO>(ib, bc + 16 * j, ks);
      }
      pa0.issue(r + 1, nxt);
      quad(0, 0, fa, fb, acc);
      // P2
      pa1.issue(r + 1, nxt + HALF);
      quad(0, 1, fa, fb, acc);
      // P3
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[ks][i] = frag2<T, AKO>(ia, 64 + 16 * i, ks);
      pb0.issue(r + 2, cur + 2 * HALF);
      quad(1, 1, fa, fb, acc);
      // P4
      pb1.issue(r + 2, cur + 3 * HALF);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      pb0.fix(r + 1, nxt + 2 * HALF);
      pb1.fix(r + 1, nxt + 3 * HALF);
      quad(1, 0, fa, fb, acc);
    }
    if (!late) __builtin_amdgcn_s_barrier();  // re-align the two wave rows
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // trailing zero-page DMAs before LDS reuse
    __builtin_amdgcn_s_barrier();
  }

  // The A3 schedule (balanced reads as BAL): per K-tile r, P1 reads A rows 0-63 + B
  // columns 0-31 and restages A0 of r+2, P2 reads B columns 32-63 and restages A1 of r+2,
  // P3 reads A rows 64-127, P4 restages both B halves of r+2 into B's current slot and
  // waits for K-tile r+1 with the 8 youngest DMAs (A and B of r+2) still in flight.
  template <bool MM, class HA, class HB>
  TT_DEV static void run3(int nk, char* lds, uint32_t base, const HA& pa0, const HA& pa1, const HB& pb0, const HB& pb1,
                          f32x4 (&acc)[TM][TN]) {
    const int wave = threadIdx.x >> 6;
    const int wr = wave >> 2, bh = (wave & 3) >> 1, bc = (wave & 1) * 64;
    pa0.issue(0, base);
    pa1.issue(0, base + HALF);
    pb0.issue(0, base + BOFF);
    pb1.issue(0, base + BOFF + HALF);
    pa0.issue(1, base + 2 * HALF);
    pa1.issue(1, base + 3 * HALF);
    pb0.issue(1, base + BOFF + 2 * HALF);
    pb1.issue(1, base + BOFF + 3 * HALF);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    pb0.fix(0, base + BOFF);
    pb1.fix(0, base + BOFF + HALF);
    __builtin_amdgcn_s_barrier();
    const bool late = __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256;  // wave row 1
    if (TT_PRIO_HALF && late) __builtin_amdgcn_s_setprio(1);
    if (late) __builtin_amdgcn_s_barrier();
    uint4 fa[2][4], fb[2][4];
    int as = 0;  // A slot of K-tile r (r mod 3)
    for (int r = 0; r < nk; ++r) {
      const int an = as == 0 ? 2 : as - 1;  // slot of K-tile r+2 = slot of r-1
      const int bs = r & 1;
      const char* ia = lds + as * (2 * HALF) + wr * HALF;
      const char* ib = lds + BOFF + bs * (2 * HALF) + bh * HALF;
      const uint32_t anx = base + (uint32_t)an * (2 * HALF), bcur = base + BOFF + (uint32_t)bs * (2 * HALF);
      if constexpr (MM) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
          for (int i = 0; i < 4; ++i) fa[ks][i] = frag2<T, AKO>(ia, 16 * i, ks);
#pragma unroll
          for (int j = 0; j < 2; ++j) fb[ks][j] = frag2<T, BKO>(ib, bc + 16 * j, ks);
        }
      }
      pa0.issue(r + 2, anx);
      quad(0, 0, fa, fb, acc, MM);
      if constexpr (MM) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int j = 2; j < 4; ++j) fb[ks][j] = frag2<T, BKO>(ib, bc + 16 * j, ks);
      }
      pa1.issue(r + 2, anx + HALF);
      quad(0, 1, fa, fb, acc, MM);
      if constexpr (MM) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < 4; ++i) fa[ks][i] = frag2<T, AKO>(ia, 64 + 16 * i, ks);
      }
      quad(1, 1, fa, fb, acc, MM);
      pb0.issue(r + 2, bcur);
      pb1.issue(r + 2, bcur + HALF);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      {  // K-tile r+1 (B slot (r+1) & 1) has landed for this wave's DMAs
        const uint32_t bnx = base + BOFF + (uint32_t)(bs ^ 1) * (2 * HALF);
        pb0.fix(r + 1, bnx);
        pb1.fix(r + 1, bnx + HALF);
      }
      quad(1, 0, fa, fb, acc, MM);
      as = as == 2 ? 0 : as + 1;
    }
    if (!late) __builtin_amdgcn_s_barrier();  // re-align the two wave rows
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // trailing zero-page DMAs before LDS reuse
    __builtin_amdgcn_s_barrier();
  }
};

// XCD-aware 1-D workgroup order: ids are dealt round-robin over the 8 XCDs, so remap
// them (bijectively) to give every XCD a contiguous run; callers enumerate tiles with the
// fastest index being the one whose tiles share an operand panel.
TT_DEV int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, loc = bid >> 3;
  const int q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// ---- common loaders ------------------------------------------------------------
// K-contig loaders: rowptr(r) = row r of the tile at k = 0 (or nullptr past the end);
// at(r, k) = element (r, k) (or nullptr). K-outer loaders: at(k, col) = element (k, tile
// column col) (or nullptr), raw_at = the same ignoring any row shift.
template <typename T>
struct KCPlain {  // rows [r0, r0+ROWS) of a row-major [rows][ld] matrix
  static constexpr bool SHIFTED = false, KSPLIT = false;
  const T* base; long ld; int r0, rows;
  TT_DEV const T* rowptr(int r) const { int g = r0 + r; return g < rows ? base + (long)g * ld : nullptr; }
  TT_DEV const T* at(int r, int k) const { const T* p = rowptr(r); return p ? p + k : nullptr; }
};
// K-contig operand whose columns [0, ksplit) come from base0 and [ksplit, K) from base1
// (same rows and ld): the GRU dL/dgh operand, whose r|z columns are shared with dL/dgx.
template <typename T>
struct KCSplit {  // ksplit: a multiple of the K-tile for the 8-phase loop
  static constexpr bool SHIFTED = false, KSPLIT = true;
  const T* base0; const T* base1; long ld; int r0, rows, ksplit;
  TT_DEV const T* rowptr(int r) const { int g = r0 + r; return g < rows ? base0 + (long)g * ld : nullptr; }
  TT_DEV const T* at(int r, int k) const {
    const int g = r0 + r;
    if (g >= rows) return nullptr;
    return k < ksplit ? base0 + (long)g * ld + k : base1 + (long)g * ld + (k - ksplit);
  }
};
template <typename T>
struct KOPlain {  // columns [c0, c0+128) of a row-major [K][ld] matrix
  static constexpr bool SHIFTED = false, KSPLIT = false;
  const T* base; long ld; int c0, ncols;
  const T* base1 = nullptr;  // columns >= csplit (absolute) come from base1 + (col - csplit)
  int csplit = 0x7fffffff;
  TT_DEV const T* raw_at(long k, int col) const {
    const int gc = c0 + col;
    return gc < csplit ? base + k * ld + gc : base1 + k * ld + (gc - csplit);
  }
  TT_DEV const T* at(long k, int col) const { return raw_at(k, col); }
  // element offset of tile column col from base (k = 0): the buffer form of raw_at; base1
  // must lie in the same rows (same ld) at or after base
  TT_DEV long col_off(int col) const {
    const int gc = c0 + col;
    return gc < csplit ? (long)gc : (long)(base1 - base) + (gc - csplit);
  }
};
// K-outer operand whose k index is (b*T + t) and whose source row is (b*T + t + shift),
// zero when t+shift falls outside [0,T). Used for the GRU h_{s-1} operand of dW_hh.
template <typename T>
struct KOShift {
  static constexpr bool SHIFTED = true, KSPLIT = false;
  const T* base; long ld; int c0, ncols, T_, shift;
  TT_DEV const T* raw_at(long k, int col) const { return base + k * ld + c0 + col; }
  TT_DEV const T* at(long k, int col) const {
    const int t = (int)(k % T_);
    const int ts = t + shift;
    if (ts < 0 || ts >= T_) return nullptr;
    return base + (k + shift) * ld + c0 + col;
  }
};

}  // namespace ttg
