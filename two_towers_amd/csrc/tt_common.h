// Shared device helpers for the two-tower HIP path (gfx950 / CDNA4 only).
//
// Element types: the path runs in one of two arithmetic types, chosen per call:
//   TT_F32  = 0 : fp32 storage, exact-f32 MFMA (v_mfma_f32_16x16x4_f32)
//   TT_BF16 = 1 : bf16 storage, v_mfma_f32_16x16x32_bf16, fp32 accumulation
// bf16 values travel as raw uint16_t bits so no HIP bf16 class is needed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define TT_F32 0
#define TT_BF16 1

typedef uint16_t bf16_t;
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define TT_DEV __device__ __forceinline__

TT_DEV float bf2f(bf16_t b) { return __uint_as_float(((uint32_t)b) << 16); }
// Round-to-nearest-even; lowers to v_cvt_pk_bf16_f32 (keeps NaN a NaN).
TT_DEV bf16_t f2bf(float f) { __bf16 h = (__bf16)f; return __builtin_bit_cast(bf16_t, h); }

template <typename T> struct Elt;
template <> struct Elt<float> {
  static constexpr int EPC = 4;  // elements per 16-byte chunk
  TT_DEV static float ld(const float* p) { return *p; }
  TT_DEV static void st(float* p, float v) { *p = v; }
  TT_DEV static float cvt(float v) { return v; }
};
template <> struct Elt<bf16_t> {
  static constexpr int EPC = 8;
  TT_DEV static float ld(const bf16_t* p) { return bf2f(*p); }
  TT_DEV static void st(bf16_t* p, float v) { *p = f2bf(v); }
  TT_DEV static bf16_t cvt(float v) { return f2bf(v); }
};

// 8 consecutive elements <-> fp32 registers, one or two 16-byte accesses.
TT_DEV void ld8(const float* p, float (&f)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
TT_DEV void ld8(const bf16_t* p, float (&f)[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
  }
}
TT_DEV void st8(float* p, const float (&f)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(f[4], f[5], f[6], f[7]);
}
TT_DEV void st8(bf16_t* p, const float (&f)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}

// Streaming stores: buffer_store_dwordx4 ... sc1 writes through and DROPS the line from
// the XCD's L2 (MI355X_MICROARCH.md, store flavours), so multi-GB output streams do not
// evict the operands that the other workgroups of the XCD are still re-reading.
// The descriptor base must be wave-uniform; byte offsets are per lane (< 2 GiB).
typedef unsigned tt_u32x4 __attribute__((vector_size(16)));
TT_DEV __amdgpu_buffer_rsrc_t tt_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
TT_DEV uint4 pack8bf(const float (&f)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
  return make_uint4(w[0], w[1], w[2], w[3]);
}
// 16-byte buffer store (default cache policy); an offset past num_records is dropped.
// The soffset field is always the constant 0 and `soff` is folded into the per-lane
// offset: a wide (> 8-byte) buffer store whose soffset is an SGPR gets no hazard
// protection from the compiler (LLVM's GCNHazardRecognizer exempts that form), and
// on gfx950 a VALU write of the data VGPRs right after such a store replaced part of
// the stored data — the round-2 saved-gh_n corruption (DESIGN.md §3;
// tools/check_store_hazard.py checks the built library for the form).
TT_DEV void st16_buf(__amdgpu_buffer_rsrc_t r, uint32_t voff, int soff, uint4 v) {
  tt_u32x4 w = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(w, r, (int)(voff + (uint32_t)soff), 0, 0);
}
TT_DEV void st16_buf_sc1(__amdgpu_buffer_rsrc_t r, uint32_t voff, int soff, uint4 v) {
  tt_u32x4 w = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(w, r, (int)(voff + (uint32_t)soff), 0, 16);
}
// Buffer resource of num_records 0x7fffffff bytes, or 0 (every load reads zero) if !on.
TT_DEV __amdgpu_buffer_rsrc_t tt_rsrc_n(const void* base, bool on) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, on ? 0x7fffffff : 0, 0x00020000);
}
// 16-byte buffer load; an offset past num_records returns zeros.
template <int AUX = 0>
TT_DEV uint4 ld16_buf(__amdgpu_buffer_rsrc_t r, uint32_t voff, int soff) {
  const tt_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, soff, AUX);
  return make_uint4(v[0], v[1], v[2], v[3]);
}
template <int AUX>
TT_DEV void st16_buf_aux(__amdgpu_buffer_rsrc_t r, int off, uint4 v) {  // 2 nt, 17 sc0 sc1
  tt_u32x4 w = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(w, r, off, 0, AUX);
}
TT_DEV void st16_sc1(__amdgpu_buffer_rsrc_t r, int off, uint4 v) {
  tt_u32x4 w = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(w, r, off, 0, 16);
}
TT_DEV void st8_sc1(__amdgpu_buffer_rsrc_t r, int off, const float (&f)[8], float*) {
  st16_sc1(r, off, make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3])));
  st16_sc1(r, off + 16, make_uint4(__float_as_uint(f[4]), __float_as_uint(f[5]), __float_as_uint(f[6]), __float_as_uint(f[7])));
}
TT_DEV void st8_sc1(__amdgpu_buffer_rsrc_t r, int off, const float (&f)[8], bf16_t*) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
  st16_sc1(r, off, make_uint4(w[0], w[1], w[2], w[3]));
}

// Full-line epilogue stores from a transposed-accumulate 16x16 tile pair. After the
// column-pair v_permlane16_swap, lane l holds two 16-byte chunks of its row (l & 15): v0 =
// 8 columns c.. of the pair's first 32 columns, v1 = the same 8 columns + 32; one store
// instruction of them writes 16 rows x 64 B (16 half lines). row_pair exchanges v1 of rows
// 0-7 with v0 of rows 8-15 (lane l <-> l ^ 8, one v_mov_dpp row_ror:8 per dword), so that
// store `da` writes rows 0-7 whole (8 lanes x 16 B = 128 B per row) and `db` rows 8-15:
// lane l stores da at row (l & 7), db at row (l & 7) + 8, both at column c + (l & 8 ? 32 : 0).
TT_DEV uint32_t dpp_ror8(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x128 /* row_ror:8 */, 0xF, 0xF, false);
}
TT_DEV void row_pair(const uint4& v0, const uint4& v1, uint4& da, uint4& db) {
  const bool lo = (threadIdx.x & 8) == 0;
  uint4 s = lo ? v1 : v0, r;
  r.x = dpp_ror8(s.x);
  r.y = dpp_ror8(s.y);
  r.z = dpp_ror8(s.z);
  r.w = dpp_ror8(s.w);
  da = lo ? v0 : r;
  db = lo ? r : v1;
}

// 8 elements held raw (16 B bf16 / 32 B fp32) so loads can be issued long before use.
template <typename T>
struct Raw8 {
  uint4 a, b;
  TT_DEV void load(const T* p) {
    a = *reinterpret_cast<const uint4*>(p);
    if constexpr (sizeof(T) == 4) b = *reinterpret_cast<const uint4*>(p + 4);
  }
  TT_DEV void zero() { a = b = make_uint4(0, 0, 0, 0); }
  TT_DEV void get(float (&f)[8]) const {
    if constexpr (sizeof(T) == 4) {
      f[0] = __uint_as_float(a.x); f[1] = __uint_as_float(a.y); f[2] = __uint_as_float(a.z); f[3] = __uint_as_float(a.w);
      f[4] = __uint_as_float(b.x); f[5] = __uint_as_float(b.y); f[6] = __uint_as_float(b.z); f[7] = __uint_as_float(b.w);
    } else {
      const uint32_t w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        f[2 * i] = __uint_as_float(w[i] << 16);
        f[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
      }
    }
  }
};

// v_rcp_f32 (1 ulp): a plain 1.0f / x compiles to the ~11-instruction IEEE division
// sequence, which dominated the GRU epilogues' VALU time.
TT_DEV float tt_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
TT_DEV float tt_sigmoid(float x) { return tt_rcp(1.0f + __expf(-x)); }
TT_DEV float tt_tanh(float x) {
  // tanh(x) = 1 - 2/(exp(2x)+1); saturates cleanly for large |x|.
  float e = __expf(2.0f * x);
  return 1.0f - 2.0f * tt_rcp(e + 1.0f);
}

// 1 - tanh(x)^2 without cancellation: 4 e^{-2|x|} / (1 + e^{-2|x|})^2.
TT_DEV float tt_sech2(float x) {
  const float e = __expf(-2.0f * fabsf(x));
  const float r = tt_rcp(1.0f + e);
  return 4.0f * e * r * r;
}

// sigma(x) and sigma(-x) = 1 - sigma(x) from one exp and one reciprocal, without the
// cancellation of 1 - sigma(x) and without overflow: E = e^{-|x|} in (0, 1].
TT_DEV void tt_sigmoid_pair(float x, float& s, float& sm) {
  const float e = __expf(-fabsf(x));
  const float p = tt_rcp(1.0f + e);  // sigma(|x|)
  const float q = e * p;                 // sigma(-|x|)
  s = x >= 0.f ? p : q;
  sm = x >= 0.f ? q : p;
}
// tanh(x) and 1 - tanh(x)^2 from one exp and one reciprocal (E = e^{-2|x|}).
TT_DEV void tt_tanh_sech2(float x, float& th, float& sech2) {
  const float e = __expf(-2.0f * fabsf(x));
  const float r = tt_rcp(1.0f + e);
  const float t = (1.0f - e) * r;
  th = x >= 0.f ? t : -t;
  sech2 = 4.0f * e * r * r;
}

// Counter-based dropout mask shared by the forward (GRU layer-0 output) and
// backward (input-projection gradient) kernels, and restated in oracle/.
// keep(seed, row, col) with row = b*T + t, col in [0, 2H).
TT_DEV uint32_t tt_hash3(uint32_t seed, uint32_t row, uint32_t col) {
  uint32_t h = seed * 0x9E3779B1u ^ (row * 0x85EBCA77u) ^ (col * 0xC2B2AE3Du + 0x27D4EB2Fu);
  h ^= h >> 16; h *= 0x7FEB352Du; h ^= h >> 15; h *= 0x846CA68Bu; h ^= h >> 16;
  return h;
}
// Returns the multiplier (0 or 1/(1-p)); threshold = p * 2^24.
TT_DEV float tt_dropout_scale(uint32_t seed, uint32_t row, uint32_t col, uint32_t thresh, float inv_keep) {
  return ((tt_hash3(seed, row, col) >> 8) < thresh) ? 0.0f : inv_keep;
}

TT_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
TT_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// Reduce over the 16 lanes that share (lane>>4) — one MFMA C-tile row group.
TT_DEV float sum16(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
TT_DEV float max16(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
