// HBM-bound helpers: Word2Vec row gather, float->padded packing, casts, column sums.
#include <algorithm>

#include "tt_api.h"
#include "tt_common.h"

namespace {

// One 16-byte chunk per thread; consecutive threads walk a row, so both the
// table row read and the output row write are fully coalesced 16 B/lane.
__global__ __launch_bounds__(256) void embed_gather_kernel(const uint4* __restrict__ table, long vocab,
                                                           int cpr, const int32_t* __restrict__ ids,
                                                           long n, uint4* __restrict__ out) {
  const long total = n * cpr;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const long row = e / cpr;
    const int c = (int)(e - row * cpr);
    const int id = ids[row];
    uint4 v = make_uint4(0, 0, 0, 0);
    if (id >= 0 && id < vocab) v = table[(long)id * cpr + c];
    out[e] = v;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void pack_rows_kernel(const float* __restrict__ src, long n, int e, int ep,
                                                        T* __restrict__ out) {
  const long total = n * ep;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / ep;
    const int c = (int)(i - r * ep);
    Elt<T>::st(out + i, c < e ? src[r * e + c] : 0.f);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void cast_kernel(const float* __restrict__ x, long n, T* __restrict__ y) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) Elt<T>::st(y + i, x[i]);
}

// Column sums in a fixed order, so bias and LayerNorm gradients are bit-for-bit
// reproducible run to run (no float atomics): one 1024-thread workgroup per 64
// columns, wave w adds rows w, w+16, w+32, ... of its column (lane), then the 16 wave
// sums are added in wave order. Callers pass partial-row buffers (a few hundred rows).
__global__ __launch_bounds__(1024) void colsum_kernel(const float* __restrict__ x, long rows, int cols, long ld,
                                                      int accumulate, float* __restrict__ out) {
  __shared__ float red[16][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (c < cols)
    for (long r = wave; r < rows; r += 16) s += x[r * ld + c];
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += red[w][lane];
    out[c] = accumulate ? out[c] + t : t;
  }
}

__global__ __launch_bounds__(256) void sum_kernel(const float* __restrict__ x, long n, float scale,
                                                  float* __restrict__ out) {
  __shared__ float part[4];
  float s = 0.f;
  for (long i = threadIdx.x; i < n; i += 256) s += x[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = scale * (part[0] + part[1] + part[2] + part[3]);
}

struct PackArgs {
  tt_pack_job j[16];
  long start[17];  // prefix sums of rows * dcols / 4 (4-element groups per job)
  int n;
};
__global__ __launch_bounds__(256) void pack_multi_kernel(PackArgs a) {
  const long total = a.start[a.n];
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    int k = 0;
    while (k + 1 < a.n && i >= a.start[k + 1]) ++k;
    const tt_pack_job& J = a.j[k];
    const long q = i - a.start[k];
    const int g4 = J.dcols / 4;
    const long r = q / g4;
    const int c = (int)(q - r * g4) * 4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < J.cols) {
      v = *reinterpret_cast<const float4*>(J.src + r * J.lds + c);
      if (J.src2) {
        const float4 w = *reinterpret_cast<const float4*>(J.src2 + r * J.lds + c);
        v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
      }
    }
    if (J.dst_bf16) {
      const uint2 o = make_uint2((uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16),
                                 (uint32_t)f2bf(v.z) | ((uint32_t)f2bf(v.w) << 16));
      *reinterpret_cast<uint2*>(static_cast<bf16_t*>(J.dst) + r * J.ldd + c) = o;
    } else {
      *reinterpret_cast<float4*>(static_cast<float*>(J.dst) + r * J.ldd + c) = v;
    }
  }
}

inline unsigned grid_for(long work, int per_block = 256, int cap = 8192) {
  long g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (unsigned)std::min<long>(g, cap);
}

}  // namespace

extern "C" int tt_embed_gather(int dtype, const void* table, long vocab, int ep, const int32_t* ids, long n,
                               void* out, void* stream) {
  TT_CHECK_ARG(dtype == TT_DT_F32 || dtype == TT_DT_BF16, "tt_embed_gather: bad dtype");
  const int esz = dtype == TT_DT_BF16 ? 2 : 4;
  TT_CHECK_ARG((ep * esz) % 16 == 0, "tt_embed_gather: ep*sizeof(dtype) must be a multiple of 16 (ep=%d)", ep);
  if (n == 0) return 0;
  const int cpr = ep * esz / 16;
  hipLaunchKernelGGL(embed_gather_kernel, dim3(grid_for(n * cpr)), dim3(256), 0, (hipStream_t)stream,
                     (const uint4*)table, vocab, cpr, ids, n, (uint4*)out);
  TT_CHECK_LAUNCH("embed_gather_kernel");
  return 0;
}

extern "C" int tt_pack_rows(int dtype, const float* src, long n, int e, int ep, void* out, void* stream) {
  TT_CHECK_ARG(ep >= e, "tt_pack_rows: ep < e");
  if (n == 0) return 0;
  dim3 g(grid_for(n * ep));
  if (dtype == TT_DT_BF16)
    hipLaunchKernelGGL(pack_rows_kernel<bf16_t>, g, dim3(256), 0, (hipStream_t)stream, src, n, e, ep, (bf16_t*)out);
  else
    hipLaunchKernelGGL(pack_rows_kernel<float>, g, dim3(256), 0, (hipStream_t)stream, src, n, e, ep, (float*)out);
  TT_CHECK_LAUNCH("pack_rows_kernel");
  return 0;
}

extern "C" int tt_pack_multi(const tt_pack_job* jobs, int njobs, void* stream) {
  TT_CHECK_ARG(njobs >= 0 && njobs <= 16 && (njobs == 0 || jobs), "tt_pack_multi: njobs %d not in [0,16]", njobs);
  PackArgs a{};
  a.n = njobs;
  a.start[0] = 0;
  for (int k = 0; k < njobs; ++k) {
    const tt_pack_job& J = jobs[k];
    TT_CHECK_ARG(J.src && J.dst && J.rows >= 0 && J.cols >= 0 && J.dcols >= J.cols, "tt_pack_multi: job %d", k);
    TT_CHECK_ARG(J.cols % 4 == 0 && J.dcols % 4 == 0 && J.lds % 4 == 0 && J.ldd % 4 == 0 && J.lds >= J.cols &&
                     J.ldd >= J.dcols,
                 "tt_pack_multi: job %d: cols, dcols and leading dimensions must be multiples of 4", k);
    const bool src_ok = ((uintptr_t)J.src | (uintptr_t)J.src2) % 16 == 0;
    TT_CHECK_ARG(src_ok && (uintptr_t)J.dst % (J.dst_bf16 ? 8 : 16) == 0, "tt_pack_multi: job %d: misaligned operand", k);
    a.j[k] = J;
    a.start[k + 1] = a.start[k] + (long)J.rows * (J.dcols / 4);
  }
  if (a.start[njobs] == 0) return 0;
  hipLaunchKernelGGL(pack_multi_kernel, dim3(grid_for(a.start[njobs], 256, 4096)), dim3(256), 0, (hipStream_t)stream, a);
  TT_CHECK_LAUNCH("pack_multi_kernel");
  return 0;
}

extern "C" int tt_cast(int dtype, const float* x, long n, void* y, void* stream) {
  if (n == 0) return 0;
  dim3 g(grid_for(n));
  if (dtype == TT_DT_BF16)
    hipLaunchKernelGGL(cast_kernel<bf16_t>, g, dim3(256), 0, (hipStream_t)stream, x, n, (bf16_t*)y);
  else
    hipLaunchKernelGGL(cast_kernel<float>, g, dim3(256), 0, (hipStream_t)stream, x, n, (float*)y);
  TT_CHECK_LAUNCH("cast_kernel");
  return 0;
}

extern "C" int tt_colsum(const float* x, long rows, int cols, long ld, float* out, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (cols == 0) return 0;
  if (rows == 0) {
    if (!accumulate) TT_CHECK_HIP(hipMemsetAsync(out, 0, sizeof(float) * cols, st));
    return 0;
  }
  hipLaunchKernelGGL(colsum_kernel, dim3(tt_ceil_div(cols, 64)), dim3(1024), 0, st, x, rows, cols, ld, accumulate,
                     out);
  TT_CHECK_LAUNCH("colsum_kernel");
  return 0;
}

extern "C" int tt_sum(const float* x, long n, float scale, float* out, void* stream) {
  hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, x, n, scale, out);
  TT_CHECK_LAUNCH("sum_kernel");
  return 0;
}
