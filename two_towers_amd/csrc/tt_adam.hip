// Multi-tensor Adam: one launch updates every parameter of the model.
#include <math.h>

#include "tt_api.h"
#include "tt_common.h"

namespace {

constexpr int MAXT = 48;
constexpr int CHUNK = 4096;  // elements per workgroup

struct AdamArgs {
  float* p[MAXT];
  const float* g[MAXT];
  float* m[MAXT];
  float* v[MAXT];
  long start[MAXT + 1];  // prefix sums of sizes
  const int* skip;       // device word: non-zero -> leave every tensor unchanged (or null)
  int nt;
  float b2, omb1, omb2, eps, wd, step_size, bc2_sqrt;
};

// Matches torch.optim.adam._single_tensor_adam (foreach=False, capturable=False):
//   exp_avg.lerp_(grad, 1-b1); exp_avg_sq.mul_(b2).addcmul_(grad, grad, value=1-b2)
//   denom = exp_avg_sq.sqrt() / bias_correction2_sqrt + eps
//   param.addcdiv_(exp_avg, denom, value=-lr/bias_correction1)
__global__ __launch_bounds__(256) void adam_kernel(AdamArgs a) {
  if (a.skip && *a.skip != 0) return;  // an invalid forward fed this step
  const long e0 = (long)blockIdx.x * CHUNK;
  const long total = a.start[a.nt];
  int t = 0;
  while (t + 1 < a.nt && a.start[t + 1] <= e0) ++t;
  for (long e = e0 + threadIdx.x; e < min(total, e0 + CHUNK); e += 256) {
    while (e >= a.start[t + 1]) ++t;
    const long i = e - a.start[t];
    float g = a.g[t][i];
    float p = a.p[t][i];
    if (a.wd != 0.f) g = g + a.wd * p;
    float m = a.m[t][i];
    float v = a.v[t][i];
    m = m + a.omb1 * (g - m);  // lerp, weight < 0.5 branch
    v = v * a.b2 + a.omb2 * g * g;
    const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
    p = p + (-a.step_size * m) / denom;
    a.m[t][i] = m;
    a.v[t][i] = v;
    a.p[t][i] = p;
  }
}

}  // namespace

extern "C" int tt_adam_multi(float* const* params, const float* const* grads, float* const* exp_avg,
                             float* const* exp_avg_sq, const long* sizes, int ntensors, float lr, float beta1,
                             float beta2, float eps, float weight_decay, int step, const int32_t* skip,
                             void* stream) {
  TT_CHECK_ARG(ntensors >= 0 && ntensors <= MAXT, "tt_adam_multi: at most %d tensors per call", MAXT);
  TT_CHECK_ARG(step >= 1, "tt_adam_multi: step must be >= 1");
  if (ntensors == 0) return 0;
  AdamArgs a{};
  a.start[0] = 0;
  for (int i = 0; i < ntensors; ++i) {
    a.p[i] = params[i];
    a.g[i] = grads[i];
    a.m[i] = exp_avg[i];
    a.v[i] = exp_avg_sq[i];
    a.start[i + 1] = a.start[i] + sizes[i];
  }
  a.nt = ntensors;
  a.skip = skip;
  a.b2 = beta2; a.omb1 = (float)(1.0 - (double)beta1); a.omb2 = (float)(1.0 - (double)beta2);
  a.eps = eps; a.wd = weight_decay;
  const double bc1 = 1.0 - pow((double)beta1, step);
  const double bc2 = 1.0 - pow((double)beta2, step);
  a.step_size = (float)(lr / bc1);
  a.bc2_sqrt = (float)sqrt(bc2);
  const long total = a.start[ntensors];
  if (total == 0) return 0;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)tt_ceil_div(total, CHUNK)), dim3(256), 0, (hipStream_t)stream, a);
  TT_CHECK_LAUNCH("adam_kernel");
  return 0;
}
