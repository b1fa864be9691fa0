// Host-side helpers for the C-ABI layer: error capture and launch checks.
#pragma once
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include "../../include/tt_hip.h"

namespace tt {
void set_error(const char* fmt, ...);
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
