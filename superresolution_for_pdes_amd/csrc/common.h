// srpde-mi355x: shared helpers for the gfx950 HIP kernels behind include/srpde.h.
//
// Conventions (see DESIGN.md "Data layout in HBM"):
//  * activations are NHWC fp32 ("channels-last"); a tensor VIEW is (ptr, ld) where
//    ld = row stride in floats between consecutive pixels, so a channel slice of a
//    wider tensor (virtual concat) is addressed without a copy;
//  * pixel index p = (n*H + y)*W + x, P = N*H*W;
//  * every entry point is stream-ordered on the hipStream_t it is given, never
//    allocates, never synchronises the host, and returns 0 / negative arg error /
//    positive hipError_t.  The message is kept in a thread-local buffer.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <algorithm>

#include "../../include/srpde.h"

namespace srpde {

void set_error(const char* fmt, ...);
// the main kernel a conv entry point launched, as rocprofv3 names it (srpde_last_kernel; bench.py's roofline)
void note_kernel(const char* fmt, ...);

constexpr int kErrArg = -1;
constexpr int kErrShape = -2;
constexpr int kErrAlign = -3;
constexpr int kErrWorkspace = -4;

#define SRPDE_CHECK_ARG(cond, ...)                        \
  do {                                                    \
    if (!(cond)) {                                        \
      ::srpde::set_error(__VA_ARGS__);                    \
      return ::srpde::kErrArg;                            \
    }                                                     \
  } while (0)

#define SRPDE_LAUNCH_CHECK(name)                                            \
  do {                                                                      \
    hipError_t e_ = hipGetLastError();                                      \
    if (e_ != hipSuccess) {                                                 \
      ::srpde::set_error("%s: launch failed: %s", name, hipGetErrorString(e_)); \
      return (int)e_;                                                       \
    }                                                                       \
  } while (0)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

inline int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// h3 operand scales (conv_h3.hip header): the power-of-two exponent that brings max|x| (float
// bits) just under 2^15, and 2^e as a float.  Every producer and consumer of a split forms the
// scale with these two, so a split written by one kernel is read back exactly by another.
__device__ __forceinline__ int h3_exp(unsigned bits) {
  const int e = (int)((bits >> 23) & 0xffu);
  if (e == 0) return bits ? 100 : 0;            // zero / denormal maximum
  if (e == 0xff) return 0;                      // inf / nan: propagate
  return min(max(15 - (e - 126), -100), 100);   // max < 2^(e-126)
}
__device__ __forceinline__ float exp2i(int e) { return __uint_as_float((unsigned)(e + 127) << 23); }

}  // namespace srpde
