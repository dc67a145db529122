// Bicubic resize with align_corners=True for single-channel fields, gfx950.
//
// Replaces F.interpolate(u, size=(ho, wo), mode='bicubic', align_corners=True) of the
// interpolation baselines the reference compares its cascade against
// (src/resolution_comparison_enhanced.py:43-65 multi-level, :386-392 direct).  Semantics of
// aten::upsample_bicubic2d (align_corners=True): source coordinate s = dst * (in-1)/(out-1) in
// fp32, i = floor(s), t = s - i, Keys' cubic convolution with A = -0.75 over taps i-1..i+2,
// taps clamped to the border (upsample_get_value_bounded); rows interpolated along x first,
// then the four row values along y.  fp32 arithmetic, as the reference's .float() fields.
//
// Memory-bound and tiny (a 640^2 field is 1.6 MB): one thread per output pixel, the 16 taps
// come from L2 (a row of the source is reused by the 2-3 output rows that map into it).
#include "common.h"

namespace srpde {

__device__ __forceinline__ void cubic_coeffs(float t, float c[4]) {
  const float A = -0.75f;
  const float x1 = t + 1.0f;                  // cubic_convolution2
  c[0] = ((A * x1 - 5.0f * A) * x1 + 8.0f * A) * x1 - 4.0f * A;
  c[1] = ((A + 2.0f) * t - (A + 3.0f)) * t * t + 1.0f;      // cubic_convolution1
  const float x2 = 1.0f - t;
  c[2] = ((A + 2.0f) * x2 - (A + 3.0f)) * x2 * x2 + 1.0f;
  const float x3 = x2 + 1.0f;                 // (1 - t) + 1, as aten (not 2 - t: one rounding differs)
  c[3] = ((A * x3 - 5.0f * A) * x3 + 8.0f * A) * x3 - 4.0f * A;
}

__global__ __launch_bounds__(256) void resize_bicubic_ac_kernel(const float* __restrict__ x, float* __restrict__ out,
                                                               int planes, int h, int w, int ho, int wo, float sy,
                                                               float sx) {
  const long long total = (long long)planes * ho * wo;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const long long pl = e / ((long long)ho * wo);
    const int rem = (int)(e - pl * ho * wo);
    const int oy = rem / wo, ox = rem - oy * wo;
    // rounded products (no contraction into the fractional parts below), as aten computes them
    float ry, rx;
    {
#pragma clang fp contract(off)
      ry = sy * (float)oy;
      rx = sx * (float)ox;
    }
    const int iy = (int)floorf(ry), ix = (int)floorf(rx);
    float cy[4], cx[4];
    cubic_coeffs(ry - (float)iy, cy);
    cubic_coeffs(rx - (float)ix, cx);
    int xs[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) xs[j] = min(max(ix - 1 + j, 0), w - 1);
    const float* src = x + pl * h * w;
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float* row = src + (size_t)min(max(iy - 1 + k, 0), h - 1) * w;
      const float r = row[xs[0]] * cx[0] + row[xs[1]] * cx[1] + row[xs[2]] * cx[2] + row[xs[3]] * cx[3];
      acc += r * cy[k];
    }
    out[e] = acc;
  }
}

}  // namespace srpde

using namespace srpde;

extern "C" {

int srpde_resize_bicubic_ac(const float* x, float* out, int planes, int h, int w, int ho, int wo,
                            hipStream_t stream) {
  SRPDE_CHECK_ARG(x && out && planes > 0 && h > 0 && w > 0 && ho > 0 && wo > 0, "srpde_resize_bicubic_ac: bad args");
  const float sy = ho > 1 ? (float)(h - 1) / (float)(ho - 1) : 0.f;
  const float sx = wo > 1 ? (float)(w - 1) / (float)(wo - 1) : 0.f;
  const long long total = (long long)planes * ho * wo;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(resize_bicubic_ac_kernel, dim3(blocks), dim3(256), 0, stream, x, out, planes, h, w, ho, wo, sy,
                     sx);
  SRPDE_LAUNCH_CHECK("srpde_resize_bicubic_ac");
  return 0;
}

}  // extern "C"
