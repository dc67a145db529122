// Bilinear x2 (align_corners=True) source indices and weights, shared by the upsample kernels
// (pointwise.hip) and the convolutions that read an upsampled input without materialising it (h4).
#pragma once
#include "common.h"

namespace srpde {

// align_corners=True: src = dst * (in-1)/(out-1) (float, as aten area_pixel_compute_scale),
// i0 = floor(src), i1 = i0 + (i0 < in-1), l1 = src - i0, l0 = 1 - l1.
struct Lerp { int i0, i1; float l0, l1; };
__device__ __forceinline__ Lerp lerp_index(int o, int in, int out) {
  const float scale = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
  // rounded product, as aten's area_pixel_compute_source_index: with contraction on, the compiler
  // may fuse src - i0 below into fma(scale, o, -i0) (it did once packed-FP32 ops were disabled), which
  // moves the weights by up to an ulp of src (~2e-6 at src ~ 19) and the interpolated values with them
  float src;
  {
#pragma clang fp contract(off)
    src = scale * (float)o;
  }
  Lerp r;
  r.i0 = (int)src;
  r.i1 = r.i0 + (r.i0 < in - 1 ? 1 : 0);
  r.l1 = src - (float)r.i0;
  r.l0 = 1.f - r.l1;
  return r;
}


}  // namespace srpde
