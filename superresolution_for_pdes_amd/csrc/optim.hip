// Fused clip_grad_norm_ + AdamW over ONE flat fp32 parameter buffer (gfx950).
//
// Reference: src/train_enhanced.py:74-75 (torch.nn.utils.clip_grad_norm_(params, 1.0);
// optimizer.step()) with optim.AdamW(lr=2e-4, weight_decay=1e-4) at :308.  The update
// order mirrors torch's foreach AdamW: p *= 1 - lr*wd; m = lerp(m, g, 1-b1);
// v = b2 v + (1-b2) g^2; p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps).
// The clip coefficient min(1, max_norm/(||g|| + 1e-6)) is computed ON DEVICE from a
// deterministic fp64 norm reduction and read by the update kernel: no host sync.
// grad_scale folds the data-parallel 1/world_size average into the same pass.
#include "common.h"

namespace srpde {

__global__ __launch_bounds__(256) void sqnorm_partial_kernel(const float* __restrict__ g, long long n,
                                                             float scale, double* __restrict__ part) {
  __shared__ double red[256];
  double s = 0.0;
  const long long n4 = n >> 2;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    const float4 v = reinterpret_cast<const float4*>(g)[i];
    const float a = v.x * scale, b = v.y * scale, c = v.z * scale, d = v.w * scale;
    s += (double)a * a + (double)b * b + (double)c * c + (double)d * d;
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const float a = g[n4 * 4 + threadIdx.x] * scale;
    s += (double)a * a;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// coef[0] = clip coefficient, coef[1] = total norm
__global__ void clip_coef_kernel(const double* __restrict__ part, int nblk, float max_norm, float* __restrict__ coef) {
  __shared__ double red[256];
  double s = 0.0;
  for (int k = threadIdx.x; k < nblk; k += 256) s += part[k];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float total = (float)sqrt(red[0]);
    float c = max_norm / (total + 1e-6f);
    if (!(max_norm > 0.f)) c = 1.f;
    coef[0] = c < 1.f ? c : 1.f;
    coef[1] = total;
  }
}

__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, long long n,
                                                    float lr, float beta1, float beta2, float eps, float wd,
                                                    float step_size, float bc2_sqrt, const float* __restrict__ coef,
                                                    float grad_scale) {
  const float gs = grad_scale * (coef ? coef[0] : 1.f);
  const float decay = 1.f - lr * wd;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float gi = g[i] * gs;
    float pi = p[i] * decay;
    float mi = m[i];
    mi = mi + (1.f - beta1) * (gi - mi);
    float vi = v[i] * beta2;
    vi = vi + (1.f - beta2) * gi * gi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi = pi + step_size * (mi / denom);
    p[i] = pi; m[i] = mi; v[i] = vi;
  }
}

}  // namespace srpde

using namespace srpde;

extern "C" {

size_t srpde_grad_norm_workspace_size(void) { return 1024 * sizeof(double); }

int srpde_clip_coef(const float* g, long long n, float grad_scale, float max_norm, float* coef, void* workspace,
                    size_t ws_bytes, hipStream_t stream) {
  SRPDE_CHECK_ARG(g && coef && workspace && ws_bytes >= 1024 * sizeof(double) && aligned16(g),
                  "srpde_clip_coef: bad args");
  const int nb = (int)std::min<long long>(1024, std::max<long long>(1, (n / 4 + 255) / 256));
  hipLaunchKernelGGL(sqnorm_partial_kernel, dim3(nb), dim3(256), 0, stream, g, n, grad_scale,
                     static_cast<double*>(workspace));
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(256), 0, stream, static_cast<const double*>(workspace), nb,
                     max_norm, coef);
  SRPDE_LAUNCH_CHECK("srpde_clip_coef");
  return 0;
}

int srpde_adamw_step(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1, float beta2,
                     float eps, float weight_decay, int step, const float* coef, float grad_scale,
                     hipStream_t stream) {
  SRPDE_CHECK_ARG(p && g && m && v && n > 0 && step >= 1, "srpde_adamw_step: bad args");
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  const float step_size = (float)(-(double)lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  const int blocks = (int)std::min<long long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(adamw_kernel, dim3(blocks), dim3(256), 0, stream, p, g, m, v, n, lr, beta1, beta2, eps,
                     weight_decay, step_size, bc2_sqrt, coef, grad_scale);
  SRPDE_LAUNCH_CHECK("srpde_adamw_step");
  return 0;
}

}  // extern "C"
