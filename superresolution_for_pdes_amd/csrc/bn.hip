// BatchNorm2d (train / eval) + ReLU for NHWC fp32, gfx950.
//
// Reference semantics (src/models.py:17,19,44-48,58,60 -> nn.BatchNorm2d defaults, then
// F.relu / nn.ReLU): train mode normalises with the biased batch variance, updates
// running_mean / running_var (unbiased) with momentum 0.1 and num_batches_tracked += 1;
// eval mode uses the running statistics.  eps = 1e-5.
//
// Batch statistics come from the conv epilogue's per-row-block (mean, M2) partials
// (conv.hip) merged here with Chan's parallel formula in fp64, in a fixed tree order
// (deterministic).  The backward recomputes x_hat and the ReLU mask from the conv
// output y instead of storing them.
#include "common.h"

namespace srpde {

struct Chan {
  double n, mean, m2;
};
__device__ __forceinline__ Chan chan_merge(Chan a, Chan b) {
  if (b.n == 0.0) return a;
  if (a.n == 0.0) return b;
  const double n = a.n + b.n, d = b.mean - a.mean;
  Chan r;
  r.n = n;
  r.mean = a.mean + d * (b.n / n);
  r.m2 = a.m2 + b.m2 + d * d * (a.n * b.n / n);
  return r;
}

// one block per channel.  The equal-count row blocks (all but a ragged last one) merge without a
// division per partial: with a shift s (block 0's mean), each thread sums (mean_b - s), (mean_b -
// s)^2 and M2_b in fp64; one fixed-order tree combines the threads; then
// mean = s + S1 / k  and  M2 = sum M2_b + n * (S2 - S1^2 / k)  (the parallel-variance identity for k
// blocks of n rows), and the ragged block joins with one Chan merge.  (A Chan merge per partial is
// a dependent chain of fp64 divisions: 50 of them per thread at the 40x40 layers.)  Also bumps
// num_batches_tracked (block 0), which used to be a launch of its own.
// 1024 threads, four partials in flight per thread: the kernel is latency-bound (one block per
// channel reads nblk strided float2), e.g. 12,800 partials per channel at the 40x40 layers.
// channel c's batch statistics from the fp64 sums over its nfull equal-count row blocks (shift = block 0's
// mean; s1 = sum (mean_b - shift), s2 = sum (mean_b - shift)^2, sm = sum M2_b) and the ragged last block: mean /
// invstd, running statistics, num_batches_tracked (c == 0) and, with scale_out, the fused consumer's affine
__device__ __forceinline__ void fin_channel(int c, const float2* __restrict__ stats, int nblk, int nfull,
                                            int rows_per_blk, long long P, int C, double shift, double s1, double s2,
                                            double sm, float* running_mean, float* running_var, float momentum,
                                            float eps, float* __restrict__ mean_out, float* __restrict__ invstd_out,
                                            long long* num_batches_tracked, const float* __restrict__ gamma,
                                            const float* __restrict__ beta, float* __restrict__ scale_out,
                                            float* __restrict__ shift_out, unsigned* amax, float sqrt_pm1) {
  Chan acc{0.0, 0.0, 0.0};
  if (nfull > 0) {
    const double k = (double)nfull, n0 = (double)rows_per_blk;
    const double m2 = sm + n0 * fmax(s2 - s1 * s1 / k, 0.0);
    acc = Chan{k * n0, shift + s1 / k, m2};
  }
  for (int b = nfull; b < nblk; ++b) {   // the ragged last block, if any
    const float2 v = stats[(size_t)b * C + c];
    const long long rem = P - (long long)b * rows_per_blk;
    const double cnt = (double)(rem < rows_per_blk ? rem : rows_per_blk);
    acc = chan_merge(acc, Chan{cnt, (double)v.x, (double)v.y});
  }
  const double n = acc.n, mean = acc.mean, m2 = acc.m2;
  const double var_b = m2 / n;
  const double var_u = n > 1.0 ? m2 / (n - 1.0) : var_b;
  mean_out[c] = (float)mean;
  invstd_out[c] = (float)(1.0 / sqrt(var_b + (double)eps));
  if (running_mean) running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
  if (running_var) running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)var_u;
  if (c == 0 && num_batches_tracked) *num_batches_tracked += 1;
  if (scale_out) {   // bn_affine_kernel's outputs for this channel, from the same float mean / invstd
    const float sc = gamma[c] * invstd_out[c];
    scale_out[c] = sc;
    shift_out[c] = beta[c] - mean_out[c] * sc;
    if (amax) atomicMax(amax, __float_as_uint(fabsf(gamma[c]) * sqrt_pm1 + fabsf(beta[c])));
  }
}

constexpr int FIN_T = 1024;
__global__ __launch_bounds__(FIN_T) void bn_train_finalize_kernel(
    const float2* __restrict__ stats, int nblk, int rows_per_blk, long long P, int C,
    float* running_mean, float* running_var, float momentum, float eps,
    float* __restrict__ mean_out, float* __restrict__ invstd_out, long long* num_batches_tracked,
    const float* __restrict__ gamma = nullptr, const float* __restrict__ beta = nullptr,
    float* __restrict__ scale_out = nullptr, float* __restrict__ shift_out = nullptr, unsigned* amax = nullptr,
    float sqrt_pm1 = 0.f) {
  const int c = blockIdx.x;
  __shared__ double s1[FIN_T], s2[FIN_T], sm[FIN_T];
  const long long nfull_ll = P / rows_per_blk;
  const int nfull = (int)(nfull_ll < nblk ? nfull_ll : nblk);
  const double shift = nfull > 0 ? (double)stats[c].x : 0.0;
  double a1 = 0.0, a2 = 0.0, am = 0.0;
  int b = threadIdx.x;
  for (; b + 3 * FIN_T < nfull; b += 4 * FIN_T) {
    float2 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = stats[(size_t)(b + u * FIN_T) * C + c];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const double d = (double)v[u].x - shift;
      a1 += d;
      a2 = fma(d, d, a2);
      am += (double)v[u].y;
    }
  }
  for (; b < nfull; b += FIN_T) {
    const float2 v = stats[(size_t)b * C + c];
    const double d = (double)v.x - shift;
    a1 += d;
    a2 = fma(d, d, a2);
    am += (double)v.y;
  }
  s1[threadIdx.x] = a1; s2[threadIdx.x] = a2; sm[threadIdx.x] = am;
  __syncthreads();
  for (int s = FIN_T / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      s1[threadIdx.x] += s1[threadIdx.x + s];
      s2[threadIdx.x] += s2[threadIdx.x + s];
      sm[threadIdx.x] += sm[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0)
    fin_channel(c, stats, nblk, nfull, rows_per_blk, P, C, shift, s1[0], s2[0], sm[0], running_mean, running_var,
                momentum, eps, mean_out, invstd_out, num_batches_tracked, gamma, beta, scale_out, shift_out, amax,
                sqrt_pm1);
}

// The same statistics in two coalesced passes (srpde_bn_train_finalize_ws): one block per channel reads one float2 of
// each 128-B line, so a 40 x 40 layer's 20,480 partials per channel are 20,480 line requests on each of only C CUs
// (36 us at C = 64).  Pass 1: (16-channel group, row slice) blocks, a wave reading 4 rows x 16 channels = four whole
// lines per instruction, fp64 sums per channel and slice into ws [S][C][3]; pass 2: one wave per channel loads
// the S slices at once and sums them in order, then finishes as fin_channel.  Same expressions; the sums are ordered per slice, then over slices.
constexpr int FIN_SPLIT_MAX = 64;
__global__ __launch_bounds__(256) void bn_stats_split_kernel(const float2* __restrict__ stats, int nfull, int rows,
                                                             int C, double* __restrict__ ws) {
  __shared__ double red[3][16][17];
  const int cl = threadIdx.x & 15, ph = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl, sl = blockIdx.y;
  const int b0 = sl * rows, b1 = min(nfull, b0 + rows);
  double a1 = 0.0, a2 = 0.0, am = 0.0;
  if (c < C && nfull > 0) {
    const double shift = (double)stats[c].x;
    int b = b0 + ph;
    for (; b + 48 < b1; b += 64) {
      float2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = stats[(size_t)(b + 16 * u) * C + c];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const double d = (double)v[u].x - shift;
        a1 += d;
        a2 = fma(d, d, a2);
        am += (double)v[u].y;
      }
    }
    for (; b < b1; b += 16) {
      const float2 v = stats[(size_t)b * C + c];
      const double d = (double)v.x - shift;
      a1 += d;
      a2 = fma(d, d, a2);
      am += (double)v.y;
    }
  }
  red[0][ph][cl] = a1; red[1][ph][cl] = a2; red[2][ph][cl] = am;
  __syncthreads();
  if (ph < 3 && c < C) {   // three threads per channel: one sum each, phases in order
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[ph][k][cl];
    ws[((size_t)sl * C + c) * 3 + ph] = t;
  }
}

__global__ __launch_bounds__(64) void bn_finalize_split_kernel(const float2* __restrict__ stats, const double* __restrict__ ws,
                                                               int nsl, int nblk, int rows_per_blk, long long P, int C,
                                                               float* running_mean, float* running_var, float momentum,
                                                               float eps, float* __restrict__ mean_out,
                                                               float* __restrict__ invstd_out,
                                                               long long* num_batches_tracked,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, float* __restrict__ scale_out,
                                                               float* __restrict__ shift_out, unsigned* amax, float sqrt_pm1) {
  // one wave per channel: every slice's sums loaded at once (lane k: slice k), then summed in slice order
  __shared__ double part[3][FIN_SPLIT_MAX];
  const int c = blockIdx.x, k = threadIdx.x;
  if (k < nsl) {
    const double* w = ws + ((size_t)k * C + c) * 3;
    part[0][k] = w[0]; part[1][k] = w[1]; part[2][k] = w[2];
  }
  __syncthreads();
  if (k != 0) return;
  const long long nfull_ll = P / rows_per_blk;
  const int nfull = (int)(nfull_ll < nblk ? nfull_ll : nblk);
  double s1 = 0.0, s2 = 0.0, sm = 0.0;
  for (int j = 0; j < nsl; ++j) {
    s1 += part[0][j]; s2 += part[1][j]; sm += part[2][j];
  }
  fin_channel(c, stats, nblk, nfull, rows_per_blk, P, C, nfull > 0 ? (double)stats[c].x : 0.0, s1, s2, sm,
              running_mean, running_var, momentum, eps, mean_out, invstd_out, num_batches_tracked, gamma, beta,
              scale_out, shift_out, amax, sqrt_pm1);
}

// row slices of pass 1: ~4 blocks per CU-sized wave of work, at least 64 rows (4 per phase) per slice
static int fin_slices(int nfull, int C) {
  const int groups = (C + 15) / 16;
  int sl = (1024 / groups + 3) / 4;
  sl = std::max(1, std::min(sl, FIN_SPLIT_MAX));
  sl = std::min(sl, std::max(1, nfull / 64));
  return sl;
}

__global__ void bn_eval_prepare_kernel(const float* rm, const float* rv, int C, float eps, float* mean_out,
                                       float* invstd_out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) {
    mean_out[c] = rm[c];
    invstd_out[c] = 1.0f / sqrtf(rv[c] + eps);
  }
}

// per-channel affine of train-mode BN (a = relu(y*scale + shift)) for a consumer that applies it
// on the fly (the h3 convolution's input transform), and a rigorous bound on max|a|:
// Samuelson, |y - mean| <= sqrt(P-1) * std_biased, so |a| <= |gamma| sqrt(P-1) + |beta|
__global__ __launch_bounds__(256) void bn_affine_kernel(const float* __restrict__ mean, const float* __restrict__ invstd,
                                                        const float* __restrict__ gamma, const float* __restrict__ beta,
                                                        int C, float sqrt_pm1, float* __restrict__ scale,
                                                        float* __restrict__ shift, unsigned* amax) {
  float m = 0.f;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float sc = gamma[c] * invstd[c];
    scale[c] = sc;
    shift[c] = beta[c] - mean[c] * sc;
    m = fmaxf(m, fabsf(gamma[c]) * sqrt_pm1 + fabsf(beta[c]));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  __shared__ float wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0 && amax) atomicMax(amax, __float_as_uint(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]))));
}


// *amax = max(*amax, block max of v) as float bits (v >= 0): the max|x| word the h3
// convolutions (conv_h3.hip) derive their power-of-two operand scale from
__device__ __forceinline__ void block_amax(float v, unsigned* amax) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  __shared__ float wmax[16];
  const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  if ((threadIdx.x & 63) == 0) wmax[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = 0.f;
    for (int k = 0; k < nw; ++k) m = fmaxf(m, wmax[k]);
    atomicMax(amax, __float_as_uint(m));
  }
}

// out = relu((y - mean) * invstd * gamma + beta)
__global__ __launch_bounds__(256) void bn_relu_fwd_kernel(const float* __restrict__ y, int ldy,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float* __restrict__ out,
                                                          int ldo, long long P, int C, int relu, unsigned* amax) {
  const int C4 = C >> 2;
  const long long total = P * C4;
  float mx = 0.f;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const long long p = e / C4;
    const int c = (int)(e - p * C4) * 4;
    const float4 v = *reinterpret_cast<const float4*>(y + p * ldy + c);
    const float4 mu = *reinterpret_cast<const float4*>(mean + c);
    const float4 is = *reinterpret_cast<const float4*>(invstd + c);
    const float4 g = *reinterpret_cast<const float4*>(gamma + c);
    const float4 b = *reinterpret_cast<const float4*>(beta + c);
    float4 o;
    o.x = (v.x - mu.x) * is.x * g.x + b.x;
    o.y = (v.y - mu.y) * is.y * g.y + b.y;
    o.z = (v.z - mu.z) * is.z * g.z + b.z;
    o.w = (v.w - mu.w) * is.w * g.w + b.w;
    if (relu) {
      o.x = fmaxf(o.x, 0.f); o.y = fmaxf(o.y, 0.f); o.z = fmaxf(o.z, 0.f); o.w = fmaxf(o.w, 0.f);
    }
    *reinterpret_cast<float4*>(out + p * ldo + c) = o;
    mx = fmaxf(mx, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
  }
  if (amax) block_amax(mx, amax);
}

// Generic per-channel column reduction layout used by the backward passes:
// block b owns rows [b*rows_per_blk, ...), threads tile (row, channel-quad).
// rows a thread keeps in flight in the row loops below (bn_rows): one outstanding row per thread left
// these HBM-bound kernels latency-bound at 2-3 TB/s.  The per-thread order of the rows (and of the sums
// over them) is unchanged.
constexpr int BN_U = 4;

__device__ __forceinline__ void thread_rc(int C, int* c4, int* r0, int* rstride) {
  const int C4 = C >> 2;
  *c4 = threadIdx.x % C4;
  *r0 = threadIdx.x / C4;
  *rstride = blockDim.x / C4;
}

// rows p0, p0 + rs, ... < pe of (y, da) at channel quad c, handed in order to row(p, y quad, da quad): BN_U
// rows loaded before the first is used, the last partial group one row at a time
template <typename F>
__device__ __forceinline__ void bn_rows(long long p0, long long pe, int rs, const float* __restrict__ y, int ldy,
                                        const float* __restrict__ da, int ldda, int c, F&& row) {
  for (; p0 + (BN_U - 1) * rs < pe; p0 += BN_U * rs) {
    float4 vv[BN_U], dd[BN_U];
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      vv[u] = *reinterpret_cast<const float4*>(y + (p0 + u * rs) * ldy + c);
      dd[u] = *reinterpret_cast<const float4*>(da + (p0 + u * rs) * ldda + c);
    }
    __builtin_amdgcn_sched_barrier(0);   // (the scheduler would sink each load to its row)
#pragma unroll
    for (int u = 0; u < BN_U; ++u) row(p0 + u * rs, vv[u], dd[u]);
  }
  for (; p0 < pe; p0 += rs)
    row(p0, *reinterpret_cast<const float4*>(y + p0 * ldy + c), *reinterpret_cast<const float4*>(da + p0 * ldda + c));
}

// partial sums of dz and dz*xhat per (block, channel); dz = da * [bn_out > 0]
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const float* __restrict__ y, int ldy,
                                                            const float* __restrict__ da, int ldda,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ invstd,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, long long P, int C,
                                                            int rows_per_blk, int relu,
                                                            float2* __restrict__ part,
                                                            float* __restrict__ da_max = nullptr) {
  extern __shared__ float4 red4[];  // [2][256]
  int c4, r0, rs;
  thread_rc(C, &c4, &r0, &rs);
  const int active = (C >> 2) * rs;
  const int c = c4 * 4;
  float4 s1 = make_float4(0.f, 0.f, 0.f, 0.f), s2 = s1;
  float dmax = 0.f;
  if ((int)threadIdx.x < active) {
    const float4 mu = *reinterpret_cast<const float4*>(mean + c);
    const float4 is = *reinterpret_cast<const float4*>(invstd + c);
    const float4 g = *reinterpret_cast<const float4*>(gamma + c);
    const float4 b = *reinterpret_cast<const float4*>(beta + c);
    const long long pb = (long long)blockIdx.x * rows_per_blk;
    const long long pe = min(P, pb + rows_per_blk);
    auto row = [&](long long, const float4& v, const float4& d) {
      dmax = fmaxf(dmax, fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fmaxf(fabsf(d.z), fabsf(d.w))));
      float xh, dz;
#define BN_ACC(X)                                              \
  xh = (v.X - mu.X) * is.X;                                    \
  dz = (!(relu & 1) || xh * g.X + b.X > 0.f) ? d.X : 0.f;      \
  s1.X += dz;                                                  \
  s2.X += dz * xh;
      BN_ACC(x) BN_ACC(y) BN_ACC(z) BN_ACC(w)
#undef BN_ACC
    };
    bn_rows(pb + r0, pe, rs, y, ldy, da, ldda, c, row);
  }
  red4[threadIdx.x] = s1;
  red4[256 + threadIdx.x] = s2;
  __syncthreads();
  if ((int)threadIdx.x < (C >> 2)) {
    float4 t1 = make_float4(0.f, 0.f, 0.f, 0.f), t2 = t1;
    for (int r = 0; r < rs; ++r) {
      const float4 a = red4[r * (C >> 2) + threadIdx.x], b2 = red4[256 + r * (C >> 2) + threadIdx.x];
      t1.x += a.x; t1.y += a.y; t1.z += a.z; t1.w += a.w;
      t2.x += b2.x; t2.y += b2.y; t2.z += b2.z; t2.w += b2.w;
    }
    float2* o = part + (size_t)blockIdx.x * C + c;
    o[0] = make_float2(t1.x, t2.x); o[1] = make_float2(t1.y, t2.y);
    o[2] = make_float2(t1.z, t2.z); o[3] = make_float2(t1.w, t2.w);
  }
  if (da_max != nullptr) {   // this block's max|da| -> its slot (block-uniform branch)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) dmax = fmaxf(dmax, __shfl_xor(dmax, o, 64));
    __syncthreads();
    float* wmx = reinterpret_cast<float*>(red4);
    if ((threadIdx.x & 63) == 0) wmx[threadIdx.x >> 6] = dmax;
    __syncthreads();
    if (threadIdx.x == 0) da_max[blockIdx.x] = fmaxf(fmaxf(wmx[0], wmx[1]), fmaxf(wmx[2], wmx[3]));
  }
}

// The attention gate's gating gradient accumulated into dg (pointwise.hip att_bwd_gating_kernel's
// expressions: dg[p][c] += dsa[p] * wg[c]) together with the backward reduction of the BN (+ ReLU) whose
// output gradient dg then is (bn_bwd_reduce_kernel's expressions and partial layout) -- the bridge's last BN
// under att3's gating signal (src/models.py:46-48, 88): one pass instead of the gating pass plus a
// reduction pass that re-read dg.
__global__ __launch_bounds__(256) void gating_bn_reduce_kernel(const float* __restrict__ dsa, const float* __restrict__ wg,
                                                               float* dg, int lddg, const float* __restrict__ y,
                                                               int ldy, const float* __restrict__ mean,
                                                               const float* __restrict__ invstd,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, long long P, int C,
                                                               int rows_per_blk, int relu, float2* __restrict__ part,
                                                               float* __restrict__ da_max) {
  extern __shared__ float4 red4[];  // [2][256]
  int c4, r0, rs;
  thread_rc(C, &c4, &r0, &rs);
  const int active = (C >> 2) * rs;
  const int c = c4 * 4;
  float4 s1 = make_float4(0.f, 0.f, 0.f, 0.f), s2 = s1;
  float dmax = 0.f;
  if ((int)threadIdx.x < active) {
    const float4 mu = *reinterpret_cast<const float4*>(mean + c);
    const float4 is = *reinterpret_cast<const float4*>(invstd + c);
    const float4 g = *reinterpret_cast<const float4*>(gamma + c);
    const float4 b = *reinterpret_cast<const float4*>(beta + c);
    const float4 w = *reinterpret_cast<const float4*>(wg + c);
    const long long pb = (long long)blockIdx.x * rows_per_blk;
    const long long pe = min(P, pb + rows_per_blk);
    auto row = [&](long long p, const float4& v, const float4& old) {
      const float sp = dsa[p];
      float4 d = make_float4(sp * w.x, sp * w.y, sp * w.z, sp * w.w);
      d.x += old.x; d.y += old.y; d.z += old.z; d.w += old.w;
      *reinterpret_cast<float4*>(dg + p * lddg + c) = d;
      dmax = fmaxf(dmax, fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fmaxf(fabsf(d.z), fabsf(d.w))));
      float xh, dz;
#define GBN_ACC(X)                                             \
  xh = (v.X - mu.X) * is.X;                                    \
  dz = (!(relu & 1) || xh * g.X + b.X > 0.f) ? d.X : 0.f;      \
  s1.X += dz;                                                  \
  s2.X += dz * xh;
      GBN_ACC(x) GBN_ACC(y) GBN_ACC(z) GBN_ACC(w)
#undef GBN_ACC
    };
    bn_rows(pb + r0, pe, rs, y, ldy, dg, lddg, c, row);
  }
  red4[threadIdx.x] = s1;
  red4[256 + threadIdx.x] = s2;
  __syncthreads();
  if ((int)threadIdx.x < (C >> 2)) {
    float4 t1 = make_float4(0.f, 0.f, 0.f, 0.f), t2 = t1;
    for (int r = 0; r < rs; ++r) {
      const float4 a = red4[r * (C >> 2) + threadIdx.x], b2 = red4[256 + r * (C >> 2) + threadIdx.x];
      t1.x += a.x; t1.y += a.y; t1.z += a.z; t1.w += a.w;
      t2.x += b2.x; t2.y += b2.y; t2.z += b2.z; t2.w += b2.w;
    }
    float2* o = part + (size_t)blockIdx.x * C + c;
    o[0] = make_float2(t1.x, t2.x); o[1] = make_float2(t1.y, t2.y);
    o[2] = make_float2(t1.z, t2.z); o[3] = make_float2(t1.w, t2.w);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) dmax = fmaxf(dmax, __shfl_xor(dmax, o, 64));
  __syncthreads();
  float* wmx = reinterpret_cast<float*>(red4);
  if ((threadIdx.x & 63) == 0) wmx[threadIdx.x >> 6] = dmax;
  __syncthreads();
  if (threadIdx.x == 0) da_max[blockIdx.x] = fmaxf(fmaxf(wmx[0], wmx[1]), fmaxf(wmx[2], wmx[3]));
}

// fp64 column sums of [nblk][C] float2 partials -> out0[C], out1[C]; one block per channel
__global__ __launch_bounds__(256) void colsum2_kernel(const float2* __restrict__ part, int nblk, int C,
                                                      float* out0, float* out1, double* keep0, double* keep1) {
  const int c = blockIdx.x;
  __shared__ double a[256], b[256];
  double x = 0.0, yv = 0.0;
  for (int k = threadIdx.x; k < nblk; k += 256) {
    const float2 v = part[(size_t)k * C + c];
    x += v.x; yv += v.y;
  }
  a[threadIdx.x] = x; b[threadIdx.x] = yv;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) { a[threadIdx.x] += a[threadIdx.x + s]; b[threadIdx.x] += b[threadIdx.x + s]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (out0) out0[c] = (float)a[0];
    if (out1) out1[c] = (float)b[0];
    if (keep0) keep0[c] = a[0];
    if (keep1) keep1[c] = b[0];
  }
}

// train mode: dy = gamma*invstd*(dz - sum(dz)/P - xhat*sum(dz*xhat)/P); eval mode (flags bit 1: the
// normalisation used the running statistics, constants w.r.t. the input): dy = gamma*invstd*dz.
// Partial column sums of dy (conv bias grad).  flags bit 0: ReLU after the BN.
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const float* __restrict__ y, int ldy,
                                                           const float* __restrict__ da, int ldda,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const double* __restrict__ sdz,
                                                           const double* __restrict__ sdzx, long long P, int C,
                                                           int rows_per_blk, int relu, float* __restrict__ dy,
                                                           int lddy, float2* __restrict__ bias_part, unsigned* amax) {
  extern __shared__ float4 red4[];
  float mx = 0.f;
  int c4, r0, rs;
  thread_rc(C, &c4, &r0, &rs);
  const int active = (C >> 2) * rs;
  const int c = c4 * 4;
  float4 sb = make_float4(0.f, 0.f, 0.f, 0.f);
  if ((int)threadIdx.x < active) {
    const float4 mu = *reinterpret_cast<const float4*>(mean + c);
    const float4 is = *reinterpret_cast<const float4*>(invstd + c);
    const float4 g = *reinterpret_cast<const float4*>(gamma + c);
    const float4 b = *reinterpret_cast<const float4*>(beta + c);
    const double invP = (relu & 2) ? 0.0 : 1.0 / (double)P;
    float4 m1, m2, k;
    m1.x = (float)(sdz[c] * invP); m1.y = (float)(sdz[c + 1] * invP);
    m1.z = (float)(sdz[c + 2] * invP); m1.w = (float)(sdz[c + 3] * invP);
    m2.x = (float)(sdzx[c] * invP); m2.y = (float)(sdzx[c + 1] * invP);
    m2.z = (float)(sdzx[c + 2] * invP); m2.w = (float)(sdzx[c + 3] * invP);
    k.x = g.x * is.x; k.y = g.y * is.y; k.z = g.z * is.z; k.w = g.w * is.w;
    const long long pb = (long long)blockIdx.x * rows_per_blk;
    const long long pe = min(P, pb + rows_per_blk);
    auto row = [&](long long p, const float4& v, const float4& d) {
      float4 o;
      float xh, dz;
#define BN_APPLY(X)                                            \
  xh = (v.X - mu.X) * is.X;                                    \
  dz = (!(relu & 1) || xh * g.X + b.X > 0.f) ? d.X : 0.f;      \
  o.X = (dz - m1.X - xh * m2.X) * k.X;                         \
  sb.X += o.X;
      BN_APPLY(x) BN_APPLY(y) BN_APPLY(z) BN_APPLY(w)
#undef BN_APPLY
      *reinterpret_cast<float4*>(dy + p * lddy + c) = o;
      mx = fmaxf(mx, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
    };
    bn_rows(pb + r0, pe, rs, y, ldy, da, ldda, c, row);
  }
  if (amax) block_amax(mx, amax);
  if (bias_part == nullptr) return;
  red4[threadIdx.x] = sb;
  __syncthreads();
  if ((int)threadIdx.x < (C >> 2)) {
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int r = 0; r < rs; ++r) {
      const float4 a = red4[r * (C >> 2) + threadIdx.x];
      t.x += a.x; t.y += a.y; t.z += a.z; t.w += a.w;
    }
    float2* o = bias_part + (size_t)blockIdx.x * C + c;
    o[0] = make_float2(t.x, 0.f); o[1] = make_float2(t.y, 0.f);
    o[2] = make_float2(t.z, 0.f); o[3] = make_float2(t.w, 0.f);
  }
}

// The BN (+ReLU) backward apply of bn_bwd_apply_kernel (the same expressions, with the float m1 / m2
// of bn_bwd_coef_kernel) written as the h3 operand split of dy for the dgrad and weight gradient that
// consume it (srpde_conv_fwd_h3_presplit, srpde_conv_wgrad_h3p): dy * s = hi + lo, hi / lo fp16 planes
// [2][P][Cp], s = 2^h3_exp(dy_amax) from the rigorous bound of bn_bwd_coef_kernel -- no fp32 dy is
// written and the dgrad does no split work.  Cp = C rounded up to the 32-channel h3 chunk, channels
// C..Cp-1 zero (out_bn2's 16 channels: its dgrad and weight gradient then run on the h3 kernels).
// Each thread owns one channel quad of a run of rows.
__global__ __launch_bounds__(256) void bn_bwd_apply_split_kernel(const float* __restrict__ y, int ldy,
                                                                 const float* __restrict__ da, int ldda,
                                                                 const float* __restrict__ mean,
                                                                 const float* __restrict__ invstd,
                                                                 const float* __restrict__ gamma,
                                                                 const float* __restrict__ beta,
                                                                 const float* __restrict__ m1v,
                                                                 const float* __restrict__ m2v, long long P, int C,
                                                                 int Cp, int rows_per_blk, int relu,
                                                                 const unsigned* __restrict__ dy_amax,
                                                                 _Float16* __restrict__ planes) {
  typedef _Float16 half4 __attribute__((ext_vector_type(4)));
  int c4, r0, rs;
  thread_rc(Cp, &c4, &r0, &rs);
  if ((int)threadIdx.x >= (Cp >> 2) * rs) return;
  const int c = c4 * 4;
  const size_t plane = (size_t)P * Cp;
  const long long pb = (long long)blockIdx.x * rows_per_blk;
  const long long pe = min(P, pb + rows_per_blk);
  if (c >= C) {   // the zero channels padding the planes to Cp (a multiple of 32, the h3 chunk)
    const half4 z = {0, 0, 0, 0};
    for (long long p = pb + r0; p < pe; p += rs) {
      *reinterpret_cast<half4*>(planes + (size_t)p * Cp + c) = z;
      *reinterpret_cast<half4*>(planes + plane + (size_t)p * Cp + c) = z;
    }
    return;
  }
  const float4 mu = *reinterpret_cast<const float4*>(mean + c);
  const float4 is = *reinterpret_cast<const float4*>(invstd + c);
  const float4 g = *reinterpret_cast<const float4*>(gamma + c);
  const float4 b = *reinterpret_cast<const float4*>(beta + c);
  const float4 m1 = *reinterpret_cast<const float4*>(m1v + c);
  const float4 m2 = *reinterpret_cast<const float4*>(m2v + c);
  const float4 k = make_float4(g.x * is.x, g.y * is.y, g.z * is.z, g.w * is.w);
  const float s = exp2i(h3_exp(*dy_amax));
  auto row = [&](long long p, const float4& v, const float4& d) {
    float o[4];
    float xh, dz;
#define BN_APPLY_S(I, X)                                       \
  xh = (v.X - mu.X) * is.X;                                    \
  dz = (!(relu & 1) || xh * g.X + b.X > 0.f) ? d.X : 0.f;      \
  o[I] = (dz - m1.X - xh * m2.X) * k.X;
    BN_APPLY_S(0, x) BN_APPLY_S(1, y) BN_APPLY_S(2, z) BN_APPLY_S(3, w)
#undef BN_APPLY_S
    half4 hi, lo;
#pragma unroll
    for (int q = 0; q < 4; ++q) {   // conv_h3.hip split2h: hi = fp16(x s), lo = fp16(x s - hi)
      const float xs = o[q] * s;
      const _Float16 h = (_Float16)xs;
      hi[q] = h;
      lo[q] = (_Float16)(xs - (float)h);
    }
    *reinterpret_cast<half4*>(planes + (size_t)p * Cp + c) = hi;
    *reinterpret_cast<half4*>(planes + plane + (size_t)p * Cp + c) = lo;
  };
  bn_rows(pb + r0, pe, rs, y, ldy, da, ldda, c, row);
}

// The BN (+ReLU) backward's per-channel apply coefficients for a consumer that computes dy on the
// fly (srpde_conv_dgrad_h3_bnb): m1 = sum(dz)/P, m2 = sum(dz*xhat)/P as float, exactly as
// bn_bwd_apply_kernel forms them (0 in eval mode); the conv-bias gradient sum(dy) in fp64
// (= gamma*invstd*(sum dz - P*m1 - m2*sum xhat), sum xhat = 0 for train-mode batch statistics:
// 0 up to rounding, as the reference's autograd value); and a rigorous bound on max|dy| for the
// consumer's operand scale: |dy_c| <= |gamma_c invstd_c| (max|da| + |m1_c| + max|xhat| |m2_c|),
// max|xhat| <= sqrt(P-1) (Samuelson) in train mode.  One block.
__global__ __launch_bounds__(256) void bn_bwd_coef_kernel(const double* __restrict__ sdz, const double* __restrict__ sdzx,
                                                         long long P, int C, const float* __restrict__ invstd,
                                                         const float* __restrict__ gamma, int eval,
                                                         const float* __restrict__ da_max, int n_da_max,
                                                         float* __restrict__ m1, float* __restrict__ m2,
                                                         float* __restrict__ dbias, unsigned* dy_amax) {
  __shared__ float red[256];
  float a = 0.f;
  for (int k = threadIdx.x; k < n_da_max; k += 256) a = fmaxf(a, da_max[k]);
  red[threadIdx.x] = a;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + st]);
    __syncthreads();
  }
  const float amax_da = red[0];
  __syncthreads();
  const double invP = eval ? 0.0 : 1.0 / (double)P;
  const float xmax = eval ? 0.f : sqrtf((float)(P > 1 ? P - 1 : 1));
  float b = 0.f;
  for (int c = threadIdx.x; c < C; c += 256) {
    const float k = gamma[c] * invstd[c];
    const float a1 = (float)(sdz[c] * invP), a2 = (float)(sdzx[c] * invP);
    m1[c] = a1;
    m2[c] = a2;
    if (dbias) dbias[c] = (float)((double)k * (sdz[c] - (double)P * (double)a1 * (eval ? 0.0 : 1.0)));
    b = fmaxf(b, fabsf(k) * (amax_da + fabsf(a1) + xmax * fabsf(a2)));
  }
  red[threadIdx.x] = b;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + st]);
    __syncthreads();
  }
  if (threadIdx.x == 0) *dy_amax = __float_as_uint(red[0] * 1.0001f);   // covers the float rounding of the sum
}

// BN + ReLU of a ConvBlock output that a 2x2 max-pool reads next (models.py:79-80): each thread
// forms the four pixels of one pooling window for 4 channels with bn_relu_fwd_kernel's expressions,
// stores them, and stores their max in maxpool2_fwd's comparison order (first max wins) -- the pool
// no longer re-reads the activation.  amax: max|out| (the pooled tensor's bound as well).
__global__ __launch_bounds__(256) void bn_relu_pool_fwd_kernel(const float* __restrict__ y, int ldy,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ invstd,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, float* __restrict__ out,
                                                               int ldo, float* __restrict__ pool, int ldp, int n, int H,
                                                               int W, int C, int relu, unsigned* amax) {
  const int C4 = C >> 2, Wo = W >> 1, Ho = H >> 1;
  const long long total = (long long)n * Ho * Wo * C4;
  float mx = 0.f;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const long long q = e / C4;
    const int c = (int)(e - q * C4) * 4;
    const int ox = (int)(q % Wo);
    const long long t = q / Wo;
    const int oy = (int)(t % Ho);
    const long long nb = t / Ho;
    const long long p00 = (nb * H + 2 * oy) * W + 2 * ox;
    const long long pp[4] = {p00, p00 + 1, p00 + W, p00 + W + 1};
    const float4 mu = *reinterpret_cast<const float4*>(mean + c);
    const float4 is = *reinterpret_cast<const float4*>(invstd + c);
    const float4 g = *reinterpret_cast<const float4*>(gamma + c);
    const float4 b = *reinterpret_cast<const float4*>(beta + c);
    float4 o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 v = *reinterpret_cast<const float4*>(y + pp[k] * ldy + c);
      float4 r;
      r.x = (v.x - mu.x) * is.x * g.x + b.x;
      r.y = (v.y - mu.y) * is.y * g.y + b.y;
      r.z = (v.z - mu.z) * is.z * g.z + b.z;
      r.w = (v.w - mu.w) * is.w * g.w + b.w;
      if (relu) {
        r.x = fmaxf(r.x, 0.f); r.y = fmaxf(r.y, 0.f); r.z = fmaxf(r.z, 0.f); r.w = fmaxf(r.w, 0.f);
      }
      *reinterpret_cast<float4*>(out + pp[k] * ldo + c) = r;
      mx = fmaxf(mx, fmaxf(fmaxf(fabsf(r.x), fabsf(r.y)), fmaxf(fabsf(r.z), fabsf(r.w))));
      o[k] = r;
    }
    float4 m;
#define MX(X) { float v = o[0].X; if (o[1].X > v) v = o[1].X; if (o[2].X > v) v = o[2].X; if (o[3].X > v) v = o[3].X; m.X = v; }
    MX(x) MX(y) MX(z) MX(w)
#undef MX
    *reinterpret_cast<float4*>(pool + q * ldp + c) = m;
  }
  if (amax) block_amax(mx, amax);
}

// bn_relu_pool_fwd_kernel for one sample per block, which also forms the attention gate's channel
// branch of the activation (models.py:106-112, 119-121: m = mean over the pixels, h = relu(W1 m + b1),
// ca = sigmoid(W2 h + b2), as att_channel_fwd_kernel) from the sums of the values it writes, so the
// activation is not re-read for it.  C / 4 divides 256; Cr = C / 8.
template <bool POOL>
__global__ __launch_bounds__(256) void bn_relu_pool_att_fwd_kernel(
    const float* __restrict__ y, int ldy, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ out, int ldo,
    float* __restrict__ pool, int ldp, int H, int W, int C, unsigned* amax, const float* __restrict__ w1,
    const float* __restrict__ b1, const float* __restrict__ w2, const float* __restrict__ b2, float* __restrict__ mo,
    float* __restrict__ ho, float* __restrict__ cao) {
  __shared__ float4 red4[256];
  __shared__ float ms[256], hs[32];
  const int nb = blockIdx.x, C4 = C >> 2, Wo = W >> 1, Ho = H >> 1, Cr = C >> 3;
  const int c4 = threadIdx.x % C4, rs = 256 / C4, c = 4 * c4;
  const float4 mu = *reinterpret_cast<const float4*>(mean + c);
  const float4 is = *reinterpret_cast<const float4*>(invstd + c);
  const float4 g = *reinterpret_cast<const float4*>(gamma + c);
  const float4 b = *reinterpret_cast<const float4*>(beta + c);
  float mx = 0.f;
  float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
  const long long pbase = (long long)nb * H * W;
  constexpr int NPX = POOL ? 4 : 1;   // pixels per work item: a pooling window, or one pixel
  for (int q = threadIdx.x / C4; q < (POOL ? Ho * Wo : H * W); q += rs) {
    long long pp[4];
    if (POOL) {
      const int oy = q / Wo, ox = q - oy * Wo;
      const long long p00 = pbase + (long long)(2 * oy) * W + 2 * ox;
      pp[0] = p00; pp[1] = p00 + 1; pp[2] = p00 + W; pp[3] = p00 + W + 1;
    } else {
      pp[0] = pbase + q;
    }
    float4 o[4];
#pragma unroll
    for (int k = 0; k < NPX; ++k) {
      const float4 v = *reinterpret_cast<const float4*>(y + pp[k] * ldy + c);
      float4 r;
      r.x = fmaxf((v.x - mu.x) * is.x * g.x + b.x, 0.f);
      r.y = fmaxf((v.y - mu.y) * is.y * g.y + b.y, 0.f);
      r.z = fmaxf((v.z - mu.z) * is.z * g.z + b.z, 0.f);
      r.w = fmaxf((v.w - mu.w) * is.w * g.w + b.w, 0.f);
      if (out) *reinterpret_cast<float4*>(out + pp[k] * ldo + c) = r;
      mx = fmaxf(mx, fmaxf(fmaxf(r.x, r.y), fmaxf(r.z, r.w)));
      sum.x += r.x; sum.y += r.y; sum.z += r.z; sum.w += r.w;
      o[k] = r;
    }
    if (POOL) {
      float4 m;
#define MX(X) { float v = o[0].X; if (o[1].X > v) v = o[1].X; if (o[2].X > v) v = o[2].X; if (o[3].X > v) v = o[3].X; m.X = v; }
      MX(x) MX(y) MX(z) MX(w)
#undef MX
      *reinterpret_cast<float4*>(pool + ((long long)nb * Ho * Wo + q) * ldp + c) = m;
    }
  }
  if (amax) block_amax(mx, amax);
  red4[threadIdx.x] = sum;
  __syncthreads();
  if ((int)threadIdx.x < C4) {
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int r = 0; r < rs; ++r) {
      const float4 a = red4[r * C4 + threadIdx.x];
      t.x += a.x; t.y += a.y; t.z += a.z; t.w += a.w;
    }
    const float inv = 1.f / (float)(H * W);
    const int cc = threadIdx.x * 4;
    ms[cc] = t.x * inv; ms[cc + 1] = t.y * inv; ms[cc + 2] = t.z * inv; ms[cc + 3] = t.w * inv;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < C; j += blockDim.x) mo[(long long)nb * C + j] = ms[j];
  for (int r = threadIdx.x; r < Cr; r += blockDim.x) {
    float a = b1[r];
    for (int cc = 0; cc < C; ++cc) a += w1[r * C + cc] * ms[cc];
    a = fmaxf(a, 0.f);
    hs[r] = a;
    ho[(long long)nb * Cr + r] = a;
  }
  __syncthreads();
  for (int cc = threadIdx.x; cc < C; cc += blockDim.x) {
    float a = b2[cc];
    for (int r = 0; r < Cr; ++r) a += w2[cc * Cr + r] * hs[r];
    cao[(long long)nb * C + cc] = 1.f / (1.f + expf(-a));
  }
}

// BN + ReLU of the bridge output with the spatial attention of the gate it drives (models.py:44-48,
// 124-125: sa = sigmoid(conv1x1(b)) for att3, whose gating input b is): a pixel's channels are spread
// over whole waves (C / 4 >= 64 threads), its 1x1 conv reduced by shuffles and across the waves in
// LDS, so b is not re-read for it.  Few, long blocks for the max|out| atomic.
__global__ __launch_bounds__(256) void bn_relu_gate_fwd_kernel(const float* __restrict__ y, int ldy,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ invstd,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, float* __restrict__ out,
                                                               int ldo, long long P, int C, const float* __restrict__ wg,
                                                               const float* __restrict__ bg, float* __restrict__ sa,
                                                               unsigned* amax) {
  __shared__ float wred[4];
  const int C4 = C >> 2, ppb = 256 / C4, wpp = C4 >> 6;
  const int c = 4 * (threadIdx.x % C4), pl = threadIdx.x / C4, wave = threadIdx.x >> 6;
  const float4 mu = *reinterpret_cast<const float4*>(mean + c);
  const float4 is = *reinterpret_cast<const float4*>(invstd + c);
  const float4 g = *reinterpret_cast<const float4*>(gamma + c);
  const float4 b = *reinterpret_cast<const float4*>(beta + c);
  const float4 wv = *reinterpret_cast<const float4*>(wg + c);
  const float bias = bg[0];
  float mx = 0.f;
  for (long long p0 = (long long)blockIdx.x * ppb; p0 < P; p0 += (long long)gridDim.x * ppb) {
    const long long p = p0 + pl;
    float dot = 0.f;
    if (p < P) {
      const float4 v = *reinterpret_cast<const float4*>(y + p * ldy + c);
      float4 r;
      r.x = fmaxf((v.x - mu.x) * is.x * g.x + b.x, 0.f);
      r.y = fmaxf((v.y - mu.y) * is.y * g.y + b.y, 0.f);
      r.z = fmaxf((v.z - mu.z) * is.z * g.z + b.z, 0.f);
      r.w = fmaxf((v.w - mu.w) * is.w * g.w + b.w, 0.f);
      if (out) *reinterpret_cast<float4*>(out + p * ldo + c) = r;
      mx = fmaxf(mx, fmaxf(fmaxf(r.x, r.y), fmaxf(r.z, r.w)));
      dot = r.x * wv.x + r.y * wv.y + r.z * wv.z + r.w * wv.w;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o, 64);
    if ((threadIdx.x & 63) == 0) wred[wave] = dot;
    __syncthreads();
    if ((threadIdx.x % C4) == 0 && p < P) {
      float t = 0.f;
      for (int k = 0; k < wpp; ++k) t += wred[pl * wpp + k];
      sa[p] = 1.f / (1.f + expf(-(t + bias)));
    }
    __syncthreads();
  }
  if (amax) block_amax(mx, amax);
}

// The gradient of an encoder block's output e = relu(bn2(y)) in one pass, and that BatchNorm's backward reduction:
// e feeds both the AttentionGate of its skip connection (models.py:119-130, :93 / :90) and the 2x2 max-pool of the
// next block (:79-80), so de = (dout * sa) * ca + dm (the gate's input gradient, att_bwd_dx_kernel's expression) plus
// the pooled gradient routed to each window's first maximum (maxpool2_bwd_px_kernel's comparison order).  Before:
// att_bwd_dx wrote de, maxpool2_bwd read it back and rewrote it, and bn_bwd_reduce read it a third time; here it is
// written once and the partial sums (sum dz, sum dz * xhat; bn_bwd_reduce_kernel's expressions, per thread in a
// fixed pixel order) and the per-block max|de| leave with it.  de is equal bit for bit to the three-pass result.
// Block (C / 4, 256 / (C / 4)): one channel quad of one pooling window per thread, a grid-stride walk over windows.
__global__ __launch_bounds__(256) void att_pool_bn_bwd_kernel(
    const float* __restrict__ dout, int lddo, const float* __restrict__ ca, const float* __restrict__ sa,
    const float* __restrict__ dm, const float* __restrict__ a, int lda, const float* __restrict__ dp, int lddp,
    const float* __restrict__ y, int ldy, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ de, int ldde, int H, int W,
    unsigned npool, float2* __restrict__ part, float* __restrict__ da_max) {
  extern __shared__ float4 red4[];   // [2][256]
  const int C4 = blockDim.x, C = 4 * C4, c = threadIdx.x * 4;
  const unsigned Wo = W >> 1, Ho = H >> 1, HW = (unsigned)(H * W);
  const float4 mu = *reinterpret_cast<const float4*>(mean + c);
  const float4 is = *reinterpret_cast<const float4*>(invstd + c);
  const float4 g = *reinterpret_cast<const float4*>(gamma + c);
  const float4 b = *reinterpret_cast<const float4*>(beta + c);
  float4 s1 = make_float4(0.f, 0.f, 0.f, 0.f), s2 = s1;
  float dmax = 0.f;
  for (unsigned q = blockIdx.x * blockDim.y + threadIdx.y; q < npool; q += gridDim.x * blockDim.y) {
    const unsigned ox = q % Wo, t = q / Wo, oy = t % Ho, n = t / Ho;
    const size_t p0 = ((size_t)n * H + 2 * oy) * W + 2 * ox;
    const size_t p[4] = {p0, p0 + 1, p0 + W, p0 + W + 1};
    float4 v[4], d[4], yv[4];
    float sv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k] = *reinterpret_cast<const float4*>(a + p[k] * lda + c);
      d[k] = *reinterpret_cast<const float4*>(dout + p[k] * lddo + c);
      yv[k] = *reinterpret_cast<const float4*>(y + p[k] * ldy + c);
      sv[k] = sa[p[k]];
    }
    const float4 gp = *reinterpret_cast<const float4*>(dp + (size_t)q * lddp + c);
    const float4 cav = *reinterpret_cast<const float4*>(ca + (size_t)n * C + c);
    const float4 dmv = *reinterpret_cast<const float4*>(dm + (size_t)n * C + c);
    (void)HW;
    float4 o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float s = sv[k];
      o[k].x = (d[k].x * s) * cav.x + dmv.x; o[k].y = (d[k].y * s) * cav.y + dmv.y;
      o[k].z = (d[k].z * s) * cav.z + dmv.z; o[k].w = (d[k].w * s) * cav.w + dmv.w;
    }
    // (the routed add by selects, not o[am]: a dynamic index put o in scratch)
#define ARG(X)                                                     \
  {                                                                \
    int am = 0; float mv = v[0].X;                                 \
    if (v[1].X > mv) { mv = v[1].X; am = 1; }                      \
    if (v[2].X > mv) { mv = v[2].X; am = 2; }                      \
    if (v[3].X > mv) { mv = v[3].X; am = 3; }                      \
    o[0].X = am == 0 ? o[0].X + gp.X : o[0].X;                     \
    o[1].X = am == 1 ? o[1].X + gp.X : o[1].X;                     \
    o[2].X = am == 2 ? o[2].X + gp.X : o[2].X;                     \
    o[3].X = am == 3 ? o[3].X + gp.X : o[3].X;                     \
  }
    ARG(x) ARG(y) ARG(z) ARG(w)
#undef ARG
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      *reinterpret_cast<float4*>(de + p[k] * ldde + c) = o[k];
      dmax = fmaxf(dmax, fmaxf(fmaxf(fabsf(o[k].x), fabsf(o[k].y)), fmaxf(fabsf(o[k].z), fabsf(o[k].w))));
      float xh, dz;
#define BN_ACC(X)                                              \
  xh = (yv[k].X - mu.X) * is.X;                                \
  dz = (xh * g.X + b.X > 0.f) ? o[k].X : 0.f;                  \
  s1.X += dz;                                                  \
  s2.X += dz * xh;
      BN_ACC(x) BN_ACC(y) BN_ACC(z) BN_ACC(w)
#undef BN_ACC
    }
  }
  const int tid = threadIdx.y * C4 + threadIdx.x;
  red4[tid] = s1;
  red4[256 + tid] = s2;
  __syncthreads();
  if (threadIdx.y == 0) {
    float4 t1 = make_float4(0.f, 0.f, 0.f, 0.f), t2 = t1;
    for (int r = 0; r < (int)blockDim.y; ++r) {
      const float4 u1 = red4[r * C4 + threadIdx.x], u2 = red4[256 + r * C4 + threadIdx.x];
      t1.x += u1.x; t1.y += u1.y; t1.z += u1.z; t1.w += u1.w;
      t2.x += u2.x; t2.y += u2.y; t2.z += u2.z; t2.w += u2.w;
    }
    float2* o2 = part + (size_t)blockIdx.x * C + c;
    o2[0] = make_float2(t1.x, t2.x); o2[1] = make_float2(t1.y, t2.y);
    o2[2] = make_float2(t1.z, t2.z); o2[3] = make_float2(t1.w, t2.w);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) dmax = fmaxf(dmax, __shfl_xor(dmax, o, 64));
  __syncthreads();
  float* wmx = reinterpret_cast<float*>(red4);
  if ((tid & 63) == 0) wmx[tid >> 6] = dmax;
  __syncthreads();
  if (tid == 0) da_max[blockIdx.x] = fmaxf(fmaxf(wmx[0], wmx[1]), fmaxf(wmx[2], wmx[3]));
}

static int att_pool_blocks(int n, int h, int w, int c) {
  const long long npool = (long long)n * (h / 2) * (w / 2);
  const int py = 256 / (c / 4);
  return (int)std::min<long long>(1024, (npool + py - 1) / py);
}

static int bwd_blocks(long long P, int C, int* rows_per_blk) {
  // ~1024 blocks; rows per block a multiple of the rows a block covers per sweep
  const int rs = 256 / (C >> 2);
  long long rpb = (P + 1023) / 1024;
  rpb = (rpb + rs - 1) / rs * rs;
  if (rpb < rs) rpb = rs;
  *rows_per_blk = (int)rpb;
  return (int)((P + rpb - 1) / rpb);
}

}  // namespace srpde

using namespace srpde;

extern "C" {

int srpde_bn_train_finalize(const float* stats, int nblk, int rows_per_blk, long long P, int C,
                            float* running_mean, float* running_var, long long* num_batches_tracked,
                            float momentum, float eps, float* mean_out, float* invstd_out, hipStream_t stream) {
  SRPDE_CHECK_ARG(stats && mean_out && invstd_out && C > 0 && nblk > 0, "srpde_bn_train_finalize: bad args");
  hipLaunchKernelGGL(bn_train_finalize_kernel, dim3(C), dim3(FIN_T), 0, stream,
                     reinterpret_cast<const float2*>(stats), nblk, rows_per_blk, P, C, running_mean, running_var,
                     momentum, eps, mean_out, invstd_out, num_batches_tracked);
  SRPDE_LAUNCH_CHECK("srpde_bn_train_finalize");
  return 0;
}

int srpde_bn_train_finalize_affine(const float* stats, int nblk, int rows_per_blk, long long P, int C,
                                   float* running_mean, float* running_var, long long* num_batches_tracked,
                                   float momentum, float eps, float* mean_out, float* invstd_out, const float* gamma,
                                   const float* beta, float* scale, float* shift, unsigned* amax_bound,
                                   hipStream_t stream) {
  SRPDE_CHECK_ARG(stats && mean_out && invstd_out && gamma && beta && scale && shift && C > 0 && nblk > 0 && P > 0,
                  "srpde_bn_train_finalize_affine: bad args");
  hipLaunchKernelGGL(bn_train_finalize_kernel, dim3(C), dim3(FIN_T), 0, stream,
                     reinterpret_cast<const float2*>(stats), nblk, rows_per_blk, P, C, running_mean, running_var,
                     momentum, eps, mean_out, invstd_out, num_batches_tracked, gamma, beta, scale, shift, amax_bound,
                     (float)sqrt((double)(P - 1)));
  SRPDE_LAUNCH_CHECK("srpde_bn_train_finalize_affine");
  return 0;
}

size_t srpde_bn_finalize_workspace_size(int nblk, int C) {
  (void)nblk;   // (the slice count is capped; the partial count only sets the slice length)
  return (size_t)FIN_SPLIT_MAX * (C > 0 ? C : 0) * 3 * sizeof(double);
}

int srpde_bn_train_finalize_ws(const float* stats, int nblk, int rows_per_blk, long long P, int C, float* running_mean,
                               float* running_var, long long* num_batches_tracked, float momentum, float eps,
                               float* mean_out, float* invstd_out, const float* gamma, const float* beta, float* scale,
                               float* shift, unsigned* amax_bound, void* workspace, size_t ws_bytes,
                               hipStream_t stream) {
  SRPDE_CHECK_ARG(stats && mean_out && invstd_out && workspace && C > 0 && nblk > 0 && P > 0 && rows_per_blk > 0,
                  "srpde_bn_train_finalize_ws: bad args");
  SRPDE_CHECK_ARG((scale == nullptr) == (shift == nullptr) && (scale == nullptr || (gamma && beta)),
                  "srpde_bn_train_finalize_ws: scale / shift need gamma / beta");
  if (ws_bytes < srpde_bn_finalize_workspace_size(nblk, C)) {
    set_error("srpde_bn_train_finalize_ws: workspace %zu < %zu bytes", ws_bytes, srpde_bn_finalize_workspace_size(nblk, C));
    return kErrWorkspace;
  }
  const long long nfull_ll = P / rows_per_blk;
  const int nfull = (int)(nfull_ll < nblk ? nfull_ll : nblk);
  const int nsl = fin_slices(nfull, C);
  const int rows = nfull > 0 ? ceil_div(nfull, nsl) : 0;
  double* ws = static_cast<double*>(workspace);
  hipLaunchKernelGGL(bn_stats_split_kernel, dim3(ceil_div(C, 16), nsl), dim3(256), 0, stream,
                     reinterpret_cast<const float2*>(stats), nfull, rows, C, ws);
  SRPDE_LAUNCH_CHECK("srpde_bn_train_finalize_ws(slices)");
  hipLaunchKernelGGL(bn_finalize_split_kernel, dim3(C), dim3(64), 0, stream,
                     reinterpret_cast<const float2*>(stats), ws, nsl, nblk, rows_per_blk, P, C, running_mean,
                     running_var, momentum, eps, mean_out, invstd_out, num_batches_tracked, gamma, beta, scale, shift,
                     scale ? amax_bound : nullptr, (float)sqrt((double)(P - 1)));
  SRPDE_LAUNCH_CHECK("srpde_bn_train_finalize_ws");
  return 0;
}

int srpde_bn_eval_prepare(const float* running_mean, const float* running_var, int C, float eps, float* mean_out,
                          float* invstd_out, hipStream_t stream) {
  SRPDE_CHECK_ARG(running_mean && running_var && mean_out && invstd_out, "srpde_bn_eval_prepare: null");
  hipLaunchKernelGGL(bn_eval_prepare_kernel, dim3(ceil_div(C, 256)), dim3(256), 0, stream, running_mean,
                     running_var, C, eps, mean_out, invstd_out);
  SRPDE_LAUNCH_CHECK("srpde_bn_eval_prepare");
  return 0;
}

int srpde_bn_relu_fwd(const float* y, int ldy, const float* mean, const float* invstd, const float* gamma,
                      const float* beta, float* out, int ldo, long long P, int C, int relu, unsigned* amax,
                      hipStream_t stream) {
  SRPDE_CHECK_ARG(y && mean && invstd && gamma && beta && out, "srpde_bn_relu_fwd: null");
  SRPDE_CHECK_ARG(C % 4 == 0 && ldy % 4 == 0 && ldo % 4 == 0, "srpde_bn_relu_fwd: C/ld must be multiples of 4");
  const long long total = P * (C / 4);
  // with an amax word: fewer, longer blocks (one same-address atomic per block)
  const int blocks = (int)std::min<long long>((total + 255) / 256, amax ? 1024 : 8192);
  hipLaunchKernelGGL(bn_relu_fwd_kernel, dim3(blocks), dim3(256), 0, stream, y, ldy, mean, invstd, gamma, beta,
                     out, ldo, P, C, relu, amax);
  SRPDE_LAUNCH_CHECK("srpde_bn_relu_fwd");
  return 0;
}

int srpde_bn_relu_pool_fwd(const float* y, int ldy, const float* mean, const float* invstd, const float* gamma,
                           const float* beta, float* out, int ldo, float* pool, int ldp, int n, int h, int w, int C,
                           int relu, unsigned* amax, hipStream_t stream) {
  SRPDE_CHECK_ARG(y && mean && invstd && gamma && beta && out && pool, "srpde_bn_relu_pool_fwd: null");
  SRPDE_CHECK_ARG(C % 4 == 0 && ldy % 4 == 0 && ldo % 4 == 0 && ldp % 4 == 0 && h % 2 == 0 && w % 2 == 0,
                  "srpde_bn_relu_pool_fwd: C / ld must be multiples of 4, h and w even");
  const long long total = (long long)n * (h / 2) * (w / 2) * (C / 4);
  const int blocks = (int)std::min<long long>((total + 255) / 256, amax ? 1024 : 8192);
  hipLaunchKernelGGL(bn_relu_pool_fwd_kernel, dim3(blocks), dim3(256), 0, stream, y, ldy, mean, invstd, gamma, beta,
                     out, ldo, pool, ldp, n, h, w, C, relu, amax);
  SRPDE_LAUNCH_CHECK("srpde_bn_relu_pool_fwd");
  return 0;
}

int srpde_bn_relu_pool_att_fwd(const float* y, int ldy, const float* mean, const float* invstd, const float* gamma,
                               const float* beta, float* out, int ldo, float* pool, int ldp, int n, int h, int w,
                               int C, unsigned* amax, const float* w1, const float* b1, const float* w2,
                               const float* b2, float* m, float* hbuf, float* ca, hipStream_t stream) {
  SRPDE_CHECK_ARG(y && mean && invstd && gamma && beta && w1 && b1 && w2 && b2 && m && hbuf && ca,
                  "srpde_bn_relu_pool_att_fwd: null");   // out nullable: the activation is not written
  SRPDE_CHECK_ARG(C % 32 == 0 && C <= 256 && 256 % (C / 4) == 0 && ldy % 4 == 0 && ldo % 4 == 0 &&
                      (pool == nullptr || (ldp % 4 == 0 && h % 2 == 0 && w % 2 == 0)),
                  "srpde_bn_relu_pool_att_fwd: C a multiple of 32 <= 256, ld multiples of 4, h and w even");
  if (pool)
    hipLaunchKernelGGL(bn_relu_pool_att_fwd_kernel<true>, dim3(n), dim3(256), 0, stream, y, ldy, mean, invstd, gamma,
                       beta, out, ldo, pool, ldp, h, w, C, amax, w1, b1, w2, b2, m, hbuf, ca);
  else
    hipLaunchKernelGGL(bn_relu_pool_att_fwd_kernel<false>, dim3(n), dim3(256), 0, stream, y, ldy, mean, invstd, gamma,
                       beta, out, ldo, pool, ldp, h, w, C, amax, w1, b1, w2, b2, m, hbuf, ca);
  SRPDE_LAUNCH_CHECK("srpde_bn_relu_pool_att_fwd");
  return 0;
}

int srpde_bn_relu_gate_fwd(const float* y, int ldy, const float* mean, const float* invstd, const float* gamma,
                           const float* beta, float* out, int ldo, long long P, int C, const float* wg,
                           const float* bg, float* sa, unsigned* amax, hipStream_t stream) {
  SRPDE_CHECK_ARG(y && mean && invstd && gamma && beta && wg && bg && sa, "srpde_bn_relu_gate_fwd: null");   // out nullable
  SRPDE_CHECK_ARG((C == 256 || C == 512 || C == 1024) && ldy % 4 == 0 && ldo % 4 == 0,
                  "srpde_bn_relu_gate_fwd: C 256, 512 or 1024, ld multiples of 4");
  const long long ppb = 256 / (C / 4);
  const int blocks = (int)std::min<long long>((P + ppb - 1) / ppb, 1024);
  hipLaunchKernelGGL(bn_relu_gate_fwd_kernel, dim3(blocks), dim3(256), 0, stream, y, ldy, mean, invstd, gamma, beta,
                     out, ldo, P, C, wg, bg, sa, amax);
  SRPDE_LAUNCH_CHECK("srpde_bn_relu_gate_fwd");
  return 0;
}

int srpde_bn_affine(const float* mean, const float* invstd, const float* gamma, const float* beta, int C, long long P,
                    float* scale, float* shift, unsigned* amax_bound, hipStream_t stream) {
  SRPDE_CHECK_ARG(mean && invstd && gamma && beta && scale && shift && C > 0 && P > 0, "srpde_bn_affine: bad args");
  hipLaunchKernelGGL(bn_affine_kernel, dim3(1), dim3(256), 0, stream, mean, invstd, gamma, beta, C,
                     (float)sqrt((double)(P - 1)), scale, shift, amax_bound);
  SRPDE_LAUNCH_CHECK("srpde_bn_affine");
  return 0;
}

size_t srpde_bn_relu_bwd_workspace_size(long long P, int C) {
  int rpb;
  const int nblk = bwd_blocks(P, C, &rpb);
  return (size_t)nblk * C * sizeof(float2) * 2 + (size_t)C * sizeof(double) * 2;
}

int srpde_bn_relu_bwd(const float* y, int ldy, const float* da, int ldda, const float* mean, const float* invstd,
                      const float* gamma, const float* beta, float* dy, int lddy, float* dgamma, float* dbeta,
                      float* dbias, long long P, int C, int relu, unsigned* amax, void* workspace,
                      size_t ws_bytes, hipStream_t stream) {
  SRPDE_CHECK_ARG(y && da && mean && invstd && gamma && beta && dy && workspace, "srpde_bn_relu_bwd: null");
  SRPDE_CHECK_ARG(C % 4 == 0 && C <= 1024 && ldy % 4 == 0 && ldda % 4 == 0 && lddy % 4 == 0,
                  "srpde_bn_relu_bwd: C/ld must be multiples of 4 (C<=1024)");
  int rpb;
  const int nblk = bwd_blocks(P, C, &rpb);
  const size_t need = srpde_bn_relu_bwd_workspace_size(P, C);
  if (ws_bytes < need) {
    set_error("srpde_bn_relu_bwd: workspace %zu < %zu", ws_bytes, need);
    return kErrWorkspace;
  }
  float2* part = static_cast<float2*>(workspace);
  float2* bpart = part + (size_t)nblk * C;
  double* sdz = reinterpret_cast<double*>(bpart + (size_t)nblk * C);
  double* sdzx = sdz + C;
  const size_t lds = 2 * 256 * sizeof(float4);
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(nblk), dim3(256), lds, stream, y, ldy, da, ldda, mean, invstd,
                     gamma, beta, P, C, rpb, relu, part);
  SRPDE_LAUNCH_CHECK("srpde_bn_relu_bwd(reduce)");
  hipLaunchKernelGGL(colsum2_kernel, dim3(C), dim3(256), 0, stream, part, nblk, C, dbeta, dgamma, sdz, sdzx);
  SRPDE_LAUNCH_CHECK("srpde_bn_relu_bwd(colsum)");
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(nblk), dim3(256), lds, stream, y, ldy, da, ldda, mean, invstd,
                     gamma, beta, sdz, sdzx, P, C, rpb, relu, dy, lddy, dbias ? bpart : nullptr, amax);
  SRPDE_LAUNCH_CHECK("srpde_bn_relu_bwd(apply)");
  if (dbias) {
    hipLaunchKernelGGL(colsum2_kernel, dim3(C), dim3(256), 0, stream, bpart, nblk, C, dbias, (float*)nullptr,
                       (double*)nullptr, (double*)nullptr);
    SRPDE_LAUNCH_CHECK("srpde_bn_relu_bwd(bias)");
  }
  return 0;
}

int srpde_bn_relu_bwd_part(const float* y, int ldy, const float* da, int ldda, const float* mean, const float* invstd,
                           const float* gamma, const float* beta, float* dy, int lddy, float* dgamma, float* dbeta,
                           float* dbias, long long P, int C, int relu, unsigned* amax, const void* part, int nblk,
                           void* workspace, size_t ws_bytes, hipStream_t stream) {
  SRPDE_CHECK_ARG(y && da && mean && invstd && gamma && beta && dy && workspace && part && nblk > 0,
                  "srpde_bn_relu_bwd_part: null");
  SRPDE_CHECK_ARG(C % 4 == 0 && C <= 1024 && ldy % 4 == 0 && ldda % 4 == 0 && lddy % 4 == 0,
                  "srpde_bn_relu_bwd_part: C/ld must be multiples of 4 (C<=1024)");
  int rpb;
  const int ablk = bwd_blocks(P, C, &rpb);
  const size_t need = srpde_bn_relu_bwd_workspace_size(P, C);
  if (ws_bytes < need) {
    set_error("srpde_bn_relu_bwd_part: workspace %zu < %zu", ws_bytes, need);
    return kErrWorkspace;
  }
  float2* bpart = static_cast<float2*>(workspace) + (size_t)ablk * C;
  double* sdz = reinterpret_cast<double*>(bpart + (size_t)ablk * C);
  double* sdzx = sdz + C;
  hipLaunchKernelGGL(colsum2_kernel, dim3(C), dim3(256), 0, stream, static_cast<const float2*>(part), nblk, C, dbeta,
                     dgamma, sdz, sdzx);
  SRPDE_LAUNCH_CHECK("srpde_bn_relu_bwd_part(colsum)");
  const size_t lds = 2 * 256 * sizeof(float4);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(ablk), dim3(256), lds, stream, y, ldy, da, ldda, mean, invstd, gamma,
                     beta, sdz, sdzx, P, C, rpb, relu, dy, lddy, dbias ? bpart : nullptr, amax);
  SRPDE_LAUNCH_CHECK("srpde_bn_relu_bwd_part(apply)");
  if (dbias) {
    hipLaunchKernelGGL(colsum2_kernel, dim3(C), dim3(256), 0, stream, bpart, ablk, C, dbias, (float*)nullptr,
                       (double*)nullptr, (double*)nullptr);
    SRPDE_LAUNCH_CHECK("srpde_bn_relu_bwd_part(bias)");
  }
  return 0;
}

// Everything the fused dgrad (srpde_conv_dgrad_h3_bnb) needs to apply this BN's backward on the
// fly: dgamma, dbeta, dbias, the float m1 / m2 vectors and the dy operand-scale bound word.  `part`:
// the (sum dz, sum dz*xhat) partials already produced by the dgrad that wrote da (nblk row blocks,
// with that dgrad's per-tile max|da| in da_max[n_da_max]); null: one reduction pass over y and da
// here (which also takes max|da|).  flags: SRPDE_BN_RELU | SRPDE_BN_EVAL.
int srpde_bn_bwd_apply_split(const float* y, int ldy, const float* da, int ldda, const float* mean,
                             const float* invstd, const float* gamma, const float* beta, const float* m1,
                             const float* m2, long long P, int C, int flags, const unsigned* dy_amax, void* planes,
                             hipStream_t stream) {
  SRPDE_CHECK_ARG(y && da && mean && invstd && gamma && beta && m1 && m2 && dy_amax && planes && P > 0,
                  "srpde_bn_bwd_apply_split: null argument");
  SRPDE_CHECK_ARG(C % 4 == 0 && C <= 1024 && ldy % 4 == 0 && ldda % 4 == 0 && aligned16(y) && aligned16(da) &&
                      aligned16(planes), "srpde_bn_bwd_apply_split: C / ld multiples of 4, 16-byte aligned");
  const int Cp = (C + 31) / 32 * 32;
  int rpb;
  const int nblk = bwd_blocks(P, Cp, &rpb);
  hipLaunchKernelGGL(bn_bwd_apply_split_kernel, dim3(nblk), dim3(256), 0, stream, y, ldy, da, ldda, mean, invstd,
                     gamma, beta, m1, m2, P, C, Cp, rpb, flags & SRPDE_BN_RELU, dy_amax, static_cast<_Float16*>(planes));
  SRPDE_LAUNCH_CHECK("srpde_bn_bwd_apply_split");
  return 0;
}

size_t srpde_bn_bwd_prepare_workspace_size(long long P, int C) {
  int rpb;
  const int nblk = bwd_blocks(P, C, &rpb);
  return (size_t)nblk * C * sizeof(float2) + (size_t)C * sizeof(double) * 2 + (size_t)nblk * sizeof(float) + 64;
}

int srpde_bn_bwd_prepare(const float* y, int ldy, const float* da, int ldda, const float* mean, const float* invstd,
                         const float* gamma, const float* beta, long long P, int C, int flags, const void* part,
                         int nblk_part, const float* da_max, int n_da_max, float* m1, float* m2, float* dgamma,
                         float* dbeta, float* dbias, unsigned* dy_amax, void* workspace, size_t ws_bytes,
                         hipStream_t stream) {
  SRPDE_CHECK_ARG(y && da && mean && invstd && gamma && beta && m1 && m2 && dy_amax && workspace && P > 0,
                  "srpde_bn_bwd_prepare: null argument");
  SRPDE_CHECK_ARG(C % 4 == 0 && C <= 1024 && ldy % 4 == 0 && ldda % 4 == 0, "srpde_bn_bwd_prepare: C / ld");
  SRPDE_CHECK_ARG(part == nullptr || (da_max && n_da_max > 0 && nblk_part > 0),
                  "srpde_bn_bwd_prepare: fused partials need the producer's max|da| slots");
  if (ws_bytes < srpde_bn_bwd_prepare_workspace_size(P, C)) {
    set_error("srpde_bn_bwd_prepare: workspace too small");
    return kErrWorkspace;
  }
  int rpb;
  const int nblk = bwd_blocks(P, C, &rpb);
  float2* wpart = static_cast<float2*>(workspace);
  double* sdz = reinterpret_cast<double*>(wpart + (size_t)nblk * C);
  double* sdzx = sdz + C;
  float* wmax = reinterpret_cast<float*>(sdzx + C);
  const float2* use_part = static_cast<const float2*>(part);
  int np = nblk_part;
  if (part == nullptr) {
    const size_t lds = 2 * 256 * sizeof(float4);
    hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(nblk), dim3(256), lds, stream, y, ldy, da, ldda, mean, invstd,
                       gamma, beta, P, C, rpb, flags & SRPDE_BN_RELU, wpart, wmax);
    SRPDE_LAUNCH_CHECK("srpde_bn_bwd_prepare(reduce)");
    use_part = wpart;
    np = nblk;
    da_max = wmax;
    n_da_max = nblk;
  }
  hipLaunchKernelGGL(colsum2_kernel, dim3(C), dim3(256), 0, stream, use_part, np, C, dbeta, dgamma, sdz, sdzx);
  SRPDE_LAUNCH_CHECK("srpde_bn_bwd_prepare(colsum)");
  hipLaunchKernelGGL(bn_bwd_coef_kernel, dim3(1), dim3(256), 0, stream, sdz, sdzx, P, C, invstd, gamma,
                     (flags & SRPDE_BN_EVAL) ? 1 : 0, da_max, n_da_max, m1, m2, dbias, dy_amax);
  SRPDE_LAUNCH_CHECK("srpde_bn_bwd_prepare(coef)");
  return 0;
}

int srpde_gating_bn_reduce_blocks(long long P, int C) {
  int rpb;
  return bwd_blocks(P, C, &rpb);
}

int srpde_gating_bn_reduce(const float* dsa, const float* wg, float* dg, int lddg, const float* y, int ldy,
                           const float* mean, const float* invstd, const float* gamma, const float* beta, long long P,
                           int C, int flags, void* part, float* da_max, hipStream_t stream) {
  SRPDE_CHECK_ARG(dsa && wg && dg && y && mean && invstd && gamma && beta && part && da_max && P > 0,
                  "srpde_gating_bn_reduce: null argument");
  SRPDE_CHECK_ARG(C % 4 == 0 && C <= 1024 && (256 % (C / 4)) == 0 && lddg % 4 == 0 && ldy % 4 == 0 && aligned16(dg) &&
                      aligned16(y),
                  "srpde_gating_bn_reduce: C / 4 must divide 256, row strides multiples of 4, 16-byte aligned");
  int rpb;
  const int nblk = bwd_blocks(P, C, &rpb);
  hipLaunchKernelGGL(gating_bn_reduce_kernel, dim3(nblk), dim3(256), 2 * 256 * sizeof(float4), stream, dsa, wg, dg, lddg,
                     y, ldy, mean, invstd, gamma, beta, P, C, rpb, flags & SRPDE_BN_RELU, static_cast<float2*>(part),
                     da_max);
  SRPDE_LAUNCH_CHECK("srpde_gating_bn_reduce");
  return 0;
}

int srpde_att_pool_bn_bwd_blocks(int n, int h, int w, int c) { return att_pool_blocks(n, h, w, c); }

int srpde_att_pool_bn_bwd(const float* dout, int lddo, const float* ca, const float* sa, const float* dm, const float* a,
                          int lda, const float* dp, int lddp, const float* y, int ldy, const float* mean,
                          const float* invstd, const float* gamma, const float* beta, float* de, int ldde, int n, int h,
                          int w, int c, void* part, float* da_max, hipStream_t stream) {
  SRPDE_CHECK_ARG(dout && ca && sa && dm && a && dp && y && mean && invstd && gamma && beta && de && part && da_max,
                  "srpde_att_pool_bn_bwd: null argument");
  const int c4 = c / 4;
  SRPDE_CHECK_ARG(c % 4 == 0 && c4 >= 1 && c4 <= 64 && (c4 & (c4 - 1)) == 0 && h % 2 == 0 && w % 2 == 0 &&
                      lddo % 4 == 0 && lda % 4 == 0 && lddp % 4 == 0 && ldy % 4 == 0 && ldde % 4 == 0 &&
                      (long long)n * h * w < (1LL << 31),
                  "srpde_att_pool_bn_bwd: c / 4 a power of two <= 64, even h / w, row strides multiples of 4");
  const int nb = att_pool_blocks(n, h, w, c);
  hipLaunchKernelGGL(att_pool_bn_bwd_kernel, dim3(nb), dim3(c4, 256 / c4), 2 * 256 * sizeof(float4), stream, dout,
                     lddo, ca, sa, dm, a, lda, dp, lddp, y, ldy, mean, invstd, gamma, beta, de, ldde, h, w,
                     (unsigned)(n * (h / 2) * (w / 2)), static_cast<float2*>(part), da_max);
  SRPDE_LAUNCH_CHECK("srpde_att_pool_bn_bwd");
  return 0;
}

}  // extern "C"
