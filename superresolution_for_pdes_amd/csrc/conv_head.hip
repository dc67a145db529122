// The U-Net's output head in inference, one pass: out_conv2 (3x3, 32 -> 16) -> out_bn2 with its
// running statistics -> ReLU -> final (1x1, 16 -> 1) -> + the coarse input channel
// (src/models.py:59-61, 98-101 in eval mode).  out_conv2 has 16 output channels: on the 64- / 128-column
// convolution tiles half or more of every MFMA was padding, and its 105 MB output was written only for
// the head to read it back (h3r 0.25 ms + head 26 us at batch 1024).
//
// One workgroup (4 waves) per 128 output pixels: the split halo tile of the 32 input channels (h3: the
// operand scaled by 2^h3_exp(max|z|) and cut into fp16 hi / lo pieces, 160-B rows as h4's S tile) is
// built once in LDS; each wave owns 32 pixels x all 16 channels, with the 9 taps' weight fragments (both
// planes) held in 72 VGPRs for the whole tile, and runs h3's three MFMAs per tap and 16-row block
// (al*bh, ah*bl, ah*bh -- the 16x16x32 product order of conv_fwd_h4 / h3r, one 32-channel chunk), so the
// conv values equal the h3 kernels'.  The epilogue undoes the operand scales, adds the bias, applies
// BN + ReLU (ep_bn_relu), dots the 16 channels with the final weights across the 16 lanes that hold a
// pixel's row and adds the residual.
#include "conv_h3.h"

namespace srpde {

struct HeadArgs {
  const float* z; int ldz;          // [P][32] the head's input (out_conv1's activation)
  const unsigned* amax;             // max|z| word
  const _Float16* wsp;              // [2][16][288] out_conv2's h3 weight planes
  const int* wexp;                  // [16]
  const float* bias;                // [16] or null
  const float* mean; const float* invstd; const float* gamma; const float* beta;   // out_bn2 (eval)
  const float* wf; const float* bf; // final 1x1 [16], [1]
  const float* xin; int xin_c;      // the U-Net input, NCHW: the residual is channel 0
  int N, H, W, P;
  float* out;                       // [P]
};

// 128-pixel tiles: the 34 KiB halo tile lets four workgroups share a CU, so one's loads overlap the
// others' MFMAs (256-pixel tiles, two per CU: 184 us at batch 1024, latency-bound)
constexpr int HEAD_BM = 128, HEAD_SR = 160, HEAD_RB = HEAD_BM / 64;   // 16-row blocks per wave
constexpr int HEAD_IT = 4;   // halo-tile tasks per thread: (128 + 2 (w + 1)) * 4 <= 4 * 256, w <= 63

__global__ __launch_bounds__(256, 3) void conv_head_eval_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, lq = lane >> 4;
  const int W = a.W, HW = a.H * a.W, halo = W + 1, arows = HEAD_BM + 2 * halo;
  const int zrel = arows * HEAD_SR;   // a zero 16-B x 8 row for taps outside the image
  const int m0 = blockIdx.x * HEAD_BM, pix0 = m0 - halo;
  const int ea = h3_exp(*a.amax);
  const float sa = exp2i(ea);

  // the weight fragments: B[k][n] = W[n][tap][k], lane (n = l16, k = 8 lq .. 8 lq + 7), both planes
  half8 bh[9], bl[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const size_t o = (size_t)l16 * 288 + t * 32 + lq * 8;
    bh[t] = *reinterpret_cast<const half8*>(a.wsp + o);
    bl[t] = *reinterpret_cast<const half8*>(a.wsp + 16 * 288 + o);
  }
  // the channel scale to undo and the BN / head constants of this lane's channel n = l16: loaded with
  // the tile, not after the MFMAs
  const int we = a.wexp[l16], e = ea + we;
  const float bn = a.bias ? a.bias[l16] : 0.f;
  const float mu = a.mean[l16], is = a.invstd[l16], ga = a.gamma[l16], be = a.beta[l16], wfn = a.wf[l16];
  const float bfv = a.bf[0];
  // the split halo tile: task (row r, 8 channels c8); rows outside the tensor are zero.  Every task's
  // loads are issued before any is split (HEAD_IT tasks per thread: w <= 63), not one round trip each
  if (tid < 32) reinterpret_cast<float*>(lds + zrel)[tid] = 0.f;
  float4 v[HEAD_IT][2];
#pragma unroll
  for (int k = 0; k < HEAD_IT; ++k) {
    const int sg = tid + 256 * k, r = sg >> 2, c8 = sg & 3;
    const int pix = pix0 + r;
    v[k][0] = v[k][1] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (sg < arows * 4 && pix >= 0 && pix < a.P) {
      v[k][0] = *reinterpret_cast<const float4*>(a.z + (size_t)pix * a.ldz + c8 * 8);
      v[k][1] = *reinterpret_cast<const float4*>(a.z + (size_t)pix * a.ldz + c8 * 8 + 4);
    }
  }
#pragma unroll
  for (int k = 0; k < HEAD_IT; ++k) {
    const int sg = tid + 256 * k, r = sg >> 2, c8 = sg & 3;
    if (sg < arows * 4) {
      half8 hv, lv;
      split2h(v[k][0], v[k][1], sa, hv, lv);
      *reinterpret_cast<half8*>(lds + r * HEAD_SR + c8 * 16) = hv;
      *reinterpret_cast<half8*>(lds + r * HEAD_SR + 64 + c8 * 16) = lv;
    }
  }
  __syncthreads();

  const bool wide = e > 126 || e < -126;
  const float ia = exp2i(-ea), cs = wide ? exp2i(-we) : exp2i(-e);

#pragma unroll
  for (int i = 0; i < HEAD_RB; ++i) {
    const int rr = wave * (16 * HEAD_RB) + i * 16 + l16;   // this lane's A row (pixel) in the tile
    const int m = m0 + rr;
    int yy = -(1 << 20), xx = 0;
    if (m < a.P) {
      const int rem = m % HW;
      yy = rem / W;
      xx = rem - yy * W;
    }
    floatx4 part;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ky = t / 3, kx = t % 3;
      const int iy = yy + ky - 1, ix = xx + kx - 1;
      const bool ok = iy >= 0 && iy < a.H && ix >= 0 && ix < W;
      const int o = ok ? (rr + ky * W + kx) * HEAD_SR + lq * 16 : zrel;
      const half8 ah = *reinterpret_cast<const half8*>(lds + o);
      const half8 al = *reinterpret_cast<const half8*>(lds + o + 64);
      floatx4 c0 = t == 0 ? __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[t], floatx4{}, 0, 0, 0)
                          : __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[t], part, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[t], c0, 0, 0, 0);
      part = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[t], c0, 0, 0, 0);
    }
    // lane holds D[4 lq + r][l16]: pixel m0 + 16 (HEAD_RB wave + i) + 4 lq + r, channel l16
    float s[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = wide ? part[r] * ia : part[r];
      v = __builtin_fmaf(v, cs, bn);
      v = ep_bn_relu(v, mu, is, ga, be);
      s[r] = v * wfn;
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
      for (int r = 0; r < 4; ++r) s[r] += __shfl_xor(s[r], o, 64);
    if (l16 == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = m0 + wave * (16 * HEAD_RB) + i * 16 + lq * 4 + r;
        if (p < a.P) {
          const int nn = p / HW, q = p - nn * HW;
          a.out[p] = (s[r] + bfv) + a.xin[(size_t)nn * a.xin_c * HW + q];
        }
      }
    }
  }
}

// out_conv2 in training (src/models.py:58, 99: conv 32 -> 16 feeding out_bn2 with batch statistics), the
// forward of srpde_conv_fwd_h3 for that shape: the eval head's tile and MFMA layout (128 pixels per
// workgroup, the 32-channel split halo tile in LDS, 16 output channels per wave with the nine taps' weight
// fragments in registers -- no padding of the 16 channels to a 32- or 64-column tile) with the training
// epilogue of the conv kernels: y (16 channels), the (mean, M2) BN partials of the 128-row block (the
// srpde_conv_h3_stats_rows_for block of this shape) and the stored input split (H3Args::xsplit) for the
// weight gradient; out_bn1's BN + ReLU (H3Args::in_scale / in_shift) is applied in the split.  Same
// products in the same order as h3r's 32-column tile, so y equals it bit for bit (tests/test_gpu_h5.py).
__global__ __launch_bounds__(256, 3) void conv_fwd_n16_kernel(ConvParams p, H3Args h) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, lq = lane >> 4;
  const int W = p.W, HW = p.H * p.W, halo = W + 1, arows = HEAD_BM + 2 * halo;
  const int zrel = arows * HEAD_SR;
  float* red = reinterpret_cast<float*>(lds + zrel + 128);   // [4 waves][16] cross-wave sums
  const int m0 = blockIdx.x * HEAD_BM, pix0 = m0 - halo;
  const int ea = h3_exp(*h.amax0);
  const float sa = exp2i(ea);
  half8 bh[9], bl[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const size_t o = (size_t)l16 * 288 + t * 32 + lq * 8;
    bh[t] = *reinterpret_cast<const half8*>(h.wsp + o);
    bl[t] = *reinterpret_cast<const half8*>(h.wsp + 16 * 288 + o);
  }
  const int we = h.wexp[l16], e = ea + we;
  const float bn = p.bias ? p.bias[l16] : 0.f;
  if (tid < 32) reinterpret_cast<float*>(lds + zrel)[tid] = 0.f;
  float4 v[HEAD_IT][2];
#pragma unroll
  for (int k = 0; k < HEAD_IT; ++k) {
    const int sg = tid + 256 * k, r = sg >> 2, c8 = sg & 3;
    const int pix = pix0 + r;
    v[k][0] = v[k][1] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (sg < arows * 4 && pix >= 0 && pix < p.P) {
      v[k][0] = *reinterpret_cast<const float4*>(p.x0 + (size_t)pix * p.ldx0 + c8 * 8);
      v[k][1] = *reinterpret_cast<const float4*>(p.x0 + (size_t)pix * p.ldx0 + c8 * 8 + 4);
    }
  }
  const size_t xplane = (size_t)p.P * 32;
#pragma unroll
  for (int k = 0; k < HEAD_IT; ++k) {
    const int sg = tid + 256 * k, r = sg >> 2, c8 = sg & 3;
    if (sg < arows * 4) {
      const int pix = pix0 + r;
      const bool inside = pix >= 0 && pix < p.P;
      float4 a0 = v[k][0], a1 = v[k][1];
      if (h.in_scale != nullptr) {   // the producer's BN + ReLU; rows outside the tensor stay 0
        const float4 s0 = *reinterpret_cast<const float4*>(h.in_scale + c8 * 8);
        const float4 s1 = *reinterpret_cast<const float4*>(h.in_scale + c8 * 8 + 4);
        const float4 t0 = *reinterpret_cast<const float4*>(h.in_shift + c8 * 8);
        const float4 t1 = *reinterpret_cast<const float4*>(h.in_shift + c8 * 8 + 4);
#define N16_AFF(V, S, T, X) V.X = inside ? fmaxf(V.X * S.X + T.X, 0.f) : 0.f;
        N16_AFF(a0, s0, t0, x) N16_AFF(a0, s0, t0, y) N16_AFF(a0, s0, t0, z) N16_AFF(a0, s0, t0, w)
        N16_AFF(a1, s1, t1, x) N16_AFF(a1, s1, t1, y) N16_AFF(a1, s1, t1, z) N16_AFF(a1, s1, t1, w)
#undef N16_AFF
      }
      half8 hv, lv;
      split2h(a0, a1, sa, hv, lv);
      *reinterpret_cast<half8*>(lds + r * HEAD_SR + c8 * 16) = hv;
      *reinterpret_cast<half8*>(lds + r * HEAD_SR + 64 + c8 * 16) = lv;
      if (h.xsplit != nullptr && r >= halo && r < halo + HEAD_BM && inside) {   // the tile's own rows
        _Float16* o = h.xsplit + (size_t)pix * 32 + c8 * 8;
        *reinterpret_cast<half8*>(o) = hv;
        *reinterpret_cast<half8*>(o + xplane) = lv;
      }
    }
  }
  __syncthreads();

  const bool wide = e > 126 || e < -126;
  const float ia = exp2i(-ea), cs = wide ? exp2i(-we) : exp2i(-e);
  float yv[HEAD_RB][4];
#pragma unroll
  for (int i = 0; i < HEAD_RB; ++i) {
    const int rr = wave * (16 * HEAD_RB) + i * 16 + l16;   // this lane's A row (pixel) in the tile
    const int m = m0 + rr;
    int yy = -(1 << 20), xx = 0;
    if (m < p.P) {
      const int rem = m % HW;
      yy = rem / W;
      xx = rem - yy * W;
    }
    floatx4 part;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ky = t / 3, kx = t % 3;
      const int iy = yy + ky - 1, ix = xx + kx - 1;
      const bool ok = iy >= 0 && iy < p.H && ix >= 0 && ix < W;
      const int o = ok ? (rr + ky * W + kx) * HEAD_SR + lq * 16 : zrel;
      const half8 ah = *reinterpret_cast<const half8*>(lds + o);
      const half8 al = *reinterpret_cast<const half8*>(lds + o + 64);
      floatx4 c0 = t == 0 ? __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[t], floatx4{}, 0, 0, 0)
                          : __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[t], part, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[t], c0, 0, 0, 0);
      part = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[t], c0, 0, 0, 0);
    }
    // lane holds D[4 lq + r][l16]: pixel m0 + 16 (HEAD_RB wave + i) + 4 lq + r, channel l16
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int px = m0 + wave * (16 * HEAD_RB) + i * 16 + lq * 4 + r;
      const float y = __builtin_fmaf(wide ? part[r] * ia : part[r], cs, bn);
      yv[i][r] = y;
      if (px < p.P) p.y[(size_t)px * p.ldy + l16] = y;
    }
  }
  if (p.stats == nullptr) return;
  // (mean, M2) of channel l16 over the block's valid rows: lane sums, the 4 lq lanes of a channel, then the
  // 4 waves through LDS (two passes: the mean first)
  const int cnt = min(HEAD_BM, p.P - m0);
  auto chan_sum = [&](float t) {
    t += __shfl_xor(t, 16, 64);
    t += __shfl_xor(t, 32, 64);
    if (lq == 0) red[wave * 16 + l16] = t;
    __syncthreads();
    const float s = (red[l16] + red[16 + l16]) + (red[32 + l16] + red[48 + l16]);
    __syncthreads();
    return s;
  };
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < HEAD_RB; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int px = m0 + wave * (16 * HEAD_RB) + i * 16 + lq * 4 + r;
      if (px < p.P) t += yv[i][r];
    }
  const float mean = chan_sum(t) / (float)cnt;
  t = 0.f;
#pragma unroll
  for (int i = 0; i < HEAD_RB; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int px = m0 + wave * (16 * HEAD_RB) + i * 16 + lq * 4 + r;
      const float d = yv[i][r] - mean;
      if (px < p.P) t = __builtin_fmaf(d, d, t);
    }
  const float m2 = chan_sum(t);
  if (tid < 16) p.stats[(size_t)blockIdx.x * 16 + tid] = make_float2(mean, m2);
}

bool n16_supported(int c0, int c1, int cout, int w, int dil) {
  return c0 == 32 && c1 == 0 && cout == 16 && dil == 1 && w > 0 && w <= 63 &&
         (size_t)(HEAD_BM + 2 * (w + 1)) * HEAD_SR + 128 + 256 <= 80 * 1024;
}

int launch_fwd_n16(const ConvParams& p, const H3Args& h, hipStream_t st) {
  const size_t lds = (size_t)(HEAD_BM + 2 * (p.W + 1)) * HEAD_SR + 128 + 256;
  note_kernel("conv_fwd_n16_kernel");
  hipLaunchKernelGGL(conv_fwd_n16_kernel, dim3(ceil_div(p.P, HEAD_BM)), dim3(256), lds, st, p, h);
  SRPDE_LAUNCH_CHECK("srpde_conv_fwd_h3(n16)");
  return 0;
}

}  // namespace srpde

using namespace srpde;

extern "C" {

int srpde_conv_head_eval_supported(int w) {
  return (w > 0 && w <= 63 && (size_t)(HEAD_BM + 2 * (w + 1)) * HEAD_SR + 128 <= 80 * 1024) ? 1 : 0;
}

int srpde_conv_head_eval(const float* z, int ldz, const unsigned* amax_z, const void* wsplit, const int* wexp,
                         const float* bias, const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                         const float* bn_beta, const float* wf, const float* bf, const float* xin, int xin_c, int n,
                         int h, int w, float* out, hipStream_t stream) {
  SRPDE_CHECK_ARG(z && amax_z && wsplit && wexp && bn_mean && bn_invstd && bn_gamma && bn_beta && wf && bf && xin &&
                      out && xin_c >= 1,
                  "srpde_conv_head_eval: null pointer");
  SRPDE_CHECK_ARG(n > 0 && h > 0 && w > 0 && (long long)n * h * w < (1LL << 31) && ldz % 4 == 0 && ldz >= 32 &&
                      aligned16(z) && aligned16(wsplit),
                  "srpde_conv_head_eval: bad shape / stride / alignment");
  HeadArgs a;
  a.z = z; a.ldz = ldz; a.amax = amax_z;
  a.wsp = static_cast<const _Float16*>(wsplit); a.wexp = wexp; a.bias = bias;
  a.mean = bn_mean; a.invstd = bn_invstd; a.gamma = bn_gamma; a.beta = bn_beta;
  a.wf = wf; a.bf = bf; a.xin = xin; a.xin_c = xin_c;
  a.N = n; a.H = h; a.W = w; a.P = n * h * w; a.out = out;
  const size_t lds = (size_t)(HEAD_BM + 2 * (w + 1)) * HEAD_SR + 128;
  SRPDE_CHECK_ARG(srpde_conv_head_eval_supported(w), "srpde_conv_head_eval: image rows too wide for the tile (w=%d > 63)",
                  w);
  note_kernel("conv_head_eval_kernel");
  hipLaunchKernelGGL(conv_head_eval_kernel, dim3(ceil_div(a.P, HEAD_BM)), dim3(256), lds, stream, a);
  SRPDE_LAUNCH_CHECK("srpde_conv_head_eval");
  return 0;
}

}  // extern "C"
