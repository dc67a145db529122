// Implicit-GEMM 3x3 / 1x1 convolution for gfx950 on fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces the aten convolution / convolution_backward calls that reference
// src/models.py makes through nn.Conv2d (ConvBlock.conv1/conv2 models.py:16,18;
// bridge[0],[3] models.py:43,46 with dilation 2; out_conv1/2 models.py:57,59).
//
//   forward :  Y[p][n] = bias[n] + sum_{t,c} X[p + sign*off(t)][c] * Wp[n][t][c]
//   dgrad   :  the same kernel with sign = -1 and Wd[c][t][n] = W[n][c][t]
//   wgrad   :  dW[n][t][c] = sum_p dY[p][n] * X[p + off(t)][c]   (split-K over pixels,
//              deterministic slab reduction -- no float atomics)
//
// X may be a *virtual concat* of two NHWC views (x0: c0 channels, x1: c1 channels) so
// torch.cat in UNet.forward (models.py:87,90,93) never materialises.  The forward
// epilogue adds the bias, stores Y and emits per-(row-block, channel) BatchNorm
// partial statistics (block mean, block M2) for the train-mode BN that always follows
// (models.py:22-23,44,47,96-97): the batch statistics never re-read Y from HBM.
#include "conv_common.h"

namespace srpde {



constexpr int BK = 16;      // k (tap*Cin + c) per stage
constexpr int LDK = BK + 4; // padded LDS row: conflict-free ds_read_b128 over 32 rows


template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256) void conv_igemm_fwd_kernel(ConvParams p) {
  constexpr int TM = BM / WM, TN = BN / WN, TI = TM / 32, TJ = TN / 32;
  constexpr int A_LOADS = BM / 64;                         // float4 per thread per stage
  constexpr int B_ROWS_PER_PASS = 64;
  constexpr int B_LOADS = BN >= 64 ? BN / 64 : 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* As = smem;                        // [2][BM][LDK]
  float* Bs = smem + 2 * BM * LDK;         // [2][BN][LDK]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wmi = wave % WM, wni = wave / WM;
  const int nbn = (p.Cout + BN - 1) / BN;
  const int nbm = (p.P + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, nbm * nbn);
  const int mt = wg / nbn, nt = wg - mt * nbn;
  const int m0 = mt * BM, n0 = nt * BN;
  const int HW = p.H * p.W;
  const int kc = p.ksize >> 1;

  // per-thread A rows (pixel coordinates), fixed for the whole K loop
  const int col4 = tid & 3;
  int a_nb[A_LOADS], a_y[A_LOADS], a_x[A_LOADS];
#pragma unroll
  for (int i = 0; i < A_LOADS; ++i) {
    const int m = m0 + (tid >> 2) + i * 64;
    if (m < p.P) {
      const int n = m / HW, rem = m - n * HW, yy = rem / p.W;
      a_nb[i] = n * HW; a_y[i] = yy; a_x[i] = rem - yy * p.W;
    } else {
      a_nb[i] = -1; a_y[i] = 0; a_x[i] = 0;
    }
  }

  float4 ra[A_LOADS], rb[B_LOADS];
  auto load_stage = [&](int s) {
    const int k = s * BK + col4 * 4;
    int tap = 0, c = 0;
    bool kin = k < p.K;
    if (kin) { tap = k / p.Cin; c = k - tap * p.Cin; }
    const int ky = tap / p.ksize, kx = tap - ky * p.ksize;
    const int oy = (ky - kc) * p.dil * p.sign, ox = (kx - kc) * p.dil * p.sign;
    const float* src; int ld, cc;
    if (c < p.c0) { src = p.x0; ld = p.ldx0; cc = c; } else { src = p.x1; ld = p.ldx1; cc = c - p.c0; }
#pragma unroll
    for (int i = 0; i < A_LOADS; ++i) {
      const int iy = a_y[i] + oy, ix = a_x[i] + ox;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (kin && a_nb[i] >= 0 && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W)
        v = *reinterpret_cast<const float4*>(src + (size_t)(a_nb[i] + iy * p.W + ix) * ld + cc);
      ra[i] = v;
    }
#pragma unroll
    for (int j = 0; j < B_LOADS; ++j) {
      const int row = (tid >> 2) + j * B_ROWS_PER_PASS;
      const int nn = n0 + row;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row < BN && nn < p.Cout && kin)
        v = *reinterpret_cast<const float4*>(p.w + (size_t)nn * p.K + k);
      rb[j] = v;
    }
  };
  auto store_stage = [&](int buf) {
    float* a = As + buf * BM * LDK;
    float* b = Bs + buf * BN * LDK;
#pragma unroll
    for (int i = 0; i < A_LOADS; ++i)
      *reinterpret_cast<float4*>(a + ((tid >> 2) + i * 64) * LDK + col4 * 4) = ra[i];
#pragma unroll
    for (int j = 0; j < B_LOADS; ++j) {
      const int row = (tid >> 2) + j * B_ROWS_PER_PASS;
      if (row < BN) *reinterpret_cast<float4*>(b + row * LDK + col4 * 4) = rb[j];
    }
  };

  floatx16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nsteps = (p.K + BK - 1) / BK;
  load_stage(0);
  store_stage(0);
  __syncthreads();

  const int lr = lane & 31, lh = lane >> 5;
  const int wm0 = wmi * TM, wn0 = wni * TN;
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) load_stage(s + 1);
    const float* a = As + buf * BM * LDK;
    const float* b = Bs + buf * BN * LDK;
    // two-level accumulation: each stage's 16-term MFMA chain starts from zero and is
    // then added into the running sum, so fp32 rounding grows ~sqrt(16)+sqrt(K/16)
    // instead of ~sqrt(K) (matches mkldnn's blocked accumulation accuracy)
    floatx16 part[TI][TJ];
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      const int kk = g * 8 + lh * 4;
      float4 av[TI], bv[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) av[i] = *reinterpret_cast<const float4*>(a + (wm0 + i * 32 + lr) * LDK + kk);
#pragma unroll
      for (int j = 0; j < TJ; ++j) bv[j] = *reinterpret_cast<const float4*>(b + (wn0 + j * 32 + lr) * LDK + kk);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const floatx16 c0 = g == 0 ? floatx16{} : part[i][j];
          part[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].x, bv[j].x, c0, 0, 0, 0);
          part[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].y, bv[j].y, part[i][j], 0, 0, 0);
          part[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].z, bv[j].z, part[i][j], 0, 0, 0);
          part[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].w, bv[j].w, part[i][j], 0, 0, 0);
        }
    }
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] += part[i][j];
    if (s + 1 < nsteps) store_stage(buf ^ 1);
    __syncthreads();
  }

  // ---------------- epilogue: bias, (eval) BN + ReLU, store, BN partial statistics -------------
  // the shared h3 epilogue (conv_common.h): 16-B row stores through LDS (the K loop ended with a
  // barrier, LDS is free), per-SRB-row statistics, the eval-mode BN + ReLU and max word (ep_*)
  x6_finish<BM, BN, WM, WN, BM>(p, acc, false, wg, nbm * nbn, 0, m0, n0, wmi, wni, lane, smem,
                                (p.ldy % 4 == 0 && (reinterpret_cast<uintptr_t>(p.y) & 15) == 0)
                                    ? smem + 2 * WM * TI * BN : nullptr);
}

// ------------------ the 4-channel-input 3x3 forward (enc1.conv1, models.py:16) ------------------
// The U-Net's first conv reads the 3-channel input (padded to 4, the zero 4th channel meeting zero
// weights) and writes 64 channels: K = 9 taps x 4 channels is far too short for the K-chunked kernels
// (conv_igemm_fwd_kernel: 278 us at B = 1024, ~1.5 TB/s), and the pass is bound by the 64-channel
// write.  Here a wave owns 64 pixels x 64 output channels and keeps the whole 64 x 36 weight tile in
// registers: per tap it loads one fp32 of its 16 pixels' 4 channels per lane straight into the MFMA
// operand (16-B pixels, a 256-B contiguous wave load) and runs 16 v_mfma_f32_16x16x4_f32 (weights as
// the A operand, so a lane's accumulator is 4 consecutive channels of one pixel: 16-B row stores).
// Epilogue: bias, the eval-mode BN + ReLU and max word (ep_*), BN partial statistics per 256 rows
// (a workgroup's 4 waves), the same (mean, M2) layout as the other forward kernels.
typedef float c4x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256, 3) void conv_fwd_c4_kernel(ConvParams p) {
  constexpr int NPB = 4, NCB = 4;                  // 16-pixel blocks per wave, 16-channel blocks per tile
  __shared__ float red[4][64];
  __shared__ __attribute__((aligned(16))) float stg[4][16 * 68];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l16 = lane & 15, lg = lane >> 4;       // B column (pixel) / K row (channel); D row group
  const int m0 = blockIdx.x * 256, n0 = blockIdx.y * 64;
  const int HW = p.H * p.W;
  // the weight tile as A operands: W[n0 + 16 cb + l16][tap][lg]
  float wa[9][NCB];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) wa[t][cb] = p.w[(size_t)(n0 + cb * 16 + l16) * 36 + t * 4 + lg];
  int pn[NPB], py[NPB], px[NPB];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    const int m = m0 + wave * 64 + pb * 16 + l16;
    if (m < p.P) {
      const int nn = m / HW, rem = m - nn * HW;
      pn[pb] = nn * HW; py[pb] = rem / p.W; px[pb] = rem - py[pb] * p.W;
    } else {
      pn[pb] = -1; py[pb] = 0; px[pb] = 0;
    }
  }
  c4x4 acc[NPB][NCB];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb)
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) acc[pb][cb] = c4x4{0.f, 0.f, 0.f, 0.f};
  // every tap's operand loads issued before the first MFMA (unconditional loads of a clamped address,
  // the out-of-image ones zeroed after): one memory round trip per wave instead of one per tap
  float xb[9][NPB];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int oy = (t / 3 - 1) * p.dil * p.sign, ox = (t % 3 - 1) * p.dil * p.sign;
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb) {
      const int iy = py[pb] + oy, ix = px[pb] + ox;
      const bool ok = pn[pb] >= 0 && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
      const float v = p.x0[(size_t)(ok ? pn[pb] + iy * p.W + ix : 0) * 4 + lg];
      xb[t][pb] = ok ? v : 0.f;
    }
  }
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
        acc[pb][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t][cb], xb[t][pb], acc[pb][cb], 0, 0, 0);
  // lane: pixel m0 + 64 wave + 16 pb + l16, channels n0 + 16 cb + 4 lg + 0..3
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    const int c = n0 + cb * 16 + lg * 4;
    const float4 b4 = p.bias ? *reinterpret_cast<const float4*>(p.bias + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 mu, is, ga, be;
    if (p.ep_mean) {
      mu = *reinterpret_cast<const float4*>(p.ep_mean + c);
      is = *reinterpret_cast<const float4*>(p.ep_invstd + c);
      ga = *reinterpret_cast<const float4*>(p.ep_gamma + c);
      be = *reinterpret_cast<const float4*>(p.ep_beta + c);
    }
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb) {
      c4x4& v = acc[pb][cb];
      v[0] += b4.x; v[1] += b4.y; v[2] += b4.z; v[3] += b4.w;
      if (p.ep_mean) {
        v[0] = ep_bn_relu(v[0], mu.x, is.x, ga.x, be.x);
        v[1] = ep_bn_relu(v[1], mu.y, is.y, ga.y, be.y);
        v[2] = ep_bn_relu(v[2], mu.z, is.z, ga.z, be.z);
        v[3] = ep_bn_relu(v[3], mu.w, is.w, ga.w, be.w);
      }
    }
  }
  // the output leaves through a per-wave LDS stage, 16 pixels at a time: a lane holds 4 channels of one
  // pixel per accumulator (64-B pieces of 16 rows per store instruction); staged, each store
  // instruction writes 4 whole 256-B rows (rows padded to 68 floats: conflict-free 16-B writes)
  float* st = stg[wave];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
      *reinterpret_cast<float4*>(st + l16 * 68 + cb * 16 + lg * 4) =
          make_float4(acc[pb][cb][0], acc[pb][cb][1], acc[pb][cb][2], acc[pb][cb][3]);
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's stage writes are done
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int row = k * 4 + (lane >> 4), c4 = (lane & 15) * 4;
      const float4 v = *reinterpret_cast<const float4*>(st + row * 68 + c4);
      const int m = m0 + wave * 64 + pb * 16 + row;
      if (m < p.P) *reinterpret_cast<float4*>(p.y + (size_t)m * p.ldy + n0 + c4) = v;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // the reads are back before the next block overwrites the stage
    __builtin_amdgcn_wave_barrier();
  }
  if (p.ep_amax != nullptr) {
    float mx = 0.f;
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
        if (pn[pb] >= 0)
#pragma unroll
          for (int r = 0; r < 4; ++r) mx = fmaxf(mx, fabsf(acc[pb][cb][r]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    if (lane == 0) red[wave][0] = mx;
    __syncthreads();
    if (threadIdx.x == 0)
      atomicMax(p.ep_amax, __float_as_uint(fmaxf(fmaxf(red[0][0], red[1][0]), fmaxf(red[2][0], red[3][0]))));
  }
  if (p.stats == nullptr) return;
  // statistics of the workgroup's 256 rows: per channel the mean, then M2 about it
  const int cnt = min(256, p.P - m0);
  float mean[NCB][4];
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = 0.f;
#pragma unroll
        for (int pb = 0; pb < NPB; ++pb) {
          const float v = acc[pb][cb][r];
          if (pass == 0) {
            s += pn[pb] >= 0 ? v : 0.f;
          } else {
            const float d = v - mean[cb][r];
            s = pn[pb] >= 0 ? __builtin_fmaf(d, d, s) : s;
          }
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) s += __shfl_xor(s, o, 64);
        if (l16 == 0) red[wave][cb * 16 + lg * 4 + r] = s;
      }
    __syncthreads();
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int cl = cb * 16 + lg * 4 + r;
        const float t = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
        if (pass == 0) mean[cb][r] = t / (float)cnt;
        else if (wave == 0 && l16 == 0) p.stats[(size_t)blockIdx.x * p.Cout + n0 + cl] = make_float2(mean[cb][r], t);
      }
    __syncthreads();
  }
}

static bool c4_ok(const ConvParams& p) {
  // Cout % 128 != 0: the 256-row statistics blocks srpde_conv_stats_rows_per_block gives those widths
  return p.ksize == 3 && p.c0 == 4 && p.c1 == 0 && p.ldx0 == 4 && p.Cout % 64 == 0 && p.Cout % 128 != 0 &&
         p.ldy % 4 == 0 &&
         (reinterpret_cast<uintptr_t>(p.y) & 15) == 0 && !p.accumulate;
}

static int launch_fwd_c4(const ConvParams& p, hipStream_t st) {
  note_kernel("conv_fwd_c4_kernel");
  hipLaunchKernelGGL(conv_fwd_c4_kernel, dim3(ceil_div(p.P, 256), p.Cout / 64), dim3(256), 0, st, p);
  SRPDE_LAUNCH_CHECK("srpde_conv_fwd(c4)");
  return 0;
}

// ---------------------- forward v2: LDS-DMA staged, BK = 32 ----------------------
// For Cin % 32 == 0 (every layer but enc1.conv1 fwd and out_conv2 dgrad).  Operand tiles
// go HBM/L2 -> LDS with buffer_load ... lds (no VGPR staging, no ds_write): each wave
// instruction fills 1 KiB lane-linearly; the 16-B chunk a lane fetches is pre-swizzled
// on the SOURCE side (chunk c of row r sits in slot c ^ ((r>>1)&7)) so the ds_read_b128
// operand reads are bank-conflict free.  Out-of-image taps (zero padding) and rows past
// P / Cout use an out-of-range buffer offset: the hardware range check returns zeros.

template <int BM, int BN, int WM, int WN, int HP>
__global__ __launch_bounds__(256, 2) void conv_fwd_v2_kernel(ConvParams p) {
  constexpr int TM = BM / WM, TN = BN / WN, TI = TM / 32, TJ = TN / 32;
  constexpr int AI = BM / 32;   // A wave-instructions (1 KiB each) per wave per stage
  constexpr int BI = BN / 32;   // B wave-instructions per wave per stage
  constexpr int STAGE = (BM + BN) * ROW2;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* lds = reinterpret_cast<char*>(smem);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wmi = wave % WM, wni = wave / WM;
  const int nbn = (p.Cout + BN - 1) / BN;
  const int nbm = (p.P + BM - 1) / BM;
  // tiles [0, nfull) whole (XCD-aware order); the last ntail tiles as tsplit K-pieces each,
  // so the final partially-filled round of workgroups is spread over more CUs
  const int nfull = nbm * nbn - p.ntail;
  int wg, piece = 0;
  if ((int)blockIdx.x < nfull) {
    wg = xcd_remap(blockIdx.x, nfull);
  } else {
    const int q = blockIdx.x - nfull;
    wg = nfull + q / p.tsplit;
    piece = q - (q / p.tsplit) * p.tsplit;
  }
  const bool tail = wg >= nfull;
  const int mt = wg / nbn, nt = wg - mt * nbn;
  const int m0 = mt * BM, n0 = nt * BN;
  const int HW = p.H * p.W;
  const int kc = p.ksize >> 1;

  const int32x4 rs0 = make_rsrc(p.x0, (unsigned)((size_t)p.P * p.ldx0 * 4));
  const int32x4 rs1 = make_rsrc(p.c1 ? p.x1 : p.x0, (unsigned)((size_t)p.P * (p.c1 ? p.ldx1 : p.ldx0) * 4));
  const int32x4 rsw = make_rsrc(p.w, (unsigned)((size_t)p.Cout * p.K * 4));

  // per-lane A rows, fixed over the K loop: byte offset of (pixel, swizzled chunk) in each
  // source, and a bitmask of the taps whose shifted pixel lies inside the image (padding)
  unsigned a_o0[AI], a_o1[AI], a_mask[AI];
  const int ld1 = p.c1 ? p.ldx1 : p.ldx0;
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int q = (wave * AI + i) * 64 + lane;
    const int r = q >> 3;
    const int c4 = swz(r, q & 7) * 4;
    const int m = m0 + r;
    unsigned mask = 0;
    int pix = 0;
    if (m < p.P) {
      const int n = m / HW, rem = m - n * HW, yy = rem / p.W, xx = rem - yy * p.W;
      pix = m;
      for (int t = 0; t < p.ksize * p.ksize; ++t) {
        const int ky = t / p.ksize, kx = t - ky * p.ksize;
        const int iy = yy + (ky - kc) * p.dil * p.sign, ix = xx + (kx - kc) * p.dil * p.sign;
        if (iy >= 0 && iy < p.H && ix >= 0 && ix < p.W) mask |= 1u << t;
      }
      (void)n;
    }
    a_mask[i] = mask;
    a_o0[i] = (unsigned)((pix * p.ldx0 + c4) * 4);
    a_o1[i] = (unsigned)((pix * ld1 + c4) * 4);
  }
  int b_off[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int q = (wave * BI + j) * 64 + lane;
    const int r = q >> 3;
    const int nn = n0 + r;
    b_off[j] = nn < p.Cout ? (nn * p.K + swz(r, q & 7) * 4) * 4 : -1;
  }

  // this block's K range in BK2 stages (a tail piece covers a contiguous share)
  const int nall = p.K / BK2;
  const int s_beg = tail ? (piece * nall) / p.tsplit : 0;
  const int s_end = tail ? ((piece + 1) * nall) / p.tsplit : nall;
  // scalar K-walk state of the next stage to issue.  Stages run channel-chunk-major, tap
  // minor (stage s = chunk * taps + tap): the taps of one 32-channel chunk re-read the same
  // ~(BM + halo) x 128 B of activations back to back, so they hit in L2 instead of being
  // re-fetched once per tap after a whole-Cin sweep.
  const int taps = p.ksize * p.ksize;
  int nx_tap = s_beg % taps, nx_ch = (s_beg / taps) * BK2;
  int nx_ky = nx_tap / p.ksize, nx_kx = nx_tap - nx_ky * p.ksize;
  auto issue = [&](int s, int buf) {
    (void)s;
    const int tap = nx_tap, ch0 = nx_ch;
    const int k0 = tap * p.Cin + ch0;
    const int tsh = ((nx_ky - kc) * p.W + (nx_kx - kc)) * p.dil * p.sign;  // pixel shift of this tap
    const bool second = ch0 >= p.c0;
    const int32x4 rs = second ? rs1 : rs0;
    const int ld = second ? ld1 : p.ldx0;
    const int cb = second ? ch0 - p.c0 : ch0;
    const unsigned sadd = (unsigned)((tsh * ld + cb) * 4);
    ++nx_tap;
    if (++nx_kx == p.ksize) { nx_kx = 0; ++nx_ky; }
    if (nx_tap == taps) {
      nx_tap = 0; nx_ky = 0; nx_kx = 0;
      nx_ch += BK2;
    }
    char* abase = lds + buf * STAGE;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const unsigned base = second ? a_o1[i] : a_o0[i];
      const unsigned off = ((a_mask[i] >> tap) & 1u) ? base + sadd : OOB;
      dma16(rs, off, lds_addr_of(abase + (wave * AI + i) * 1024));
    }
    char* bbase = abase + BM * ROW2;
#pragma unroll
    for (int j = 0; j < BI; ++j) {
      const unsigned off = b_off[j] >= 0 ? (unsigned)(b_off[j] + k0 * 4) : OOB;
      dma16(rsw, off, lds_addr_of(bbase + (wave * BI + j) * 1024));
    }
  };

  floatx16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int lr = lane & 31, lh = lane >> 5;
  const int wm0 = wmi * TM, wn0 = wni * TN;
  issue(s_beg, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // two-level accumulation: an MFMA chain of HP stages (32*HP products) starts from zero
  // and is then added into acc -- fp32 error ~sqrt(32 HP) + sqrt(K/(32 HP)) instead of
  // ~sqrt(K); HP*32 ~ sqrt(K) balances both (mkldnn-level accuracy).
  floatx16 part[TI][TJ];
  for (int s = s_beg; s < s_end; ++s) {
    const int buf = (s - s_beg) & 1;
    if (s + 1 < s_end) issue(s + 1, buf ^ 1);
    const char* a = lds + buf * STAGE;
    const char* b = a + BM * ROW2;
    const bool fresh = ((s - s_beg) % HP) == 0;
#pragma unroll
    for (int g = 0; g < BK2 / 8; ++g) {
      const int c = 2 * g + lh;
      float4 av[TI], bv[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int r = wm0 + i * 32 + lr;
        av[i] = *reinterpret_cast<const float4*>(a + r * ROW2 + swz(r, c) * 16);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int r = wn0 + j * 32 + lr;
        bv[j] = *reinterpret_cast<const float4*>(b + r * ROW2 + swz(r, c) * 16);
      }
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const floatx16 c0 = (g == 0 && fresh) ? floatx16{} : part[i][j];
          part[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].x, bv[j].x, c0, 0, 0, 0);
          part[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].y, bv[j].y, part[i][j], 0, 0, 0);
          part[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].z, bv[j].z, part[i][j], 0, 0, 0);
          part[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].w, bv[j].w, part[i][j], 0, 0, 0);
        }
    }
    if ((s - s_beg + 1) % HP == 0 || s + 1 == s_end) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] += part[i][j];
    }
    // stage-(s+1) DMA of this wave has landed, then every wave's (and every wave is done
    // reading stage s, whose buffer the next step's DMA overwrites)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  if (tail) {  // raw partial tile -> workspace [tail tile][piece][BM][BN]; conv_tail_fixup finishes
    float* dst = p.part + ((size_t)(wg - nfull) * p.tsplit + piece) * (BM * BN);
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          dst[rl * BN + wn0 + j * 32 + lr] = acc[i][j][r];
        }
    return;
  }

  // ---------------- epilogue: bias, store, BN partial statistics -----------------
  float bcol[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int col = n0 + wn0 + j * 32 + lr;
    bcol[j] = (p.bias != nullptr && col < p.Cout) ? p.bias[col] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int col = n0 + wn0 + j * 32 + lr;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const float v = acc[i][j][r] + bcol[j];
        acc[i][j][r] = v;
        if (row < p.P && col < p.Cout) {
          float* dst = p.y + (size_t)row * p.ldy + col;
          *dst = p.accumulate ? *dst + v : v;
        }
      }
    }
  if (p.stats == nullptr) return;
  float* red = smem;
  const int cnt = min(BM, p.P - m0);
  float mean[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        s += (row < p.P) ? acc[i][j][r] : 0.f;
      }
    s += __shfl_xor(s, 32, 64);
    if (lh == 0) red[wmi * BN + wn0 + j * 32 + lr] = s;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < WM; ++w) s += red[w * BN + wn0 + j * 32 + lr];
    mean[j] = s / (float)cnt;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const float d = acc[i][j][r] - mean[j];
        s += (row < p.P) ? d * d : 0.f;
      }
    s += __shfl_xor(s, 32, 64);
    if (lh == 0) red[wmi * BN + wn0 + j * 32 + lr] = s;
  }
  __syncthreads();
  if (wmi == 0 && lh == 0) {
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int cl = wn0 + j * 32 + lr, col = n0 + cl;
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) s += red[w * BN + cl];
      if (col < p.Cout) p.stats[(size_t)mt * p.Cout + col] = make_float2(mean[j], s);
    }
  }
}


// ------------------------------ weight gradient --------------------------------


constexpr int BKP = 16;  // pixels per stage

// The BN (+ReLU) backward applied to the weight gradient's dY operand as it is loaded (enc1.conv1, whose only
// consumer of dy is this fp32 weight gradient: no dgrad): dy = gamma invstd (dz - m1 - xhat m2), dz = da masked by
// the recomputed BN output > 0 -- bn_bwd_apply_kernel's expressions with srpde_bn_bwd_prepare's m1 / m2, so the
// same dy bits, never written.
struct WgradBn {
  const float* y; int ldy;
  const float *mean, *invstd, *gamma, *beta, *m1, *m2;
  int relu;
};

template <int BM, int BN, int WM, int WN, bool BNB = false>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradParams p, WgradBn bn = {}) {
  constexpr int TM = BM / WM, TN = BN / WN, TI = TM / 32, TJ = TN / 32;
  constexpr int LDA = BM + 4, LDB = BN + 4;
  constexpr int A_V4_ROW = BM / 4, B_V4_ROW = BN / 4;
  constexpr int A_TOTAL = BKP * A_V4_ROW, B_TOTAL = BKP * B_V4_ROW;
  constexpr int A_LOADS = (A_TOTAL + 255) / 256, B_LOADS = (B_TOTAL + 255) / 256;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* As = smem;                    // [2][BKP][LDA]
  float* Bs = smem + 2 * BKP * LDA;    // [2][BKP][LDB]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wmi = wave % WM, wni = wave / WM;
  const int nbm = (p.Cout + BM - 1) / BM, nbn = (p.K + BN - 1) / BN;
  const int ntile = nbm * nbn;
  const int split = blockIdx.x / ntile;
  const int tile = blockIdx.x - split * ntile;
  const int mt = tile / nbn, nt = tile - mt * nbn;
  const int m0 = mt * BM, n0 = nt * BN;
  const int pbeg = split * p.chunk;
  const int pend = min(p.P, pbeg + p.chunk);
  const int HW = p.H * p.W;
  const int kc = p.ksize >> 1;

  // B columns handled by this thread are fixed: decode (tap, channel source) once
  int b_oy[B_LOADS], b_ox[B_LOADS], b_cc[B_LOADS], b_src[B_LOADS];
  bool b_ok[B_LOADS];
#pragma unroll
  for (int j = 0; j < B_LOADS; ++j) {
    const int e = tid + j * 256;
    const int c4 = e % B_V4_ROW;
    const int k = n0 + c4 * 4;
    b_ok[j] = (e < B_TOTAL) && (k < p.K);
    const int tap = b_ok[j] ? k / p.Cin : 0;
    const int c = b_ok[j] ? k - tap * p.Cin : 0;
    const int ky = tap / p.ksize, kx = tap - ky * p.ksize;
    b_oy[j] = (ky - kc) * p.dil; b_ox[j] = (kx - kc) * p.dil;
    b_src[j] = c < p.c0 ? 0 : 1;
    b_cc[j] = c < p.c0 ? c : c - p.c0;
  }

  float4 ra[A_LOADS], rb[B_LOADS];
  auto load_stage = [&](int pbase) {
#pragma unroll
    for (int i = 0; i < A_LOADS; ++i) {
      const int e = tid + i * 256;
      const int c4 = e % A_V4_ROW, pr = e / A_V4_ROW;
      const int px = pbase + pr, col = m0 + c4 * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < A_TOTAL && px < pend && col < p.Cout) {
        v = *reinterpret_cast<const float4*>(p.dy + (size_t)px * p.lddy + col);
        if constexpr (BNB) {
          const float4 yv = *reinterpret_cast<const float4*>(bn.y + (size_t)px * bn.ldy + col);
          const float4 mu = *reinterpret_cast<const float4*>(bn.mean + col);
          const float4 is = *reinterpret_cast<const float4*>(bn.invstd + col);
          const float4 g = *reinterpret_cast<const float4*>(bn.gamma + col);
          const float4 bb = *reinterpret_cast<const float4*>(bn.beta + col);
          const float4 m1 = *reinterpret_cast<const float4*>(bn.m1 + col);
          const float4 m2 = *reinterpret_cast<const float4*>(bn.m2 + col);
          float xh, dz;
#define WG_BN(X)                                                     \
  xh = (yv.X - mu.X) * is.X;                                         \
  dz = (!(bn.relu & 1) || xh * g.X + bb.X > 0.f) ? v.X : 0.f;        \
  v.X = (dz - m1.X - xh * m2.X) * (g.X * is.X);
          WG_BN(x) WG_BN(y) WG_BN(z) WG_BN(w)
#undef WG_BN
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int j = 0; j < B_LOADS; ++j) {
      const int e = tid + j * 256;
      const int pr = e / B_V4_ROW;
      const int px = pbase + pr;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (b_ok[j] && px < pend) {
        const int n = px / HW, rem = px - n * HW, yy = rem / p.W, xx = rem - yy * p.W;
        const int iy = yy + b_oy[j], ix = xx + b_ox[j];
        if (iy >= 0 && iy < p.H && ix >= 0 && ix < p.W) {
          const size_t q = (size_t)(n * HW + iy * p.W + ix);
          v = b_src[j] == 0 ? *reinterpret_cast<const float4*>(p.x0 + q * p.ldx0 + b_cc[j])
                            : *reinterpret_cast<const float4*>(p.x1 + q * p.ldx1 + b_cc[j]);
        }
      }
      rb[j] = v;
    }
  };
  auto store_stage = [&](int buf) {
    float* a = As + buf * BKP * LDA;
    float* b = Bs + buf * BKP * LDB;
#pragma unroll
    for (int i = 0; i < A_LOADS; ++i) {
      const int e = tid + i * 256;
      if (e < A_TOTAL) *reinterpret_cast<float4*>(a + (e / A_V4_ROW) * LDA + (e % A_V4_ROW) * 4) = ra[i];
    }
#pragma unroll
    for (int j = 0; j < B_LOADS; ++j) {
      const int e = tid + j * 256;
      if (e < B_TOTAL) *reinterpret_cast<float4*>(b + (e / B_V4_ROW) * LDB + (e % B_V4_ROW) * 4) = rb[j];
    }
  };

  floatx16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nsteps = (pend - pbeg + BKP - 1) / BKP;
  const int lr = lane & 31, lh = lane >> 5;
  const int wm0 = wmi * TM, wn0 = wni * TN;
  if (nsteps > 0) {
    load_stage(pbeg);
    store_stage(0);
  }
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) load_stage(pbeg + (s + 1) * BKP);
    const float* a = As + buf * BKP * LDA;
    const float* b = Bs + buf * BKP * LDB;
#pragma unroll
    for (int kq = 0; kq < BKP / 2; ++kq) {
      const int kr = kq * 2 + lh;
      float av[TI], bv[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) av[i] = a[kr * LDA + wm0 + i * 32 + lr];
#pragma unroll
      for (int j = 0; j < TJ; ++j) bv[j] = b[kr * LDB + wn0 + j * 32 + lr];
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (s + 1 < nsteps) store_stage(buf ^ 1);
    __syncthreads();
  }

  float* out = p.part + (size_t)split * p.Cout * p.K;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int col = n0 + wn0 + j * 32 + lr;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row < p.Cout && col < p.K) out[(size_t)row * p.K + col] = acc[i][j][r];
      }
    }
}

// ------------------- weight gradient v2: LDS-DMA staged, BKW pixels -------------------
// For c0 % 32 == 0 and c1 % 32 == 0.  Both GEMM operands are pixel-major in HBM (dY[p][m],
// X[p + off(tap)][c]); a stage is BKW pixels of each.  LDS keeps every operand as 32-column
// groups [group][pixel][32 floats] (128-B rows; group stride padded by 128 B so the two groups
// a half-wave reads sit on different banks).  One DMA wave-instruction fills 8 pixels x 32
// columns of ONE group, so its (tap, source tensor) is wave-uniform; padding taps and pixels
// past the chunk use the out-of-range offset (hardware zero fill).  MFMA operands need no
// transpose: lane (r, h) reads QA consecutive dY channels of pixel 2kp+h with one ds_read, and
// channel q of that read feeds output tile q, whose rows are the interleaved channels
// wm0 + QA*r + q (same for the QB X columns).
constexpr int BKW = 32;                  // pixels per stage (= 4 waves x 8-pixel row blocks)
constexpr int GSTR = BKW * 128 + 128;    // LDS bytes per 32-column group (+128 B bank pad)

template <int Q>
struct vecf;
template <> struct vecf<1> { typedef float t; };
template <> struct vecf<2> { typedef float2 t; };
template <> struct vecf<4> { typedef float4 t; };
__device__ __forceinline__ float vget(float v, int) { return v; }
__device__ __forceinline__ float vget(float2 v, int q) { return q == 0 ? v.x : v.y; }
__device__ __forceinline__ float vget(float4 v, int q) { return q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w; }

template <int BM, int BN, int WM, int WN, int HP>
__global__ __launch_bounds__(256, 2) void conv_wgrad_v2_kernel(WgradParams p) {
  constexpr int TM = BM / WM, TN = BN / WN, QA = TM / 32, QB = TN / 32;
  constexpr int GA = BM / 32, GB = BN / 32;  // column groups; wave w loads row block w of each
  static_assert(BKW == 32, "4 waves x 8 rows");
  static_assert(QA == 1 || QA == 2 || QA == 4, "QA");
  static_assert(QB == 1 || QB == 2 || QB == 4, "QB");
  constexpr int STAGE = (GA + GB) * GSTR;
  typedef typename vecf<QA>::t va_t;
  typedef typename vecf<QB>::t vb_t;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* lds = reinterpret_cast<char*>(smem);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wmi = wave % WM, wni = wave / WM;
  const int nbm = (p.Cout + BM - 1) / BM, nbn = (p.K + BN - 1) / BN;
  const int ntile = nbm * nbn;
  // consecutive logical blocks = tiles of one pixel chunk -> same XCD (shared dY / X rows)
  const int bid = xcd_remap(blockIdx.x, ntile * p.splits);
  const int split = bid / ntile, tile = bid - split * ntile;
  const int mt = tile / nbn, nt = tile - mt * nbn;
  const int m0 = mt * BM, n0 = nt * BN;
  const int pbeg = split * p.chunk, pend = min(p.P, pbeg + p.chunk);
  const int HW = p.H * p.W, kc = p.ksize >> 1;

  const int32x4 rsy = make_rsrc(p.dy, (unsigned)((size_t)p.P * p.lddy * 4));
  const int32x4 rs0 = make_rsrc(p.x0, (unsigned)((size_t)p.P * p.ldx0 * 4));
  const int ld1 = p.c1 ? p.ldx1 : p.ldx0;
  const int32x4 rs1 = make_rsrc(p.c1 ? p.x1 : p.x0, (unsigned)((size_t)p.P * ld1 * 4));
  const int sub = lane >> 3, c4 = (lane & 7) * 4;

  // per-group constants (wave-uniform): dY column byte offset / validity, and for X the tap
  // shift, the source tensor and the channel byte offset of the group's first column
  int a_colb[GA];
  bool a_ok[GA];
#pragma unroll
  for (int g = 0; g < GA; ++g) {
    const int m = m0 + 32 * g + c4;
    a_ok[g] = m < p.Cout;
    a_colb[g] = m * 4;
  }
  int b_dy[GB], b_dx[GB], b_sh[GB], b_chb[GB];
  bool b_ok[GB], b_second[GB];
#pragma unroll
  for (int g = 0; g < GB; ++g) {
    const int kg = n0 + 32 * g;
    b_ok[g] = kg < p.K;
    const int tap = b_ok[g] ? kg / p.Cin : 0;
    const int ch = kg - tap * p.Cin;
    const int ky = tap / p.ksize, kx = tap - ky * p.ksize;
    b_dy[g] = (ky - kc) * p.dil;
    b_dx[g] = (kx - kc) * p.dil;
    b_sh[g] = b_dy[g] * p.W + b_dx[g];
    b_second[g] = ch >= p.c0;
    b_chb[g] = ((b_second[g] ? ch - p.c0 : ch) + c4) * 4;
  }

  auto issue = [&](int pbase, int buf) {
    const int pix = pbase + wave * 8 + sub;
    const bool pok = pix < pend;
    const int n = pix / HW, rem = pix - n * HW, yy = rem / p.W, xx = rem - yy * p.W;
    char* abase = lds + buf * STAGE + wave * 1024;
#pragma unroll
    for (int g = 0; g < GA; ++g) {
      const unsigned off = (pok && a_ok[g]) ? (unsigned)(pix * p.lddy * 4 + a_colb[g]) : OOB;
      dma16(rsy, off, lds_addr_of(abase + g * GSTR));
    }
    char* bbase = abase + GA * GSTR;
#pragma unroll
    for (int g = 0; g < GB; ++g) {
      const int iy = yy + b_dy[g], ix = xx + b_dx[g];
      const bool ok = pok && b_ok[g] && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
      const int ld = b_second[g] ? ld1 : p.ldx0;
      const unsigned off = ok ? (unsigned)((pix + b_sh[g]) * ld * 4 + b_chb[g]) : OOB;
      dma16(b_second[g] ? rs1 : rs0, off, lds_addr_of(bbase + g * GSTR));
    }
  };

  floatx16 acc[QA][QB], part[QA][QB];
#pragma unroll
  for (int i = 0; i < QA; ++i)
#pragma unroll
    for (int j = 0; j < QB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int lr = lane & 31, lh = lane >> 5;
  const int wm0 = wmi * TM, wn0 = wni * TN;
  // per-lane operand read offsets inside a stage (pixel row lh; + 256 B per k-pair)
  const int ma = wm0 + QA * lr, nb = wn0 + QB * lr;
  const int a_rd = (ma >> 5) * GSTR + (ma & 31) * 4 + lh * 128;
  const int b_rd = GA * GSTR + (nb >> 5) * GSTR + (nb & 31) * 4 + lh * 128;

  const int nsteps = (pend - pbeg + BKW - 1) / BKW;
  if (nsteps > 0) issue(pbeg, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) issue(pbeg + (s + 1) * BKW, buf ^ 1);
    const char* st = lds + buf * STAGE;
    const bool fresh = (s % HP) == 0;
#pragma unroll
    for (int kp = 0; kp < BKW / 2; ++kp) {
      const va_t av = *reinterpret_cast<const va_t*>(st + a_rd + kp * 256);
      const vb_t bv = *reinterpret_cast<const vb_t*>(st + b_rd + kp * 256);
#pragma unroll
      for (int i = 0; i < QA; ++i)
#pragma unroll
        for (int j = 0; j < QB; ++j) {
          const floatx16 c0 = (kp == 0 && fresh) ? floatx16{} : part[i][j];
          part[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(vget(av, i), vget(bv, j), c0, 0, 0, 0);
        }
    }
    if ((s + 1) % HP == 0 || s + 1 == nsteps) {
#pragma unroll
      for (int i = 0; i < QA; ++i)
#pragma unroll
        for (int j = 0; j < QB; ++j) acc[i][j] += part[i][j];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // slab [split][Cout][K]: tile (i, j) element (row rc, col lr) is dW[wm0+QA*rc+i][wn0+QB*lr+j]
  float* out = p.part + (size_t)split * p.Cout * p.K;
  const int n = n0 + nb;
  if (n < p.K) {
#pragma unroll
    for (int i = 0; i < QA; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rc = (r & 3) + 8 * (r >> 2) + 4 * lh;
        const int m = m0 + wm0 + QA * rc + i;
        if (m < p.Cout) {
          float* dst = out + (size_t)m * p.K + n;
          if constexpr (QB == 1) {
            dst[0] = acc[i][0][r];
          } else if constexpr (QB == 2) {
            *reinterpret_cast<float2*>(dst) = make_float2(acc[i][0][r], acc[i][1][r]);
          } else {
            *reinterpret_cast<float4*>(dst) = make_float4(acc[i][0][r], acc[i][1][r], acc[i][2][r], acc[i][3][r]);
          }
        }
      }
  }
}

// first level of a two-level slab sum (few elements, many slabs: enc1.conv1's 2304 weights over
// ~2048 slabs): slab g*G <- sum of slabs [g*G, g*G + G) in order, one thread per (element, group).
// A whole group's G loads are issued before the in-order sum (one load in flight per thread made it
// latency-bound: ~250 us per call for ~19 MB)
template <int G>
__global__ void slab_group_sum_kernel(float* __restrict__ part, int splits, long long total) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long ngroups = (splits + G - 1) / G;
  if (i >= total * ngroups) return;
  const long long g = i / total, e = i - g * total;
  const int q0 = (int)(g * G), q1 = min(splits, q0 + G);
  float s = 0.f;
  if (q1 - q0 == G) {
    float v[G];
#pragma unroll
    for (int u = 0; u < G; ++u) v[u] = part[(size_t)(q0 + u) * total + e];
#pragma unroll
    for (int u = 0; u < G; ++u) s += v[u];
  } else {
    for (int q = q0; q < q1; ++q) s += part[(size_t)q * total + e];
  }
  part[(size_t)q0 * total + e] = s;
}

// sum the split-K slabs in fixed order, write dW in torch layout [Cout][Cin_real][k][k]
// (slab q at part + q * stride * cout * K: stride > 1 after slab_group_sum_kernel)
__global__ void wgrad_reduce_kernel(const float* __restrict__ part, float* __restrict__ dw, int splits,
                                    int cout, int cin, int cin_real, int taps, int accumulate, int stride) {
  // iterate in slab (k-contiguous) order so the split reads coalesce; the transposed
  // store into torch's [Cout][Cin][kh][kw] layout is the scattered side (written once)
  // block = 64 consecutive slab elements x 4 split groups; fixed-order combine
  __shared__ float red[4][64];
  const long long K = (long long)taps * cin;
  const long long total = (long long)cout * K;
  const int el = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const long long e = (long long)blockIdx.x * 64 + el;
  float s = 0.f;
  if (e < total) {
    const size_t qs = (size_t)stride * cout * K;
    int q = grp;
    for (; q + 28 < splits; q += 32) {   // eight of this thread's slabs loaded before their in-order sum
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(q + 4 * u) * qs + e];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; q < splits; q += 4) s += part[(size_t)q * qs + e];
  }
  red[grp][el] = s;
  __syncthreads();
  if (grp == 0 && e < total) {
    const float v = (red[0][el] + red[1][el]) + (red[2][el] + red[3][el]);
    const int n = (int)(e / K);
    const int k = (int)(e - (long long)n * K);
    const int t = k / cin, c = k - t * cin;
    if (c < cin_real) {
      const long long dst = ((long long)n * cin_real + c) * taps + t;
      dw[dst] = accumulate ? dw[dst] + v : v;
    }
  }
}

int wgrad_reduce(const float* part, float* dw, int splits, int cout, int cin, int cin_real, int taps, int accumulate,
                 hipStream_t stream) {
  const long long total = (long long)cout * taps * cin;
  const int blocks = (int)((total + 63) / 64);
  int stride = 1;
  if (total < 65536 && splits >= 128) {   // too few elements to keep the chip busy: sum groups of 32 first
    constexpr int G = 32;
    const long long work = total * ((splits + G - 1) / G);
    hipLaunchKernelGGL(slab_group_sum_kernel<G>, dim3((int)((work + 255) / 256)), dim3(256), 0, stream,
                       const_cast<float*>(part), splits, total);
    SRPDE_LAUNCH_CHECK("srpde_conv_wgrad(reduce groups)");
    stride = G;
    splits = (splits + G - 1) / G;
  }
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, stream, part, dw, splits, cout, cin, cin_real,
                     taps, accumulate, stride);
  SRPDE_LAUNCH_CHECK("srpde_conv_wgrad(reduce)");
  return 0;
}

// W[Cout][Cin_real][k][k] -> Wf[Cout][taps][Cin] and Wd[Cin][taps][Cout] (Cin >= Cin_real, zero pad)
__global__ void pack_weights_kernel(const float* __restrict__ w, float* __restrict__ wf, float* __restrict__ wd,
                                    int cout, int cin, int cin_real, int taps) {
  const long long total = (long long)cout * taps * cin;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % cin);
    const long long r = e / cin;
    const int t = (int)(r % taps);
    const int n = (int)(r / taps);
    const float v = c < cin_real ? w[((long long)n * cin_real + c) * taps + t] : 0.f;
    if (wf) wf[e] = v;
    if (wd) wd[((long long)c * taps + t) * cout + n] = v;
  }
}

// -------------------------------- host side ------------------------------------
template <int BM, int BN, int WM, int WN>
static int launch_fwd(const ConvParams& p, hipStream_t st) {
  const int nbm = ceil_div(p.P, BM), nbn = ceil_div(p.Cout, BN);
  const size_t lds = (size_t)2 * (BM + BN) * LDK * sizeof(float);
  hipLaunchKernelGGL((conv_igemm_fwd_kernel<BM, BN, WM, WN>), dim3(nbm * nbn), dim3(256), lds, st, p);
  SRPDE_LAUNCH_CHECK("srpde_conv_fwd");
  return 0;
}


template <int BM, int BN, int WM, int WN, int HP>
static int launch_fwd_v2(ConvParams p, hipStream_t st, void* ws, size_t ws_bytes) {
  const int nbm = ceil_div(p.P, BM), nbn = ceil_div(p.Cout, BN);
  const int T = nbm * nbn;
  const size_t lds = (size_t)2 * (BM + BN) * ROW2;
  // workgroups resident at once (occupancy x CUs), queried once per instantiation
  static int slots = [&] {
    int per_cu = 0, dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, conv_fwd_v2_kernel<BM, BN, WM, WN, HP>, 256, lds);
    return std::max(1, per_cu) * std::max(1, cus);
  }();
  // tail split: when the last round of workgroups would be under half full, cut its tiles
  // into F K-pieces so that round runs on ~F x more CUs for 1/F of the time
  plan_tail(p, T, slots, BM, BN, ws, ws_bytes);
  const int grid = T - p.ntail + p.ntail * p.tsplit;
  hipLaunchKernelGGL((conv_fwd_v2_kernel<BM, BN, WM, WN, HP>), dim3(grid), dim3(256), lds, st, p);
  SRPDE_LAUNCH_CHECK("srpde_conv_fwd(v2)");
  if (p.ntail > 0) {
    hipLaunchKernelGGL((conv_tail_fixup_kernel<BM, BN>), dim3(p.ntail), dim3(1024), 0, st, p);
    SRPDE_LAUNCH_CHECK("srpde_conv_fwd(tail fixup)");
  }
  return 0;
}


static bool v2_ok(const ConvParams& p) {
  const long long maxld = std::max(p.ldx0, p.c1 ? p.ldx1 : 0);
  return p.c0 % 32 == 0 && p.c1 % 32 == 0 && (long long)p.P * maxld * 4 < (1LL << 31) &&
         (long long)p.Cout * p.K * 4 < (1LL << 31);
}

static int fwd_config(int cout) { return cout % 128 == 0 ? 0 : (cout % 64 == 0 ? 1 : 2); }
static int fwd_bm(int cfg) { return cfg == 0 ? 128 : 256; }

template <int BM, int BN, int WM, int WN>
static int launch_wgrad(const WgradParams& p, hipStream_t st, const WgradBn* bn = nullptr) {
  const int nb = ceil_div(p.Cout, BM) * ceil_div(p.K, BN) * p.splits;
  const size_t lds = (size_t)2 * BKP * ((BM + 4) + (BN + 4)) * sizeof(float);
  if (bn != nullptr)
    hipLaunchKernelGGL((conv_wgrad_kernel<BM, BN, WM, WN, true>), dim3(nb), dim3(256), lds, st, p, *bn);
  else
    hipLaunchKernelGGL((conv_wgrad_kernel<BM, BN, WM, WN, false>), dim3(nb), dim3(256), lds, st, p, WgradBn{});
  SRPDE_LAUNCH_CHECK("srpde_conv_wgrad");
  return 0;
}

template <int BM, int BN, int WM, int WN>
static int launch_wgrad_v2(const WgradParams& p, hipStream_t st) {
  const int nb = ceil_div(p.Cout, BM) * ceil_div(p.K, BN) * p.splits;
  const size_t lds = (size_t)2 * (BM / 32 + BN / 32) * GSTR;
  hipLaunchKernelGGL((conv_wgrad_v2_kernel<BM, BN, WM, WN, 2>), dim3(nb), dim3(256), lds, st, p);
  SRPDE_LAUNCH_CHECK("srpde_conv_wgrad(v2)");
  return 0;
}

static bool wgrad_v2_ok(const WgradParams& p) {
  const long long maxld = std::max(std::max(p.ldx0, p.c1 ? p.ldx1 : 0), p.lddy);
  return p.c0 % 32 == 0 && p.c1 % 32 == 0 && (long long)p.P * maxld * 4 < (1LL << 31);
}

static void wgrad_tiles(int cout, int K, int* bm, int* bn) {
  if (cout >= 128) { *bm = 128; *bn = 128; }
  else if (cout >= 64) { *bm = 64; *bn = K <= 64 ? 64 : 256; }   // K <= 64: enc1.conv1 (3 -> 4 channels)
  else { *bm = 32; *bn = 256; }
}

static void wgrad_split(int P, int cout, int K, int* chunk, int* splits) {
  int bm, bn;
  wgrad_tiles(cout, K, &bm, &bn);
  const long long tiles = (long long)ceil_div(cout, bm) * ceil_div(K, bn);
  // at most 2048 workgroups (= whole rounds of 256 CUs x 1|2 resident): rounding the split
  // count UP would leave a nearly empty last round (e.g. 36 tiles x 57 = 2052 = 4 rounds + 4)
  long long want = std::max(1LL, 2048 / tiles);
  long long c = (P + want - 1) / want;
  c = (c + BKW - 1) / BKW * BKW;  // multiple of both stage sizes (BKP | BKW)
  if (c < 256) c = 256;
  *chunk = (int)c;
  *splits = ceil_div(P, c);
}

}  // namespace srpde

using namespace srpde;

extern "C" {

size_t srpde_conv_stats_blocks(int n, int h, int w, int cout) {
  return (size_t)ceil_div((long long)n * h * w, fwd_bm(fwd_config(cout)));
}

int srpde_conv_stats_rows_per_block(int cout) { return fwd_bm(fwd_config(cout)); }

// tail-split scratch: at most one round of workgroups worth of fp32 tiles (<= 1024 slots)
size_t srpde_conv_fwd_workspace_size(int cout) {
  const int bm = fwd_bm(fwd_config(cout));
  const int bn = cout % 128 == 0 ? 128 : (cout % 64 == 0 ? 64 : 32);
  return (size_t)1024 * bm * bn * sizeof(float);
}

int srpde_conv_fwd(const float* x0, int c0, int ldx0, const float* x1, int c1, int ldx1,
                   const float* wpack, const float* bias, float* y, int ldy,
                   int n, int h, int w, int cout, int ksize, int dil, int sign, int accumulate,
                   float* stats, const float* ep_mean, const float* ep_invstd, const float* ep_gamma,
                   const float* ep_beta, unsigned* ep_amax, void* workspace, size_t ws_bytes, hipStream_t stream) {
  SRPDE_CHECK_ARG(x0 && wpack && y, "srpde_conv_fwd: null pointer");
  SRPDE_CHECK_ARG(n > 0 && h > 0 && w > 0 && cout > 0, "srpde_conv_fwd: bad shape");
  SRPDE_CHECK_ARG(ksize == 1 || ksize == 3, "srpde_conv_fwd: ksize must be 1 or 3");
  SRPDE_CHECK_ARG(sign == 1 || sign == -1, "srpde_conv_fwd: sign must be +-1");
  SRPDE_CHECK_ARG(c0 % 4 == 0 && c1 % 4 == 0 && ldx0 % 4 == 0 && (c1 == 0 || ldx1 % 4 == 0),
                  "srpde_conv_fwd: channel counts / strides must be multiples of 4 (c0=%d c1=%d)", c0, c1);
  SRPDE_CHECK_ARG(c1 == 0 || x1 != nullptr, "srpde_conv_fwd: x1 null with c1>0");
  SRPDE_CHECK_ARG(aligned16(x0) && aligned16(wpack) && (c1 == 0 || aligned16(x1)),
                  "srpde_conv_fwd: inputs must be 16-byte aligned");
  SRPDE_CHECK_ARG((long long)n * h * w < (1LL << 31), "srpde_conv_fwd: too many pixels");
  ConvParams p;
  p.x0 = x0; p.c0 = c0; p.ldx0 = ldx0;
  p.x1 = x1; p.c1 = c1; p.ldx1 = ldx1 > 0 ? ldx1 : 4;
  p.w = wpack; p.bias = bias; p.y = y; p.ldy = ldy;
  p.stats = reinterpret_cast<float2*>(stats);
  p.N = n; p.H = h; p.W = w; p.Cout = cout; p.ksize = ksize; p.dil = dil; p.sign = sign; p.accumulate = accumulate;
  p.P = n * h * w; p.Cin = c0 + c1; p.K = ksize * ksize * p.Cin;
  p.ntail = 0; p.tsplit = 1; p.part = nullptr;
  SRPDE_CHECK_ARG(ep_mean == nullptr || (ep_invstd && ep_gamma && ep_beta && !accumulate && stats == nullptr &&
                                         cout % 4 == 0 && !v2_ok(p)),
                  "srpde_conv_fwd: the epilogue BN + ReLU needs mean/invstd/gamma/beta, no accumulate / stats, "
                  "cout %% 4 == 0, and a layer the register-staged kernel takes (cin %% 32 != 0)");
  p.ep_mean = ep_mean; p.ep_invstd = ep_invstd; p.ep_gamma = ep_gamma; p.ep_beta = ep_beta;
  p.ep_amax = ep_mean != nullptr ? ep_amax : nullptr;
  if (c4_ok(p)) return launch_fwd_c4(p, stream);
  if (v2_ok(p)) {
    switch (fwd_config(cout)) {
      case 0: return launch_fwd_v2<128, 128, 2, 2, 4>(p, stream, workspace, ws_bytes);
      case 1: return launch_fwd_v2<256, 64, 4, 1, 4>(p, stream, workspace, ws_bytes);
      default: return launch_fwd_v2<256, 32, 4, 1, 4>(p, stream, workspace, ws_bytes);
    }
  }
  switch (fwd_config(cout)) {
    case 0: return launch_fwd<128, 128, 2, 2>(p, stream);
    case 1: return launch_fwd<256, 64, 4, 1>(p, stream);
    default: return launch_fwd<256, 32, 4, 1>(p, stream);
  }
}

size_t srpde_conv_wgrad_workspace_size(int n, int h, int w, int cout, int cin, int ksize) {
  const int P = n * h * w, K = ksize * ksize * cin;
  int chunk, splits;
  wgrad_split(P, cout, K, &chunk, &splits);
  return (size_t)splits * cout * K * sizeof(float);
}

static int conv_wgrad_impl(const float* dy, int lddy, const float* x0, int c0, int ldx0, const float* x1, int c1,
                           int ldx1, float* dw, int cin_real, int accumulate, int n, int h, int w, int cout,
                           int ksize, int dil, void* workspace, size_t ws_bytes, hipStream_t stream,
                           const unsigned* amax_dy = nullptr, const unsigned* amax0 = nullptr,
                           const unsigned* amax1 = nullptr, const WgradBn* bn = nullptr) {
  SRPDE_CHECK_ARG(dy && x0 && dw && workspace, "srpde_conv_wgrad: null pointer");
  SRPDE_CHECK_ARG(c0 % 4 == 0 && c1 % 4 == 0 && lddy % 4 == 0 && ldx0 % 4 == 0 && cout % 4 == 0,
                  "srpde_conv_wgrad: channel counts / strides must be multiples of 4");
  SRPDE_CHECK_ARG(c1 == 0 || (x1 && ldx1 % 4 == 0), "srpde_conv_wgrad: bad x1");
  SRPDE_CHECK_ARG(cin_real <= c0 + c1, "srpde_conv_wgrad: cin_real > cin");
  WgradParams p;
  p.dy = dy; p.lddy = lddy; p.x0 = x0; p.c0 = c0; p.ldx0 = ldx0; p.x1 = x1; p.c1 = c1;
  p.ldx1 = ldx1 > 0 ? ldx1 : 4;
  p.N = n; p.H = h; p.W = w; p.Cout = cout; p.ksize = ksize; p.dil = dil;
  p.P = n * h * w; p.Cin = c0 + c1; p.K = ksize * ksize * p.Cin;
  wgrad_split(p.P, cout, p.K, &p.chunk, &p.splits);
  const size_t need = (size_t)p.splits * cout * p.K * sizeof(float);
  if (ws_bytes < need) {
    set_error("srpde_conv_wgrad: workspace %zu < %zu bytes", ws_bytes, need);
    return kErrWorkspace;
  }
  p.part = static_cast<float*>(workspace);
  int bm, bn_cols, rc;
  wgrad_tiles(cout, p.K, &bm, &bn_cols);
  if (bn != nullptr) {   // the fp32 kernel with the BN apply on its dY loads (srpde_conv_wgrad_bnb)
    if (bm == 128) rc = launch_wgrad<128, 128, 2, 2>(p, stream, bn);
    else if (bm == 64)
      rc = bn_cols == 64 ? launch_wgrad<64, 64, 2, 2>(p, stream, bn) : launch_wgrad<64, 256, 1, 4>(p, stream, bn);
    else rc = launch_wgrad<32, 256, 1, 4>(p, stream, bn);
  } else if (amax_dy) {
    SRPDE_CHECK_ARG(c0 % 32 == 0 && c1 % 32 == 0 && cout % 16 == 0 && wgrad_v2_ok(p) && amax0 && (c1 == 0 || amax1),
                    "srpde_conv_wgrad_h3: needs c0, c1 multiples of 32, cout of 16 and the amax words (c0=%d c1=%d cout=%d)",
                    c0, c1, cout);
    rc = launch_wgrad_h3(p, amax_dy, amax0, amax1, stream);
  } else if (wgrad_v2_ok(p)) {
    if (bm == 128) rc = launch_wgrad_v2<128, 128, 2, 2>(p, stream);
    else if (bm == 64) rc = launch_wgrad_v2<64, 128, 1, 4>(p, stream);   // 64x128: two workgroups per CU
    else rc = launch_wgrad_v2<32, 256, 1, 4>(p, stream);
  } else {
    if (bm == 128) rc = launch_wgrad<128, 128, 2, 2>(p, stream);
    else if (bm == 64) rc = bn_cols == 64 ? launch_wgrad<64, 64, 2, 2>(p, stream) : launch_wgrad<64, 256, 1, 4>(p, stream);
    else rc = launch_wgrad<32, 256, 1, 4>(p, stream);
  }
  if (rc) return rc;
  return wgrad_reduce(p.part, dw, p.splits, cout, p.Cin, cin_real, ksize * ksize, accumulate, stream);
}

int srpde_conv_wgrad(const float* dy, int lddy, const float* x0, int c0, int ldx0, const float* x1, int c1,
                     int ldx1, float* dw, int cin_real, int accumulate, int n, int h, int w, int cout, int ksize,
                     int dil, void* workspace, size_t ws_bytes, hipStream_t stream) {
  return conv_wgrad_impl(dy, lddy, x0, c0, ldx0, x1, c1, ldx1, dw, cin_real, accumulate, n, h, w, cout, ksize, dil,
                         workspace, ws_bytes, stream);
}

int srpde_conv_wgrad_bnb(const float* da, int ldda, const float* y, int ldy, const float* mean, const float* invstd,
                         const float* gamma, const float* beta, const float* m1, const float* m2, int flags,
                         const float* x0, int c0, int ldx0, float* dw, int cin_real, int accumulate, int n, int h,
                         int w, int cout, int ksize, int dil, void* workspace, size_t ws_bytes, hipStream_t stream) {
  SRPDE_CHECK_ARG(da && y && mean && invstd && gamma && beta && m1 && m2 && ldy % 4 == 0,
                  "srpde_conv_wgrad_bnb: null argument / y stride");
  const WgradBn bn{y, ldy, mean, invstd, gamma, beta, m1, m2, flags & SRPDE_BN_RELU};
  return conv_wgrad_impl(da, ldda, x0, c0, ldx0, nullptr, 0, 0, dw, cin_real, accumulate, n, h, w, cout, ksize, dil,
                         workspace, ws_bytes, stream, nullptr, nullptr, nullptr, &bn);
}

int srpde_conv_wgrad_h3(const float* dy, int lddy, const unsigned* amax_dy, const float* x0, int c0, int ldx0,
                        const unsigned* amax0, const float* x1, int c1, int ldx1, const unsigned* amax1, float* dw,
                        int cin_real, int accumulate, int n, int h, int w, int cout, int ksize, int dil,
                        void* workspace, size_t ws_bytes, hipStream_t stream) {
  SRPDE_CHECK_ARG(amax_dy, "srpde_conv_wgrad_h3: null amax_dy");
  return conv_wgrad_impl(dy, lddy, x0, c0, ldx0, x1, c1, ldx1, dw, cin_real, accumulate, n, h, w, cout, ksize, dil,
                         workspace, ws_bytes, stream, amax_dy, amax0, amax1);
}

int srpde_pack_conv_weights(const float* w, float* wfwd, float* wdgrad, int cout, int cin, int cin_real, int ksize,
                            hipStream_t stream) {
  SRPDE_CHECK_ARG(w && (wfwd || wdgrad), "srpde_pack_conv_weights: null pointer");
  SRPDE_CHECK_ARG(cin >= cin_real && cin % 4 == 0, "srpde_pack_conv_weights: bad cin");
  const int taps = ksize * ksize;
  const long long total = (long long)cout * taps * cin;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(pack_weights_kernel, dim3(blocks), dim3(256), 0, stream, w, wfwd, wdgrad, cout, cin, cin_real,
                     taps);
  SRPDE_LAUNCH_CHECK("srpde_pack_conv_weights");
  return 0;
}

}  // extern "C"
