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

  float* red = smem;  // [WM][BN] -- the K loop ended with a barrier, LDS is free
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


// --------------- forward x6: fp32 products from 3-way bf16 splits --------------------
// gfx950 has no xf32 MFMA and its fp32 MFMA runs at 1/16 of the bf16 rate.  Every fp32
// operand x is split exactly into x = hi + mid + lo (three RNE bf16 pieces: 24 significand
// bits) and a*b is formed from the six partial products whose magnitude reaches 2^-16 of
// the leading one:  ah*bh + ah*bm + am*bh + am*bm + ah*bl + al*bh  (dropped terms <= 2^-23
// relative), each on v_mfma_f32_32x32x16_bf16 with fp32 accumulation -- an fp32 GEMM to
// within fp32 rounding (checked against fp64 in tests/test_gpu_kernels.py) at up to 16/6 x
// the fp32-MFMA rate.  Weights are split once per step into three bf16 planes
// (srpde_split_weights); activations arrive fp32 by LDS-DMA exactly as in v2 and are split
// in registers right after their ds_read, so the A side needs no extra HBM or LDS bytes.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// upper 16 bits of two floats packed as a bf16 pair (element 0 = lo_e, element 1 = hi_e)
__device__ __forceinline__ unsigned pack_hi16(float lo_e, float hi_e) {
  return __builtin_amdgcn_perm(__float_as_uint(hi_e), __float_as_uint(lo_e), 0x07060302u);
}

// Truncation split (exact): hi = top 8 significant bits, r = x - hi (exact), mid = top 8
// bits of r, lo = r - mid (exact and itself a bf16).  x == hi + mid + lo bit-for-bit; two
// AND/SUB pairs and three byte-permutes per element pair, no conversions.
__device__ __forceinline__ void split3(const float4 a, const float4 b, bf16x8& hi, bf16x8& mi, bf16x8& lo) {
  typedef float f2v __attribute__((ext_vector_type(2)));
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  auto trunc2 = [](f2v x) {
    return f2v{__uint_as_float(__float_as_uint(x.x) & 0xffff0000u), __uint_as_float(__float_as_uint(x.y) & 0xffff0000u)};
  };
  u32x4 H, M, L;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f2v x = {v[2 * k], v[2 * k + 1]};
    const f2v r = x - trunc2(x);      // v_pk_add_f32
    const f2v q = r - trunc2(r);
    H[k] = pack_hi16(x.x, x.y);
    M[k] = pack_hi16(r.x, r.y);
    L[k] = pack_hi16(q.x, q.y);
  }
  hi = __builtin_bit_cast(bf16x8, H);
  mi = __builtin_bit_cast(bf16x8, M);
  lo = __builtin_bit_cast(bf16x8, L);
}

// 32-bf16 (64-B) weight rows: 16-B chunk c of row r sits in slot c ^ ((r >> 2) & 3)
__device__ __forceinline__ int swzb(int r, int c) { return c ^ ((r >> 2) & 3); }


template <int BM, int BN, int WM, int WN, int SRB, int HP>
__global__ __launch_bounds__(WM * WN * 64, WM * WN >= 8 ? 1 : 2) void conv_fwd_x6_kernel(ConvParams p, const __bf16* __restrict__ wsp) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN, TI = TM / 32, TJ = TN / 32;
  constexpr int AI = BM / (8 * NW);        // A DMA wave-instructions (8 rows x 128 B) per wave
  constexpr int BTOT = 3 * BN / 16;        // B DMA instructions per stage (16 rows x 64 B)
  constexpr int BPW = (BTOT + NW - 1) / NW;
  constexpr int A_BYTES = BM * ROW2;
  constexpr int BP_BYTES = BN * 64;        // one bf16 plane of the B tile
  constexpr int STAGE = A_BYTES + 3 * BP_BYTES;
  constexpr int NSB = BM / SRB;
  static_assert(AI >= 1 && BM % (8 * NW) == 0, "A DMA split");
  static_assert(BM % SRB == 0 && WM % NSB == 0, "statistics sub-blocks");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* lds = reinterpret_cast<char*>(smem);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wmi = wave % WM, wni = wave / WM;
  const int nbn = (p.Cout + BN - 1) / BN;
  const int nbm = (p.P + BM - 1) / BM;
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
  const size_t plane = (size_t)p.Cout * p.K;   // bf16 elements per weight plane
  const int32x4 rsw = make_rsrc(wsp, (unsigned)(3 * plane * 2));

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
  // B: instruction q = plane * (BN/16) + 16-row block; lane -> (row, slot), fetches chunk swzb^-1
  int b_off[BPW];
#pragma unroll
  for (int j = 0; j < BPW; ++j) {
    const int q = wave + j * NW;
    const int pl = q / (BN / 16), rb = q - pl * (BN / 16);
    const int r = rb * 16 + (lane >> 2);
    const int c = swzb(r, lane & 3);
    const int nn = n0 + r;
    b_off[j] = (q < BTOT && nn < p.Cout) ? (int)((pl * plane + (size_t)nn * p.K + c * 8) * 2) : -1;
  }

  const int nall = p.K / BK2;
  const int s_beg = tail ? (piece * nall) / p.tsplit : 0;
  const int s_end = tail ? ((piece + 1) * nall) / p.tsplit : nall;
  const int taps = p.ksize * p.ksize;
  int nx_tap = s_beg % taps, nx_ch = (s_beg / taps) * BK2;
  int nx_ky = nx_tap / p.ksize, nx_kx = nx_tap - nx_ky * p.ksize;
  auto issue = [&](int buf) {
    const int tap = nx_tap, ch0 = nx_ch;
    const int k0 = tap * p.Cin + ch0;
    const int tsh = ((nx_ky - kc) * p.W + (nx_kx - kc)) * p.dil * p.sign;
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
    char* bbase = abase + A_BYTES;
#pragma unroll
    for (int j = 0; j < BPW; ++j) {
      const int q = wave + j * NW;
      if (q < BTOT) {
        const unsigned off = b_off[j] >= 0 ? (unsigned)(b_off[j] + k0 * 2) : OOB;
        dma16(rsw, off, lds_addr_of(bbase + q * 1024));
      }
    }
  };

  floatx16 acc[TI][TJ], part[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int lr = lane & 31, lh = lane >> 5;
  const int wm0 = wmi * TM, wn0 = wni * TN;
  issue(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // one stage; FRESH (compile time) starts the partial chain from a literal zero
  auto stage = [&](int s, auto fresh_tag) {
    constexpr bool FRESH = decltype(fresh_tag)::value;
    const int buf = (s - s_beg) & 1;
    if (s + 1 < s_end && !(p.dbg & 1)) issue(buf ^ 1);
    const char* a = lds + buf * STAGE;
    const char* b = a + A_BYTES;
#pragma unroll
    for (int g = 0; g < BK2 / 16; ++g) {
      bf16x8 ah[TI], am[TI], al[TI], bh[TJ], bm[TJ], bl[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int r = wm0 + i * 32 + lr;
        const int c = 4 * g + 2 * lh;
        const float4 x0 = *reinterpret_cast<const float4*>(a + r * ROW2 + swz(r, c) * 16);
        const float4 x1 = *reinterpret_cast<const float4*>(a + r * ROW2 + swz(r, c + 1) * 16);
        split3(x0, x1, ah[i], am[i], al[i]);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int r = wn0 + j * 32 + lr;
        const int o = r * 64 + swzb(r, 2 * g + lh) * 16;
        bh[j] = *reinterpret_cast<const bf16x8*>(b + o);
        bm[j] = *reinterpret_cast<const bf16x8*>(b + BP_BYTES + o);
        bl[j] = *reinterpret_cast<const bf16x8*>(b + 2 * BP_BYTES + o);
      }
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          floatx16 c0;
          if (FRESH && g == 0)
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], floatx16{}, 0, 0, 0);  // small terms first
          else
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], part[i][j], 0, 0, 0);
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], c0, 0, 0, 0);
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bm[j], c0, 0, 0, 0);
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bh[j], c0, 0, 0, 0);
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bm[j], c0, 0, 0, 0);
          part[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], c0, 0, 0, 0);
        }
    }
    if (!(p.dbg & 2)) {   // (dbg bit 2: diagnostics only, results wrong)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  };
  for (int s = s_beg; s < s_end; s += HP) {
    stage(s, std::true_type{});
#pragma unroll
    for (int h = 1; h < HP; ++h)
      if (s + h < s_end) stage(s + h, std::false_type{});
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] += part[i][j];
  }

  x6_finish<BM, BN, WM, WN, SRB>(p, acc, tail, wg, nfull, piece, m0, n0, wmi, wni, lane, smem);
}

// x6p: the same convolution with the activations arriving pre-split (three bf16 planes
// [3][P][c], srpde_split_planes): both operands are DMA'd as bf16 and read as MFMA fragments
// directly -- no VALU split in the loop.  A rows are 64 B per plane per stage (swzb swizzle,
// source-side, like the weights).
template <int BM, int BN, int WM, int WN, int SRB, int HP>
__global__ __launch_bounds__(WM * WN * 64, WM * WN >= 8 ? 1 : 2) void conv_fwd_x6p_kernel(ConvParams p, const __bf16* __restrict__ wsp) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN, TI = TM / 32, TJ = TN / 32;
  constexpr int ATOT = 3 * BM / 16, APW = (ATOT + NW - 1) / NW;   // A DMA instructions (16 rows x 64 B)
  constexpr int BTOT = 3 * BN / 16, BPW = (BTOT + NW - 1) / NW;
  constexpr int AP_BYTES = BM * 64, BP_BYTES = BN * 64;
  constexpr int STAGE = 3 * (AP_BYTES + BP_BYTES);
  constexpr int NSB = BM / SRB;
  static_assert(BM % SRB == 0 && WM % NSB == 0, "statistics sub-blocks");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* lds = reinterpret_cast<char*>(smem);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wmi = wave % WM, wni = wave / WM;
  const int nbn = (p.Cout + BN - 1) / BN;
  const int nbm = (p.P + BM - 1) / BM;
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

  const int32x4 rs0 = make_rsrc(p.x0p, (unsigned)((size_t)3 * p.P * p.c0 * 2));
  const int c1s = p.c1 ? p.c1 : p.c0;
  const int32x4 rs1 = make_rsrc(p.c1 ? p.x1p : p.x0p, (unsigned)((size_t)3 * p.P * c1s * 2));
  const size_t plane = (size_t)p.Cout * p.K;
  const int32x4 rsw = make_rsrc(wsp, (unsigned)(3 * plane * 2));

  // A instructions: q = plane * (BM/16) + 16-row block; lane -> (row, slot), fetches chunk swzb
  unsigned a_o0[APW], a_o1[APW], a_mask[APW];
#pragma unroll
  for (int i = 0; i < APW; ++i) {
    const int q = wave + i * NW;
    const int pl = q / (BM / 16), rb = q - pl * (BM / 16);
    const int r = rb * 16 + (lane >> 2);
    const int c = swzb(r, lane & 3);
    const int m = m0 + r;
    unsigned mask = 0;
    int pix = 0;
    if (q < ATOT && m < p.P) {
      const int rem = m % HW, yy = rem / p.W, xx = rem - yy * p.W;
      pix = m;
      for (int t = 0; t < p.ksize * p.ksize; ++t) {
        const int ky = t / p.ksize, kx = t - ky * p.ksize;
        const int iy = yy + (ky - kc) * p.dil * p.sign, ix = xx + (kx - kc) * p.dil * p.sign;
        if (iy >= 0 && iy < p.H && ix >= 0 && ix < p.W) mask |= 1u << t;
      }
    }
    a_mask[i] = mask;
    a_o0[i] = (unsigned)(((size_t)pl * p.P * p.c0 + (size_t)pix * p.c0 + c * 8) * 2);
    a_o1[i] = (unsigned)(((size_t)pl * p.P * c1s + (size_t)pix * c1s + c * 8) * 2);
  }
  int b_off[BPW];
#pragma unroll
  for (int j = 0; j < BPW; ++j) {
    const int q = wave + j * NW;
    const int pl = q / (BN / 16), rb = q - pl * (BN / 16);
    const int r = rb * 16 + (lane >> 2);
    const int c = swzb(r, lane & 3);
    const int nn = n0 + r;
    b_off[j] = (q < BTOT && nn < p.Cout) ? (int)((pl * plane + (size_t)nn * p.K + c * 8) * 2) : -1;
  }

  const int nall = p.K / BK2;
  const int s_beg = tail ? (piece * nall) / p.tsplit : 0;
  const int s_end = tail ? ((piece + 1) * nall) / p.tsplit : nall;
  const int taps = p.ksize * p.ksize;
  int nx_tap = s_beg % taps, nx_ch = (s_beg / taps) * BK2;
  int nx_ky = nx_tap / p.ksize, nx_kx = nx_tap - nx_ky * p.ksize;
  auto issue = [&](int buf) {
    const int tap = nx_tap, ch0 = nx_ch;
    const int k0 = tap * p.Cin + ch0;
    const int tsh = ((nx_ky - kc) * p.W + (nx_kx - kc)) * p.dil * p.sign;
    const bool second = ch0 >= p.c0;
    const int32x4 rs = second ? rs1 : rs0;
    const int cs = second ? c1s : p.c0;
    const int cb = second ? ch0 - p.c0 : ch0;
    const unsigned sadd = (unsigned)((tsh * cs + cb) * 2);
    ++nx_tap;
    if (++nx_kx == p.ksize) { nx_kx = 0; ++nx_ky; }
    if (nx_tap == taps) {
      nx_tap = 0; nx_ky = 0; nx_kx = 0;
      nx_ch += BK2;
    }
    char* abase = lds + buf * STAGE;
#pragma unroll
    for (int i = 0; i < APW; ++i) {
      const int q = wave + i * NW;
      if (q < ATOT) {
        const unsigned base = second ? a_o1[i] : a_o0[i];
        const unsigned off = ((a_mask[i] >> tap) & 1u) ? base + sadd : OOB;
        dma16(rs, off, lds_addr_of(abase + q * 1024));
      }
    }
    char* bbase = abase + 3 * AP_BYTES;
#pragma unroll
    for (int j = 0; j < BPW; ++j) {
      const int q = wave + j * NW;
      if (q < BTOT) {
        const unsigned off = b_off[j] >= 0 ? (unsigned)(b_off[j] + k0 * 2) : OOB;
        dma16(rsw, off, lds_addr_of(bbase + q * 1024));
      }
    }
  };

  floatx16 acc[TI][TJ], part[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int lr = lane & 31, lh = lane >> 5;
  const int wm0 = wmi * TM, wn0 = wni * TN;
  issue(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  auto stage = [&](int s, auto fresh_tag) {
    constexpr bool FRESH = decltype(fresh_tag)::value;
    const int buf = (s - s_beg) & 1;
    if (s + 1 < s_end) issue(buf ^ 1);
    const char* a = lds + buf * STAGE;
    const char* b = a + 3 * AP_BYTES;
#pragma unroll
    for (int g = 0; g < BK2 / 16; ++g) {
      bf16x8 ah[TI], am[TI], al[TI], bh[TJ], bm[TJ], bl[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int r = wm0 + i * 32 + lr;
        const int o = r * 64 + swzb(r, 2 * g + lh) * 16;
        ah[i] = *reinterpret_cast<const bf16x8*>(a + o);
        am[i] = *reinterpret_cast<const bf16x8*>(a + AP_BYTES + o);
        al[i] = *reinterpret_cast<const bf16x8*>(a + 2 * AP_BYTES + o);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int r = wn0 + j * 32 + lr;
        const int o = r * 64 + swzb(r, 2 * g + lh) * 16;
        bh[j] = *reinterpret_cast<const bf16x8*>(b + o);
        bm[j] = *reinterpret_cast<const bf16x8*>(b + BP_BYTES + o);
        bl[j] = *reinterpret_cast<const bf16x8*>(b + 2 * BP_BYTES + o);
      }
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          floatx16 c0;
          if (FRESH && g == 0)
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], floatx16{}, 0, 0, 0);
          else
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], part[i][j], 0, 0, 0);
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], c0, 0, 0, 0);
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bm[j], c0, 0, 0, 0);
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bh[j], c0, 0, 0, 0);
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bm[j], c0, 0, 0, 0);
          part[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], c0, 0, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  for (int s = s_beg; s < s_end; s += HP) {
    stage(s, std::true_type{});
#pragma unroll
    for (int h = 1; h < HP; ++h)
      if (s + h < s_end) stage(s + h, std::false_type{});
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] += part[i][j];
  }
  x6_finish<BM, BN, WM, WN, SRB>(p, acc, tail, wg, nfull, piece, m0, n0, wmi, wni, lane, smem);
}

// [P][c] fp32 view -> three bf16 planes [3][P][c] (truncation split: hi, mid, lo exact)
__global__ void split_planes_kernel(const float* __restrict__ x, int ldx, int c, long long P,
                                    __bf16* __restrict__ out) {
  const int cq = c / 8;
  const long long total = P * cq;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const long long r = e / cq;
    const int ch = (int)(e - r * cq) * 8;
    const float* src = x + r * ldx + ch;
    const float4 a = *reinterpret_cast<const float4*>(src);
    const float4 b = *reinterpret_cast<const float4*>(src + 4);
    bf16x8 h, m, l;
    split3(a, b, h, m, l);
    const long long o = r * c + ch;
    *reinterpret_cast<bf16x8*>(out + o) = h;
    *reinterpret_cast<bf16x8*>(out + P * c + o) = m;
    *reinterpret_cast<bf16x8*>(out + 2 * P * c + o) = l;
  }
}

// fp32 -> three bf16 planes [3][n] (hi, mid, lo) for the x6 kernels' weight operand
__global__ void split_weights_kernel(const float* __restrict__ w, __bf16* __restrict__ out, long long n) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const float v = w[e];
    const __bf16 h = (__bf16)v;
    const float r = v - (float)h;
    const __bf16 m = (__bf16)r;
    out[e] = h;
    out[n + e] = m;
    out[2 * n + e] = (__bf16)(r - (float)m);
  }
}

// ------------------------------ weight gradient --------------------------------


constexpr int BKP = 16;  // pixels per stage

template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradParams p) {
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
      if (e < A_TOTAL && px < pend && col < p.Cout)
        v = *reinterpret_cast<const float4*>(p.dy + (size_t)px * p.lddy + col);
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

// ------------------- weight gradient x6: 3-way bf16 split, 6 MFMA products -------------------
// dW tile [BM couts][BN k-columns] over a pixel chunk, 16 pixels per stage.  Both operands
// are pixel-major in HBM and the MFMA wants 8 consecutive PIXELS per lane, so each stage is
// register-staged (one pixel row x 8 columns per task), split into hi/mid/lo bf16 and
// written as three [16 pixel][columns] bf16 images; the MFMA fragments come back through
// ds_read_b64_tr_b16 (hardware transpose: a 16-lane group reads 4 pixel rows x 16 columns
// and each lane receives its column's 4 pixels).  Chunk XOR swizzle s(row) keeps the four
// rows of a transposed read on distinct banks.  One barrier per stage (double-buffered
// images); partial MFMA chains of HP stages (two-level accumulation, as the forward).
constexpr int BKX = 16;    // pixels per wgrad-x6 stage

template <int BM, int BN, int WM, int WN, int HP>
__global__ __launch_bounds__(256, 2) void conv_wgrad_x6_kernel(WgradParams p) {
  constexpr int TM = BM / WM, TN = BN / WN, TI = TM / 32, TJ = TN / 32;
  constexpr int RA = BM * 2, RBB = BN * 2;             // image row bytes (bf16)
  constexpr int IMG_A = BKX * RA, IMG_B = BKX * RBB;    // one plane
  constexpr int STAGE = 3 * (IMG_A + IMG_B);
  constexpr int TA = (2 * BM + 255) / 256, TB = (2 * BN + 255) / 256;   // staging tasks per thread
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* lds = reinterpret_cast<char*>(smem);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wmi = wave % WM, wni = wave / WM;
  const int nbm = (p.Cout + BM - 1) / BM, nbn = (p.K + BN - 1) / BN;
  const int ntile = nbm * nbn;
  const int bid = xcd_remap(blockIdx.x, ntile * p.splits);
  const int split = bid / ntile, tile = bid - split * ntile;
  const int mt = tile / nbn, nt = tile - mt * nbn;
  const int m0 = mt * BM, n0 = nt * BN;
  const int pbeg = split * p.chunk, pend = min(p.P, pbeg + p.chunk);
  const int HW = p.H * p.W, kc = p.ksize >> 1;
  const int ld1 = p.c1 ? p.ldx1 : p.ldx0;

  // staging tasks: (pixel row, 8-column chunk); A = dY[pix][m0 + 8c ..], B = X[pix + off][k ..]
  int a_row[TA], a_col[TA];
  bool a_on[TA];
#pragma unroll
  for (int i = 0; i < TA; ++i) {
    const int q = tid + 256 * i;
    a_on[i] = q < 2 * BM;
    a_row[i] = q / (BM / 8);
    a_col[i] = (q % (BM / 8)) * 8;
  }
  int b_row[TB], b_col[TB], b_dy[TB], b_dx[TB], b_sh[TB], b_ch[TB];
  bool b_on[TB], b_second[TB];
#pragma unroll
  for (int i = 0; i < TB; ++i) {
    const int q = tid + 256 * i;
    b_row[i] = q / (BN / 8);
    b_col[i] = (q % (BN / 8)) * 8;
    const int k = n0 + b_col[i];
    b_on[i] = q < 2 * BN && k < p.K;
    const int tap = b_on[i] ? k / p.Cin : 0;
    const int ch = k - tap * p.Cin;
    const int ky = tap / p.ksize, kx = tap - ky * p.ksize;
    b_dy[i] = (ky - kc) * p.dil;
    b_dx[i] = (kx - kc) * p.dil;
    b_sh[i] = b_dy[i] * p.W + b_dx[i];
    b_second[i] = ch >= p.c0;
    b_ch[i] = b_second[i] ? ch - p.c0 : ch;
  }

  // image coordinates of each B task's pixel, advanced by BKX pixels per stage (no divisions
  // in the loop; BKX < 2 W for every layer here, W >= 10)
  int b_y[TB], b_x[TB];
#pragma unroll
  for (int i = 0; i < TB; ++i) {
    const int pix = pbeg + b_row[i];
    const int rem = pix % HW;
    b_y[i] = rem / p.W;
    b_x[i] = rem - b_y[i] * p.W;
  }
  auto advance = [&]() {
#pragma unroll
    for (int i = 0; i < TB; ++i) {
      int x = b_x[i] + BKX, y = b_y[i];
      while (x >= p.W) { x -= p.W; ++y; }
      while (y >= p.H) y -= p.H;
      b_x[i] = x; b_y[i] = y;
    }
  };
  // two register sets: stage s+2 is loaded while stage s computes and stage s+1 is stored
  float4 ra[2][TA][2], rb[2][TB][2];
  auto load_stage = [&](int pbase, auto set_tag) {
    constexpr int SET = decltype(set_tag)::value;
#pragma unroll
    for (int i = 0; i < TA; ++i) {
      const int pix = pbase + a_row[i], m = m0 + a_col[i];
      float4 v0 = make_float4(0.f, 0.f, 0.f, 0.f), v1 = v0;
      if (a_on[i] && pix < pend && m < p.Cout) {
        const float* src = p.dy + (size_t)pix * p.lddy + m;
        v0 = *reinterpret_cast<const float4*>(src);
        v1 = *reinterpret_cast<const float4*>(src + 4);   // Cout % 8 == 0
      }
      ra[SET][i][0] = v0; ra[SET][i][1] = v1;
    }
#pragma unroll
    for (int i = 0; i < TB; ++i) {
      const int pix = pbase + b_row[i];
      float4 v0 = make_float4(0.f, 0.f, 0.f, 0.f), v1 = v0;
      if (b_on[i] && pix < pend) {
        const int iy = b_y[i] + b_dy[i], ix = b_x[i] + b_dx[i];
        if (iy >= 0 && iy < p.H && ix >= 0 && ix < p.W) {
          const float* src = b_second[i] ? p.x1 + (size_t)(pix + b_sh[i]) * ld1 + b_ch[i]
                                         : p.x0 + (size_t)(pix + b_sh[i]) * p.ldx0 + b_ch[i];
          v0 = *reinterpret_cast<const float4*>(src);
          v1 = *reinterpret_cast<const float4*>(src + 4);
        }
      }
      rb[SET][i][0] = v0; rb[SET][i][1] = v1;
    }
  };
  auto store_stage = [&](auto set_tag) {   // set SET -> LDS buffer SET
    constexpr int SET = decltype(set_tag)::value;
    char* base = lds + SET * STAGE;
#pragma unroll
    for (int i = 0; i < TA; ++i) {
      if (!a_on[i]) continue;
      bf16x8 h, m, l;
      split3(ra[SET][i][0], ra[SET][i][1], h, m, l);
      const int o = wx_off<RA>(a_row[i], a_col[i] >> 3);
      *reinterpret_cast<bf16x8*>(base + o) = h;
      *reinterpret_cast<bf16x8*>(base + IMG_A + o) = m;
      *reinterpret_cast<bf16x8*>(base + 2 * IMG_A + o) = l;
    }
#pragma unroll
    for (int i = 0; i < TB; ++i) {
      if (tid + 256 * i >= 2 * BN) continue;
      bf16x8 h, m, l;
      split3(rb[SET][i][0], rb[SET][i][1], h, m, l);
      const int o = 3 * IMG_A + wx_off<RBB>(b_row[i], b_col[i] >> 3);
      *reinterpret_cast<bf16x8*>(base + o) = h;
      *reinterpret_cast<bf16x8*>(base + IMG_B + o) = m;
      *reinterpret_cast<bf16x8*>(base + 2 * IMG_B + o) = l;
    }
  };

  floatx16 acc[TI][TJ], part[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int lr = lane & 31, lh = lane >> 5;
  const int wm0 = wmi * TM, wn0 = wni * TN;
  const int nsteps = (pend - pbeg + BKX - 1) / BKX;

  // stage s (parity PAR = s & 1 at compile time): LDS buffer PAR holds it
  auto stage = [&](int s, auto fresh_tag, auto par_tag) {
    constexpr bool FRESH = decltype(fresh_tag)::value;
    constexpr int PAR = decltype(par_tag)::value;
    if (s + 2 < nsteps) {
      load_stage(pbeg + (s + 2) * BKX, par_tag);
      advance();
    }
    const char* img = lds + PAR * STAGE;
    bf16x8 ah[TI], am[TI], al[TI];
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      ah[i] = tr_frag<bf16x8, RA>(img, wm0 + 32 * i, lane);
      am[i] = tr_frag<bf16x8, RA>(img + IMG_A, wm0 + 32 * i, lane);
      al[i] = tr_frag<bf16x8, RA>(img + 2 * IMG_A, wm0 + 32 * i, lane);
    }
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const bf16x8 bh = tr_frag<bf16x8, RBB>(img + 3 * IMG_A, wn0 + 32 * j, lane);
      const bf16x8 bm = tr_frag<bf16x8, RBB>(img + 3 * IMG_A + IMG_B, wn0 + 32 * j, lane);
      const bf16x8 bl = tr_frag<bf16x8, RBB>(img + 3 * IMG_A + 2 * IMG_B, wn0 + 32 * j, lane);
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        floatx16 c0;
        if (FRESH)
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh, floatx16{}, 0, 0, 0);
        else
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh, part[i][j], 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl, c0, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bm, c0, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bh, c0, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bm, c0, 0, 0, 0);
        part[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh, c0, 0, 0, 0);
      }
    }
    if (s + 1 < nsteps) store_stage(std::integral_constant<int, 1 - PAR>{});
    __syncthreads();
  };

  typedef std::integral_constant<int, 0> P0;
  typedef std::integral_constant<int, 1> P1;
  if (nsteps > 0) {
    load_stage(pbeg, P0{});
    advance();
    store_stage(P0{});
  }
  if (nsteps > 1) {
    load_stage(pbeg + BKX, P1{});
    advance();
  }
  __syncthreads();
  static_assert(HP == 4, "stage parities are unrolled for HP = 4");
  for (int s = 0; s < nsteps; s += HP) {
    stage(s, std::true_type{}, P0{});
    if (s + 1 < nsteps) stage(s + 1, std::false_type{}, P1{});
    if (s + 2 < nsteps) stage(s + 2, std::false_type{}, P0{});
    if (s + 3 < nsteps) stage(s + 3, std::false_type{}, P1{});
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] += part[i][j];
  }

  // slab [split][Cout][K]
  float* out = p.part + (size_t)split * p.Cout * p.K;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int n = n0 + wn0 + 32 * j + lr;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < p.Cout && n < p.K) out[(size_t)m * p.K + n] = acc[i][j][r];
      }
    }
}

// first level of a two-level slab sum (few elements, many slabs: enc1.conv1's 2304 weights over
// ~2048 slabs): slab g*G <- sum of slabs [g*G, g*G + G) in order, one thread per (element, group)
__global__ void slab_group_sum_kernel(float* __restrict__ part, int splits, int G, long long total) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long ngroups = (splits + G - 1) / G;
  if (i >= total * ngroups) return;
  const long long g = i / total, e = i - g * total;
  const int q0 = (int)(g * G), q1 = min(splits, q0 + G);
  float s = 0.f;
  for (int q = q0; q < q1; ++q) s += part[(size_t)q * total + e];
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
  if (e < total)
    for (int q = grp; q < splits; q += 4) s += part[(size_t)q * stride * cout * K + e];
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
    hipLaunchKernelGGL(slab_group_sum_kernel, dim3((int)((work + 255) / 256)), dim3(256), 0, stream,
                       const_cast<float*>(part), splits, G, total);
    SRPDE_LAUNCH_CHECK("srpde_conv_wgrad(reduce groups)");
    stride = G;
    splits = (splits + G - 1) / G;
  }
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, stream, part, dw, splits, cout, cin, cin_real,
                     taps, accumulate, stride);
  SRPDE_LAUNCH_CHECK("srpde_conv_wgrad(reduce)");
  return 0;
}

// ------ weight gradient of a conv on a <= 3-channel input, with its BN (+ReLU) backward applied on the fly ------
// enc1.conv1 (models.py:16,21 on the 3-channel input): dW[co][ci][tap] = sum_p dy[p][co] x[p + off(tap)][ci]
// is a Cout x 27 sum of outer products over every pixel -- HBM-bound on reading dy, so dy is never
// written: each thread forms dy = gamma*invstd*(dz - m1 - xhat*m2) (dz = da where the BN+ReLU output
// is positive) for 4 channels of a pixel row from da and y with bn_bwd_apply_kernel's expressions,
// and accumulates its 9 taps x 3 input channels x 4 products in fp32.  Rows of a block are combined
// across lanes and waves in a fixed order and written as one slab [split][Cout][27] (k = tap*3 + ci,
// the other wgrad kernels' K order), summed in fixed order by wgrad_reduce.  x: NHWC rows of ldx >= 4
// floats (channels past 3 ignored).
// Per block: a contiguous pixel range walked in tiles of TP pixels.  Each tile's y and da rows come
// in as float4 loads (every thread TP*C/1024 of each, all in flight), dy is formed in registers and
// parked in LDS next to the tile's x halo (TP + 2*(W+1)*dil rows, zero outside the tensor); then a
// thread owns one channel of a quarter of the tile's pixels and does the 27 products per pixel from
// LDS (x reads are wave-wide broadcasts).
constexpr int C3_TP = 64;
template <int C>
__global__ __launch_bounds__(256) void wgrad_bnb_c3_kernel(const float* __restrict__ y, int ldy,
                                                           const float* __restrict__ da, int ldda,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const float* __restrict__ m1v, const float* __restrict__ m2v,
                                                           int relu, const float* __restrict__ x, int ldx, int H, int W,
                                                           int dil, int P, int chunk, float* __restrict__ part) {
  constexpr int TP = C3_TP, KK = 27, C4 = C / 4;
  constexpr int RS = 256 / C;                 // pixel groups in the product phase
  constexpr int LPT = TP * C4 / 256;          // float4 loads per thread per tensor and tile
  static_assert(256 % C == 0 && (TP * C4) % 256 == 0 && TP % RS == 0, "tile geometry");
  extern __shared__ float4 c3_lds[];
  float* dys = reinterpret_cast<float*>(c3_lds);                  // [TP][C]
  float4* xs = c3_lds + TP * C4;                                   // [TP + 2 * halo][4]
  float (*red)[9][C] = reinterpret_cast<float (*)[9][C]>(c3_lds);   // after the last tile: [RS][9][C]
  const int tid = threadIdx.x;
  const int halo = (W + 1) * dil, HW = H * W;
  // load-phase coordinates: float4 j of a tile is (pixel j / C4, channels 4 * (j % C4))
  const int lc = 4 * (tid % C4);
  const float4 mu = *reinterpret_cast<const float4*>(mean + lc);
  const float4 is = *reinterpret_cast<const float4*>(invstd + lc);
  const float4 g = *reinterpret_cast<const float4*>(gamma + lc);
  const float4 b = *reinterpret_cast<const float4*>(beta + lc);
  const float4 m1 = *reinterpret_cast<const float4*>(m1v + lc);
  const float4 m2 = *reinterpret_cast<const float4*>(m2v + lc);
  const float4 k = make_float4(g.x * is.x, g.y * is.y, g.z * is.z, g.w * is.w);
  // product-phase coordinates
  const int c = tid % C, q = C == 64 ? __builtin_amdgcn_readfirstlane(tid / C) : tid / C;
  float acc[KK];
#pragma unroll
  for (int i = 0; i < KK; ++i) acc[i] = 0.f;
  const int pb = blockIdx.x * chunk, pe = min(P, pb + chunk);
  for (int t0 = pb; t0 < pe; t0 += TP) {
    float4 v[LPT], d[LPT];
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int pp = t0 + (tid + 256 * i) / C4;
      if (pp < pe) {
        v[i] = *reinterpret_cast<const float4*>(y + (size_t)pp * ldy + lc);
        d[i] = *reinterpret_cast<const float4*>(da + (size_t)pp * ldda + lc);
      } else {
        v[i] = d[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    const int nx = TP + 2 * halo;
    for (int j = tid; j < nx; j += 256) {
      const int pp = t0 - halo + j;
      xs[j] = (pp >= 0 && pp < P) ? *reinterpret_cast<const float4*>(x + (size_t)pp * ldx) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int j = tid + 256 * i, pl = j / C4;
      float4 o;
      float xh, dz;
#define BN_APPLY(X)                                            \
  xh = (v[i].X - mu.X) * is.X;                                 \
  dz = (!(relu & 1) || xh * g.X + b.X > 0.f) ? d[i].X : 0.f;   \
  o.X = (dz - m1.X - xh * m2.X) * k.X;
      BN_APPLY(x) BN_APPLY(y) BN_APPLY(z) BN_APPLY(w)
#undef BN_APPLY
      if (t0 + pl >= pe) o = make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(dys + pl * C + lc) = o;
    }
    __syncthreads();
    {
      // this thread's pixels t0 + q, t0 + q + RS, ...: image coordinates stepped incrementally (q is
      // wave-uniform when a wave holds one pixel row of channels, so this is scalar work there)
      const int p0 = t0 + q;
      int rem = p0 % HW;
      int py = rem / W, px = rem - py * W;
      for (int pl = q; pl < TP; pl += RS) {
        const float o = dys[pl * C + c];
#pragma unroll
        for (int ty = 0; ty < 3; ++ty) {
          if ((unsigned)(py + (ty - 1) * dil) >= (unsigned)H) continue;
#pragma unroll
          for (int tx = 0; tx < 3; ++tx) {
            if ((unsigned)(px + (tx - 1) * dil) >= (unsigned)W) continue;
            const float4 xv = xs[pl + halo + ((ty - 1) * W + (tx - 1)) * dil];
            float* a = acc + (ty * 3 + tx) * 3;
            a[0] += o * xv.x; a[1] += o * xv.y; a[2] += o * xv.z;
          }
        }
        px += RS;
        while (px >= W) { px -= W; if (++py == H) py = 0; }
      }
    }
    __syncthreads();
  }
  // combine the RS pixel groups in three rounds of nine k-values (keeps the LDS footprint at one
  // tile, so a weight-gradient workgroup of the side stream still fits next to this block)
  float* out = part + (size_t)blockIdx.x * C * KK;
#pragma unroll
  for (int rd = 0; rd < 3; ++rd) {
#pragma unroll
    for (int i = 0; i < 9; ++i) red[q][i][c] = acc[rd * 9 + i];
    __syncthreads();
    for (int e = tid; e < C * 9; e += 256) {
      const int co = e / 9, kk = e - co * 9;
      float t = 0.f;
#pragma unroll
      for (int r = 0; r < RS; ++r) t += red[r][kk][co];
      out[co * KK + rd * 9 + kk] = t;
    }
    __syncthreads();
  }
}

static void wgrad_bnb_c3_split(long long P, int C, int* chunk, int* splits) {
  // ~2048 blocks (8 per CU), chunks a multiple of the rows a block covers per sweep
  const int rs = C3_TP;
  long long c = (P + 2047) / 2048;
  c = (c + rs - 1) / rs * rs;
  *chunk = (int)c;
  *splits = (int)((P + c - 1) / c);
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


template <int BM, int BN, int WM, int WN, int SRB>
static int launch_fwd_x6(ConvParams p, const __bf16* wsp, hipStream_t st, void* ws, size_t ws_bytes) {
  constexpr int NT = WM * WN * 64;
  const int nbm = ceil_div(p.P, BM), nbn = ceil_div(p.Cout, BN);
  const int T = nbm * nbn;
  const size_t lds = (size_t)2 * (BM * ROW2 + 3 * BN * 64);
  static int slots = [&] {
    int per_cu = 0, dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, conv_fwd_x6_kernel<BM, BN, WM, WN, SRB, 2>, NT, lds);
    if (getenv("SRPDE_CONV_VERBOSE"))
      fprintf(stderr, "conv_fwd_x6<%d,%d,%d,%d>: %d workgroups/CU (LDS %zu B)\n", BM, BN, WM, WN, per_cu, lds);
    return std::max(1, per_cu) * std::max(1, cus);
  }();
  plan_tail(p, T, slots, BM, BN, ws, ws_bytes);
  static const int dbg = [] { const char* e = getenv("SRPDE_CONV_DBG"); return e ? atoi(e) : 0; }();
  p.dbg = dbg;
  const int grid = T - p.ntail + p.ntail * p.tsplit;
  hipLaunchKernelGGL((conv_fwd_x6_kernel<BM, BN, WM, WN, SRB, 2>), dim3(grid), dim3(NT), lds, st, p, wsp);
  SRPDE_LAUNCH_CHECK("srpde_conv_fwd_x6");
  if (p.ntail > 0) {
    hipLaunchKernelGGL((conv_tail_fixup_kernel<BM, BN, SRB>), dim3(p.ntail), dim3(1024), 0, st, p);
    SRPDE_LAUNCH_CHECK("srpde_conv_fwd_x6(tail fixup)");
  }
  return 0;
}

template <int BM, int BN, int WM, int WN, int SRB>
static int launch_fwd_x6p(ConvParams p, const __bf16* wsp, hipStream_t st, void* ws, size_t ws_bytes) {
  constexpr int NT = WM * WN * 64;
  const int nbm = ceil_div(p.P, BM), nbn = ceil_div(p.Cout, BN);
  const int T = nbm * nbn;
  const size_t lds = (size_t)2 * 3 * (BM + BN) * 64;
  static int slots = [&] {
    int per_cu = 0, dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, conv_fwd_x6p_kernel<BM, BN, WM, WN, SRB, 2>, NT, lds);
    return std::max(1, per_cu) * std::max(1, cus);
  }();
  plan_tail(p, T, slots, BM, BN, ws, ws_bytes);
  const int grid = T - p.ntail + p.ntail * p.tsplit;
  hipLaunchKernelGGL((conv_fwd_x6p_kernel<BM, BN, WM, WN, SRB, 2>), dim3(grid), dim3(NT), lds, st, p, wsp);
  SRPDE_LAUNCH_CHECK("srpde_conv_fwd_x6p");
  if (p.ntail > 0) {
    hipLaunchKernelGGL((conv_tail_fixup_kernel<BM, BN, SRB>), dim3(p.ntail), dim3(1024), 0, st, p);
    SRPDE_LAUNCH_CHECK("srpde_conv_fwd_x6p(tail fixup)");
  }
  return 0;
}

// stages per partial MFMA chain (SRPDE_CONV_HP, tuning/diagnostics only; 1000 = no split)
static int conv_hp() {
  static int hp = [] {
    const char* e = getenv("SRPDE_CONV_HP");
    return e ? atoi(e) : 4;
  }();
  return hp;
}

static bool v2_ok(const ConvParams& p) {
  const long long maxld = std::max(p.ldx0, p.c1 ? p.ldx1 : 0);
  return p.c0 % 32 == 0 && p.c1 % 32 == 0 && (long long)p.P * maxld * 4 < (1LL << 31) &&
         (long long)p.Cout * p.K * 4 < (1LL << 31);
}

static int fwd_config(int cout) { return cout % 128 == 0 ? 0 : (cout % 64 == 0 ? 1 : 2); }
static int fwd_bm(int cfg) { return cfg == 0 ? 128 : 256; }

template <int BM, int BN, int WM, int WN>
static int launch_wgrad(const WgradParams& p, hipStream_t st) {
  const int nb = ceil_div(p.Cout, BM) * ceil_div(p.K, BN) * p.splits;
  const size_t lds = (size_t)2 * BKP * ((BM + 4) + (BN + 4)) * sizeof(float);
  hipLaunchKernelGGL((conv_wgrad_kernel<BM, BN, WM, WN>), dim3(nb), dim3(256), lds, st, p);
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

template <int BM, int BN, int WM, int WN>
static int launch_wgrad_x6(const WgradParams& p, hipStream_t st) {
  const int nb = ceil_div(p.Cout, BM) * ceil_div(p.K, BN) * p.splits;
  const size_t lds = (size_t)2 * 3 * BKX * 2 * (BM + BN);
  hipLaunchKernelGGL((conv_wgrad_x6_kernel<BM, BN, WM, WN, 4>), dim3(nb), dim3(256), lds, st, p);
  SRPDE_LAUNCH_CHECK("srpde_conv_wgrad_x6");
  return 0;
}

// Cout = 64 tile: 64x256 (1 workgroup/CU by LDS) or 64x128 (2/CU); SRPDE_WGRAD64 tuning
static bool wgrad64_wide() {
  static const bool wide = [] {
    const char* e = getenv("SRPDE_WGRAD64");
    return e && atoi(e) != 0;
  }();
  return wide;
}

static bool wgrad_v2_ok(const WgradParams& p) {
  static const bool on = [] {
    const char* e = getenv("SRPDE_WGRAD_V2");  // tuning/diagnostics: 0 = register-staged kernel
    return !e || atoi(e) != 0;
  }();
  const long long maxld = std::max(std::max(p.ldx0, p.c1 ? p.ldx1 : 0), p.lddy);
  return on && p.c0 % 32 == 0 && p.c1 % 32 == 0 && (long long)p.P * maxld * 4 < (1LL << 31);
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
                   float* stats, void* workspace, size_t ws_bytes, hipStream_t stream) {
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
  p.ntail = 0; p.tsplit = 1; p.part = nullptr; p.dbg = 0;
  if (v2_ok(p)) {
    switch (fwd_config(cout)) {
      case 0:
        switch (conv_hp()) {
          case 1: return launch_fwd_v2<128, 128, 2, 2, 1>(p, stream, workspace, ws_bytes);
          case 2: return launch_fwd_v2<128, 128, 2, 2, 2>(p, stream, workspace, ws_bytes);
          case 1000: return launch_fwd_v2<128, 128, 2, 2, 1000000>(p, stream, workspace, ws_bytes);
          default: return launch_fwd_v2<128, 128, 2, 2, 4>(p, stream, workspace, ws_bytes);
        }
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

int srpde_conv_x6_supported(int c0, int c1, int cout) {
  return c0 % 32 == 0 && c1 % 32 == 0 && cout % 32 == 0 && c0 + c1 > 0 ? 1 : 0;
}

int srpde_split_weights(const float* w, void* planes, long long n, hipStream_t stream) {
  SRPDE_CHECK_ARG(w && planes && n > 0, "srpde_split_weights: bad arguments");
  const int blocks = (int)std::min<long long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(split_weights_kernel, dim3(blocks), dim3(256), 0, stream, w, static_cast<__bf16*>(planes), n);
  SRPDE_LAUNCH_CHECK("srpde_split_weights");
  return 0;
}

int srpde_conv_fwd_x6(const float* x0, int c0, int ldx0, const float* x1, int c1, int ldx1, const void* wsplit,
                      const float* bias, float* y, int ldy, int n, int h, int w, int cout, int ksize, int dil,
                      int sign, int accumulate, float* stats, void* workspace, size_t ws_bytes, hipStream_t stream) {
  SRPDE_CHECK_ARG(x0 && wsplit && y, "srpde_conv_fwd_x6: null pointer");
  SRPDE_CHECK_ARG(n > 0 && h > 0 && w > 0 && cout > 0, "srpde_conv_fwd_x6: bad shape");
  SRPDE_CHECK_ARG(ksize == 1 || ksize == 3, "srpde_conv_fwd_x6: ksize must be 1 or 3");
  SRPDE_CHECK_ARG(sign == 1 || sign == -1, "srpde_conv_fwd_x6: sign must be +-1");
  SRPDE_CHECK_ARG(srpde_conv_x6_supported(c0, c1, cout), "srpde_conv_fwd_x6: needs c0, c1, cout multiples of 32 "
                  "(c0=%d c1=%d cout=%d)", c0, c1, cout);
  SRPDE_CHECK_ARG(ldx0 % 4 == 0 && (c1 == 0 || ldx1 % 4 == 0), "srpde_conv_fwd_x6: strides must be multiples of 4");
  SRPDE_CHECK_ARG(c1 == 0 || x1 != nullptr, "srpde_conv_fwd_x6: x1 null with c1>0");
  SRPDE_CHECK_ARG(aligned16(x0) && aligned16(wsplit) && (c1 == 0 || aligned16(x1)),
                  "srpde_conv_fwd_x6: inputs must be 16-byte aligned");
  ConvParams p;
  p.x0 = x0; p.c0 = c0; p.ldx0 = ldx0;
  p.x1 = x1; p.c1 = c1; p.ldx1 = ldx1 > 0 ? ldx1 : 4;
  p.w = nullptr; p.bias = bias; p.y = y; p.ldy = ldy;
  p.stats = reinterpret_cast<float2*>(stats);
  p.N = n; p.H = h; p.W = w; p.Cout = cout; p.ksize = ksize; p.dil = dil; p.sign = sign; p.accumulate = accumulate;
  p.P = n * h * w; p.Cin = c0 + c1; p.K = ksize * ksize * p.Cin;
  p.ntail = 0; p.tsplit = 1; p.part = nullptr; p.dbg = 0;
  SRPDE_CHECK_ARG(v2_ok(p) && 3LL * cout * p.K * 2 < (1LL << 31), "srpde_conv_fwd_x6: tensor too large");
  const __bf16* wsp = static_cast<const __bf16*>(wsplit);
  // waves stacked along M (WN = 1) so each activation fragment is split by one wave only
  static const int layout = [] {
    const char* e = getenv("SRPDE_X6_LAYOUT");   // tuning/diagnostics: 1 = 2-D wave grid
    return e ? atoi(e) : 0;
  }();
  switch (fwd_config(cout)) {
    case 0:
      if (layout == 2) return launch_fwd_x6<128, 128, 4, 1, 128>(p, wsp, stream, workspace, ws_bytes);
      return layout == 1 ? launch_fwd_x6<256, 128, 4, 2, 128>(p, wsp, stream, workspace, ws_bytes)
                         : launch_fwd_x6<256, 128, 8, 1, 128>(p, wsp, stream, workspace, ws_bytes);
    case 1:
      return layout == 1 ? launch_fwd_x6<256, 64, 4, 2, 256>(p, wsp, stream, workspace, ws_bytes)
                         : launch_fwd_x6<256, 64, 8, 1, 256>(p, wsp, stream, workspace, ws_bytes);
    default: return launch_fwd_x6<256, 32, 8, 1, 256>(p, wsp, stream, workspace, ws_bytes);
  }
}

int srpde_split_planes(const float* x, int ldx, int c, long long P, void* planes, hipStream_t stream) {
  SRPDE_CHECK_ARG(x && planes && P > 0 && c > 0, "srpde_split_planes: bad arguments");
  SRPDE_CHECK_ARG(c % 8 == 0 && ldx % 4 == 0 && aligned16(x) && aligned16(planes),
                  "srpde_split_planes: c %% 8, ldx %% 4 and 16-byte alignment required (c=%d ldx=%d)", c, ldx);
  const long long total = P * (c / 8);
  const int blocks = (int)std::min<long long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(split_planes_kernel, dim3(blocks), dim3(256), 0, stream, x, ldx, c, P,
                     static_cast<__bf16*>(planes));
  SRPDE_LAUNCH_CHECK("srpde_split_planes");
  return 0;
}

int srpde_conv_fwd_x6p(const void* x0p, int c0, const void* x1p, int c1, const void* wsplit, const float* bias,
                       float* y, int ldy, int n, int h, int w, int cout, int ksize, int dil, int sign, int accumulate,
                       float* stats, void* workspace, size_t ws_bytes, hipStream_t stream) {
  SRPDE_CHECK_ARG(x0p && wsplit && y, "srpde_conv_fwd_x6p: null pointer");
  SRPDE_CHECK_ARG(n > 0 && h > 0 && w > 0 && cout > 0, "srpde_conv_fwd_x6p: bad shape");
  SRPDE_CHECK_ARG(ksize == 1 || ksize == 3, "srpde_conv_fwd_x6p: ksize must be 1 or 3");
  SRPDE_CHECK_ARG(sign == 1 || sign == -1, "srpde_conv_fwd_x6p: sign must be +-1");
  SRPDE_CHECK_ARG(srpde_conv_x6_supported(c0, c1, cout), "srpde_conv_fwd_x6p: needs c0, c1, cout multiples of 32 "
                  "(c0=%d c1=%d cout=%d)", c0, c1, cout);
  SRPDE_CHECK_ARG(c1 == 0 || x1p != nullptr, "srpde_conv_fwd_x6p: x1p null with c1>0");
  SRPDE_CHECK_ARG(aligned16(x0p) && aligned16(wsplit) && (c1 == 0 || aligned16(x1p)),
                  "srpde_conv_fwd_x6p: inputs must be 16-byte aligned");
  ConvParams p;
  p.x0 = nullptr; p.c0 = c0; p.ldx0 = c0;
  p.x1 = nullptr; p.c1 = c1; p.ldx1 = c1 > 0 ? c1 : 4;
  p.x0p = static_cast<const __bf16*>(x0p); p.x1p = static_cast<const __bf16*>(x1p);
  p.w = nullptr; p.bias = bias; p.y = y; p.ldy = ldy;
  p.stats = reinterpret_cast<float2*>(stats);
  p.N = n; p.H = h; p.W = w; p.Cout = cout; p.ksize = ksize; p.dil = dil; p.sign = sign; p.accumulate = accumulate;
  p.P = n * h * w; p.Cin = c0 + c1; p.K = ksize * ksize * p.Cin;
  p.ntail = 0; p.tsplit = 1; p.part = nullptr; p.dbg = 0;
  SRPDE_CHECK_ARG(3LL * p.P * std::max(c0, c1) * 2 < (1LL << 31) && 3LL * cout * p.K * 2 < (1LL << 31),
                  "srpde_conv_fwd_x6p: tensor too large");
  const __bf16* wsp = static_cast<const __bf16*>(wsplit);
  switch (fwd_config(cout)) {
    case 0: return launch_fwd_x6p<256, 128, 8, 1, 128>(p, wsp, stream, workspace, ws_bytes);
    case 1: return launch_fwd_x6p<256, 64, 8, 1, 256>(p, wsp, stream, workspace, ws_bytes);
    default: return launch_fwd_x6p<256, 32, 8, 1, 256>(p, wsp, stream, workspace, ws_bytes);
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
                           int ksize, int dil, void* workspace, size_t ws_bytes, hipStream_t stream, bool x6,
                           const unsigned* amax_dy = nullptr, const unsigned* amax0 = nullptr,
                           const unsigned* amax1 = nullptr) {
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
  int bm, bn, rc;
  wgrad_tiles(cout, p.K, &bm, &bn);
  if (amax_dy) {
    SRPDE_CHECK_ARG(c0 % 32 == 0 && c1 % 32 == 0 && cout % 16 == 0 && wgrad_v2_ok(p) && amax0 && (c1 == 0 || amax1),
                    "srpde_conv_wgrad_h3: needs c0, c1 multiples of 32, cout of 16 and the amax words (c0=%d c1=%d cout=%d)",
                    c0, c1, cout);
    rc = launch_wgrad_h3(p, amax_dy, amax0, amax1, stream);
  } else if (x6) {
    SRPDE_CHECK_ARG(srpde_conv_x6_supported(c0, c1, cout) && wgrad_v2_ok(p),
                    "srpde_conv_wgrad_x6: needs c0, c1, cout multiples of 32 (c0=%d c1=%d cout=%d)", c0, c1, cout);
    if (bm == 128) rc = launch_wgrad_x6<128, 128, 2, 2>(p, stream);
    else if (bm == 64) rc = launch_wgrad_x6<64, 256, 1, 4>(p, stream);
    else rc = launch_wgrad_x6<32, 256, 1, 4>(p, stream);
  } else if (wgrad_v2_ok(p)) {
    if (bm == 128) rc = launch_wgrad_v2<128, 128, 2, 2>(p, stream);
    else if (bm == 64) rc = wgrad64_wide() ? launch_wgrad_v2<64, 256, 1, 4>(p, stream)
                                           : launch_wgrad_v2<64, 128, 1, 4>(p, stream);
    else rc = launch_wgrad_v2<32, 256, 1, 4>(p, stream);
  } else {
    if (bm == 128) rc = launch_wgrad<128, 128, 2, 2>(p, stream);
    else if (bm == 64) rc = bn == 64 ? launch_wgrad<64, 64, 2, 2>(p, stream) : launch_wgrad<64, 256, 1, 4>(p, stream);
    else rc = launch_wgrad<32, 256, 1, 4>(p, stream);
  }
  if (rc) return rc;
  return wgrad_reduce(p.part, dw, p.splits, cout, p.Cin, cin_real, ksize * ksize, accumulate, stream);
}

int srpde_conv_wgrad(const float* dy, int lddy, const float* x0, int c0, int ldx0, const float* x1, int c1,
                     int ldx1, float* dw, int cin_real, int accumulate, int n, int h, int w, int cout, int ksize,
                     int dil, void* workspace, size_t ws_bytes, hipStream_t stream) {
  return conv_wgrad_impl(dy, lddy, x0, c0, ldx0, x1, c1, ldx1, dw, cin_real, accumulate, n, h, w, cout, ksize, dil,
                         workspace, ws_bytes, stream, false);
}

int srpde_conv_wgrad_x6(const float* dy, int lddy, const float* x0, int c0, int ldx0, const float* x1, int c1,
                        int ldx1, float* dw, int cin_real, int accumulate, int n, int h, int w, int cout, int ksize,
                        int dil, void* workspace, size_t ws_bytes, hipStream_t stream) {
  return conv_wgrad_impl(dy, lddy, x0, c0, ldx0, x1, c1, ldx1, dw, cin_real, accumulate, n, h, w, cout, ksize, dil,
                         workspace, ws_bytes, stream, true);
}

int srpde_conv_wgrad_h3(const float* dy, int lddy, const unsigned* amax_dy, const float* x0, int c0, int ldx0,
                        const unsigned* amax0, const float* x1, int c1, int ldx1, const unsigned* amax1, float* dw,
                        int cin_real, int accumulate, int n, int h, int w, int cout, int ksize, int dil,
                        void* workspace, size_t ws_bytes, hipStream_t stream) {
  SRPDE_CHECK_ARG(amax_dy, "srpde_conv_wgrad_h3: null amax_dy");
  return conv_wgrad_impl(dy, lddy, x0, c0, ldx0, x1, c1, ldx1, dw, cin_real, accumulate, n, h, w, cout, ksize, dil,
                         workspace, ws_bytes, stream, false, amax_dy, amax0, amax1);
}

size_t srpde_conv_wgrad_bnb_c3_workspace_size(long long P, int cout) {
  int chunk, splits;
  wgrad_bnb_c3_split(P, cout, &chunk, &splits);
  return (size_t)splits * cout * 27 * sizeof(float);
}

int srpde_conv_wgrad_bnb_c3(const float* y, int ldy, const float* da, int ldda, const float* mean, const float* invstd,
                            const float* gamma, const float* beta, const float* m1, const float* m2, int flags,
                            const float* x, int ldx, float* dw, int accumulate, int n, int h, int w, int cout, int dil,
                            void* workspace, size_t ws_bytes, hipStream_t stream) {
  SRPDE_CHECK_ARG(y && da && mean && invstd && gamma && beta && m1 && m2 && x && dw && workspace,
                  "srpde_conv_wgrad_bnb_c3: null pointer");
  SRPDE_CHECK_ARG((cout == 64 || cout == 32 || cout == 16) && ldy % 4 == 0 && ldda % 4 == 0 && ldx >= 4 &&
                      ldx % 4 == 0 && aligned16(y) && aligned16(da) && aligned16(x),
                  "srpde_conv_wgrad_bnb_c3: needs cout 16/32/64, 16-byte rows and ldx >= 4 (cout=%d ldx=%d)", cout, ldx);
  const long long P = (long long)n * h * w;
  int chunk, splits;
  wgrad_bnb_c3_split(P, cout, &chunk, &splits);
  const size_t need = (size_t)splits * cout * 27 * sizeof(float);
  if (ws_bytes < need) {
    set_error("srpde_conv_wgrad_bnb_c3: workspace %zu < %zu bytes", ws_bytes, need);
    return kErrWorkspace;
  }
  float* part = static_cast<float*>(workspace);
  const int relu = flags & 1;
  SRPDE_CHECK_ARG(P < (1LL << 31) / 64, "srpde_conv_wgrad_bnb_c3: tensor too large");
  const size_t lds = std::max((size_t)C3_TP * cout + (size_t)(C3_TP + 2 * (w + 1) * dil) * 4,
                              (size_t)(256 / cout) * 9 * cout) * sizeof(float);
  SRPDE_CHECK_ARG(lds <= 96 * 1024, "srpde_conv_wgrad_bnb_c3: image too wide (w=%d dil=%d)", w, dil);
#define L(C)                                                                                                     \
  hipLaunchKernelGGL(wgrad_bnb_c3_kernel<C>, dim3(splits), dim3(256), lds, stream, y, ldy, da, ldda, mean, invstd, \
                     gamma, beta, m1, m2, relu, x, ldx, h, w, dil, (int)P, chunk, part)
  if (cout == 64) L(64);
  else if (cout == 32) L(32);
  else L(16);
#undef L
  SRPDE_LAUNCH_CHECK("srpde_conv_wgrad_bnb_c3");
  return wgrad_reduce(part, dw, splits, cout, 3, 3, 9, accumulate, stream);
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
