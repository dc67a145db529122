// "h5": the 3x3 convolution forward at W = 40 into 64 or 32 output channels (enc1.conv2, dec1.conv1,
// dec1.conv2, out_conv1: nn.Conv2d at src/models.py:16,18,57 inside ConvBlock.forward :21-24 and
// UNet.forward :78,93,96).  Same h3 arithmetic as conv_h3.hip / conv_h4.hip (scaled two-piece fp16
// operands, three fp16 MFMA products per fp32 product, one partial chain per 32-channel chunk folded
// into the accumulator), same products in the same order, same epilogue expressions: the conv output
// equals the h3 / h4 kernels' bit for bit (tests/test_gpu_h5.py).  What is different is the data flow
// (DESIGN.md 3.7):
//  * A tile is 8 whole image rows of one sample (320 pixels).  Its halo tile lives in LDS as a
//    zero-padded (8 + 2) x (40 + 2) image of 160-byte rows (hi 64 B | lo 64 B | 32 unused), so every
//    tap of every lane is ONE compile-time LDS offset from the lane's pixel: no per-tap address math,
//    no out-of-image masks (the pad ring and, at a sample's top / bottom, the halo rows are zeros).
//    160-byte rows keep the 16x16x32 fragment reads conflict-free at any row shift.
//  * The weights never touch LDS: each wave loads the B fragments of its output channels for tap
//    tau + 2 straight into registers (buffer loads, L1 / L2 resident), so there is no weight ring, no
//    weight DMA and no per-tap barrier.
//  * Two halo buffers: while the nine taps of chunk c run from one, every wave converts its share of
//    chunk c + 1 (register-staged fp32 loads -> fused input BN / gate -> scaled split -> LDS) into the
//    other, spread over the taps so the VALU work issues beside the partner wave's MFMAs.  One
//    workgroup barrier per chunk.  The last chunk of a tile converts the first chunk of the
//    workgroup's next tile (persistent workgroups walk contiguous tile ranges, so a tile's top halo
//    rows were its predecessor's bottom rows: L2 hits on the same XCD).
//  * The MFMA operands are swapped (weights as A, pixels as B): a lane's accumulator holds four
//    consecutive output channels of one pixel, so the epilogue stores 16-byte NHWC pieces straight
//    from registers and the BN statistics of a wave's 80 pixels (two image rows) reduce in registers
//    and across a 16-lane DPP row -- one (mean, M2) partial per 80 rows, no LDS.
// Layout per wave (8 waves, 2 per SIMD): output channels 32*(w & 1) .. + 32 (two 16-channel blocks;
// one at Cout = 32), pixels 80*(w >> 1) .. + 80 (five 16-pixel blocks).
#include <atomic>

#include "conv_h3.h"

namespace srpde {

__device__ floatx4 h5_bload(int32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4f32");

namespace {
constexpr int kW = 40;                       // image width (compile-time: the pad geometry)
constexpr int kTR = 8;                       // image rows per tile
constexpr int kM = kTR * kW;                 // 320 output pixels per tile
constexpr int kPW = kW + 2;                  // padded row
constexpr int kSROWS = (kTR + 2) * kPW;      // 420 halo-image rows
constexpr int kSR = 160;                     // bytes per halo-image row: hi 64 | lo 64 | 32 unused
constexpr int kSBUF = kSROWS * kSR;          // 67200 B per buffer
constexpr int kNPB = 5;                      // 16-pixel blocks per wave
constexpr int kSRB = 80;                     // rows per BN-statistics partial (one wave's pixels)
constexpr int kLDS = 2 * kSBUF + 64;         // two buffers + the max|y| reduction scratch
constexpr int kHaloPix = (kTR + 2) * kW;     // 400 halo pixels converted per chunk (4 units of 8 channels each)
}  // namespace

// weight register slots: the B fragments of tap tau + H5_WSLOTS - 1 are loaded at tap tau (18 taps per
// chunk pair must be a multiple of it)
#ifndef H5_WSLOTS
#define H5_WSLOTS 2
#endif
static_assert(18 % H5_WSLOTS == 0, "weight slots");
// timing-only diagnostics (results wrong when non-zero; an A/B library is built with
// SRPDE_EXTRA_FLAGS=-DH5_DBG=<bits>): 1 = no convert in the taps, 2 = no MFMAs, 4 = no epilogue stores,
// 8 = no weight loads in the taps
#ifndef H5_DBG
#define H5_DBG 0
#endif

template <int B, int E, typename F>
__device__ __forceinline__ void h5_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    h5_for<B + 1, E>(f);
  }
}

// sum over the 16 lanes of a DPP row, every lane receiving it (row rotations by 8, 4, 2, 1)
__device__ __forceinline__ float h5_row_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xf, 0xf, false));
  return v;
}

__device__ __forceinline__ half8 h5_half8(floatx4 v) { return __builtin_bit_cast(half8, v); }

// kernel variants: what the launch carries besides the plain conv + bias (each variant compiles only its
// own code, which keeps the register budget: the all-in-one kernel spilled)
constexpr int H5_AFF = 1;     // fused input BN + ReLU (H3Args::in_scale / in_shift)
constexpr int H5_GATE = 2;    // attention-gated second input (H3Args::x1_ca / x1_sa)
constexpr int H5_TRAIN = 4;   // BN statistics partials + the stored input split (ConvParams::stats, H3Args::xsplit)
constexpr int H5_EPBN = 8;    // eval-mode BN + ReLU epilogue + max|y| (ConvParams::ep_*)

// NCB: 16-channel output blocks per wave (2: Cout 64, 1: Cout 32); MODE: H5_* bits
template <int NCB, int MODE>
__global__ __launch_bounds__(512, 1) void conv_fwd_h5_kernel(ConvParams p, H3Args h) {
  constexpr bool AFF = (MODE & H5_AFF) != 0, GATE = (MODE & H5_GATE) != 0;
  constexpr bool TRAIN = (MODE & H5_TRAIN) != 0, EPBN = (MODE & H5_EPBN) != 0;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* lds = reinterpret_cast<char*>(smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, lq = lane >> 4;
  const int cp = wave & 1, q = wave >> 1;
  const int tps = p.H / kTR;                   // tiles per sample
  const int ntiles = p.N * tps;
  const int t_beg = (int)((long long)blockIdx.x * ntiles / gridDim.x);
  const int t_end = (int)((long long)(blockIdx.x + 1) * ntiles / gridDim.x);
  if (t_beg >= t_end) return;                  // uniform over the workgroup
  const int nch = p.Cin >> 5;                  // even (host check)
  const int HW = p.H * kW;

  unsigned abits = *h.amax0;
  if (p.c1 != 0) abits = max(abits, *h.amax1);
  const int ea = h3_exp(abits);
  const float sa = exp2i(ea);

  // the pad columns of both halo images are zeros for the whole launch
  if (tid < 320) {
    const int b = tid / 160, r = tid - b * 160, iy = r >> 4, side = (r >> 3) & 1, c = r & 7;
    *reinterpret_cast<float4*>(lds + b * kSBUF + (iy * kPW + side * (kPW - 1)) * kSR + c * 16) =
        make_float4(0.f, 0.f, 0.f, 0.f);
  }

  // the lane's B fragment (pixel 16 j + l16 of the wave's 80, 8 channels at 16 lq) of tap (ky, kx) is
  // at halo-image row (r + ky) * 42 + x + kx, r / x the pixel's tile row / column
  unsigned ab0[kNPB], ab1[kNPB];
#pragma unroll
  for (int j = 0; j < kNPB; ++j) {
    const int tp = 80 * q + 16 * j + l16;
    const int r = tp / kW, x = tp - kW * r;
    ab0[j] = (unsigned)((r * kPW + x) * kSR + lq * 16);
    ab1[j] = ab0[j] + kSBUF;
  }

  // weights: [2][Cout][K] planes, K = tap * Cin + channel; the lane's A fragment of output block cb is
  // row 16 cb + l16, 8 channels at 8 lq of the tap's 32-channel chunk
  const unsigned plane = (unsigned)p.Cout * (unsigned)p.K;
  const int32x4 rsw = make_rsrc(h.wsp, 2u * plane * 2u);
  unsigned wvo[NCB];
#pragma unroll
  for (int c = 0; c < NCB; ++c) wvo[c] = ((16u * (unsigned)(cp * NCB + c) + (unsigned)l16) * (unsigned)p.K + 8u * lq) * 2u;
  half8 wh[H5_WSLOTS][NCB], wl[H5_WSLOTS][NCB];   // taps tau .. tau + PD (slot tau % H5_WSLOTS)
  auto wload = [&](auto slot_tag, int ch, int tt) {
    constexpr int S = decltype(slot_tag)::value;
    const int so = (tt * p.Cin + ch * 32) * 2;
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
      wh[S][c] = h5_half8(h5_bload(rsw, (int)wvo[c], so, 0));
      wl[S][c] = h5_half8(h5_bload(rsw, (int)wvo[c], so + (int)(plane * 2u), 0));
    }
  };

  // ---- the convert: halo pixel (iy, x), iy = 0 .. 9 (tile rows -1 .. 8), 8 channels c8 per unit;
  // unit i of a lane is halo pixel 128 i + tid / 4 (i = 3 only for tid < 64: 400 pixels)
  const int c8 = tid & 3;
  const int32x4 rs0 = make_rsrc(p.x0, (unsigned)((size_t)p.P * p.ldx0 * 4));
  const int32x4 rs1 = make_rsrc(p.c1 ? p.x1 : p.x0, (unsigned)((size_t)p.P * (p.c1 ? p.ldx1 : p.ldx0) * 4));
  const unsigned xplane = (unsigned)p.P * (unsigned)p.Cin;
  floatx4 cv[2][2];
  auto unit_pos = [&](int i, int ttile, int& iy, int& x, int& gp, bool& valid) {
    const int pi = i * 128 + (tid >> 2);
    iy = pi / kW;
    x = pi - kW * iy;
    const int kk = ttile - (ttile / tps) * tps;
    valid = !(iy == 0 && kk == 0) && !(iy == kTR + 1 && kk == tps - 1);
    gp = ttile * kM + (iy - 1) * kW + x;
  };
  auto cv_issue = [&](auto g_tag, int ttile, int tch) {
    constexpr int G = decltype(g_tag)::value;
    const bool second = tch * 32 >= p.c0;
    const int ld = second ? p.ldx1 : p.ldx0;
    const int cb = (second ? tch * 32 - p.c0 : tch * 32) + c8 * 8;
    h5_for<0, 2>([&](auto u_tag) {
      constexpr int U = decltype(u_tag)::value, I = 2 * G + U;
      int iy, x, gp;
      bool valid;
      unit_pos(I, ttile, iy, x, gp, valid);
      // unit 3 exists for tid < 64 only (400 halo pixels); a zero fill past it
      const bool on = I < 3 || (tid >> 2) + 384 < kHaloPix;
      const unsigned vo = (on && valid) ? (unsigned)((gp * ld + cb) * 4) : OOB;
      cv[U][0] = h5_bload(second ? rs1 : rs0, (int)vo, 0, 0);
      cv[U][1] = h5_bload(second ? rs1 : rs0, (int)(vo + 16u), 0, 0);
    });
  };
  auto cv_process = [&](auto g_tag, int ttile, int tch) {
    constexpr int G = decltype(g_tag)::value;
    const int buf = tch & 1;
    const bool second = tch * 32 >= p.c0;
    const bool gate = GATE && second;
    float4 s0, s1, t0, t1;
    if constexpr (AFF) {
      const int cc = tch * 32 + c8 * 8;
      s0 = *reinterpret_cast<const float4*>(h.in_scale + cc);
      s1 = *reinterpret_cast<const float4*>(h.in_scale + cc + 4);
      t0 = *reinterpret_cast<const float4*>(h.in_shift + cc);
      t1 = *reinterpret_cast<const float4*>(h.in_shift + cc + 4);
    }
    h5_for<0, 2>([&](auto u_tag) {
      constexpr int U = decltype(u_tag)::value, I = 2 * G + U;
      if (I < 3 || (tid >> 2) + 384 < kHaloPix) {   // (uniform per wave: unit 3 is wave 0's)
        int iy, x, gp;
        bool valid;
        unit_pos(I, ttile, iy, x, gp, valid);
        float4 v0 = make_float4(cv[U][0][0], cv[U][0][1], cv[U][0][2], cv[U][0][3]);
        float4 v1 = make_float4(cv[U][1][0], cv[U][1][1], cv[U][1][2], cv[U][1][3]);
        if (gate) gate8(v0, v1, h, valid ? gp : -1, p.P, HW, p.c1, tch * 32 - p.c0 + c8 * 8);
        if constexpr (AFF) {   // fused BN + ReLU of the producer; rows outside the sample stay 0
          const bool inside = valid;
#define AFF(V, S, T, X) V.X = inside ? fmaxf(V.X * S.X + T.X, 0.f) : 0.f;
          AFF(v0, s0, t0, x) AFF(v0, s0, t0, y) AFF(v0, s0, t0, z) AFF(v0, s0, t0, w)
          AFF(v1, s1, t1, x) AFF(v1, s1, t1, y) AFF(v1, s1, t1, z) AFF(v1, s1, t1, w)
#undef AFF
        }
        half8 hv, lv;
        split2h(v0, v1, sa, hv, lv);
        char* dst = lds + buf * kSBUF + (iy * kPW + x + 1) * kSR + c8 * 16;
        *reinterpret_cast<half8*>(dst) = hv;
        *reinterpret_cast<half8*>(dst + 64) = lv;
        if (TRAIN && iy >= 1 && iy <= kTR) {   // the tile's own pixels: the stored input split
          _Float16* o = h.xsplit + (size_t)gp * p.Cin + tch * 32 + c8 * 8;
          *reinterpret_cast<half8*>(o) = hv;
          *reinterpret_cast<half8*>(o + xplane) = lv;
        }
      }
    });
  };

  floatx4 acc[NCB][kNPB], part[NCB][kNPB];
  half8 xh[3], xl[3];   // fragment window (see tap)
  float amax_run = 0.f;

  // one tap T (0 .. 17) of the chunk pair (cc, cc + 1) of tile t: chunk cc + T / 9 from halo buffer T / 9
  auto tap = [&](auto T_tag, int cc, int t, bool has_next) {
    constexpr int T = decltype(T_tag)::value;
    constexpr int B = T / 9, TT = T % 9, SL = T % H5_WSLOTS;
    const int ch = cc + B;
    // weights of tap T + 2 into slot (T + 2) % 3 (the chunk after the last is chunk 0 of the next tile)
    {
      constexpr int T2 = T + H5_WSLOTS - 1;
      int ch2 = cc + T2 / 9;
      if (ch2 >= nch) ch2 -= nch;
      if constexpr (!(H5_DBG & 8)) wload(std::integral_constant<int, T2 % H5_WSLOTS>{}, ch2, T2 % 9);
    }
    // the convert of the chunk that follows this one (buffer B ^ 1): this tile's ch + 1, or the next
    // tile's chunk 0; loads at tap 0 / 3, split + LDS writes at tap 3 / 6 (a load group is waited for
    // three taps after its issue, when the weights issued after it are)
    const bool cv_next_tile = ch + 1 >= nch;
    const bool cv_on = (!cv_next_tile || has_next) && !(H5_DBG & 1);
    const int cv_tile = cv_next_tile ? t + 1 : t, cv_ch = cv_next_tile ? 0 : ch + 1;
    if constexpr (TT == 0) {
      if (cv_on) cv_issue(std::integral_constant<int, 0>{}, cv_tile, cv_ch);
    }
    if constexpr (TT == 3) {
      if (cv_on) {
        cv_process(std::integral_constant<int, 0>{}, cv_tile, cv_ch);
        cv_issue(std::integral_constant<int, 1>{}, cv_tile, cv_ch);
      }
    }
    if constexpr (TT == 6) {
      if (cv_on) cv_process(std::integral_constant<int, 1>{}, cv_tile, cv_ch);
    }
    if constexpr (TT == 0) {
      if (B == 1 || cc > 0) {   // fold the previous chunk's partial chain (two-level accumulation)
#pragma unroll
        for (int c = 0; c < NCB; ++c)
#pragma unroll
          for (int j = 0; j < kNPB; ++j) acc[c][j] += part[c][j];
      }
    }
    h5_for<0, kNPB>([&](auto j_tag) {
      constexpr int J = decltype(j_tag)::value;
      // fragments: a sliding window of three blocks over the 90 blocks (18 taps x 5) of a chunk pair;
      // block g sits in slot g % 3, block g + 2 is read after block g's MFMAs
      constexpr int G = 5 * T + J, SX = G % 3;
      constexpr int G2 = (G + 2) % 90, T2 = G2 / 5, J2 = G2 % 5, B2 = T2 / 9, TT2 = T2 % 9;
      constexpr int TOFF2 = ((TT2 / 3) * kPW + TT2 % 3) * kSR;
#pragma unroll
      for (int c = 0; c < NCB && !(H5_DBG & 2); ++c) {
        floatx4 c0;
        if constexpr (TT == 0)   // a chunk's partial chain starts from zero; small terms first
          c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[SL][c], xl[SX], floatx4{}, 0, 0, 0);
        else
          c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[SL][c], xl[SX], part[c][J], 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[SL][c], xh[SX], c0, 0, 0, 0);
        part[c][J] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[SL][c], xh[SX], c0, 0, 0, 0);
      }
      if constexpr (TT == 8 && J == 3) {
        // every wave has read the last fragments of this chunk (blocks 3, 4 of tap 8 in flight to its
        // registers) and written its share of the next chunk: after the barrier the next chunk's buffer
        // is complete and this chunk's buffer free
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
      {
        const unsigned a = (B2 ? ab1[J2] : ab0[J2]) + TOFF2;
        xh[G2 % 3] = *reinterpret_cast<const half8*>(lds + a);
        xl[G2 % 3] = *reinterpret_cast<const half8*>(lds + a + 64);
      }
      // keep the block's order (its MFMAs, then one block's reads): the scheduler would otherwise hoist
      // reads into fresh registers and run out of them
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  // prologue: the first tile's chunk 0 into buffer 0, the weights of taps 0 and 1
  cv_issue(std::integral_constant<int, 0>{}, t_beg, 0);
  cv_process(std::integral_constant<int, 0>{}, t_beg, 0);
  cv_issue(std::integral_constant<int, 1>{}, t_beg, 0);
  cv_process(std::integral_constant<int, 1>{}, t_beg, 0);
  h5_for<0, H5_WSLOTS - 1>([&](auto s_tag) { wload(s_tag, 0, decltype(s_tag)::value); });
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    xh[j] = *reinterpret_cast<const half8*>(lds + ab0[j]);
    xl[j] = *reinterpret_cast<const half8*>(lds + ab0[j] + 64);
  }

  const float ia = exp2i(-ea);
  for (int t = t_beg; t < t_end; ++t) {
    const bool has_next = t + 1 < t_end;
#pragma unroll
    for (int c = 0; c < NCB; ++c)
#pragma unroll
      for (int j = 0; j < kNPB; ++j) acc[c][j] = floatx4{};
    for (int cc = 0; cc < nch; cc += 2) {
      h5_for<0, 18>([&](auto T_tag) { tap(T_tag, cc, t, has_next); });
    }

    // ---- epilogue: scales, bias, (eval) BN + ReLU, 16-B stores, (train) BN statistics
    const int pix0 = t * kM + 80 * q;   // the wave's first pixel
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
      const int col0 = 16 * (cp * NCB + c) + 4 * lq;
      float v[kNPB][4];
      const int4 we = *reinterpret_cast<const int4*>(h.wexp + col0);
      const float4 bi = p.bias != nullptr ? *reinterpret_cast<const float4*>(p.bias + col0) : make_float4(0.f, 0.f, 0.f, 0.f);
      const int wer[4] = {we.x, we.y, we.z, we.w};
      const float bir[4] = {bi.x, bi.y, bi.z, bi.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int e = ea + wer[r];
        float cs;
        bool pre = false;
        if (e > 126 || e < -126) {   // (conv_fwd_h4_kernel: the operand scale undone in two steps)
          pre = true;
          cs = exp2i(-wer[r]);
        } else {
          cs = exp2i(-e);
        }
#pragma unroll
        for (int j = 0; j < kNPB; ++j) {
          float a = acc[c][j][r] + part[c][j][r];   // the last chunk's fold
          if (pre) a *= ia;
          v[j][r] = __builtin_fmaf(a, cs, bir[r]);
        }
      }
      if constexpr (EPBN) {   // eval-mode BN + ReLU (ConvParams::ep_*)
        const float4 mu = *reinterpret_cast<const float4*>(p.ep_mean + col0);
        const float4 is = *reinterpret_cast<const float4*>(p.ep_invstd + col0);
        const float4 ga = *reinterpret_cast<const float4*>(p.ep_gamma + col0);
        const float4 be = *reinterpret_cast<const float4*>(p.ep_beta + col0);
        const float mur[4] = {mu.x, mu.y, mu.z, mu.w}, isr[4] = {is.x, is.y, is.z, is.w};
        const float gar[4] = {ga.x, ga.y, ga.z, ga.w}, ber[4] = {be.x, be.y, be.z, be.w};
#pragma unroll
        for (int j = 0; j < kNPB; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[j][r] = ep_bn_relu(v[j][r], mur[r], isr[r], gar[r], ber[r]);
            amax_run = fmaxf(amax_run, fabsf(v[j][r]));
          }
      }
#pragma unroll
      for (int j = 0; j < kNPB; ++j) {
        float4* dst = reinterpret_cast<float4*>(p.y + (size_t)(pix0 + 16 * j + l16) * p.ldy + col0);
        float4 o = make_float4(v[j][0], v[j][1], v[j][2], v[j][3]);
        if (p.accumulate) {
          const float4 prev = *dst;
          o = make_float4(prev.x + o.x, prev.y + o.y, prev.z + o.z, prev.w + o.w);
        }
        if ((H5_DBG & 4) && o.x != 123.f) continue;
        *dst = o;
      }
      if constexpr (TRAIN) {   // (mean, M2) of the wave's 80 pixels per channel
        float mean[4], m2[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < kNPB; ++j) s += v[j][r];
          mean[r] = h5_row_sum(s) / (float)kSRB;
          float m = 0.f;
#pragma unroll
          for (int j = 0; j < kNPB; ++j) {
            const float d = v[j][r] - mean[r];
            m = __builtin_fmaf(d, d, m);
          }
          m2[r] = h5_row_sum(m);
        }
        if (l16 == 0) {
          float2* st = p.stats + (size_t)(pix0 / kSRB) * p.Cout + col0;
          st[0] = make_float2(mean[0], m2[0]);
          st[1] = make_float2(mean[1], m2[1]);
          st[2] = make_float2(mean[2], m2[2]);
          st[3] = make_float2(mean[3], m2[3]);
        }
      }
    }
  }
  if (EPBN && p.ep_amax != nullptr) {   // max|y| of the workgroup's tiles -> one atomicMax
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) amax_run = fmaxf(amax_run, __shfl_xor(amax_run, o, 64));
    float* red = reinterpret_cast<float*>(lds + 2 * kSBUF);
    if (lane == 0) red[wave] = amax_run;
    __syncthreads();
    if (tid == 0) {
      float m = 0.f;
      for (int k = 0; k < 8; ++k) m = fmaxf(m, red[k]);
      atomicMax(p.ep_amax, __float_as_uint(m));
    }
  }
}

// ---------------------------------- host side ---------------------------------------
static std::atomic<int> g_h5{1};

bool h5_on() { return g_h5.load(std::memory_order_relaxed) != 0; }
int h5_set(int on) {
  const int prev = h5_on() ? 1 : 0;
  if (on >= 0) g_h5.store(on ? 1 : 0);
  return prev;
}

// the shapes h5 takes (forward, no upsampled input): W = 40, H a multiple of 8, Cout 64 or 32, input
// channels a multiple of 64 (chunk pairs), the first input a multiple of 32
bool h5_supported(int c0, int c1, int cout, int h, int w, int dil) {
  return h5_on() && w == kW && h > 0 && h % kTR == 0 && dil == 1 && (cout == 64 || cout == 32) && c0 % 32 == 0 &&
         c1 % 32 == 0 && (c0 + c1) % 64 == 0 && (c0 + c1) > 0;
}

int h5_stats_rows() { return kSRB; }

template <int NCB, int MODE>
static void launch_h5_variant(const ConvParams& p, const H3Args& h, int grid, hipStream_t st) {
  hipLaunchKernelGGL((conv_fwd_h5_kernel<NCB, MODE>), dim3(grid), dim3(512), kLDS, st, p, h);
}

template <int NCB>
static int launch_h5_ncb(const ConvParams& p, const H3Args& h, int grid, hipStream_t st) {
  const bool aff = h.in_scale != nullptr, gate = h.x1_ca != nullptr, epbn = p.ep_mean != nullptr;
  const bool train = p.stats != nullptr || h.xsplit != nullptr;
  // the U-Net's uses: eval (BN + ReLU epilogue, gated concat input), train (statistics + stored split,
  // fused input BN or gated concat input), and the plain conv
  if (!aff && !gate && !train && epbn) launch_h5_variant<NCB, H5_EPBN>(p, h, grid, st);
  else if (!aff && gate && !train && epbn) launch_h5_variant<NCB, H5_GATE | H5_EPBN>(p, h, grid, st);
  else if (aff && !gate && train && !epbn) launch_h5_variant<NCB, H5_AFF | H5_TRAIN>(p, h, grid, st);
  else if (!aff && gate && train && !epbn) launch_h5_variant<NCB, H5_GATE | H5_TRAIN>(p, h, grid, st);
  else if (!aff && !gate && train && !epbn) launch_h5_variant<NCB, H5_TRAIN>(p, h, grid, st);
  else if (!aff && !gate && !train && !epbn) launch_h5_variant<NCB, 0>(p, h, grid, st);
  else if (!aff && gate && !train && !epbn) launch_h5_variant<NCB, H5_GATE>(p, h, grid, st);
  else if (aff && !gate && !train && !epbn) launch_h5_variant<NCB, H5_AFF>(p, h, grid, st);
  else {
    set_error("srpde_conv_fwd_h3(h5): no kernel variant for this combination (in_scale %d, gate %d, stats/xsplit %d, "
              "ep %d)", (int)aff, (int)gate, (int)train, (int)epbn);
    return kErrArg;
  }
  return 0;
}

int launch_fwd_h5(const ConvParams& p, const H3Args& h, hipStream_t st) {
  static const int cus = [] {
    int dev = 0, c = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    return std::max(1, c);
  }();
  const int ntiles = p.N * (p.H / kTR);
  const int grid = std::min(ntiles, cus);
  const int rc = p.Cout == 64 ? launch_h5_ncb<2>(p, h, grid, st) : launch_h5_ncb<1>(p, h, grid, st);
  if (rc != 0) return rc;
  SRPDE_LAUNCH_CHECK("srpde_conv_fwd_h3(h5)");
  return 0;
}

}  // namespace srpde
