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
//  * Weights: a tap's [2 planes][Cout][32] fp16 tile goes through a 3-slot LDS ring, DMA'd (buffer_load ...
//    lds) three taps ahead by the four "loader" waves, one workgroup barrier per tap; every wave reads its A
//    fragments of the next tap into registers.
//  * Two halo buffers: while the nine taps of chunk c run from one, the four "converter" waves convert chunk
//    c + 1 (register-staged fp32 loads -> fused input BN / gate -> scaled split -> LDS) into the other,
//    one or two units per tap.  A SIMD runs one wave of each role.  The last chunk of a tile converts the
//    first chunk of the workgroup's next tile (persistent workgroups walk contiguous tile ranges, so a
//    tile's top halo rows were its predecessor's bottom rows: L2 hits on the same XCD).
//  * The MFMA operands are swapped (weights as A, pixels as B): a lane's accumulator holds four
//    consecutive output channels of one pixel, so the epilogue stores 16-byte NHWC pieces straight
//    from registers and the BN statistics of a wave's 80 pixels (two image rows) reduce in registers
//    and across a 16-lane DPP row -- one (mean, M2) partial per 80 rows, no LDS.  The epilogue of a
//    tile runs inside the next tile's taps 7 .. 8 (its accumulators are dead there), between MFMAs.
// Layout per wave (8 waves, 2 per SIMD): output channels 32*(w & 1) .. + 32 (two 16-channel blocks;
// one at Cout = 32), pixels 80*(w >> 1) .. + 80 (five 16-pixel blocks).
#include <atomic>

#include "conv_h3.h"

namespace srpde {

__device__ floatx4 h5_bload(int32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4f32");

// 16-B-per-lane LDS-DMA (buffer_load_dwordx4 ... lds) with a uniform byte offset in soffset and the wave-uniform LDS
// destination in M0 (conv_h4.hip dma16s): inline asm, invisible to the compiler's waitcnt pass -- the issuing
// (loader) waves count these loads themselves
__device__ __forceinline__ void h5_dma16(int32x4 rsrc, unsigned voff, unsigned soff, unsigned lds_addr) {
  asm volatile(
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %0, %1, %2 offen lds"
      :
      : "v"(voff), "s"(rsrc), "s"(__builtin_amdgcn_readfirstlane(soff)), "{m0}"(__builtin_amdgcn_readfirstlane(lds_addr))
      : "memory");
}

// 16-B buffer store as inline asm: the loader waves count their vector-memory operations exactly in the tap
// waits (a store to a buffer of 0 records is dropped but still counted).  The s_nop is the wait state a VALU
// write of the store's data registers needs after a store of more than 8 bytes: the compiler's hazard pass
// does not see an asm store, and without it the first data register was measured overwritten before the
// store read it
__device__ __forceinline__ void h5_st16(floatx4 v, unsigned voff, int32x4 rsrc, unsigned soff) {
  asm volatile("buffer_store_dwordx4 %0, %1, %2, %3 offen\n\ts_nop 1" ::"v"(v), "v"(voff), "s"(rsrc),
               "s"(__builtin_amdgcn_readfirstlane(soff))
               : "memory");
}

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
constexpr int kOffW = 2 * kSBUF;             // the weight ring: 3 slots of one tap [2 planes][64 rows][64 B]
constexpr int kWSLOT = 8192;
constexpr int kOffP = kOffW + 3 * kWSLOT;     // per output channel: cs, bias, eval BN mean / invstd / gamma / beta, pm
constexpr int kOffA = kOffP + 8 * 64 * 4;     // the fused input BN's scale / shift per input channel (<= 192)
constexpr int kOffR = kOffA + 2 * 192 * 4;    // the max|y| reduction
constexpr int kLDS = kOffR + 64;
constexpr int kHaloPix = (kTR + 2) * kW;     // 400 halo pixels converted per chunk (4 units of 8 channels each)
}  // namespace

// timing-only diagnostics (results wrong when non-zero; an A/B library is built with
// SRPDE_EXTRA_FLAGS=-DH5_DBG=<bits>): 1 = no convert in the taps, 2 = no MFMAs, 4 = no epilogue stores,
// 8 = no weight loads in the taps, 32 = no pixel-fragment reads in the taps, 64 = halo loads out of bounds (zeros), 16 = phase timestamps (every wave stores s_memtime before and after every tap
// barrier and around the epilogue of its SECOND tile into room past the output: y + P * ldy + 512 * blockIdx.x +
// 64 * wave 64-bit words; tools/h5_phase_ts.py)
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
constexpr int H5_ACC = 16;    // y += conv (ConvParams::accumulate)
constexpr int H5_UP = 32;     // x0 is the bilinear x2 upsample of H3Args::up_src, interpolated in the convert

// NCB: 16-channel output blocks per wave (2: Cout 64, 1: Cout 32); MODE: H5_* bits
template <int NCB, int MODE>
__global__ __launch_bounds__(512, 1) void conv_fwd_h5_kernel(ConvParams p, H3Args h) {
  constexpr bool AFF = (MODE & H5_AFF) != 0, GATE = (MODE & H5_GATE) != 0;
  constexpr bool TRAIN = (MODE & H5_TRAIN) != 0, EPBN = (MODE & H5_EPBN) != 0, ACC = (MODE & H5_ACC) != 0;
  constexpr bool UP = (MODE & H5_UP) != 0;
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

  // the epilogue's per-channel parameters and the fused input BN's scale / shift, staged in LDS once (the
  // epilogue then issues no global loads, whose waits would also wait for the weight DMAs)
  {
    float* prm = reinterpret_cast<float*>(lds + kOffP);
    if (tid < p.Cout) {
      const int c = tid;
      // the operand scales undone: acc * 2^-(ea + wexp) as (acc * pm) * cs, in two exact steps where
      // 2^-(ea + wexp) is no normal float (conv_fwd_h4_kernel); pm = 1 or 2^-ea (a multiply by 1 is exact)
      const int e = ea + h.wexp[c];
      const bool two = e > 126 || e < -126;
      prm[c] = exp2i(two ? -h.wexp[c] : -e);
      prm[384 + c] = two ? exp2i(-ea) : 1.f;
      prm[64 + c] = p.bias != nullptr ? p.bias[c] : 0.f;
      if constexpr (EPBN) {
        prm[128 + c] = p.ep_mean[c];
        prm[192 + c] = p.ep_invstd[c];
        prm[256 + c] = p.ep_gamma[c];
        prm[320 + c] = p.ep_beta[c];
      }
    }
    if constexpr (AFF) {
      float* aff = reinterpret_cast<float*>(lds + kOffA);
      if (tid < p.Cin) {
        aff[tid] = h.in_scale[tid];
        aff[192 + tid] = h.in_shift[tid];
      }
    }
  }

  // the lane's B fragment (pixel 16 j + l16 of the wave's 80, 8 channels at 16 lq) of tap (ky, kx) is
  // at halo-image row (r + ky) * 42 + x + kx, r / x the pixel's tile row / column
  unsigned ab0[kNPB];   // (+ kSBUF for buffer 1, added at each read: kept as registers they were spilled)
#pragma unroll
  for (int j = 0; j < kNPB; ++j) {
    const int tp = 80 * q + 16 * j + l16;
    const int r = tp / kW, x = tp - kW * r;
    ab0[j] = (unsigned)((r * kPW + x) * kSR + lq * 16);
  }

  // Roles: waves 4 .. 7 DMA the weights into the LDS ring, waves 0 .. 3 load and convert the halo tiles.  The
  // MFMA work is the same for every wave; a SIMD runs one wave of each role (waves w and w + 4).
  const bool loader = wave >= 4;

  // weights: [2][Cout][K] planes, K = tap * Cin + channel.  A tap's tile ([2][Cout][32] fp16, 8 KiB at
  // Cout 64) goes through a 3-slot LDS ring: at tap tau every wave reads its A fragments of tap tau + 1 into
  // registers, and the loader waves DMA tap tau + 3 into the slot tap tau used (its fragments were read
  // during tau - 1); before the barrier of tap tau + 1 a loader waits for its DMA of tap tau + 2 (issued at
  // tau - 1).  One barrier per tap.  Ring rows are the 64-B k-rows of conv_h4.hip with the same 16-B chunk
  // swizzle (swzh), conflict-free reads.  Piece pc (1 KiB, one DMA): plane pc / (2 NCB), 16-row block
  // pc % (2 NCB); lane -> row (lane >> 2), slot lane & 3 holding source chunk swzh(row, lane & 3).  Loader
  // wave 4 + k DMAs pieces NCB k .. NCB k + NCB - 1.
  const unsigned plane = (unsigned)p.Cout * (unsigned)p.K;
  const int32x4 rsw = make_rsrc(h.wsp, 2u * plane * 2u);
  unsigned wsrc[NCB], wdst[NCB];   // per piece of this loader wave: source bytes (tap 0, chunk 0), ring offset
#pragma unroll
  for (int k = 0; k < NCB; ++k) {
    const int pc = (wave & 3) * NCB + k, pl = pc / (2 * NCB), rb = pc % (2 * NCB);
    const int r = rb * 16 + (lane >> 2);
    wsrc[k] = ((unsigned)pl * plane + (unsigned)r * (unsigned)p.K + (unsigned)swzh(r, lane & 3) * 8u) * 2u;
    wdst[k] = (unsigned)(kOffW + pl * (NCB * 2048) + rb * 1024);   // + slot * kWSLOT (+ lane * 16 by the DMA)
  }
  const unsigned lds0 = lds_addr_of(lds);
  const unsigned wfr = (unsigned)(kOffW + l16 * 64 + swzh(l16, lq) * 16);        // A fragment, + cb * 1024
  auto wdma = [&](int ch, int tt, int slot) {
#pragma unroll
    for (int k = 0; k < NCB; ++k) h5_dma16(rsw, wsrc[k], (unsigned)((tt * p.Cin + ch * 32) * 2), lds0 + wdst[k] + slot * kWSLOT);
  };
  half8 wh[2][NCB], wl[2][NCB];               // A fragments of taps tau (slot tau % 2) and tau + 1
  auto wfrag = [&](auto r_tag, int slot) {
    constexpr int R = decltype(r_tag)::value;
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
      const unsigned a = wfr + slot * kWSLOT + (cp * NCB + c) * 1024;
      wh[R][c] = *reinterpret_cast<const half8*>(lds + a);
      wl[R][c] = *reinterpret_cast<const half8*>(lds + a + NCB * 2048);
    }
  };
  floatx4 stg[8];   // the converters' staged halo loads

  // ---- the convert (waves 0 .. 3): halo pixel (iy, x), iy = 0 .. 9 (tile rows -1 .. 8), 8 channels c8 per
  // unit; unit i of a lane is halo pixel 64 i + tid / 4, i = 0 .. 6 (unit 6: tid < 64 only, 400 pixels);
  // group 0 = units 0 .. 3 (loaded at tap 0 of a chunk, converted at tap 3), group 1 = units 4 .. 6 (tap 3 -> 6)
  const int c8 = tid & 3;
  const int32x4 rs0 = make_rsrc(p.x0, (unsigned)((size_t)p.P * p.ldx0 * 4));
  const int32x4 rs1 = make_rsrc(p.c1 ? p.x1 : p.x0, (unsigned)((size_t)p.P * (p.c1 ? p.ldx1 : p.ldx0) * 4));
  const unsigned xplane = (unsigned)p.P * (unsigned)p.Cin;
  auto unit_pos = [&](int i, int ttile, int& iy, int& x, int& gp, bool& valid) {
    int tq = tid >> 2;
    asm volatile("" : "+v"(tq));   // recomputed at each use: hoisted out of the tile loop they were spilled
    const int pi = i * 64 + tq;
    iy = pi / kW;
    x = pi - kW * iy;
    const int kk = ttile - (ttile / tps) * tps;
    valid = !(iy == 0 && kk == 0) && !(iy == kTR + 1 && kk == tps - 1);
    gp = ttile * kM + (iy - 1) * kW + x;
  };
  // unit U's two loads live in staging slot U % 4 (units 4 .. 6 reuse the slots of units 0 .. 2)
  auto cv_issue = [&](auto u_tag, int ttile, int tch) {
    constexpr int U = decltype(u_tag)::value, SS = U % 4;
    const bool second = tch * 32 >= p.c0;
    const int ld = second ? p.ldx1 : p.ldx0;
    const int cb = (second ? tch * 32 - p.c0 : tch * 32) + c8 * 8;
    int iy, x, gp;
    bool valid;
    unit_pos(U, ttile, iy, x, gp, valid);
    const bool on = U < 6 || (tid >> 2) + 384 < kHaloPix;   // unit 6: tid < 64; a zero fill past it
    const unsigned vo = (on && valid && !(H5_DBG & 64)) ? (unsigned)((gp * ld + cb) * 4) : OOB;
    stg[2 * SS] = h5_bload(second ? rs1 : rs0, (int)vo, 0, 0);
    stg[2 * SS + 1] = h5_bload(second ? rs1 : rs0, (int)(vo + 16u), 0, 0);
  };
  auto cv_process = [&](auto u_tag, int ttile, int tch) {
    constexpr int U = decltype(u_tag)::value, SS = U % 4;
    if (U == 6 && (tid >> 2) + 384 >= kHaloPix) return;   // (uniform per wave: unit 6 is wave 0's)
    const int buf = tch & 1;
    const bool second = tch * 32 >= p.c0;
    int iy, x, gp;
    bool valid;
    unit_pos(U, ttile, iy, x, gp, valid);
    float4 v0 = make_float4(stg[2 * SS][0], stg[2 * SS][1], stg[2 * SS][2], stg[2 * SS][3]);
    float4 v1 = make_float4(stg[2 * SS + 1][0], stg[2 * SS + 1][1], stg[2 * SS + 1][2], stg[2 * SS + 1][3]);
    if (GATE && second) gate8n(v0, v1, h, ttile / tps, valid ? gp : -1, p.c1, tch * 32 - p.c0 + c8 * 8);
    if constexpr (AFF) {   // fused BN + ReLU of the producer; rows outside the sample stay 0
      const float* aff = reinterpret_cast<const float*>(lds + kOffA) + tch * 32 + c8 * 8;
      const float4 s0 = *reinterpret_cast<const float4*>(aff), s1 = *reinterpret_cast<const float4*>(aff + 4);
      const float4 t0 = *reinterpret_cast<const float4*>(aff + 192), t1 = *reinterpret_cast<const float4*>(aff + 196);
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
    if (TRAIN && h.xsplit != nullptr && iy >= 1 && iy <= kTR) {   // the tile's own pixels: the stored input split
      _Float16* o = h.xsplit + (size_t)gp * p.Cin + tch * 32 + c8 * 8;
      *reinterpret_cast<half8*>(o) = hv;
      *reinterpret_cast<half8*>(o + xplane) = lv;
    }
  };
  // UP (the decoder's upsampled input, eval): unit U of a chunk of x0 interpolates its halo pixel from the
  // four low-res pixels of up_src, upsample_gate_fwd_px_kernel's / conv_fwd_h4's expression; its 8 loads fill
  // the whole staging array (one unit in flight: loaded at one tap, converted at the next)
  const int32x4 rsu = make_rsrc(UP ? h.up_src : p.x0, UP ? (unsigned)((size_t)p.N * h.up_h * h.up_w * h.up_ld * 4) : 0u);
  auto up_src = [&](int U, int ttile, Lerp& ly, Lerp& lx, int& b0, bool& valid) {
    int iy, x, gp;
    unit_pos(U, ttile, iy, x, gp, valid);
    const int nn = ttile / tps, oy = (ttile - nn * tps) * kTR + iy - 1;
    ly = lerp_index(valid ? oy : 0, h.up_h, p.H);
    lx = lerp_index(x, h.up_w, kW);
    b0 = nn * h.up_h * h.up_w;
  };
  auto cv_issue_up = [&](auto u_tag, int ttile, int tch) {
    constexpr int U = decltype(u_tag)::value;
    Lerp ly, lx;
    int b0;
    bool valid;
    up_src(U, ttile, ly, lx, b0, valid);
    const bool on = (U < 6 || (tid >> 2) + 384 < kHaloPix) && valid;
    const int cb = tch * 32 + c8 * 8;
    const int src[4] = {b0 + ly.i0 * h.up_w + lx.i0, b0 + ly.i0 * h.up_w + lx.i1, b0 + ly.i1 * h.up_w + lx.i0,
                        b0 + ly.i1 * h.up_w + lx.i1};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned vo = on ? (unsigned)((src[k] * h.up_ld + cb) * 4) : OOB;
      stg[2 * k] = h5_bload(rsu, (int)vo, 0, 0);
      stg[2 * k + 1] = h5_bload(rsu, (int)(vo + 16u), 0, 0);
    }
  };
  auto cv_process_up = [&](auto u_tag, int ttile, int tch) {
    constexpr int U = decltype(u_tag)::value;
    if (U == 6 && (tid >> 2) + 384 >= kHaloPix) return;   // (uniform per wave: unit 6 is wave 0's)
    Lerp ly, lx;
    int b0;
    bool valid;
    up_src(U, ttile, ly, lx, b0, valid);
    float o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int hf = q >> 2, c = q & 3;
      const float a = stg[hf][c], b = stg[2 + hf][c], d = stg[4 + hf][c], f = stg[6 + hf][c];
      // ly.l0 (lx.l0 a + lx.l1 b) + ly.l1 (lx.l0 d + lx.l1 f), contracted as the compiler contracts it in
      // upsample_gate_fwd_px_kernel and conv_fwd_h4 (each sum: fma of its first product onto the second)
      const float t0 = __builtin_fmaf(lx.l0, a, lx.l1 * b), t1 = __builtin_fmaf(lx.l0, d, lx.l1 * f);
      o[q] = __builtin_fmaf(ly.l0, t0, ly.l1 * t1);
    }
    const float4 v0 = make_float4(o[0], o[1], o[2], o[3]), v1 = make_float4(o[4], o[5], o[6], o[7]);
    int iy, x, gp;
    bool vv;
    unit_pos(U, ttile, iy, x, gp, vv);
    half8 hv, lv;
    split2h(v0, v1, sa, hv, lv);
    char* dst = lds + (tch & 1) * kSBUF + (iy * kPW + x + 1) * kSR + c8 * 16;
    *reinterpret_cast<half8*>(dst) = hv;
    *reinterpret_cast<half8*>(dst + 64) = lv;
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using I4 = std::integral_constant<int, 4>;
  using I5 = std::integral_constant<int, 5>;
  using I6 = std::integral_constant<int, 6>;

  floatx4 acc[NCB][kNPB], part[NCB][kNPB];
  half8 xh[3], xl[3];   // fragment window (see tap)
  float amax_run = 0.f;
  int tile_no = 0, nts = 0;
  auto stamp = [&]() {
    if constexpr ((H5_DBG & 16) != 0) {
      if (tile_no == 1 && nts < 64) {
        const unsigned long long tv = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_s_waitcnt(0xc07f);
        reinterpret_cast<unsigned long long*>(p.y + (size_t)p.P * p.ldy)[(size_t)blockIdx.x * 512 + wave * 64 + nts] = tv;
      }
      ++nts;
    }
  };

  // ---- epilogue of 16-channel block C of a finished tile, from acc (the tile's sums): scales, bias, (eval)
  // BN + ReLU, 16-B stores, (train) BN statistics.  Deferred into taps 9 - NCB .. 8 of the next tile's first chunk
  // pair -- acc is dead there until the fold at tap 9 -- so its VALU work issues between that tap's MFMAs.  It
  // runs at those taps of EVERY chunk pair, branch-free: its stores go to buffers of 0 records (dropped, and
  // max|y| not updated) except in the first pair of a tile that has a predecessor in this workgroup; the last
  // tile's epilogue runs after the loop.  Stores are inline asm, which the loader waves count in their tap waits.
  unsigned eyo[NCB], eso[NCB];   // byte offsets of the lane's outputs / BN partials within a tile
#pragma unroll
  for (int c = 0; c < NCB; ++c) {
    const int col0 = 16 * (cp * NCB + c) + 4 * lq;
    eyo[c] = (unsigned)(((80 * q + l16) * p.ldy + col0) * 4);
    eso[c] = l16 == 0 ? (unsigned)((q * p.Cout + col0) * 8) : OOB;
  }
  int32x4 eyr = make_rsrc(p.y, 0u), esr = make_rsrc(p.stats, 0u);   // the epilogue's tile (0 records: none)
  unsigned eso_t = 0;                                                // + its BN partial rows
  bool e_on = false;
  auto epi_tile = [&](int tt, bool on) {
    e_on = on;
    eyr = make_rsrc(p.y + (size_t)tt * kM * p.ldy, on ? (unsigned)(kM * p.ldy * 4) : 0u);
    if constexpr (TRAIN) {
      esr = make_rsrc(p.stats, on && p.stats != nullptr ? (unsigned)(p.P / kSRB * p.Cout * 8) : 0u);
      eso_t = (unsigned)(tt * (kM / kSRB) * p.Cout * 8);
    }
  };
  float4 ecs, epm, ebi, emu, eis, ega, ebe;
  auto epi_prm = [&](int C) {
    const float* prm = reinterpret_cast<const float*>(lds + kOffP) + 16 * (cp * NCB + C) + 4 * lq;
    ecs = *reinterpret_cast<const float4*>(prm);
    ebi = *reinterpret_cast<const float4*>(prm + 64);
    epm = *reinterpret_cast<const float4*>(prm + 384);
    if constexpr (EPBN) {
      emu = *reinterpret_cast<const float4*>(prm + 128);
      eis = *reinterpret_cast<const float4*>(prm + 192);
      ega = *reinterpret_cast<const float4*>(prm + 256);
      ebe = *reinterpret_cast<const float4*>(prm + 320);
    }
  };
  auto epi_blk = [&](auto c_tag, auto j_tag, float(&v)[4]) {
    constexpr int C = decltype(c_tag)::value, J = decltype(j_tag)::value;
    const float cs[4] = {ecs.x, ecs.y, ecs.z, ecs.w}, pm[4] = {epm.x, epm.y, epm.z, epm.w};
    const float bi[4] = {ebi.x, ebi.y, ebi.z, ebi.w};
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = __builtin_fmaf(acc[C][J][r] * pm[r], cs[r], bi[r]);
    if constexpr (EPBN) {   // eval-mode BN + ReLU (ConvParams::ep_*)
      const float mu[4] = {emu.x, emu.y, emu.z, emu.w}, is[4] = {eis.x, eis.y, eis.z, eis.w};
      const float ga[4] = {ega.x, ega.y, ega.z, ega.w}, be[4] = {ebe.x, ebe.y, ebe.z, ebe.w};
      float m = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = ep_bn_relu(v[r], mu[r], is[r], ga[r], be[r]);
        m = fmaxf(m, fabsf(v[r]));
      }
      amax_run = e_on ? fmaxf(amax_run, m) : amax_run;
    }
    floatx4 o = {v[0], v[1], v[2], v[3]};
    const unsigned so = (unsigned)(J * 16 * p.ldy * 4);
    if constexpr (ACC) {
      const floatx4 prev = h5_bload(eyr, (int)(eyo[C] + so), 0, 0);
      o = floatx4{prev[0] + o[0], prev[1] + o[1], prev[2] + o[2], prev[3] + o[3]};
    }
    if constexpr (!(H5_DBG & 4)) h5_st16(o, eyo[C], eyr, so);
  };
  auto epi_stats = [&](auto c_tag, const float(&v)[kNPB][4]) {   // (mean, M2) of the wave's 80 pixels
    constexpr int C = decltype(c_tag)::value;
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
    if constexpr (!(H5_DBG & 4)) {
      h5_st16(floatx4{mean[0], m2[0], mean[1], m2[1]}, eso[C], esr, eso_t);
      h5_st16(floatx4{mean[2], m2[2], mean[3], m2[3]}, eso[C] + 16u, esr, eso_t);
    }
  };
  auto epi_full = [&](auto c_tag) {
    constexpr int C = decltype(c_tag)::value;
    epi_prm(C);
    float v[kNPB][4];
    h5_for<0, kNPB>([&](auto j_tag) { epi_blk(c_tag, j_tag, v[decltype(j_tag)::value]); });
    if constexpr (TRAIN) epi_stats(c_tag, v);
  };
  // the deferred epilogue runs block C at tap kEpiT0 + C: the last taps of the first chunk, where the converters'
  // staging registers are free again
  constexpr int kEpiT0 = 9 - NCB;
  // vector-memory operations a loader wave issues at tap T after that tap's weight DMA (the deferred epilogue)
  constexpr auto epi_ns = [](int T) {
    return (!ACC && !(H5_DBG & 4) && T >= kEpiT0 && T < 9) ? kNPB + (TRAIN ? 2 : 0) : 0;
  };

  // one tap T (0 .. 17) of the chunk pair (cc, cc + 1) of tile t: chunk cc + T / 9 from halo buffer T / 9
  auto tap = [&](auto T_tag, int cc, int t, bool has_next) {
    constexpr int T = decltype(T_tag)::value;
    constexpr int B = T / 9, TT = T % 9, SL = T % 2;
    const int ch = cc + B;
    // one barrier per tap: after it the ring slot of tap T + 1 is complete (DMA'd at tap T - 2, waited for by
    // its loader just below) and the slot of tap T (read during tap T - 1) free
    stamp();
    // DMA of tap T + 1 (issued at tap T - 2) landed: younger are the DMA of tap T + 2 and the epilogue stores
    // of taps T - 2 and T - 1
    if (loader) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NCB + epi_ns(T - 2) + epi_ns(T - 1)) : "memory");
    asm volatile("s_barrier" ::: "memory");
    stamp();
    if constexpr (!(H5_DBG & 8)) {
      wfrag(std::integral_constant<int, (T + 1) % 2>{}, (T + 1) % 3);   // A fragments of tap T + 1
      if (loader) {
        constexpr int T3 = T + 3;
        int ch3 = cc + T3 / 9;
        if (ch3 >= nch) ch3 -= nch;
        wdma(ch3, T3 % 9, T % 3);                                       // tap T + 3 into tap T's slot
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // the convert of the chunk that follows this one (buffer B ^ 1): this tile's ch + 1, or the next
    // tile's chunk 0; loads at tap 0 / 3, split + LDS writes at tap 3 / 6 (a load group is waited for
    // three taps after its issue, when the weights issued after it are)
    const bool cv_next_tile = ch + 1 >= nch;
    const bool cv_on = (!cv_next_tile || has_next) && !(H5_DBG & 1);
    const int cv_tile = cv_next_tile ? t + 1 : t, cv_ch = cv_next_tile ? 0 : ch + 1;
    // schedule (one or two units converted per tap, loads two to three taps ahead): tap 0 loads units
    // 0 .. 3; tap 2 converts 0, 1 and loads 4, 5; tap 3 converts 2; tap 4 converts 3 and loads 6; taps 5,
    // 6, 7 convert 4, 5, 6.  Every LDS write lands before the barrier of tap 8, after which the next chunk
    // is read.
    const bool cv_up = UP && cv_ch * 32 < p.c0;   // a chunk of the upsampled input: one unit per tap
    if (!loader && cv_on && cv_up) {
      if constexpr (UP) {
        if constexpr (TT >= 1 && TT <= 7) cv_process_up(std::integral_constant<int, TT - 1>{}, cv_tile, cv_ch);
        if constexpr (TT <= 6) cv_issue_up(std::integral_constant<int, TT>{}, cv_tile, cv_ch);
      }
    } else if (!loader && cv_on) {
      if constexpr (TT == 0) {
        cv_issue(I0{}, cv_tile, cv_ch); cv_issue(I1{}, cv_tile, cv_ch);
        cv_issue(I2{}, cv_tile, cv_ch); cv_issue(I3{}, cv_tile, cv_ch);
      }
      if constexpr (TT == 2) {
        cv_process(I0{}, cv_tile, cv_ch); cv_process(I1{}, cv_tile, cv_ch);
        cv_issue(I4{}, cv_tile, cv_ch); cv_issue(I5{}, cv_tile, cv_ch);
      }
      if constexpr (TT == 3) cv_process(I2{}, cv_tile, cv_ch);
      if constexpr (TT == 4) {
        cv_process(I3{}, cv_tile, cv_ch);
        cv_issue(I6{}, cv_tile, cv_ch);
      }
      if constexpr (TT == 5) cv_process(I4{}, cv_tile, cv_ch);
      if constexpr (TT == 6) cv_process(I5{}, cv_tile, cv_ch);
      if constexpr (TT == 7) cv_process(I6{}, cv_tile, cv_ch);
    }
    constexpr bool EPI = !ACC && T >= kEpiT0 && T < 9;   // the deferred epilogue's block T - kEpiT0 at this tap
    constexpr int EC = EPI ? T - kEpiT0 : 0;
    [[maybe_unused]] float ev[kNPB][4];
    if constexpr (EPI) epi_prm(EC);
    if constexpr (TT == 0) {   // fold the previous chunk's partial chain (two-level accumulation)
      if (B == 1 && cc == 0) {   // the tile's first chunk: 0 + part (no zeroing pass)
#pragma unroll
        for (int c = 0; c < NCB; ++c)
#pragma unroll
          for (int j = 0; j < kNPB; ++j) acc[c][j] = part[c][j];
      } else if (B == 1 || cc > 0) {
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
      if constexpr (!(H5_DBG & 32)) {
        unsigned a = ab0[J2];
        if constexpr (B2 != 0) {
          asm volatile("" : "+v"(a));   // (not hoisted into a second register array)
          a += kSBUF;
        }
        a += TOFF2;
        xh[G2 % 3] = *reinterpret_cast<const half8*>(lds + a);
        xl[G2 % 3] = *reinterpret_cast<const half8*>(lds + a + 64);
      }
      if constexpr (EPI) {
        epi_blk(std::integral_constant<int, EC>{}, j_tag, ev[J]);
        if constexpr (TRAIN && J == kNPB - 1) epi_stats(std::integral_constant<int, EC>{}, ev);
      }
      // keep the block's order (its MFMAs, then one block's reads): the scheduler would otherwise hoist
      // reads into fresh registers and run out of them
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  // prologue: the first tile's chunk 0 into buffer 0, the ring's first taps
  __syncthreads();   // (the staged parameters, before the first convert reads them)
  if (!loader && UP) {   // (chunk 0 of an UP launch is always a chunk of the upsampled input)
    h5_for<0, 7>([&](auto u_tag) {
      cv_issue_up(u_tag, t_beg, 0);
      cv_process_up(u_tag, t_beg, 0);
    });
  } else if (!loader) {
    cv_issue(I0{}, t_beg, 0); cv_issue(I1{}, t_beg, 0); cv_issue(I2{}, t_beg, 0); cv_issue(I3{}, t_beg, 0);
    cv_process(I0{}, t_beg, 0); cv_process(I1{}, t_beg, 0); cv_process(I2{}, t_beg, 0); cv_process(I3{}, t_beg, 0);
    cv_issue(I4{}, t_beg, 0); cv_issue(I5{}, t_beg, 0); cv_issue(I6{}, t_beg, 0);
    cv_process(I4{}, t_beg, 0); cv_process(I5{}, t_beg, 0); cv_process(I6{}, t_beg, 0);
  } else {   // the ring's taps 0, 1, 2
    wdma(0, 0, 0);
    wdma(0, 1, 1);
    wdma(0, 2, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  wfrag(std::integral_constant<int, 0>{}, 0);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    xh[j] = *reinterpret_cast<const half8*>(lds + ab0[j]);
    xl[j] = *reinterpret_cast<const half8*>(lds + ab0[j] + 64);
  }
  // (tap 0's DMA overwrites ring slot 0: this wave's reads of it are complete before the barrier)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  for (int t = t_beg; t < t_end; ++t) {
    const bool has_next = t + 1 < t_end;
    for (int cc = 0; cc < nch; cc += 2) {
      if constexpr (!ACC) epi_tile(t - 1, cc == 0 && t > t_beg);   // the previous tile's epilogue, taps 9 - NCB .. 8
      h5_for<0, 18>([&](auto T_tag) { tap(T_tag, cc, t, has_next); });
    }
    // the last chunk's fold: acc = the tile's sums
#pragma unroll
    for (int c = 0; c < NCB; ++c)
#pragma unroll
      for (int j = 0; j < kNPB; ++j) acc[c][j] += part[c][j];
    if constexpr (ACC) {   // (y += conv: not deferred, the loads of y would stall the taps)
      epi_tile(t, true);
      h5_for<0, NCB>([&](auto c_tag) { epi_full(c_tag); });
    }
    stamp();
    ++tile_no;
    nts = 0;
  }
  if constexpr (!ACC) {   // the last tile's epilogue
    epi_tile(t_end - 1, true);
    h5_for<0, NCB>([&](auto c_tag) { epi_full(c_tag); });
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the last (unused) weight DMAs, before the workgroup ends
  if (EPBN && p.ep_amax != nullptr) {   // max|y| of the workgroup's tiles -> one atomicMax
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) amax_run = fmaxf(amax_run, __shfl_xor(amax_run, o, 64));
    float* red = reinterpret_cast<float*>(lds + kOffR);
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
// the shapes h5 takes (forward; an upsampled input: h5_up_supported): W = 40, H a multiple of 8, Cout 64 or 32, input
// channels a multiple of 64 (chunk pairs), the first input a multiple of 32
bool h5_supported(int c0, int c1, int cout, int h, int w, int dil) {
  return w == kW && h > 0 && h % kTR == 0 && dil == 1 && (cout == 64 || cout == 32) && c0 % 32 == 0 &&
         c1 % 32 == 0 && (c0 + c1) % 64 == 0 && (c0 + c1) > 0;
}

int h5_stats_rows() { return kSRB; }

template <int NCB, int MODE>
static void launch_h5_variant(const ConvParams& p, const H3Args& h, int grid, hipStream_t st) {
  note_kernel("conv_fwd_h5_kernel<%d, %d>", NCB, MODE);
  hipLaunchKernelGGL((conv_fwd_h5_kernel<NCB, MODE>), dim3(grid), dim3(512), kLDS, st, p, h);
}

template <int NCB>
static int launch_h5_ncb(const ConvParams& p, const H3Args& h, int grid, hipStream_t st) {
  const bool aff = h.in_scale != nullptr, gate = h.x1_ca != nullptr, epbn = p.ep_mean != nullptr;
  const bool train = p.stats != nullptr || h.xsplit != nullptr;
  if (h.up_src != nullptr) {   // the eval decoder's dec1.conv1: upsampled x0, gated x1, BN + ReLU epilogue
    if (!(gate && epbn && !aff && !train && !p.accumulate)) {
      set_error("srpde_conv_fwd_h3(h5): an upsampled x0 only with a gated x1 and the eval BN epilogue");
      return kErrArg;
    }
    launch_h5_variant<NCB, H5_UP | H5_GATE | H5_EPBN>(p, h, grid, st);
    return 0;
  }
  if (p.accumulate) {   // (not in the U-Net's forward: the plain conv only)
    if (aff || gate || train || epbn) {
      set_error("srpde_conv_fwd_h3(h5): accumulate only without in_scale / gate / statistics / ep");
      return kErrArg;
    }
    launch_h5_variant<NCB, H5_ACC>(p, h, grid, st);
    return 0;
  }
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
