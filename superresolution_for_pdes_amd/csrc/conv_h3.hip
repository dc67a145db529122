// "h3" convolution family for gfx950: fp32-accurate 3x3 convolution from two-piece fp16
// splits on the fp16 MFMA (v_mfma_f32_32x32x16_f16), three partial products per fp32 product.
//
// Same contract as srpde_conv_fwd (conv.hip header comment; reference nn.Conv2d calls at
// src/models.py:16,18,43,46,57,59): forward (sign +1) and dgrad (sign -1, dgrad-packed
// weights), virtual concat of two NHWC inputs, fused bias + BatchNorm partial statistics.
//
// Arithmetic.  Every operand is scaled by a power of two so that the tensor's max|x| lands
// just under 2^15, then split x*s = hi + lo with hi = fp16_rne(x*s) and lo = fp16_rne(x*s - hi):
// 22 significant bits, representation error <= 2^-23 relative (fp32 itself keeps 24).  The
// product a*b is  al*bh + ah*bl + ah*bh  (the dropped al*bl is <= 2^-22 relative and of random
// sign); each partial product is exact in fp32 and accumulated in fp32 by the MFMA.  The
// scales are exact powers of two and are undone in the epilogue.  Activation scales come from
// a max|x| word the producing kernel wrote with atomicMax (bn_relu_fwd / bn_relu_bwd, or
// srpde_absmax); weight scales are per packed row (srpde_split_weights_h3).  fp16 has 11
// significant bits against bf16's 8, so two pieces and three products replace the x6
// kernels' three pieces and six products: half the MFMA work at the same accuracy class.
//
// Data movement.  A 3x3 tap only shifts the pixel rows an output tile reads, so the A
// operand of one 32-channel chunk is staged ONCE as a halo tile -- the tile's BM pixel rows
// plus (W+1)*dil rows either side -- and the nine taps read it at nine row offsets (7x fewer
// A bytes than per-tap staging).  Taps that fall outside the image (padding, row and image
// wrap) read a zeroed LDS row instead.  The halo tile lands fp32 (buffer_load ... lds DMA,
// no VGPR staging) and is scaled and split into hi / lo fp16 planes in LDS once per chunk, so
// each element is split once, not once per tap; the nine tap stages then read MFMA fragments
// of both operands straight from LDS.  The next chunk's halo tile is DMA'd in slices during
// the current chunk's stages; the weight tile of each tap stage is double-buffered.  One
// partial MFMA chain per chunk (two-level fp32 accumulation).
#include <atomic>

#include "conv_common.h"
#include "conv_h3.h"

namespace srpde {

// TWO_LEVEL: one partial MFMA chain per channel chunk folded into the accumulator (needs twice
// the accumulator registers); otherwise one fp32 MFMA chain over all of K, as a CPU GEMM sums.
// TPS: taps per stage (one barrier per stage; the weight stage holds TPS taps).
template <int BM, int BN, int WM, int WN, int SRB, bool TWO_LEVEL, int TPS, bool BNB = false, bool PRE = false>
__global__ __launch_bounds__(WM * WN * 64, 8 / (WM * WN)) void conv_fwd_h3_kernel(ConvParams p, H3Args h) {
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int TM = BM / WM, TN = BN / WN, TI = TM / 32, TJ = TN / 32;
  constexpr int BTOT = 2 * BN / 16;        // B DMA instructions per stage (16 rows x 64 B)
  constexpr int BPW = (BTOT + NW - 1) / NW;
  constexpr int BP_BYTES = BN * 64;        // one fp16 plane of the B tile (one tap)
  constexpr int B_TAP = 2 * BP_BYTES;      // hi + lo planes of one tap
  constexpr int B_STAGE = TPS * B_TAP;
  constexpr int NS = (9 + TPS - 1) / TPS;  // stages per channel chunk
  constexpr int AQ = (64 / NW + NS - 2) / (NS - 1);   // halo-slice DMAs per wave in stages 0..NS-2 (64 / NW per wave
                                                      // and chunk: arows <= 512)
  constexpr int AD = BNB ? 2 : 1;               // DMAs per halo slice (BNB: the gradient and the BN input)
  static_assert(BM % SRB == 0 && WM % (BM / SRB) == 0, "statistics sub-blocks");
  static_assert(TPS >= 1 && TPS <= 3, "taps per stage");
  static_assert(!(BNB && PRE), "one input transform");
  // LDS: F = fp32 halo tile (DMA target, 128-B rows) | S = its split, 128-B rows of eight 16-B
  //      chunks: hi pieces of channel group c8 in chunk c8, lo pieces in chunk 4 + c8, chunk k at
  //      slot swz(r, k) (conflict-free reads at any tap shift; a row's four fragments of one
  //      lane are XOR 32 / 64 / 96 of each other) | B = two weight stages | 128 zero bytes
  //      (the padding row, 128-B aligned so the XORs stay in it) | 1 KiB DMA sink
  // PRE (the input arrives as its h3 split, [2][P][Cin] fp16 hi / lo planes scaled by 2^h3_exp(amax0)):
  //      no F and no convert -- two S-layout buffers of arows + 1 rows (the last one zero), chunk c's
  //      halo tile DMA'd straight into buffer c & 1 in S order (source-side swizzle) while the other
  //      buffer is read | B | 1 KiB DMA sink
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* lds = reinterpret_cast<char*>(smem);
  const int arows = h.arows;
  const int abuf = (arows + 1) * 128;           // PRE: bytes per A buffer
  char* const fbuf = lds;
  char* const fbuf2 = fbuf + arows * ROW2;      // BNB: fp32 halo tile of the BN input y
  const int soff = PRE ? 0 : (BNB ? 2 : 1) * arows * ROW2;   // S, as a byte offset from lds
  char* const sbuf = lds + soff;
  char* const bbuf0 = PRE ? lds + 2 * abuf : sbuf + arows * 128;
  char* const zrow = PRE ? lds + arows * 128 : bbuf0 + 2 * B_STAGE;
  const int zoff = PRE ? arows * 128 : soff + arows * 128 + 2 * B_STAGE;   // PRE: relative to the buffer
  char* const sink = PRE ? bbuf0 + 2 * B_STAGE : zrow + 128;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
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

  if (tid < 32) reinterpret_cast<float*>(zrow)[tid] = 0.f;
  if (PRE && tid >= 32 && tid < 64) reinterpret_cast<float*>(zrow + abuf)[tid - 32] = 0.f;   // buffer 1's zero row

  const int32x4 rs0 = make_rsrc(p.x0, (unsigned)((size_t)p.P * p.ldx0 * 4));
  const int32x4 rs1 = make_rsrc(p.c1 ? p.x1 : p.x0, (unsigned)((size_t)p.P * (p.c1 ? p.ldx1 : p.ldx0) * 4));
  const size_t plane = (size_t)p.Cout * p.K;   // fp16 elements per weight plane
  const int32x4 rsw = make_rsrc(h.wsp, (unsigned)(2 * plane * 2));
  const int32x4 rsy = BNB ? make_rsrc(h.bnb_y, (unsigned)((size_t)p.P * h.bnb_ldy * 4)) : rs0;
  const int ld1 = p.c1 ? p.ldx1 : p.ldx0;

  // activation scale (shared by both inputs of a virtual concat)
  unsigned ab = h.amax0 ? *h.amax0 : 0u;
  if (p.c1 && h.amax1) ab = max(ab, *h.amax1);
  const int ea = h3_exp(ab);
  const float sa = exp2i(ea);

  // per tap: the LDS byte offset of this lane's A fragment (hi pieces; lo = XOR 64) of its 16x16x32
  // row (lane & 15 of each 16-row block, chunk lane >> 4) shifted by the tap; the zero row for taps
  // outside the image.  Computed once per tile.
  const int lr = lane & 31;
  const int l16 = lane & 15, lq = lane >> 4;
  const int wmi = wave % WM, wni = wave / WM;
  const int wm0 = wmi * TM, wn0 = wni * TN;
  constexpr int TI16 = 2 * TI, TJ16 = 2 * TJ;
  // (the image row / column of each of this lane's rows; the nine tap offsets are formed per tap from
  // them -- a [9][TI16] table held 18 VGPRs through the loop)
  int ayy[TI16], axx[TI16];
#pragma unroll
  for (int i = 0; i < TI16; ++i) {
    const int m = m0 + wm0 + i * 16 + l16;
    int yy = -(1 << 20), xx = 0;   // rows past the tensor: every tap reads the zero row
    if (m < p.P) {
      const int rem = m % HW;
      yy = rem / p.W;
      xx = rem - yy * p.W;
    }
    ayy[i] = yy;
    axx[i] = xx;
  }
  auto aoff_of = [&](auto tap_tag, int i) -> int {
    constexpr int t = decltype(tap_tag)::value;
    const int ky = p.sign > 0 ? t / 3 : 2 - t / 3, kx = p.sign > 0 ? t % 3 : 2 - t % 3;
    const int iy = ayy[i] + (t / 3 - 1) * p.dil * p.sign, ix = axx[i] + (t % 3 - 1) * p.dil * p.sign;
    const int r = wm0 + i * 16 + l16 + (ky * p.W + kx) * p.dil;
    return (iy >= 0 && iy < p.H && ix >= 0 && ix < p.W) ? soff + r * 128 + swz(r, lq) * 16 : zoff;
  };
  // B: instruction q = plane * (BN/16) + 16-row block; lane -> (row, slot), fetches chunk swzh^-1
  int b_off[BPW];
#pragma unroll
  for (int j = 0; j < BPW; ++j) {
    const int q = wave + j * NW;
    const int pl = q / (BN / 16), rb = q - pl * (BN / 16);
    const int r = rb * 16 + (lane >> 2);
    const int c = swzh(r, lane & 3);
    const int nn = n0 + r;
    b_off[j] = (q < BTOT && nn < p.Cout) ? (int)((pl * plane + (size_t)nn * p.K + c * 8) * 2) : -1;
  }

  const int nch = p.Cin / BK2;
  const int c_beg = tail ? (piece * nch) / p.tsplit : 0;
  const int c_end = tail ? ((piece + 1) * nch) / p.tsplit : nch;
  const int na = arows / 8;                   // A DMA instructions per chunk (8 rows x 128 B)
  const int pix0 = m0 - h.halo;

  const size_t xplane = (size_t)p.P * p.Cin;
  // A slice `q` of chunk `ch` (8 halo rows, fp32) into F; q >= na: a zero-fill DMA into the sink,
  // so every wave issues the same number of vector-memory ops per stage (exact vmcnt counts)
  auto issue_a = [&](int ch, int q) {
    if constexpr (PRE) {   // 8 rows x 128 B of S into buffer ch & 1: lane slot (lane & 7) holds chunk
                           // slot ^ ((r >> 1) & 7) (swz is an involution): hi (< 4) or lo plane piece
      const int r = q * 8 + (lane >> 3);
      const int pix = pix0 + r;
      const bool real = q < na;
      const int k = (lane & 7) ^ ((r >> 1) & 7);
      const unsigned off = (real && pix >= 0 && pix < p.P)
                               ? (unsigned)(((k >= 4 ? xplane : 0) + (size_t)pix * p.Cin + ch * BK2 + (k & 3) * 8) * 2)
                               : OOB;
      dma16(rs0, off, lds_addr_of(real ? lds + (ch & 1) * abuf + q * 1024 : sink));
      return;
    }
    const int ch0 = ch * BK2;
    const bool second = ch0 >= p.c0;
    const int32x4 rs = second ? rs1 : rs0;
    const int ld = second ? ld1 : p.ldx0;
    const int cb = second ? ch0 - p.c0 : ch0;
    const int r = q * 8 + (lane >> 3);
    const int pix = pix0 + r;
    const bool real = q < na;
    const unsigned off = (real && pix >= 0 && pix < p.P) ? (unsigned)((pix * ld + cb + swz(r, lane & 7) * 4) * 4) : OOB;
    dma16(rs, off, lds_addr_of(real ? fbuf + q * 1024 : sink));
    if constexpr (BNB) {
      const unsigned offy = (real && pix >= 0 && pix < p.P) ? (unsigned)((pix * h.bnb_ldy + cb + swz(r, lane & 7) * 4) * 4)
                                                            : OOB;
      dma16(rsy, offy, lds_addr_of(real ? fbuf2 + q * 1024 : sink));
    }
  };
  auto issue_b = [&](int ch, int st, int buf) {   // the TPS taps of stage `st` of chunk `ch`
#pragma unroll
    for (int u = 0; u < TPS; ++u) {
      const int tap = st * TPS + u;
      if (tap < 9) {
        const int k0 = tap * p.Cin + ch * BK2;
        char* bbase = bbuf0 + buf * B_STAGE + u * B_TAP;
#pragma unroll
        for (int j = 0; j < BPW; ++j) {
          const int q = wave + j * NW;
          if (q < BTOT) {
            const unsigned off = b_off[j] >= 0 ? (unsigned)(b_off[j] + k0 * 2) : OOB;
            dma16(rsw, off, lds_addr_of(bbase + q * 1024));
          }
        }
      }
    }
  };
  // F (fp32, landed) -> S: scale and split every halo element once per chunk
  // (the N-tile-0 workgroup of each row tile also stores its own rows' pieces to h.xsplit)
  const bool wsplit = !PRE && h.xsplit != nullptr && nt == 0;
  struct BnbCoef { float mu[8], is[8], ga[8], be[8], m1[8], m2[8]; };
  auto convert = [&](int ch) {
    BnbCoef bq;
    if constexpr (BNB) {   // this thread's 8 channels (sg & 3 == tid & 3 for every task of the loop below)
      const int cc = ch * BK2 + (tid & 3) * 8;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        bq.mu[k] = h.bnb_mean[cc + k]; bq.is[k] = h.bnb_invstd[cc + k];
        bq.ga[k] = h.bnb_gamma[cc + k]; bq.be[k] = h.bnb_beta[cc + k];
        bq.m1[k] = h.bnb_m1[cc + k]; bq.m2[k] = h.bnb_m2[cc + k];
      }
    }
    (void)bq;
    for (int sg = tid; sg < arows * 4; sg += NT) {
      const int r = sg >> 2, c8 = sg & 3;
      float4 v0 = *reinterpret_cast<const float4*>(fbuf + r * ROW2 + swz(r, 2 * c8) * 16);
      float4 v1 = *reinterpret_cast<const float4*>(fbuf + r * ROW2 + swz(r, 2 * c8 + 1) * 16);
      if constexpr (BNB) {   // fused BN (+ReLU) backward: da (F) and y (F2) -> dy; rows outside the tensor stay 0
        const bool inside = pix0 + r >= 0 && pix0 + r < p.P;
        const float4 y0 = *reinterpret_cast<const float4*>(fbuf2 + r * ROW2 + swz(r, 2 * c8) * 16);
        const float4 y1 = *reinterpret_cast<const float4*>(fbuf2 + r * ROW2 + swz(r, 2 * c8 + 1) * 16);
        float vv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        const float yy8[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          // the same expressions as bn_bwd_apply_kernel (bn.hip)
          const float xh = (yy8[k] - bq.mu[k]) * bq.is[k];
          const float dz = (!h.bnb_relu || xh * bq.ga[k] + bq.be[k] > 0.f) ? vv[k] : 0.f;
          vv[k] = inside ? (dz - bq.m1[k] - xh * bq.m2[k]) * (bq.ga[k] * bq.is[k]) : 0.f;
        }
        v0 = make_float4(vv[0], vv[1], vv[2], vv[3]);
        v1 = make_float4(vv[4], vv[5], vv[6], vv[7]);
      }
      if (h.x1_ca != nullptr && ch * BK2 >= p.c0) gate8(v0, v1, h, pix0 + r, p.P, p.H * p.W, p.c1, ch * BK2 - p.c0 + c8 * 8);
      if (h.in_scale != nullptr) {   // fused BN + ReLU of the producer; rows outside the tensor stay 0
        const int cc = ch * BK2 + c8 * 8, pix = pix0 + r;
        const bool inside = pix >= 0 && pix < p.P;
        const float4 s0 = *reinterpret_cast<const float4*>(h.in_scale + cc);
        const float4 s1 = *reinterpret_cast<const float4*>(h.in_scale + cc + 4);
        const float4 t0 = *reinterpret_cast<const float4*>(h.in_shift + cc);
        const float4 t1 = *reinterpret_cast<const float4*>(h.in_shift + cc + 4);
#define AFF(V, S, T, X) V.X = inside ? fmaxf(V.X * S.X + T.X, 0.f) : 0.f;
        AFF(v0, s0, t0, x) AFF(v0, s0, t0, y) AFF(v0, s0, t0, z) AFF(v0, s0, t0, w)
        AFF(v1, s1, t1, x) AFF(v1, s1, t1, y) AFF(v1, s1, t1, z) AFF(v1, s1, t1, w)
#undef AFF
      }
      half8 hv, lv;
      split2h(v0, v1, sa, hv, lv);
      *reinterpret_cast<half8*>(sbuf + r * 128 + swz(r, c8) * 16) = hv;
      *reinterpret_cast<half8*>(sbuf + r * 128 + swz(r, 4 + c8) * 16) = lv;
      if (wsplit) {
        const int pix = pix0 + r;
        if (r >= h.halo && r < h.halo + BM && pix < p.P) {
          _Float16* dst = h.xsplit + (size_t)pix * p.Cin + ch * BK2 + c8 * 8;
          *reinterpret_cast<half8*>(dst) = hv;
          *reinterpret_cast<half8*>(dst + xplane) = lv;
        }
      }
    }
  };

  floatx4 acc[TI16][TJ16];
  floatx4 part[TWO_LEVEL ? TI16 : 1][TWO_LEVEL ? TJ16 : 1];
  auto chain = [&](int i, int j) -> floatx4& {
    if constexpr (TWO_LEVEL) return part[i][j];
    else return acc[i][j];
  };
#pragma unroll
  for (int i = 0; i < TI16; ++i)
#pragma unroll
    for (int j = 0; j < TJ16; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.f;

  // prologue: whole halo tile of the first chunk + first weight stage
  if (!(SRPDE_CONV_DBG & 32))   // diagnostics: 32 = no prologue halo DMA, 64 = no prologue convert
    for (int q = wave; q < na; q += NW) issue_a(c_beg, q);
  issue_b(c_beg, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (!PRE && !(SRPDE_CONV_DBG & 64)) convert(c_beg);
  __syncthreads();

  int sidx = 0;      // stage counter (B buffer parity)
  int acur = 0;      // PRE: byte offset of the current chunk's A buffer
  // one tap: the A fragments and the first column block's B fragments, then one column block's
  // MFMAs per further B read pair (without the schedule the compiler parks each read right before
  // its MFMA and exposes its latency)
  // A fragments of the next tap, read during the current tap's last MFMA group (within a chunk the
  // A tile does not change, so they stay valid across the stage barrier); tap 0 of a chunk reads its own.
  // Pre-split inputs only: the convert path's registers leave no room for them in the other kernels
  // (48 B of scratch, forward +3 %; presplit dgrad -2.4 %, tools/gpu/lib_ab.sh)
  constexpr bool PF = PRE;
  half8 pah[TI16], pal[TI16];
  auto tap_body = [&](const char* b, auto tap_tag) {
    constexpr int TAP = decltype(tap_tag)::value;
    half8 ah[TI16], al[TI16], bh[TJ16], bl[TJ16];
    const char* abase = PRE ? lds + acur : lds;
#pragma unroll
    for (int i = 0; i < TI16; ++i) {   // lo pieces: XOR 64 (see the LDS layout)
      if constexpr (TAP == 0 || !PF) {
        const int o = aoff_of(std::integral_constant<int, TAP>{}, i);
        ah[i] = *reinterpret_cast<const half8*>(abase + o);
        al[i] = *reinterpret_cast<const half8*>(abase + (o ^ 64));
      } else {
        ah[i] = pah[i];
        al[i] = pal[i];
      }
    }
#pragma unroll
    for (int j = 0; j < TJ16; ++j) {
      const int r = wn0 + j * 16 + l16;
      const int o = r * 64 + swzh(r, lq) * 16;
      bh[j] = *reinterpret_cast<const half8*>(b + o);
      bl[j] = *reinterpret_cast<const half8*>(b + BP_BYTES + o);
    }
#pragma unroll
    for (int j = 0; j < TJ16; ++j)
#pragma unroll
      for (int i = 0; i < TI16; ++i) {
        floatx4 c0;
        if (TWO_LEVEL && TAP == 0)   // a chunk's partial chain starts from zero
          c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], floatx4{}, 0, 0, 0);
        else   // small terms first
          c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], chain(i, j), 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j], c0, 0, 0, 0);
        chain(i, j) = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], c0, 0, 0, 0);
      }
    if constexpr (PF && TAP < 8) {
#pragma unroll
      for (int i = 0; i < TI16; ++i) {
        const int o = aoff_of(std::integral_constant<int, (TAP < 8 ? TAP + 1 : 8)>{}, i);
        pah[i] = *reinterpret_cast<const half8*>(abase + o);
        pal[i] = *reinterpret_cast<const half8*>(abase + (o ^ 64));
      }
    }
    __builtin_amdgcn_sched_group_barrier(0x100, (TAP == 0 || !PF) ? 2 * TI16 + 2 : 2, 0);
#pragma unroll
    for (int j = 1; j < TJ16; ++j) {
      __builtin_amdgcn_sched_group_barrier(0x008, 3 * TI16, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
    if constexpr (PF && TAP < 8) __builtin_amdgcn_sched_group_barrier(0x100, 2 * TI16, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 3 * TI16, 0);
  };
  auto stage = [&](int ch, auto st_tag) {
    constexpr int ST = decltype(st_tag)::value;
    // prefetch: the next weight stage, then AQ slices of the next chunk's halo tile (F is free:
    // the current chunk was converted to S before its first stage)
    const bool more = ch + 1 < c_end;
    const bool dma = !(SRPDE_CONV_DBG & 1);   // diagnostics (SRPDE_CONV_DBG, results wrong): 1 = no DMA in the loop
    // waves 4..7 issue the stage's LDS-DMA pieces between its two taps, waves 0..3 before them: the two
    // waves of a SIMD issue out of phase, each under the other's MFMAs (fwd -1.7 %, dgrad -0.6 % on the
    // deep layers, tools/gpu/dma_ab.sh)
    const bool late_b = wave >= 4 && TPS > 1;
    const bool late_a = late_b;
    auto dma_b = [&]() {
      if (dma && ST < NS - 1) issue_b(ch, ST + 1, (sidx + 1) & 1);
      else if (dma && more) issue_b(ch + 1, 0, (sidx + 1) & 1);
    };
    auto dma_a = [&]() {
      if (dma && ST < NS - 1 && more) {
#pragma unroll
        for (int u = 0; u < AQ; ++u) issue_a(ch + 1, wave + (ST * AQ + u) * NW);
      }
    };
    if (!late_b) dma_b();
    if (!late_a) dma_a();
    const char* b = bbuf0 + (sidx & 1) * B_STAGE;
    if (!(SRPDE_CONV_DBG & 128)) {   // diagnostics: 128 = no MFMA work
      tap_body(b, std::integral_constant<int, ST * TPS>{});
      if (late_b) dma_b();
      if (late_a) dma_a();
      if constexpr (TPS > 1 && ST * TPS + 1 < 9) tap_body(b + B_TAP, std::integral_constant<int, ST * TPS + 1>{});
      if constexpr (TPS > 2 && ST * TPS + 2 < 9) tap_body(b + 2 * B_TAP, std::integral_constant<int, ST * TPS + 2>{});
    } else {
      if (late_b) dma_b();
      if (late_a) dma_a();
    }
    ++sidx;
    // the next stage's weights must have landed; the halo slices issued after them may still be
    // in flight (they are waited for by the next stage's count, long before the chunk ends)
    if (ST < NS - 1 && more && h.relax)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(AQ * AD) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!(SRPDE_CONV_DBG & 2)) __syncthreads();   // diagnostics: 2 = no stage barrier
  };
  for (int ch = c_beg; ch < c_end; ++ch) {
    if constexpr (PRE) acur = (ch & 1) * abuf;
    stage(ch, std::integral_constant<int, 0>{});
    if constexpr (NS > 1) stage(ch, std::integral_constant<int, 1>{});
    if constexpr (NS > 2) stage(ch, std::integral_constant<int, 2>{});
    if constexpr (NS > 3) stage(ch, std::integral_constant<int, 3>{});
    if constexpr (NS > 4) stage(ch, std::integral_constant<int, 4>{});
    if constexpr (NS > 5) stage(ch, std::integral_constant<int, 5>{});
    if constexpr (NS > 6) stage(ch, std::integral_constant<int, 6>{});
    if constexpr (NS > 7) stage(ch, std::integral_constant<int, 7>{});
    if constexpr (NS > 8) stage(ch, std::integral_constant<int, 8>{});
    // two-level accumulation: one partial chain per channel chunk (9 taps x 32 channels)
    if constexpr (TWO_LEVEL) {
#pragma unroll
      for (int i = 0; i < TI16; ++i)
#pragma unroll
        for (int j = 0; j < TJ16; ++j) acc[i][j] += part[i][j];
    }
    if (!PRE && ch + 1 < c_end && !(SRPDE_CONV_DBG & 4)) {   // the next chunk's halo tile has landed in F (vmcnt(0) + barrier)
      convert(ch + 1);                      // (diagnostics: 4 = no per-chunk convert)
      __syncthreads();
    }
  }
  // the 32x32x16 accumulator layout of the epilogue
  floatx16 acc32[TI][TJ];
  acc16_to_32<TI, TJ>(acc, acc32);
  // the scales to undo: acc * 2^-(ea + wexp[col]), exact; applied by the epilogue in the same FMA
  // as the bias.  A combined exponent outside the normal range (operands of extreme magnitude)
  // takes the activation scale here first, so no intermediate under- or overflows.
  float colscale[TJ];
  const float ia = exp2i(-ea);
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int col = n0 + wn0 + j * 32 + lr;
    const int we = col < p.Cout ? h.wexp[col] : 0;
    const int e = ea + we;
    if (e > 126 || e < -126) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc32[i][j][r] *= ia;
      colscale[j] = exp2i(-we);
    } else {
      colscale[j] = exp2i(-e);
    }
    if (col >= p.Cout) colscale[j] = 0.f;
  }
  if (SRPDE_CONV_DBG & 16) {   // diagnostics: 16 = no epilogue (one store per lane keeps the MFMAs live)
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) t += acc32[i][j][0] * colscale[j] + acc32[i][j][15];
    if (t == 123.f) p.y[tid] = t;
    return;
  }
  // the halo buffer F is free now: reduction scratch [2][WM][BN] floats, then 2 KiB per wave of store stage
  x6_finish<BM, BN, WM, WN, SRB>(p, acc32, tail, wg, nfull, piece, m0, n0, wmi, wni, lane, smem,
                                 h.wide ? smem + 2 * WM * BN : nullptr, colscale);
}

// ------------- h3r: register-staged halo tiles, 4 waves, two workgroups per CU -------------
// The shallow-K layers (output tiles of 64 / 32 channels: the 40x40 convolutions and the dgrads
// into 64 channels) run only 2-6 channel chunks per tile, so the per-tile work -- tap-address
// setup, halo split, bias + BatchNorm-statistics epilogue, DMA latency at the prologue -- weighs
// as much as the MFMAs, and with one 8-wave workgroup per CU (conv_fwd_h3_kernel: fp32 halo tile
// F + its split S + weight stages = 120 KiB of LDS) every wave of the CU reaches those phases at
// the same barriers and the MFMA pipes idle through them.  Here the next chunk's halo tile is
// loaded into VGPRs (buffer_load_dwordx4, issued after the chunk's last fragment reads, so the
// prefetch registers never live together with the fragments) instead of into an fp32 LDS tile,
// and split from registers into S after the chunk: no F, so a workgroup needs S + a ring of NB
// weight stages (<= 78 KiB) and two workgroups share a CU -- one's setup / split / epilogue and
// halo-load latency run under the other's MFMAs.  The weight ring is fed NB - 1 stages ahead,
// across chunk boundaries (a one-stage lead does not cover an L2 round trip under load: one tap
// is 24 MFMAs per wave).  A workgroup is 4 waves stacked
// along M, each 64 rows x BN columns (8 fragment reads per 12 MFMAs at BN = 64, against 6 per 6
// in the 8-wave 32-row layout).  Same arithmetic (the same split, product order and two-level
// accumulation per chunk) and the same epilogue, statistics blocks and output as the 8-wave kernel.
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ f32x4 llvm_raw_buffer_load_f4(int32x4 rsrc, int voffset, int soffset,
                                         int aux) __asm("llvm.amdgcn.raw.buffer.load.v4f32");

// PRE: the input arrives as its h3 split ([2][P][Cin] fp16 planes, conv_fwd_h3_kernel): the halo
// tasks load the hi / lo pieces and the convert only stores them
template <int BN, int TPS, int NTK, int NB, bool PRE = false>
__global__ __launch_bounds__(256, 2) void conv_fwd_h3r_kernel(ConvParams p, H3Args h) {
  constexpr int BM = 256, WM = 4, WN = 1, NW = 4, NT = 256, SRB = 128;
  constexpr int TM = BM / WM, TN = BN / WN, TI = TM / 32, TJ = TN / 32;
  constexpr int BTOT = 2 * BN / 16;        // B DMA instructions per tap (16 rows x 64 B)
  constexpr int BPW = (BTOT + NW - 1) / NW;
  constexpr int BP_BYTES = BN * 64;
  constexpr int B_TAP = 2 * BP_BYTES;
  constexpr int B_STAGE = TPS * B_TAP;
  constexpr int NS = (9 + TPS - 1) / TPS;
  constexpr int DPS = TPS * BPW;           // weight DMAs per wave per stage (spares into the sink: exact counts)
  static_assert(NB >= 2 && NB <= NS + 1, "weight ring");
  // LDS: 128 zero bytes (the padding row) | S (arows 128-B rows: hi / lo fp16 pieces of 32
  // channels, slot swz(r, k)) | NB weight stages | 1 KiB DMA sink.  Every A-fragment offset is
  // below 64 KiB, so the per-tap offsets of a lane's two row blocks share one VGPR.
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* lds = reinterpret_cast<char*>(smem);
  const int arows = h.arows;
  char* const zrow = lds;
  char* const sbuf = lds + 128;
  char* const bbuf0 = sbuf + arows * 128;
  char* const sink = bbuf0 + NB * B_STAGE;
  constexpr int zoff = 0;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
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

  if (tid < 32) reinterpret_cast<float*>(zrow)[tid] = 0.f;

  const int32x4 rs0 = make_rsrc(p.x0, (unsigned)((size_t)p.P * p.ldx0 * 4));
  const int32x4 rs1 = make_rsrc(p.c1 ? p.x1 : p.x0, (unsigned)((size_t)p.P * (p.c1 ? p.ldx1 : p.ldx0) * 4));
  const size_t plane = (size_t)p.Cout * p.K;
  const int32x4 rsw = make_rsrc(h.wsp, (unsigned)(2 * plane * 2));
  const int ld1 = p.c1 ? p.ldx1 : p.ldx0;

  unsigned ab = h.amax0 ? *h.amax0 : 0u;
  if (p.c1 && h.amax1) ab = max(ab, *h.amax1);
  const int ea = h3_exp(ab);
  const float sa = exp2i(ea);

  const int lr = lane & 31;
  const int l16 = lane & 15, lq = lane >> 4;
  const int wmi = wave, wni = 0;
  const int wm0 = wmi * TM, wn0 = 0;
  constexpr int TI16 = 2 * TI, TJ16 = 2 * TJ;
  static_assert(TI16 == 4, "four 16-row blocks per wave: two packed offset words per tap");
  // per tap and 16-row block: the LDS byte offset of this lane's 16x16x32 A fragment (hi pieces;
  // lo = XOR 64), two blocks' offsets per 32-bit word
  unsigned apk[9][2];
#pragma unroll
  for (int i = 0; i < TI16; ++i) {
    const int m = m0 + wm0 + i * 16 + l16;
    int yy = -(1 << 20), xx = 0;
    if (m < p.P) {
      const int rem = m % HW;
      yy = rem / p.W;
      xx = rem - yy * p.W;
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ky = p.sign > 0 ? t / 3 : 2 - t / 3, kx = p.sign > 0 ? t % 3 : 2 - t % 3;
      const int iy = yy + (t / 3 - 1) * p.dil * p.sign, ix = xx + (t % 3 - 1) * p.dil * p.sign;
      const int r = wm0 + i * 16 + l16 + (ky * p.W + kx) * p.dil;
      const unsigned ao = (iy >= 0 && iy < p.H && ix >= 0 && ix < p.W) ? 128 + r * 128 + swz(r, lq) * 16 : zoff;
      if (i % 2 == 0) apk[t][i / 2] = ao;
      else apk[t][i / 2] |= ao << 16;
    }
  }
  int b_off[BPW];
#pragma unroll
  for (int j = 0; j < BPW; ++j) {
    const int q = wave + j * NW;
    const int pl = q / (BN / 16), rb = q - pl * (BN / 16);
    const int r = rb * 16 + (lane >> 2);
    const int c = swzh(r, lane & 3);
    const int nn = n0 + r;
    b_off[j] = (q < BTOT && nn < p.Cout) ? (int)((pl * plane + (size_t)nn * p.K + c * 8) * 2) : -1;
  }

  const int nch = p.Cin / BK2;
  const int c_beg = tail ? (piece * nch) / p.tsplit : 0;
  const int c_end = tail ? ((piece + 1) * nch) / p.tsplit : nch;
  const int ntask = arows * 4;                // (halo row, 8-channel group) tasks of one chunk
  const int pix0 = m0 - h.halo;

  // the halo tile of chunk `ch`, task k of this thread -> pf[k] (8 fp32 channels; rows outside
  // the tensor and tasks past the tile: the range check returns zeros)
  f32x4 pf[NTK][2];
  auto load_task = [&](int ch, int k) {
    const int ch0 = ch * BK2;
    const bool second = ch0 >= p.c0;
    const int32x4 rs = second ? rs1 : rs0;
    const int ld = second ? ld1 : p.ldx0;
    const int cb = second ? ch0 - p.c0 : ch0;
    int t = tid;
    asm volatile("" : "+v"(t));   // recompute the task addresses per call (no registers held across the loop)
    const int sg = t + NT * k;
    const int r = sg >> 2, c8 = sg & 3;
    const int pix = pix0 + r;
    if constexpr (PRE) {
      const unsigned off = (sg < ntask && pix >= 0 && pix < p.P) ? (unsigned)((pix * p.Cin + cb + c8 * 8) * 2) : OOB;
      pf[k][0] = llvm_raw_buffer_load_f4(rs0, (int)off, 0, 0);
      pf[k][1] = llvm_raw_buffer_load_f4(rs0, off == OOB ? (int)OOB : (int)(off + (unsigned)(p.P * p.Cin * 2)), 0, 0);
      return;
    }
    const unsigned off = (sg < ntask && pix >= 0 && pix < p.P) ? (unsigned)((pix * ld + cb + c8 * 8) * 4) : OOB;
    pf[k][0] = llvm_raw_buffer_load_f4(rs, (int)off, 0, 0);
    pf[k][1] = llvm_raw_buffer_load_f4(rs, (int)(off + 16u), 0, 0);
  };
  // the TPS taps of stage `st` of chunk `ch` into ring slot `buf`; exactly DPS DMAs per wave
  // (missing taps / rows, or ch < 0 = past the last stage: zero fills into the sink)
  auto issue_b = [&](int ch, int st, int buf) {
#pragma unroll
    for (int u = 0; u < TPS; ++u) {
      const int tap = st * TPS + u;
      const int k0 = tap * p.Cin + ch * BK2;
      char* bbase = bbuf0 + buf * B_STAGE + u * B_TAP;
#pragma unroll
      for (int j = 0; j < BPW; ++j) {
        const int q = wave + j * NW;
        const bool real = ch >= 0 && tap < 9 && q < BTOT;
        const unsigned off = (real && b_off[j] >= 0) ? (unsigned)(b_off[j] + k0 * 2) : OOB;
        dma16(rsw, off, lds_addr_of(real ? bbase + q * 1024 : sink));
      }
    }
  };
  const bool wsplit = h.xsplit != nullptr && nt == 0;
  const size_t xplane = (size_t)p.P * p.Cin;
  // registers (chunk ch) -> S: scale and split every halo element once per chunk
  auto convert = [&](int ch) {
    int t = tid;
    asm volatile("" : "+v"(t));   // as in load_task
    // fused BN + ReLU of the producer: every task of a thread has the same 8 channels (t & 3),
    // so their (scale, shift) are loaded once per chunk, not once per task
    float4 s0, s1, t0, t1;
    const bool gate = !PRE && h.x1_ca != nullptr && ch * BK2 >= p.c0;   // the attention-gated second input
    if (h.in_scale != nullptr) {
      const int cc = ch * BK2 + (t & 3) * 8;
      s0 = *reinterpret_cast<const float4*>(h.in_scale + cc);
      s1 = *reinterpret_cast<const float4*>(h.in_scale + cc + 4);
      t0 = *reinterpret_cast<const float4*>(h.in_shift + cc);
      t1 = *reinterpret_cast<const float4*>(h.in_shift + cc + 4);
    }
#pragma unroll
    for (int k = 0; k < NTK; ++k) {
      const int sg = t + NT * k;
      if (PRE && sg < ntask) {
        const int r = sg >> 2, c8 = sg & 3;
        *reinterpret_cast<half8*>(sbuf + r * 128 + swz(r, c8) * 16) = __builtin_bit_cast(half8, pf[k][0]);
        *reinterpret_cast<half8*>(sbuf + r * 128 + swz(r, 4 + c8) * 16) = __builtin_bit_cast(half8, pf[k][1]);
      } else if (sg < ntask) {
        const int r = sg >> 2, c8 = sg & 3;
        float4 v0 = make_float4(pf[k][0].x, pf[k][0].y, pf[k][0].z, pf[k][0].w);
        float4 v1 = make_float4(pf[k][1].x, pf[k][1].y, pf[k][1].z, pf[k][1].w);
        if (gate) gate8(v0, v1, h, pix0 + r, p.P, p.H * p.W, p.c1, ch * BK2 - p.c0 + c8 * 8);
        if (h.in_scale != nullptr) {   // rows outside the tensor stay 0
          const int pix = pix0 + r;
          const bool inside = pix >= 0 && pix < p.P;
#define AFF(V, S, T, X) V.X = inside ? fmaxf(__builtin_fmaf(V.X, S.X, T.X), 0.f) : 0.f;
          AFF(v0, s0, t0, x) AFF(v0, s0, t0, y) AFF(v0, s0, t0, z) AFF(v0, s0, t0, w)
          AFF(v1, s1, t1, x) AFF(v1, s1, t1, y) AFF(v1, s1, t1, z) AFF(v1, s1, t1, w)
#undef AFF
        }
        half8 hv, lv;
        split2h(v0, v1, sa, hv, lv);
        *reinterpret_cast<half8*>(sbuf + r * 128 + swz(r, c8) * 16) = hv;
        *reinterpret_cast<half8*>(sbuf + r * 128 + swz(r, 4 + c8) * 16) = lv;
        if (wsplit) {
          const int pix = pix0 + r;
          if (r >= h.halo && r < h.halo + BM && pix < p.P) {
            _Float16* dst = h.xsplit + (size_t)pix * p.Cin + ch * BK2 + c8 * 8;
            *reinterpret_cast<half8*>(dst) = hv;
            *reinterpret_cast<half8*>(dst + xplane) = lv;
          }
        }
      }
    }
  };

  floatx4 acc[TI16][TJ16], part[TI16][TJ16];

  // prologue: the first chunk's halo tile + the first NB - 1 weight stages
#pragma unroll
  for (int k = 0; k < NTK; ++k) load_task(c_beg, k);
#pragma unroll
  for (int s = 0; s < NB - 1; ++s) {
    const int c = c_beg + s / NS;
    issue_b(c < c_end ? c : -1, s % NS, s);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  convert(c_beg);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < TI16; ++i)
#pragma unroll
    for (int j = 0; j < TJ16; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.f;

  int cur = 0;   // ring slot of the current stage
  auto tap_body = [&](const char* b, auto tap_tag) {
    constexpr int TAP = decltype(tap_tag)::value;
    unsigned pk[2] = {apk[TAP][0], apk[TAP][1]};
    asm volatile("" : "+v"(pk[0]), "+v"(pk[1]));   // the fragment addresses are formed here, not hoisted
                                                    // out of the chunk loop (live addresses would spill)
    half8 bh[TJ16], bl[TJ16];
#pragma unroll
    for (int j = 0; j < TJ16; ++j) {
      const int r = wn0 + j * 16 + l16;
      const int o = r * 64 + swzh(r, lq) * 16;
      bh[j] = *reinterpret_cast<const half8*>(b + o);
      bl[j] = *reinterpret_cast<const half8*>(b + BP_BYTES + o);
    }
#pragma unroll
    for (int i = 0; i < TI16; ++i) {
      const int ao = (i % 2 == 0) ? (int)(pk[i / 2] & 0xffffu) : (int)(pk[i / 2] >> 16);
      const half8 ah = *reinterpret_cast<const half8*>(lds + ao);
      const half8 al = *reinterpret_cast<const half8*>(lds + (ao ^ 64));
#pragma unroll
      for (int j = 0; j < TJ16; ++j) {
        floatx4 c0;
        if (TAP == 0)
          c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[j], floatx4{}, 0, 0, 0);
        else
          c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[j], part[i][j], 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[j], c0, 0, 0, 0);
        part[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[j], c0, 0, 0, 0);
      }
      // one row block's A fragments live at a time (the register budget of two workgroups per CU);
      // the other workgroup's waves cover the read latency
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto stage = [&](int ch, auto st_tag) {
    constexpr int ST = decltype(st_tag)::value;
    const bool more = ch + 1 < c_end;
    {   // the ring slot the previous stage read (every wave is past its barrier) gets stage + NB - 1
      constexpr int TGT = ST + NB - 1;
      const int c = ch + TGT / NS;
      issue_b(c < c_end ? c : -1, TGT % NS, cur == 0 ? NB - 1 : cur - 1);
    }
    const char* b = bbuf0 + cur * B_STAGE;
    if (!(SRPDE_CONV_DBG & 128)) {   // diagnostics (SRPDE_CONV_DBG, results wrong): 128 = no MFMA work
      tap_body(b, std::integral_constant<int, ST * TPS>{});
      if constexpr (TPS > 1 && ST * TPS + 1 < 9) tap_body(b + B_TAP, std::integral_constant<int, ST * TPS + 1>{});
      if constexpr (TPS > 2 && ST * TPS + 2 < 9) tap_body(b + 2 * B_TAP, std::integral_constant<int, ST * TPS + 2>{});
    }
    cur = cur == NB - 1 ? 0 : cur + 1;
    if (ST == NS - 1) {
      // two-level accumulation: the chunk's partial chain folds into the accumulator here, so it
      // is dead before the prefetch registers come alive
#pragma unroll
      for (int i = 0; i < TI16; ++i)
#pragma unroll
        for (int j = 0; j < TJ16; ++j) acc[i][j] += part[i][j];
      // the next chunk's halo tile, after the chunk's last fragment reads; the split after the
      // chunk needs it (and every weight stage issued so far) landed
      if (more) {
#pragma unroll
        for (int k = 0; k < NTK; ++k) load_task(ch + 1, k);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      // the next stage's weights must have landed; the NB - 2 stages issued after them may still
      // be in flight (vector-memory loads complete in order)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NB - 2) * DPS) : "memory");
    }
    __syncthreads();
  };
  for (int ch = c_beg; ch < c_end; ++ch) {
    stage(ch, std::integral_constant<int, 0>{});
    if constexpr (NS > 1) stage(ch, std::integral_constant<int, 1>{});
    if constexpr (NS > 2) stage(ch, std::integral_constant<int, 2>{});
    if constexpr (NS > 3) stage(ch, std::integral_constant<int, 3>{});
    if constexpr (NS > 4) stage(ch, std::integral_constant<int, 4>{});
    if constexpr (NS > 5) stage(ch, std::integral_constant<int, 5>{});
    if constexpr (NS > 6) stage(ch, std::integral_constant<int, 6>{});
    if constexpr (NS > 7) stage(ch, std::integral_constant<int, 7>{});
    if constexpr (NS > 8) stage(ch, std::integral_constant<int, 8>{});
    if (ch + 1 < c_end) {   // every wave is past the chunk's last stage barrier: S is free
      if (!(SRPDE_CONV_DBG & 4)) convert(ch + 1);   // diagnostics: 4 = no per-chunk split
      __syncthreads();
    }
  }
  floatx16 acc32[TI][TJ];   // the 32x32x16 accumulator layout of the epilogue
  acc16_to_32<TI, TJ>(acc, acc32);
  float colscale[TJ];
  const float ia = exp2i(-ea);
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int col = n0 + wn0 + j * 32 + lr;
    const int we = col < p.Cout ? h.wexp[col] : 0;
    const int e = ea + we;
    if (e > 126 || e < -126) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc32[i][j][r] *= ia;
      colscale[j] = exp2i(-we);
    } else {
      colscale[j] = exp2i(-e);
    }
    if (col >= p.Cout) colscale[j] = 0.f;
  }
  if (SRPDE_CONV_DBG & 16) {   // diagnostics: 16 = no epilogue (one store per lane keeps the MFMAs live)
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) t += acc32[i][j][0] * colscale[j] + acc32[i][j][15];
    if (t == 123.f) p.y[tid] = t;
    return;
  }
  // S is free now: reduction scratch [2][WM * TI][BN] floats, then 2 KiB per wave of store stage
  x6_finish<BM, BN, WM, WN, SRB>(p, acc32, tail, wg, nfull, piece, m0, n0, wmi, wni, lane, smem,
                                 h.wide ? smem + 2 * WM * TI * BN : nullptr, colscale);
}

// ------------------- weight gradient h3: scaled 2-way fp16 split, 3 MFMA products -------------------
// Same tiling and staging as conv_wgrad_x6 (conv.hip): dW tile [BM couts][BN k-columns] over a
// pixel chunk (split-K), 16 pixels per stage, register-staged pixel rows split into hi / lo
// fp16 images and read back as transposed MFMA fragments (ds_read_b64_tr_b16).
constexpr int BKH = 16;    // pixels per stage

struct H3W {
  const unsigned* ady;   // max|dY| word
  const unsigned* ax0;   // max|x0| word
  const unsigned* ax1;   // max|x1| word (c1 > 0)
};

template <int BM, int BN, int WM, int WN, int HP>
__global__ __launch_bounds__(256, 2) void conv_wgrad_h3_kernel(WgradParams p, H3W sc) {
  constexpr int TM = BM / WM, TN = BN / WN, TI = TM / 32, TJ = TN / 32;
  constexpr int RA = BM * 2, RBB = BN * 2;             // image row bytes (fp16)
  constexpr int IMG_A = BKH * RA, IMG_B = BKH * RBB;    // one plane
  constexpr int STAGE = 2 * (IMG_A + IMG_B);
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
  // operand scales: dY (A) and the forward input (B, both halves of a virtual concat)
  const int ea = h3_exp(*sc.ady);
  unsigned bb = *sc.ax0;
  if (p.c1) bb = max(bb, *sc.ax1);
  const int eb = h3_exp(bb);
  const float sa = exp2i(ea), sb = exp2i(eb);

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

  // image coordinates of each B task's pixel, advanced by BKH pixels per stage (no divisions
  // in the loop; BKH < 2 W for every layer here, W >= 10)
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
      int x = b_x[i] + BKH, y = b_y[i];
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
      half8 h, l;
      split2h(ra[SET][i][0], ra[SET][i][1], sa, h, l);
      const int o = wx_off<RA>(a_row[i], a_col[i] >> 3);
      *reinterpret_cast<half8*>(base + o) = h;
      *reinterpret_cast<half8*>(base + IMG_A + o) = l;
    }
#pragma unroll
    for (int i = 0; i < TB; ++i) {
      if (tid + 256 * i >= 2 * BN) continue;
      half8 h, l;
      split2h(rb[SET][i][0], rb[SET][i][1], sb, h, l);
      const int o = 2 * IMG_A + wx_off<RBB>(b_row[i], b_col[i] >> 3);
      *reinterpret_cast<half8*>(base + o) = h;
      *reinterpret_cast<half8*>(base + IMG_B + o) = l;
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
  const int nsteps = (pend - pbeg + BKH - 1) / BKH;

  // stage s (parity PAR = s & 1 at compile time): LDS buffer PAR holds it
  auto stage = [&](int s, auto fresh_tag, auto par_tag) {
    constexpr bool FRESH = decltype(fresh_tag)::value;
    constexpr int PAR = decltype(par_tag)::value;
    if (s + 2 < nsteps) {
      load_stage(pbeg + (s + 2) * BKH, par_tag);
      advance();
    }
    const char* img = lds + PAR * STAGE;
    half8 ah[TI], al[TI];
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      ah[i] = tr_frag<half8, RA>(img, wm0 + 32 * i, lane);
      al[i] = tr_frag<half8, RA>(img + IMG_A, wm0 + 32 * i, lane);
    }
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const half8 bh = tr_frag<half8, RBB>(img + 2 * IMG_A, wn0 + 32 * j, lane);
      const half8 bl = tr_frag<half8, RBB>(img + 2 * IMG_A + IMG_B, wn0 + 32 * j, lane);
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        floatx16 c0;
        if (FRESH)
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh, floatx16{}, 0, 0, 0);   // small terms first
        else
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh, part[i][j], 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl, c0, 0, 0, 0);
        part[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh, c0, 0, 0, 0);
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
    load_stage(pbeg + BKH, P1{});
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

  // slab [split][Cout][K], scales undone (exact powers of two)
  const float unscale_a = exp2i(-ea), unscale_b = exp2i(-eb);
  float* out = p.part + (size_t)split * p.Cout * p.K;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int n = n0 + wn0 + 32 * j + lr;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < p.Cout && n < p.K) out[(size_t)m * p.K + n] = (acc[i][j][r] * unscale_a) * unscale_b;
      }
    }
}

// ------------- weight gradient h3p: both operands arrive pre-split (fp16 hi / lo planes) -------------
// dW[m][k] = sum_p dY[p][m] * X[p + off(tap(k))][c(k)] as an fp16 GEMM over a pixel chunk (split-K):
// A = dY pieces [2][P][Cout] (stored by the dgrad kernel), B = input pieces [2][P][Cin] (stored by
// the forward kernel), each scaled by its tensor's power of two.  A stage is PS pixel rows of
// both operands' hi and lo planes, DMA'd straight into swizzled LDS images (buffer_load ... lds;
// taps that leave the image and rows past the chunk are zero-filled by the range check), and
// the MFMA fragments come back through ds_read_b64_tr_b16.  A ring of NST stages keeps NST-1
// stages of DMA in flight; every wave issues exactly DPW DMA ops per stage (spare ones go to a
// sink) so the waits are exact vmcnt counts.  No VALU work in the loop.
struct H3P {
  const _Float16* dyp;     // [2][P][Cout]
  const _Float16* xp;      // [2][P][Cin]
  const unsigned* ady;     // max|dY| word (the dgrad split's scale)
  const unsigned* ax0;     // max|x0|, max|x1| words (the forward split's scale)
  const unsigned* ax1;
  // h3h with the fp32 input (srpde_conv_wgrad_h3x): the forward's input transform, repeated where the
  // input rows are staged -- the producing BatchNorm + ReLU of x0 (in_scale / in_shift) and the
  // AttentionGate of x1 (x1_ca [N][c1], x1_sa [P]); null: none
  const float* in_scale;
  const float* in_shift;
  const float* x1_ca;
  const float* x1_sa;
};

// byte offsets (relative to an image base) of the two transposed 4-row reads that give lane
// `lane` its 8 k-values of column col0 + (lane & 31) -- tr_frag's addressing, hoisted out of the loop
template <int RB>
__device__ __forceinline__ int2 tr_offsets(int col0, int lane) {
  const int h = lane >> 5, q = (lane & 15) >> 2, pp = lane & 3;
  const int col = col0 + (lane & 16) + 4 * pp;
  return make_int2(wx_off<RB>(8 * h + q, col >> 3) + 2 * (col & 7), wx_off<RB>(8 * h + 4 + q, col >> 3) + 2 * (col & 7));
}
// the fragment at LDS byte pointers p0 / p1 (a tr_offsets pair added to an image base; compile-time
// parts of the base fold into the instructions' offset fields)
// compiler-visible raw buffer loads (the compiler counts them in its own waits; offsets past the buffer read 0)
__device__ floatx4 h3x_bload4(int32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4f32");
__device__ float h3x_bload1(int32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.f32");
typedef __attribute__((address_space(3))) char lds_char;
__device__ __forceinline__ half8 tr_read(const lds_char* p0, const lds_char* p1) {
  typedef short v4i16 __attribute__((ext_vector_type(4)));
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)p0);
  const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)p1);
  const v8i16 c = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  return __builtin_bit_cast(half8, c);
}

template <int RB>
__device__ __forceinline__ int wx_swz(int row) { return (wx_off<RB>(row, 0) - row * RB) >> 4; }

template <int B, int E, typename F>
__device__ __forceinline__ void h3_for(F&& f) {   // f(integral_constant<B>), ..., f(integral_constant<E - 1>)
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    h3_for<B + 1, E>(f);
  }
}

// timing-only diagnostics of the weight gradient (A/B builds, results wrong when non-zero): 1 = no stage wait /
// barrier, 2 = no DMA in the stage loop (with the DMA, bridge.3's weight gradient took 1.39 ms, without it
// 1.07 ms; issued right after the stage barrier, a stage's 48 DMA wave-instructions held up its first
// MFMAs: spread over the stage's MFMA groups 1.26 ms, tools/gpu/wgrad_variants.sh)
#ifndef H3H_DBG
#define H3H_DBG 0
#endif
#ifndef H3P_DBG
#define H3P_DBG 0
#endif

template <int BM, int BN, int WM, int WN, int PS, int NST, int HP>
__global__ __launch_bounds__(WM * WN * 64, 1) void conv_wgrad_h3p_kernel(WgradParams p, H3P q) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN, TI = TM / 32, TJ = TN / 32;
  constexpr int RA = BM * 2, RBB = BN * 2;              // image row bytes
  constexpr int IMG_A = PS * RA, IMG_B = PS * RBB;       // one plane
  constexpr int STAGE = 2 * (IMG_A + IMG_B);
  constexpr int NA = 2 * IMG_A / 1024, NB = 2 * IMG_B / 1024;   // DMA wave-instructions per stage
  constexpr int DA = (NA + NW - 1) / NW, DB = (NB + NW - 1) / NW, DPW = DA + DB;   // DMA ops per wave per stage
  static_assert(IMG_A % 1024 == 0 && IMG_B % 1024 == 0, "images must be whole KiB");
  static_assert(PS % 16 == 0 && (NST - 2) * DPW <= 63, "stage geometry");
  // (the per-issue coordinate advance wraps at most one image row and one image: PS < H * W)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* lds = reinterpret_cast<char*>(smem);
  char* const sink = lds + NST * STAGE;

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
  const int nsteps = (pend - pbeg + PS - 1) / PS;
  const int kc = p.ksize >> 1;

  const int32x4 rsa = make_rsrc(q.dyp, (unsigned)((size_t)2 * p.P * p.lddy * 2));
  const int32x4 rsb = make_rsrc(q.xp, (unsigned)((size_t)2 * p.P * p.Cin * 2));
  const size_t aplane = (size_t)p.P * p.lddy * 2, bplane = (size_t)p.P * p.Cin * 2;   // bytes

  // this wave's DMA ops: A op j is A instruction wave + j*NW, B op j is B instruction wave + j*NW
  // (past NA / NB: a spare zero-fill into the sink).  LDS destinations are wave-uniform; per lane: a
  // running byte offset (advanced by one stage of pixels per issue) and, for B, the image
  // coordinates of its pixel.
  const int psy = PS / p.W, psx = PS - psy * p.W;       // one stage of pixels in image rows / columns
  const unsigned astep = (unsigned)(PS * p.lddy * 2), bstep = (unsigned)(PS * p.Cin * 2);
  int a_row[DA];
  unsigned a_off[DA];
  bool a_ok[DA];
#pragma unroll
  for (int j = 0; j < DA; ++j) {
    const int w = min(wave + j * NW, NA - 1);
    const int pl = w / (NA / 2), idx = w - pl * (NA / 2);
    const int byte = idx * 1024 + lane * 16;
    const int row = byte / RA, slot = (byte - row * RA) >> 4;
    const int m = m0 + 8 * (slot ^ wx_swz<RA>(row));
    a_row[j] = row;
    a_ok[j] = m < p.Cout && wave + j * NW < NA;
    a_off[j] = (unsigned)(pl * aplane + ((size_t)(pbeg + row) * p.lddy + m) * 2);
  }
  int b_row[DB], b_dy[DB], b_dx[DB], b_y[DB], b_x[DB];
  unsigned b_off[DB];
  bool b_ok[DB];
#pragma unroll
  for (int j = 0; j < DB; ++j) {
    const int w = min(wave + j * NW, NB - 1);
    const int pl = w / (NB / 2), idx = w - pl * (NB / 2);
    const int byte = idx * 1024 + lane * 16;
    const int row = byte / RBB, slot = (byte - row * RBB) >> 4;
    const int k = n0 + 8 * (slot ^ wx_swz<RBB>(row));
    b_row[j] = row;
    b_ok[j] = k < p.K && wave + j * NW < NB;
    const int tap = k < p.K ? k / p.Cin : 0, c = k - tap * p.Cin;
    const int ky = tap / p.ksize, kx = tap - ky * p.ksize;
    b_dy[j] = (ky - kc) * p.dil;
    b_dx[j] = (kx - kc) * p.dil;
    const long long src = (long long)(pbeg + row) + b_dy[j] * p.W + b_dx[j];   // may be < 0 (then unused)
    b_off[j] = (unsigned)((long long)pl * (long long)bplane + (src * p.Cin + c) * 2);
    const int rem = (pbeg + row) % (p.H * p.W);
    b_y[j] = rem / p.W;
    b_x[j] = rem - b_y[j] * p.W;
  }
  // issue stage `s` into ring slot s % NST (always DA + DB ops per wave; past the chunk: zero fill); ops
  // [OLO, OHI) of the wave's A-then-B list (issue_part), all of them (issue)
  auto issue_part = [&](int s, int slot, auto olo_tag, auto ohi_tag) {
    constexpr int OLO = decltype(olo_tag)::value, OHI = decltype(ohi_tag)::value;
    char* st = lds + slot * STAGE;
    const int pbase = pbeg + s * PS;
    const bool full = pbase + PS <= pend;                // wave-uniform: no row of the stage is past the chunk
#pragma unroll
    for (int j = 0; j < DA; ++j) {
      if (j < OLO || j >= OHI) continue;
      const int w = wave + j * NW;
      const int pl = w / (NA / 2), idx = w - pl * (NA / 2);
      const bool in = full || pbase + a_row[j] < pend;
      dma16(rsa, (a_ok[j] && in) ? a_off[j] : OOB, lds_addr_of(w < NA ? st + pl * IMG_A + idx * 1024 : sink));
      a_off[j] += astep;
    }
#pragma unroll
    for (int j = 0; j < DB; ++j) {
      if (DA + j < OLO || DA + j >= OHI) continue;
      const int w = wave + j * NW;
      const int pl = w / (NB / 2), idx = w - pl * (NB / 2);
      const bool ok = b_ok[j] && (full || pbase + b_row[j] < pend) && (unsigned)(b_y[j] + b_dy[j]) < (unsigned)p.H &&
                      (unsigned)(b_x[j] + b_dx[j]) < (unsigned)p.W;
      dma16(rsb, ok ? b_off[j] : OOB, lds_addr_of(w < NB ? st + 2 * IMG_A + pl * IMG_B + idx * 1024 : sink));
      b_off[j] += bstep;
      int x = b_x[j] + psx, y = b_y[j] + psy;   // image coordinates of the next stage's pixel
      if (x >= p.W) { x -= p.W; ++y; }
      if (y >= p.H) y -= p.H;
      b_x[j] = x; b_y[j] = y;
    }
  };
  auto issue = [&](int s, int slot) {
    issue_part(s, slot, std::integral_constant<int, 0>{}, std::integral_constant<int, DPW>{});
  };

  const int ea = h3_exp(*q.ady);
  unsigned xb = *q.ax0;
  if (p.c1) xb = max(xb, *q.ax1);
  const int eb = h3_exp(xb);

  floatx16 acc[TI][TJ], part[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int wm0 = wmi * TM, wn0 = wni * TN;

  int2 oa[TI], ob[TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i) oa[i] = tr_offsets<RA>(wm0 + 32 * i, lane);
#pragma unroll
  for (int j = 0; j < TJ; ++j) ob[j] = tr_offsets<RBB>(wn0 + 32 * j, lane);
#pragma unroll
  for (int s = 0; s < NST - 1; ++s) issue(s, s);
  // stage s lives in ring slot s % NST; the stage loop is unrolled by NST so the slot (and with
  // it every LDS address offset) is a compile-time constant
  auto stage = [&](int s, auto fresh_tag, auto slot_tag) {
    constexpr bool FRESH = decltype(fresh_tag)::value;
    constexpr int SLOT = decltype(slot_tag)::value;
    if constexpr (!(H3P_DBG & 1)) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 2) * DPW) : "memory");
      __syncthreads();
    }
    const lds_char* sb = (const lds_char*)(uintptr_t)lds_addr_of(lds) + SLOT * STAGE;
    const lds_char* va[TI][2];   // this stage's per-lane fragment addresses (+ immediates below)
    const lds_char* vb[TJ][2];
#pragma unroll
    for (int i = 0; i < TI; ++i) { va[i][0] = sb + oa[i].x; va[i][1] = sb + oa[i].y; }
#pragma unroll
    for (int j = 0; j < TJ; ++j) { vb[j][0] = sb + 2 * IMG_A + ob[j].x; vb[j][1] = sb + 2 * IMG_A + ob[j].y; }
#pragma unroll
    for (int kk = 0; kk < PS / 16; ++kk) {
      half8 ah[TI], al[TI];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        ah[i] = tr_read(va[i][0] + kk * 16 * RA, va[i][1] + kk * 16 * RA);
        al[i] = tr_read(va[i][0] + IMG_A + kk * 16 * RA, va[i][1] + IMG_A + kk * 16 * RA);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const half8 bh = tr_read(vb[j][0] + kk * 16 * RBB, vb[j][1] + kk * 16 * RBB);
        const half8 bl = tr_read(vb[j][0] + IMG_B + kk * 16 * RBB, vb[j][1] + IMG_B + kk * 16 * RBB);
        if constexpr (!(H3P_DBG & 2)) {   // stage s + 2's DMA ops, spread over this stage's MFMA groups
          constexpr int NG = (PS / 16) * TJ, PER = (DPW + NG - 1) / NG;
          h3_for<0, PS / 16>([&](auto kk_tag) {
            h3_for<0, TJ>([&](auto j_tag) {
              constexpr int G = decltype(kk_tag)::value * TJ + decltype(j_tag)::value;
              if (kk == decltype(kk_tag)::value && j == decltype(j_tag)::value && G * PER < DPW)
                issue_part(s + NST - 1, (SLOT + NST - 1) % NST, std::integral_constant<int, G * PER>{},
                           std::integral_constant<int, (G + 1) * PER < DPW ? (G + 1) * PER : DPW>{});
            });
          });
        }
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          floatx16 c0;
          if (FRESH && kk == 0)
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh, floatx16{}, 0, 0, 0);   // small terms first
          else
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh, part[i][j], 0, 0, 0);
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl, c0, 0, 0, 0);
          part[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh, c0, 0, 0, 0);
        }
      }
    }
  };
  static_assert(HP == NST && NST == 3, "one partial chain per ring revolution (3 stages)");
  for (int s = 0; s < nsteps; s += 3) {
    stage(s, std::true_type{}, std::integral_constant<int, 0>{});
    if (s + 1 < nsteps) stage(s + 1, std::false_type{}, std::integral_constant<int, 1>{});
    if (s + 2 < nsteps) stage(s + 2, std::false_type{}, std::integral_constant<int, 2>{});
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] += part[i][j];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // spare DMAs land before the workgroup retires

  // slab [split][Cout][K], scales undone (exact powers of two)
  const float ua = exp2i(-ea), ub = exp2i(-eb);
  float* out = p.part + (size_t)split * p.Cout * p.K;
  const int lr = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int n = n0 + wn0 + 32 * j + lr;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < p.Cout && n < p.K) out[(size_t)m * p.K + n] = (acc[i][j][r] * ua) * ub;
      }
    }
}

// ------------- weight gradient h3h: the input operand staged once as a ring of pixel rows -------------
// Same GEMM and operands as h3p (dW[m][tap*Cin + c] = sum_p dY[p][m] X[p + off(tap)][c] from the
// stored fp16 splits), for a tile of BM output channels x one 32-channel input chunk x all nine taps.
// In h3p every 32-channel column group of a tap DMA's its own copy of the shifted input rows, so each
// input element is loaded nine times per pass and the kernel is bound by LDS-DMA issue (~60+ cycles
// per 1 KiB piece, MI355X_MICROARCH.md) at ~0.4 pieces per MFMA.  Here the input chunk lives in LDS
// as a ring of CAP pixel rows (slot = row & (CAP - 1)): each stage DMA's only its PS new rows (the
// rows (W + 1) * dil ahead of the stage), and wave t reads tap t's B fragments at a row shift of
// off(t) = dy * W + dx.  Input rows a tap must not see (it leaves the image: padding, row and image
// wrap) are read from a zero row instead, per lane: each lane addresses one pixel row of the
// transposed read.  Nine waves, one per tap, each a BM x 32 tile.  ~0.11 pieces per MFMA.
//
// XF (srpde_conv_wgrad_h3x): the input rows come from the fp32 activations instead of a stored split,
// so the training forward writes no split planes (4 B per input element).  Two more waves (loaders)
// stage them: each stage's rows are loaded into registers two stages ahead, put through the forward's
// input transform (fused BN + ReLU of x0, attention gate of x1) and split with the forward's scale, and
// written into the ring one stage ahead, before that stage's barrier -- the ring then holds exactly the
// bits the forward's stored split held.  The loaders issue no LDS-DMA, so the compiler's own waits
// count their loads; the MFMA waves DMA only the dY pieces.
template <int BM, int PS, int NST, int CAP, int XF>
__global__ __launch_bounds__(XF ? 704 : 576, 1) void conv_wgrad_h3h_kernel(WgradParams p, H3P q, int cc_n) {
  constexpr int NW = 9, TI = BM / 32;
  constexpr int RA = BM * 2;                   // A image row bytes (one plane)
  constexpr int IMG_A = PS * RA;               // one plane of one stage
  constexpr int NA = 2 * IMG_A / 1024;         // A pieces per stage
  constexpr int NBP = PS / 16;                 // B pieces per plane per stage (16 rows x 64 B)
  constexpr int NB = XF ? 0 : 2 * NBP;
  constexpr int TOT = NA + NB;                 // pieces per stage
  constexpr int DLO = TOT / NW, NHI = TOT % NW;   // waves < NHI issue DLO + 1 pieces per stage
  constexpr int RING = (CAP + 1) * 64;         // one plane of the input ring + its zero row
  static_assert(IMG_A % 1024 == 0 && PS % 16 == 0 && (NST == 3 || NST == 4), "stage geometry");
  static_assert((CAP & (CAP - 1)) == 0 && CAP >= 64, "ring rows: a power of two");
  static_assert((NST - 2) * (DLO + 1) <= 63, "vmcnt range");
  static_assert(!XF || PS == 64, "XF: two loader waves stage 64 rows x 8 channel quads");
  static_assert(XF >= 0 && XF <= 2, "XF: 0 stored split, 1 fp32 input, 2 fp32 input with the gate's loads");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* lds = reinterpret_cast<char*>(smem);
  char* const abuf = lds;                              // [NST][2][PS][RA]
  char* const bring = abuf + NST * 2 * IMG_A;          // [2][CAP][64]
  char* const zrow = bring + CAP * 64;                 // the hi plane's zero row (lo: + RING)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nbm = (p.Cout + BM - 1) / BM;
  const int ntile = nbm * cc_n;
  const int bid = xcd_remap(blockIdx.x, ntile * p.splits);
  const int split = bid / ntile, tile = bid - split * ntile;
  const int mt = tile / cc_n, cc = tile - mt * cc_n;
  const int m0 = mt * BM, c0 = cc * 32;
  const int pbeg = split * p.chunk, pend = min(p.P, pbeg + p.chunk);
  const int nsteps = (pend - pbeg + PS - 1) / PS;
  const int halo = (p.W + 1) * p.dil;
  const int rbase = (pbeg + halo + 15) & ~15;          // first row the stages DMA (16-aligned)
  const int rlo = (pbeg - halo) & ~15;                 // first row of the prologue (may be < 0)

  if (threadIdx.x < 8)
    reinterpret_cast<float4*>(zrow + (threadIdx.x >> 2) * RING)[threadIdx.x & 3] = make_float4(0.f, 0.f, 0.f, 0.f);

  const int32x4 rsa = make_rsrc(q.dyp, (unsigned)((size_t)2 * p.P * p.lddy * 2));
  const int32x4 rsb = make_rsrc(q.xp, (unsigned)((size_t)2 * p.P * p.Cin * 2));
  const unsigned aplane = (unsigned)((size_t)p.P * p.lddy * 2), bplane = (unsigned)((size_t)p.P * p.Cin * 2);

  // B piece of rows [r, r + 16) of plane pl: lane -> row r + lane / 4, 16-B chunk lane % 4
  auto bpiece = [&](int r, int pl) {
    const int row = r + (lane >> 2);
    const unsigned off = (row >= 0 && row < p.P)
                             ? pl * bplane + (unsigned)(((size_t)row * p.Cin + c0 + 8 * (lane & 3)) * 2)
                             : OOB;
    dma16(rsb, off, lds_addr_of(bring + pl * RING + (r & (CAP - 1)) * 64));
  };
  // this wave's pieces of stage s (ring slot SLOT): piece u = wave + j * NW; u < NA: A, else B
  auto issue = [&](int s, int slot) {
    const int p0 = pbeg + s * PS;
    const bool full = p0 + PS <= pend;
#pragma unroll
    for (int j = 0; j < DLO + 1; ++j) {
      const int u = wave + j * NW;
      if (j == DLO && wave >= NHI) break;
      if (u < NA) {
        const int pl = u / (NA / 2), idx = u - pl * (NA / 2);
        const int byte = idx * 1024 + lane * 16;
        const int row = byte / RA, sl = (byte - row * RA) >> 4;
        const int m = m0 + 8 * (sl ^ wx_swz<RA>(row));
        const bool ok = m < p.Cout && (full || p0 + row < pend);
        dma16(rsa, ok ? pl * aplane + (unsigned)(((size_t)(p0 + row) * p.lddy + m) * 2) : OOB,
              lds_addr_of(abuf + (slot * 2 + pl) * IMG_A + idx * 1024));
      } else {
        const int v = u - NA, pl = v / NBP, g = v - pl * NBP;
        bpiece(rbase + s * PS + 16 * g, pl);
      }
    }
  };
  if constexpr (XF) {
    if (wave >= NW) {   // the loader waves: 64 rows x 8 channel quads per stage, 4 rows per lane
      typedef _Float16 half4 __attribute__((ext_vector_type(4)));
      const int lt = tid - NW * 64, qd = lt & 7, rw = lt >> 3;
      const bool second = c0 >= p.c0;
      const float* __restrict__ xs = second ? p.x1 : p.x0;
      const int ld = second ? p.ldx1 : p.ldx0;
      const int cb = (second ? c0 - p.c0 : c0) + 4 * qd;
      const bool aff = !second && q.in_scale != nullptr;
      const bool gate = XF == 2 && second && q.x1_ca != nullptr;
      float4 as = make_float4(1.f, 1.f, 1.f, 1.f), at = make_float4(0.f, 0.f, 0.f, 0.f);
      if (aff) {
        as = *reinterpret_cast<const float4*>(q.in_scale + cb);
        at = *reinterpret_cast<const float4*>(q.in_shift + cb);
      }
      unsigned xw = *q.ax0;
      if (p.c1) xw = max(xw, *q.ax1);
      const float sc = exp2i(h3_exp(xw));
      const int HW = p.H * p.W;
      // buffer loads: a row outside the tensor reads zeros at an out-of-range offset instead of branching, so
      // every stage issues the same loads and the compiler's waits count them exactly (a branch around a load
      // made them all vmcnt(0)); the gate's loads read zeros from an empty buffer where there is no gate
      const int32x4 rsx = make_rsrc(xs, (unsigned)((size_t)p.P * ld * 4));
      const int32x4 rsg = make_rsrc(q.x1_ca, gate ? (unsigned)((size_t)p.N * p.c1 * 4) : 0u);
      const int32x4 rss = make_rsrc(q.x1_sa, gate ? (unsigned)((size_t)p.P * 4) : 0u);
      struct Rows { floatx4 v[4], g[4]; float s[4]; };
      auto load = [&](int R, Rows& b) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = R + rw + 16 * j;
          const bool in = r >= 0 && r < p.P;
          b.v[j] = h3x_bload4(rsx, in ? (int)(((unsigned)r * ld + cb) * 4u) : (int)OOB, 0, 0);
          if constexpr (XF == 2) {   // the gate-capable variant (dec1.conv1)
            b.g[j] = h3x_bload4(rsg, in ? (int)(((unsigned)(r / HW) * p.c1 + cb) * 4u) : (int)OOB, 0, 0);
            b.s[j] = h3x_bload1(rss, in ? r * 4 : (int)OOB, 0, 0);
          }
        }
      };
      // the forward's transform (conv_h5.hip cv_process / gate8n) and split (split2h) of rows < rend
      auto put = [&](int R, const Rows& b, int rend) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = R + rw + 16 * j;
          if (r >= rend) continue;
          float v[4] = {b.v[j][0], b.v[j][1], b.v[j][2], b.v[j][3]};
          if (r >= 0 && r < p.P) {
            if (aff) {
              v[0] = fmaxf(v[0] * as.x + at.x, 0.f); v[1] = fmaxf(v[1] * as.y + at.y, 0.f);
              v[2] = fmaxf(v[2] * as.z + at.z, 0.f); v[3] = fmaxf(v[3] * as.w + at.w, 0.f);
            }
            if (gate) {
              const float s = b.s[j];
              v[0] = (v[0] * b.g[j][0]) * s; v[1] = (v[1] * b.g[j][1]) * s;
              v[2] = (v[2] * b.g[j][2]) * s; v[3] = (v[3] * b.g[j][3]) * s;
            }
          }
          half4 hi, lo;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float xv = v[k] * sc;
            const _Float16 hv = (_Float16)xv;
            hi[k] = hv;
            lo[k] = (_Float16)(xv - (float)hv);
          }
          char* d = bring + (r & (CAP - 1)) * 64 + qd * 8;
          *reinterpret_cast<half4*>(d) = hi;
          *reinterpret_cast<half4*>(d + RING) = lo;
        }
      };
      Rows b0, b1, b2;
      // the rows every stage assumes resident and stage 0's: three groups in flight at once where they fit
      if (rbase + PS - rlo <= 3 * 64) {
        load(rlo, b0);
        load(rlo + 64, b1);
        load(rlo + 128, b2);
        put(rlo, b0, rbase + PS);
        put(rlo + 64, b1, rbase + PS);
        put(rlo + 128, b2, rbase + PS);
      } else {
        for (int R = rlo; R < rbase; R += 64) {
          load(R, b0);
          put(R, b0, rbase);
        }
        load(rbase, b0);
        put(rbase, b0, 0x7fffffff);
      }
      load(rbase + PS, b1);
      load(rbase + 2 * PS, b2);
      // stage s (after its barrier): stage s + 3's loads into the set stage s's rows left, then stage
      // s + 1's rows (loaded two stages ago) into the ring.  Unconditional: past the chunk they load rows
      // nobody reads (or zeros) into ring rows ahead of every stage's reach
      auto step = [&](int s, Rows& tgt, const Rows& src) {
        __syncthreads();
        load(rbase + (s + 3) * PS, tgt);
        put(rbase + (s + 1) * PS, src, 0x7fffffff);
      };
      int s = 0;
      for (; s + 3 <= nsteps; s += 3) {
        step(s, b0, b1);
        step(s + 1, b1, b2);
        step(s + 2, b2, b0);
      }
      if (s < nsteps) step(s, b0, b1);
      if (s + 1 < nsteps) step(s + 1, b1, b2);
      return;
    }
  }
  // prologue: the input rows [rlo, rbase) every later stage assumes resident
  if constexpr (!XF) {
    const int ng = (rbase - rlo) >> 4;
    for (int v = wave; v < 2 * ng; v += NW) bpiece(rlo + 16 * (v >> 1), v & 1);
  }

  const int ea = h3_exp(*q.ady);
  unsigned xb = *q.ax0;
  if (p.c1) xb = max(xb, *q.ax1);
  const int eb = h3_exp(xb);

  floatx16 acc[TI], part[TI];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;

  int2 oa[TI];
#pragma unroll
  for (int i = 0; i < TI; ++i) oa[i] = tr_offsets<RA>(32 * i, lane);
  // this wave's tap and the lane's four pixel rows of a stage (kk, half): image coordinates
  const int ty = wave / 3, tx = wave - 3 * (wave / 3);
  const int dyo = (ty - 1) * p.dil, dxo = (tx - 1) * p.dil;
  const int toff = dyo * p.W + dxo;
  const int colb = 2 * ((lane & 16) + 4 * (lane & 3));
  const int h = lane >> 5, qq = (lane & 15) >> 2;
  const int HW = p.H * p.W;
  const int psy = PS / p.W, psx = PS - psy * p.W;
  int px[NBP][2], py[NBP][2];
#pragma unroll
  for (int kk = 0; kk < NBP; ++kk)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pl = pbeg + 16 * kk + 8 * h + 4 * j + qq;
      const int rem = pl % HW;
      py[kk][j] = rem / p.W;
      px[kk][j] = rem - py[kk][j] * p.W;
    }

#pragma unroll
  for (int s = 0; s < NST - 1; ++s) issue(s, s);
  const unsigned zaddr = lds_addr_of(zrow) + colb;
  const unsigned bbase = lds_addr_of(bring) + colb;
  auto stage = [&](int s, auto fresh_tag, auto slot_tag) {
    constexpr bool FRESH = decltype(fresh_tag)::value;
    constexpr int SLOT = decltype(slot_tag)::value;
    if (wave < NHI) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 2) * (DLO + 1)) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 2) * DLO) : "memory");
    __syncthreads();

    const lds_char* sa = (const lds_char*)(uintptr_t)lds_addr_of(abuf) + SLOT * 2 * IMG_A;
    const int p0 = pbeg + s * PS;
    // fragments of kk + 1 are read while kk's MFMAs run (register double buffer)
    auto bfrag = [&](int kk, half8& bh, half8& bl) {
      // B rows of this lane for tap `wave`: the shifted input row, or the zero row (both planes
      // keep one past the ring, so hi and lo addresses differ by RING either way)
      unsigned ba[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bool ok = (unsigned)(py[kk][j] + dyo) < (unsigned)p.H && (unsigned)(px[kk][j] + dxo) < (unsigned)p.W;
        const int row = p0 + 16 * kk + 8 * h + 4 * j + qq + toff;
        ba[j] = ok ? bbase + (unsigned)((row & (CAP - 1)) * 64) : zaddr;
      }
      bh = tr_read((const lds_char*)(uintptr_t)ba[0], (const lds_char*)(uintptr_t)ba[1]);
      bl = tr_read((const lds_char*)(uintptr_t)(ba[0] + RING), (const lds_char*)(uintptr_t)(ba[1] + RING));
    };
    auto afrag = [&](int kk, half8* ah, half8* al) {
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        ah[i] = tr_read(sa + oa[i].x + kk * 16 * RA, sa + oa[i].y + kk * 16 * RA);
        al[i] = tr_read(sa + IMG_A + oa[i].x + kk * 16 * RA, sa + IMG_A + oa[i].y + kk * 16 * RA);
      }
    };
    // H3H_DBG & 1 (timing diagnostic, wrong results): the last tap's wave issues no MFMAs, leaving eight
    // MFMA waves, two per SIMD
    const bool mskip = (H3H_DBG & 1) && wave == NW - 1;
    half8 bh[2], bl[2], ah[2][TI], al[2][TI];
    bfrag(0, bh[0], bl[0]);
    afrag(0, ah[0], al[0]);
#pragma unroll
    for (int kk = 0; kk < NBP; ++kk) {
      const int cur = kk & 1;
      if (kk + 1 < NBP) {
        bfrag(kk + 1, bh[cur ^ 1], bl[cur ^ 1]);
        afrag(kk + 1, ah[cur ^ 1], al[cur ^ 1]);
      }
#pragma unroll
      for (int i = 0; i < TI && !mskip; ++i) {
        floatx16 c0v;
        if (FRESH && kk == 0)
          c0v = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[cur][i], bh[cur], floatx16{}, 0, 0, 0);   // small terms first
        else
          c0v = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[cur][i], bh[cur], part[i], 0, 0, 0);
        c0v = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[cur][i], bl[cur], c0v, 0, 0, 0);
        part[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[cur][i], bh[cur], c0v, 0, 0, 0);
      }
      if (kk == 0) issue(s + NST - 1, (SLOT + NST - 1) % NST);   // stage s + 2's DMA after the first MFMAs
    }
    // the lane's pixels of the next stage
#pragma unroll
    for (int kk = 0; kk < NBP; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        int x = px[kk][j] + psx, y = py[kk][j] + psy;
        if (x >= p.W) { x -= p.W; ++y; }
        if (y >= p.H) y -= p.H;
        px[kk][j] = x; py[kk][j] = y;
      }
  };
  for (int s = 0; s < nsteps; s += NST) {
    stage(s, std::true_type{}, std::integral_constant<int, 0>{});
    if (s + 1 < nsteps) stage(s + 1, std::false_type{}, std::integral_constant<int, 1>{});
    if (s + 2 < nsteps) stage(s + 2, std::false_type{}, std::integral_constant<int, 2>{});
    if constexpr (NST > 3)
      if (s + 3 < nsteps) stage(s + 3, std::false_type{}, std::integral_constant<int, NST - 1>{});
#pragma unroll
    for (int i = 0; i < TI; ++i) acc[i] += part[i];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // spare DMAs land before the workgroup retires

  // slab [split][Cout][K], k = tap * Cin + c; scales undone (exact powers of two)
  const float ua = exp2i(-ea), ub = exp2i(-eb);
  float* out = p.part + (size_t)split * p.Cout * p.K;
  const int lr = lane & 31, lh = lane >> 5;
  const int n = wave * p.Cin + c0 + lr;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (m < p.Cout) out[(size_t)m * p.K + n] = (acc[i][r] * ua) * ub;
    }
}

// ------------- weight gradient h3g: h3h's input-row ring for 128 output channels per tile -------------
// The deep layers (Cout 128-512 at W = 10 / 20) ran h3p's 256 x 128 / 128 x 256 tiles: one tap per column
// tile, so every tap DMA'd its own shifted copy of the input rows (~0.25 LDS-DMA pieces per MFMA, each ~60
// issue cycles among the MFMAs) and both operands were re-read once per column tile.  Here a tile is 128 output
// channels x one 32-channel input chunk x all nine taps: the input chunk is staged ONCE as h3h's ring of pixel
// rows, and the nine taps read it at row shifts.  Twelve MFMA waves: wave (mi, ty) owns the 32-row m block mi
// and the three taps of kernel row ty (dx = -dil, 0, +dil), i.e. three 32 x 32 accumulators; per 16-pixel step
// it reads one A fragment pair (dY hi / lo) and three B pairs and issues nine MFMA chains of three products.
// 40 DMA pieces per 64-pixel stage for 432 MFMAs (0.09 per MFMA, h3p 0.25).  Measured (profiles/r06_h3g_ab.txt,
// r06_pmc_h3g.txt): the DMA saving is paid back in issue -- the per-lane tap masks and ring addresses of three taps
// cost 7-8 VALU per MFMA at 164 VGPRs, three waves per SIMD -- so the W = 10 layers stay on h3p (+5-10 % here) and
// h3g takes only the W = 20 shapes whose K leaves h3p's last column tile partly empty.  Same products, same per-stage partial
// chains folded into the accumulator every three stages, same slab layout as h3h: the slabs equal h3p's up to
// the order of the three-stage partial sums.  Out-of-image taps read a zero row per lane (the tap's shift is
// folded into the address, so the lane's address is the shifted row or the zero row).
template <int PS, int NST, int CAP, int W, int DIL>
__global__ __launch_bounds__(768, 1) void conv_wgrad_h3g_kernel(WgradParams p, H3P q, int cc_n) {
  constexpr int BM = 128, NW = 12;
  constexpr int RA = BM * 2;                   // A image row bytes (one plane)
  constexpr int IMG_A = PS * RA;               // one plane of one stage
  constexpr int NA = 2 * IMG_A / 1024;         // A pieces per stage
  constexpr int NBP = PS / 16;                 // B pieces per plane per stage (16 rows x 64 B)
  constexpr int TOT = NA + 2 * NBP;            // pieces per stage (+ the mirror copy of ring rows 0 .. 15)
  constexpr int DLO = TOT / NW, NHI = TOT % NW;   // waves < NHI issue DLO + 1 pieces per stage
  constexpr int NJ = DLO + (NHI ? 1 : 0);
  // ring plane: CAP rows, then rows CAP .. CAP + 15 mirroring rows 0 .. 15 (a lane's row index base + lrow,
  // lrow <= 11, never wraps), then the zero row
  constexpr int RING = (CAP + 17) * 64;
  constexpr int ZROW = CAP + 16;
  constexpr int HALO = (W + 1) * DIL;
  static_assert(IMG_A % 1024 == 0 && PS % 16 == 0 && NST == 3, "stage geometry");
  static_assert((CAP & (CAP - 1)) == 0 && 2 * HALO + 15 + 3 * PS <= CAP, "ring rows: a power of two holding a stage's reach");
  static_assert((NST - 2) * (DLO + 1) <= 62, "vmcnt range");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* lds = reinterpret_cast<char*>(smem);
  char* const abuf = lds;                              // [NST][2][PS][RA]
  char* const bring = abuf + NST * 2 * IMG_A;          // [2][CAP + 17][64]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nbm = (p.Cout + BM - 1) / BM;
  const int ntile = nbm * cc_n;
  const int bid = xcd_remap(blockIdx.x, ntile * p.splits);
  const int split = bid / ntile, tile = bid - split * ntile;
  const int mt = tile / cc_n, cc = tile - mt * cc_n;
  const int m0 = mt * BM, c0 = cc * 32;
  const int pbeg = split * p.chunk, pend = min(p.P, pbeg + p.chunk);
  const int nsteps = (pend - pbeg + PS - 1) / PS;
  const int rbase = (pbeg + HALO + 15) & ~15;          // first row the stages DMA (16-aligned)
  const int rlo = (pbeg - HALO) & ~15;                 // first row of the prologue (may be < 0)

  if (threadIdx.x < 8)
    reinterpret_cast<float4*>(bring + ZROW * 64 + (threadIdx.x >> 2) * RING)[threadIdx.x & 3] =
        make_float4(0.f, 0.f, 0.f, 0.f);

  const int32x4 rsa = make_rsrc(q.dyp, (unsigned)((size_t)2 * p.P * p.lddy * 2));
  const int32x4 rsb = make_rsrc(q.xp, (unsigned)((size_t)2 * p.P * p.Cin * 2));
  const unsigned aplane = (unsigned)((size_t)p.P * p.lddy * 2), bplane = (unsigned)((size_t)p.P * p.Cin * 2);
  const unsigned bring_a = lds_addr_of(bring);

  // B piece of rows [r, r + 16) of plane pl (r 16-aligned): lane -> row r + lane / 4, 16-B chunk lane % 4; the
  // piece landing in ring rows 0 .. 15 goes to the mirror rows as well (one more DMA: the stage waits assume
  // the minimum count per wave, so an extra op only makes them stricter)
  auto bpiece = [&](int r, int pl) {
    const int row = r + (lane >> 2);
    const unsigned off = (row >= 0 && row < p.P)
                             ? pl * bplane + (unsigned)(((size_t)row * p.Cin + c0 + 8 * (lane & 3)) * 2)
                             : OOB;
    const int slot = r & (CAP - 1);
    dma16(rsb, off, bring_a + pl * RING + slot * 64);
    if (slot == 0) dma16(rsb, off, bring_a + pl * RING + CAP * 64);
  };
  // this wave's pieces: piece u = wave + j * NW of every stage; u < NA: A (dY rows), else B (input rows).  The
  // per-lane source offsets advance by one stage of rows per issue (stages are issued in order)
  // (the lane's row / column of an A piece: m beyond Cout and rows past the chunk read zeros)
  auto a_geom = [&](int u, int& row, int& m) {
    const int idx = u - (u / (NA / 2)) * (NA / 2);
    const int byte = idx * 1024 + lane * 16;
    row = byte / RA;
    const int sl = (byte - row * RA) >> 4;
    m = m0 + 8 * (sl ^ wx_swz<RA>(row));
  };
  unsigned a_off[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int u = min(wave + j * NW, NA - 1);
    int row, m;
    a_geom(u, row, m);
    a_off[j] = m < p.Cout ? (u / (NA / 2)) * aplane + (unsigned)(((size_t)(pbeg + row) * p.lddy + m) * 2) : OOB;
  }
  const unsigned astep = (unsigned)(PS * p.lddy * 2);
  auto issue = [&](int s, int slot) {
    const int p0 = pbeg + s * PS;
    const bool full = p0 + PS <= pend;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int u = wave + j * NW;
      if (j == DLO && wave >= NHI) break;
      if (u < NA) {
        const int pl = u / (NA / 2), idx = u - pl * (NA / 2);
        bool ok = a_off[j] < OOB;
        if (!full) {
          int row, m;
          a_geom(u, row, m);
          ok = ok && p0 + row < pend;
        }
        dma16(rsa, ok ? a_off[j] : OOB, lds_addr_of(abuf + (slot * 2 + pl) * IMG_A + idx * 1024));
      } else {
        const int v = u - NA, pl = v / NBP, g = v - pl * NBP;
        bpiece(rbase + s * PS + 16 * g, pl);
      }
      if (a_off[j] < OOB) a_off[j] += astep;
    }
  };
  // prologue: the input rows [rlo, rbase) every later stage assumes resident
  {
    const int ng = (rbase - rlo) >> 4;
    for (int v = wave; v < 2 * ng; v += NW) bpiece(rlo + 16 * (v >> 1), v & 1);
  }

  const int ea = h3_exp(*q.ady);
  unsigned xb = *q.ax0;
  if (p.c1) xb = max(xb, *q.ax1);
  const int eb = h3_exp(xb);

  const int mi = wave & 3, ty = wave >> 2;
  floatx16 acc[3], part[3];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  const int2 oa = tr_offsets<RA>(32 * mi, lane);
  // the lane's pixel rows of a 16-pixel step: 8h + 4j + qq (j = 0, 1: the two transposed 4-row reads)
  const int dyo = (ty - 1) * DIL;
  const int colb = 2 * ((lane & 16) + 4 * (lane & 3));
  const int lrow = 8 * (lane >> 5) + ((lane & 15) >> 2);
  const int HWp = p.H * W;
  const unsigned lane_b = bring_a + (unsigned)(lrow * 64 + colb);   // + the row index base * 64
  const unsigned zaddr = bring_a + (unsigned)(ZROW * 64 + colb);
  int rs0 = pbeg % HWp;   // pixel-in-image of the stage's first pixel (uniform), advanced by PS per stage
  static_assert(PS + 16 * (PS / 16) <= 2 * 100, "one wrap per add (H * W >= 100)");

#pragma unroll
  for (int s = 0; s < NST - 1; ++s) issue(s, s);
  // B row addresses of the lane for the wave's three taps at step (kk, j) of the stage at pixel p0: uniform
  // parts in scalars (the pixel-in-image of p0 + 16 kk + 4 j, the ring index of its shifted rows), per lane the
  // row offset lrow, its wrap into the next image row / image, and the tap masks
  auto baddr = [&](int P0, int R0, unsigned (&ba)[3]) {
    if (R0 >= HWp) R0 -= HWp;                            // uniform: the pixel-in-image of P0
    int r = R0 + lrow;
    r = (int)min((unsigned)r, (unsigned)(r - HWp));      // wrap into the next image
    const int y = r / W, x = r - y * W;
    const bool yok = (unsigned)(y + dyo) < (unsigned)p.H;
    const int ib = __builtin_amdgcn_readfirstlane((P0 + dyo * W - DIL) & (CAP - 1));   // tap 0's row index base
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const bool ok = yok && (t == 1 || (t == 0 ? x >= DIL : x < W - DIL));
      const unsigned a = lane_b + (unsigned)(((ib + t * DIL) & (CAP - 1)) * 64);
      ba[t] = ok ? a : zaddr;
    }
  };
  auto stage = [&](int s, auto fresh_tag, auto slot_tag) {
    constexpr bool FRESH = decltype(fresh_tag)::value;
    constexpr int SLOT = decltype(slot_tag)::value;
    if (wave < NHI) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 2) * (DLO + 1)) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 2) * DLO) : "memory");
    __syncthreads();

    const lds_char* sa = (const lds_char*)(uintptr_t)lds_addr_of(abuf) + SLOT * 2 * IMG_A;
    const int p0 = pbeg + s * PS;
    unsigned ba0[3], ba1[3];
    baddr(p0, rs0, ba0);
    baddr(p0 + 4, rs0 + 4, ba1);
#pragma unroll
    for (int kk = 0; kk < NBP; ++kk) {
      const half8 ah = tr_read(sa + oa.x + kk * 16 * RA, sa + oa.y + kk * 16 * RA);
      const half8 al = tr_read(sa + IMG_A + oa.x + kk * 16 * RA, sa + IMG_A + oa.y + kk * 16 * RA);
      half8 bh[3], bl[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        bh[t] = tr_read((const lds_char*)(uintptr_t)ba0[t], (const lds_char*)(uintptr_t)ba1[t]);
        bl[t] = tr_read((const lds_char*)(uintptr_t)ba0[t] + RING, (const lds_char*)(uintptr_t)ba1[t] + RING);
      }
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        floatx16 c0v;
        if (FRESH && kk == 0)
          c0v = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[t], floatx16{}, 0, 0, 0);   // small terms first
        else
          c0v = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[t], part[t], 0, 0, 0);
        c0v = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[t], c0v, 0, 0, 0);
        part[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[t], c0v, 0, 0, 0);
      }
      if (kk + 1 < NBP) {   // the next step's addresses (VALU beside this step's MFMAs)
        baddr(p0 + 16 * (kk + 1), rs0 + 16 * (kk + 1), ba0);
        baddr(p0 + 16 * (kk + 1) + 4, rs0 + 16 * (kk + 1) + 4, ba1);
      }
      if (kk == 0) issue(s + NST - 1, (SLOT + NST - 1) % NST);   // stage s + 2's DMA after the first MFMAs
    }
    rs0 += PS;
    if (rs0 >= HWp) rs0 -= HWp;
  };
  for (int s = 0; s < nsteps; s += NST) {
    stage(s, std::true_type{}, std::integral_constant<int, 0>{});
    if (s + 1 < nsteps) stage(s + 1, std::false_type{}, std::integral_constant<int, 1>{});
    if (s + 2 < nsteps) stage(s + 2, std::false_type{}, std::integral_constant<int, 2>{});
#pragma unroll
    for (int t = 0; t < 3; ++t) acc[t] += part[t];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // spare DMAs land before the workgroup retires

  // slab [split][Cout][K], k = tap * Cin + c; scales undone (exact powers of two)
  const float ua = exp2i(-ea), ub = exp2i(-eb);
  float* out = p.part + (size_t)split * p.Cout * p.K;
  const int lr = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int n = (3 * ty + t) * p.Cin + c0 + lr;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + 32 * mi + (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (m < p.Cout) out[(size_t)m * p.K + n] = (acc[t][r] * ua) * ub;
    }
  }
}

// fp32 packed weights [rows][K] -> fp16 hi / lo planes [2][rows][K] with a power-of-two scale
// per row (one wave per row)
__global__ __launch_bounds__(256) void split_weights_h3_kernel(const float* __restrict__ w, _Float16* __restrict__ out,
                                                               int* __restrict__ wexp, int rows, int K) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* src = w + (size_t)row * K;
  float m = 0.f;
  for (int k = lane; k < K; k += 64) m = fmaxf(m, fabsf(src[k]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  const int e = h3_exp(__float_as_uint(m));
  const float s = exp2i(e);
  _Float16* hi = out + (size_t)row * K;
  _Float16* lo = out + (size_t)rows * K + (size_t)row * K;
  for (int k = lane; k < K; k += 64) {
    const float v = src[k] * s;
    const _Float16 hv = (_Float16)v;
    hi[k] = hv;
    lo[k] = (_Float16)(v - (float)hv);
  }
  if (lane == 0) wexp[row] = e;
}

// All conv layers' h3 weight planes in one launch, straight from torch's [Cout][Cin][3][3]:
// forward rows  n in [0, Cout):   k = tap*Cin_pad + c  ->  W[n][c][tap]   (c >= Cin_real: 0)
// dgrad rows    c in [0, Cin_pad): k = tap*Cout + n    ->  W[n][c][tap]
// one wave per row: max|row| -> power-of-two scale -> hi / lo fp16 planes.  desc (device int64,
// H3W_DESC per layer): w, cout, cin_real, cin_pad, planes_f, exp_f, planes_d, exp_d, row_begin,
// cout_pad (rows of a layer: Cout forward rows then Cin_pad dgrad rows; planes_f / planes_d may be 0;
// dgrad rows hold k = tap*cout_pad + n, zero for n >= cout: out_conv2's 16 channels as a 32-channel
// dgrad input, matching srpde_bn_bwd_apply_split's padded planes).
constexpr int H3W_DESC = 10;
constexpr int H3W_TMAX = 512;   // dgrad rows of layers with cout <= this stage their source through LDS

__global__ __launch_bounds__(256) void prepare_weights_h3_kernel(const long long* __restrict__ desc, int nlayers,
                                                                 int total_rows) {
  __shared__ float T[H3W_TMAX * 37];   // a block's 4 rows' sources (the staged paths below)
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= total_rows) return;
  int l = 0;
  while (l + 1 < nlayers && desc[(l + 1) * H3W_DESC + 8] <= row) ++l;
  const long long* d = desc + l * H3W_DESC;
  const float* w = reinterpret_cast<const float*>(d[0]);
  const int cout = (int)d[1], cin_real = (int)d[2], cin_pad = (int)d[3], cout_pad = (int)d[9];
  int r = row - (int)d[8];
  const bool fwd = r < cout;
  if (!fwd) r -= cout;
  _Float16* planes = reinterpret_cast<_Float16*>(fwd ? d[4] : d[6]);
  int* wexp = reinterpret_cast<int*>(fwd ? d[5] : d[7]);
  if (planes == nullptr) return;   // uniform over the block: its 4 rows are of one layer and kind
  const int inner = fwd ? cin_pad : cout_pad;      // k = tap * inner + i
  const int K = 9 * inner;
  const int rows = fwd ? cout : cin_pad;
  if (fwd && 4 * cin_real * 9 <= H3W_TMAX * 37 && cin_pad % 8 == 0) {
    // forward rows n0..n0+3: their sources are 4 * cin_real * 9 contiguous floats, staged once
    const int n0 = r - (threadIdx.x >> 6), span = cin_real * 9;
    const float* src = w + (size_t)n0 * span;
    for (int e = threadIdx.x; e < 4 * span; e += 256) T[e] = src[e];
    __syncthreads();
    const float* t = T + (threadIdx.x >> 6) * span;
    // max |w| over the staged source itself (the zero padding adds nothing): no per-element division
    float m = 0.f;
    for (int k = lane; k < span; k += 64) m = fmaxf(m, fabsf(t[k]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    const int e = h3_exp(__float_as_uint(m));
    const float sc = exp2i(e);
    _Float16* hi = planes + (size_t)r * K;
    _Float16* lo = planes + (size_t)rows * K + (size_t)r * K;
    for (int k0 = lane * 8; k0 < K; k0 += 512) {   // 8 consecutive k of one tap per lane (cin_pad % 8 == 0)
      const int tap = k0 / cin_pad, c0 = k0 - tap * cin_pad;
      half8 hv, lv;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float x = (c0 + i < cin_real ? t[(c0 + i) * 9 + tap] : 0.f) * sc;
        const _Float16 h = (_Float16)x;
        hv[i] = h;
        lv[i] = (_Float16)(x - (float)h);
      }
      *reinterpret_cast<half8*>(hi + k0) = hv;
      *reinterpret_cast<half8*>(lo + k0) = lv;
    }
    if (lane == 0) wexp[r] = e;
    return;
  }
  if (!fwd && cout_pad <= H3W_TMAX) {
    // dgrad rows c0..c0+3 of this block: the source W[n][c0..c0+3][0..8] is 36 contiguous floats
    // per n -- staged through LDS once by the block, so HBM / L2 reads are row-contiguous (a wave
    // walking k = tap * cout + n directly reads one scattered 4-B word per cache line, 18 times)
    const int c0 = r - (threadIdx.x >> 6);
    for (int e = threadIdx.x; e < cout_pad * 36; e += 256) {
      const int n = e / 36, q = e - n * 36;
      T[n * 37 + q] = (n < cout && c0 + q / 9 < cin_real) ? w[((size_t)n * cin_real + c0) * 9 + q] : 0.f;
    }
    __syncthreads();
    const int cq = (threadIdx.x >> 6) * 9;   // this wave's row within the staged columns
    float m = 0.f;
    for (int n = lane; n < cout_pad; n += 64)
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) m = fmaxf(m, fabsf(T[n * 37 + cq + tap]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    const int e = h3_exp(__float_as_uint(m));
    const float sc = exp2i(e);
    _Float16* hi = planes + (size_t)r * K;
    _Float16* lo = planes + (size_t)rows * K + (size_t)r * K;
    for (int k0 = lane * 8; k0 < K; k0 += 512) {   // 8 consecutive k (same tap: cout_pad % 8 == 0) per lane
      const int tap = k0 / cout_pad, n = k0 - tap * cout_pad;
      half8 hv, lv;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float v = T[(n + i) * 37 + cq + tap] * sc;
        const _Float16 h = (_Float16)v;
        hv[i] = h;
        lv[i] = (_Float16)(v - (float)h);
      }
      *reinterpret_cast<half8*>(hi + k0) = hv;
      *reinterpret_cast<half8*>(lo + k0) = lv;
    }
    if (lane == 0) wexp[r] = e;
    return;
  }
  auto val = [&](int k) -> float {
    const int tap = k / inner, i = k - tap * inner;
    const int n = fwd ? r : i, c = fwd ? i : r;
    return (c < cin_real && n < cout) ? w[((size_t)n * cin_real + c) * 9 + tap] : 0.f;
  };
  float m = 0.f;
  for (int k = lane; k < K; k += 64) m = fmaxf(m, fabsf(val(k)));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  const int e = h3_exp(__float_as_uint(m));
  const float sc = exp2i(e);
  _Float16* hi = planes + (size_t)r * K;
  _Float16* lo = planes + (size_t)rows * K + (size_t)r * K;
  for (int k = lane; k < K; k += 64) {
    const float v = val(k) * sc;
    const _Float16 hv = (_Float16)v;
    hi[k] = hv;
    lo[k] = (_Float16)(v - (float)hv);
  }
  if (lane == 0) wexp[r] = e;
}

// *amax = max(*amax, max|x|) over a [P][c] view (float bits; caller zeroes *amax)
__global__ __launch_bounds__(256) void absmax_kernel(const float* __restrict__ x, int ldx, int c, long long P,
                                                     unsigned* amax) {
  const int c4 = c >> 2;
  const long long total = P * c4;
  float m = 0.f;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const long long r = e / c4;
    const float4 v = *reinterpret_cast<const float4*>(x + r * ldx + (e - r * c4) * 4);
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  __shared__ float wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(amax, __float_as_uint(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]))));
}

// ---------------------------------- host side ---------------------------------------
// tile configs: 1 = 256x128, 2 = 256x64, 3 = 256x32.  (A 256x256 single-level tile with a 4x2
// wave grid measured no faster on bridge.3 -- 1.194 vs 1.197 ms -- at 3x the fp32 summation
// error, so every config keeps the two-level accumulation.)
static int h3_cfg(int cout) { return cout % 128 == 0 ? 1 : (cout % 64 == 0 ? 2 : 3); }
static int h3_bn(int cfg) { return cfg == 1 ? 128 : cfg == 2 ? 64 : 32; }
constexpr int H3_BM = 256;
// rows per BatchNorm-statistics block of every h3 forward launch (srpde_conv_h3_stats_rows)
constexpr int H3_SRB = 128;

static int h3_arows(int w, int dil, int bm = H3_BM) { return (bm + 2 * (w + 1) * dil + 7) / 8 * 8; }

static size_t h3_lds(int bn, int arows, int tps = 1, bool bnb = false, bool pre = false) {
  if (pre) return (size_t)2 * (arows + 1) * 128 + (size_t)2 * tps * 2 * bn * 64 + 1024;
  return (size_t)arows * ((bnb ? 2 : 1) * ROW2 + 128) + (size_t)2 * tps * 2 * bn * 64 + 128 + 1024;
}
// taps per stage: two when the weight double-buffer fits in LDS (three measured within noise)
static int h3_tps(int bn, int arows, bool pre = false) {
  int t = 2;
  while (t > 1 && h3_lds(bn, arows, t, false, pre) > 160 * 1024) --t;
  return t;
}

template <int BM, int BN, int WM, int WN, int SRB, bool TWO_LEVEL, int TPS, bool BNB = false, bool PRE = false>
static int launch_fwd_h3(ConvParams p, H3Args h, hipStream_t st, void* ws, size_t ws_bytes) {
  constexpr int NT = WM * WN * 64;
  const int nbm = ceil_div(p.P, BM), nbn = ceil_div(p.Cout, BN);
  const int T = nbm * nbn;
  const size_t lds = h3_lds(BN, h.arows, TPS, BNB, PRE);
  if ((size_t)h.arows * ROW2 < (size_t)(2 * WM * BN + WM * WN * 512) * 4) h.wide = 0;   // F too small to stage
  static const int cus = [] {
    int dev = 0, c = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    return std::max(1, c);
  }();
  // resident workgroups: by waves (8 per CU) and by LDS
  const int slots = cus * std::max(1, std::min(8 / (WM * WN), (int)((160 * 1024) / lds)));
  plan_tail(p, T, slots, BM, BN, ws, ws_bytes);
  const int nch = p.Cin / BK2;
  if (p.ntail > 0 && p.tsplit > nch) p.tsplit = nch;   // pieces are whole channel chunks
  if (p.tsplit < 2) { p.ntail = 0; p.tsplit = 1; }
  const int grid = T - p.ntail + p.ntail * p.tsplit;
  note_kernel("conv_fwd_h3_kernel<%d, %d, %d, %d, %d, %s, %d, %s, %s>", BM, BN, WM, WN, SRB, TWO_LEVEL ? "true" : "false",
              TPS, BNB ? "true" : "false", PRE ? "true" : "false");
  hipLaunchKernelGGL((conv_fwd_h3_kernel<BM, BN, WM, WN, SRB, TWO_LEVEL, TPS, BNB, PRE>), dim3(grid), dim3(NT), lds, st,
                     p, h);
  SRPDE_LAUNCH_CHECK("srpde_conv_fwd_h3");
  if (p.ntail > 0) return launch_tail_fixup<BM, BN, SRB>(p, st);
  return 0;
}

// h3r (register-staged halo, two workgroups per CU): LDS = S + two weight stages + the zero row
constexpr int H3R_NTK = 6;   // halo tasks per thread: arows <= 6 * 256 / 4 = 384
constexpr int H3R_NB = 4;    // weight ring depth (stages of one tap)
static size_t h3r_lds(int bn, int arows, int tps) {   // zero row | S | weight ring | DMA sink
  return 128 + (size_t)arows * 128 + (size_t)H3R_NB * tps * 2 * bn * 64 + 1024;
}
static int h3r_tps(int bn) { (void)bn; return 1; }
// the h3r kernel takes this shape: an output tile of <= 64 channels, a halo tile that fits the
// registers, and two workgroups' LDS per CU
static bool h3r_fits(int bn, int arows, int fam) {
  return !(fam & FAM_NO_H3R) && bn <= 64 && arows <= H3R_NTK * 256 / 4 && 2 * h3r_lds(bn, arows, h3r_tps(bn)) <= 160 * 1024;
}

template <int BN, int TPS, bool PRE = false>
static int launch_fwd_h3r(ConvParams p, H3Args h, hipStream_t st, void* ws, size_t ws_bytes) {
  constexpr int BM = 256, WM = 4, SRB = 128;
  const int nbm = ceil_div(p.P, BM), nbn = ceil_div(p.Cout, BN);
  const int T = nbm * nbn;
  const size_t lds = h3r_lds(BN, h.arows, TPS);
  if ((size_t)h.arows * 128 < (size_t)(2 * WM * 2 * BN + WM * 512) * 4) h.wide = 0;   // S too small to stage
  static int slots = [&] {
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return std::max(1, cus) * 2;   // resident workgroups: two per CU
  }();
  plan_tail(p, T, slots, BM, BN, ws, ws_bytes);
  const int nch = p.Cin / BK2;
  if (p.ntail > 0 && p.tsplit > nch) p.tsplit = nch;
  if (p.tsplit < 2) { p.ntail = 0; p.tsplit = 1; }
  const int grid = T - p.ntail + p.ntail * p.tsplit;
  note_kernel("conv_fwd_h3r_kernel<%d, %d, %d, %d, %s>", BN, TPS, H3R_NTK, H3R_NB, PRE ? "true" : "false");
  hipLaunchKernelGGL((conv_fwd_h3r_kernel<BN, TPS, H3R_NTK, H3R_NB, PRE>), dim3(grid), dim3(256), lds, st, p, h);
  SRPDE_LAUNCH_CHECK("srpde_conv_fwd_h3(h3r)");
  if (p.ntail > 0) return launch_tail_fixup<BM, BN, SRB>(p, st);
  return 0;
}

int launch_wgrad_h3(const WgradParams& p, const unsigned* amax_dy, const unsigned* amax0, const unsigned* amax1,
                    hipStream_t st) {
  const H3W sc{amax_dy, amax0, p.c1 ? amax1 : amax0};
  const int nb = ceil_div(p.Cout, p.Cout >= 128 ? 128 : (p.Cout >= 64 ? 64 : 32)) *
                 ceil_div(p.K, p.Cout >= 128 ? 128 : 256) * p.splits;
  if (p.Cout >= 128) {
    note_kernel("conv_wgrad_h3_kernel<128, 128, 2, 2, 4>");
    hipLaunchKernelGGL((conv_wgrad_h3_kernel<128, 128, 2, 2, 4>), dim3(nb), dim3(256), (size_t)2 * 2 * BKH * 2 * (128 + 128), st, p, sc);
  } else if (p.Cout >= 64) {
    note_kernel("conv_wgrad_h3_kernel<64, 256, 1, 4, 4>");
    hipLaunchKernelGGL((conv_wgrad_h3_kernel<64, 256, 1, 4, 4>), dim3(nb), dim3(256), (size_t)2 * 2 * BKH * 2 * (64 + 256), st, p, sc);
  } else {
    note_kernel("conv_wgrad_h3_kernel<32, 256, 1, 4, 4>");
    hipLaunchKernelGGL((conv_wgrad_h3_kernel<32, 256, 1, 4, 4>), dim3(nb), dim3(256), (size_t)2 * 2 * BKH * 2 * (32 + 256), st, p, sc);
  }
  SRPDE_LAUNCH_CHECK("srpde_conv_wgrad_h3");
  return 0;
}

// h3p tiles: Cout >= 256: 256x128 (4x2 waves); 128: 128x256 (2x4); 64: 64x256 (1x8); 32: 32x256 (1x8)
// (192-column tiles with 6 waves for K = 576 / 1728 / 3456, which avoid a partly empty last
// 256-column tile, measured slower on every layer: the waves' efficiency loss outweighs the waste)

// Cout <= 64 with K a multiple of 288 (nine taps of 32 channels: K = 576, 1728): 288-column tiles
// of nine 64x32 / 32x32 wave tiles, so no column tile is partly empty (K = 576 filled 2.25 of three
// 256-column tiles)
static bool h3p_use288(int cout, int K) {
  return cout <= 64 && K % 288 == 0;
}

static void h3p_tiles(int cout, int K, int* bm, int* bn) {
  if (cout >= 256) { *bm = 256; *bn = 128; }
  else if (cout >= 128) { *bm = 128; *bn = 256; }
  else if (cout >= 64) { *bm = 64; *bn = h3p_use288(cout, K) ? 288 : 256; }
  else { *bm = 32; *bn = h3p_use288(cout, K) ? 288 : 256; }
}

// h3g (the input-row ring for 128-channel m tiles) takes the W = 20 layers with 128 output channels and at most
// 128 input channels (enc2.conv1, enc2.conv2, dec2.conv2), whose K = 9 Cin leaves h3p's last 256-column tile
// partly empty; against h3p on the same box (profiles/r06_h3g_ab.txt): enc2.conv1 -16 %, enc2.conv2 -1 %,
// dec2.conv2 -3 %, but dec2.conv1 (Cin 384) +2 % and the W = 10 layers +5-10 % (12 waves at 164 VGPRs issue
// 7-8 VALU per MFMA for the per-lane tap masks, against h3p's 4.5 for its DMA bookkeeping), so those keep h3p
constexpr int H3G_PS = 64, H3G_CAP = 256;
static bool h3g_ok(int cout, int K, int cin, int w, int dil) {
  return cout == 128 && w == 20 && dil == 1 && cin <= 128 && K == 9 * cin && cin % 32 == 0;
}

void h3p_split(int P, int cout, int K, int w, int* chunk, int* splits) {
  int bm, bn;
  h3p_tiles(cout, K, &bm, &bn);
  const bool g = h3g_ok(cout, K, K / 9, w, 1);
  if (g) { bm = 128; bn = 288; }
  const long long tiles = (long long)ceil_div(cout, bm) * ceil_div(K, bn);
  // one workgroup per CU (LDS): ~2 rounds of 256 CUs, chunks a multiple of the 32-pixel stage.
  // The weight gradients run on a side stream next to the dgrad chain; half the workgroups of the
  // earlier 4-round target leave CUs to the critical path and halve the split-K reduction
  // (step 34.94 / 35.06 -> 34.56 / 34.59 ms same box; 256 the same, 128: 37.1 ms).
  constexpr long long target = 512;
  const long long want = std::max(1LL, target / tiles);
  long long c = (P + want - 1) / want;
  c = g ? (c + 63) / 64 * 64 : (c + 31) / 32 * 32;
  if (c < 256) c = 256;
  *chunk = (int)c;
  *splits = ceil_div(P, c);
}

// h3h: the input-row-ring weight gradient for the 288-column shapes (one 32-channel input chunk x
// nine taps per tile, the same tiles and split-K slabs as h3p's 288-column kernel) whose ring of
// H3H_CAP rows holds a stage's reach: 3 stages of H3H_PS rows + 2 (W + 1) dil + alignment.
// pixels per stage and ring rows (measured: 32-pixel stages 3-10% slower; a fourth ring stage of
// 32 or 64 pixels within 1-2%)
constexpr int H3H_PS = 64, H3H_CAP = 512;
// (Cout >= 128 would need 9 waves x 128 x 32 accumulators with the two-level chain: 168 VGPRs
// and 312 B of spill scratch at three waves per SIMD -- not built; those layers keep h3p)
static bool h3h_ok(int cout, int K, int cin, int w, int dil) {
  return h3p_use288(cout, K) && K == 9 * cin && cin % 32 == 0 && 2 * (w + 1) * dil + 15 + 3 * H3H_PS <= H3H_CAP;
}

template <int BM, int PS, int NST, int CAP, int XF>
static int launch_h3h_cfg(const WgradParams& p, const H3P& q, hipStream_t st) {
  const int cc_n = p.Cin / 32;
  const int nb = ceil_div(p.Cout, BM) * cc_n * p.splits;
  const size_t lds = (size_t)NST * 2 * PS * BM * 2 + (size_t)2 * (CAP + 1) * 64;
  note_kernel("conv_wgrad_h3h_kernel<%d, %d, %d, %d, %d>", BM, PS, NST, CAP, XF);
  hipLaunchKernelGGL((conv_wgrad_h3h_kernel<BM, PS, NST, CAP, XF>), dim3(nb), dim3(XF ? 704 : 576), lds, st, p, q,
                     cc_n);
  SRPDE_LAUNCH_CHECK(XF ? "srpde_conv_wgrad_h3x" : "srpde_conv_wgrad_h3p(h3h)");
  return 0;
}
template <int BM, int XF = 0>
static int launch_h3h(const WgradParams& p, const H3P& q, hipStream_t st) {
  return launch_h3h_cfg<BM, H3H_PS, 3, H3H_CAP, XF>(p, q, st);
}

template <int W, int DIL>
static int launch_h3g(const WgradParams& p, const H3P& q, hipStream_t st) {
  constexpr int PS = H3G_PS, NST = 3, CAP = H3G_CAP;
  const int cc_n = p.Cin / 32;
  const int nb = ceil_div(p.Cout, 128) * cc_n * p.splits;
  const size_t lds = (size_t)NST * 2 * PS * 128 * 2 + (size_t)2 * (CAP + 17) * 64;
  note_kernel("conv_wgrad_h3g_kernel<%d, %d, %d, %d, %d>", PS, NST, CAP, W, DIL);
  hipLaunchKernelGGL((conv_wgrad_h3g_kernel<PS, NST, CAP, W, DIL>), dim3(nb), dim3(768), lds, st, p, q, cc_n);
  SRPDE_LAUNCH_CHECK("srpde_conv_wgrad_h3p(h3g)");
  return 0;
}

template <int BM, int BN, int WM, int WN>
static int launch_h3p(const WgradParams& p, const H3P& q, hipStream_t st) {
  constexpr int PS = 32, NST = 3;
  const int nb = ceil_div(p.Cout, BM) * ceil_div(p.K, BN) * p.splits;
  const size_t lds = (size_t)NST * 2 * PS * 2 * (BM + BN) + 1024;
  note_kernel("conv_wgrad_h3p_kernel<%d, %d, %d, %d, %d, %d, 3>", BM, BN, WM, WN, PS, NST);
  hipLaunchKernelGGL((conv_wgrad_h3p_kernel<BM, BN, WM, WN, PS, NST, 3>), dim3(nb), dim3(WM * WN * 64), lds, st, p, q);
  SRPDE_LAUNCH_CHECK("srpde_conv_wgrad_h3p");
  return 0;
}

}  // namespace srpde

using namespace srpde;

extern "C" {

size_t srpde_conv_wgrad_h3p_workspace_size(int n, int h, int w, int cout, int cin, int ksize) {
  int chunk, splits;
  h3p_split(n * h * w, cout, ksize * ksize * cin, w, &chunk, &splits);
  return (size_t)splits * cout * ksize * ksize * cin * sizeof(float);
}

int srpde_conv_wgrad_h3p(const void* dyp, const unsigned* amax_dy, const void* xp, int c0, const unsigned* amax0,
                         int c1, const unsigned* amax1, float* dw, int cin_real, int accumulate, int n, int h, int w,
                         int cout, int ksize, int dil, void* workspace, size_t ws_bytes, hipStream_t stream) {
  SRPDE_CHECK_ARG(dyp && xp && dw && workspace && amax_dy && amax0 && (c1 == 0 || amax1),
                  "srpde_conv_wgrad_h3p: null pointer");
  SRPDE_CHECK_ARG(cout % 16 == 0 && (c0 + c1) % 8 == 0 && ksize == 3 && cin_real <= c0 + c1,
                  "srpde_conv_wgrad_h3p: needs cout %% 16 == 0, cin %% 8 == 0, ksize 3 (cout=%d cin=%d)", cout, c0 + c1);
  SRPDE_CHECK_ARG(aligned16(dyp) && aligned16(xp), "srpde_conv_wgrad_h3p: planes must be 16-byte aligned");
  WgradParams p;
  // dyp planes hold cout rounded up to the 32-channel chunk (srpde_bn_bwd_apply_split's padding); rows of
  // dw: cout (the padded rows are zero-filled by the DMA range check, their products never stored)
  p.dy = nullptr; p.lddy = (cout + 31) / 32 * 32; p.x0 = nullptr; p.c0 = c0; p.ldx0 = c0 + c1; p.x1 = nullptr; p.c1 = c1;
  p.ldx1 = c0 + c1;
  p.N = n; p.H = h; p.W = w; p.Cout = cout; p.ksize = ksize; p.dil = dil;
  p.P = n * h * w; p.Cin = c0 + c1; p.K = ksize * ksize * p.Cin;
  // the dy planes' row stride is cout rounded up to 32 (p.lddy): the bound is on that width
  SRPDE_CHECK_ARG(2LL * p.P * std::max(p.lddy, p.Cin) * 2 < (1LL << 31), "srpde_conv_wgrad_h3p: tensor too large");
  h3p_split(p.P, cout, p.K, w, &p.chunk, &p.splits);
  const size_t need = (size_t)p.splits * cout * p.K * sizeof(float);
  if (ws_bytes < need) {
    set_error("srpde_conv_wgrad_h3p: workspace %zu < %zu bytes", ws_bytes, need);
    return kErrWorkspace;
  }
  p.part = static_cast<float*>(workspace);
  const H3P q{static_cast<const _Float16*>(dyp), static_cast<const _Float16*>(xp), amax_dy, amax0, c1 ? amax1 : amax0};
  int rc;
  if (h3g_ok(cout, p.K, p.Cin, w, dil)) rc = launch_h3g<20, 1>(p, q, stream);
  else if (cout >= 256) rc = launch_h3p<256, 128, 4, 2>(p, q, stream);
  else if (cout >= 128) rc = launch_h3p<128, 256, 2, 4>(p, q, stream);
  else if (h3h_ok(cout, p.K, p.Cin, w, dil)) rc = cout >= 64 ? launch_h3h<64>(p, q, stream) : launch_h3h<32>(p, q, stream);
  else if (cout >= 64) rc = h3p_use288(cout, p.K) ? launch_h3p<64, 288, 1, 9>(p, q, stream) : launch_h3p<64, 256, 1, 8>(p, q, stream);
  else rc = h3p_use288(cout, p.K) ? launch_h3p<32, 288, 1, 9>(p, q, stream) : launch_h3p<32, 256, 1, 8>(p, q, stream);
  if (rc) return rc;
  return wgrad_reduce(p.part, dw, p.splits, cout, p.Cin, cin_real, ksize * ksize, accumulate, stream);
}

int srpde_conv_wgrad_h3g_supported(int cout, int cin, int w, int dil) {
  return cout > 0 && cin > 0 && h3g_ok(cout, 9 * cin, cin, w, dil) ? 1 : 0;
}

int srpde_conv_wgrad_h3x_supported(int c0, int c1, int cout, int w, int dil) {
  const int cin = c0 + c1;
  return cout > 0 && cout <= 64 && cout % 16 == 0 && c0 > 0 && c0 % 32 == 0 && c1 % 32 == 0 && dil > 0 &&
         h3h_ok(cout, 9 * cin, cin, w, dil);
}

int srpde_conv_wgrad_h3x(const void* dyp, const unsigned* amax_dy, const float* x0, int ldx0, int c0,
                         const unsigned* amax0, const float* in_scale, const float* in_shift, const float* x1, int ldx1,
                         int c1, const unsigned* amax1, const float* x1_ca, const float* x1_sa, float* dw, int cin_real,
                         int accumulate, int n, int h, int w, int cout, int ksize, int dil, void* workspace,
                         size_t ws_bytes, hipStream_t stream) {
  SRPDE_CHECK_ARG(dyp && amax_dy && x0 && amax0 && dw && workspace && (c1 == 0 || (x1 && amax1)),
                  "srpde_conv_wgrad_h3x: null pointer");
  SRPDE_CHECK_ARG(ksize == 3 && srpde_conv_wgrad_h3x_supported(c0, c1, cout, w, dil) && cin_real <= c0 + c1,
                  "srpde_conv_wgrad_h3x: shape not supported (cout=%d c0=%d c1=%d w=%d dil=%d)", cout, c0, c1, w, dil);
  SRPDE_CHECK_ARG((in_scale == nullptr) == (in_shift == nullptr) && (x1_ca == nullptr) == (x1_sa == nullptr) &&
                      (x1_ca == nullptr || c1 > 0),
                  "srpde_conv_wgrad_h3x: in_scale / in_shift and x1_ca / x1_sa go together (a gate needs x1)");
  SRPDE_CHECK_ARG(aligned16(dyp) && aligned16(x0) && ldx0 % 4 == 0 && ldx0 >= c0 &&
                      (c1 == 0 || (aligned16(x1) && ldx1 % 4 == 0 && ldx1 >= c1)) &&
                      (in_scale == nullptr || (aligned16(in_scale) && aligned16(in_shift))) &&
                      (x1_ca == nullptr || aligned16(x1_ca)),
                  "srpde_conv_wgrad_h3x: 16-byte aligned operands, row strides multiples of 4");
  WgradParams p;
  p.dy = nullptr; p.lddy = (cout + 31) / 32 * 32; p.x0 = x0; p.c0 = c0; p.ldx0 = ldx0; p.x1 = x1; p.c1 = c1;
  p.ldx1 = ldx1;
  p.N = n; p.H = h; p.W = w; p.Cout = cout; p.ksize = ksize; p.dil = dil;
  p.P = n * h * w; p.Cin = c0 + c1; p.K = ksize * ksize * p.Cin;
  SRPDE_CHECK_ARG(2LL * p.P * p.lddy * 2 < (1LL << 31) && (long long)p.P * std::max(ldx0, ldx1) < (1LL << 31),
                  "srpde_conv_wgrad_h3x: tensor too large");
  h3p_split(p.P, cout, p.K, w, &p.chunk, &p.splits);
  const size_t need = (size_t)p.splits * cout * p.K * sizeof(float);
  if (ws_bytes < need) {
    set_error("srpde_conv_wgrad_h3x: workspace %zu < %zu bytes", ws_bytes, need);
    return kErrWorkspace;
  }
  p.part = static_cast<float*>(workspace);
  const H3P q{static_cast<const _Float16*>(dyp), nullptr, amax_dy, amax0, c1 ? amax1 : amax0, in_scale, in_shift,
              x1_ca, x1_sa};
  int rc;
  if (x1_ca != nullptr) rc = cout > 32 ? launch_h3h<64, 2>(p, q, stream) : launch_h3h<32, 2>(p, q, stream);
  else rc = cout > 32 ? launch_h3h<64, 1>(p, q, stream) : launch_h3h<32, 1>(p, q, stream);
  if (rc) return rc;
  return wgrad_reduce(p.part, dw, p.splits, cout, p.Cin, cin_real, ksize * ksize, accumulate, stream);
}

}  // extern "C"

namespace srpde {
}  // namespace srpde

using namespace srpde;

extern "C" {

int srpde_conv_h3_stats_rows(void) { return H3_SRB; }

int srpde_conv_h3_stats_rows_for(int c0, int c1, int cout, int h, int w, int dil, int flags) {
  return !(flags & FAM_NO_H5) && h5_supported(c0, c1, cout, h, w, dil) ? h5_stats_rows() : H3_SRB;
}

int srpde_conv_h3_supported(int c0, int c1, int cout, int w, int dil, int ksize) {
  // cout % 16: a 16-channel output (out_conv2) runs on the 32-column tile with the weight rows past
  // Cout zero-filled by the DMA range check
  if (!(ksize == 3 && c0 % 32 == 0 && c1 % 32 == 0 && cout % 16 == 0 && c0 + c1 > 0 && w > 0 && dil >= 1)) return 0;
  const int bn = h3_bn(h3_cfg(cout));
  const int arows = h3_arows(w, dil);
  return (arows <= 512 && h3_lds(bn, arows) <= 160 * 1024) ? 1 : 0;
}

int srpde_split_weights_h3(const float* w, void* planes, int* wexp, int rows, int K, hipStream_t stream) {
  SRPDE_CHECK_ARG(w && planes && wexp && rows > 0 && K > 0, "srpde_split_weights_h3: bad arguments");
  hipLaunchKernelGGL(split_weights_h3_kernel, dim3(ceil_div(rows, 4)), dim3(256), 0, stream, w,
                     static_cast<_Float16*>(planes), wexp, rows, K);
  SRPDE_LAUNCH_CHECK("srpde_split_weights_h3");
  return 0;
}

int srpde_prepare_weights_h3(const long long* desc, int nlayers, int total_rows, hipStream_t stream) {
  SRPDE_CHECK_ARG(desc && nlayers > 0 && total_rows > 0, "srpde_prepare_weights_h3: bad arguments");
  hipLaunchKernelGGL(prepare_weights_h3_kernel, dim3(ceil_div(total_rows, 4)), dim3(256), 0, stream, desc, nlayers,
                     total_rows);
  SRPDE_LAUNCH_CHECK("srpde_prepare_weights_h3");
  return 0;
}

int srpde_absmax(const float* x, int ldx, int c, long long P, unsigned* amax, hipStream_t stream) {
  SRPDE_CHECK_ARG(x && amax && c % 4 == 0 && ldx % 4 == 0 && aligned16(x), "srpde_absmax: bad arguments");
  if (P <= 0) return 0;
  const long long total = P * (c / 4);
  const int blocks = (int)std::min<long long>((total + 255) / 256, 2048);
  hipLaunchKernelGGL(absmax_kernel, dim3(blocks), dim3(256), 0, stream, x, ldx, c, P, amax);
  SRPDE_LAUNCH_CHECK("srpde_absmax");
  return 0;
}

int srpde_conv_fwd_h3(const float* x0, int c0, int ldx0, const float* x1, int c1, int ldx1, const unsigned* amax0,
                      const unsigned* amax1, const void* wsplit, const int* wexp, const float* bias, float* y, int ldy,
                      int n, int h, int w, int cout, int ksize, int dil, int sign, int accumulate, float* stats,
                      void* xsplit_out, const float* in_scale, const float* in_shift, const float* bn_y,
                      int bn_ldy, const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                      const float* bn_beta, void* bn_part, float* out_max, const float* ep_mean,
                      const float* ep_invstd, const float* ep_gamma, const float* ep_beta, unsigned* ep_amax,
                      const float* x1_ca, const float* x1_sa, const float* x0_up, int up_ld, int up_h, int up_w,
                      void* workspace, size_t ws_bytes, hipStream_t stream) {
  SRPDE_CHECK_ARG((accumulate & ~(1 | FAM_MASK)) == 0, "srpde_conv_fwd_h3: accumulate: bit 0 plus family bits only");
  const int fam = accumulate & FAM_MASK;
  accumulate &= 1;
  const bool h5ok = !(fam & FAM_NO_H5), h4ok = !(fam & FAM_NO_H4);
  SRPDE_CHECK_ARG(x0 && wsplit && wexp && y && amax0, "srpde_conv_fwd_h3: null pointer");
  SRPDE_CHECK_ARG(x0_up == nullptr || (up_h * 2 == h && up_w * 2 == w && up_ld % 4 == 0 && up_ld >= c0 &&
                                       aligned16(x0_up) && in_scale == nullptr && ksize == 3 && sign == 1 &&
                                       h4ok && h4_up_supported(w, dil, cout)),
                  "srpde_conv_fwd_h3: an upsampled x0 (x0_up) needs h = 2 up_h, w = 2 up_w, no in_scale, the forward, "
                  "and a shape the h4 kernel is instantiated for (W 20 / 128 columns, W 40 / 64 columns)");
  SRPDE_CHECK_ARG((x1_ca == nullptr) == (x1_sa == nullptr) && (x1_ca == nullptr || c1 > 0),
                  "srpde_conv_fwd_h3: x1_ca / x1_sa go together and need a second input (c1 > 0)");
  SRPDE_CHECK_ARG(c1 == 0 || (x1 && amax1), "srpde_conv_fwd_h3: x1 / amax1 null with c1>0");
  SRPDE_CHECK_ARG(n > 0 && h > 0 && w > 0 && cout > 0, "srpde_conv_fwd_h3: bad shape");
  SRPDE_CHECK_ARG(sign == 1 || sign == -1, "srpde_conv_fwd_h3: sign must be +-1");
  SRPDE_CHECK_ARG(srpde_conv_h3_supported(c0, c1, cout, w, dil, ksize),
                  "srpde_conv_fwd_h3: unsupported shape (c0=%d c1=%d cout=%d w=%d dil=%d ksize=%d)", c0, c1, cout, w,
                  dil, ksize);
  SRPDE_CHECK_ARG(ldx0 % 4 == 0 && (c1 == 0 || ldx1 % 4 == 0), "srpde_conv_fwd_h3: strides must be multiples of 4");
  SRPDE_CHECK_ARG(aligned16(x0) && aligned16(wsplit) && (c1 == 0 || aligned16(x1)),
                  "srpde_conv_fwd_h3: inputs must be 16-byte aligned");
  ConvParams p;
  p.x0 = x0; p.c0 = c0; p.ldx0 = ldx0;
  p.x1 = x1; p.c1 = c1; p.ldx1 = ldx1 > 0 ? ldx1 : 4;
  p.w = nullptr; p.bias = bias; p.y = y; p.ldy = ldy;
  p.stats = reinterpret_cast<float2*>(stats);
  p.N = n; p.H = h; p.W = w; p.Cout = cout; p.ksize = ksize; p.dil = dil; p.sign = sign; p.accumulate = accumulate;
  p.P = n * h * w; p.Cin = c0 + c1; p.K = ksize * ksize * p.Cin;
  p.ntail = 0; p.tsplit = 1; p.part = nullptr;
  const long long maxld = std::max(ldx0, c1 ? ldx1 : 0);
  SRPDE_CHECK_ARG((long long)p.P * maxld * 4 < (1LL << 31) && 2LL * cout * p.K * 2 < (1LL << 31),
                  "srpde_conv_fwd_h3: tensor too large");
  H3Args a{};
  a.wsp = static_cast<const _Float16*>(wsplit);
  a.wexp = wexp;
  a.amax0 = amax0;
  a.amax1 = c1 ? amax1 : nullptr;
  a.halo = (w + 1) * dil;
  a.arows = h3_arows(w, dil);
  a.relax = 1;   // a stage waits only for its weight DMA; the halo slices land later
  a.xsplit = static_cast<_Float16*>(xsplit_out);
  SRPDE_CHECK_ARG((in_scale == nullptr) == (in_shift == nullptr) && (in_scale == nullptr || c1 == 0),
                  "srpde_conv_fwd_h3: in_scale / in_shift go together and need c1 == 0");
  a.in_scale = in_scale;
  a.in_shift = in_shift;
  a.x1_ca = x1_ca;
  a.x1_sa = x1_sa;
  a.up_src = x0_up;
  a.up_ld = up_ld; a.up_h = up_h; a.up_w = up_w;
  a.wide = ldy % 4 == 0 && aligned16(y);
  SRPDE_CHECK_ARG(bn_part == nullptr || (bn_y && bn_mean && bn_invstd && bn_gamma && bn_beta && !accumulate &&
                                          bn_ldy % 4 == 0 && cout % 4 == 0),
                  "srpde_conv_fwd_h3: the fused BN reduction needs bn_y/mean/invstd/gamma/beta and no accumulate");
  p.bn_y = bn_y; p.bn_ldy = bn_ldy; p.bn_mean = bn_mean; p.bn_invstd = bn_invstd;
  p.bn_gamma = bn_gamma; p.bn_beta = bn_beta; p.bn_part = static_cast<float2*>(bn_part);
  p.out_max = out_max;
  SRPDE_CHECK_ARG(xsplit_out == nullptr || aligned16(xsplit_out), "srpde_conv_fwd_h3: xsplit_out must be 16-byte aligned");
  SRPDE_CHECK_ARG(ep_mean == nullptr || (ep_invstd && ep_gamma && ep_beta && !accumulate && stats == nullptr &&
                                         bn_part == nullptr && cout % 4 == 0),
                  "srpde_conv_fwd_h3: the epilogue BN + ReLU needs mean/invstd/gamma/beta, no accumulate / stats / "
                  "bn_part, cout %% 4 == 0");
  p.ep_mean = ep_mean; p.ep_invstd = ep_invstd; p.ep_gamma = ep_gamma; p.ep_beta = ep_beta;
  p.ep_amax = ep_mean != nullptr ? ep_amax : nullptr;
  // out_conv2's shape in training (32 -> 16, no epilogue BN): the 16-output kernel, 128-row statistics
  if (x0_up == nullptr && sign == 1 && bn_part == nullptr && out_max == nullptr && ep_mean == nullptr && !accumulate &&
      h5ok && n16_supported(c0, c1, cout, w, dil) && ldx0 % 4 == 0 && aligned16(x0))
    return launch_fwd_n16(p, a, stream);
  // h5 takes the forward of the shapes srpde_conv_h3_stats_rows_for reports 80-row statistics for
  if (x0_up == nullptr && sign == 1 && bn_part == nullptr && out_max == nullptr && h5ok &&
      h5_supported(c0, c1, cout, h, w, dil)) {
    if (ldy % 4 == 0 && aligned16(y) && (c1 == 0 || ldx1 % 4 == 0)) return launch_fwd_h5(p, a, stream);
    SRPDE_CHECK_ARG(stats == nullptr, "srpde_conv_fwd_h3: the h5 shape (w=40, cout=%d) needs a 16-byte aligned y "
                    "with ldy %% 4 == 0 when it writes statistics", cout);
  }
  // the eval decoder's dec1.conv1 (upsampled x0, gated x1, BN + ReLU epilogue) at W = 40: h5's UP variant
  if (x0_up != nullptr && sign == 1 && bn_part == nullptr && out_max == nullptr && ep_mean != nullptr &&
      stats == nullptr && x1_ca != nullptr && !accumulate && h5ok && h5_supported(c0, c1, cout, h, w, dil) && ldy % 4 == 0 &&
      aligned16(y) && (c1 == 0 || ldx1 % 4 == 0))
    return launch_fwd_h5(p, a, stream);
  SRPDE_CHECK_ARG(x0_up == nullptr || stats == nullptr || !h5ok || !h5_supported(c0, c1, cout, h, w, dil),
                  "srpde_conv_fwd_h3: an upsampled x0 with statistics at an h5 shape (w=40, cout=%d): the statistics "
                  "blocks would not be the srpde_conv_h3_stats_rows_for ones", cout);
  if (x0_up != nullptr || (h4ok && h4_supported(w, dil, cout, false)))
    return launch_fwd_h4(p, a, false, stream, workspace, ws_bytes);
  if (h3r_fits(h3_bn(h3_cfg(cout)), a.arows, fam)) {
    if (h3_cfg(cout) == 2) return launch_fwd_h3r<64, 1>(p, a, stream, workspace, ws_bytes);
    return launch_fwd_h3r<32, 1>(p, a, stream, workspace, ws_bytes);
  }
  const int tps = h3_tps(h3_bn(h3_cfg(cout)), a.arows);
#define H3_LAUNCH(BN_)                                                                        \
  (tps == 2 ? launch_fwd_h3<256, BN_, 8, 1, H3_SRB, true, 2>(p, a, stream, workspace, ws_bytes) \
            : launch_fwd_h3<256, BN_, 8, 1, H3_SRB, true, 1>(p, a, stream, workspace, ws_bytes))
  switch (h3_cfg(cout)) {
    case 1: return H3_LAUNCH(128);
    case 2: return H3_LAUNCH(64);
    default: return H3_LAUNCH(32);
  }
#undef H3_LAUNCH
}

// srpde_conv_fwd_h3 on an input that arrives as its h3 split (planes [2][P][c] fp16 hi / lo of
// x * 2^h3_exp(*amax), e.g. srpde_bn_bwd_apply_split's dy): the halo tiles are DMA'd / loaded as
// fp16 pieces straight into the MFMA operand layout, no fp32 tile, no split work and nothing to
// store for the weight gradient (which reads the same planes).
int srpde_conv_fwd_h3_presplit(const void* xsplit, int c, const unsigned* amax, const void* wsplit, const int* wexp,
                               const float* bias, float* y, int ldy, int n, int h, int w, int cout, int ksize,
                               int dil, int sign, int accumulate, float* stats, const float* bn_y, int bn_ldy,
                               const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                               const float* bn_beta, void* bn_part, float* out_max, void* workspace, size_t ws_bytes,
                               hipStream_t stream) {
  SRPDE_CHECK_ARG((accumulate & ~(1 | FAM_MASK)) == 0, "srpde_conv_fwd_h3_presplit: accumulate: bit 0 plus family bits");
  const int fam = accumulate & FAM_MASK;
  accumulate &= 1;
  SRPDE_CHECK_ARG(xsplit && amax && wsplit && wexp && y, "srpde_conv_fwd_h3_presplit: null pointer");
  SRPDE_CHECK_ARG(n > 0 && h > 0 && w > 0 && cout > 0 && (sign == 1 || sign == -1), "srpde_conv_fwd_h3_presplit: bad shape");
  SRPDE_CHECK_ARG(srpde_conv_h3_supported(c, 0, cout, w, dil, ksize),
                  "srpde_conv_fwd_h3_presplit: unsupported shape (c=%d cout=%d w=%d dil=%d)", c, cout, w, dil);
  SRPDE_CHECK_ARG(aligned16(xsplit) && aligned16(wsplit), "srpde_conv_fwd_h3_presplit: 16-byte alignment");
  ConvParams p;
  p.x0 = static_cast<const float*>(xsplit); p.c0 = c; p.ldx0 = c;   // [2][P][c] fp16 == P * c floats of bytes
  p.x1 = nullptr; p.c1 = 0; p.ldx1 = 4;
  p.w = nullptr; p.bias = bias; p.y = y; p.ldy = ldy;
  p.stats = reinterpret_cast<float2*>(stats);
  p.N = n; p.H = h; p.W = w; p.Cout = cout; p.ksize = ksize; p.dil = dil; p.sign = sign; p.accumulate = accumulate;
  p.P = n * h * w; p.Cin = c; p.K = ksize * ksize * c;
  p.ntail = 0; p.tsplit = 1; p.part = nullptr;
  SRPDE_CHECK_ARG((long long)p.P * c * 4 < (1LL << 31) && 2LL * cout * p.K * 2 < (1LL << 31),
                  "srpde_conv_fwd_h3_presplit: tensor too large");
  SRPDE_CHECK_ARG(bn_part == nullptr || (bn_y && bn_mean && bn_invstd && bn_gamma && bn_beta && !accumulate &&
                                          bn_ldy % 4 == 0 && cout % 4 == 0),
                  "srpde_conv_fwd_h3_presplit: the fused BN reduction needs bn_y/mean/invstd/gamma/beta, no accumulate");
  p.bn_y = bn_y; p.bn_ldy = bn_ldy; p.bn_mean = bn_mean; p.bn_invstd = bn_invstd;
  p.bn_gamma = bn_gamma; p.bn_beta = bn_beta; p.bn_part = static_cast<float2*>(bn_part);
  p.out_max = out_max;
  H3Args a{};
  a.wsp = static_cast<const _Float16*>(wsplit);
  a.wexp = wexp;
  a.amax0 = amax;
  a.amax1 = nullptr;
  a.halo = (w + 1) * dil;
  a.arows = h3_arows(w, dil);
  a.relax = 1;
  a.xsplit = nullptr;
  a.in_scale = nullptr; a.in_shift = nullptr;
  a.wide = ldy % 4 == 0 && aligned16(y);
  if (!(fam & FAM_NO_H4) && h4_supported(w, dil, cout, false))
    return launch_fwd_h4(p, a, true, stream, workspace, ws_bytes);
  if (h3r_fits(h3_bn(h3_cfg(cout)), a.arows, fam)) {
    if (h3_cfg(cout) == 2) return launch_fwd_h3r<64, 1, true>(p, a, stream, workspace, ws_bytes);
    return launch_fwd_h3r<32, 1, true>(p, a, stream, workspace, ws_bytes);
  }
  const int bn = h3_bn(h3_cfg(cout));
  SRPDE_CHECK_ARG(h3_lds(bn, a.arows, 1, false, true) <= 160 * 1024, "srpde_conv_fwd_h3_presplit: LDS (w=%d dil=%d)", w,
                  dil);
  const int tps = h3_tps(bn, a.arows, true);
#define H3P_LAUNCH(BN_)                                                                                   \
  (tps == 2 ? launch_fwd_h3<256, BN_, 8, 1, H3_SRB, true, 2, false, true>(p, a, stream, workspace, ws_bytes) \
            : launch_fwd_h3<256, BN_, 8, 1, H3_SRB, true, 1, false, true>(p, a, stream, workspace, ws_bytes))
  switch (h3_cfg(cout)) {
    case 1: return H3P_LAUNCH(128);
    case 2: return H3P_LAUNCH(64);
    default: return H3P_LAUNCH(32);
  }
#undef H3P_LAUNCH
}

// dgrad with the BatchNorm (+ReLU) backward apply fused into the operand transform (BNB kernels):
// dx = conv^T(dy) with dy = gamma*invstd*(dz - m1 - xhat*m2) computed per halo element from the
// BN output gradient da and the BN input y (no dy tensor in HBM).  m1 / m2 / the dy operand-scale
// bound come from srpde_bn_bwd_prepare.  Stores dy's split (dysplit_out) for srpde_conv_wgrad_h3p,
// optionally the next BN-backward reduction (bn_* / bn_part) and per-tile max|dx| (dx_max).
int srpde_conv_dgrad_h3_bnb(const float* da, int ldda, const unsigned* dy_amax, const float* bn_y_in, int bn_ldy_in,
                            const float* mean, const float* invstd, const float* gamma, const float* beta,
                            const float* m1, const float* m2, int flags, const void* wsplit, const int* wexp,
                            float* dx, int lddx, int n, int h, int w, int cout_dy, int cin_dx, int dil,
                            void* dysplit_out, const float* bn_y, int bn_ldy, const float* bn_mean,
                            const float* bn_invstd, const float* bn_gamma, const float* bn_beta, void* bn_part,
                            float* dx_max, void* workspace, size_t ws_bytes, hipStream_t stream) {
  SRPDE_CHECK_ARG(da && dy_amax && bn_y_in && mean && invstd && gamma && beta && m1 && m2 && wsplit && wexp && dx &&
                  dysplit_out, "srpde_conv_dgrad_h3_bnb: null pointer");
  SRPDE_CHECK_ARG(n > 0 && h > 0 && w > 0 && cout_dy > 0 && cin_dx > 0, "srpde_conv_dgrad_h3_bnb: bad shape");
  SRPDE_CHECK_ARG(srpde_conv_h3_supported(cout_dy, 0, cin_dx, w, dil, 3),
                  "srpde_conv_dgrad_h3_bnb: unsupported shape (cout_dy=%d cin_dx=%d w=%d dil=%d)", cout_dy, cin_dx, w,
                  dil);
  SRPDE_CHECK_ARG(ldda % 4 == 0 && bn_ldy_in % 4 == 0 && aligned16(da) && aligned16(bn_y_in) && aligned16(wsplit) &&
                  aligned16(dysplit_out), "srpde_conv_dgrad_h3_bnb: 16-byte alignment / ld % 4");
  ConvParams p;
  p.x0 = da; p.c0 = cout_dy; p.ldx0 = ldda;
  p.x1 = nullptr; p.c1 = 0; p.ldx1 = 4;
  p.w = nullptr; p.bias = nullptr; p.y = dx; p.ldy = lddx;
  p.stats = nullptr;
  p.N = n; p.H = h; p.W = w; p.Cout = cin_dx; p.ksize = 3; p.dil = dil; p.sign = -1; p.accumulate = 0;
  p.P = n * h * w; p.Cin = cout_dy; p.K = 9 * p.Cin;
  p.ntail = 0; p.tsplit = 1; p.part = nullptr;
  SRPDE_CHECK_ARG((long long)p.P * std::max(ldda, bn_ldy_in) * 4 < (1LL << 31) && 2LL * cin_dx * p.K * 2 < (1LL << 31),
                  "srpde_conv_dgrad_h3_bnb: tensor too large");
  SRPDE_CHECK_ARG(bn_part == nullptr || (bn_y && bn_mean && bn_invstd && bn_gamma && bn_beta && bn_ldy % 4 == 0 &&
                                          cin_dx % 4 == 0), "srpde_conv_dgrad_h3_bnb: bad fused-reduction arguments");
  p.bn_y = bn_y; p.bn_ldy = bn_ldy; p.bn_mean = bn_mean; p.bn_invstd = bn_invstd;
  p.bn_gamma = bn_gamma; p.bn_beta = bn_beta; p.bn_part = static_cast<float2*>(bn_part);
  p.out_max = dx_max;
  H3Args a{};
  a.wsp = static_cast<const _Float16*>(wsplit);
  a.wexp = wexp;
  a.amax0 = dy_amax;
  a.amax1 = nullptr;
  a.halo = (w + 1) * dil;
  a.arows = h3_arows(w, dil);
  a.relax = 1;
  a.xsplit = static_cast<_Float16*>(dysplit_out);
  a.in_scale = nullptr; a.in_shift = nullptr;
  a.wide = lddx % 4 == 0 && aligned16(dx);
  a.bnb_y = bn_y_in; a.bnb_ldy = bn_ldy_in;
  a.bnb_mean = mean; a.bnb_invstd = invstd; a.bnb_gamma = gamma; a.bnb_beta = beta;
  a.bnb_m1 = m1; a.bnb_m2 = m2;
  a.bnb_relu = flags & 1;
  const int bn = h3_bn(h3_cfg(cin_dx));
  SRPDE_CHECK_ARG(h3_lds(bn, a.arows, 1, true) <= 160 * 1024, "srpde_conv_dgrad_h3_bnb: LDS (w=%d dil=%d)", w, dil);
  SRPDE_CHECK_ARG(h3_cfg(cin_dx) != 1, "srpde_conv_dgrad_h3_bnb: 128-column tiles not provided (cin_dx=%d)", cin_dx);
  // one tap per stage: the second fp32 halo tile takes the second weight stage's LDS.  (The
  // 128-column tile does not fit its registers with the fused transform -- 46 VGPRs of scratch --
  // so outputs with a multiple of 128 channels keep srpde_bn_relu_bwd + srpde_conv_fwd_h3.)
  if (h3_cfg(cin_dx) == 2) return launch_fwd_h3<256, 64, 8, 1, H3_SRB, true, 1, true>(p, a, stream, workspace, ws_bytes);
  return launch_fwd_h3<256, 32, 8, 1, H3_SRB, true, 1, true>(p, a, stream, workspace, ws_bytes);
}

// Number of output tiles (= out_max slots) srpde_conv_fwd_h3 uses for this shape; 0 if unsupported.
long long srpde_conv_h3_tiles(long long P, int cin, int cout, int w, int dil) {
  if (P <= 0 || !srpde_conv_h3_supported(cin, 0, cout, w, dil, 3)) return 0;
  const int bm = H3_BM;
  const int bn = h3_bn(h3_cfg(cout));
  return ((P + bm - 1) / bm) * ((cout + bn - 1) / bn);
}

int srpde_conv_h3_bnb_supported(int cout_dy, int cin_dx, int w, int dil) {
  if (!srpde_conv_h3_supported(cout_dy, 0, cin_dx, w, dil, 3) || h3_cfg(cin_dx) == 1) return 0;
  return h3_lds(h3_bn(h3_cfg(cin_dx)), h3_arows(w, dil), 1, true) <= 160 * 1024 ? 1 : 0;
}

}  // extern "C"
