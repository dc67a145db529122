// "h4": the 256 x 128 (and 256 x 64) implicit-GEMM 3x3 convolution (forward and dgrad) of
// conv_h3.hip (conv_fwd_h3_kernel<256, BN, 8, 1, 128, true, ...>), rebuilt around its main loop so
// the MFMA pipes stay fed.  Instantiated for W = 10 (dilation 1, 2) and 20 with 128- or 64-column
// tiles, and for W = 40 with 64-column tiles (the W = 40 layers took the 4-wave h3r kernel before).  Same arithmetic, fragments, product order, two-level accumulation and
// epilogue as that kernel, so the outputs are bit-identical to it (tests/test_gpu_kernels.py
// ::test_conv_h4_equals_h3); reference calls: nn.Conv2d at src/models.py:16,18,43,46 and their
// autograd convolution_backward (input gradient).
//
// What changed, and why (round 3's phase ablation and instruction counts of the h3 loop,
// DESIGN.md 3.6):
//  * One tap per weight stage in a ring of four slots, filled three taps ahead.  A wave waits
//    for its own DMA of tap tau+1 at the end of tap tau-1, so after that tap's barrier every
//    wave may read tap tau+1's B fragments -- the B fragments of the next tap (and, within a
//    chunk, its A fragments) are read during the current tap's MFMAs, and a wave leaves each
//    barrier with its operands in registers.  (h3: the fragments of each column block were read
//    right before its MFMAs, 16 exposed lgkmcnt waits per tap.)
//  * B fragment pairs are read two column blocks ahead of their MFMAs.
//  * The split halo tile S uses 160-byte rows (no XOR swizzle; 160 B is conflict-free for the
//    16x16x32 A-fragment reads at any row shift, see h4_sr_is_conflict_free in DESIGN), so a tap
//    is a constant row shift: the per-tap A addresses of a lane's two 16-row blocks are
//    precomputed once per tile as two 16-bit offsets per tap (nine VGPRs; out-of-image taps
//    point at a zero row).  W and the dilation are template parameters.
//  * Every DMA's varying part is a per-tile VGPR offset and its per-stage part a uniform SGPR
//    offset (buffer soffset): no address arithmetic or branches around the DMA issue.
//  * PRE (the input arrives as its h3 split, the pre-split dgrad): two S buffers; chunk c+1's
//    pieces are DMA'd in S layout during chunk c, so there is no convert and no stall between
//    chunks.  Otherwise the fp32 halo tile F of chunk c+1 is DMA'd during chunk c and split into S
//    between chunks, as in h3.
#include "conv_h3.h"

namespace srpde {

// 16-B-per-lane LDS-DMA with a uniform byte offset in SGPR soffset (see dma16 in conv_common.h:
// inline asm so the waitcnt pass leaves it alone; M0 = the wave-uniform LDS destination)
__device__ __forceinline__ void dma16s(int32x4 rsrc, unsigned voff, unsigned soff, unsigned lds_addr) {
  asm volatile(
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %0, %1, %2 offen lds"
      :
      : "v"(voff), "s"(rsrc), "s"(__builtin_amdgcn_readfirstlane(soff)), "{m0}"(__builtin_amdgcn_readfirstlane(lds_addr))
      : "memory");
}

// compile-time loop: f(integral_constant<int, I>) for I = B .. E-1
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

template <int W, int DIL, int BN_>
struct H4Geom {
  static constexpr int BM = 256, BN = BN_;
  static constexpr int HALO = (W + 1) * DIL;
  static constexpr int AROWS = BM + 2 * HALO;                // halo tile rows
  static constexpr int SR = 160;                             // S row bytes: hi 64 | lo 64 | 32 unused
  static constexpr int SBUF = (AROWS * SR + 1023) / 1024 * 1024;   // rows, DMA'd in 1-KiB pieces (PRE)
  static constexpr int ZREL = SBUF;                          // 128 zero bytes after each S buffer
  static constexpr int SSTRIDE = SBUF + 128;
  static constexpr int FROWS = (AROWS + 7) / 8 * 8;          // fp32 halo tile rows (8-row DMA slices)
  static constexpr int NA = FROWS / 8;                       // F slices per chunk
  static constexpr int NQ = SBUF / 1024;                     // S pieces per chunk (PRE)
  static constexpr int NBR = 4;                              // weight ring slots, one tap each
  static constexpr int BP = BN * 64;                         // one fp16 plane of a tap's weight tile
  static constexpr int BSLOT = 2 * BP;
  static constexpr int NBD = BN / 64;                        // weight DMAs (1 KiB) per wave and tap
  template <bool PRE> static constexpr int nsb() { return PRE ? 2 : 1; }
  template <bool PRE> static constexpr int off_f() { return nsb<PRE>() * SSTRIDE; }
  template <bool PRE> static constexpr int off_b() { return off_f<PRE>() + (PRE ? 0 : FROWS * 128); }
  template <bool PRE> static constexpr int off_sink() { return off_b<PRE>() + NBR * BSLOT; }
  template <bool PRE> static constexpr int lds() { return off_sink<PRE>() + 1024; }
  template <bool PRE> static constexpr int apw() { return PRE ? (NQ + 7) / 8 : (NA + 7) / 8; }
};

template <int W, int DIL, int BN, int SIGN, bool PRE>
__global__ __launch_bounds__(512, 1) void conv_fwd_h4_kernel(ConvParams p, H3Args h) {
  using G = H4Geom<W, DIL, BN>;
  constexpr int BM = G::BM, WM = 8, WN = 1, SRB = 128;
  constexpr int TI = 1, TJ = BN / 32, TI16 = 2, TJ16 = BN / 16, NBD = G::NBD;
  static_assert(BN == 64 || BN == 128, "h4 column tiles");
  constexpr int SR = G::SR, AROWS = G::AROWS, SSTRIDE = G::SSTRIDE, ZREL = G::ZREL;
  constexpr int BP = G::BP, BSLOT = G::BSLOT;
  constexpr int OFF_F = G::template off_f<PRE>(), OFF_B = G::template off_b<PRE>();
  constexpr int OFF_SINK = G::template off_sink<PRE>();   // target of the zero-fill DMAs that keep vmcnt counts exact
  constexpr int APW = G::template apw<PRE>();   // A-tile DMAs per wave and chunk, one per tap 0 .. APW-1
  static_assert(G::template lds<PRE>() <= 160 * 1024, "LDS");
  // the next chunk's A pieces are issued at taps 0 .. APW-1 and must have landed (the tap-end wait
  // leaves only that tap's DMAs in flight) before PRE's tap 8 reads them / before the convert after tap 8
  static_assert(APW <= (PRE ? 7 : 8), "A DMAs land before the next chunk's tile is read");
  static_assert(SSTRIDE + 64 < 65536 && ZREL < 65536, "16-bit fragment offsets");
  static_assert(2 * WM * BN * 4 + WM * 2048 <= AROWS * SR, "epilogue scratch fits S");

  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* lds = reinterpret_cast<char*>(smem);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nbn = p.Cout / BN;
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
  const int pix0 = m0 - G::HALO;

  // zero rows after each S buffer
  if (tid < 32) reinterpret_cast<float*>(lds + ZREL)[tid] = 0.f;
  if (PRE && tid >= 32 && tid < 64) reinterpret_cast<float*>(lds + SSTRIDE + ZREL)[tid - 32] = 0.f;

  const int32x4 rs0 = make_rsrc(p.x0, (unsigned)((size_t)p.P * p.ldx0 * 4));
  const int32x4 rs1 = make_rsrc(p.c1 ? p.x1 : p.x0, (unsigned)((size_t)p.P * (p.c1 ? p.ldx1 : p.ldx0) * 4));
  const size_t plane = (size_t)p.Cout * p.K;   // fp16 elements per weight plane
  const int32x4 rsw = make_rsrc(h.wsp, (unsigned)(2 * plane * 2));
  const int ld1 = p.c1 ? p.ldx1 : p.ldx0;

  unsigned ab = h.amax0 ? *h.amax0 : 0u;
  if (p.c1 && h.amax1) ab = max(ab, *h.amax1);
  const int ea = h3_exp(ab);
  const float sa = exp2i(ea);

  const int lr = lane & 31, l16 = lane & 15, lq = lane >> 4;
  const int wmi = wave, wni = 0, wm0 = wave * 32;

  // per tap: the S offsets (relative to the S buffer) of this lane's A fragment (hi pieces; lo +64)
  // for its two 16-row blocks, 16 bits each; taps outside the image -> the zero row
  unsigned apk[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) apk[t] = 0;
#pragma unroll
  for (int i = 0; i < TI16; ++i) {
    const int rr = wm0 + i * 16 + l16;
    const int m = m0 + rr;
    int yy = -(1 << 20), xx = 0;
    if (m < p.P) {
      const int rem = m % (p.H * W);
      yy = rem / W;
      xx = rem - yy * W;
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ky = SIGN > 0 ? t / 3 : 2 - t / 3, kx = SIGN > 0 ? t % 3 : 2 - t % 3;
      const int iy = yy + (ky - 1) * DIL, ix = xx + (kx - 1) * DIL;
      const bool ok = iy >= 0 && iy < p.H && ix >= 0 && ix < W;
      const unsigned rel = ok ? (unsigned)((rr + (ky * W + kx) * DIL) * SR + lq * 16) : (unsigned)ZREL;
      apk[t] |= rel << (16 * i);
    }
  }
  // B fragment reads: row r = 16 j + l16 of the tap's tile, 16-B chunk lq at slot swzh(r, lq)
  const unsigned b_lane = (unsigned)(OFF_B + l16 * 64 + swzh(l16, lq) * 16);
  // B DMA d of wave w: 16-row block rb of plane pl (BN = 128: row block w of both planes; BN = 64: plane
  // w / 4, row block w % 4); per-tile byte offsets, the tap / chunk part is soffset
  unsigned b_voff[NBD], b_lds[NBD];
#pragma unroll
  for (int d = 0; d < NBD; ++d) {
    const int pl = NBD == 2 ? d : wave >> 2, rb = NBD == 2 ? wave : wave & 3;
    const int r = rb * 16 + (lane >> 2);
    const int c = swzh(r, lane & 3);
    b_voff[d] = (unsigned)((pl * plane + (size_t)(n0 + r) * p.K + c * 8) * 2);
    b_lds[d] = (unsigned)(pl * BP + rb * 1024);
  }

  const int nch = p.Cin / BK2;
  const int c_beg = tail ? (piece * nch) / p.tsplit : 0;
  const int c_end = tail ? ((piece + 1) * nch) / p.tsplit : nch;
  const size_t xplane = (size_t)p.P * p.Cin;
  const unsigned lds0 = lds_addr_of(lds);

  // A-tile DMA u of this wave: PRE, S piece q = wave + 8 u = bytes [1024 q, +1024) of an S buffer, 16 B
  // per lane, ten per 160-B row (per-tile lane offsets); otherwise F slice q = halo rows 8q .. 8q+7,
  // 16-B chunk k of row r at slot swz(r, k) (offsets formed per DMA: the registers are worth more)
  unsigned a_voff[PRE ? APW : 1];
  if constexpr (PRE) {
#pragma unroll
    for (int u = 0; u < APW; ++u) {
      const int q = wave + 8 * u;
      const int b = q * 1024 + lane * 16;
      const int r = b / SR, slot = (b - r * SR) >> 4;
      const int pix = pix0 + r;
      a_voff[u] = (slot < 8 && r < AROWS && pix >= 0 && pix < p.P)
                      ? (unsigned)(((slot >= 4 ? xplane : 0) + (size_t)pix * p.Cin + (slot & 3) * 8) * 2)
                      : OOB;
    }
  }
  // the A-tile DMA u for chunk ch.  Every wave issues exactly the same DMAs per tap whatever the
  // tile: a piece past the tile (q >= NQ / NA) or past the tile's last chunk (!real) is a zero
  // fill into the sink, so the vmcnt counts of the tap loop stay exact.
  auto issue_a = [&](int ch, int u, bool real) {
    const int q = wave + 8 * u;
    if (!real || q >= (PRE ? G::NQ : G::NA)) {
      dma16s(rs0, OOB, 0u, lds0 + (unsigned)OFF_SINK);
      return;
    }
    if constexpr (PRE) {
      dma16s(rs0, a_voff[u], (unsigned)(ch * BK2 * 2), lds0 + (unsigned)((ch & 1) * SSTRIDE + q * 1024));
    } else {
      const int ch0 = ch * BK2;
      const bool second = ch0 >= p.c0;   // the second input of a virtual concat (own rows, own stride)
      const int r = q * 8 + (lane >> 3);
      const int pix = pix0 + r;
      const unsigned voff =
          (pix >= 0 && pix < p.P) ? (unsigned)((pix * (second ? ld1 : p.ldx0) + swz(r, lane & 7) * 4) * 4) : OOB;
      dma16s(second ? rs1 : rs0, voff, (unsigned)((second ? ch0 - p.c0 : ch0) * 4), lds0 + (unsigned)(OFF_F + q * 1024));
    }
  };
  // the weight tile of tap `tap` of chunk `ch` into ring slot `slot` (!real: zero fills into the sink)
  auto issue_b = [&](int ch, int tap, int slot, bool real) {
    const unsigned soff = (unsigned)((tap * p.Cin + ch * BK2) * 2);
#pragma unroll
    for (int d = 0; d < NBD; ++d)
      dma16s(rsw, real ? b_voff[d] : OOB, real ? soff : 0u,
             lds0 + (unsigned)(real ? OFF_B + slot * BSLOT + b_lds[d] : OFF_SINK));
  };

  // F (chunk ch, landed) -> S: scale and split every halo element once per chunk; the N-tile-0
  // workgroup of each row tile also stores its own rows' pieces to h.xsplit
  const bool wsplit = !PRE && h.xsplit != nullptr && nt == 0;
  auto convert = [&](int ch) {
    float4 s0, s1, t0, t1;
    const int c8 = tid & 3;   // every task of this thread has the same 8 channels
    const bool gate = h.x1_ca != nullptr && ch * BK2 >= p.c0;   // the attention-gated second input
    if (h.in_scale != nullptr) {
      const int cc = ch * BK2 + c8 * 8;
      s0 = *reinterpret_cast<const float4*>(h.in_scale + cc);
      s1 = *reinterpret_cast<const float4*>(h.in_scale + cc + 4);
      t0 = *reinterpret_cast<const float4*>(h.in_shift + cc);
      t1 = *reinterpret_cast<const float4*>(h.in_shift + cc + 4);
    }
#pragma unroll
    for (int k = 0; k < (AROWS * 4 + 511) / 512; ++k) {
      const int sg = tid + 512 * k;
      if (sg >= AROWS * 4) break;
      const int r = sg >> 2;
      const char* f = lds + OFF_F + r * 128;
      float4 v0 = *reinterpret_cast<const float4*>(f + swz(r, 2 * c8) * 16);
      float4 v1 = *reinterpret_cast<const float4*>(f + swz(r, 2 * c8 + 1) * 16);
      if (gate) gate8(v0, v1, h, pix0 + r, p.P, p.H * W, p.c1, ch * BK2 - p.c0 + c8 * 8);
      if (h.in_scale != nullptr) {   // fused BN + ReLU of the producer; rows outside the tensor stay 0
        const int pix = pix0 + r;
        const bool inside = pix >= 0 && pix < p.P;
#define AFF(V, S, T, X) V.X = inside ? fmaxf(V.X * S.X + T.X, 0.f) : 0.f;
        AFF(v0, s0, t0, x) AFF(v0, s0, t0, y) AFF(v0, s0, t0, z) AFF(v0, s0, t0, w)
        AFF(v1, s1, t1, x) AFF(v1, s1, t1, y) AFF(v1, s1, t1, z) AFF(v1, s1, t1, w)
#undef AFF
      }
      half8 hv, lv;
      split2h(v0, v1, sa, hv, lv);
      *reinterpret_cast<half8*>(lds + r * SR + c8 * 16) = hv;
      *reinterpret_cast<half8*>(lds + r * SR + 64 + c8 * 16) = lv;
      if (wsplit) {
        const int pix = pix0 + r;
        if (r >= G::HALO && r < G::HALO + BM && pix < p.P) {
          _Float16* dst = h.xsplit + (size_t)pix * p.Cin + ch * BK2 + c8 * 8;
          *reinterpret_cast<half8*>(dst) = hv;
          *reinterpret_cast<half8*>(dst + xplane) = lv;
        }
      }
    }
  };

  floatx4 acc[TI16][TJ16], part[TI16][TJ16];
#pragma unroll
  for (int i = 0; i < TI16; ++i)
#pragma unroll
    for (int j = 0; j < TJ16; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.f;

  // prologue: the first chunk's A tile, the weights of its first three taps
#pragma unroll
  for (int u = 0; u < APW; ++u) issue_a(c_beg, u, true);
#pragma unroll
  for (int t = 0; t < 3; ++t) issue_b(c_beg, t, t, true);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (!PRE) {
    convert(c_beg);
    __syncthreads();
  }

  // fragments carried from one tap to the next
  half8 ah[TI16], al[TI16], bh0, bl0, bh1, bl1;
  auto read_a = [&](int t_dyn_unused, unsigned pk, unsigned sbase, half8 (&xh)[TI16], half8 (&xl)[TI16]) {
    (void)t_dyn_unused;
#pragma unroll
    for (int i = 0; i < TI16; ++i) {
      const unsigned o = sbase + (i == 0 ? (pk & 0xffffu) : (pk >> 16));
      xh[i] = *reinterpret_cast<const half8*>(lds + o);
      xl[i] = *reinterpret_cast<const half8*>(lds + o + 64);
    }
  };
  {
    const unsigned sb = PRE ? (unsigned)((c_beg & 1) * SSTRIDE) : 0u;
    read_a(0, apk[0], sb, ah, al);
    const unsigned bb = b_lane;   // slot 0
    bh0 = *reinterpret_cast<const half8*>(lds + bb);
    bl0 = *reinterpret_cast<const half8*>(lds + bb + BP);
    bh1 = *reinterpret_cast<const half8*>(lds + bb + 1024);
    bl1 = *reinterpret_cast<const half8*>(lds + bb + BP + 1024);
  }

  // column blocks a B fragment pair is read ahead of its MFMAs: two where the registers allow (PRE: 243
  // VGPRs; BN = 64: half the accumulators), one with the convert path's registers at BN = 128 (two: 24
  // VGPRs of spill)
  constexpr int BPF = (PRE || BN == 64) ? 2 : 1;
  int slot0 = 0;   // ring slot of the chunk's tap 0 (taps of a tile use slots 0, 1, 2, 3, 0, ...)
  // one tap: MFMAs of column block j with the B fragments of block j + 2 (or of the next tap)
  // in flight; the next tap's A fragments read at block TJ16 / 2 - 1 (within the chunk)
  auto tap = [&](int ch, auto tap_tag) {
    constexpr int T = decltype(tap_tag)::value;
    const int slot = (slot0 + T) & 3;
    const bool more = ch + 1 < c_end;
    const unsigned bcur = b_lane + (unsigned)(slot * BSLOT);
    const unsigned bnext = b_lane + (unsigned)(((slot + 1) & 3) * BSLOT);
    const unsigned sb = PRE ? (unsigned)((ch & 1) * SSTRIDE) : 0u;
    const unsigned sbn = PRE ? (unsigned)(((ch + 1) & 1) * SSTRIDE) : 0u;
    // DMAs of this tap: the next chunk's A-tile piece T (T < APW), then the weights of tap tau + 3
    if constexpr (!(SRPDE_CONV_DBG & 1)) {   // (timing-only diagnostics, conv_common.h: 1 = no DMA in the taps)
      if constexpr (T < APW) issue_a(ch + 1, T, more);
      constexpr int T3 = T + 3;
      if constexpr (T3 < 9) issue_b(ch, T3, (slot + 3) & 3, true);
      else issue_b(ch + 1, T3 - 9, (slot + 3) & 3, more);
    }
    half8 bh[TJ16], bl[TJ16], nah[TI16], nal[TI16];
    bh[0] = bh0; bl[0] = bl0;
    if constexpr (BPF > 1) { bh[1] = bh1; bl[1] = bl1; }
    static_for<0, TJ16>([&](auto j_tag) {
      constexpr int j = decltype(j_tag)::value;
      if constexpr (j + BPF < TJ16) {
        bh[j + BPF] = *reinterpret_cast<const half8*>(lds + bcur + (j + BPF) * 1024);
        bl[j + BPF] = *reinterpret_cast<const half8*>(lds + bcur + BP + (j + BPF) * 1024);
      } else if constexpr (j + BPF - TJ16 < 2) {   // the next tap's first column blocks (landed: its DMA
                                                    // was waited for before the last barrier)
        constexpr int jn = j + BPF - TJ16;
        half8& xh = jn == 0 ? bh0 : bh1;
        half8& xl = jn == 0 ? bl0 : bl1;
        xh = *reinterpret_cast<const half8*>(lds + bnext + jn * 1024);
        xl = *reinterpret_cast<const half8*>(lds + bnext + BP + jn * 1024);
      }
      // the next tap's A fragments: within the chunk; PRE also across it (the next chunk's S buffer
      // has landed: its pieces were issued at taps < APW and waited for with tap 8's weights)
      constexpr bool RA = j == TJ16 / 2 - 1 && (T < 8 || PRE);
      if constexpr (RA) read_a(0, apk[T < 8 ? T + 1 : 0], T < 8 ? sb : sbn, nah, nal);
#pragma unroll
      for (int i = 0; i < TI16 && !(SRPDE_CONV_DBG & 128); ++i) {   // diagnostics: 128 = no MFMAs
        floatx4 c0;
        if (T == 0)   // a chunk's partial chain starts from zero
          c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], floatx4{}, 0, 0, 0);
        else          // small terms first
          c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], part[i][j], 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j], c0, 0, 0, 0);
        part[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], c0, 0, 0, 0);
      }
      constexpr int NRB = (j + BPF < TJ16 || j + BPF - TJ16 < 2) ? 2 : 0;
      __builtin_amdgcn_sched_group_barrier(0x100, NRB + (RA ? 2 * TI16 : 0), 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 3 * TI16, 0);
    });
    if constexpr (T < 8 || PRE) {
#pragma unroll
      for (int i = 0; i < TI16; ++i) {
        ah[i] = nah[i];
        al[i] = nal[i];
      }
    }
    // after this barrier the next tap tau + 1 reads its own weights (issued at tap tau - 2) AND the first
    // column blocks of tap tau + 2's (issued at tap tau - 1): only this tap's DMAs may still be in
    // flight (exact counts: every wave issues NCUR DMAs per tap, zero fills included; the prologue
    // before the first tap drained to 0).  Round 4 waited for tap tau - 2 only, so the bnext reads of
    // the following tap could see a slot before its DMA landed: a run-to-run race that showed under
    // load (tools/diag_race.py: dgrad outputs changed in the first column blocks of a tile).
    constexpr int NCUR = NBD + (T < APW ? 1 : 0);
    // a bare s_barrier: no lgkmcnt(0) drain of the next tap's fragment reads still in flight (they read
    // slot tau + 1 and the S tile, which no DMA issued after this barrier writes); the asm is a
    // compiler memory barrier, so no LDS read moves above it
    if constexpr (SRPDE_CONV_DBG & 2)   // diagnostics: 2 = no tap barrier
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NCUR) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(NCUR) : "memory");
  };

  for (int ch = c_beg; ch < c_end; ++ch) {
    tap(ch, std::integral_constant<int, 0>{});
    tap(ch, std::integral_constant<int, 1>{});
    tap(ch, std::integral_constant<int, 2>{});
    tap(ch, std::integral_constant<int, 3>{});
    tap(ch, std::integral_constant<int, 4>{});
    tap(ch, std::integral_constant<int, 5>{});
    tap(ch, std::integral_constant<int, 6>{});
    tap(ch, std::integral_constant<int, 7>{});
    tap(ch, std::integral_constant<int, 8>{});
    slot0 = (slot0 + 9) & 3;
    // two-level accumulation: one partial chain per channel chunk (9 taps x 32 channels)
#pragma unroll
    for (int i = 0; i < TI16; ++i)
#pragma unroll
      for (int j = 0; j < TJ16; ++j) acc[i][j] += part[i][j];
    if constexpr (!PRE) {
      if (ch + 1 < c_end) {   // the next chunk's halo tile has landed in F (its DMAs preceded the last wait)
        if (!(SRPDE_CONV_DBG & 4)) convert(ch + 1);   // diagnostics: 4 = no per-chunk convert
        __syncthreads();
        read_a(0, apk[0], 0u, ah, al);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the trailing zero-fill DMAs, before LDS is reused

  floatx16 acc32[TI][TJ];
  acc16_to_32<TI, TJ>(acc, acc32);
  // the scales to undo: acc * 2^-(ea + wexp[col]) (conv_fwd_h3_kernel)
  float colscale[TJ];
  const float ia = exp2i(-ea);
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int col = n0 + j * 32 + lr;
    const int we = h.wexp[col];
    const int e = ea + we;
    if (e > 126 || e < -126) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc32[0][j][r] *= ia;
      colscale[j] = exp2i(-we);
    } else {
      colscale[j] = exp2i(-e);
    }
  }
  if constexpr (SRPDE_CONV_DBG & 16) {   // diagnostics: 16 = no epilogue (one store per lane keeps the MFMAs live)
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < TJ; ++j) t += acc32[0][j][0] * colscale[j] + acc32[0][j][15];
    if (t == 123.f) p.y[tid] = t;
    return;
  }
  // S is free now: reduction scratch [2][WM][BN] floats, then 2 KiB per wave of store stage
  x6_finish<BM, BN, WM, WN, SRB>(p, acc32, tail, wg, nfull, piece, m0, n0, wmi, wni, lane, smem,
                                 h.wide ? smem + 2 * WM * BN : nullptr, colscale);
}

// ---------------------------------- host side ---------------------------------------
template <int W, int DIL, int BN_, int SIGN, bool PRE>
static int launch_h4_cfg(ConvParams p, H3Args h, hipStream_t st, void* ws, size_t ws_bytes) {
  using G = H4Geom<W, DIL, BN_>;
  constexpr int BM = G::BM, BN = G::BN;
  const int T = ceil_div(p.P, BM) * (p.Cout / BN);
  static const int cus = [] {
    int dev = 0, c = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    return std::max(1, c);
  }();
  plan_tail(p, T, cus, BM, BN, ws, ws_bytes);   // one workgroup per CU (LDS)
  const int nch = p.Cin / BK2;
  if (p.ntail > 0 && p.tsplit > nch) p.tsplit = nch;
  if (p.tsplit < 2) { p.ntail = 0; p.tsplit = 1; }
  const int grid = T - p.ntail + p.ntail * p.tsplit;
  hipLaunchKernelGGL((conv_fwd_h4_kernel<W, DIL, BN, SIGN, PRE>), dim3(grid), dim3(512), G::template lds<PRE>(), st, p, h);
  SRPDE_LAUNCH_CHECK("srpde_conv_fwd_h3(h4)");
  if (p.ntail > 0) return launch_tail_fixup<BM, BN, 128>(p, st);
  return 0;
}

// the column tile: 128 where the weight ring and two S buffers fit LDS (W <= 20), else 64
static int h4_bn(int w, int cout) { return (cout % 128 == 0 && w <= 20) ? 128 : 64; }

bool h4_supported(int w, int dil, int cout, bool bnb) {
  if (bnb || cout % 64 != 0) return false;
  return (w == 10 && (dil == 1 || dil == 2)) || (w == 20 && dil == 1) || (w == 40 && dil == 1);
}

int launch_fwd_h4(const ConvParams& p, const H3Args& h, bool pre, hipStream_t st, void* ws, size_t ws_bytes) {
#define H4_CASE(W_, D_, BN_)                                                                          \
  if (p.W == W_ && p.dil == D_ && h4_bn(W_, p.Cout) == BN_) {                                         \
    if (pre) return p.sign > 0 ? launch_h4_cfg<W_, D_, BN_, 1, true>(p, h, st, ws, ws_bytes)          \
                               : launch_h4_cfg<W_, D_, BN_, -1, true>(p, h, st, ws, ws_bytes);        \
    return p.sign > 0 ? launch_h4_cfg<W_, D_, BN_, 1, false>(p, h, st, ws, ws_bytes)                  \
                      : launch_h4_cfg<W_, D_, BN_, -1, false>(p, h, st, ws, ws_bytes);                \
  }
  H4_CASE(10, 1, 128)
  H4_CASE(10, 2, 128)
  H4_CASE(20, 1, 128)
  H4_CASE(10, 1, 64)
  H4_CASE(10, 2, 64)
  H4_CASE(20, 1, 64)
  H4_CASE(40, 1, 64)
#undef H4_CASE
  set_error("srpde_conv_fwd_h3(h4): no instantiation for W=%d dil=%d cout=%d", p.W, p.dil, p.Cout);
  return kErrArg;
}

}  // namespace srpde
