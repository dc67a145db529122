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
//  * One tap per weight stage in a ring of NBR slots (4 at 128 columns, 6 .. 8 at 64), filled
//    PD = NBR - 1 taps ahead.  A wave waits for its own DMA of tap tau+2 at the end of tap tau,
//    so after that tap's barrier every wave may read tap tau+2's B fragments -- the B fragments
//    of the next tap (and, within a chunk, its A fragments) are read during the current tap's
//    MFMAs, and a wave leaves each barrier with its operands in registers.  (h3: the fragments of each column block were read
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

// A/B switch for the DMA placement in a tap (1: all waves at the top of the tap, the round-4 first form)
#ifndef H4_DMA_EARLY
#define H4_DMA_EARLY 1
#endif
// A/B switch: s_setprio 1 for waves 4-7 (MI355X_MICROARCH.md, two waves per SIMD, item 4; measured: no
// change on six layers, tools/gpu/multi_ab.sh "prio")
#ifndef H4_PRIO
#define H4_PRIO 0
#endif
// A/B switch: the tap barrier after every second tap (taps 1, 3, 5, 7, 8 of a chunk) where the weight
// ring has >= 6 slots; the prefetch distance drops by one tap (PD = slots - 2) so that the two taps
// between barriers never DMA into a slot a slower wave still reads.  Measured: no change (30 conv
// passes 15.463 -> 15.447 ms, forward within noise; run-to-run race check clean;
// profiles/r04s_h4_bar2_ab.txt) -- the per-tap overhead is not the barrier
#ifndef H4_BAR2
#define H4_BAR2 0
#endif

typedef float h4f32x4 __attribute__((ext_vector_type(4)));
__device__ h4f32x4 h4_buffer_load_f4(int32x4 rsrc, int voffset, int soffset,
                                     int aux) __asm("llvm.amdgcn.raw.buffer.load.v4f32");
__device__ __forceinline__ float4 f4_of(h4f32x4 v) { return make_float4(v[0], v[1], v[2], v[3]); }
__device__ float h4_buffer_load_f1(int32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.f32");

// conv_h3.h gate8 (the same expressions) with buffer loads: the attention vectors' 64-bit base pointers, held
// in VGPRs across the persistent loop, were the last spilled registers of the 128-column instantiations
__device__ __forceinline__ void gate8_h4(float4& v0, float4& v1, const H3Args& h, int pix, int P, int HW, int c1,
                                         int cc1) {
  if (pix < 0 || pix >= P) return;
  const int n = pix / HW;
  const int32x4 rca = make_rsrc(h.x1_ca, (unsigned)((P / HW) * c1 * 4)), rsa = make_rsrc(h.x1_sa, (unsigned)(P * 4));
  const float4 a0 = f4_of(h4_buffer_load_f4(rca, (n * c1 + cc1) * 4, 0, 0));
  const float4 a1 = f4_of(h4_buffer_load_f4(rca, (n * c1 + cc1) * 4 + 16, 0, 0));
  const float s = h4_buffer_load_f1(rsa, pix * 4, 0, 0);
  v0.x = (v0.x * a0.x) * s; v0.y = (v0.y * a0.y) * s; v0.z = (v0.z * a0.z) * s; v0.w = (v0.w * a0.w) * s;
  v1.x = (v1.x * a1.x) * s; v1.y = (v1.y * a1.y) * s; v1.z = (v1.z * a1.z) * s; v1.w = (v1.w * a1.w) * s;
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
  static constexpr int BP = BN * 64;                         // one fp16 plane of a tap's weight tile
  static constexpr int BSLOT = 2 * BP;
  static constexpr int NBD = BN / 64;                        // weight DMAs (1 KiB) per wave and tap
  // persistent workgroups (one per CU running tile after tile, each tile's first chunk loaded during the
  // previous tile's last chunk) with 64-column tiles; at 128 columns the loop-carried state plus the
  // epilogue exceed 256 VGPRs (~170 spilled), so those run one tile per workgroup
  static constexpr bool PERSIST = BN == 64;
  template <bool PRE> static constexpr int nsb() { return PRE ? 2 : 1; }
  template <bool PRE> static constexpr int off_f() { return nsb<PRE>() * SSTRIDE; }
  template <bool PRE> static constexpr int off_b() { return off_f<PRE>() + (PRE ? 0 : FROWS * 128); }
  // weight ring slots (one tap each): as many as LDS holds, 4 .. 8.  Tap tau issues the weights of tap
  // tau + PD (PD = slots - 1) into the slot tap tau - 1 used.  64-column tiles (8-KiB slots) get 6 or 7:
  // their taps are half as long, and with PD = 3 the weight DMA latency was exposed (the MFMA-free
  // build of enc1.conv2 took 0.43 of its 0.65 ms, one DMA round trip per tap)
  template <bool PRE> static constexpr int nbr() {
    constexpr int base = PRE ? 2 * SSTRIDE : SSTRIDE + FROWS * 128;
    constexpr int n = (160 * 1024 - base - 1024) / BSLOT;
    return n > 8 ? 8 : n;
  }
  template <bool PRE> static constexpr int off_sink() { return off_b<PRE>() + nbr<PRE>() * BSLOT; }
  template <bool PRE> static constexpr int lds() { return off_sink<PRE>() + 1024; }
  template <bool PRE> static constexpr int apw() { return PRE ? (NQ + 7) / 8 : (NA + 7) / 8; }
};

// one work item of a persistent workgroup: a whole output tile, or one K-piece of a split tail tile
struct H4Tile {
  int wg, piece, m0, n0, pix0, c_beg, c_end;
  int lo;   // UP: the first low-res source pixel the tile's halo reads
  bool tail;
};

// UP: x0 is the bilinear x2 upsample of h.up_src (forward, non-PRE only), interpolated from low-res rows
// DMA'd into F in the per-chunk convert
template <int W, int DIL, int BN, int SIGN, bool PRE, bool UP = false>
__global__ __launch_bounds__(512, 1) void conv_fwd_h4_kernel(ConvParams p, H3Args h) {
  using G = H4Geom<W, DIL, BN>;
  constexpr int BM = G::BM, WM = 8, WN = 1, SRB = 128;
  constexpr int TI = 1, TJ = BN / 32, TI16 = 2, TJ16 = BN / 16, NBD = G::NBD;
  static_assert(BN == 64 || BN == 128, "h4 column tiles");
  constexpr int SR = G::SR, AROWS = G::AROWS, SSTRIDE = G::SSTRIDE, ZREL = G::ZREL;
  constexpr int BP = G::BP, BSLOT = G::BSLOT;
  constexpr int OFF_F = G::template off_f<PRE>(), OFF_B = G::template off_b<PRE>();
  constexpr int OFF_SINK = G::template off_sink<PRE>();   // target of the zero-fill DMAs that keep vmcnt counts exact
  constexpr int APW = G::template apw<PRE>();   // A-tile DMAs per wave and chunk
  constexpr int NBR = G::template nbr<PRE>();   // weight ring slots
  constexpr bool BAR2 = H4_BAR2 && NBR >= 6;    // a tap barrier after every second tap (H4_BAR2 above)
  constexpr int PD = BAR2 ? NBR - 2 : NBR - 1;  // prefetch distance (taps)
  static_assert(NBR >= 4 && G::template lds<PRE>() <= 160 * 1024, "LDS");
  // a tap-end wait leaves the DMAs of the last WIN taps in flight (see the barrier in tap()); the next
  // chunk's A pieces, APT per tap in taps 0 .. TA-1, must have landed by PRE's tap 8 (it reads them) /
  // by the convert after tap 8
  // (BAR2: a wait must also cover the window's second tap, so one tap fewer stays in flight)
  constexpr int WIN = BAR2 ? PD - 3 : PD - 2;
  constexpr int TA = (PRE ? 8 : 9) - WIN;
  constexpr int APT = (APW + TA - 1) / TA;
  static_assert(APT <= 2 && TA >= 1, "A DMAs land before the next chunk's tile is read");
  static_assert(SSTRIDE + 64 < 65536 && ZREL < 65536, "16-bit fragment offsets");
  static_assert(2 * WM * BN * 4 + WM * 2048 <= AROWS * SR, "epilogue scratch fits S");
  static_assert(!UP || (!PRE && SIGN > 0 && DIL == 1), "the upsampled input: forward, fp32 input");
  // UP: the low-res rows of a tile's halo, at most (AROWS / W + 2) / 2 + 3 source image rows (two images
  // when the tile crosses one's end), fit F's FROWS rows
  static_assert(!UP || ((AROWS / W + 2) / 2 + 3) * (W / 2) <= G::FROWS, "upsample source rows fit F");

  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* lds = reinterpret_cast<char*>(smem);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nbn = p.Cout / BN;
  const int nbm = (p.P + BM - 1) / BM;
  const int nfull = nbm * nbn - p.ntail;
  const int nitems = nfull + p.ntail * p.tsplit;
  const int nch = p.Cin / BK2;
  // work item -> tile: the whole tiles in XCD-aware order (blocks sharing an A row panel on one XCD;
  // a persistent workgroup b stays on XCD b % 8 and takes items b, b + grid, ..., grid % 8 == 0), then
  // the K-pieces of the split tail
  auto tile_of = [&](int it) {
    H4Tile t;
    if (it < nfull) {
      t.wg = xcd_remap(it, nfull);
      t.piece = 0;
    } else {
      const int q = it - nfull;
      t.wg = nfull + q / p.tsplit;
      t.piece = q - (q / p.tsplit) * p.tsplit;
    }
    t.tail = t.wg >= nfull;
    const int mt = t.wg / nbn, nt = t.wg - mt * nbn;
    t.m0 = mt * BM;
    t.n0 = nt * BN;
    t.pix0 = t.m0 - G::HALO;
    t.c_beg = t.tail ? (t.piece * nch) / p.tsplit : 0;
    t.c_end = t.tail ? ((t.piece + 1) * nch) / p.tsplit : nch;
    t.lo = 0;
    if constexpr (UP) {   // the low-res row of the tile's first in-tensor halo pixel, x = 0
      const int pf = max(t.pix0, 0), HWh = p.H * W;
      const int nn = pf / HWh, yy = (pf - nn * HWh) / W;
      t.lo = nn * h.up_h * h.up_w + lerp_index(yy, h.up_h, p.H).i0 * h.up_w;
    }
    return t;
  };

  // zero rows after each S buffer
  if (tid < 32) reinterpret_cast<float*>(lds + ZREL)[tid] = 0.f;
  if (PRE && tid >= 32 && tid < 64) reinterpret_cast<float*>(lds + SSTRIDE + ZREL)[tid - 32] = 0.f;

  const int32x4 rs0 = make_rsrc(p.x0, (unsigned)((size_t)p.P * p.ldx0 * 4));
  const int32x4 rs1 = make_rsrc(p.c1 ? p.x1 : p.x0, (unsigned)((size_t)p.P * (p.c1 ? p.ldx1 : p.ldx0) * 4));
  const int Plo = UP ? p.N * h.up_h * h.up_w : 0;
  const int32x4 rsu = make_rsrc(UP ? h.up_src : p.x0, UP ? (unsigned)((size_t)Plo * h.up_ld * 4) : 0u);
  const unsigned plane = (unsigned)p.Cout * (unsigned)p.K;   // fp16 elements per weight plane
  const int32x4 rsw = make_rsrc(h.wsp, 2u * plane * 2u);
  const int ld1 = p.c1 ? p.ldx1 : p.ldx0;

  unsigned ab = h.amax0 ? *h.amax0 : 0u;
  if (p.c1 && h.amax1) ab = max(ab, *h.amax1);
  const int ea = h3_exp(ab);
  const float sa = exp2i(ea);

  const int lr = lane & 31, l16 = lane & 15, lq = lane >> 4;
  const int wmi = wave, wni = 0, wm0 = wave * 32;

  // B fragment reads: row r = 16 j + l16 of the tap's tile, 16-B chunk lq at slot swzh(r, lq)
  const unsigned b_lane = (unsigned)(OFF_B + l16 * 64 + swzh(l16, lq) * 16);
  const unsigned xplane = (unsigned)p.P * (unsigned)p.Cin;
  const unsigned lds0 = lds_addr_of(lds);
  // diagnostics 256: wave 0 of each workgroup records s_memtime at phase boundaries past the output
  // (y + P * ldy + 64 * blockIdx.x floats: the caller allocates the room; tools/h4_phase_ts.py)
  int nts = 0;
  auto stamp = [&]() {
    if constexpr ((SRPDE_CONV_DBG & 256) != 0) {
      if (wave == 0 && nts < 32) {   // wave-uniform (a lane-divergent branch upsets the scalar operands)
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_s_waitcnt(0xc07f);
        reinterpret_cast<unsigned long long*>(p.y + (size_t)p.P * p.ldy)[(size_t)blockIdx.x * 32 + nts] = t;
      }
      ++nts;
    }
  };

  // the A-tile DMA u of a tile's chunk ch.  PRE: S piece q = wave + 8 u = bytes [1024 q, +1024) of S
  // buffer `buf`, 16 B per lane, ten per 160-B row; otherwise F slice q = halo rows 8q .. 8q+7, 16-B
  // chunk k of row r at slot swz(r, k).  Offsets are formed per DMA (registers are worth more).  Every
  // wave issues exactly the same DMAs per tap whatever the tile: a piece past the tile (q >= NQ / NA)
  // or with nothing to load (!real) is a zero fill into the sink, so the vmcnt counts stay exact.
  // per-lane DMA constants, formed once (tile-independent; the per-DMA work is a few VALU ops and scalar
  // selects, no branches).  PRE A piece u: its S row r and 16-B slot (hi 0-3, lo 4-7, 8-9 the unused
  // 32 B of a 160-B row), bit 31 = the piece lies inside the tile and is loaded.  B DMA d: the lane's
  // byte offset in the weight planes of column tile 0.
  constexpr int NAU = PRE ? ((APW + APT - 1) / APT) * APT : 1;
  unsigned apre[NAU], bofs[NBD];
  if constexpr (PRE) {
#pragma unroll
    for (int u = 0; u < NAU; ++u) {
      const int q = wave + 8 * u;
      const int b = q * 1024 + lane * 16;
      const int r = b / SR, slot = (b - r * SR) >> 4;
      apre[u] = (unsigned)r | ((unsigned)(slot & 7) << 16) | ((q < G::NQ && slot < 8 && r < AROWS) ? 0x80000000u : 0u);
    }
  }
#pragma unroll
  for (int d = 0; d < NBD; ++d) {
    const int pl = NBD == 2 ? d : wave >> 2, rb = NBD == 2 ? wave : wave & 3;
    const int r = rb * 16 + (lane >> 2);
    bofs[d] = (pl * plane + (unsigned)r * (unsigned)p.K + swzh(r, lane & 3) * 8) * 2u;
  }

  // the A-tile DMA u of a tile's chunk ch.  PRE: S piece q = wave + 8 u = bytes [1024 q, +1024) of S
  // buffer `buf`, 16 B per lane, ten per 160-B row; otherwise F slice q = halo rows 8q .. 8q+7, 16-B
  // chunk k of row r at slot swz(r, k).  Every wave issues exactly the same DMAs per tap whatever the
  // tile: a piece past the tile (q >= NQ / NA) or with nothing to load (!real) is a zero fill into the
  // sink, so the vmcnt counts stay exact.
  auto issue_a = [&](const H4Tile& t, int ch, int u, bool real, int buf) {
    const int pix0 = t.pix0;
    const int q = wave + 8 * u;
    const bool qin = q < (PRE ? G::NQ : G::NA);
    if constexpr (PRE) {
      const unsigned pk = apre[u];
      const int pix = pix0 + (int)(pk & 0xffffu);
      const unsigned slot = (pk >> 16) & 7u;
      const bool ok = real && (pk >> 31) && pix >= 0 && pix < p.P;
      const unsigned voff = ((slot >= 4 ? xplane : 0u) + (unsigned)pix * (unsigned)p.Cin + (slot & 3u) * 8u) * 2u;
      dma16s(rs0, ok ? voff : OOB, (unsigned)(ch * BK2 * 2),
             lds0 + (unsigned)(real && qin ? buf * SSTRIDE + q * 1024 : OFF_SINK));
    } else {
      const int ch0 = ch * BK2;
      const bool second = ch0 >= p.c0;   // the second input of a virtual concat (own rows, own stride)
      int ln = lane;   // laundered: formed per DMA, not hoisted into registers held across the loop
      asm volatile("" : "+v"(ln));
      const int r = q * 8 + (ln >> 3);
      if (UP && !second) {   // F row r = low-res pixel t.lo + r
        const int lp = t.lo + r;
        const bool ok = real && qin && lp < Plo;
        const unsigned voff = (unsigned)((lp * h.up_ld + swz(r, ln & 7) * 4) * 4);
        dma16s(rsu, ok ? voff : OOB, (unsigned)(ch0 * 4), lds0 + (unsigned)(real && qin ? OFF_F + q * 1024 : OFF_SINK));
        return;
      }
      const int pix = pix0 + r;
      const bool ok = real && qin && pix >= 0 && pix < p.P;
      const unsigned voff = (unsigned)((pix * (second ? ld1 : p.ldx0) + swz(r, ln & 7) * 4) * 4);
      dma16s(second ? rs1 : rs0, ok ? voff : OOB, (unsigned)((second ? ch0 - p.c0 : ch0) * 4),
             lds0 + (unsigned)(real && qin ? OFF_F + q * 1024 : OFF_SINK));
    }
  };
  // the weight tile of tap `tap` of a tile's chunk `ch` into ring slot `slot`: DMA d of wave w is the
  // 16-row block rb of plane pl (BN = 128: row block w of both planes; BN = 64: plane w / 4, row block
  // w % 4); !real: zero fills into the sink
  auto issue_b = [&](int n0, int ch, int tap, int slot, bool real) {
    const unsigned soff = (unsigned)((tap * p.Cin + ch * BK2) * 2);
    const unsigned nofs = (unsigned)n0 * (unsigned)p.K * 2u;
#pragma unroll
    for (int d = 0; d < NBD; ++d) {
      const int pl = NBD == 2 ? d : wave >> 2, rb = NBD == 2 ? wave : wave & 3;
      dma16s(rsw, real ? bofs[d] + nofs : OOB, real ? soff : 0u,
             lds0 + (unsigned)(real ? OFF_B + slot * BSLOT + pl * BP + rb * 1024 : OFF_SINK));
    }
  };

  // F (chunk ch of tile t, landed) -> S: scale and split every halo element once per chunk; the
  // N-tile-0 workgroup of each row tile also stores its own rows' pieces to h.xsplit
  auto convert = [&](const H4Tile& t, int ch) {
    const bool wsplit = h.xsplit != nullptr && t.n0 == 0;
    float4 s0, s1, t0, t1;
    const int c8 = tid & 3;   // every task of this thread has the same 8 channels
    const bool gate = h.x1_ca != nullptr && ch * BK2 >= p.c0;   // the attention-gated second input
    if constexpr ((SRPDE_CONV_DBG & 512) != 0) {   // diagnostics: 512 = no scale / shift loads (identity BN)
      s0 = s1 = make_float4(1.f, 1.f, 1.f, 1.f);
      t0 = t1 = make_float4(0.f, 0.f, 0.f, 0.f);
    } else if (h.in_scale != nullptr) {
      // buffer loads: the per-lane part of the address is one 32-bit offset (c8 * 32 B), the chunk's in the
      // scalar offset -- a 64-bit per-lane pointer held across the persistent loop spilled (8 VGPRs) in the
      // 128-column instantiations
      const unsigned nb = (unsigned)((p.c0 + p.c1) * 4);
      const int32x4 rsc = make_rsrc(h.in_scale, nb), rsh = make_rsrc(h.in_shift, nb);
      const int vo = c8 * 32, so = ch * BK2 * 4;
      s0 = f4_of(h4_buffer_load_f4(rsc, vo, so, 0));
      s1 = f4_of(h4_buffer_load_f4(rsc, vo + 16, so, 0));
      t0 = f4_of(h4_buffer_load_f4(rsh, vo, so, 0));
      t1 = f4_of(h4_buffer_load_f4(rsh, vo + 16, so, 0));
    }
    // (UP: not unrolled -- unrolled, the interpolating convert spilled 48-50 VGPRs; eval forward -1 %)
#pragma unroll (UP ? 1 : (AROWS * 4 + 511) / 512)
    for (int k = 0; k < (AROWS * 4 + 511) / 512; ++k) {
      const int sg = tid + 512 * k;
      if (sg >= AROWS * 4) break;
      const int r = sg >> 2;
      float4 v0, v1;
      if (UP && ch * BK2 < p.c0) {
        // the upsampled input: up(x)[pix] from the four low-res rows in F, upsample_gate_fwd_px_kernel's
        // expression (bit-identical to the materialised tensor); rows outside the tensor are 0
        const int pix = t.pix0 + r;
        v0 = v1 = make_float4(0.f, 0.f, 0.f, 0.f);
        if (pix >= 0 && pix < p.P) {
          const int HWh = p.H * W, nn = pix / HWh, rem = pix - nn * HWh, oy = rem / W, ox = rem - oy * W;
          const Lerp ly = lerp_index(oy, h.up_h, p.H), lx = lerp_index(ox, h.up_w, W);
          const int b0 = nn * h.up_h * h.up_w - t.lo;
          const int fa = min(b0 + ly.i0 * h.up_w + lx.i0, G::FROWS - 1), fb = min(b0 + ly.i0 * h.up_w + lx.i1, G::FROWS - 1);
          const int fd = min(b0 + ly.i1 * h.up_w + lx.i0, G::FROWS - 1), ff = min(b0 + ly.i1 * h.up_w + lx.i1, G::FROWS - 1);
#pragma unroll
          for (int hf = 0; hf < 2; ++hf) {
            const int k = 2 * c8 + hf;
            const float4 a = *reinterpret_cast<const float4*>(lds + OFF_F + fa * 128 + swz(fa, k) * 16);
            const float4 b = *reinterpret_cast<const float4*>(lds + OFF_F + fb * 128 + swz(fb, k) * 16);
            const float4 d = *reinterpret_cast<const float4*>(lds + OFF_F + fd * 128 + swz(fd, k) * 16);
            const float4 f = *reinterpret_cast<const float4*>(lds + OFF_F + ff * 128 + swz(ff, k) * 16);
            float4 o;
#define UPL(X) o.X = ly.l0 * (lx.l0 * a.X + lx.l1 * b.X) + ly.l1 * (lx.l0 * d.X + lx.l1 * f.X);
            UPL(x) UPL(y) UPL(z) UPL(w)
#undef UPL
            (hf == 0 ? v0 : v1) = o;
          }
        }
      } else {
        const char* f = lds + OFF_F + r * 128;
        v0 = *reinterpret_cast<const float4*>(f + swz(r, 2 * c8) * 16);
        v1 = *reinterpret_cast<const float4*>(f + swz(r, 2 * c8 + 1) * 16);
      }
      if (gate) gate8_h4(v0, v1, h, t.pix0 + r, p.P, p.H * W, p.c1, ch * BK2 - p.c0 + c8 * 8);
      if (h.in_scale != nullptr) {   // fused BN + ReLU of the producer; rows outside the tensor stay 0
        const int pix = t.pix0 + r;
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
        const int pix = t.pix0 + r;
        if (r >= G::HALO && r < G::HALO + BM && pix < p.P) {
          _Float16* dst = h.xsplit + (size_t)pix * p.Cin + ch * BK2 + c8 * 8;
          *reinterpret_cast<half8*>(dst) = hv;
          *reinterpret_cast<half8*>(dst + xplane) = lv;
        }
      }
    }
  };

  // fragments carried from one tap to the next
  floatx4 acc[TI16][TJ16], part[TI16][TJ16];
  half8 ah[TI16], al[TI16], bh0, bl0, bh1, bl1;
  auto read_a = [&](unsigned pk, unsigned sbase, half8 (&xh)[TI16], half8 (&xl)[TI16]) {
#pragma unroll
    for (int i = 0; i < TI16; ++i) {
      const unsigned o = sbase + (i == 0 ? (pk & 0xffffu) : (pk >> 16));
      xh[i] = *reinterpret_cast<const half8*>(lds + o);
      xl[i] = *reinterpret_cast<const half8*>(lds + o + 64);
    }
  };

  // column blocks a B fragment pair is read ahead of its MFMAs: two where the registers allow (PRE;
  // BN = 64: half the accumulators), one with the convert path's registers at BN = 128
  constexpr int BPF = (PRE || BN == 64) ? 2 : 1;
  int slot0 = 0;   // ring slot of the chunk's tap 0 (taps use slots 0, 1, .., NBR - 1, 0, ... across chunks and tiles)
  int gch = 0;     // chunks this workgroup has run: PRE's S buffer of a chunk is gch & 1
  unsigned apk[9];

  // one tap of chunk ch of tile `cur`: MFMAs of column block j with the B fragments of block j + BPF
  // (or of the next tap) in flight; the next tap's A fragments read at block TJ16 / 2 - 1.  Its DMAs:
  // pieces of the next chunk's A tile (taps < TA) and the weights of tap tau + PD -- the next chunk being the
  // tile's own or, in its last chunk, the first chunk of the workgroup's next tile (`nxt`, `has_next`)
  auto tap = [&](const H4Tile& cur, const H4Tile& nxt, bool has_next, int ch, auto tap_tag) {
    constexpr int T = decltype(tap_tag)::value;
    const int slot = (slot0 + T) % NBR;
    const bool last = ch + 1 == cur.c_end;
    const H4Tile& tn = last ? nxt : cur;
    const int chn = last ? nxt.c_beg : ch + 1;
    const bool more = !last || has_next;
    const unsigned bcur = b_lane + (unsigned)(slot * BSLOT);
    const unsigned bnext = b_lane + (unsigned)(((slot + 1) % NBR) * BSLOT);
    const unsigned sb = PRE ? (unsigned)((gch & 1) * SSTRIDE) : 0u;
    const unsigned sbn = PRE ? (unsigned)(((gch + 1) & 1) * SSTRIDE) : 0u;
    // the tap's DMAs (H4_DMA_EARLY = 0: issued between MFMA groups -- block 1 in waves 0-3, block
    // TJ16 / 2 + 1 in waves 4-7, a SIMD's two waves being w and w + 4 -- so the two waves of a SIMD
    // issue them at different times, each under MFMAs already in the pipe)
    auto issue_tap = [&]() {
      if constexpr (!(SRPDE_CONV_DBG & 1)) {   // (timing-only diagnostics, conv_common.h: 1 = no DMA in the taps)
        if constexpr (T * APT < APW) {
#pragma unroll
          for (int a = 0; a < APT; ++a) issue_a(tn, chn, T * APT + a, more, (gch + 1) & 1);
        }
        constexpr int TP = T + PD;
        if constexpr (TP < 9) issue_b(cur.n0, ch, TP, (slot + PD) % NBR, true);
        else issue_b(tn.n0, chn, TP - 9, (slot + PD) % NBR, more);
      }
    };
    constexpr int JD0 = H4_DMA_EARLY ? 0 : 1, JD1 = H4_DMA_EARLY ? 0 : TJ16 / 2 + 1;
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
      // the next tap's A fragments: within the chunk; PRE also across it (the next chunk's S buffer has
      // landed: its pieces were issued at taps < APW and waited for by tap 7's end).  In a tile's last
      // chunk tap 8 reads them with this tile's offsets: unused, re-read after the epilogue.
      constexpr bool RA = j == TJ16 / 2 - 1 && (T < 8 || PRE);
      if constexpr (RA) read_a(apk[T < 8 ? T + 1 : 0], T < 8 ? sb : sbn, nah, nal);
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
      if constexpr (j == JD0 && JD0 == JD1) {
        issue_tap();
      } else {
        if constexpr (j == JD0) {
          if (wave < 4) issue_tap();
        }
        if constexpr (j == JD1) {
          if (wave >= 4) issue_tap();
        }
      }
    });
    if constexpr (T < 8 || PRE) {
#pragma unroll
      for (int i = 0; i < TI16; ++i) {
        ah[i] = nah[i];
        al[i] = nal[i];
      }
    }
    // after this barrier the next tap tau + 1 reads its own weights AND the first column blocks of tap
    // tau + 2's (issued at tap tau + 2 - PD): only the DMAs of the last WIN = PD - 2 taps may still be in
    // flight (exact counts: every wave issues nc(T) DMAs at tap T, zero fills included; the prologue
    // drained to 0; a tile's epilogue stores only add to the count, and loads complete in order, so
    // the wait never releases early).  Round 4 first allowed one tap more, so the bnext reads of
    // the following tap could see a slot before its DMA landed: a run-to-run race under load
    // (tools/diag_race.py: dgrad outputs changed in the first column blocks of a tile).
    // in flight after the wait: the DMAs of taps T - WIN + 1 .. T (every tap T' of a chunk issues nc(T'))
    constexpr auto nc = [](int t) { return NBD + ((t + 9) % 9 * APT < APW ? APT : 0); };
    constexpr int NCUR = [&] {
      int n = 0;
      for (int k = T - WIN + 1; k <= T; ++k) n += nc(k);
      return n;
    }();
    // a bare s_barrier: no lgkmcnt(0) drain of the next tap's fragment reads still in flight (they read
    // slot tau + 1 and the S tile, which no DMA issued after this barrier writes); the asm is a
    // compiler memory barrier, so no LDS read moves above it
    if constexpr (BAR2 && T % 2 == 0 && T != 8) {
      // no barrier: the last one (tap T - 1, or tap 8 of the previous chunk) covered this window's reads
    } else if constexpr (SRPDE_CONV_DBG & 2) {   // diagnostics: 2 = no tap barrier
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NCUR) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(NCUR) : "memory");
    }
  };

  // persistent: workgroup b takes items b, b + grid, ...; the first tile's first chunk and the weights of
  // its first PD taps are loaded here, every later tile's during the previous tile's last chunk
  if (H4_PRIO && wave >= 4) __builtin_amdgcn_s_setprio(1);   // the younger half: static priority
  stamp();
  int it = blockIdx.x;
  H4Tile cur = tile_of(it);
#pragma unroll
  for (int u = 0; u < APW; ++u) issue_a(cur, cur.c_beg, u, true, 0);
#pragma unroll
  for (int t = 0; t < PD; ++t) issue_b(cur.n0, cur.c_beg, t, t, true);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (!PRE) {
    convert(cur, cur.c_beg);
    __syncthreads();
  }

  while (true) {
    stamp();
    const int itn = it + (int)gridDim.x;
    const bool has_next = G::PERSIST && itn < nitems;
    const H4Tile nxt = has_next ? tile_of(itn) : cur;

    // per tap: the S offsets (relative to the S buffer) of this lane's A fragment (hi pieces; lo +64)
    // for its two 16-row blocks, 16 bits each; taps outside the image -> the zero row
#pragma unroll
    for (int t = 0; t < 9; ++t) apk[t] = 0;
#pragma unroll
    for (int i = 0; i < TI16; ++i) {
      const int rr = wm0 + i * 16 + l16;
      const int m = cur.m0 + rr;
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
#pragma unroll
    for (int i = 0; i < TI16; ++i)
#pragma unroll
      for (int j = 0; j < TJ16; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.f;
    read_a(apk[0], PRE ? (unsigned)((gch & 1) * SSTRIDE) : 0u, ah, al);
    {
      const unsigned bb = b_lane + (unsigned)(slot0 * BSLOT);
      bh0 = *reinterpret_cast<const half8*>(lds + bb);
      bl0 = *reinterpret_cast<const half8*>(lds + bb + BP);
      bh1 = *reinterpret_cast<const half8*>(lds + bb + 1024);
      bl1 = *reinterpret_cast<const half8*>(lds + bb + BP + 1024);
    }

    for (int ch = cur.c_beg; ch < cur.c_end; ++ch) {
      tap(cur, nxt, has_next, ch, std::integral_constant<int, 0>{});
      tap(cur, nxt, has_next, ch, std::integral_constant<int, 1>{});
      tap(cur, nxt, has_next, ch, std::integral_constant<int, 2>{});
      tap(cur, nxt, has_next, ch, std::integral_constant<int, 3>{});
      tap(cur, nxt, has_next, ch, std::integral_constant<int, 4>{});
      tap(cur, nxt, has_next, ch, std::integral_constant<int, 5>{});
      tap(cur, nxt, has_next, ch, std::integral_constant<int, 6>{});
      tap(cur, nxt, has_next, ch, std::integral_constant<int, 7>{});
      tap(cur, nxt, has_next, ch, std::integral_constant<int, 8>{});
      stamp();
      slot0 = (slot0 + 9) % NBR;
      ++gch;
      // two-level accumulation: one partial chain per channel chunk (9 taps x 32 channels)
#pragma unroll
      for (int i = 0; i < TI16; ++i)
#pragma unroll
        for (int j = 0; j < TJ16; ++j) acc[i][j] += part[i][j];
      if constexpr (!PRE) {
        if (ch + 1 < cur.c_end) {   // the next chunk's halo tile has landed in F (its DMAs preceded the last wait)
          if (!(SRPDE_CONV_DBG & 4)) convert(cur, ch + 1);   // diagnostics: 4 = no per-chunk convert
          __syncthreads();
          stamp();
          read_a(apk[0], 0u, ah, al);
        }
      }
    }

    floatx16 acc32[TI][TJ];
    acc16_to_32<TI, TJ>(acc, acc32);
    // the scales to undo: acc * 2^-(ea + wexp[col]) (conv_fwd_h3_kernel)
    float colscale[TJ];
    const float ia = exp2i(-ea);
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int col = cur.n0 + j * 32 + lr;
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
    } else {
      // scratch: the S buffer of the chunk just finished (no DMA targets it: the next tile's first chunk
      // went to F, or to the other S buffer), [2][WM][BN] floats of reduction, then 2 KiB per wave of store
      // stage; the next tile's DMAs in flight target the weight ring only
      float* scr = smem + (PRE ? ((gch + 1) & 1) * (SSTRIDE / 4) : 0);
      x6_finish<BM, BN, WM, WN, SRB>(p, acc32, cur.tail, cur.wg, nfull, cur.piece, cur.m0, cur.n0, wmi, wni, lane,
                                     scr, h.wide ? scr + 2 * WM * BN : nullptr, colscale);
    }
    stamp();
    if (!has_next) break;
    __syncthreads();   // every wave is past the epilogue's use of the scratch
    if constexpr (!PRE) {
      convert(nxt, nxt.c_beg);   // its halo tile landed in F during the last chunk
      __syncthreads();
    }
    cur = nxt;
    it = itn;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the trailing zero-fill DMAs, before the workgroup ends
}

// ---------------------------------- host side ---------------------------------------
template <int W, int DIL, int BN_, int SIGN, bool PRE, bool UP = false>
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
  // persistent: one workgroup per CU (LDS), each running items b, b + grid, ... (whole tiles, then the
  // K-pieces of the split tail)
  const int nitems = T - p.ntail + p.ntail * p.tsplit;
  const int grid = G::PERSIST ? std::min(nitems, cus) : nitems;
  note_kernel("conv_fwd_h4_kernel<%d, %d, %d, %d, %s, %s>", W, DIL, BN, SIGN, PRE ? "true" : "false", UP ? "true" : "false");
  hipLaunchKernelGGL((conv_fwd_h4_kernel<W, DIL, BN, SIGN, PRE, UP>), dim3(grid), dim3(512), G::template lds<PRE>(), st,
                     p, h);
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

bool h4_up_supported(int w, int dil, int cout) {
  return dil == 1 && cout % 64 == 0 && ((w == 20 && h4_bn(w, cout) == 128) || (w == 40 && h4_bn(w, cout) == 64));
}

int launch_fwd_h4(const ConvParams& p, const H3Args& h, bool pre, hipStream_t st, void* ws, size_t ws_bytes) {
  if (h.up_src != nullptr) {   // the upsampled input: the decoder's first convs (forward)
    if (!pre && p.sign > 0 && p.dil == 1 && p.W == 20 && h4_bn(20, p.Cout) == 128)
      return launch_h4_cfg<20, 1, 128, 1, false, true>(p, h, st, ws, ws_bytes);
    if (!pre && p.sign > 0 && p.dil == 1 && p.W == 40 && h4_bn(40, p.Cout) == 64)
      return launch_h4_cfg<40, 1, 64, 1, false, true>(p, h, st, ws, ws_bytes);
    set_error("srpde_conv_fwd_h3: no upsampled-input instantiation for W=%d dil=%d cout=%d", p.W, p.dil, p.Cout);
    return kErrArg;
  }
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
