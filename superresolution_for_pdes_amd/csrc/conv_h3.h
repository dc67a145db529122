// srpde-mi355x: device pieces shared by the h3 convolution kernels (conv_h3.hip, conv_h4.hip):
// the fp16 two-piece split, the B-tile swizzle, the 16x16 -> 32x32 accumulator regrouping and
// the kernel argument block.  Arithmetic and layouts: conv_h3.hip header comment.
#pragma once
#include "conv_common.h"
#include "resample.h"

namespace srpde {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split2h(const float4 a, const float4 b, float s, half8& hi, half8& lo) {
  const float v[8] = {a.x * s, a.y * s, a.z * s, a.w * s, b.x * s, b.y * s, b.z * s, b.w * s};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const _Float16 h = (_Float16)v[k];
    hi[k] = h;
    lo[k] = (_Float16)(v[k] - (float)h);
  }
}

// 32-half (64-B) weight rows: 16-B chunk c of row r sits in slot c ^ g((r >> 2) & 3), g = (0, 2, 3, 1):
// conflict-free for the 16x16x32 B-fragment reads (lane: row (lane & 15), chunk lane >> 4) of every
// ds_read_b128 lane group (MI355X_MICROARCH.md, LDS table)
__device__ __forceinline__ int swzh(int r, int c) { return c ^ ((0x78 >> (2 * ((r >> 2) & 3))) & 3); }

typedef float floatx4 __attribute__((ext_vector_type(4)));

// The main loops run v_mfma_f32_16x16x32_f16 (one 32-channel chunk of a tap per instruction): at
// equal cycles per FLOP the 16x16 shape holds a higher clock under load on random data than
// 32x32x16 (tools/mfma_peak.hip: 2058 vs 1791-1861 TF dense, profiles/r03_mfma_shapes.txt).  The
// epilogue (x6_finish) keeps the 32x32x16 accumulator layout; a 32x32 block is four 16x16 blocks
// (a, b) (rows 16a.., cols 16b..), regrouped in registers by two lane swaps per dword:
// X = (a, 0), Y = (a, 1) at one element q -> permlane16_swap -> permlane32_swap gives the 32x32
// elements 4 (2a) + q and 4 (2a + 1) + q.
template <int TI, int TJ>
__device__ __forceinline__ void acc16_to_32(const floatx4 (&a16)[2 * TI][2 * TJ], floatx16 (&a32)[TI][TJ]) {
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const auto r1 = __builtin_amdgcn_permlane16_swap(__float_as_uint(a16[2 * i + a][2 * j][q]),
                                                           __float_as_uint(a16[2 * i + a][2 * j + 1][q]), false, false);
          const auto r2 = __builtin_amdgcn_permlane32_swap(r1[0], r1[1], false, false);
          a32[i][j][8 * a + q] = __uint_as_float(r2[0]);
          a32[i][j][8 * a + 4 + q] = __uint_as_float(r2[1]);
        }
}

struct H3Args {
  const _Float16* wsp;     // [2][Cout][K] hi / lo planes
  const int* wexp;         // [Cout] weight scale exponents
  const unsigned* amax0;   // max|x0| (float bits), or null
  const unsigned* amax1;   // max|x1|, or null
  int halo;                // (W + 1) * dil
  int arows;               // BM + 2 * halo, rounded up to 8 (<= 512: at most 8 slices per wave)
  int relax;               // 1: a stage waits only for its weight DMA (halo slices land later)
  _Float16* xsplit;        // optional [2][P][Cin] hi / lo planes of the (scaled) input, written
                           // as a by-product of the split for the weight-gradient kernel
  const float* in_scale;   // optional per-channel affine + ReLU applied to x0 in the split
  const float* in_shift;   // (the producing BatchNorm, fused; c1 == 0)
  int wide;                // 1: the epilogue stores 16-B rows through LDS (ldy % 4 == 0, y 16-B aligned)
  // BNB kernels (dgrad with the BatchNorm(+ReLU) backward apply fused into the operand transform):
  // x0 is the gradient da of the BN + ReLU output; the operand is
  //   dy = gamma*invstd * (dz - m1 - xhat*m2),  xhat = (y - mean)*invstd,  dz = da * [xhat*gamma + beta > 0]
  // (m1 = m2 = 0 in eval mode), computed per halo element from a second fp32 halo tile of y
  const float* bnb_y; int bnb_ldy;
  const float* bnb_mean; const float* bnb_invstd; const float* bnb_gamma; const float* bnb_beta;
  const float* bnb_m1; const float* bnb_m2;
  int bnb_relu;
  // optional AttentionGate of a virtual concat's second input, fused into the input transform
  // (models.py:119-130 feeding dec*.conv1 at :87,:90,:93): x1 element (p, c) enters as
  // (x1[p][c] * ca[n][c]) * sa[p], n = p / (H W) -- att_apply_kernel's expression (pointwise.hip)
  const float* x1_ca;      // [N][c1]
  const float* x1_sa;      // [P]
  // optional: x0 is up(x0_up), the bilinear x2 (align_corners) upsample of an [N][up_h][up_w] NHWC
  // tensor (row stride up_ld), formed in the operand transform (models.py:70,89,92: the decoder's
  // upsampled input is never written)
  const float* up_src;
  int up_ld, up_h, up_w;
};

// the gate above on 8 consecutive channels cc1.. (channel index inside x1) of pixel pix; rows
// outside the tensor are left alone (they are zero fills)
__device__ __forceinline__ void gate8(float4& v0, float4& v1, const H3Args& h, int pix, int P, int HW, int c1,
                                      int cc1) {
  if (pix < 0 || pix >= P) return;
  const int n = pix / HW;
  const float4 a0 = *reinterpret_cast<const float4*>(h.x1_ca + (size_t)n * c1 + cc1);
  const float4 a1 = *reinterpret_cast<const float4*>(h.x1_ca + (size_t)n * c1 + cc1 + 4);
  const float s = h.x1_sa[pix];
  v0.x = (v0.x * a0.x) * s; v0.y = (v0.y * a0.y) * s; v0.z = (v0.z * a0.z) * s; v0.w = (v0.w * a0.w) * s;
  v1.x = (v1.x * a1.x) * s; v1.y = (v1.y * a1.y) * s; v1.z = (v1.z * a1.z) * s; v1.w = (v1.w * a1.w) * s;
}

// gate8 with the pixel's sample index n known (no division by H W; h5 has it from the tile index)
__device__ __forceinline__ void gate8n(float4& v0, float4& v1, const H3Args& h, int n, int pix, int c1, int cc1) {
  if (pix < 0) return;
  const float4 a0 = *reinterpret_cast<const float4*>(h.x1_ca + (size_t)n * c1 + cc1);
  const float4 a1 = *reinterpret_cast<const float4*>(h.x1_ca + (size_t)n * c1 + cc1 + 4);
  const float s = h.x1_sa[pix];
  v0.x = (v0.x * a0.x) * s; v0.y = (v0.y * a0.y) * s; v0.z = (v0.z * a0.z) * s; v0.w = (v0.w * a0.w) * s;
  v1.x = (v1.x * a1.x) * s; v1.y = (v1.y * a1.y) * s; v1.z = (v1.z * a1.z) * s; v1.w = (v1.w * a1.w) * s;
}

// the K-split tail's fixup: one block per statistics sub-block of each tail tile (twice the blocks of a
// whole-tile fixup for the same work: the tail has few tiles; 32.15 -> 32.12 ms per step) unless the
// per-tile max|out| slot is wanted
template <int BM, int BN, int SRB>
static int launch_tail_fixup(const ConvParams& p, hipStream_t st) {
  if constexpr (BM > SRB) {
    if (p.out_max == nullptr) {
      hipLaunchKernelGGL((conv_tail_fixup_kernel<BM, BN, SRB, SRB>), dim3(p.ntail, BM / SRB), dim3(1024), 0, st, p);
      SRPDE_LAUNCH_CHECK("srpde_conv_fwd_h3(tail fixup)");
      return 0;
    }
  }
  hipLaunchKernelGGL((conv_tail_fixup_kernel<BM, BN, SRB>), dim3(p.ntail), dim3(1024), 0, st, p);
  SRPDE_LAUNCH_CHECK("srpde_conv_fwd_h3(tail fixup)");
  return 0;
}

// h4 (conv_h4.hip): the 256 x 128 forward / dgrad kernel for the shapes it is instantiated for
bool h4_supported(int w, int dil, int cout, bool bnb);
bool h4_up_supported(int w, int dil, int cout);   // the upsampled-input forward (H3Args::up_src)
int launch_fwd_h4(const ConvParams& p, const H3Args& h, bool pre, hipStream_t st, void* ws, size_t ws_bytes);

// kernel-family bits of srpde_conv_fwd_h3's / srpde_conv_fwd_h3_presplit's `accumulate` argument (bit 0 is the
// accumulate flag itself) and of srpde_conv_h3_stats_rows_for's `flags`: per call, no library state.  The families
// compute the same outputs bit for bit; the bits let tests compare them and tuning time them.
constexpr int FAM_NO_H5 = 2, FAM_NO_H4 = 4, FAM_NO_H3R = 8, FAM_MASK = FAM_NO_H5 | FAM_NO_H4 | FAM_NO_H3R;

// the 16-output forward of out_conv2 in training (conv_head.hip): c0 == 32, c1 == 0, cout == 16, w <= 63
// (taken with the h5 kernels: FAM_NO_H5 routes it back to h3r)
bool n16_supported(int c0, int c1, int cout, int w, int dil);
int launch_fwd_n16(const ConvParams& p, const H3Args& h, hipStream_t st);
// h5 (conv_h5.hip): the W = 40 forward into 64 / 32 channels (8-row tiles, weight taps through an LDS ring)
bool h5_supported(int c0, int c1, int cout, int h, int w, int dil);
int h5_stats_rows();
int launch_fwd_h5(const ConvParams& p, const H3Args& h, hipStream_t st);

}  // namespace srpde
