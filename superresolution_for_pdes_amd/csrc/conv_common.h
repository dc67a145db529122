// srpde-mi355x: pieces shared by the implicit-GEMM convolution kernels (conv.hip, conv_h3.hip):
// the parameter block, LDS-DMA helpers, XCD-aware tile order, the K-split tail fixup and the
// bias/store/BN-statistics epilogue of the 32x32 MFMA accumulator tiles.
#pragma once
#include <algorithm>
#include <cstdlib>
#include "common.h"

// Timing-only diagnostics of the h3 kernels (phase ablation): a compile-time bit set,
// 0 in the product build -- an A/B library is built with SRPDE_EXTRA_FLAGS=-DSRPDE_CONV_DBG=<bits>
// (results wrong when non-zero).  1 = no DMA in the loop, 2 = no stage barrier, 4 = no per-chunk
// convert, 16 = no epilogue, 32 = no prologue halo DMA, 64 = no prologue convert, 128 = no MFMAs,
// 256 = phase timestamps past the output (h4; tools/h4_phase_ts.py), 512 = no input scale / shift loads in
// the h4 convert (identity BN).
#ifndef SRPDE_CONV_DBG
#define SRPDE_CONV_DBG 0
#endif

namespace srpde {

typedef float floatx16 __attribute__((ext_vector_type(16)));

struct ConvParams {
  const float* x0; int c0; int ldx0;
  const float* x1; int c1; int ldx1;
  const float* w;       // [Cout][taps][Cin] packed, Cin = c0 + c1
  const float* bias;    // [Cout] or null
  float* y; int ldy;    // output view
  float2* stats;        // [mblocks][Cout] (mean, M2) or null
  int N, H, W, Cout, ksize, dil, sign, accumulate;
  int P, K, Cin;
  // tail split (v2 only): the last `ntail` tiles are computed as `tsplit` K-pieces each,
  // written raw to `part`, and finished (sum, bias, store, BN partials) by conv_tail_fixup
  int ntail, tsplit;
  float* part;
  // optional fused BatchNorm-backward reduction (h3 dgrad): the output is the gradient of a
  // BN + ReLU output a = relu(gamma * (bn_y - mean) * invstd + beta); per (SRB-row block, channel)
  // the epilogue writes (sum dz, sum dz * xhat), dz = out * [a > 0], xhat = (bn_y - mean) * invstd
  const float* bn_y = nullptr;
  int bn_ldy = 0;
  const float* bn_mean = nullptr;
  const float* bn_invstd = nullptr;
  const float* bn_gamma = nullptr;
  const float* bn_beta = nullptr;
  float2* bn_part = nullptr;
  // optional: every output tile writes max|out| of its own elements to out_max[tile] (no atomics;
  // the consumer reduces the [ntiles] slots) -- the operand-scale bound of the BN backward that
  // reads this output next (srpde_bn_bwd_prepare)
  float* out_max = nullptr;
  // optional eval-mode BatchNorm + ReLU applied by the epilogue (models.py:22-23 with running
  // statistics): out = relu((conv + bias - mean) * invstd * gamma + beta), the expression of
  // bn_relu_fwd_kernel; ep_amax (nullable) receives max|out| (one atomicMax per workgroup)
  const float* ep_mean = nullptr;
  const float* ep_invstd = nullptr;
  const float* ep_gamma = nullptr;
  const float* ep_beta = nullptr;
  unsigned* ep_amax = nullptr;
};

// relu((v - mean) * invstd * gamma + beta): bn_relu_fwd_kernel's expression (bn.hip)
__device__ __forceinline__ float ep_bn_relu(float v, float mu, float is, float g, float b) {
  return fmaxf((v - mu) * is * g + b, 0.f);
}

__device__ __forceinline__ int xcd_remap(int bid, int total) {
  // bijective: blocks that share an A row-panel land on one XCD (MI355X L2 per XCD)
  const int xcd = bid & 7, q = total >> 3, r = total & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

typedef int int32x4 __attribute__((ext_vector_type(4)));

__device__ void llvm_raw_buffer_load_lds(int32x4 rsrc, __attribute__((address_space(3))) unsigned* lds, int size,
                                         int voffset, int soffset, int offset,
                                         int aux) __asm("llvm.amdgcn.raw.buffer.load.lds");

__device__ __forceinline__ int32x4 make_rsrc(const void* base, unsigned bytes) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(base);
  int32x4 r;
  r.x = (int)(unsigned)(a & 0xffffffffu);
  r.y = (int)(unsigned)((a >> 32) & 0xffffu);
  r.z = (int)bytes;
  r.w = 0x00020000;
  return r;
}

constexpr int BK2 = 32;                 // k per stage (one tap, 32 channels)
constexpr int ROW2 = BK2 * 4;           // 128-byte LDS rows
constexpr unsigned OOB = 0x80000000u;   // beyond num_records -> zero fill

__device__ __forceinline__ int swz(int r, int c) { return c ^ ((r >> 1) & 7); }

// One 16-B-per-lane LDS-DMA (buffer_load_dwordx4 ... lds) as inline asm.  Issued through the
// builtin, hipcc treats the DMA as an LDS store that may alias the following ds_reads and
// emits s_waitcnt vmcnt(0) right after it, serialising the prefetch behind the compute;
// as asm it is invisible to the waitcnt pass and we count vmcnt ourselves (vmcnt(0) before
// the stage barrier).  The wave-uniform LDS destination goes in M0 through the "{m0}" operand
// constraint, so the compiler allocates M0 (no save / restore); the s_nop covers the M0-write
// -> LDS-DMA read hazard the compiler cannot see inside the asm.
__device__ __forceinline__ void dma16(int32x4 rsrc, unsigned voff, unsigned lds_addr) {
  asm volatile(
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %0, %1, 0 offen lds"
      :
      : "v"(voff), "s"(rsrc), "{m0}"(__builtin_amdgcn_readfirstlane(lds_addr))
      : "memory");
}

__device__ __forceinline__ unsigned lds_addr_of(const void* p) {
  return (unsigned)(uintptr_t)((__attribute__((address_space(3))) const char*)p);
}

// Finish the split tail tiles: fixed-order sum of the K-pieces, bias, store (or accumulate),
// and the same per-row-block BN partials (mean, M2) the main epilogue writes.
// SRB = rows per BN-statistics block (srpde_conv_stats_rows_per_block); a tile of BM rows
// writes BM / SRB statistics rows.
// BMB: rows of the tile one block finishes (BM, or SRB with blockIdx.y the statistics sub-block: twice
// the blocks for the same work when the tail has few tiles; needs out_max == nullptr)
template <int BM, int BN, int SRB = BM, int BMB = BM>
__global__ __launch_bounds__(1024) void conv_tail_fixup_kernel(ConvParams p) {
  constexpr int CQ = BN / 4;          // column quads
  constexpr int G = 1024 / CQ;        // row groups
  constexpr int RPT = BMB / G;        // rows per thread
  constexpr int NSB = BMB / SRB;      // statistics sub-blocks per block
  static_assert(RPT >= 1 && BMB % G == 0 && BM % BMB == 0, "fixup geometry");
  static_assert(BMB % SRB == 0 && SRB % G == 0, "fixup statistics geometry");
  __shared__ float4 red[G][CQ];
  const int nbn = (p.Cout + BN - 1) / BN, nbm = (p.P + BM - 1) / BM;
  const int nfull = nbm * nbn - p.ntail;
  const int wg = nfull + blockIdx.x;
  const int mt = wg / nbn, nt = wg - mt * nbn;
  const int rbase = blockIdx.y * BMB;  // first tile row of this block
  const int m0 = mt * BM + rbase, n0 = nt * BN;
  const int cq = threadIdx.x % CQ, g = threadIdx.x / CQ;
  const int col = n0 + cq * 4;
  const bool cok = col < p.Cout;  // Cout % 4 == 0
  const float* src = p.part + (size_t)blockIdx.x * p.tsplit * (BM * BN);
  const float4 bias = (p.bias != nullptr && cok) ? *reinterpret_cast<const float4*>(p.bias + col)
                                                  : make_float4(0.f, 0.f, 0.f, 0.f);
  float4 v[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int r = g + i * G;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = 0; k < p.tsplit; ++k) {
      const float4 q = *reinterpret_cast<const float4*>(src + (size_t)k * (BM * BN) + (rbase + r) * BN + cq * 4);
      a.x += q.x; a.y += q.y; a.z += q.z; a.w += q.w;
    }
    a.x += bias.x; a.y += bias.y; a.z += bias.z; a.w += bias.w;
    if (p.ep_mean != nullptr && cok) {   // eval-mode BN + ReLU (see ConvParams)
      const int c = col;
      a.x = ep_bn_relu(a.x, p.ep_mean[c], p.ep_invstd[c], p.ep_gamma[c], p.ep_beta[c]);
      a.y = ep_bn_relu(a.y, p.ep_mean[c + 1], p.ep_invstd[c + 1], p.ep_gamma[c + 1], p.ep_beta[c + 1]);
      a.z = ep_bn_relu(a.z, p.ep_mean[c + 2], p.ep_invstd[c + 2], p.ep_gamma[c + 2], p.ep_beta[c + 2]);
      a.w = ep_bn_relu(a.w, p.ep_mean[c + 3], p.ep_invstd[c + 3], p.ep_gamma[c + 3], p.ep_beta[c + 3]);
    }
    v[i] = a;
    const int row = m0 + r;
    if (row < p.P && cok) {
      float* dst = p.y + (size_t)row * p.ldy + col;
      if (p.accumulate) {
        const float4 o = *reinterpret_cast<const float4*>(dst);
        *reinterpret_cast<float4*>(dst) = make_float4(o.x + a.x, o.y + a.y, o.z + a.z, o.w + a.w);
      } else {
        *reinterpret_cast<float4*>(dst) = a;
      }
    }
  }
  constexpr int IPS = RPT / NSB;      // a thread's rows per statistics sub-block
  if (p.ep_amax != nullptr) {         // max|out| of the block's rows -> one atomicMax
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < RPT; ++i)
      if (m0 + g + i * G < p.P && cok)
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[i].x), fabsf(v[i].y)), fmaxf(fabsf(v[i].z), fabsf(v[i].w))));
    red[g][cq] = make_float4(mx, 0.f, 0.f, 0.f);
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.f;
      for (int k = 0; k < G; ++k)
        for (int c = 0; c < CQ; ++c) t = fmaxf(t, red[k][c].x);
      atomicMax(p.ep_amax, __float_as_uint(t));
    }
    __syncthreads();
  }
  if (BMB == BM && p.out_max != nullptr) {   // max|out| of this tile -> its slot (whole-tile blocks only)
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < RPT; ++i)
      if (m0 + g + i * G < p.P && cok)
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[i].x), fabsf(v[i].y)), fmaxf(fabsf(v[i].z), fabsf(v[i].w))));
    red[g][cq] = make_float4(mx, 0.f, 0.f, 0.f);
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.f;
      for (int k = 0; k < G; ++k)
        for (int c = 0; c < CQ; ++c) t = fmaxf(t, red[k][c].x);
      p.out_max[wg] = t;
    }
    __syncthreads();
  }
  if (p.bn_part != nullptr) {         // fused BN-backward reduction (as x6_finish)
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 mu = cok ? *reinterpret_cast<const float4*>(p.bn_mean + col) : z4;
    const float4 is = cok ? *reinterpret_cast<const float4*>(p.bn_invstd + col) : z4;
    const float4 ga = cok ? *reinterpret_cast<const float4*>(p.bn_gamma + col) : z4;
    const float4 be = cok ? *reinterpret_cast<const float4*>(p.bn_beta + col) : z4;
#pragma unroll
    for (int sb = 0; sb < NSB; ++sb) {
      const int rb = m0 + sb * SRB;
      if (rb >= p.P) break;           // uniform over the block
      float4 s1 = z4, s2 = z4;
#pragma unroll
      for (int i = sb * IPS; i < (sb + 1) * IPS; ++i) {
        const int row = m0 + g + i * G;
        if (row < p.P && cok) {
          const float4 yv = *reinterpret_cast<const float4*>(p.bn_y + (size_t)row * p.bn_ldy + col);
          float xh, dz;
#define BNP_ACC(X)                                     \
  xh = (yv.X - mu.X) * is.X;                           \
  dz = __builtin_fmaf(xh, ga.X, be.X) > 0.f ? v[i].X : 0.f; \
  s1.X += dz;                                          \
  s2.X = __builtin_fmaf(dz, xh, s2.X);
          BNP_ACC(x) BNP_ACC(y) BNP_ACC(z) BNP_ACC(w)
#undef BNP_ACC
        }
      }
      red[g][cq] = s1;
      __syncthreads();
      float4 t1 = z4;
      if (g == 0)
        for (int k = 0; k < G; ++k) {
          const float4 q = red[k][cq];
          t1.x += q.x; t1.y += q.y; t1.z += q.z; t1.w += q.w;
        }
      __syncthreads();
      red[g][cq] = s2;
      __syncthreads();
      if (g == 0 && cok) {
        float4 t2 = z4;
        for (int k = 0; k < G; ++k) {
          const float4 q = red[k][cq];
          t2.x += q.x; t2.y += q.y; t2.z += q.z; t2.w += q.w;
        }
        float2* bp = p.bn_part + (size_t)(rb / SRB) * p.Cout + col;
        bp[0] = make_float2(t1.x, t2.x); bp[1] = make_float2(t1.y, t2.y);
        bp[2] = make_float2(t1.z, t2.z); bp[3] = make_float2(t1.w, t2.w);
      }
      __syncthreads();
    }
  }
  if (p.stats == nullptr) return;
#pragma unroll
  for (int sb = 0; sb < NSB; ++sb) {
    const int rb = m0 + sb * SRB;
    const int cnt = min(SRB, p.P - rb);
    if (cnt <= 0) break;              // uniform over the block
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = sb * IPS; i < (sb + 1) * IPS; ++i)
      if (m0 + g + i * G < p.P) { s.x += v[i].x; s.y += v[i].y; s.z += v[i].z; s.w += v[i].w; }
    red[g][cq] = s;
    __syncthreads();
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = 0; k < G; ++k) {
      const float4 q = red[k][cq];
      t.x += q.x; t.y += q.y; t.z += q.z; t.w += q.w;
    }
    const float inv = 1.f / (float)cnt;
    const float4 mean = make_float4(t.x * inv, t.y * inv, t.z * inv, t.w * inv);
    __syncthreads();
    float4 m2 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = sb * IPS; i < (sb + 1) * IPS; ++i) {
      if (m0 + g + i * G < p.P) {
        const float dx = v[i].x - mean.x, dy = v[i].y - mean.y, dz = v[i].z - mean.z, dw = v[i].w - mean.w;
        m2.x += dx * dx; m2.y += dy * dy; m2.z += dz * dz; m2.w += dw * dw;
      }
    }
    red[g][cq] = m2;
    __syncthreads();
    if (g == 0 && cok) {
      float4 u = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int k = 0; k < G; ++k) {
        const float4 q = red[k][cq];
        u.x += q.x; u.y += q.y; u.z += q.z; u.w += q.w;
      }
      float2* st = p.stats + (size_t)(rb / SRB) * p.Cout + col;
      st[0] = make_float2(mean.x, u.x); st[1] = make_float2(mean.y, u.y);
      st[2] = make_float2(mean.z, u.z); st[3] = make_float2(mean.w, u.w);
    }
    __syncthreads();
  }
}

// epilogue shared by the x6 / h3 forward kernels: raw tail-piece tiles, or bias + store + BN
// partial statistics per SRB rows.  Reduction scratch: smem[2][WM * TI][BN] floats.  `stage`
// (nullable): 2 KiB of LDS per wave, past the reduction scratch, through which the output leaves as 16-B row stores (needs ldy % 4 == 0 and
// a 16-B aligned y): 4 dwordx4 stores per lane and 32x32 block instead of 16 dword stores.
// `colscale` (nullable): per accumulator column block j, an exact power-of-two scale still to be
// applied (h3: the operand scales); it is fused with the bias into one FMA (bit-identical to the
// separate multiply and add, the multiply being exact).  A tile whose rows all lie inside the
// tensor (every tile but the last row tile) takes a path without per-row bounds checks.
template <int BM, int BN, int WM, int WN, int SRB, bool FULL>
__device__ __forceinline__ void x6_finish_body(const ConvParams& p, floatx16 (&acc)[BM / WM / 32][BN / WN / 32],
                                               int m0, int n0, int wmi, int wni, int lane, float* smem,
                                               float* stage, const float (&bcol)[BN / WN / 32]) {
  constexpr int TM = BM / WM, TN = BN / WN, TI = TM / 32, TJ = TN / 32;
  constexpr int NSB = BM / SRB, WPS = WM / NSB;
  const int lr = lane & 31, lh = lane >> 5;
  const int wm0 = wmi * TM, wn0 = wni * TN;
  auto row_ok = [&](int row) { return FULL || row < p.P; };
  // fused BN-backward reduction: issue every load of the BN input up front (clamped addresses,
  // masked in the sums) so they overlap each other and the stores instead of serialising
  float byv[TI][TJ][16];
  if (p.bn_part != nullptr) {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int col = min(n0 + wn0 + j * 32 + lr, p.Cout - 1);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row0 = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          const int row = FULL ? row0 : min(row0, p.P - 1);
          byv[i][j][r] = __builtin_nontemporal_load(p.bn_y + (size_t)row * p.bn_ldy + col);
        }
      }
  }
  if (stage != nullptr) {
    // each 16-row half of a wave's 32x32 block goes through the wave's LDS stage as [16][32]
    // floats and comes back as one float4 of a row per lane (8 lanes per 128-B row)
    float* st = stage + (wni * WM + wmi) * 512;
    const int rr = lane >> 3, c4 = (lane & 7) * 4;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int col = n0 + wn0 + j * 32 + c4;
        const bool cok = col < p.Cout;
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
          for (int r = 8 * hf; r < 8 * hf + 8; ++r)
            st[((r & 3) + 8 * ((r >> 2) & 1) + 4 * lh) * 32 + lr] = acc[i][j][r];
          __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the wave's stage writes are done
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const float4 v = *reinterpret_cast<const float4*>(st + (8 * k + rr) * 32 + c4);
            const int row = m0 + wm0 + i * 32 + 16 * hf + 8 * k + rr;
            if (row_ok(row) && cok) {
              float4* dst = reinterpret_cast<float4*>(p.y + (size_t)row * p.ldy + col);
              if (p.accumulate) {
                const float4 o = *dst;
                *dst = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
              } else {
                *dst = v;
              }
            }
          }
          __builtin_amdgcn_wave_barrier();
        }
      }
  } else {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int col = n0 + wn0 + j * 32 + lr;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (row_ok(row) && col < p.Cout) {
            float* dst = p.y + (size_t)row * p.ldy + col;
            *dst = p.accumulate ? *dst + acc[i][j][r] : acc[i][j][r];
          }
        }
      }
  }
  if (p.out_max != nullptr) {         // max|out| of this tile -> out_max[tile] (one store per workgroup)
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const bool cok = n0 + wn0 + j * 32 + lr < p.Cout;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (row_ok(row) && cok) mx = fmaxf(mx, fabsf(acc[i][j][r]));
        }
      }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    __syncthreads();                  // smem may still hold the store stage's last reads
    if (lane == 0) smem[wni * WM + wmi] = mx;
    __syncthreads();
    if (wmi == 0 && wni == 0 && lane == 0) {
      float t = 0.f;
      for (int k = 0; k < WM * WN; ++k) t = fmaxf(t, smem[k]);
      const int nbn = (p.Cout + BN - 1) / BN;
      p.out_max[(m0 / BM) * nbn + n0 / BN] = t;
    }
    __syncthreads();
  }
  if (p.ep_amax != nullptr) {         // max|out| of this tile -> one atomicMax per workgroup
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const bool cok = n0 + wn0 + j * 32 + lr < p.Cout;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (row_ok(row) && cok) mx = fmaxf(mx, fabsf(acc[i][j][r]));
        }
      }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    __syncthreads();                  // smem may still hold the store stage's last reads
    if (lane == 0) smem[wni * WM + wmi] = mx;
    __syncthreads();
    if (wmi == 0 && wni == 0 && lane == 0) {
      float t = 0.f;
      for (int k = 0; k < WM * WN; ++k) t = fmaxf(t, smem[k]);
      atomicMax(p.ep_amax, __float_as_uint(t));
    }
    __syncthreads();
  }
  if (p.bn_part != nullptr) {         // fused BN-backward reduction of the layer below (see ConvParams)
    float* red = smem;                // [2][WM * TI][BN]: one partial per 32-row block
    const int sb = wmi / WPS;
    const int rb0 = m0 + sb * SRB;
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int col = n0 + wn0 + j * 32 + lr;
      const bool cok = col < p.Cout;
      const float mu = cok ? p.bn_mean[col] : 0.f, is = cok ? p.bn_invstd[col] : 0.f;
      const float ga = cok ? p.bn_gamma[col] : 0.f, be = cok ? p.bn_beta[col] : 0.f;
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (row_ok(row) && cok) {
            // explicit FMAs: the same instructions in every kernel instantiation (equal bits)
            const float xh = (byv[i][j][r] - mu) * is;
            const float dz = __builtin_fmaf(xh, ga, be) > 0.f ? acc[i][j][r] : 0.f;
            s1 += dz;
            s2 = __builtin_fmaf(dz, xh, s2);
          }
        }
        s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 32, 64);
        if (lh == 0) {
          red[(wmi * TI + i) * BN + wn0 + j * 32 + lr] = s1;
          red[(WM + wmi) * TI * BN + i * BN + wn0 + j * 32 + lr] = s2;
        }
      }
    }
    __syncthreads();
    if (wmi % WPS == 0 && lh == 0 && rb0 < p.P) {
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int cl = wn0 + j * 32 + lr, col = n0 + cl;
        float t1 = 0.f, t2 = 0.f;
#pragma unroll
        for (int w = 0; w < WPS * TI; ++w) {
          t1 += red[(sb * WPS * TI + w) * BN + cl];
          t2 += red[WM * TI * BN + (sb * WPS * TI + w) * BN + cl];
        }
        if (col < p.Cout) p.bn_part[(size_t)(rb0 / SRB) * p.Cout + col] = make_float2(t1, t2);
      }
    }
    __syncthreads();
  }
  if (p.stats == nullptr) return;
  // per-32-row-block column partials [WM * TI][BN], combined in row order: the statistics of a
  // tile do not depend on how its rows are dealt to waves (equal bits across wave layouts)
  float* red = smem;
  const int sb = wmi / WPS;           // this wave's statistics sub-block
  const int rb0 = m0 + sb * SRB;
  const int cnt = FULL ? SRB : min(SRB, p.P - rb0);
  float mean[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j)
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      float s = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        s += row_ok(row) ? acc[i][j][r] : 0.f;
      }
      s += __shfl_xor(s, 32, 64);
      if (lh == 0) red[(wmi * TI + i) * BN + wn0 + j * 32 + lr] = s;
    }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < WPS * TI; ++w) s += red[(sb * WPS * TI + w) * BN + wn0 + j * 32 + lr];
    mean[j] = cnt > 0 ? s / (float)cnt : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < TJ; ++j)
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      float s = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const float d = acc[i][j][r] - mean[j];
        s = row_ok(row) ? __builtin_fmaf(d, d, s) : s;   // the same FMA on both paths (bit-equal tiles)
      }
      s += __shfl_xor(s, 32, 64);
      if (lh == 0) red[(wmi * TI + i) * BN + wn0 + j * 32 + lr] = s;
    }
  __syncthreads();
  if (wmi % WPS == 0 && lh == 0 && cnt > 0) {
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int cl = wn0 + j * 32 + lr, col = n0 + cl;
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < WPS * TI; ++w) s += red[(sb * WPS * TI + w) * BN + cl];
      if (col < p.Cout) p.stats[(size_t)(rb0 / SRB) * p.Cout + col] = make_float2(mean[j], s);
    }
  }
}

template <int BM, int BN, int WM, int WN, int SRB>
__device__ __forceinline__ void x6_finish(const ConvParams& p, floatx16 (&acc)[BM / WM / 32][BN / WN / 32], bool tail,
                                          int wg, int nfull, int piece, int m0, int n0, int wmi, int wni, int lane,
                                          float* smem, float* stage = nullptr, const float* colscale = nullptr) {
  constexpr int TM = BM / WM, TN = BN / WN, TI = TM / 32, TJ = TN / 32;
  const int lr = lane & 31, lh = lane >> 5;
  const int wm0 = wmi * TM, wn0 = wni * TN;
  if (tail) {
    float* dst = p.part + ((size_t)(wg - nfull) * p.tsplit + piece) * (BM * BN);
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const float cs = colscale ? colscale[j] : 1.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          dst[rl * BN + wn0 + j * 32 + lr] = acc[i][j][r] * cs;
        }
      }
    return;
  }

  // ---------------- epilogue: bias (fused with the operand scale), store, BN statistics --------
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
      const float cs = colscale ? colscale[j] : 1.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = __builtin_fmaf(acc[i][j][r], cs, bcol[j]);
    }
  if (p.ep_mean != nullptr) {         // eval-mode BN + ReLU (see ConvParams)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int col = n0 + wn0 + j * 32 + lr;
      const bool cok = col < p.Cout;
      const float mu = cok ? p.ep_mean[col] : 0.f, is = cok ? p.ep_invstd[col] : 0.f;
      const float ga = cok ? p.ep_gamma[col] : 0.f, be = cok ? p.ep_beta[col] : 0.f;
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = ep_bn_relu(acc[i][j][r], mu, is, ga, be);
    }
  }
  if (m0 + BM <= p.P)
    x6_finish_body<BM, BN, WM, WN, SRB, true>(p, acc, m0, n0, wmi, wni, lane, smem, stage, bcol);
  else
    x6_finish_body<BM, BN, WM, WN, SRB, false>(p, acc, m0, n0, wmi, wni, lane, smem, stage, bcol);
}

// ------------------------------ weight gradient --------------------------------
struct WgradParams {
  const float* dy; int lddy;          // [P][Cout] view
  const float* x0; int c0; int ldx0;  // forward input (virtual concat)
  const float* x1; int c1; int ldx1;
  float* part;                        // [splits][Cout][K]
  int N, H, W, Cout, ksize, dil;
  int P, K, Cin, chunk, splits;
};

// 16-bit MFMA operand images for the weight-gradient kernels: [pixel][column] rows of RB
// bytes, read back transposed (8 consecutive pixels of one column per lane)
template <int RB>
__device__ __forceinline__ int wx_off(int row, int ch) {   // byte offset of 16-B chunk ch of a row
  constexpr int sh = RB >= 256 ? 0 : (RB == 128 ? 1 : -1);
  const int s = sh < 0 ? 0 : (((row >> sh) & 3) << 2) & (RB / 16 - 1);
  return row * RB + 16 * (ch ^ s);
}

template <typename V, int RB>
__device__ __forceinline__ V tr_frag(const char* img, int col0, int lane) {
  // 8 k-values (pixels 8h .. 8h+7) of column col0 + (lane & 31): two transposed 4-row reads
  const int h = lane >> 5, q = (lane & 15) >> 2, pp = lane & 3;
  const int col = col0 + (lane & 16) + 4 * pp;   // this lane's 4-column address slot
  typedef short v4i16 __attribute__((ext_vector_type(4)));
  const int o0 = wx_off<RB>(8 * h + q, col >> 3) + 2 * (col & 7);
  const int o1 = wx_off<RB>(8 * h + 4 + q, col >> 3) + 2 * (col & 7);
  const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4i16*)(uintptr_t)lds_addr_of(img + o0));
  const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4i16*)(uintptr_t)lds_addr_of(img + o1));
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  const v8i16 c = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  return __builtin_bit_cast(V, c);
}

// h3 weight-gradient launcher (conv_h3.hip): raw scaled-back slabs into p.part
int launch_wgrad_h3(const WgradParams& p, const unsigned* amax_dy, const unsigned* amax0, const unsigned* amax1,
                    hipStream_t st);

// fixed-order sum of split-K weight-gradient slabs [splits][Cout][taps*Cin] into torch's
// [Cout][Cin_real][k][k] layout (conv.hip)
int wgrad_reduce(const float* part, float* dw, int splits, int cout, int cin, int cin_real, int taps, int accumulate,
                 hipStream_t stream);

// ---------------- host: K-split of the last, under-filled round of tiles ----------------
// tail split plan shared by the LDS-DMA forward kernels (see launch_fwd_v2)
static void plan_tail(ConvParams& p, int T, int slots, int BM, int BN, void* ws, size_t ws_bytes) {
  p.ntail = 0; p.tsplit = 1; p.part = nullptr;
  const int nall = p.K / BK2;
  const int rem = T % slots;
  if (T >= slots && rem > 0 && 2 * rem <= slots && ws != nullptr) {
    int F = std::min(std::min(slots / rem, nall / 2), 8);
    while (F >= 2 && (size_t)rem * F * BM * BN * sizeof(float) > ws_bytes) --F;
    if (F >= 2) { p.ntail = rem; p.tsplit = F; p.part = static_cast<float*>(ws); }
  }
}

}  // namespace srpde
