// Variants of upsample_gate_fwd_px_kernel (pointwise.hip) for the cross-process corruption hunt
// (tools/race_up.py UPMODE=k0..k4): which ingredient makes its output unrepeatable while another
// process runs the h3 convolutions.  Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC.
#include <hip/hip_runtime.h>

struct Lerp { int i0, i1; float l0, l1; };
__device__ __forceinline__ Lerp lerp_index(unsigned o, int n, int no) {
  Lerp r;
  const float s = no > 1 ? (float)(n - 1) / (float)(no - 1) : 0.f;
  const float f = s * (float)o;
  r.i0 = (int)f;
  r.i1 = r.i0 < n - 1 ? r.i0 + 1 : r.i0;
  r.l1 = f - (float)r.i0;
  r.l0 = 1.f - r.l1;
  return r;
}

// MODE 0: as pointwise.hip; 1: out stored after the reduction; 2: no reduction (dummy sa);
// 3: no reduction, a dummy ds_bpermute after the store; 4: no reduction, a static LDS round trip
template <int MODE>
__global__ __launch_bounds__(256) void victim_kernel(const float* __restrict__ x, int ldx, float* __restrict__ out,
                                                     int ldo, unsigned npix, int H, int W, int Ho, int Wo,
                                                     const float* __restrict__ wg, const float* __restrict__ bg,
                                                     float* __restrict__ sa) {
  const unsigned q = blockIdx.x * blockDim.y + threadIdx.y;
  const bool on = q < npix;
  const unsigned qq = on ? q : 0;
  const unsigned ox = qq % (unsigned)Wo, t = qq / (unsigned)Wo, oy = t % (unsigned)Ho, n = t / (unsigned)Ho;
  const int c = threadIdx.x * 4;
  const Lerp ly = lerp_index(oy, H, Ho), lx = lerp_index(ox, W, Wo);
  const float* base = x + (size_t)n * H * W * ldx + c;
  const float4 a = *reinterpret_cast<const float4*>(base + (size_t)(ly.i0 * W + lx.i0) * ldx);
  const float4 b = *reinterpret_cast<const float4*>(base + (size_t)(ly.i0 * W + lx.i1) * ldx);
  const float4 d = *reinterpret_cast<const float4*>(base + (size_t)(ly.i1 * W + lx.i0) * ldx);
  const float4 f = *reinterpret_cast<const float4*>(base + (size_t)(ly.i1 * W + lx.i1) * ldx);
  float4 o;
#define UP(X) o.X = ly.l0 * (lx.l0 * a.X + lx.l1 * b.X) + ly.l1 * (lx.l0 * d.X + lx.l1 * f.X);
  UP(x) UP(y) UP(z) UP(w)
#undef UP
  if (MODE != 1 && on) *reinterpret_cast<float4*>(out + (size_t)q * ldo + c) = o;
  const float4 wv = *reinterpret_cast<const float4*>(wg + c);
  float acc = o.x * wv.x + o.y * wv.y + o.z * wv.z + o.w * wv.w;
  if (MODE <= 1) {
    for (int off = 1; off < (int)blockDim.x; off <<= 1) acc += __shfl_xor(acc, off, 64);
  } else if (MODE == 3) {
    acc += __shfl_xor(acc, 1, 64);
  } else if (MODE == 4) {
    __shared__ float s[256];
    const int tid = threadIdx.y * blockDim.x + threadIdx.x;
    s[tid] = acc;
    __syncthreads();
    acc += s[tid ^ 1];
  }
  if (on && threadIdx.x == 0) sa[q] = 1.f / (1.f + expf(-(acc + bg[0])));
  if (MODE == 1 && on) *reinterpret_cast<float4*>(out + (size_t)q * ldo + c) = o;
}

extern "C" int victim_upsample_gate(int mode, const float* x, float* out, int n, int h, int w, int c,
                                    const float* wg, const float* bg, float* sa, hipStream_t st) {
  const int c4 = c / 4, py = 256 / c4, ho = 2 * h, wo = 2 * w;
  const unsigned npix = (unsigned)(n * ho * wo);
  dim3 g((npix + py - 1) / py), blk(c4, py);
#define L(M) hipLaunchKernelGGL(victim_kernel<M>, g, blk, 0, st, x, c, out, c, npix, h, w, ho, wo, wg, bg, sa)
  switch (mode) {
    case 0: L(0); break;
    case 1: L(1); break;
    case 2: L(2); break;
    case 3: L(3); break;
    default: L(4); break;
  }
#undef L
  return (int)hipGetLastError();
}

// Noise: LDS-DMA loops (16-B per lane buffer_load ... lds, as conv_common.h's dma16), every access
// in bounds (mode 0) or out of range -> zero fill (mode 1); mode 2: plain global loads, no LDS-DMA
typedef int v4i __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void dma_noise_kernel(const float* src, unsigned bytes, int iters, int mode,
                                                        float* sinkout) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const unsigned long long a = reinterpret_cast<unsigned long long>(src);
  v4i r;
  r.x = (int)(unsigned)(a & 0xffffffffu);
  r.y = (int)(unsigned)((a >> 32) & 0xffffu);
  r.z = (int)bytes;
  r.w = 0x00020000;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  float acc = 0.f;
  for (int it = 0; it < iters; ++it) {
    const unsigned row = (blockIdx.x * 4 + wave + it * 977u) % (bytes / 1024u);
    const unsigned off = mode == 1 ? 0x80000000u : row * 1024u + lane * 16u;
    if (mode == 2) {
      const float4 v = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(src) + off);
      acc += v.x;
    } else {
      const unsigned lds = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)(smem) + (wave * 4 + (it & 3)) * 1024);
      asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" : : "v"(off), "s"(r),
                   "{m0}"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
      if ((it & 3) == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  acc += smem[threadIdx.x];
  if (acc == 12345.f) sinkout[0] = acc;
}

extern "C" int dma_noise(int mode, const float* src, unsigned bytes, int blocks, int iters, float* sinkout,
                         hipStream_t st) {
  hipLaunchKernelGGL(dma_noise_kernel, dim3(blocks), dim3(256), 16 * 1024, st, src, bytes, iters, mode, sinkout);
  return (int)hipGetLastError();
}

// Noise: mode 3 = v_permlane16_swap / v_permlane32_swap loops (as conv_h3.hip's acc16_to_32);
// mode 4 = 16x16x32 f16 MFMA chains
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void valu_noise_kernel(int iters, int mode, float* sinkout) {
  unsigned x0 = threadIdx.x * 2654435761u, x1 = x0 ^ 0x9e3779b9u;
  f4 c = {0.f, 0.f, 0.f, 0.f};
  h8 a, b;
  for (int k = 0; k < 8; ++k) { a[k] = (_Float16)(threadIdx.x * 0.01f + k); b[k] = (_Float16)(k * 0.5f); }
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  typedef __bf16 b8 __attribute__((ext_vector_type(8)));
  typedef float f16v __attribute__((ext_vector_type(16)));
  h4 a4 = {a[0], a[1], a[2], a[3]}, b4 = {b[0], b[1], b[2], b[3]};
  b8 ab, bb;
  for (int k = 0; k < 8; ++k) { ab[k] = (__bf16)(float)a[k]; bb[k] = (__bf16)(float)b[k]; }
  const float fa = threadIdx.x * 0.001f, fb = 0.5f;
  f16v c16 = {};
  for (int it = 0; it < iters; ++it) {
    if (mode == 3) {
      const auto r1 = __builtin_amdgcn_permlane16_swap(x0, x1, false, false);
      const auto r2 = __builtin_amdgcn_permlane32_swap(r1[0], r1[1], false, false);
      x0 = r2[0] + 1u;
      x1 = r2[1] ^ (unsigned)it;
    } else if (mode == 4) {
      c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    } else if (mode == 5) {
      c16 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c16, 0, 0, 0);
    } else if (mode == 6) {
      c = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c, 0, 0, 0);
    } else if (mode == 7) {
      c16 = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, b4, c16, 0, 0, 0);
    } else if (mode == 8) {
      c = __builtin_amdgcn_mfma_f32_16x16x4f32(fa, fb, c, 0, 0, 0);
    } else {
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, c, 0, 0, 0);
    }
  }
  if (x0 == 12345u || c[0] == 12345.f || c16[3] == 12345.f) sinkout[0] = (float)x1 + c[1];
}

extern "C" int valu_noise(int mode, int blocks, int iters, float* sinkout, hipStream_t st) {
  hipLaunchKernelGGL(valu_noise_kernel, dim3(blocks), dim3(256), 0, st, iters, mode, sinkout);
  return (int)hipGetLastError();
}
