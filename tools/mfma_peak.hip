// Sustained dense MFMA rate on this MI355X: v_mfma_f32_32x32x16_f16 chains with no memory
// traffic, 2 or 4 waves per SIMD, every CU busy.  Sets the practical ceiling the conv kernels
// are measured against (tools/gpu_mfma_peak.sh).
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_peak.hip -o tools/mfma_peak && ./tools/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int CHAINS>
__global__ __launch_bounds__(512, 1) void mfma_loop(float* out, int iters) {
  extern __shared__ float lds_unused[];
  if (iters < 0) lds_unused[threadIdx.x] = 0.f;
  half8 a, b;
  for (int k = 0; k < 8; ++k) {
    a[k] = (_Float16)(threadIdx.x * 1e-3f + k);
    b[k] = (_Float16)(k * 0.5f);
  }
  floatx16 acc[CHAINS];
  for (int c = 0; c < CHAINS; ++c)
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[c], 0, 0, 0);
  }
  float s = 0.f;
  for (int c = 0; c < CHAINS; ++c)
    for (int r = 0; r < 16; ++r) s += acc[c][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// the conv kernels' pattern: per (i, j) tile a chain of three dependent products
// (al*bh -> +ah*bl -> +ah*bh) on its partial accumulator, TILES tiles per wave
template <int TILES>
__global__ __launch_bounds__(512, 1) void mfma_chain3(float* out, int iters) {
  extern __shared__ float lds_unused[];
  if (iters < 0) lds_unused[threadIdx.x] = 0.f;
  half8 a0, a1, b0, b1;
  for (int k = 0; k < 8; ++k) {
    a0[k] = (_Float16)(threadIdx.x * 1e-3f + k);
    a1[k] = (_Float16)(threadIdx.x * 2e-3f - k);
    b0[k] = (_Float16)(k * 0.5f);
    b1[k] = (_Float16)(k * 0.25f + 1.f);
  }
  floatx16 acc[TILES];
  for (int c = 0; c < TILES; ++c)
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < TILES; ++c) {
      floatx16 c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, acc[c], 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, c0, 0, 0, 0);
      acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, c0, 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int c = 0; c < TILES; ++c)
    for (int r = 0; r < 16; ++r) s += acc[c][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// realistic operand toggling: each iteration's fragments are fresh pseudo-random fp16 bit patterns
// (an LCG in the low mantissa bits of precomputed values), as the conv kernels' data are
template <int TILES>
__global__ __launch_bounds__(512, 1) void mfma_random(float* out, int iters) {
  extern __shared__ float lds_unused[];
  if (iters < 0) lds_unused[threadIdx.x] = 0.f;
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  u32x4 ra, rb;
  unsigned seed = threadIdx.x * 2654435761u + blockIdx.x * 40503u;
  for (int k = 0; k < 4; ++k) {
    seed = seed * 1664525u + 1013904223u; ra[k] = (seed & 0x03ff03ffu) | 0x38003800u;
    seed = seed * 1664525u + 1013904223u; rb[k] = (seed & 0x03ff03ffu) | 0x38003800u;
  }
  floatx16 acc[TILES];
  for (int c = 0; c < TILES; ++c)
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  for (int it = 0; it < iters; ++it) {
    const u32x4 ma = (u32x4){(unsigned)it * 0x00010001u, (unsigned)it * 0x00030003u, (unsigned)it * 0x00050005u,
                             (unsigned)it * 0x00070007u} & 0x03ff03ffu;
    const half8 a = __builtin_bit_cast(half8, ra ^ ma), b = __builtin_bit_cast(half8, rb ^ (ma << 1));
    const half8 a2 = __builtin_bit_cast(half8, ra ^ (ma >> 1)), b2 = __builtin_bit_cast(half8, rb ^ (ma << 2));
#pragma unroll
    for (int c = 0; c < TILES; ++c) {
      floatx16 c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a2, b, acc[c], 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b2, c0, 0, 0, 0);
      acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int c = 0; c < TILES; ++c)
    for (int r = 0; r < 16; ++r) s += acc[c][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}


// the same work as mfma_random on v_mfma_f32_16x16x32_f16 (MI355X_MICROARCH.md: the 16x16 shape holds
// a higher clock under load on random data): per 32x32 tile-equivalent two independent 16x16
// accumulators, each a chain of three products, per iteration (equal FLOP per iteration)
typedef float floatx4 __attribute__((ext_vector_type(4)));
template <int TILES>
__global__ __launch_bounds__(512, 1) void mfma_random16(float* out, int iters) {
  extern __shared__ float lds_unused[];
  if (iters < 0) lds_unused[threadIdx.x] = 0.f;
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  u32x4 ra, rb;
  unsigned seed = threadIdx.x * 2654435761u + blockIdx.x * 40503u;
  for (int k = 0; k < 4; ++k) {
    seed = seed * 1664525u + 1013904223u; ra[k] = (seed & 0x03ff03ffu) | 0x38003800u;
    seed = seed * 1664525u + 1013904223u; rb[k] = (seed & 0x03ff03ffu) | 0x38003800u;
  }
  floatx4 acc[2 * TILES];
  for (int c = 0; c < 2 * TILES; ++c)
    for (int r = 0; r < 4; ++r) acc[c][r] = 0.f;
  for (int it = 0; it < iters; ++it) {
    const u32x4 ma = (u32x4){(unsigned)it * 0x00010001u, (unsigned)it * 0x00030003u, (unsigned)it * 0x00050005u,
                             (unsigned)it * 0x00070007u} & 0x03ff03ffu;
    const half8 a = __builtin_bit_cast(half8, ra ^ ma), b = __builtin_bit_cast(half8, rb ^ (ma << 1));
    const half8 a2 = __builtin_bit_cast(half8, ra ^ (ma >> 1)), b2 = __builtin_bit_cast(half8, rb ^ (ma << 2));
#pragma unroll
    for (int c = 0; c < 2 * TILES; ++c) {
      floatx4 c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2, b, acc[c], 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b2, c0, 0, 0, 0);
      acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c0, 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int c = 0; c < 2 * TILES; ++c)
    for (int r = 0; r < 4; ++r) s += acc[c][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
static void timeit(const char* name, K kern, int blocks, float* out, int iters, double mfma_per_iter,
                   size_t lds = 0) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(512), lds, 0, out, iters);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(512), lds, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 32 * 32 * 16 * mfma_per_iter * iters * (blocks * 8.0);
  printf("%-40s %.3f ms  %.1f TFLOP/s dense  (%.1f%% of 2516.8)\n", name, ms, flops / ms / 1e9,
         100.0 * flops / ms / 1e9 / 2516.8);
}

int main() {
  int dev = 0, cus = 0, clk = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
  float* out;
  const int blocks = cus * 4;   // 4 rounds of one 512-thread block per CU
  hipMalloc(&out, sizeof(float) * blocks * 512);
  const int iters = 20000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL((mfma_loop<4>), dim3(blocks), dim3(512), 0, 0, out, iters);
    hipEventRecord(e0);
    hipLaunchKernelGGL((mfma_loop<4>), dim3(blocks), dim3(512), 0, 0, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = 2.0 * 32 * 32 * 16 * 4.0 * iters * (blocks * 8.0);   // per wave: 4 chains x iters
    printf("fp16 32x32x16 MFMA, 8 waves/CU, %d CUs (clock attr %d kHz): %.3f ms, %.1f TFLOP/s dense "
           "(%.1f TF fp32-product units at 3 products)\n",
           cus, clk, ms, flops / ms / 1e9, flops / ms / 1e9 / 3);
  }
  timeit("chains of 3 dependent, 1 tile/wave", mfma_chain3<1>, blocks, out, 8000, 3);
  timeit("chains of 3 dependent, 2 tiles/wave", mfma_chain3<2>, blocks, out, 4000, 6);
  timeit("chains of 3 dependent, 4 tiles/wave", mfma_chain3<4>, blocks, out, 2000, 12);
  timeit("1 independent chain/wave", mfma_loop<1>, blocks, out, 20000, 1);
  // one 512-thread workgroup per CU (100 KB of LDS each): 2 waves per SIMD, as the conv kernels
  timeit("3-chains x4, 1 WG/CU (2 waves/SIMD)", mfma_chain3<4>, blocks, out, 2000, 12, 100 * 1024);
  timeit("4 chains, 1 WG/CU (2 waves/SIMD)", mfma_loop<4>, blocks, out, 5000, 4, 100 * 1024);
  timeit("random operands, 3-chains x4, 1 WG/CU", mfma_random<4>, blocks, out, 2000, 12, 100 * 1024);
  timeit("random operands, 3-chains x4, 1 WG/CU", mfma_random<4>, blocks, out, 8000, 12, 100 * 1024);
  // flops counted in 32x32x16 units (the 16x16x32 kernel does equal work per iteration)
  timeit("16x16x32 random, 3-chains x8, 1 WG/CU", mfma_random16<4>, blocks, out, 2000, 12, 100 * 1024);
  timeit("16x16x32 random, 3-chains x8, 1 WG/CU", mfma_random16<4>, blocks, out, 8000, 12, 100 * 1024);
  timeit("random operands, 3-chains x4, 1 WG/CU (again)", mfma_random<4>, blocks, out, 8000, 12, 100 * 1024);
  hipFree(out);
  return 0;
}
