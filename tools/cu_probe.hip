// Which CUs a CU-masked stream's workgroups land on (hipExtStreamCreateWithCUMask): every workgroup of a
// spinning kernel records its XCC_ID and HW_ID (SE / SH / CU) hardware registers; the host prints, per mask,
// how many distinct CUs each XCC and shader engine ran workgroups on.  A diagnostic (not part of the library)
// from the round-6 CU-reservation experiment: mask bit i = XCD i % 8, engine (i / 8) % 4, CU i / 32.
//   hipcc --offload-arch=gfx950 -O2 tools/cu_probe.hip -o tools/bin/cu_probe && tools/bin/cu_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <set>
#include <vector>

__global__ void probe_kernel(unsigned* out, long long spin) {
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID, all 32 bits
  const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
  const long long t0 = clock64();
  while (clock64() - t0 < spin) {
  }
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
  }
}

static void run(const char* name, const std::vector<uint32_t>& mask, unsigned* d_out, int nblk) {
  hipStream_t s;
  if (mask.empty()) {
    if (hipStreamCreate(&s) != hipSuccess) return;
  } else if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
    printf("%s: stream creation failed\n", name);
    return;
  }
  hipLaunchKernelGGL(probe_kernel, dim3(nblk), dim3(64), 0, s, d_out, 200000LL);
  hipStreamSynchronize(s);
  std::vector<unsigned> h(2 * nblk);
  hipMemcpy(h.data(), d_out, h.size() * 4, hipMemcpyDeviceToHost);
  std::set<unsigned> cus;
  int per_xcc[16] = {0};
  std::set<unsigned> per_se[16][8];
  for (int b = 0; b < nblk; ++b) {
    const unsigned hw = h[2 * b], xcc = h[2 * b + 1] & 0xF;
    const unsigned cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
    const unsigned key = (xcc << 16) | (se << 8) | (sh << 4) | cu;
    if (cus.insert(key).second) per_xcc[xcc]++;
    per_se[xcc][se].insert((sh << 4) | cu);
  }
  printf("%-28s total CUs %3zu | per XCC:", name, cus.size());
  for (int x = 0; x < 8; ++x) printf(" %2d", per_xcc[x]);
  printf(" | XCC0 per SE:");
  for (int e = 0; e < 8; ++e) printf(" %zu", per_se[0][e].size());
  printf(" | XCC1 per SE:");
  for (int e = 0; e < 8; ++e) printf(" %zu", per_se[1][e].size());
  printf("\n");
  hipStreamDestroy(s);
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int words = ncu / 32;
  printf("CUs %d, mask words %d\n", ncu, words);
  const int nblk = 8192;
  unsigned* d_out;
  hipMalloc(&d_out, 2 * nblk * 4);
  run("full", {}, d_out, nblk);
  std::vector<uint32_t> m(words, 0xFFFFFFFFu);
  m[0] = 0;
  run("word0 cleared", m, d_out, nblk);
  for (int d = 0; d < words; ++d) m[d] = 0xFFFFFFFEu;
  run("bit0 of every word cleared", m, d_out, nblk);
  for (int d = 0; d < words; ++d) m[d] = 0xFFFFFFFFu;
  for (int i = 0; i < 8; ++i) m[0] &= ~(1u << i);
  run("bits 0-7 cleared", m, d_out, nblk);
  for (int d = 0; d < words; ++d) m[d] = 0xFFFFFF00u;
  run("bits 0-7 of every word", m, d_out, nblk);
  for (int d = 0; d < words; ++d) m[d] = 0x00FFFFFFu;
  run("bits 24-31 of every word", m, d_out, nblk);
  for (int d = 0; d < words; ++d) {
    uint32_t clear = 0;
    for (int q = 0; q < 4; ++q) clear |= 1u << ((d * 4 + q) % 8 + 8 * (q / 8));
    m[d] = ~clear;
  }
  run("per-word pattern", m, d_out, nblk);
  hipFree(d_out);
  return 0;
}
