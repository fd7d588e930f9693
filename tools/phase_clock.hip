// Per-phase cycle breakdown of k_verify (profiling tool, not part of the library).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/phase_clock tools/phase_clock.hip
//   ./tools/phase_clock [n] [occ]
// Inputs are random bytes: every lane runs the same instruction stream whatever the
// verdict (only sc_halfsize's trip count depends on the data, and random k is its
// typical case), so the phase costs equal those of a valid batch.
#define MV_PHASE_CLOCKS
#include "../mysticeti_amd/csrc/kernels.hip"

#include <stdio.h>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
  const int occ = argc > 2 ? atoi(argv[2]) : 2;
  std::vector<uint8_t> h(128 * (size_t)n);
  uint64_t x = 0x9e3779b97f4a7c15ull;
  for (auto& b : h) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    b = (uint8_t)x;
  }
  uint8_t *msg, *sig, *pk, *st;
  uint4 *btab, *scr;
  unsigned long long* ph;
  const size_t waves = (size_t)((n + 255) / 256) * 4;
  CK(hipMalloc(&msg, 32 * (size_t)n));
  CK(hipMalloc(&sig, 64 * (size_t)n));
  CK(hipMalloc(&pk, 32 * (size_t)n));
  CK(hipMalloc(&st, n));
  CK(hipMalloc(&btab, mvk::btable_bytes()));
  CK(hipMalloc(&scr, mvk::verify_scratch_bytes(n)));
  CK(hipMalloc(&ph, waves * 16 * sizeof(unsigned long long)));
  CK(hipMemcpy(msg, h.data(), 32 * (size_t)n, hipMemcpyHostToDevice));
  CK(hipMemcpy(sig, h.data() + 32 * (size_t)n, 64 * (size_t)n, hipMemcpyHostToDevice));
  CK(hipMemcpy(pk, h.data() + 96 * (size_t)n, 32 * (size_t)n, hipMemcpyHostToDevice));
  CK(mvk::launch_btable_init(btab, 0));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(mv::g_phase_buf), &ph, sizeof(ph)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms = 0;
  const dim3 grid((n + 255) / 256), block(256);
  for (int rep = 0; rep < 3; rep++) {
    CK(hipEventRecord(e0, 0));
    if (occ == 1)
      hipLaunchKernelGGL(mv::k_verify<1>, grid, block, 0, 0, msg, sig, pk, nullptr, n, btab, scr, st, (const uint32_t*)nullptr);
    else if (occ == 3)
      hipLaunchKernelGGL(mv::k_verify<3>, grid, block, 0, 0, msg, sig, pk, nullptr, n, btab, scr, st, (const uint32_t*)nullptr);
    else
      hipLaunchKernelGGL(mv::k_verify<2>, grid, block, 0, 0, msg, sig, pk, nullptr, n, btab, scr, st, (const uint32_t*)nullptr);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
  }
  std::vector<unsigned long long> p(waves * 16);
  CK(hipMemcpy(p.data(), ph, p.size() * 8, hipMemcpyDeviceToHost));
  // (from, to) phase-clock indices
  const int span[7][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 4}, {4, 5}, {5, 6}, {6, 7}};
  const char* names[7] = {"sha512+reduce", "halfsize", "muladd+recode", "decompress_x2", "tables",
                          "ladder(32 windows)", "cofactor+store"};
  double sum[7] = {0};
  for (size_t w = 0; w < waves; w++)
    for (int i = 0; i < 7; i++) sum[i] += (double)(p[w * 16 + span[i][1]] - p[w * 16 + span[i][0]]);
  printf("{\"n\": %u, \"occ\": %d, \"kernel_ms\": %.4f, \"rate\": %.4g, \"wave_cycles\": {", n, occ, ms,
         n / (ms * 1e-3));
  for (int i = 0; i < 7; i++) printf("%s\"%s\": %.0f", i ? ", " : "", names[i], sum[i] / waves);
  printf("}}\n");
  return 0;
}
