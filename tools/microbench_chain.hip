// Latency of one dependent chain of field operations on a single wave (the online path's
// floor): fe_sq / fe_mul (one lane per element, fe25519.h) against feq_sq (four lanes per
// element, fe_q4.h). One 64-lane workgroup, ITERS dependent operations, hipEvent timing.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I mysticeti_amd/csrc tools/microbench_chain.hip -o tools/microbench_chain
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "fe25519.h"
#include "fe_q4.h"
#include "fe_r16.h"
#include "hash_dev.h"

using namespace mv;
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e_)); return 1; } } while (0)

__global__ void __launch_bounds__(64) k_chain_sq(uint32_t* out, int iters) {
  fe a;
  for (int i = 0; i < 9; i++) a.v[i] = threadIdx.x * 7 + i + 1;
#pragma unroll 1
  for (int it = 0; it < iters; it++) fe_sq(a, a);
  uint32_t s = 0;
  for (int i = 0; i < 9; i++) s += a.v[i];
  out[threadIdx.x] = s;
}
__global__ void __launch_bounds__(64) k_chain_mul(uint32_t* out, int iters) {
  fe a, b;
  for (int i = 0; i < 9; i++) {
    a.v[i] = threadIdx.x * 7 + i + 1;
    b.v[i] = threadIdx.x * 3 + i + 5;
  }
#pragma unroll 1
  for (int it = 0; it < iters; it++) fe_mul(a, a, b);
  uint32_t s = 0;
  for (int i = 0; i < 9; i++) s += a.v[i];
  out[threadIdx.x] = s;
}
__global__ void __launch_bounds__(64) k_chain_q4(uint32_t* out, int iters) {
  feq a;
  for (int i = 0; i < 3; i++) a.r[i] = threadIdx.x * 7 + i + 1;
  if ((threadIdx.x & 3) != 0) a.r[2] = 0;
#pragma unroll 1
  for (int it = 0; it < iters; it++) feq_sq(a, a);
  out[threadIdx.x] = a.r[0] + a.r[1] + a.r[2];
}

__global__ void __launch_bounds__(64) k_chain_r16(uint32_t* out, int iters) {
  const r16::Consts K = r16::consts();
  fer a;
  a.v = (threadIdx.x & 15) < 9 ? threadIdx.x * 7 + 1 : 0u;
#pragma unroll 1
  for (int it = 0; it < iters; it++) fer_sq(a, a, K);
  out[threadIdx.x] = a.v;
}

// SHA-512 of 96 bytes (the challenge input), each input the previous digest's words
__global__ void __launch_bounds__(64) k_chain_sha(uint32_t* out, int iters) {
  uint32_t in[24], h[16];
  for (int i = 0; i < 24; i++) in[i] = threadIdx.x * 7 + i;
#pragma unroll 1
  for (int it = 0; it < iters / 16; it++) {
    sha512_short(h, in, 96);
    for (int i = 0; i < 16; i++) in[i] = h[i];
  }
  out[threadIdx.x] = in[0] + in[5];
}

typedef void (*kfn)(uint32_t*, int);
static int run(const char* name, kfn k, uint32_t* d) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float best[2] = {1e30f, 1e30f};
  const int iters[2] = {256, 4352};
  for (int rep = 0; rep < 5; rep++)
    for (int j = 0; j < 2; j++) {
      CHECK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, iters[j]);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best[j]) best[j] = ms;
    }
  // the difference of two chain lengths cancels the launch overhead
  const double us = (best[1] - best[0]) * 1e3 / (iters[1] - iters[0]);
  printf("{\"kernel\": \"%s\", \"us_per_op\": %.4f, \"ns_per_op\": %.1f}\n", name, us, us * 1e3);
  return 0;
}

int main() {
  uint32_t* d;
  CHECK(hipMalloc(&d, 64 * sizeof(uint32_t)));
  if (run("fe_sq (1 lane)", k_chain_sq, d) || run("fe_mul (1 lane)", k_chain_mul, d) ||
      run("feq_sq (4 lanes)", k_chain_q4, d) || run("fer_sq (16-lane row)", k_chain_r16, d) ||
      run("sha512_short 96 B (1 lane), per 16 ops = 1 hash", k_chain_sha, d))
    return 1;
  return 0;
}
