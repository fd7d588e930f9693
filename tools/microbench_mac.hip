#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e_)); return 1; } } while (0)
constexpr int ITERS = 16384;
// 4 independent chains, exactly the Step<4>::mac block
__global__ void __launch_bounds__(256) k_mac4(uint32_t* out, uint32_t a, uint32_t b, int iters) {
  uint64_t q0 = threadIdx.x, q1 = q0 + 1, q2 = q0 + 2, q3 = q0 + 3; uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
      uint64_t s0, s1, s2, s3;
      asm volatile("v_mad_u64_u32 %0, %8, %12, %13, %0\n\tv_mad_u64_u32 %1, %9, %12, %13, %1\n\tv_mad_u64_u32 %2, %10, %12, %13, %2\n\tv_mad_u64_u32 %3, %11, %12, %13, %3\n\t"
                   "v_addc_co_u32 %4, %8, %4, 0, %8\n\tv_addc_co_u32 %5, %9, %5, 0, %9\n\tv_addc_co_u32 %6, %10, %6, 0, %10\n\tv_addc_co_u32 %7, %11, %7, 0, %11"
                   : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "=&s"(s0), "=&s"(s1), "=&s"(s2), "=&s"(s3)
                   : "v"(a), "v"(b));
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(q0 + q1 + q2 + q3) + c0 + c1 + c2 + c3;
}
// 4 independent addc chains (VOP3b, SGPR carry), 8 instrs per asm
__global__ void __launch_bounds__(256) k_addc4(uint32_t* out, uint32_t a, uint32_t b, int iters) {
  uint32_t r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3; uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++)
      asm volatile("v_addc_co_u32 %0, %4, %0, %8, %4\n\tv_addc_co_u32 %1, %5, %1, %8, %5\n\tv_addc_co_u32 %2, %6, %2, %8, %6\n\tv_addc_co_u32 %3, %7, %3, %8, %7\n\t"
                   "v_addc_co_u32 %0, %4, %0, %8, %4\n\tv_addc_co_u32 %1, %5, %1, %8, %5\n\tv_addc_co_u32 %2, %6, %2, %8, %6\n\tv_addc_co_u32 %3, %7, %3, %8, %7"
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3) : "v"(a));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r0 + r1 + r2 + r3;
}
// only mads, 4 chains
__global__ void __launch_bounds__(256) k_mad4(uint32_t* out, uint32_t a, uint32_t b, int iters) {
  uint64_t q0 = threadIdx.x, q1 = q0 + 1, q2 = q0 + 2, q3 = q0 + 3;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
      uint64_t s0, s1, s2, s3;
      asm volatile("v_mad_u64_u32 %0, %4, %8, %9, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_mad_u64_u32 %2, %6, %8, %9, %2\n\tv_mad_u64_u32 %3, %7, %8, %9, %3\n\t"
                   "v_mad_u64_u32 %0, %4, %8, %9, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_mad_u64_u32 %2, %6, %8, %9, %2\n\tv_mad_u64_u32 %3, %7, %8, %9, %3"
                   : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "=&s"(s0), "=&s"(s1), "=&s"(s2), "=&s"(s3) : "v"(a), "v"(b));
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(q0 + q1 + q2 + q3);
}
// VOP2 add with vcc carry chain, 4 chains is impossible (single vcc): e32 add_u32 x8 independent
__global__ void __launch_bounds__(256) k_add8(uint32_t* out, uint32_t a, uint32_t b, int iters) {
  uint32_t r[8]; for (int i = 0; i < 8; i++) r[i] = threadIdx.x + i;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++)
#pragma unroll
      for (int i = 0; i < 8; i++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[i]) : "v"(a));
  }
  uint32_t s = 0; for (int i = 0; i < 8; i++) s += r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
typedef void (*kfn)(uint32_t*, uint32_t, uint32_t, int);
int run(const char* name, kfn k, double instr_per_iter, uint32_t* d, int blocks, int occ_waves) {
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 3u, 5u, 64); CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0)); hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 3u, 5u, ITERS); CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  double instr = (double)blocks * 256 / 64 * ITERS * instr_per_iter;  // wave-instructions
  printf("{\"kernel\": \"%s\", \"waves_per_cu\": %d, \"wave_instr_per_s\": %.4e, \"lane_instr_per_s\": %.4e, \"ms\": %.2f}\n", name, occ_waves, instr / (ms * 1e-3), 64 * instr / (ms * 1e-3), ms);
  return 0;
}
int main() {
  uint32_t* d; CHECK(hipMalloc(&d, 256 * 64 * 256 * 4));
  for (int wpc : {4, 8, 16, 32}) {
    int blocks = 256 * wpc / 4;
    run("mac4_block(8 instr)", k_mac4, 8 * 8, d, blocks, wpc);
    run("addc4_vop3b", k_addc4, 8 * 8, d, blocks, wpc);
    run("mad4", k_mad4, 8 * 8, d, blocks, wpc);
    run("add_u32_vop2", k_add8, 8 * 8, d, blocks, wpc);
  }
  return 0;
}
