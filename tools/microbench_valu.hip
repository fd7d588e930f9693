// VALU integer-throughput microbenchmark for gfx950 (MI355X).
//
// Fixes the roofline denominator for the verify kernels: the
// field arithmetic lives on 32x32->64 multiply-accumulates, whose issue rate the
// CDNA4 guides do not state. Every kernel runs ACC independent dependency chains
// per lane, so the loop is issue-bound, and reports lane-ops/s over the whole
// chip plus the single-wave dependent-chain latency.
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/microbench_valu.hip -o tools/microbench_valu
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 65536;
constexpr int ACC = 8;

// One op per macro invocation on accumulator i.
#define OP_MAD64(i)   asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(q[i]) : "v"(a), "v"(b) : "vcc")
#define OP_MULLO(i)   asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(r[i]) : "v"(b))
#define OP_MULHI(i)   asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(r[i]) : "v"(b))
#define OP_MAD24(i)   asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(r[i]) : "v"(b), "v"(a))
#define OP_MULHI24(i) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(r[i]) : "v"(b))
#define OP_ADD(i)     asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[i]) : "v"(b))
#define OP_ADDC(i)    asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(r[i]) : "v"(b) : "vcc")
#define OP_ALIGN(i)   asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(r[i]) : "v"(b))
#define OP_XOR3(i)    asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r[i]) : "v"(b), "v"(a))
#define OP_ADD3(i)    asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(b), "v"(a))
#define OP_LSHR64(i)  asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(q[i]))
#define OP_FMA64(i)   asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[i]) : "v"(dx), "v"(dy))
#define OP_CNDMASK(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r[i]) : "v"(b))
#define OP_MOV(i)     asm volatile("v_mov_b32 %0, %1" : "=v"(r[i]) : "v"(r[(i + 1) % ACC]))
#define OP_LSHLADD64(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(q[i]) : "v"(q[(i + 1) % ACC]))
#define OP_MAC(i)     asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %3, %0\n\tv_addc_co_u32 %1, s[40:41], %1, 0, s[40:41]" : "+v"(q[i]), "+v"(r[i]) : "v"(a), "v"(b) : "s40", "s41")

#define KERNEL(NAME, OPM, OPS_PER)                                                     \
  __global__ void __launch_bounds__(256) k_##NAME(uint32_t* out, uint32_t a, uint32_t b, int iters) { \
    uint64_t q[ACC]; uint32_t r[ACC]; double d[ACC];                                   \
    double dx = (double)a * 1e-9, dy = (double)b * 1e-9;                               \
    _Pragma("unroll") for (int i = 0; i < ACC; i++) {                                  \
      q[i] = threadIdx.x + i; r[i] = threadIdx.x * 7 + i; d[i] = i; }                  \
    for (int it = 0; it < iters; it++) {                                               \
      _Pragma("unroll") for (int i = 0; i < ACC; i++) { OPM(i); }                      \
      _Pragma("unroll") for (int i = 0; i < ACC; i++) { OPM(i); }                      \
      _Pragma("unroll") for (int i = 0; i < ACC; i++) { OPM(i); }                      \
      _Pragma("unroll") for (int i = 0; i < ACC; i++) { OPM(i); }                      \
    }                                                                                  \
    uint32_t s = 0;                                                                    \
    _Pragma("unroll") for (int i = 0; i < ACC; i++) s += (uint32_t)q[i] + r[i] + (uint32_t)d[i]; \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                    \
  }                                                                                    \
  __global__ void k1_##NAME(uint32_t* out, uint32_t a, uint32_t b, int iters) {        \
    uint64_t q[1]; uint32_t r[1]; double d[1];                                         \
    double dx = (double)a * 1e-9, dy = (double)b * 1e-9;                               \
    q[0] = threadIdx.x; r[0] = threadIdx.x; d[0] = 1;                                  \
    for (int it = 0; it < iters; it++) { OPM(0); OPM(0); OPM(0); OPM(0); }             \
    out[threadIdx.x] = (uint32_t)q[0] + r[0] + (uint32_t)d[0];                         \
  }

KERNEL(mad_u64_u32, OP_MAD64, 1)
KERNEL(mul_lo_u32, OP_MULLO, 1)
KERNEL(mul_hi_u32, OP_MULHI, 1)
KERNEL(mad_u32_u24, OP_MAD24, 1)
KERNEL(mul_hi_u32_u24, OP_MULHI24, 1)
KERNEL(add_u32, OP_ADD, 1)
KERNEL(add_co_addc_pair, OP_ADDC, 2)
KERNEL(alignbit_b32, OP_ALIGN, 1)
KERNEL(bitop3_xor3, OP_XOR3, 1)
KERNEL(add3_u32, OP_ADD3, 1)
KERNEL(lshrrev_b64, OP_LSHR64, 1)
KERNEL(fma_f64, OP_FMA64, 1)
KERNEL(cndmask_b32, OP_CNDMASK, 1)
KERNEL(mov_b32, OP_MOV, 1)
KERNEL(lshl_add_u64, OP_LSHLADD64, 1)

typedef void (*kfn)(uint32_t*, uint32_t, uint32_t, int);

static int run(const char* name, kfn k, kfn k1, int instrs_per_op, uint32_t* dout, int blocks) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, dout, 3u, 5u, 16);  // warm
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, dout, 3u, 5u, ITERS);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  double ops = (double)blocks * 256 * ITERS * 4 * ACC;         // lane-ops (macro invocations)
  double instr_rate = ops * instrs_per_op / (ms * 1e-3);
  // latency: single wave, single chain
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(k1, dim3(1), dim3(64), 0, 0, dout, 3u, 5u, ITERS / 16);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms1; CHECK(hipEventElapsedTime(&ms1, e0, e1));
  double lat_ns = ms1 * 1e6 / (ITERS / 16 * 4.0);
  printf("{\"instr\": \"%s\", \"lane_ops_per_s\": %.4e, \"instr_lane_rate\": %.4e, \"dep_latency_ns_per_op\": %.3f, \"ms\": %.3f}\n",
         name, ops / (ms * 1e-3), instr_rate, lat_ns, ms);
  return 0;
}

int main() {
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  int blocks = p.multiProcessorCount * 8;  // 8 x 256 threads = 32 waves per CU
  printf("{\"device\": \"%s\", \"gcn\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", p.name, p.gcnArchName,
         p.multiProcessorCount, p.clockRate);
  uint32_t* dout; CHECK(hipMalloc(&dout, (size_t)blocks * 256 * 4));
#define RUN(NAME, N) if (run(#NAME, k_##NAME, k1_##NAME, N, dout, blocks)) return 1;
  RUN(add_u32, 1)
  RUN(mad_u64_u32, 1)
  RUN(mul_lo_u32, 1)
  RUN(mul_hi_u32, 1)
  RUN(mad_u32_u24, 1)
  RUN(mul_hi_u32_u24, 1)
  RUN(add_co_addc_pair, 2)
  RUN(alignbit_b32, 1)
  RUN(bitop3_xor3, 1)
  RUN(add3_u32, 1)
  RUN(lshrrev_b64, 1)
  RUN(fma_f64, 1)
  RUN(cndmask_b32, 1)
  RUN(mov_b32, 1)
  RUN(lshl_add_u64, 1)
  return 0;
}
