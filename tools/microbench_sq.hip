// Field squaring forms for GF(2^255 - 19) on gfx950, timed on the same dependent chain
// (k_bv_prep's two exponentiation chains are ~85% of its issue, and the
// 9 x 29 squaring costs ~177 issue slots against the 128 the roofline unit counts).
//
//   fe29  fe25519.h fe_sq: 9 x 29-bit unsaturated limbs, each column one v_mad_u64_u32 chain,
//         high columns folded by 2^261 = 1216 (the product form)
//   fe32  8 x 32-bit saturated limbs, product scanning with v_mad_u64_u32's carry-out (a
//         column's products accumulate in 64 bits + a carry word), the cross products doubled
//         once per column, then r = L + 38 H (2^256 = 38 mod p)
//   fe25  10 signed limbs of 26 and 25 bits alternately (the ref10 squaring): 55 products of
//         pre-doubled and x19 / x38 operands, each column one signed v_mad_i64_i32 chain, then 12
//         rounding carries in 64 bits
//
// Both run ITERS dependent squarings per lane (a) on one wave (latency: the online path's
// floor) and (b) on the full chip, 8 waves per SIMD (throughput: issue slots per squaring =
// device cycles / 2 per SIMD over the wave-squarings it ran, at the clock the kernel saw, from
// s_memtime). Result (profiles/r06/microbench_sq.jsonl): fe32 costs 1.8x fe29 on the full chip
// (373 against 203 slots) and 2.7x on a lone wave's chain, fe25 1.24x (252 slots) and 1.2x, so
// the 9 x 29 form stays. The chains start from the same values; their results are compared mod p
// (canonical encodings).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I mysticeti_amd/csrc tools/microbench_sq.hip -o tools/microbench_sq
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "asm_ops.h"
#include "fe25519.h"

using namespace mv;
#define CHECK(x)                                                        \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      printf("HIP %s\n", hipGetErrorString(e_));                        \
      return 1;                                                         \
    }                                                                   \
  } while (0)

// ---- 8 x 32: r = a^2 mod p, a < 2^256 in, r < 2^256 out (not canonical) ----
MV_DEV void sq32(uint32_t (&r)[8], const uint32_t (&a)[8]) {
  uint32_t t[16];
  uint64_t cin = 0;  // the previous column's bits above 32
  uint32_t cin_top = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    uint64_t acc[1] = {0};
    uint32_t top[1] = {0};
#pragma unroll
    for (int i = (k > 7 ? k - 7 : 0); i < k - i; i++) {
      const uint32_t x[1] = {a[i]}, y[1] = {a[k - i]};
      Step<1>::mac(acc, top, x, y);
    }
    // double the cross products (a 97-bit shift by one)
    top[0] = (top[0] << 1) | (uint32_t)(acc[0] >> 63);
    acc[0] <<= 1;
    if ((k & 1) == 0) {
      const uint32_t x[1] = {a[k >> 1]};
      Step<1>::mac(acc, top, x, x);
    }
    // + the carry of the previous column (cin: 64 bits, cin_top: bits 64..95)
    const uint64_t s = acc[0] + cin;
    top[0] += cin_top + (s < cin ? 1u : 0u);
    t[k] = (uint32_t)s;
    cin = (s >> 32) | ((uint64_t)top[0] << 32);
    cin_top = 0;
  }
  t[15] = (uint32_t)cin;
  // r = L + 38 H
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    c = (uint64_t)t[8 + i] * 38u + t[i] + (c >> 32);
    r[i] = (uint32_t)c;
  }
  // the top carry (< 39) once more: r[0] += 38 q, rippled (r < 2^256 after it)
  uint64_t d = (uint64_t)r[0] + (c >> 32) * 38u;
  r[0] = (uint32_t)d;
#pragma unroll
  for (int i = 1; i < 8; i++) {
    d = (uint64_t)r[i] + (d >> 32);
    r[i] = (uint32_t)d;
  }
  r[0] += (uint32_t)(d >> 32) * 38u;  // (only when r was within 38 of 2^256: then r[0] is small)
}

// ---- 10 x 25.5 (ref10 layout): limb i holds bits [ceil(25.5 i), ceil(25.5 (i + 1))) ----
constexpr int B25[11] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230, 255};
MV_DEV void sq25(int32_t (&h)[10], const int32_t (&f)[10]) {
  const int32_t f0 = f[0], f1 = f[1], f2 = f[2], f3 = f[3], f4 = f[4], f5 = f[5], f6 = f[6], f7 = f[7], f8 = f[8],
                f9 = f[9];
  const int32_t f0_2 = 2 * f0, f1_2 = 2 * f1, f2_2 = 2 * f2, f3_2 = 2 * f3, f4_2 = 2 * f4, f5_2 = 2 * f5,
                f6_2 = 2 * f6, f7_2 = 2 * f7;
  const int32_t f5_38 = 38 * f5, f6_19 = 19 * f6, f7_38 = 38 * f7, f8_19 = 19 * f8, f9_38 = 38 * f9;
#define M(a, b) ((int64_t)(a) * (int64_t)(b))
  int64_t h0 = M(f0, f0) + M(f1_2, f9_38) + M(f2_2, f8_19) + M(f3_2, f7_38) + M(f4_2, f6_19) + M(f5, f5_38);
  int64_t h1 = M(f0_2, f1) + M(f2, f9_38) + M(f3_2, f8_19) + M(f4, f7_38) + M(f5_2, f6_19);
  int64_t h2 = M(f0_2, f2) + M(f1_2, f1) + M(f3_2, f9_38) + M(f4_2, f8_19) + M(f5_2, f7_38) + M(f6, f6_19);
  int64_t h3 = M(f0_2, f3) + M(f1_2, f2) + M(f4, f9_38) + M(f5_2, f8_19) + M(f6, f7_38);
  int64_t h4 = M(f0_2, f4) + M(f1_2, f3_2) + M(f2, f2) + M(f5_2, f9_38) + M(f6_2, f8_19) + M(f7, f7_38);
  int64_t h5 = M(f0_2, f5) + M(f1_2, f4) + M(f2_2, f3) + M(f6, f9_38) + M(f7_2, f8_19);
  int64_t h6 = M(f0_2, f6) + M(f1_2, f5_2) + M(f2_2, f4) + M(f3_2, f3) + M(f7_2, f9_38) + M(f8, f8_19);
  int64_t h7 = M(f0_2, f7) + M(f1_2, f6) + M(f2_2, f5) + M(f3_2, f4) + M(f8, f9_38);
  int64_t h8 = M(f0_2, f8) + M(f1_2, f7_2) + M(f2_2, f6) + M(f3_2, f5_2) + M(f4, f4) + M(f9, f9_38);
  int64_t h9 = M(f0_2, f9) + M(f1_2, f8) + M(f2_2, f7) + M(f3_2, f6) + M(f4_2, f5);
#undef M
  int64_t c;
#define CR(a, b, s) c = (a + ((int64_t)1 << (s - 1))) >> s; b += c; a -= c << s;
  CR(h0, h1, 26) CR(h4, h5, 26) CR(h1, h2, 25) CR(h5, h6, 25) CR(h2, h3, 26) CR(h6, h7, 26)
  CR(h3, h4, 25) CR(h7, h8, 25) CR(h4, h5, 26) CR(h8, h9, 26)
  c = (h9 + ((int64_t)1 << 24)) >> 25; h0 += c * 19; h9 -= c << 25;
  CR(h0, h1, 26)
#undef CR
  h[0] = (int32_t)h0; h[1] = (int32_t)h1; h[2] = (int32_t)h2; h[3] = (int32_t)h3; h[4] = (int32_t)h4;
  h[5] = (int32_t)h5; h[6] = (int32_t)h6; h[7] = (int32_t)h7; h[8] = (int32_t)h8; h[9] = (int32_t)h9;
}

// 8 words (value < 2^255) -> 10 limbs
MV_DEV void from_words25(int32_t (&h)[10], const uint32_t (&w)[8]) {
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const int b = B25[i], n = B25[i + 1] - b, q = b >> 5, r = b & 31;
    uint64_t x = w[q];
    if (q + 1 < 8) x |= (uint64_t)w[q + 1] << 32;
    h[i] = (int32_t)((x >> r) & ((1ull << n) - 1));
  }
}

// canonical 8-word encoding of a 10-limb value (ref10's reduction: q = floor(h / p), h - q p)
MV_DEV void canon25(uint32_t (&w)[8], const int32_t (&f)[10]) {
  int64_t h[10];
#pragma unroll
  for (int i = 0; i < 10; i++) h[i] = f[i];
  int64_t q = (19 * h[9] + ((int64_t)1 << 24)) >> 25;
#pragma unroll
  for (int i = 0; i < 10; i++) q = (h[i] + q) >> (B25[i + 1] - B25[i]);
  h[0] += 19 * q;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int s = B25[i + 1] - B25[i];
    const int64_t c = h[i] >> s;
    h[i + 1] += c;
    h[i] -= c << s;
  }
  h[9] &= (1 << 25) - 1;
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const int b = B25[i], q2 = b >> 5, r = b & 31;
    const uint64_t x = (uint64_t)h[i] << r;
    w[q2] |= (uint32_t)x;
    if (q2 + 1 < 8) w[q2 + 1] |= (uint32_t)(x >> 32);
  }
}

// canonical 8-word encoding of an 8 x 32 value
MV_DEV void canon32(uint32_t (&w)[8], const uint32_t (&a)[8]) {
  uint32_t x[8];
#pragma unroll
  for (int i = 0; i < 8; i++) x[i] = a[i];
  for (int pass = 0; pass < 2; pass++) {  // fold bit 255 (2^255 = 19)
    uint64_t c = (uint64_t)(x[0]) + 19u * (x[7] >> 31);
    x[7] &= 0x7fffffffu;
    x[0] = (uint32_t)c;
#pragma unroll
    for (int i = 1; i < 8; i++) {
      c = (uint64_t)x[i] + (c >> 32);
      x[i] = (uint32_t)c;
    }
  }
  // x < 2^255: subtract p once if x >= p
  const uint32_t P[8] = {0xffffffedu, 0xffffffffu, 0xffffffffu, 0xffffffffu,
                         0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu};
  uint32_t y[8];
  int64_t b = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int64_t s = (int64_t)x[i] - P[i] + b;
    y[i] = (uint32_t)s;
    b = s >> 32;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = b < 0 ? x[i] : y[i];
}

MV_DEV void start(uint32_t (&a32)[8], fe& a29, uint32_t seed) {
  // a 255-bit value from the seed, in both forms
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = seed * 2654435761u + 0x9e3779b9u * (uint32_t)(i + 1);
  w[7] &= 0x7fffffffu;
#pragma unroll
  for (int i = 0; i < 8; i++) a32[i] = w[i];
  fe_from_words(a29, w);
}

__global__ void __launch_bounds__(256) k_sq29(uint32_t* out, int iters, unsigned long long* cyc) {
  uint32_t a32[8];
  fe a;
  start(a32, a, blockIdx.x * blockDim.x + threadIdx.x);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < iters; it++) fe_sq(a, a);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  fe c;
  fe_canon(c, a);
  uint32_t w[8];
  fe_to_words(w, c);
  const size_t g = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 8; i++) out[8 * g + i] = w[i];
  if (threadIdx.x == 0) atomicMax(cyc, (unsigned long long)(t1 - t0));
}

__global__ void __launch_bounds__(256) k_sq32(uint32_t* out, int iters, unsigned long long* cyc) {
  uint32_t a[8];
  fe a29;
  start(a, a29, blockIdx.x * blockDim.x + threadIdx.x);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < iters; it++) sq32(a, a);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t w[8];
  canon32(w, a);
  const size_t g = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 8; i++) out[8 * g + i] = w[i];
  if (threadIdx.x == 0) atomicMax(cyc, (unsigned long long)(t1 - t0));
}

__global__ void __launch_bounds__(256) k_sq25(uint32_t* out, int iters, unsigned long long* cyc) {
  uint32_t a32[8];
  fe a29;
  start(a32, a29, blockIdx.x * blockDim.x + threadIdx.x);
  int32_t a[10];
  from_words25(a, a32);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < iters; it++) sq25(a, a);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t w[8];
  canon25(w, a);
  const size_t g = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 8; i++) out[8 * g + i] = w[i];
  if (threadIdx.x == 0) atomicMax(cyc, (unsigned long long)(t1 - t0));
}

typedef void (*kfn)(uint32_t*, int, unsigned long long*);

int run(const char* name, kfn k, int blocks, int iters, uint32_t* d, unsigned long long* dc, double* us, double* cyc) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 16, dc);  // warm
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemset(dc, 0, 8));
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, iters, dc);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long c = 0;
  CHECK(hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost));
  *us = ms * 1e3;
  *cyc = (double)c;
  (void)name;
  return 0;
}

int main() {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int iters = 4096;
  const int full_blocks = cus * 8;  // 256-thread blocks: 4 waves each, 8 waves per SIMD
  uint32_t *d29, *d32, *d25;
  unsigned long long* dc;
  CHECK(hipMalloc(&d29, (size_t)full_blocks * 256 * 32));
  CHECK(hipMalloc(&d32, (size_t)full_blocks * 256 * 32));
  CHECK(hipMalloc(&d25, (size_t)full_blocks * 256 * 32));
  CHECK(hipMalloc(&dc, 8));
  struct R {
    const char* name;
    kfn k;
    uint32_t* d;
  } forms[3] = {{"fe29 (9 x 29, fe_sq)", k_sq29, d29},
                {"fe32 (8 x 32, product scanning)", k_sq32, d32},
                {"fe25 (10 x 25.5 signed, ref10 squaring)", k_sq25, d25}};
  // s_memtime ticks at the shader clock; wall-clock us gives the clock
  for (const R& f : forms) {
    double us1, cyc1, usf, cycf;
    if (run(f.name, f.k, 1, iters, f.d, dc, &us1, &cyc1)) return 1;  // one workgroup: 4 waves on 4 SIMDs
    if (run(f.name, f.k, full_blocks, iters, f.d, dc, &usf, &cycf)) return 1;
    const double sq_full = (double)full_blocks * 256 * iters;
    const double ghz = cycf / (usf * 1e3);
    // issue slots per squaring at the full chip: a SIMD issues one full-rate wave64 instruction
    // per 2 cycles, so its slots = cycles / 2, over the wave-squarings it ran (lane count / 64)
    const double slots = (cycf / 2.0) / (sq_full / (cus * 4.0) / 64.0);
    printf("{\"form\": \"%s\", \"lone_wave_ns_per_sq\": %.2f, \"lone_wave_cycles_per_sq\": %.1f, "
           "\"full_chip_sq_per_s\": %.4g, \"clock_GHz\": %.3f, \"issue_slots_per_sq\": %.1f}\n",
           f.name, us1 * 1e3 / iters, cyc1 / iters, sq_full / (usf * 1e-6), ghz, slots);
  }
  // the two chains must agree mod p on every lane (canonical encodings)
  const size_t words = (size_t)full_blocks * 256 * 8;
  uint32_t* h29 = (uint32_t*)malloc(words * 4);
  uint32_t* h32 = (uint32_t*)malloc(words * 4);
  uint32_t* h25 = (uint32_t*)malloc(words * 4);
  CHECK(hipMemcpy(h29, d29, words * 4, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(h32, d32, words * 4, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(h25, d25, words * 4, hipMemcpyDeviceToHost));
  size_t bad = 0, bad25 = 0;
  for (size_t i = 0; i < words; i++) {
    bad += h29[i] != h32[i];
    bad25 += h29[i] != h25[i];
  }
  printf("{\"agree\": %s, \"words_compared\": %zu, \"mismatched_fe32\": %zu, \"mismatched_fe25\": %zu}\n",
         bad + bad25 ? "false" : "true", words, bad, bad25);
  return bad + bad25 != 0;
}
