// Probe: unaligned 8-byte global loads and LDS stores/loads (what k_b2_walk relies on) give the
// right bytes on gfx950. hipcc -O3 --offload-arch=gfx950 -o tools/unaligned_probe tools/unaligned_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
__global__ void k(const uint8_t* g, uint64_t* out, int sh) {
  __shared__ uint8_t lds[64 * 40];
  const int t = threadIdx.x;
  for (int i = t; i < 64 * 40; i += 64) lds[i] = 0xAA;
  __syncthreads();
  uint64_t v;
  memcpy(&v, g + 8 * t + sh, 8);          // unaligned global load
  memcpy(lds + 40 * t + sh + 3, &v, 8);   // unaligned LDS store
  __syncthreads();
  uint64_t r0, r1;
  memcpy(&r0, lds + 40 * t, 8);
  memcpy(&r1, lds + 40 * t + 8, 8);
  uint64_t r2;
  memcpy(&r2, lds + 40 * t + sh + 3, 8);  // unaligned LDS load
  out[3 * t] = r0; out[3 * t + 1] = r1; out[3 * t + 2] = r2;
}
int main() {
  uint8_t h[1024]; for (int i = 0; i < 1024; i++) h[i] = (uint8_t)(i * 7 + 1);
  uint8_t* g; uint64_t* o; hipMalloc(&g, 1024); hipMalloc(&o, 64 * 3 * 8);
  hipMemcpy(g, h, 1024, hipMemcpyHostToDevice);
  int bad = 0;
  for (int sh = 0; sh < 8; sh++) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, g, o, sh);
    uint64_t r[64 * 3]; hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
    for (int t = 0; t < 64; t++) {
      uint8_t want[16]; memset(want, 0xAA, 16);
      uint64_t v; memcpy(&v, h + 8 * t + sh, 8);
      for (int b = 0; b < 8; b++) if (sh + 3 + b < 16) want[sh + 3 + b] = (uint8_t)(v >> (8 * b));
      uint64_t w0, w1; memcpy(&w0, want, 8); memcpy(&w1, want + 8, 8);
      if (r[3 * t] != w0 || (sh + 3 + 8 <= 16 && r[3 * t + 1] != w1) || r[3 * t + 2] != v) bad++;
    }
  }
  printf("unaligned test: %s (%d bad)\n", bad ? "FAIL" : "ok", bad);
  return bad != 0;
}
