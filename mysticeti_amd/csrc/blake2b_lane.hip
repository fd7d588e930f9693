// BLAKE2b-256 for gfx950 with ONE lane per string: the throughput form of the block hash
// (blake2 0.10.6 Blake2b<U32> as crypto.rs:34-61 and :174-189 use
// it; RFC 7693 with nn = 32, kk = 0) for batch-size calls (config 4: 2^21 pre-images of ~8 KB).
//
// blake2b_quad.h spreads a string over four lanes to cut the compression chain 4x, which the
// online path (a few strings, latency-bound) needs. At batch size the chip is full anyway and the
// quad form pays for its layout on every round: 12 DPP moves for the diagonal step and back, four
// message reads from LDS at lane-dependent SIGMA offsets (0.40 of LDS-active cycles conflicted,
// profiles/r03/final/pmc_c4_k_b2_quad.txt) and their address arithmetic, 68 issue slots per
// lane-round for 52 of G. Here lane = string:
//
//   state     v[16] and h[8] in VGPRs; the four G's of a half-round are independent, so one wave
//             issues them back to back (no DPP, no cross-lane hazards)
//   message   the block's 16 words in VGPRs, loaded straight from HBM (8-byte loads: strings are
//             8-aligned); SIGMA is resolved at compile time (the 12 rounds are unrolled), so a
//             message word is a register operand, not an LDS read
//   plan      blake2b_quad.h's Plan: DUAL = B2(P) and B2(P || sig) share their (|P| - 1) / 128
//             common compressions; the msg digest's final block runs on a copy of h
//
// Per string and round: 8 G's x (6 v_lshl_add_u64 + 8 xor + 6 rotate) = 208 lane-slots against
// 4 x 68 = 272 in the quad form.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/mysti_verify.h"
#include "blake2b_quad.h"
#include "kernels.h"

namespace mv {
namespace b2l {

using b2q::add64;
using b2q::IV;
using b2q::Plan;
using b2q::ror16;
using b2q::ror24;
using b2q::ror32;
using b2q::ror63;
using b2q::SIGMA;

#define MV_LG(a, b, c, d, x, y) \
  a = add64(add64(a, b), x);    \
  d = ror32(d ^ a);             \
  c = add64(c, d);              \
  b = ror24(b ^ c);             \
  a = add64(add64(a, b), y);    \
  d = ror16(d ^ a);             \
  c = add64(c, d);              \
  b = ror63(b ^ c);

MV_DEV void compress(uint64_t (&h)[8], const uint64_t (&m)[16], uint64_t t, bool fin) {
  uint64_t v[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    v[i] = h[i];
    v[8 + i] = IV[i];
  }
  v[12] ^= t;  // t < 2^64: v[13] unchanged
  v[14] = fin ? ~v[14] : v[14];
#pragma unroll
  for (int r = 0; r < 12; r++) {
    MV_LG(v[0], v[4], v[8], v[12], m[SIGMA[r][0]], m[SIGMA[r][1]])
    MV_LG(v[1], v[5], v[9], v[13], m[SIGMA[r][2]], m[SIGMA[r][3]])
    MV_LG(v[2], v[6], v[10], v[14], m[SIGMA[r][4]], m[SIGMA[r][5]])
    MV_LG(v[3], v[7], v[11], v[15], m[SIGMA[r][6]], m[SIGMA[r][7]])
    MV_LG(v[0], v[5], v[10], v[15], m[SIGMA[r][8]], m[SIGMA[r][9]])
    MV_LG(v[1], v[6], v[11], v[12], m[SIGMA[r][10]], m[SIGMA[r][11]])
    MV_LG(v[2], v[7], v[8], v[13], m[SIGMA[r][12]], m[SIGMA[r][13]])
    MV_LG(v[3], v[4], v[9], v[14], m[SIGMA[r][14]], m[SIGMA[r][15]])
  }
#pragma unroll
  for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[8 + i];
}
#undef MV_LG

// Block b of the string at p, zero past lim; a word is read only when it starts below lim (the
// strings are 8-aligned and readable up to round-up(lim, 8), as for the quad form).
MV_DEV void load_block(uint64_t (&m)[16], const uint8_t* p, uint64_t b, uint64_t lim) {
  const uint64_t* src = reinterpret_cast<const uint64_t*>(p) + b * 16;
  const uint64_t base = b * 128;
  if (base + 128 <= lim) {
#pragma unroll
    for (int j = 0; j < 16; j++) m[j] = src[j];
  } else {
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint64_t pos = base + 8 * j;
      uint64_t v = 0;
      if (pos < lim) {
        v = src[j];
        const uint64_t rem = lim - pos;
        if (rem < 8) v &= (1ull << (8 * rem)) - 1;
      }
      m[j] = v;
    }
  }
}

// 64 strings per 64-lane workgroup. DUAL: out0 = B2(P) (msg), out1 = B2(P || sig) (digest) of
// the staged P || sig with |P| = len; otherwise out0 = B2(string). The message block is loaded
// at the top of its step (tools/gpu_r03z.sh: prefetching it during the previous compression
// needs 134 VGPRs and 3 waves per SIMD and measured no faster; neither did a forced 5 waves per
// SIMD (spills), a shift + add form of the 63-bit rotation, the four G's of a half-round
// written in lock-step (the scheduler pairs them the same way), nor h parked in LDS during the
// rounds (84 VGPRs, 5 waves per SIMD: 4.06 ms per 2^20 either way). Round 4: the message words
// made in registers instead of loaded (no memory traffic at all) ran the hash in the same 4.12
// ms, and the blocks moved one step ahead through LDS by direct-to-LDS loads (16 lines per load
// instruction instead of 64, 16 KB LDS per wave) ran it in 4.9 ms (profiles/r04/ab_c4_hash.txt):
// the loads are not what bounds it. The kernel is bound by VALU issue: ~2,000 instructions per
// compression per wave, 20 per G (6 v_lshl_add_u64, 8 v_xor, 4 v_perm, 2 v_alignbit: the
// instruction mix of the algorithm), no cross-lane or LDS work.
template <bool DUAL>
__global__ void __launch_bounds__(64) k_b2_lane(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ off,
                                                const uint64_t* __restrict__ len, uint32_t n,
                                                uint8_t* __restrict__ out0, uint8_t* __restrict__ out1) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  const bool live = i < n;
  Plan<DUAL> pl;
  pl.init(live ? len[i] : 0, live);
  const uint8_t* p = buf + (live ? off[i] : 0);
  const uint32_t nmax = b2q::wave_max(pl.nsteps);
  uint64_t h[8];
#pragma unroll
  for (int k = 0; k < 8; k++) h[k] = IV[k];
  h[0] ^= 0x01010020ull;  // depth 1, fanout 1, nn = 32
  for (uint32_t s = 0; s < nmax; s++) {
    uint64_t b, lim, t;
    bool fin, mfin;
    pl.at(s, b, lim, t, fin, mfin);
    uint64_t m[16];
    load_block(m, p, b, lim);
    uint64_t hs[8];
#pragma unroll
    for (int k = 0; k < 8; k++) hs[k] = h[k];
    compress(h, m, t, fin);
    if (DUAL && mfin && s < pl.nsteps) {
      uint64_t* o = reinterpret_cast<uint64_t*>(out0 + 32 * (size_t)i);
#pragma unroll
      for (int k = 0; k < 4; k++) o[k] = h[k];
    }
    if ((DUAL && mfin) || s >= pl.nsteps) {  // msg stored / string already done: keep h
#pragma unroll
      for (int k = 0; k < 8; k++) h[k] = hs[k];
    }
  }
  if (live) {
    uint64_t* o = reinterpret_cast<uint64_t*>((DUAL ? out1 : out0) + 32 * (size_t)i);
#pragma unroll
    for (int k = 0; k < 4; k++) o[k] = h[k];
  }
}

}  // namespace b2l
}  // namespace mv

namespace mvk {

hipError_t launch_blake2b_lane(const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n, uint8_t* out,
                               hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL((mv::b2l::k_b2_lane<false>), dim3((n + 63) / 64), dim3(64), 0, s, buf, off, len, n, out,
                     (uint8_t*)nullptr);
  return hipGetLastError();
}

hipError_t launch_block_hash_lane(const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n,
                                  uint8_t* msg_out, uint8_t* dig_out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL((mv::b2l::k_b2_lane<true>), dim3((n + 63) / 64), dim3(64), 0, s, buf, off, len, n, msg_out,
                     dig_out);
  return hipGetLastError();
}

}  // namespace mvk
