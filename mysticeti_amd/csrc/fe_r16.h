// GF(2^255-19) with one DPP ROW (16 lanes) per field element (gfx950), for latency-bound
// exponentiation chains: the ZIP-215 decode of R on the online block path (comb.hip).
//
// Why: a lone wave issues about one VALU instruction per 4 cycles whatever the instruction
// (tools/microbench_chain.hip: fe_sq = 104 instructions = 222 ns on one wave), so a chain of
// ~265 dependent field operations costs its instruction count. fe_q4.h's four-lane form needs
// 146 instructions per product (operand selects), no faster. Here the instruction stream is
// the same in every lane and the cross-lane moves are single DPP movs:
//
// R form: lane t (0..8) of the row holds limb t of fe25519.h's 9 x 29-bit representation;
// lanes 9..15 hold zero. A product r = a b:
//   1. lane t sums column t = sum_i a_i b_(t-i), i = 0..8: a_i by row_newbcast:i, b_(t-i) by
//      row_shr:i (zero below the row start). Lanes 9..15 thereby compute columns 9..15 (b is
//      zero at lanes >= 9); column 16 = a_8 b_8 in every lane. 9 v_mad_u64_u32 per lane.
//   2. fold (2^261 = 1216 mod p): column c >= 9's low half times 1216 to column c - 9
//      (row_shl:9), its high half times 9728 = 8 * 1216 to column c - 8 (row_shl:8; the
//      multiplier is zero where the source is column 8); column 16 into lanes 7 and 8.
//   3. carry round 1 at 32 bits: column t's high word has weight 2^(29 (t + 1) + 3), so lane t
//      adds 8 x (lane t - 1's high word) (row_shr:1) and lane 0 adds 9728 x lane 8's
//      (row_shl:8, multiplier zero elsewhere); values < 2^45.
//   4. carry round 2 at 29 bits (row_shr:1, row_shl:8 with 1216): limbs N-bounded
//      (< 2^29 + 2^16), lanes 9..15 cleared.
// Inputs may be N- or A-bounded (fe25519.h): 9 (2^30 + 2^24)^2 < 2^63.3, so no column
// overflows. The value is the residue of fe_mul's (limbs may differ: compare canonically).
#pragma once
#include "fe25519.h"

namespace mv {

struct fer {
  uint32_t v;  // limb (threadIdx.x & 15) of the element, zero in lanes 9..15
};

namespace r16 {

MV_DEV uint32_t lane() { return threadIdx.x & 15u; }

// DPP move with zero for lanes whose source is outside the row
template <int CTRL>
MV_DEV uint32_t dpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, true);
}
template <int I>
MV_DEV uint32_t bcast(uint32_t x) {  // lane I of the row, in every lane (row_newbcast:I)
  return dpp<0x150 + I>(x);
}
template <int I>
MV_DEV uint32_t shr(uint32_t x) {  // lane t reads lane t - I (row_shr:I), 0 for t < I
  if constexpr (I == 0) return x;
  else return dpp<0x110 + I>(x);
}
template <int I>
MV_DEV uint32_t shl(uint32_t x) {  // lane t reads lane t + I (row_shl:I), 0 for t + I > 15
  return dpp<0x100 + I>(x);
}

// lane-constant multipliers of the fold and carry steps
struct Consts {
  uint32_t mH;    // 9728 in lanes 1..7 (high halves of columns 9..15), else 0
  uint32_t m16l;  // 1216 in lane 7 (column 16's low half -> column 7)
  uint32_t m16h;  // 9728 in lane 8 (column 16's high half -> column 8)
  uint32_t m0w;   // 9728 in lane 0 (round 1: column 8's high word)
  uint32_t m0c;   // 1216 in lane 0 (round 2: limb 8's carry)
  uint32_t keep;  // all ones in lanes 0..8
};
MV_DEV Consts consts() {
  const uint32_t t = lane();
  Consts k;
  k.mH = (t >= 1 && t <= 7) ? 8 * R261 : 0u;
  k.m16l = t == 7 ? R261 : 0u;
  k.m16h = t == 8 ? 8 * R261 : 0u;
  k.m0w = t == 0 ? 8 * R261 : 0u;
  k.m0c = t == 0 ? R261 : 0u;
  k.keep = t < 9 ? 0xffffffffu : 0u;
  return k;
}

MV_DEV uint64_t mad(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }

}  // namespace r16

MV_DEV void fer_mul(fer& r, const fer& a, const fer& b, const r16::Consts& K) {
  using namespace r16;
  const uint32_t av = a.v, bv = b.v;
  // 1. columns 0..15 (lane t: column t), column 16 in every lane
  uint64_t col = (uint64_t)bcast<0>(av) * bv;
  col = mad(bcast<1>(av), shr<1>(bv), col);
  col = mad(bcast<2>(av), shr<2>(bv), col);
  col = mad(bcast<3>(av), shr<3>(bv), col);
  col = mad(bcast<4>(av), shr<4>(bv), col);
  col = mad(bcast<5>(av), shr<5>(bv), col);
  col = mad(bcast<6>(av), shr<6>(bv), col);
  col = mad(bcast<7>(av), shr<7>(bv), col);
  const uint32_t a8 = bcast<8>(av);
  col = mad(a8, shr<8>(bv), col);
  const uint64_t c16 = (uint64_t)a8 * bcast<8>(bv);
  // 2. fold columns 9..16
  const uint32_t lo = (uint32_t)col, hi = (uint32_t)(col >> 32);
  uint64_t v = mad(shl<9>(lo), R261, (uint64_t)lo | ((uint64_t)hi << 32));
  v = mad(shl<8>(hi), K.mH, v);
  v = mad((uint32_t)c16, K.m16l, v);
  v = mad((uint32_t)(c16 >> 32), K.m16h, v);
  // 3. carry round 1 at 32 bits
  const uint32_t vl = (uint32_t)v, vh = (uint32_t)(v >> 32);
  uint64_t w = (uint64_t)vl + ((uint64_t)shr<1>(vh) << 3);
  w = mad(shl<8>(vh), K.m0w, w);
  // 4. carry round 2 at 29 bits
  const uint32_t kk = __builtin_amdgcn_alignbit((uint32_t)(w >> 32), (uint32_t)w, 29);  // w >> 29 (< 2^16)
  uint32_t o = ((uint32_t)w & M29) + shr<1>(kk);
  o += __umul24(shl<8>(kk), K.m0c);
  r.v = o & K.keep;
}
MV_DEV void fer_sq(fer& r, const fer& a, const r16::Consts& K) { fer_mul(r, a, a, K); }
MV_DEV void fer_sqn(fer& r, const fer& a, int n, const r16::Consts& K) {
  fer_sq(r, a, K);
#pragma unroll 1
  for (int i = 1; i < n; i++) fer_sq(r, r, K);
}

// the element of fe form (every lane of the row holds it) in R form
MV_DEV void fer_from_fe(fer& r, const fe& a) {
  const uint32_t t = r16::lane();
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) x = t == (uint32_t)i ? a.v[i] : x;
  r.v = x;
}
// R form -> every lane of the row holds the whole element
MV_DEV void fe_from_fer(fe& r, const fer& x) {
  using namespace r16;
  r.v[0] = bcast<0>(x.v);
  r.v[1] = bcast<1>(x.v);
  r.v[2] = bcast<2>(x.v);
  r.v[3] = bcast<3>(x.v);
  r.v[4] = bcast<4>(x.v);
  r.v[5] = bcast<5>(x.v);
  r.v[6] = bcast<6>(x.v);
  r.v[7] = bcast<7>(x.v);
  r.v[8] = bcast<8>(x.v);
}

// x^((p-5)/8) on one row: fe_pow22501's addition chain (fe_q4.h's feq_pow_p58). mid() runs
// once x^(2^AT - 1) is formed: AT = 200 after 208 of 263 products, 40 after 45, 20 after 24 (a caller's
// workgroup barrier there lets other waves sync while the chain goes on)
struct NoMid {
  MV_DEV void operator()() const {}
};
template <int AT = 200, class Mid = NoMid>
MV_DEV void fer_pow_p58(fer& r, const fer& x, Mid mid = Mid()) {
  static_assert(AT == 20 || AT == 40 || AT == 200, "mid() positions");
  const r16::Consts K = r16::consts();
  fer t0, t1, t2, t3, t5, t7, t13, t15, a;
  fer_sq(t0, x, K);          // 2
  fer_sqn(t1, t0, 2, K);     // 8
  fer_mul(t2, x, t1, K);     // 9
  fer_mul(t3, t0, t2, K);    // 11
  fer_sq(a, t3, K);          // 22
  fer_mul(t5, t2, a, K);     // 2^5-1
  fer_sqn(a, t5, 5, K);
  fer_mul(t7, a, t5, K);     // 2^10-1
  fer_sqn(a, t7, 10, K);
  fer_mul(t1, a, t7, K);     // 2^20-1
  if constexpr (AT == 20) mid();
  fer_sqn(a, t1, 20, K);
  fer_mul(a, a, t1, K);      // 2^40-1
  if constexpr (AT == 40) mid();
  fer_sqn(a, a, 10, K);
  fer_mul(t13, a, t7, K);    // 2^50-1
  fer_sqn(a, t13, 50, K);
  fer_mul(t15, a, t13, K);   // 2^100-1
  fer_sqn(a, t15, 100, K);
  fer_mul(a, a, t15, K);     // 2^200-1
  if constexpr (AT == 200) mid();
  fer_sqn(a, a, 50, K);
  fer_mul(a, a, t13, K);     // 2^250-1
  fer_sqn(a, a, 2, K);
  fer_mul(r, a, x, K);       // 2^252-3
}

}  // namespace mv
