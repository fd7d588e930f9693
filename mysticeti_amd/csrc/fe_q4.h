// GF(2^255-19) multiplication with FOUR lanes per field element (gfx950), for latency-bound
// exponentiation chains: the ZIP-215 decode of R on the online block path (comb.hip), where
// one lane per signature runs ~265 field operations back to back and each one is ~180 issue
// slots on a single wave.
//
// Q form: lane c of an aligned quad holds rows t = 0..2 = limbs 4t + c of fe25519.h's 9 x 29-bit
// representation (row 2 is limb 8 in lane 0 and zero in lanes 1..3). A product r = a b:
//   1. every lane gathers the whole of a (9 quad broadcasts) and the window
//      bs[m] = b[m + c], m = -3..8 (zero outside 0..8), from its neighbours (DPP quad_perm;
//      bs[0], bs[4], bs[8] are its own rows);
//   2. lane c sums the columns k = 4r + c, r = 0..4: col(k) = sum_i a[i] bs[4r - i], 27
//      v_mad_u64_u32 per lane (81 products over four lanes, with a few zero ones);
//   3. the high columns fold as in fe_reduce_scan (2^261 = 1216, 2^293 = 9728 mod p): the
//      9728 half stays in the lane (column k - 8 is row r - 2), the 1216 half moves one lane
//      down (column k - 9);
//   4. two carry rounds in parallel over the columns (the first 64-bit, the second 32-bit),
//      each moving carries one lane up; column 8's carry wraps to column 0 times 1216.
// Output limbs are N-bounded (< 2^29 + 2^23), inputs may be N or A (fe25519.h's bounds), and
// the value is the same residue as fe_mul's (the limbs may differ: compare canonical forms).
#pragma once
#include "fe25519.h"

namespace mv {

struct feq {
  uint32_t r[3];
};

namespace q4 {

MV_DEV uint32_t lane() { return threadIdx.x & 3u; }

template <int CTRL>
MV_DEV uint32_t dpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
MV_DEV uint64_t dpp64(uint64_t x) {
  return (uint64_t)dpp<CTRL>((uint32_t)x) | ((uint64_t)dpp<CTRL>((uint32_t)(x >> 32)) << 32);
}
// quad_perm control: lane i reads lane (i + K) & 3
template <int K>
constexpr int rot() {
  return ((0 + K) & 3) | (((1 + K) & 3) << 2) | (((2 + K) & 3) << 4) | (((3 + K) & 3) << 6);
}
template <int K>
constexpr int bcast() {
  return K | (K << 2) | (K << 4) | (K << 6);
}

// limb j of the element, in every lane
template <int J>
MV_DEV uint32_t limb(const feq& x) {
  return dpp<bcast<J % 4>()>(x.r[J / 4]);
}
// bs[M] = limb M + c of the element in lane c (zero outside 0..8), M = -3..8
template <int M>
MV_DEV uint32_t shifted(const feq& x, uint32_t c) {
  if constexpr (M == 0 || M == 4 || M == 8) {
    return x.r[M / 4];
  } else if constexpr (M < 0) {
    // sender lane s provides limb s (row 0) to lane s - M when that lane exists
    const uint32_t sv = c + (uint32_t)(-M) < 4 ? x.r[0] : 0u;
    return dpp<rot<M & 3>()>(sv);
  } else {
    static_assert(M < 8, "row U + 1 <= 2");
    constexpr int U = M / 4, V = M % 4;
    // receiver c reads lane s = (c + V) & 3, which sends row U + 1 when s < V (c + V wrapped)
    const uint32_t sv = c < (uint32_t)V ? x.r[U + 1] : x.r[U];
    return dpp<rot<V>()>(sv);
  }
}

}  // namespace q4

// the element of fe form (every lane holds it) in Q form
MV_DEV void feq_from_fe(feq& r, const fe& a) {
  const uint32_t c = q4::lane();
#pragma unroll
  for (int t = 0; t < 3; t++) {
    const uint32_t x0 = a.v[4 * t], x1 = t < 2 ? a.v[4 * t + 1] : 0u, x2 = t < 2 ? a.v[4 * t + 2] : 0u,
                   x3 = t < 2 ? a.v[4 * t + 3] : 0u;
    const uint32_t lo = c & 1u ? x1 : x0, hi = c & 1u ? x3 : x2;
    r.r[t] = c & 2u ? hi : lo;
  }
}
// Q form -> every lane holds the whole element
MV_DEV void fe_from_feq(fe& r, const feq& x) {
  r.v[0] = q4::limb<0>(x);
  r.v[1] = q4::limb<1>(x);
  r.v[2] = q4::limb<2>(x);
  r.v[3] = q4::limb<3>(x);
  r.v[4] = q4::limb<4>(x);
  r.v[5] = q4::limb<5>(x);
  r.v[6] = q4::limb<6>(x);
  r.v[7] = q4::limb<7>(x);
  r.v[8] = q4::limb<8>(x);
}

MV_DEV void feq_mul(feq& out, const feq& a, const feq& b) {
  const uint32_t c = q4::lane();
  fe A;
  fe_from_feq(A, a);
  // bs[m + 3] = limb m + c of b, m = -3..8
  uint32_t bs[12];
  bs[0] = q4::shifted<-3>(b, c);
  bs[1] = q4::shifted<-2>(b, c);
  bs[2] = q4::shifted<-1>(b, c);
  bs[3] = q4::shifted<0>(b, c);
  bs[4] = q4::shifted<1>(b, c);
  bs[5] = q4::shifted<2>(b, c);
  bs[6] = q4::shifted<3>(b, c);
  bs[7] = q4::shifted<4>(b, c);
  bs[8] = q4::shifted<5>(b, c);
  bs[9] = q4::shifted<6>(b, c);
  bs[10] = q4::shifted<7>(b, c);
  bs[11] = q4::shifted<8>(b, c);
  // columns k = 4r + c
  uint64_t col[5];
#pragma unroll
  for (int r = 0; r < 5; r++) {
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int m = 4 * r - i;
      if (m >= -3 && m <= 8) s += (uint64_t)A.v[i] * bs[m + 3];
    }
    col[r] = s;
  }
  // fold the high columns: row 2 is high in lanes 1..3 (k = 9..11) and column 8 in lane 0;
  // rows 3 and 4 are high everywhere (row 4 is zero in lanes 1..3)
  const bool l0 = c == 0;
  const uint64_t h2 = l0 ? 0ull : col[2];
  // the 9728 halves stay in the lane: row r -> row r - 2
  uint64_t lo0 = col[0] + (uint64_t)(uint32_t)(h2 >> 32) * (8 * R261);
  uint64_t lo1 = col[1] + (uint64_t)(uint32_t)(col[3] >> 32) * (8 * R261);
  uint64_t lo2 = (l0 ? col[2] : 0ull) + (uint64_t)(uint32_t)(col[4] >> 32) * (8 * R261);
  // the 1216 halves go to column k - 9: lane c - 1 (row r - 2), or from lane 0 to lane 3 (row r - 3)
  const uint64_t f2 = (uint64_t)(uint32_t)h2 * R261, f3 = (uint64_t)(uint32_t)col[3] * R261,
                 f4 = (uint64_t)(uint32_t)col[4] * R261;
  const uint64_t s0 = l0 ? f3 : f2, s1 = l0 ? f4 : f3;
  lo0 += q4::dpp64<q4::rot<1>()>(s0);
  lo1 += q4::dpp64<q4::rot<1>()>(s1);
  // carry round 1 (64-bit): column k's carry to column k + 1 (lane c + 1, or lane 3 -> lane 0
  // one row up); column 8 (lane 0, row 2) wraps to column 0 times 1216
  {
    const uint64_t k0 = lo0 >> 29, k1 = lo1 >> 29, k2 = lo2 >> 29;
    const uint64_t g0 = q4::dpp64<q4::rot<3>()>(k0), g1 = q4::dpp64<q4::rot<3>()>(k1);
    const uint64_t w = k2 * (uint64_t)R261;  // column 8's carry, weight 2^261
    lo0 = (lo0 & M29) + (l0 ? w : g0);
    lo1 = (lo1 & M29) + (l0 ? g0 : g1);
    lo2 = (lo2 & M29) + (l0 ? g1 : 0ull);
  }
  // carry round 2 (values < 2^42): the same with 32-bit carries
  {
    const uint32_t k0 = (uint32_t)(lo0 >> 29), k1 = (uint32_t)(lo1 >> 29), k2 = (uint32_t)(lo2 >> 29);
    const uint32_t g0 = q4::dpp<q4::rot<3>()>(k0), g1 = q4::dpp<q4::rot<3>()>(k1);
    out.r[0] = ((uint32_t)lo0 & M29) + (l0 ? k2 * R261 : g0);
    out.r[1] = ((uint32_t)lo1 & M29) + (l0 ? g0 : g1);
    out.r[2] = l0 ? ((uint32_t)lo2 & M29) + g1 : 0u;
  }
}
MV_DEV void feq_sq(feq& r, const feq& a) { feq_mul(r, a, a); }
MV_DEV void feq_sqn(feq& r, const feq& a, int n) {
  feq_sq(r, a);
#pragma unroll 1
  for (int i = 1; i < n; i++) feq_sq(r, r);
}

// fe_pow_p58 (x^((p-5)/8)) on four lanes: fe_pow22501's addition chain
MV_DEV void feq_pow_p58(feq& r, const feq& x) {
  feq t0, t1, t2, t3, t5, t7, t13, t15, a;
  feq_sq(t0, x);           // 2
  feq_sqn(t1, t0, 2);      // 8
  feq_mul(t2, x, t1);      // 9
  feq_mul(t3, t0, t2);     // 11
  feq_sq(a, t3);           // 22
  feq_mul(t5, t2, a);      // 2^5-1
  feq_sqn(a, t5, 5);
  feq_mul(t7, a, t5);      // 2^10-1
  feq_sqn(a, t7, 10);
  feq_mul(t1, a, t7);      // 2^20-1
  feq_sqn(a, t1, 20);
  feq_mul(a, a, t1);       // 2^40-1
  feq_sqn(a, a, 10);
  feq_mul(t13, a, t7);     // 2^50-1
  feq_sqn(a, t13, 50);
  feq_mul(t15, a, t13);    // 2^100-1
  feq_sqn(a, t15, 100);
  feq_mul(a, a, t15);      // 2^200-1
  feq_sqn(a, a, 50);
  feq_mul(a, a, t13);      // 2^250-1
  feq_sqn(a, a, 2);
  feq_mul(r, a, x);        // 2^252-3
}

}  // namespace mv
