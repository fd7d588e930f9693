// GF(2^255-19) arithmetic for gfx950, one field element per lane.
//
// Representation: 9 unsaturated limbs of 29 bits (radix 2^29, 261 bits), so a
// whole column of a schoolbook product fits in 64 bits and needs no carry
// flags. Why not 8 x 32-bit limbs: on gfx950 every carry-consuming instruction
// (v_addc_co_u32 with an SGPR carry) issues at half rate, like v_mad_u64_u32
// itself, so a saturated MAC costs two half-rate slots; here a MAC is ONE
// v_mad_u64_u32 (tools/microbench_mac.hip, profiles/r01/). Additions become
// full-rate limb-wise v_add_u32 with no carry chain.
//
// Limb bounds (all arithmetic relies on them):
//   N  "normalised": every limb < 2^29 + 2^23. Output of mul, sq, sub, normalize.
//   A  lazy sum of two N values: every limb < 2^30 + 2^24. Output of fe_add.
// fe_mul / fe_sq accept N or A inputs: 9 * (2^30 + 2^24)^2 < 2^63.3, so the
// 64-bit column sums cannot overflow. fe_sub accepts N or A for both operands
// (its bias constant has every limb >= 1.5 * 2^30). fe_add needs N inputs;
// fe_addn (add + normalise) returns N. Reduction uses 2^261 = 1216 (mod p).
//
// Replaces (semantics only) curve25519-dalek-ng 4.1.1 FieldElement51, the
// field under ed25519-consensus (mysticeti-core/src/crypto.rs:25,188).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MV_DEV __device__ __forceinline__

#include "carry32.h"

namespace mv {

constexpr uint32_t M29 = (1u << 29) - 1;
constexpr uint32_t R261 = 1216;  // 2^261 mod p

struct fe {
  uint32_t v[9];
};

// ---- normalisation: carry pass, limbs < 2^32 in -> N out ----
MV_DEV void fe_normalize(fe& r) {
  uint32_t c;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    c = r.v[i] >> 29;
    r.v[i] &= M29;
    r.v[i + 1] += c;
  }
  c = r.v[8] >> 29;  // weight 2^261
  r.v[8] &= M29;
  r.v[0] += __umul24(c, R261);  // < 2^29 + 2^14
}

// ---- basic ops ----
MV_DEV void fe_set(fe& r, uint32_t x) {  // x < 2^29
  r.v[0] = x;
#pragma unroll
  for (int i = 1; i < 9; i++) r.v[i] = 0;
}
// lazy: N + N -> A (a multiplication input only)
MV_DEV void fe_add(fe& r, const fe& a, const fe& b) {
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = a.v[i] + b.v[i];
}
MV_DEV void fe_addn(fe& r, const fe& a, const fe& b) {  // (N|A) + (N|A) -> N
  fe_add(r, a, b);
  fe_normalize(r);
}
// a - b + C, C = 0 mod p with limbs in (2^31 - 2^29, 2^31]: never negative -> N
MV_DEV void fe_sub(fe& r, const fe& a, const fe& b) {
  r.v[0] = a.v[0] + (0x7fffed00u - b.v[0]);
#pragma unroll
  for (int i = 1; i < 9; i++) r.v[i] = a.v[i] + (0x7ffffffcu - b.v[i]);
  fe_normalize(r);
}
MV_DEV void fe_neg(fe& r, const fe& a) {
  fe z;
  fe_set(z, 0);
  fe_sub(r, z, a);
}

// Column-scanning reduction, shared by mul and sq. col(k) returns the 64-bit sum
// of column k (< 2^63.3). A high column k = 9..16 is folded as it is produced,
// without a carry chain: its 32-bit halves L, H go to the low columns with
// 2^261 = 1216 and 2^(261+32) = 2^(29*10) * 8 = 1216 * 8 (mod p) as one
// v_mad_u64_u32 each (L * 1216 -> column k-9, H * 9728 -> column k-8; the low
// sums stay < 2^63.3 + 2^42.3 + 2^44.6). Only the 9 low sums are live at a time.
template <class Col>
MV_DEV void fe_reduce_scan(fe& r, Col col) {
  uint64_t lo[9];
#pragma unroll
  for (int k = 0; k < 9; k++) lo[k] = col(k);
#pragma unroll
  for (int k = 9; k < 17; k++) {
    uint64_t c = col(k);
    // opaque: keeps the column one 64-bit MAD chain (otherwise the compiler may also
    // rebuild its low half from v_mul_lo_u32 products for the L * 1216 term)
    asm("" : "+v"(c));
    lo[k - 9] += (uint64_t)(uint32_t)c * R261;
    lo[k - 8] += (uint64_t)(uint32_t)(c >> 32) * (8 * R261);
  }
#pragma unroll
  for (int k = 0; k < 8; k++) {
    r.v[k] = (uint32_t)lo[k] & M29;
    lo[k + 1] += lo[k] >> 29;
  }
  r.v[8] = (uint32_t)lo[8] & M29;
  uint64_t t0 = (uint64_t)r.v[0] + (lo[8] >> 29) * R261;  // top < 2^35
  r.v[0] = (uint32_t)t0 & M29;
  r.v[1] += (uint32_t)(t0 >> 29);  // < 2^29 + 2^17
}

MV_DEV void fe_mul(fe& r, const fe& a, const fe& b) {
  fe_reduce_scan(r, [&](int k) {
    uint64_t c = 0;
#pragma unroll
    for (int i = (k > 8 ? k - 8 : 0); i <= (k < 8 ? k : 8); i++) c += (uint64_t)a.v[i] * b.v[k - i];
    return c;
  });
}
MV_DEV void fe_sq(fe& r, const fe& a_in) {
  // opaque limbs: otherwise the compiler rebuilds 2a from the producer's unmasked column
  // ((c << 1) & 0x3ffffffe beside c & 0x1fffffff: one extra instruction per limb)
  fe a;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    a.v[i] = a_in.v[i];
    asm("" : "+v"(a.v[i]));
  }
  uint32_t a2[9];
#pragma unroll
  for (int i = 0; i < 9; i++) a2[i] = a.v[i] << 1;  // < 2^31.01
  fe_reduce_scan(r, [&](int k) {
    uint64_t c = (k & 1) ? 0 : (uint64_t)a.v[k >> 1] * a.v[k >> 1];
#pragma unroll
    for (int i = (k > 8 ? k - 8 : 0); i < k - i; i++) c += (uint64_t)a2[i] * a.v[k - i];
    return c;
  });
}
MV_DEV void fe_sqn(fe& r, const fe& a, int n) {
  fe_sq(r, a);
#pragma unroll 1
  for (int i = 1; i < n; i++) fe_sq(r, r);
}
// multiply by a small constant c < 2^26 (N|A input)
MV_DEV void fe_mul_small(fe& r, const fe& a, uint32_t c) {
  uint64_t t[9];
#pragma unroll
  for (int i = 0; i < 9; i++) t[i] = (uint64_t)a.v[i] * c;  // < 2^56.1
#pragma unroll
  for (int k = 0; k < 8; k++) {
    r.v[k] = (uint32_t)t[k] & M29;
    t[k + 1] += t[k] >> 29;
  }
  r.v[8] = (uint32_t)t[8] & M29;
  uint64_t t0 = (uint64_t)r.v[0] + (t[8] >> 29) * R261;
  r.v[0] = (uint32_t)t0 & M29;
  r.v[1] += (uint32_t)(t0 >> 29);
}

// grouped forms kept for the curve formulas' readability (no carries: the
// compiler interleaves independent operations by itself)
MV_DEV void fe_mul2(fe& r0, const fe& a0, const fe& b0, fe& r1, const fe& a1, const fe& b1) {
  fe_mul(r0, a0, b0);
  fe_mul(r1, a1, b1);
}
MV_DEV void fe_sq2(fe& r0, const fe& a0, fe& r1, const fe& a1) {
  fe_sq(r0, a0);
  fe_sq(r1, a1);
}

// ---- canonical form / predicates ----
// fully reduced value in [0, p)
MV_DEV void fe_canon(fe& r, const fe& a) {
  fe t = a;
  fe_normalize(t);  // limbs < 2^29 + 2^14, value < 2^261 + small
  // fold bits >= 255 (limb 8 holds bits 232..260) with 2^255 = 19, twice
#pragma unroll
  for (int it = 0; it < 2; it++) {
    uint32_t q = t.v[8] >> 23;
    t.v[8] &= (1u << 23) - 1;
    t.v[0] += q * 19u;
    uint32_t c;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      c = t.v[i] >> 29;
      t.v[i] &= M29;
      t.v[i + 1] += c;
    }
  }
  // now t < 2^255 + tiny: subtract p iff t + 19 >= 2^255
  uint32_t u[9];
  uint32_t c = 19;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint32_t s = t.v[i] + c;
    c = s >> 29;
    u[i] = s & M29;
  }
  const bool ge = (u[8] >> 23) != 0;  // t + 19 >= 2^255
  u[8] &= (1u << 23) - 1;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = ge ? u[i] : t.v[i];
}
MV_DEV bool fe_is_zero(const fe& a) {
  fe c;
  fe_canon(c, a);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) o |= c.v[i];
  return o == 0;
}
MV_DEV bool fe_eq(const fe& a, const fe& b) {
  fe d;
  fe_sub(d, a, b);
  return fe_is_zero(d);
}
MV_DEV bool fe_is_negative(const fe& a) {
  fe c;
  fe_canon(c, a);
  return c.v[0] & 1u;
}
MV_DEV void fe_cmov(fe& r, const fe& a, bool c) {
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = c ? a.v[i] : r.v[i];
}
// 8 words (< 2^256) -> fe, all 256 bits kept (the top limb takes bits 232..255)
MV_DEV void fe_from_words_full(fe& r, const uint32_t w[8]) {
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int b = 29 * i, wi = b >> 5, s = b & 31;
    uint32_t lo = w[wi];
    uint32_t hi = (wi + 1 < 8) ? w[wi + 1] : 0u;
    r.v[i] = __builtin_amdgcn_alignbit(hi, lo, s) & M29;
  }
}
// 32 LE bytes as 8 words -> fe; bit 255 dropped, value NOT range-checked (ZIP-215)
MV_DEV void fe_from_words(fe& r, const uint32_t w[8]) {
  fe_from_words_full(r, w);
  r.v[8] &= (1u << 23) - 1;  // bits 232..254
}
// canonical fe -> 8 LE words
MV_DEV void fe_to_words(uint32_t w[8], const fe& a) {
  fe c;
  fe_canon(c, a);
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int b = 32 * j, li = b / 29, s = b % 29;
    uint32_t x = c.v[li] >> s;
    if (li + 1 < 9) x |= c.v[li + 1] << (29 - s);
    if (s > 26 && li + 2 < 9) x |= c.v[li + 2] << (58 - s);
    w[j] = x;
  }
}

// ---- exponentiation chains ----
// (x^(2^250-1), x^11), shared by inversion and the square-root exponent.
MV_DEV void fe_pow22501(fe& t19, fe& t3, const fe& x) {
  fe t0, t1, t2, t5, t7, t13, t15, a;
  fe_sq(t0, x);           // 2
  fe_sqn(t1, t0, 2);      // 8
  fe_mul(t2, x, t1);      // 9
  fe_mul(t3, t0, t2);     // 11
  fe_sq(a, t3);           // 22
  fe_mul(t5, t2, a);      // 2^5-1
  fe_sqn(a, t5, 5);
  fe_mul(t7, a, t5);      // 2^10-1
  fe_sqn(a, t7, 10);
  fe_mul(t1, a, t7);      // 2^20-1
  fe_sqn(a, t1, 20);
  fe_mul(a, a, t1);       // 2^40-1
  fe_sqn(a, a, 10);
  fe_mul(t13, a, t7);     // 2^50-1
  fe_sqn(a, t13, 50);
  fe_mul(t15, a, t13);    // 2^100-1
  fe_sqn(a, t15, 100);
  fe_mul(a, a, t15);      // 2^200-1
  fe_sqn(a, a, 50);
  fe_mul(t19, a, t13);    // 2^250-1
}
MV_DEV void fe_invert(fe& r, const fe& x) {
  fe t19, t3;
  fe_pow22501(t19, t3, x);
  fe_sqn(t19, t19, 5);
  fe_mul(r, t19, t3);  // p-2
}
MV_DEV void fe_pow_p58(fe& r, const fe& x) {
  fe t19, t3;
  fe_pow22501(t19, t3, x);
  fe_sqn(t19, t19, 2);
  fe_mul(r, t19, x);  // (p-5)/8
}
// Two independent exponentiations in lock-step: twice the ILP per wave.
MV_DEV void fe_sq2n(fe& a, fe& b, int n) {
#pragma unroll 1
  for (int i = 0; i < n; i++) fe_sq2(a, a, b, b);
}
MV_DEV void fe_pow_p58_x2(fe& ra, fe& rb, const fe& xa, const fe& xb) {
  fe a0, b0, a2, b2, a3, b3, a5, b5, a7, b7, a13, b13, a15, b15, ta, tb;
  fe_sq2(a0, xa, b0, xb);                          // 2
  ta = a0; tb = b0; fe_sq2n(ta, tb, 2);            // 8
  fe_mul2(a2, xa, ta, b2, xb, tb);                 // 9
  fe_mul2(a3, a0, a2, b3, b0, b2);                 // 11
  fe_sq2(ta, a3, tb, b3);                          // 22
  fe_mul2(a5, a2, ta, b5, b2, tb);                 // 2^5-1
  ta = a5; tb = b5; fe_sq2n(ta, tb, 5);
  fe_mul2(a7, ta, a5, b7, tb, b5);                 // 2^10-1
  ta = a7; tb = b7; fe_sq2n(ta, tb, 10);
  fe_mul2(a2, ta, a7, b2, tb, b7);                 // 2^20-1
  ta = a2; tb = b2; fe_sq2n(ta, tb, 20);
  fe_mul2(ta, ta, a2, tb, tb, b2);                 // 2^40-1
  fe_sq2n(ta, tb, 10);
  fe_mul2(a13, ta, a7, b13, tb, b7);               // 2^50-1
  ta = a13; tb = b13; fe_sq2n(ta, tb, 50);
  fe_mul2(a15, ta, a13, b15, tb, b13);             // 2^100-1
  ta = a15; tb = b15; fe_sq2n(ta, tb, 100);
  fe_mul2(ta, ta, a15, tb, tb, b15);               // 2^200-1
  fe_sq2n(ta, tb, 50);
  fe_mul2(ta, ta, a13, tb, tb, b13);               // 2^250-1
  fe_sq2n(ta, tb, 2);
  fe_mul2(ra, ta, xa, rb, tb, xb);                 // 2^252-3
}

// fe_pow_p58_x2 without its last multiplication: (ra, rb) = (xa, xb)^(2^252 - 4), so xa and xb
// are dead from the 9th power on (the caller multiplies by x, recomputed: 18 registers fewer
// live across the 250 squarings).
MV_DEV void fe_pow_p58_x2_nox(fe& ra, fe& rb, const fe& xa, const fe& xb) {
  fe a0, b0, a2, b2, a3, b3, a5, b5, a7, b7, a13, b13, a15, b15, ta, tb;
  fe_sq2(a0, xa, b0, xb);                          // 2
  ta = a0; tb = b0; fe_sq2n(ta, tb, 2);            // 8
  fe_mul2(a2, xa, ta, b2, xb, tb);                 // 9
  fe_mul2(a3, a0, a2, b3, b0, b2);                 // 11
  fe_sq2(ta, a3, tb, b3);                          // 22
  fe_mul2(a5, a2, ta, b5, b2, tb);                 // 2^5-1
  ta = a5; tb = b5; fe_sq2n(ta, tb, 5);
  fe_mul2(a7, ta, a5, b7, tb, b5);                 // 2^10-1
  ta = a7; tb = b7; fe_sq2n(ta, tb, 10);
  fe_mul2(a2, ta, a7, b2, tb, b7);                 // 2^20-1
  ta = a2; tb = b2; fe_sq2n(ta, tb, 20);
  fe_mul2(ta, ta, a2, tb, tb, b2);                 // 2^40-1
  fe_sq2n(ta, tb, 10);
  fe_mul2(a13, ta, a7, b13, tb, b7);               // 2^50-1
  ta = a13; tb = b13; fe_sq2n(ta, tb, 50);
  fe_mul2(a15, ta, a13, b15, tb, b13);             // 2^100-1
  ta = a15; tb = b15; fe_sq2n(ta, tb, 100);
  fe_mul2(ta, ta, a15, tb, tb, b15);               // 2^200-1
  fe_sq2n(ta, tb, 50);
  fe_mul2(ta, ta, a13, tb, tb, b13);               // 2^250-1
  fe_sq2n(ta, tb, 2);                              // 2^252-4
  ra = ta;
  rb = tb;
}

}  // namespace mv
