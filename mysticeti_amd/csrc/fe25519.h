// GF(2^255-19) arithmetic for gfx950, one field element per lane.
//
// Representation: 8 x 32-bit limbs (radix 2^32, little-endian), value held
// loosely in [0, 2^256); every operation returns a "tight" value
// < 2^255 + 2^14, which every operation accepts as input. Canonical form is
// produced only for comparisons and encoding.
//
// Multiplication is product-scanning (column-wise) on v_mad_u64_u32 with its
// carry-out into a third accumulator word (v_addc_co_u32): 3 issue slots per
// 32x32 MAC on CDNA4, where v_mad_u64_u32 issues at half the full VALU rate
// (tools/microbench_valu.hip, profiles/r01_microbench_valu*.jsonl). The
// 512-bit product is folded with 2^256 = 38 (mod p) and then 2^255 = 19.
//
// Replaces (semantics only) curve25519-dalek-ng 4.1.1 FieldElement51, the
// field under ed25519-consensus (mysticeti-core/src/crypto.rs:25,188).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MV_DEV __device__ __forceinline__

namespace mv {

struct fe {
  uint32_t v[8];
};

// ---- carry-flag primitives (wave64 carry masks live in SGPR pairs) ----
MV_DEV void mac(uint64_t& acc, uint32_t& c2, uint32_t a, uint32_t b) {
  uint64_t cm;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cm) : "v"(a), "v"(b));
  asm("v_addc_co_u32 %0, %1, %2, 0, %1" : "=v"(c2), "+s"(cm) : "v"(c2));
}
MV_DEV uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t r, cm;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cm) : "v"(a), "v"(b), "v"(c));
  return r;
}
MV_DEV uint32_t add_co(uint32_t a, uint32_t b, uint64_t& cm) {
  uint32_t r;
  asm("v_add_co_u32 %0, %1, %2, %3" : "=v"(r), "=s"(cm) : "v"(a), "v"(b));
  return r;
}
MV_DEV uint32_t addc_co(uint32_t a, uint32_t b, uint64_t& cm) {
  uint32_t r;
  asm("v_addc_co_u32 %0, %1, %2, %3, %1" : "=v"(r), "+s"(cm) : "v"(a), "v"(b));
  return r;
}
MV_DEV uint32_t addc0(uint32_t a, uint64_t& cm) {  // a + carry, carry out
  uint32_t r;
  asm("v_addc_co_u32 %0, %1, %2, 0, %1" : "=v"(r), "+s"(cm) : "v"(a));
  return r;
}
MV_DEV uint32_t sub_co(uint32_t a, uint32_t b, uint64_t& bm) {
  uint32_t r;
  asm("v_sub_co_u32 %0, %1, %2, %3" : "=v"(r), "=s"(bm) : "v"(a), "v"(b));
  return r;
}
MV_DEV uint32_t subb_co(uint32_t a, uint32_t b, uint64_t& bm) {
  uint32_t r;
  asm("v_subb_co_u32 %0, %1, %2, %3, %1" : "=v"(r), "+s"(bm) : "v"(a), "v"(b));
  return r;
}
MV_DEV uint32_t subb0(uint32_t a, uint64_t& bm) {  // a - borrow, borrow out
  uint32_t r;
  asm("v_subb_co_u32 %0, %1, %2, 0, %1" : "=v"(r), "+s"(bm) : "v"(a));
  return r;
}
// carry/borrow bit of the lane as 0/1
MV_DEV uint32_t carry_bit(uint64_t& cm) {
  uint32_t r;
  asm("v_cndmask_b32 %0, 0, 1, %1" : "=v"(r) : "s"(cm));
  return r;
}

// ---- folding ----
// r (8 limbs) + 19*h where h < 2^9 is the part of the value at or above 2^255:
// r7 keeps only its low 31 bits. Result < 2^255 + 19*2^9 (tight).
MV_DEV void fold255(fe& r, uint32_t top) {
  // top: bits >= 256 (small); h = top*2 + bit255
  uint32_t h = (top << 1) | (r.v[7] >> 31);
  r.v[7] &= 0x7fffffffu;
  uint32_t m = h * 19u;
  uint64_t cm;
  r.v[0] = add_co(r.v[0], m, cm);
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = addc0(r.v[i], cm);
}

// ---- basic ops ----
MV_DEV void fe_set(fe& r, uint32_t x) {
  r.v[0] = x;
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = 0;
}
MV_DEV void fe_add(fe& r, const fe& a, const fe& b) {
  uint64_t cm;
  r.v[0] = add_co(a.v[0], b.v[0], cm);
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = addc_co(a.v[i], b.v[i], cm);
  fold255(r, carry_bit(cm));
}
// a - b for tight a, b: a - b + 2p when it would borrow, then fold bit 255.
MV_DEV void fe_sub(fe& r, const fe& a, const fe& b) {
  uint64_t bm;
  r.v[0] = sub_co(a.v[0], b.v[0], bm);
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = subb_co(a.v[i], b.v[i], bm);
  // borrowed: value is a-b+2^256; subtract 38 to make it a-b+2p (no further borrow: a-b > -2^255-2^14)
  uint32_t m = carry_bit(bm) * 38u;
  uint64_t b2;
  r.v[0] = sub_co(r.v[0], m, b2);
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = subb0(r.v[i], b2);
  fold255(r, 0);
}
MV_DEV void fe_neg(fe& r, const fe& a) {
  fe z;
  fe_set(z, 0);
  fe_sub(r, z, a);
}
// 2^256-reduction of a 512-bit product t[16] -> tight r
MV_DEV void fe_reduce_wide(fe& r, const uint32_t t[16]) {
  uint32_t lo[8], hi[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t u = mad64(t[8 + i], 38u, (uint64_t)t[i]);  // < 2^38 + 2^32
    lo[i] = (uint32_t)u;
    hi[i] = (uint32_t)(u >> 32);
  }
  uint64_t cm;
  r.v[0] = lo[0];
  r.v[1] = add_co(lo[1], hi[0], cm);
#pragma unroll
  for (int i = 2; i < 8; i++) r.v[i] = addc_co(lo[i], hi[i - 1], cm);
  uint32_t top = addc0(hi[7], cm);  // < 2^7
  fold255(r, top);
}
MV_DEV void fe_mul(fe& r, const fe& a, const fe& b) {
  uint32_t t[16];
  uint64_t acc = 0;
  uint32_t c2 = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
#pragma unroll
    for (int i = (k > 7 ? k - 7 : 0); i <= (k < 7 ? k : 7); i++) mac(acc, c2, a.v[i], b.v[k - i]);
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)c2 << 32);
    c2 = 0;
  }
  t[15] = (uint32_t)acc;
  fe_reduce_wide(r, t);
}
// squaring: cross products once, doubled, plus the diagonal
MV_DEV void fe_sq(fe& r, const fe& a) {
  uint32_t t[16];
  uint64_t acc = 0;
  uint32_t c2 = 0;
  t[0] = 0;
#pragma unroll
  for (int k = 1; k < 14; k++) {
#pragma unroll
    for (int i = (k > 7 ? k - 7 : 0); i < k - i; i++) mac(acc, c2, a.v[i], a.v[k - i]);
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)c2 << 32);
    c2 = 0;
  }
  t[14] = (uint32_t)acc;
  t[15] = (uint32_t)(acc >> 32);
  // t = 2*t + diag
  uint32_t d[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t s = (uint64_t)a.v[i] * a.v[i];
    d[2 * i] = (uint32_t)s;
    d[2 * i + 1] = (uint32_t)(s >> 32);
  }
  uint32_t u[16];
  uint64_t cm;
  u[0] = d[0];  // t[0] == 0
  u[1] = add_co(__builtin_amdgcn_alignbit(t[1], t[0], 31), d[1], cm);
#pragma unroll
  for (int i = 2; i < 16; i++) u[i] = addc_co(__builtin_amdgcn_alignbit(t[i], t[i - 1], 31), d[i], cm);
  fe_reduce_wide(r, u);
}
MV_DEV void fe_sqn(fe& r, const fe& a, int n) {
  fe_sq(r, a);
  for (int i = 1; i < n; i++) fe_sq(r, r);
}
// multiply by a small constant (< 2^26)
MV_DEV void fe_mul_small(fe& r, const fe& a, uint32_t c) {
  uint32_t lo[8], hi[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t u = (uint64_t)a.v[i] * c;
    lo[i] = (uint32_t)u;
    hi[i] = (uint32_t)(u >> 32);
  }
  uint64_t cm;
  r.v[0] = lo[0];
  r.v[1] = add_co(lo[1], hi[0], cm);
#pragma unroll
  for (int i = 2; i < 8; i++) r.v[i] = addc_co(lo[i], hi[i - 1], cm);
  uint32_t top = addc0(hi[7], cm);
  // top * 2^256 = top * 38; fold through 2^255
  fold255(r, top);
}

// ---- canonical form / predicates ----
MV_DEV void fe_canon(fe& r, const fe& a) {
  // a tight (< 2p): subtract p iff a + 19 >= 2^255
  fe t;
  uint64_t cm;
  t.v[0] = add_co(a.v[0], 19u, cm);
#pragma unroll
  for (int i = 1; i < 8; i++) t.v[i] = addc0(a.v[i], cm);
  bool ge = (t.v[7] >> 31) != 0;
  t.v[7] &= 0x7fffffffu;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = ge ? t.v[i] : a.v[i];
}
MV_DEV bool fe_is_zero(const fe& a) {
  fe c;
  fe_canon(c, a);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= c.v[i];
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
  for (int i = 0; i < 8; i++) r.v[i] = c ? a.v[i] : r.v[i];
}
// decode 32 LE bytes given as 8 words; bit 255 dropped, value NOT range-checked (ZIP-215)
MV_DEV void fe_from_words(fe& r, const uint32_t w[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = w[i];
  r.v[7] &= 0x7fffffffu;
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
  for (int i = 0; i < n; i++) {
    fe_sq(a, a);
    fe_sq(b, b);
  }
}
MV_DEV void fe_pow_p58_x2(fe& ra, fe& rb, const fe& xa, const fe& xb) {
  fe a0, b0, a2, b2, a3, b3, a5, b5, a7, b7, a13, b13, a15, b15, ta, tb;
  fe_sq(a0, xa); fe_sq(b0, xb);                 // 2
  ta = a0; tb = b0; fe_sq2n(ta, tb, 2);         // 8
  fe_mul(a2, xa, ta); fe_mul(b2, xb, tb);       // 9
  fe_mul(a3, a0, a2); fe_mul(b3, b0, b2);       // 11
  fe_sq(ta, a3); fe_sq(tb, b3);                 // 22
  fe_mul(a5, a2, ta); fe_mul(b5, b2, tb);       // 2^5-1
  ta = a5; tb = b5; fe_sq2n(ta, tb, 5);
  fe_mul(a7, ta, a5); fe_mul(b7, tb, b5);       // 2^10-1
  ta = a7; tb = b7; fe_sq2n(ta, tb, 10);
  fe_mul(a2, ta, a7); fe_mul(b2, tb, b7);       // 2^20-1
  ta = a2; tb = b2; fe_sq2n(ta, tb, 20);
  fe_mul(ta, ta, a2); fe_mul(tb, tb, b2);       // 2^40-1
  fe_sq2n(ta, tb, 10);
  fe_mul(a13, ta, a7); fe_mul(b13, tb, b7);     // 2^50-1
  ta = a13; tb = b13; fe_sq2n(ta, tb, 50);
  fe_mul(a15, ta, a13); fe_mul(b15, tb, b13);   // 2^100-1
  ta = a15; tb = b15; fe_sq2n(ta, tb, 100);
  fe_mul(ta, ta, a15); fe_mul(tb, tb, b15);     // 2^200-1
  fe_sq2n(ta, tb, 50);
  fe_mul(ta, ta, a13); fe_mul(tb, tb, b13);     // 2^250-1
  fe_sq2n(ta, tb, 2);
  fe_mul(ra, ta, xa); fe_mul(rb, tb, xb);       // 2^252-3
}

}  // namespace mv
