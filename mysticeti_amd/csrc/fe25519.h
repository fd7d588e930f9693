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
// (tools/microbench_valu.hip). The 512-bit product is folded with
// 2^256 = 38 (mod p) and then 2^255 = 19.
//
// ILP / hazard structure: on gfx950 a VALU that reads an SGPR carry written by a
// VALU needs 2 wait states, and each product is one serial MAC chain. So every
// operation comes in an N-way form (fe_mul_n, fe_sq_n, fe_addsub_n) that runs N
// independent field operations in lock-step, instruction by instruction (volatile
// asm keeps the order): with N >= 3 every carry consumer sits >= 3 instructions
// after its producer (no s_nop) and N MAC chains overlap their latency. The
// curve formulas (ge25519.h) group their independent operations into these calls.
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
// Volatile: their relative order is the interleaving schedule.
MV_DEV void a_mad(uint64_t& acc, uint64_t& cm, uint32_t a, uint32_t b) {
  asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cm) : "v"(a), "v"(b));
}
MV_DEV void a_cnt(uint32_t& c2, uint64_t& cm) {  // c2 += carry
  asm volatile("v_addc_co_u32 %0, %1, %0, 0, %1" : "+v"(c2), "+s"(cm));
}
MV_DEV uint32_t add_co(uint32_t a, uint32_t b, uint64_t& cm) {
  uint32_t r;
  asm volatile("v_add_co_u32 %0, %1, %2, %3" : "=v"(r), "=s"(cm) : "v"(a), "v"(b));
  return r;
}
MV_DEV uint32_t addc_co(uint32_t a, uint32_t b, uint64_t& cm) {
  uint32_t r;
  asm volatile("v_addc_co_u32 %0, %1, %2, %3, %1" : "=v"(r), "+s"(cm) : "v"(a), "v"(b));
  return r;
}
MV_DEV uint32_t addc0(uint32_t a, uint64_t& cm) {  // a + carry, carry out
  uint32_t r;
  asm volatile("v_addc_co_u32 %0, %1, %2, 0, %1" : "=v"(r), "+s"(cm) : "v"(a));
  return r;
}
MV_DEV uint32_t sub_co(uint32_t a, uint32_t b, uint64_t& bm) {
  uint32_t r;
  asm volatile("v_sub_co_u32 %0, %1, %2, %3" : "=v"(r), "=s"(bm) : "v"(a), "v"(b));
  return r;
}
MV_DEV uint32_t subb_co(uint32_t a, uint32_t b, uint64_t& bm) {
  uint32_t r;
  asm volatile("v_subb_co_u32 %0, %1, %2, %3, %1" : "=v"(r), "+s"(bm) : "v"(a), "v"(b));
  return r;
}
MV_DEV uint32_t subb0(uint32_t a, uint64_t& bm) {  // a - borrow, borrow out
  uint32_t r;
  asm volatile("v_subb_co_u32 %0, %1, %2, 0, %1" : "=v"(r), "+s"(bm) : "v"(a));
  return r;
}
// carry/borrow bit of the lane as 0/1
MV_DEV uint32_t carry_bit(uint64_t& cm) {
  uint32_t r;
  asm volatile("v_cndmask_b32 %0, 0, 1, %1" : "=v"(r) : "s"(cm));
  return r;
}
// plain 32x32+64 -> 64 (no carry-out consumer)
MV_DEV uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t r, cm;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cm) : "v"(a), "v"(b), "v"(c));
  return r;
}
// one serial MAC into a 96-bit (acc, c2) accumulator (scalar arithmetic, not hot)
MV_DEV void mac(uint64_t& acc, uint32_t& c2, uint32_t a, uint32_t b) {
  uint64_t cm;
  a_mad(acc, cm, a, b);
  a_cnt(c2, cm);
}
// ---------------------------------------------------------------- N-way core

// r[c] (8 limbs) + 19*h[c], h[c] = 2*top[c] + bit255(r[c]); r7 keeps 31 bits.
template <int N>
MV_DEV void fold_n(fe (&r)[N], const uint32_t (&top)[N]) {
  uint32_t m[N];
#pragma unroll
  for (int c = 0; c < N; c++) {
    uint32_t h = (top[c] << 1) | (r[c].v[7] >> 31);
    r[c].v[7] &= 0x7fffffffu;
    m[c] = h * 19u;
  }
  uint64_t cm[N];
#pragma unroll
  for (int c = 0; c < N; c++) r[c].v[0] = add_co(r[c].v[0], m[c], cm[c]);
#pragma unroll
  for (int i = 1; i < 8; i++)
#pragma unroll
    for (int c = 0; c < N; c++) r[c].v[i] = addc0(r[c].v[i], cm[c]);
}

// Incremental 2^256-reduction: consumes the product limbs w_0..w_15 in column
// order, so only 8 limbs + one pending high word per element stay live.
//   k < 8 : lo[k] = w_k
//   k >= 8: u = w_k * 38 + lo[k-8]; r_{k-8} = lo(u) + hi(u_{k-9}) + carry
// then the 2^255 fold of the top word.
template <int N>
struct Reducer {
  fe r[N];
  uint32_t hprev[N];
  uint64_t cm[N];
  MV_DEV void step(int k, const uint32_t (&w)[N]) {
    if (k < 8) {
#pragma unroll
      for (int c = 0; c < N; c++) r[c].v[k] = w[c];
      return;
    }
    const int i = k - 8;
    uint32_t hi[N];
#pragma unroll
    for (int c = 0; c < N; c++) {
      uint64_t u = mad64(w[c], 38u, (uint64_t)r[c].v[i]);  // < 2^38 + 2^32
      r[c].v[i] = (uint32_t)u;
      hi[c] = (uint32_t)(u >> 32);
    }
    if (i == 1) {
#pragma unroll
      for (int c = 0; c < N; c++) r[c].v[1] = add_co(r[c].v[1], hprev[c], cm[c]);
    } else if (i > 1) {
#pragma unroll
      for (int c = 0; c < N; c++) r[c].v[i] = addc_co(r[c].v[i], hprev[c], cm[c]);
    }
#pragma unroll
    for (int c = 0; c < N; c++) hprev[c] = hi[c];
  }
  MV_DEV void finish(fe (&out)[N]);
};

template <int N>
MV_DEV void Reducer<N>::finish(fe (&out)[N]) {
  uint32_t top[N];
#pragma unroll
  for (int c = 0; c < N; c++) top[c] = addc0(hprev[c], cm[c]);  // < 2^7
  fold_n<N>(r, top);
#pragma unroll
  for (int c = 0; c < N; c++) out[c] = r[c];
}

template <int N>
MV_DEV void fe_mul_n(fe (&r)[N], const fe (&a)[N], const fe (&b)[N]) {
  Reducer<N> red;
  uint64_t acc[N];
  uint32_t c2[N];
#pragma unroll
  for (int c = 0; c < N; c++) {
    acc[c] = 0;
    c2[c] = 0;
  }
#pragma unroll
  for (int k = 0; k < 15; k++) {
#pragma unroll
    for (int i = (k > 7 ? k - 7 : 0); i <= (k < 7 ? k : 7); i++) {
      uint64_t cm[N];
#pragma unroll
      for (int c = 0; c < N; c++) a_mad(acc[c], cm[c], a[c].v[i], b[c].v[k - i]);
#pragma unroll
      for (int c = 0; c < N; c++) a_cnt(c2[c], cm[c]);
    }
    uint32_t w[N];
#pragma unroll
    for (int c = 0; c < N; c++) {
      w[c] = (uint32_t)acc[c];
      acc[c] = (acc[c] >> 32) | ((uint64_t)c2[c] << 32);
      c2[c] = 0;
    }
    red.step(k, w);
  }
  uint32_t w[N];
#pragma unroll
  for (int c = 0; c < N; c++) w[c] = (uint32_t)acc[c];
  red.step(15, w);
  red.finish(r);
}

// squaring: cross-product columns t_k, then u_k = 2 t_k + diag_k with a carry
// chain along the columns, fed straight into the reducer.
template <int N>
MV_DEV void fe_sq_n(fe (&r)[N], const fe (&a)[N]) {
  Reducer<N> red;
  uint64_t acc[N], cd[N];
  uint32_t c2[N], tprev[N], dhi[N];
#pragma unroll
  for (int c = 0; c < N; c++) {
    acc[c] = 0;
    c2[c] = 0;
    tprev[c] = 0;
  }
#pragma unroll
  for (int k = 0; k < 16; k++) {
    if (k >= 1 && k < 14) {
#pragma unroll
      for (int i = (k > 7 ? k - 7 : 0); i < k - i; i++) {
        uint64_t cm[N];
#pragma unroll
        for (int c = 0; c < N; c++) a_mad(acc[c], cm[c], a[c].v[i], a[c].v[k - i]);
#pragma unroll
        for (int c = 0; c < N; c++) a_cnt(c2[c], cm[c]);
      }
    }
    uint32_t t[N], d[N], w[N];
#pragma unroll
    for (int c = 0; c < N; c++) {
      t[c] = (uint32_t)acc[c];  // cross column k (0 for k = 0)
      acc[c] = (acc[c] >> 32) | ((uint64_t)c2[c] << 32);
      c2[c] = 0;
      if ((k & 1) == 0) {
        uint64_t sq = mad64(a[c].v[k >> 1], a[c].v[k >> 1], 0);
        d[c] = (uint32_t)sq;
        dhi[c] = (uint32_t)(sq >> 32);
      } else {
        d[c] = dhi[c];
      }
    }
    if (k == 0) {
#pragma unroll
      for (int c = 0; c < N; c++) w[c] = d[c];  // t_0 == 0
    } else if (k == 1) {
#pragma unroll
      for (int c = 0; c < N; c++) w[c] = add_co(__builtin_amdgcn_alignbit(t[c], tprev[c], 31), d[c], cd[c]);
    } else {
#pragma unroll
      for (int c = 0; c < N; c++) w[c] = addc_co(__builtin_amdgcn_alignbit(t[c], tprev[c], 31), d[c], cd[c]);
    }
#pragma unroll
    for (int c = 0; c < N; c++) tprev[c] = t[c];
    red.step(k, w);
  }
  red.finish(r);
}

// r[c] = a[c] + b[c] or, for bit c of SUB, a[c] - b[c] (computed as a + (2p - b)).
// Tight inputs; tight outputs.
template <int N, unsigned SUB>
MV_DEV void fe_addsub_n(fe (&r)[N], const fe (&a)[N], const fe (&b)[N]) {
  fe bb[N];
  uint64_t cm[N];
  // 2p - b for the subtractions (2p = 2^256 - 38 > tight b: no borrow out)
#pragma unroll
  for (int c = 0; c < N; c++) {
    if (SUB & (1u << c)) {
      bb[c].v[0] = sub_co(0xffffffdau, b[c].v[0], cm[c]);
    } else {
      bb[c] = b[c];
    }
  }
#pragma unroll
  for (int i = 1; i < 8; i++)
#pragma unroll
    for (int c = 0; c < N; c++)
      if (SUB & (1u << c)) bb[c].v[i] = subb_co(0xffffffffu, b[c].v[i], cm[c]);
#pragma unroll
  for (int c = 0; c < N; c++) r[c].v[0] = add_co(a[c].v[0], bb[c].v[0], cm[c]);
#pragma unroll
  for (int i = 1; i < 8; i++)
#pragma unroll
    for (int c = 0; c < N; c++) r[c].v[i] = addc_co(a[c].v[i], bb[c].v[i], cm[c]);
  uint32_t top[N];
#pragma unroll
  for (int c = 0; c < N; c++) top[c] = carry_bit(cm[c]);
  fold_n<N>(r, top);
}

// ---------------------------------------------------------------- scalar wrappers
MV_DEV void fe_set(fe& r, uint32_t x) {
  r.v[0] = x;
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = 0;
}
MV_DEV void fe_mul(fe& r, const fe& a, const fe& b) {
  fe ra[1], aa[1] = {a}, bb[1] = {b};
  fe_mul_n<1>(ra, aa, bb);
  r = ra[0];
}
MV_DEV void fe_sq(fe& r, const fe& a) {
  fe ra[1], aa[1] = {a};
  fe_sq_n<1>(ra, aa);
  r = ra[0];
}
MV_DEV void fe_add(fe& r, const fe& a, const fe& b) {
  fe ra[1], aa[1] = {a}, bb[1] = {b};
  fe_addsub_n<1, 0u>(ra, aa, bb);
  r = ra[0];
}
MV_DEV void fe_sub(fe& r, const fe& a, const fe& b) {
  fe ra[1], aa[1] = {a}, bb[1] = {b};
  fe_addsub_n<1, 1u>(ra, aa, bb);
  r = ra[0];
}
MV_DEV void fe_neg(fe& r, const fe& a) {
  fe z;
  fe_set(z, 0);
  fe_sub(r, z, a);
}
// two independent products / squares / adds
MV_DEV void fe_mul2(fe& r0, const fe& a0, const fe& b0, fe& r1, const fe& a1, const fe& b1) {
  fe r[2], a[2] = {a0, a1}, b[2] = {b0, b1};
  fe_mul_n<2>(r, a, b);
  r0 = r[0];
  r1 = r[1];
}
MV_DEV void fe_sq2(fe& r0, const fe& a0, fe& r1, const fe& a1) {
  fe r[2], a[2] = {a0, a1};
  fe_sq_n<2>(r, a);
  r0 = r[0];
  r1 = r[1];
}
MV_DEV void fe_mul3(fe& r0, const fe& a0, const fe& b0, fe& r1, const fe& a1, const fe& b1, fe& r2, const fe& a2,
                    const fe& b2) {
  fe r[3], a[3] = {a0, a1, a2}, b[3] = {b0, b1, b2};
  fe_mul_n<3>(r, a, b);
  r0 = r[0];
  r1 = r[1];
  r2 = r[2];
}
MV_DEV void fe_mul4(fe& r0, const fe& a0, const fe& b0, fe& r1, const fe& a1, const fe& b1, fe& r2, const fe& a2,
                    const fe& b2, fe& r3, const fe& a3, const fe& b3) {
  fe r[4], a[4] = {a0, a1, a2, a3}, b[4] = {b0, b1, b2, b3};
  fe_mul_n<4>(r, a, b);
  r0 = r[0];
  r1 = r[1];
  r2 = r[2];
  r3 = r[3];
}
MV_DEV void fe_sq4(fe& r0, const fe& a0, fe& r1, const fe& a1, fe& r2, const fe& a2, fe& r3, const fe& a3) {
  fe r[4], a[4] = {a0, a1, a2, a3};
  fe_sq_n<4>(r, a);
  r0 = r[0];
  r1 = r[1];
  r2 = r[2];
  r3 = r[3];
}
template <unsigned SUB>
MV_DEV void fe_addsub2(fe& r0, const fe& a0, const fe& b0, fe& r1, const fe& a1, const fe& b1) {
  fe r[2], a[2] = {a0, a1}, b[2] = {b0, b1};
  fe_addsub_n<2, SUB>(r, a, b);
  r0 = r[0];
  r1 = r[1];
}
template <unsigned SUB>
MV_DEV void fe_addsub3(fe& r0, const fe& a0, const fe& b0, fe& r1, const fe& a1, const fe& b1, fe& r2,
                       const fe& a2, const fe& b2) {
  fe r[3], a[3] = {a0, a1, a2}, b[3] = {b0, b1, b2};
  fe_addsub_n<3, SUB>(r, a, b);
  r0 = r[0];
  r1 = r[1];
  r2 = r[2];
}
template <unsigned SUB>
MV_DEV void fe_addsub4(fe& r0, const fe& a0, const fe& b0, fe& r1, const fe& a1, const fe& b1, fe& r2,
                       const fe& a2, const fe& b2, fe& r3, const fe& a3, const fe& b3) {
  fe r[4], a[4] = {a0, a1, a2, a3}, b[4] = {b0, b1, b2, b3};
  fe_addsub_n<4, SUB>(r, a, b);
  r0 = r[0];
  r1 = r[1];
  r2 = r[2];
  r3 = r[3];
}

MV_DEV void fe_sqn(fe& r, const fe& a, int n) {
  fe_sq(r, a);
#pragma unroll 1
  for (int i = 1; i < n; i++) fe_sq(r, r);
}
// multiply by a small constant (< 2^26)
MV_DEV void fe_mul_small(fe& r, const fe& a, uint32_t c) {
  uint32_t lo[8], hi[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t u = mad64(a.v[i], c, 0);
    lo[i] = (uint32_t)u;
    hi[i] = (uint32_t)(u >> 32);
  }
  uint64_t cm;
  fe rr[1];
  rr[0].v[0] = lo[0];
  rr[0].v[1] = add_co(lo[1], hi[0], cm);
#pragma unroll
  for (int i = 2; i < 8; i++) rr[0].v[i] = addc_co(lo[i], hi[i - 1], cm);
  uint32_t top[1] = {addc0(hi[7], cm)};
  fold_n<1>(rr, top);  // top < 2^26: h*19 < 2^32
  r = rr[0];
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

}  // namespace mv
