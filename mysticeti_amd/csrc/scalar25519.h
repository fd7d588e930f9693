// Scalars mod l = 2^252 + 27742317777372353535851937790883648493 on gfx950,
// one per lane, 8 little-endian 32-bit words.
//
// Replaces (semantics) curve25519-dalek-ng 4.1.1 Scalar::from_bytes_wide (the
// challenge k = SHA-512(R||A||M) mod l), Scalar::from_canonical_bytes (s < l)
// and, for signing, the scalar multiply-add S = r + k*a mod l.
#pragma once
#include "fe25519.h"

namespace mv {

__constant__ const uint32_t SC_L[8] = {0x5cf5d3ed, 0x5812631a, 0xa2f79cd6, 0x14def9de, 0, 0, 0, 0x10000000};
// mu = floor(2^512 / l), 9 words
__constant__ const uint32_t SC_MU[9] = {0x0a2c131b, 0xed9ce5a3, 0x086329a7, 0x2106215d, 0xffffffeb,
                                        0xffffffff, 0xffffffff, 0xffffffff, 0xf};

// s < l (which also rejects bit 255): Scalar::from_canonical_bytes
MV_DEV bool sc_is_canonical(const uint32_t s[8]) {
  uint64_t bm;
  (void)sub_co(s[0], SC_L[0], bm);
#pragma unroll
  for (int i = 1; i < 8; i++) (void)subb_co(s[i], SC_L[i], bm);
  return carry_bit(bm) != 0;  // borrow <=> s < l
}

// Barrett reduction (b = 2^32, k = 8) of a 512-bit value x[16] mod l.
MV_DEV void sc_reduce512(uint32_t r[8], const uint32_t x[16]) {
  // q2 = floor(x / 2^224) * mu; only words >= 9 are needed (q3)
  uint32_t q2[18];
#pragma unroll
  for (int i = 0; i < 18; i++) q2[i] = 0;
  {
    uint64_t acc = 0;
    uint32_t c2 = 0;
#pragma unroll
    for (int k = 0; k < 17; k++) {
#pragma unroll
      for (int i = (k > 8 ? k - 8 : 0); i <= (k < 8 ? k : 8); i++) mac(acc, c2, x[7 + i], SC_MU[k - i]);
      q2[k] = (uint32_t)acc;
      acc = (acc >> 32) | ((uint64_t)c2 << 32);
      c2 = 0;
    }
    q2[17] = (uint32_t)acc;
  }
  const uint32_t* q3 = q2 + 9;
  // r2 = q3 * l mod 2^288
  uint32_t r2[9];
  {
    uint64_t acc = 0;
    uint32_t c2 = 0;
#pragma unroll
    for (int k = 0; k < 9; k++) {
#pragma unroll
      for (int i = 0; i <= k; i++)
        if (k - i < 8) mac(acc, c2, q3[i], SC_L[k - i]);
      r2[k] = (uint32_t)acc;
      acc = (acc >> 32) | ((uint64_t)c2 << 32);
      c2 = 0;
    }
  }
  uint32_t rr[9];
  uint64_t bm;
  rr[0] = sub_co(x[0], r2[0], bm);
#pragma unroll
  for (int i = 1; i < 9; i++) rr[i] = subb_co(x[i], r2[i], bm);
#pragma unroll
  for (int it = 0; it < 2; it++) {
    uint32_t s[9];
    uint64_t b2;
    s[0] = sub_co(rr[0], SC_L[0], b2);
#pragma unroll
    for (int i = 1; i < 8; i++) s[i] = subb_co(rr[i], SC_L[i], b2);
    s[8] = subb0(rr[8], b2);
    bool ge = carry_bit(b2) == 0;
#pragma unroll
    for (int i = 0; i < 9; i++) rr[i] = ge ? s[i] : rr[i];
  }
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = rr[i];
}

// (a*b + c) mod l for a, b, c < 2^256
MV_DEV void sc_muladd(uint32_t r[8], const uint32_t a[8], const uint32_t b[8], const uint32_t c[8]) {
  uint32_t t[16];
  uint64_t acc = 0;
  uint32_t c2 = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
#pragma unroll
    for (int i = (k > 7 ? k - 7 : 0); i <= (k < 7 ? k : 7); i++) mac(acc, c2, a[i], b[k - i]);
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)c2 << 32);
    c2 = 0;
  }
  t[15] = (uint32_t)acc;
  uint64_t cm;
  t[0] = add_co(t[0], c[0], cm);
#pragma unroll
  for (int i = 1; i < 8; i++) t[i] = addc_co(t[i], c[i], cm);
#pragma unroll
  for (int i = 8; i < 16; i++) t[i] = addc0(t[i], cm);
  sc_reduce512(r, t);
}

// Signed radix-16 recoding of k < 2^253: 64 digits in [-8, 7], packed as
// 4-bit two's complement, digit i in bits 4(i%8).. of word i/8.
MV_DEV void sc_recode16(uint32_t out[8], const uint32_t k[8]) {
  uint32_t carry = 0;
#pragma unroll
  for (int w = 0; w < 8; w++) {
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint32_t d = ((k[w] >> (4 * j)) & 15u) + carry;
      carry = (d + 8) >> 4;  // d in [8, 16] -> digit d - 16, carry 1
      d = (d - (carry << 4)) & 15u;
      o |= d << (4 * j);
    }
    out[w] = o;
  }
}
// Signed radix-256 recoding of s < 2^253 (s < l; signing reduces its secret scalar
// mod l first): 32 digits in [-128, 127] packed as int8 bytes, digit i in byte i. The
// top digit is at most 0x10 + 1, so no carry leaves the last byte.
MV_DEV void sc_recode256(uint32_t out[8], const uint32_t s[8]) {
  uint32_t carry = 0;
#pragma unroll
  for (int w = 0; w < 8; w++) {
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      uint32_t d = ((s[w] >> (8 * j)) & 255u) + carry;
      carry = (d + 128) >> 8;  // d in [128, 256] -> digit d - 256, carry 1
      d = (d - (carry << 8)) & 255u;
      o |= d << (8 * j);
    }
    out[w] = o;
  }
}

// Signed radix-16 recoding of a value < 2^127 (4 words): 32 digits in [-8, 7]. The
// top nibble is at most 7 and absorbs the last carry (d + carry <= 7 needs x < 2^127
// with top nibble <= 6, which the half-size scalars below satisfy).
MV_DEV void sc_recode16_128(uint32_t out[4], const uint32_t x[4]) {
  uint32_t carry = 0;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint32_t d = ((x[w] >> (4 * j)) & 15u) + carry;
      carry = (d + 8) >> 4;
      d = (d - (carry << 4)) & 15u;
      o |= d << (4 * j);
    }
    out[w] = o;
  }
}

// bit length of an 8-word value (0 for 0)
MV_DEV int len256(const uint32_t x[8]) {
  int L = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) L = x[i] ? 32 * i + 32 - (int)__clz(x[i]) : L;
  return L;
}
// r = x << s mod 2^(32 NW), 0 <= s < 256 (per-lane s: funnel shifts, then a
// 3-stage word-select network instead of dynamic register indexing)
template <int NW>
MV_DEV void shl_var(uint32_t (&r)[NW], const uint32_t (&x)[NW], int s) {
  const int bsh = s & 31, ws = s >> 5;
#pragma unroll
  for (int i = NW - 1; i >= 0; i--) {
    const uint64_t pair = ((uint64_t)x[i] << 32) | (i ? x[i - 1] : 0u);
    r[i] = (uint32_t)(pair >> (32 - bsh));
  }
#pragma unroll
  for (int k = 1; k <= 4; k <<= 1) {
    const bool on = (ws & k) != 0;
#pragma unroll
    for (int i = NW - 1; i >= 0; i--) r[i] = on ? (i >= k ? r[i - k] : 0u) : r[i];
  }
}

// Half-size scalars for verification (T. Pornin, "Optimized lattice basis reduction
// in dimension 2, and fast Schnorr and EdDSA signature verification", 2020): find
// c, d with c = d*k (mod l), |c| < 2^126, 0 < d < 2^127, so that
//   [8]([s]B - [k]A - R) = O  <=>  [8]([d*s mod l]B - [c]A - [d]R) = O
// (d is invertible mod l; c - d*k is a multiple of l, which [8] kills on A's
// torsion part). The reduction is the extended-Euclid remainder sequence of (l, k),
// quotients applied as shift-subtract steps, stopped at the first remainder below
// 2^126 (Thue): its cofactor t satisfies |t| <= l / 2^126 < 2^127. t is tracked mod
// 2^128 (every intermediate cofactor is below 2^127 in magnitude). Each step drops
// len(a) + len(b) by at least one, so the loop ends within ~380 steps; for random k it
// takes ~110 (64-lane max ~125).
// Output: c as magnitude (4 words) + sign, d (4 words).
MV_DEV void sc_halfsize(uint32_t c[4], bool& c_neg, uint32_t d[4], const uint32_t k[8]) {
  uint32_t a[8], b[8], ta[4], tb[4];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a[i] = SC_L[i];
    b[i] = k[i];
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    ta[i] = 0;
    tb[i] = i == 0;
  }
  int la = 253, lb = len256(b);
  bool done = lb <= 126;
  if (done) {  // k itself is short: (c, d) = (k, 1)
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = b[i];
#pragma unroll
    for (int i = 0; i < 4; i++) ta[i] = tb[i];
  }
  while (!done) {
    const int s = la - lb;
    uint32_t bs[8], x[8];
    shl_var<8>(bs, b, s);
    uint64_t bm;
    x[0] = sub_co(a[0], bs[0], bm);
#pragma unroll
    for (int i = 1; i < 8; i++) x[i] = subb_co(a[i], bs[i], bm);
    const uint32_t over = carry_bit(bm);  // b << s > a: use b << (s - 1), s >= 1
    if (over) {
      uint64_t cm;
      uint32_t h[8];
#pragma unroll
      for (int i = 0; i < 8; i++) h[i] = (bs[i] >> 1) | (i < 7 ? bs[i + 1] << 31 : 0u);
      x[0] = add_co(x[0], h[0], cm);
#pragma unroll
      for (int i = 1; i < 8; i++) x[i] = addc_co(x[i], h[i], cm);
    }
    uint32_t ts[4];
    shl_var<4>(ts, tb, s - (int)over);
    uint64_t tm;
    ta[0] = sub_co(ta[0], ts[0], tm);
#pragma unroll
    for (int i = 1; i < 4; i++) ta[i] = subb_co(ta[i], ts[i], tm);
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = x[i];
    la = len256(a);
    if (la <= 126) {
      done = true;
    } else {
      uint64_t cm;
      (void)sub_co(a[0], b[0], cm);
#pragma unroll
      for (int i = 1; i < 8; i++) (void)subb_co(a[i], b[i], cm);
      if (carry_bit(cm)) {  // a < b: swap roles
#pragma unroll
        for (int i = 0; i < 8; i++) {
          const uint32_t t = a[i];
          a[i] = b[i];
          b[i] = t;
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const uint32_t t = ta[i];
          ta[i] = tb[i];
          tb[i] = t;
        }
        const int t = la;
        la = lb;
        lb = t;
      }
    }
  }
  // d = ta (signed); make d positive, moving the sign to c = a
  c_neg = (int32_t)ta[3] < 0;
  uint64_t nm;
  uint32_t nd[4];
  nd[0] = sub_co(0u, ta[0], nm);
#pragma unroll
  for (int i = 1; i < 4; i++) nd[i] = subb_co(0u, ta[i], nm);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    d[i] = c_neg ? nd[i] : ta[i];
    c[i] = a[i];
  }
}

// uniform-index word pick without dynamic register indexing
MV_DEV uint32_t pick8(const uint32_t a[8], int idx) {
  uint32_t r = a[0];
#pragma unroll
  for (int i = 1; i < 8; i++) r = (idx == i) ? a[i] : r;
  return r;
}
MV_DEV int digit16(const uint32_t kd[8], int i) {
  uint32_t w = pick8(kd, i >> 3);
  return ((int)(w << (28 - 4 * (i & 7)))) >> 28;
}
MV_DEV int digit256(const uint32_t sd[8], int i) {
  uint32_t w = pick8(sd, i >> 2);
  return ((int)(w << (24 - 8 * (i & 3)))) >> 24;
}

}  // namespace mv
