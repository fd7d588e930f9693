/* ORACLE / TEST INFRASTRUCTURE ONLY — see oracle.h.
 *
 * Restatement of ed25519-consensus 2.1.0 VerificationKey::verify (ZIP-215,
 * called at mysticeti-core/src/crypto.rs:188) on the arithmetic structure of
 * curve25519-dalek-ng 4.1.1's u64 backend:
 *   - GF(2^255-19) in 5 x 51-bit limbs with 128-bit products;
 *   - extended / projective / completed / (projective|affine) Niels points;
 *   - EdwardsPoint::vartime_double_scalar_mul_basepoint = Straus with a
 *     width-5 NAF for the variable point and width-8 NAF for the basepoint;
 *   - ZIP-215 decompress (y read from 255 bits without a range check), s < l,
 *     k = SHA-512(R || A || M) mod l, accept <=> [8](R - R') is the identity.
 * Signing (RFC 8032) is here only to build corpora.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "oracle.h"

typedef unsigned __int128 u128;
typedef struct {
  uint64_t v[5];
} fe;

#define M51 ((1ULL << 51) - 1)

static void fe_frombytes(fe* h, const uint8_t s[32]) {
  uint64_t w[4];
  for (int i = 0; i < 4; i++) {
    w[i] = 0;
    for (int j = 7; j >= 0; j--) w[i] = (w[i] << 8) | s[8 * i + j];
  }
  h->v[0] = w[0] & M51;
  h->v[1] = ((w[0] >> 51) | (w[1] << 13)) & M51;
  h->v[2] = ((w[1] >> 38) | (w[2] << 26)) & M51;
  h->v[3] = ((w[2] >> 25) | (w[3] << 39)) & M51;
  h->v[4] = (w[3] >> 12) & M51; /* bit 255 dropped; value NOT range-checked (ZIP-215) */
}

static void fe_carry(fe* h) {
  uint64_t c;
  c = h->v[0] >> 51; h->v[0] &= M51; h->v[1] += c;
  c = h->v[1] >> 51; h->v[1] &= M51; h->v[2] += c;
  c = h->v[2] >> 51; h->v[2] &= M51; h->v[3] += c;
  c = h->v[3] >> 51; h->v[3] &= M51; h->v[4] += c;
  c = h->v[4] >> 51; h->v[4] &= M51; h->v[0] += 19 * c;
}

static void fe_tobytes(uint8_t s[32], const fe* f) {
  fe h = *f;
  fe_carry(&h);
  fe_carry(&h);
  /* q = 1 iff h >= p */
  uint64_t q = (h.v[0] + 19) >> 51;
  q = (h.v[1] + q) >> 51;
  q = (h.v[2] + q) >> 51;
  q = (h.v[3] + q) >> 51;
  q = (h.v[4] + q) >> 51;
  h.v[0] += 19 * q;
  uint64_t c;
  c = h.v[0] >> 51; h.v[0] &= M51; h.v[1] += c;
  c = h.v[1] >> 51; h.v[1] &= M51; h.v[2] += c;
  c = h.v[2] >> 51; h.v[2] &= M51; h.v[3] += c;
  c = h.v[3] >> 51; h.v[3] &= M51; h.v[4] += c;
  h.v[4] &= M51;
  uint64_t w[4];
  w[0] = h.v[0] | (h.v[1] << 51);
  w[1] = (h.v[1] >> 13) | (h.v[2] << 38);
  w[2] = (h.v[2] >> 26) | (h.v[3] << 25);
  w[3] = (h.v[3] >> 39) | (h.v[4] << 12);
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 8; j++) s[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

static const fe FE_ZERO = {{0, 0, 0, 0, 0}};
static const fe FE_ONE = {{1, 0, 0, 0, 0}};

static inline void fe_add(fe* h, const fe* a, const fe* b) {
  for (int i = 0; i < 5; i++) h->v[i] = a->v[i] + b->v[i];
}
/* a - b computed as a + 16p - b, then carried (inputs limbs < 2^54). */
static inline void fe_sub(fe* h, const fe* a, const fe* b) {
  h->v[0] = (a->v[0] + 36028797018963664ULL) - b->v[0];
  h->v[1] = (a->v[1] + 36028797018963952ULL) - b->v[1];
  h->v[2] = (a->v[2] + 36028797018963952ULL) - b->v[2];
  h->v[3] = (a->v[3] + 36028797018963952ULL) - b->v[3];
  h->v[4] = (a->v[4] + 36028797018963952ULL) - b->v[4];
  fe_carry(h);
}
static inline void fe_neg(fe* h, const fe* a) { fe_sub(h, &FE_ZERO, a); }

static void fe_mul(fe* h, const fe* a, const fe* b) {
  const uint64_t *x = a->v, *y = b->v;
  uint64_t y1_19 = 19 * y[1], y2_19 = 19 * y[2], y3_19 = 19 * y[3], y4_19 = 19 * y[4];
  u128 c0 = (u128)x[0] * y[0] + (u128)x[4] * y1_19 + (u128)x[3] * y2_19 + (u128)x[2] * y3_19 + (u128)x[1] * y4_19;
  u128 c1 = (u128)x[1] * y[0] + (u128)x[0] * y[1] + (u128)x[4] * y2_19 + (u128)x[3] * y3_19 + (u128)x[2] * y4_19;
  u128 c2 = (u128)x[2] * y[0] + (u128)x[1] * y[1] + (u128)x[0] * y[2] + (u128)x[4] * y3_19 + (u128)x[3] * y4_19;
  u128 c3 = (u128)x[3] * y[0] + (u128)x[2] * y[1] + (u128)x[1] * y[2] + (u128)x[0] * y[3] + (u128)x[4] * y4_19;
  u128 c4 = (u128)x[4] * y[0] + (u128)x[3] * y[1] + (u128)x[2] * y[2] + (u128)x[1] * y[3] + (u128)x[0] * y[4];
  c1 += (uint64_t)(c0 >> 51);
  c2 += (uint64_t)(c1 >> 51);
  c3 += (uint64_t)(c2 >> 51);
  c4 += (uint64_t)(c3 >> 51);
  uint64_t carry = (uint64_t)(c4 >> 51);
  h->v[0] = ((uint64_t)c0 & M51) + 19 * carry;
  h->v[1] = (uint64_t)c1 & M51;
  h->v[2] = (uint64_t)c2 & M51;
  h->v[3] = (uint64_t)c3 & M51;
  h->v[4] = (uint64_t)c4 & M51;
  h->v[1] += h->v[0] >> 51;
  h->v[0] &= M51;
}

static void fe_sq(fe* h, const fe* a) {
  const uint64_t* x = a->v;
  uint64_t x0_2 = 2 * x[0], x1_2 = 2 * x[1], x3_19 = 19 * x[3], x4_19 = 19 * x[4];
  u128 c0 = (u128)x[0] * x[0] + (u128)x1_2 * x4_19 + (u128)(2 * x[2]) * x3_19;
  u128 c1 = (u128)x0_2 * x[1] + (u128)x[3] * x3_19 + (u128)(2 * x[2]) * x4_19;
  u128 c2 = (u128)x0_2 * x[2] + (u128)x[1] * x[1] + (u128)(2 * x[3]) * x4_19;
  u128 c3 = (u128)x0_2 * x[3] + (u128)x1_2 * x[2] + (u128)x[4] * x4_19;
  u128 c4 = (u128)x0_2 * x[4] + (u128)x1_2 * x[3] + (u128)x[2] * x[2];
  c1 += (uint64_t)(c0 >> 51);
  c2 += (uint64_t)(c1 >> 51);
  c3 += (uint64_t)(c2 >> 51);
  c4 += (uint64_t)(c3 >> 51);
  uint64_t carry = (uint64_t)(c4 >> 51);
  h->v[0] = ((uint64_t)c0 & M51) + 19 * carry;
  h->v[1] = (uint64_t)c1 & M51;
  h->v[2] = (uint64_t)c2 & M51;
  h->v[3] = (uint64_t)c3 & M51;
  h->v[4] = (uint64_t)c4 & M51;
  h->v[1] += h->v[0] >> 51;
  h->v[0] &= M51;
}
static void fe_sqn(fe* h, const fe* a, int n) {
  fe_sq(h, a);
  for (int i = 1; i < n; i++) fe_sq(h, h);
}

/* (x^(2^250-1), x^11) — the shared addition chain of invert and pow_p58. */
static void fe_pow22501(fe* t19, fe* t3, const fe* x) {
  fe t0, t1, t2, t4, t5, t6, t7, t8, t9, t10, t11, t12, t13, t14, t15, t16, t17, t18;
  fe_sq(&t0, x);                /* 2 */
  fe_sqn(&t1, &t0, 2);          /* 8 */
  fe_mul(&t2, x, &t1);          /* 9 */
  fe_mul(t3, &t0, &t2);         /* 11 */
  fe_sq(&t4, t3);               /* 22 */
  fe_mul(&t5, &t2, &t4);        /* 2^5-1 */
  fe_sqn(&t6, &t5, 5);
  fe_mul(&t7, &t6, &t5);        /* 2^10-1 */
  fe_sqn(&t8, &t7, 10);
  fe_mul(&t9, &t8, &t7);        /* 2^20-1 */
  fe_sqn(&t10, &t9, 20);
  fe_mul(&t11, &t10, &t9);      /* 2^40-1 */
  fe_sqn(&t12, &t11, 10);
  fe_mul(&t13, &t12, &t7);      /* 2^50-1 */
  fe_sqn(&t14, &t13, 50);
  fe_mul(&t15, &t14, &t13);     /* 2^100-1 */
  fe_sqn(&t16, &t15, 100);
  fe_mul(&t17, &t16, &t15);     /* 2^200-1 */
  fe_sqn(&t18, &t17, 50);
  fe_mul(t19, &t18, &t13);      /* 2^250-1 */
}
static void fe_invert(fe* out, const fe* x) {
  fe t19, t3, t20;
  fe_pow22501(&t19, &t3, x);
  fe_sqn(&t20, &t19, 5);
  fe_mul(out, &t20, &t3); /* 2^255-21 = p-2 */
}
static void fe_pow_p58(fe* out, const fe* x) {
  fe t19, t3, t20;
  fe_pow22501(&t19, &t3, x);
  fe_sqn(&t20, &t19, 2);
  fe_mul(out, &t20, x); /* 2^252-3 = (p-5)/8 */
}
static int fe_eq(const fe* a, const fe* b) {
  uint8_t x[32], y[32];
  fe_tobytes(x, a);
  fe_tobytes(y, b);
  return memcmp(x, y, 32) == 0;
}
static int fe_is_negative(const fe* a) {
  uint8_t x[32];
  fe_tobytes(x, a);
  return x[0] & 1;
}
static int fe_is_zero(const fe* a) { return fe_eq(a, &FE_ZERO); }

/* constants, computed once by orc_init() from their definitions */
static fe FE_D, FE_D2, FE_SQRT_M1;

/* dalek sqrt_ratio_i: returns 1 iff u/v is a square (u == 0 included); r >= 0. */
static int fe_sqrt_ratio_i(fe* r, const fe* u, const fe* v) {
  fe v3, v7, t, uv7, check, neg_u, neg_u_i, r_prime;
  fe_sq(&t, v);
  fe_mul(&v3, &t, v);
  fe_sq(&t, &v3);
  fe_mul(&v7, &t, v);
  fe_mul(&uv7, u, &v7);
  fe_pow_p58(&t, &uv7);
  fe_mul(&t, &t, &v3);
  fe_mul(r, &t, u);
  fe_sq(&t, r);
  fe_mul(&check, v, &t);
  fe_neg(&neg_u, u);
  fe_mul(&neg_u_i, &neg_u, &FE_SQRT_M1);
  int correct = fe_eq(&check, u);
  int flipped = fe_eq(&check, &neg_u);
  int flipped_i = fe_eq(&check, &neg_u_i);
  fe_mul(&r_prime, &FE_SQRT_M1, r);
  if (flipped || flipped_i) *r = r_prime;
  if (fe_is_negative(r)) fe_neg(r, r);
  return correct || flipped;
}

/* ---------------- points ---------------- */
typedef struct { fe X, Y, Z, T; } ge_ext;
typedef struct { fe X, Y, Z; } ge_proj;
typedef struct { fe X, Y, Z, T; } ge_cmp; /* completed: x = X/Z, y = Y/T */
typedef struct { fe YpX, YmX, Z, T2d; } ge_pniels;
typedef struct { fe ypx, ymx, xy2d; } ge_aniels;

static void ext_identity(ge_ext* p) {
  p->X = FE_ZERO; p->Y = FE_ONE; p->Z = FE_ONE; p->T = FE_ZERO;
}
static void ext_to_pniels(ge_pniels* n, const ge_ext* p) {
  fe_add(&n->YpX, &p->Y, &p->X);
  fe_sub(&n->YmX, &p->Y, &p->X);
  n->Z = p->Z;
  fe_mul(&n->T2d, &p->T, &FE_D2);
}
static void ext_to_proj(ge_proj* r, const ge_ext* p) { r->X = p->X; r->Y = p->Y; r->Z = p->Z; }
static void cmp_to_ext(ge_ext* r, const ge_cmp* c) {
  fe_mul(&r->X, &c->X, &c->T);
  fe_mul(&r->Y, &c->Y, &c->Z);
  fe_mul(&r->Z, &c->Z, &c->T);
  fe_mul(&r->T, &c->X, &c->Y);
}
static void cmp_to_proj(ge_proj* r, const ge_cmp* c) {
  fe_mul(&r->X, &c->X, &c->T);
  fe_mul(&r->Y, &c->Y, &c->Z);
  fe_mul(&r->Z, &c->Z, &c->T);
}
static void proj_double(ge_cmp* c, const ge_proj* p) {
  fe XX, YY, ZZ2, XpY, XpY2, YYpXX, YYmXX;
  fe_sq(&XX, &p->X);
  fe_sq(&YY, &p->Y);
  fe_sq(&ZZ2, &p->Z);
  fe_add(&ZZ2, &ZZ2, &ZZ2);
  fe_add(&XpY, &p->X, &p->Y);
  fe_sq(&XpY2, &XpY);
  fe_add(&YYpXX, &YY, &XX);
  fe_sub(&YYmXX, &YY, &XX);
  fe_sub(&c->X, &XpY2, &YYpXX);
  c->Y = YYpXX;
  c->Z = YYmXX;
  fe_sub(&c->T, &ZZ2, &YYmXX);
}
static void ext_add_pniels(ge_cmp* c, const ge_ext* p, const ge_pniels* q, int sub) {
  fe YpX, YmX, PP, MM, TT2d, ZZ, ZZ2;
  fe_add(&YpX, &p->Y, &p->X);
  fe_sub(&YmX, &p->Y, &p->X);
  fe_mul(&PP, &YpX, sub ? &q->YmX : &q->YpX);
  fe_mul(&MM, &YmX, sub ? &q->YpX : &q->YmX);
  fe_mul(&TT2d, &p->T, &q->T2d);
  fe_mul(&ZZ, &p->Z, &q->Z);
  fe_add(&ZZ2, &ZZ, &ZZ);
  fe_sub(&c->X, &PP, &MM);
  fe_add(&c->Y, &PP, &MM);
  if (sub) {
    fe_sub(&c->Z, &ZZ2, &TT2d);
    fe_add(&c->T, &ZZ2, &TT2d);
  } else {
    fe_add(&c->Z, &ZZ2, &TT2d);
    fe_sub(&c->T, &ZZ2, &TT2d);
  }
}
static void ext_add_aniels(ge_cmp* c, const ge_ext* p, const ge_aniels* q, int sub) {
  fe YpX, YmX, PP, MM, Txy2d, Z2;
  fe_add(&YpX, &p->Y, &p->X);
  fe_sub(&YmX, &p->Y, &p->X);
  fe_mul(&PP, &YpX, sub ? &q->ymx : &q->ypx);
  fe_mul(&MM, &YmX, sub ? &q->ypx : &q->ymx);
  fe_mul(&Txy2d, &p->T, &q->xy2d);
  fe_add(&Z2, &p->Z, &p->Z);
  fe_sub(&c->X, &PP, &MM);
  fe_add(&c->Y, &PP, &MM);
  if (sub) {
    fe_sub(&c->Z, &Z2, &Txy2d);
    fe_add(&c->T, &Z2, &Txy2d);
  } else {
    fe_add(&c->Z, &Z2, &Txy2d);
    fe_sub(&c->T, &Z2, &Txy2d);
  }
}
static void ext_add(ge_ext* r, const ge_ext* p, const ge_ext* q) {
  ge_pniels n;
  ge_cmp c;
  ext_to_pniels(&n, q);
  ext_add_pniels(&c, p, &n, 0);
  cmp_to_ext(r, &c);
}
static void ext_sub(ge_ext* r, const ge_ext* p, const ge_ext* q) {
  ge_pniels n;
  ge_cmp c;
  ext_to_pniels(&n, q);
  ext_add_pniels(&c, p, &n, 1);
  cmp_to_ext(r, &c);
}
static void ext_double(ge_ext* r, const ge_ext* p) {
  ge_proj q;
  ge_cmp c;
  ext_to_proj(&q, p);
  proj_double(&c, &q);
  cmp_to_ext(r, &c);
}
static void ext_neg(ge_ext* r, const ge_ext* p) {
  fe_neg(&r->X, &p->X);
  r->Y = p->Y;
  r->Z = p->Z;
  fe_neg(&r->T, &p->T);
}
static int ext_is_identity(const ge_ext* p) {
  /* compress(P) == compress(identity)  <=>  X == 0 and Y == Z (mod p) */
  return fe_is_zero(&p->X) && fe_eq(&p->Y, &p->Z);
}
static void ext_compress(uint8_t s[32], const ge_ext* p) {
  fe zi, x, y;
  fe_invert(&zi, &p->Z);
  fe_mul(&x, &p->X, &zi);
  fe_mul(&y, &p->Y, &zi);
  fe_tobytes(s, &y);
  s[31] ^= (uint8_t)(fe_is_negative(&x) << 7);
}
/* CompressedEdwardsY::decompress, ZIP-215 rules. */
static int ext_decompress(ge_ext* p, const uint8_t s[32]) {
  fe u, v, yy;
  fe_frombytes(&p->Y, s);
  p->Z = FE_ONE;
  fe_sq(&yy, &p->Y);
  fe_sub(&u, &yy, &FE_ONE);
  fe_mul(&v, &yy, &FE_D);
  fe_add(&v, &v, &FE_ONE);
  if (!fe_sqrt_ratio_i(&p->X, &u, &v)) return 0;
  if (s[31] >> 7) fe_neg(&p->X, &p->X); /* x == 0 with sign bit set: accepted */
  fe_mul(&p->T, &p->X, &p->Y);
  return 1;
}

/* ---------------- scalars mod l ---------------- */
/* l = 2^252 + 27742317777372353535851937790883648493, little-endian 32-bit words */
static const uint32_t L32[8] = {0x5cf5d3ed, 0x5812631a, 0xa2f79cd6, 0x14def9de, 0, 0, 0, 0x10000000};
/* mu = floor(2^512 / l), 9 words */
static const uint32_t MU32[9] = {0x0a2c131b, 0xed9ce5a3, 0x086329a7, 0x2106215d,
                                 0xffffffeb, 0xffffffff, 0xffffffff, 0xffffffff, 0xf};

/* Barrett reduction (HAC 14.42, b = 2^32, k = 8) of a 512-bit LE integer mod l. */
static void sc_reduce512(uint32_t r[8], const uint32_t x[16]) {
  /* q1 = floor(x / b^(k-1)) : words 7..15 */
  const uint32_t* q1 = x + 7;
  uint32_t q2[18];
  memset(q2, 0, sizeof q2);
  for (int i = 0; i < 9; i++) {
    uint64_t c = 0;
    for (int j = 0; j < 9; j++) {
      uint64_t t = (uint64_t)q1[i] * MU32[j] + q2[i + j] + c;
      q2[i + j] = (uint32_t)t;
      c = t >> 32;
    }
    q2[i + 9] = (uint32_t)c;
  }
  const uint32_t* q3 = q2 + 9; /* floor(q2 / b^(k+1)) */
  /* r2 = (q3 * l) mod b^(k+1) */
  uint32_t r2[9];
  memset(r2, 0, sizeof r2);
  for (int i = 0; i < 9; i++) {
    uint64_t c = 0;
    for (int j = 0; j < 8 && i + j < 9; j++) {
      uint64_t t = (uint64_t)q3[i] * L32[j] + r2[i + j] + c;
      r2[i + j] = (uint32_t)t;
      c = t >> 32;
    }
    if (i + 8 < 9) r2[i + 8] += (uint32_t)c;
  }
  /* r = (x mod b^(k+1)) - r2, wrapping mod b^(k+1) */
  uint32_t rr[9];
  int64_t br = 0;
  for (int i = 0; i < 9; i++) {
    int64_t t = (int64_t)x[i] - (int64_t)r2[i] + br;
    rr[i] = (uint32_t)t;
    br = t >> 32;
  }
  for (int it = 0; it < 2; it++) { /* r < 3l: at most two subtractions */
    uint32_t s[9];
    int64_t b = 0;
    for (int i = 0; i < 9; i++) {
      int64_t t = (int64_t)rr[i] - (int64_t)(i < 8 ? L32[i] : 0) + b;
      s[i] = (uint32_t)t;
      b = t >> 32;
    }
    if (b == 0) memcpy(rr, s, sizeof s);
  }
  memcpy(r, rr, 32);
}

static void sc_from_bytes_wide(uint32_t r[8], const uint8_t in[64]) {
  uint32_t x[16];
  for (int i = 0; i < 16; i++)
    x[i] = (uint32_t)in[4 * i] | ((uint32_t)in[4 * i + 1] << 8) | ((uint32_t)in[4 * i + 2] << 16) |
           ((uint32_t)in[4 * i + 3] << 24);
  sc_reduce512(r, x);
}
void orc_scalar_reduce_wide(const uint8_t in[64], uint8_t out[32]) {
  uint32_t r[8];
  sc_from_bytes_wide(r, in);
  for (int i = 0; i < 32; i++) out[i] = (uint8_t)(r[i / 4] >> (8 * (i % 4)));
}
static void sc_to_bytes(uint8_t out[32], const uint32_t r[8]) {
  for (int i = 0; i < 32; i++) out[i] = (uint8_t)(r[i / 4] >> (8 * (i % 4)));
}
/* Scalar::from_canonical_bytes: high bit clear and value < l */
static int sc_is_canonical(const uint8_t s[32]) {
  if (s[31] >> 7) return 0;
  for (int i = 7; i >= 0; i--) {
    uint32_t w = (uint32_t)s[4 * i] | ((uint32_t)s[4 * i + 1] << 8) | ((uint32_t)s[4 * i + 2] << 16) |
                 ((uint32_t)s[4 * i + 3] << 24);
    if (w < L32[i]) return 1;
    if (w > L32[i]) return 0;
  }
  return 0; /* == l */
}
/* width-w NAF of a scalar < 2^255 (bytes LE): 256 digits, odd, |d| < 2^(w-1) */
static void sc_naf(int8_t naf[256], const uint8_t s[32], int w) {
  uint64_t x[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++)
    for (int j = 7; j >= 0; j--) x[i] = (x[i] << 8) | s[8 * i + j];
  memset(naf, 0, 256);
  int width = 1 << w, mask = width - 1;
  int pos = 0, carry = 0;
  while (pos < 256) {
    int idx = pos / 64, bit = pos % 64;
    uint64_t bits = (bit < 64 - w) ? (x[idx] >> bit) : ((x[idx] >> bit) | (x[idx + 1] << (64 - bit)));
    int window = carry + (int)(bits & (uint64_t)mask);
    if ((window & 1) == 0) {
      pos += 1;
      continue;
    }
    if (window < width / 2) {
      carry = 0;
      naf[pos] = (int8_t)window;
    } else {
      carry = 1;
      naf[pos] = (int8_t)(window - width);
    }
    pos += w;
  }
}

static ge_ext GE_B;
static ge_aniels B_ODD[64]; /* B, 3B, ..., 127B */
static void pniels_to_aniels(ge_aniels* a, const ge_ext* p) {
  fe zi, x, y, xy;
  fe_invert(&zi, &p->Z);
  fe_mul(&x, &p->X, &zi);
  fe_mul(&y, &p->Y, &zi);
  fe_add(&a->ypx, &y, &x);
  fe_sub(&a->ymx, &y, &x);
  fe_mul(&xy, &x, &y);
  fe_mul(&a->xy2d, &xy, &FE_D2);
}

static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static void orc_init(void) {
  /* d = -121665/121666 */
  fe n121665 = {{121665, 0, 0, 0, 0}}, n121666 = {{121666, 0, 0, 0, 0}}, inv;
  fe_invert(&inv, &n121666);
  fe_mul(&FE_D, &n121665, &inv);
  fe_neg(&FE_D, &FE_D);
  fe_add(&FE_D2, &FE_D, &FE_D);
  fe_carry(&FE_D2);
  /* sqrt(-1) = 2^((p-1)/4) */
  fe two = {{2, 0, 0, 0, 0}}, t;
  /* (p-1)/4 = 2^253 - 5: compute 2^(2^253-5) = 2^(2^253) / 2^5 via exponent chain on base 2 */
  /* 2^((p-1)/4) = (2^((p-5)/8))^2 * 2 ; (p-5)/8 = 2^252-3 */
  fe_pow_p58(&t, &two);
  fe_sq(&t, &t);
  fe_mul(&FE_SQRT_M1, &t, &two);
  /* B: y = 4/5, x non-negative */
  fe four = {{4, 0, 0, 0, 0}}, five = {{5, 0, 0, 0, 0}}, y;
  fe_invert(&inv, &five);
  fe_mul(&y, &four, &inv);
  uint8_t enc[32];
  fe_tobytes(enc, &y);
  ext_decompress(&GE_B, enc);
  ge_ext b2, cur;
  ext_double(&b2, &GE_B);
  cur = GE_B;
  for (int i = 0; i < 64; i++) {
    pniels_to_aniels(&B_ODD[i], &cur);
    ext_add(&cur, &cur, &b2);
  }
}
static void ensure_init(void) { pthread_once(&g_once, orc_init); }

/* EdwardsPoint::vartime_double_scalar_mul_basepoint(a, A, b) = [a]A + [b]B */
static void double_scalar_mul_basepoint(ge_ext* out, const uint8_t a[32], const ge_ext* A, const uint8_t b[32]) {
  int8_t a_naf[256], b_naf[256];
  sc_naf(a_naf, a, 5);
  sc_naf(b_naf, b, 8);
  int i = 255;
  while (i >= 0 && a_naf[i] == 0 && b_naf[i] == 0) i--;
  ge_pniels tableA[8];
  ge_ext A2, cur = *A;
  ext_double(&A2, A);
  for (int k = 0; k < 8; k++) {
    ext_to_pniels(&tableA[k], &cur);
    ext_add(&cur, &cur, &A2);
  }
  ge_proj r;
  r.X = FE_ZERO; r.Y = FE_ONE; r.Z = FE_ONE;
  for (; i >= 0; i--) {
    ge_cmp t;
    ge_ext e;
    proj_double(&t, &r);
    if (a_naf[i] > 0) {
      cmp_to_ext(&e, &t);
      ext_add_pniels(&t, &e, &tableA[a_naf[i] / 2], 0);
    } else if (a_naf[i] < 0) {
      cmp_to_ext(&e, &t);
      ext_add_pniels(&t, &e, &tableA[-a_naf[i] / 2], 1);
    }
    if (b_naf[i] > 0) {
      cmp_to_ext(&e, &t);
      ext_add_aniels(&t, &e, &B_ODD[b_naf[i] / 2], 0);
    } else if (b_naf[i] < 0) {
      cmp_to_ext(&e, &t);
      ext_add_aniels(&t, &e, &B_ODD[-b_naf[i] / 2], 1);
    }
    cmp_to_proj(&r, &t);
  }
  out->X = r.X; out->Y = r.Y; out->Z = r.Z;
  fe_mul(&out->X, &r.X, &r.Z);
  fe_mul(&out->Y, &r.Y, &r.Z);
  fe_sq(&out->Z, &r.Z);
  fe_mul(&out->T, &r.X, &r.Y);
}

int orc_point_decodes(const uint8_t enc[32]) {
  ensure_init();
  ge_ext p;
  return ext_decompress(&p, enc);
}

/* VerificationKey (ed25519-consensus 2.1.0): the key bytes and -A, decoded once at
 * VerificationKey::try_from; the reference's committee keys are built that way once per
 * authority (crypto.rs:25, committee.rs:83-87), so per-block verifies start from -A. */
struct orc_vk {
  uint8_t bytes[32];
  int ok;
  ge_ext minusA;
};
size_t orc_vk_size(void) { return sizeof(struct orc_vk); }
int orc_vk_init(orc_vk* vk, const uint8_t pk[32]) {
  ensure_init();
  ge_ext A;
  memcpy(vk->bytes, pk, 32);
  vk->ok = ext_decompress(&A, pk);
  if (vk->ok) ext_neg(&vk->minusA, &A);
  return vk->ok;
}

int orc_ed25519_verify_vk(const orc_vk* vk, const uint8_t sig[64], const uint8_t* msg, size_t msg_len) {
  ensure_init();
  if (!vk->ok) return ORC_SIG_MALFORMED_KEY;
  const uint8_t* pk = vk->bytes;
  const ge_ext minusA = vk->minusA;
  ge_ext R, Rp, diff;
  if (!sc_is_canonical(sig + 32)) return ORC_SIG_INVALID;
  if (!ext_decompress(&R, sig)) return ORC_SIG_INVALID;
  uint8_t h[64], k[32];
  uint8_t stackbuf[64 + 256];
  uint8_t* buf = msg_len <= 256 ? stackbuf : (uint8_t*)malloc(64 + msg_len);
  memcpy(buf, sig, 32);
  memcpy(buf + 32, pk, 32);
  memcpy(buf + 64, msg, msg_len);
  orc_sha512(buf, 64 + msg_len, h);
  if (buf != stackbuf) free(buf);
  uint32_t kw[8];
  sc_from_bytes_wide(kw, h);
  sc_to_bytes(k, kw);
  double_scalar_mul_basepoint(&Rp, k, &minusA, sig + 32);
  ext_sub(&diff, &R, &Rp);
  ext_double(&diff, &diff);
  ext_double(&diff, &diff);
  ext_double(&diff, &diff);
  return ext_is_identity(&diff) ? ORC_SIG_OK : ORC_SIG_INVALID;
}

int orc_ed25519_verify(const uint8_t pk[32], const uint8_t sig[64], const uint8_t* msg, size_t msg_len) {
  orc_vk vk;
  if (!orc_vk_init(&vk, pk)) return ORC_SIG_MALFORMED_KEY; /* VerificationKey::try_from */
  return orc_ed25519_verify_vk(&vk, sig, msg, msg_len);
}

static void clamp_secret(uint8_t a[32], const uint8_t h[32]) {
  memcpy(a, h, 32);
  a[0] &= 248;
  a[31] &= 127;
  a[31] |= 64;
}
static void basepoint_mul(ge_ext* out, const uint8_t s[32]) {
  uint8_t zero[32] = {0};
  ge_ext id;
  ext_identity(&id);
  double_scalar_mul_basepoint(out, zero, &id, s);
}

void orc_ed25519_pubkey(const uint8_t seed[32], uint8_t pk[32]) {
  ensure_init();
  uint8_t h[64], a[32];
  ge_ext A;
  orc_sha512(seed, 32, h);
  clamp_secret(a, h);
  uint8_t a_wide[64] = {0}, a_red[32];
  memcpy(a_wide, a, 32);
  orc_scalar_reduce_wide(a_wide, a_red); /* [a]B == [a mod l]B; keeps the NAF within 256 digits */
  basepoint_mul(&A, a_red);
  ext_compress(pk, &A);
}

/* r = (a*b + c) mod l, all 32-byte LE */
static void sc_muladd(uint8_t out[32], const uint8_t a[32], const uint8_t b[32], const uint8_t c[32]) {
  uint32_t aw[8], bw[8], x[16];
  for (int i = 0; i < 8; i++) {
    aw[i] = (uint32_t)a[4 * i] | ((uint32_t)a[4 * i + 1] << 8) | ((uint32_t)a[4 * i + 2] << 16) |
            ((uint32_t)a[4 * i + 3] << 24);
    bw[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
            ((uint32_t)b[4 * i + 3] << 24);
  }
  memset(x, 0, sizeof x);
  for (int i = 0; i < 8; i++) {
    uint64_t cy = 0;
    for (int j = 0; j < 8; j++) {
      uint64_t t = (uint64_t)aw[i] * bw[j] + x[i + j] + cy;
      x[i + j] = (uint32_t)t;
      cy = t >> 32;
    }
    x[i + 8] = (uint32_t)cy;
  }
  uint64_t cy = 0;
  for (int i = 0; i < 16; i++) {
    uint64_t cw = i < 8 ? ((uint32_t)c[4 * i] | ((uint32_t)c[4 * i + 1] << 8) | ((uint32_t)c[4 * i + 2] << 16) |
                           ((uint32_t)c[4 * i + 3] << 24))
                        : 0;
    uint64_t t = (uint64_t)x[i] + cw + cy;
    x[i] = (uint32_t)t;
    cy = t >> 32;
  }
  uint32_t r[8];
  sc_reduce512(r, x);
  sc_to_bytes(out, r);
}

void orc_ed25519_sign(const uint8_t seed[32], const uint8_t* msg, size_t msg_len, uint8_t sig[64]) {
  ensure_init();
  uint8_t h[64], a[32], pk[32], rh[64], r[32], kh[64], k[32];
  ge_ext A, Rp;
  orc_sha512(seed, 32, h);
  clamp_secret(a, h);
  uint8_t a_wide[64] = {0}, a_red[32];
  memcpy(a_wide, a, 32);
  orc_scalar_reduce_wide(a_wide, a_red);
  basepoint_mul(&A, a_red);
  ext_compress(pk, &A);
  uint8_t buf[32 + 256];
  if (msg_len > 256) return;
  memcpy(buf, h + 32, 32);
  memcpy(buf + 32, msg, msg_len);
  orc_sha512(buf, 32 + msg_len, rh);
  orc_scalar_reduce_wide(rh, r);
  basepoint_mul(&Rp, r);
  ext_compress(sig, &Rp);
  uint8_t kbuf[64 + 256];
  memcpy(kbuf, sig, 32);
  memcpy(kbuf + 32, pk, 32);
  memcpy(kbuf + 64, msg, msg_len);
  orc_sha512(kbuf, 64 + msg_len, kh);
  orc_scalar_reduce_wide(kh, k);
  sc_muladd(sig + 32, k, a_red, r);
}

/* ---------------- threaded batches (persistent pool, pool.c) ---------------- */
typedef struct {
  const uint8_t *pk, *sig, *msg, *seed;
  uint8_t *status, *pk_out, *sig_out;
} batch_job;

static void verify_item(void* arg, size_t i) {
  batch_job* j = (batch_job*)arg;
  j->status[i] = (uint8_t)orc_ed25519_verify(j->pk + 32 * i, j->sig + 64 * i, j->msg + 32 * i, 32);
}
static void sign_item(void* arg, size_t i) {
  batch_job* j = (batch_job*)arg;
  orc_ed25519_pubkey(j->seed + 32 * i, j->pk_out + 32 * i);
  orc_ed25519_sign(j->seed + 32 * i, j->msg + 32 * i, 32, j->sig_out + 64 * i);
}

void orc_ed25519_verify_batch(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg32, size_t n,
                              uint8_t* status, int threads) {
  ensure_init();
  batch_job j = {pk, sig, msg32, NULL, status, NULL, NULL};
  orc_parallel_for(n, threads, 64, verify_item, &j);
}
void orc_ed25519_sign_batch(const uint8_t* seed, const uint8_t* msg32, size_t n, uint8_t* pk, uint8_t* sig,
                            int threads) {
  ensure_init();
  batch_job j = {NULL, NULL, msg32, seed, NULL, pk, sig};
  orc_parallel_for(n, threads, 64, sign_item, &j);
}
