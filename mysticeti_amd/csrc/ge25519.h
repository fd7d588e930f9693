// Edwards25519 group arithmetic on gfx950 (one point per lane).
//
// Coordinates (a = -1 twisted Edwards, d = -121665/121666):
//   p3     extended (X:Y:Z:T), x = X/Z, y = Y/Z, xy = T/Z
//   p2     projective (X:Y:Z)
//   p1p1   completed ((X:Z),(Y:T)), output of add/double before normalisation
//   cached (Y+X, Y-X, Z, 2dT)  -- variable-base table entries (scratch in HBM)
//   precomp(y+x, y-x, 2dxy)    -- fixed-base B table entries (LDS)
// Unified formulas (Hisil-Wong-Carter-Dawson 2008), so identity entries need no
// branch: every lane runs the same instruction stream.
//
// Replaces (semantics) curve25519-dalek-ng 4.1.1 EdwardsPoint / ProjectiveNiels /
// AffineNiels as used by ed25519-consensus 2.1.0 (mysticeti-core/src/crypto.rs:188).
#pragma once
#include "fe25519.h"

namespace mv {

struct p3 { fe X, Y, Z, T; };
struct p2 { fe X, Y, Z; };
struct p1p1 { fe X, Y, Z, T; };
struct cached { fe YpX, YmX, Z, T2d; };
struct precomp { fe ypx, ymx, xy2d; };

// curve constants, little-endian 32-bit words
__constant__ const uint32_t K_D[8] = {0x135978a3, 0x75eb4dca, 0x4141d8ab, 0x00700a4d,
                                      0x7779e898, 0x8cc74079, 0x2b6ffe73, 0x52036cee};
__constant__ const uint32_t K_D2[8] = {0x26b2f159, 0xebd69b94, 0x8283b156, 0x00e0149a,
                                       0xeef3d130, 0x198e80f2, 0x56dffce7, 0x2406d9dc};
__constant__ const uint32_t K_SQRTM1[8] = {0x4a0ea0b0, 0xc4ee1b27, 0xad2fe478, 0x2f431806,
                                           0x3dfbd7a7, 0x2b4d0099, 0x4fc1df0b, 0x2b832480};

MV_DEV void fe_const(fe& r, const uint32_t* c) {
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = c[i];
  fe_from_words_full(r, w);
}

MV_DEV void p3_identity(p3& p) {
  fe_set(p.X, 0); fe_set(p.Y, 1); fe_set(p.Z, 1); fe_set(p.T, 0);
}
MV_DEV void p2_identity(p2& p) {
  fe_set(p.X, 0); fe_set(p.Y, 1); fe_set(p.Z, 1);
}
MV_DEV void cached_identity(cached& c) {
  fe_set(c.YpX, 1); fe_set(c.YmX, 1); fe_set(c.Z, 1); fe_set(c.T2d, 0);
}

// Bounds (fe25519.h): p3 / p2 coordinates are N; p1p1 coordinates are N or A
// (all multiplication inputs); cached entries: YpX A, the rest N.
MV_DEV void p1p1_to_p2(p2& r, const p1p1& c) {
  fe_mul(r.X, c.X, c.T);
  fe_mul(r.Y, c.Y, c.Z);
  fe_mul(r.Z, c.Z, c.T);
}
MV_DEV void p1p1_to_p3(p3& r, const p1p1& c) {
  fe_mul(r.X, c.X, c.T);
  fe_mul(r.Y, c.Y, c.Z);
  fe_mul(r.Z, c.Z, c.T);
  fe_mul(r.T, c.X, c.Y);
}
MV_DEV void p3_to_cached(cached& r, const p3& p) {
  fe d2;
  fe_const(d2, K_D2);
  fe_add(r.YpX, p.Y, p.X);
  fe_sub(r.YmX, p.Y, p.X);
  r.Z = p.Z;
  fe_mul(r.T2d, p.T, d2);
}
// 2P from projective: 4 squarings (dbl-2008-hwcd, a = -1)
MV_DEV void p2_dbl(p1p1& r, const p2& p) {
  fe XX, YY, ZZ, S, S2, ZZ2;
  fe_add(S, p.X, p.Y);
  fe_sq(XX, p.X);
  fe_sq(YY, p.Y);
  fe_sq(ZZ, p.Z);
  fe_sq(S2, S);
  fe_add(r.Y, YY, XX);   // A
  fe_sub(r.Z, YY, XX);   // N
  fe_add(ZZ2, ZZ, ZZ);   // A
  fe_sub(r.X, S2, r.Y);  // N
  fe_sub(r.T, ZZ2, r.Z); // N
}
MV_DEV void p3_dbl(p1p1& r, const p3& p) {
  p2 q;
  q.X = p.X; q.Y = p.Y; q.Z = p.Z;
  p2_dbl(r, q);
}
// P + Q (Q cached): 4 multiplications
MV_DEV void p3_add_cached(p1p1& r, const p3& p, const cached& q) {
  fe PP, MM, TT, ZZ, ZZ2, ypx, ymx;
  fe_add(ypx, p.Y, p.X);
  fe_sub(ymx, p.Y, p.X);
  fe_mul(PP, ypx, q.YpX);
  fe_mul(MM, ymx, q.YmX);
  fe_mul(TT, p.T, q.T2d);
  fe_mul(ZZ, p.Z, q.Z);
  fe_add(ZZ2, ZZ, ZZ);      // A
  fe_sub(r.X, PP, MM);      // N
  fe_add(r.Y, PP, MM);      // A
  fe_addn(r.Z, ZZ2, TT);    // A + N: normalised
  fe_sub(r.T, ZZ2, TT);     // N
}
// P + Q (Q precomp, Z = 1): 3 multiplications
MV_DEV void p3_add_precomp(p1p1& r, const p3& p, const precomp& q) {
  fe PP, MM, TT, Z2, ypx, ymx;
  fe_add(ypx, p.Y, p.X);
  fe_sub(ymx, p.Y, p.X);
  fe_mul(PP, ypx, q.ypx);
  fe_mul(MM, ymx, q.ymx);
  fe_mul(TT, p.T, q.xy2d);
  fe_add(Z2, p.Z, p.Z);
  fe_sub(r.X, PP, MM);
  fe_add(r.Y, PP, MM);
  fe_addn(r.Z, Z2, TT);
  fe_sub(r.T, Z2, TT);
}
// conditional negation of table entries: -(x, y) = (-x, y) swaps y+x / y-x and negates xy
MV_DEV void cached_cneg(cached& c, bool neg) {
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint32_t a = c.YpX.v[i], b = c.YmX.v[i];
    c.YpX.v[i] = neg ? b : a;
    c.YmX.v[i] = neg ? a : b;
  }
  fe n;
  fe_neg(n, c.T2d);
  fe_cmov(c.T2d, n, neg);
}
MV_DEV void precomp_cneg(precomp& c, bool neg) {
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint32_t a = c.ypx.v[i], b = c.ymx.v[i];
    c.ypx.v[i] = neg ? b : a;
    c.ymx.v[i] = neg ? a : b;
  }
  fe n;
  fe_neg(n, c.xy2d);
  fe_cmov(c.xy2d, n, neg);
}
MV_DEV void p3_neg(p3& r, const p3& p) {
  fe_neg(r.X, p.X);
  r.Y = p.Y;
  r.Z = p.Z;
  fe_neg(r.T, p.T);
}
// compress(P) == compress(identity)  <=>  X == 0 and Y == Z (mod p)
MV_DEV bool p3_is_identity(const p3& p) { return fe_is_zero(p.X) && fe_eq(p.Y, p.Z); }

// sqrt_ratio_i(u, v) post-processing, given r0 = u*v^3*(u*v^7)^((p-5)/8):
// returns whether u/v is a square (u == 0 included) and the non-negative root.
MV_DEV bool sqrt_ratio_finish(fe& r, const fe& u, const fe& v, const fe& r0) {
  fe i, check, t, ui;
  fe_const(i, K_SQRTM1);
  fe_sq(t, r0);
  fe_mul(check, v, t);
  fe_add(t, check, u);          // check == -u
  bool flipped = fe_is_zero(t);
  bool correct = fe_eq(check, u);
  fe_mul(ui, u, i);
  fe_add(t, check, ui);         // check == -u*i
  bool flipped_i = fe_is_zero(t);
  fe ri;
  fe_mul(ri, r0, i);
  r = r0;
  fe_cmov(r, ri, flipped || flipped_i);
  fe nr;
  fe_neg(nr, r);
  fe_cmov(r, nr, fe_is_negative(r));
  return correct || flipped;
}

// ZIP-215 decompression of two encodings at once (A and R of one signature):
// y from 255 bits without a range check, x = +-sqrt((y^2-1)/(dy^2+1)), sign bit
// applied even when x == 0 (dalek CompressedEdwardsY::decompress semantics).
MV_DEV void decompress_x2(p3& A, bool& okA, const uint32_t ea[8], p3& R, bool& okR, const uint32_t er[8]) {
  fe d, one;
  fe_const(d, K_D);
  fe_set(one, 1);
  fe ya, yr, ua, ur, va, vr, t;
  fe_from_words(ya, ea);
  fe_from_words(yr, er);
  fe_sq(t, ya);
  fe_sub(ua, t, one);
  fe_mul(va, t, d);
  fe_add(va, va, one);
  fe_sq(t, yr);
  fe_sub(ur, t, one);
  fe_mul(vr, t, d);
  fe_add(vr, vr, one);
  // r0 = u v^3 (u v^7)^((p-5)/8)
  fe v3a, v3r, ea7, er7;
  fe_sq(t, va); fe_mul(v3a, t, va);
  fe_sq(t, vr); fe_mul(v3r, t, vr);
  fe_sq(t, v3a); fe_mul(ea7, t, va); fe_mul(ea7, ea7, ua);
  fe_sq(t, v3r); fe_mul(er7, t, vr); fe_mul(er7, er7, ur);
  fe pa, pr;
  fe_pow_p58_x2(pa, pr, ea7, er7);
  fe_mul(pa, pa, v3a); fe_mul(pa, pa, ua);
  fe_mul(pr, pr, v3r); fe_mul(pr, pr, ur);
  fe xa, xr;
  okA = sqrt_ratio_finish(xa, ua, va, pa);
  okR = sqrt_ratio_finish(xr, ur, vr, pr);
  fe n;
  fe_neg(n, xa);
  fe_cmov(xa, n, (ea[7] >> 31) != 0);
  fe_neg(n, xr);
  fe_cmov(xr, n, (er[7] >> 31) != 0);
  A.X = xa; A.Y = ya; fe_set(A.Z, 1); fe_mul(A.T, xa, ya);
  R.X = xr; R.Y = yr; fe_set(R.Z, 1); fe_mul(R.T, xr, yr);
}

// One ZIP-215 decompression (single exponentiation chain: about half the registers of
// decompress_x2, for kernels that trade its ILP for occupancy).
MV_DEV void decompress1(p3& A, bool& okA, const uint32_t ea[8]) {
  fe d, one, ya, ua, va, t, v3a, ea7, pa, xa, n;
  fe_const(d, K_D);
  fe_set(one, 1);
  fe_from_words(ya, ea);
  fe_sq(t, ya);
  fe_sub(ua, t, one);
  fe_mul(va, t, d);
  fe_add(va, va, one);
  fe_sq(t, va); fe_mul(v3a, t, va);
  fe_sq(t, v3a); fe_mul(ea7, t, va); fe_mul(ea7, ea7, ua);
  fe_pow_p58(pa, ea7);
  fe_mul(pa, pa, v3a); fe_mul(pa, pa, ua);
  okA = sqrt_ratio_finish(xa, ua, va, pa);
  fe_neg(n, xa);
  fe_cmov(xa, n, (ea[7] >> 31) != 0);
  A.X = xa; A.Y = ya; fe_set(A.Z, 1); fe_mul(A.T, xa, ya);
}

// decompress1 with nothing but the chain live across fe_pow_p58: y, u, v and v^3 are
// recomputed from the encoding afterwards (2 squarings + 2 multiplications, under 2% of
// the decode), so a lane-per-signature kernel fits its target occupancy without spilling.
MV_DEV void decompress1_lean(p3& A, bool& okA, const uint32_t ea[8]) {
  fe pa;
  {
    fe d, one, ya, ua, va, t, ea7;
    fe_const(d, K_D);
    fe_set(one, 1);
    fe_from_words(ya, ea);
    fe_sq(t, ya);
    fe_sub(ua, t, one);
    fe_mul(va, t, d);
    fe_add(va, va, one);
    fe_sq(t, va); fe_mul(ea7, t, va);      // v^3
    fe_sq(t, ea7); fe_mul(ea7, t, va); fe_mul(ea7, ea7, ua);  // u v^7
    fe_pow_p58(pa, ea7);
  }
  fe d, one, ya, ua, va, t, v3a, xa, n;
  fe_const(d, K_D);
  fe_set(one, 1);
  fe_from_words(ya, ea);
  fe_sq(t, ya);
  fe_sub(ua, t, one);
  fe_mul(va, t, d);
  fe_add(va, va, one);
  fe_sq(t, va); fe_mul(v3a, t, va);
  fe_mul(pa, pa, v3a); fe_mul(pa, pa, ua);
  okA = sqrt_ratio_finish(xa, ua, va, pa);
  fe_neg(n, xa);
  fe_cmov(xa, n, (ea[7] >> 31) != 0);
  A.X = xa; A.Y = ya; fe_set(A.Z, 1); fe_mul(A.T, xa, ya);
}

// Two decompress1_lean's with their exponentiation chains interleaved (fe_pow_p58_x2: two
// independent squarings per step, twice the ILP of one chain); only the two chain states are
// live across them, the rest is recomputed from the encodings afterwards.
// The encodings come from get(which, words) (0: A, 1: R), called before and again after the
// chains, so a kernel can park them in LDS instead of holding 16 registers across the chains.
template <class Get>
MV_DEV void decompress2_lean(p3& A, bool& okA, p3& R, bool& okR, Get get) {
  fe pa, pr;
  {
    fe xa, xr;
    {
      fe d, one, y, u, v, t;
      uint32_t ea[8], er[8];
      get(0, ea);
      get(1, er);
      fe_const(d, K_D);
      fe_set(one, 1);
      fe_from_words(y, ea);
      fe_sq(t, y);
      fe_sub(u, t, one);
      fe_mul(v, t, d);
      fe_add(v, v, one);
      fe_sq(t, v); fe_mul(xa, t, v);
      fe_sq(t, xa); fe_mul(xa, t, v); fe_mul(xa, xa, u);  // u v^7 of A
      fe_from_words(y, er);
      fe_sq(t, y);
      fe_sub(u, t, one);
      fe_mul(v, t, d);
      fe_add(v, v, one);
      fe_sq(t, v); fe_mul(xr, t, v);
      fe_sq(t, xr); fe_mul(xr, t, v); fe_mul(xr, xr, u);  // u v^7 of R
    }
    fe_pow_p58_x2_nox(pa, pr, xa, xr);  // (u v^7)^(2^252 - 4): the last factor u v^7 below
  }
  auto finish = [](p3& P, bool& ok, const uint32_t e[8], fe& p) {
    fe d, one, y, u, v, t, v3, x, n;
    fe_const(d, K_D);
    fe_set(one, 1);
    fe_from_words(y, e);
    fe_sq(t, y);
    fe_sub(u, t, one);
    fe_mul(v, t, d);
    fe_add(v, v, one);
    fe_sq(t, v); fe_mul(v3, t, v);
    fe_sq(t, v3); fe_mul(t, t, v); fe_mul(t, t, u);  // u v^7
    fe_mul(p, p, t);                                 // (u v^7)^((p - 5) / 8)
    fe_mul(p, p, v3); fe_mul(p, p, u);
    ok = sqrt_ratio_finish(x, u, v, p);
    fe_neg(n, x);
    fe_cmov(x, n, (e[7] >> 31) != 0);
    P.X = x; P.Y = y; fe_set(P.Z, 1); fe_mul(P.T, x, y);
  };
  uint32_t e[8];
  get(0, e);
  finish(A, okA, e, pa);
  get(1, e);
  finish(R, okR, e, pr);
}

}  // namespace mv
