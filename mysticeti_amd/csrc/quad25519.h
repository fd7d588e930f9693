// Edwards25519 point arithmetic with FOUR lanes per point (gfx950): lane c of an aligned
// quad holds coordinate c of an extended point (X, Y, Z, T). For the latency-bound tails of
// the batch path (k_bv_final's Horner over the window sums), where one lane per point runs a
// doubling's 8 field operations back to back: here the four squarings of a doubling, and the
// four multiplications of each of its halves, run one per lane, so a doubling is one
// squaring and one multiplication deep, plus quad broadcasts (DPP quad_perm, full rate).
// The operation sequence per value is exactly ge25519.h's (p2_dbl + p1p1_to_p3, and
// p3_to_cached + p3_add_cached + p1p1_to_p3), so results and limb bounds are identical.
// All four lanes of a quad must be active.
#pragma once
#include "fe25519.h"
#include "ge25519.h"

namespace mv {

MV_DEV uint32_t qlane() { return threadIdx.x & 3u; }

// every lane of the quad takes limb-wise the value of quad lane K
template <int K>
MV_DEV void fe_qget(fe& r, const fe& a) {
  constexpr int ctrl = K | (K << 2) | (K << 4) | (K << 6);
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.v[i], ctrl, 0xf, 0xf, false);
}
// r = a[c] for quad lane c
MV_DEV void fe_qsel(fe& r, uint32_t c, const fe& a0, const fe& a1, const fe& a2, const fe& a3) {
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint32_t lo = c & 1u ? a1.v[i] : a0.v[i];
    const uint32_t hi = c & 1u ? a3.v[i] : a2.v[i];
    r.v[i] = c & 2u ? hi : lo;
  }
}

// v = coordinate c of P  ->  coordinate c of 2P (P extended; p2_dbl + p1p1_to_p3)
MV_DEV void qp_dbl(fe& v) {
  const uint32_t c = qlane();
  fe X, Y, S, in, sq;
  fe_qget<0>(X, v);
  fe_qget<1>(Y, v);
  fe_add(S, X, Y);
  fe_qsel(in, c, v, v, v, S);  // lanes 0..2 square X, Y, Z; lane 3 squares X + Y
  fe_sq(sq, in);
  fe XX, YY, ZZ, S2, rX, rY, rZ, rT, ZZ2, o1, o2;
  fe_qget<0>(XX, sq);
  fe_qget<1>(YY, sq);
  fe_qget<2>(ZZ, sq);
  fe_qget<3>(S2, sq);
  fe_add(rY, YY, XX);   // A
  fe_sub(rZ, YY, XX);   // N
  fe_add(ZZ2, ZZ, ZZ);  // A
  fe_sub(rX, S2, rY);   // N
  fe_sub(rT, ZZ2, rZ);  // N
  // X = rX rT, Y = rY rZ, Z = rZ rT, T = rX rY
  fe_qsel(o1, c, rX, rY, rZ, rX);
  fe_qsel(o2, c, rT, rZ, rT, rY);
  fe_mul(v, o1, o2);
}
MV_DEV void qp_dbl_n(fe& v, int n) {
#pragma unroll 1
  for (int i = 0; i < n; i++) qp_dbl(v);
}

// v = coordinate c of P, w = coordinate c of Q  ->  v = coordinate c of P + Q
MV_DEV void qp_add(fe& v, const fe& w) {
  const uint32_t c = qlane();
  fe d2, X2, Y2, cy, cm, t2d, cq;
  fe_const(d2, K_D2);
  fe_qget<0>(X2, w);
  fe_qget<1>(Y2, w);
  fe_add(cy, Y2, X2);  // cached(Q): Y + X (A), Y - X (N), Z, 2dT
  fe_sub(cm, Y2, X2);
  fe_mul(t2d, w, d2);
  fe_qsel(cq, c, cy, cm, w, t2d);
  fe X1, Y1, ypx, ymx, o1, prod;
  fe_qget<0>(X1, v);
  fe_qget<1>(Y1, v);
  fe_add(ypx, Y1, X1);
  fe_sub(ymx, Y1, X1);
  // lane 0: PP = (Y1 + X1)(Y2 + X2), 1: MM = (Y1 - X1)(Y2 - X2), 2: ZZ = Z1 Z2, 3: TT = T1 2dT2
  fe_qsel(o1, c, ypx, ymx, v, v);
  fe_mul(prod, o1, cq);
  fe PP, MM, ZZ, TT, ZZ2, rX, rY, rZ, rT, a1, a2;
  fe_qget<0>(PP, prod);
  fe_qget<1>(MM, prod);
  fe_qget<2>(ZZ, prod);
  fe_qget<3>(TT, prod);
  fe_add(ZZ2, ZZ, ZZ);    // A
  fe_sub(rX, PP, MM);     // N
  fe_add(rY, PP, MM);     // A
  fe_addn(rZ, ZZ2, TT);   // N
  fe_sub(rT, ZZ2, TT);    // N
  fe_qsel(a1, c, rX, rY, rZ, rX);
  fe_qsel(a2, c, rT, rZ, rT, rY);
  fe_mul(v, a1, a2);
}

// v = coordinate c of a curve point P -> whether [8]P is the identity (the same in every lane of
// the quad), i.e. whether P lies in the 8-torsion E[8]. On -x^2 + y^2 = 1 + d x^2 y^2 those are
// exactly the points with x = 0 (orders 1, 2), y = 0 (order 4: (+-sqrt(-1), 0)) or
// x^2 + y^2 = 0 (order 8: 2P has y = (y^2 + x^2) / (2 + x^2 - y^2) = 0, i.e. 2P is of order 4;
// conversely 2P of order 4 has y = 0). The three tests are homogeneous, so X and Y of the
// extended point serve: one squaring deep, against [8]P's three doublings and the identity test
// (tests/test_torsion_predicate.py checks the equivalence over E[8] + multiples of B).
MV_DEV bool qp_in_torsion(const fe& v) {
  fe sq, Y2, s;
  fe_sq(sq, v);  // lane 0: X^2, lane 1: Y^2
  fe_qget<1>(Y2, sq);
  fe_addn(s, sq, Y2);  // lane 0: X^2 + Y^2
  const uint32_t bits = (fe_is_zero(v) ? 1u : 0u) | (fe_is_zero(s) ? 2u : 0u);
  const uint32_t b0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)bits, 0x00, 0xf, 0xf, false);  // lane 0's
  const uint32_t b1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)bits, 0x55, 0xf, 0xf, false);  // lane 1's
  return (b0 & 3u) != 0 || (b1 & 1u) != 0;  // X = 0 or X^2 + Y^2 = 0; Y = 0
}

// coordinate c of the extended point stored as 9 uint4 (p3_to_quads layout: X, Y, Z, T limbs)
MV_DEV void qp_load(fe& v, const uint4* base, size_t idx) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(base + idx * 9) + 9 * qlane();
#pragma unroll
  for (int i = 0; i < 9; i++) v.v[i] = w[i];
}

MV_DEV void qp_identity(fe& v) {
  const uint32_t c = qlane();
  fe_set(v, c == 1u || c == 2u ? 1u : 0u);
}
MV_DEV void qp_store(uint4* base, size_t idx, const fe& v) {
  uint32_t* w = reinterpret_cast<uint32_t*>(base + idx * 9) + 9 * qlane();
#pragma unroll
  for (int i = 0; i < 9; i++) w[i] = v.v[i];
}

}  // namespace mv
