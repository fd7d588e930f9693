// Edwards25519 points with one DPP ROW (16 lanes) per coordinate: a whole wave holds one
// extended point, row c = coordinate c (X, Y, Z, T) in fe_r16.h's R form. For the longest
// latency chain of the batch path, k_bv_final's Horner over the window sums (240 doublings):
// quad25519.h runs a doubling as one squaring and one multiplication deep with a whole
// 9-limb product per lane (~0.22 us each on a lone wave); here each of those products is
// one fer_mul on a row (~0.13 us), and the moves between coordinates are one ds_bpermute
// per value instead of nine DPP moves. The operation sequence is quad25519.h's (qp_dbl,
// qp_add), so every result is the same residue; limbs may differ (one parallel carry round
// here where fe25519.h carries serially), so compare canonically.
#pragma once
#include "fe25519.h"
#include "fe_r16.h"
#include "ge25519.h"

namespace mv {
namespace r4 {

MV_DEV uint32_t row() { return (threadIdx.x >> 4) & 3u; }

// every row takes row K's element (lane t of each row reads lane 16 K + t)
template <int K>
MV_DEV fer get(const fer& x) {
  fer r;
  r.v = (uint32_t)__shfl((int)x.v, 16 * K + (int)(threadIdx.x & 15u), 64);
  return r;
}
// row c takes a_c
MV_DEV fer sel(const fer& a0, const fer& a1, const fer& a2, const fer& a3) {
  const uint32_t c = row();
  const uint32_t lo = c & 1u ? a1.v : a0.v, hi = c & 1u ? a3.v : a2.v;
  fer r;
  r.v = c & 2u ? hi : lo;
  return r;
}

// one parallel carry round at 29 bits: limbs < 2^32 in -> N out (lanes 1..8 < 2^29 + 8, lane 0
// < 2^29 + 7 * 1216); limb 8's carry goes to limb 0 times 2^261 = 1216 (mod p)
MV_DEV fer carry(uint32_t x, const r16::Consts& K) {
  using namespace r16;
  const uint32_t k = x >> 29;
  uint32_t o = (x & M29) + shr<1>(k);
  o += __umul24(shl<8>(k), K.m0c);
  fer r;
  r.v = o & K.keep;
  return r;
}
// lazy: N + N -> A (a multiplication input only; fe_add)
MV_DEV fer add(const fer& a, const fer& b) {
  fer r;
  r.v = a.v + b.v;
  return r;
}
// (N|A) + (N|A) -> N (fe_addn)
MV_DEV fer addn(const fer& a, const fer& b, const r16::Consts& K) { return carry(a.v + b.v, K); }
// a - b + C, C = 0 mod p with limbs in (2^31 - 2^29, 2^31] (fe_sub's): -> N
MV_DEV fer sub(const fer& a, const fer& b, const r16::Consts& K) {
  const uint32_t t = r16::lane();
  const uint32_t c = t == 0 ? 0x7fffed00u : (t < 9 ? 0x7ffffffcu : 0u);
  return carry(a.v + (c - b.v), K);
}

// v = coordinate row() of P  ->  coordinate row() of 2P (qp_dbl)
MV_DEV void dbl(fer& v, const r16::Consts& K) {
  const fer X = get<0>(v), Y = get<1>(v);
  const fer S = add(X, Y);
  fer sq;
  fer_sq(sq, sel(v, v, v, S), K);  // rows 0..2 square X, Y, Z; row 3 squares X + Y
  const fer XX = get<0>(sq), YY = get<1>(sq), ZZ = get<2>(sq), S2 = get<3>(sq);
  const fer rY = add(YY, XX);   // A
  const fer rZ = sub(YY, XX, K);  // N
  const fer ZZ2 = add(ZZ, ZZ);  // A
  const fer rX = sub(S2, rY, K);  // N
  const fer rT = sub(ZZ2, rZ, K);  // N
  // X = rX rT, Y = rY rZ, Z = rZ rT, T = rX rY
  fer_mul(v, sel(rX, rY, rZ, rX), sel(rT, rZ, rT, rY), K);
}

// v = coordinate row() of P, w = coordinate row() of Q  ->  v = coordinate row() of P + Q
// (qp_add); d2r = 2d in R form
MV_DEV void addp(fer& v, const fer& w, const fer& d2r, const r16::Consts& K) {
  const fer X2 = get<0>(w), Y2 = get<1>(w);
  const fer cy = add(Y2, X2), cm = sub(Y2, X2, K);  // cached(Q): Y + X (A), Y - X (N), Z, 2dT
  fer t2d;
  fer_mul(t2d, w, d2r, K);
  const fer cq = sel(cy, cm, w, t2d);
  const fer X1 = get<0>(v), Y1 = get<1>(v);
  const fer ypx = add(Y1, X1), ymx = sub(Y1, X1, K);
  // row 0: PP = (Y1 + X1)(Y2 + X2), 1: MM = (Y1 - X1)(Y2 - X2), 2: ZZ = Z1 Z2, 3: TT = T1 2dT2
  fer prod;
  fer_mul(prod, sel(ypx, ymx, v, v), cq, K);
  const fer PP = get<0>(prod), MM = get<1>(prod), ZZ = get<2>(prod), TT = get<3>(prod);
  const fer ZZ2 = add(ZZ, ZZ);        // A
  const fer rX = sub(PP, MM, K);      // N
  const fer rY = add(PP, MM);         // A
  const fer rZ = addn(ZZ2, TT, K);    // N
  const fer rT = sub(ZZ2, TT, K);     // N
  fer_mul(v, sel(rX, rY, rZ, rX), sel(rT, rZ, rT, rY), K);
}

// coordinate row() of the extended point stored as 9 uint4 (p3_to_quads layout: X, Y, Z, T
// limbs, 9 words each)
MV_DEV fer load(const uint4* base, size_t idx) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(base + idx * 9) + 9 * row();
  const uint32_t t = r16::lane();
  fer r;
  r.v = t < 9 ? w[t] : 0u;
  return r;
}
MV_DEV void store(uint32_t* w36, const fer& v) {
  const uint32_t t = r16::lane();
  if (t < 9) w36[9 * row() + t] = v.v;
}
MV_DEV void store(uint4* base, size_t idx, const fer& v) { store(reinterpret_cast<uint32_t*>(base + idx * 9), v); }
// the identity (0 : 1 : 1 : 0)
MV_DEV fer identity() {
  fer r;
  r.v = (r16::lane() == 0 && (row() == 1u || row() == 2u)) ? 1u : 0u;
  return r;
}

}  // namespace r4
}  // namespace mv
