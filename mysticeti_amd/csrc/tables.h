// Fixed-base tables and shared per-lane helpers of the verify / sign / batch kernels
// (gfx950). Table entries are stored in the field's limb form (9 x 29-bit words
// per element): B entries (precomp, 27 words + 1 pad = 7 uint4) in LDS, variable-base
// entries (cached, 36 words = 9 uint4) in HBM scratch.
#pragma once
#include "fe25519.h"
#include "ge25519.h"
#include "scalar25519.h"

namespace mv {

constexpr int BT_ENTRIES = 129;  // [0..128]B, then [0..128](2^124 B)
constexpr int BT_QUADS = 7;
constexpr int BT_TABLE = BT_ENTRIES * BT_QUADS;  // uint4 per fixed-base table
constexpr int AT_ENTRIES = 9;    // [0..8](-A), [0..8](-R)
constexpr int AT_QUADS = 9;
constexpr int AT_TABLE = AT_ENTRIES * AT_QUADS;  // uint4 per lane per variable-base table
// batch-path points (k_bv_prep -> k_bv_bucket, and the fallback): affine precomp, 27 limb
// words padded to one 128-B line, so a bucket's gather touches one line (112-B packed
// records measured the same: 1.67 vs 1.68 ms per 2^20 batch)
constexpr int PT_QUADS = 8;

template <int NW>
MV_DEV void words_to_quads(uint4 (&q)[(NW + 3) / 4], const uint32_t (&w)[NW]) {
#pragma unroll
  for (int i = 0; i < (NW + 3) / 4; i++)
    q[i] = make_uint4(w[4 * i], 4 * i + 1 < NW ? w[4 * i + 1] : 0u, 4 * i + 2 < NW ? w[4 * i + 2] : 0u,
                      4 * i + 3 < NW ? w[4 * i + 3] : 0u);
}
template <int NW>
MV_DEV void quads_to_words(uint32_t (&w)[NW], const uint4 (&q)[(NW + 3) / 4]) {
#pragma unroll
  for (int i = 0; i < (NW + 3) / 4; i++) {
    w[4 * i] = q[i].x;
    if (4 * i + 1 < NW) w[4 * i + 1] = q[i].y;
    if (4 * i + 2 < NW) w[4 * i + 2] = q[i].z;
    if (4 * i + 3 < NW) w[4 * i + 3] = q[i].w;
  }
}
MV_DEV void cached_to_quads(uint4 (&q)[9], const cached& c) {
  uint32_t w[36];
#pragma unroll
  for (int i = 0; i < 9; i++) {
    w[i] = c.YpX.v[i];
    w[9 + i] = c.YmX.v[i];
    w[18 + i] = c.Z.v[i];
    w[27 + i] = c.T2d.v[i];
  }
  words_to_quads<36>(q, w);
}
MV_DEV void quads_to_cached(cached& c, const uint4 (&q)[9]) {
  uint32_t w[36];
  quads_to_words<36>(w, q);
#pragma unroll
  for (int i = 0; i < 9; i++) {
    c.YpX.v[i] = w[i];
    c.YmX.v[i] = w[9 + i];
    c.Z.v[i] = w[18 + i];
    c.T2d.v[i] = w[27 + i];
  }
}
MV_DEV void precomp_to_quads(uint4 (&q)[7], const precomp& c) {
  uint32_t w[27];
#pragma unroll
  for (int i = 0; i < 9; i++) {
    w[i] = c.ypx.v[i];
    w[9 + i] = c.ymx.v[i];
    w[18 + i] = c.xy2d.v[i];
  }
  words_to_quads<27>(q, w);
}

MV_DEV void lds_btab_load(uint4* sm, const uint4* g, int quads) {
  for (int i = threadIdx.x; i < quads; i += blockDim.x) sm[i] = g[i];
  __syncthreads();
}
// B-table lookup with sign: digit in [-128, 128]
MV_DEV void btab_get(precomp& p, const uint4* sm, int digit) {
  int e = digit < 0 ? -digit : digit;
  const uint4* qp = sm + e * BT_QUADS;
  uint4 q[7];
#pragma unroll
  for (int i = 0; i < 7; i++) q[i] = qp[i];
  uint32_t w[27];
  quads_to_words<27>(w, q);
#pragma unroll
  for (int i = 0; i < 9; i++) {
    p.ypx.v[i] = w[i];
    p.ymx.v[i] = w[9 + i];
    p.xy2d.v[i] = w[18 + i];
  }
  precomp_cneg(p, digit < 0);
}

MV_DEV void load8(uint32_t w[8], const uint8_t* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}
MV_DEV void store8(uint8_t* p, const uint32_t w[8]) {
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4(w[0], w[1], w[2], w[3]);
  q[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

// encode a point: y with the sign of x in bit 255
MV_DEV void p3_compress(uint32_t out[8], const p3& p) {
  fe zi, x, y;
  fe_invert(zi, p.Z);
  fe_mul(x, p.X, zi);
  fe_mul(y, p.Y, zi);
  uint32_t xw[8];
  fe_to_words(xw, x);
  fe_to_words(out, y);
  out[7] |= (xw[0] & 1u) << 31;
}

// [s]B for s < 2^253 given as signed radix-256 digits (LDS table)
MV_DEV void basemul(p3& out, const uint32_t sd[8], const uint4* btab) {
  p2 P;
  p2_identity(P);
  p3 P3;
  p1p1 Q;
  precomp pre;
  for (int w = 31; w >= 0; w--) {
    if (w != 31) {
      for (int i = 0; i < 7; i++) {
        p2_dbl(Q, P);
        p1p1_to_p2(P, Q);
      }
      p2_dbl(Q, P);
      p1p1_to_p3(P3, Q);
    } else {
      p3_identity(P3);
    }
    btab_get(pre, btab, digit256(sd, w));
    p3_add_precomp(Q, P3, pre);
    if (w != 0) p1p1_to_p2(P, Q);
  }
  p1p1_to_p3(out, Q);
}

MV_DEV void quads_to_precomp(precomp& p, const uint4 (&q)[7]) {
  uint32_t w[27];
  quads_to_words<27>(w, q);
#pragma unroll
  for (int i = 0; i < 9; i++) {
    p.ypx.v[i] = w[i];
    p.ymx.v[i] = w[9 + i];
    p.xy2d.v[i] = w[18 + i];
  }
}
// the extended point (ypx - ymx, ypx + ymx, 2, xy2d / d) = (2x, 2y, 2, 2xy) of an affine
// precomp entry (y+x, y-x, 2dxy)
__constant__ const uint32_t K_DINV[8] = {0xcdc9f843, 0x25e0f276, 0x4279542e, 0x0b5dd698,
                                         0xcdb9cf66, 0x2b162114, 0x14d5ce43, 0x40907ed2};
MV_DEV void precomp_to_p3(p3& r, const precomp& c) {
  fe dinv;
  fe_const(dinv, K_DINV);
  fe_sub(r.X, c.ypx, c.ymx);
  fe_addn(r.Y, c.ypx, c.ymx);
  fe_set(r.Z, 2);
  fe_mul(r.T, c.xy2d, dinv);
}

MV_DEV void p3_to_quads(uint4 (&q)[9], const p3& p) {
  uint32_t w[36];
#pragma unroll
  for (int i = 0; i < 9; i++) {
    w[i] = p.X.v[i];
    w[9 + i] = p.Y.v[i];
    w[18 + i] = p.Z.v[i];
    w[27 + i] = p.T.v[i];
  }
  words_to_quads<36>(q, w);
}
MV_DEV void quads_to_p3(p3& p, const uint4 (&q)[9]) {
  uint32_t w[36];
  quads_to_words<36>(w, q);
#pragma unroll
  for (int i = 0; i < 9; i++) {
    p.X.v[i] = w[i];
    p.Y.v[i] = w[9 + i];
    p.Z.v[i] = w[18 + i];
    p.T.v[i] = w[27 + i];
  }
}

}  // namespace mv
