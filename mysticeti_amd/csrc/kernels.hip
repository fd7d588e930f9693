// HIP kernels of the StatementBlock verification engine (gfx950 only).
//
//   k_btable_init    fixed-base tables [j]B and [j](2^124 B), j = 0..128, affine
//                    (y+x, y-x, 2dxy)
//   k_verify         ZIP-215 ed25519 verify, one signature per lane (ed25519-consensus
//                    VerificationKey::verify, called at mysticeti-core/src/crypto.rs:188),
//                    on half-size scalars (scalar25519.h sc_halfsize)
//   k_sign           RFC 8032 signing, one per lane (crypto.rs:199-223, corpus generation)
//   (BLAKE2b: blake2b_quad.hip for small calls, blake2b_lane.hip at batch size; the
//   launch_blake2b / launch_block_hash entry points below route between them)
//   k_selftest       field / scalar primitives for the parity tests
//
// The verify kernel is INT32-VALU bound: HBM traffic is 128 B of
// input per signature plus the per-lane variable-base tables (2 x 9 cached points,
// written once, read 32 times each, L2/MALL-resident per wave).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/mysti_verify.h"
#include "fe25519.h"
#include "fe_q4.h"
#include "fe_r16.h"
#include "ge25519.h"
#include "hash_dev.h"
#include "kernels.h"
#include "scalar25519.h"
#include "tables.h"
#include "comb.h"

namespace mv {

// Per-wave variable-base table scratch. Lane-major: each lane owns 2 x 81 contiguous
// uint4 ([table][entry][quad]), so one entry gather reads 144 contiguous bytes per lane
// (2 cache lines) and the whole line is used (a wave-major layout coalesces the build's
// stores, but a random-digit gather then touches ~5 partly used lines per 8 lanes per quad).
constexpr int TAB_LANE_STRIDE = 2 * AT_TABLE, TAB_QUAD_STRIDE = 1;
constexpr int TAB_ENTRY_STRIDE = AT_QUADS * TAB_QUAD_STRIDE;
constexpr int TAB_TABLE_STRIDE = AT_ENTRIES * TAB_ENTRY_STRIDE;  // A table -> R table
MV_DEV void atab_put(uint4* tab, int e, const cached& c) {
  uint4* p = tab + e * TAB_ENTRY_STRIDE;
  uint4 q[9];
  cached_to_quads(q, c);
#pragma unroll
  for (int i = 0; i < 9; i++) p[i * TAB_QUAD_STRIDE] = q[i];
}
// raw entry load; the sign is applied at use time (cached_cneg) so the gather's
// latency hides behind the window's doublings
MV_DEV void atab_load(cached& c, const uint4* tab, int digit) {
  int e = digit < 0 ? -digit : digit;
  const uint4* p = tab + e * TAB_ENTRY_STRIDE;
  uint4 q[9];
#pragma unroll
  for (int i = 0; i < 9; i++) q[i] = p[i * TAB_QUAD_STRIDE];
  quads_to_cached(c, q);
}

// ---------------------------------------------------------------- kernels
__global__ void __launch_bounds__(256) k_btable_init(uint4* out) {
  const int j = threadIdx.x;
  const int t = blockIdx.x;  // 0: B, 1: 2^124 B
  if (j >= BT_ENTRIES) return;
  // B = decompress(4/5, sign 0)
  const uint32_t by[8] = {0x66666658, 0x66666666, 0x66666666, 0x66666666,
                          0x66666666, 0x66666666, 0x66666666, 0x66666666};
  p3 B, R;
  bool okB, okR;
  decompress_x2(B, okB, by, R, okR, by);
  if (t == 1) {
    p2 P;
    p1p1 Q;
    P.X = B.X;
    P.Y = B.Y;
    P.Z = B.Z;
    for (int i = 0; i < 123; i++) {
      p2_dbl(Q, P);
      p1p1_to_p2(P, Q);
    }
    p2_dbl(Q, P);
    p1p1_to_p3(B, Q);
  }
  p3 acc;
  p3_identity(acc);
  cached cb;
  p3_to_cached(cb, B);
  for (int i = 0; i < j; i++) {
    p1p1 q;
    p3_add_cached(q, acc, cb);
    p1p1_to_p3(acc, q);
  }
  fe zi, x, y, xy, d2;
  fe_invert(zi, acc.Z);
  fe_mul(x, acc.X, zi);
  fe_mul(y, acc.Y, zi);
  fe_const(d2, K_D2);
  precomp pc;
  fe_add(pc.ypx, y, x);
  fe_sub(pc.ymx, y, x);
  fe_mul(xy, x, y);
  fe_mul(pc.xy2d, xy, d2);
  fe_canon(pc.ypx, pc.ypx);
  fe_canon(pc.ymx, pc.ymx);
  fe_canon(pc.xy2d, pc.xy2d);
  uint4 q[7];
  precomp_to_quads(q, pc);
  uint4* o = out + t * BT_TABLE + j * BT_QUADS;
#pragma unroll
  for (int i = 0; i < 7; i++) o[i] = q[i];
}

// Per-wave scratch layout (uint4 units): the two variable-base tables of the 64 lanes
// ([0..8](-A) or [0..8](A) by the sign of c, then [0..8](-R)), then the recoded
// scalars [group][lane], parked in HBM during the ladder instead of holding 16 VGPRs.
constexpr int SCR_DIG = 2 * AT_TABLE * 64;  // 4 groups x uint4 (c, d, e lo, e hi)
constexpr int WAVE_QUADS = 2 * AT_TABLE + 4;  // 166 per lane

// [0..8]P as cached points into a per-wave table
MV_DEV void vtab_build(uint4* tab, const p3& P) {
  cached c1, c;
  cached_identity(c);
  atab_put(tab, 0, c);
  p3_to_cached(c1, P);
  atab_put(tab, 1, c1);
  p3 cur = P;
  for (int j = 2; j <= 8; j++) {
    p1p1 t;
    p3_add_cached(t, cur, c1);
    p1p1_to_p3(cur, t);
    p3_to_cached(c, cur);
    atab_put(tab, j, c);
  }
}

// What the batch path's k_bv_prep already decoded (the fallback re-verifies from it): R at
// pts[i] and A at pts[n + i] (affine precomp), or A from the committee's comb table entry
// [0][1] = [1](-A) when it was summed per key; status[i] != 0 is prep's final verdict
// (s >= l or a point that does not decode) and stays.
struct PrepView {
  const uint4* pts;   // nullptr: decode A and R here
  uint32_t n;
  const uint4* comb;  // non-null: A of key b from the comb tables
};

// One signature per lane. pk rows are read at key_idx[i] when key_idx != nullptr.
// MINW = minimum waves per SIMD (2 -> <= 256 VGPRs, 1 -> <= 512).
//
// Checks [8]([e]B - [c]A - [d]R) == O with e = d*s mod l, (c, d) = sc_halfsize(k),
// which holds iff the ZIP-215 equation [8]([s]B - [k]A - R) == O does (see
// sc_halfsize). e's signed radix-256 digits 0..15 go against [j]B at the even 4-bit
// windows, digits 16..31 against [j](2^124 B) at the odd ones, so every one of the
// 32 windows does 4 doublings and three additions (A, R, B or 2^124 B).
template <int MINW>
__global__ void __launch_bounds__(256, MINW)
    k_verify(const uint8_t* __restrict__ msg, const uint8_t* __restrict__ sig, const uint8_t* __restrict__ pk,
             const uint32_t* __restrict__ key_idx, uint32_t n, const uint4* __restrict__ btab_g,
             uint4* __restrict__ scratch, uint8_t* __restrict__ status, const uint32_t* __restrict__ skip,
             uint32_t skip_group, PrepView pv) {
  // batch fallback (batch.hip): nothing to do for a group whose equation held (skip_group
  // is a multiple of the block size, so the test is uniform over the block)
  if (skip && skip[skip_group ? blockIdx.x * blockDim.x / skip_group : 0]) return;
  __shared__ uint4 btab[2 * BT_TABLE];
  lds_btab_load(btab, btab_g, 2 * BT_TABLE);
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t idx = gid < n ? gid : n - 1;
  const int lane = threadIdx.x & 63;
  uint4* wave_tab = scratch + (size_t)(gid >> 6) * (WAVE_QUADS * 64);
  uint4* wave_dig = wave_tab + SCR_DIG;
  uint4* tabA = wave_tab + lane * TAB_LANE_STRIDE;
  uint4* tabR = tabA + TAB_TABLE_STRIDE;

  bool okA, okR, s_ok;
  {
    uint32_t aw[8], rw[8], sw[8], mw[8];
    load8(aw, pk + 32 * (size_t)(key_idx ? key_idx[idx] : idx));
    load8(rw, sig + 64 * (size_t)idx);
    load8(sw, sig + 64 * (size_t)idx + 32);
    load8(mw, msg + 32 * (size_t)idx);

    s_ok = sc_is_canonical(sw);
    // k = SHA-512(R || A || M) mod l over the original encodings
    uint32_t kin[24], h[16], k[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      kin[i] = rw[i];
      kin[8 + i] = aw[i];
      kin[16 + i] = mw[i];
    }
    sha512_short(h, kin, 96);
    sc_reduce512(k, h);
    uint32_t c[4], d[8], e[8], zero[8];
    bool c_neg;
    sc_halfsize(c, c_neg, d, k);
#pragma unroll
    for (int i = 0; i < 8; i++) zero[i] = 0;
#pragma unroll
    for (int i = 4; i < 8; i++) d[i] = 0;
    sc_muladd(e, d, sw, zero);
    uint32_t cd[4], dd[4], ed[8];
    sc_recode16_128(cd, c);
    sc_recode16_128(dd, d);
    sc_recode256(ed, e);
#pragma unroll
    for (int g = 0; g < 4; g++) wave_dig[g * 64 + lane] = make_uint4(cd[g], dd[g], ed[g], ed[4 + g]);

    p3 A, R, nR;
    if (pv.pts) {  // decoded by k_bv_prep; lanes prep already rejected keep its verdict
      const bool prep_ok = status[idx] == 0;
      okA = prep_ok;
      okR = prep_ok;
      s_ok = s_ok && prep_ok;
      uint4 q[7];
      precomp pc;
      const uint4* pr = pv.pts + (size_t)idx * PT_QUADS;
#pragma unroll
      for (int k = 0; k < 7; k++) q[k] = pr[k];
      quads_to_precomp(pc, q);
      precomp_to_p3(R, pc);
      const uint4* pa = pv.comb ? pv.comb + (size_t)(key_idx ? key_idx[idx] : idx) * CT_TABLE + CT_QUADS
                                : pv.pts + ((size_t)pv.n + idx) * PT_QUADS;
#pragma unroll
      for (int k = 0; k < 7; k++) q[k] = pa[k];
      quads_to_precomp(pc, q);
      if (pv.comb) precomp_cneg(pc, true);  // the tables hold -A
      precomp_to_p3(A, pc);
    } else {
      decompress_x2(A, okA, aw, R, okR, rw);
    }
    // -[c]A = [|c|](-A) for c >= 0, [|c|]A for c < 0
    if (!c_neg) p3_neg(A, A);
    vtab_build(tabA, A);
    p3_neg(nR, R);
    vtab_build(tabR, nR);
  }

  p2 P;
  p3 P3;
  p1p1 Q;
  cached ca, cr;
  precomp pb;
  // 4 groups of 8 windows; a group's digit quad is loaded one group ahead, each
  // window's two table gathers are issued before its doublings and consumed after.
  uint4 dw_next = wave_dig[3 * 64 + lane];
  for (int g = 3; g >= 0; g--) {
    const uint4 dw = dw_next;
    if (g > 0) dw_next = wave_dig[(g - 1) * 64 + lane];
    for (int j = 7; j >= 0; j--) {
      const int w = 8 * g + j;
      const int dc = ((int)(dw.x << (28 - 4 * j))) >> 28;
      const int dd = ((int)(dw.y << (28 - 4 * j))) >> 28;
      atab_load(ca, tabA, dc);
      atab_load(cr, tabR, dd);
      if (w != 31) {
        for (int i = 0; i < 3; i++) {
          p2_dbl(Q, P);
          p1p1_to_p2(P, Q);
        }
        p2_dbl(Q, P);
        p1p1_to_p3(P3, Q);
      } else {
        p3_identity(P3);
      }
      cached_cneg(ca, dc < 0);
      p3_add_cached(Q, P3, ca);
      p1p1_to_p3(P3, Q);
      cached_cneg(cr, dd < 0);
      p3_add_cached(Q, P3, cr);
      p1p1_to_p3(P3, Q);
      // even window 2i: digit i of e (B); odd window 2i+1: digit 16+i (2^124 B)
      const uint32_t ew = (j & 1) ? dw.w : dw.z;
      const int de = ((int)(ew << (24 - 8 * (j >> 1)))) >> 24;
      btab_get(pb, btab + (j & 1) * BT_TABLE, de);
      p3_add_precomp(Q, P3, pb);
      p1p1_to_p2(P, Q);
    }
  }
  // cofactored check: [8]([e]B - [c]A - [d]R) == identity
#pragma unroll 1
  for (int i = 0; i < 3; i++) {
    p2_dbl(Q, P);
    p1p1_to_p2(P, Q);
  }
  const bool ident = fe_is_zero(P.X) && fe_eq(P.Y, P.Z);
  if (gid < n && !(pv.pts && !okA)) {  // (prep's own verdicts stay)
    uint8_t st = !okA ? 2 : ((s_ok && okR && ident) ? 0 : 1);
    status[gid] = st;
  }
}

// RFC 8032: (pk, R || S) from (seed, 32-byte msg)
__global__ void __launch_bounds__(256, 2)
    k_sign(const uint8_t* __restrict__ seed, const uint8_t* __restrict__ msg, uint32_t n,
           const uint4* __restrict__ btab_g, uint8_t* __restrict__ pk_out, uint8_t* __restrict__ sig_out) {
  __shared__ uint4 btab[BT_TABLE];
  lds_btab_load(btab, btab_g, BT_TABLE);
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t idx = gid < n ? gid : n - 1;
  uint32_t sw[8], mw[8], h[16];
  load8(sw, seed + 32 * (size_t)idx);
  load8(mw, msg + 32 * (size_t)idx);
  sha512_short(h, sw, 32);
  uint32_t a[16];
#pragma unroll
  for (int i = 0; i < 8; i++) a[i] = h[i];
  a[0] &= 0xfffffff8u;
  a[7] = (a[7] & 0x7fffffffu) | 0x40000000u;
#pragma unroll
  for (int i = 8; i < 16; i++) a[i] = 0;
  uint32_t ared[8], sd[8];
  sc_reduce512(ared, a);  // [a]B == [a mod l]B keeps the top digit in range
  sc_recode256(sd, ared);
  p3 P;
  basemul(P, sd, btab);
  uint32_t pkw[8];
  p3_compress(pkw, P);
  // r = SHA-512(prefix || M) mod l
  uint32_t rin[16], rh[16], r[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    rin[i] = h[8 + i];
    rin[8 + i] = mw[i];
  }
  sha512_short(rh, rin, 64);
  sc_reduce512(r, rh);
  sc_recode256(sd, r);
  basemul(P, sd, btab);
  uint32_t Rw[8];
  p3_compress(Rw, P);
  uint32_t kin[24], kh[16], k[8], S[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    kin[i] = Rw[i];
    kin[8 + i] = pkw[i];
    kin[16 + i] = mw[i];
  }
  sha512_short(kh, kin, 96);
  sc_reduce512(k, kh);
  sc_muladd(S, k, ared, r);
  if (gid < n) {
    store8(pk_out + 32 * (size_t)gid, pkw);
    store8(sig_out + 64 * (size_t)gid, Rw);
    store8(sig_out + 64 * (size_t)gid + 32, S);
  }
}

// Field / scalar primitives on 16-word lane inputs (parity tests).
__global__ void __launch_bounds__(64) k_selftest(int op, const uint32_t* __restrict__ in, uint32_t n,
                                                 const uint4* __restrict__ btab_g, uint32_t* __restrict__ out) {
  __shared__ uint4 btab[2 * BT_TABLE];
  lds_btab_load(btab, btab_g, 2 * BT_TABLE);
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n) return;
  uint32_t x[16], y[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    x[i] = in[16 * (size_t)gid + i];
    y[i] = 0;
  }
  fe a, b, r;
  fe_from_words_full(a, x);
  fe_from_words_full(b, x + 8);
  switch (op) {
    case 0: fe_mul(r, a, b); fe_canon(r, r); break;
    case 1: fe_sq(r, a); fe_canon(r, r); break;
    case 2: fe_add(r, a, b); fe_canon(r, r); break;
    case 3: fe_sub(r, a, b); fe_canon(r, r); break;
    case 4: fe_invert(r, a); fe_canon(r, r); break;
    case 5: fe_pow_p58(r, a); fe_canon(r, r); break;
    case 6: fe_mul_small(r, a, x[8]); fe_canon(r, r); break;
    case 7: {  // ZIP-215 decode of a: x (canonical) and the ok flag in word 8
      p3 A, B;
      bool oa, ob;
      decompress_x2(A, oa, x, B, ob, x);
      fe_canon(r, A.X);
      y[8] = oa ? 1u : 0u;
      break;
    }
    case 8: {
      uint32_t k[8];
      sc_reduce512(k, x);
#pragma unroll
      for (int i = 0; i < 8; i++) out[16 * (size_t)gid + i] = k[i];
#pragma unroll
      for (int i = 8; i < 16; i++) out[16 * (size_t)gid + i] = 0;
      return;
    }
    case 9: {  // sha512 of 64 bytes
      sha512_short(y, x, 64);
#pragma unroll
      for (int i = 0; i < 16; i++) out[16 * (size_t)gid + i] = y[i];
      return;
    }
    case 15: {  // sha512 of 96 bytes (the R || A || M challenge input): the 64 input bytes, then their first 32
      uint32_t m96[24];
#pragma unroll
      for (int i = 0; i < 16; i++) m96[i] = x[i];
#pragma unroll
      for (int i = 0; i < 8; i++) m96[16 + i] = x[i];
      sha512_short(y, m96, 96);
#pragma unroll
      for (int i = 0; i < 16; i++) out[16 * (size_t)gid + i] = y[i];
      return;
    }
    // four lanes per element (fe_q4.h): every lane of a quad must hold the same input
    case 16: {
      feq qa, qb, qr;
      feq_from_fe(qa, a);
      feq_from_fe(qb, b);
      feq_mul(qr, qa, qb);
      fe_from_feq(r, qr);
      fe_canon(r, r);
      break;
    }
    case 17: {
      feq qa, qr;
      feq_from_fe(qa, a);
      feq_pow_p58(qr, qa);
      fe_from_feq(r, qr);
      fe_canon(r, r);
      break;
    }
    case 18: {  // a^(2^50) by repeated squaring
      feq qa, qr;
      feq_from_fe(qa, a);
      feq_sqn(qr, qa, 50);
      fe_from_feq(r, qr);
      fe_canon(r, r);
      break;
    }
    // one DPP row per element (fe_r16.h): every lane of a 16-lane row must hold the same input
    case 19: {
      fer ra, rb, rr;
      fer_from_fe(ra, a);
      fer_from_fe(rb, b);
      fer_mul(rr, ra, rb, r16::consts());
      fe_from_fer(r, rr);
      fe_canon(r, r);
      break;
    }
    case 20: {
      fer ra, rr;
      fer_from_fe(ra, a);
      fer_pow_p58(rr, ra);
      fe_from_fer(r, rr);
      fe_canon(r, r);
      break;
    }
    case 21: {  // a^(2^50) by repeated squaring
      fer ra, rr;
      fer_from_fe(ra, a);
      fer_sqn(rr, ra, 50, r16::consts());
      fe_from_fer(r, rr);
      fe_canon(r, r);
      break;
    }
    case 10: fe_set(r, sc_is_canonical(x) ? 1 : 0); break;
    case 11: {  // [a]B encoding for a scalar a < 2^253
      uint32_t sd[8];
      sc_recode256(sd, x);
      p3 P;
      basemul(P, sd, btab);
      uint32_t enc[8];
      p3_compress(enc, P);
#pragma unroll
      for (int i = 0; i < 8; i++) out[16 * (size_t)gid + i] = enc[i];
#pragma unroll
      for (int i = 8; i < 16; i++) out[16 * (size_t)gid + i] = 0;
      return;
    }
    case 13: {  // sc_halfsize of k < l: c words 0..3, c_neg word 4, d words 8..11
      uint32_t c[4], d[4];
      bool neg;
      sc_halfsize(c, neg, d, x);
#pragma unroll
      for (int i = 0; i < 16; i++) y[i] = 0;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        y[i] = c[i];
        y[8 + i] = d[i];
      }
      y[4] = neg;
#pragma unroll
      for (int i = 0; i < 16; i++) out[16 * (size_t)gid + i] = y[i];
      return;
    }
    case 14: {  // [a](2^124 B) encoding via the second fixed-base table
      uint32_t sd[8];
      sc_recode256(sd, x);
      p3 P;
      basemul(P, sd, btab + BT_TABLE);
      uint32_t enc[8];
      p3_compress(enc, P);
#pragma unroll
      for (int i = 0; i < 8; i++) out[16 * (size_t)gid + i] = enc[i];
#pragma unroll
      for (int i = 8; i < 16; i++) out[16 * (size_t)gid + i] = 0;
      return;
    }
    case 12: {  // fe_canon of raw 255-bit input
      fe_from_words(r, x);
      fe_canon(r, r);
      break;
    }
    default: fe_set(r, 0);
  }
  {
    uint32_t rw[8];
    fe_to_words(rw, r);
#pragma unroll
    for (int i = 0; i < 8; i++) y[i] = rw[i];
  }
#pragma unroll
  for (int i = 0; i < 16; i++) out[16 * (size_t)gid + i] = y[i];
}

// The number of invalid signatures (status MV_SIG_INVALID: the failures a combined equation
// can see; s >= l and undecodable points are excluded from it exactly) of n statuses, added to
// *count (zeroed by the launcher): the single-path feedback of the batch policy (engine.cpp
// enqueue_batch), one atomic per wave. 256 threads x 16 bytes per thread per block.
__global__ void __launch_bounds__(256) k_count_rejects(const uint8_t* __restrict__ status, uint32_t n,
                                                       uint32_t* __restrict__ count) {
  const uint32_t base = (blockIdx.x * 256 + threadIdx.x) * 16;
  uint32_t c = 0;
  if (base + 16 <= n) {
    const uint4 w = *reinterpret_cast<const uint4*>(status + base);
    const uint32_t x[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
      // bytes equal to 1 -> y's zero bytes; nonzero bytes of y get their high bit set
      const uint32_t y = x[k] ^ 0x01010101u;
      const uint32_t nz = (((y & 0x7f7f7f7fu) + 0x7f7f7f7fu) | y) & 0x80808080u;
      c += 4u - (uint32_t)__builtin_popcount(nz);
    }
  } else {
    for (uint32_t i = base; i < n && i < base + 16; i++) c += status[i] == MV_SIG_INVALID;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) c += (uint32_t)__shfl_xor((int)c, m);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(count, c);
}

}  // namespace mv

// ---------------------------------------------------------------- launchers
namespace mvk {

hipError_t launch_count_rejects(const uint8_t* status, uint32_t n, uint32_t* count, hipStream_t s) {
  hipError_t e = hipMemsetAsync(count, 0, sizeof(uint32_t), s);
  if (e != hipSuccess || n == 0) return e;
  hipLaunchKernelGGL(mv::k_count_rejects, dim3((n + 4095) / 4096), dim3(256), 0, s, status, n, count);
  return hipGetLastError();
}

size_t verify_scratch_bytes(uint32_t n) {
  size_t waves = (size_t)((n + 255) / 256) * 4;  // every wave of the 256-thread grid owns a slot
  return waves * mv::WAVE_QUADS * 64 * sizeof(uint4);
}
// MV_VERIFY_OCC (A/B): k_verify's waves per SIMD, 1, 2 (default) or 3
static int verify_variant(const Knobs& kn) { return kn.verify_occ == 1 || kn.verify_occ == 3 ? (int)kn.verify_occ : 2; }
size_t btable_bytes() { return 2 * mv::BT_TABLE * sizeof(uint4); }

hipError_t launch_btable_init(void* d_btab, hipStream_t s) {
  hipLaunchKernelGGL(mv::k_btable_init, dim3(2), dim3(256), 0, s, (uint4*)d_btab);
  return hipGetLastError();
}
hipError_t launch_verify(const Knobs& kn, const uint8_t* msg, const uint8_t* sig, const uint8_t* pk, const uint32_t* key_idx,
                         uint32_t n, const void* btab, void* scratch, uint8_t* status, hipStream_t s,
                         const uint32_t* skip, uint32_t skip_group, const void* prep_pts, const void* prep_comb) {
  if (n == 0) return hipSuccess;
  const mv::PrepView pv{static_cast<const uint4*>(prep_pts), n, static_cast<const uint4*>(prep_comb)};
  if (verify_variant(kn) == 1)
    hipLaunchKernelGGL(mv::k_verify<1>, dim3((n + 255) / 256), dim3(256), 0, s, msg, sig, pk, key_idx, n,
                       (const uint4*)btab, (uint4*)scratch, status, skip, skip_group, pv);
  else if (verify_variant(kn) == 3)
    hipLaunchKernelGGL(mv::k_verify<3>, dim3((n + 255) / 256), dim3(256), 0, s, msg, sig, pk, key_idx, n,
                       (const uint4*)btab, (uint4*)scratch, status, skip, skip_group, pv);
  else
    hipLaunchKernelGGL(mv::k_verify<2>, dim3((n + 255) / 256), dim3(256), 0, s, msg, sig, pk, key_idx, n,
                       (const uint4*)btab, (uint4*)scratch, status, skip, skip_group, pv);
  return hipGetLastError();
}
hipError_t launch_sign(const uint8_t* seed, const uint8_t* msg, uint32_t n, const void* btab, uint8_t* pk,
                       uint8_t* sig, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(mv::k_sign, dim3((n + 255) / 256), dim3(256), 0, s, seed, msg, n, (const uint4*)btab, pk, sig);
  return hipGetLastError();
}
// BLAKE2b launchers: four lanes per string on small calls (blake2b_quad.hip), one lane per
// string at batch size (blake2b_lane.hip)
hipError_t launch_blake2b(const Knobs& kn, const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n,
                          uint8_t* out, hipStream_t s) {
  return launch_blake2b_quad(kn, buf, off, len, n, out, s);
}
hipError_t launch_block_hash(const Knobs& kn, const uint8_t* buf, const uint64_t* off, const uint64_t* len,
                             uint32_t n, uint8_t* msg_out, uint8_t* dig_out, hipStream_t s) {
  return launch_block_hash_quad(kn, buf, off, len, n, msg_out, dig_out, s);
}
hipError_t launch_selftest(int op, const uint32_t* in, uint32_t n, const void* btab, uint32_t* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(mv::k_selftest, dim3((n + 63) / 64), dim3(64), 0, s, op, in, n, (const uint4*)btab, out);
  return hipGetLastError();
}

}  // namespace mvk
