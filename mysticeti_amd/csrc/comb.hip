// Committee-key ed25519 verification on per-key comb tables (gfx950).
//
// The block path verifies signatures by a committee of at most 512 authorities
// (types.rs:118-121) whose keys are known before any block arrives: the reference
// decodes each VerificationKey once, when the committee is loaded (committee.rs:83-87,
// crypto.rs:25). mv_set_committee does the same and also builds, per key, the comb
// table
//     C_A[i][j] = [j * 256^i](-A),   i = 0..31, j = 0..128,
// as affine precomp points (y+x, y-x, 2dxy), one 128-byte line per entry (528 KB per
// key); mv_create builds C_B for the base point. With the signed radix-256 digits s_i
// of s and k_i of k = SHA-512(R || A || M) mod l,
//     R' = [s]B - [k]A = sum_i C_B[i][s_i] + sum_i C_A[i][k_i]
// is 64 mixed additions and no doublings (k_verify's half-size ladder: 128 doublings,
// 96 additions and a per-signature table). The predicate is k_verify's, the ZIP-215
// rule of ed25519_consensus::VerificationKey::verify (crypto.rs:188): s < l, R decodes,
// [8](R - R') == O.
//
// k_verify_comb: 64 signatures per 256-thread workgroup, one ROLE per wave. The lanes of
// a wave run in lock-step, so a signature's four dependency chains go to four waves
// (four SIMDs), not to four lanes:
//   wave 0   ZIP-215 decode of R: one exponentiation chain, ~265 field ops
//   wave 1   the 32 B-table entries of s's digits                  32 additions
//   wave 2   SHA-512 k; the A-table entries of k's digits 0..15    16 additions
//   wave 3   SHA-512 k; the A-table entries of k's digits 16..31   16 additions
// Wave 0 then adds the three partial sums (through LDS), subtracts them from R, clears
// the cofactor and tests for the identity. A 64-block batch (config 5) is one
// workgroup whose latency is wave 0's ~310 field ops; at full load the kernel does ~860
// field ops per signature against k_verify's ~2,335.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "fe25519.h"
#include "fe_r16.h"
#include "ge25519.h"
#include "hash_dev.h"
#include "quad25519.h"
#include "kernels.h"
#include "scalar25519.h"
#include "tables.h"
#include "comb.h"
#include "blake2b_quad.h"
#include "block_verdict.h"
#include "ingest_dev.h"

namespace mv {

// encoding of B: y = 4/5, sign 0
__constant__ const uint32_t K_BENC[8] = {0x66666658, 0x66666666, 0x66666666, 0x66666666,
                                         0x66666666, 0x66666666, 0x66666666, 0x66666666};

// Thread per (point b, row i, entry j): C[b][i][j] = [j * 256^i](+-P_b), P_b decoded
// from enc[b] with the ZIP-215 rules (B when enc == nullptr); ok[b] = P_b decodes.
__global__ void __launch_bounds__(256) k_comb_init(const uint8_t* __restrict__ enc, uint32_t nb, int negate,
                                                   uint4* __restrict__ tab, uint8_t* __restrict__ ok_out) {
  constexpr uint32_t PER = CT_ROWS * CT_ENTRIES;
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= nb * PER) return;
  const uint32_t b = gid / PER, r = gid % PER, i = r / CT_ENTRIES, j = r % CT_ENTRIES;
  uint32_t ew[8];
  if (enc) {
    load8(ew, enc + 32 * (size_t)b);
  } else {
#pragma unroll
    for (int k = 0; k < 8; k++) ew[k] = K_BENC[k];
  }
  p3 P;
  bool ok;
  decompress1(P, ok, ew);
  if (negate) p3_neg(P, P);
  // [j]P from the top bit down, then 8i doublings
  cached c;
  p3_to_cached(c, P);
  p3 Q;
  p3_identity(Q);
  p1p1 t;
  for (int bit = 7; bit >= 0; bit--) {
    p3_dbl(t, Q);
    p1p1_to_p3(Q, t);
    if ((j >> bit) & 1u) {
      p3_add_cached(t, Q, c);
      p1p1_to_p3(Q, t);
    }
  }
  for (uint32_t d = 0; d < 8 * i; d++) {
    p3_dbl(t, Q);
    p1p1_to_p3(Q, t);
  }
  fe zi, x, y, xy, d2;
  fe_invert(zi, Q.Z);
  fe_mul(x, Q.X, zi);
  fe_mul(y, Q.Y, zi);
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
  uint4* o = tab + (size_t)b * CT_TABLE + (size_t)i * CT_ROW + (size_t)j * CT_QUADS;
#pragma unroll
  for (int k = 0; k < 7; k++) o[k] = q[k];
  o[7] = make_uint4(0, 0, 0, 0);
  if (ok_out && i == 0 && j == 0) ok_out[b] = ok ? 1 : 0;
}

// P += Q (both extended)
MV_DEV void ct_acc(p3& P, const p3& Q) {
  cached c;
  p1p1 t;
  p3_to_cached(c, Q);
  p3_add_cached(t, P, c);
  p1p1_to_p3(P, t);
}

// the signature status of block gid, or its block verdict when the kernel carries it
MV_DEV void put_status(uint8_t* status, const mvk::BlockVerdictOut& bv, uint32_t gid, uint8_t sig_status) {
  if (bv.status)
    bv.status[gid] = block_verdict(bv.facts, bv.claimed, bv.msg_digest, bv.digest, sig_status, gid);
  else
    status[gid] = sig_status;
}

__global__ void __launch_bounds__(256) k_verify_comb(const uint8_t* msg, const uint8_t* __restrict__ sig,
                                                     const uint8_t* __restrict__ pk, const uint32_t* __restrict__ key_idx,
                                                     uint32_t n, const uint4* __restrict__ combB,
                                                     const uint4* __restrict__ combA,
                                                     const uint8_t* __restrict__ key_ok, uint8_t* __restrict__ status,
                                                     const mvk::BlockVerdictOut bv) {
  __shared__ uint4 part[3][9][64];  // partial sums of waves 1..3, [quad][lane]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t gid = blockIdx.x * 64 + lane;
  const uint32_t idx = gid < n ? gid : n - 1;
  const uint32_t key = key_idx[idx];
  p3 R;
  bool okR = false, s_ok = false;
  if (wave == 0) {
    uint32_t rw[8], sw[8];
    load8(rw, sig + 64 * (size_t)idx);
    load8(sw, sig + 64 * (size_t)idx + 32);
    s_ok = sc_is_canonical(sw);
    decompress1(R, okR, rw);
  } else {
    p3 acc;
    if (wave == 1) {
      uint32_t sw[8], sd[8];
      load8(sw, sig + 64 * (size_t)idx + 32);
      sc_recode256(sd, sw);
      ct_sum(acc, combB, sd, 0, CT_ROWS);
    } else {
      // k = SHA-512(R || A || M) mod l over the encodings as received (A = the
      // committee key's bytes)
      uint32_t kin[24], h[16], k[8], kd[8];
      load8(kin, sig + 64 * (size_t)idx);
      load8(kin + 8, pk + 32 * (size_t)key);
      load8(kin + 16, msg + 32 * (size_t)idx);
      sha512_short(h, kin, 96);
      sc_reduce512(k, h);
      sc_recode256(kd, k);
      const int r0 = (wave - 2) * (CT_ROWS / 2);
      ct_sum(acc, combA + (size_t)key * CT_TABLE, kd, r0, r0 + CT_ROWS / 2);
    }
    uint4 q[9];
    p3_to_quads(q, acc);
#pragma unroll
    for (int k = 0; k < 9; k++) part[wave - 1][k][lane] = q[k];
  }
  __syncthreads();
  if (wave == 0) {
    p3 S, X;
    uint4 q[9];
#pragma unroll
    for (int k = 0; k < 9; k++) q[k] = part[0][k][lane];
    quads_to_p3(S, q);
#pragma unroll
    for (int k = 0; k < 9; k++) q[k] = part[1][k][lane];
    quads_to_p3(X, q);
    ct_acc(S, X);
#pragma unroll
    for (int k = 0; k < 9; k++) q[k] = part[2][k][lane];
    quads_to_p3(X, q);
    ct_acc(S, X);
    p3_neg(S, S);
    ct_acc(R, S);  // R - R'
    p2 P;
    p1p1 t;
    P.X = R.X;
    P.Y = R.Y;
    P.Z = R.Z;
#pragma unroll 1
    for (int d = 0; d < 3; d++) {  // cofactor
      p2_dbl(t, P);
      p1p1_to_p2(P, t);
    }
    const bool ident = fe_is_zero(P.X) && fe_eq(P.Y, P.Z);
    if (gid < n) put_status(status, bv, gid, !key_ok[key] ? 2 : ((s_ok && okR && ident) ? 0 : 1));
  }
}

// ---------------------------------------------------------------- online path: short chains
// k_verify_comb16: the same predicate with every dependent chain cut short, for the online
// path (64-block calls), where k_verify_comb's latency is its longest single-lane chain: the
// R decode (~265 field operations) and the 32 B-table additions, ~80 us each on one lane.
// C16_SIGS signatures per workgroup:
//   role 0 (one 16-lane DPP row per signature): ZIP-215 decode of R, its (p-5)/8
//           power on fe_r16.h (~2x shorter per product than one lane), then the combination
//   roles 1..4 (one quad per signature each): the C_B entries of s's digits in four
//           blocks of 8 rows, point additions on quad25519.h's layout (lane c holds
//           coordinate c; it loads only the entry coordinate its product needs)
//   roles 5..8: SHA-512 k, then the C_A entries of k's digits in four blocks of 8 rows
// The table roles' sums are reduced (LDS, then lane shuffles) while role 0 finishes its decode
// (a barrier inside the power chain), then role 0's lanes 0..3 of each row subtract the sum
// from R as a quad, clear the cofactor and test for the identity. Same predicate, same status
// as k_verify_comb.
template <int AT = 200, class Mid = NoMid>
MV_DEV void decompress1_r16(p3& A, bool& okA, const uint32_t ea[8], Mid mid = Mid()) {
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
  {
    fer x, r;
    fer_from_fe(x, ea7);
    fer_pow_p58<AT>(r, x, mid);
    fe_from_fer(pa, r);
  }
  fe_mul(pa, pa, v3a); fe_mul(pa, pa, ua);
  okA = sqrt_ratio_finish(xa, ua, va, pa);
  fe_neg(n, xa);
  fe_cmov(xa, n, (ea[7] >> 31) != 0);
  A.X = xa; A.Y = ya; fe_set(A.Z, 1); fe_mul(A.T, xa, ya);
}

// v = coordinate c of P (extended) -> coordinate c of P + e, e = a table entry (affine
// precomp, p3_add_precomp's sequence): lane 0 multiplies Y + X by e's y + x, lane 1 Y - X by
// y - x, lane 2 Z by 2, lane 3 T by 2dxy (`op` is the lane's operand, the entry's sign applied)
MV_DEV void qp_madd(fe& v, const fe& op) {
  const uint32_t c = qlane();
  fe X1, Y1, ypx, ymx, o1, prod;
  fe_qget<0>(X1, v);
  fe_qget<1>(Y1, v);
  fe_add(ypx, Y1, X1);
  fe_sub(ymx, Y1, X1);
  fe_qsel(o1, c, ypx, ymx, v, v);
  fe_mul(prod, o1, op);
  fe PP, MM, Z2, TT, rX, rY, rZ, rT, a1, a2;
  fe_qget<0>(PP, prod);
  fe_qget<1>(MM, prod);
  fe_qget<2>(Z2, prod);
  fe_qget<3>(TT, prod);
  fe_sub(rX, PP, MM);   // N
  fe_add(rY, PP, MM);   // A
  fe_addn(rZ, Z2, TT);  // N
  fe_sub(rT, Z2, TT);   // N
  fe_qsel(a1, c, rX, rY, rZ, rX);
  fe_qsel(a2, c, rT, rZ, rT, rY);
  fe_mul(v, a1, a2);
}
// the operand lane c needs from entry |d| of a comb row (CT_QUADS uint4: y+x, y-x, 2dxy limbs)
MV_DEV void q_entry(fe& op, const uint4* row, int digit) {
  const uint32_t c = qlane();
  const bool neg = digit < 0;
  const int e = neg ? -digit : digit;
  // lane 0 takes y+x (y-x when negated), lane 1 the other, lane 3 2dxy, lane 2 the constant 2
  const uint32_t part = c == 0 ? (neg ? 1u : 0u) : (c == 1 ? (neg ? 0u : 1u) : 2u);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(row + e * CT_QUADS) + 9 * part;
#pragma unroll
  for (int i = 0; i < 9; i++) op.v[i] = w[i];
}
MV_DEV void q_entry_fix(fe& op, int digit) {
  const uint32_t c = qlane();
  if (c == 3 && digit < 0) fe_neg(op, op);  // -(2dxy)
  if (c == 2) fe_set(op, 2);
}
// sum over rows [r0, r1) of the comb entries of the signed radix-256 digits sd, coordinate form;
// the entries of the next two rows are in flight during an addition (loaded unconditionally, rows
// past r1 - 1 clamped to it: loads under a branch are waited on inside it, see ct_sum)
MV_DEV void q_ct_sum(fe& v, const uint4* tab, const uint32_t sd[8], int r0, int r1) {
  qp_identity(v);
  fe op0, op1;
  const int r01 = r0 + 1 < r1 ? r0 + 1 : r1 - 1;
  int d0 = digit256(sd, r0), d1 = digit256(sd, r01);
  q_entry(op0, tab + (size_t)r0 * CT_ROW, d0);
  q_entry(op1, tab + (size_t)r01 * CT_ROW, d1);
#pragma unroll 1
  for (int i = r0; i < r1; i++) {
    fe cur = op0;
    const int dcur = d0;
    op0 = op1;
    d0 = d1;
    const int in = i + 2 < r1 ? i + 2 : r1 - 1;
    d1 = digit256(sd, in);
    q_entry(op1, tab + (size_t)in * CT_ROW, d1);
    q_entry_fix(cur, dcur);
    qp_madd(v, cur);
  }
}

// the same over rows r0 .. r0 + NR - 1 (r0 a multiple of 4) with every row's entry in flight
// before the first addition: row I's entry is loaded, then rows I + 1 .. (recursively: no array,
// whose unrolled indices the compiler left to scratch), then row I is added
template <int I, int NR, bool FRESH>
MV_DEV void q_ct_rows(fe& v, const uint4* tab, const uint32_t (&w)[NR / 4], int r0) {
  const int d = ((int)(w[I >> 2] << (24 - 8 * (I & 3)))) >> 24;
  fe op;
  q_entry(op, tab + (size_t)(r0 + I) * CT_ROW, d);
  if constexpr (I + 1 < NR) {
    q_ct_rows<I + 1, NR, FRESH>(v, tab, w, r0);
  } else if constexpr (FRESH) {
    qp_identity(v);
  }
  q_entry_fix(op, d);
  qp_madd(v, op);
}
// FRESH: v = the sum; else v += the sum
template <int NR, bool FRESH = true>
MV_DEV void q_ct_sum_pf(fe& v, const uint4* tab, const uint32_t sd[8], int r0) {
  static_assert(NR % 4 == 0, "whole digit words");
  uint32_t w[NR / 4];
#pragma unroll
  for (int i = 0; i < NR / 4; i++) w[i] = pick8(sd, (r0 >> 2) + i);
  q_ct_rows<0, NR, FRESH>(v, tab, w, r0);
}

// 4 signatures per workgroup: one wave decodes (4 rows), one wave holds the four B roles and
// one the four A roles (16 lanes each), so every wave has a SIMD of its own; with 16
// signatures per workgroup (12 waves, 3 per SIMD) SHA-512 k took 27 us instead of ~10
constexpr uint32_t C16_SIGS = 4;    // signatures per k_verify_comb16 workgroup
constexpr uint32_t C16_TROLES = 8;  // table-sum roles: four over the B rows, four over the A rows
// + one spare wave, which ingests (with the other three) when the kernel parses its blocks and
// then hashes the block digests
constexpr uint32_t C16_THREADS = 16 * C16_SIGS + C16_TROLES * 4 * C16_SIGS + 64;
// the kernel's wall clock (100 MHz): online-service diagnostics
MV_DEV uint64_t on_now() { return (uint64_t)wall_clock64(); }

// 8 little-endian words at any byte address (9 aligned words funnel-shifted; the block buffers
// are readable 16 bytes past each block)
MV_DEV void load8_unaligned(uint32_t w[8], const uint8_t* p) {
  const uint32_t* q = reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
  uint32_t a[9];
#pragma unroll
  for (int i = 0; i < 9; i++) a[i] = q[i];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = sh ? __builtin_amdgcn_alignbyte(a[i + 1], a[i], sh) : a[i];
}

// One workgroup's share (signatures 4 wg .. 4 wg + 3) of the short-chain comb verify: the body
// of k_verify_comb16, also run job by job by the resident online service (k_online below).
// Two barriers: 0 after the ingest, 1 when role 0 has decoded R and the A wave has S = [s]B - [k]A.
// Between them the waves meet through LDS flags (spins with s_sleep; every wave has its own
// SIMD; the spare wave hashes the block digests):
//   role 0 (wave 0, one 16-lane row per signature)  the ZIP-215 decode of R
//   B wave (four roles of quads)   8 B rows each; then, once the A wave has published k's
//                                  digits, 4 A rows each (rows 16..31); a lane tree over its roles
//   A wave (four roles of quads)   the messages' digests, SHA-512 k, k's digits -> LDS; 4 A rows
//                                  each (rows 0..15); a lane tree; + the B wave's total = S
// then role 0: R - S, and the torsion test of qp_in_torsion (= [8](R - S) is the identity).
// stamp (online job 0, MV_ONLINE_TRACE): barrier 0 (wave 1), the B rows done, S done, R decoded, barrier 1;
// [7] digests done, [8] k's digits published.
MV_DEV void comb16_wg(uint32_t wg, const uint8_t* msg, const uint8_t* sig, const uint8_t* __restrict__ pk,
                      const uint32_t* key_idx, uint32_t n, const uint4* __restrict__ combB,
                      const uint4* __restrict__ combA, const uint8_t* __restrict__ key_ok,
                      uint8_t* __restrict__ status, const mvk::BlockVerdictOut& bv, const mvk::BlockHashIn& hin,
                      const mvk::BlockIngestIn& ing, uint64_t* stamp = nullptr) {
  __shared__ uint32_t part_b[C16_SIGS][36];  // the B wave's total, coordinate c at words 9c..
  __shared__ uint32_t part_s[C16_SIGS][36];  // S
  __shared__ uint32_t kdl[C16_SIGS][8];      // k's radix-256 digits, A wave -> B wave
  __shared__ uint32_t kflag, bflag;          // kdl written; part_b written
  constexpr int BROWS = CT_ROWS / 4;         // B rows per role
  constexpr int AROWS = CT_ROWS / 8;         // A rows per role (each wave takes half of them)
  const uint32_t t = threadIdx.x;
  static_assert(C16_THREADS == 4 * 64 && C16_SIGS == 4, "one ingest wave per block of the workgroup");
  static_assert(4 * C16_SIGS * (C16_TROLES / 2) == 64, "the B roles fill one wave, the A roles another");
  if (t == 0) {  // read after barrier 0
    kflag = 0;
    bflag = 0;
  }
  // With the ingest (ing.buf), role 0 does not wait for it: it decodes R speculatively from the
  // raw block's last 64 bytes (the signature is the bincode's last field, crypto.rs:309-347) and
  // meets barrier 0 inside its power chain (after 24 of 263 products, about when the parse is
  // done); waves 1..3 parse the blocks (wave 1 also the fourth) and meet it after. Role 0 then
  // checks its R against the parsed signature and decodes again if a block differs (trailing
  // bytes, a malformed block).
  const uint32_t wv = __builtin_amdgcn_readfirstlane(t >> 6);
#ifndef MV_SPEC_MAX
#define MV_SPEC_MAX 3  // blocks per workgroup up to which role 0 decodes speculatively
#endif
  // speculation when waves 1..3 can parse the workgroup's blocks one each; with four blocks all
  // four waves parse (one each) and role 0 decodes after barrier 0
  const bool spec = ing.buf && n - wg * C16_SIGS <= MV_SPEC_MAX;  // workgroup-uniform
  if (ing.buf && (!spec || wv != 0)) {  // barrier 0 after the parse (ingest_dev.h)
    __shared__ IngestLds igl[C16_SIGS];
    const CommitteeView cv{ing.stakes, ing.n_auth, ing.epoch, ing.quorum_thr};
    const IngestOut io{ing.stage, ing.pre_off, ing.pre_len, ing.sig, ing.key_idx, ing.facts, ing.claimed};
    const uint32_t first = spec ? wv - 1 : wv, step = spec ? C16_SIGS - 1 : C16_SIGS;
    for (uint32_t j = first; j < C16_SIGS; j += step) {
      const uint32_t bi = wg * C16_SIGS + j;
      if (bi < n) ingest_block<true>(bi, ing.buf, ing.off, ing.len, cv, io, igl[wv]);
    }
    __threadfence();  // its outputs are read by the other waves after the barrier
    __syncthreads();  // barrier 0
  } else if (!ing.buf) {
    __syncthreads();  // barrier 0
  }
  if (stamp && t == 64) __hip_atomic_store(stamp, on_now(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (__builtin_amdgcn_readfirstlane(t) >= C16_THREADS - 64) {  // the spare wave: the block digests, barrier 1
    if (hin.stage) {
      // B2(P || sig), the staged signature after each pre-image (one quad per block): off the
      // A wave's chain, which then hashes P alone (DUAL's extra final blocks no longer delay k)
      b2q::quad_hash_range<false, 1, true, true, 64>(wg * C16_SIGS, C16_SIGS, hin.stage, hin.pre_off, hin.pre_len,
                                                     n, hin.digest, nullptr);
      __threadfence();  // read by role 0's verdict after barrier 1
    }
    __syncthreads();
    return;
  }
  const bool row_role = t < 16 * C16_SIGS;
  const uint32_t role = row_role ? 0u : 1u + (t - 16 * C16_SIGS) / (4 * C16_SIGS);
  const uint32_t sq = row_role ? t >> 4 : (t >> 2) & (C16_SIGS - 1), c = t & 3u;
  const uint32_t gid = wg * C16_SIGS + sq;
  const uint32_t idx = gid < n ? gid : n - 1;
  uint32_t key = 0;  // role 0 reads it after barrier 0, inside its branch
  fe v;  // coordinate c of this role's point
  bool okR = false, s_ok = false;
  // the branches around the barriers and the flags are wave-uniform (readfirstlane: scalar branches)
  if (__builtin_amdgcn_readfirstlane(role) == 0) {  // every lane of the row holds the signature's R and s
    uint32_t rw[8], sw[8];
    p3 R;
    if (spec) {
      // speculative: the raw block's R (a block shorter than a signature reads a word of the
      // signature array instead -- in bounds, wrong, decoded again below)
      const uint64_t L = ing.len[idx];
      load8_unaligned(rw, L >= 64 ? ing.buf + ing.off[idx] + L - 64 : sig + 64 * (size_t)idx);
#ifndef MV_SPEC_AT
#define MV_SPEC_AT 20  // barrier 0 after 24 of the chain's products, about when the parse is done (40: 2% fewer blocks/s, r04at)
#endif
      decompress1_r16<MV_SPEC_AT>(R, okR, rw, [&] { __syncthreads(); });  // barrier 0
      uint32_t pw[8];
      load8(pw, sig + 64 * (size_t)idx);  // the parsed R
      bool same = true;
#pragma unroll
      for (int i = 0; i < 8; i++) same = same && pw[i] == rw[i];
      if (__ballot(!same)) decompress1_r16(R, okR, pw);  // some row guessed wrong: decode the parsed R
    } else {
      load8(rw, sig + 64 * (size_t)idx);
      decompress1_r16(R, okR, rw);
    }
    load8(sw, sig + 64 * (size_t)idx + 32);
    s_ok = sc_is_canonical(sw);
    key = key_idx[idx];
    fe_qsel(v, c, R.X, R.Y, R.Z, R.T);
    if (stamp && t == 0) __hip_atomic_store(stamp + 3, on_now(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
    key = key_idx[idx];
    const uint4* tabA = combA + (size_t)key * CT_TABLE;
    const uint32_t tr = role - 1;  // 0 .. 3: the B wave's roles; 4 .. 7: the A wave's
    const bool b_wave = __builtin_amdgcn_readfirstlane(tr) < C16_TROLES / 2;
    const uint32_t wr = tr & 3u;  // the role within its wave: lanes 16 wr .. 16 wr + 15
    if (b_wave) {
      uint32_t sw[8], sd[8], kd[8];
      load8(sw, sig + 64 * (size_t)idx + 32);
      sc_recode256(sd, sw);
      q_ct_sum_pf<BROWS>(v, combB, sd, (int)wr * BROWS);
      if (stamp && t == 64) __hip_atomic_store(stamp + 1, on_now(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      while (__hip_atomic_load(&kflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) __builtin_amdgcn_s_sleep(1);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
      for (int i = 0; i < 8; i++) kd[i] = kdl[sq][i];
      q_ct_sum_pf<AROWS, false>(v, tabA, kd, CT_ROWS / 2 + (int)wr * AROWS);
    } else {
      if (hin.stage) {
        // the signed message's digest of this workgroup's blocks first (one quad per block, quads
        // 0 .. C16_SIGS - 1 of the A wave): M = B2(P) feeds the challenge below (the block digest
        // B2(P || sig) is the spare wave's)
        b2q::quad_hash_range<false, 1, true, true>(wg * C16_SIGS, C16_SIGS, hin.stage, hin.pre_off, hin.pre_len, n,
                                                    hin.msg_digest, nullptr);
        __threadfence();  // the digests are read back below (other lanes) and by role 0's verdict
      }
      if (stamp && t == 128) __hip_atomic_store(stamp + 7, on_now(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      // k = SHA-512(R || A || M) mod l over the encodings as received (A = the committee key's
      // bytes). A workgroup with one distinct signature (a one-block request) runs it on the
      // scalar unit (sha512s_96, wave-uniform operands); otherwise every lane runs its own
      uint32_t h[16], k[8], kd[8];
#ifndef MV_SCALAR_SHA
#define MV_SCALAR_SHA 0
#endif
      if (MV_SCALAR_SHA && n - wg * C16_SIGS == 1) {
        const uint32_t g2 = wg * C16_SIGS;
        const uint32_t k2 = __builtin_amdgcn_readfirstlane(key_idx[g2]);
        uint32_t kin[24];
#pragma unroll
        for (int i = 0; i < 8; i++) {
          kin[i] = __builtin_amdgcn_readfirstlane(reinterpret_cast<const uint32_t*>(sig + 64 * (size_t)g2)[i]);
          kin[8 + i] = __builtin_amdgcn_readfirstlane(reinterpret_cast<const uint32_t*>(pk + 32 * (size_t)k2)[i]);
          kin[16 + i] = __builtin_amdgcn_readfirstlane(reinterpret_cast<const uint32_t*>(msg + 32 * (size_t)g2)[i]);
        }
        sha512s_96(h, kin);
      } else {
        uint32_t kin[24];
        load8(kin, sig + 64 * (size_t)idx);
        load8(kin + 8, pk + 32 * (size_t)key);
        load8(kin + 16, msg + 32 * (size_t)idx);
        sha512_short(h, kin, 96);
      }
      sc_reduce512(k, h);
      sc_recode256(kd, k);
      if (wr == 0 && c == 0) {
#pragma unroll
        for (int i = 0; i < 8; i++) kdl[sq][i] = kd[i];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (t == 128) __hip_atomic_store(&kflag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (stamp && t == 128) __hip_atomic_store(stamp + 8, on_now(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      q_ct_sum_pf<AROWS>(v, tabA, kd, (int)wr * AROWS);
    }
    // the wave's four roles -> role 0 of the wave (lanes 16 h up)
    for (uint32_t h = 2; h >= 1; h >>= 1) {
      fe w;
#pragma unroll
      for (int i = 0; i < 9; i++) w.v[i] = (uint32_t)__shfl_down((int)v.v[i], 4 * C16_SIGS * h, 64);
      if (wr < h) qp_add(v, w);
    }
    if (b_wave) {
      if (wr == 0) {
#pragma unroll
        for (int i = 0; i < 9; i++) part_b[sq][9 * c + i] = v.v[i];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (t == 64) __hip_atomic_store(&bflag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
      while (__hip_atomic_load(&bflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) __builtin_amdgcn_s_sleep(1);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      fe w;
#pragma unroll
      for (int i = 0; i < 9; i++) w.v[i] = part_b[sq][9 * c + i];
      qp_add(v, w);
      if (wr == 0) {
#pragma unroll
        for (int i = 0; i < 9; i++) part_s[sq][9 * c + i] = v.v[i];
      }
      if (stamp && t == 128) __hip_atomic_store(stamp + 2, on_now(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  __syncthreads();  // barrier 1
  if (stamp && t == 0) __hip_atomic_store(stamp + 4, on_now(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (role == 0) {  // lanes 0..3 of each row form the quad (the other lanes repeat it)
    fe S;
#pragma unroll
    for (int i = 0; i < 9; i++) S.v[i] = part_s[sq][9 * c + i];
    // R' = S = [s]B - [k]A (the A tables hold -A); R - R': -S has X and T negated
    fe nS;
    fe_neg(nS, S);
    fe_cmov(S, nS, c == 0 || c == 3);
    qp_add(v, S);
    const bool small = qp_in_torsion(v);
    if ((t & 15u) == 0 && gid < n) put_status(status, bv, gid, !key_ok[key] ? 2 : ((s_ok && okR && small) ? 0 : 1));
  }
}

__global__ void __launch_bounds__(C16_THREADS) k_verify_comb16(const uint8_t* msg, const uint8_t* sig,  // not restrict: the ingest phase writes it
                                                               const uint8_t* __restrict__ pk,
                                                               const uint32_t* key_idx,  // likewise
                                                               uint32_t n,
                                                               const uint4* __restrict__ combB,
                                                               const uint4* __restrict__ combA,
                                                               const uint8_t* __restrict__ key_ok,
                                                               uint8_t* __restrict__ status,
                                                               const mvk::BlockVerdictOut bv,
                                                               const mvk::BlockHashIn hin,
                                                               const mvk::BlockIngestIn ing) {
  comb16_wg(blockIdx.x, msg, sig, pk, key_idx, n, combB, combA, key_ok, status, bv, hin, ing);
}

// The resident online service (kernels.h OnlineArgs). Every branch around a barrier is
// uniform (the role is the workgroup's, decisions are broadcast through LDS), and every wait
// loop also tests the launch's end, so all waves leave.
constexpr uint32_t ON_BATCH = 64;  // the poller's window (requests it can move per pass): one wave's lanes
constexpr uint32_t ON_COPY_UNROLL = 8;  // 16-B input loads per poller thread in flight
static_assert(IG_WIN == mvk::INGEST_WINDOW_BYTES, "the host's eligibility test uses the ingest window");
static_assert(ON_BATCH <= mvk::ONLINE_SLOTS && ON_BATCH <= 64 && mvk::ONLINE_SLOTS % 64 == 0,
              "the window's lanes cover distinct slots, one wave");

// Workgroup 0: moves published requests from page-locked memory into HBM, appends their jobs.
MV_DEV void online_poller(const mvk::OnlineArgs& A) {
  mvk::OnlineCtl* ctl = A.ctl;
  mvk::OnlineDev* dev = A.dev;
  __shared__ uint32_t sh[5];              // kind (0 idle, 1 move, 2 exit), ready lo / hi, count, advance
  __shared__ uint32_t pre[ON_BATCH + 1];  // 16-B chunk prefix over the batch's inputs
  __shared__ uint32_t nblk[ON_BATCH];
  __shared__ uint32_t qoff[ON_BATCH];     // request - ready of each moved request
  __shared__ uint64_t dstp[ON_BATCH];     // where its input goes: its slot's scratch
  const uint32_t t = threadIdx.x;
  const uint64_t t_start = on_now();
  uint64_t t_busy = t_start;
  uint64_t why = 0;  // wave 0: why the launch ends (mvk::ONLINE_EXIT_*)
  if (t == 0) {  // this launch's setup: tickets of earlier launches are void
    const unsigned long long tl = __hip_atomic_load(&dev->jobs_tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&dev->jobs_head, tl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&dev->quit, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&dev->epoch, A.launch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (;;) {
    if (t < 64) {
      // wave 0: every published request of the window [ready, ready + ON_BATCH), in any order:
      // a caller that publishes late (descheduled between reserving its number and writing
      // its seq) does not hold back the requests behind it (round 4 moved only the
      // consecutive prefix, and 99 concurrent callers stalled behind one). `moved[slot]`
      // (request + 1, poller-only) marks the ones already moved; `ready` advances over the
      // moved prefix. The window is at most the ring: the slots of its lanes are distinct.
      // Polls are relaxed (an acquire invalidates the caches every time: the working
      // workgroups' comb tables with them); one acquire fence once requests are seen. The
      // window's seq words are read together (one PCIe round trip): a request is published
      // once its seq holds its number + 1, which the host writes after its bytes.
      uint32_t kind = 0;
      const uint64_t rdy = __hip_atomic_load(&dev->ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      bool fresh = false, moved = false;
      uint32_t nb = 0, cb = 0;
      const uint64_t q = rdy + t;
      const uint32_t slot = (uint32_t)(q % mvk::ONLINE_SLOTS);
      if (t < ON_BATCH) {
        // moved[] (HBM) and seq (PCIe) read side by side; n and copy_bytes after seq. (Reading the
        // 16-byte descriptor in one nontemporal load instead served requests only after the
        // launch's idle exit, ~10 ms: that load is not system-coherent; profiles/r05/c5_desc_ab.txt)
        const unsigned long long mvq = __hip_atomic_load(&dev->moved[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const mvk::OnlineReq* r = A.reqs + slot;
        const uint64_t sq = __hip_atomic_load(&r->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        moved = mvq == q + 1;
        fresh = !moved && sq == q + 1;
        if (fresh) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: the slot's bytes after seq
          nb = r->n;
          cb = r->copy_bytes;
        }
      }
      const uint64_t fm = __ballot(fresh);
      const uint32_t cnt = (uint32_t)__builtin_popcountll(fm);
      // the moved prefix after this pass (lanes past the window count as not moved)
      const uint64_t notdone = __ballot(!(fresh || moved) || t >= ON_BATCH);
      const uint32_t adv = notdone ? (uint32_t)__builtin_ctzll(notdone) : 64u;
      const uint64_t now = on_now();
      if (fresh) {
        const uint32_t i = (uint32_t)__builtin_popcountll(fm & ((1ull << t) - 1));  // rank among the fresh
        qoff[i] = t;
        nblk[i] = nb;
        pre[i] = (cb + 15) / 16;  // chunk count, prefixed below
        __hip_atomic_store(&ctl->trace[slot][0], now, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      if (cnt || adv) {
        kind = 1;
        t_busy = now;
      } else if (__hip_atomic_load(&ctl->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
        kind = 2;
        why = mvk::ONLINE_EXIT_STOP;
      } else if (now - t_busy > A.idle_ticks) {
        kind = 2;
        why = mvk::ONLINE_EXIT_IDLE;
      } else if (now - t_start > A.max_ticks) {
        kind = 2;
        why = mvk::ONLINE_EXIT_MAX;
      }
      if (t == 0) {
        sh[0] = kind;
        sh[1] = (uint32_t)rdy;
        sh[2] = (uint32_t)(rdy >> 32);
        sh[3] = cnt;
        sh[4] = adv;
      }
    }
    __syncthreads();
    const uint32_t kind = sh[0], cnt = sh[3], adv = sh[4];
    const uint64_t rdy = (uint64_t)sh[1] | ((uint64_t)sh[2] << 32);
    if (kind == 2) {
      if (t == 0) {
        __hip_atomic_store(&dev->quit, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        // the exit record for the host's bounded stop (diagnostics when a launch will not end)
        __hip_atomic_store(&ctl->exit_why, why, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&ctl->exit_ready, rdy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&ctl->exit_head,
                           (uint64_t)__hip_atomic_load(&dev->jobs_head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&ctl->exit_tail,
                           (uint64_t)__hip_atomic_load(&dev->jobs_tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      return;
    }
    if (kind == 0) {
      __syncthreads();  // sh[] is rewritten by the next pass only after every wave read it
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    if (t == 0) {  // chunk prefix; each request's input goes to its slot's scratch
      uint32_t c = 0;
      for (uint32_t i = 0; i < cnt; i++) {
        const uint32_t k = pre[i];
        pre[i] = c;
        c += k;
        dstp[i] = (uint64_t)(A.scr + mvk::ONLINE_SCR_STRIDE * (uint32_t)((rdy + qoff[i]) % mvk::ONLINE_SLOTS));
      }
      pre[cnt] = c;
    }
    __syncthreads();
    // inputs: 16-byte chunk k of the batch by thread k (mod the workgroup), all independent;
    // ON_COPY_UNROLL loads per thread in flight before their stores, so a round of PCIe reads
    // moves 256 x 8 x 16 B = 32 KB (one round trip instead of one per 4 KB: a 64-block request
    // of config-1 blocks is ~25 KB)
    const uint32_t total = pre[cnt];
    // (a lane past the end copies its own 16 bytes of HBM sink onto themselves: no branch around
    // the loads, so they all stay in registers and in flight together, and no extra PCIe read)
    if (total <= blockDim.x) {  // one chunk per thread at most (a few small requests): one load each
      if (t < total) {
        uint32_t i = 0;
        while (pre[i + 1] <= t) i++;
        const uint32_t slot = (uint32_t)((rdy + qoff[i]) % mvk::ONLINE_SLOTS), c = t - pre[i];
        reinterpret_cast<uint4*>(dstp[i])[c] = reinterpret_cast<const uint4*>(A.in_host + mvk::ONLINE_IN_STRIDE * slot)[c];
      }
    } else for (uint32_t k0 = 0; k0 < total; k0 += blockDim.x * ON_COPY_UNROLL) {
      uint64_t src[ON_COPY_UNROLL], dst[ON_COPY_UNROLL];
#pragma unroll
      for (uint32_t u = 0; u < ON_COPY_UNROLL; u++) {
        const uint32_t kk = k0 + u * blockDim.x + t;
        const bool live = kk < total;
        const uint32_t k = live ? kk : 0u;
        uint32_t i = 0;
        while (pre[i + 1] <= k) i++;
        const uint32_t slot = (uint32_t)((rdy + qoff[i]) % mvk::ONLINE_SLOTS), c = k - pre[i];
        const uint64_t sink = (uint64_t)(dev->sink + 2 * t);
        src[u] = live ? (uint64_t)(A.in_host + mvk::ONLINE_IN_STRIDE * slot + 16 * (size_t)c) : sink;
        dst[u] = live ? dstp[i] + 16 * (uint64_t)c : sink;
      }
      uint64_t lo[ON_COPY_UNROLL], hi[ON_COPY_UNROLL];
#pragma unroll
      for (uint32_t u = 0; u < ON_COPY_UNROLL; u++) {
        const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(src[u]);
        lo[u] = x.x;
        hi[u] = x.y;
      }
#pragma unroll
      for (uint32_t u = 0; u < ON_COPY_UNROLL; u++) *reinterpret_cast<ulonglong2*>(dst[u]) = make_ulonglong2(lo[u], hi[u]);
    }
    __threadfence();  // the inputs before the jobs (agent scope)
    __syncthreads();
    if (t == 0) {
      unsigned long long jt = __hip_atomic_load(&dev->jobs_tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (uint32_t i = 0; i < cnt; i++) {
        const uint64_t q = rdy + qoff[i];
        const uint32_t slot = (uint32_t)(q % mvk::ONLINE_SLOTS), nj = (nblk[i] + C16_SIGS - 1) / C16_SIGS;
        dev->n[slot] = nblk[i];
        __hip_atomic_store(&dev->moved[slot], (unsigned long long)(q + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (nj == 0)  // a void request: complete it here
          __hip_atomic_store(&ctl->done[slot], q + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        else
          for (uint32_t j = 0; j < nj; j++, jt++) dev->jobs[jt % mvk::ONLINE_JOBS] = ((unsigned long long)q << 8) | j;
      }
      __hip_atomic_store(&dev->ready, (unsigned long long)(rdy + adv), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&dev->jobs_tail, jt, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (t < cnt)
      __hip_atomic_store(&ctl->trace[(rdy + qoff[t]) % mvk::ONLINE_SLOTS][1], on_now(), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();  // pre[] / nblk[] / qoff[] / sh[] are rewritten by the next pass
  }
}

// Workgroups 1..: take a ticket, wait until the ring's tail passes it, run that job from HBM,
// hand its outputs to the host.
MV_DEV void online_worker(const mvk::OnlineArgs& A) {
  mvk::OnlineCtl* ctl = A.ctl;
  mvk::OnlineDev* dev = A.dev;
  __shared__ uint32_t job[4];  // kind (1 work, 2 exit), request lo / hi, job
  const uint32_t t = threadIdx.x;
  const uint64_t t_start = on_now();
  bool setup = false;
  for (;;) {
    if (t == 0) {
      uint32_t kind = 2, j = 0;
      uint64_t q = 0;
      while (!setup) {  // the poller has voided earlier tickets
        if (__hip_atomic_load(&dev->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == A.launch) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          setup = true;
        } else if (on_now() - t_start > A.max_ticks + A.idle_ticks) {
          break;
        } else {
          __builtin_amdgcn_s_sleep(2);
        }
      }
      if (setup) {
        const unsigned long long tk = __hip_atomic_fetch_add(&dev->jobs_head, 1ull, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT);
        for (;;) {  // relaxed polls, one acquire fence when the ticket's job is there
          if (tk < __hip_atomic_load(&dev->jobs_tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            const unsigned long long e = dev->jobs[tk % mvk::ONLINE_JOBS];
            q = e >> 8;
            j = (uint32_t)(e & 0xffu);
            kind = 1;
            break;
          }
          if (__hip_atomic_load(&dev->quit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
              on_now() - t_start > A.max_ticks + A.idle_ticks)
            break;  // the launch is over (this ticket is voided by the next launch)
          __builtin_amdgcn_s_sleep(2);
        }
        if (kind == 1 && j == 0)
          __hip_atomic_store(&ctl->trace[q % mvk::ONLINE_SLOTS][2], on_now(), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
      }
      job[0] = kind;
      job[1] = (uint32_t)q;
      job[2] = (uint32_t)(q >> 32);
      job[3] = j;
    }
    __syncthreads();
    const uint32_t kind = job[0];
    const uint64_t q = (uint64_t)job[1] | ((uint64_t)job[2] << 32);
    const uint32_t j = __builtin_amdgcn_readfirstlane(job[3]);
    __syncthreads();  // job[] is rewritten by the next claim only after every wave read it
    if (kind == 2) return;
    const uint32_t slot = __builtin_amdgcn_readfirstlane((uint32_t)(q % mvk::ONLINE_SLOTS));
    const uint32_t n = __builtin_amdgcn_readfirstlane(dev->n[slot]);
    // the slot's HBM scratch (kernels.h layout): everything below is uniform address arithmetic
    uint8_t* sc = A.scr + mvk::ONLINE_SCR_STRIDE * slot;
    const uint64_t* off = reinterpret_cast<const uint64_t*>(sc);
    uint8_t* out = sc + mvk::ONLINE_O_OUT;
    uint8_t* md = out;
    uint8_t* bd = out + 32 * mvk::ONLINE_MAX_BLOCKS;
    uint8_t* st = out + 64 * mvk::ONLINE_MAX_BLOCKS;
    uint8_t* stage = sc + mvk::ONLINE_O_STAGE;
    uint64_t* poff = reinterpret_cast<uint64_t*>(sc + mvk::ONLINE_O_POFF);
    uint64_t* plen = reinterpret_cast<uint64_t*>(sc + mvk::ONLINE_O_PLEN);
    uint8_t* sig = sc + mvk::ONLINE_O_SIG;
    uint32_t* kidx = reinterpret_cast<uint32_t*>(sc + mvk::ONLINE_O_KIDX);
    uint32_t* facts = reinterpret_cast<uint32_t*>(sc + mvk::ONLINE_O_FACTS);
    uint8_t* claimed = sc + mvk::ONLINE_O_CLAIMED;
    const mvk::BlockVerdictOut bv{facts, claimed, md, bd, st};
    const mvk::BlockHashIn hin{stage, poff, plen, md, bd};
    const mvk::BlockIngestIn ing{sc + 16 * (size_t)n, off, off + n, A.stakes, A.n_auth, A.epoch, A.quorum_thr,
                                 stage, poff, plen, sig, kidx, facts, claimed};
    uint64_t* stamp = j == 0 ? &ctl->trace[slot][4] : nullptr;
    comb16_wg(j, md, sig, A.pk, kidx, n, (const uint4*)A.combB, (const uint4*)A.combA, A.key_ok,
              sc + mvk::ONLINE_O_SST, bv, hin, ing, stamp);
    __syncthreads();  // the job's digests and verdicts are in HBM (workgroup scope)
    if (stamp && t == 0) __hip_atomic_store(stamp + 5, on_now(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // this job's blocks: md and bd (8 words each), status -> page-locked output
    uint8_t* oh = A.out_host + mvk::ONLINE_OUT_STRIDE * slot;
    const uint32_t b0 = j * C16_SIGS, nb = n - b0 < C16_SIGS ? n - b0 : C16_SIGS;
    if (t < 16 * nb) {
      const uint32_t b = b0 + t / 16, w = t % 16;  // words 0..7 md, 8..15 bd
      const size_t o = w < 8 ? 32 * (size_t)b + 4 * w : 32 * ((size_t)mvk::ONLINE_MAX_BLOCKS + b) + 4 * (w - 8);
      *reinterpret_cast<uint32_t*>(oh + o) = *reinterpret_cast<const uint32_t*>(out + o);
    } else if (t >= 64 && t < 64 + nb) {
      const size_t o = 64 * (size_t)mvk::ONLINE_MAX_BLOCKS + b0 + (t - 64);
      oh[o] = out[o];
    }
    if (t < 128) __threadfence_system();  // the writers' outputs (waves 0, 1) before the done word
    __syncthreads();
    if (stamp && t == 0) __hip_atomic_store(stamp + 6, on_now(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (t == 0) {
      const uint32_t nj = (n + C16_SIGS - 1) / C16_SIGS;
      const uint32_t prev = __hip_atomic_fetch_add(&dev->jobs_done[slot], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (prev + 1 == nj) {
        __hip_atomic_store(&dev->jobs_done[slot], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&ctl->trace[slot][3], on_now(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&ctl->done[slot], q + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

__global__ void __launch_bounds__(C16_THREADS) k_online(const mvk::OnlineArgs A) {
  // liveness: this workgroup runs launch A.launch, then has left it (the host's bounded stop
  // reads these words when a launch does not end in time)
  uint32_t* live = &A.ctl->wg[blockIdx.x];
  if (threadIdx.x == 0) __hip_atomic_store(live, A.launch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (blockIdx.x == 0)
    online_poller(A);
  else
    online_worker(A);
  if (threadIdx.x == 0)
    __hip_atomic_store(live, A.launch | mvk::ONLINE_WG_LEFT, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The same predicate split in two, for small batches of long blocks (config 5, 8-KB
// pre-images), where k_b2_quad's serial chain of ~65 compressions is the latency path. The
// terms that need only the signature run in the same launch as the hash, on workgroups of
// their own (no cross-stream events: each costs ~10 us of queue drain on this path):
//   k_hash_comb_pre  workgroups [0, nh): quad BLAKE2b of 16 blocks each (blake2b_quad.h);
//                    [nh, nh + np): s < l and the ZIP-215 decode of R, 64 signatures each;
//                    [nh + np, nh + 2 np): -[s]B on C_B, 64 signatures each
//   k_comb_post      k = SHA-512(R || A || M) mod l, then the A-table entries of k's digits
//                    on eight roles of quads, a tree over the roles, [8], identity test (below).
// k_comb_post's latency is a SHA-512 and 4 + 5 two-product-deep additions instead of the R
// decode.
__global__ void __launch_bounds__(64) k_hash_comb_pre(const uint8_t* __restrict__ stage,
                                                      const uint64_t* __restrict__ poff,
                                                      const uint64_t* __restrict__ plen, uint8_t* __restrict__ md,
                                                      uint8_t* __restrict__ bd, const uint8_t* __restrict__ sig,
                                                      uint32_t n, uint32_t nh, uint32_t np,
                                                      const uint4* __restrict__ combB, uint4* __restrict__ rbuf,
                                                      uint4* __restrict__ sbuf, uint8_t* __restrict__ qflags) {
  const uint32_t blk = blockIdx.x;
  if (blk < nh) {
    b2q::quad_hash<true, 1, true>(blk, stage, poff, plen, n, md, bd);  // latency form: reads hoisted
    return;
  }
  const bool role_r = blk < nh + np;
  const uint32_t gid = (blk - nh - (role_r ? 0 : np)) * 64 + threadIdx.x;
  const uint32_t idx = gid < n ? gid : n - 1;
  uint4 q[9];
  if (role_r) {
    uint32_t rw[8], sw[8];
    load8(rw, sig + 64 * (size_t)idx);
    load8(sw, sig + 64 * (size_t)idx + 32);
    const bool s_ok = sc_is_canonical(sw);
    p3 R;
    bool okR;
    decompress1(R, okR, rw);
    p3_to_quads(q, R);
    if (gid < n) {
#pragma unroll
      for (int k = 0; k < 9; k++) rbuf[(size_t)gid * 9 + k] = q[k];
      qflags[gid] = (s_ok ? 1 : 0) | (okR ? 2 : 0);
    }
  } else {
    uint32_t sw[8], sd[8];
    load8(sw, sig + 64 * (size_t)idx + 32);
    sc_recode256(sd, sw);
    p3 acc;
    ct_sum(acc, combB, sd, 0, CT_ROWS);
    p3_neg(acc, acc);
    p3_to_quads(q, acc);
    if (gid < n) {
#pragma unroll
      for (int k = 0; k < 9; k++) sbuf[(size_t)gid * 9 + k] = q[k];
    }
  }
}

// k_comb_post: POST_SIGS signatures per workgroup, eight roles of one quad per signature
// (quad25519.h's coordinate layout: every point operation is two products deep):
//   phase 1  wave 0: k = SHA-512(R || A || M) mod l, one lane per signature, digits to LDS;
//            role 7 meanwhile: R - [s]B from k_hash_comb_pre's two points
//   phase 2  role w: the C_A entries of k's digits 4w .. 4w + 3 (four additions)
//   phase 3  a 3-level tree over the roles' sums; role 0: R - [s]B - sum (the tables hold -A),
//            [8], identity test
constexpr uint32_t POST_SIGS = 4;  // two waves per workgroup: each on a SIMD of its own
constexpr int POST_ROLES = 8;
__global__ void __launch_bounds__(4 * POST_SIGS * POST_ROLES) k_comb_post(const uint8_t* msg,  // not restrict: bv writes it
                                                                         const uint8_t* __restrict__ sig,
                                                                         const uint8_t* __restrict__ pk,
                                                                         const uint32_t* __restrict__ key_idx, uint32_t n,
                                                                         const uint4* __restrict__ combA,
                                                                         const uint8_t* __restrict__ key_ok,
                                                                         const uint4* __restrict__ rbuf,
                                                                         const uint4* __restrict__ sbuf,
                                                                         const uint8_t* __restrict__ qflags,
                                                                         uint8_t* __restrict__ status,
                                                                         const mvk::BlockVerdictOut bv) {
  __shared__ uint32_t part[POST_ROLES][POST_SIGS][36];  // per-role sums, coordinate c at words 9c..
  __shared__ uint32_t skd[8][POST_SIGS];                // k's signed radix-256 digits, [word][sig]
  const uint32_t t = threadIdx.x, role = t / (4 * POST_SIGS), sq = (t >> 2) & (POST_SIGS - 1), c = t & 3u;
  const uint32_t gid = blockIdx.x * POST_SIGS + sq;
  const uint32_t idx = gid < n ? gid : n - 1;
  const uint32_t key = key_idx[idx];
  if (t < POST_SIGS) {  // k once per signature (wave 0, lanes 0 .. POST_SIGS - 1)
    const uint32_t g2 = blockIdx.x * POST_SIGS + t, i2 = g2 < n ? g2 : n - 1;
    uint32_t kin[24], h[16], k[8], kd[8];
    load8(kin, sig + 64 * (size_t)i2);
    load8(kin + 8, pk + 32 * (size_t)key_idx[i2]);
    load8(kin + 16, msg + 32 * (size_t)i2);
    sha512_short(h, kin, 96);
    sc_reduce512(k, h);
    sc_recode256(kd, k);
#pragma unroll
    for (int i = 0; i < 8; i++) skd[i][t] = kd[i];
  } else if (role == POST_ROLES - 1) {  // R - [s]B (k_hash_comb_pre's R and -[s]B), coordinate form
    const uint32_t* rw = reinterpret_cast<const uint32_t*>(rbuf + (size_t)idx * 9) + 9 * c;
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(sbuf + (size_t)idx * 9) + 9 * c;
    fe v, w;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      v.v[i] = rw[i];
      w.v[i] = sw[i];
    }
    qp_add(v, w);
#pragma unroll
    for (int i = 0; i < 9; i++) part[0][sq][9 * c + i] = v.v[i];  // role 0's slot is free until phase 3
  }
  __syncthreads();
  fe v;
  {
    uint32_t kd[8];
#pragma unroll
    for (int i = 0; i < 8; i++) kd[i] = skd[i][sq];
    const int r0 = (int)role * (CT_ROWS / POST_ROLES);
    q_ct_sum(v, combA + (size_t)key * CT_TABLE, kd, r0, r0 + CT_ROWS / POST_ROLES);  // -[k_w]A
  }
  fe rs;  // R - [s]B, read by role 0 before its slot is overwritten
  if (role == 0) {
#pragma unroll
    for (int i = 0; i < 9; i++) rs.v[i] = part[0][sq][9 * c + i];
  }
  __syncthreads();
  // tree over the roles' sums: role w < h adds role w + h's
  for (uint32_t h = POST_ROLES / 2; h >= 1; h >>= 1) {
    if (role >= h && role < 2 * h) {
#pragma unroll
      for (int i = 0; i < 9; i++) part[role][sq][9 * c + i] = v.v[i];
    }
    __syncthreads();
    if (role < h) {
      fe w;
#pragma unroll
      for (int i = 0; i < 9; i++) w.v[i] = part[role + h][sq][9 * c + i];
      qp_add(v, w);
    }
    __syncthreads();
  }
  if (role == 0) {
    // v = -[k]A; R - [s]B + [k]A = R - R': negate v (X and T), add R - [s]B
    fe nv;
    fe_neg(nv, v);
    fe_cmov(v, nv, c == 0 || c == 3);
    qp_add(v, rs);
    const bool small = qp_in_torsion(v);  // [8](R - R') is the identity
    const uint8_t f = qflags[idx];
    if (c == 0 && gid < n) put_status(status, bv, gid, !key_ok[key] ? 2 : (((f & 3) == 3 && small) ? 0 : 1));
  }
}

}  // namespace mv

// ---------------------------------------------------------------- launchers
namespace mvk {

size_t comb_table_bytes(uint32_t nbases) { return (size_t)nbases * mv::CT_TABLE * sizeof(uint4); }

hipError_t launch_comb_init(const uint8_t* enc, uint32_t nb, int negate, void* tab, uint8_t* ok, hipStream_t s) {
  if (nb == 0) return hipSuccess;
  const uint32_t threads = nb * mv::CT_ROWS * mv::CT_ENTRIES;
  hipLaunchKernelGGL(mv::k_comb_init, dim3((threads + 255) / 256), dim3(256), 0, s, enc, nb, negate, (uint4*)tab, ok);
  return hipGetLastError();
}

bool comb_short_chain(const Knobs& kn, uint32_t n) {
  return kn.comb_quad >= 0 ? kn.comb_quad != 0 : n <= 64u * 256u;
}

hipError_t launch_verify_comb(const Knobs& kn, const uint8_t* msg, const uint8_t* sig, const uint8_t* pk, const uint32_t* key_idx,
                              uint32_t n, const void* combB, const void* combA, const uint8_t* key_ok,
                              uint8_t* status, hipStream_t s, const BlockVerdictOut* bv, const BlockHashIn* hin,
                              const BlockIngestIn* ing) {
  if ((hin || ing) && !comb_short_chain(kn, n)) return hipErrorInvalidValue;  // the caller parses / hashes first
  if (n == 0) return hipSuccess;
  const BlockVerdictOut none{};
  // short chains (k_verify_comb16: a row per R decode, quads for the table sums) up to 64
  // workgroups of 256 signatures' worth (the online path); MV_COMB_QUAD=0 / 1 forces
  // k_verify_comb / k_verify_comb16 (A/B, tests)
  const BlockHashIn nohash{};
  const BlockIngestIn noingest{};
  if (comb_short_chain(kn, n))
    hipLaunchKernelGGL(mv::k_verify_comb16, dim3((n + mv::C16_SIGS - 1) / mv::C16_SIGS), dim3(mv::C16_THREADS), 0, s,
                       msg, sig, pk, key_idx, n, (const uint4*)combB, (const uint4*)combA, key_ok, status,
                       bv ? *bv : none, hin ? *hin : nohash, ing ? *ing : noingest);
  else
    hipLaunchKernelGGL(mv::k_verify_comb, dim3((n + 63) / 64), dim3(256), 0, s, msg, sig, pk, key_idx, n,
                       (const uint4*)combB, (const uint4*)combA, key_ok, status, bv ? *bv : none);
  return hipGetLastError();
}

hipError_t launch_online(const OnlineArgs& a, uint32_t grid, hipStream_t s) {
  if (grid < 2) return hipErrorInvalidValue;  // a poller and at least one worker
  hipLaunchKernelGGL(mv::k_online, dim3(grid), dim3(mv::C16_THREADS), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_hash_comb_pre(const uint8_t* stage, const uint64_t* poff, const uint64_t* plen, uint32_t n,
                                uint8_t* md, uint8_t* bd, const uint8_t* sig, const void* combB, void* rbuf,
                                void* sbuf, uint8_t* qflags, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint32_t nh = (n + 15) / 16, np = (n + 63) / 64;
  hipLaunchKernelGGL(mv::k_hash_comb_pre, dim3(nh + 2 * np), dim3(64), 0, s, stage, poff, plen, md, bd, sig, n, nh,
                     np, (const uint4*)combB, (uint4*)rbuf, (uint4*)sbuf, qflags);
  return hipGetLastError();
}

hipError_t launch_comb_post(const uint8_t* msg, const uint8_t* sig, const uint8_t* pk, const uint32_t* key_idx,
                            uint32_t n, const void* combA, const uint8_t* key_ok, const void* rbuf,
                            const void* sbuf, const uint8_t* qflags, uint8_t* status, hipStream_t s,
                            const BlockVerdictOut* bv) {
  if (n == 0) return hipSuccess;
  const BlockVerdictOut none{};
  hipLaunchKernelGGL(mv::k_comb_post, dim3((n + mv::POST_SIGS - 1) / mv::POST_SIGS), dim3(4 * mv::POST_SIGS * mv::POST_ROLES),
                     0, s, msg, sig, pk, key_idx, n,
                     (const uint4*)combA, key_ok, (const uint4*)rbuf, (const uint4*)sbuf, qflags, status, bv ? *bv : none);
  return hipGetLastError();
}

}  // namespace mvk
