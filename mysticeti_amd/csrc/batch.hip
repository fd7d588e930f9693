// Batch ed25519 verification on gfx950: one random linear combination of the whole
// batch, checked as a single multi-scalar multiplication (bucket method), with an
// exact per-signature fallback on the device when the combined equation fails.
//
// Semantics: ed25519-consensus 2.1.0 `batch::Verifier` (the ZIP-215 batch rule that
// is designed to agree with the single `VerificationKey::verify` called at
// mysticeti-core/src/crypto.rs:188): for signatures (A_i, R_i, s_i) with challenges
// k_i and independent uniformly random 127-bit z_i,
//     [8]( -[sum z_i s_i]B + sum [z_i]R_i + sum [z_i k_i]A_i ) == O.
// Every individually valid signature satisfies [8]([s_i]B - [k_i]A_i - R_i) = O, so a
// batch of valid signatures always passes; a batch holding an invalid one passes with
// probability <= 2^-127 over the z_i. Per-signature preconditions (s < l, A and R
// decode) are decided exactly in k_bv_prep and excluded from the combination. When
// the combination fails, k_verify (kernels.hip) re-verifies every signature of the
// batch individually (it reads the batch flag and exits at once when it passed), so
// every verdict is the single-verify verdict.
//
// Pipeline (one batch of n signatures, all on one stream):
//   k_bv_prep     lane per signature: SHA-512 challenge, ZIP-215 decode of A and R,
//                 z_i = BLAKE2b(secret || call || i), scalars z_i and z_i k_i mod l,
//                 affine points (y+x, y-x, 2dxy) to HBM, sum z_i s_i
//   k_part_*, k_fine_sort   two-pass counting sort of the (bucket, point) entries
//                 (LDS histograms and ranks; no global atomics; the _lds forms stage
//                 their output in LDS and store it coalesced)
//   k_bv_bucket   lane per bucket: the bucket's sum T (k_bv_bucket_bal + _fix: the
//                 same sums with an equal number of entries per lane)
//   k_bv_reduce   tree over the buckets (fan-in 8) of the pairs (V, T) per window
//                 (_q: four lanes per element, _r: a wave per element on small levels)
//   k_bv_final    Horner over the 16 window sums (one DPP row per coordinate with one
//                 equation), -[sum z s]B, [8], identity test
// Sub-batch equations: the batch may be cut into up to BV_MAXG groups of whole 1024-
// signature chunks, each with its own buckets and its own combined equation (one flag per
// group). The fallback then re-verifies only the groups whose equation failed, so k bad
// signatures cost at most k groups of single verifies instead of the whole batch.
// Windows: signed radix 2^16, |digit| <= 2^15; R scalars (z < 2^127) use windows 0..7,
// A scalars (< l < 2^253) windows 0..15.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "fe25519.h"
#include "ge25519.h"
#include "hash_dev.h"
#include "kernels.h"
#include "scalar25519.h"
#include "tables.h"
#include "comb.h"
#include "quad25519.h"
#include "pt_r16.h"

namespace mv {

constexpr int BV_C = 16;                    // window bits
constexpr int BV_NB = 1 << (BV_C - 1);      // bucket magnitudes 1..2^15 per window
constexpr int BV_NW = 16;                   // windows
constexpr int BV_NWR = 8;                   // windows of the 127-bit R scalars
constexpr uint32_t BV_NKG = BV_NW * BV_NB;  // bucket keys per group, key = w * NB + |d| - 1
constexpr int BV_FINE_BITS = 8;             // bucket sort: partition = key >> 8 (window +
constexpr int BV_NPG = BV_NKG >> BV_FINE_BITS;  // 7 high magnitude bits), then 256 buckets
constexpr int BV_FAN = 8;                   // reduction fan-in
constexpr int BV_MAXG = mvk::BATCH_MAX_GROUPS;  // sub-batch equations per batch
constexpr int P3_QUADS = 9;
constexpr int SC_QUADS = 3;                 // z (4 words), z*k mod l (8 words)
constexpr int BSUM_WORDS = 12;              // z * s < 2^381

// signed radix-2^16 digit w of a little-endian scalar, running carry in/out;
// digit in [-2^15, 2^15 - 1] (v = 16 bits + carry <= 2^16)
MV_DEV int bv_digit(uint32_t word, int half, uint32_t& carry) {
  const uint32_t v = (half ? (word >> 16) : (word & 0xffffu)) + carry;
  carry = v >= (1u << 15) ? 1u : 0u;
  return (int)v - (int)(carry << 16);
}

// Calls fn(window, digit, isA) for every nonzero digit of (z, zk). z < 2^127 and
// zk < 2^253 leave the top windows (7 and 15) with a value <= 2^15 after the carry,
// so they take it unsigned: no carry window, and no bucket collects half the batch.
template <class Fn>
MV_DEV void bv_for_digits(const uint32_t z[4], const uint32_t zk[8], Fn fn) {
  uint32_t carry = 0;
#pragma unroll
  for (int w = 0; w < 7; w++) {
    const int d = bv_digit(z[w >> 1], w & 1, carry);
    if (d) fn(w, d, 0);
  }
  {
    const int d = (int)((z[3] >> 16) + carry);
    if (d) fn(7, d, 0);
  }
  carry = 0;
#pragma unroll
  for (int w = 0; w < 15; w++) {
    const int d = bv_digit(zk[w >> 1], w & 1, carry);
    if (d) fn(w, d, 1);
  }
  {
    const int d = (int)((zk[7] >> 16) + carry);
    if (d) fn(15, d, 1);
  }
}

MV_DEV uint32_t bv_key(int w, int d) { return (uint32_t)w * BV_NB + (uint32_t)(d < 0 ? -d : d) - 1u; }

MV_DEV void precomp_from_affine(precomp& pc, const p3& P) {
  fe d2;
  fe_const(d2, K_D2);
  fe_addn(pc.ypx, P.Y, P.X);
  fe_sub(pc.ymx, P.Y, P.X);
  fe_mul(pc.xy2d, P.T, d2);  // P.Z = 1, P.T = xy
}

MV_DEV void pt_store(uint4* pts, size_t idx, const precomp& pc) {
  uint4 q[7];
  precomp_to_quads(q, pc);
  uint4* p = pts + idx * PT_QUADS;
#pragma unroll
  for (int i = 0; i < 7; i++) p[i] = q[i];
  if (PT_QUADS == 8) p[7] = make_uint4(0, 0, 0, 0);  // whole-line writes
}
MV_DEV void pt_load(precomp& pc, const uint4* pts, uint32_t idx) {
  const uint4* p = pts + (size_t)idx * PT_QUADS;
  uint4 q[7];
#pragma unroll
  for (int i = 0; i < 7; i++) q[i] = p[i];
  quads_to_precomp(pc, q);
}
MV_DEV void p3_store(uint4* a, size_t idx, const p3& P) {
  uint4 q[9];
  p3_to_quads(q, P);
  uint4* p = a + idx * P3_QUADS;
#pragma unroll
  for (int i = 0; i < 9; i++) p[i] = q[i];
}
MV_DEV void p3_load(p3& P, const uint4* a, size_t idx) {
  const uint4* p = a + idx * P3_QUADS;
  uint4 q[9];
#pragma unroll
  for (int i = 0; i < 9; i++) q[i] = p[i];
  quads_to_p3(P, q);
}
// P += Q (both extended)
MV_DEV void p3_acc(p3& P, const p3& Q) {
  cached c;
  p1p1 t;
  p3_to_cached(c, Q);
  p3_add_cached(t, P, c);
  p1p1_to_p3(P, t);
}
MV_DEV void p3_dbl_n(p3& P, int n) {
  if (n <= 0) return;
  p2 q;
  p1p1 t;
  q.X = P.X; q.Y = P.Y; q.Z = P.Z;
  for (int i = 1; i < n; i++) {
    p2_dbl(t, q);
    p1p1_to_p2(q, t);
  }
  p2_dbl(t, q);
  p1p1_to_p3(P, t);
}

// ---------------------------------------------------------------- k_bv_prep
struct BvKey {
  uint32_t w[10];  // 32-byte secret, 64-bit call counter
};

// Committee keys (block path): A of key b is entry [0][1] = [1](-A_b) of its comb table
// (comb.hip, built by mv_set_committee with the same ZIP-215 decode), negated here.
struct CommitteeA {
  const uint4* tab;  // nullptr: decode A per signature
  const uint8_t* ok;
  uint32_t stride;   // uint4 per key table
  uint32_t aggregate;  // 1: A's term is summed per key (k_bv_keyacc / keycol / keysum), no A points
};

#ifndef MV_PREP_OCC
#define MV_PREP_OCC 3
#endif
__global__ void __launch_bounds__(256, MV_PREP_OCC)
    k_bv_prep(const uint8_t* __restrict__ msg, const uint8_t* __restrict__ sig, const uint8_t* __restrict__ pk,
              const uint32_t* __restrict__ key_idx, uint32_t n, BvKey key, CommitteeA ca, uint4* __restrict__ pts,
              uint4* __restrict__ scal, unsigned long long* __restrict__ bsum, uint8_t* __restrict__ status,
              uint32_t blk0, uint32_t group_sigs) {
  __shared__ unsigned long long sbsum[BSUM_WORDS];
  // A, s and z wait in LDS across the decodes ([word][thread]: no bank conflicts), so each
  // input byte is read from HBM once and none of them holds registers during the chains. A
  // compiler memory barrier before each read-back keeps the compiler from forwarding the
  // thread's own stores (which would keep the values live in registers after all); volatile
  // would not do: it turns the accesses into 64-bit-addressed flat ones
  __shared__ uint32_t va[8][256], vs[8][256], vz[4][256];
#ifdef MV_PREP_X2
  __shared__ uint32_t vr[8][256];  // R's encoding, parked like A's across the two chains
#endif
  const uint32_t t = threadIdx.x;
  if (threadIdx.x < BSUM_WORDS) sbsum[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t blk = blockIdx.x + blk0;  // launches may cover a chunk of the batch
  const uint32_t gid = blk * blockDim.x + threadIdx.x;
  const bool live = gid < n;
  const uint32_t idx = live ? gid : n - 1;

  uint32_t aw[8], rw[8], sw[8], mw[8];
  const uint32_t kid = key_idx ? key_idx[idx] : idx;
  load8(aw, pk + 32 * (size_t)kid);
  load8(rw, sig + 64 * (size_t)idx);
  load8(sw, sig + 64 * (size_t)idx + 32);
  load8(mw, msg + 32 * (size_t)idx);
  const bool s_ok = sc_is_canonical(sw);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    va[i][t] = aw[i];
    vs[i][t] = sw[i];
  }
  // scalars first (cheap, and their inputs die before the long decode):
  // k = SHA-512(R || A || M) mod l, z = BLAKE2b(secret || call || i) < 2^127, z k mod l
  uint32_t z[4], zk[8];
  {
    uint32_t k[8];
    {
      uint32_t kin[24], h[16];
#pragma unroll
      for (int i = 0; i < 8; i++) {
        kin[i] = rw[i];
        kin[8 + i] = aw[i];
        kin[16 + i] = mw[i];
      }
      sha512_short(h, kin, 96);
      sc_reduce512(k, h);
    }
    uint64_t m[16], h[8];
#pragma unroll
    for (int i = 0; i < 5; i++) m[i] = (uint64_t)key.w[2 * i] | ((uint64_t)key.w[2 * i + 1] << 32);
    m[5] = gid;
#pragma unroll
    for (int i = 6; i < 16; i++) m[i] = 0;
    b2_init256(h);
    b2_compress(h, m, 48, true);
    z[0] = (uint32_t)h[0];
    z[1] = (uint32_t)(h[0] >> 32);
    z[2] = (uint32_t)h[1];
    z[3] = (uint32_t)(h[1] >> 32) & 0x7fffffffu;  // z < 2^127
    uint32_t z8[8], zero[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      z8[i] = i < 4 ? z[i] : 0u;
      zero[i] = 0;
    }
    sc_muladd(zk, z8, k, zero);
  }
  uint4* sc = scal + (size_t)idx * SC_QUADS;
#pragma unroll
  for (int i = 0; i < 4; i++) vz[i][t] = z[i];
  if (live) {
    sc[0] = make_uint4(z[0], z[1], z[2], z[3]);
    sc[1] = make_uint4(zk[0], zk[1], zk[2], zk[3]);
    sc[2] = make_uint4(zk[4], zk[5], zk[6], zk[7]);
  }

  bool okA, okR;
  {
    precomp pc;
    if (ca.tab) {  // committee key: R is the only decode
      p3 P;
      decompress1_lean(P, okR, rw);
      precomp_from_affine(pc, P);
      if (live) pt_store(pts, gid, pc);
      okA = ca.ok[kid] != 0;
      if (!ca.aggregate) {
        const uint4* e = ca.tab + (size_t)kid * ca.stride + 8;  // row 0, entry 1 (8 uint4 per entry)
        uint4 q[7];
#pragma unroll
        for (int k = 0; k < 7; k++) q[k] = e[k];
        quads_to_precomp(pc, q);
        precomp_cneg(pc, true);  // -(-A) = A
        fe_canon(pc.xy2d, pc.xy2d);
        if (live) pt_store(pts, (size_t)n + gid, pc);
      }
    } else {
#ifdef MV_PREP_X2
    // (A/B) both chains interleaved: twice the ILP per lane
    p3 P, Q;
#pragma unroll
    for (int i = 0; i < 8; i++) vr[i][t] = rw[i];
    decompress2_lean(Q, okA, P, okR, [&](int which, uint32_t (&e)[8]) {
      asm volatile("" ::: "memory");  // re-read from LDS (not forwarded from registers)
#pragma unroll
      for (int i = 0; i < 8; i++) e[i] = which ? vr[i][t] : va[i][t];
    });
    precomp_from_affine(pc, P);
    if (live) pt_store(pts, gid, pc);
    precomp_from_affine(pc, Q);
    if (live) pt_store(pts, (size_t)n + gid, pc);
#else
    // one decode at a time at 3 waves/SIMD beat the two decodes in lock-step (decompress_x2)
    // at 2 waves/SIMD: 241 vs 220 M verifies/s for the whole batch path
    p3 P;
    decompress1_lean(P, okR, rw);
    precomp_from_affine(pc, P);
    if (live) pt_store(pts, gid, pc);
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < 8; i++) aw[i] = va[i][t];  // from LDS: not held across R's decode
    decompress1_lean(P, okA, aw);
    precomp_from_affine(pc, P);
    if (live) pt_store(pts, (size_t)n + gid, pc);
#endif
    }
  }
  const bool ok = live && okA && okR && s_ok;
  if (live) {
    if (!ok) {  // excluded from the combination: no bucket entries
      const uint4 zq = make_uint4(0, 0, 0, 0);
      sc[0] = zq;
      sc[1] = zq;
      sc[2] = zq;
    }
    status[gid] = !okA ? 2 : (ok ? 0 : 1);
  }
  // z and s from LDS rather than 12 registers held across the decodes
  asm volatile("" ::: "memory");
#pragma unroll
  for (int i = 0; i < 4; i++) z[i] = ok ? vz[i][t] : 0u;
#pragma unroll
  for (int i = 0; i < 8; i++) sw[i] = vs[i][t];
  // z * s (12 words, not reduced), summed per workgroup
  {
    uint64_t acc = 0;
    uint32_t c2 = 0;
#pragma unroll
    for (int c = 0; c < 11; c++) {
#pragma unroll
      for (int i = 0; i < 4; i++)
        if (c - i >= 0 && c - i < 8) mac(acc, c2, z[i], sw[c - i]);
      atomicAdd(&sbsum[c], (unsigned long long)(uint32_t)acc);
      acc = (acc >> 32) | ((uint64_t)c2 << 32);
      c2 = 0;
    }
    atomicAdd(&sbsum[11], (unsigned long long)(uint32_t)acc);
  }
  __syncthreads();
  // the workgroup's column sums into its group's (zeroed before the first prep launch); the
  // final check then reads 12 words per group instead of reducing a per-workgroup array
  if (threadIdx.x < BSUM_WORDS)
    atomicAdd(&bsum[(size_t)(blk * 256u / group_sigs) * BSUM_WORDS + threadIdx.x], sbsum[threadIdx.x]);
}

// ---------------------------------------------------------------- bucket sort
// Two-pass counting sort of the (bucket key, point) entries without global atomics:
//   k_part_count               chunk = 1024 signatures: entries per partition (LDS)
//   k_part_scan / k_part_top   exclusive offsets of every (chunk, partition) run
//   k_part_scatter             per chunk: entries (key, point) into their
//                              partition, runs ordered by chunk, ranks from LDS atomics
//   k_fine_sort                workgroup per partition: counting sort by the low 8 key
//                              bits in LDS -> final bucket lists and bucket offsets
// Sub-batches (groups): the batch's chunks are cut into `count` contiguous groups of `cpg`
// chunks, and every group has its own buckets (key = g * BV_NKG + local key), so the
// pipeline checks one combined equation per group. A chunk lies inside one group, so the
// per-chunk counts stay group-local (BV_NPG partitions per chunk).
template <int NT = 256>
MV_DEV uint32_t block_excl_scan256(uint32_t v, uint32_t* sm, uint32_t& total) {
  const int t = threadIdx.x;
  sm[t] = v;
  __syncthreads();
  for (int o = 1; o < NT; o <<= 1) {
    uint32_t x = t >= o ? sm[t - o] : 0u;
    __syncthreads();
    sm[t] += x;
    __syncthreads();
  }
  total = sm[NT - 1];
  const uint32_t incl = sm[t];
  __syncthreads();
  return incl - v;
}

constexpr int PART_CHUNK = 1024;  // signatures per k_part_count / k_part_scatter block

struct BvGroups {
  uint32_t count;  // groups (sub-batch equations)
  uint32_t cpg;    // chunks per group: signature i is in group i / (cpg * PART_CHUNK)
};

MV_DEV void load_scalars(uint32_t z[4], uint32_t zk[8], const uint4* scal, uint32_t i) {
  const uint4* sc = scal + (size_t)i * SC_QUADS;
  const uint4 q0 = sc[0], q1 = sc[1], q2 = sc[2];
  z[0] = q0.x; z[1] = q0.y; z[2] = q0.z; z[3] = q0.w;
  zk[0] = q1.x; zk[1] = q1.y; zk[2] = q1.z; zk[3] = q1.w;
  zk[4] = q2.x; zk[5] = q2.y; zk[6] = q2.z; zk[7] = q2.w;
}
// chunk c = 1024 signatures: entries per (group-local) partition -> pcount[c][p]
// skipA: the A scalars are summed per committee key instead (no A bucket entries)
__global__ void __launch_bounds__(PART_CHUNK) k_part_count(const uint4* __restrict__ scal, uint32_t n, uint32_t skipA,
                                                           uint32_t* __restrict__ pcount) {
  __shared__ uint32_t hist[BV_NPG];
  for (int i = threadIdx.x; i < BV_NPG; i += PART_CHUNK) hist[i] = 0;
  __syncthreads();
  const uint32_t gid = blockIdx.x * PART_CHUNK + threadIdx.x;
  if (gid < n) {
    uint32_t z[4], zk[8];
    load_scalars(z, zk, scal, gid);
    if (skipA) {
#pragma unroll
      for (int i = 0; i < 8; i++) zk[i] = 0;
    }
    bv_for_digits(z, zk, [&](int w, int d, int) { atomicAdd(&hist[bv_key(w, d) >> BV_FINE_BITS], 1u); });
  }
  __syncthreads();
  for (int i = threadIdx.x; i < BV_NPG; i += PART_CHUNK) pcount[(size_t)blockIdx.x * BV_NPG + i] = hist[i];
}
// block b: group b / 32, its partitions [64 (b % 32), + 64), SCAN_SUB chunk subgroups of the
// group's chunks (one group of 1,024 chunks: 64 chunks per thread, not 256); row reads are
// 256-B coalesced. poff[c][p] = entries of partition (g, p) in the group's chunks before c;
// ptot[g * BV_NPG + p] = partition size.
constexpr int SCAN_SUB = 16;
__global__ void __launch_bounds__(64 * SCAN_SUB) k_part_scan(const uint32_t* __restrict__ pcount, uint32_t nchunk,
                                                             BvGroups G, uint32_t* __restrict__ poff,
                                                             uint32_t* __restrict__ ptot) {
  __shared__ uint32_t gsum[SCAN_SUB][64];
  constexpr uint32_t BPG = BV_NPG / 64;
  const uint32_t pl = threadIdx.x & 63, q = threadIdx.x >> 6;
  const uint32_t g = blockIdx.x / BPG;
  const uint32_t p = (blockIdx.x % BPG) * 64 + pl;
  const uint32_t cg0 = g * G.cpg, cg1 = min(nchunk, cg0 + G.cpg);
  const uint32_t per = (cg1 - cg0 + SCAN_SUB - 1) / SCAN_SUB;
  const uint32_t c0 = min(cg1, cg0 + q * per), c1 = min(cg1, c0 + per);
  uint32_t sum = 0;
  for (uint32_t c = c0; c < c1; c++) sum += pcount[(size_t)c * BV_NPG + p];
  gsum[q][pl] = sum;
  __syncthreads();
  uint32_t run = 0;
  for (uint32_t k = 0; k < q; k++) run += gsum[k][pl];
  for (uint32_t c = c0; c < c1; c++) {
    const uint32_t v = pcount[(size_t)c * BV_NPG + p];
    poff[(size_t)c * BV_NPG + p] = run;
    run += v;
  }
  if (q == SCAN_SUB - 1) ptot[g * BV_NPG + p] = run;
}
// exclusive scan of the partition totals (all groups) -> pstart[0..total]
__global__ void __launch_bounds__(256) k_part_top(const uint32_t* __restrict__ ptot, uint32_t total,
                                                  uint32_t* __restrict__ pstart) {
  __shared__ uint32_t sm[256];
  const uint32_t per = total / 256;  // total is a multiple of BV_NPG
  const uint32_t* src = ptot + (size_t)per * threadIdx.x;
  uint32_t sum = 0;
  for (uint32_t i = 0; i < per; i++) sum += src[i];
  uint32_t all;
  uint32_t run = block_excl_scan256(sum, sm, all);
  for (uint32_t i = 0; i < per; i++) {
    const uint32_t v = src[i];
    pstart[(size_t)per * threadIdx.x + i] = run;
    run += v;
  }
  if (threadIdx.x == 0) pstart[total] = all;
}
// (scal, n: the signatures [base, base + n) of a batch of nall; point refs are batch-wide)
__global__ void __launch_bounds__(PART_CHUNK) k_part_scatter(const uint4* __restrict__ scal, uint32_t n,
                                                             const uint32_t* __restrict__ poff,
                                                             const uint32_t* __restrict__ pstart, BvGroups G,
                                                             uint32_t skipA, uint32_t nall, uint32_t base,
                                                             unsigned long long* __restrict__ tmp) {
  __shared__ uint32_t rank[BV_NPG];
  for (int i = threadIdx.x; i < BV_NPG; i += PART_CHUNK) rank[i] = 0;
  __syncthreads();
  const uint32_t gid = blockIdx.x * PART_CHUNK + threadIdx.x;
  if (gid < n) {
    const uint32_t g = blockIdx.x / G.cpg;
    uint32_t z[4], zk[8];
    load_scalars(z, zk, scal, gid);
    if (skipA) {
#pragma unroll
      for (int i = 0; i < 8; i++) zk[i] = 0;
    }
    const uint32_t* po = poff + (size_t)blockIdx.x * BV_NPG;
    const uint32_t* ps = pstart + (size_t)g * BV_NPG;
    bv_for_digits(z, zk, [&](int w, int d, int isA) {
      const uint32_t key = bv_key(w, d);
      const uint32_t p = key >> BV_FINE_BITS;
      const uint32_t r = atomicAdd(&rank[p], 1u);
      const uint32_t pt = isA ? nall + base + gid : base + gid;
      tmp[ps[p] + po[p] + r] = ((unsigned long long)(g * BV_NKG + key) << 32) | (pt << 1) | (d < 0 ? 1u : 0u);
    });
  }
}
// The same scatter with coalesced stores (MV_SCATTER_LDS): window by window, the block's entries
// are first placed in LDS in partition order (the chunk's per-partition counts from
// k_part_count, scanned), then thread i stores LDS entry i, so consecutive threads write
// consecutive words of a partition's run instead of one scattered 8-byte word per entry (the
// direct form wrote 2.7x the entry bytes, profiles/r05/pmc/pmc_c2_k_part_scatter.txt). Entry
// order inside a run changes, which no later stage depends on (the fine sort orders by key,
// and a bucket's sum does not depend on the order of its points).
constexpr uint32_t BV_PPW_ = BV_NB >> BV_FINE_BITS;  // partitions per window (128)
__global__ void __launch_bounds__(PART_CHUNK) k_part_scatter_lds(const uint4* __restrict__ scal, uint32_t n,
                                                                 const uint32_t* __restrict__ pcount,
                                                                 const uint32_t* __restrict__ poff,
                                                                 const uint32_t* __restrict__ pstart, BvGroups G,
                                                                 uint32_t skipA, uint32_t nall, uint32_t base,
                                                                 unsigned long long* __restrict__ tmp) {
  __shared__ unsigned long long buf[2 * PART_CHUNK];  // one window's entries (<= 2 per signature)
  __shared__ uint32_t lofs[BV_PPW_ + 1], gpos[BV_PPW_], rank[BV_PPW_];
  const uint32_t gid = blockIdx.x * PART_CHUNK + threadIdx.x;
  const bool live = gid < n;
  const uint32_t g = blockIdx.x / G.cpg;
  // the signature's digits, all windows (bv_for_digits' carries), kept in registers
  int dR[8], dA[16];
#pragma unroll
  for (int w = 0; w < 8; w++) dR[w] = 0;
#pragma unroll
  for (int w = 0; w < 16; w++) dA[w] = 0;
  if (live) {
    uint32_t z[4], zk[8];
    load_scalars(z, zk, scal, gid);
    if (skipA) {
#pragma unroll
      for (int i = 0; i < 8; i++) zk[i] = 0;
    }
    bv_for_digits(z, zk, [&](int w, int d, int isA) {
      if (isA) dA[w] = d; else dR[w < 8 ? w : 0] = d;
    });
  }
  const uint32_t* pc = pcount + (size_t)blockIdx.x * BV_NPG;
  const uint32_t* po = poff + (size_t)blockIdx.x * BV_NPG;
  const uint32_t* ps = pstart + (size_t)g * BV_NPG;
  const uint32_t ptR = base + gid, ptA = nall + base + gid;
#pragma unroll 1
  for (int w = 0; w < BV_NW; w++) {
    // this window's partitions: chunk-local offsets (wave 0 scans 128 counts), global run starts
    if (threadIdx.x < 64) {
      const uint32_t l = threadIdx.x, p0 = (uint32_t)w * BV_PPW_ + 2 * l;
      const uint32_t c0 = pc[p0], c1 = pc[p0 + 1];
      uint32_t incl = c0 + c1;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t x = (uint32_t)__shfl_up((int)incl, o);
        if (l >= (uint32_t)o) incl += x;
      }
      const uint32_t ex = incl - c0 - c1;
      lofs[2 * l] = ex;
      lofs[2 * l + 1] = ex + c0;
      if (l == 63) lofs[BV_PPW_] = incl;
      gpos[2 * l] = ps[p0] + po[p0];
      gpos[2 * l + 1] = ps[p0 + 1] + po[p0 + 1];
      rank[2 * l] = 0;
      rank[2 * l + 1] = 0;
    }
    __syncthreads();
    auto place = [&](int d, uint32_t pt) {
      const uint32_t key = bv_key(w, d), pl = (key >> BV_FINE_BITS) & (BV_PPW_ - 1);
      const uint32_t r = atomicAdd(&rank[pl], 1u);
      buf[lofs[pl] + r] = ((unsigned long long)(g * BV_NKG + key) << 32) | (pt << 1) | (d < 0 ? 1u : 0u);
    };
    if (w < 8 && dR[w]) place(dR[w], ptR);
    if (dA[w]) place(dA[w], ptA);
    __syncthreads();
    const uint32_t tot = lofs[BV_PPW_];
    for (uint32_t i = threadIdx.x; i < tot; i += PART_CHUNK) {
      const unsigned long long e = buf[i];
      const uint32_t pl = ((uint32_t)(e >> 32) >> BV_FINE_BITS) & (BV_PPW_ - 1);
      tmp[gpos[pl] + (i - lofs[pl])] = e;
    }
    __syncthreads();
  }
}

// block -> partition P: the partition's entries sorted by bucket into ents; offs[key] for
// its 256 keys. FINE_NT threads over 256 bins (a partition holds ~8K entries, window 15's
// ~32K: digits stop at 2^13), so the ranked stores of the blocks in flight merge in L2. The
// biggest partitions (window 15's) of every group are scheduled first.
constexpr uint32_t BV_PPW = BV_NB >> BV_FINE_BITS;  // partitions per window (128)
constexpr int FINE_NT = 1024;
__global__ void __launch_bounds__(FINE_NT) k_fine_sort(const unsigned long long* __restrict__ tmp,
                                                       const uint32_t* __restrict__ pstart, uint32_t ngroups,
                                                       uint32_t* __restrict__ ents, uint32_t* __restrict__ offs) {
  constexpr int NF = 1 << BV_FINE_BITS;
  __shared__ uint32_t cnt[NF];
  const uint32_t span = ngroups * BV_PPW;
  const uint32_t w = BV_NW - 1 - blockIdx.x / span;
  const uint32_t g = (blockIdx.x % span) / BV_PPW;
  const uint32_t p = g * BV_NPG + w * BV_PPW + blockIdx.x % BV_PPW;
  const uint32_t s = pstart[p], e = pstart[p + 1];
  if (threadIdx.x < NF) cnt[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t i = s + threadIdx.x; i < e; i += FINE_NT) atomicAdd(&cnt[(uint32_t)(tmp[i] >> 32) & (NF - 1)], 1u);
  __syncthreads();
  static_assert(NF == 256, "wave 0 scans four bins per lane");
  if (threadIdx.x < 64) {  // wave 0 alone (no barrier inside): exclusive scan of the bins
    const uint32_t l = threadIdx.x;
    uint32_t c[4], sum = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      c[k] = cnt[4 * l + k];
      sum += c[k];
    }
    uint32_t incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t x = (uint32_t)__shfl_up((int)incl, o);
      if (l >= (uint32_t)o) incl += x;
    }
    uint32_t ex = incl - sum;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      offs[(size_t)p * NF + 4 * l + k] = s + ex;
      cnt[4 * l + k] = ex;
      ex += c[k];
    }
    if (p == ngroups * BV_NPG - 1 && l == 0) offs[(size_t)ngroups * BV_NKG] = e;
  }
  __syncthreads();
  for (uint32_t i = s + threadIdx.x; i < e; i += FINE_NT) {
    const unsigned long long v = tmp[i];
    const uint32_t r = atomicAdd(&cnt[(uint32_t)(v >> 32) & (NF - 1)], 1u);
    ents[s + r] = (uint32_t)v;
  }
}

// The same sort with its output staged in LDS (MV_FINE_LDS): a partition of <= FINE_LDS entries
// is read once into registers (16 per thread) and counted; the count's atomic returns each
// entry's rank in its bin, so after the scan an entry's place is its bin's start + its rank (one
// LDS atomic per entry instead of round 5's two); the entries are placed in LDS in bucket order
// and stored coalesced; the direct form read each entry twice and stored one scattered word per
// entry. Larger partitions (window 15's at 2^20 signatures: ~32K) take the direct form.
// Bank conflicts stay ~65% of the LDS cycles either way (profiles/r06/pmc_c2s1_k_fine_sort_lds_*):
// 64 lanes' random bins (and random ranks for the placement) land on 64 banks at random, about
// four to a bank; the kernel is 0.16 ms of the 3.2-ms step.
constexpr uint32_t FINE_LDS = 16384;
constexpr int FINE_FPT = FINE_LDS / FINE_NT;
__global__ void __launch_bounds__(FINE_NT) k_fine_sort_lds(const unsigned long long* __restrict__ tmp,
                                                           const uint32_t* __restrict__ pstart, uint32_t ngroups,
                                                           uint32_t* __restrict__ ents, uint32_t* __restrict__ offs) {
  constexpr int NF = 1 << BV_FINE_BITS;
  __shared__ uint32_t cnt[NF];
  __shared__ uint32_t obuf[FINE_LDS];
  const uint32_t span = ngroups * BV_PPW;
  const uint32_t w = BV_NW - 1 - blockIdx.x / span;
  const uint32_t g = (blockIdx.x % span) / BV_PPW;
  const uint32_t p = g * BV_NPG + w * BV_PPW + blockIdx.x % BV_PPW;
  const uint32_t s = pstart[p], e = pstart[p + 1], m = e - s;
  const bool staged = m <= FINE_LDS;  // (uniform in the block)
  if (threadIdx.x < NF) cnt[threadIdx.x] = 0;
  __syncthreads();
  uint32_t ent[FINE_FPT], br[FINE_FPT];  // entry; bin << 16 | its rank in the bin
  static_assert(FINE_LDS <= (1u << 16), "ranks fit 16 bits");
  if (staged) {
#pragma unroll
    for (int k = 0; k < FINE_FPT; k++) {
      const uint32_t i = threadIdx.x + (uint32_t)k * FINE_NT;
      const unsigned long long v = i < m ? tmp[s + i] : 0ull;
      ent[k] = (uint32_t)v;
      br[k] = ((uint32_t)(v >> 32) & (NF - 1)) << 16;
    }
#pragma unroll
    for (int k = 0; k < FINE_FPT; k++)
      if (threadIdx.x + (uint32_t)k * FINE_NT < m) br[k] |= atomicAdd(&cnt[br[k] >> 16], 1u);
  } else {
    for (uint32_t i = s + threadIdx.x; i < e; i += FINE_NT) atomicAdd(&cnt[(uint32_t)(tmp[i] >> 32) & (NF - 1)], 1u);
  }
  __syncthreads();
  static_assert(NF == 256, "wave 0 scans four bins per lane");
  if (threadIdx.x < 64) {  // wave 0 alone (no barrier inside): exclusive scan of the bins
    const uint32_t l = threadIdx.x;
    uint32_t c[4], sum = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      c[k] = cnt[4 * l + k];
      sum += c[k];
    }
    uint32_t incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t x = (uint32_t)__shfl_up((int)incl, o);
      if (l >= (uint32_t)o) incl += x;
    }
    uint32_t ex = incl - sum;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      offs[(size_t)p * NF + 4 * l + k] = s + ex;
      cnt[4 * l + k] = ex;
      ex += c[k];
    }
    if (p == ngroups * BV_NPG - 1 && l == 0) offs[(size_t)ngroups * BV_NKG] = e;
  }
  __syncthreads();
  if (staged) {
#pragma unroll
    for (int k = 0; k < FINE_FPT; k++)
      if (threadIdx.x + (uint32_t)k * FINE_NT < m) obuf[cnt[br[k] >> 16] + (br[k] & 0xffffu)] = ent[k];
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < m; i += FINE_NT) ents[s + i] = obuf[i];
  } else {
    for (uint32_t i = s + threadIdx.x; i < e; i += FINE_NT) {
      const unsigned long long x = tmp[i];
      const uint32_t r = atomicAdd(&cnt[(uint32_t)(x >> 32) & (NF - 1)], 1u);
      ents[s + r] = (uint32_t)x;
    }
  }
}

// ---------------------------------------------------------------- buckets
// Lane = segment of `seg` consecutive buckets (g, w, j*seg .. j*seg + seg - 1), consumed from
// the top bucket down: T = running sum of the segment's buckets, V = sum of T after every
// bucket = sum_b (b + 1) B_{j*seg + b}. The segment then stands for V + (j * seg) T in the
// window's sum (k_bv_reduce). seg = 1: T only (V = T). Windows are laid out high-first in the
// grid (window 15's buckets hold four times the entries), every group's windows side by side,
// and each point is loaded one add ahead.
// 3 workgroups per CU (168 VGPRs, 16 spilled) beat 2 (175 VGPRs, no spill): the gathers
// need the third wave per SIMD (config 2: bucket 1.71 -> 1.44-1.50 ms as run, +0.8% step rate)
#ifndef MV_BUCKET_OCC
#define MV_BUCKET_OCC 3
#endif
#ifndef MV_BUCKET_PF2
#define MV_BUCKET_PF2 1  // k_bv_bucket_bal: unconditional point prefetch (0: the old branch, A/B)
#endif
__global__ void __launch_bounds__(256, MV_BUCKET_OCC) k_bv_bucket(const uint4* __restrict__ pts, const uint32_t* __restrict__ offs,
                                                   const uint32_t* __restrict__ ents, uint32_t ngroups, uint32_t seg,
                                                   uint32_t nw, uint4* __restrict__ segV, uint4* __restrict__ segT) {
  const uint32_t nsw = BV_NB / seg;  // segments per (group, window) row
  const uint32_t lin = blockIdx.x * blockDim.x + threadIdx.x;
  if (lin >= ngroups * nw * nsw) return;  // windows nw.. carry no entries (per-key A term)
  const uint32_t span = ngroups * nsw;
  const uint32_t w = nw - 1 - lin / span;
  const uint32_t g = (lin % span) / nsw, j = lin % nsw;
  const uint32_t sidx = (g * BV_NW + w) * nsw + j;  // segment index, row-major
  const uint32_t key0 = g * BV_NKG + w * BV_NB + j * seg;
  // the running sum V waits in LDS ([word][thread]: conflict-free) while the bucket's points
  // are added into T, so it holds no registers across the inner loop (no spill at 3 WG/CU)
  __shared__ uint32_t sV[36][256];
  const uint32_t tid = threadIdx.x;
  auto v_load = [&](p3& V) {
#pragma unroll
    for (int i = 0; i < 9; i++) {
      V.X.v[i] = sV[i][tid];
      V.Y.v[i] = sV[9 + i][tid];
      V.Z.v[i] = sV[18 + i][tid];
      V.T.v[i] = sV[27 + i][tid];
    }
  };
  auto v_store = [&](const p3& V) {
#pragma unroll
    for (int i = 0; i < 9; i++) {
      sV[i][tid] = V.X.v[i];
      sV[9 + i][tid] = V.Y.v[i];
      sV[18 + i][tid] = V.Z.v[i];
      sV[27 + i][tid] = V.T.v[i];
    }
  };
  p3 T;
  p3_identity(T);
  if (seg > 1) v_store(T);  // V = identity
  const uint32_t e_lo = offs[key0];
  uint32_t e = offs[key0 + seg];
  uint4 q[7];
  uint32_t ent = 0;
  if (e > e_lo) {
    e--;
    ent = ents[e];
    const uint4* p = pts + (size_t)(ent >> 1) * PT_QUADS;
#pragma unroll
    for (int i = 0; i < 7; i++) q[i] = p[i];
  }
  uint32_t b1 = offs[key0 + seg];
  for (int b = (int)seg - 1; b >= 0; b--) {
    const uint32_t b0 = offs[key0 + b];
    for (uint32_t k = b1; k > b0; k--) {
      precomp pc;
      quads_to_precomp(pc, q);
      const bool neg = ent & 1u;
      if (e > e_lo) {  // next point in flight during this add
        e--;
        ent = ents[e];
        const uint4* p = pts + (size_t)(ent >> 1) * PT_QUADS;
#pragma unroll
        for (int i = 0; i < 7; i++) q[i] = p[i];
      }
      precomp_cneg(pc, neg);
      p1p1 t;
      p3_add_precomp(t, T, pc);
      p1p1_to_p3(T, t);
    }
    b1 = b0;
    if (seg > 1) {
      p3 V;
      v_load(V);
      p3_acc(V, T);
      v_store(V);
    }
  }
  if (seg > 1) {
    p3 V;
    v_load(V);
    p3_store(segV, sidx, V);
  }
  p3_store(segT, sidx, T);
}

// Balanced buckets (seg = 1, MV_BUCKET_BAL): one lane per bucket leaves a wave as slow as its
// fullest bucket — bucket sizes are Poisson (mean 32-128 by window), and the wave's max of 64
// kept lanes busy ~75% of the time (SQ_THREAD_CYCLES_VALU / (64 x SQ_INSTS_VALU),
// profiles/r05/pmc/pmc_c2_k_bv_bucket.txt). Here every lane adds the same number L of entries:
// lane j takes entries [j L, (j + 1) L) of the whole key-sorted list (all groups and windows:
// ents is sorted by key = g * BV_NKG + w * BV_NB + |d| - 1). A bucket that starts in the lane's
// range is written to segT by it (complete, or its first piece); the piece of a bucket that
// began before the range goes to carry[j], which k_bv_bucket_fix adds to segT. Empty buckets
// are written (identity) by k_bv_bucket_fix too.
// offs_key(x): the largest key k in [k0, nk) with offs[k] <= x (offs nondecreasing, offs[k0] <= x)
MV_DEV uint32_t bv_key_of(const uint32_t* __restrict__ offs, uint32_t k0, uint32_t nk, uint32_t x) {
  uint32_t lo = k0, hi = nk;  // offs[lo] <= x, answer in [lo, hi)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (offs[mid] <= x) lo = mid; else hi = mid;
  }
  return lo;
}

__global__ void __launch_bounds__(256, MV_BUCKET_OCC) k_bv_bucket_bal(const uint4* __restrict__ pts,
                                                                     const uint32_t* __restrict__ offs,
                                                                     const uint32_t* __restrict__ ents, uint32_t nk,
                                                                     uint32_t nlanes, uint4* __restrict__ carry,
                                                                     uint4* __restrict__ segT) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nlanes) return;
  const uint32_t e0 = offs[0], e1 = offs[nk];
  const uint32_t L = (e1 - e0 + nlanes - 1) / nlanes;
  const uint32_t lo = min(e0 + j * L, e1), hi = min(lo + L, e1);
  if (lo >= hi) return;
  uint32_t b = bv_key_of(offs, 0, nk, lo);  // the bucket holding entry lo (non-empty)
  uint32_t nb = offs[b + 1];                // its end
  bool head = offs[b] < lo;                 // began before this lane: the piece is a carry
  // a piece: the carry, or the bucket's sum
  auto emit = [&](uint32_t key, const p3& P) {
    if (head)
      p3_store(carry, j, P);
    else
      p3_store(segT, key, P);
  };
  p3 T;
  p3_identity(T);
  uint4 q[7];
  uint32_t ent = ents[lo];
#if MV_BUCKET_PF2
  uint32_t ent_n = ents[min(lo + 1, hi - 1)];  // the entry after the one in flight
#endif
  {
    const uint4* p = pts + (size_t)(ent >> 1) * PT_QUADS;
#pragma unroll
    for (int i = 0; i < 7; i++) q[i] = p[i];
  }
  for (uint32_t x = lo; x < hi; x++) {
    precomp pc;
    quads_to_precomp(pc, q);
    const bool neg = ent & 1u;
#if MV_BUCKET_PF2
    // next point in flight during this add, loaded unconditionally (the last lap reloads entry
    // hi - 1): a load under a branch made the compiler copy the quads into the loop's registers
    // inside the branch, waiting on the loads at once; and the entry index one lap further ahead
    ent = ent_n;
    ent_n = ents[min(x + 2, hi - 1)];
    {
      const uint4* p = pts + (size_t)(ent >> 1) * PT_QUADS;
#pragma unroll
      for (int i = 0; i < 7; i++) q[i] = p[i];
    }
#else
    if (x + 1 < hi) {  // next point in flight during this add
      ent = ents[x + 1];
      const uint4* p = pts + (size_t)(ent >> 1) * PT_QUADS;
#pragma unroll
      for (int i = 0; i < 7; i++) q[i] = p[i];
    }
#endif
    precomp_cneg(pc, neg);
    p1p1 t;
    p3_add_precomp(t, T, pc);
    p1p1_to_p3(T, t);
    if (x + 1 == nb) {  // bucket b complete (in this lane)
      emit(b, T);
      head = false;
      p3_identity(T);
      if (x + 1 < hi) {  // the next non-empty bucket: usually b + 1, else search (empty runs)
        const uint32_t n2 = offs[b + 2];
        if (n2 > nb) { b++; nb = n2; }
        else { b = bv_key_of(offs, b + 1, nk, x + 1); nb = offs[b + 1]; }
      }
    }
  }
  if (hi != nb) emit(b, T);  // the range ends inside bucket b
}

// One lane per bucket key (g, w < nw, |d| - 1): empty -> identity; a bucket whose entries run
// past the lane that began it gets the carries of the lanes it continues into.
__global__ void __launch_bounds__(256) k_bv_bucket_fix(const uint32_t* __restrict__ offs, uint32_t nk,
                                                       uint32_t ngroups, uint32_t nw, uint32_t nlanes,
                                                       const uint4* __restrict__ carry, uint4* __restrict__ segT) {
  const uint32_t lin = blockIdx.x * blockDim.x + threadIdx.x;
  if (lin >= ngroups * nw * BV_NB) return;
  const uint32_t g = lin / (nw * BV_NB), r = lin % (nw * BV_NB);
  const uint32_t key = g * BV_NKG + r;  // (w, |d| - 1) = (r / NB, r % NB), w < nw
  const uint32_t e0 = offs[0], e1 = offs[nk];
  const uint32_t L = (e1 - e0 + nlanes - 1) / nlanes;
  const uint32_t lo = offs[key], hi = offs[key + 1];
  if (lo == hi) {
    p3 I;
    p3_identity(I);
    p3_store(segT, key, I);
    return;
  }
  const uint32_t j0 = (lo - e0) / L, j1 = (hi - 1 - e0) / L;
  if (j1 == j0) return;
  p3 T;
  p3_load(T, segT, key);
  for (uint32_t j = j0 + 1; j <= j1; j++) {
    p3 C;
    p3_load(C, carry, j);
    p3_acc(T, C);
  }
  p3_store(segT, key, T);
}

// ---------------------------------------------------------------- reduction
#ifndef MV_REDUCE_PF
#define MV_REDUCE_PF 1  // inputs loaded one step ahead (0: the old load-then-use order, A/B)
#endif
// Rows = (group, window); row r holds cnt_in elements. Elements (V, T) with indices
// m = 0..cnt-1 stand for V + (m * scale) T. Groups of FAN consecutive elements m = FAN*q + t
// become one element with index q:
//   V' = sum V_t + scale * sum_t t T_t,   T' = sum T_t,   scale' = FAN * scale.
// scale is a power of two (log2 = shift): the multiplication is `shift` doublings.
// First level with one bucket per segment (inV == nullptr): the elements are the buckets,
// m = |d| - 1, so V_m = T_m and scale = 1: V' = sum_t (t + 1) T_t, the sum of the running sums.
// Output rows are compact, r = g * nw + w; the first level (from_keys) reads the bucket
// kernel's key-space layout, row (g, w) at (g * BV_NW + w) * cnt_in.
__global__ void __launch_bounds__(64) k_bv_reduce(const uint4* __restrict__ inV, const uint4* __restrict__ inT,
                                                  uint32_t cnt_in, int fan, int shift, uint32_t rows, uint32_t nw,
                                                  uint32_t from_keys, uint4* __restrict__ outV,
                                                  uint4* __restrict__ outT) {
  const uint32_t cnt_out = (cnt_in + fan - 1) / fan;
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= cnt_out * rows) return;
  const uint32_t r = gid / cnt_out, q = gid % cnt_out;
  const uint32_t rin = from_keys ? (r / nw) * BV_NW + r % nw : r;
  const size_t base = (size_t)rin * cnt_in + (size_t)q * fan;
  const int m = (int)min((uint32_t)fan, cnt_in - q * fan);
  p3 U, Sx, X;
  p3_identity(U);
  p3_identity(Sx);
  // each step's point(s) loaded one step ahead (the lane is a lone latency chain)
  if (!inV) {
#if MV_REDUCE_PF == 0
    for (int t = m - 1; t >= 0; t--) {
      p3_load(X, inT, base + t);
      p3_acc(U, X);
      p3_acc(Sx, U);
    }
    p3_store(outV, gid, Sx);
    p3_store(outT, gid, U);
    return;
#endif
    p3_load(X, inT, base + m - 1);
    for (int t = m - 1; t >= 0; t--) {
      const p3 Xc = X;
      if (t > 0) p3_load(X, inT, base + t - 1);
      p3_acc(U, Xc);
      p3_acc(Sx, U);
    }
    p3_store(outV, gid, Sx);
    p3_store(outT, gid, U);
    return;
  }
  p3 Vs, Y;
  p3_identity(Vs);
#if MV_REDUCE_PF == 0
  for (int t = m - 1; t >= 0; t--) {
    p3_load(X, inT, base + t);
    p3_acc(U, X);
    if (t > 0) p3_acc(Sx, U);
    p3_load(Y, inV, base + t);
    p3_acc(Vs, Y);
  }
  p3_dbl_n(Sx, shift);
  p3_acc(Vs, Sx);
  p3_store(outV, gid, Vs);
  p3_store(outT, gid, U);
  return;
#endif
  p3_load(X, inT, base + m - 1);
  p3_load(Y, inV, base + m - 1);
  for (int t = m - 1; t >= 0; t--) {
    const p3 Xc = X, Yc = Y;
    if (t > 0) {
      p3_load(X, inT, base + t - 1);
      p3_load(Y, inV, base + t - 1);
    }
    p3_acc(U, Xc);
    if (t > 0) p3_acc(Sx, U);  // sum_{t>=1} sum_{t'>=t} T_t' = sum t' T_t'
    p3_acc(Vs, Yc);
  }
  p3_dbl_n(Sx, shift);
  p3_acc(Vs, Sx);
  p3_store(outV, gid, Vs);
  p3_store(outT, gid, U);
}

// ---------------------------------------------------------------- per-key A term
// Committee keys (the block path): every signature of key b has A = A_b, so
//     sum_i [z_i k_i] A_i = sum_b [c_b] A_b,   c_b = sum_{i: key i = b} z_i k_i mod l,
// one fixed-base multiplication per (group, key) on the key's comb table (32 mixed
// additions) instead of 16 bucket entries per signature.
constexpr int BV_MAXKEYS = 512;  // committee size bound (types.rs:118-121)

// chunk c = 1024 signatures: column sums of z k per key -> kpart[c][key][8] (u64 words,
// each < 2^42). Excluded signatures have z k = 0 (k_bv_prep).
__global__ void __launch_bounds__(PART_CHUNK) k_bv_keyacc(const uint4* __restrict__ scal,
                                                          const uint32_t* __restrict__ key_idx, uint32_t n,
                                                          uint32_t nkeys, unsigned long long* __restrict__ kpart) {
  __shared__ unsigned long long ks[BV_MAXKEYS * 8];
  for (uint32_t i = threadIdx.x; i < nkeys * 8; i += PART_CHUNK) ks[i] = 0;
  __syncthreads();
  const uint32_t gid = blockIdx.x * PART_CHUNK + threadIdx.x;
  if (gid < n) {
    const uint4* sc = scal + (size_t)gid * SC_QUADS;
    const uint4 q1 = sc[1], q2 = sc[2];
    const uint32_t w[8] = {q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
    const uint32_t key = key_idx[gid];
    if (key < nkeys && (w[0] | w[1] | w[2] | w[3] | w[4] | w[5] | w[6] | w[7])) {
#pragma unroll
      for (int k = 0; k < 8; k++) atomicAdd(&ks[key * 8 + k], (unsigned long long)w[k]);
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nkeys * 8; i += PART_CHUNK) kpart[(size_t)blockIdx.x * nkeys * 8 + i] = ks[i];
}

// The per-key term in two launches, wide enough that neither is a latency chain on a few
// lanes (round 3's one-workgroup-per-group form walked every chunk of every key on one lane:
// 0.44 ms per 2^20 config-4 blocks):
//   k_bv_keycol  workgroup (g, b): c_b = sum over the group's chunks of kpart (256 lanes, then
//                an LDS tree), reduced mod l and recoded; then lane r < 32 adds table row r's
//                entry of c_b's digit r to the identity and a 5-level tree sums the 32 rows:
//                keyp[g][b] = [c_b](-A_b)
//   k_bv_keysum  workgroup g: the group's keys' points by a tree -> asum[g] = +sum_b [c_b] A_b
__global__ void __launch_bounds__(256) k_bv_keycol(const unsigned long long* __restrict__ kpart, uint32_t nchunk,
                                                   uint32_t cpg, uint32_t nkeys, const uint4* __restrict__ combA,
                                                   uint4* __restrict__ keyp) {
  __shared__ unsigned long long cs[8][256];
  __shared__ uint32_t sd_s[8];
  __shared__ uint4 red[P3_QUADS][CT_ROWS];
  const uint32_t g = blockIdx.x / nkeys, b = blockIdx.x % nkeys, t = threadIdx.x;
  const uint32_t c0 = g * cpg, c1 = min(nchunk, c0 + cpg);
  unsigned long long col[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t c = c0 + t; c < c1; c += blockDim.x) {
    const unsigned long long* p = kpart + ((size_t)c * nkeys + b) * 8;
#pragma unroll
    for (int k = 0; k < 8; k++) col[k] += p[k];
  }
#pragma unroll
  for (int k = 0; k < 8; k++) cs[k][t] = col[k];
  __syncthreads();
  for (uint32_t h = blockDim.x / 2; h > 0; h >>= 1) {
    if (t < h) {
#pragma unroll
      for (int k = 0; k < 8; k++) cs[k][t] += cs[k][t + h];
    }
    __syncthreads();
  }
  if (t == 0) {
    uint32_t x[16], r[8], sd[8];
    unsigned long long carry = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const unsigned long long v = cs[k][0] + carry;  // column sums < 2^62: no overflow
      x[k] = (uint32_t)v;
      carry = v >> 32;
    }
    x[8] = (uint32_t)carry;
    x[9] = (uint32_t)(carry >> 32);
#pragma unroll
    for (int k = 10; k < 16; k++) x[k] = 0;
    sc_reduce512(r, x);
    sc_recode256(sd, r);
#pragma unroll
    for (int k = 0; k < 8; k++) sd_s[k] = sd[k];
  }
  __syncthreads();
  if (t < CT_ROWS) {  // row t's entry of digit t, as a point
    uint32_t sd[8];
#pragma unroll
    for (int k = 0; k < 8; k++) sd[k] = sd_s[k];
    p3 P;
    ct_sum(P, combA + (size_t)b * CT_TABLE, sd, (int)t, (int)t + 1);
    uint4 q[9];
    p3_to_quads(q, P);
#pragma unroll
    for (int k = 0; k < 9; k++) red[k][t] = q[k];
  }
  __syncthreads();
  for (uint32_t h = CT_ROWS / 2; h > 0; h >>= 1) {
    if (t < h) {
      p3 A, B;
      uint4 q[9];
#pragma unroll
      for (int k = 0; k < 9; k++) q[k] = red[k][t];
      quads_to_p3(A, q);
#pragma unroll
      for (int k = 0; k < 9; k++) q[k] = red[k][t + h];
      quads_to_p3(B, q);
      p3_acc(A, B);
      p3_to_quads(q, A);
#pragma unroll
      for (int k = 0; k < 9; k++) red[k][t] = q[k];
    }
    __syncthreads();
  }
  if (t < P3_QUADS) keyp[((size_t)g * BV_MAXKEYS + b) * P3_QUADS + t] = red[t][0];
}

__global__ void __launch_bounds__(256) k_bv_keysum(const uint4* __restrict__ keyp, uint32_t nkeys,
                                                   uint4* __restrict__ asum) {
  __shared__ uint4 red[P3_QUADS][256];
  const uint32_t g = blockIdx.x, t = threadIdx.x;
  p3 acc;
  p3_identity(acc);
  for (uint32_t b = t; b < nkeys; b += blockDim.x) {
    p3 P;
    p3_load(P, keyp, (size_t)g * BV_MAXKEYS + b);
    p3_acc(acc, P);
  }
  uint4 q[9];
  p3_to_quads(q, acc);
#pragma unroll
  for (int k = 0; k < 9; k++) red[k][t] = q[k];
  __syncthreads();
  for (uint32_t h = blockDim.x / 2; h > 0; h >>= 1) {
    if (t < h) {
      p3 A, B;
#pragma unroll
      for (int k = 0; k < 9; k++) q[k] = red[k][t];
      quads_to_p3(A, q);
#pragma unroll
      for (int k = 0; k < 9; k++) q[k] = red[k][t + h];
      quads_to_p3(B, q);
      p3_acc(A, B);
      p3_to_quads(q, A);
#pragma unroll
      for (int k = 0; k < 9; k++) red[k][t] = q[k];
    }
    __syncthreads();
  }
  if (t == 0) {
#pragma unroll
    for (int k = 0; k < 9; k++) q[k] = red[k][0];
    quads_to_p3(acc, q);
    p3_neg(acc, acc);  // the tables hold -A
    p3_store(asum, g, acc);
  }
}

// The same reduction with four lanes per element (quad25519.h), for the levels with few
// elements, where one lane per element leaves the chip idle and the level's time is one
// lane's chain of 8 x 3 additions and the doublings.
__global__ void __launch_bounds__(256) k_bv_reduce_q(const uint4* __restrict__ inV, const uint4* __restrict__ inT,
                                                     uint32_t cnt_in, int fan, int shift, uint32_t rows, uint32_t nw,
                                                     uint32_t from_keys, uint4* __restrict__ outV,
                                                     uint4* __restrict__ outT) {
  const uint32_t cnt_out = (cnt_in + fan - 1) / fan;
  const uint32_t gid = (blockIdx.x * blockDim.x + threadIdx.x) >> 2;  // one element per quad
  if (gid >= cnt_out * rows) return;
  const uint32_t r = gid / cnt_out, q = gid % cnt_out;
  const uint32_t rin = from_keys ? (r / nw) * BV_NW + r % nw : r;
  const size_t base = (size_t)rin * cnt_in + (size_t)q * fan;
  const int m = (int)min((uint32_t)fan, cnt_in - q * fan);
  fe U, Sx, X;
  qp_identity(U);
  qp_identity(Sx);
  // each step's point(s) loaded one step ahead (a quad is a lone latency chain)
  if (!inV) {
#if MV_REDUCE_PF == 0
    for (int t = m - 1; t >= 0; t--) {
      qp_load(X, inT, base + t);
      qp_add(U, X);
      qp_add(Sx, U);
    }
    qp_store(outV, gid, Sx);
    qp_store(outT, gid, U);
    return;
#endif
    qp_load(X, inT, base + m - 1);
    for (int t = m - 1; t >= 0; t--) {
      const fe Xc = X;
      if (t > 0) qp_load(X, inT, base + t - 1);
      qp_add(U, Xc);
      qp_add(Sx, U);
    }
    qp_store(outV, gid, Sx);
    qp_store(outT, gid, U);
    return;
  }
  fe Vs, Y;
  qp_identity(Vs);
#if MV_REDUCE_PF == 0
  for (int t = m - 1; t >= 0; t--) {
    qp_load(X, inT, base + t);
    qp_add(U, X);
    if (t > 0) qp_add(Sx, U);
    qp_load(Y, inV, base + t);
    qp_add(Vs, Y);
  }
  qp_dbl_n(Sx, shift);
  qp_add(Vs, Sx);
  qp_store(outV, gid, Vs);
  qp_store(outT, gid, U);
  return;
#endif
  qp_load(X, inT, base + m - 1);
  qp_load(Y, inV, base + m - 1);
  for (int t = m - 1; t >= 0; t--) {
    const fe Xc = X, Yc = Y;
    if (t > 0) {
      qp_load(X, inT, base + t - 1);
      qp_load(Y, inV, base + t - 1);
    }
    qp_add(U, Xc);
    if (t > 0) qp_add(Sx, U);
    qp_add(Vs, Yc);
  }
  qp_dbl_n(Sx, shift);
  qp_add(Vs, Sx);
  qp_store(outV, gid, Vs);
  qp_store(outT, gid, U);
}

// The same level with one WAVE per element, one DPP row per coordinate (pt_r16.h), for the
// small top levels (<= MV_REDUCE_ROWS elements: at most a wave or so per SIMD, where a quad's
// lone chain of 24 additions is issue-bound): the element's 2 x fan inputs are loaded at once
// (one word per lane each) and every point operation is two row products deep. On a big level
// the quad form stays: a wave per element issues ~5x the instructions per element.
__global__ void __launch_bounds__(256) k_bv_reduce_r(const uint4* __restrict__ inV, const uint4* __restrict__ inT,
                                                     uint32_t cnt_in, int fan, int shift, uint32_t rows, uint32_t nw,
                                                     uint32_t from_keys, uint4* __restrict__ outV,
                                                     uint4* __restrict__ outT) {
  const uint32_t cnt_out = (cnt_in + fan - 1) / fan;
  const uint32_t gid = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;  // one element per wave
  if (gid >= cnt_out * rows) return;                                  // (uniform in the wave)
  const uint32_t r = gid / cnt_out, q = gid % cnt_out;
  const uint32_t rin = from_keys ? (r / nw) * BV_NW + r % nw : r;
  const size_t base = (size_t)rin * cnt_in + (size_t)q * fan;
  const int m = (int)min((uint32_t)fan, cnt_in - q * fan);
  const r16::Consts K = r16::consts();
  fe d2;
  fe_const(d2, K_D2);
  fer d2r;
  fer_from_fe(d2r, d2);
  fer T[BV_FAN], V[BV_FAN];
#pragma unroll
  for (int t = 0; t < BV_FAN; t++) {
    T[t] = t < m ? r4::load(inT, base + t) : r4::identity();
    V[t] = (inV && t < m) ? r4::load(inV, base + t) : r4::identity();
  }
  fer U = r4::identity(), Sx = r4::identity();
  if (!inV) {
#pragma unroll
    for (int t = BV_FAN - 1; t >= 0; t--) {
      if (t < m) {
        r4::addp(U, T[t], d2r, K);
        r4::addp(Sx, U, d2r, K);
      }
    }
    r4::store(outV, gid, Sx);
    r4::store(outT, gid, U);
    return;
  }
  fer Vs = r4::identity();
#pragma unroll
  for (int t = BV_FAN - 1; t >= 0; t--) {
    if (t < m) {
      r4::addp(U, T[t], d2r, K);
      if (t > 0) r4::addp(Sx, U, d2r, K);
      r4::addp(Vs, V[t], d2r, K);
    }
  }
#pragma unroll 1
  for (int i = 0; i < shift; i++) r4::dbl(Sx, K);
  r4::addp(Vs, Sx, d2r, K);
  r4::store(outV, gid, Vs);
  r4::store(outT, gid, U);
}

// ---------------------------------------------------------------- final check
// One 128-thread block. Quad g of wave 0: Horner over group g's window sums (V of the last
// reduction level, one per window), four lanes per point. Lane g of wave 1, meanwhile:
// -[sum z s mod l]B of group g from its column sums (k_bv_prep) on the comb table of B.
// flags[1 + g] = group g's equation held; flags[0] = all.
// rows (one group): the Horner on all of wave 0, one DPP row per coordinate (pt_r16.h), then
// quad 0 continues from its result
__global__ void __launch_bounds__(128) k_bv_final(const uint4* __restrict__ winV, uint32_t nw,
                                                  const uint4* __restrict__ asum,
                                                  const unsigned long long* __restrict__ bsum, uint32_t ngroups,
                                                  const uint4* __restrict__ combB, uint32_t* __restrict__ flags,
                                                  uint32_t rows) {
  __shared__ uint4 sbp[BV_MAXG][P3_QUADS];
  __shared__ uint4 shp[P3_QUADS];
  __shared__ uint32_t sflag[BV_MAXG];
  const uint32_t lane = threadIdx.x & 63;
  if (threadIdx.x >= 64) {
    if (lane < ngroups) {
      // x = sum z s mod l from the group's 12 column sums (each < 2^64)
      uint32_t x[16];
      unsigned long long carry = 0;
#pragma unroll
      for (int c = 0; c < BSUM_WORDS; c++) {
        const unsigned long long v = bsum[(size_t)lane * BSUM_WORDS + c];
        const unsigned long long lo = (v & 0xffffffffull) + (carry & 0xffffffffull);
        x[c] = (uint32_t)lo;
        carry = (v >> 32) + (carry >> 32) + (lo >> 32);
      }
      x[12] = (uint32_t)carry;
      x[13] = (uint32_t)(carry >> 32);
      x[14] = x[15] = 0;
      uint32_t r[8], sd[8];
      sc_reduce512(r, x);
      sc_recode256(sd, r);
      // [x]B on the comb table of B (mv_create): 32 mixed additions, no doublings (a ladder
      // would be 248 doublings, as long as the Horner chain beside it)
      p3 P;
      ct_sum(P, combB, sd, 0, CT_ROWS);
      p3_neg(P, P);
      uint4 q[9];
      p3_to_quads(q, P);
#pragma unroll
      for (int i = 0; i < 9; i++) sbp[lane][i] = q[i];
    }
  }
  // Horner over group g's window sums on quad g of wave 0 (quad25519.h: a doubling is one
  // squaring and one multiplication deep), then the per-key A term
  const uint32_t g = lane >> 2;
  fe v;
  if (threadIdx.x < 64 && rows && ngroups == 1) {
    const r16::Consts K = r16::consts();
    fe d2;
    fe_const(d2, K_D2);
    fer d2r;
    fer_from_fe(d2r, d2);
    fer pv = r4::load(winV, nw - 1);
#pragma unroll 1
    for (int w = (int)nw - 2; w >= 0; w--) {
      const fer wv = r4::load(winV, w);
#pragma unroll 1
      for (int i = 0; i < BV_C; i++) r4::dbl(pv, K);
      r4::addp(pv, wv, d2r, K);
    }
    if (asum) r4::addp(pv, r4::load(asum, 0), d2r, K);
    r4::store(reinterpret_cast<uint32_t*>(shp), pv);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the rows' stores before quad 0 reads
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (g == 0) qp_load(v, shp, 0);
  } else if (threadIdx.x < 64 && g < ngroups) {
    const size_t row0 = (size_t)g * nw;
    qp_load(v, winV, row0 + nw - 1);
    for (int w = (int)nw - 2; w >= 0; w--) {
      fe wv;
      qp_load(wv, winV, row0 + w);
      qp_dbl_n(v, BV_C);
      qp_add(v, wv);
    }
    if (asum) {  // the per-key A term of the group (k_bv_keysum)
      fe av;
      qp_load(av, asum, g);
      qp_add(v, av);
    }
  }
  __syncthreads();
  if (threadIdx.x < 64 && g < ngroups) {
    fe bv;
    qp_load(bv, &sbp[0][0], g);
    qp_add(v, bv);
    qp_dbl_n(v, 3);  // cofactor
    // identity <=> X == 0 and Y == Z (mod p)
    fe Y, Z;
    fe_qget<1>(Y, v);
    fe_qget<2>(Z, v);
    const bool x0 = fe_is_zero(v);
    const bool yz = fe_eq(Y, Z);
    if ((lane & 3) == 0) sflag[g] = x0 && yz ? 1u : 0u;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t all = 1;
    for (uint32_t gg = 0; gg < ngroups; gg++) {
      flags[1 + gg] = sflag[gg];
      all &= sflag[gg];
    }
    flags[0] = all;
  }
}

}  // namespace mv

// ---------------------------------------------------------------- launchers
namespace mvk {

namespace {
constexpr size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
struct BatchLayout {
  size_t pts, scal, pcount, poff, ptot, pstart, tmp, offs, ents, segV, segT, rV0, rT0, rV1, rT1, bsum, kpart, keyp,
      asum, flag, total;
  BatchLayout(uint32_t n, uint32_t groups) {
    using namespace mv;
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o += align256(bytes); return r; };
    pts = take((size_t)2 * n * PT_QUADS * 16);
    scal = take((size_t)n * SC_QUADS * 16);
    const size_t nchunk = (n + PART_CHUNK - 1) / PART_CHUNK;
    pcount = take(nchunk * BV_NPG * 4);
    poff = take(nchunk * BV_NPG * 4);
    ptot = take((size_t)groups * BV_NPG * 4);
    pstart = take(((size_t)groups * BV_NPG + 1) * 4);
    tmp = take((size_t)(BV_NWR + BV_NW) * n * 8);
    offs = take(((size_t)groups * BV_NKG + 1) * 4);
    ents = take((size_t)(BV_NWR + BV_NW) * n * 4);
    // segments of >= 2 buckets, or the balanced bucket kernel's carries (one per lane)
    segV = take((size_t)groups * BV_NKG / 2 * P3_QUADS * 16);
    segT = take((size_t)groups * BV_NKG * P3_QUADS * 16);
    const size_t lv = (size_t)groups * (BV_NKG / BV_FAN) * P3_QUADS * 16;
    rV0 = take(lv); rT0 = take(lv); rV1 = take(lv); rT1 = take(lv);
    bsum = take((size_t)BV_MAXG * BSUM_WORDS * 8);  // per group
    kpart = take(nchunk * BV_MAXKEYS * 8 * 8);
    keyp = take((size_t)BV_MAXG * BV_MAXKEYS * P3_QUADS * 16);
    asum = take((size_t)BV_MAXG * P3_QUADS * 16);
    flag = take((1 + BV_MAXG) * 4);
    total = o;
  }
};
// group geometry: `want` groups of whole 1024-signature chunks
mv::BvGroups batch_groups(uint32_t n, uint32_t want) {
  const uint32_t nchunk = (n + mv::PART_CHUNK - 1) / mv::PART_CHUNK;
  uint32_t g = want < 1 ? 1 : (want > (uint32_t)mv::BV_MAXG ? (uint32_t)mv::BV_MAXG : want);
  if (g > nchunk) g = nchunk;
  const uint32_t cpg = (nchunk + g - 1) / g;
  return mv::BvGroups{(nchunk + cpg - 1) / cpg, cpg};
}
// MV_NO_KEY_AGG=1 (experiments): committee keys keep one A bucket entry per signature
bool agg_disabled(const Knobs& kn) { return kn.no_key_agg != 0; }

// reduction levels with at most this many elements run four lanes per element
// (MV_REDUCE_QUAD=<n> for experiments; 0 = never)
uint32_t reduce_quad_max(const Knobs& kn) { return (uint32_t)kn.reduce_quad; }

// buckets per bucket-kernel lane (a power of two): MV_BV_SEG=<k> for experiments
uint32_t bucket_segment(const Knobs& kn) {
  uint32_t seg = kn.bv_seg > 0 ? (uint32_t)kn.bv_seg : 1u;  // 1: measured best for 1..16 groups with the quad reduce
  if (seg > 64) seg = 64;
  return 1u << (31 - __builtin_clz(seg));
}
}  // namespace

size_t batch_scratch_bytes(uint32_t n, uint32_t groups) { return BatchLayout(n, groups).total; }

uint32_t batch_group_size(uint32_t n, uint32_t groups) {
  return batch_groups(n, groups).cpg * mv::PART_CHUNK;
}

hipError_t launch_verify_batch(const Knobs& kn, const uint8_t* msg, const uint8_t* sig, const uint8_t* pk, const uint32_t* key_idx,
                               uint32_t n, uint32_t groups, const uint32_t key[10], const void* btab,
                               void* bscratch, void* vscratch, uint8_t* status, hipStream_t s,
                               uint32_t** flag_out, hipEvent_t* ev, const void* comb_a, const uint8_t* key_ok,
                               uint32_t n_keys, const void* comb_b, const ChunkGate* gate, const hipEvent_t* chain) {
  using namespace mv;
  // optional stage events (engine stage timing): ev[0] before prep, ev[i + 1] after stage i
  auto mark = [&](int i) { if (ev) (void)hipEventRecord(ev[i], s); };
  if (n == 0) return hipSuccess;
  const BvGroups G = batch_groups(n, groups);
  const BatchLayout L(n, G.count);
  char* base = static_cast<char*>(bscratch);
  uint4* pts = (uint4*)(base + L.pts);
  uint4* scal = (uint4*)(base + L.scal);
  uint32_t* pcount = (uint32_t*)(base + L.pcount);
  uint32_t* poff = (uint32_t*)(base + L.poff);
  uint32_t* ptot = (uint32_t*)(base + L.ptot);
  uint32_t* pstart = (uint32_t*)(base + L.pstart);
  unsigned long long* tmp = (unsigned long long*)(base + L.tmp);
  uint32_t* offs = (uint32_t*)(base + L.offs);
  uint32_t* ents = (uint32_t*)(base + L.ents);
  uint4* segV = (uint4*)(base + L.segV);
  uint4* segT = (uint4*)(base + L.segT);
  uint4* rv[2] = {(uint4*)(base + L.rV0), (uint4*)(base + L.rV1)};
  uint4* rt[2] = {(uint4*)(base + L.rT0), (uint4*)(base + L.rT1)};
  unsigned long long* bsum = (unsigned long long*)(base + L.bsum);
  unsigned long long* kpart = (unsigned long long*)(base + L.kpart);
  uint4* keyp = (uint4*)(base + L.keyp);
  uint4* asum = (uint4*)(base + L.asum);
  uint32_t* flag = (uint32_t*)(base + L.flag);
  if (flag_out) *flag_out = flag;
  const uint32_t nblk = (n + 255) / 256;
  hipError_t e;
  BvKey k;
  for (int i = 0; i < 10; i++) k.w[i] = key[i];
  const uint32_t nchunk = (n + PART_CHUNK - 1) / PART_CHUNK;
  const uint32_t nparts = G.count * BV_NPG;
  mark(0);
  // committee keys with their comb tables: A from the tables, and its term summed per key
  const bool com = key_idx && key_ok && comb_a;
  const bool agg = com && n_keys > 0 && n_keys <= (uint32_t)BV_MAXKEYS && !agg_disabled(kn);
  CommitteeA ca{com ? static_cast<const uint4*>(comb_a) : nullptr, key_ok,
                (uint32_t)(comb_table_bytes(1) / sizeof(uint4)), agg ? 1u : 0u};
  const uint32_t nw = agg ? BV_NWR : BV_NW;  // windows with bucket entries
  e = hipMemsetAsync(bsum, 0, (size_t)BV_MAXG * BSUM_WORDS * 8, s);  // k_bv_prep accumulates per group
  if (e != hipSuccess) return e;
  const uint32_t seg = bucket_segment(kn);
  const uint32_t nk = G.count * BV_NKG;
  // bucket sums of the sorted entries of m signatures
  auto buckets = [&](uint64_t m) {
    if (seg == 1 && kn.bucket_bal > 0) {
      // equal entries per lane (the carries in segV: at most one per lane): 64 per lane, but at
      // least 3 waves per SIMD (196,608 lanes) while lanes keep >= 8 entries, so a small batch or
      // segment still fills the chip instead of running a few long lanes
      const uint64_t est = m * (nw + BV_NWR);  // entries: at most one per window of z and of z k
      uint64_t want = kn.bucket_bal > 1 ? est / (uint64_t)kn.bucket_bal
                                        : std::max<uint64_t>(est / 64, std::min<uint64_t>(est / 8, 196608));
      const uint32_t cap = nk / 2;
      uint32_t nl = (uint32_t)std::min<uint64_t>(cap, std::max<uint64_t>(256, (want + 255) / 256 * 256));
      hipLaunchKernelGGL(k_bv_bucket_bal, dim3(nl / 256), dim3(256), 0, s, pts, offs, ents, nk, nl, segV, segT);
      hipLaunchKernelGGL(k_bv_bucket_fix, dim3(G.count * nw * BV_NB / 256), dim3(256), 0, s, offs, nk, G.count, nw, nl,
                         segV, segT);
    } else {
      hipLaunchKernelGGL(k_bv_bucket, dim3(G.count * nw * (BV_NB / seg) / 256), dim3(256), 0, s, pts, offs, ents,
                         G.count, seg, nw, segV, segT);
    }
  };
  if (gate && gate->n) {
    const uint32_t* end = gate->end;
    if (end[gate->n - 1] != n) return hipErrorInvalidValue;
    for (uint32_t c = 0, lo = 0; c < gate->n; lo = end[c++]) {
      const uint32_t hi = end[c];
      if (hi <= lo || lo % 256 || (hi % 256 && hi != n)) return hipErrorInvalidValue;
      if ((e = hipStreamWaitEvent(s, gate->ready[c], 0)) != hipSuccess) return e;
      hipLaunchKernelGGL(k_bv_prep, dim3((hi - lo + 255) / 256), dim3(256), 0, s, msg, sig, pk, key_idx, n, k, ca,
                         pts, scal, bsum, status, lo / 256, G.cpg * PART_CHUNK);
    }
  } else {
    if (chain && chain[0] && (e = hipStreamWaitEvent(s, chain[0], 0)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_bv_prep, dim3(nblk), dim3(256), 0, s, msg, sig, pk, key_idx, n, k, ca, pts, scal, bsum,
                       status, 0u, G.cpg * PART_CHUNK);
    if (chain && (e = hipEventRecord(chain[1], s)) != hipSuccess) return e;
  }
  {
    mark(1);
    hipLaunchKernelGGL(k_part_count, dim3(nchunk), dim3(PART_CHUNK), 0, s, scal, n, agg ? 1u : 0u, pcount);
    hipLaunchKernelGGL(k_part_scan, dim3(G.count * (BV_NPG / 64)), dim3(64 * SCAN_SUB), 0, s, pcount, nchunk, G, poff,
                       ptot);
    hipLaunchKernelGGL(k_part_top, dim3(1), dim3(256), 0, s, ptot, nparts, pstart);
    if (kn.scatter_lds)
      hipLaunchKernelGGL(k_part_scatter_lds, dim3(nchunk), dim3(PART_CHUNK), 0, s, scal, n, pcount, poff, pstart, G,
                         agg ? 1u : 0u, n, 0u, tmp);
    else
      hipLaunchKernelGGL(k_part_scatter, dim3(nchunk), dim3(PART_CHUNK), 0, s, scal, n, poff, pstart, G,
                         agg ? 1u : 0u, n, 0u, tmp);
    if (kn.fine_lds)
      hipLaunchKernelGGL(k_fine_sort_lds, dim3(nparts), dim3(FINE_NT), 0, s, tmp, pstart, G.count, ents, offs);
    else
      hipLaunchKernelGGL(k_fine_sort, dim3(nparts), dim3(FINE_NT), 0, s, tmp, pstart, G.count, ents, offs);
    mark(2);
    // buckets per bucket-kernel lane: one per lane while the grid is small; with many groups,
    // a lane walks `seg` buckets and emits their running sums, so the bucket cells never go
    // through memory and the reduction stays the size of one group's
    buckets(n);
  }
  if (agg) {
    hipLaunchKernelGGL(k_bv_keyacc, dim3(nchunk), dim3(PART_CHUNK), 0, s, scal, key_idx, n, n_keys, kpart);
    hipLaunchKernelGGL(k_bv_keycol, dim3(G.count * n_keys), dim3(256), 0, s, kpart, nchunk, G.cpg, n_keys,
                       static_cast<const uint4*>(comb_a), keyp);
    hipLaunchKernelGGL(k_bv_keysum, dim3(G.count), dim3(256), 0, s, keyp, n_keys, asum);
  }
  mark(3);
  const uint4* inV = seg > 1 ? segV : nullptr;  // one bucket per segment: V = T
  const uint4* inT = segT;
  const uint32_t rows = G.count * nw;
  uint32_t cnt = BV_NB / seg;
  int shift = 31 - __builtin_clz(seg);  // log2(seg)
  int pp = 0;
  while (cnt > 1) {
    const int fan = cnt >= (uint32_t)BV_FAN ? BV_FAN : (int)cnt;
    const uint32_t out = (cnt + fan - 1) / fan;
    const uint32_t lanes = out * rows;
    if (lanes <= (uint32_t)kn.reduce_rows)  // small top level: a wave per element
      hipLaunchKernelGGL(k_bv_reduce_r, dim3((64 * lanes + 255) / 256), dim3(256), 0, s, inV, inT, cnt, fan, shift,
                         rows, nw, inT == segT ? 1u : 0u, rv[pp], rt[pp]);
    else if (lanes <= reduce_quad_max(kn))  // latency-bound level: four lanes per element
      hipLaunchKernelGGL(k_bv_reduce_q, dim3((4 * lanes + 255) / 256), dim3(256), 0, s, inV, inT, cnt, fan, shift,
                         rows, nw, inT == segT ? 1u : 0u, rv[pp], rt[pp]);
    else
      hipLaunchKernelGGL(k_bv_reduce, dim3((lanes + 63) / 64), dim3(64), 0, s, inV, inT, cnt, fan, shift, rows, nw,
                         inT == segT ? 1u : 0u, rv[pp], rt[pp]);
    inV = rv[pp];
    inT = rt[pp];
    pp ^= 1;
    shift += fan == 8 ? 3 : (fan == 4 ? 2 : 1);
    cnt = out;
  }
  mark(4);
  hipLaunchKernelGGL(k_bv_final, dim3(1), dim3(128), 0, s, inV, nw, agg ? (const uint4*)asum : nullptr, bsum,
                     G.count, static_cast<const uint4*>(comb_b), flag, kn.final_rows ? 1u : 0u);
  mark(5);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  // exact fallback: re-verifies the signatures of every group whose equation failed
  // (R and A as k_bv_prep decoded them: no decompression)
  e = launch_verify(kn, msg, sig, pk, key_idx, n, btab, vscratch, status, s, flag + 1, G.cpg * PART_CHUNK, pts,
                    ca.tab && ca.aggregate ? comb_a : nullptr);
  mark(6);
  return e;
}

}  // namespace mvk
