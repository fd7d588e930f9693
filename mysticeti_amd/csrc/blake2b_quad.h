// BLAKE2b-256 with FOUR lanes per string: the device code of blake2b_quad.hip (its header
// comment describes the design), shared with comb.hip's latency-path kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef MV_DEV
#define MV_DEV __device__ __forceinline__
#endif

namespace mv {
namespace b2q {

// RFC 7693 §2.7 message schedule (rounds 10 and 11 reuse rows 0 and 1)
constexpr uint8_t SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

// LDS layout of a message block: word w of string j sits at u64 index
// WH[w] * 16 NS * 4 + 4 j + WG[w] of the buffer ([rank][string][class]). A ds_read_b64 half-wave
// is 8 quads (strings) x 4 lanes, and lane q of every quad reads the same word SIGMA[r][...];
// quad j's four reads land on 8-byte bank slots 4 j + WG[w] (mod 32), so they are conflict-
// free when the four words have distinct classes WG. No class map makes all 40 distinct
// SIGMA word quadruples rainbow (exhaustive search); this one (local search) costs 1.60 LDS
// cycles per half-wave read on average, against 2.65 for rows padded to 17 words.
constexpr uint8_t WG[16] = {0, 0, 2, 0, 1, 0, 3, 3, 1, 3, 2, 1, 3, 1, 2, 2};
constexpr uint8_t WH[16] = {0, 1, 0, 2, 0, 3, 0, 1, 1, 2, 1, 2, 3, 3, 2, 3};
template <int NS>
constexpr uint32_t woff(int w) { return (uint32_t)WH[w] * 64u * NS + WG[w]; }  // u64 units from the string's base

// The u64 offset lane q reads in round r, slot k (0/1: column step x/y, 2/3: diagonal step
// x/y) is woff(SIGMA[r][8 (k >> 1) + 2q + (k & 1)]); packed 8 bits per lane (NS = 1) or 16
// bits per lane (NS = 2).
template <int NS>
constexpr uint64_t msel(int r, int k) {
  uint64_t c = 0;
  for (int q = 0; q < 4; q++)
    c |= (uint64_t)woff<NS>(SIGMA[r][8 * (k >> 1) + 2 * q + (k & 1)]) << ((NS == 1 ? 8 : 16) * q);
  return c;
}
template <int NS>
struct Sel {
  uint64_t v[12][4];
};
template <int NS>
constexpr Sel<NS> make_sel() {
  Sel<NS> s{};
  for (int r = 0; r < 12; r++)
    for (int k = 0; k < 4; k++) s.v[r][k] = msel<NS>(r, k);
  return s;
}
template <int NS>
constexpr Sel<NS> SEL = make_sel<NS>();
template <int NS>
MV_DEV uint32_t sel_at(int r, int k, uint32_t q) {
  if (NS == 1) return __builtin_amdgcn_ubfe((uint32_t)SEL<1>.v[r][k], 8 * q, 8);  // one v_bfe_u32
  return (uint32_t)(SEL<NS>.v[r][k] >> (16 * q)) & 0xffffu;
}

constexpr uint64_t IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                            0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                            0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

// a plain 64-bit add: the compiler selects v_lshl_add_u64 itself and, unlike for an inline-asm
// one, knows its hazards (no s_nop after every add)
MV_DEV uint64_t add64(uint64_t a, uint64_t b) { return a + b; }
MV_DEV uint64_t pack(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
MV_DEV uint64_t ror32(uint64_t x) { return (x >> 32) | (x << 32); }
MV_DEV uint64_t ror24(uint64_t x) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return pack(__builtin_amdgcn_perm(hi, lo, 0x06050403u), __builtin_amdgcn_perm(lo, hi, 0x06050403u));
}
MV_DEV uint64_t ror16(uint64_t x) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return pack(__builtin_amdgcn_perm(hi, lo, 0x05040302u), __builtin_amdgcn_perm(lo, hi, 0x05040302u));
}
MV_DEV uint64_t ror63(uint64_t x) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return pack(__builtin_amdgcn_alignbit(lo, hi, 31), __builtin_amdgcn_alignbit(hi, lo, 31));
}
// lane q of each quad takes x from lane (q + K) & 3
template <int K>
MV_DEV uint64_t qrot(uint64_t x) {
  constexpr int ctrl = ((0 + K) & 3) | (((1 + K) & 3) << 2) | (((2 + K) & 3) << 4) | (((3 + K) & 3) << 6);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)x, ctrl, 0xf, 0xf, true);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(x >> 32), ctrl, 0xf, 0xf, true);
  return pack(lo, hi);
}

#define MV_QG(x, y)         \
  a = add64(add64(a, b), x); \
  d = ror32(d ^ a);          \
  c = add64(c, d);           \
  b = ror24(b ^ c);          \
  a = add64(add64(a, b), y); \
  d = ror16(d ^ a);          \
  c = add64(c, d);           \
  b = ror63(b ^ c);

// One compression of the quad's block m[16] (LDS) for each of NS strings, interleaved: the
// strings' G chains are independent, so one string's instructions fill the other's
// dependency and DPP-hazard gaps, and the message-word addresses are computed once for
// both. (h0, h1) = (h[q], h[4 + q]); (iv0, iv1) = (IV[q], IV[4 + q]); t = byte counter
// (< 2^64), fin = final block.
// HOIST (the latency path: one wave per SIMD): no per-round barrier, so the scheduler issues
// the message reads ahead of the G chains and the LDS latency leaves the critical path
template <int NS, bool HOIST = false>
MV_DEV void compress(uint64_t (&h0)[NS], uint64_t (&h1)[NS], const uint64_t* const (&m)[NS], uint32_t q,
                     uint64_t iv0, uint64_t iv1, const uint64_t (&t)[NS], const bool (&fin)[NS]) {
  uint64_t va[NS], vb[NS], vc[NS], vd[NS];
#pragma unroll
  for (int k = 0; k < NS; k++) {
    va[k] = h0[k];
    vb[k] = h1[k];
    vc[k] = iv0;
    vd[k] = iv1 ^ (q == 0 ? t[k] : 0ull);        // v[12] ^= t (t_hi = 0: v[13] unchanged)
    vd[k] = (q == 2 && fin[k]) ? ~vd[k] : vd[k];  // v[14] = ~v[14] on the final block
  }
#pragma unroll
  for (int r = 0; r < 12; r++) {
    // keep each round's message reads in their round: hoisting all 48 ahead of the chain
    // (what the scheduler does unchecked) doubles the VGPRs and halves the waves per SIMD
    if (!HOIST) asm volatile("" ::: "memory");
    const uint32_t qq = q;
    const uint32_t i0 = sel_at<NS>(r, 0, qq), i1 = sel_at<NS>(r, 1, qq);
    const uint32_t i2 = sel_at<NS>(r, 2, qq), i3 = sel_at<NS>(r, 3, qq);
    uint64_t x0[NS], y0[NS], x1[NS], y1[NS];
#pragma unroll
    for (int k = 0; k < NS; k++) {
      x0[k] = m[k][i0];
      y0[k] = m[k][i1];
      x1[k] = m[k][i2];
      y1[k] = m[k][i3];
    }
#pragma unroll
    for (int k = 0; k < NS; k++) {
      uint64_t a = va[k], b = vb[k], c = vc[k], d = vd[k];
      MV_QG(x0[k], y0[k])
      va[k] = a; vb[k] = b; vc[k] = c; vd[k] = d;
    }
#pragma unroll
    for (int k = 0; k < NS; k++) {
      vb[k] = qrot<1>(vb[k]);
      vc[k] = qrot<2>(vc[k]);
      vd[k] = qrot<3>(vd[k]);
    }
#pragma unroll
    for (int k = 0; k < NS; k++) {
      uint64_t a = va[k], b = vb[k], c = vc[k], d = vd[k];
      MV_QG(x1[k], y1[k])
      va[k] = a; vb[k] = b; vc[k] = c; vd[k] = d;
    }
#pragma unroll
    for (int k = 0; k < NS; k++) {
      vb[k] = qrot<3>(vb[k]);
      vc[k] = qrot<2>(vc[k]);
      vd[k] = qrot<1>(vd[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < NS; k++) {
    h0[k] ^= va[k] ^ vc[k];
    h1[k] ^= vb[k] ^ vd[k];
  }
}
#undef MV_QG

MV_DEV uint32_t wave_min32(uint32_t x) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, m));
  return x;
}
MV_DEV uint32_t wave_max(uint32_t x) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, m));
  return x;
}

// What step s of a string hashes. DUAL (the block path, staged P || sig with L = |P|):
// steps [0, common) are the compressions B2(P) and B2(P || sig) share, step `common` is the
// final block of B2(P) (msg), steps after it finish B2(P || sig) (digest). Otherwise one
// hash of L bytes. Steps at or past the string's count load nothing (lim = 0).
template <bool DUAL>
struct Plan {
  uint64_t L, common, last;
  uint32_t nsteps;
  MV_DEV void init(uint64_t len, bool live) {
    L = len;
    if (DUAL) {
      common = L == 0 ? 0 : (L - 1) / 128;
      last = (L + 63) / 128;
      nsteps = live ? (uint32_t)(last + 2) : 0u;
    } else {
      common = ~0ull;
      last = L == 0 ? 0 : (L - 1) / 128;
      nsteps = live ? (uint32_t)(last + 1) : 0u;
    }
  }
  // block index, length limit, counter, final flag, msg-final flag
  MV_DEV void at(uint32_t s, uint64_t& b, uint64_t& lim, uint64_t& t, bool& fin, bool& mfin) const {
    if (DUAL) {
      mfin = s == common;
      b = s < common ? s : (mfin ? common : s - 1);
      lim = mfin ? L : L + 64;
      fin = mfin || b == last;
      t = mfin ? L : (b == last ? L + 64 : 128 * (b + 1));
    } else {
      mfin = false;
      b = s;
      lim = L;
      fin = b == last;
      t = fin ? L : 128 * (b + 1);
    }
    if (s >= nsteps) lim = 0;
  }
};

// Lane q's quarter (words 4q .. 4q+3) of block b, zero past lim; a word is read only when it
// starts below lim (the strings are 8-aligned and readable up to round-up(lim, 8)).
MV_DEV void load_quarter(uint64_t w[4], const uint8_t* p, uint64_t b, uint64_t lim, uint32_t q) {
  const uint64_t* src = reinterpret_cast<const uint64_t*>(p) + b * 16 + 4 * q;
  const uint64_t base = b * 128 + 32 * q;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint64_t pos = base + 8 * j;
    uint64_t v = 0;
    if (pos < lim) {
      v = src[j];
      const uint64_t rem = lim - pos;
      if (rem < 8) v &= (1ull << (8 * rem)) - 1;
    }
    w[j] = v;
  }
}

// 16 * NS strings per 64-lane workgroup: quad qd takes strings 16 k + qd, k < NS. DUAL:
// out0 = B2(P) (msg), out1 = B2(P || sig) (digest); otherwise out0 = B2(string).
// WAVE: one wave of a larger workgroup runs this alone (k_verify_comb16's online hash): its
// steps are ordered by wave-scope fences instead of workgroup barriers. Strings
// [first, first + count) of the n, count <= 16 NS (quad qd takes string first + 16 k + qd).
template <bool WAVE>
MV_DEV void qh_sync() {
  if (WAVE) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}
// EXTRA: bytes hashed past len[i] (the staged signature after a pre-image: the block digest alone)
template <bool DUAL, int NS, bool HOIST = false, bool WAVE = false, uint32_t EXTRA = 0>
MV_DEV void quad_hash_range(uint32_t first, uint32_t count, const uint8_t* __restrict__ buf,
                            const uint64_t* __restrict__ off, const uint64_t* __restrict__ len, uint32_t n,
                            uint8_t* __restrict__ out0, uint8_t* __restrict__ out1) {
  // [buffer][word rank][string][word class] (WG/WH above)
  __shared__ uint64_t mbuf[2][4][16 * NS][4];
  const uint32_t lane = threadIdx.x & 63u, q = lane & 3, qd = lane >> 2;
  uint32_t wo[4];  // offsets of this lane's quarter (words 4q .. 4q+3) from the string's base
#pragma unroll
  for (int j = 0; j < 4; j++) wo[j] = (uint32_t)WH[4 * q + j] * 64u * NS + WG[4 * q + j];
  uint32_t idx[NS];
  bool live[NS];
  const uint8_t* p[NS];
  Plan<DUAL> pl[NS];
  uint32_t nsteps_max = 0, nfull_min = 0xffffffffu;
#pragma unroll
  for (int k = 0; k < NS; k++) {
    idx[k] = first + 16 * k + qd;
    live[k] = 16 * k + qd < count && idx[k] < n;
    p[k] = buf + (live[k] ? off[idx[k]] : 0);
    pl[k].init(live[k] ? len[idx[k]] + EXTRA : 0, live[k]);
    nsteps_max = max(nsteps_max, pl[k].nsteps);
    // whole 128-byte blocks that are neither final nor the message's last (the shared prefix)
    const uint64_t c = live[k] ? (DUAL ? pl[k].common : pl[k].last) : 0;
    nfull_min = min(nfull_min, (uint32_t)(c > 0xffffffffull ? 0xffffffffull : c));
  }
  const uint32_t nmax = wave_max(nsteps_max);
  const uint32_t nfull = min(wave_min32(nfull_min), nmax);
  const uint64_t iv0 = IV[q], iv1 = IV[4 + q];
  uint64_t h0[NS], h1[NS];
#pragma unroll
  for (int k = 0; k < NS; k++) {
    h0[k] = iv0 ^ (q == 0 ? 0x01010020ull : 0ull);  // depth 1, fanout 1, nn = 32
    h1[k] = iv1;
  }
  uint64_t w[NS][4];
  const uint64_t* mrow[NS];
  uint64_t t[NS];
  bool fin[NS];
  // Steps [0, nfull): whole blocks of every string of the wave: no plan, no masking,
  // counters 128 (s + 1). The remaining steps go through the plans.
#pragma unroll
  for (int k = 0; k < NS; k++) {
    if (nfull > 0) {
      const uint64_t* src = reinterpret_cast<const uint64_t*>(p[k]) + 4 * q;
#pragma unroll
      for (int j = 0; j < 4; j++) w[k][j] = src[j];
    } else {
      uint64_t b, lim, tt;
      bool f, mf;
      pl[k].at(0, b, lim, tt, f, mf);
      load_quarter(w[k], p[k], b, lim, q);
    }
#pragma unroll
    for (int j = 0; j < 4; j++) (&mbuf[0][0][16 * k + qd][0])[wo[j]] = w[k][j];
  }
  for (uint32_t s = 0; s < nfull; s++) {
    qh_sync<WAVE>();
#pragma unroll
    for (int k = 0; k < NS; k++) {
      if (s + 1 < nfull) {  // the next whole block, in flight during this compression
        const uint64_t* src = reinterpret_cast<const uint64_t*>(p[k]) + (size_t)(s + 1) * 16 + 4 * q;
#pragma unroll
        for (int j = 0; j < 4; j++) w[k][j] = src[j];
      } else {
        uint64_t b, lim, tt;
        bool f, mf;
        pl[k].at(s + 1, b, lim, tt, f, mf);
        load_quarter(w[k], p[k], b, lim, q);
      }
      mrow[k] = &mbuf[s & 1][0][16 * k + qd][0];
      t[k] = 128ull * (s + 1);
      fin[k] = false;
    }
    compress<NS, HOIST>(h0, h1, mrow, q, iv0, iv1, t, fin);
#pragma unroll
    for (int k = 0; k < NS; k++)
#pragma unroll
      for (int j = 0; j < 4; j++) (&mbuf[(s + 1) & 1][0][16 * k + qd][0])[wo[j]] = w[k][j];
  }
  for (uint32_t s = nfull; s < nmax; s++) {
    qh_sync<WAVE>();
    bool mfin[NS];
    uint64_t s0[NS], s1[NS];
#pragma unroll
    for (int k = 0; k < NS; k++) {
      uint64_t bn, limn, tn, b, lim;
      bool finn, mfinn;
      pl[k].at(s + 1, bn, limn, tn, finn, mfinn);
      load_quarter(w[k], p[k], bn, limn, q);  // next block, in flight during this compression
      pl[k].at(s, b, lim, t[k], fin[k], mfin[k]);
      mrow[k] = &mbuf[s & 1][0][16 * k + qd][0];
      s0[k] = h0[k];
      s1[k] = h1[k];
    }
    compress<NS, HOIST>(h0, h1, mrow, q, iv0, iv1, t, fin);
#pragma unroll
    for (int k = 0; k < NS; k++) {
      if (DUAL && mfin[k] && s < pl[k].nsteps) reinterpret_cast<uint64_t*>(out0 + 32 * (size_t)idx[k])[q] = h0[k];
      if ((DUAL && mfin[k]) || s >= pl[k].nsteps) {  // msg stored / string already done: keep h
        h0[k] = s0[k];
        h1[k] = s1[k];
      }
#pragma unroll
      for (int j = 0; j < 4; j++) (&mbuf[(s + 1) & 1][0][16 * k + qd][0])[wo[j]] = w[k][j];
    }
  }
#pragma unroll
  for (int k = 0; k < NS; k++)
    if (live[k]) reinterpret_cast<uint64_t*>((DUAL ? out1 : out0) + 32 * (size_t)idx[k])[q] = h0[k];
}
// 16 NS strings per 64-lane workgroup (block blk)
template <bool DUAL, int NS, bool HOIST = false>
MV_DEV void quad_hash(uint32_t blk, const uint8_t* __restrict__ buf, const uint64_t* __restrict__ off,
                      const uint64_t* __restrict__ len, uint32_t n, uint8_t* __restrict__ out0,
                      uint8_t* __restrict__ out1) {
  quad_hash_range<DUAL, NS, HOIST, false>(blk * 16 * NS, 16 * NS, buf, off, len, n, out0, out1);
}


}  // namespace b2q
}  // namespace mv
