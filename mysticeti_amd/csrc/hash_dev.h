// Per-lane SHA-512 (FIPS 180-4) and BLAKE2b (RFC 7693) compressions for gfx950.
//
// SHA-512 is the ed25519 challenge hash k = H(R || A || M) (ed25519-consensus
// 2.1.0 over sha2 0.9.9); BLAKE2b-256 is mysticeti's BlockHasher
// (mysticeti-core/src/crypto.rs:34, Blake2b<U32>). 64-bit words are held as
// VGPR pairs; rotations lower to v_alignbit_b32 pairs, 3-input logic to
// v_bitop3_b32 (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#ifndef MV_DEV
#define MV_DEV __device__ __forceinline__
#endif

namespace mv {

// 64-bit rotate right by a constant n (after inlining): two v_alignbit_b32, or a register swap
MV_DEV uint64_t rotr64(uint64_t x, int n) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (n == 32) return ((uint64_t)lo << 32) | hi;
  if (n == 8 || n == 16 || n == 24) {  // byte rotations: v_perm_b32 (full rate; v_alignbit is half)
    const uint32_t k = (uint32_t)n >> 3, sel = (k | (k + 1) << 8 | (k + 2) << 16 | (k + 3) << 24);
    return ((uint64_t)__builtin_amdgcn_perm(lo, hi, sel) << 32) | __builtin_amdgcn_perm(hi, lo, sel);
  }
  if (n < 32)
    return ((uint64_t)__builtin_amdgcn_alignbit(lo, hi, n) << 32) | __builtin_amdgcn_alignbit(hi, lo, n);
  return ((uint64_t)__builtin_amdgcn_alignbit(hi, lo, n - 32) << 32) | __builtin_amdgcn_alignbit(lo, hi, n - 32);
}
MV_DEV uint64_t shr64(uint64_t x, int n) {  // n < 32
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return ((uint64_t)(hi >> n) << 32) | __builtin_amdgcn_alignbit(hi, lo, n);
}
// 3-input logic per 32-bit half (v_bitop3_b32, gfx950): 0x96 = a ^ b ^ c, 0xE8 = majority
template <int IMM>
MV_DEV uint64_t bitop3_64(uint64_t a, uint64_t b, uint64_t c) {
  const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, IMM);
  const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), IMM);
  return ((uint64_t)hi << 32) | lo;
}
MV_DEV uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

__constant__ const uint64_t SHA512_K[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL, 0x3956c25bf348b538ULL,
    0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL, 0xd807aa98a3030242ULL, 0x12835b0145706fbeULL,
    0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL, 0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL,
    0xc19bf174cf692694ULL, 0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL, 0x983e5152ee66dfabULL,
    0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL, 0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL,
    0x06ca6351e003826fULL, 0x142929670a0e6e70ULL, 0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL,
    0x53380d139d95b3dfULL, 0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL, 0xd192e819d6ef5218ULL,
    0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL, 0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL,
    0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL, 0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL,
    0x682e6ff3d6b2b8a3ULL, 0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL, 0xca273eceea26619cULL,
    0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL, 0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL,
    0x113f9804bef90daeULL, 0x1b710b35131c471bULL, 0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL,
    0x431d67c49c100d4cULL, 0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

MV_DEV void sha512_init(uint64_t st[8]) {
  st[0] = 0x6a09e667f3bcc908ULL; st[1] = 0xbb67ae8584caa73bULL; st[2] = 0x3c6ef372fe94f82bULL;
  st[3] = 0xa54ff53a5f1d36f1ULL; st[4] = 0x510e527fade682d1ULL; st[5] = 0x9b05688c2b3e6c1fULL;
  st[6] = 0x1f83d9abfb41bd6bULL; st[7] = 0x5be0cd19137e2179ULL;
}

// Round T of the compression, every index a constant: the a..h rotation is register renaming
// (the slot of a round's new a is the old h's, of its new e the old d's), rotations are
// v_alignbit_b32 pairs, the three-input XORs and the majority one v_bitop3_b32 per half, Ch a
// v_bfi_b32 per half.
template <int T>
MV_DEV void sha512_round(uint64_t (&v)[8], uint64_t (&w)[16]) {
  constexpr int j = T & 15, r = T & 7;
  if constexpr (T >= 16) {
    const uint64_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
    const uint64_t s0 = bitop3_64<0x96>(rotr64(w15, 1), rotr64(w15, 8), shr64(w15, 7));
    const uint64_t s1 = bitop3_64<0x96>(rotr64(w2, 19), rotr64(w2, 61), shr64(w2, 6));
    w[j] += s0 + w[(j + 9) & 15] + s1;
  }
  uint64_t& h = v[(15 - r) & 7];
  uint64_t& d = v[(11 - r) & 7];
  const uint64_t a = v[(8 - r) & 7], b = v[(9 - r) & 7], c = v[(10 - r) & 7];
  const uint64_t e = v[(12 - r) & 7], f = v[(13 - r) & 7], g = v[(14 - r) & 7];
  const uint64_t S1 = bitop3_64<0x96>(rotr64(e, 14), rotr64(e, 18), rotr64(e, 41));
  const uint64_t ch = (e & f) | (~e & g);
  const uint64_t t1 = h + S1 + ch + SHA512_K[T] + w[j];
  const uint64_t S0 = bitop3_64<0x96>(rotr64(a, 28), rotr64(a, 34), rotr64(a, 39));
  const uint64_t maj = bitop3_64<0xE8>(a, b, c);
  d += t1;            // the next round's e
  h = t1 + S0 + maj;  // the next round's a
}
template <int... T>
MV_DEV void sha512_rounds(uint64_t (&v)[8], uint64_t (&w)[16], std::integer_sequence<int, T...>) {
  (sha512_round<T>(v, w), ...);
}

// One compression; w[16] = the block as big-endian 64-bit words (clobbered). Straight-line
// code: 80 rounds with constant indices (the looped form kept the state in a register array
// indexed at run time and cost ~2.5x the instructions).
MV_DEV void sha512_compress(uint64_t st[8], uint64_t w_in[16]) {
  uint64_t v[8], w[16];
#pragma unroll
  for (int i = 0; i < 8; i++) v[i] = st[i];
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = w_in[i];
  sha512_rounds(v, w, std::make_integer_sequence<int, 80>{});
#pragma unroll
  for (int i = 0; i < 8; i++) st[i] += v[i];
}

// The same compression in plain 64-bit C++ (shifts for the rotations, no VALU-only intrinsics):
// called on wave-uniform values, it compiles to scalar-unit code (s_lshr_b64 / s_xor_b64 /
// s_add_u32 + s_addc_u32), which a lone wave issues about one per cycle, against one VALU
// instruction per 4 cycles -- the latency form for one signature (comb.hip's online job).
MV_DEV uint64_t rotr64s(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
template <int T>
MV_DEV void sha512s_round(uint64_t (&v)[8], uint64_t (&w)[16]) {
  constexpr int j = T & 15, r = T & 7;
  if constexpr (T >= 16) {
    const uint64_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
    const uint64_t s0 = rotr64s(w15, 1) ^ rotr64s(w15, 8) ^ (w15 >> 7);
    const uint64_t s1 = rotr64s(w2, 19) ^ rotr64s(w2, 61) ^ (w2 >> 6);
    w[j] += s0 + w[(j + 9) & 15] + s1;
  }
  uint64_t& h = v[(15 - r) & 7];
  uint64_t& d = v[(11 - r) & 7];
  const uint64_t a = v[(8 - r) & 7], b = v[(9 - r) & 7], c = v[(10 - r) & 7];
  const uint64_t e = v[(12 - r) & 7], f = v[(13 - r) & 7], g = v[(14 - r) & 7];
  const uint64_t S1 = rotr64s(e, 14) ^ rotr64s(e, 18) ^ rotr64s(e, 41);
  const uint64_t ch = (e & f) ^ (~e & g);
  const uint64_t t1 = h + S1 + ch + SHA512_K[T] + w[j];
  const uint64_t S0 = rotr64s(a, 28) ^ rotr64s(a, 34) ^ rotr64s(a, 39);
  const uint64_t maj = (a & b) | (c & (a | b));
  d += t1;
  h = t1 + S0 + maj;
}
template <int... T>
MV_DEV void sha512s_rounds(uint64_t (&v)[8], uint64_t (&w)[16], std::integer_sequence<int, T...>) {
  (sha512s_round<T>(v, w), ...);
}
// SHA-512 of 96 bytes given as 24 little-endian 32-bit words, all wave-uniform; out as
// sha512_short's (16 little-endian words of the digest)
MV_DEV void sha512s_96(uint32_t out[16], const uint32_t in[24]) {
  uint64_t w[16], v[8], st[8];
#pragma unroll
  for (int i = 0; i < 12; i++)
    w[i] = ((uint64_t)__builtin_bswap32(in[2 * i]) << 32) | __builtin_bswap32(in[2 * i + 1]);
  w[12] = 0x8000000000000000ull;
  w[13] = 0;
  w[14] = 0;
  w[15] = 96 * 8;
  sha512_init(st);
#pragma unroll
  for (int i = 0; i < 8; i++) v[i] = st[i];
  sha512s_rounds(v, w, std::make_integer_sequence<int, 80>{});
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t le = bswap64(st[i] + v[i]);
    out[2 * i] = (uint32_t)le;
    out[2 * i + 1] = (uint32_t)(le >> 32);
  }
}

// SHA-512 of up to 111 bytes given as little-endian 32-bit words (nbytes % 4 == 0);
// out = 16 little-endian 32-bit words of the 64-byte digest.
MV_DEV void sha512_short(uint32_t out[16], const uint32_t* in, int nbytes) {
  uint64_t w[16];
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = 0;
  // pack bytes big-endian into 64-bit words: word i = bytes 8i..8i+7
#pragma unroll
  for (int i = 0; i < 28; i++) {
    if (4 * i < nbytes) {
      uint32_t be = __builtin_bswap32(in[i]);
      if (i & 1) w[i >> 1] |= (uint64_t)be;
      else w[i >> 1] |= (uint64_t)be << 32;
    }
  }
  // padding: 0x80 after the message, bit length in the last word
  int pi = nbytes >> 3, pb = nbytes & 7;
#pragma unroll
  for (int i = 0; i < 14; i++)
    if (i == pi) w[i] |= 0x80ULL << (56 - 8 * pb);
  w[15] = (uint64_t)nbytes * 8;
  uint64_t st[8];
  sha512_init(st);
  sha512_compress(st, w);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t le = bswap64(st[i]);
    out[2 * i] = (uint32_t)le;
    out[2 * i + 1] = (uint32_t)(le >> 32);
  }
}

// ---------------- BLAKE2b ----------------
__constant__ const uint64_t B2_IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                        0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                        0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

MV_DEV void b2_init256(uint64_t h[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) h[i] = B2_IV[i];
  h[0] ^= 0x01010000ULL ^ 32ULL;  // depth 1, fanout 1, no key, 32-byte digest
}

#define MV_B2G(a, b, c, d, x, y)   \
  do {                             \
    v[a] = v[a] + v[b] + (x);      \
    v[d] = rotr64(v[d] ^ v[a], 32); \
    v[c] = v[c] + v[d];            \
    v[b] = rotr64(v[b] ^ v[c], 24); \
    v[a] = v[a] + v[b] + (y);      \
    v[d] = rotr64(v[d] ^ v[a], 16); \
    v[c] = v[c] + v[d];            \
    v[b] = rotr64(v[b] ^ v[c], 63); \
  } while (0)

#define MV_B2ROUND(s0, s1, s2, s3, s4, s5, s6, s7, s8, s9, s10, s11, s12, s13, s14, s15) \
  MV_B2G(0, 4, 8, 12, m[s0], m[s1]);                                                     \
  MV_B2G(1, 5, 9, 13, m[s2], m[s3]);                                                     \
  MV_B2G(2, 6, 10, 14, m[s4], m[s5]);                                                    \
  MV_B2G(3, 7, 11, 15, m[s6], m[s7]);                                                    \
  MV_B2G(0, 5, 10, 15, m[s8], m[s9]);                                                    \
  MV_B2G(1, 6, 11, 12, m[s10], m[s11]);                                                  \
  MV_B2G(2, 7, 8, 13, m[s12], m[s13]);                                                   \
  MV_B2G(3, 4, 9, 14, m[s14], m[s15]);

// m[16] little-endian message words; t = bytes hashed so far incl. this block
MV_DEV void b2_compress(uint64_t h[8], const uint64_t m[16], uint64_t t, bool last) {
  uint64_t v[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    v[i] = h[i];
    v[i + 8] = B2_IV[i];
  }
  v[12] ^= t;
  v[14] = last ? ~v[14] : v[14];
  MV_B2ROUND(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  MV_B2ROUND(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3)
  MV_B2ROUND(11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4)
  MV_B2ROUND(7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8)
  MV_B2ROUND(9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13)
  MV_B2ROUND(2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9)
  MV_B2ROUND(12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11)
  MV_B2ROUND(13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10)
  MV_B2ROUND(6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5)
  MV_B2ROUND(10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0)
  MV_B2ROUND(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  MV_B2ROUND(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3)
#pragma unroll
  for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[i + 8];
}

}  // namespace mv
