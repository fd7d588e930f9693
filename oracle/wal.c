/* ORACLE / TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement of the reference's WAL replay check:
 *   - crc32fast 1.3.2 `hash` (Cargo.lock:777, used at mysticeti-core/src/wal.rs:173-177 and :250):
 *     CRC-32/ISO-HDLC -- reflected polynomial 0xEDB88320, initial value and final xor 0xFFFFFFFF.
 *     Restated byte at a time from a 256-entry table (the textbook form of the same CRC);
 *     pinned to zlib.crc32 by tests/golden/wal.json.
 *   - WalWriter::writev position arithmetic (wal.rs:150-188): an entry of v_len payload bytes takes
 *     len = v_len + 16 bytes; if it would straddle a map boundary (offset(pos) != offset(pos+len-1))
 *     the writer first pads with zeros up to the boundary.
 *   - header (wal.rs:211-223): 16 bytes little-endian u128 = crc (u64) | len (u32) << 64 | tag (u32) << 96.
 *   - WalIterator::next / try_position (wal.rs:314-346) over WalReader::try_read (wal.rs:233-261):
 *       position >= end_position              -> end of iteration
 *       fewer than 16 bytes left in the map   -> no entry here (read_header None, wal.rs:297-300)
 *       len == 0 and crc == 0                 -> no entry here
 *       len == 0 and crc != 0                 -> panic "Non-zero crc at len 0"      (status 2)
 *       len < 16 or entry past its map        -> panic in Bytes::slice (wal.rs:249)  (status 3)
 *       crc32(payload) != crc                 -> panic "Crc mismatch"               (status 1)
 *     "no entry here": at the first position of a map the iteration ends; elsewhere it retries
 *     once at the start of the next map (wal.rs:321-330).
 *   The reference panics at the first failing entry; the restatement reports it (with its
 *   status) as the last entry and stops.
 * Bytes at or past `size` read as zero (the mapping's tail past the end of the file).
 */
#include <stdint.h>
#include <string.h>

#include "oracle.h"

#if defined(__x86_64__)
#include <immintrin.h>
#endif

static uint32_t crc_table[256];
static int crc_table_ready;

__attribute__((constructor)) static void crc_init(void) {  /* at load: no race between pool threads */
  if (crc_table_ready) return;
  for (uint32_t b = 0; b < 256; b++) {
    uint32_t c = b;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
    crc_table[b] = c;
  }
  crc_table_ready = 1;
}

static uint32_t crc_bytes(uint32_t c, const uint8_t* p, size_t n) {
  for (size_t i = 0; i < n; i++) c = (c >> 8) ^ crc_table[(c ^ p[i]) & 0xff];
  return c;
}

uint32_t orc_crc32_table(const uint8_t* p, size_t n) { return crc_bytes(0xFFFFFFFFu, p, n) ^ 0xFFFFFFFFu; }

#if defined(__x86_64__)
/* crc32fast 1.3.2's x86_64 path (specialized::pclmulqdq, selected at run time when the CPU has
 * PCLMULQDQ and SSE4.1): the register is folded 64 bytes at a time with carry-less multiplies,
 * then reduced to 32 bits (Barrett). Restated from the published method (Gopal et al., "Fast
 * CRC Computation for Generic Polynomials Using PCLMULQDQ Instruction", Intel 2009) with its
 * bit-reflected constants for the CRC-32 polynomial. Takes and returns the raw register;
 * n >= 64 and a multiple of 16. */
__attribute__((target("pclmul,sse4.1"))) static uint32_t crc_fold(uint32_t crc, const uint8_t* buf, size_t len) {
  const __m128i k1k2 = _mm_set_epi64x(0x01c6e41596ll, 0x0154442bd4ll);
  const __m128i k3k4 = _mm_set_epi64x(0x00ccaa009ell, 0x01751997d0ll);
  const __m128i k5k0 = _mm_set_epi64x(0, 0x0163cd6124ll);
  const __m128i poly = _mm_set_epi64x(0x01f7011641ll, 0x01db710641ll);
  __m128i x0, x1, x2, x3, x4, x5, x6, x7, x8;
  x1 = _mm_loadu_si128((const __m128i*)(buf + 0x00));
  x2 = _mm_loadu_si128((const __m128i*)(buf + 0x10));
  x3 = _mm_loadu_si128((const __m128i*)(buf + 0x20));
  x4 = _mm_loadu_si128((const __m128i*)(buf + 0x30));
  x1 = _mm_xor_si128(x1, _mm_cvtsi32_si128((int)crc));
  x0 = k1k2;
  buf += 64;
  len -= 64;
  while (len >= 64) {  /* four independent 128-bit lanes, each folded 512 bits forward */
    x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
    x6 = _mm_clmulepi64_si128(x2, x0, 0x00);
    x7 = _mm_clmulepi64_si128(x3, x0, 0x00);
    x8 = _mm_clmulepi64_si128(x4, x0, 0x00);
    x1 = _mm_clmulepi64_si128(x1, x0, 0x11);
    x2 = _mm_clmulepi64_si128(x2, x0, 0x11);
    x3 = _mm_clmulepi64_si128(x3, x0, 0x11);
    x4 = _mm_clmulepi64_si128(x4, x0, 0x11);
    x1 = _mm_xor_si128(_mm_xor_si128(x1, x5), _mm_loadu_si128((const __m128i*)(buf + 0x00)));
    x2 = _mm_xor_si128(_mm_xor_si128(x2, x6), _mm_loadu_si128((const __m128i*)(buf + 0x10)));
    x3 = _mm_xor_si128(_mm_xor_si128(x3, x7), _mm_loadu_si128((const __m128i*)(buf + 0x20)));
    x4 = _mm_xor_si128(_mm_xor_si128(x4, x8), _mm_loadu_si128((const __m128i*)(buf + 0x30)));
    buf += 64;
    len -= 64;
  }
  x0 = k3k4;  /* fold the four lanes into one (128 bits forward each) */
  x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
  x1 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x1, x0, 0x11), x2), x5);
  x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
  x1 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x1, x0, 0x11), x3), x5);
  x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
  x1 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x1, x0, 0x11), x4), x5);
  while (len >= 16) {
    x2 = _mm_loadu_si128((const __m128i*)buf);
    x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
    x1 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x1, x0, 0x11), x2), x5);
    buf += 16;
    len -= 16;
  }
  /* 128 -> 64 bits */
  x2 = _mm_clmulepi64_si128(x1, x0, 0x10);
  x3 = _mm_setr_epi32(~0, 0, ~0, 0);
  x1 = _mm_xor_si128(_mm_srli_si128(x1, 8), x2);
  x0 = k5k0;
  x2 = _mm_srli_si128(x1, 4);
  x1 = _mm_and_si128(x1, x3);
  x1 = _mm_xor_si128(_mm_clmulepi64_si128(x1, x0, 0x00), x2);
  /* Barrett reduction to 32 bits */
  x0 = poly;
  x2 = _mm_and_si128(x1, x3);
  x2 = _mm_clmulepi64_si128(x2, x0, 0x10);
  x2 = _mm_and_si128(x2, x3);
  x2 = _mm_clmulepi64_si128(x2, x0, 0x00);
  x1 = _mm_xor_si128(x1, x2);
  return (uint32_t)_mm_extract_epi32(x1, 1);
}
static int have_pclmul(void) {
  static int v = -1;
  if (v < 0) v = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
  return v;
}
#endif

/* crc32fast::hash: the folded path for >= 64 bytes where the CPU has it, bytes for the rest */
uint32_t orc_crc32(const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
#if defined(__x86_64__)
  if (n >= 64 && have_pclmul()) {
    const size_t m = n & ~(size_t)15;
    c = crc_fold(c, p, m);
    p += m;
    n -= m;
  }
#endif
  return crc_bytes(c, p, n) ^ 0xFFFFFFFFu;
}

void orc_crc32_batch(const uint8_t* buf, const uint64_t* off, const uint64_t* len, size_t n, uint32_t* out) {
  for (size_t i = 0; i < n; i++) out[i] = orc_crc32(buf + off[i], len[i]);
}

uint64_t orc_wal_layout(const uint64_t* payload_len, size_t n, uint32_t map_bits, uint64_t start, uint64_t* pos) {
  const uint64_t mask = ~((1ull << map_bits) - 1);
  uint64_t p = start;
  for (size_t i = 0; i < n; i++) {
    const uint64_t len = payload_len[i] + 16;
    if ((p & mask) != ((p + len - 1) & mask)) p = (p + len - 1) & mask;  /* zero padding to the boundary */
    pos[i] = p;
    p += len;
  }
  return p;
}

static uint8_t byte_at(const uint8_t* img, uint64_t size, uint64_t i) { return i < size ? img[i] : 0; }

static uint64_t le64_at(const uint8_t* img, uint64_t size, uint64_t i) {
  uint64_t v = 0;
  for (int k = 7; k >= 0; k--) v = (v << 8) | byte_at(img, size, i + (uint64_t)k);
  return v;
}

/* try_read: 0 = no entry, 1 = entry (status in *st) */
static int try_read(const uint8_t* img, uint64_t size, uint32_t map_bits, uint64_t p, uint32_t* tag, uint32_t* plen,
                    uint8_t* st) {
  const uint64_t msize = 1ull << map_bits, base = p & ~(msize - 1), boff = p - base;
  if (msize - boff < 16) return 0;
  const uint64_t crc = le64_at(img, size, p), hi = le64_at(img, size, p + 8);
  const uint64_t len = hi & 0xffffffffull;
  *tag = (uint32_t)(hi >> 32);
  *plen = 0;
  if (len == 0) {
    if (crc == 0) return 0;
    *st = ORC_WAL_NONZERO_CRC_LEN0;
    return 1;
  }
  if (len < 16 || boff + len > msize) {
    *st = ORC_WAL_BAD_LENGTH;
    return 1;
  }
  *plen = (uint32_t)(len - 16);
  uint32_t c;
  if (p + len <= size) {
    c = orc_crc32(img + p + 16, len - 16);
  } else {  /* payload runs past the image: zeros */
    c = 0xFFFFFFFFu;
    for (uint64_t i = p + 16; i < p + len; i++) c = (c >> 8) ^ crc_table[(c ^ byte_at(img, size, i)) & 0xff];
    c ^= 0xFFFFFFFFu;
  }
  *st = (uint64_t)c == crc ? ORC_WAL_OK : ORC_WAL_CRC_MISMATCH;
  return 1;
}

uint64_t orc_wal_iter(const uint8_t* img, uint64_t size, uint64_t end_pos, uint32_t map_bits, uint64_t* pos,
                      uint32_t* tag, uint32_t* len, uint8_t* status, uint64_t cap) {
  const uint64_t msize = 1ull << map_bits;
  uint64_t count = 0, p = 0;
  for (;;) {
    uint32_t t, l;
    uint8_t st = ORC_WAL_OK;
    int got = 0;
    uint64_t at = p;
    if (at < end_pos) got = try_read(img, size, map_bits, at, &t, &l, &st);
    if (!got && at < end_pos && (at & (msize - 1)) != 0) {  /* retry once at the next map */
      at = (at & ~(msize - 1)) + msize;
      if (at < end_pos) got = try_read(img, size, map_bits, at, &t, &l, &st);
    }
    if (!got) break;
    if (count < cap) {
      pos[count] = at;
      tag[count] = t;
      len[count] = l;
      status[count] = st;
    }
    count++;
    if (st != ORC_WAL_OK) break;  /* the reference panics here */
    p = at + (uint64_t)l + 16;
  }
  return count;
}
