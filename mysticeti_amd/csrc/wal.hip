// WAL replay check on gfx950: crc32fast::hash (CRC-32/ISO-HDLC) of
// every WAL entry's payload, and the entry walk of WalIterator (mysticeti-core/src/wal.rs:
// 226-346) over a WAL image in HBM.
//
// CRC: one wave per byte string D = [a, b). The string is cut into rows of 256 bytes that
// END at b (the first row is padded in front); lane l owns 32-bit word l of every row and
// folds its words by Horner with the linear map "advance 256 bytes":
//     u_l <- A256(u_l) ^ w_{l,j}
// so u_l = XOR_j shift(w_{l,j}, 256 (R-1-j)). The lanes then combine in a 6-level tree
// (shifts by 4, 8, ..., 128 bytes) and a final 4-byte shift. Every shift is a GF(2)-linear
// map applied as four 256-entry table lookups (one per state byte). The initial value
// 0xFFFFFFFF is folded in as a 4-byte prefix P with crc_raw(0, P) = 0xFFFFFFFF placed just
// before a (zeros before it change nothing from state 0), so no per-string variable shift
// is needed. Unaligned b: each lane reads the two aligned dwords around its word and
// funnel-shifts them (v_alignbyte_b32).
// Tables in LDS: A256 (the hot one, 4 x 256 words) replicated 8 times so that lanes l and
// l' with l != l' (mod 8) never hit one bank; the tree's six maps once (56 KiB in all, one
// copy per 1024-thread workgroup, two workgroups per CU). The kernel is bound by HBM latency,
// not by the LDS: 32 bank-aligned copies (no conflicts at all, 152 KiB, one workgroup per CU)
// measured 3.18 ms per 2^20 entries and 16 copies 2.52, against 2.31 for this form at 8 waves
// per SIMD (profiles/r04/wal/ab_tables_occupancy_r04p.txt).
//
// Walk: one lane per map of 2^map_bits bytes. Every map that holds entries starts with one
// (the writer pads an entry that would straddle a map, wal.rs:155-167), so maps walk
// independently; the host then joins them in the reference's iteration order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mysti_verify.h"
#include "kernels.h"

#ifndef MV_DEV
#define MV_DEV __device__ __forceinline__
#endif

namespace mv {
namespace wal {

#ifndef MV_WAL_REP
#define MV_WAL_REP 8
#endif
constexpr int REP = MV_WAL_REP;              // copies of A256 (bank spread)
constexpr int A_WORDS = 4 * 256 * REP;       // [byte t][value e][copy c]
constexpr int S_LEVELS = 6;                  // shifts by 4 << k bytes, k < 6
constexpr int S_WORDS = S_LEVELS * 4 * 256;  // [k][byte t][value e]
constexpr int T_WORDS = 256;                 // the byte table (1-byte shift), global only
constexpr uint32_t PREFIX = 0x9226f562u;     // crc_raw(0, PREFIX as 4 LE bytes) = 0xFFFFFFFF
constexpr int WG = 1024;                     // threads per crc workgroup
#ifndef MV_WAL_ROWS
#define MV_WAL_ROWS 8  // rows in flight per batch; 8 fits the 64-VGPR budget of 8 waves per SIMD
#endif
constexpr int WAL_ROWS = MV_WAL_ROWS;
#ifndef MV_WAL_WPE
#define MV_WAL_WPE 8  // waves per SIMD the register budget is cut for: two 1024-thread workgroups per CU
#endif
#define MV_WAL_ATTR __attribute__((amdgpu_waves_per_eu(MV_WAL_WPE)))        // 256-B rows in flight per wave

// a wave-uniform 64-bit value from lane 0
MV_DEV uint64_t bcast64(uint64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x), hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
  return ((uint64_t)hi << 32) | lo;
}

struct Lds {
  uint32_t a[A_WORDS];
#ifndef MV_WAL_SGLOBAL
  uint32_t s[S_WORDS];
#endif
};

MV_DEV void lds_fill(Lds& L, const uint32_t* __restrict__ tables) {
  for (int i = threadIdx.x; i < A_WORDS + S_WORDS; i += blockDim.x) {
    if (i < A_WORDS) L.a[i] = tables[i];
#ifndef MV_WAL_SGLOBAL
    else L.s[i - A_WORDS] = tables[i];
#endif
  }
  __syncthreads();
}

MV_DEV uint32_t adv256(const Lds& L, uint32_t u, uint32_t c) {
  return L.a[(0 * 256 + (u & 255)) * REP + c] ^ L.a[(1 * 256 + ((u >> 8) & 255)) * REP + c] ^
         L.a[(2 * 256 + ((u >> 16) & 255)) * REP + c] ^ L.a[(3 * 256 + (u >> 24)) * REP + c];
}
// the tree's shift maps: in LDS, or (MV_WAL_SGLOBAL) read through the caches
MV_DEV const uint32_t* s_tab(const Lds& L, const uint32_t* __restrict__ tables) {
#ifdef MV_WAL_SGLOBAL
  return tables + A_WORDS;
#else
  return L.s;
#endif
}
MV_DEV uint32_t shiftk(const uint32_t* S, int k, uint32_t u) {
  const uint32_t* s = S + k * 1024;
  return s[u & 255] ^ s[256 + ((u >> 8) & 255)] ^ s[512 + ((u >> 16) & 255)] ^ s[768 + (u >> 24)];
}
MV_DEV uint32_t ld32(const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); }  // (nt loads: no gain)

// crc_raw(0xFFFFFFFF, base[a, b)) (the CRC register before the final xor), on the whole wave.
// Reads only the aligned dwords that hold bytes of [a, b).
MV_DEV uint32_t crc_raw_wave(const uint8_t* __restrict__ base, uint64_t a, uint64_t b, const Lds& L,
                              const uint32_t* S) {
  const uint32_t lane = threadIdx.x & 63, c = lane & (REP - 1);
  const uint64_t len = b - a;
  const uint64_t R = (len + 4 + 255) / 256;
  const uint32_t sh = (uint32_t)(b & 3);
  const int64_t a4 = (int64_t)(a & ~3ull);
  const uint64_t Z = (uint64_t)PREFIX << 32;  // virtual bytes a-8 .. a-1: 0 0 0 0 P0 P1 P2 P3
  uint32_t u = 0;
  // rows 0, 1: may hold bytes before a (zeros, then the prefix P); their loads go out first
  uint32_t w01[2] = {0u, 0u};
  int64_t q01[2];
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const int64_t x = (int64_t)b - 256 * (int64_t)(R - j) + 4 * (int64_t)lane;
    q01[j] = x - (int64_t)a;
    if ((uint64_t)j < R && q01[j] > -4) {
      const int64_t xa = x - sh;
      const uint32_t A = xa >= a4 ? ld32(base + xa) : 0u;
      const uint32_t B = sh ? ld32(base + xa + 4) : 0u;
      w01[j] = sh ? __builtin_amdgcn_alignbyte(B, A, sh) : A;
    }
  }
  // rows 2 .. R-1 in batches of WAL_ROWS loads in flight (the kernel is bound by HBM latency:
  // ~1-2 us per round trip, so each lane keeps a batch outstanding); the last batch is partial,
  // its rows past R neither loaded nor folded: one round trip, not one per leftover row
  const uint8_t* pr = base + (int64_t)b - 256 * (int64_t)(R - 2) + 4 * (int64_t)lane - sh;
  for (uint64_t j0 = 2;; j0 += WAL_ROWS, pr += 256 * WAL_ROWS) {
    uint32_t A[WAL_ROWS], B[WAL_ROWS];
#pragma unroll
    for (int k = 0; k < WAL_ROWS; k++) {
      const bool live = j0 + k < R;  // wave-uniform
      A[k] = live ? ld32(pr + 256 * k) : 0u;
      B[k] = live && sh ? ld32(pr + 256 * k + 4) : 0u;
    }
    if (j0 == 2) {
#pragma unroll
      for (int j = 0; j < 2; j++) {
        if ((uint64_t)j >= R) break;
        uint32_t w = w01[j];
        const int64_t q = q01[j];
        if (q < 0) {
          const uint32_t keep = q <= -4 ? 0u : (0xffffffffu << (8 * (uint32_t)(-q)));
          w = q < -8 ? 0u : ((w & keep) | (uint32_t)(Z >> (8 * (q + 8))));
        }
        u = adv256(L, u, c) ^ w;
      }
    }
#pragma unroll
    for (int k = 0; k < WAL_ROWS; k++)
      if (j0 + k < R) u = adv256(L, u, c) ^ (sh ? __builtin_amdgcn_alignbyte(B[k], A[k], sh) : A[k]);
    if (j0 + WAL_ROWS >= R) break;
  }
  // lanes: val over [g, g + 2^(k+1)) = shift(val[g, g + 2^k), 4 * 2^k) ^ val[g + 2^k, ...)
#pragma unroll
  for (int k = 0; k < S_LEVELS; k++) {
    const uint32_t v = (uint32_t)__shfl_down((int)u, 1 << k);
    if ((lane & ((2u << k) - 1)) == 0) u = shiftk(S, k, u) ^ v;
  }
  u = shiftk(S, 0, u);  // lane 63's word ends 4 bytes before the end
  return (uint32_t)__shfl((int)u, 0);
}

// state <- state advanced over n zero bytes (crc_raw(state, 0^n)); rare paths only
MV_DEV uint32_t zeros_shift(const Lds& L, const uint32_t* S, const uint32_t* __restrict__ tbyte, uint32_t s,
                            uint64_t n) {
  const uint32_t c = threadIdx.x & (REP - 1);
  for (; n >= 256; n -= 256) s = adv256(L, s, c);
  for (int k = S_LEVELS - 1; k >= 0; k--)
    if (n >= (4u << k)) {
      s = shiftk(S, k, s);
      n -= 4u << k;
    }
  for (; n; n--) s = (s >> 8) ^ tbyte[s & 255];
  return s;
}

// ------------------------------------------------------------------ crc32 of n strings
__global__ void __launch_bounds__(WG) MV_WAL_ATTR k_crc32_batch(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ off,
                                                    const uint64_t* __restrict__ len, uint32_t n,
                                                    const uint32_t* __restrict__ tables, uint32_t* __restrict__ out) {
  __shared__ Lds L;
  lds_fill(L, tables);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t waves = gridDim.x * (WG / 64);
  for (uint32_t i = blockIdx.x * (WG / 64) + threadIdx.x / 64; i < n; i += waves) {
    const uint64_t a = bcast64(off[i]), b = a + bcast64(len[i]);
    const uint32_t r = crc_raw_wave(buf, a, b, L, s_tab(L, tables));
    if (lane == 0) out[i] = ~r;
  }
}

// ------------------------------------------------------------------ WAL walk
// map flags (the iteration after this map's entries)
// EMPTY: no entry at the map start, the iteration ends before the map; NEXT: it continues at
// the next map's start; END: it reached end_pos; BAD: the last record failed (a reference panic)
constexpr uint8_t MAP_EMPTY = mvk::WAL_MAP_EMPTY, MAP_NEXT = mvk::WAL_MAP_NEXT, MAP_END = mvk::WAL_MAP_END,
                  MAP_BAD = mvk::WAL_MAP_BAD;

MV_DEV uint64_t le64_bounded(const uint8_t* img, uint64_t size, uint64_t p) {
  if (p + 8 <= size) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(img + (p & ~3ull));
    const uint32_t s = (uint32_t)(p & 3);
    const uint32_t w0 = w[0], w1 = w[1], w2 = s ? w[2] : 0u;
    const uint32_t lo = s ? __builtin_amdgcn_alignbyte(w1, w0, s) : w0;
    const uint32_t hi = s ? __builtin_amdgcn_alignbyte(w2, w1, s) : w1;
    return ((uint64_t)hi << 32) | lo;
  }
  uint64_t v = 0;
  for (int k = 7; k >= 0; k--) v = (v << 8) | (p + k < size ? img[p + k] : 0u);
  return v;
}

// record = position | status << 60 (status: MV_WAL_OK for an entry whose crc is still to check)
// The walk is a chain of dependent header reads (~1 us of HBM latency each, ~1,800 per 16-MiB map
// of config-4 blocks). It runs ahead speculatively: the headers at p + k * stride, k < WALK_AHEAD,
// are loaded together, stride = the last entry's length (WAL entries of one kind share a length);
// they are then consumed in order while each entry's length equals the stride, and the walk
// re-aims at the first that differs. The checks, records and flags are those of the one-at-a-time
// walk (wal.rs:285-346) in the same order; a mispredicted header is never used.
constexpr int WALK_AHEAD = 8;
// a header's 16 bytes at q as five aligned dwords, loaded without a branch (so the run-ahead
// loads are all in flight together); `fast` false (the header would reach past the image, or the
// image is shorter than 20 bytes): the consumer reads it byte-wise (le64_bounded)
struct WalkHdr {
  uint32_t w[5];
  bool fast;
};
MV_DEV void hdr_load(WalkHdr& h, const uint8_t* img, uint64_t size, uint64_t q) {
  h.fast = size >= 20 && q <= size - 20;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(img + (h.fast ? (q & ~3ull) : 0ull));
#pragma unroll
  for (int i = 0; i < 5; i++) h.w[i] = w[i];
}
MV_DEV void hdr_get(const WalkHdr& h, const uint8_t* img, uint64_t size, uint64_t q, uint64_t& crc, uint64_t& hi) {
  if (h.fast) {
    const uint32_t s = (uint32_t)(q & 3);
    auto fn = [&](int i) { return s ? __builtin_amdgcn_alignbyte(h.w[i + 1], h.w[i], s) : h.w[i]; };
    crc = ((uint64_t)fn(1) << 32) | fn(0);
    hi = ((uint64_t)fn(3) << 32) | fn(2);
  } else {
    crc = le64_bounded(img, size, q);
    hi = le64_bounded(img, size, q + 8);
  }
}
__global__ void __launch_bounds__(64) k_wal_walk(const uint8_t* __restrict__ img, uint64_t size, uint64_t end_pos,
                                                 uint32_t map_bits, uint32_t nmaps, uint32_t cap_pm,
                                                 const uint64_t* __restrict__ moff,
                                                 unsigned long long* __restrict__ rec, uint32_t* __restrict__ mcount,
                                                 uint8_t* __restrict__ mflag) {
  const uint32_t m = blockIdx.x * 64 + threadIdx.x;
  if (m >= nmaps) return;
  const uint64_t msize = 1ull << map_bits, start = (uint64_t)m << map_bits;
  uint64_t p = start, stride = 0;
  uint32_t count = 0;
  uint8_t flag = MAP_NEXT;
  // moff (the second walk): map m's records at rec + moff[m], as many as the first walk counted
  unsigned long long* r = moff ? rec + moff[m] : rec + (size_t)m * cap_pm;
  if (moff) cap_pm = mcount[m];
  bool done = false, have_next = false;
  WalkHdr hd[WALK_AHEAD], hn[WALK_AHEAD];
  while (!done) {
    if (have_next) {
#pragma unroll
      for (int k = 0; k < WALK_AHEAD; k++) hd[k] = hn[k];
    } else {
#pragma unroll
      for (int k = 0; k < WALK_AHEAD; k++) hdr_load(hd[k], img, size, p + (uint64_t)k * stride);
    }
    const int ahead = stride ? WALK_AHEAD : 1;
    // the round after this one, in flight while this one is consumed (it is used only if all of
    // this round's entries have the stride)
    have_next = stride != 0;
    if (have_next) {
#pragma unroll
      for (int k = 0; k < WALK_AHEAD; k++) hdr_load(hn[k], img, size, p + (uint64_t)(WALK_AHEAD + k) * stride);
    }
#pragma unroll
    for (int k = 0; k < WALK_AHEAD; k++) {
      if (k >= ahead) break;
      // the entry at p (= the k-th speculative position: the lengths so far equal the stride)
      if (p >= end_pos) {
        flag = p == start ? MAP_EMPTY : MAP_END;
        done = true;
        break;
      }
      const uint64_t boff = p - start;
      if (msize - boff < 16) {  // no room for a header (wal.rs:297-300)
        flag = MAP_NEXT;
        done = true;
        break;
      }
      uint64_t crc, hi;
      hdr_get(hd[k], img, size, p, crc, hi);
      const uint64_t len = hi & 0xffffffffull;
      if (len == 0) {
        if (crc == 0) {
          flag = boff == 0 ? MAP_EMPTY : MAP_NEXT;
        } else {
          if (count < cap_pm) r[count] = p | ((unsigned long long)MV_WAL_NONZERO_CRC_LEN0 << 60);
          count++;
          flag = MAP_BAD;
        }
        done = true;
        break;
      }
      if (len < 16 || boff + len > msize) {
        if (count < cap_pm) r[count] = p | ((unsigned long long)MV_WAL_BAD_LENGTH << 60);
        count++;
        flag = MAP_BAD;
        done = true;
        break;
      }
      if (count < cap_pm) r[count] = p;
      count++;
      p += len;
      if (len != stride) {  // the next speculative header is not at p: re-aim
        stride = len;
        have_next = false;
        break;
      }
    }
  }
  mcount[m] = count;
  mflag[m] = flag;
}

// records of map m -> entries [moff[m], moff[m] + mcount[m])
__global__ void __launch_bounds__(256) k_wal_compact(const unsigned long long* __restrict__ rec, uint32_t cap_pm,
                                                     const uint32_t* __restrict__ mcount,
                                                     const uint64_t* __restrict__ moff,
                                                     unsigned long long* __restrict__ ent) {
  const uint32_t m = blockIdx.x;
  const uint32_t c = mcount[m];
  const uint64_t o = moff[m];
  for (uint32_t i = threadIdx.x; i < c; i += 256) ent[o + i] = rec[(size_t)m * cap_pm + i];
}

// one wave per entry: header, crc of the payload, verdict; the first failing entry index
// goes to *first_fail (atomic min)
__global__ void __launch_bounds__(WG) MV_WAL_ATTR k_wal_crc(const uint8_t* __restrict__ img, uint64_t size,
                                                const unsigned long long* __restrict__ ent, uint64_t total,
                                                const uint32_t* __restrict__ tables, uint64_t* __restrict__ out_pos,
                                                uint32_t* __restrict__ out_tag, uint32_t* __restrict__ out_len,
                                                uint8_t* __restrict__ out_status, uint64_t cap,
                                                unsigned long long* __restrict__ first_fail) {
  __shared__ Lds L;
  lds_fill(L, tables);
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t waves = (uint64_t)gridDim.x * (WG / 64);
  const uint32_t* tbyte = tables + A_WORDS + S_WORDS;
  const uint32_t* S = s_tab(L, tables);
  for (uint64_t e = blockIdx.x * (WG / 64) + threadIdx.x / 64; e < total; e += waves) {
    const uint64_t r = bcast64(ent[e]);
    const uint64_t p = r & ((1ull << 60) - 1);
    uint32_t st = (uint32_t)(r >> 60);
    const uint64_t crc = bcast64(le64_bounded(img, size, p)), hi = bcast64(le64_bounded(img, size, p + 8));
    const uint64_t len = hi & 0xffffffffull;
    const uint32_t tag = (uint32_t)(hi >> 32);
    uint32_t plen = 0;
    if (st == MV_WAL_OK) {
      plen = (uint32_t)(len - 16);
      const uint64_t a = p + 16, b = p + len;
      uint32_t raw;
      if (b <= size) {
        raw = crc_raw_wave(img, a, b, L, S);
      } else {  // the file ends inside the payload: the rest reads as zeros
        raw = a < size ? crc_raw_wave(img, a, size, L, S) : 0xffffffffu;
        raw = zeros_shift(L, S, tbyte, raw, b - (a < size ? size : a));
      }
      st = (uint64_t)(~raw) == crc ? MV_WAL_OK : MV_WAL_CRC_MISMATCH;
    }
    if (lane == 0) {
      if (e < cap) {
        out_pos[e] = p;
        out_tag[e] = tag;
        out_len[e] = plen;
        out_status[e] = (uint8_t)st;
      }
      if (st != MV_WAL_OK) atomicMin(first_fail, (unsigned long long)e);
    }
  }
}

}  // namespace wal
}  // namespace mv

namespace mvk {

size_t wal_table_words() { return mv::wal::A_WORDS + mv::wal::S_WORDS + mv::wal::T_WORDS; }

// host: A256 (replicated), the tree shifts, the byte table
void wal_build_tables(uint32_t* out) {
  using namespace mv::wal;
  uint32_t T[256];
  for (uint32_t b = 0; b < 256; b++) {
    uint32_t c = b;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
    T[b] = c;
  }
  auto shift = [&](uint32_t s, int n) {
    for (int i = 0; i < n; i++) s = (s >> 8) ^ T[s & 255];
    return s;
  };
  for (int t = 0; t < 4; t++)
    for (int e = 0; e < 256; e++) {
      const uint32_t v = shift((uint32_t)e << (8 * t), 256);
      for (int c = 0; c < REP; c++) out[(t * 256 + e) * REP + c] = v;
    }
  for (int k = 0; k < S_LEVELS; k++)
    for (int t = 0; t < 4; t++)
      for (int e = 0; e < 256; e++) out[A_WORDS + k * 1024 + t * 256 + e] = shift((uint32_t)e << (8 * t), 4 << k);
  for (int e = 0; e < 256; e++) out[A_WORDS + S_WORDS + e] = T[e];
}

static uint32_t crc_grid(uint64_t items, int cus) {
  const uint64_t per_wg = mv::wal::WG / 64;
  uint64_t g = (items + per_wg - 1) / per_wg;
  const uint64_t cap = (uint64_t)(163840 / sizeof(mv::wal::Lds)) * (uint64_t)cus;  // 1024-thread workgroups per CU (LDS)
  return (uint32_t)(g < 1 ? 1 : (g > cap ? cap : g));
}

hipError_t launch_crc32(const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n,
                        const uint32_t* tables, uint32_t* out, int cus, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(mv::wal::k_crc32_batch, dim3(crc_grid(n, cus)), dim3(mv::wal::WG), 0, s, buf, off, len, n,
                     tables, out);
  return hipGetLastError();
}

hipError_t launch_wal_walk(const uint8_t* img, uint64_t size, uint64_t end_pos, uint32_t map_bits, uint32_t nmaps,
                           uint32_t cap_pm, const uint64_t* moff, unsigned long long* rec, uint32_t* mcount,
                           uint8_t* mflag, hipStream_t s) {
  if (nmaps == 0) return hipSuccess;
  hipLaunchKernelGGL(mv::wal::k_wal_walk, dim3((nmaps + 63) / 64), dim3(64), 0, s, img, size, end_pos, map_bits, nmaps,
                     cap_pm, moff, rec, mcount, mflag);
  return hipGetLastError();
}

hipError_t launch_wal_compact(const unsigned long long* rec, uint32_t cap_pm, const uint32_t* mcount,
                              const uint64_t* moff, uint32_t nmaps, unsigned long long* ent, hipStream_t s) {
  if (nmaps == 0) return hipSuccess;
  hipLaunchKernelGGL(mv::wal::k_wal_compact, dim3(nmaps), dim3(256), 0, s, rec, cap_pm, mcount, moff, ent);
  return hipGetLastError();
}

hipError_t launch_wal_crc(const uint8_t* img, uint64_t size, const unsigned long long* ent, uint64_t total,
                          const uint32_t* tables, uint64_t* out_pos, uint32_t* out_tag, uint32_t* out_len,
                          uint8_t* out_status, uint64_t cap, unsigned long long* first_fail, int cus, hipStream_t s) {
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(mv::wal::k_wal_crc, dim3(crc_grid(total, cus)), dim3(mv::wal::WG), 0, s, img, size, ent, total,
                     tables, out_pos, out_tag, out_len, out_status, cap, first_fail);
  return hipGetLastError();
}

}  // namespace mvk
