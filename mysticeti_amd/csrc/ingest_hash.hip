// Fused device ingest + BLAKE2b for the block path:
// bincode Data<StatementBlock> bytes in HBM -> the signed pre-image, both digests, and the
// facts StatementBlock::verify checks, without staging the pre-image in HBM.
//
// k_block_ingest (ingest.hip) + k_b2_quad (blake2b_quad.hip) write the 8 KB pre-image of a
// config-4 block to HBM and read it back: 2.85x the bincode's bytes. Here one QUAD (four lanes)
// owns a block from its first bincode byte to its digests, 16 blocks per 64-lane workgroup:
//
//   bincode ring   4 lines of 128 B per quad in LDS; every step the quad loads up to two more
//                  lines (16-B loads, 32 B per lane), issued before the compression and stored
//                  after it, so the HBM latency hides behind the hash
//   transcoder     parses the block from the ring in the reference's order and emits its
//                  pre-image (crypto.rs:85-128, types.rs:661-691, 751-755) into a 2-block
//                  pre-image ring. Every piece of the pre-image is an optional tag byte
//                  followed by dwords taken from the bincode (byte-swapped for the big-endian
//                  integers): the quad's lanes write output dwords j = q, q + 4, ... as
//                  alignbyte(F[j], F[j-1]) at the stream's byte offset
//   hash           compress<1, LIN> of blake2b_quad.h straight from the pre-image ring (one
//                  column of the state per lane, SIGMA words at linear offsets; the ring's
//                  quad stride of 36 u64 measures 1.98 LDS cycles per half-wave read on the
//                  bank model, against 1.60 for the class layout that needed a copy)
//
// The DUAL plan of quad_hash: the (|P| - 1) / 128 compressions that B2(P) and B2(P || sig)
// share run as soon as their blocks exist; the transcoder holds the signature back until the
// msg digest's final (masked) block has been compressed, then appends it for the block digest.
// The rules (bounds, checks, error order) are k_block_ingest's, which states them with the
// reference file:line; tests/test_gpu_ingest.py and test_gpu_blocks.py hold this kernel, the
// host codec (MV_FLAG_HOST_PARSE) and the oracle to the same verdicts and digests.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mysti_verify.h"
#include "blake2b_quad.h"
#include "block_verdict.h"
#include "kernels.h"

namespace mv {
namespace ih {

constexpr uint32_t BR_LINES = 4;           // bincode ring: lines of 128 B per quad
constexpr uint32_t BR_DW = BR_LINES * 32;  // dwords
constexpr uint32_t BR_STRIDE = BR_DW + 4;  // quad stride (dwords): quads 4 banks apart
constexpr uint32_t PR_U64 = 36;            // pre-image ring: 2 message blocks + pad (u64)
constexpr uint32_t SHARE_CHUNK = 64;       // Share payload bytes per piece
constexpr uint32_t MAX_STMT = 137;         // longest statement header: Vote Reject(Some)
constexpr uint64_t VR_MAX = 1024 * 1024;   // VoteRange::verify MAX_LEN (types.rs:448)

enum : uint32_t { PH_HDR, PH_INC, PH_NST, PH_ST, PH_SHARE, PH_TR, PH_WAITMSG, PH_DONE, PH_FAIL };
enum : uint32_t { FK_LOC, FK_BE128, FK_RAW };

struct Args {
  const uint8_t* buf;
  uint64_t buf_bytes;
  const uint64_t* off;
  const uint64_t* len;
  uint32_t n;
  const uint64_t* stakes;
  uint32_t n_auth;
  uint64_t epoch, quorum_thr;
  uint8_t* sig_out;
  uint32_t* key_idx;
  uint32_t* facts;
  uint8_t* claimed;
  uint8_t* md;
  uint8_t* bd;
};

MV_DEV uint32_t vr_code(uint64_t s0, uint64_t s1) {  // VoteRange::verify (types.rs:440-460)
  return s1 < s0 ? 1u : (s1 - s0 >= VR_MAX ? 2u : (s1 >= VR_MAX ? 3u : 0u));
}

// The quad's view of its block: bincode ring, pre-image ring, stream state.
struct Quad {
  const uint32_t* br;  // bincode ring (absolute line x at dwords (32 x) mod BR_DW)
  uint32_t* pr32;      // pre-image ring (stream dword j at j mod 64)
  uint32_t d;          // block start within its 16-byte aligned base
  uint32_t q;          // lane within the quad
  uint32_t pre_dw, pk, pend;  // stream: complete dwords, pending bytes (< 4) and their value

  // dword at block byte `pos` (any alignment; the bytes must be in the ring)
  MV_DEV uint32_t dw(uint32_t pos) const {
    const uint32_t a = d + pos, i = a >> 2;
    return __builtin_amdgcn_alignbyte(br[(i + 1) & (BR_DW - 1)], br[i & (BR_DW - 1)], a & 3u);
  }
  MV_DEV uint64_t u64(uint32_t pos) const { return (uint64_t)dw(pos) | ((uint64_t)dw(pos + 4) << 32); }
  MV_DEV uint32_t u8(uint32_t pos) const { return dw(pos) & 0xffu; }

  // dword j of a piece's F: LOC = a BlockReference / locator (BE authority, BE round, the
  // digest as it lies, then BE u64 extras at +56, +64), BE128 = the u128 creation time
  // big-endian, RAW = bytes as they lie (the last dword masked to fb bytes)
  MV_DEV uint32_t fdw(uint32_t kind, uint32_t base, uint32_t j, uint32_t fb) const {
    uint32_t off;
    bool sw;
    if (kind == FK_LOC) {
      if (j < 4) {
        off = 8 * (j >> 1) + ((j & 1) ? 0u : 4u);
        sw = true;
      } else if (j < 12) {
        off = 24 + 4 * (j - 4);
        sw = false;
      } else {
        const uint32_t jj = j - 12;
        off = 56 + 8 * (jj >> 1) + ((jj & 1) ? 0u : 4u);
        sw = true;
      }
    } else if (kind == FK_BE128) {
      off = 12 - 4 * j;
      sw = true;
    } else {
      off = 4 * j;
      sw = false;
    }
    uint32_t v = dw(base + off);
    if (sw) v = __builtin_bswap32(v);
    if (kind == FK_RAW && (fb & 3u) && j == ((fb + 3) >> 2) - 1) v &= (1u << (8 * (fb & 3u))) - 1;
    return v;
  }

  MV_DEV uint32_t pre_hi() const { return 4 * pre_dw + pk; }

  // appends [tag byte] || F (fb bytes) to the stream; the quad's lanes write dwords q, q + 4, ...
  MV_DEV void emit(int tag, uint32_t kind, uint32_t base, uint32_t fb) {
    uint32_t pre = pend, k = pk;
    if (tag >= 0) {
      pre |= (uint32_t)tag << (8 * k);
      k++;
    }
    if (k == 4) {
      if (q == 0) pr32[pre_dw & 63] = pre;
      pre_dw++;
      pre = 0;
      k = 0;
    }
    const uint32_t tb = k + fb, nw = (tb + 3) >> 2, nF = (fb + 3) >> 2;
    const uint32_t top = k ? pre << (8 * (4 - k)) : 0u;  // the prefix's k bytes at the top of F[-1]
    for (uint32_t j = q; j < nw; j += 4) {
      const uint32_t fj = j < nF ? fdw(kind, base, j, fb) : 0u;
      uint32_t out = fj;
      if (k) {
        const uint32_t fp = j == 0 ? top : fdw(kind, base, j - 1, fb);
        out = __builtin_amdgcn_alignbyte(fj, fp, 4 - k);
      }
      pr32[(pre_dw + j) & 63] = out;
    }
    pre_dw += tb >> 2;
    pk = tb & 3u;
    pend = pk ? pr32[pre_dw & 63] : 0u;  // written above by one of the quad's lanes (LDS in order)
  }
  // zeroes the stream from its end to the end of its 128-byte block (the final block's mask)
  MV_DEV void flush() {
    const uint32_t start = pre_dw + (pk ? 1u : 0u);
    const uint32_t end = ((pre_hi() + 127) >> 7) << 5;
    for (uint32_t j = start + q; j < end; j += 4) pr32[j & 63] = 0u;
  }
};

__global__ void __launch_bounds__(64) k_block_ingest_hash(Args A) {
  __shared__ uint32_t bring[16 * BR_STRIDE];
  __shared__ uint64_t pring[16 * PR_U64];
  __shared__ uint32_t seen[16][16];  // authorities of round r - 1 among the includes (<= 512)
  const uint32_t lane = threadIdx.x, q = lane & 3u, qd = lane >> 2;
  const uint32_t i = blockIdx.x * 16 + qd;
  const bool live = i < A.n;
#pragma unroll
  for (uint32_t k = 0; k < 4; k++) seen[qd][q + 4 * k] = 0;

  const uint64_t o = live ? A.off[i] : 0;
  const uint64_t L64 = live ? A.len[i] : 0;
  // network frames are at most 16 MiB (network.rs:216): block positions fit 32 bits
  const uint32_t L = L64 > 0x7fffffffull ? 0x7fffffffu : (uint32_t)L64;
  // lines are 128 B from the 16-byte aligned address at or below the block's first byte
  const uintptr_t abs0 = reinterpret_cast<uintptr_t>(A.buf + o);
  const uint8_t* const gbase = reinterpret_cast<const uint8_t*>(abs0 & ~(uintptr_t)15);
  const uint8_t* const gend = A.buf + A.buf_bytes;
  Quad Q;
  Q.br = bring + qd * BR_STRIDE;
  Q.pr32 = reinterpret_cast<uint32_t*>(pring + qd * PR_U64);
  Q.d = (uint32_t)(abs0 & 15u);
  Q.q = q;
  Q.pre_dw = 0;
  Q.pk = 0;
  Q.pend = 0;
  uint32_t* const brw = bring + qd * BR_STRIDE;
  const uint64_t* const pr = pring + qd * PR_U64;

  uint32_t phase = live ? PH_HDR : PH_DONE;
  uint32_t p = 0;                  // next bincode element (block-relative)
  uint32_t cnt = 0, total = 0;     // include / statement counters
  uint32_t share_pos = 0, share_rem = 0, share_first = 0, sig_p = 0;
  uint64_t me_a = 0, me_r = 0;
  uint32_t inc_first = 0, vr_first = 0;
  const uint32_t n_lines = (live && L) ? ((Q.d + L - 1) >> 7) + 1 : 0;
  uint32_t ld_next = 0;            // next absolute line of the block to load
  // hash state (lane q: columns q of the 4 x 4 working matrix)
  const uint64_t iv0 = b2q::IV[q], iv1 = b2q::IV[4 + q];
  uint64_t h0 = iv0 ^ (q == 0 ? 0x01010020ull : 0ull), h1 = iv1;
  uint32_t s = 0, common = 0, last = 0, nsteps = 0, Lpre = 0;
  bool pdone = false, hdone = !live;

  auto fail = [&]() {
    phase = PH_FAIL;
    const uint32_t w = q >= 2 ? 0xffffffffu : 0u;  // s = 2^256 - 1: outside the batch equation
    reinterpret_cast<uint4*>(A.sig_out + 64 * (size_t)i)[q] = make_uint4(w, w, w, w);
    if (q == 0) {
      A.key_idx[i] = 0;
      A.facts[i] = 0;
    }
  };

  for (;;) {
    // ---- (1) loads: up to two more lines, the ring keeping every byte from `keep` on
    const uint32_t keep = phase == PH_SHARE ? share_pos : (phase == PH_WAITMSG ? sig_p : p);
    const bool parsing = phase < PH_DONE;
    const uint32_t want = parsing ? min(((Q.d + keep) >> 7) + BR_LINES, n_lines) : 0u;
    const uint32_t nl = want > ld_next ? min(want - ld_next, 2u) : 0u;
    uint4 ld[4];
#pragma unroll
    for (int h = 0; h < 4; h++) {
      const uint8_t* src = gbase + (size_t)(ld_next + (h >> 1)) * 128 + 32 * q + 16 * (h & 1);
      ld[h] = ((uint32_t)(h >> 1) < nl && src < gend) ? *reinterpret_cast<const uint4*>(src) : make_uint4(0, 0, 0, 0);
    }

    // ---- (2) one compression, for the quads whose next block is in the pre-image ring
    bool ready = false, fin = false, mfin = false;
    uint32_t b = 0;
    uint64_t t = 0;
    if (!hdone) {
      if (phase == PH_FAIL) {
        hdone = true;
      } else if (!pdone) {  // P continues past block s: a shared, non-final block
        if (Q.pre_hi() >= 128 * (s + 1)) {
          ready = true;
          b = s;
          t = 128ull * (s + 1);
        }
      } else {  // quad_hash's DUAL plan with L = |P|
        mfin = s == common;
        b = s < common ? s : (mfin ? common : s - 1);
        fin = mfin || b == last;
        t = mfin ? (uint64_t)Lpre : (b == last ? (uint64_t)Lpre + 64 : 128ull * (b + 1));
        ready = s < nsteps && (s <= common || phase == PH_DONE);
      }
    }
    __syncthreads();  // the transcoder's ring stores before the hash reads them
    if (__ballot(ready)) {
      uint64_t hh0[1] = {h0}, hh1[1] = {h1};
      const uint64_t* const mrow[1] = {pr + (b & 1u) * 16};
      const uint64_t tt[1] = {t};
      const bool ff[1] = {fin};
      b2q::compress<1, true>(hh0, hh1, mrow, q, iv0, iv1, tt, ff);
      if (ready) {
        if (mfin) {  // B2(P) done: the chain continues from the shared prefix for B2(P || sig)
          reinterpret_cast<uint64_t*>(A.md + 32 * (size_t)i)[q] = hh0[0];
        } else {
          h0 = hh0[0];
          h1 = hh1[0];
        }
        s++;
        if (pdone && s == nsteps) {
          reinterpret_cast<uint64_t*>(A.bd + 32 * (size_t)i)[q] = h0;
          hdone = true;
        }
      }
    }

    // ---- (3) the loaded lines into the bincode ring
#pragma unroll
    for (int h = 0; h < 4; h++)
      if ((uint32_t)(h >> 1) < nl) {
        const uint32_t x = ((ld_next + (h >> 1)) * 32 + 8 * q + 4 * (h & 1)) & (BR_DW - 1);
        brw[x] = ld[h].x;
        brw[x + 1] = ld[h].y;
        brw[x + 2] = ld[h].z;
        brw[x + 3] = ld[h].w;
      }
    ld_next += nl;
    __syncthreads();

    // ---- (4) transcode until the next block to hash is complete (at most one block ahead)
    const uint32_t avail = ld_next ? min(ld_next * 128 - Q.d, L) : 0u;  // block bytes [.., avail) loaded
    const uint32_t bnext = (pdone && s > common) ? s - 1 : s;
    bool blocked = false;
    for (;;) {
      const bool go = !blocked && Q.pre_hi() <= 128 * (bnext + 1) &&
                      (phase < PH_WAITMSG || (phase == PH_WAITMSG && s > common));
      if (!__ballot(go)) break;
      if (!go) continue;
      if (phase == PH_HDR) {
        // reference (authority, round, digest with its u64 length 32) and the include count
        if (L < 64) {
          fail();
        } else if (avail < 64) {
          blocked = true;
        } else if (Q.u64(16) != 32) {
          fail();
        } else {
          me_a = Q.u64(0);
          me_r = Q.u64(8);
          const uint64_t n_inc = Q.u64(56);
          if (n_inc > (uint64_t)((L - 64) / 56)) {
            fail();
          } else {
            reinterpret_cast<uint2*>(A.claimed + 32 * (size_t)i)[q] = make_uint2(Q.dw(24 + 8 * q), Q.dw(28 + 8 * q));
            Q.emit(-1, FK_LOC, 0, 16);  // BE authority, BE round
            p = 64;
            cnt = 0;
            total = (uint32_t)n_inc;
            phase = total ? PH_INC : PH_NST;
          }
        }
      } else if (phase == PH_INC) {  // includes (types.rs:349-362), threshold clock's authorities
        if (avail < p + 56) {
          blocked = true;
        } else if (Q.u64(p + 16) != 32) {
          fail();
        } else {
          const uint64_t a = Q.u64(p), r = Q.u64(p + 8);
          if (!inc_first)
            inc_first = a >= A.n_auth ? MV_BLOCK_INCLUDE_UNKNOWN_AUTHORITY : (r >= me_r ? MV_BLOCK_INCLUDE_ROUND : 0u);
          if (me_r > 0 && r == me_r - 1 && a < A.n_auth) {
            const uint32_t wd = (uint32_t)a >> 5, bit = 1u << (a & 31);
            const uint32_t sv = seen[qd][wd];
            if (!(sv & bit)) seen[qd][wd] = sv | bit;  // the quad's four lanes store the same word
          }
          Q.emit(-1, FK_LOC, p, 48);
          p += 56;
          if (++cnt == total) phase = PH_NST;
        }
      } else if (phase == PH_NST) {
        if (p + 8 > L) {
          fail();
        } else if (avail < p + 8) {
          blocked = true;
        } else {
          const uint64_t n_st = Q.u64(p);
          p += 8;
          cnt = 0;
          total = n_st > 0xffffffffull ? 0xffffffffu : (uint32_t)n_st;  // a bad count fails on bounds
          phase = total ? PH_ST : PH_TR;
        }
      } else if (phase == PH_ST) {
        if (p + 4 > L) {
          fail();
        } else if (avail < min(L, p + MAX_STMT)) {
          blocked = true;
        } else {
          const uint32_t tag = Q.dw(p);
          bool next = false;
          if (tag == 0) {  // Share: u64 length, bytes (no length in the pre-image)
            if (p + 12 > L) {
              fail();
            } else {
              const uint64_t l = Q.u64(p + 4);
              if (l > (uint64_t)(L - p - 12)) {
                fail();
              } else {
                share_pos = p + 12;
                share_rem = (uint32_t)l;
                share_first = 1;
                phase = PH_SHARE;
              }
            }
          } else if (tag == 1) {  // Vote: locator (ref 56 + offset 8), u32 vote, [u8 option, [locator]]
            if (p + 72 > L || Q.u64(p + 20) != 32) {
              fail();
            } else {
              const uint32_t vote = Q.dw(p + 68);
              if (vote == 0) {
                Q.emit(1, FK_LOC, p + 4, 56);
                p += 72;
                next = true;
              } else if (vote == 1 && p + 73 <= L) {
                const uint32_t some = Q.u8(p + 72);
                if (some == 0) {
                  Q.emit(2, FK_LOC, p + 4, 56);
                  p += 73;
                  next = true;
                } else if (some == 1 && p + 137 <= L && Q.u64(p + 89) == 32) {
                  Q.emit(3, FK_LOC, p + 4, 56);
                  Q.emit(-1, FK_LOC, p + 73, 56);
                  p += 137;
                  next = true;
                } else {
                  fail();
                }
              } else {
                fail();
              }
            }
          } else if (tag == 2) {  // VoteRange: ref 56, start, end
            if (p + 76 > L || Q.u64(p + 20) != 32) {
              fail();
            } else {
              if (!vr_first) vr_first = vr_code(Q.u64(p + 60), Q.u64(p + 68));
              Q.emit(4, FK_LOC, p + 4, 64);
              p += 76;
              next = true;
            }
          } else {
            fail();
          }
          if (next && ++cnt == total) phase = PH_TR;
        }
      } else if (phase == PH_SHARE) {  // [0] || payload, SHARE_CHUNK bytes per piece
        const uint32_t chunk = min(share_rem, SHARE_CHUNK);
        if (avail < share_pos + chunk) {
          blocked = true;
        } else {
          Q.emit(share_first ? 0 : -1, FK_RAW, share_pos, chunk);
          share_first = 0;
          share_pos += chunk;
          share_rem -= chunk;
          if (!share_rem) {
            p = share_pos;
            phase = ++cnt == total ? PH_TR : PH_ST;
          }
        }
      } else if (phase == PH_TR) {  // creation time (u128), epoch marker, epoch, signature
        if (p + 97 > L) {
          fail();
        } else if (avail < p + 97) {
          blocked = true;
        } else {
          const uint32_t marker = Q.u8(p + 16);
          const uint64_t ep = Q.u64(p + 17);
          if (marker > 1 || Q.u64(p + 25) != 64) {
            fail();
          } else {
            Q.emit(-1, FK_BE128, p, 16);
            Q.emit((int)marker, FK_LOC, p + 17, 8);
            Lpre = Q.pre_hi();
            pdone = true;
            common = (Lpre - 1) >> 7;
            last = (Lpre + 63) >> 7;
            nsteps = last + 2;
            Q.flush();  // B2(P)'s final block, zero past |P|
            sig_p = p + 33;
            // threshold clock (threshold_clock.rs:12-35): stake of the distinct round r - 1
            // authorities; lane q sums seen words q, q + 4, ..., eight loads in flight at a time
            uint64_t stake = 0;
            for (uint32_t w = q; w < 16; w += 4) {
              uint32_t bits = seen[qd][w];
              while (bits) {
                uint64_t v[8];
#pragma unroll
                for (int k = 0; k < 8; k++) {
                  const uint32_t a = bits ? 32 * w + (uint32_t)__builtin_ctz(bits) : 0u;  // a set bit is < n_auth
                  const uint64_t x = A.stakes[a];
                  v[k] = bits ? x : 0ull;
                  bits &= bits - 1;
                }
#pragma unroll
                for (int k = 0; k < 8; k++) stake += v[k];
              }
            }
            stake += (uint64_t)__shfl_xor((unsigned long long)stake, 1);
            stake += (uint64_t)__shfl_xor((unsigned long long)stake, 2);
            const uint32_t f = BF_PARSED | (ep == A.epoch ? BF_EPOCH_OK : 0u) | (me_a < A.n_auth ? BF_AUTHOR_OK : 0u) |
                               (me_r == 0 ? BF_GENESIS : 0u) | (vr_first << BF_VR_SHIFT) |
                               (stake > A.quorum_thr ? BF_QUORUM : 0u) | (inc_first << BF_INC_SHIFT);
            const bool sig_decides = (f & BF_EPOCH_OK) && (f & BF_AUTHOR_OK) && !(f & BF_GENESIS);
            uint4 sw = make_uint4(Q.dw(sig_p + 16 * q), Q.dw(sig_p + 16 * q + 4), Q.dw(sig_p + 16 * q + 8),
                                  Q.dw(sig_p + 16 * q + 12));
            if (!sig_decides && q >= 2) sw = make_uint4(~0u, ~0u, ~0u, ~0u);
            reinterpret_cast<uint4*>(A.sig_out + 64 * (size_t)i)[q] = sw;
            if (q == 0) {
              A.key_idx[i] = me_a < A.n_auth ? (uint32_t)me_a : 0u;
              A.facts[i] = f;
            }
            phase = PH_WAITMSG;
          }
        }
      } else if (phase == PH_WAITMSG) {  // B2(P) is done: P || sig for the block digest
        Q.emit(-1, FK_RAW, sig_p, 64);
        Q.flush();
        phase = PH_DONE;
      }
    }
    if (!__ballot(!hdone)) break;
  }
}

}  // namespace ih
}  // namespace mv

namespace mvk {

hipError_t launch_block_ingest_hash(const uint8_t* buf, uint64_t buf_bytes, const uint64_t* off, const uint64_t* len,
                                    uint32_t n, const uint64_t* stakes, uint32_t n_auth, uint64_t epoch,
                                    uint64_t quorum_thr, uint8_t* sig, uint32_t* key_idx, uint32_t* facts,
                                    uint8_t* claimed, uint8_t* md, uint8_t* bd, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const mv::ih::Args a{buf, buf_bytes, off, len, n, stakes, n_auth, epoch, quorum_thr, sig, key_idx, facts, claimed,
                       md, bd};
  hipLaunchKernelGGL(mv::ih::k_block_ingest_hash, dim3((n + 15) / 16), dim3(64), 0, s, a);
  return hipGetLastError();
}

}  // namespace mvk
