// The per-block verdict of StatementBlock::verify (types.rs:315-376) from the ingest facts, the
// claimed and computed digests and the signature status: k_block_verdict (ingest.hip) and,
// fused into their last wave, the committee comb kernels of the online path (comb.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mysti_verify.h"

#ifndef MV_DEV
#define MV_DEV __device__ __forceinline__
#endif

namespace mv {

constexpr uint32_t BF_PARSED = 1u, BF_EPOCH_OK = 2u, BF_AUTHOR_OK = 4u, BF_GENESIS = 8u, BF_QUORUM = 32u;
constexpr int BF_INC_SHIFT = 8;  // first failing include: MV_BLOCK_INCLUDE_* or 0
constexpr int BF_VR_SHIFT = 16;  // first failing VoteRange: vr_code() or 0

MV_DEV bool digest_same(const uint8_t* claimed, const uint8_t* digest, uint32_t i) {
  const uint4* a = reinterpret_cast<const uint4*>(claimed + 32 * (size_t)i);
  const uint4* b = reinterpret_cast<const uint4*>(digest + 32 * (size_t)i);
  const uint4 a0 = a[0], a1 = a[1], b0 = b[0], b1 = b[1];
  return ((a0.x ^ b0.x) | (a0.y ^ b0.y) | (a0.z ^ b0.z) | (a0.w ^ b0.w) | (a1.x ^ b1.x) | (a1.y ^ b1.y) |
          (a1.z ^ b1.z) | (a1.w ^ b1.w)) == 0;
}

// status of block i in the order of StatementBlock::verify. A block that does not deserialize
// has no pre-image: its two digests are zeroed, so every output is deterministic.
MV_DEV uint8_t block_verdict(const uint32_t* facts, const uint8_t* claimed, uint8_t* msg_digest, uint8_t* digest,
                             uint8_t sig_status, uint32_t i) {
  const uint32_t f = facts[i];
  if (!(f & BF_PARSED)) {
    const uint4 z = make_uint4(0, 0, 0, 0);
    uint4* m4 = reinterpret_cast<uint4*>(msg_digest + 32 * (size_t)i);
    uint4* d4 = reinterpret_cast<uint4*>(digest + 32 * (size_t)i);
    m4[0] = z;
    m4[1] = z;
    d4[0] = z;
    d4[1] = z;
    return MV_BLOCK_PARSE_ERROR;
  }
  const bool same = digest_same(claimed, digest, i);
  const uint32_t inc = (f >> BF_INC_SHIFT) & 0xffu;
  const uint32_t vr = (f >> BF_VR_SHIFT) & 3u;
  return !same                     ? MV_BLOCK_DIGEST_MISMATCH
         : !(f & BF_EPOCH_OK)      ? MV_BLOCK_EPOCH_MISMATCH
         : !(f & BF_AUTHOR_OK)     ? MV_BLOCK_UNKNOWN_AUTHOR
         : (f & BF_GENESIS)        ? MV_BLOCK_GENESIS
         : sig_status != MV_SIG_OK ? MV_BLOCK_SIG_INVALID
         : inc                     ? (uint8_t)inc
         : vr == 1                 ? MV_BLOCK_VOTE_RANGE
         : vr == 2                 ? MV_BLOCK_VOTE_RANGE_TOO_LONG
         : vr == 3                 ? MV_BLOCK_VOTE_RANGE_END_TOO_LARGE
         : !(f & BF_QUORUM)        ? MV_BLOCK_THRESHOLD_CLOCK
                                   : MV_BLOCK_OK;
}

}  // namespace mv
