// Host-side StatementBlock codec of the engine: bincode Data<StatementBlock> bytes
// -> signed pre-image + the fields StatementBlock::verify checks on the host.
//
//   bincode field order  types.rs:93-114 (StatementBlock), :49-54 (BlockReference),
//                        :57-64 (BaseStatement), :31-35 (Vote), :384-394 (locators),
//                        crypto.rs:309-347 (length-checked 32/64-byte arrays);
//                        bincode 1.3.3 defaults (LE fixint, u64 lengths, u32 tags,
//                        trailing bytes allowed) as used by Data::from_bytes (data.rs:43-52)
//   pre-image            BlockDigest::digest_without_signature (crypto.rs:85-128) with the
//                        CryptoHash encodings of crypto.rs:150-170 and types.rs:661-691
//   host checks          types.rs:333-374 (epoch, author, genesis, includes, VoteRange,
//                        threshold clock) -- the crypto checks run on the GPU
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace mvh {

struct Committee {
  std::vector<uint8_t> pks;     // n x 32
  std::vector<uint64_t> stakes; // n
  uint64_t epoch = 0;
  uint64_t quorum_threshold = 0;  // 2 * total / 3 (committee.rs:56-57); quorum <=> stake > it
  uint32_t size() const { return (uint32_t)stakes.size(); }
};

// Outcome of the host-side part of StatementBlock::verify for one block.
struct BlockFacts {
  bool parsed = false;
  uint64_t author = 0, round = 0, epoch = 0;
  uint8_t claimed_digest[32];
  uint8_t signature[64];
  uint8_t include_error = 0;  // 0, MV_BLOCK_INCLUDE_UNKNOWN_AUTHORITY or MV_BLOCK_INCLUDE_ROUND (first failing include)
  uint8_t vote_range_error = 0;  // first failing VoteRange: MV_BLOCK_VOTE_RANGE* or 0
  bool threshold_ok = false;
  uint64_t preimage_len = 0;
};

// Parses `len` bytes; on success writes the pre-image to `pre` (capacity `cap`, may be
// nullptr to size only) and fills `f`. Returns false on a bincode error.
bool parse_block(const uint8_t* buf, size_t len, const Committee* committee, uint8_t* pre, size_t cap,
                 BlockFacts& f);

// The final verdict (MV_BLOCK_*) in the order of StatementBlock::verify, given the GPU's
// digest and signature results.
uint8_t block_verdict(const BlockFacts& f, const Committee& c, const uint8_t computed_digest[32], uint8_t sig_status);

}  // namespace mvh
