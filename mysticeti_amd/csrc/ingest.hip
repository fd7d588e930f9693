// Device-side StatementBlock ingest for gfx950: bincode
// Data<StatementBlock> bytes resident in HBM -> the signed pre-image P || sig, staged for
// k_block_hash, plus the facts StatementBlock::verify checks; one block per lane.
// k_block_verdict folds the digest comparison, the signature verdict and those facts into
// one status in the reference's error order (types.rs:315-376).
//
//   bincode     types.rs:93-114 (StatementBlock), :49-54 (BlockReference), :57-64
//               (BaseStatement), :31-35 (Vote), :384-394 (locators), crypto.rs:309-347
//               (length-checked 32/64-byte arrays); bincode 1.3.3 defaults (LE fixint, u64
//               lengths, u32 tags, trailing bytes allowed) as Data::from_bytes uses them
//               (data.rs:43-52)
//   pre-image   BlockDigest::digest_without_signature (crypto.rs:85-128) with the
//               CryptoHash encodings of crypto.rs:150-170, types.rs:661-691 and 751-755
//   checks      epoch, author, genesis and includes (types.rs:333-362), VoteRange::verify
//               (types.rs:440-460), the threshold clock (threshold_clock.rs:12-35)
// block_codec.cpp states the same rules on the host (MV_FLAG_HOST_PARSE); the GPU tests hold
// both paths and the oracle to the same verdicts and digests, malformed input included.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/mysti_verify.h"
#include "hash_dev.h"
#include "block_verdict.h"
#include "kernels.h"
#include "ingest_dev.h"

namespace mv {

// Lane per block over global memory (the reference implementation of the ingest; the
// product launches k_block_ingest, which falls back to ingest_lane for oversize blocks).
__global__ void __launch_bounds__(256) k_block_parse(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ off,
                                                     const uint64_t* __restrict__ len, uint32_t n, CommitteeView cv,
                                                     IngestOut io) {
  __shared__ uint32_t seen[16][256];  // per-lane authority bitmap, [word][lane]
  const uint32_t t = threadIdx.x;
  const uint32_t i = blockIdx.x * 256 + t;
#pragma unroll
  for (int k = 0; k < 16; k++) seen[k][t] = 0;
  if (i >= n) return;
  ingest_lane(buf, off[i], len[i], i, cv, io, &seen[0][t], 256);
}

// ---------------------------------------------------------------- wave per block
// k_block_ingest: one 64-lane workgroup per block (ingest_dev.h's ingest_block).
__global__ void __launch_bounds__(64) k_block_ingest(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ off,
                                                     const uint64_t* __restrict__ len, uint32_t n, CommitteeView cv,
                                                     IngestOut io) {
  __shared__ IngestLds L;
  ingest_block<false>(blockIdx.x, buf, off, len, cv, io, L);
}

// Between the hashes and the signature check: a parsed block whose digest differs from the
// claimed one gets DIGEST_MISMATCH whatever its signature (types.rs:327-332 comes before the
// signature check at :346-348), so its s is set to 2^256 - 1 (>= l): it is then excluded
// from the batch equation like the blocks ingest rejects ahead of the signature.
__global__ void __launch_bounds__(256) k_block_digest_gate(const uint8_t* __restrict__ claimed,
                                                           const uint8_t* __restrict__ digest,
                                                           const uint32_t* __restrict__ facts, uint32_t n,
                                                           uint8_t* __restrict__ sig) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !(facts[i] & BF_PARSED) || digest_same(claimed, digest, i)) return;
  uint4* s4 = reinterpret_cast<uint4*>(sig + 64 * (size_t)i + 32);
  s4[0] = make_uint4(~0u, ~0u, ~0u, ~0u);
  s4[1] = make_uint4(~0u, ~0u, ~0u, ~0u);
}

// status[i] in the order of StatementBlock::verify (types.rs:315-376), block_verdict.h
__global__ void __launch_bounds__(256) k_block_verdict(const uint32_t* __restrict__ facts,
                                                       const uint8_t* __restrict__ claimed,
                                                       uint8_t* __restrict__ msg_digest,
                                                       uint8_t* __restrict__ digest,
                                                       const uint8_t* __restrict__ sig_status, uint32_t n,
                                                       uint8_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  status[i] = block_verdict(facts, claimed, msg_digest, digest, sig_status[i], i);
}

}  // namespace mv

// ---------------------------------------------------------------- launchers
namespace mvk {

hipError_t launch_block_parse(const Knobs& kn, const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n,
                              const uint64_t* stakes, uint32_t n_auth, uint64_t epoch, uint64_t quorum_thr,
                              uint8_t* stage, uint64_t* pre_off, uint64_t* pre_len, uint8_t* sig, uint32_t* key_idx,
                              uint32_t* facts, uint8_t* claimed, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const mv::CommitteeView cv{stakes, n_auth, epoch, quorum_thr};
  const mv::IngestOut io{stage, pre_off, pre_len, sig, key_idx, facts, claimed};
  if (kn.ingest_lane)  // A/B (MV_INGEST_LANE=1): the lane-per-block kernel
    hipLaunchKernelGGL(mv::k_block_parse, dim3((n + 255) / 256), dim3(256), 0, s, buf, off, len, n, cv, io);
  else  // (capping its workgroups per CU with padded LDS, to leave room for the other stream's
        // kernels, measured slower: 79 vs 103 M config-4 blocks/s, profiles/r03/ab/)
    hipLaunchKernelGGL(mv::k_block_ingest, dim3(n), dim3(64), 0, s, buf, off, len, n, cv, io);
  return hipGetLastError();
}

hipError_t launch_block_digest_gate(const uint8_t* claimed, const uint8_t* digest, const uint32_t* facts, uint32_t n,
                                    uint8_t* sig, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(mv::k_block_digest_gate, dim3((n + 255) / 256), dim3(256), 0, s, claimed, digest, facts, n, sig);
  return hipGetLastError();
}

hipError_t launch_block_verdict(const uint32_t* facts, const uint8_t* claimed, uint8_t* msg_digest, uint8_t* digest,
                                const uint8_t* sig_status, uint32_t n, uint8_t* status, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(mv::k_block_verdict, dim3((n + 255) / 256), dim3(256), 0, s, facts, claimed, msg_digest, digest,
                     sig_status, n, status);
  return hipGetLastError();
}

}  // namespace mvk
