// BLAKE2b-256 for gfx950 with FOUR lanes per string (blake2 0.10.6
// Blake2b<U32> as crypto.rs:34-61 and :174-189 use it; RFC 7693 with nn = 32, kk = 0).
//
// Lane q of a quad holds column q of the 4x4 working matrix, (v[q], v[4+q], v[8+q], v[12+q]),
// and runs one G per half-round: the column step as is, the diagonal step after rotating the
// b, c, d rows across the quad by 1, 2, 3 lanes (DPP quad_perm, full rate) and back. The
// message block sits in LDS (128 B per string, double-buffered, each lane loads a quarter of
// the next block from HBM during the current compression); each lane reads the four words
// its G's add in a round at SIGMA-derived indices.
//
// Why four lanes: a compression is a chain of 12 rounds, so a lane-per-string kernel runs
// each string's 96 G's back to back. Four lanes cut that chain 4x (the latency path, 64
// blocks per call, is bound by it) and shrink the state to 8 VGPRs + 4 for h, so the
// throughput kernel runs at full occupancy instead of ~160 VGPRs per lane.
//
// 64-bit adds are v_lshl_add_u64 (one half-rate instruction, not an add/addc pair); the 24-
// and 16-bit rotations are byte permutes (v_perm_b32); 32 is a register swap.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/mysti_verify.h"
#include "blake2b_quad.h"
#include "kernels.h"

namespace mv {
namespace b2q {

#define MV_B2Q_BOUNDS __launch_bounds__(64, NS == 1 ? 4 : 3)
template <bool DUAL, int NS>
__global__ void MV_B2Q_BOUNDS k_b2_quad(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ off,
                                        const uint64_t* __restrict__ len, uint32_t n, uint8_t* __restrict__ out0,
                                        uint8_t* __restrict__ out1) {
  quad_hash<DUAL, NS>(blockIdx.x, buf, off, len, n, out0, out1);
}
// the online path's form (a few waves on an idle chip): message reads hoisted out of their
// rounds, so the LDS latency leaves the compression chain (more VGPRs, fewer waves: fine here)
__global__ void __launch_bounds__(64) k_b2_quad_lat(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ off,
                                                    const uint64_t* __restrict__ len, uint32_t n,
                                                    uint8_t* __restrict__ out0, uint8_t* __restrict__ out1) {
  quad_hash<true, 1, true>(blockIdx.x, buf, off, len, n, out0, out1);
}


}  // namespace b2q
}  // namespace mv

namespace mvk {

// strings per quad: 1 (the default: measured on config 4, 2 interleaved strings per quad ran
// at the same speed -- 5.16 vs 5.11 ms -- with 60% more VGPRs). MV_B2Q_NS=2 selects the
// interleaved kernel (experiments).
static int b2q_ns(const Knobs& kn) { return kn.b2q_ns == 2 ? 2 : 1; }
// batch-size calls: the lane-per-string kernel (blake2b_lane.hip) unless MV_B2_LANE=0
static bool b2_lane(const Knobs& kn, uint32_t n) { return kn.b2_lane != 0 && n >= MV_BATCH_MIN; }

hipError_t launch_blake2b_quad(const Knobs& kn, const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n, uint8_t* out,
                               hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (b2_lane(kn, n)) return launch_blake2b_lane(buf, off, len, n, out, s);
  if (b2q_ns(kn) == 2)
    hipLaunchKernelGGL((mv::b2q::k_b2_quad<false, 2>), dim3((n + 31) / 32), dim3(64), 0, s, buf, off, len, n, out,
                       (uint8_t*)nullptr);
  else
    hipLaunchKernelGGL((mv::b2q::k_b2_quad<false, 1>), dim3((n + 15) / 16), dim3(64), 0, s, buf, off, len, n, out,
                       (uint8_t*)nullptr);
  return hipGetLastError();
}

hipError_t launch_block_hash_quad(const Knobs& kn, const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n,
                                  uint8_t* msg_out, uint8_t* dig_out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (b2_lane(kn, n)) return launch_block_hash_lane(buf, off, len, n, msg_out, dig_out, s);
  if (n < MV_BATCH_MIN)  // the online path (comb verify): latency form
    hipLaunchKernelGGL(mv::b2q::k_b2_quad_lat, dim3((n + 15) / 16), dim3(64), 0, s, buf, off, len, n, msg_out, dig_out);
  else if (b2q_ns(kn) == 2)
    hipLaunchKernelGGL((mv::b2q::k_b2_quad<true, 2>), dim3((n + 31) / 32), dim3(64), 0, s, buf, off, len, n, msg_out,
                       dig_out);
  else
    hipLaunchKernelGGL((mv::b2q::k_b2_quad<true, 1>), dim3((n + 15) / 16), dim3(64), 0, s, buf, off, len, n, msg_out,
                       dig_out);
  return hipGetLastError();
}

}  // namespace mvk
