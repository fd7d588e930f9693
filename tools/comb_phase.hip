// Phase timing of the online comb verify (diagnostics, not shipped): a copy of
// k_verify_comb16 (comb.hip, included whole) with s_memrealtime stamps (100 MHz) per role,
// on 64 random signatures over 100 random committee keys (timing does not depend on validity).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I mysticeti_amd/csrc tools/comb_phase.hip -o tools/comb_phase
#include "../mysticeti_amd/csrc/comb.hip"

#include <stdio.h>
#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

namespace mv {
MV_DEV uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

// stamps: [role][0 start, 1 role work done, 2 after the first barrier, 3 end] (lane 0 of each
// role, workgroup 0); table roles 5..8 also stamp the end of SHA-512 in slot 3
__global__ void __launch_bounds__(C16_THREADS) k_comb16_phases(const uint8_t* msg, const uint8_t* __restrict__ sig,
                                                               const uint8_t* __restrict__ pk,
                                                               const uint32_t* __restrict__ key_idx, uint32_t n,
                                                               const uint4* __restrict__ combB,
                                                               const uint4* __restrict__ combA,
                                                               uint8_t* __restrict__ status, uint64_t* ts) {
  __shared__ uint32_t part[C16_TROLES][C16_SIGS][36];
  constexpr int ROWS = CT_ROWS / (C16_TROLES / 2);
  const uint64_t t0 = now();
  const uint32_t t = threadIdx.x;
  const bool row_role = t < 16 * C16_SIGS;
  const uint32_t role = row_role ? 0u : 1u + (t - 16 * C16_SIGS) / (4 * C16_SIGS);
  const uint32_t sq = row_role ? t >> 4 : (t >> 2) & (C16_SIGS - 1), c = t & 3u;
  const uint32_t gid = blockIdx.x * C16_SIGS + sq;
  const uint32_t idx = gid < n ? gid : n - 1;
  const uint32_t key = key_idx[idx];
  const bool stamp = blockIdx.x == 0 && (row_role ? t == 0 : (t - 16 * C16_SIGS) % (4 * C16_SIGS) == 0);
  fe v;
  bool okR = false, s_ok = false;
  if (role == 0) {
    uint32_t rw[8], sw[8];
    load8(rw, sig + 64 * (size_t)idx);
    load8(sw, sig + 64 * (size_t)idx + 32);
    s_ok = sc_is_canonical(sw);
    p3 R;
    decompress1_r16(R, okR, rw);
    fe_qsel(v, c, R.X, R.Y, R.Z, R.T);
  } else {
    const uint32_t tr = role - 1;
    if (tr < C16_TROLES / 2) {
      uint32_t sw[8], sd[8];
      load8(sw, sig + 64 * (size_t)idx + 32);
      sc_recode256(sd, sw);
      const int r0 = (int)tr * ROWS;
      q_ct_sum(v, combB, sd, r0, r0 + ROWS);
    } else {
      uint32_t kin[24], h[16], k[8], kd[8];
      load8(kin, sig + 64 * (size_t)idx);
      load8(kin + 8, pk + 32 * (size_t)key);
      load8(kin + 16, msg + 32 * (size_t)idx);
      sha512_short(h, kin, 96);
      sc_reduce512(k, h);
      sc_recode256(kd, k);
      if (stamp) ts[role * 4 + 3] = now();
      const int r0 = (int)(tr - C16_TROLES / 2) * ROWS;
      q_ct_sum(v, combA + (size_t)key * CT_TABLE, kd, r0, r0 + ROWS);
    }
#pragma unroll
    for (int i = 0; i < 9; i++) part[tr][sq][9 * c + i] = v.v[i];
  }
  const uint64_t t1 = now();
  __syncthreads();
  const uint64_t t2 = now();
  fe w;
  for (uint32_t h = C16_TROLES / 2; h >= 1; h >>= 1) {
    if (role >= 1 && role - 1 < h) {
#pragma unroll
      for (int i = 0; i < 9; i++) w.v[i] = part[role - 1 + h][sq][9 * c + i];
      qp_add(v, w);
#pragma unroll
      for (int i = 0; i < 9; i++) part[role - 1][sq][9 * c + i] = v.v[i];
    }
    __syncthreads();
  }
  if (role == 0) {
    fe S;
#pragma unroll
    for (int i = 0; i < 9; i++) S.v[i] = part[0][sq][9 * c + i];
    fe nS;
    fe_neg(nS, S);
    fe_cmov(S, nS, c == 0 || c == 3);
    qp_add(v, S);
    qp_dbl(v);
    qp_dbl(v);
    qp_dbl(v);
    fe Z;
    fe_qget<2>(Z, v);
    const bool zx = fe_is_zero(v);
    const bool eyz = fe_eq(v, Z);
    const uint32_t bits = (zx ? 1u : 0u) | (eyz ? 2u : 0u);
    if ((t & 15u) == 0 && gid < n) status[gid] = (uint8_t)(bits + (s_ok ? 4 : 0) + (okR ? 8 : 0));
  }
  const uint64_t t3 = now();
  if (stamp) {
    ts[role * 4 + 0] = t0;
    ts[role * 4 + 1] = t1;
    ts[role * 4 + 2] = t2;
    if (role <= C16_TROLES / 2) ts[role * 4 + 3] = t3;
  }
}
}  // namespace mv

int main() {
  const uint32_t n = 64, nkeys = 100;
  std::vector<uint8_t> enc(32 * nkeys), msg(32 * n), sig(64 * n), pk(32 * n);
  uint32_t x = 12345;
  auto rnd = [&] { x = x * 1664525u + 1013904223u; return (uint8_t)(x >> 24); };
  for (auto& b : enc) b = rnd();
  for (auto& b : msg) b = rnd();
  for (auto& b : sig) b = rnd();
  std::vector<uint32_t> kidx(n);
  for (uint32_t i = 0; i < n; i++) kidx[i] = i % nkeys;
  uint8_t *d_enc, *d_msg, *d_sig, *d_ok, *d_st;
  uint32_t* d_kidx;
  void *d_B, *d_A;
  uint64_t* d_ts;
  CHECK(hipMalloc(&d_enc, enc.size()));
  CHECK(hipMalloc(&d_msg, msg.size()));
  CHECK(hipMalloc(&d_sig, sig.size()));
  CHECK(hipMalloc(&d_ok, nkeys));
  CHECK(hipMalloc(&d_st, n));
  CHECK(hipMalloc(&d_kidx, 4 * n));
  CHECK(hipMalloc(&d_ts, 8 * 9 * 4));
  CHECK(hipMalloc(&d_B, mvk::comb_table_bytes(1)));
  CHECK(hipMalloc(&d_A, mvk::comb_table_bytes(nkeys)));
  CHECK(hipMemcpy(d_enc, enc.data(), enc.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_msg, msg.data(), msg.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_sig, sig.data(), sig.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_kidx, kidx.data(), 4 * n, hipMemcpyHostToDevice));
  CHECK(mvk::launch_comb_init(nullptr, 1, 0, d_B, nullptr, 0));
  CHECK(mvk::launch_comb_init(d_enc, nkeys, 1, d_A, d_ok, 0));
  CHECK(hipDeviceSynchronize());
  std::vector<std::vector<double>> ph(9 * 4);
  for (int rep = 0; rep < 30; rep++) {
    CHECK(hipMemset(d_ts, 0, 8 * 36));
    hipLaunchKernelGGL(mv::k_comb16_phases, dim3(n / mv::C16_SIGS), dim3(mv::C16_THREADS), 0, 0, d_msg, d_sig, d_enc,
                       d_kidx, n, (const uint4*)d_B, (const uint4*)d_A, d_st, d_ts);
    CHECK(hipDeviceSynchronize());
    uint64_t ts[36];
    CHECK(hipMemcpy(ts, d_ts, sizeof(ts), hipMemcpyDeviceToHost));
    uint64_t base = ts[0];
    for (int r = 0; r < 9; r++) base = std::min(base, ts[4 * r]);
    for (int i = 0; i < 36; i++) ph[i].push_back(ts[i] ? (ts[i] - base) / 100.0 : -1.0);  // 100 MHz -> us
  }
  const char* names[9] = {"R decode (rows)", "B rows 0-7", "B rows 8-15", "B rows 16-23", "B rows 24-31",
                          "SHA + A rows 0-7", "SHA + A rows 8-15", "SHA + A rows 16-23", "SHA + A rows 24-31"};
  for (int r = 0; r < 9; r++) {
    double m[4];
    for (int k = 0; k < 4; k++) {
      auto v = ph[4 * r + k];
      std::sort(v.begin(), v.end());
      m[k] = v[v.size() / 2];
    }
    printf("{\"role\": %d, \"what\": \"%s\", \"start_us\": %.1f, \"work_done_us\": %.1f, \"after_barrier_us\": %.1f, \"slot3_us\": %.1f}\n",
           r, names[r], m[0], m[1], m[2], m[3]);
  }
  return 0;
}
