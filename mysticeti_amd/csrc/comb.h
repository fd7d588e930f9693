// Per-key comb tables (comb.hip builds them at mv_set_committee / mv_create) and the
// lookup-and-add shared by the comb verify (comb.hip) and the batch path's per-key term
// (batch.hip): C[i][j] = [j * 256^i](+-P), i = 0..31, j = 0..128, affine precomp points
// (y+x, y-x, 2dxy), one 128-byte line per entry.
#pragma once
#include "fe25519.h"
#include "ge25519.h"
#include "scalar25519.h"
#include "tables.h"

namespace mv {

constexpr int CT_QUADS = 8;      // 27 limb words, padded to one 128-B line
constexpr int CT_ENTRIES = 129;  // j = 0..128
constexpr int CT_ROWS = 32;      // radix-256 digit positions
constexpr int CT_ROW = CT_ENTRIES * CT_QUADS;
constexpr int CT_TABLE = CT_ROWS * CT_ROW;  // uint4 per base point

MV_DEV void ct_load(uint4 (&q)[7], const uint4* row, int digit) {
  const int e = digit < 0 ? -digit : digit;
  const uint4* p = row + e * CT_QUADS;
#pragma unroll
  for (int k = 0; k < 7; k++) q[k] = p[k];
}

// acc = sum over rows i in [r0, r1) of C[i][digit i of sd] (signed radix-256 digits);
// each entry is loaded one addition ahead, unconditionally (the last lap reloads row r1 - 1): a
// load under a branch has the compiler copy the quads inside the branch, waiting on them at once
MV_DEV void ct_sum(p3& acc, const uint4* tab, const uint32_t sd[8], int r0, int r1) {
  p3_identity(acc);
  uint4 q[7];
  int dg = digit256(sd, r0);
  ct_load(q, tab + (size_t)r0 * CT_ROW, dg);
#pragma unroll 1
  for (int i = r0; i < r1; i++) {
    precomp pc;
    quads_to_precomp(pc, q);
    const bool neg = dg < 0;
    const int in = i + 1 < r1 ? i + 1 : r1 - 1;
    dg = digit256(sd, in);
    ct_load(q, tab + (size_t)in * CT_ROW, dg);
    precomp_cneg(pc, neg);
    p1p1 t;
    p3_add_precomp(t, acc, pc);
    p1p1_to_p3(acc, t);
  }
}

}  // namespace mv
