// 32-bit carry-chain primitives (v_add_co / v_addc with SGPR carries) for the
// scalar-mod-l arithmetic (scalar25519.h). Not used by the field layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef MV_DEV
#define MV_DEV __device__ __forceinline__
#endif

namespace mv {

// ---- carry-flag primitives (wave64 carry masks live in SGPR pairs) ----
// Volatile: their relative order is the interleaving schedule.
MV_DEV void a_mad(uint64_t& acc, uint64_t& cm, uint32_t a, uint32_t b) {
  asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cm) : "v"(a), "v"(b));
}
MV_DEV void a_cnt(uint32_t& c2, uint64_t& cm) {  // c2 += carry
  asm volatile("v_addc_co_u32 %0, %1, %0, 0, %1" : "+v"(c2), "+s"(cm));
}
MV_DEV uint32_t add_co(uint32_t a, uint32_t b, uint64_t& cm) {
  uint32_t r;
  asm volatile("v_add_co_u32 %0, %1, %2, %3" : "=v"(r), "=s"(cm) : "v"(a), "v"(b));
  return r;
}
MV_DEV uint32_t addc_co(uint32_t a, uint32_t b, uint64_t& cm) {
  uint32_t r;
  asm volatile("v_addc_co_u32 %0, %1, %2, %3, %1" : "=v"(r), "+s"(cm) : "v"(a), "v"(b));
  return r;
}
MV_DEV uint32_t addc0(uint32_t a, uint64_t& cm) {  // a + carry, carry out
  uint32_t r;
  asm volatile("v_addc_co_u32 %0, %1, %2, 0, %1" : "=v"(r), "+s"(cm) : "v"(a));
  return r;
}
MV_DEV uint32_t sub_co(uint32_t a, uint32_t b, uint64_t& bm) {
  uint32_t r;
  asm volatile("v_sub_co_u32 %0, %1, %2, %3" : "=v"(r), "=s"(bm) : "v"(a), "v"(b));
  return r;
}
MV_DEV uint32_t subb_co(uint32_t a, uint32_t b, uint64_t& bm) {
  uint32_t r;
  asm volatile("v_subb_co_u32 %0, %1, %2, %3, %1" : "=v"(r), "+s"(bm) : "v"(a), "v"(b));
  return r;
}
MV_DEV uint32_t subb0(uint32_t a, uint64_t& bm) {  // a - borrow, borrow out
  uint32_t r;
  asm volatile("v_subb_co_u32 %0, %1, %2, 0, %1" : "=v"(r), "+s"(bm) : "v"(a));
  return r;
}
// carry/borrow bit of the lane as 0/1
MV_DEV uint32_t carry_bit(uint64_t& cm) {
  uint32_t r;
  asm volatile("v_cndmask_b32 %0, 0, 1, %1" : "=v"(r) : "s"(cm));
  return r;
}
// plain 32x32+64 -> 64 (no carry-out consumer)
MV_DEV uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t r, cm;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cm) : "v"(a), "v"(b), "v"(c));
  return r;
}
// one serial MAC into a 96-bit (acc, c2) accumulator (scalar arithmetic, not hot)
MV_DEV void mac(uint64_t& acc, uint32_t& c2, uint32_t a, uint32_t b) {
  uint64_t cm;
  a_mad(acc, cm, a, b);
  a_cnt(c2, cm);
}

}  // namespace mv
