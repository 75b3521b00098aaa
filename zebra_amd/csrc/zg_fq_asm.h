// zg_fq_asm.h -- gfx950 Montgomery multiplication for Fq, Finely Integrated Product
// Scanning (FIPS) with a 3-word column accumulator. Each 32x32 product is ONE
// v_mad_u64_u32 into the 64-bit {lo, mid} pair whose carry-out (an SGPR lane mask) feeds
// ONE v_addc_co_u32 into the top word: 2 VALU instructions per MAC, 288 MACs per product.
// (The compiler's own lowering of the same C needs 4-5 instructions per MAC: it cannot
// use the mad's carry-out.)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "zg_constants.h"

namespace zg {

struct Acc3 {
  uint64_t lm;  // low + middle words
  uint32_t h;   // high word
};

__device__ __forceinline__ void mac3(Acc3& a, uint32_t x, uint32_t y) {
  uint64_t c;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(a.lm), "=s"(c) : "v"(x), "v"(y));
  asm("v_addc_co_u32 %0, vcc, 0, %0, %1" : "+v"(a.h) : "s"(c) : "vcc");
}
__device__ __forceinline__ void mac3s(Acc3& a, uint32_t x, uint32_t ys) {  // y uniform (SGPR)
  uint64_t c;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(a.lm), "=s"(c) : "v"(x), "s"(ys));
  asm("v_addc_co_u32 %0, vcc, 0, %0, %1" : "+v"(a.h) : "s"(c) : "vcc");
}
__device__ __forceinline__ uint32_t shift3(Acc3& a) {
  uint32_t lo = (uint32_t)a.lm;
  a.lm = (a.lm >> 32) | ((uint64_t)a.h << 32);
  a.h = 0;
  return lo;
}

// ---- multi-limb add / sub / select on VALU carry chains (device only).
// The C formulation (uint64_t sums, >> 32 carries) compiles to 64-bit shift-adds and moves,
// ~5 instructions per limb; these are 1 (v_add_co / v_addc_co / v_sub_co / v_subb_co with
// the carry in an SGPR-pair lane mask) plus 1 v_cndmask per limb for a reduction.
__device__ __forceinline__ uint32_t asm_add_co(uint32_t a, uint32_t b, uint64_t& co) {
  uint32_t r;
  asm volatile("v_add_co_u32 %0, %1, %2, %3" : "=v"(r), "=s"(co) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t asm_addc(uint32_t a, uint32_t b, uint64_t ci, uint64_t& co) {
  uint32_t r;
  asm volatile("v_addc_co_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(co) : "v"(a), "v"(b), "s"(ci));
  return r;
}
__device__ __forceinline__ uint32_t asm_sub_co(uint32_t a, uint32_t b, uint64_t& bo) {
  uint32_t r;
  asm volatile("v_sub_co_u32 %0, %1, %2, %3" : "=v"(r), "=s"(bo) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t asm_subb(uint32_t a, uint32_t b, uint64_t bi, uint64_t& bo) {
  uint32_t r;
  asm volatile("v_subb_co_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(bo) : "v"(a), "v"(b), "s"(bi));
  return r;
}
// m (lane mask) set -> t, else f
__device__ __forceinline__ uint32_t asm_sel(uint32_t f, uint32_t t, uint64_t m) {
  uint32_t r;
  asm volatile("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
  return r;
}

// r = a + b (N limbs), returns the carry-out mask
template <int N>
__device__ __forceinline__ uint64_t mp_add(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint64_t c;
  r[0] = asm_add_co(a[0], b[0], c);
#pragma unroll
  for (int i = 1; i < N; i++) r[i] = asm_addc(a[i], b[i], c, c);
  return c;
}
// r = a - b (N limbs), returns the borrow-out mask
template <int N>
__device__ __forceinline__ uint64_t mp_sub(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint64_t c;
  r[0] = asm_sub_co(a[0], b[0], c);
#pragma unroll
  for (int i = 1; i < N; i++) r[i] = asm_subb(a[i], b[i], c, c);
  return c;
}
// a < 2m -> a mod m
template <int N>
__device__ __forceinline__ void mp_reduce_once(uint32_t* r, const uint32_t* a, const uint32_t* m) {
  uint32_t d[N];
  const uint64_t bo = mp_sub<N>(d, a, m);
#pragma unroll
  for (int i = 0; i < N; i++) r[i] = asm_sel(d[i], a[i], bo);  // borrow: a < m, keep a
}
// (a + b) mod m for a, b < m
template <int N>
__device__ __forceinline__ void mp_add_mod(uint32_t* r, const uint32_t* a, const uint32_t* b, const uint32_t* m) {
  uint32_t s[N];
  mp_add<N>(s, a, b);  // < 2m < 2^(32N): no carry-out
  mp_reduce_once<N>(r, s, m);
}
// (a - b) mod m for a, b < m
template <int N>
__device__ __forceinline__ void mp_sub_mod(uint32_t* r, const uint32_t* a, const uint32_t* b, const uint32_t* m) {
  uint32_t d[N], e[N];
  const uint64_t bo = mp_sub<N>(d, a, b);
  mp_add<N>(e, d, m);
#pragma unroll
  for (int i = 0; i < N; i++) r[i] = asm_sel(d[i], e[i], bo);  // borrow: a < b, add m back
}

#include "zg_fips.h"

}  // namespace zg
