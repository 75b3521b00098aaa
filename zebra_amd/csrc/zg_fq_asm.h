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

// r = a * b * 2^-384 mod p ; a, b < p  ->  r < p
__device__ __forceinline__ void fq_mul_fips(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  constexpr int N = 12;
  uint32_t m[N];
  Acc3 acc = {0, 0};
#pragma unroll
  for (int i = 0; i < N; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) {
      mac3(acc, a[j], b[i - j]);
      mac3s(acc, m[j], FQ_P[i - j]);
    }
    mac3(acc, a[i], b[0]);
    m[i] = (uint32_t)acc.lm * FQ_INV;
    mac3s(acc, m[i], FQ_P[0]);
    shift3(acc);
  }
  uint32_t t[N];
#pragma unroll
  for (int i = N; i < 2 * N - 1; i++) {
#pragma unroll
    for (int j = i - N + 1; j < N; j++) {
      mac3(acc, a[j], b[i - j]);
      mac3s(acc, m[j], FQ_P[i - j]);
    }
    t[i - N] = shift3(acc);
  }
  t[N - 1] = (uint32_t)acc.lm;  // < 2p < 2^382: no further carry
  // conditional subtraction
  uint32_t d[N], borrow = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    uint64_t s = (uint64_t)t[i] - FQ_P[i] - borrow;
    d[i] = (uint32_t)s;
    borrow = (uint32_t)(s >> 63);
  }
#pragma unroll
  for (int i = 0; i < N; i++) r[i] = borrow ? t[i] : d[i];
}

}  // namespace zg
