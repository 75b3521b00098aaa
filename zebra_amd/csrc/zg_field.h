// zg_field.h -- BLS12-381 prime fields for gfx950: Fq (381-bit, 12 x 32-bit limbs) and
// Fr (255-bit, 8 x 32-bit limbs), Montgomery form (R = 2^384 / 2^256).
//
// Restates the arithmetic of pairing 0.14.2 `bls12_381::{Fq, Fr}` (6/4 x 64-bit limbs
// there) in the limb width CDNA4's VALU multiplies natively:
// every 32x32->64 product + 64-bit addend is one v_mad_u64_u32. MFMA is not used.
//
// Montgomery multiplication is the "no-carry" CIOS form: both moduli have a top limb
// below 2^31 - 1, so the running accumulator never needs an (N+1)-th word.
//
// Functions are __host__ __device__ so tests/native can execute the identical code on
// the CPU (test harness only; the product path launches it on the GPU).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "zg_constants.h"
#include "zg_fq_asm.h"

#define ZG_HD __host__ __device__
#define ZG_INL __host__ __device__ __forceinline__
// ZG_INLINE_ALL (a translation unit that defines it before any zebra header): every ZG_NOINL
// function is inlined into the unit's kernels -- no call frames, so no private segment for a kernel
// whose whole call tree fits its register budget (zg_decode_sqrt.hip)
#ifdef ZG_INLINE_ALL
#define ZG_NOINL __host__ __device__ __forceinline__
#else
#define ZG_NOINL __host__ __device__ __attribute__((noinline))
#endif
// ZG_DEC_INL: functions the decode unit (zg_decode.hip, ZG_TU_DECODE) inlines into its kernels -- the
// point wrappers that take their arguments by pointer / reference and B's square root, whose call
// frames were that kernel's private segment -- and that stay out of line everywhere else
#ifdef ZG_TU_DECODE
#define ZG_DEC_INL __host__ __device__ __forceinline__
#else
#define ZG_DEC_INL ZG_NOINL
#endif
#define ZG_POW_FN ZG_DEC_INL inline

// ZG_FQ29 (default): Fq products in 29-bit digits (zg_fq29.h / gen_fq29.py); 0: the 32-bit-word
// FIPS asm (zg_fips.h) on the device
#ifndef ZG_FQ29
#define ZG_FQ29 1
#endif
#include "zg_fq29_gen.h"

namespace zg {

struct FqM {
  static constexpr int N = 12;
  static constexpr uint32_t INV = FQ_INV;
  ZG_INL static uint32_t p(int i) { return FQ_P[i]; }
};
struct FrM {
  static constexpr int N = 8;
  static constexpr uint32_t INV = FR_INV;
  ZG_INL static uint32_t p(int i) { return FR_R[i]; }
};

template <class M>
struct Fp {
  uint32_t l[M::N];
};
using Fq = Fp<FqM>;
using Fr = Fp<FrM>;

template <class M>
ZG_INL Fp<M> fp_zero() {
  Fp<M> r;
#pragma unroll
  for (int i = 0; i < M::N; i++) r.l[i] = 0;
  return r;
}

ZG_INL Fq fq_one() {
  Fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = FQ_ONE[i];
  return r;
}
ZG_INL Fr fr_one() {
  Fr r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = FR_ONE[i];
  return r;
}
ZG_INL Fq fq_const(const uint32_t* c) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = c[i];
  return r;
}

template <class M>
ZG_INL bool fp_is_zero(const Fp<M>& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < M::N; i++) acc |= a.l[i];
  return acc == 0;
}

template <class M>
ZG_INL bool fp_eq(const Fp<M>& a, const Fp<M>& b) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < M::N; i++) acc |= a.l[i] ^ b.l[i];
  return acc == 0;
}

// r = a - p if a >= p else a   (a < 2p)
template <class M>
ZG_INL Fp<M> fp_reduce_once(const Fp<M>& a) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t m[M::N];
#pragma unroll
  for (int i = 0; i < M::N; i++) m[i] = M::p(i);
  Fp<M> r;
  mp_reduce_once<M::N>(r.l, a.l, m);
  return r;
#else
  Fp<M> d;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < M::N; i++) {
    uint64_t t = (uint64_t)a.l[i] - M::p(i) - borrow;
    d.l[i] = (uint32_t)t;
    borrow = (uint32_t)(t >> 63);
  }
  Fp<M> r;
#pragma unroll
  for (int i = 0; i < M::N; i++) r.l[i] = borrow ? a.l[i] : d.l[i];
  return r;
#endif
}

template <class M>
ZG_INL Fp<M> fp_add(const Fp<M>& a, const Fp<M>& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t m[M::N];
#pragma unroll
  for (int i = 0; i < M::N; i++) m[i] = M::p(i);
  Fp<M> r;
  if constexpr (M::N == 12)
    fqa_add(r.l, a.l, b.l);
  else
    mp_add_mod<M::N>(r.l, a.l, b.l, m);
  return r;
#else
  Fp<M> s;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < M::N; i++) {
    uint64_t t = (uint64_t)a.l[i] + b.l[i] + c;
    s.l[i] = (uint32_t)t;
    c = (uint32_t)(t >> 32);
  }
  return fp_reduce_once<M>(s);
#endif
}

template <class M>
ZG_INL Fp<M> fp_sub(const Fp<M>& a, const Fp<M>& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t m[M::N];
#pragma unroll
  for (int i = 0; i < M::N; i++) m[i] = M::p(i);
  Fp<M> r;
  if constexpr (M::N == 12)
    fqa_sub(r.l, a.l, b.l);
  else
    mp_sub_mod<M::N>(r.l, a.l, b.l, m);
  return r;
#else
  Fp<M> d;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < M::N; i++) {
    uint64_t t = (uint64_t)a.l[i] - b.l[i] - borrow;
    d.l[i] = (uint32_t)t;
    borrow = (uint32_t)(t >> 63);
  }
  // add back p masked by borrow
  uint32_t mask = 0u - borrow;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < M::N; i++) {
    uint64_t t = (uint64_t)d.l[i] + (M::p(i) & mask) + c;
    d.l[i] = (uint32_t)t;
    c = (uint32_t)(t >> 32);
  }
  return d;
#endif
}

template <class M>
ZG_INL Fp<M> fp_neg(const Fp<M>& a) {
  return fp_sub<M>(fp_zero<M>(), a);
}

template <class M>
ZG_INL Fp<M> fp_dbl(const Fp<M>& a) {
  return fp_add<M>(a, a);
}

// Montgomery product, no-carry CIOS. a, b < p  ->  result < p.
template <class M>
ZG_INL Fp<M> fp_mul_inl(const Fp<M>& a, const Fp<M>& b) {
  constexpr int N = M::N;
  uint32_t t[N];
#pragma unroll
  for (int j = 0; j < N; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    const uint32_t bi = b.l[i];
    uint64_t A = (uint64_t)a.l[0] * bi + t[0];
    t[0] = (uint32_t)A;
    A >>= 32;
    const uint32_t m = t[0] * M::INV;
    uint64_t C = ((uint64_t)m * M::p(0) + t[0]) >> 32;
#pragma unroll
    for (int j = 1; j < N; j++) {
      A = (uint64_t)a.l[j] * bi + t[j] + A;
      t[j] = (uint32_t)A;
      A >>= 32;
      C = (uint64_t)m * M::p(j) + t[j] + C;
      t[j - 1] = (uint32_t)C;
      C >>= 32;
    }
    t[N - 1] = (uint32_t)(C + A);
  }
  Fp<M> r;
#pragma unroll
  for (int j = 0; j < N; j++) r.l[j] = t[j];
  return fp_reduce_once<M>(r);
}

// Out-of-line multiply: the tower above calls this ~54x per Fq12 product; inlining all of
// them would blow the instruction cache. Operands cross the call as ext_vector values so
// the AMDGPU calling convention keeps them in VGPRs (a by-value aggregate of 12 dwords
// would go through scratch).
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

ZG_NOINL inline u32x16 fq_mul_v(u32x8 a0, u32x4 a1, u32x8 b0, u32x4 b1) {
  Fq a, b;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a.l[i] = a0[i];
    b.l[i] = b0[i];
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    a.l[8 + i] = a1[i];
    b.l[8 + i] = b1[i];
  }
  Fq r;
#if ZG_FQ29
  fq29_mul(r.l, a.l, b.l);     // 29-bit digits, carry-free v_mad_u64_u32 columns (host: same code)
#elif defined(__HIP_DEVICE_COMPILE__)
  fq_mul_fips(r.l, a.l, b.l);  // gfx950: v_mad_u64_u32 carry-out product scanning
#else
  r = fp_mul_inl<FqM>(a, b);   // host build of the test harness (tests/native): portable CIOS
#endif
  u32x16 o;
#pragma unroll
  for (int i = 0; i < 12; i++) o[i] = r.l[i];
  o[12] = o[13] = o[14] = o[15] = 0;
  return o;
}
ZG_INL Fq fq_mul(const Fq& a, const Fq& b) {
  u32x8 a0, b0;
  u32x4 a1, b1;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a0[i] = a.l[i];
    b0[i] = b.l[i];
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    a1[i] = a.l[8 + i];
    b1[i] = b.l[8 + i];
  }
  u32x16 o = fq_mul_v(a0, a1, b0, b1);
  Fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = o[i];
  return r;
}
ZG_NOINL inline u32x8 fr_mul_v(u32x8 a0, u32x8 b0) {
  Fr a, b;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a.l[i] = a0[i];
    b.l[i] = b0[i];
  }
  Fr r;
#if ZG_FQ29
  fr29_mul(r.l, a.l, b.l);     // 29-bit digits, carry-free columns (host: same code)
#elif defined(__HIP_DEVICE_COMPILE__)
  fr_mul_fips(r.l, a.l, b.l);  // gfx950: v_mad_u64_u32 carry-out product scanning
#else
  r = fp_mul_inl<FrM>(a, b);   // host build of the test harness (tests/native): portable CIOS
#endif
  u32x8 o;
#pragma unroll
  for (int i = 0; i < 8; i++) o[i] = r.l[i];
  return o;
}
ZG_INL Fr fr_mul(const Fr& a, const Fr& b) {
  u32x8 a0, b0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a0[i] = a.l[i];
    b0[i] = b.l[i];
  }
  u32x8 o = fr_mul_v(a0, b0);
  Fr r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = o[i];
  return r;
}

#if ZG_FQ29
ZG_NOINL inline u32x16 fq_sqr_v(u32x8 a0, u32x4 a1) {
  Fq a;
#pragma unroll
  for (int i = 0; i < 8; i++) a.l[i] = a0[i];
#pragma unroll
  for (int i = 0; i < 4; i++) a.l[8 + i] = a1[i];
  Fq r;
  fq29_sqr(r.l, a.l);  // 105 + 196 digit products (a < 2p)
  u32x16 o;
#pragma unroll
  for (int i = 0; i < 12; i++) o[i] = r.l[i];
  o[12] = o[13] = o[14] = o[15] = 0;
  return o;
}
ZG_INL Fq fq_sqr(const Fq& a) {
  u32x8 a0;
  u32x4 a1;
#pragma unroll
  for (int i = 0; i < 8; i++) a0[i] = a.l[i];
#pragma unroll
  for (int i = 0; i < 4; i++) a1[i] = a.l[8 + i];
  u32x16 o = fq_sqr_v(a0, a1);
  Fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = o[i];
  return r;
}
#else
ZG_INL Fq fq_sqr(const Fq& a) { return fq_mul(a, a); }
#endif
ZG_INL Fq fq_add(const Fq& a, const Fq& b) { return fp_add<FqM>(a, b); }
ZG_INL Fq fq_sub(const Fq& a, const Fq& b) { return fp_sub<FqM>(a, b); }
ZG_INL Fq fq_neg(const Fq& a) { return fp_neg<FqM>(a); }
ZG_INL Fq fq_dbl(const Fq& a) { return fp_add<FqM>(a, a); }
ZG_INL bool fq_is_zero(const Fq& a) { return fp_is_zero<FqM>(a); }
ZG_INL bool fq_eq(const Fq& a, const Fq& b) { return fp_eq<FqM>(a, b); }
ZG_INL Fr fr_add(const Fr& a, const Fr& b) { return fp_add<FrM>(a, b); }

// a^e for an exponent given as little-endian limbs (square-and-multiply, MSB first).
ZG_NOINL inline void fq_pow_limbs_p(Fq* out, const Fq* a, const uint32_t* e, int nbits) {
  Fq r = fq_one();
  const Fq base = *a;
  for (int i = nbits - 1; i >= 0; i--) {
    r = fq_sqr(r);
    if ((e[i >> 5] >> (i & 31)) & 1u) r = fq_mul(r, base);
  }
  *out = r;
}
ZG_INL Fq fq_pow_limbs(const Fq& a, const uint32_t* e, int nbits) {
  Fq r;
  fq_pow_limbs_p(&r, &a, e, nbits);
  return r;
}

// Variable-time inverse (binary extended Euclid) of a Montgomery-form element: public data
// only. Returns the Montgomery form of the inverse. a != 0.
ZG_NOINL inline Fq fq_inv_vartime(Fq a) {
  if (fq_is_zero(a)) return a;  // never reached for a Miller product; guards the loop
  Fq u = a, v, x1 = fp_zero<FqM>(), x2 = fp_zero<FqM>();
  for (int i = 0; i < 12; i++) v.l[i] = FQ_P[i];
  x1.l[0] = 1;
  auto is_one = [](const Fq& z) {
    uint32_t acc = z.l[0] ^ 1u;
    for (int i = 1; i < 12; i++) acc |= z.l[i];
    return acc == 0;
  };
  auto half = [](Fq& x) {  // x = x / 2 mod p  (x < p)
    uint32_t c = 0;
    if (x.l[0] & 1u) {
      for (int i = 0; i < 12; i++) {
        uint64_t s = (uint64_t)x.l[i] + FQ_P[i] + c;
        x.l[i] = (uint32_t)s;
        c = (uint32_t)(s >> 32);
      }
    }
    for (int i = 0; i < 11; i++) x.l[i] = (x.l[i] >> 1) | (x.l[i + 1] << 31);
    x.l[11] = (x.l[11] >> 1) | (c << 31);
  };
  auto shr1 = [](Fq& x) {
    for (int i = 0; i < 11; i++) x.l[i] = (x.l[i] >> 1) | (x.l[i + 1] << 31);
    x.l[11] >>= 1;
  };
  while (!is_one(u) && !is_one(v)) {
    while (!(u.l[0] & 1u)) {
      shr1(u);
      half(x1);
    }
    while (!(v.l[0] & 1u)) {
      shr1(v);
      half(x2);
    }
    // u >= v ?
    uint32_t borrow = 0;
    Fq d;
    for (int i = 0; i < 12; i++) {
      uint64_t t = (uint64_t)u.l[i] - v.l[i] - borrow;
      d.l[i] = (uint32_t)t;
      borrow = (uint32_t)(t >> 63);
    }
    if (!borrow) {
      u = d;
      x1 = fq_sub(x1, x2);
    } else {
      uint32_t b2 = 0;
      for (int i = 0; i < 12; i++) {
        uint64_t t = (uint64_t)v.l[i] - u.l[i] - b2;
        v.l[i] = (uint32_t)t;
        b2 = (uint32_t)(t >> 63);
      }
      x2 = fq_sub(x2, x1);
    }
  }
  Fq inv_plain = is_one(u) ? x1 : x2;       // (aR)^-1 as an integer mod p
  return fq_mul(inv_plain, fq_const(FQ_R3));  // (aR)^-1 * R^3 / R = a^-1 R
}


// fq_inv (Montgomery form in and out) is Pornin's binary GCD, zg_bingcd.h: branch-free, a fixed
// 26 outer steps (the same work on every lane of a wave), ~20 k instructions against ~280 k for
// Fermat and a lane-divergent loop for fq_inv_vartime
// constant-time Fermat inverse (kept for reference / tests)
ZG_INL Fq fq_inv_fermat(const Fq& a) { return fq_pow_limbs(a, FQ_EXP_INV, 381); }

// a^((p-3)/4) by a sliding-window chain of zg_constants.h.
#ifndef ZG_SQRT_W
#define ZG_SQRT_W 4
#endif
#if ZG_FQ29 && (ZG_SQRT_W == 3 || ZG_SQRT_W == 4)
// w = 4 (375 squarings + 79 multiplications, 8 odd powers) or w = 3 (377 + 106, 4 odd powers): the
// chain is the same for every lane, so the table index is wave-uniform and a switch on it reads
// fixed registers -- the table stays in VGPRs (112 or 56) instead of the private segment a
// runtime-indexed array needs.
#if ZG_SQRT_W == 4
#define ZG_SQ_CHAIN FQ_PM3_4_CHAIN4
#define ZG_SQ_CHAIN_LEN FQ_PM3_4_CHAIN4_LEN
#else
#define ZG_SQ_CHAIN FQ_PM3_4_CHAIN3
#define ZG_SQ_CHAIN_LEN FQ_PM3_4_CHAIN3_LEN
#endif
struct Fq29D {
  uint32_t d[14];
};
// s = T_k for a wave-uniform k: eight separate values and copies in the arms of a switch, so
// nothing indexes an array at run time
ZG_INL void fq29d_pick8(uint32_t* s, const Fq29D& T0, const Fq29D& T1, const Fq29D& T2, const Fq29D& T3,
                        const Fq29D& T4, const Fq29D& T5, const Fq29D& T6, const Fq29D& T7, int k) {
  Fq29D v;
  switch (k) {
    case 0: v = T0; break;
    case 1: v = T1; break;
    case 2: v = T2; break;
    case 3: v = T3; break;
    case 4: v = T4; break;
    case 5: v = T5; break;
    case 6: v = T6; break;
    default: v = T7; break;
  }
#pragma unroll
  for (int w = 0; w < 14; w++) s[w] = v.d[w];
}
#endif
ZG_POW_FN void fq_pow_pm3_4_p(Fq* out, const Fq* ap) {
#if ZG_FQ29 && (ZG_SQRT_W == 3 || ZG_SQRT_W == 4)
  // digit-resident chain (Montgomery R' = 2^406, zg_fq29_gen.h fq29d_*)
  Fq29D T0, T1, T2, T3;
  uint32_t a2[14], r[14], t[14], s[14];
  fq29d_from_mont(T0.d, ap->l);
  fq29d_sqr(a2, T0.d);
  fq29d_mul(T1.d, T0.d, a2);
  fq29d_mul(T2.d, T1.d, a2);
  fq29d_mul(T3.d, T2.d, a2);
#if ZG_SQRT_W == 4
  Fq29D T4, T5, T6, T7;
  fq29d_mul(T4.d, T3.d, a2);
  fq29d_mul(T5.d, T4.d, a2);
  fq29d_mul(T6.d, T5.d, a2);
  fq29d_mul(T7.d, T6.d, a2);
#else
  const Fq29D &T4 = T3, &T5 = T3, &T6 = T3, &T7 = T3;  // never picked
#endif
  fq29d_pick8(r, T0, T1, T2, T3, T4, T5, T6, T7, ZG_SQ_CHAIN[0][1] >> 1);
  for (int i = 1; i < ZG_SQ_CHAIN_LEN; i++) {
    for (int q = 0; q < ZG_SQ_CHAIN[i][0]; q++) {
      fq29d_sqr(t, r);
#pragma unroll
      for (int w = 0; w < 14; w++) r[w] = t[w];
    }
    const int o = ZG_SQ_CHAIN[i][1];
    if (o) {
      fq29d_pick8(s, T0, T1, T2, T3, T4, T5, T6, T7, o >> 1);
      fq29d_mul(t, r, s);
#pragma unroll
      for (int w = 0; w < 14; w++) r[w] = t[w];
    }
  }
  fq29d_to_mont(out->l, r);
#elif ZG_FQ29
  // w = 5 (375 squarings + 67 multiplications; 16 odd powers, a runtime-indexed table)
  uint32_t tbl[16][14], a2[14], r[14], t[14];
  fq29d_from_mont(tbl[0], ap->l);
  fq29d_sqr(a2, tbl[0]);
  for (int k = 1; k < 16; k++) fq29d_mul(tbl[k], tbl[k - 1], a2);
#pragma unroll
  for (int w = 0; w < 14; w++) r[w] = tbl[FQ_PM3_4_CHAIN[0][1] >> 1][w];
  for (int i = 1; i < FQ_PM3_4_CHAIN_LEN; i++) {
    for (int s = 0; s < FQ_PM3_4_CHAIN[i][0]; s++) {
      fq29d_sqr(t, r);
#pragma unroll
      for (int w = 0; w < 14; w++) r[w] = t[w];
    }
    const int o = FQ_PM3_4_CHAIN[i][1];
    if (o) {
      fq29d_mul(t, r, tbl[o >> 1]);
#pragma unroll
      for (int w = 0; w < 14; w++) r[w] = t[w];
    }
  }
  fq29d_to_mont(out->l, r);
#else
  Fq tbl[16];
  tbl[0] = *ap;
  const Fq a2 = fq_sqr(tbl[0]);
  for (int k = 1; k < 16; k++) tbl[k] = fq_mul(tbl[k - 1], a2);
  Fq r = tbl[FQ_PM3_4_CHAIN[0][1] >> 1];
  for (int i = 1; i < FQ_PM3_4_CHAIN_LEN; i++) {
    for (int s = 0; s < FQ_PM3_4_CHAIN[i][0]; s++) r = fq_sqr(r);
    const int o = FQ_PM3_4_CHAIN[i][1];
    if (o) r = fq_mul(r, tbl[o >> 1]);
  }
  *out = r;
#endif
}
ZG_INL Fq fq_pow_pm3_4(const Fq& a) {
  Fq r;
  fq_pow_pm3_4_p(&r, &a);
  return r;
}

// Returns true and sets *out if a is a square (pairing Fq::sqrt: p = 3 mod 4, root a^((p+1)/4)).
ZG_INL bool fq_sqrt(const Fq& a, Fq* out) {
  Fq s = fq_mul(fq_pow_pm3_4(a), a);
  *out = s;
  return fq_eq(fq_sqr(s), a);
}

// a / 2 (Montgomery form is preserved: (aR)/2 = (a/2)R)
ZG_INL Fq fq_half(const Fq& a) {
  Fq x = a;
  uint32_t c = 0;
  const uint32_t odd = 0u - (x.l[0] & 1u);
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t s = (uint64_t)x.l[i] + (FQ_P[i] & odd) + c;
    x.l[i] = (uint32_t)s;
    c = (uint32_t)(s >> 32);
  }
#pragma unroll
  for (int i = 0; i < 11; i++) x.l[i] = (x.l[i] >> 1) | (x.l[i + 1] << 31);
  x.l[11] = (x.l[11] >> 1) | (c << 31);
  return x;
}

// canonical (non-Montgomery) limbs <-> Montgomery
ZG_INL Fq fq_to_mont(const Fq& a) { return fq_mul(a, fq_const(FQ_R2)); }
ZG_INL Fq fq_from_mont(const Fq& a) {
  Fq one;
#pragma unroll
  for (int i = 0; i < 12; i++) one.l[i] = i == 0 ? 1u : 0u;
  return fq_mul(a, one);
}

// Compare canonical integers (non-Montgomery limbs): a > b
template <class M>
ZG_INL bool fp_gt_canon(const Fp<M>& a, const Fp<M>& b) {
  // a > b  <=>  b - a borrows
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < M::N; i++) {
    uint64_t t = (uint64_t)b.l[i] - a.l[i] - borrow;
    borrow = (uint32_t)(t >> 63);
  }
  return borrow != 0;
}

// canonical limbs < modulus ?
template <class M>
ZG_INL bool fp_lt_modulus(const Fp<M>& a) {
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < M::N; i++) {
    uint64_t t = (uint64_t)a.l[i] - M::p(i) - borrow;
    borrow = (uint32_t)(t >> 63);
  }
  return borrow != 0;
}

// 48 big-endian bytes -> canonical limbs
ZG_INL Fq fq_limbs_from_be(const uint8_t* b) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint8_t* q = b + 44 - 4 * i;
    r.l[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
  return r;
}
ZG_INL void fq_limbs_to_be(const Fq& a, uint8_t* b) {
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint8_t* q = b + 44 - 4 * i;
    q[0] = (uint8_t)(a.l[i] >> 24);
    q[1] = (uint8_t)(a.l[i] >> 16);
    q[2] = (uint8_t)(a.l[i] >> 8);
    q[3] = (uint8_t)a.l[i];
  }
}
// 32 little-endian bytes -> canonical Fr limbs
ZG_INL Fr fr_limbs_from_le(const uint8_t* b) {
  Fr r;
#pragma unroll
  for (int i = 0; i < 8; i++)
    r.l[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
             ((uint32_t)b[4 * i + 3] << 24);
  return r;
}
ZG_INL Fr fr_to_mont(const Fr& a) {
  Fr r2;
#pragma unroll
  for (int i = 0; i < 8; i++) r2.l[i] = FR_R2[i];
  return fr_mul(a, r2);
}
ZG_INL Fr fr_from_mont(const Fr& a) {
  Fr one;
#pragma unroll
  for (int i = 0; i < 8; i++) one.l[i] = i == 0 ? 1u : 0u;
  return fr_mul(a, one);
}

}  // namespace zg
