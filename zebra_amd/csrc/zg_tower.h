// zg_tower.h -- the BLS12-381 extension tower on gfx950 (restates pairing 0.14.2
// Fq2/Fq6/Fq12):
//   Fq2  = Fq[u]  / (u^2 + 1)
//   Fq6  = Fq2[v] / (v^3 - xi),  xi = u + 1
//   Fq12 = Fq6[w] / (w^2 - v)
// Products use Karatsuba at every level (Fq2 mul = 3 Fq mul, Fq6 mul = 6 Fq2 mul,
// Fq12 mul = 3 Fq6 mul = 54 Fq mul). Sparse line products (mul_by_014) cost 13 Fq2 mul.
#pragma once
#include "zg_bingcd.h"  // fq_inv (includes zg_field.h)

namespace zg {

struct Fq2 {
  Fq c0, c1;
};
struct Fq6 {
  Fq2 c0, c1, c2;
};
struct Fq12 {
  Fq6 c0, c1;
};

// ------------------------------------------------------------------ Fq2
ZG_INL Fq2 f2_zero() { return {fp_zero<FqM>(), fp_zero<FqM>()}; }
ZG_INL Fq2 f2_one() { return {fq_one(), fp_zero<FqM>()}; }
ZG_INL Fq2 f2_const(const uint32_t c[2][12]) { return {fq_const(c[0]), fq_const(c[1])}; }
// device: both coefficients' carry chains in one interleaved asm statement (zg_fips.h)
ZG_INL Fq2 f2_add(const Fq2& a, const Fq2& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  Fq2 r;
  f2a_add(r.c0.l, a.c0.l, b.c0.l, r.c1.l, a.c1.l, b.c1.l);
  return r;
#else
  return {fq_add(a.c0, b.c0), fq_add(a.c1, b.c1)};
#endif
}
ZG_INL Fq2 f2_sub(const Fq2& a, const Fq2& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  Fq2 r;
  f2a_sub(r.c0.l, a.c0.l, b.c0.l, r.c1.l, a.c1.l, b.c1.l);
  return r;
#else
  return {fq_sub(a.c0, b.c0), fq_sub(a.c1, b.c1)};
#endif
}
ZG_INL Fq2 f2_neg(const Fq2& a) { return f2_sub({fp_zero<FqM>(), fp_zero<FqM>()}, a); }
ZG_INL Fq2 f2_dbl(const Fq2& a) { return f2_add(a, a); }
ZG_INL Fq2 f2_conj(const Fq2& a) { return {a.c0, fq_neg(a.c1)}; }
ZG_INL bool f2_is_zero(const Fq2& a) { return fq_is_zero(a.c0) && fq_is_zero(a.c1); }
ZG_INL bool f2_eq(const Fq2& a, const Fq2& b) { return fq_eq(a.c0, b.c0) && fq_eq(a.c1, b.c1); }

ZG_INL Fq2 f2_mul(const Fq2& a, const Fq2& b) {
  Fq t0 = fq_mul(a.c0, b.c0);
  Fq t1 = fq_mul(a.c1, b.c1);
  Fq t2 = fq_mul(fq_add(a.c0, a.c1), fq_add(b.c0, b.c1));
  return {fq_sub(t0, t1), fq_sub(fq_sub(t2, t0), t1)};
}
ZG_INL Fq2 f2_sqr(const Fq2& a) {
  Fq t = fq_mul(a.c0, a.c1);
  return {fq_mul(fq_add(a.c0, a.c1), fq_sub(a.c0, a.c1)), fq_dbl(t)};
}
ZG_INL Fq2 f2_mul_fq(const Fq2& a, const Fq& s) { return {fq_mul(a.c0, s), fq_mul(a.c1, s)}; }
// multiply by xi = u + 1
ZG_INL Fq2 f2_mul_nr(const Fq2& a) {
#if defined(__HIP_DEVICE_COMPILE__)
  Fq2 r;
  f2a_sub_add(r.c0.l, a.c0.l, a.c1.l, r.c1.l, a.c0.l, a.c1.l);
  return r;
#else
  return {fq_sub(a.c0, a.c1), fq_add(a.c0, a.c1)};
#endif
}
ZG_NOINL inline void f2_inv_p(Fq2* r, const Fq2* ap) {
  const Fq2 a = *ap;
  Fq t = fq_inv(fq_add(fq_sqr(a.c0), fq_sqr(a.c1)));
  *r = {fq_mul(a.c0, t), fq_neg(fq_mul(a.c1, t))};
}
ZG_INL Fq2 f2_inv(const Fq2& a) {
  Fq2 r;
  f2_inv_p(&r, &a);
  return r;
}
ZG_NOINL inline void f2_pow_limbs_p(Fq2* out, const Fq2* a, const uint32_t* e, int nbits) {
  Fq2 r = f2_one();
  const Fq2 base = *a;
  for (int i = nbits - 1; i >= 0; i--) {
    r = f2_sqr(r);
    if ((e[i >> 5] >> (i & 31)) & 1u) r = f2_mul(r, base);
  }
  *out = r;
}
ZG_INL Fq2 f2_pow_limbs(const Fq2& a, const uint32_t* e, int nbits) {
  Fq2 r;
  f2_pow_limbs_p(&r, &a, e, nbits);
  return r;
}
// Square root in Fq2 by the norm ("complex") method: two Fq exponentiations by (p-3)/4
// instead of the two Fq2 exponentiations of pairing's Fq2::sqrt (Algorithm 9 of eprint
// 2012/685); ~920 vs ~2,660 Fq multiplications. The decoders pick the sign of y from the
// encoding flag afterwards, so which of the two roots is returned does not matter
// (SURVEY.md 8(a) row a4). For a = a0 + a1 u with a1 != 0:
//   g = sqrt(a0^2 + a1^2) (a is a square in Fq2 iff its norm is a square in Fq),
//   d = (a0 + g)/2 != 0, e = d^((p-3)/4):
//   d a square:  y = e d + (a1 e / 2) u          ((e d)^2 = d, 1/(e d) = e)
//   otherwise :  y = a1 e / 2 - (e d) u          (-d is a square; (p-3)/4 is even)
ZG_DEC_INL inline bool f2_sqrt(const Fq2& a, Fq2* out) {
  // one call site of the exponentiation (pass 0: a0, or the norm n; pass 1: d), so a unit that
  // inlines it (ZG_DEC_INL) holds one copy
  const bool c1z = fq_is_zero(a.c1);
  const Fq n = c1z ? a.c0 : fq_add(fq_sqr(a.c0), fq_sqr(a.c1));
  Fq x = n, e0 = n, d = n;
  bool ok = true;
  for (int pass = 0; pass < 2; pass++) {
    const Fq e = fq_pow_pm3_4(x);
    if (pass == 1) {
      e0 = e;
      break;
    }
    if (c1z) {  // a in Fq: sqrt(a0) or sqrt(-a0) u; (-a0)^((p-3)/4) == e too: (p-3)/4 is even
      e0 = e;
      break;
    }
    const Fq g = fq_mul(e, n);
    if (!fq_eq(fq_sqr(g), n)) {
      ok = false;
      break;
    }
    d = fq_half(fq_add(a.c0, g));
    x = d;
  }
  if (!ok) return false;
  if (c1z) {
    const Fq s = fq_mul(e0, a.c0);
    if (fq_eq(fq_sqr(s), a.c0)) {
      *out = {s, fp_zero<FqM>()};
      return true;
    }
    const Fq t = fq_neg(s);  // e * (-a0)
    *out = {fp_zero<FqM>(), t};
    return fq_eq(fq_sqr(t), fq_neg(a.c0));
  }
  const Fq ed = fq_mul(e0, d);
  const Fq h = fq_half(fq_mul(a.c1, e0));
  Fq2 y;
  if (fq_eq(fq_sqr(ed), d))
    y = {ed, h};
  else
    y = {h, fq_neg(ed)};
  *out = y;
  return f2_eq(f2_sqr(y), a);
}

// ------------------------------------------------------------------ Fq6
ZG_INL Fq6 f6_zero() { return {f2_zero(), f2_zero(), f2_zero()}; }
ZG_INL Fq6 f6_one() { return {f2_one(), f2_zero(), f2_zero()}; }
ZG_INL Fq6 f6_add(const Fq6& a, const Fq6& b) {
  return {f2_add(a.c0, b.c0), f2_add(a.c1, b.c1), f2_add(a.c2, b.c2)};
}
ZG_INL Fq6 f6_sub(const Fq6& a, const Fq6& b) {
  return {f2_sub(a.c0, b.c0), f2_sub(a.c1, b.c1), f2_sub(a.c2, b.c2)};
}
ZG_INL Fq6 f6_neg(const Fq6& a) { return {f2_neg(a.c0), f2_neg(a.c1), f2_neg(a.c2)}; }
// multiply by v: (c0, c1, c2) -> (xi c2, c0, c1)
ZG_INL Fq6 f6_mul_nr(const Fq6& a) { return {f2_mul_nr(a.c2), a.c0, a.c1}; }
ZG_INL bool f6_is_zero(const Fq6& a) { return f2_is_zero(a.c0) && f2_is_zero(a.c1) && f2_is_zero(a.c2); }
ZG_INL bool f6_eq(const Fq6& a, const Fq6& b) {
  return f2_eq(a.c0, b.c0) && f2_eq(a.c1, b.c1) && f2_eq(a.c2, b.c2);
}

ZG_INL Fq6 f6_mul(const Fq6& a, const Fq6& b) {
  Fq2 t0 = f2_mul(a.c0, b.c0);
  Fq2 t1 = f2_mul(a.c1, b.c1);
  Fq2 t2 = f2_mul(a.c2, b.c2);
  Fq2 c0 = f2_add(f2_mul_nr(f2_sub(f2_sub(f2_mul(f2_add(a.c1, a.c2), f2_add(b.c1, b.c2)), t1), t2)), t0);
  Fq2 c1 = f2_add(f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c1), f2_add(b.c0, b.c1)), t0), t1), f2_mul_nr(t2));
  Fq2 c2 = f2_add(f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c2), f2_add(b.c0, b.c2)), t0), t2), t1);
  return {c0, c1, c2};
}
// a * (b0 + b1 v)   (5 Fq2 mul)
ZG_INL Fq6 f6_mul_by_01(const Fq6& a, const Fq2& b0, const Fq2& b1) {
  Fq2 t0 = f2_mul(a.c0, b0);
  Fq2 t1 = f2_mul(a.c1, b1);
  Fq2 c0 = f2_add(f2_mul_nr(f2_mul(f2_add(a.c1, a.c2), b1)), t0);
  c0 = f2_sub(c0, f2_mul_nr(t1));
  Fq2 c1 = f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c1), f2_add(b0, b1)), t0), t1);
  Fq2 c2 = f2_add(f2_sub(f2_mul(f2_add(a.c0, a.c2), b0), t0), t1);
  return {c0, c1, c2};
}
// a * (b1 v)   (3 Fq2 mul)
ZG_INL Fq6 f6_mul_by_1(const Fq6& a, const Fq2& b1) {
  return {f2_mul_nr(f2_mul(a.c2, b1)), f2_mul(a.c0, b1), f2_mul(a.c1, b1)};
}
ZG_INL Fq6 f6_inv(const Fq6& a) {
  Fq2 c0 = f2_sub(f2_sqr(a.c0), f2_mul_nr(f2_mul(a.c1, a.c2)));
  Fq2 c1 = f2_sub(f2_mul_nr(f2_sqr(a.c2)), f2_mul(a.c0, a.c1));
  Fq2 c2 = f2_sub(f2_sqr(a.c1), f2_mul(a.c0, a.c2));
  Fq2 t = f2_add(f2_mul(a.c0, c0), f2_mul_nr(f2_add(f2_mul(a.c2, c1), f2_mul(a.c1, c2))));
  Fq2 ti = f2_inv(t);
  return {f2_mul(c0, ti), f2_mul(c1, ti), f2_mul(c2, ti)};
}

// ------------------------------------------------------------------ Fq12
ZG_INL Fq12 f12_one() { return {f6_one(), f6_zero()}; }
ZG_INL Fq12 f12_conj(const Fq12& a) { return {a.c0, f6_neg(a.c1)}; }
ZG_INL bool f12_eq(const Fq12& a, const Fq12& b) { return f6_eq(a.c0, b.c0) && f6_eq(a.c1, b.c1); }
ZG_INL bool f12_is_zero(const Fq12& a) { return f6_is_zero(a.c0) && f6_is_zero(a.c1); }
ZG_INL bool f12_is_one(const Fq12& a) { return f12_eq(a, f12_one()); }

ZG_INL Fq12 f12_mul_inl(const Fq12& a, const Fq12& b) {
  Fq6 t0 = f6_mul(a.c0, b.c0);
  Fq6 t1 = f6_mul(a.c1, b.c1);
  Fq6 c1 = f6_sub(f6_sub(f6_mul(f6_add(a.c0, a.c1), f6_add(b.c0, b.c1)), t0), t1);
  return {f6_add(t0, f6_mul_nr(t1)), c1};
}
// complex squaring: (a0 + a1 w)^2 = (a0^2 + v a1^2) + 2 a0 a1 w, with 2 Fq6 products
ZG_INL Fq12 f12_sqr_inl(const Fq12& a) {
  Fq6 ab = f6_mul(a.c0, a.c1);
  Fq6 c0 = f6_mul(f6_add(a.c0, a.c1), f6_add(a.c0, f6_mul_nr(a.c1)));
  c0 = f6_sub(f6_sub(c0, ab), f6_mul_nr(ab));
  return {c0, f6_add(ab, ab)};
}
// f * ((c0 + c1 v) + (c4 v) w)   -- pairing Fq12::mul_by_014, 13 Fq2 mul
ZG_INL Fq12 f12_mul_by_014_inl(const Fq12& f, const Fq2& c0, const Fq2& c1, const Fq2& c4) {
  Fq6 aa = f6_mul_by_01(f.c0, c0, c1);
  Fq6 bb = f6_mul_by_1(f.c1, c4);
  Fq6 s = f6_mul_by_01(f6_add(f.c0, f.c1), c0, f2_add(c1, c4));
  return {f6_add(aa, f6_mul_nr(bb)), f6_sub(f6_sub(s, aa), bb)};
}
ZG_INL Fq12 f12_inv_inl(const Fq12& a) {
  Fq6 t = f6_sub(f6_mul(a.c0, a.c0), f6_mul_nr(f6_mul(a.c1, a.c1)));
  Fq6 ti = f6_inv(t);
  return {f6_mul(a.c0, ti), f6_neg(f6_mul(a.c1, ti))};
}

// Frobenius x -> x^(p^k), k in {1, 2, 3}
ZG_INL Fq12 f12_frob_inl(const Fq12& a, int k) {
  const uint32_t(*c61)[12];
  const uint32_t(*c62)[12];
  const uint32_t(*c12)[12];
  if (k == 1) {
    c61 = FROB6_C1_1; c62 = FROB6_C2_1; c12 = FROB12_C1_1;
  } else if (k == 2) {
    c61 = FROB6_C1_2; c62 = FROB6_C2_2; c12 = FROB12_C1_2;
  } else {
    c61 = FROB6_C1_3; c62 = FROB6_C2_3; c12 = FROB12_C1_3;
  }
  const bool odd = k & 1;
  auto fr2 = [&](const Fq2& x) { return odd ? f2_conj(x) : x; };
  Fq2 g61 = f2_const(c61), g62 = f2_const(c62), g12 = f2_const(c12);
  Fq6 a0 = {fr2(a.c0.c0), f2_mul(fr2(a.c0.c1), g61), f2_mul(fr2(a.c0.c2), g62)};
  Fq6 a1 = {fr2(a.c1.c0), f2_mul(fr2(a.c1.c1), g61), f2_mul(fr2(a.c1.c2), g62)};
  a1 = {f2_mul(a1.c0, g12), f2_mul(a1.c1, g12), f2_mul(a1.c2, g12)};
  return {a0, a1};
}

// ---- out-of-line Fq12 operations (pointer arguments; the Fq2/Fq6 work inside stays in VGPRs)
ZG_NOINL inline void f12_mul_p(Fq12* r, const Fq12* a, const Fq12* b) { *r = f12_mul_inl(*a, *b); }
ZG_NOINL inline void f12_sqr_p(Fq12* r, const Fq12* a) { *r = f12_sqr_inl(*a); }
ZG_NOINL inline void f12_inv_p(Fq12* r, const Fq12* a) { *r = f12_inv_inl(*a); }
ZG_NOINL inline void f12_frob_p(Fq12* r, const Fq12* a, int k) { *r = f12_frob_inl(*a, k); }
ZG_NOINL inline void f12_mul_by_014_p(Fq12* r, const Fq12* f, const Fq2* c0, const Fq2* c1, const Fq2* c4) {
  *r = f12_mul_by_014_inl(*f, *c0, *c1, *c4);
}
ZG_INL Fq12 f12_mul(const Fq12& a, const Fq12& b) { Fq12 r; f12_mul_p(&r, &a, &b); return r; }
ZG_INL Fq12 f12_sqr(const Fq12& a) { Fq12 r; f12_sqr_p(&r, &a); return r; }
ZG_INL Fq12 f12_inv(const Fq12& a) { Fq12 r; f12_inv_p(&r, &a); return r; }
ZG_INL Fq12 f12_frob(const Fq12& a, int k) { Fq12 r; f12_frob_p(&r, &a, k); return r; }
ZG_INL Fq12 f12_mul_by_014(const Fq12& f, const Fq2& c0, const Fq2& c1, const Fq2& c4) {
  Fq12 r;
  f12_mul_by_014_p(&r, &f, &c0, &c1, &c4);
  return r;
}

// f^x then conjugate (pairing final-exp exp_by_x for the negative BLS parameter)
ZG_NOINL inline void f12_pow_u64_p(Fq12* out, const Fq12* ap, uint64_t e) {
  const Fq12 a = *ap;
  Fq12 r = f12_one();
  bool started = false;
  for (int i = 63; i >= 0; i--) {
    if (started) r = f12_sqr(r);
    if ((e >> i) & 1ull) {
      r = started ? f12_mul(r, a) : a;
      started = true;
    }
  }
  *out = r;
}
ZG_INL Fq12 f12_pow_u64(const Fq12& a, uint64_t e) {
  Fq12 r;
  f12_pow_u64_p(&r, &a, e);
  return r;
}

// ------------------------------------------------------------------ GT encoding
// 576 B: the 12 Fq coefficients in tower order, each 48-byte big-endian canonical.
ZG_INL void f12_to_bytes(const Fq12& a, uint8_t* out) {
  const Fq2* c[6] = {&a.c0.c0, &a.c0.c1, &a.c0.c2, &a.c1.c0, &a.c1.c1, &a.c1.c2};
  for (int i = 0; i < 6; i++) {
    fq_limbs_to_be(fq_from_mont(c[i]->c0), out + 96 * i);
    fq_limbs_to_be(fq_from_mont(c[i]->c1), out + 96 * i + 48);
  }
}
ZG_INL Fq12 f12_from_bytes(const uint8_t* in) {
  Fq12 a;
  Fq2* c[6] = {&a.c0.c0, &a.c0.c1, &a.c0.c2, &a.c1.c0, &a.c1.c1, &a.c1.c2};
  for (int i = 0; i < 6; i++) {
    c[i]->c0 = fq_to_mont(fq_limbs_from_be(in + 96 * i));
    c[i]->c1 = fq_to_mont(fq_limbs_from_be(in + 96 * i + 48));
  }
  return a;
}

}  // namespace zg
