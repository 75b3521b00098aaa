// zg_bn254.h -- BN254 ("alt_bn128", the `bn` crate) on gfx950 for PGHR13 Sprout proofs
// (crypto/src/pghr13.rs). One lane per proof.
//
//   Fq      8 x 32-bit limbs, Montgomery R = 2^256; products by the product-scanning FIPS
//           Montgomery multiply (zg_fips.h bq_mul_fips), out of line to keep kernels small
//   tower   Fq2 = Fq[u]/(u^2 + 1), Fq6 = Fq2[v]/(v^3 - xi), Fq12 = Fq6[w]/(w^2 - v), xi = 9 + u;
//           an Fq12 element A + B w holds the coefficients of w^0, w^2, w^4 (A) and w^1, w^3, w^5
//           (B) of the oracle's Fq2[w]/(w^6 - xi) form (oracle/bn254.py)
//   G1      y^2 = x^3 + 3, Jacobian coordinates; G2 (D-type twist) y^2 = x^3 + 3 / xi
//   decode  G1::from_compressed / G2::from_compressed / AffineG{1,2}::new of the bn crate
//           (restated in oracle/bn254.py): prefixes 2/3 (y parity) and 10/11 (y_gt), G2's x a
//           512-bit big-endian blob c1 p + c0, G2 points checked for order r
//   pairing optimal ate (loop 6u + 2, then the pi(Q), -pi^2(Q) steps) with homogeneous G2
//           coordinates and lines scaled by Fq2 factors (killed by the final exponentiation),
//           then the final exponentiation: easy part (p^6 - 1)(p^2 + 1), hard part the
//           Fuentes-Castaneda chain (three exponentiations by -u), i.e. the reduced pairing to
//           the power 2u(6u^2 + 3u + 1) -- oracle.bn254.final_exponentiation_fc, byte for byte
#pragma once
#include "zg_bingcd.h"

namespace zg {

struct BqM {
  static constexpr int N = 8;
  static constexpr uint32_t INV = BQ_INV;
  ZG_INL static uint32_t p(int i) { return BQ_P[i]; }
};
using Bq = Fp<BqM>;

ZG_INL Bq bq_c(const uint32_t* c) {
  Bq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = c[i];
  return r;
}
ZG_INL Bq bq_zero() { return fp_zero<BqM>(); }
ZG_INL Bq bq_one() { return bq_c(BQ_ONE); }

ZG_NOINL inline u32x8 bq_mul_v(u32x8 a0, u32x8 b0) {
  Bq a, b, r;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a.l[i] = a0[i];
    b.l[i] = b0[i];
  }
#if ZG_FQ29
  bq29_mul(r.l, a.l, b.l);  // 29-bit digits (zg_fq29_gen.h; host: same code)
#elif defined(__HIP_DEVICE_COMPILE__)
  bq_mul_fips(r.l, a.l, b.l);
#else
  r = fp_mul_inl<BqM>(a, b);
#endif
  u32x8 o;
#pragma unroll
  for (int i = 0; i < 8; i++) o[i] = r.l[i];
  return o;
}
ZG_INL Bq bq_mul(const Bq& a, const Bq& b) {
  u32x8 a0, b0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a0[i] = a.l[i];
    b0[i] = b.l[i];
  }
  const u32x8 o = bq_mul_v(a0, b0);
  Bq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = o[i];
  return r;
}
ZG_INL Bq bq_sqr(const Bq& a) { return bq_mul(a, a); }
ZG_INL Bq bq_add(const Bq& a, const Bq& b) { return fp_add<BqM>(a, b); }
ZG_INL Bq bq_sub(const Bq& a, const Bq& b) { return fp_sub<BqM>(a, b); }
ZG_INL Bq bq_neg(const Bq& a) { return fp_neg<BqM>(a); }
ZG_INL Bq bq_dbl(const Bq& a) { return fp_add<BqM>(a, a); }
ZG_INL bool bq_is_zero(const Bq& a) { return fp_is_zero<BqM>(a); }
ZG_INL bool bq_eq(const Bq& a, const Bq& b) { return fp_eq<BqM>(a, b); }
ZG_INL Bq bq_to_mont(const Bq& a) { return bq_mul(a, bq_c(BQ_R2)); }
ZG_INL Bq bq_from_mont(const Bq& a) {
  Bq one = bq_zero();
  one.l[0] = 1;
  return bq_mul(a, one);
}
// (a R)^-1 R^3 R^-1 = a^-1 R (public values: binary GCD)
ZG_INL Bq bq_inv(const Bq& a) { return bq_mul(fp_inv_vt<BqM, ZG_INV_T_FR>(a), bq_c(BQ_R3)); }
ZG_INL Bq bq_pow(const Bq& a, const uint32_t* e, int nbits) {
  Bq r = bq_one();
  for (int i = nbits - 1; i >= 0; i--) {
    r = bq_sqr(r);
    if ((e[i >> 5] >> (i & 31)) & 1u) r = bq_mul(r, a);
  }
  return r;
}
// p = 3 mod 4: a^((p+1)/4), false for a non-residue
ZG_INL bool bq_sqrt(const Bq& a, Bq* r) {
  const Bq s = bq_pow(a, BQ_EXP_SQRT, 254);
  *r = s;
  return bq_eq(bq_sqr(s), a);
}

// ---- Fq2
struct Bq2 {
  Bq c0, c1;
};
ZG_INL Bq2 b2_c(const uint32_t* c) { return {bq_c(c), bq_c(c + 8)}; }
ZG_INL Bq2 b2_zero() { return {bq_zero(), bq_zero()}; }
ZG_INL Bq2 b2_one() { return {bq_one(), bq_zero()}; }
ZG_INL Bq2 b2_add(const Bq2& a, const Bq2& b) { return {bq_add(a.c0, b.c0), bq_add(a.c1, b.c1)}; }
ZG_INL Bq2 b2_sub(const Bq2& a, const Bq2& b) { return {bq_sub(a.c0, b.c0), bq_sub(a.c1, b.c1)}; }
ZG_INL Bq2 b2_neg(const Bq2& a) { return {bq_neg(a.c0), bq_neg(a.c1)}; }
ZG_INL Bq2 b2_dbl(const Bq2& a) { return {bq_dbl(a.c0), bq_dbl(a.c1)}; }
ZG_INL Bq2 b2_conj(const Bq2& a) { return {a.c0, bq_neg(a.c1)}; }
ZG_INL bool b2_is_zero(const Bq2& a) { return bq_is_zero(a.c0) && bq_is_zero(a.c1); }
ZG_INL bool b2_eq(const Bq2& a, const Bq2& b) { return bq_eq(a.c0, b.c0) && bq_eq(a.c1, b.c1); }
// Fq2 products out of line (operands as ext_vector values, which the AMDGPU calling convention
// keeps in VGPRs): the tower above calls them hundreds of times per kernel
ZG_INL u32x16 b2_pack(const Bq2& a) {
  u32x16 v;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    v[i] = a.c0.l[i];
    v[8 + i] = a.c1.l[i];
  }
  return v;
}
ZG_INL Bq2 b2_unpack(const u32x16& v) {
  Bq2 a;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a.c0.l[i] = v[i];
    a.c1.l[i] = v[8 + i];
  }
  return a;
}
ZG_NOINL inline u32x16 b2_mul_v(u32x16 x, u32x16 y) {
  const Bq2 a = b2_unpack(x), b = b2_unpack(y);
  const Bq t0 = bq_mul(a.c0, b.c0), t1 = bq_mul(a.c1, b.c1);
  const Bq t2 = bq_mul(bq_add(a.c0, a.c1), bq_add(b.c0, b.c1));
  return b2_pack({bq_sub(t0, t1), bq_sub(bq_sub(t2, t0), t1)});
}
ZG_NOINL inline u32x16 b2_sqr_v(u32x16 x) {
  const Bq2 a = b2_unpack(x);
  const Bq t = bq_mul(a.c0, a.c1);
  return b2_pack({bq_mul(bq_add(a.c0, a.c1), bq_sub(a.c0, a.c1)), bq_dbl(t)});
}
ZG_INL Bq2 b2_mul(const Bq2& a, const Bq2& b) { return b2_unpack(b2_mul_v(b2_pack(a), b2_pack(b))); }
ZG_INL Bq2 b2_sqr(const Bq2& a) { return b2_unpack(b2_sqr_v(b2_pack(a))); }
ZG_INL Bq2 b2_mul_fq(const Bq2& a, const Bq& s) { return {bq_mul(a.c0, s), bq_mul(a.c1, s)}; }
// xi a = (9 + u)(a0 + a1 u) = (9 a0 - a1) + (a0 + 9 a1) u
ZG_INL Bq2 b2_mul_xi(const Bq2& a) {
  const Bq a0_8 = bq_dbl(bq_dbl(bq_dbl(a.c0))), a1_8 = bq_dbl(bq_dbl(bq_dbl(a.c1)));
  return {bq_sub(bq_add(a0_8, a.c0), a.c1), bq_add(bq_add(a1_8, a.c1), a.c0)};
}
ZG_INL Bq2 b2_inv(const Bq2& a) {
  const Bq t = bq_inv(bq_add(bq_sqr(a.c0), bq_sqr(a.c1)));
  return {bq_mul(a.c0, t), bq_neg(bq_mul(a.c1, t))};
}
ZG_INL Bq2 b2_pow(const Bq2& a, const uint32_t* e, int nbits) {
  Bq2 r = b2_one();
  for (int i = nbits - 1; i >= 0; i--) {
    r = b2_sqr(r);
    if ((e[i >> 5] >> (i & 31)) & 1u) r = b2_mul(r, a);
  }
  return r;
}
// a square root in Fq2 = Fq[u]/(u^2 + 1) by the norm ("complex") method, false for a non-residue:
// s = sqrt(a0^2 + a1^2); x = t^((p+1)/4) for t = (a0 + s)/2 -- if x^2 == t the root is
// (x, a1 / 2x), else x^2 == -t (p = 3 mod 4) and (a0 - s)/2 = -a1^2 / 4t is the square of a1 / 2x,
// the root (a1 / 2x, x). Two Fq exponentiations and one inversion, against two Fq2 exponentiations
// of eprint 2012/685 algorithm 9 (round 2's form): any root serves, bn_g2_decode picks y or -y by the
// encoding's flag afterwards.
ZG_INL bool b2_sqrt(const Bq2& a, Bq2* r) {
  if (bq_is_zero(a.c1)) {  // a in Fq: sqrt(a0), or sqrt(-a0) u (-1 is a non-residue)
    Bq s;
    if (bq_sqrt(a.c0, &s)) {
      *r = {s, bq_zero()};
      return true;
    }
    const bool ok = bq_sqrt(bq_neg(a.c0), &s);
    *r = {bq_zero(), s};
    return ok;
  }
  Bq s;
  if (!bq_sqrt(bq_add(bq_sqr(a.c0), bq_sqr(a.c1)), &s)) return false;
  Bq t = bq_add(a.c0, s);
  t = bq_mul(t, bq_c(BQ_HALF));  // (a0 + s) / 2 != 0 since a1 != 0
  const Bq x = bq_pow(t, BQ_EXP_SQRT, 254);
  const Bq w = bq_mul(a.c1, bq_inv(bq_dbl(x)));
  *r = bq_eq(bq_sqr(x), t) ? Bq2{x, w} : Bq2{w, x};
  return b2_eq(b2_sqr(*r), a);
}

// ---- Fq6
struct Bq6 {
  Bq2 c0, c1, c2;
};
ZG_INL Bq6 b6_zero() { return {b2_zero(), b2_zero(), b2_zero()}; }
ZG_INL Bq6 b6_one() { return {b2_one(), b2_zero(), b2_zero()}; }
ZG_INL Bq6 b6_add(const Bq6& a, const Bq6& b) { return {b2_add(a.c0, b.c0), b2_add(a.c1, b.c1), b2_add(a.c2, b.c2)}; }
ZG_INL Bq6 b6_sub(const Bq6& a, const Bq6& b) { return {b2_sub(a.c0, b.c0), b2_sub(a.c1, b.c1), b2_sub(a.c2, b.c2)}; }
ZG_INL Bq6 b6_neg(const Bq6& a) { return {b2_neg(a.c0), b2_neg(a.c1), b2_neg(a.c2)}; }
ZG_INL Bq6 b6_mul_v(const Bq6& a) { return {b2_mul_xi(a.c2), a.c0, a.c1}; }
ZG_INL Bq6 b6_mul(const Bq6& a, const Bq6& b) {
  const Bq2 t0 = b2_mul(a.c0, b.c0), t1 = b2_mul(a.c1, b.c1), t2 = b2_mul(a.c2, b.c2);
  const Bq2 c0 = b2_add(t0, b2_mul_xi(b2_sub(b2_sub(b2_mul(b2_add(a.c1, a.c2), b2_add(b.c1, b.c2)), t1), t2)));
  const Bq2 c1 = b2_add(b2_sub(b2_sub(b2_mul(b2_add(a.c0, a.c1), b2_add(b.c0, b.c1)), t0), t1), b2_mul_xi(t2));
  const Bq2 c2 = b2_add(b2_sub(b2_sub(b2_mul(b2_add(a.c0, a.c2), b2_add(b.c0, b.c2)), t0), t2), t1);
  return {c0, c1, c2};
}
ZG_INL Bq6 b6_mul_b2(const Bq6& a, const Bq2& s) { return {b2_mul(a.c0, s), b2_mul(a.c1, s), b2_mul(a.c2, s)}; }
// a (b0 + b1 v): 5 Fq2 products
ZG_INL Bq6 b6_mul_01(const Bq6& a, const Bq2& b0, const Bq2& b1) {
  const Bq2 t0 = b2_mul(a.c0, b0), t1 = b2_mul(a.c1, b1);
  const Bq2 c0 = b2_add(t0, b2_mul_xi(b2_mul(a.c2, b1)));
  const Bq2 c1 = b2_sub(b2_sub(b2_mul(b2_add(a.c0, a.c1), b2_add(b0, b1)), t0), t1);
  const Bq2 c2 = b2_add(b2_mul(a.c2, b0), t1);
  return {c0, c1, c2};
}
ZG_INL Bq6 b6_inv(const Bq6& a) {
  const Bq2 t0 = b2_sub(b2_sqr(a.c0), b2_mul_xi(b2_mul(a.c1, a.c2)));
  const Bq2 t1 = b2_sub(b2_mul_xi(b2_sqr(a.c2)), b2_mul(a.c0, a.c1));
  const Bq2 t2 = b2_sub(b2_sqr(a.c1), b2_mul(a.c0, a.c2));
  const Bq2 det = b2_add(b2_mul(a.c0, t0), b2_mul_xi(b2_add(b2_mul(a.c2, t1), b2_mul(a.c1, t2))));
  const Bq2 di = b2_inv(det);
  return {b2_mul(t0, di), b2_mul(t1, di), b2_mul(t2, di)};
}

// ---- Fq12
struct Bq12 {
  Bq6 c0, c1;
};
ZG_INL Bq12 b12_one() { return {b6_one(), b6_zero()}; }
ZG_INL Bq12 b12_conj(const Bq12& a) { return {a.c0, b6_neg(a.c1)}; }
ZG_INL Bq12 b12_mul(const Bq12& a, const Bq12& b) {
  const Bq6 t0 = b6_mul(a.c0, b.c0), t1 = b6_mul(a.c1, b.c1);
  const Bq6 c1 = b6_sub(b6_sub(b6_mul(b6_add(a.c0, a.c1), b6_add(b.c0, b.c1)), t0), t1);
  return {b6_add(t0, b6_mul_v(t1)), c1};
}
ZG_INL Bq12 b12_sqr(const Bq12& a) {
  const Bq6 ab = b6_mul(a.c0, a.c1);
  const Bq6 t = b6_mul(b6_add(a.c0, a.c1), b6_add(a.c0, b6_mul_v(a.c1)));
  return {b6_sub(b6_sub(t, ab), b6_mul_v(ab)), b6_add(ab, ab)};
}
ZG_INL Bq12 b12_inv(const Bq12& a) {
  const Bq6 t = b6_inv(b6_sub(b6_mul(a.c0, a.c0), b6_mul_v(b6_mul(a.c1, a.c1))));
  return {b6_mul(a.c0, t), b6_neg(b6_mul(a.c1, t))};
}
// f * (a0 + b0 w + b1 w^3) (a line: A = (a0, 0, 0), B = (b0, b1, 0)): 13 Fq2 products
ZG_INL Bq12 b12_mul_line(const Bq12& f, const Bq2& a0, const Bq2& b0, const Bq2& b1) {
  const Bq6 t0 = b6_mul_b2(f.c0, a0);
  const Bq6 t1 = b6_mul_01(f.c1, b0, b1);
  const Bq6 s = b6_mul_01(b6_add(f.c0, f.c1), b2_add(a0, b0), b1);
  return {b6_add(t0, b6_mul_v(t1)), b6_sub(b6_sub(s, t0), t1)};
}
ZG_INL bool b12_is_one(const Bq12& a) {
  const Bq12 o = b12_one();
  return b2_eq(a.c0.c0, o.c0.c0) && b2_is_zero(a.c0.c1) && b2_is_zero(a.c0.c2) && b2_is_zero(a.c1.c0) &&
         b2_is_zero(a.c1.c1) && b2_is_zero(a.c1.c2);
}
// a^(p^k), k in {1, 2, 3}: coefficient of w^i: conj^k, times xi^(i (p^k - 1) / 6)
ZG_INL Bq12 b12_frob(const Bq12& a, int k) {
  auto cj = [&](const Bq2& x) { return (k & 1) ? b2_conj(x) : x; };
  const uint32_t* g1 = k == 1 ? BQ_FROB1_1 : k == 2 ? BQ_FROB2_1 : BQ_FROB3_1;
  const uint32_t* g2 = k == 1 ? BQ_FROB1_2 : k == 2 ? BQ_FROB2_2 : BQ_FROB3_2;
  const uint32_t* g3 = k == 1 ? BQ_FROB1_3 : k == 2 ? BQ_FROB2_3 : BQ_FROB3_3;
  const uint32_t* g4 = k == 1 ? BQ_FROB1_4 : k == 2 ? BQ_FROB2_4 : BQ_FROB3_4;
  const uint32_t* g5 = k == 1 ? BQ_FROB1_5 : k == 2 ? BQ_FROB2_5 : BQ_FROB3_5;
  Bq12 r;
  r.c0.c0 = cj(a.c0.c0);                       // w^0
  r.c0.c1 = b2_mul(cj(a.c0.c1), b2_c(g2));     // w^2
  r.c0.c2 = b2_mul(cj(a.c0.c2), b2_c(g4));     // w^4
  r.c1.c0 = b2_mul(cj(a.c1.c0), b2_c(g1));     // w^1
  r.c1.c1 = b2_mul(cj(a.c1.c1), b2_c(g3));     // w^3
  r.c1.c2 = b2_mul(cj(a.c1.c2), b2_c(g5));     // w^5
  return r;
}
// a^2 for a in the cyclotomic subgroup (after the easy part of the final exponentiation):
// Granger-Scott, the three Fq4 squarings (z0, z1), (z2, z3), (z4, z5) of the coefficients
// z0 = c0.c0, z4 = c0.c1, z3 = c0.c2, z2 = c1.c0, z1 = c1.c1, z5 = c1.c2 -- 6 Fq2 products
// against 12 for b12_sqr
ZG_INL void b12_fp4_sqr(const Bq2& a, const Bq2& b, Bq2* t0, Bq2* t1) {
  const Bq2 ab = b2_mul(a, b);
  *t0 = b2_sub(b2_sub(b2_mul(b2_add(a, b), b2_add(b2_mul_xi(b), a)), ab), b2_mul_xi(ab));
  *t1 = b2_add(ab, ab);
}
ZG_INL Bq12 b12_csqr(const Bq12& x) {
  Bq2 t0, t1, t2, t3, t4, t5;
  b12_fp4_sqr(x.c0.c0, x.c1.c1, &t0, &t1);
  b12_fp4_sqr(x.c1.c0, x.c0.c2, &t2, &t3);
  b12_fp4_sqr(x.c0.c1, x.c1.c2, &t4, &t5);
  auto tri_m2 = [](const Bq2& t, const Bq2& z) {  // 3 t - 2 z
    const Bq2 d = b2_sub(t, z);
    return b2_add(b2_add(d, d), t);
  };
  auto tri_p2 = [](const Bq2& t, const Bq2& z) {  // 3 t + 2 z
    const Bq2 d = b2_add(t, z);
    return b2_add(b2_add(d, d), t);
  };
  Bq12 r;
  r.c0.c0 = tri_m2(t0, x.c0.c0);
  r.c1.c1 = tri_p2(t1, x.c1.c1);
  r.c1.c0 = tri_p2(b2_mul_xi(t5), x.c1.c0);
  r.c0.c2 = tri_m2(t4, x.c0.c2);
  r.c0.c1 = tri_m2(t2, x.c0.c1);
  r.c1.c2 = tri_p2(t3, x.c1.c2);
  return r;
}
// f^(-u) for f in the cyclotomic subgroup (inverse = conjugate)
ZG_INL Bq12 b12_exp_by_neg_u(const Bq12& f) {
  Bq12 r = f;
  for (int i = 61; i >= 0; i--) {  // u has 63 bits; the top one is the initial r
    r = b12_csqr(r);
    if ((BN_U >> i) & 1ull) r = b12_mul(r, f);
  }
  return b12_conj(r);
}
// the final exponentiation (see the header): oracle.bn254.final_exponentiation_fc
ZG_INL Bq12 bn_final_exp(const Bq12& f) {
  Bq12 t = b12_mul(b12_conj(f), b12_inv(f));
  t = b12_mul(b12_frob(t, 2), t);
  const Bq12 a = b12_exp_by_neg_u(t);
  const Bq12 b = b12_csqr(a);
  const Bq12 c = b12_csqr(b);
  const Bq12 d = b12_mul(c, b);
  const Bq12 e = b12_exp_by_neg_u(d);
  const Bq12 g = b12_exp_by_neg_u(b12_csqr(e));
  const Bq12 k = b12_mul(b12_mul(b12_conj(g), e), b12_conj(d));
  const Bq12 l = b12_mul(k, b);
  const Bq12 n = b12_mul(t, b12_mul(k, e));
  const Bq12 r = b12_mul(b12_frob(k, 2), b12_mul(b12_frob(l, 1), n));
  return b12_mul(b12_frob(b12_mul(b12_conj(t), l), 3), r);
}

// ---- G1 (Jacobian, Z = 0 is the identity)
struct BJ1 {
  Bq X, Y, Z;
};
struct BA1 {
  Bq x, y;
  bool inf;
};
ZG_INL BJ1 bj1_inf() { return {bq_one(), bq_one(), bq_zero()}; }
ZG_INL BJ1 bj1_from(const BA1& a) { return a.inf ? bj1_inf() : BJ1{a.x, a.y, bq_one()}; }
ZG_INL bool bj1_is_inf(const BJ1& p) { return bq_is_zero(p.Z); }
// dbl-2009-l (a = 0)
ZG_INL BJ1 bj1_dbl(const BJ1& p) {
  const Bq A = bq_sqr(p.X), B = bq_sqr(p.Y), C = bq_sqr(B);
  const Bq t = bq_sub(bq_sub(bq_sqr(bq_add(p.X, B)), A), C);
  const Bq D = bq_dbl(t), E = bq_add(bq_dbl(A), A), F = bq_sqr(E);
  const Bq X3 = bq_sub(F, bq_dbl(D));
  const Bq C8 = bq_dbl(bq_dbl(bq_dbl(C)));
  return {X3, bq_sub(bq_mul(E, bq_sub(D, X3)), C8), bq_dbl(bq_mul(p.Y, p.Z))};
}
// p + q (q affine), madd-2007-bl with the special cases
ZG_INL BJ1 bj1_add_aff(const BJ1& p, const BA1& q) {
  if (q.inf) return p;
  if (bj1_is_inf(p)) return bj1_from(q);
  const Bq Z1Z1 = bq_sqr(p.Z);
  const Bq U2 = bq_mul(q.x, Z1Z1), S2 = bq_mul(q.y, bq_mul(p.Z, Z1Z1));
  const Bq H = bq_sub(U2, p.X), rr = bq_dbl(bq_sub(S2, p.Y));
  if (bq_is_zero(H)) return bq_is_zero(rr) ? bj1_dbl(p) : bj1_inf();
  const Bq HH = bq_sqr(H), I = bq_dbl(bq_dbl(HH)), J = bq_mul(H, I), V = bq_mul(p.X, I);
  const Bq X3 = bq_sub(bq_sub(bq_sqr(rr), J), bq_dbl(V));
  const Bq Y3 = bq_sub(bq_mul(rr, bq_sub(V, X3)), bq_dbl(bq_mul(p.Y, J)));
  const Bq Z3 = bq_sub(bq_sub(bq_sqr(bq_add(p.Z, H)), Z1Z1), HH);
  return {X3, Y3, Z3};
}
// p + q, both Jacobian (add-2007-bl with the special cases)
ZG_INL BJ1 bj1_add(const BJ1& p, const BJ1& q) {
  if (bj1_is_inf(p)) return q;
  if (bj1_is_inf(q)) return p;
  const Bq Z1Z1 = bq_sqr(p.Z), Z2Z2 = bq_sqr(q.Z);
  const Bq U1 = bq_mul(p.X, Z2Z2), U2 = bq_mul(q.X, Z1Z1);
  const Bq S1 = bq_mul(bq_mul(p.Y, q.Z), Z2Z2), S2 = bq_mul(bq_mul(q.Y, p.Z), Z1Z1);
  const Bq H = bq_sub(U2, U1), rr = bq_dbl(bq_sub(S2, S1));
  if (bq_is_zero(H)) return bq_is_zero(rr) ? bj1_dbl(p) : bj1_inf();
  const Bq I = bq_sqr(bq_dbl(H)), J = bq_mul(H, I), V = bq_mul(U1, I);
  const Bq X3 = bq_sub(bq_sub(bq_sqr(rr), J), bq_dbl(V));
  const Bq Y3 = bq_sub(bq_mul(rr, bq_sub(V, X3)), bq_dbl(bq_mul(S1, J)));
  const Bq Z3 = bq_mul(bq_sub(bq_sub(bq_sqr(bq_add(p.Z, q.Z)), Z1Z1), Z2Z2), H);
  return {X3, Y3, Z3};
}
ZG_INL BA1 bj1_to_aff(const BJ1& p) {
  if (bj1_is_inf(p)) return {bq_zero(), bq_zero(), true};
  const Bq zi = bq_inv(p.Z), zi2 = bq_sqr(zi);
  return {bq_mul(p.X, zi2), bq_mul(p.Y, bq_mul(zi2, zi)), false};
}
// [k] q for k given as nbits little-endian limbs (from the top)
ZG_INL BJ1 bj1_mul(const BA1& q, const uint32_t* k, int nbits) {
  BJ1 acc = bj1_inf();
  for (int i = nbits - 1; i >= 0; i--) {
    acc = bj1_dbl(acc);
    if ((k[i >> 5] >> (i & 31)) & 1u) acc = bj1_add_aff(acc, q);
  }
  return acc;
}
ZG_INL BA1 ba1_neg(const BA1& a) { return {a.x, bq_neg(a.y), a.inf}; }
ZG_INL BA1 ba1_add(const BA1& a, const BA1& b) { return bj1_to_aff(bj1_add_aff(bj1_from(a), b)); }
// the GLV endomorphism of G1: phi(x, y) = (beta x, y) = [lambda](x, y), lambda^2 + lambda + 1 = 0 mod r
ZG_INL BA1 ba1_phi(const BA1& a) { return {bq_mul(a.x, bq_c(BQ_BETA)), a.y, a.inf}; }
// [a + b lambda] q for 64-bit a = k[0..1], b = k[2..3] (LE limbs): one joint double-and-add over the
// two halves with the table q, phi(q), q + phi(q) -- 64 doublings and ~48 mixed additions against
// 128 and ~64 for a 128-bit scalar. Distinct (a, b) give distinct scalars mod r: the lattice
// {(x, y): x + y lambda = 0 mod r} has no non-zero vector with both |x|, |y| < 2^64 (its reduced
// basis has both vectors of norm ~2^127), so 128 random bits give 2^128 distinct weights.
ZG_INL BJ1 bj1_mul_glv(const BA1& q, const uint32_t* k) {
  if (q.inf) return bj1_inf();
  const BA1 f = ba1_phi(q);
  const BA1 s = ba1_add(q, f);  // q + phi(q) != O: phi(q) = -q would need lambda = -1
  BJ1 acc = bj1_inf();
  for (int i = 63; i >= 0; i--) {
    acc = bj1_dbl(acc);
    const uint32_t ba = (k[i >> 5] >> (i & 31)) & 1u, bb = (k[2 + (i >> 5)] >> (i & 31)) & 1u;
    if (ba | bb) acc = bj1_add_aff(acc, ba & bb ? s : ba ? q : f);
  }
  return acc;
}

// ---- G2 on the twist (homogeneous projective for the Miller loop, Jacobian for [r] Q)
struct BA2 {
  Bq2 x, y;
};
struct BJ2 {
  Bq2 X, Y, Z;
};
ZG_INL BJ2 bj2_dbl(const BJ2& p) {
  const Bq2 A = b2_sqr(p.X), B = b2_sqr(p.Y), C = b2_sqr(B);
  const Bq2 t = b2_sub(b2_sub(b2_sqr(b2_add(p.X, B)), A), C);
  const Bq2 D = b2_dbl(t), E = b2_add(b2_dbl(A), A), F = b2_sqr(E);
  const Bq2 X3 = b2_sub(F, b2_dbl(D));
  const Bq2 C8 = b2_dbl(b2_dbl(b2_dbl(C)));
  return {X3, b2_sub(b2_mul(E, b2_sub(D, X3)), C8), b2_dbl(b2_mul(p.Y, p.Z))};
}
ZG_INL BJ2 bj2_add_aff(const BJ2& p, const BA2& q) {
  if (b2_is_zero(p.Z)) return {q.x, q.y, b2_one()};
  const Bq2 Z1Z1 = b2_sqr(p.Z);
  const Bq2 U2 = b2_mul(q.x, Z1Z1), S2 = b2_mul(q.y, b2_mul(p.Z, Z1Z1));
  const Bq2 H = b2_sub(U2, p.X), rr = b2_dbl(b2_sub(S2, p.Y));
  if (b2_is_zero(H)) return b2_is_zero(rr) ? bj2_dbl(p) : BJ2{b2_one(), b2_one(), b2_zero()};
  const Bq2 HH = b2_sqr(H), I = b2_dbl(b2_dbl(HH)), J = b2_mul(H, I), V = b2_mul(p.X, I);
  const Bq2 X3 = b2_sub(b2_sub(b2_sqr(rr), J), b2_dbl(V));
  const Bq2 Y3 = b2_sub(b2_mul(rr, b2_sub(V, X3)), b2_dbl(b2_mul(p.Y, J)));
  const Bq2 Z3 = b2_sub(b2_sub(b2_sqr(b2_add(p.Z, H)), Z1Z1), HH);
  return {X3, Y3, Z3};
}
// AffineG2::new's order check, [r] Q == O, as the bn crate runs it (kept for tests; the product
// uses ba2_in_subgroup below)
ZG_INL bool ba2_in_subgroup_r(const BA2& q) {
  BJ2 acc = {b2_one(), b2_one(), b2_zero()};
  for (int i = 253; i >= 0; i--) {
    acc = bj2_dbl(acc);
    if ((BN_R[i >> 5] >> (i & 31)) & 1u) acc = bj2_add_aff(acc, q);
  }
  return b2_is_zero(acc.Z);
}
ZG_INL bool ba2_on_curve(const BA2& q) {
  return b2_eq(b2_sqr(q.y), b2_add(b2_mul(b2_sqr(q.x), q.x), b2_c(BQ_B2)));
}
ZG_INL bool ba1_on_curve(const BA1& p) {
  Bq three = bq_add(bq_dbl(bq_one()), bq_one());
  return bq_eq(bq_sqr(p.y), bq_add(bq_mul(bq_sqr(p.x), p.x), three));
}

// Miller-loop line through T (homogeneous twist point), scaled by an Fq2 factor: the Fq12 element
// c0 y_P + (c1 x_P) w + c3 w^3 (oracle.bn254._line times 2 Y Z^2 for a doubling, times
// x_Q Z - X for an addition)
struct BLine {
  Bq2 c0, c1, c3;
};
struct BH2 {  // homogeneous: x = X / Z, y = Y / Z
  Bq2 X, Y, Z;
};
ZG_INL BLine bh2_dbl_step(BH2* t) {
  const Bq2 X = t->X, Y = t->Y, Z = t->Z;
  const Bq2 XX = b2_sqr(X), YZ = b2_mul(Y, Z);
  const Bq2 w3 = b2_add(b2_dbl(XX), XX);  // 3 X^2
  BLine l;
  l.c0 = b2_dbl(b2_mul(YZ, Z));                                      // 2 Y Z^2
  l.c1 = b2_neg(b2_mul(w3, Z));                                      // -3 X^2 Z
  l.c3 = b2_sub(b2_mul(w3, X), b2_dbl(b2_mul(b2_sqr(Y), Z)));        // 3 X^3 - 2 Y^2 Z
  // dbl-2007-bl (homogeneous, a = 0)
  const Bq2 s = b2_dbl(YZ), ss = b2_sqr(s), sss = b2_mul(s, ss);
  const Bq2 R = b2_mul(Y, s), RR = b2_sqr(R);
  const Bq2 B = b2_sub(b2_sub(b2_sqr(b2_add(X, R)), XX), RR);
  const Bq2 h = b2_sub(b2_sqr(w3), b2_dbl(B));
  t->X = b2_mul(h, s);
  t->Y = b2_sub(b2_mul(w3, b2_sub(B, h)), b2_dbl(RR));
  t->Z = sss;
  return l;
}
ZG_INL BLine bh2_add_step(BH2* t, const BA2& q) {
  const Bq2 th = b2_sub(b2_mul(q.y, t->Z), t->Y);  // theta
  const Bq2 L = b2_sub(b2_mul(q.x, t->Z), t->X);   // lambda
  BLine l;
  l.c0 = L;
  l.c1 = b2_neg(th);
  l.c3 = b2_sub(b2_mul(th, q.x), b2_mul(L, q.y));
  // madd-1998-cmo (homogeneous)
  const Bq2 uu = b2_sqr(th), vv = b2_sqr(L), vvv = b2_mul(L, vv);
  const Bq2 R = b2_mul(vv, t->X);
  const Bq2 A = b2_sub(b2_sub(b2_mul(uu, t->Z), vvv), b2_dbl(R));
  t->X = b2_mul(L, A);
  t->Y = b2_sub(b2_mul(th, b2_sub(R, A)), b2_mul(vvv, t->Y));
  t->Z = b2_mul(vvv, t->Z);
  return l;
}
ZG_INL Bq12 b12_mul_bline(const Bq12& f, const BLine& l, const BA1& p) {
  return b12_mul_line(f, b2_mul_fq(l.c0, p.y), b2_mul_fq(l.c1, p.x), l.c3);
}
// pi(Q), pi^2(Q) on the twist
ZG_INL BA2 ba2_frob(const BA2& q) {
  return {b2_mul(b2_conj(q.x), b2_c(BQ_FROB1_2)), b2_mul(b2_conj(q.y), b2_c(BQ_FROB1_3))};
}
ZG_INL BA2 ba2_frob2(const BA2& q) { return {b2_mul(q.x, b2_c(BQ_FROB2_2)), b2_mul(q.y, b2_c(BQ_FROB2_3))}; }

// G2 membership as psi(Q) == [6u^2] Q (a 127-bit scalar: half the doublings of [r] Q; round 3's
// first form, kept for the host test). psi (untwist-Frobenius-twist, ba2_frob) satisfies
// psi^2 - t psi + p = 0 on E'(Fq2) and acts on G2 as [p] = [p mod r] = [6u^2]. The endomorphism
// psi - [6u^2] has degree (6u^2)^2 - t 6u^2 + p = p - 6u^2 = r (t = 6u^2 + 1), so its kernel is
// exactly G2: for Q on the twist, psi(Q) = [6u^2] Q  <=>  [r] Q = O (AffineG2::new).
ZG_INL bool ba2_in_subgroup_6u2(const BA2& q) {
  static constexpr uint32_t SIX_U2[4] = {0xe87cfd46u, 0xf83e9682u, 0xeeb859fbu, 0x6f4d8248u};  // 6u^2
  BJ2 acc = {q.x, q.y, b2_one()};
  for (int i = 125; i >= 0; i--) {  // bit 126 is the leading one
    acc = bj2_dbl(acc);
    if ((SIX_U2[i >> 5] >> (i & 31)) & 1u) acc = bj2_add_aff(acc, q);
  }
  if (b2_is_zero(acc.Z)) return false;  // [6u^2] Q = O while psi(Q) is finite
  const BA2 s = ba2_frob(q);
  const Bq2 z2 = b2_sqr(acc.Z);
  return b2_eq(acc.X, b2_mul(s.x, z2)) && b2_eq(acc.Y, b2_mul(s.y, b2_mul(z2, acc.Z)));
}
// Jacobian p + q (add-2007-bl with the special cases), psi and psi^2 on Jacobian points (conjugation
// is a field automorphism, so psi(X : Y : Z) = (conj X g2 : conj Y g3 : conj Z))
ZG_INL bool bj2_is_inf(const BJ2& p) { return b2_is_zero(p.Z); }
ZG_INL BJ2 bj2_add(const BJ2& p, const BJ2& q) {
  if (bj2_is_inf(p)) return q;
  if (bj2_is_inf(q)) return p;
  const Bq2 Z1Z1 = b2_sqr(p.Z), Z2Z2 = b2_sqr(q.Z);
  const Bq2 U1 = b2_mul(p.X, Z2Z2), U2 = b2_mul(q.X, Z1Z1);
  const Bq2 S1 = b2_mul(b2_mul(p.Y, q.Z), Z2Z2), S2 = b2_mul(b2_mul(q.Y, p.Z), Z1Z1);
  const Bq2 H = b2_sub(U2, U1), rr = b2_dbl(b2_sub(S2, S1));
  if (b2_is_zero(H)) return b2_is_zero(rr) ? bj2_dbl(p) : BJ2{b2_one(), b2_one(), b2_zero()};
  const Bq2 I = b2_sqr(b2_dbl(H)), J = b2_mul(H, I), V = b2_mul(U1, I);
  const Bq2 X3 = b2_sub(b2_sub(b2_sqr(rr), J), b2_dbl(V));
  const Bq2 Y3 = b2_sub(b2_mul(rr, b2_sub(V, X3)), b2_dbl(b2_mul(S1, J)));
  const Bq2 Z3 = b2_mul(b2_sub(b2_sub(b2_sqr(b2_add(p.Z, q.Z)), Z1Z1), Z2Z2), H);
  return {X3, Y3, Z3};
}
ZG_INL BJ2 bj2_psi(const BJ2& p) {
  return {b2_mul(b2_conj(p.X), b2_c(BQ_FROB1_2)), b2_mul(b2_conj(p.Y), b2_c(BQ_FROB1_3)), b2_conj(p.Z)};
}
ZG_INL BJ2 bj2_psi2(const BJ2& p) { return {b2_mul(p.X, b2_c(BQ_FROB2_2)), b2_mul(p.Y, b2_c(BQ_FROB2_3)), p.Z}; }
ZG_INL bool bj2_eq(const BJ2& p, const BJ2& q) {
  if (bj2_is_inf(p) || bj2_is_inf(q)) return bj2_is_inf(p) && bj2_is_inf(q);
  const Bq2 Z1Z1 = b2_sqr(p.Z), Z2Z2 = b2_sqr(q.Z);
  return b2_eq(b2_mul(p.X, Z2Z2), b2_mul(q.X, Z1Z1)) &&
         b2_eq(b2_mul(b2_mul(p.Y, q.Z), Z2Z2), b2_mul(b2_mul(q.Y, p.Z), Z1Z1));
}
// G2 membership (round 3) as  [u + 1] Q + psi([u] Q) + psi^2([u] Q) == psi^3([2u] Q)  -- a 63-bit
// scalar, half the doublings of the psi == [6u^2] form (El Housni-Guillevic-Piellard's test for BN
// curves). Why it is exact here: #E'(Fq2) = r h' with h' = 2p - r = 10069 * 5864401 * 1875725156269 *
// (a 178-bit prime), all distinct primes != r, so every Sylow subgroup of E'(Fq2) is cyclic of prime
// order and the endomorphism E = [u + 1] + psi [u] + psi^2 [u] - psi^3 [2u] acts on each as a
// scalar. E vanishes on G2 and on no point of order l for each l | h' (checked on a generator of each
// component: tests/test_pghr13.py::test_host_g2_membership_*), so ker E = G2 exactly and the test
// decides like AffineG2::new's [r] Q = O.
ZG_INL bool ba2_in_subgroup(const BA2& q) {
  BJ2 a = {q.x, q.y, b2_one()};
  for (int i = 61; i >= 0; i--) {  // [u] Q, u = BN_U (bit 62 the leading one)
    a = bj2_dbl(a);
    if ((BN_U >> i) & 1ull) a = bj2_add_aff(a, q);
  }
  const BJ2 pa = bj2_psi(a);
  BJ2 l = bj2_add_aff(a, q);          // [u + 1] Q
  l = bj2_add(l, pa);                  // + psi([u] Q)
  l = bj2_add(l, bj2_psi(pa));         // + psi^2([u] Q)
  const BJ2 r = bj2_psi(bj2_psi2(bj2_dbl(a)));  // psi^3([2u] Q)
  return bj2_eq(l, r);
}

#define ZG_BN_ATE_BITS 65  // 6u + 2
ZG_INL bool bn_ate_bit(int i) { return (BN_ATE[i >> 5] >> (i & 31)) & 1u; }

// the optimal ate Miller function of one pair, lines computed along the loop
ZG_INL Bq12 bn_miller_single(const BA1& p, const BA2& Q) {
  BH2 t = {Q.x, Q.y, b2_one()};
  Bq12 f = b12_one();
  for (int bit = ZG_BN_ATE_BITS - 2; bit >= 0; bit--) {
    f = b12_sqr(f);
    f = b12_mul_bline(f, bh2_dbl_step(&t), p);
    if (bn_ate_bit(bit)) f = b12_mul_bline(f, bh2_add_step(&t, Q), p);
  }
  f = b12_mul_bline(f, bh2_add_step(&t, ba2_frob(Q)), p);
  const BA2 q2 = ba2_frob2(Q);
  return b12_mul_bline(f, bh2_add_step(&t, {q2.x, b2_neg(q2.y)}), p);
}

// G1::from_compressed (33 bytes)
ZG_INL bool bn_g1_decode(const uint8_t* b, BA1* out) {
  const uint8_t sign = b[0];
  if (sign != 2 && sign != 3) return false;
  Bq x;
  for (int i = 0; i < 8; i++) {
    const uint8_t* q = b + 1 + 28 - 4 * i;
    x.l[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
  if (!fp_lt_modulus<BqM>(x)) return false;
  const Bq xm = bq_to_mont(x);
  const Bq three = bq_add(bq_dbl(bq_one()), bq_one());
  Bq y;
  if (!bq_sqrt(bq_add(bq_mul(bq_sqr(xm), xm), three), &y)) return false;
  const bool odd = bq_from_mont(y).l[0] & 1u;
  if ((sign == 2) == odd) y = bq_neg(y);
  *out = {xm, y, false};
  return true;
}

// G2::from_compressed (65 bytes): x from the 512-bit blob U = c1 p + c0 (long division), y by
// the y_gt flag, then the order check
ZG_INL bool bn_g2_decode(const uint8_t* b, BA2* out) {
  const uint8_t sign = b[0];
  if (sign != 10 && sign != 11) return false;
  // U / p by shift-subtract over the 512 bits (MSB first); remainder < p < 2^254
  uint32_t rem[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, quo[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  bool q_big = false;  // quotient >= 2^256 (then certainly >= p)
  for (int i = 0; i < 512; i++) {
    const uint32_t bit = (b[1 + (i >> 3)] >> (7 - (i & 7))) & 1u;
#pragma unroll
    for (int k = 8; k > 0; k--) rem[k] = (rem[k] << 1) | (rem[k - 1] >> 31);
    rem[0] = (rem[0] << 1) | bit;
    // rem >= p ?
    uint32_t t[9];
    uint64_t br = 0;
#pragma unroll
    for (int k = 0; k < 9; k++) {
      const uint64_t d = (uint64_t)rem[k] - (k < 8 ? BQ_P[k] : 0u) - br;
      t[k] = (uint32_t)d;
      br = (d >> 63) & 1u;
    }
    const bool ge = br == 0;
    q_big |= (quo[7] >> 31) != 0;  // the quotient is about to exceed 256 bits
#pragma unroll
    for (int k = 7; k > 0; k--) quo[k] = (quo[k] << 1) | (quo[k - 1] >> 31);
    quo[0] = (quo[0] << 1) | (ge ? 1u : 0u);
#pragma unroll
    for (int k = 0; k < 9; k++) rem[k] = ge ? t[k] : rem[k];
  }
  Bq c0, c1;
  for (int k = 0; k < 8; k++) {
    c0.l[k] = rem[k];
    c1.l[k] = quo[k];
  }
  if (q_big || !fp_lt_modulus<BqM>(c1)) return false;  // Fq2::from_slice: c1 must be < p
  BA2 q;
  q.x = {bq_to_mont(c0), bq_to_mont(c1)};
  Bq2 y;
  if (!b2_sqrt(b2_add(b2_mul(b2_sqr(q.x), q.x), b2_c(BQ_B2)), &y)) return false;
  // y_gt: y > -y in the order c1 p + c0 (compare c1, then c0, canonical)
  const Bq2 yn = b2_neg(y);
  const Bq y0 = bq_from_mont(y.c0), y1 = bq_from_mont(y.c1), n0 = bq_from_mont(yn.c0), n1 = bq_from_mont(yn.c1);
  const bool gt = bq_eq(y1, n1) ? fp_gt_canon<BqM>(y0, n0) : fp_gt_canon<BqM>(y1, n1);
  if ((sign == 10) == gt) y = yn;
  q.y = y;
  if (!ba2_in_subgroup(q)) return false;
  *out = q;
  return true;
}


}  // namespace zg
