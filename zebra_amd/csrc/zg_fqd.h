// zg_fqd.h -- lazy digit-resident Fq and G1 Jacobian arithmetic for point-operation chains
// (the decode kernels' subgroup checks and GLV products r_i A_i).
//
// FqD holds an Fq value as 14 normalized 29-bit digits in Montgomery form R' = 2^406 (the
// representation of zg_fq29_gen.h fq29d_*), NOT reduced mod p: the value is below K p for a bound
// K that the formulas below track by hand (comments: bounds in units of p). A product
// (fq29d_mul / fq29d_sqr; their column sums stay below 2^64 for any normalized 14-digit inputs)
// of a < Ka p and b < Kb p returns (a b + m p) / 2^406 < (Ka Kb p / 2^406 + 1) p < 2p whenever
// Ka Kb < 2^25 (p < 2^381). Sums and differences are digit-wise with one carry normalization and
// are never reduced. A chain of point operations therefore splits, repacks and canonicalises
// nothing between its products (the word form of zg_field.h does all three in every fq_mul) and
// pays one conversion in and one out per point.
//
// A difference c_a a - c_b b is formed as c_a a + (k p - c_b b) with k p held in "borrowed"
// digits (digits 0..12 raised by c_b 2^29, digits 1..13 lowered by c_b): each digit of
// k p - c_b b is non-negative for normalized b with c_b b <= (k - 1) p and c_b <= 13
// (floor(p / 2^377) = 13 covers the lowered top digit).
#pragma once
#include "zg_curve.h"

namespace zg {

struct FqD {
  uint32_t d[14];
};

// k p in digits 0..13, digits 0..12 raised by s 2^29 and digits 1..13 lowered by s
struct FqDK {
  uint32_t d[14];
};
constexpr FqDK fqd_kp(uint32_t k, uint32_t s) {
  uint32_t w[13] = {};
  uint64_t c = 0;
  for (int i = 0; i < 12; i++) {
    const uint64_t m = (uint64_t)FQ_P[i] * k + c;
    w[i] = (uint32_t)m;
    c = m >> 32;
  }
  w[12] = (uint32_t)c;
  FqDK r = {};
  for (int L = 0; L < 14; L++) {
    const int bit = 29 * L, wi = bit >> 5, off = bit & 31;
    uint64_t v = (uint64_t)w[wi] >> off;
    if (wi + 1 < 13) v |= (uint64_t)w[wi + 1] << (32 - off);
    r.d[L] = L < 13 ? (uint32_t)(v & 0x1fffffffu) : (uint32_t)v;
  }
  for (int L = 0; L < 14; L++) {
    if (L < 13) r.d[L] += s << 29;
    if (L > 0) r.d[L] -= s;
  }
  return r;
}

// R' mod p = 2^406 mod p: the FqD form of 1
static constexpr uint32_t FQD_ONE[14] = {0x03a9fb84u, 0x0ba00690u, 0x071288f1u, 0x0f59bcc5u, 0x126cb614u,
                                         0x0585bf36u, 0x1b85ac3du, 0x1cf856fau, 0x1891ecbdu, 0x1a7eec05u,
                                         0x155a88f0u, 0x0741ac6du, 0x1317c30fu, 0x00000009u};

// carry normalization (value unchanged); digits must leave room for the carries (< 2^32 - 8)
ZG_INL void fqd_norm(uint32_t* d) {
#pragma unroll
  for (int i = 0; i < 13; i++) {
    d[i + 1] += d[i] >> 29;
    d[i] &= FQ29_MASK;
  }
}

ZG_INL FqD fqd_one() {
  FqD r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = FQD_ONE[i];
  return r;
}
ZG_INL FqD fqd_zero() {
  FqD r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = 0u;
  return r;
}
// ZG_FQD_CALL (default 1): the products are two out-of-line functions with register arguments
// (as fq_mul_v / fq_sqr_v), so a chain's code stays small (a fully inlined subgroup check is
// ~16 k instructions, past the instruction cache a decode wave shares); 0 inlines them
#ifndef ZG_FQD_CALL
#define ZG_FQD_CALL 1
#endif
#if ZG_FQD_CALL
ZG_NOINL inline u32x16 fqd_mul_v(u32x16 a, u32x16 b) {
  uint32_t x[14], y[14], r[14];
#pragma unroll
  for (int i = 0; i < 14; i++) {
    x[i] = a[i];
    y[i] = b[i];
  }
  fq29d_mul(r, x, y);
  u32x16 o;
#pragma unroll
  for (int i = 0; i < 14; i++) o[i] = r[i];
  o[14] = o[15] = 0;
  return o;
}
ZG_NOINL inline u32x16 fqd_sqr_v(u32x16 a) {
  uint32_t x[14], r[14];
#pragma unroll
  for (int i = 0; i < 14; i++) x[i] = a[i];
  fq29d_sqr(r, x);
  u32x16 o;
#pragma unroll
  for (int i = 0; i < 14; i++) o[i] = r[i];
  o[14] = o[15] = 0;
  return o;
}
ZG_INL u32x16 fqd_pack(const FqD& a) {
  u32x16 v;
#pragma unroll
  for (int i = 0; i < 14; i++) v[i] = a.d[i];
  v[14] = v[15] = 0;
  return v;
}
ZG_INL FqD fqd_unpack(const u32x16& v) {
  FqD r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = v[i];
  return r;
}
ZG_INL FqD fqd_mul(const FqD& a, const FqD& b) { return fqd_unpack(fqd_mul_v(fqd_pack(a), fqd_pack(b))); }
ZG_INL FqD fqd_sqr(const FqD& a) { return fqd_unpack(fqd_sqr_v(fqd_pack(a))); }
#else
ZG_INL FqD fqd_mul(const FqD& a, const FqD& b) {  // < 2p for Ka Kb < 2^25
  FqD r;
  fq29d_mul(r.d, a.d, b.d);
  return r;
}
ZG_INL FqD fqd_sqr(const FqD& a) {  // < 2p for Ka < 2^12
  FqD r;
  fq29d_sqr(r.d, a.d);
  return r;
}
#endif
// c a (c a small positive integer)
template <int C>
ZG_INL FqD fqd_smul(const FqD& a) {
  FqD r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = C * a.d[i];
  fqd_norm(r.d);
  return r;
}
ZG_INL FqD fqd_add(const FqD& a, const FqD& b) {
  FqD r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = a.d[i] + b.d[i];
  fqd_norm(r.d);
  return r;
}
// CA a - CB b + K p   (requires CB b <= (K - 1) p, CB <= 13; result < CA a + K p)
template <int K, int CA, int CB>
ZG_INL FqD fqd_sub(const FqD& a, const FqD& b) {
  constexpr FqDK kp = fqd_kp(K, CB);
  static_assert(CB >= 1 && CB <= 13 && CA >= 0 && CA + CB <= 6, "digit budget");
  FqD r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = CA * a.d[i] + (kp.d[i] - CB * b.d[i]);
  fqd_norm(r.d);
  return r;
}
// a - b - c + K p   (requires b + c <= (K - 1) p; result < a + K p)
template <int K>
ZG_INL FqD fqd_sub2(const FqD& a, const FqD& b, const FqD& c) {
  constexpr FqDK kp = fqd_kp(K, 2);
  FqD r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = a.d[i] + (kp.d[i] - b.d[i] - c.d[i]);
  fqd_norm(r.d);
  return r;
}
// v == 0 mod p for a product output or any v < 2p (normalized digits are unique: v is 0 or p)
ZG_INL bool fqd_is_zero2(const FqD& v) {
  constexpr FqDK p1 = fqd_kp(1, 0);
  bool z0 = true, z1 = true;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    z0 = z0 && v.d[i] == 0u;
    z1 = z1 && v.d[i] == p1.d[i];
  }
  return z0 || z1;
}
// v == 0 mod p for v < 4p
ZG_INL bool fqd_is_zero4(const FqD& v) {
  constexpr FqDK p1 = fqd_kp(1, 0), p2 = fqd_kp(2, 0), p3 = fqd_kp(3, 0);
  bool z0 = true, z1 = true, z2 = true, z3 = true;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    z0 = z0 && v.d[i] == 0u;
    z1 = z1 && v.d[i] == p1.d[i];
    z2 = z2 && v.d[i] == p2.d[i];
    z3 = z3 && v.d[i] == p3.d[i];
  }
  return z0 || z1 || z2 || z3;
}

// word Montgomery form (R = 2^384, any value < 2^384) -> FqD (< 2p)
ZG_INL FqD fqd_from(const Fq& a) {
  FqD r;
  fq29d_from_mont(r.d, a.l);
  return r;
}
// FqD (any value < 2^21 p) -> canonical word Montgomery form
ZG_INL Fq fqd_to(const FqD& a) {
  Fq r;
  fq29d_to_mont(r.l, a.d);
  return r;
}

// ------------------------------------------------------------------ G1 Jacobian (y^2 = x^3 + 4)
// Invariant of every G1D below: X < 35p, Y < 19p, Z < 4p; infinity is Z == 0 mod p.
struct G1D {
  FqD x, y, z;
};

ZG_INL bool g1d_is_inf(const G1D& p) { return fqd_is_zero4(p.z); }
ZG_INL G1D g1d_from_aff(const FqD& x, const FqD& y) { return {x, y, fqd_one()}; }
ZG_INL G1D g1d_infinity() { return {fqd_one(), fqd_one(), fqd_zero()}; }
// canonical word-form Jacobian (the same point; Z = 0 stays infinity)
ZG_INL G1J g1d_to_jac(const G1D& p) { return {fqd_to(p.x), fqd_to(p.y), fqd_to(p.z)}; }

// dbl-2009-l (a = 0), 7 products. In: the invariant. Out: X < 31p, Y < 19p, Z < 4p.
// Infinity (Z = 0) doubles to Z = 2 Y Z = 0.
ZG_INL G1D g1d_dbl(const G1D& p) {
  const FqD A = fqd_sqr(p.x);                              // < 2
  const FqD B = fqd_sqr(p.y);                              // < 2
  const FqD C = fqd_sqr(B);                                // < 2
  const FqD T = fqd_sqr(fqd_add(p.x, B));                  // (X + B < 37)^2: < 2
  const FqD D = fqd_smul<2>(fqd_sub2<5>(T, A, C));         // 2 (T - A - C + 5p): < 14 (A + C < 4)
  const FqD E = fqd_smul<3>(A);                            // < 6
  const FqD F = fqd_sqr(E);                                // < 2
  const FqD X3 = fqd_sub<29, 1, 2>(F, D);                  // F - 2D + 29p: < 31 (2D < 28)
  const FqD Y3a = fqd_mul(E, fqd_sub<32, 1, 1>(D, X3));    // (D - X3 + 32p < 46) E: < 2
  const FqD Y3 = fqd_sub<17, 1, 1>(Y3a, fqd_smul<8>(C));   // - 8C + 17p: < 19 (8C < 16)
  const FqD Z3 = fqd_smul<2>(fqd_mul(p.y, p.z));           // < 4
  return {X3, Y3, Z3};
}

// g1d_dbl on a whole wave for a lone doubling chain (K4's top-window scaling, zg_msm.hip): the same
// formulas and bounds, so the same digits, with the seven products of dbl-2009-l in three levels of
// independent products, one per lane (lanes 0..2), exchanged through `xch` (3 FqD of LDS, the wave's
// own): {A = X^2, B = Y^2, YZ}, {C = B^2, T = (X + B)^2, F = (3A)^2}, {E (D - X3)}. Every lane of the
// wave calls it with the same p and gets the result.
ZG_INL FqD fqd_pick3(int k, const FqD& a, const FqD& b, const FqD& c) {
  FqD r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.d[i] = k == 0 ? a.d[i] : k == 1 ? b.d[i] : c.d[i];
  return r;
}
ZG_INL void fqd_xch_put(FqD* xch, int lane, const FqD& v) {
  if (lane < 3) xch[lane] = v;
  __syncthreads();
}
ZG_INL G1D g1d_dbl_wave(const G1D& p, FqD* xch) {
  const int lane = threadIdx.x & 63, k = lane < 3 ? lane : 0;
  // level 1: A = X X, B = Y Y, YZ = Y Z
  const FqD m1 = fqd_mul(fqd_pick3(k, p.x, p.y, p.y), fqd_pick3(k, p.x, p.y, p.z));
  fqd_xch_put(xch, lane, m1);
  const FqD A = xch[0], B = xch[1], YZ = xch[2];
  __syncthreads();
  // level 2: C = B^2, T = (X + B)^2, F = E^2 with E = 3 A
  const FqD E = fqd_smul<3>(A);
  const FqD m2 = fqd_sqr(fqd_pick3(k, B, fqd_add(p.x, B), E));
  fqd_xch_put(xch, lane, m2);
  const FqD C = xch[0], T = xch[1], F = xch[2];
  __syncthreads();
  const FqD D = fqd_smul<2>(fqd_sub2<5>(T, A, C));
  const FqD X3 = fqd_sub<29, 1, 2>(F, D);
  // level 3: E (D - X3)
  const FqD m3 = fqd_mul(E, fqd_sub<32, 1, 1>(D, X3));
  fqd_xch_put(xch, lane, m3);
  const FqD Y3a = xch[0];
  __syncthreads();
  const FqD Y3 = fqd_sub<17, 1, 1>(Y3a, fqd_smul<8>(C));
  const FqD Z3 = fqd_smul<2>(YZ);
  return {X3, Y3, Z3};
}

// madd-2007-bl with complete case handling: p + q for q affine and finite, qx < 2p, qy < 4p.
// In: the invariant. Out: X < 9p, Y < 7p, Z < 4p (or g1d_dbl's, or q itself). 11 products.
ZG_INL G1D g1d_add_aff(const G1D& p, const FqD& qx, const FqD& qy) {
  if (g1d_is_inf(p)) return g1d_from_aff(qx, qy);
  const FqD Z1Z1 = fqd_sqr(p.z);                           // < 2
  const FqD U2 = fqd_mul(qx, Z1Z1);                        // < 2
  const FqD S2 = fqd_mul(fqd_mul(qy, p.z), Z1Z1);          // < 2
  const FqD H = fqd_sub<36, 1, 1>(U2, p.x);                // U2 - X1 + 36p: < 38 (X1 < 35)
  const FqD rr = fqd_sub<39, 2, 2>(S2, p.y);               // 2 S2 - 2 Y1 + 39p: < 43 (2 Y1 < 38)
  const FqD HH = fqd_sqr(H);                               // < 2
  const FqD RR = fqd_sqr(rr);                              // < 2
  // H == 0 mod p <=> H^2 == 0 (and rr likewise): P == +-Q
  if (fqd_is_zero2(HH)) {
    if (fqd_is_zero2(RR)) return g1d_dbl(p);
    return g1d_infinity();
  }
  const FqD I = fqd_smul<4>(HH);                           // < 8
  const FqD J = fqd_mul(H, I);                             // < 2
  const FqD V = fqd_mul(p.x, I);                           // < 2
  const FqD X3 = fqd_sub2<7>(RR, J, fqd_smul<2>(V));       // rr^2 - J - 2V + 7p: < 9 (J + 2V < 6)
  const FqD Y3a = fqd_mul(rr, fqd_sub<10, 1, 1>(V, X3));   // (V - X3 + 10p < 12) rr: < 2
  const FqD Y3 = fqd_sub<5, 1, 2>(Y3a, fqd_mul(p.y, J));   // - 2 Y1 J + 5p: < 7 (2 Y1 J < 4)
  const FqD Z3 = fqd_smul<2>(fqd_mul(p.z, H));             // (Z1 + H)^2 - Z1Z1 - HH = 2 Z1 H: < 4
  return {X3, Y3, Z3};
}

// add-2007-bl with complete case handling: p + q, both in the invariant (either may be infinity).
// Out: X < 9p, Y < 7p, Z < 4p (or g1d_dbl's, or p / q itself). 16 products.
ZG_INL G1D g1d_add_full(const G1D& p, const G1D& q) {
  if (g1d_is_inf(p)) return q;
  if (g1d_is_inf(q)) return p;
  const FqD Z1Z1 = fqd_sqr(p.z);                           // (Z1 < 4)^2: < 2
  const FqD Z2Z2 = fqd_sqr(q.z);                           // < 2
  const FqD U1 = fqd_mul(p.x, Z2Z2);                       // 35 x 2: < 2
  const FqD U2 = fqd_mul(q.x, Z1Z1);                       // < 2
  const FqD S1 = fqd_mul(fqd_mul(p.y, q.z), Z2Z2);         // (19 x 4 -> < 2) x 2: < 2
  const FqD S2 = fqd_mul(fqd_mul(q.y, p.z), Z1Z1);         // < 2
  const FqD H = fqd_sub<3, 1, 1>(U2, U1);                  // U2 - U1 + 3p: < 5 (U1 < 2)
  const FqD rr = fqd_sub<5, 2, 2>(S2, S1);                 // 2 S2 - 2 S1 + 5p: < 9 (2 S1 < 4)
  const FqD HH = fqd_sqr(H);                               // < 2
  const FqD RR = fqd_sqr(rr);                              // < 2
  // H == 0 mod p <=> H^2 == 0 (and rr likewise): P == +-Q
  if (fqd_is_zero2(HH)) {
    if (fqd_is_zero2(RR)) return g1d_dbl(p);
    return g1d_infinity();
  }
  const FqD I = fqd_smul<4>(HH);                           // (2H)^2: < 8
  const FqD J = fqd_mul(H, I);                             // 5 x 8: < 2
  const FqD V = fqd_mul(U1, I);                            // < 2
  const FqD X3 = fqd_sub2<7>(RR, J, fqd_smul<2>(V));       // rr^2 - J - 2V + 7p: < 9 (J + 2V < 6)
  const FqD Y3a = fqd_mul(rr, fqd_sub<10, 1, 1>(V, X3));   // (V - X3 + 10p < 12) x (rr < 9): < 2
  const FqD Y3 = fqd_sub<5, 1, 2>(Y3a, fqd_mul(S1, J));    // - 2 S1 J + 5p: < 7 (2 S1 J < 4)
  const FqD Z3 = fqd_smul<2>(fqd_mul(fqd_mul(p.z, q.z), H));  // 2 Z1 Z2 H: (16 -> < 2) x 5 -> < 2, x 2: < 4
  return {X3, Y3, Z3};
}

// -x for x < 2p: 3p - x < 3p
ZG_INL FqD fqd_neg2(const FqD& x) { return fqd_sub<3, 0, 1>(fqd_zero(), x); }

// G1 subgroup check (zg_curve.h g1_in_subgroup, same test): sigma(P) == -[x^2] P with the
// 127 doublings and 16 mixed additions in FqD
ZG_DEC_INL inline bool g1_in_subgroup_d(const G1A& p) {
  if (p.inf) return true;
  const FqD px = fqd_from(p.x), py = fqd_from(p.y);
  G1D q = g1d_from_aff(px, py);
  for (int i = 126; i >= 0; i--) {  // bit 127 of x^2 is the leading one
    q = g1d_dbl(q);
    if ((X2_ABS[i >> 5] >> (i & 31)) & 1u) q = g1d_add_aff(q, px, py);
  }
  const G1A s = {fq_mul(p.x, fq_const(G1_BETA)), fq_neg(p.y), false};
  return jac_eq_aff(g1d_to_jac(q), s);
}

}  // namespace zg
