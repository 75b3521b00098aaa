// zg_curve.h -- G1 (y^2 = x^3 + 4 over Fq) and G2 (y^2 = x^3 + 4(u+1) over Fq2) on gfx950.
// Restates pairing 0.14.2 curve semantics: Jacobian
// arithmetic, compressed/uncompressed decoding (`into_affine`), subgroup membership.
//
// Subgroup checks use endomorphisms instead of pairing's naive [r]P (mathematically
// equivalent):
//   G1:  P in G1  <=>  sigma(P) = [-x^2] P,   sigma(x, y) = (beta x, y)      (Bowe 2019/814)
//   G2:  Q in G2  <=>  psi(Q)   = [u] Q,      psi = twist o Frobenius o untwist (Scott 2021/1130)
// Both are exercised against on-curve non-subgroup points in tests/.
#pragma once
#include "zg_tower.h"

namespace zg {

// ---- generic field-op overloads so one Jacobian template serves G1 and G2
ZG_INL Fq F_add(const Fq& a, const Fq& b) { return fq_add(a, b); }
ZG_INL Fq F_sub(const Fq& a, const Fq& b) { return fq_sub(a, b); }
ZG_INL Fq F_mul(const Fq& a, const Fq& b) { return fq_mul(a, b); }
ZG_INL Fq F_sqr(const Fq& a) { return fq_sqr(a); }
ZG_INL Fq F_dbl(const Fq& a) { return fq_dbl(a); }
ZG_INL Fq F_neg(const Fq& a) { return fq_neg(a); }
ZG_INL bool F_is_zero(const Fq& a) { return fq_is_zero(a); }
ZG_INL bool F_eq(const Fq& a, const Fq& b) { return fq_eq(a, b); }
ZG_INL Fq2 F_add(const Fq2& a, const Fq2& b) { return f2_add(a, b); }
ZG_INL Fq2 F_sub(const Fq2& a, const Fq2& b) { return f2_sub(a, b); }
ZG_INL Fq2 F_mul(const Fq2& a, const Fq2& b) { return f2_mul(a, b); }
ZG_INL Fq2 F_sqr(const Fq2& a) { return f2_sqr(a); }
ZG_INL Fq2 F_dbl(const Fq2& a) { return f2_dbl(a); }
ZG_INL Fq2 F_neg(const Fq2& a) { return f2_neg(a); }
ZG_INL bool F_is_zero(const Fq2& a) { return f2_is_zero(a); }
ZG_INL bool F_eq(const Fq2& a, const Fq2& b) { return f2_eq(a, b); }
template <class F> ZG_INL F F_one();
template <> ZG_INL Fq F_one<Fq>() { return fq_one(); }
template <> ZG_INL Fq2 F_one<Fq2>() { return f2_one(); }
template <class F> ZG_INL F F_zero();
template <> ZG_INL Fq F_zero<Fq>() { return fp_zero<FqM>(); }
template <> ZG_INL Fq2 F_zero<Fq2>() { return f2_zero(); }

template <class F>
struct Aff {
  F x, y;
  bool inf;
};
template <class F>
struct Jac {
  F x, y, z;  // z == 0  <=>  point at infinity
};
using G1A = Aff<Fq>;
using G1J = Jac<Fq>;
using G2A = Aff<Fq2>;
using G2J = Jac<Fq2>;

template <class F>
ZG_INL Jac<F> jac_infinity() {
  return {F_one<F>(), F_one<F>(), F_zero<F>()};
}
template <class F>
ZG_INL bool jac_is_inf(const Jac<F>& p) {
  return F_is_zero(p.z);
}
template <class F>
ZG_INL Jac<F> jac_from_aff(const Aff<F>& a) {
  return a.inf ? jac_infinity<F>() : Jac<F>{a.x, a.y, F_one<F>()};
}

// dbl-2009-l (a = 0): 2M + 5S
template <class F>
ZG_INL Jac<F> jac_dbl_inl(const Jac<F>& p) {
  F A = F_sqr(p.x);
  F B = F_sqr(p.y);
  F C = F_sqr(B);
  F D = F_dbl(F_sub(F_sub(F_sqr(F_add(p.x, B)), A), C));
  F E = F_add(F_dbl(A), A);
  F Fv = F_sqr(E);
  F X3 = F_sub(Fv, F_dbl(D));
  F C8 = F_dbl(F_dbl(F_dbl(C)));
  F Y3 = F_sub(F_mul(E, F_sub(D, X3)), C8);
  F Z3 = F_dbl(F_mul(p.y, p.z));
  return {X3, Y3, Z3};
}

template <class F>
ZG_NOINL void jac_dbl_p(Jac<F>* r, const Jac<F>* p) { *r = jac_dbl_inl(*p); }
template <class F>
ZG_INL Jac<F> jac_dbl(const Jac<F>& p) { Jac<F> r; jac_dbl_p(&r, &p); return r; }

// add-2007-bl with complete case handling (P == Q -> dbl, P == -Q -> infinity)
template <class F>
ZG_INL Jac<F> jac_add_inl(const Jac<F>& p, const Jac<F>& q) {
  if (jac_is_inf(p)) return q;
  if (jac_is_inf(q)) return p;
  F Z1Z1 = F_sqr(p.z);
  F Z2Z2 = F_sqr(q.z);
  F U1 = F_mul(p.x, Z2Z2);
  F U2 = F_mul(q.x, Z1Z1);
  F S1 = F_mul(F_mul(p.y, q.z), Z2Z2);
  F S2 = F_mul(F_mul(q.y, p.z), Z1Z1);
  F H = F_sub(U2, U1);
  F rr = F_dbl(F_sub(S2, S1));
  if (F_is_zero(H)) {
    if (F_is_zero(rr)) return jac_dbl(p);
    return jac_infinity<F>();
  }
  F I = F_sqr(F_dbl(H));
  F J = F_mul(H, I);
  F V = F_mul(U1, I);
  F X3 = F_sub(F_sub(F_sqr(rr), J), F_dbl(V));
  F Y3 = F_sub(F_mul(rr, F_sub(V, X3)), F_dbl(F_mul(S1, J)));
  F Z3 = F_mul(F_sub(F_sub(F_sqr(F_add(p.z, q.z)), Z1Z1), Z2Z2), H);
  return {X3, Y3, Z3};
}

// the same with the doubling case inlined too (no out-of-line call with pointers to the
// caller's frame: kernels that must not touch scratch)
template <class F>
ZG_INL Jac<F> jac_add_full(const Jac<F>& p, const Jac<F>& q) {
  if (jac_is_inf(p)) return q;
  if (jac_is_inf(q)) return p;
  F Z1Z1 = F_sqr(p.z);
  F Z2Z2 = F_sqr(q.z);
  F U1 = F_mul(p.x, Z2Z2);
  F U2 = F_mul(q.x, Z1Z1);
  F S1 = F_mul(F_mul(p.y, q.z), Z2Z2);
  F S2 = F_mul(F_mul(q.y, p.z), Z1Z1);
  F H = F_sub(U2, U1);
  F rr = F_dbl(F_sub(S2, S1));
  if (F_is_zero(H)) {
    if (F_is_zero(rr)) return jac_dbl_inl(p);
    return jac_infinity<F>();
  }
  F I = F_sqr(F_dbl(H));
  F J = F_mul(H, I);
  F V = F_mul(U1, I);
  F X3 = F_sub(F_sub(F_sqr(rr), J), F_dbl(V));
  F Y3 = F_sub(F_mul(rr, F_sub(V, X3)), F_dbl(F_mul(S1, J)));
  F Z3 = F_mul(F_sub(F_sub(F_sqr(F_add(p.z, q.z)), Z1Z1), Z2Z2), H);
  return {X3, Y3, Z3};
}

template <class F>
ZG_NOINL void jac_add_p(Jac<F>* r, const Jac<F>* p, const Jac<F>* q) { *r = jac_add_inl(*p, *q); }
template <class F>
ZG_INL Jac<F> jac_add(const Jac<F>& p, const Jac<F>& q) { Jac<F> r; jac_add_p(&r, &p, &q); return r; }

// madd-2007-bl: p Jacobian + q affine (finite), complete case handling
template <class F>
ZG_INL Jac<F> jac_add_aff_inl(const Jac<F>& p, const Aff<F>& q) {
  if (q.inf) return p;
  if (jac_is_inf(p)) return Jac<F>{q.x, q.y, F_one<F>()};
  F Z1Z1 = F_sqr(p.z);
  F U2 = F_mul(q.x, Z1Z1);
  F S2 = F_mul(F_mul(q.y, p.z), Z1Z1);
  F H = F_sub(U2, p.x);
  F rr = F_dbl(F_sub(S2, p.y));
  if (F_is_zero(H)) {
    if (F_is_zero(rr)) return jac_dbl_inl(p);  // inlined: no pointer to p (keeps p out of scratch)
    return jac_infinity<F>();
  }
  F HH = F_sqr(H);
  F I = F_dbl(F_dbl(HH));
  F J = F_mul(H, I);
  F V = F_mul(p.x, I);
  F X3 = F_sub(F_sub(F_sqr(rr), J), F_dbl(V));
  F Y3 = F_sub(F_mul(rr, F_sub(V, X3)), F_dbl(F_mul(p.y, J)));
  F Z3 = F_sub(F_sub(F_sqr(F_add(p.z, H)), Z1Z1), HH);
  return {X3, Y3, Z3};
}

template <class F>
ZG_NOINL void jac_add_aff_p(Jac<F>* r, const Jac<F>* p, const Aff<F>* q) { *r = jac_add_aff_inl(*p, *q); }
template <class F>
ZG_INL Jac<F> jac_add_aff(const Jac<F>& p, const Aff<F>& q) { Jac<F> r; jac_add_aff_p(&r, &p, &q); return r; }

template <class F>
ZG_INL Jac<F> jac_neg(const Jac<F>& p) {
  return {p.x, F_neg(p.y), p.z};
}

// [k] q for a scalar given as little-endian 32-bit limbs (canonical, not Montgomery).
template <class F>
ZG_NOINL void jac_mul_limbs_p(Jac<F>* out, const Aff<F>* qp, const uint32_t* k, int nbits) {
  const Aff<F> q = *qp;
  Jac<F> acc = jac_infinity<F>();
  for (int i = nbits - 1; i >= 0; i--) {  // point ops inlined: acc stays in registers
    acc = jac_dbl_inl(acc);
    if ((k[i >> 5] >> (i & 31)) & 1u) acc = jac_add_aff_inl(acc, q);
  }
  *out = acc;
}
template <class F>
ZG_INL Jac<F> jac_mul_limbs(const Aff<F>& q, const uint32_t* k, int nbits) {
  Jac<F> r;
  jac_mul_limbs_p(&r, &q, k, nbits);
  return r;
}
template <class F>
ZG_INL Jac<F> jac_mul_u64(const Aff<F>& q, uint64_t k) {
  uint32_t l[2] = {(uint32_t)k, (uint32_t)(k >> 32)};
  return jac_mul_limbs(q, l, 64);
}

ZG_INL Fq F_inv(const Fq& a) { return fq_inv(a); }
ZG_INL Fq2 F_inv(const Fq2& a) { return f2_inv(a); }
template <class F>
ZG_INL Aff<F> jac_to_aff(const Jac<F>& p) {
  if (jac_is_inf(p)) return {F_zero<F>(), F_zero<F>(), true};
  F zi = F_inv(p.z);
  F zi2 = F_sqr(zi);
  return {F_mul(p.x, zi2), F_mul(p.y, F_mul(zi2, zi)), false};
}
// p (Jacobian) == q (affine, finite)?
template <class F>
ZG_INL bool jac_eq_aff(const Jac<F>& p, const Aff<F>& q) {
  if (jac_is_inf(p)) return q.inf;
  if (q.inf) return false;
  F z2 = F_sqr(p.z);
  return F_eq(F_mul(q.x, z2), p.x) && F_eq(F_mul(q.y, F_mul(z2, p.z)), p.y);
}

// ------------------------------------------------------------------ subgroup checks
ZG_NOINL inline bool g1_in_subgroup(const G1A& p) {
  if (p.inf) return true;
  // [x^2] P  with x^2 < 2^128 (positive), then sigma(P) == -[x^2]P; the point ops are inlined
  // so the Jacobian state stays in registers (the exponent is uniform: no divergence)
  G1J q = jac_from_aff(p);
  for (int i = 126; i >= 0; i--) {  // bit 127 of x^2 is the leading one
    q = jac_dbl_inl(q);
    if ((X2_ABS[i >> 5] >> (i & 31)) & 1u) q = jac_add_aff_inl(q, p);
  }
  G1A s = {fq_mul(p.x, fq_const(G1_BETA)), fq_neg(p.y), false};
  return jac_eq_aff(q, s);
}
ZG_INL G2A g2_psi(const G2A& p) {
  return {f2_mul(f2_conj(p.x), f2_const(PSI_X)), f2_mul(f2_conj(p.y), f2_const(PSI_Y)), p.inf};
}
ZG_NOINL inline bool g2_in_subgroup(const G2A& p) {
  if (p.inf) return true;
  // [u]P = -[|u|]P ; check psi(P) == [u]P  <=>  -psi(P) == [|u|] P
  G2J q = jac_mul_u64(p, BLS_X);
  G2A s = g2_psi(p);
  s.y = f2_neg(s.y);
  return jac_eq_aff(q, s);
}

ZG_INL bool g1_on_curve(const G1A& p) {
  if (p.inf) return true;
  Fq rhs = fq_add(fq_mul(fq_sqr(p.x), p.x), fq_const(FQ_B4));
  return fq_eq(fq_sqr(p.y), rhs);
}
ZG_INL bool g2_on_curve(const G2A& p) {
  if (p.inf) return true;
  Fq2 rhs = f2_add(f2_mul(f2_sqr(p.x), p.x), f2_const(FQ2_B));
  return f2_eq(f2_sqr(p.y), rhs);
}

// "lexicographically greatest" of y vs -y (pairing Ord; Fq2 compares c1 first).
// For a canonical y != 0:  y > -y  <=>  y > (p-1)/2.
ZG_INL bool fq_lex_greatest(const Fq& y_mont) {
  Fq c = fq_from_mont(y_mont);
  Fq half;
#pragma unroll
  for (int i = 0; i < 12; i++) half.l[i] = 0;
  // (p-1)/2 = p >> 1
#pragma unroll
  for (int i = 0; i < 12; i++) half.l[i] = (FQ_P[i] >> 1) | (i < 11 ? (FQ_P[i + 1] << 31) : 0u);
  return fp_gt_canon<FqM>(c, half);
}
ZG_INL bool f2_lex_greatest(const Fq2& y) {
  if (!fq_is_zero(y.c1)) return fq_lex_greatest(y.c1);
  return fq_lex_greatest(y.c0);
}

// ------------------------------------------------------------------ decoding
// Decode outcomes
enum : int { DEC_OK = 0, DEC_INFINITY = 1, DEC_ERR = 2 };

// pairing 0.14 G1Compressed::into_affine (subgroup-checked). 48 bytes.
ZG_NOINL inline int g1_decompress(const uint8_t* b, G1A* out, bool check_subgroup = true) {
  uint8_t f = b[0];
  if (!(f & 0x80)) return DEC_ERR;  // UnexpectedCompressionMode
  if (f & 0x40) {                   // infinity: remaining bits (incl. 0x20) must be zero
    uint8_t acc = f & 0x3f;
    for (int i = 1; i < 48; i++) acc |= b[i];
    if (acc) return DEC_ERR;
    out->inf = true;
    return DEC_INFINITY;
  }
  const bool greatest = f & 0x20;
  uint8_t tmp[48];
  for (int i = 0; i < 48; i++) tmp[i] = b[i];
  tmp[0] &= 0x1f;
  Fq x = fq_limbs_from_be(tmp);
  if (!fp_lt_modulus<FqM>(x)) return DEC_ERR;
  x = fq_to_mont(x);
  Fq rhs = fq_add(fq_mul(fq_sqr(x), x), fq_const(FQ_B4));
  Fq y;
  if (!fq_sqrt(rhs, &y)) return DEC_ERR;  // NotOnCurve
  // pick y if (y < -y) ^ greatest, else -y
  const bool y_gt = fq_lex_greatest(y);          // y > -y (false when y == 0)
  const bool y_lt = !y_gt && !fq_is_zero(y);     // y < -y
  if (!(y_lt ^ greatest)) y = fq_neg(y);
  out->x = x;
  out->y = y;
  out->inf = false;
  if (check_subgroup && !g1_in_subgroup(*out)) return DEC_ERR;
  return DEC_OK;
}

// pairing 0.14 G2Compressed::into_affine. 96 bytes: x.c1 (flags) || x.c0.
ZG_DEC_INL inline int g2_decompress(const uint8_t* b, G2A* out, bool check_subgroup = true) {
  uint8_t f = b[0];
  if (!(f & 0x80)) return DEC_ERR;
  if (f & 0x40) {
    uint8_t acc = f & 0x3f;
    for (int i = 1; i < 96; i++) acc |= b[i];
    if (acc) return DEC_ERR;
    out->inf = true;
    return DEC_INFINITY;
  }
  const bool greatest = f & 0x20;
  uint8_t tmp[48];
  for (int i = 0; i < 48; i++) tmp[i] = b[i];
  tmp[0] &= 0x1f;
  Fq x1 = fq_limbs_from_be(tmp);
  Fq x0 = fq_limbs_from_be(b + 48);
  if (!fp_lt_modulus<FqM>(x1) || !fp_lt_modulus<FqM>(x0)) return DEC_ERR;
  Fq2 x = {fq_to_mont(x0), fq_to_mont(x1)};
  Fq2 rhs = f2_add(f2_mul(f2_sqr(x), x), f2_const(FQ2_B));
  Fq2 y;
  if (!f2_sqrt(rhs, &y)) return DEC_ERR;
  const bool y_gt = f2_lex_greatest(y);
  const bool y_lt = !y_gt && !f2_is_zero(y);
  if (!(y_lt ^ greatest)) y = f2_neg(y);
  out->x = x;
  out->y = y;
  out->inf = false;
  if (check_subgroup && !g2_in_subgroup(*out)) return DEC_ERR;
  return DEC_OK;
}

// pairing 0.14 G1Uncompressed::into_affine. 96 bytes x || y.
ZG_NOINL inline int g1_decode_uncompressed(const uint8_t* b, G1A* out) {
  uint8_t f = b[0];
  if (f & 0x80) return DEC_ERR;
  if (f & 0x40) {
    uint8_t acc = f & 0x3f;
    for (int i = 1; i < 96; i++) acc |= b[i];
    if (acc) return DEC_ERR;
    out->inf = true;
    return DEC_INFINITY;
  }
  if (f & 0x20) return DEC_ERR;
  uint8_t tmp[48];
  for (int i = 0; i < 48; i++) tmp[i] = b[i];
  tmp[0] &= 0x1f;
  Fq x = fq_limbs_from_be(tmp), y = fq_limbs_from_be(b + 48);
  if (!fp_lt_modulus<FqM>(x) || !fp_lt_modulus<FqM>(y)) return DEC_ERR;
  out->x = fq_to_mont(x);
  out->y = fq_to_mont(y);
  out->inf = false;
  if (!g1_on_curve(*out) || !g1_in_subgroup(*out)) return DEC_ERR;
  return DEC_OK;
}

// pairing 0.14 G2Uncompressed::into_affine. 192 bytes x.c1 || x.c0 || y.c1 || y.c0.
ZG_NOINL inline int g2_decode_uncompressed(const uint8_t* b, G2A* out) {
  uint8_t f = b[0];
  if (f & 0x80) return DEC_ERR;
  if (f & 0x40) {
    uint8_t acc = f & 0x3f;
    for (int i = 1; i < 192; i++) acc |= b[i];
    if (acc) return DEC_ERR;
    out->inf = true;
    return DEC_INFINITY;
  }
  if (f & 0x20) return DEC_ERR;
  uint8_t tmp[48];
  for (int i = 0; i < 48; i++) tmp[i] = b[i];
  tmp[0] &= 0x1f;
  Fq v[4] = {fq_limbs_from_be(tmp), fq_limbs_from_be(b + 48), fq_limbs_from_be(b + 96),
             fq_limbs_from_be(b + 144)};
  for (int i = 0; i < 4; i++)
    if (!fp_lt_modulus<FqM>(v[i])) return DEC_ERR;
  out->x = {fq_to_mont(v[1]), fq_to_mont(v[0])};
  out->y = {fq_to_mont(v[3]), fq_to_mont(v[2])};
  out->inf = false;
  if (!g2_on_curve(*out) || !g2_in_subgroup(*out)) return DEC_ERR;
  return DEC_OK;
}

// ------------------------------------------------------------------ encoding (synthetic data)
ZG_INL void g1_compress(const G1A& p, uint8_t* b) {
  if (p.inf) {
    b[0] = 0xc0;
    for (int i = 1; i < 48; i++) b[i] = 0;
    return;
  }
  fq_limbs_to_be(fq_from_mont(p.x), b);
  b[0] |= 0x80;
  if (fq_lex_greatest(p.y)) b[0] |= 0x20;
}
ZG_INL void g2_compress(const G2A& p, uint8_t* b) {
  if (p.inf) {
    b[0] = 0xc0;
    for (int i = 1; i < 96; i++) b[i] = 0;
    return;
  }
  fq_limbs_to_be(fq_from_mont(p.x.c1), b);
  fq_limbs_to_be(fq_from_mont(p.x.c0), b + 48);
  b[0] |= 0x80;
  if (f2_lex_greatest(p.y)) b[0] |= 0x20;
}

}  // namespace zg
