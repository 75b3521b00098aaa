// zg_pairing.h -- optimal-ate Miller loop and final exponentiation for BLS12-381 on gfx950.
//
// Restates pairing 0.14.2 `Bls12::miller_loop`, `G2Prepared` (doubling_step /
// addition_step, Algorithms 26/27 of eprint 2010/354) and `Bls12::final_exponentiation`
// (SURVEY.md 8(a) rows a9-a11). The line coefficients and their evaluation are the same
// as the crate's, so per-proof Miller values are identical field elements; the final
// exponentiation is the crate's chain, whose exponent is 3 * (p^12 - 1) / r, so GT
// values are bit-identical to bellman's (they are cubes of the textbook pairing).
#pragma once
#include "zg_curve.h"

namespace zg {

struct Line {
  Fq2 c0, c1, c2;
};

// bits of (x >> 1) after its leading one, MSB first: x >> 1 = 0x6900800000008000 (63 bits)
#define ZG_XH 0x6900800000008000ull
#define ZG_XH_TOP 61

// pairing doubling_step: r <- 2r, returns the line coefficients
ZG_NOINL inline Line line_double(G2J& r) {
  Fq2 tmp0 = f2_sqr(r.x);
  Fq2 tmp1 = f2_sqr(r.y);
  Fq2 tmp2 = f2_sqr(tmp1);
  Fq2 tmp3 = f2_sub(f2_sub(f2_sqr(f2_add(tmp1, r.x)), tmp0), tmp2);
  tmp3 = f2_dbl(tmp3);
  Fq2 tmp4 = f2_add(f2_dbl(tmp0), tmp0);
  Fq2 tmp6 = f2_add(r.x, tmp4);
  Fq2 tmp5 = f2_sqr(tmp4);
  Fq2 zsq = f2_sqr(r.z);
  Fq2 nx = f2_sub(f2_sub(tmp5, tmp3), tmp3);
  Fq2 nz = f2_sub(f2_sub(f2_sqr(f2_add(r.z, r.y)), tmp1), zsq);
  Fq2 ny = f2_mul(f2_sub(tmp3, nx), tmp4);
  tmp2 = f2_dbl(f2_dbl(f2_dbl(tmp2)));
  ny = f2_sub(ny, tmp2);
  tmp3 = f2_neg(f2_dbl(f2_mul(tmp4, zsq)));
  tmp6 = f2_sub(f2_sub(f2_sqr(tmp6), tmp0), tmp5);
  tmp1 = f2_dbl(f2_dbl(tmp1));
  tmp6 = f2_sub(tmp6, tmp1);
  tmp0 = f2_dbl(f2_mul(nz, zsq));
  r = {nx, ny, nz};
  return {tmp0, tmp3, tmp6};
}

// pairing addition_step: r <- r + q (q affine), returns the line coefficients
ZG_NOINL inline Line line_add(G2J& r, const G2A& q) {
  Fq2 zsq = f2_sqr(r.z);
  Fq2 ysq = f2_sqr(q.y);
  Fq2 t0 = f2_mul(zsq, q.x);
  Fq2 t1 = f2_mul(f2_sub(f2_sub(f2_sqr(f2_add(q.y, r.z)), ysq), zsq), zsq);
  Fq2 t2 = f2_sub(t0, r.x);
  Fq2 t3 = f2_sqr(t2);
  Fq2 t4 = f2_dbl(f2_dbl(t3));
  Fq2 t5 = f2_mul(t4, t2);
  Fq2 t6 = f2_sub(f2_sub(t1, r.y), r.y);
  Fq2 t9 = f2_mul(t6, q.x);
  Fq2 t7 = f2_mul(t4, r.x);
  Fq2 nx = f2_sub(f2_sub(f2_sub(f2_sqr(t6), t5), t7), t7);
  Fq2 nz = f2_sub(f2_sub(f2_sqr(f2_add(r.z, t2)), zsq), t3);
  Fq2 t10 = f2_add(q.y, nz);
  Fq2 t8 = f2_mul(f2_sub(t7, nx), t6);
  t0 = f2_dbl(f2_mul(r.y, t5));
  Fq2 ny = f2_sub(t8, t0);
  t10 = f2_sub(f2_sub(f2_sqr(t10), ysq), f2_sqr(nz));
  t9 = f2_sub(f2_dbl(t9), t10);
  t10 = f2_dbl(nz);
  t6 = f2_neg(t6);
  t1 = f2_dbl(t6);
  r = {nx, ny, nz};
  return {t10, t1, t9};
}

// pairing `ell`: f *= (c2 + (c1 * px) v + (c0 * py) v w)
ZG_INL Fq12 ell(const Fq12& f, const Line& c, const Fq& px, const Fq& py) {
  return f12_mul_by_014(f, c.c2, f2_mul_fq(c.c1, px), f2_mul_fq(c.c0, py));
}

// Miller loop of one pair with G2 lines computed on the fly. p, q finite (callers skip
// infinity pairs exactly like the crate). Result already conjugated (u < 0).
ZG_NOINL inline Fq12 miller_loop_1(const G1A& p, const G2A& q) {
  Fq12 f = f12_one();
  G2J r = {q.x, q.y, f2_one()};
  for (int i = ZG_XH_TOP; i >= 0; i--) {
    f = ell(f, line_double(r), p.x, p.y);
    if ((ZG_XH >> i) & 1ull) f = ell(f, line_add(r, q), p.x, p.y);
    f = f12_sqr(f);
  }
  f = ell(f, line_double(r), p.x, p.y);
  return f12_conj(f);
}

// number of line coefficient triples per prepared G2 point
#define ZG_NCOEFF 68

// G2Prepared::from_affine into a caller buffer of ZG_NCOEFF lines
ZG_NOINL inline void g2_prepare(const G2A& q, Line* out) {
  G2J r = {q.x, q.y, f2_one()};
  int n = 0;
  for (int i = ZG_XH_TOP; i >= 0; i--) {
    out[n++] = line_double(r);
    if ((ZG_XH >> i) & 1ull) out[n++] = line_add(r, q);
  }
  out[n++] = line_double(r);
}

// Miller loop of one pair with prepared lines (e.g. -gamma, -delta of a VK).
ZG_NOINL inline Fq12 miller_loop_prepared(const G1A& p, const Line* coeffs) {
  Fq12 f = f12_one();
  int n = 0;
  for (int i = ZG_XH_TOP; i >= 0; i--) {
    f = ell(f, coeffs[n++], p.x, p.y);
    if ((ZG_XH >> i) & 1ull) f = ell(f, coeffs[n++], p.x, p.y);
    f = f12_sqr(f);
  }
  f = ell(f, coeffs[n++], p.x, p.y);
  return f12_conj(f);
}

ZG_INL Fq12 exp_by_x(const Fq12& f, uint64_t x) { return f12_conj(f12_pow_u64(f, x)); }

// Bls12::final_exponentiation (pairing 0.14.2 chain). f must be non-zero.
ZG_NOINL inline Fq12 final_exponentiation(const Fq12& f) {
  Fq12 f1 = f12_conj(f);
  Fq12 f2 = f12_inv(f);
  Fq12 r = f12_mul(f1, f2);
  f2 = r;
  r = f12_mul(f12_frob(r, 2), f2);
  const uint64_t x = BLS_X;
  Fq12 y0 = f12_sqr(r);
  Fq12 y1 = exp_by_x(y0, x);
  Fq12 y2 = exp_by_x(y1, x >> 1);
  Fq12 y3 = f12_conj(r);
  y1 = f12_mul(y1, y3);
  y1 = f12_conj(y1);
  y1 = f12_mul(y1, y2);
  y2 = exp_by_x(y1, x);
  y3 = exp_by_x(y2, x);
  y1 = f12_conj(y1);
  y3 = f12_mul(y3, y1);
  y1 = f12_conj(y1);
  y1 = f12_frob(y1, 3);
  y2 = f12_frob(y2, 2);
  y1 = f12_mul(y1, y2);
  y2 = exp_by_x(y3, x);
  y2 = f12_mul(y2, y0);
  y2 = f12_mul(y2, r);
  y1 = f12_mul(y1, y2);
  y2 = f12_frob(y3, 1);
  y1 = f12_mul(y1, y2);
  return y1;
}

}  // namespace zg
