// zg_lines.h -- the straight-line R-chain step functions (lane = proof): pairing 0.14.2's
// doubling_step / addition_step (zg_pairing.h line_double / line_add, the same formulas) in the
// 29-bit-digit Fq2 products, each scaled line coefficient stored as soon as it is known. Used by
// k_batch_lines_lane (zg_lines.hip); __host__ __device__, so tests/native runs the same code.
#pragma once
#include "zg_batch.h"

namespace zg {

// x^2 (canonical x), x y (x < 2p per coefficient, y canonical), x s: the 29-bit-digit forms.
// Each product is fenced by scheduling barriers: the scheduler would otherwise interleave the
// independent products of a step for ILP and keep all their digit vectors live at once (742
// spilled VGPRs); fenced, only the step's live values plus one product's digits are resident.
#if defined(__HIP_DEVICE_COMPILE__)
#define LS_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define LS_FENCE()
#endif
ZG_INL Fq2 ls_sqr(const Fq2& a) {
  LS_FENCE();
  const Fq d = fq_sub(a.c0, a.c1);
  Fq2 r;
  f2_sqr29(r.c0.l, r.c1.l, a.c0.l, a.c1.l, d.l);
  LS_FENCE();
  return r;
}
ZG_INL Fq2 ls_mul(const Fq2& a, const Fq2& b) {
  LS_FENCE();
  Fq2 r;
  f2_mul29(r.c0.l, r.c1.l, a.c0.l, a.c1.l, b.c0.l, b.c1.l);
  LS_FENCE();
  return r;
}
ZG_INL Fq2 ls_mulfq(const Fq2& a, const Fq& s) {
  LS_FENCE();
  Fq2 r;
  f2_mul_fq29(r.c0.l, r.c1.l, a.c0.l, a.c1.l, s.l);
  LS_FENCE();
  return r;
}

// The running point R = (X, Y, Z) lives in a per-lane state store St (get / put of coordinate 0, 1,
// 2): LDS on the device (LinesLds, conflict-free lane-contiguous rows), a plain struct on the host.
// Each coordinate is read where a product needs it and rewritten as soon as its new value is known,
// so registers hold at most four step temporaries next to one product's digits: the step fits 256
// VGPRs (two waves per SIMD) without the 672 B/lane of scratch spills of round 3's register-resident
// state.
struct LinesHost {
  Fq2 v[3];
  ZG_HD Fq2 get(int i) const { return v[i]; }
  ZG_HD void put(int i, const Fq2& x) { v[i] = x; }
};

// pairing doubling_step (line_double of zg_pairing.h), the scaled line stored as soon as each
// coefficient is known. tmp4 = 3 tmp0 is re-formed where used (two additions) instead of held.
template <class St>
ZG_INL void ls_double(St& st, const G1A* pa, Fq2* dst, bool act) {
  const Fq2 tmp1 = ls_sqr(st.get(1));
  const Fq2 zsq = ls_sqr(st.get(2));
  {
    const Fq2 nz = f2_sub(f2_sub(ls_sqr(f2_add(st.get(2), st.get(1))), tmp1), zsq);
    dst[2] = act ? ls_mulfq(f2_dbl(ls_mul(nz, zsq)), pa->y) : f2_one();  // c0 py
    st.put(2, nz);
  }
  const Fq2 tmp0 = ls_sqr(st.get(0));
  dst[1] = act ? ls_mulfq(f2_neg(f2_dbl(ls_mul(f2_add(f2_dbl(tmp0), tmp0), zsq))), pa->x) : f2_one();  // c1 px
  const Fq2 tmp5 = ls_sqr(f2_add(f2_dbl(tmp0), tmp0));
  dst[0] = act ? f2_sub(f2_sub(f2_sub(ls_sqr(f2_add(st.get(0), f2_add(f2_dbl(tmp0), tmp0))), tmp0), tmp5),
                        f2_dbl(f2_dbl(tmp1)))
               : f2_one();
  const Fq2 tmp2 = ls_sqr(tmp1);
  const Fq2 tmp3 = f2_dbl(f2_sub(f2_sub(ls_sqr(f2_add(tmp1, st.get(0))), tmp0), tmp2));
  const Fq2 nx = f2_sub(f2_sub(tmp5, tmp3), tmp3);
  st.put(0, nx);
  st.put(1, f2_sub(ls_mul(f2_sub(tmp3, nx), f2_add(f2_dbl(tmp0), tmp0)), f2_dbl(f2_dbl(f2_dbl(tmp2)))));
}

// pairing addition_step (line_add of zg_pairing.h) with q affine (read from HBM where used), scaled
// line. qy^2 is formed twice (one squaring per addition step, 5 per loop) instead of held.
template <class St>
ZG_INL void ls_add(St& st, const G2A* pq, const G1A* pa, Fq2* dst, bool act) {
  const Fq2 zsq = ls_sqr(st.get(2));
  const Fq2 t2 = f2_sub(ls_mul(zsq, pq->x), st.get(0));
  const Fq2 t6 = f2_sub(f2_sub(ls_mul(f2_sub(f2_sub(ls_sqr(f2_add(pq->y, st.get(2))), ls_sqr(pq->y)), zsq), zsq),
                               st.get(1)),
                        st.get(1));
  const Fq2 t3 = ls_sqr(t2);
  st.put(2, f2_sub(f2_sub(ls_sqr(f2_add(st.get(2), t2)), zsq), t3));  // nz
  dst[2] = act ? ls_mulfq(f2_dbl(st.get(2)), pa->y) : f2_one();       // c0 py
  dst[1] = act ? ls_mulfq(f2_dbl(f2_neg(t6)), pa->x) : f2_one();      // c1 px
  {
    const Fq2 nz = st.get(2);
    const Fq2 t10 = f2_sub(f2_sub(ls_sqr(f2_add(pq->y, nz)), ls_sqr(pq->y)), ls_sqr(nz));
    dst[0] = act ? f2_sub(f2_dbl(ls_mul(t6, pq->x)), t10) : f2_one();
  }
  const Fq2 t4 = f2_dbl(f2_dbl(t3));
  const Fq2 t5 = ls_mul(t4, t2);
  const Fq2 t7 = ls_mul(t4, st.get(0));
  const Fq2 nx = f2_sub(f2_sub(f2_sub(ls_sqr(t6), t5), t7), t7);
  const Fq2 ny = f2_sub(ls_mul(f2_sub(t7, nx), t6), f2_dbl(ls_mul(st.get(1), t5)));
  st.put(0, nx);
  st.put(1, ny);
}

// ---- the affine R-chain (ZG_LINES_AFFINE, round 6; zg_lines.hip k_batch_lines_aff) ----
// Fq products in 29-bit digits, fenced like the Fq2 ones above
ZG_INL Fq ls_fqmul(const Fq& a, const Fq& b) {
  LS_FENCE();
  Fq r;
  fq29_mul(r.l, a.l, b.l);
  LS_FENCE();
  return r;
}
ZG_INL Fq ls_fqsqr(const Fq& a) {
  LS_FENCE();
  Fq r;
  fq29_sqr(r.l, a.l);
  LS_FENCE();
  return r;
}
// N(d) = d0^2 + d1^2 (u^2 = -1): 1 / d = conj(d) / N(d); N(d) = 0 only for d = 0 (-1 is a non-residue mod p)
ZG_INL Fq ls_norm(const Fq2& d) { return fq_add(ls_fqsqr(d.c0), ls_fqsqr(d.c1)); }

// the G2 generator (Montgomery): the point an R-chain lane without a B to check walks, so that its
// denominators never vanish (its lines are not used)
ZG_HD inline G2A g2_generator() {
  static constexpr uint32_t X0[12] = {0x02940a10u, 0xf5f28fa2u, 0x87b4961au, 0xb3f5fb26u, 0x3e2ae580u, 0xa1a893b5u,
                                      0x1a3caee9u, 0x9894999du, 0x1863366bu, 0x6f67b763u, 0x4350bcd7u, 0x05819192u};
  static constexpr uint32_t X1[12] = {0x9e23f606u, 0xa5a9c075u, 0xbccd60c3u, 0xaaa0c59du, 0xe2867806u, 0x3bb17e18u,
                                      0x8541b367u, 0x1b1ab6ccu, 0xf2158547u, 0xc2b6ed0eu, 0x7360edf3u, 0x11922a09u};
  static constexpr uint32_t Y0[12] = {0x60494c4au, 0x4c730af8u, 0x5e369c5au, 0x597cfa1fu, 0xaa0a635au, 0xe7e6856cu,
                                      0x6e0d495fu, 0xbbefb5e9u, 0xf0ef25a2u, 0x07d3a975u, 0x7e80dae5u, 0x0083fd8eu};
  static constexpr uint32_t Y1[12] = {0xdf64b05du, 0xadc0fc92u, 0x2b1461dcu, 0x18aa270au, 0x3be4eba0u, 0x86adac6au,
                                      0xc93da33au, 0x79495c4eu, 0xa43ccaedu, 0xe7175850u, 0x63de1bf2u, 0x0b2bc2a1u};
  G2A g;
  for (int i = 0; i < 12; i++) {
    g.x.c0.l[i] = X0[i];
    g.x.c1.l[i] = X1[i];
    g.y.c0.l[i] = Y0[i];
    g.y.c1.l[i] = Y1[i];
  }
  g.inf = false;
  return g;
}

// One affine step of G2Prepared's chain, given 1 / N(d) for its denominator d (2y for a doubling,
// xQ - x for an addition): lambda = num conj(d) / N(d), (x, y) <- (lambda^2 - x - x', lambda (x - x3) - y),
// and the line through the point with slope lambda normalised by its v w coefficient and by py:
//   a = (lambda x - y) / py, b = -lambda px / py   (ab = (1/py, px/py); 0 for a proof without a line:
//   the line v w, FE-trivial). Same group law as ls_double / ls_add (pairing's doubling_step /
//   addition_step, which give these lines times an element of Fq2).
ZG_INL void ls_aff_step(Fq2& x, Fq2& y, const G2A* q, bool dbl, const Fq& ninv, const Fq2& ab, Fq2* a_out,
                        Fq2* b_out) {
  const Fq2 d = dbl ? f2_dbl(y) : f2_sub(q->x, x);
  const Fq2 dinv = ls_mulfq(f2_conj(d), ninv);
  Fq2 num;
  if (dbl) {
    const Fq2 x2 = ls_sqr(x);
    num = f2_add(f2_dbl(x2), x2);
  } else {
    num = f2_sub(q->y, y);
  }
  const Fq2 lam = ls_mul(num, dinv);
  const Fq2 x3 = f2_sub(ls_sqr(lam), dbl ? f2_dbl(x) : f2_add(x, q->x));
  const Fq2 c2 = f2_sub(ls_mul(lam, x), y);
  *a_out = ls_mulfq(c2, ab.c0);
  *b_out = f2_neg(ls_mulfq(lam, ab.c1));
  y = f2_sub(c2, ls_mul(lam, x3));
  x = x3;
}

}  // namespace zg
