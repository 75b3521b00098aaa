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

}  // namespace zg
