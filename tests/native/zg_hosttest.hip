// TEST HARNESS ONLY -- runs the product's __host__ __device__ arithmetic (zebra_amd/csrc)
// on the CPU so the CPU-only test tier can check it against the oracle without a GPU.
// Never linked into, or loaded by, the product library.
#include <string.h>
#include "../../zebra_amd/csrc/zg_coop.h"
#include "../../zebra_amd/csrc/zg_groth16.h"
#include "../../zebra_amd/csrc/zg_bingcd.h"
#include "../../zebra_amd/csrc/zg_bn254.h"
#include "../../zebra_amd/csrc/zg_lines.h"
#include "../../zebra_amd/csrc/zg_msm.h"

using namespace zg;

static Fq ld_fq(const uint8_t* b) { return fq_to_mont(fq_limbs_from_be(b)); }
static void st_fq(const Fq& a, uint8_t* b) { fq_limbs_to_be(fq_from_mont(a), b); }

extern "C" {

// G1 subgroup check and GLV product r A in the word form (zg_curve.h / zg_groth16.h) and in lazy
// digits (zg_fqd.h) for an affine point (x, y: 48-byte BE, canonical, on the curve): res[0..1]
// the two subgroup verdicts; out_w / out_d the affine [k0 + k1 lambda] P (96 B each, zero bytes
// for infinity) from the word / digit GLV with k0 = 2a + 1, k1 = b
void zgt_g1_check_glv(const uint8_t* x, const uint8_t* y, uint64_t a, uint64_t b, int* res, uint8_t* out_w,
                      uint8_t* out_d) {
  const G1A p = {ld_fq(x), ld_fq(y), false};
  res[0] = g1_in_subgroup(p);
  res[1] = g1_in_subgroup_d(p);
  const G1A w = jac_to_aff(g1_glv_mul(p, a, b));
  const G1A d = jac_to_aff(g1_glv_mul_d(p, a, b));
  const G1A d2 = jac_to_aff(g1_glv_mul_w2(p, a, b));
  res[2] = d2.inf == d.inf && (d.inf || (fq_eq(d2.x, d.x) && fq_eq(d2.y, d.y)));
  memset(out_w, 0, 96);
  memset(out_d, 0, 96);
  if (!w.inf) {
    st_fq(w.x, out_w);
    st_fq(w.y, out_w + 48);
  }
  if (!d.inf) {
    st_fq(d.x, out_d);
    st_fq(d.y, out_d + 48);
  }
}

static void st_aff(const G1J& j, uint8_t* out) {
  const G1A a = jac_to_aff(j);
  memset(out, 0, 96);
  if (!a.inf) {
    st_fq(a.x, out);
    st_fq(a.y, out + 48);
  }
}
static G1J jac_scaled(const uint8_t* x, const uint8_t* y, const uint8_t* z) {
  const Fq zz = ld_fq(z);
  if (fq_is_zero(zz)) return jac_infinity<Fq>();
  const Fq z2 = fq_sqr(zz);
  return {fq_mul(ld_fq(x), z2), fq_mul(ld_fq(y), fq_mul(z2, zz)), zz};
}
static G1D g1d_of(const G1J& j) { return {fqd_from(j.x), fqd_from(j.y), fqd_from(j.z)}; }

// K4's lazy-digit point sums (zg_fqd.h) against the word form (zg_curve.h): p = (x1, y1) and
// q = (x2, y2) as Jacobian points scaled by z1 / z2 (zero: infinity). out_w / out_d: affine p + q
// by jac_add_full / g1d_add_full; out_mw / out_md: p - (x2, y2) by jac_add_aff_inl / g1d_add_aff
// with the negated y < 3p of the bucket phase (96 B each, zero bytes for infinity)
void zgt_g1d_add(const uint8_t* x1, const uint8_t* y1, const uint8_t* z1, const uint8_t* x2, const uint8_t* y2,
                 const uint8_t* z2, uint8_t* out_w, uint8_t* out_d, uint8_t* out_mw, uint8_t* out_md) {
  const G1J p = jac_scaled(x1, y1, z1), q = jac_scaled(x2, y2, z2);
  st_aff(jac_add_full(p, q), out_w);
  st_aff(g1d_to_jac(g1d_add_full(g1d_of(p), g1d_of(q))), out_d);
  const G1A qa = {ld_fq(x2), fq_neg(ld_fq(y2)), false};
  st_aff(jac_add_aff_inl(p, qa), out_mw);
  st_aff(g1d_to_jac(g1d_add_aff(g1d_of(p), fqd_from(ld_fq(x2)), fqd_neg2(fqd_from(ld_fq(y2))))), out_md);
}

// K4's signed-digit windows (zg_msm.h msm_shape / msm_digit) of the scalar lo + 2^64 hi for a
// batch of npad padded proofs: digits[w], shifts[w], widths[w]; returns the window count, or -1
// when the final carry is not zero; shape[] = c, w, nb, parts
int zgt_msm_digits(uint64_t lo, uint32_t hi, uint64_t npad, int* digits, int* shifts, int* widths, int* shape) {
  const MsmShape S = msm_shape((size_t)npad);
  shape[0] = S.c;
  shape[1] = S.w;
  shape[2] = S.nb;
  shape[3] = S.parts;
  int carry = 0;
  for (int w = 0; w < S.w; w++) {
    digits[w] = msm_digit(lo, hi, S, w, &carry);
    shifts[w] = S.shift(w);
    widths[w] = S.width(w);
  }
  return carry ? -1 : S.w;
}

// the R-chain of zg_lines.h (k_batch_lines_lane) for one proof: B (x.c0 x.c1 y.c0 y.c1) and
// P = r A (x y), 48-byte BE each, canonical -> 68 x 3 scaled line coefficients (Fq2 as c0 || c1,
// BE) and, for comparison, the same from g2_prepare + the ell scaling (zg_pairing.h)
void zgt_lines_lane(const uint8_t* q, const uint8_t* p, uint8_t* out_lane, uint8_t* out_ref) {
  G2A B = {{ld_fq(q), ld_fq(q + 48)}, {ld_fq(q + 96), ld_fq(q + 144)}, false};
  G1A P = {ld_fq(p), ld_fq(p + 48), false};
  auto st2 = [](const Fq2& v, uint8_t* o) {
    st_fq(v.c0, o);
    st_fq(v.c1, o + 48);
  };
  LinesHost r = {{B.x, B.y, f2_one()}};
  Fq2 l[3];
  int n = 0;
  for (int i = ZG_XH_TOP; i >= -1; i--) {
    ls_double(r, &P, l, true);
    for (int j = 0; j < 3; j++) st2(l[j], out_lane + (n * 3 + j) * 96);
    n++;
    if (i >= 0 && ((ZG_XH >> i) & 1ull)) {
      ls_add(r, &B, &P, l, true);
      for (int j = 0; j < 3; j++) st2(l[j], out_lane + (n * 3 + j) * 96);
      n++;
    }
  }
  static Line ref[ZG_NCOEFF];
  g2_prepare(B, ref);
  for (int k = 0; k < ZG_NCOEFF; k++) {
    st2(ref[k].c2, out_ref + (k * 3 + 0) * 96);
    st2(f2_mul_fq(ref[k].c1, P.x), out_ref + (k * 3 + 1) * 96);
    st2(f2_mul_fq(ref[k].c0, P.y), out_ref + (k * 3 + 2) * 96);
  }
}

// the affine R-chain step of zg_lines.h (k_batch_lines_aff's ls_aff_step) for one proof, with every
// denominator inverted directly (the kernel batches them by Montgomery's trick): 68 (a, b) pairs of
// the unit-normalised lines, Fq2 as c0 || c1 BE, and the final affine point [x] B (x.c0 x.c1 y.c0 y.c1)
void zgt_lines_affine(const uint8_t* q, const uint8_t* p, uint8_t* out, uint8_t* last) {
  G2A B = {{ld_fq(q), ld_fq(q + 48)}, {ld_fq(q + 96), ld_fq(q + 144)}, false};
  const Fq px = ld_fq(p), py = ld_fq(p + 48);
  const Fq ipy = fq_inv(py);
  const Fq2 ab = {ipy, fq_mul(px, ipy)};
  Fq2 x = B.x, y = B.y;
  int n = 0;
  auto step = [&](bool dbl) {
    const Fq2 d = dbl ? f2_dbl(y) : f2_sub(B.x, x);
    const Fq ninv = fq_inv(ls_norm(d));
    Fq2 a, b;
    ls_aff_step(x, y, &B, dbl, ninv, ab, &a, &b);
    st_fq(a.c0, out + (n * 2) * 96);
    st_fq(a.c1, out + (n * 2) * 96 + 48);
    st_fq(b.c0, out + (n * 2 + 1) * 96);
    st_fq(b.c1, out + (n * 2 + 1) * 96 + 48);
    n++;
  };
  for (int i = ZG_XH_TOP; i >= -1; i--) {
    step(true);
    if (i >= 0 && ((ZG_XH >> i) & 1ull)) step(false);
  }
  st_fq(x.c0, last);
  st_fq(x.c1, last + 48);
  st_fq(y.c0, last + 96);
  st_fq(y.c1, last + 144);
}

// the products of zg_debug_field_mul (zebra_amd/csrc/zg_debug.hip) on the host: same field ids
void zgt_field_mul(int field, const uint32_t* a, const uint32_t* b, uint32_t* r) {
  switch (field) {
    case 0: fq29_mul(r, a, b); break;
    case 1: fq29_sqr(r, a); break;
    case 2: f2_mul29(r, r + 12, a, a + 12, b, b + 12); break;
    case 3: fr29_mul(r, a, b); break;
    default: bq29_mul(r, a, b); break;
  }
}

void zgt_fq_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) { st_fq(fq_mul(ld_fq(a), ld_fq(b)), out); }
void zgt_fq_add(const uint8_t* a, const uint8_t* b, uint8_t* out) { st_fq(fq_add(ld_fq(a), ld_fq(b)), out); }
void zgt_fq_sub(const uint8_t* a, const uint8_t* b, uint8_t* out) { st_fq(fq_sub(ld_fq(a), ld_fq(b)), out); }
void zgt_fq_inv(const uint8_t* a, uint8_t* out) { st_fq(fq_inv(ld_fq(a)), out); }
int zgt_fq_sqrt(const uint8_t* a, uint8_t* out) {
  Fq s;
  bool ok = fq_sqrt(ld_fq(a), &s);
  st_fq(s, out);
  return ok;
}
void zgt_fr_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) {
  Fr x = fr_to_mont(fr_limbs_from_le(a)), y = fr_to_mont(fr_limbs_from_le(b));
  Fr r = fr_from_mont(fr_mul(x, y));
  memcpy(out, r.l, 32);
}
// binary-GCD inverse on a plain residue (Fr: LE 32 bytes, Fq: BE 48 bytes)
void zgt_fr_inv_vt(const uint8_t* a, uint8_t* out) {
  Fr r = fp_inv_vt<FrM, ZG_INV_T_FR>(fr_limbs_from_le(a));
  memcpy(out, r.l, 32);
}
void zgt_fr_inv_vt_mont(const uint8_t* a, uint8_t* out) {
  Fr r = fr_from_mont(fr_inv_vt(fr_to_mont(fr_limbs_from_le(a))));
  memcpy(out, r.l, 32);
}
void zgt_fq_inv_vt(const uint8_t* a, uint8_t* out) { fq_limbs_to_be(fp_inv_vt<FqM, ZG_INV_T_FQ>(fq_limbs_from_be(a)), out); }
// BN254 (PGHR13): the device's codecs and pairing on the CPU; points canonical LE
static void st_bq(const Bq& a, uint8_t* o) {
  const Bq c = bq_from_mont(a);
  memcpy(o, c.l, 32);
}
static Bq ld_bq(const uint8_t* b) {
  Bq x;
  memcpy(x.l, b, 32);
  return bq_to_mont(x);
}
// BN254 G2 membership of the twist point with x = (x0, x1) and the chosen square root of the curve
// equation (32-byte LE canonical coordinates): res[0] = psi(Q) == [6u^2] Q (the product's
// ba2_in_subgroup), res[1] = [r] Q == O (AffineG2::new); returns 0 if x is not on the twist
int zgt_bn_g2_membership(const uint8_t* x0, const uint8_t* x1, const uint8_t* y0, const uint8_t* y1, int* res) {
  const BA2 q = {{ld_bq(x0), ld_bq(x1)}, {ld_bq(y0), ld_bq(y1)}};
  if (!ba2_on_curve(q)) return 0;
  res[0] = ba2_in_subgroup(q);
  res[1] = ba2_in_subgroup_r(q);
  return 1;
}

// BN254 G1 GLV: res[0] = [a + b lambda] q (bj1_mul_glv, k = a || b as 16 LE bytes) equals [s] q for
// the 32-byte LE scalar s; res[1] = phi(q) equals [lambda] q (BN_LAMBDA)
int zgt_bn_glv_check(const uint8_t* qx, const uint8_t* qy, const uint8_t* k, const uint8_t* s, int* res) {
  const BA1 q = {ld_bq(qx), ld_bq(qy), false};
  if (!ba1_on_curve(q)) return 0;
  uint32_t kw[4], sw[8];
  for (int l = 0; l < 4; l++) kw[l] = (uint32_t)k[4 * l] | ((uint32_t)k[4 * l + 1] << 8) | ((uint32_t)k[4 * l + 2] << 16) | ((uint32_t)k[4 * l + 3] << 24);
  for (int l = 0; l < 8; l++) sw[l] = (uint32_t)s[4 * l] | ((uint32_t)s[4 * l + 1] << 8) | ((uint32_t)s[4 * l + 2] << 16) | ((uint32_t)s[4 * l + 3] << 24);
  auto eq = [](const BA1& a, const BA1& b) { return a.inf == b.inf && (a.inf || (bq_eq(a.x, b.x) && bq_eq(a.y, b.y))); };
  res[0] = eq(bj1_to_aff(bj1_mul_glv(q, kw)), bj1_to_aff(bj1_mul(q, sw, 256)));
  res[1] = eq(ba1_phi(q), bj1_to_aff(bj1_mul(q, BN_LAMBDA, 256)));
  return 1;
}

int zgt_bn_g1_decode(const uint8_t* in, uint8_t* out) {
  BA1 p;
  if (!bn_g1_decode(in, &p)) return 0;
  st_bq(p.x, out);
  st_bq(p.y, out + 32);
  return 1;
}
int zgt_bn_g2_decode(const uint8_t* in, uint8_t* out) {
  BA2 q;
  if (!bn_g2_decode(in, &q)) return 0;
  st_bq(q.x.c0, out);
  st_bq(q.x.c1, out + 32);
  st_bq(q.y.c0, out + 64);
  st_bq(q.y.c1, out + 96);
  return 1;
}
void zgt_bn_pairing(const uint8_t* g1, const uint8_t* g2, uint8_t* gt) {
  const BA1 p = {ld_bq(g1), ld_bq(g1 + 32), false};
  const BA2 q = {{ld_bq(g2), ld_bq(g2 + 32)}, {ld_bq(g2 + 64), ld_bq(g2 + 96)}};
  const Bq12 f = bn_final_exp(bn_miller_single(p, q));
  const Bq2 cs[6] = {f.c0.c0, f.c1.c0, f.c0.c1, f.c1.c1, f.c0.c2, f.c1.c2};
  for (int k = 0; k < 6; k++) {
    st_bq(cs[k].c0, gt + 64 * k);
    st_bq(cs[k].c1, gt + 64 * k + 32);
  }
}
void zgt_f12_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) {
  f12_to_bytes(f12_mul(f12_from_bytes(a), f12_from_bytes(b)), out);
}
void zgt_f12_sqr(const uint8_t* a, uint8_t* out) { f12_to_bytes(f12_sqr(f12_from_bytes(a)), out); }
void zgt_f12_inv(const uint8_t* a, uint8_t* out) { f12_to_bytes(f12_inv(f12_from_bytes(a)), out); }
void zgt_f12_frob(const uint8_t* a, int k, uint8_t* out) { f12_to_bytes(f12_frob(f12_from_bytes(a), k), out); }
void zgt_final_exp(const uint8_t* a, uint8_t* out) { f12_to_bytes(final_exponentiation(f12_from_bytes(a)), out); }
int zgt_f2_sqrt(const uint8_t* a, uint8_t* out) {
  Fq2 x = {ld_fq(a), ld_fq(a + 48)}, s;
  bool ok = f2_sqrt(x, &s);
  st_fq(s.c0, out);
  st_fq(s.c1, out + 48);
  return ok;
}

// decode: returns DEC_* ; writes affine x||y (canonical BE)
int zgt_g1_decompress(const uint8_t* b, uint8_t* out) {
  G1A p;
  int r = g1_decompress(b, &p);
  if (r == DEC_OK) {
    st_fq(p.x, out);
    st_fq(p.y, out + 48);
  }
  return r;
}
int zgt_g2_decompress(const uint8_t* b, uint8_t* out) {
  G2A p;
  int r = g2_decompress(b, &p);
  if (r == DEC_OK) {
    st_fq(p.x.c0, out);
    st_fq(p.x.c1, out + 48);
    st_fq(p.y.c0, out + 96);
    st_fq(p.y.c1, out + 144);
  }
  return r;
}
// [r] P with the batch-scalar GLV path (r from 16 bytes, zg_groth16.h); affine x || y out
void zgt_g1_glv_mul(const uint8_t* xy, const uint8_t* r16, uint8_t* out) {
  uint64_t a, b;
  batch_scalar_ab(r16, &a, &b);
  G1A r = jac_to_aff(g1_glv_mul({ld_fq(xy), ld_fq(xy + 48), false}, a, b));
  st_fq(r.x, out);
  st_fq(r.y, out + 48);
}
// the batch scalar as a canonical little-endian Fr
void zgt_batch_scalar(const uint8_t* r16, uint8_t* out) {
  uint64_t a, b;
  batch_scalar_ab(r16, &a, &b);
  Fr v = fr_from_mont(batch_scalar_fr(a, b));
  memcpy(out, v.l, 32);
}
int zgt_g1_in_subgroup(const uint8_t* xy) { return g1_in_subgroup({ld_fq(xy), ld_fq(xy + 48), false}); }
int zgt_g2_in_subgroup(const uint8_t* xy) {
  return g2_in_subgroup({{ld_fq(xy), ld_fq(xy + 48)}, {ld_fq(xy + 96), ld_fq(xy + 144)}, false});
}

// miller loop of affine P (x||y) and Q (x0||x1||y0||y1), conjugated
void zgt_miller(const uint8_t* p, const uint8_t* q, uint8_t* out) {
  G1A P = {ld_fq(p), ld_fq(p + 48), false};
  G2A Q = {{ld_fq(q), ld_fq(q + 48)}, {ld_fq(q + 96), ld_fq(q + 144)}, false};
  f12_to_bytes(miller_loop_1(P, Q), out);
}

// prepare a VK from raw uncompressed bytes; returns vk_prepare code; alpha_beta out
static DevVK g_vk;
int zgt_vk_prepare(const uint8_t* raw_fields /*96+96+192+192+96+192*/, int n_ic, const uint8_t* ic, uint8_t* ab) {
  RawVK raw;
  const uint8_t* p = raw_fields;
  memcpy(raw.alpha_g1, p, 96); p += 96;
  memcpy(raw.beta_g1, p, 96); p += 96;
  memcpy(raw.beta_g2, p, 192); p += 192;
  memcpy(raw.gamma_g2, p, 192); p += 192;
  memcpy(raw.delta_g1, p, 96); p += 96;
  memcpy(raw.delta_g2, p, 192);
  raw.n_ic = n_ic;
  for (int i = 0; i < n_ic; i++) memcpy(raw.ic[i], ic + 96 * i, 96);
  int r = vk_prepare(raw, &g_vk, nullptr);
  if (r == 0) f12_to_bytes(g_vk.alpha_beta, ab);
  return r;
}
int zgt_verify_single(const uint8_t* proof, const uint8_t* inputs, int k, uint8_t* gt) {
  Fq12 g;
  uint8_t st = verify_single(g_vk, proof, inputs, k, &g);
  if (st == ST_OK || st == ST_VERIFY_FAILED) f12_to_bytes(g, gt);
  return st;
}

// lazy linear form of the cooperative engine: sum_t c_t x_t mod p for raw 384-bit limbs x_t
// (little-endian 32-bit words, 12 per value); returns the result's limbs
void zgt_lazy_form(const uint32_t* xs, const int* cs, int n, int canon, uint32_t* out) {
  LazyAcc a;
  lazy_zero(a);
  for (int t = 0; t < n; t++) {
    Fq x;
    for (int i = 0; i < 12; i++) x.l[i] = xs[12 * t + i];
    lazy_term(a, x, cs[t]);
  }
  Fq r = lazy_finish(a, canon != 0);
  for (int i = 0; i < 12; i++) out[i] = r.l[i];
}

}  // extern "C"
