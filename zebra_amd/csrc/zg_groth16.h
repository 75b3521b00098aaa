// zg_groth16.h -- bellman 0.1.0 groth16 semantics on gfx950 (per-thread building blocks).
//
//   Proof::<Bls12>::read   (called at verification/src/sapling.rs:158,203,
//                           crypto/src/groth16.rs:54)        -> proof_decode_point
//   prepare_verifying_key  (crypto/src/json/groth16.rs:14,21,27) -> vk_prepare
//   verify_proof           (verification/src/sapling.rs:162,207, sprout.rs:73-77)
//                                                            -> verify_single
// SURVEY.md 8(a) rows a1-a4, a8.
#pragma once
#include "zg_pairing.h"
#include "zg_fqd.h"

namespace zg {

enum : uint8_t {
  ST_OK = 0,
  ST_DECODE_INVALID = 1,
  ST_MALFORMED_VK = 2,
  ST_VERIFY_FAILED = 3,
  ST_INPUT_NONCANONICAL = 4,
  ST_PENDING = 255,
};

#define ZG_MAX_IC 10
#define ZG_MAX_INPUTS 9
#define ZG_NKINDS 3
#define ZG_SHIFTS 8  // lanes per VK-side scalar (4 byte-digits of the comb each)

// Fixed-base comb tables of the VK-side MSM (k_node_msm): for each base B (ic[0..9], alpha)
// the affine multiples d * 2^(8 w) * B, w = 0..31, d = 1..255, so a 255-bit scalar is the sum of
// its 32 byte-digits' table points -- 32 mixed additions split over ZG_SHIFTS = 8 lanes
// (4 each), no doublings. 33 bases x 8,160 points x 96 B = 25.8 MB per device: HBM is plentiful,
// the latency of every VK-side MSM (batch roots and bisection nodes) is what counts.
#define ZG_COMB_BASES (ZG_MAX_IC + 1)
#define ZG_COMB_W 32
#define ZG_COMB_D 255
#define ZG_COMB_WORDS 24  // x, y Montgomery limbs
#define ZG_COMB_POINTS (ZG_COMB_BASES * ZG_COMB_W * ZG_COMB_D)

// A prepared verifying key, resident in HBM.
struct DevVK {
  int loaded;
  int ic_len;
  G1A alpha;
  G2A beta, gamma, delta;
  G1A ic[ZG_MAX_IC];
  Fq12 alpha_beta;                 // alpha_g1_beta_g2 (final-exponentiated)
  Line neg_gamma_lines[ZG_NCOEFF]; // G2Prepared(-gamma)
  Line neg_delta_lines[ZG_NCOEFF]; // G2Prepared(-delta)
  Line beta_lines[ZG_NCOEFF];      // G2Prepared(beta)  (batch alpha/beta term)
  // comb tables of ic[0..9] and alpha (base 10), ZG_COMB_W x ZG_COMB_D points each, in a
  // per-device buffer shared by every context that loaded this key (k_vk_comb fills it)
  const uint32_t* comb;
};

// Raw uncompressed VK as uploaded by the host (crypto/src/json/groth16.rs:33-49 fields).
struct RawVK {
  uint8_t alpha_g1[96], beta_g1[96], beta_g2[192], gamma_g2[192], delta_g1[96], delta_g2[192];
  uint8_t ic[ZG_MAX_IC][96];
  int n_ic;
};

// prepare_verifying_key. Returns 0 on success, 1 + field index on a decode failure.
ZG_NOINL inline int vk_prepare(const RawVK& raw, DevVK* vk, const uint32_t* comb) {
  vk->comb = comb;
  G1A beta_g1, delta_g1;
  if (g1_decode_uncompressed(raw.alpha_g1, &vk->alpha) == DEC_ERR) return 1;
  if (g1_decode_uncompressed(raw.beta_g1, &beta_g1) == DEC_ERR) return 2;
  if (g2_decode_uncompressed(raw.beta_g2, &vk->beta) == DEC_ERR) return 3;
  if (g2_decode_uncompressed(raw.gamma_g2, &vk->gamma) == DEC_ERR) return 4;
  if (g1_decode_uncompressed(raw.delta_g1, &delta_g1) == DEC_ERR) return 5;
  if (g2_decode_uncompressed(raw.delta_g2, &vk->delta) == DEC_ERR) return 6;
  for (int i = 0; i < raw.n_ic; i++)
    if (g1_decode_uncompressed(raw.ic[i], &vk->ic[i]) == DEC_ERR) return 7 + i;
  vk->ic_len = raw.n_ic;
  // E::pairing(alpha, beta): miller_loop skips infinity pairs -> f = 1 -> FE(1) = 1
  if (!vk->alpha.inf && !vk->beta.inf)
    vk->alpha_beta = final_exponentiation(miller_loop_1(vk->alpha, vk->beta));
  else
    vk->alpha_beta = f12_one();
  G2A ng = vk->gamma, nd = vk->delta;
  ng.y = f2_neg(ng.y);
  nd.y = f2_neg(nd.y);
  if (!ng.inf) g2_prepare(ng, vk->neg_gamma_lines);
  if (!nd.inf) g2_prepare(nd, vk->neg_delta_lines);
  if (!vk->beta.inf) g2_prepare(vk->beta, vk->beta_lines);
  vk->loaded = 1;
  return 0;
}

// ---- batch scalars: 16 bytes per proof = two little-endian u64 (a, b),
//   r_i = k0 + k1 lambda mod r,  k0 = 2a + 1 (odd, < 2^65),  k1 = b,  lambda = -x^2 mod r.
// The map is injective (k0 < x^2) and hits 2^128 distinct non-zero scalars, so a batch with
// an invalid proof passes with probability <= 2^-128. sigma(x, y) = (beta x, y) acts as
// [lambda] on G1, so r_i P = k0 P + k1 sigma(P) (GLV), evaluated with the sign-aligned column
// recoding of Faz-Hernandez, Longa and Sanchez (2013): column j adds s_j (P + e_j sigma(P)),
// s_j = +-1, e_j in {0, 1}, and P + sigma(P) = -sigma^2(P) = (beta^2 x, -y) is affine, so every
// one of the 65 columns is one doubling and one mixed addition of a table point selected
// branch-free per lane (vs 128 doublings + 128 lane-divergent additions for a 128-bit scalar).
ZG_INL void batch_scalar_ab(const uint8_t* r16, uint64_t* a, uint64_t* b) {
  uint64_t x = 0, y = 0;
  for (int k = 7; k >= 0; k--) {
    x = (x << 8) | r16[k];
    y = (y << 8) | r16[8 + k];
  }
  *a = x;
  *b = y;
}
// r_i as a Montgomery Fr
ZG_INL Fr batch_scalar_fr(uint64_t a, uint64_t b) {
  Fr k0 = fp_zero<FrM>(), k1 = fp_zero<FrM>(), lam;
  const uint64_t lo = (a << 1) | 1u, hi = a >> 63;  // 2a + 1
  k0.l[0] = (uint32_t)lo;
  k0.l[1] = (uint32_t)(lo >> 32);
  k0.l[2] = (uint32_t)hi;
  k1.l[0] = (uint32_t)b;
  k1.l[1] = (uint32_t)(b >> 32);
  for (int i = 0; i < 8; i++) lam.l[i] = FR_LAMBDA[i];
  return fr_add(fr_to_mont(k0), fr_mul(fr_to_mont(k1), lam));
}
// [k0 + k1 lambda] p for p in G1 (affine, finite), k0 = 2a + 1, k1 = b
ZG_NOINL inline void g1_glv_mul_p(G1J* out, const G1A* pp, uint64_t a, uint64_t b) {
  const G1A p = *pp;
  const Fq bx = fq_mul(p.x, fq_const(G1_BETA2)), ny = fq_neg(p.y);
  // sign-aligned recoding of k1 against the digits s_j = a_j ? +1 : -1 (j < 64), s_64 = +1
  uint64_t k1 = b, e = 0;
  for (int j = 0; j < 64; j++) {
    const uint64_t ej = k1 & 1u, neg = ((a >> j) & 1u) ^ 1u;
    e |= ej << j;
    k1 = (k1 >> 1) + (ej & neg);
  }
  const bool etop = k1 & 1u;  // k1 is 0 or 1 here
  G1J q = {etop ? bx : p.x, etop ? ny : p.y, fq_one()};
  // dbl + madd inlined: the Jacobian state stays in registers across the out-of-line fq_mul
  // leaf calls (passing it by pointer to noinline point ops sent it through scratch)
  for (int j = 63; j >= 0; j--) {
    const bool ej = (e >> j) & 1u, neg = !((a >> j) & 1u);
    const G1A t = {ej ? bx : p.x, (ej != neg) ? ny : p.y, false};
    q = jac_add_aff_inl(jac_dbl_inl(q), t);
  }
  *out = q;
}
ZG_INL G1J g1_glv_mul(const G1A& p, uint64_t a, uint64_t b) {
  G1J r;
  g1_glv_mul_p(&r, &p, a, b);
  return r;
}
// the same product with the 64 doublings and mixed additions in lazy digits (zg_fqd.h)
ZG_DEC_INL inline void g1_glv_mul_d_p(G1J* out, const G1A* pp, uint64_t a, uint64_t b) {
  const FqD px = fqd_from(pp->x), py = fqd_from(pp->y);
  const FqD bx = fqd_mul(px, fqd_from(fq_const(G1_BETA2))), ny = fqd_neg2(py);  // < 2p, < 3p
  uint64_t k1 = b, e = 0;
  for (int j = 0; j < 64; j++) {
    const uint64_t ej = k1 & 1u, neg = ((a >> j) & 1u) ^ 1u;
    e |= ej << j;
    k1 = (k1 >> 1) + (ej & neg);
  }
  const bool etop = k1 & 1u;
  G1D q = g1d_from_aff(etop ? bx : px, etop ? ny : py);
  for (int j = 63; j >= 0; j--) {
    const bool ej = (e >> j) & 1u, neg = !((a >> j) & 1u);
    q = g1d_add_aff(g1d_dbl(q), ej ? bx : px, (ej != neg) ? ny : py);
  }
  *out = g1d_to_jac(q);
}
ZG_INL G1J g1_glv_mul_d(const G1A& p, uint64_t a, uint64_t b) {
  G1J r;
  g1_glv_mul_d_p(&r, &p, a, b);
  return r;
}
// The same product two columns at a time: q = 4q + s_j E(e_j, e_{j-1}, s_j s_{j-1}) with
// E = 2 (P + e_j sigma P) + r (P + e_{j-1} sigma P), r = +-1 -- eight affine entries built once
// (one doubling, five mixed additions, one batched inversion; sigma(X, Y, Z) = (beta X, Y, Z) and
// 3P + 3 sigma P = -sigma^2(3P) come free), then 64 doublings and 32 mixed additions instead of
// 64 + 64. The table is indexed per lane (private memory): 8 x 2 FqD.
ZG_NOINL inline void g1_glv_mul_w2_p(G1J* out, const G1A* pp, uint64_t a, uint64_t b) {
  const FqD px = fqd_from(pp->x), py = fqd_from(pp->y);
  const FqD be = fqd_from(fq_const(G1_BETA)), be2 = fqd_from(fq_const(G1_BETA2));
  const FqD sx = fqd_mul(px, be), s2x = fqd_mul(px, be2), ny = fqd_neg2(py);  // sigma P x, sigma^2 P x, -y
  const G1D P1 = g1d_from_aff(px, py);
  const G1D P2 = g1d_dbl(P1);
  G1D J[5];
  J[0] = g1d_add_aff(P2, px, py);                              // 3P
  J[1] = g1d_add_aff(J[0], sx, py);                            // 3P + sigma P
  J[2] = g1d_add_aff(J[1], sx, py);                            // 3P + 2 sigma P
  J[3] = g1d_add_aff(P1, sx, ny);                              // P - sigma P
  J[4] = g1d_add_aff(G1D{fqd_mul(P2.x, be), P2.y, P2.z}, px, py);  // sigma(2P) + P
  // batched inversion of the five Z (Montgomery's trick; an infinite entry only for a point outside
  // G1, whose product is discarded by k_decode_finish)
  FqD c[5];
  c[0] = J[0].z;
  for (int k = 1; k < 5; k++) c[k] = fqd_mul(c[k - 1], J[k].z);
  FqD inv = fqd_from(fq_inv(fqd_to(c[4])));
  FqD tx[8], ty[8];
  for (int k = 4; k >= 0; k--) {
    const FqD zi = k ? fqd_mul(inv, c[k - 1]) : inv;
    if (k) inv = fqd_mul(inv, J[k].z);
    const FqD zi2 = fqd_sqr(zi);
    const FqD x = fqd_mul(J[k].x, zi2), y = fqd_mul(J[k].y, fqd_mul(zi2, zi));
    // entry index (e_j << 2) | (e_{j-1} << 1) | (r == -1)
    const int idx = k == 0 ? 0 : k == 1 ? 2 : k == 2 ? 4 : k == 3 ? 3 : 5;
    tx[idx] = x;
    ty[idx] = y;
    if (k == 0) {  // 3P + 3 sigma P = -sigma^2(3P)
      tx[6] = fqd_mul(x, be2);
      ty[6] = fqd_neg2(y);
    }
  }
  tx[1] = px;   // P
  ty[1] = py;
  tx[7] = s2x;  // P + sigma P = (beta^2 x, -y)
  ty[7] = ny;
  // the sign-aligned recoding of g1_glv_mul_d_p: k0 = 2a + 1 = sum s_j 2^j, s_j = +-1 (s_64 = +1)
  uint64_t k1 = b, e = 0;
  for (int j = 0; j < 64; j++) {
    const uint64_t ej = k1 & 1u, neg = ((a >> j) & 1u) ^ 1u;
    e |= ej << j;
    k1 = (k1 >> 1) + (ej & neg);
  }
  const bool etop = k1 & 1u;
  G1D q = g1d_from_aff(etop ? s2x : px, etop ? ny : py);
  for (int jj = 31; jj >= 0; jj--) {
    const int j = 2 * jj + 1;
    const uint32_t ej = (e >> j) & 1u, el = (e >> (j - 1)) & 1u;
    const uint32_t sj = (a >> j) & 1u, sl = (a >> (j - 1)) & 1u;  // 1: s = +1
    const int idx = (int)((ej << 2) | (el << 1) | (sj ^ sl));
    const FqD y = ty[idx];
    q = g1d_add_aff(g1d_dbl(g1d_dbl(q)), tx[idx], sj ? y : fqd_sub<4, 0, 1>(fqd_zero(), y));  // -y < 4p
  }
  *out = g1d_to_jac(q);
}
ZG_INL G1J g1_glv_mul_w2(const G1A& p, uint64_t a, uint64_t b) {
  G1J r;
  g1_glv_mul_w2_p(&r, &p, a, b);
  return r;
}

// Decode A || B || C (192 B) with bellman's rules: every point subgroup-checked and the
// point at infinity rejected. Returns true on success.
ZG_INL bool proof_decode(const uint8_t* pb, G1A* a, G2A* b, G1A* c) {
  if (g1_decompress(pb, a) != DEC_OK) return false;
  if (g2_decompress(pb + 48, b) != DEC_OK) return false;
  if (g1_decompress(pb + 144, c) != DEC_OK) return false;
  return true;
}

// 32-byte LE inputs -> canonical Fr limbs; false if any is >= r
ZG_INL bool inputs_canonical(const uint8_t* in, int k, Fr* x) {
  bool ok = true;
  for (int j = 0; j < k; j++) {
    x[j] = fr_limbs_from_le(in + 32 * j);
    ok = ok && fp_lt_modulus<FrM>(x[j]);
  }
  return ok;
}

// acc = ic[0] + sum_j x_j ic[j+1]  (bellman verify_proof; canonical scalars)
ZG_NOINL inline G1J compute_acc(const DevVK& vk, const Fr* x, int k) {
  G1J acc = jac_from_aff(vk.ic[0]);
  for (int j = 0; j < k; j++) acc = jac_add(acc, jac_mul_limbs(vk.ic[j + 1], x[j].l, 255));
  return acc;
}

// bellman verify_proof for one proof: status and the final-exponentiated left-hand side
// final_exponentiation(miller_loop([(A, B), (acc, -gamma), (C, -delta)])).
ZG_NOINL inline uint8_t verify_single(const DevVK& vk, const uint8_t* pb, const uint8_t* in, int k, Fq12* gt) {
  Fr x[ZG_MAX_INPUTS];
  if (!inputs_canonical(in, k, x)) return ST_INPUT_NONCANONICAL;
  G1A a, c;
  G2A b;
  if (!proof_decode(pb, &a, &b, &c)) return ST_DECODE_INVALID;
  if (k + 1 != vk.ic_len) return ST_MALFORMED_VK;
  G1A acc = jac_to_aff(compute_acc(vk, x, k));
  Fq12 f = miller_loop_1(a, b);
  if (!acc.inf && !vk.gamma.inf) f = f12_mul(f, miller_loop_prepared(acc, vk.neg_gamma_lines));
  if (!vk.delta.inf) f = f12_mul(f, miller_loop_prepared(c, vk.neg_delta_lines));
  *gt = final_exponentiation(f);
  return f12_eq(*gt, vk.alpha_beta) ? ST_OK : ST_VERIFY_FAILED;
}

}  // namespace zg
