// zg_jubjub.h -- Jubjub and RedJubjub on gfx950: the Sapling signature
// checks that sit next to the Groth16 proofs in accept_sapling, batched on the GPU.
//
//   edwards::Point::read + is_small_order   verification/src/sapling.rs:108-128,177-189,280-292
//   redjubjub::PublicKey::verify             sapling.rs:131-137 (spend_auth_sig, generator
//                                            SpendingKeyGenerator, message rk || sighash) and
//                                            :216-244 (binding_sig, ValueCommitmentRandomness,
//                                            message bvk || sighash)
//   binding verification key                 sapling.rs:82-94,216-226,247-269: sum cv(spends)
//                                            - sum cv(outputs) - [valueBalance] G_v
// (sapling-crypto @21084bde, not vendored; restated in oracle/sapling_sig.py, which the
// reference's real transactions pin.)
//
// Jubjub is the a = -1 twisted Edwards curve -x^2 + y^2 = 1 + d x^2 y^2 over Fr (the BLS12-381
// scalar field); d is a non-square, so the extended-coordinate addition law used here
// (add-2008-hwcd, dbl-2008-hwcd) is complete. Scalars live in Fs = Z / r_J.
// RedJubjub verify (sapling-crypto redjubjub.rs): c = BLAKE2b-512("Zcash_RedJubjubH",
// Rbar || M) mod r_J; Rbar must decode, Sbar < r_J; valid iff [8](-[S] P_G + R + [c] vk) = O.
// [S] P_G uses fixed-base comb tables of the generators (8-bit digits, 32 mixed additions);
// [c] vk is a 252-bit double-and-add.
#pragma once
#include "zg_prep.h"

namespace zg {

struct FsM {
  static constexpr int N = 8;
  static constexpr uint32_t INV = FS_INV;
  ZG_INL static uint32_t p(int i) { return FS_R[i]; }
};
using Fs = Fp<FsM>;

#define ZG_JJ_GENS 3  // 0 SpendingKeyGenerator, 1 ValueCommitmentRandomness, 2 ValueCommitmentValue
#define ZG_JJ_COMB_W 32
#define ZG_JJ_COMB_D 255
#define ZG_JJ_COMB_WORDS 16  // x, y Montgomery Fr limbs
#define ZG_JJ_COMB_POINTS (ZG_JJ_GENS * ZG_JJ_COMB_W * ZG_JJ_COMB_D)

struct JExt {
  Fr X, Y, Z, T;  // x = X / Z, y = Y / Z, x y = T / Z
};

ZG_INL Fr jj_const(const uint32_t* c) {
  Fr r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = c[i];
  return r;
}
ZG_INL JExt jx_zero() { return {fp_zero<FrM>(), fr_one(), fr_one(), fp_zero<FrM>()}; }
ZG_INL JExt jx_from_aff(const Fr& x, const Fr& y) { return {x, y, fr_one(), fr_mul(x, y)}; }
ZG_INL JExt jx_neg(const JExt& p) { return {fp_neg<FrM>(p.X), p.Y, p.Z, fp_neg<FrM>(p.T)}; }

// add-2008-hwcd with a = -1 (H = B + A): complete on Jubjub
ZG_INL JExt jx_add(const JExt& p, const JExt& q) {
  const Fr A = fr_mul(p.X, q.X);
  const Fr B = fr_mul(p.Y, q.Y);
  const Fr C = fr_mul(fr_mul(p.T, q.T), jj_const(JUBJUB_D));
  const Fr D = fr_mul(p.Z, q.Z);
  const Fr E = fp_sub<FrM>(fp_sub<FrM>(fr_mul(fr_add(p.X, p.Y), fr_add(q.X, q.Y)), A), B);
  const Fr F = fp_sub<FrM>(D, C), G = fr_add(D, C), H = fr_add(B, A);
  return {fr_mul(E, F), fr_mul(G, H), fr_mul(F, G), fr_mul(E, H)};
}
// mixed: q affine (x, y), T2 = x y
ZG_INL JExt jx_add_aff(const JExt& p, const Fr& x, const Fr& y) {
  const Fr A = fr_mul(p.X, x);
  const Fr B = fr_mul(p.Y, y);
  const Fr C = fr_mul(fr_mul(p.T, fr_mul(x, y)), jj_const(JUBJUB_D));
  const Fr D = p.Z;
  const Fr E = fp_sub<FrM>(fp_sub<FrM>(fr_mul(fr_add(p.X, p.Y), fr_add(x, y)), A), B);
  const Fr F = fp_sub<FrM>(D, C), G = fr_add(D, C), H = fr_add(B, A);
  return {fr_mul(E, F), fr_mul(G, H), fr_mul(F, G), fr_mul(E, H)};
}
// dbl-2008-hwcd with a = -1
ZG_INL JExt jx_dbl(const JExt& p) {
  const Fr A = fr_mul(p.X, p.X);
  const Fr B = fr_mul(p.Y, p.Y);
  const Fr Z2 = fr_mul(p.Z, p.Z);
  const Fr C = fr_add(Z2, Z2);
  const Fr D = fp_neg<FrM>(A);
  const Fr E = fp_sub<FrM>(fp_sub<FrM>(fr_mul(fr_add(p.X, p.Y), fr_add(p.X, p.Y)), A), B);
  const Fr G = fr_add(D, B), F = fp_sub<FrM>(G, C), H = fp_sub<FrM>(D, B);
  return {fr_mul(E, F), fr_mul(G, H), fr_mul(F, G), fr_mul(E, H)};
}
ZG_INL bool jx_is_zero(const JExt& p) { return fp_is_zero<FrM>(p.X) && fp_eq<FrM>(p.Y, p.Z); }

// [k] p, k little-endian 32-bit limbs (canonical), nbits from the top
ZG_INL JExt jx_mul(const JExt& p, const uint32_t* k, int nbits) {
  JExt acc = jx_zero();
  for (int i = nbits - 1; i >= 0; i--) {
    acc = jx_dbl(acc);
    if ((k[i >> 5] >> (i & 31)) & 1u) acc = jx_add(acc, p);
  }
  return acc;
}

ZG_INL void jx_to_aff(const JExt& p, Fr* x, Fr* y) {
  const Fr zi = prep_fr_inv(p.Z);
  *x = fr_mul(p.X, zi);
  *y = fr_mul(p.Y, zi);
}

// edwards::Point::write: y (canonical, LE) with x's parity in bit 255
ZG_INL void jj_write(const Fr& x, const Fr& y, uint8_t* out) {
  const Fr xc = fr_from_mont(x), yc = fr_from_mont(y);
  for (int i = 0; i < 8; i++)
    for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(yc.l[i] >> (8 * k));
  out[31] |= (uint8_t)((xc.l[0] & 1u) << 7);
}

// the comb table point d * 2^(8 w) * G_gen
ZG_INL void jj_comb_point(const uint32_t* comb, int gen, int w, int d, Fr* x, Fr* y) {
  const uint32_t* e = comb + ((size_t)(gen * ZG_JJ_COMB_W + w) * ZG_JJ_COMB_D + (d - 1)) * ZG_JJ_COMB_WORDS;
#pragma unroll
  for (int l = 0; l < 8; l++) {
    x->l[l] = e[l];
    y->l[l] = e[8 + l];
  }
}
// [s] G_gen for a canonical scalar s (LE limbs, < 2^256): 32 byte-digit lookups
ZG_INL JExt jj_fixed_mul(const uint32_t* comb, int gen, const uint32_t* s) {
  JExt acc = jx_zero();
  for (int w = 0; w < ZG_JJ_COMB_W; w++) {
    const int d = (s[w >> 2] >> (8 * (w & 3))) & 0xff;
    if (!d) continue;
    Fr x, y;
    jj_comb_point(comb, gen, w, d, &x, &y);
    acc = jx_add_aff(acc, x, y);
  }
  return acc;
}

// ---- BLAKE2b-512 of at most 128 bytes with a 16-byte personalization (one compression)
__device__ __constant__ const uint8_t JJ_SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};
__device__ __constant__ const uint64_t JJ_IV[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                                                  0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                                                  0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
__device__ inline uint64_t jj_rotr(uint64_t x, int k) { return (x >> k) | (x << (64 - k)); }
// m: the message block as 16 LE words (zero-padded), len bytes of it; out: 8 LE words
__device__ inline void blake2b512_block(const uint64_t* m, int len, const char* personal, uint64_t* out) {
  uint64_t h[8], v[16];
  for (int i = 0; i < 8; i++) h[i] = JJ_IV[i];
  h[0] ^= 0x01010000ull ^ 64ull;
  for (int w = 0; w < 2; w++) {
    uint64_t p = 0;
    for (int b = 7; b >= 0; b--) p = (p << 8) | (uint8_t)personal[8 * w + b];
    h[6 + w] ^= p;
  }
  for (int i = 0; i < 8; i++) {
    v[i] = h[i];
    v[i + 8] = JJ_IV[i];
  }
  v[12] ^= (uint64_t)len;
  v[14] = ~v[14];
  for (int r = 0; r < 12; r++) {
    const uint8_t* s = JJ_SIGMA[r];
#define JJ_G(a, b, c, d, x, y)           \
  v[a] = v[a] + v[b] + (x);              \
  v[d] = jj_rotr(v[d] ^ v[a], 32);       \
  v[c] = v[c] + v[d];                    \
  v[b] = jj_rotr(v[b] ^ v[c], 24);       \
  v[a] = v[a] + v[b] + (y);              \
  v[d] = jj_rotr(v[d] ^ v[a], 16);       \
  v[c] = v[c] + v[d];                    \
  v[b] = jj_rotr(v[b] ^ v[c], 63);
    JJ_G(0, 4, 8, 12, m[s[0]], m[s[1]]);
    JJ_G(1, 5, 9, 13, m[s[2]], m[s[3]]);
    JJ_G(2, 6, 10, 14, m[s[4]], m[s[5]]);
    JJ_G(3, 7, 11, 15, m[s[6]], m[s[7]]);
    JJ_G(0, 5, 10, 15, m[s[8]], m[s[9]]);
    JJ_G(1, 6, 11, 12, m[s[10]], m[s[11]]);
    JJ_G(2, 7, 8, 13, m[s[12]], m[s[13]]);
    JJ_G(3, 4, 9, 14, m[s[14]], m[s[15]]);
#undef JJ_G
  }
  for (int i = 0; i < 8; i++) out[i] = h[i] ^ v[i] ^ v[i + 8];
}

// 512-bit LE value mod r_J, canonical: lo R^2 + hi R^3 (Montgomery, R = 2^256), then out
ZG_INL Fs fs_from_512(const uint64_t* h) {
  Fs lo, hi;
  for (int i = 0; i < 4; i++) {
    lo.l[2 * i] = (uint32_t)h[i];
    lo.l[2 * i + 1] = (uint32_t)(h[i] >> 32);
    hi.l[2 * i] = (uint32_t)h[4 + i];
    hi.l[2 * i + 1] = (uint32_t)(h[4 + i] >> 32);
  }
  Fs r2, r3, one;
  for (int i = 0; i < 8; i++) {
    r2.l[i] = FS_R2[i];
    r3.l[i] = FS_R3[i];
    one.l[i] = i == 0 ? 1u : 0u;
  }
  const Fs m = fp_add<FsM>(fp_mul_inl<FsM>(lo, r2), fp_mul_inl<FsM>(hi, r3));
  return fp_mul_inl<FsM>(m, one);
}

// edwards::Point::read from device memory (no local byte copy); false = Invalid
ZG_INL bool jj_read(const uint8_t* in, Fr* x, Fr* y) {
  Fr yc = fr_limbs_from_le(in);
  const bool sign = yc.l[7] >> 31;
  yc.l[7] &= 0x7fffffffu;
  if (!fp_lt_modulus<FrM>(yc)) return false;  // y is not in field
  const Fr ym = fr_to_mont(yc);
  const Fr y2 = fr_mul(ym, ym);
  const Fr num = fp_sub<FrM>(y2, fr_one());
  const Fr den = fr_add(fr_mul(jj_const(JUBJUB_D), y2), fr_one());
  Fr xm;
  if (!prep_fr_sqrt(fr_mul(num, prep_fr_inv(den)), &xm)) return false;  // not on curve
  if ((bool)(fr_from_mont(xm).l[0] & 1u) != sign) xm = fp_neg<FrM>(xm);
  *x = xm;
  *y = ym;
  return true;
}

// 8P == O
ZG_INL bool jj_small_order(const Fr& x, const Fr& y) {
  JExt p = jx_from_aff(x, y);
  p = jx_dbl(jx_dbl(jx_dbl(p)));
  return jx_is_zero(p);
}

}  // namespace zg
