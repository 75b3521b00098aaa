// zg_prep.h -- host-side public-input preparation of the Groth16 checks (SURVEY.md 8(a)
// rows a5-a7), in C++ over the same Fr arithmetic as the device code (zg_field.h, host path):
//
//   accept_spend   verification/src/sapling.rs:101-155  -> zg_prep_spend   (7 Fr)
//   accept_output  verification/src/sapling.rs:171-200  -> zg_prep_output  (5 Fr)
//   sprout::verify verification/src/sprout.rs:16-153    -> zg_prep_joinsplit (9 Fr), zg_hsig
//
// Jubjub (sapling-crypto @21084bde `edwards::Point::read`, not vendored; call sites
// sapling.rs:108-128,177-189) is the a = -1 twisted Edwards curve -x^2 + y^2 = 1 + d x^2 y^2
// over Fr of BLS12-381: a point is 32 bytes, little-endian y with the sign of x in bit 255;
// y >= r is invalid, x = sqrt((y^2 - 1) / (d y^2 + 1)) must exist, and x is negated when its
// parity differs from the sign bit. The small-order test is 8P == identity (sapling.rs:290-292).
// The RedJubjub signatures checked between these steps in the reference (sapling.rs:131-137)
// are not Groth16 and stay with the caller.
#pragma once
#include <string.h>

#include "zg_blake2b.h"
#include "zg_field.h"

namespace zg {

// error classes, in the reference's check order
enum : int {
  PREP_OK = 0,
  PREP_VALUE_COMMITMENT_INVALID = 1,     // SpendError/OutputError::ValueCommitment(Invalid)
  PREP_VALUE_COMMITMENT_SMALL_ORDER = 2, // ...::ValueCommitment(SmallOrder)
  PREP_ANCHOR = 3,                       // SpendError::Anchor (not in field)
  PREP_RANDOMIZED_KEY_INVALID = 4,       // SpendError::RandomizedKey(Invalid)
  PREP_RANDOMIZED_KEY_SMALL_ORDER = 5,   // SpendError::RandomizedKey(SmallOrder)
  PREP_NOTE_COMMITMENT = 6,              // OutputError::NoteCommitment (not in field)
  PREP_EPHEMERAL_KEY_INVALID = 7,        // OutputError::EphemeralKey(Invalid)
  PREP_EPHEMERAL_KEY_SMALL_ORDER = 8,    // OutputError::EphemeralKey(SmallOrder)
};

// ---- Fr helpers (host; Montgomery form unless noted)
ZG_HD inline Fr prep_fr_const(const uint32_t* c) {
  Fr r;
  for (int i = 0; i < 8; i++) r.l[i] = c[i];
  return r;
}
#if defined(__HIP_DEVICE_COMPILE__)
ZG_HD inline Fr prep_fr_mul(const Fr& a, const Fr& b) { return fr_mul(a, b); }
#else
// the host's product: 4 x 64-bit CIOS over unsigned __int128, the same Montgomery form (R = 2^256) and
// the same canonical result as fr_mul's 8 x 32-bit words -- ~10x faster on the host, where a window's
// descriptions are prepared (two Jubjub decodes per Sapling description, ~1,100 products each)
inline Fr prep_fr_mul(const Fr& a, const Fr& b) {
  static constexpr uint64_t M[4] = {0xffffffff00000001ull, 0x53bda402fffe5bfeull, 0x3339d80809a1d805ull,
                                    0x73eda753299d7d48ull};
  static constexpr uint64_t INV = 0xfffffffeffffffffull;  // -r^-1 mod 2^64
  typedef unsigned __int128 u128;
  uint64_t x[4], y[4], t[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    x[i] = a.l[2 * i] | (uint64_t)a.l[2 * i + 1] << 32;
    y[i] = b.l[2 * i] | (uint64_t)b.l[2 * i + 1] << 32;
  }
  for (int i = 0; i < 4; i++) {
    uint64_t c = 0;
    for (int j = 0; j < 4; j++) {
      const u128 p = (u128)x[j] * y[i] + t[j] + c;
      t[j] = (uint64_t)p;
      c = (uint64_t)(p >> 64);
    }
    u128 s = (u128)t[4] + c;
    t[4] = (uint64_t)s;
    const uint64_t t5 = (uint64_t)(s >> 64);
    const uint64_t m = t[0] * INV;
    u128 p = (u128)m * M[0] + t[0];
    c = (uint64_t)(p >> 64);
    for (int j = 1; j < 4; j++) {
      p = (u128)m * M[j] + t[j] + c;
      t[j - 1] = (uint64_t)p;
      c = (uint64_t)(p >> 64);
    }
    s = (u128)t[4] + c;
    t[3] = (uint64_t)s;
    t[4] = t5 + (uint64_t)(s >> 64);
  }
  // t < 2r: one conditional subtraction
  uint64_t d[4], bw = 0;
  for (int j = 0; j < 4; j++) {
    const u128 q = (u128)t[j] - M[j] - bw;
    d[j] = (uint64_t)q;
    bw = (uint64_t)(q >> 64) & 1u;
  }
  const bool ge = t[4] || !bw;
  Fr r;
  for (int i = 0; i < 4; i++) {
    const uint64_t v = ge ? d[i] : t[i];
    r.l[2 * i] = (uint32_t)v;
    r.l[2 * i + 1] = (uint32_t)(v >> 32);
  }
  return r;
}
#endif
ZG_HD inline Fr prep_fr_sqr(const Fr& a) { return prep_fr_mul(a, a); }
ZG_HD inline Fr prep_fr_sub(const Fr& a, const Fr& b) { return fp_sub<FrM>(a, b); }
ZG_HD inline Fr prep_fr_neg(const Fr& a) { return fp_neg<FrM>(a); }
ZG_HD inline bool prep_fr_eq(const Fr& a, const Fr& b) { return fp_eq<FrM>(a, b); }
ZG_HD inline Fr prep_fr_pow(const Fr& a, const uint32_t* e, int nbits) {
  Fr r = fr_one();
  for (int i = nbits - 1; i >= 0; i--) {
    r = prep_fr_sqr(r);
    if ((e[i >> 5] >> (i & 31)) & 1u) r = prep_fr_mul(r, a);
  }
  return r;
}
ZG_HD inline Fr prep_fr_inv(const Fr& a) { return prep_fr_pow(a, FR_EXP_INV, 255); }

// Tonelli-Shanks (r - 1 = 2^32 t); returns false for a non-residue (detected by the order search). Any root: the caller fixes
// the sign from the encoding.
ZG_HD inline bool prep_fr_sqrt(const Fr& a, Fr* out) {
  if (fp_is_zero<FrM>(a)) {
    *out = a;
    return true;
  }
  const Fr one = fr_one();
  Fr w = prep_fr_pow(a, FR_TS_TM1_2, 223);  // a^((t-1)/2)
  Fr x = prep_fr_mul(a, w);                      // a^((t+1)/2)
  Fr b = prep_fr_mul(x, w);                      // a^t
  Fr z = prep_fr_const(FR_TS_ROOT);
  int v = 32;
  while (!prep_fr_eq(b, one)) {
    int k = 0;
    Fr b2k = b;
    while (!prep_fr_eq(b2k, one)) {
      b2k = prep_fr_sqr(b2k);
      k++;
      // a non-residue: b = a^t has order exactly 2^32 (a^((r-1)/2) = -1), so the order search
      // reaches v = 32 on the first pass; a residue's never does (this replaces the Legendre
      // exponentiation the round-1 code ran first)
      if (k >= v) return false;
    }
    Fr ww = z;
    for (int j = 0; j < v - k - 1; j++) ww = prep_fr_sqr(ww);
    z = prep_fr_sqr(ww);
    b = prep_fr_mul(b, z);
    x = prep_fr_mul(x, ww);
    v = k;
  }
  *out = x;
  return true;
}

// 32 little-endian bytes -> canonical Fr limbs; false if >= r
ZG_HD inline bool prep_fr_from_repr(const uint8_t* b, Fr* canon) {
  *canon = fr_limbs_from_le(b);
  return fp_lt_modulus<FrM>(*canon);
}
ZG_HD inline void prep_fr_to_le(const Fr& canon, uint8_t* b) {
  for (int i = 0; i < 8; i++)
    for (int k = 0; k < 4; k++) b[4 * i + k] = (uint8_t)(canon.l[i] >> (8 * k));
}

struct JubjubPt {
  Fr x, y;  // affine, Montgomery
};

// edwards::Point::read; false = Invalid
ZG_HD inline bool jubjub_read(const uint8_t* in, JubjubPt* p) {
  uint8_t b[32];
  memcpy(b, in, 32);
  const bool sign = b[31] >> 7;
  b[31] &= 0x7f;
  Fr y;
  if (!prep_fr_from_repr(b, &y)) return false;  // y is not in field
  y = fr_to_mont(y);
  const Fr y2 = prep_fr_sqr(y);
  const Fr num = prep_fr_sub(y2, fr_one());
  const Fr den = fr_add(prep_fr_mul(prep_fr_const(JUBJUB_D), y2), fr_one());
  Fr x;
  if (!prep_fr_sqrt(prep_fr_mul(num, prep_fr_inv(den)), &x)) return false;  // not on curve
  const Fr xc = fr_from_mont(x);
  if ((bool)(xc.l[0] & 1u) != sign) x = prep_fr_neg(x);
  p->x = x;
  p->y = y;
  return true;
}

// 8P == identity, in projective (X : Y : Z) with dbl-2008-bbjlp (a = -1)
ZG_HD inline bool jubjub_is_small_order(const JubjubPt& p) {
  Fr X = p.x, Y = p.y, Z = fr_one();
  for (int r = 0; r < 3; r++) {
    const Fr B = prep_fr_sqr(fr_add(X, Y));
    const Fr C = prep_fr_sqr(X);
    const Fr D = prep_fr_sqr(Y);
    const Fr E = prep_fr_neg(C);
    const Fr F = fr_add(E, D);
    const Fr H = prep_fr_sqr(Z);
    const Fr J = prep_fr_sub(F, fr_add(H, H));
    X = prep_fr_mul(prep_fr_sub(prep_fr_sub(B, C), D), J);
    Y = prep_fr_mul(F, prep_fr_sub(E, D));
    Z = prep_fr_mul(F, J);
  }
  return fp_is_zero<FrM>(X) && prep_fr_eq(Y, Z);
}

// require_non_small_order_point: 0 ok, 1 invalid, 2 small order
ZG_HD inline int jubjub_read_checked(const uint8_t* b, JubjubPt* p) {
  if (!jubjub_read(b, p)) return 1;
  return jubjub_is_small_order(*p) ? 2 : 0;
}

ZG_HD inline void prep_put(uint8_t* out, int j, const Fr& mont) { prep_fr_to_le(fr_from_mont(mont), out + 32 * j); }

// multipack of a 32-byte LE value with CAPACITY 254 (sapling.rs:140-142): low 254 bits, then the top 2
ZG_HD inline void prep_multipack_nf(const uint8_t* nf, uint8_t* lo, uint8_t* hi) {
  memcpy(lo, nf, 32);
  lo[31] &= 0x3f;
  memset(hi, 0, 32);
  hi[0] = nf[31] >> 6;
}

// accept_spend public input [rk.x, rk.y, cv.x, cv.y, anchor, nf0, nf1]
ZG_HD inline int prep_spend(const uint8_t* cv, const uint8_t* anchor, const uint8_t* nf, const uint8_t* rk, uint8_t* out) {
  JubjubPt cvp, rkp;
  const int c = jubjub_read_checked(cv, &cvp);
  if (c == 1) return PREP_VALUE_COMMITMENT_INVALID;
  if (c == 2) return PREP_VALUE_COMMITMENT_SMALL_ORDER;
  Fr a;
  if (!prep_fr_from_repr(anchor, &a)) return PREP_ANCHOR;
  const int r = jubjub_read_checked(rk, &rkp);
  if (r == 1) return PREP_RANDOMIZED_KEY_INVALID;
  if (r == 2) return PREP_RANDOMIZED_KEY_SMALL_ORDER;
  prep_put(out, 0, rkp.x);
  prep_put(out, 1, rkp.y);
  prep_put(out, 2, cvp.x);
  prep_put(out, 3, cvp.y);
  prep_fr_to_le(a, out + 32 * 4);
  prep_multipack_nf(nf, out + 32 * 5, out + 32 * 6);
  return PREP_OK;
}

// accept_output public input [cv.x, cv.y, epk.x, epk.y, cmu]
ZG_HD inline int prep_output(const uint8_t* cv, const uint8_t* cmu, const uint8_t* epk, uint8_t* out) {
  JubjubPt cvp, ep;
  const int c = jubjub_read_checked(cv, &cvp);
  if (c == 1) return PREP_VALUE_COMMITMENT_INVALID;
  if (c == 2) return PREP_VALUE_COMMITMENT_SMALL_ORDER;
  Fr cm;
  if (!prep_fr_from_repr(cmu, &cm)) return PREP_NOTE_COMMITMENT;
  const int e = jubjub_read_checked(epk, &ep);
  if (e == 1) return PREP_EPHEMERAL_KEY_INVALID;
  if (e == 2) return PREP_EPHEMERAL_KEY_SMALL_ORDER;
  prep_put(out, 0, cvp.x);
  prep_put(out, 1, cvp.y);
  prep_put(out, 2, ep.x);
  prep_put(out, 3, ep.y);
  prep_fr_to_le(cm, out + 32 * 4);
  return PREP_OK;
}

// hSig = BLAKE2b-256(personal "ZcashComputehSig"; random_seed || nf0 || nf1 || pubkey)
inline void prep_hsig(const uint8_t* seed, const uint8_t* nf0, const uint8_t* nf1, const uint8_t* pubkey,
                      uint8_t* out) {
  static const uint8_t personal[16] = {'Z', 'c', 'a', 's', 'h', 'C', 'o', 'm', 'p', 'u', 't', 'e', 'h', 'S', 'i', 'g'};
  Blake2b h(32, personal);
  h.update(seed, 32);
  h.update(nf0, 32);
  h.update(nf1, 32);
  h.update(pubkey, 32);
  h.final(out);
}

// sprout.rs:42-58,86-153: the 2176-bit string (bytes MSB-first) of anchor, hSig, nf0, mac0,
// nf1, mac1, cm0, cm1, vpub_old (u64 LE), vpub_new (u64 LE), cut into `chunk`-bit pieces, each
// read with its first bit as the least significant -> 9 field elements (32 B LE). chunk = 254
// (bls::Fr::CAPACITY, into_bls_frs: the Groth16 branch) or 253 (into_bn_frs: the PHGR branch,
// sprout.rs:119-133); either way a piece is < 2^254 and below the field's modulus.
inline void prep_joinsplit_bits(const uint8_t* anchor, const uint8_t* seed, const uint8_t* nf0, const uint8_t* nf1,
                                const uint8_t* mac0, const uint8_t* mac1, const uint8_t* cm0, const uint8_t* cm1,
                                uint64_t vpub_old, uint64_t vpub_new, const uint8_t* pubkey, int chunk,
                                uint8_t* out) {
  uint8_t hsig[32], vo[8], vn[8];
  prep_hsig(seed, nf0, nf1, pubkey, hsig);
  for (int k = 0; k < 8; k++) {
    vo[k] = (uint8_t)(vpub_old >> (8 * k));
    vn[k] = (uint8_t)(vpub_new >> (8 * k));
  }
  const uint8_t* parts[10] = {anchor, hsig, nf0, mac0, nf1, mac1, cm0, cm1, vo, vn};
  const int lens[10] = {32, 32, 32, 32, 32, 32, 32, 32, 8, 8};
  memset(out, 0, 9 * 32);
  int bit = 0;
  for (int p = 0; p < 10; p++)
    for (int k = 0; k < lens[p]; k++)
      for (int j = 7; j >= 0; j--, bit++)
        if ((parts[p][k] >> j) & 1u) {
          const int c = bit / chunk, pos = bit % chunk;
          out[32 * c + pos / 8] |= (uint8_t)(1u << (pos % 8));
        }
}

inline void prep_joinsplit(const uint8_t* anchor, const uint8_t* seed, const uint8_t* nf0, const uint8_t* nf1,
                           const uint8_t* mac0, const uint8_t* mac1, const uint8_t* cm0, const uint8_t* cm1,
                           uint64_t vpub_old, uint64_t vpub_new, const uint8_t* pubkey, uint8_t* out) {
  prep_joinsplit_bits(anchor, seed, nf0, nf1, mac0, mac1, cm0, cm1, vpub_old, vpub_new, pubkey, 254, out);
}

}  // namespace zg
