// ORACLE / CPU BASELINE (test + bench infrastructure only; never the product path).
//
// A C++ restatement of the reference's per-proof CPU path -- bellman 0.1.0 verify_proof on
// pairing 0.14.2 -- with the same algorithmic structure
// as the reference: one proof at a time, 6 x 64-bit-limb Montgomery Fq, Proof::read with
// naive [r]P subgroup checks, the IC sum as naive 255-bit double-and-add per input, a
// 3-pair Miller loop with G2Prepared lines for B (and -gamma/-delta prepared once per VK),
// and pairing's final-exponentiation chain. Proofs are spread over std::threads, one proof
// per task, mirroring the rayon fan-out of verification/src/accept_chain.rs:76-81.
//
// Only tests/ and bench.py's cpu_baseline leg load this (oracle/_build/libzgcpu.so).
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

typedef unsigned __int128 u128;

namespace cpu {

// ---------------------------------------------------------------- Fq (6 x 64)
static const uint64_t P[6] = {0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL,
                              0x64774b84f38512bfULL, 0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL};
static const uint64_t PINV = 0x89f3fffcfffcfffdULL;  // -p^-1 mod 2^64
static const uint64_t R2[6] = {0xf4df1f341c341746ULL, 0x0a76e6a609d104f1ULL, 0x8de5476c4c95b6d5ULL,
                               0x67eb88a9939d83c0ULL, 0x9a793e85b519952dULL, 0x11988fe592cae3aaULL};
static const uint64_t ONE[6] = {0x760900000002fffdULL, 0xebf4000bc40c0002ULL, 0x5f48985753c758baULL,
                                0x77ce585370525745ULL, 0x5c071a97a256ec6dULL, 0x15f65ec3fa80e493ULL};

struct Fq {
  uint64_t v[6];
};

static inline bool geq_p(const uint64_t* a) {
  for (int i = 5; i >= 0; i--) {
    if (a[i] > P[i]) return true;
    if (a[i] < P[i]) return false;
  }
  return true;
}
static inline void sub_p(uint64_t* a) {
  uint64_t b = 0;
  for (int i = 0; i < 6; i++) {
    u128 t = (u128)a[i] - P[i] - b;
    a[i] = (uint64_t)t;
    b = (uint64_t)(t >> 127);
  }
}
static inline Fq add(const Fq& a, const Fq& b) {
  Fq r;
  uint64_t c = 0;
  for (int i = 0; i < 6; i++) {
    u128 t = (u128)a.v[i] + b.v[i] + c;
    r.v[i] = (uint64_t)t;
    c = (uint64_t)(t >> 64);
  }
  if (geq_p(r.v)) sub_p(r.v);
  return r;
}
static inline Fq sub(const Fq& a, const Fq& b) {
  Fq r;
  uint64_t br = 0;
  for (int i = 0; i < 6; i++) {
    u128 t = (u128)a.v[i] - b.v[i] - br;
    r.v[i] = (uint64_t)t;
    br = (uint64_t)(t >> 127);
  }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < 6; i++) {
      u128 t = (u128)r.v[i] + P[i] + c;
      r.v[i] = (uint64_t)t;
      c = (uint64_t)(t >> 64);
    }
  }
  return r;
}
static inline Fq neg(const Fq& a) {
  Fq z = {{0, 0, 0, 0, 0, 0}};
  return sub(z, a);
}
static inline Fq dbl(const Fq& a) { return add(a, a); }
// CIOS with the "no-carry" shortcut (p's top limb < 2^62, so t + a b_i + m p never needs a 7th or
// 8th word: the running value stays below 2p after every outer step). Same Montgomery product as
// pairing 0.14's (a b R^-1 mod p, canonical), fewer additions per step.
static inline Fq mul(const Fq& a, const Fq& b) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
#pragma GCC unroll 6
  for (int i = 0; i < 6; i++) {
    u128 s = (u128)a.v[0] * b.v[i] + t[0];
    uint64_t A = (uint64_t)(s >> 64);
    const uint64_t t0 = (uint64_t)s;
    const uint64_t m = t0 * PINV;
    s = (u128)m * P[0] + t0;
    uint64_t C = (uint64_t)(s >> 64);
#pragma GCC unroll 5
    for (int j = 1; j < 6; j++) {
      s = (u128)a.v[j] * b.v[i] + t[j] + A;
      A = (uint64_t)(s >> 64);
      s = (u128)m * P[j] + (uint64_t)s + C;
      C = (uint64_t)(s >> 64);
      t[j - 1] = (uint64_t)s;
    }
    t[5] = C + A;
  }
  Fq r;
  memcpy(r.v, t, 48);
  if (geq_p(r.v)) sub_p(r.v);
  return r;
}
// pairing 0.14 Fq::square: the 15 off-diagonal limb products once, doubled, plus the 6
// squares, then the Montgomery reduction of the 12-limb value
static inline Fq sqr(const Fq& a) {
  uint64_t t[12] = {0};
  for (int i = 0; i < 5; i++) {
    uint64_t c = 0;
    for (int j = i + 1; j < 6; j++) {
      u128 s = (u128)a.v[i] * a.v[j] + t[i + j] + c;
      t[i + j] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    t[i + 6] = c;
  }
  t[11] = t[10] >> 63;
  for (int i = 10; i >= 1; i--) t[i] = (t[i] << 1) | (t[i - 1] >> 63);
  t[0] <<= 1;
  uint64_t c = 0;
  for (int i = 0; i < 6; i++) {
    u128 s = (u128)a.v[i] * a.v[i] + t[2 * i] + c;
    t[2 * i] = (uint64_t)s;
    u128 s2 = (u128)t[2 * i + 1] + (uint64_t)(s >> 64);
    t[2 * i + 1] = (uint64_t)s2;
    c = (uint64_t)(s2 >> 64);
  }
  // mont_reduce: t[0..12) * 2^-384 mod p
  uint64_t carry2 = 0;
  for (int i = 0; i < 6; i++) {
    const uint64_t k = t[i] * PINV;
    uint64_t cc = 0;
    for (int j = 0; j < 6; j++) {
      u128 s = (u128)k * P[j] + t[i + j] + cc;
      t[i + j] = (uint64_t)s;
      cc = (uint64_t)(s >> 64);
    }
    u128 s = (u128)t[i + 6] + cc + carry2;
    t[i + 6] = (uint64_t)s;
    carry2 = (uint64_t)(s >> 64);
  }
  Fq r;
  memcpy(r.v, t + 6, 48);
  if (carry2 || geq_p(r.v)) sub_p(r.v);
  return r;
}
static inline bool is_zero(const Fq& a) { return !(a.v[0] | a.v[1] | a.v[2] | a.v[3] | a.v[4] | a.v[5]); }
static inline bool eq(const Fq& a, const Fq& b) { return !memcmp(a.v, b.v, 48); }
static Fq one() {
  Fq r;
  memcpy(r.v, ONE, 48);
  return r;
}
static Fq from_canon(const uint64_t* c) {
  Fq a, r2;
  memcpy(a.v, c, 48);
  memcpy(r2.v, R2, 48);
  return mul(a, r2);
}
static void to_canon(const Fq& a, uint64_t* c) {
  Fq o = {{1, 0, 0, 0, 0, 0}};
  Fq r = mul(a, o);
  memcpy(c, r.v, 48);
}
static Fq pow_limbs(const Fq& a, const uint64_t* e, int nbits) {
  Fq r = one();
  for (int i = nbits - 1; i >= 0; i--) {
    r = sqr(r);
    if ((e[i >> 6] >> (i & 63)) & 1) r = mul(r, a);
  }
  return r;
}
static uint64_t EXP_INV[6], EXP_SQRT[6], EXP_PM3_4[6], EXP_HALF[6];
static void init_exps() {
  // p-2, (p+1)/4, (p-3)/4, (p-1)/2
  uint64_t t[6];
  memcpy(t, P, 48);
  memcpy(EXP_INV, P, 48);
  EXP_INV[0] -= 2;
  // (p+1)/4
  memcpy(t, P, 48);
  t[0] += 1;
  for (int i = 0; i < 6; i++) EXP_SQRT[i] = (t[i] >> 2) | (i < 5 ? t[i + 1] << 62 : 0);
  memcpy(t, P, 48);
  t[0] -= 3;
  for (int i = 0; i < 6; i++) EXP_PM3_4[i] = (t[i] >> 2) | (i < 5 ? t[i + 1] << 62 : 0);
  memcpy(t, P, 48);
  t[0] -= 1;
  for (int i = 0; i < 6; i++) EXP_HALF[i] = (t[i] >> 1) | (i < 5 ? t[i + 1] << 63 : 0);
}
// pairing 0.14 Fq::inverse: binary extended Euclid on the Montgomery representation
// (Guide to Pairing-based Cryptography, Algorithm 16): u = aR, b = R^2 -> b = a^-1 R
static inline bool is_one_raw(const uint64_t* u) { return u[0] == 1 && !(u[1] | u[2] | u[3] | u[4] | u[5]); }
static inline void shr1(uint64_t* u) {
  for (int i = 0; i < 5; i++) u[i] = (u[i] >> 1) | (u[i + 1] << 63);
  u[5] >>= 1;
}
static inline bool lt_raw(const uint64_t* a, const uint64_t* b) {
  for (int i = 5; i >= 0; i--) {
    if (a[i] != b[i]) return a[i] < b[i];
  }
  return false;
}
static inline void sub_raw(uint64_t* a, const uint64_t* b) {
  uint64_t br = 0;
  for (int i = 0; i < 6; i++) {
    u128 t = (u128)a[i] - b[i] - br;
    a[i] = (uint64_t)t;
    br = (uint64_t)(t >> 127);
  }
}
static inline void half_mod(uint64_t* x) {  // x / 2 mod p (x < p)
  if (x[0] & 1) {
    uint64_t c = 0;
    for (int i = 0; i < 6; i++) {
      u128 t = (u128)x[i] + P[i] + c;
      x[i] = (uint64_t)t;
      c = (uint64_t)(t >> 64);
    }
  }
  shr1(x);
}
static Fq inv(const Fq& a) {
  if (is_zero(a)) return a;  // (callers never invert zero: pairing returns None)
  uint64_t u[6], v[6], b[6], c[6] = {0, 0, 0, 0, 0, 0};
  memcpy(u, a.v, 48);
  memcpy(v, P, 48);
  memcpy(b, R2, 48);
  while (!is_one_raw(u) && !is_one_raw(v)) {
    while (!(u[0] & 1)) {
      shr1(u);
      half_mod(b);
    }
    while (!(v[0] & 1)) {
      shr1(v);
      half_mod(c);
    }
    if (lt_raw(v, u)) {
      sub_raw(u, v);
      Fq x, y;
      memcpy(x.v, b, 48);
      memcpy(y.v, c, 48);
      memcpy(b, sub(x, y).v, 48);
    } else {
      sub_raw(v, u);
      Fq x, y;
      memcpy(x.v, c, 48);
      memcpy(y.v, b, 48);
      memcpy(c, sub(x, y).v, 48);
    }
  }
  Fq r;
  memcpy(r.v, is_one_raw(u) ? b : c, 48);
  return r;
}

// ---------------------------------------------------------------- tower
struct Fq2 {
  Fq c0, c1;
};
struct Fq6 {
  Fq2 c0, c1, c2;
};
struct Fq12 {
  Fq6 c0, c1;
};
static Fq2 add(const Fq2& a, const Fq2& b) { return {add(a.c0, b.c0), add(a.c1, b.c1)}; }
static Fq2 sub(const Fq2& a, const Fq2& b) { return {sub(a.c0, b.c0), sub(a.c1, b.c1)}; }
static Fq2 neg(const Fq2& a) { return {neg(a.c0), neg(a.c1)}; }
static Fq2 dbl(const Fq2& a) { return {dbl(a.c0), dbl(a.c1)}; }
static Fq2 mul(const Fq2& a, const Fq2& b) {
  Fq t0 = mul(a.c0, b.c0), t1 = mul(a.c1, b.c1);
  return {sub(t0, t1), sub(sub(mul(add(a.c0, a.c1), add(b.c0, b.c1)), t0), t1)};
}
static Fq2 sqr(const Fq2& a) { return {mul(add(a.c0, a.c1), sub(a.c0, a.c1)), dbl(mul(a.c0, a.c1))}; }
static Fq2 mulfq(const Fq2& a, const Fq& s) { return {mul(a.c0, s), mul(a.c1, s)}; }
static Fq2 mulnr(const Fq2& a) { return {sub(a.c0, a.c1), add(a.c0, a.c1)}; }
static Fq2 conj(const Fq2& a) { return {a.c0, neg(a.c1)}; }
static bool is_zero(const Fq2& a) { return is_zero(a.c0) && is_zero(a.c1); }
static bool eq(const Fq2& a, const Fq2& b) { return eq(a.c0, b.c0) && eq(a.c1, b.c1); }
static Fq2 inv(const Fq2& a) {
  Fq t = inv(add(sqr(a.c0), sqr(a.c1)));
  return {mul(a.c0, t), neg(mul(a.c1, t))};
}
static Fq2 one2() { return {one(), Fq{{0}}}; }
static Fq2 pow2(const Fq2& a, const uint64_t* e, int nbits) {
  Fq2 r = one2();
  for (int i = nbits - 1; i >= 0; i--) {
    r = sqr(r);
    if ((e[i >> 6] >> (i & 63)) & 1) r = mul(r, a);
  }
  return r;
}
static Fq6 add(const Fq6& a, const Fq6& b) { return {add(a.c0, b.c0), add(a.c1, b.c1), add(a.c2, b.c2)}; }
static Fq6 sub(const Fq6& a, const Fq6& b) { return {sub(a.c0, b.c0), sub(a.c1, b.c1), sub(a.c2, b.c2)}; }
static Fq6 neg(const Fq6& a) { return {neg(a.c0), neg(a.c1), neg(a.c2)}; }
static Fq6 mulnr(const Fq6& a) { return {mulnr(a.c2), a.c0, a.c1}; }
static Fq6 mul(const Fq6& a, const Fq6& b) {
  Fq2 t0 = mul(a.c0, b.c0), t1 = mul(a.c1, b.c1), t2 = mul(a.c2, b.c2);
  return {add(mulnr(sub(sub(mul(add(a.c1, a.c2), add(b.c1, b.c2)), t1), t2)), t0),
          add(sub(sub(mul(add(a.c0, a.c1), add(b.c0, b.c1)), t0), t1), mulnr(t2)),
          add(sub(sub(mul(add(a.c0, a.c2), add(b.c0, b.c2)), t0), t2), t1)};
}
static Fq6 inv(const Fq6& a) {
  Fq2 c0 = sub(sqr(a.c0), mulnr(mul(a.c1, a.c2)));
  Fq2 c1 = sub(mulnr(sqr(a.c2)), mul(a.c0, a.c1));
  Fq2 c2 = sub(sqr(a.c1), mul(a.c0, a.c2));
  Fq2 t = inv(add(mul(a.c0, c0), mulnr(add(mul(a.c2, c1), mul(a.c1, c2)))));
  return {mul(c0, t), mul(c1, t), mul(c2, t)};
}
static bool is_zero(const Fq6& a) { return is_zero(a.c0) && is_zero(a.c1) && is_zero(a.c2); }
static bool eq(const Fq6& a, const Fq6& b) { return eq(a.c0, b.c0) && eq(a.c1, b.c1) && eq(a.c2, b.c2); }
static Fq12 mul(const Fq12& a, const Fq12& b) {
  Fq6 t0 = mul(a.c0, b.c0), t1 = mul(a.c1, b.c1);
  return {add(t0, mulnr(t1)), sub(sub(mul(add(a.c0, a.c1), add(b.c0, b.c1)), t0), t1)};
}
static Fq12 sqr(const Fq12& a) {
  Fq6 ab = mul(a.c0, a.c1);
  Fq6 c0 = sub(sub(mul(add(a.c0, a.c1), add(a.c0, mulnr(a.c1))), ab), mulnr(ab));
  return {c0, add(ab, ab)};
}
static Fq12 conj(const Fq12& a) { return {a.c0, neg(a.c1)}; }
static Fq12 inv(const Fq12& a) {
  Fq6 t = inv(sub(mul(a.c0, a.c0), mulnr(mul(a.c1, a.c1))));
  return {mul(a.c0, t), neg(mul(a.c1, t))};
}
static Fq12 one12() {
  Fq2 z = {Fq{{0}}, Fq{{0}}};
  return {{one2(), z, z}, {z, z, z}};
}
static bool eq(const Fq12& a, const Fq12& b) { return eq(a.c0, b.c0) && eq(a.c1, b.c1); }
static bool is_zero(const Fq12& a) { return is_zero(a.c0) && is_zero(a.c1); }
// Fq6 * (b0 + b1 v) and Fq6 * (b1 v): pairing mul_by_01 / mul_by_1
static Fq6 mul01(const Fq6& a, const Fq2& b0, const Fq2& b1) {
  Fq2 t0 = mul(a.c0, b0), t1 = mul(a.c1, b1);
  return {sub(add(mulnr(mul(add(a.c1, a.c2), b1)), t0), mulnr(t1)), sub(sub(mul(add(a.c0, a.c1), add(b0, b1)), t0), t1),
          add(sub(mul(add(a.c0, a.c2), b0), t0), t1)};
}
static Fq6 mul1(const Fq6& a, const Fq2& b1) { return {mulnr(mul(a.c2, b1)), mul(a.c0, b1), mul(a.c1, b1)}; }
// f * (c0 + c1 v + c4 v w): pairing Fq12::mul_by_014 (13 Fq2 products)
static Fq12 mul014(const Fq12& f, const Fq2& c0, const Fq2& c1, const Fq2& c4) {
  Fq6 aa = mul01(f.c0, c0, c1), bb = mul1(f.c1, c4);
  Fq6 s = mul01(add(f.c0, f.c1), c0, add(c1, c4));
  return {add(aa, mulnr(bb)), sub(sub(s, aa), bb)};
}
static Fq2 FROB6_1[4], FROB6_2[4], FROB12[4];  // index k = 1..3
static Fq12 frob(const Fq12& a, int k) {
  auto f2 = [&](const Fq2& x) { return (k & 1) ? conj(x) : x; };
  Fq6 a0 = {f2(a.c0.c0), mul(f2(a.c0.c1), FROB6_1[k]), mul(f2(a.c0.c2), FROB6_2[k])};
  Fq6 a1 = {f2(a.c1.c0), mul(f2(a.c1.c1), FROB6_1[k]), mul(f2(a.c1.c2), FROB6_2[k])};
  a1 = {mul(a1.c0, FROB12[k]), mul(a1.c1, FROB12[k]), mul(a1.c2, FROB12[k])};
  return {a0, a1};
}
static Fq12 pow_u64(const Fq12& a, uint64_t e) {
  Fq12 r = one12();
  for (int i = 63; i >= 0; i--) {
    r = sqr(r);
    if ((e >> i) & 1) r = mul(r, a);
  }
  return r;
}
static const uint64_t BLS_X = 0xd201000000010000ULL;
static Fq12 exp_by_x(const Fq12& f, uint64_t x) { return conj(pow_u64(f, x)); }
static Fq12 final_exp(const Fq12& f) {  // pairing 0.14.2 chain
  Fq12 r = mul(conj(f), inv(f));
  Fq12 f2 = r;
  r = mul(frob(r, 2), f2);
  Fq12 y0 = sqr(r);
  Fq12 y1 = exp_by_x(y0, BLS_X);
  Fq12 y2 = exp_by_x(y1, BLS_X >> 1);
  Fq12 y3 = conj(r);
  y1 = mul(y1, y3);
  y1 = conj(y1);
  y1 = mul(y1, y2);
  y2 = exp_by_x(y1, BLS_X);
  y3 = exp_by_x(y2, BLS_X);
  y1 = conj(y1);
  y3 = mul(y3, y1);
  y1 = conj(y1);
  y1 = frob(y1, 3);
  y2 = frob(y2, 2);
  y1 = mul(y1, y2);
  y2 = exp_by_x(y3, BLS_X);
  y2 = mul(y2, y0);
  y2 = mul(y2, r);
  y1 = mul(y1, y2);
  y2 = frob(y3, 1);
  y1 = mul(y1, y2);
  return y1;
}

// ---------------------------------------------------------------- curves (templated Jacobian)
template <class F>
struct Pt {
  F x, y, z;  // z = 0: infinity
};
template <class F>
static F fzero() {
  F z;
  memset(&z, 0, sizeof(z));
  return z;
}
static Fq fone(Fq*) { return one(); }
static Fq2 fone(Fq2*) { return one2(); }
template <class F>
static Pt<F> infinity() {
  F o = fone((F*)nullptr);
  return {o, o, fzero<F>()};
}
template <class F>
static bool is_inf(const Pt<F>& p) {
  return is_zero(p.z);
}
template <class F>
static Pt<F> pdbl(const Pt<F>& p) {
  if (is_inf(p)) return p;
  F A = sqr(p.x), B = sqr(p.y), C = sqr(B);
  F D = dbl(sub(sub(sqr(add(p.x, B)), A), C));
  F E = add(dbl(A), A), Fv = sqr(E);
  F X3 = sub(Fv, dbl(D));
  F Y3 = sub(mul(E, sub(D, X3)), dbl(dbl(dbl(C))));
  F Z3 = dbl(mul(p.y, p.z));
  return {X3, Y3, Z3};
}
template <class F>
static Pt<F> padd(const Pt<F>& p, const Pt<F>& q) {
  if (is_inf(p)) return q;
  if (is_inf(q)) return p;
  F Z1Z1 = sqr(p.z), Z2Z2 = sqr(q.z);
  F U1 = mul(p.x, Z2Z2), U2 = mul(q.x, Z1Z1);
  F S1 = mul(mul(p.y, q.z), Z2Z2), S2 = mul(mul(q.y, p.z), Z1Z1);
  F H = sub(U2, U1), rr = dbl(sub(S2, S1));
  if (is_zero(H)) return is_zero(rr) ? pdbl(p) : infinity<F>();
  F I = sqr(dbl(H)), J = mul(H, I), V = mul(U1, I);
  F X3 = sub(sub(sqr(rr), J), dbl(V));
  F Y3 = sub(mul(rr, sub(V, X3)), dbl(mul(S1, J)));
  F Z3 = mul(sub(sub(sqr(add(p.z, q.z)), Z1Z1), Z2Z2), H);
  return {X3, Y3, Z3};
}
template <class F>
static Pt<F> pmul(const Pt<F>& p, const uint64_t* k, int nbits) {  // naive double-and-add
  Pt<F> acc = infinity<F>();
  for (int i = nbits - 1; i >= 0; i--) {
    acc = pdbl(acc);
    if ((k[i >> 6] >> (i & 63)) & 1) acc = padd(acc, p);
  }
  return acc;
}
template <class F>
static void to_affine(const Pt<F>& p, F* x, F* y) {
  F zi = inv(p.z), zi2 = sqr(zi);
  *x = mul(p.x, zi2);
  *y = mul(p.y, mul(zi2, zi));
}
static const uint64_t RMOD[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL,
                                 0x73eda753299d7d48ULL};
template <class F>
static bool in_subgroup(const Pt<F>& p) {  // pairing 0.14: [r]P == O
  return is_inf(pmul(p, RMOD, 255));
}

static Fq B4;
static Fq2 B2;
static void load_be(const uint8_t* b, uint64_t* c) {
  for (int i = 0; i < 6; i++) {
    uint64_t w = 0;
    for (int k = 0; k < 8; k++) w = (w << 8) | b[40 - 8 * i + k];
    c[i] = w;
  }
}
static bool lt_p(const uint64_t* c) { return !geq_p(c); }
static bool canon_gt_half(const Fq& y) {  // y > (p-1)/2 canonical
  uint64_t c[6];
  to_canon(y, c);
  for (int i = 5; i >= 0; i--) {
    if (c[i] > EXP_HALF[i]) return true;
    if (c[i] < EXP_HALF[i]) return false;
  }
  return false;
}
static bool fq_sqrt(const Fq& a, Fq* out) {
  Fq s = pow_limbs(a, EXP_SQRT, 380);
  *out = s;
  return eq(sqr(s), a);
}
static bool fq2_sqrt(const Fq2& a, Fq2* out) {
  if (is_zero(a)) {
    *out = a;
    return true;
  }
  Fq2 a1 = pow2(a, EXP_PM3_4, 379);
  Fq2 alpha = mul(sqr(a1), a);
  Fq2 a0 = mul(conj(alpha), alpha);
  Fq2 m1 = {neg(one()), Fq{{0}}};
  if (eq(a0, m1)) return false;
  a1 = mul(a1, a);
  if (eq(alpha, m1)) {
    *out = {neg(a1.c1), a1.c0};
    return true;
  }
  *out = mul(a1, pow2(add(alpha, one2()), EXP_HALF, 380));
  return true;
}

// bellman Proof::read point decoders (compressed); false on any failure incl. infinity
static bool g1_read(const uint8_t* b, Pt<Fq>* out) {
  if (!(b[0] & 0x80) || (b[0] & 0x40)) return false;  // wrong mode / infinity (rejected anyway)
  bool greatest = b[0] & 0x20;
  uint8_t t[48];
  memcpy(t, b, 48);
  t[0] &= 0x1f;
  uint64_t c[6];
  load_be(t, c);
  if (!lt_p(c)) return false;
  Fq x = from_canon(c), y;
  if (!fq_sqrt(add(mul(sqr(x), x), B4), &y)) return false;
  bool y_gt = canon_gt_half(y);
  bool y_lt = !y_gt && !is_zero(y);
  if (!(y_lt ^ greatest)) y = neg(y);
  *out = {x, y, one()};
  return in_subgroup(*out);
}
static bool g2_read(const uint8_t* b, Pt<Fq2>* out) {
  if (!(b[0] & 0x80) || (b[0] & 0x40)) return false;
  bool greatest = b[0] & 0x20;
  uint8_t t[48];
  memcpy(t, b, 48);
  t[0] &= 0x1f;
  uint64_t c1[6], c0[6];
  load_be(t, c1);
  load_be(b + 48, c0);
  if (!lt_p(c1) || !lt_p(c0)) return false;
  Fq2 x = {from_canon(c0), from_canon(c1)}, y;
  if (!fq2_sqrt(add(mul(sqr(x), x), B2), &y)) return false;
  bool y_gt = !is_zero(y.c1) ? canon_gt_half(y.c1) : canon_gt_half(y.c0);
  bool y_lt = !y_gt && !is_zero(y);
  if (!(y_lt ^ greatest)) y = neg(y);
  *out = {x, y, one2()};
  return in_subgroup(*out);
}
// uncompressed (VK)
static int g1_read_unc(const uint8_t* b, Pt<Fq>* out) {
  if (b[0] & 0x80) return -1;
  if (b[0] & 0x40) {
    uint8_t acc = b[0] & 0x3f;
    for (int i = 1; i < 96; i++) acc |= b[i];
    if (acc) return -1;
    *out = infinity<Fq>();
    return 0;
  }
  if (b[0] & 0x20) return -1;
  uint8_t t[96];
  memcpy(t, b, 96);
  t[0] &= 0x1f;
  uint64_t cx[6], cy[6];
  load_be(t, cx);
  load_be(t + 48, cy);
  if (!lt_p(cx) || !lt_p(cy)) return -1;
  Fq x = from_canon(cx), y = from_canon(cy);
  if (!eq(sqr(y), add(mul(sqr(x), x), B4))) return -1;
  *out = {x, y, one()};
  return in_subgroup(*out) ? 0 : -1;
}
static int g2_read_unc(const uint8_t* b, Pt<Fq2>* out) {
  if (b[0] & 0x80) return -1;
  if (b[0] & 0x40) {
    uint8_t acc = b[0] & 0x3f;
    for (int i = 1; i < 192; i++) acc |= b[i];
    if (acc) return -1;
    *out = infinity<Fq2>();
    return 0;
  }
  if (b[0] & 0x20) return -1;
  uint8_t t[192];
  memcpy(t, b, 192);
  t[0] &= 0x1f;
  uint64_t c[4][6];
  for (int i = 0; i < 4; i++) {
    load_be(t + 48 * i, c[i]);
    if (!lt_p(c[i])) return -1;
  }
  Fq2 x = {from_canon(c[1]), from_canon(c[0])}, y = {from_canon(c[3]), from_canon(c[2])};
  if (!eq(sqr(y), add(mul(sqr(x), x), B2))) return -1;
  *out = {x, y, one2()};
  return in_subgroup(*out) ? 0 : -1;
}

// ---------------------------------------------------------------- pairing
struct Coeff {
  Fq2 c0, c1, c2;
};
static Coeff doubling_step(Pt<Fq2>& r) {
  Fq2 tmp0 = sqr(r.x), tmp1 = sqr(r.y), tmp2 = sqr(tmp1);
  Fq2 tmp3 = dbl(sub(sub(sqr(add(tmp1, r.x)), tmp0), tmp2));
  Fq2 tmp4 = add(dbl(tmp0), tmp0), tmp6 = add(r.x, tmp4), tmp5 = sqr(tmp4), zsq = sqr(r.z);
  Fq2 nx = sub(sub(tmp5, tmp3), tmp3);
  Fq2 nz = sub(sub(sqr(add(r.z, r.y)), tmp1), zsq);
  Fq2 ny = sub(mul(sub(tmp3, nx), tmp4), dbl(dbl(dbl(tmp2))));
  tmp3 = neg(dbl(mul(tmp4, zsq)));
  tmp6 = sub(sub(sub(sqr(tmp6), tmp0), tmp5), dbl(dbl(tmp1)));
  tmp0 = dbl(mul(nz, zsq));
  r = {nx, ny, nz};
  return {tmp0, tmp3, tmp6};
}
static Coeff addition_step(Pt<Fq2>& r, const Fq2& qx, const Fq2& qy) {
  Fq2 zsq = sqr(r.z), ysq = sqr(qy), t0 = mul(zsq, qx);
  Fq2 t1 = mul(sub(sub(sqr(add(qy, r.z)), ysq), zsq), zsq);
  Fq2 t2 = sub(t0, r.x), t3 = sqr(t2), t4 = dbl(dbl(t3)), t5 = mul(t4, t2);
  Fq2 t6 = sub(sub(t1, r.y), r.y), t9 = mul(t6, qx), t7 = mul(t4, r.x);
  Fq2 nx = sub(sub(sub(sqr(t6), t5), t7), t7);
  Fq2 nz = sub(sub(sqr(add(r.z, t2)), zsq), t3);
  Fq2 t10 = add(qy, nz);
  Fq2 t8 = mul(sub(t7, nx), t6);
  Fq2 ny = sub(t8, dbl(mul(r.y, t5)));
  t10 = sub(sub(sqr(t10), ysq), sqr(nz));
  t9 = sub(dbl(t9), t10);
  r = {nx, ny, nz};
  return {dbl(nz), dbl(neg(t6)), t9};
}
static const uint64_t XH = 0x6900800000008000ULL;
static void prepare(const Fq2& qx, const Fq2& qy, std::vector<Coeff>& out) {
  out.clear();
  Pt<Fq2> r = {qx, qy, one2()};
  for (int i = 61; i >= 0; i--) {
    out.push_back(doubling_step(r));
    if ((XH >> i) & 1) out.push_back(addition_step(r, qx, qy));
  }
  out.push_back(doubling_step(r));
}
struct PairIn {
  Fq px, py;
  const Coeff* c;
};
static Fq12 miller(const PairIn* pairs, int np) {
  Fq12 f = one12();
  int idx = 0;
  auto ell = [&](const PairIn& p, const Coeff& c) { f = mul014(f, c.c2, mulfq(c.c1, p.px), mulfq(c.c0, p.py)); };
  for (int i = 61; i >= 0; i--) {
    for (int j = 0; j < np; j++) ell(pairs[j], pairs[j].c[idx]);
    idx++;
    if ((XH >> i) & 1) {
      for (int j = 0; j < np; j++) ell(pairs[j], pairs[j].c[idx]);
      idx++;
    }
    f = sqr(f);
  }
  for (int j = 0; j < np; j++) ell(pairs[j], pairs[j].c[idx]);
  return conj(f);
}

// ---------------------------------------------------------------- VK + verify
struct VK {
  int loaded = 0;
  std::vector<Pt<Fq>> ic;
  Fq12 ab;
  std::vector<Coeff> ng, nd;
  bool ng_inf = true, nd_inf = true;
};
static VK g_vk[3];

static void init_consts() {
  static bool done = false;
  if (done) return;
  init_exps();
  uint64_t four[6] = {4, 0, 0, 0, 0, 0};
  B4 = from_canon(four);
  B2 = {B4, B4};
  // Frobenius constants gamma = xi^((p^k - 1)/d), computed by exponentiation in Fq2
  Fq2 xi = {one(), one()};
  // exponents as 6*k-limb integers: compute (p^k - 1)/d with simple bigint
  for (int k = 1; k <= 3; k++) {
    // p^k as up to 18 limbs
    uint64_t pk[18] = {0};
    pk[0] = 1;
    for (int m = 0; m < k; m++) {
      uint64_t res[18] = {0};
      for (int i = 0; i < 18; i++) {
        if (!pk[i]) continue;
        u128 c = 0;
        for (int j = 0; j < 6 && i + j < 18; j++) {
          u128 s = (u128)pk[i] * P[j] + res[i + j] + c;
          res[i + j] = (uint64_t)s;
          c = s >> 64;
        }
        for (int t = i + 6; c && t < 18; t++) {
          u128 s = (u128)res[t] + c;
          res[t] = (uint64_t)s;
          c = s >> 64;
        }
      }
      memcpy(pk, res, sizeof(pk));
    }
    pk[0] -= 1;  // p^k - 1 (p^k odd)
    auto divsmall = [&](const uint64_t* a, uint64_t d, uint64_t* q) {
      u128 rem = 0;
      for (int i = 17; i >= 0; i--) {
        u128 cur = (rem << 64) | a[i];
        q[i] = (uint64_t)(cur / d);
        rem = cur % d;
      }
    };
    uint64_t e3[18], e6[18], e32[18];
    divsmall(pk, 3, e3);
    divsmall(pk, 6, e6);
    memcpy(e32, e3, sizeof(e32));
    u128 c = 0;  // e32 = 2 * e3
    for (int i = 0; i < 18; i++) {
      u128 s = ((u128)e32[i] << 1) + c;
      e32[i] = (uint64_t)s;
      c = s >> 64;
    }
    FROB6_1[k] = pow2(xi, e3, 18 * 64);
    FROB6_2[k] = pow2(xi, e32, 18 * 64);
    FROB12[k] = pow2(xi, e6, 18 * 64);
  }
  done = true;
}

static int verify_one(const VK& vk, const uint8_t* pb, const uint8_t* in, int k, Fq12* gt) {
  // canonical inputs
  uint64_t x[9][4];
  for (int j = 0; j < k && j < 9; j++) {
    for (int w = 0; w < 4; w++) {
      uint64_t v = 0;
      for (int b = 7; b >= 0; b--) v = (v << 8) | in[32 * j + 8 * w + b];
      x[j][w] = v;
    }
    bool lt = false;
    for (int w = 3; w >= 0; w--) {
      if (x[j][w] < RMOD[w]) {
        lt = true;
        break;
      }
      if (x[j][w] > RMOD[w]) break;
    }
    if (!lt) return 4;
  }
  Pt<Fq> A, C;
  Pt<Fq2> B;
  if (!g1_read(pb, &A) || !g2_read(pb + 48, &B) || !g1_read(pb + 144, &C)) return 1;
  if (k + 1 != (int)vk.ic.size()) return 2;
  Pt<Fq> acc = vk.ic[0];
  for (int j = 0; j < k; j++) acc = padd(acc, pmul(vk.ic[j + 1], x[j], 255));
  std::vector<Coeff> bl;
  Fq2 bx, by;
  to_affine(B, &bx, &by);
  prepare(bx, by, bl);
  PairIn pairs[3];
  int np = 0;
  Fq ax, ay, cx, cy;
  to_affine(A, &ax, &ay);
  pairs[np++] = {ax, ay, bl.data()};
  if (!is_inf(acc) && !vk.ng_inf) {
    Fq px, py;
    to_affine(acc, &px, &py);
    pairs[np++] = {px, py, vk.ng.data()};
  }
  if (!vk.nd_inf) {
    to_affine(C, &cx, &cy);
    pairs[np++] = {cx, cy, vk.nd.data()};
  }
  *gt = final_exp(miller(pairs, np));
  return eq(*gt, vk.ab) ? 0 : 3;
}

static void f12_bytes(const Fq12& a, uint8_t* out) {
  const Fq2* c[6] = {&a.c0.c0, &a.c0.c1, &a.c0.c2, &a.c1.c0, &a.c1.c1, &a.c1.c2};
  for (int i = 0; i < 6; i++)
    for (int h = 0; h < 2; h++) {
      uint64_t v[6];
      to_canon(h ? c[i]->c1 : c[i]->c0, v);
      uint8_t* o = out + 96 * i + 48 * h;
      for (int l = 0; l < 6; l++)
        for (int b = 0; b < 8; b++) o[40 - 8 * l + b] = (uint8_t)(v[l] >> (56 - 8 * b));
    }
}

}  // namespace cpu

extern "C" {

// prepare_verifying_key from uncompressed fields (alpha|betaG1|betaG2|gamma|deltaG1|deltaG2)
int zgcpu_vk_load(int kind, const uint8_t* fields, int n_ic, const uint8_t* ic, uint8_t* ab_out) {
  using namespace cpu;
  init_consts();
  if (kind < 0 || kind > 2) return -1;
  VK vk;
  Pt<Fq> alpha, beta1, delta1;
  Pt<Fq2> beta, gamma, delta;
  const uint8_t* p = fields;
  if (g1_read_unc(p, &alpha) || g1_read_unc(p + 96, &beta1) || g2_read_unc(p + 192, &beta) ||
      g2_read_unc(p + 384, &gamma) || g1_read_unc(p + 576, &delta1) || g2_read_unc(p + 672, &delta))
    return -2;
  for (int i = 0; i < n_ic; i++) {
    Pt<Fq> q;
    if (g1_read_unc(ic + 96 * i, &q)) return -2;
    vk.ic.push_back(q);
  }
  if (!is_inf(alpha) && !is_inf(beta)) {
    Fq ax, ay;
    Fq2 bx, by;
    to_affine(alpha, &ax, &ay);
    to_affine(beta, &bx, &by);
    std::vector<Coeff> bl;
    prepare(bx, by, bl);
    PairIn pr = {ax, ay, bl.data()};
    vk.ab = final_exp(miller(&pr, 1));
  } else {
    vk.ab = one12();
  }
  if (!is_inf(gamma)) {
    Fq2 gx, gy;
    to_affine(gamma, &gx, &gy);
    prepare(gx, neg(gy), vk.ng);
    vk.ng_inf = false;
  }
  if (!is_inf(delta)) {
    Fq2 dx, dy;
    to_affine(delta, &dx, &dy);
    prepare(dx, neg(dy), vk.nd);
    vk.nd_inf = false;
  }
  vk.loaded = 1;
  g_vk[kind] = vk;
  if (ab_out) f12_bytes(vk.ab, ab_out);
  return 0;
}

// verify n proofs, one per task on `threads` std::threads (bellman semantics per proof)
int zgcpu_verify(size_t n, const uint8_t* proofs, const uint8_t* kinds, const uint8_t* inputs,
                 const uint8_t* n_inputs, uint8_t* status, uint8_t* gts, int threads) {
  using namespace cpu;
  init_consts();
  static const int KN[3] = {7, 5, 9};
  for (size_t i = 0; i < n; i++)
    if (kinds[i] > 2 || !g_vk[kinds[i]].loaded) return -3;
  if (threads < 1) threads = 1;
  std::atomic<size_t> next(0);
  auto work = [&]() {
    for (;;) {
      size_t i = next.fetch_add(1);
      if (i >= n) break;
      int k = n_inputs ? n_inputs[i] : KN[kinds[i]];
      Fq12 gt;
      int st = k > 9 ? 2 : verify_one(g_vk[kinds[i]], proofs + 192 * i, inputs + 288 * i, k, &gt);
      status[i] = (uint8_t)st;
      if (gts && (st == 0 || st == 3)) f12_bytes(gt, gts + 576 * i);
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; t++) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  return 0;
}

// calibration of the port: single-thread timings of its building blocks on
// the first proof of kind `kind` (its A, B and the key's -delta / -gamma lines), so the per-proof
// figure can be set against bellman-class estimates. out[0] ns per Fq product (a dependent chain),
// out[1] ns per Fq squaring, out[2] us per 3-pair Miller loop, out[3] us per final exponentiation,
// out[4] us per G2Prepared (68 line coefficients), out[5] us per 255-bit G1 scalar product (one IC
// term, also the [r]P subgroup check), out[6] us per G2 [r]Q subgroup check, out[7] us per proof
// (verify_one). Returns 0, or -1 if the proof does not decode / the key is not loaded.
int zgcpu_bench_ops(int kind, const uint8_t* proof, const uint8_t* inputs, int k, int reps, double* out) {
  using namespace cpu;
  init_consts();
  if (kind < 0 || kind > 2 || !g_vk[kind].loaded || reps < 1) return -1;
  const VK& vk = g_vk[kind];
  Pt<Fq> A, C;
  Pt<Fq2> B;
  if (!g1_read(proof, &A) || !g2_read(proof + 48, &B) || !g1_read(proof + 144, &C)) return -1;
  using clk = std::chrono::steady_clock;
  auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
  Fq ax, ay, cx, cy;
  to_affine(A, &ax, &ay);
  to_affine(C, &cx, &cy);
  // Fq product / square chains
  const int nm = 200000;
  Fq x = ax, y = ay;
  auto t0 = clk::now();
  for (int i = 0; i < nm; i++) x = mul(x, y);
  auto t1 = clk::now();
  for (int i = 0; i < nm; i++) y = sqr(y);
  auto t2 = clk::now();
  out[0] = 1e3 * us(t0, t1) / nm;
  out[1] = 1e3 * us(t1, t2) / nm;
  volatile uint64_t sink = x.v[0] ^ y.v[0];
  (void)sink;
  // G2Prepared, 3-pair Miller loop, final exponentiation
  Fq2 bx, by;
  to_affine(B, &bx, &by);
  std::vector<Coeff> bl;
  t0 = clk::now();
  for (int r = 0; r < reps; r++) {
    bl.clear();
    prepare(bx, by, bl);
  }
  t1 = clk::now();
  out[4] = us(t0, t1) / reps;
  PairIn pairs[3] = {{ax, ay, bl.data()}, {cx, cy, vk.ng.data()}, {cx, cy, vk.nd.data()}};
  Fq12 f = one12();
  t0 = clk::now();
  for (int r = 0; r < reps; r++) f = miller(pairs, 3);
  t1 = clk::now();
  out[2] = us(t0, t1) / reps;
  Fq12 g = f;
  t0 = clk::now();
  for (int r = 0; r < reps; r++) g = final_exp(f);
  t1 = clk::now();
  out[3] = us(t0, t1) / reps;
  // one 255-bit G1 product (an IC term; the naive [r]P check has the same shape) and the G2 check
  uint64_t sc[4] = {0x0123456789abcdefULL, 0xfedcba9876543210ULL, 0x0f1e2d3c4b5a6978ULL, 0x3fffffffffffffffULL};
  Pt<Fq> pa = A;
  t0 = clk::now();
  for (int r = 0; r < reps; r++) pa = pmul(A, sc, 255);
  t1 = clk::now();
  out[5] = us(t0, t1) / reps;
  Pt<Fq2> pb = B;
  t0 = clk::now();
  for (int r = 0; r < reps; r++) pb = pmul(B, RMOD, 255);
  t1 = clk::now();
  out[6] = us(t0, t1) / reps;
  Fq12 gt;
  t0 = clk::now();
  for (int r = 0; r < reps; r++) verify_one(vk, proof, inputs, k, &gt);
  t1 = clk::now();
  out[7] = us(t0, t1) / reps;
  sink = pa.x.v[0] ^ pb.x.c0.v[0] ^ g.c0.c0.c0.v[0];
  return 0;
}

}  // extern "C"
