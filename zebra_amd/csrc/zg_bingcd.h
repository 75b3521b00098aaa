// zg_bingcd.h -- variable-time modular inversion by binary GCD with 64-bit approximations
// (T. Pornin, "Optimized Binary GCD for Modular Inversion", 2020, algorithm 2; here 30 divsteps
// per outer step on 64-bit approximations).
//
// For PUBLIC values only (tree hashes, decoded points): the running time depends on the input.
// It replaces Fermat's a^(p-2) (log2 p squarings + multiplications, ~380 Fr products) where an
// inversion sits on a latency-critical chain: 17 outer steps (Fr) of 30 divsteps on 64-bit
// approximations of a and b (their low 30 and top 34 bits), each followed by one linear update
// of the full a, b (exact division by 2^30) and of the Bezout pair u, v (Montgomery division by
// 2^30, so that a = y u and b = y v mod p hold throughout). 2 len(p) - 1 divsteps suffice for
// b to reach gcd(y, p) = 1 (then v = y^-1); y = 0 returns 0, as a^(p-2) does.
#pragma once
#include "zg_field.h"

namespace zg {

#define ZG_INV_T_FR 17  // ceil((2 * 255 - 1) / 30)
#define ZG_INV_T_FQ 26  // ceil((2 * 381 - 1) / 30)

// acc (N + 2 limbs, two's complement) += (neg ? -1 : 1) * a * m, a unsigned N limbs, m < 2^32
template <int N>
ZG_INL void bg_mac(uint32_t* acc, const uint32_t* a, uint32_t m, bool neg) {
  const uint32_t mask = neg ? 0xffffffffu : 0u;
  uint64_t c = 0, s = neg ? 1u : 0u;
#pragma unroll
  for (int i = 0; i < N + 2; i++) {
    uint32_t p = 0;
    if (i < N) {
      c += (uint64_t)a[i] * m;
      p = (uint32_t)c;
      c >>= 32;
    } else if (i == N) {
      p = (uint32_t)c;
    }
    s += (uint64_t)acc[i] + (p ^ mask);
    acc[i] = (uint32_t)s;
    s >>= 32;
  }
}

// t (N + 2 limbs, two's complement) >>= S (0 < S < 32), arithmetic
template <int N, int S>
ZG_INL void bg_shr(uint32_t* t) {
#pragma unroll
  for (int i = 0; i < N + 1; i++) t[i] = (t[i] >> S) | (t[i + 1] << (32 - S));
  t[N + 1] = (uint32_t)((int32_t)t[N + 1] >> S);
}

template <int N>
ZG_INL bool bg_neg_p(const uint32_t* t) {
  return (int32_t)t[N + 1] < 0;
}

// t = -t when c (N + 2 limbs)
template <int N>
ZG_INL void bg_cneg(uint32_t* t, bool c) {
  const uint32_t mask = c ? 0xffffffffu : 0u;
  uint64_t s = c ? 1u : 0u;
#pragma unroll
  for (int i = 0; i < N + 2; i++) {
    s += (uint64_t)(t[i] ^ mask);
    t[i] = (uint32_t)s;
    s >>= 32;
  }
}

// t += c ? sign * p : 0 (N + 2 limbs)
template <class M>
ZG_INL void bg_cadd_p(uint32_t* t, bool c, bool sub) {
  constexpr int N = M::N;
  const uint32_t mask = sub ? 0xffffffffu : 0u;
  uint64_t s = sub ? 1u : 0u;
#pragma unroll
  for (int i = 0; i < N + 2; i++) {
    const uint32_t pi = c ? ((i < N ? M::p(i) : 0u) ^ mask) : 0u;
    s += (uint64_t)t[i] + pi;
    t[i] = (uint32_t)s;
    s >>= 32;
  }
  (void)s;
}

// limb i of a (i may be anything in [0, N]; N gives 0): a select chain, no indexed registers
template <int N>
ZG_INL uint32_t bg_limb(const uint32_t* a, int i) {
  uint32_t v = 0;
#pragma unroll
  for (int j = 0; j < N; j++) v = i == j ? a[j] : v;
  return v;
}

template <int N>
ZG_INL int bg_bitlen(const uint32_t* a) {
  int n = 0;
#pragma unroll
  for (int j = 0; j < N; j++) n = a[j] ? 32 * j + 32 - __builtin_clz(a[j]) : n;
  return n;
}

// 64 bits of a starting at bit `off` (0 <= off < 32 N)
template <int N>
ZG_INL uint64_t bg_bits64(const uint32_t* a, int off) {
  const int w = off >> 5, sh = off & 31;
  const uint64_t lo = bg_limb<N>(a, w), mid = bg_limb<N>(a, w + 1), hi = bg_limb<N>(a, w + 2);
  const uint64_t x = lo | (mid << 32);
  return sh ? (x >> sh) | (hi << (64 - sh)) : x;
}

// y^-1 mod p for a residue y in [0, p) (any representation: the caller fixes Montgomery factors).
// T outer steps of 30 divsteps each, T * 30 >= 2 len(p) - 1 (Fr: 17, Fq: 26). The update
// factors of one outer step stay within [-2^30, 2^30], so each pair (f, g) travels packed in one
// 64-bit word f + 2^32 g (the divsteps are linear in it) and is unpacked once per step.
template <class M, int T>
ZG_INL Fp<M> fp_inv_vt(const Fp<M>& y) {
  constexpr int N = M::N;
  constexpr int K = 30;
  uint32_t a[N], b[N], u[N], v[N];
#pragma unroll
  for (int i = 0; i < N; i++) {
    a[i] = y.l[i];
    b[i] = M::p(i);
    u[i] = i == 0 ? 1u : 0u;
    v[i] = 0;
  }
  for (int it = 0; it < T; it++) {
    int n = bg_bitlen<N>(a);
    const int nb = bg_bitlen<N>(b);
    n = n > nb ? n : nb;
    n = n > 64 ? n : 64;
    // low K bits and top 64 - K bits of a and b
    const uint64_t low = (1ull << K) - 1;
    uint64_t xa = ((uint64_t)a[0] & low) | (bg_bits64<N>(a, n - (64 - K)) << K);
    uint64_t xb = ((uint64_t)b[0] & low) | (bg_bits64<N>(b, n - (64 - K)) << K);
    uint64_t p0 = 1, p1 = 1ull << 32;  // (f0, g0) = (1, 0), (f1, g1) = (0, 1)
#pragma unroll 6
    for (int j = 0; j < K; j++) {
      const bool odd = xa & 1;
      const bool sw = odd && xa < xb;
      const uint64_t ta = sw ? xb : xa, tb = sw ? xa : xb;
      const uint64_t tp0 = sw ? p1 : p0, tp1 = sw ? p0 : p1;
      xa = (ta - (odd ? tb : 0)) >> 1;
      xb = tb;
      p0 = tp0 - (odd ? tp1 : 0);
      p1 = tp1 << 1;
    }
    int64_t f0 = (int32_t)(uint32_t)p0, f1 = (int32_t)(uint32_t)p1;
    int64_t g0 = ((int64_t)p0 - f0) >> 32, g1 = ((int64_t)p1 - f1) >> 32;
    // (a, b) <- ((a f0 + b g0) / 2^K, (a f1 + b g1) / 2^K), signs folded into the factors
    uint32_t na[N + 2], nb2[N + 2];
#pragma unroll
    for (int i = 0; i < N + 2; i++) na[i] = nb2[i] = 0;
    bg_mac<N>(na, a, (uint32_t)(f0 < 0 ? -f0 : f0), f0 < 0);
    bg_mac<N>(na, b, (uint32_t)(g0 < 0 ? -g0 : g0), g0 < 0);
    bg_mac<N>(nb2, a, (uint32_t)(f1 < 0 ? -f1 : f1), f1 < 0);
    bg_mac<N>(nb2, b, (uint32_t)(g1 < 0 ? -g1 : g1), g1 < 0);
    bg_shr<N, K>(na);
    bg_shr<N, K>(nb2);
    const bool fa = bg_neg_p<N>(na), fb = bg_neg_p<N>(nb2);
    bg_cneg<N>(na, fa);
    bg_cneg<N>(nb2, fb);
    f0 = fa ? -f0 : f0;
    g0 = fa ? -g0 : g0;
    f1 = fb ? -f1 : f1;
    g1 = fb ? -g1 : g1;
#pragma unroll
    for (int i = 0; i < N; i++) {
      a[i] = na[i];
      b[i] = nb2[i];
    }
    // (u, v) <- ((u f0 + v g0) / 2^K, (u f1 + v g1) / 2^K) mod p (Montgomery division): with
    // |f0| + |g0| <= 2^K and u, v < p the quotient lies in (-p, 2p)
    uint32_t nu[N + 2], nv[N + 2];
#pragma unroll
    for (int i = 0; i < N + 2; i++) nu[i] = nv[i] = 0;
    bg_mac<N>(nu, u, (uint32_t)(f0 < 0 ? -f0 : f0), f0 < 0);
    bg_mac<N>(nu, v, (uint32_t)(g0 < 0 ? -g0 : g0), g0 < 0);
    bg_mac<N>(nv, u, (uint32_t)(f1 < 0 ? -f1 : f1), f1 < 0);
    bg_mac<N>(nv, v, (uint32_t)(g1 < 0 ? -g1 : g1), g1 < 0);
    uint32_t pm[N];
#pragma unroll
    for (int i = 0; i < N; i++) pm[i] = M::p(i);
    bg_mac<N>(nu, pm, (nu[0] * M::INV) & (uint32_t)low, false);
    bg_mac<N>(nv, pm, (nv[0] * M::INV) & (uint32_t)low, false);
    bg_shr<N, K>(nu);
    bg_shr<N, K>(nv);
    bg_cadd_p<M>(nu, bg_neg_p<N>(nu), false);
    bg_cadd_p<M>(nv, bg_neg_p<N>(nv), false);
    {
      uint32_t tu[N + 2], tv[N + 2];
#pragma unroll
      for (int i = 0; i < N + 2; i++) {
        tu[i] = nu[i];
        tv[i] = nv[i];
      }
      bg_cadd_p<M>(tu, true, true);
      bg_cadd_p<M>(tv, true, true);
      const bool ku = !bg_neg_p<N>(tu), kv = !bg_neg_p<N>(tv);
#pragma unroll
      for (int i = 0; i < N; i++) {
        u[i] = ku ? tu[i] : nu[i];
        v[i] = kv ? tv[i] : nv[i];
      }
    }
  }
  // b == 1 unless y == 0 (then v == 0 too)
  Fp<M> r;
#pragma unroll
  for (int i = 0; i < N; i++) r.l[i] = v[i];
  return r;
}

// Montgomery-form inverse of a Montgomery-form Fr (public values): (a R)^-1 R^3 R^-1 = a^-1 R
ZG_INL Fr fr_inv_vt(const Fr& a) {
  Fr r3;
#pragma unroll
  for (int i = 0; i < 8; i++) r3.l[i] = FR_R3[i];
  return fr_mul(fp_inv_vt<FrM, ZG_INV_T_FR>(a), r3);
}

// Montgomery-form inverse of a Montgomery-form Fq: a fixed number of branch-free steps whatever
// the value (every lane of a wave runs the same instruction stream), so it also serves values
// derived from the secret batch scalars (the affine r_i A_i of the decode kernel).
ZG_NOINL inline Fq fq_inv(Fq a) {
  Fq r3;
#pragma unroll
  for (int i = 0; i < 12; i++) r3.l[i] = FQ_R3[i];
  return fq_mul(fp_inv_vt<FqM, ZG_INV_T_FQ>(a), r3);
}

}  // namespace zg
