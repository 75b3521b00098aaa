// zg_merkle.h -- the note-commitment tree hashes on gfx950: the two
// TreeHash::combine functions of storage/src/tree_state.rs, one lane per hash.
//
//   Sprout   sha256_compress(left, right)       crypto/src/lib.rs:188-198, tree_state.rs:175-177:
//            the SHA-256 compression of the one block left || right from the standard IV, no
//            padding, the state words written big-endian
//   Sapling  pedersen_hash(left, right, depth)  crypto/src/lib.rs:250-275, tree_state.rs:188-190:
//            sapling-crypto's Pedersen hash (not vendored; restated in oracle/merkle.py) of the
//            6 personalization bits MerkleTree(depth) then the 255 low bits of left and of
//            right (LE), the affine u coordinate written LE
//
// Pedersen on the GPU: the 516 input bits are 172 3-bit chunks, 63 per generator
// G_j = find_group_hash(LE32(j), "Zcash_PH"). Chunk i of a segment contributes
// enc(a, b, c) 2^(4 i) G_j with enc = (1 - 2c)(1 + a + 2b) in {+-1..+-4}. Since G_j has prime
// order r_J, summing the digits as integers instead of in Fs gives the same point, so two
// chunks at a time index a fixed table of (enc0 + 16 enc1) 2^(8 w) G_j (6-bit code, 64 entries
// per window, the last window of a full segment holds one chunk): 32 + 32 + 23 = 87 mixed
// additions with no doubling, then one inversion for the affine u. The table holds
// 3 x 32 x 64 niels points (y + x, y - x, 2 d x y), 96 B each (576 KiB, L2 resident), built on
// the device by k_ph_table on first use.
#pragma once
#include "../../include/zg.h"  // ZG_TREE_SPROUT / ZG_TREE_SAPLING
#include "zg_bingcd.h"
#include "zg_jubjub.h"

namespace zg {

#define ZG_PH_GENS 3
#define ZG_PH_WIN 32
#define ZG_PH_CODES 64
#define ZG_PH_WORDS 24  // y + x, y - x, 2 d x y (Montgomery Fr)
#define ZG_PH_POINTS (ZG_PH_GENS * ZG_PH_WIN * ZG_PH_CODES)
#define ZG_PH_TABLE_BYTES ((size_t)ZG_PH_POINTS * ZG_PH_WORDS * 4)

// The Pedersen additions multiply with the inlined product-scanning Montgomery product
// (fr29_mul: 29-bit digits, one carry-free v_mad_u64_u32 per digit product; round 1: fr_mul_fips)
// rather than the out-of-line fr_mul call: a hash
// group is a lone wave on a latency-bound chain of tree levels, so its time is the number of
// instructions it issues.
ZG_INL Fr ph_mul(const Fr& a, const Fr& b) {
#if ZG_FQ29
  Fr r;
  fr29_mul(r.l, a.l, b.l);  // 29-bit digits, one carry-free v_mad_u64_u32 per digit product (zg_fq29_gen.h)
  return r;
#elif defined(__HIP_DEVICE_COMPILE__)
  Fr r;
  fr_mul_fips(r.l, a.l, b.l);  // gfx950: v_mad_u64_u32 carry-out product scanning (zg_fips.h)
  return r;
#else
  return fp_mul_inl<FrM>(a, b);
#endif
}

// add-2008-hwcd-3 (a = -1, k = 2d), q given as a niels point (affine): 7 multiplications
ZG_INL JExt jx_add_niels(const JExt& p, const Fr& ypx, const Fr& ymx, const Fr& k) {
  const Fr A = ph_mul(fp_sub<FrM>(p.Y, p.X), ymx);
  const Fr B = ph_mul(fr_add(p.Y, p.X), ypx);
  const Fr C = ph_mul(p.T, k);
  const Fr D = fr_add(p.Z, p.Z);
  const Fr E = fp_sub<FrM>(B, A), F = fp_sub<FrM>(D, C), G = fr_add(D, C), H = fr_add(B, A);
  return {ph_mul(E, F), ph_mul(G, H), ph_mul(F, G), ph_mul(E, H)};
}
// add-2008-hwcd (a = -1), both extended: 9 multiplications (d folded into 2d T2 / 2 = d T2)
ZG_INL JExt ph_add(const JExt& p, const JExt& q) {
  const Fr A = ph_mul(p.X, q.X);
  const Fr B = ph_mul(p.Y, q.Y);
  const Fr C = ph_mul(ph_mul(p.T, q.T), jj_const(JUBJUB_D));
  const Fr D = ph_mul(p.Z, q.Z);
  const Fr E = fp_sub<FrM>(fp_sub<FrM>(ph_mul(fr_add(p.X, p.Y), fr_add(q.X, q.Y)), A), B);
  const Fr F = fp_sub<FrM>(D, C), G = fr_add(D, C), H = fr_add(B, A);
  return {ph_mul(E, F), ph_mul(G, H), ph_mul(F, G), ph_mul(E, H)};
}

// enc(a, b, c) of a 3-bit chunk (a = bit 0): (1 - 2c)(1 + a + 2b)
ZG_INL int ph_enc(uint32_t chunk) {
  const int m = 1 + (int)(chunk & 1u) + 2 * (int)((chunk >> 1) & 1u);
  return (chunk & 4u) ? -m : m;
}

// the personalized input of MerkleTree(depth): bit i of s (17 LE words, 516 bits used)
ZG_INL void ph_stream(const uint32_t* lw, const uint32_t* rw, int depth, uint32_t* s) {
#pragma unroll
  for (int i = 0; i < 17; i++) s[i] = 0;
  // bits 0..5 depth, 6..260 left bits 0..254, 261..515 right bits 0..254
  s[0] = (uint32_t)depth & 63u;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint32_t v = k == 7 ? (lw[k] & 0x7fffffffu) : lw[k];
    s[k] |= v << 6;
    s[k + 1] |= v >> 26;
  }
  // right starts at bit 261 = word 8, bit 5
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint32_t v = k == 7 ? (rw[k] & 0x7fffffffu) : rw[k];
    s[k + 8] |= v << 5;
    s[k + 9] |= v >> 27;
  }
}

// 17-way select: word k of the stream (k in [0, 17]; 17 gives 0) without indexed registers
ZG_INL uint32_t ph_word(const uint32_t* s, int k) {
  uint32_t v = 0;
#pragma unroll
  for (int j = 0; j < 17; j++) v = k == j ? s[j] : v;
  return v;
}

// Pedersen MerkleTree(depth) hash of two LE 256-bit words -> the canonical u coordinate, on a
// group of LANES consecutive lanes (all active, `sub` = the lane's index in the group):
// lane j adds the table points of windows j, j + 8, ... (11 of the 87), the 8 partial sums meet
// in a 3-round xor butterfly (full additions), and every lane of the group then holds the sum;
// the affine u = X / Z uses the binary-GCD inverse (public data). Only sub == 0 writes `out`.
// A lone wave's Fr product costs ~1.1 us (its ~450 VALU instructions at 4 cycles each), so a
// hash's latency is the instructions one lane runs: ceil(87 / LANES) niels additions plus
// log2(LANES) butterfly additions plus the inversion (8 lanes: 11 + 3; 32 lanes: 3 + 5). Wide
// groups shorten the latency-bound upper tree levels, narrow ones spend less on butterflies
// where a level has enough hashes to fill the chip (zg_merkle.hip picks per launch).
#define ZG_PH_LANES_NARROW 8
#define ZG_PH_LANES_WIDE 32
#define ZG_PH_WINDOWS 87
template <int LANES>
ZG_INL void ph_merkle(const uint32_t* lw, const uint32_t* rw, int depth, const uint32_t* table, int sub,
                      uint32_t* out) {
  uint32_t s[17];
  ph_stream(lw, rw, depth, s);
  JExt acc = jx_zero();
  for (int w = sub; w < ZG_PH_WINDOWS; w += LANES) {
    const int g = w >> 5, wi = w & 31;
    const int pos = 3 * (63 * g + 2 * wi);  // the window's first stream bit
    const int k = pos >> 5, sh = pos & 31;
    const uint32_t lo = ph_word(s, k), hi = ph_word(s, k + 1);
    const uint32_t code = ((lo >> sh) | (sh ? hi << (32 - sh) : 0u)) & (wi == ZG_PH_WIN - 1 ? 7u : 63u);
    const uint4* e = (const uint4*)(table + ((size_t)((g * ZG_PH_WIN + wi) * ZG_PH_CODES) + code) * ZG_PH_WORDS);
    Fr ypx, ymx, kk;
    const uint4 e0 = e[0], e1 = e[1], e2 = e[2], e3 = e[3], e4 = e[4], e5 = e[5];
    ypx.l[0] = e0.x, ypx.l[1] = e0.y, ypx.l[2] = e0.z, ypx.l[3] = e0.w;
    ypx.l[4] = e1.x, ypx.l[5] = e1.y, ypx.l[6] = e1.z, ypx.l[7] = e1.w;
    ymx.l[0] = e2.x, ymx.l[1] = e2.y, ymx.l[2] = e2.z, ymx.l[3] = e2.w;
    ymx.l[4] = e3.x, ymx.l[5] = e3.y, ymx.l[6] = e3.z, ymx.l[7] = e3.w;
    kk.l[0] = e4.x, kk.l[1] = e4.y, kk.l[2] = e4.z, kk.l[3] = e4.w;
    kk.l[4] = e5.x, kk.l[5] = e5.y, kk.l[6] = e5.z, kk.l[7] = e5.w;
    acc = jx_add_niels(acc, ypx, ymx, kk);
  }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
  for (int m = 1; m < LANES; m <<= 1) {
    JExt o;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      o.X.l[i] = (uint32_t)__shfl_xor((int)acc.X.l[i], m);
      o.Y.l[i] = (uint32_t)__shfl_xor((int)acc.Y.l[i], m);
      o.Z.l[i] = (uint32_t)__shfl_xor((int)acc.Z.l[i], m);
      o.T.l[i] = (uint32_t)__shfl_xor((int)acc.T.l[i], m);
    }
    acc = ph_add(acc, o);
  }
#endif
  if (sub) return;
  const Fr x = fr_from_mont(fr_mul(acc.X, fr_inv_vt(acc.Z)));
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = x.l[i];
}

// ---- SHA-256 compression of one 64-byte block (no padding), FIPS 180-4 section 6.2.2
__device__ __constant__ const uint32_t ZG_SHA256_K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

__device__ __forceinline__ uint32_t sha_rotr(uint32_t x, int k) { return (x >> k) | (x << (32 - k)); }

// lw, rw: the 32 + 32 message bytes as LE words (byte order of H256); out likewise
__device__ __forceinline__ void sha256_compress_words(const uint32_t* lw, const uint32_t* rw, uint32_t* out) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    w[i] = __builtin_bswap32(lw[i]);
    w[8 + i] = __builtin_bswap32(rw[i]);
  }
  const uint32_t iv[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                          0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  uint32_t a = iv[0], b = iv[1], c = iv[2], d = iv[3], e = iv[4], f = iv[5], g = iv[6], h = iv[7];
#pragma unroll
  for (int t = 0; t < 64; t++) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
      const uint32_t s0 = sha_rotr(w15, 7) ^ sha_rotr(w15, 18) ^ (w15 >> 3);
      const uint32_t s1 = sha_rotr(w2, 17) ^ sha_rotr(w2, 19) ^ (w2 >> 10);
      wt = w[t & 15] = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
    }
    const uint32_t t1 = h + (sha_rotr(e, 6) ^ sha_rotr(e, 11) ^ sha_rotr(e, 25)) + ((e & f) ^ (~e & g)) +
                        ZG_SHA256_K[t] + wt;
    const uint32_t t2 = (sha_rotr(a, 2) ^ sha_rotr(a, 13) ^ sha_rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  out[0] = __builtin_bswap32(iv[0] + a);
  out[1] = __builtin_bswap32(iv[1] + b);
  out[2] = __builtin_bswap32(iv[2] + c);
  out[3] = __builtin_bswap32(iv[3] + d);
  out[4] = __builtin_bswap32(iv[4] + e);
  out[5] = __builtin_bswap32(iv[5] + f);
  out[6] = __builtin_bswap32(iv[6] + g);
  out[7] = __builtin_bswap32(iv[7] + h);
}

// LANES lanes per hash: Pedersen on a group (8 or 32), SHA-256 on one lane (LANES = 1)
template <int KIND, int LANES>
ZG_INL void tree_combine(const uint32_t* l, const uint32_t* r, int depth, const uint32_t* table, int sub,
                         uint32_t* out) {
  uint32_t lw[8], rw[8];
  const uint4* l4 = (const uint4*)l;
  const uint4* r4 = (const uint4*)r;
  const uint4 a0 = l4[0], a1 = l4[1], b0 = r4[0], b1 = r4[1];
  lw[0] = a0.x, lw[1] = a0.y, lw[2] = a0.z, lw[3] = a0.w, lw[4] = a1.x, lw[5] = a1.y, lw[6] = a1.z, lw[7] = a1.w;
  rw[0] = b0.x, rw[1] = b0.y, rw[2] = b0.z, rw[3] = b0.w, rw[4] = b1.x, rw[5] = b1.y, rw[6] = b1.z, rw[7] = b1.w;
  uint32_t o[8];
  if (KIND == ZG_TREE_SPROUT) {
    sha256_compress_words(lw, rw, o);
  } else {
    ph_merkle<LANES>(lw, rw, depth, table, sub, o);
    if (sub) return;
  }
  uint4* o4 = (uint4*)out;
  o4[0] = make_uint4(o[0], o[1], o[2], o[3]);
  o4[1] = make_uint4(o[4], o[5], o[6], o[7]);
}

// ---- one level of the window algorithm (zg_merkle.hip): the nodes of a tree level as held on
// the device. Node i of the level: i >= base -> w[i - base] (i - base < cnt, else the level's
// empty root), i == base - 1 -> f1, i == base - 2 -> f2 (frontier slots of the input state).
struct TreeLevel {
  const uint32_t* w;
  long long base, cnt;
  const uint32_t* f1;
  const uint32_t* f2;
  const uint32_t* empty;
};

ZG_INL const uint32_t* tree_node(const TreeLevel& L, long long i) {
  if (i >= L.base) return i - L.base < L.cnt ? L.w + 8 * (i - L.base) : L.empty;
  return i == L.base - 1 ? L.f1 : L.f2;
}

}  // namespace zg
