// zg_pghr13.hip -- PGHR13 Sprout proofs on BN254: the kernels and the
// host side of zg_pghr13_verify / zg_bn254_pairing.
//
// Reference: crypto/src/pghr13.rs:69-105 (Proof::from_raw, verify), called per PHGR JoinSplit by
// verification/src/sprout.rs:61-67. verify checks five pairing equalities; here, per proof, the five
// are folded into one product with random 128-bit weights rho_1..rho_5:
//
//   e(a, A) e(P1', P2) e(rho3 c, C) e(rho4 k, G) e(P5, GB2) e(P6, Z) e(P7, b) == 1
//   P1' = -(rho1 a' + rho2 b' + rho3 c' + rho5 c)     P5 = -rho4 (acc + a + c)     P6 = -rho5 h
//   (and P0 = rho1 a: with rho1 random too, one proof's check and the batch's share its operands)
//   P7  = rho2 vk.b - rho4 gammaBeta1 + rho5 (acc + a)
//
// which holds for all rho iff each equality holds (a false proof passes with probability
// ~2^-128 over the rho, drawn from getrandom(2) per call). A call is decided by ONE check: the six
// key pairs on the batch's operand sums, the proofs' own b pairs, one final exponentiation; only a
// failing call runs the per-proof path (one 7-pair multi-Miller loop + final exponentiation each).
//
//   key (once per device): k_bn_vk (points, AffineG1/G2::new checks), k_bn_lines (the 6 fixed G2
//     points' lines), k_bn_comb (byte-window combs of ic[], vk.b, gammaBeta1)
//   main stream: k_pghr_decode_g1 (wave per point), k_pghr_accp (input combs), k_pghr_prep
//     (statuses, acc), k_pghr_g2status, k_pghr_straus (the key pairs' operand sums, Straus over the
//     GLV halves), k_pghr_ssum / k_pghr_bsum_final, k_pghr_bseg
//     (every pair of the batch by loop segment), k_bn_tree (per-segment products), k_pghr_segcopy,
//     k_fe_easy, k_pghr_fe_coop (one wave)
//   side stream: k_pghr_decode_g2 (Fq2 sqrt + G2 membership), k_pghr_blines (b's lines -> HBM) and
//     k_pghr_p7 (the b pairs' operands), concurrent with the G1 chain and the Straus sums
//   per-proof path (a failing batch): k_pghr_rho + k_pghr_combine (every P_i), k_pghr_miller,
//     k_fe_easy, k_fe_exp<1..3>, k_fe_last
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <utility>
#include <string>
#include <vector>

#include "../../include/zg.h"
#include "zg_bn254.h"

namespace zg {

#define ZG_BN_MAX_IC 16
#define ZG_BN_FIXED_Q 6  // vk.a, P2 (G2::one), vk.c, vk.gamma, vk.gamma_beta_2, vk.z
#define ZG_BN_NLINES 102  // 64 doublings + 36 additions (popcount of the low 64 bits of 6u + 2) + 2
constexpr int bn_lines_needed() {
  int n = 2;  // the pi(Q), -pi^2(Q) steps
  for (int i = ZG_BN_ATE_BITS - 2; i >= 0; i--) n += 1 + (int)((BN_ATE[i >> 5] >> (i & 31)) & 1u);
  return n;
}
static_assert(bn_lines_needed() <= ZG_BN_NLINES, "line table rows");
#define ZG_BN_COMB_BASES (ZG_BN_MAX_IC + 2)
#define ZG_BN_COMB_W 32
#define ZG_BN_COMB_D 255
#define ZG_BN_PTS 7

struct BnVK {
  BA2 q[ZG_BN_FIXED_Q];  // a, P2, c, gamma, gamma_beta_2, z
  BA1 b, gb1;
  BA1 ic[ZG_BN_MAX_IC];
  int ic_len;
  int err;  // 0 ok, 1 a point is not on its curve / not of order r
};

// canonical big-endian words (the host's JSON) -> Montgomery points, with the bn crate's checks
__global__ void k_bn_vk(const uint32_t* raw, int ic_len, BnVK* vk) {
  if (blockIdx.x | threadIdx.x) return;
  // raw layout (each Fq 8 LE words, canonical): 5 G2 (x.c0, x.c1, y.c0, y.c1), b, gb1, ic[ic_len]
  int err = 0;
  auto fq = [&](int w) { return bq_to_mont(bq_c(raw + 8 * w)); };
  for (int k = 0; k < 5; k++) {  // a, c, gamma, gb2, z into q[0], q[2..5]
    BA2 q = {{fq(4 * k), fq(4 * k + 1)}, {fq(4 * k + 2), fq(4 * k + 3)}};
    if (!ba2_on_curve(q) || !ba2_in_subgroup(q)) err = 1;
    vk->q[k == 0 ? 0 : k + 1] = q;
  }
  vk->q[1] = {b2_c(BN_G2_X), b2_c(BN_G2_Y)};
  int w = 20;
  auto g1 = [&]() {
    BA1 p = {fq(w), fq(w + 1), false};
    w += 2;
    if (!ba1_on_curve(p)) err = 1;
    return p;
  };
  vk->b = g1();
  vk->gb1 = g1();
  for (int i = 0; i < ic_len; i++) vk->ic[i] = g1();
  vk->ic_len = ic_len;
  vk->err = err;
}

// the lines of fixed point j in Miller-loop order: per bit (top excluded) a doubling line, then
// an addition line when the bit is set; then the pi(Q) and -pi^2(Q) lines
__global__ void __launch_bounds__(64) k_bn_lines(const BnVK* vk, BLine* lines) {
  const int j = threadIdx.x;
  if (blockIdx.x || j >= ZG_BN_FIXED_Q) return;
  const BA2 q = vk->q[j];
  BH2 t = {q.x, q.y, b2_one()};
  BLine* o = lines + (size_t)j * ZG_BN_NLINES;
  int n = 0;
  for (int i = ZG_BN_ATE_BITS - 2; i >= 0; i--) {
    o[n++] = bh2_dbl_step(&t);
    if (bn_ate_bit(i)) o[n++] = bh2_add_step(&t, q);
  }
  const BA2 q1 = ba2_frob(q), q2 = ba2_frob2(q);
  o[n++] = bh2_add_step(&t, q1);
  o[n++] = bh2_add_step(&t, {q2.x, b2_neg(q2.y)});
}

// comb tables: entry (base, w, d) = d 2^(8 w) base, affine Montgomery (x, y), 16 words
__global__ void __launch_bounds__(64) k_bn_comb(const BnVK* vk, uint32_t* table) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ZG_BN_COMB_BASES * ZG_BN_COMB_W * ZG_BN_COMB_D) return;
  const int d = t % ZG_BN_COMB_D + 1, w = (t / ZG_BN_COMB_D) % ZG_BN_COMB_W, base = t / (ZG_BN_COMB_D * ZG_BN_COMB_W);
  BA1 p = {bq_zero(), bq_zero(), true};
  if (base < vk->ic_len)
    p = vk->ic[base];
  else if (base == ZG_BN_MAX_IC)
    p = vk->b;
  else if (base == ZG_BN_MAX_IC + 1)
    p = vk->gb1;
  uint32_t k[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int bit = 8 * w;
  k[bit >> 5] = (uint32_t)d << (bit & 31);
  const BA1 r = p.inf ? p : bj1_to_aff(bj1_mul(p, k, 256));
  uint32_t* e = table + (size_t)t * 16;
  for (int l = 0; l < 8; l++) {
    e[l] = r.inf ? 0u : r.x.l[l];
    e[8 + l] = r.inf ? 0u : r.y.l[l];
  }
}

// [s] base_j from the comb table (s: nbytes little-endian bytes)
// phi: the table's points mapped by the G1 endomorphism (beta x, y), i.e. [s lambda] of the base
ZG_INL BJ1 bn_comb_mul(BJ1 acc, const uint32_t* comb, int base, const uint8_t* s, int nbytes, bool phi = false) {
  for (int w = 0; w < nbytes; w++) {
    const int d = s[w];
    if (!d) continue;
    const uint32_t* e = comb + ((size_t)(base * ZG_BN_COMB_W + w) * ZG_BN_COMB_D + (d - 1)) * 16;
    BA1 p;
    for (int l = 0; l < 8; l++) {
      p.x.l[l] = e[l];
      p.y.l[l] = e[8 + l];
    }
    p.inf = false;
    if (phi) p.x = bq_mul(p.x, bq_c(BQ_BETA));
    acc = bj1_add_aff(acc, p);
  }
  return acc;
}

#define ZG_PGHR_DEC 9
struct PghrPts {  // per proof, written by k_pghr_combine
  BA1 p[ZG_BN_PTS];
  BA2 qb;
};

// the proof's points as decoded, acc + a and acc + a + c (k_pghr_prep -> k_pghr_rho / k_pghr_combine)
struct PghrDec {
  BA1 pt[ZG_PGHR_DEC];  // a, a', b', c, c', k, h, acc + a, acc + a + c
  BA2 qb;
};

// Proof::from_raw's point decodes: the seven G1 points one per one-wave block (grid y; 64 proofs;
// bytes a 0, a' 33, b' 131, c 164, c' 197, k 230, h 263) and the G2 point b (bytes 66..130: the
// Fq2 square root and the G2 membership test, far heavier) in a launch of its own, lane per proof,
// so the light waves do not hold a block open behind it -> dec, verdicts -> okb[8 i + w] (w = 2: b).
__device__ __constant__ const int16_t PGHR_DEC_OFF[7] = {0, 33, 131, 164, 197, 230, 263};
__device__ __constant__ const int8_t PGHR_DEC_OK[7] = {0, 1, 3, 4, 5, 6, 7};
__global__ void __launch_bounds__(64) k_pghr_decode_g1(int n, const uint8_t* proofs, PghrDec* dec, uint8_t* okb) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  const int w = blockIdx.y;  // slot w of dec.pt
  if (i >= n) return;
  BA1 a;
  const bool ok = bn_g1_decode(proofs + (size_t)296 * i + PGHR_DEC_OFF[w], &a);
  if (ok) dec[i].pt[w] = a;
  okb[8 * (size_t)i + PGHR_DEC_OK[w]] = ok;
}
__global__ void __launch_bounds__(64) k_pghr_decode_g2(int n, const uint8_t* proofs, PghrDec* dec, uint8_t* okb) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  BA2 q;
  const bool ok = bn_g2_decode(proofs + (size_t)296 * i + 66, &q);
  if (ok) dec[i].qb = q;
  okb[8 * (size_t)i + 2] = ok;
}

// x_j ic_{j+1} for the nine input slots, one per one-wave block (grid y; byte-window combs, 32
// mixed additions each) -> accp[9 i + j] (infinity past the proof's input count); canonicity is
// k_pghr_prep's
__global__ void __launch_bounds__(64) k_pghr_accp(int n, const uint8_t* inputs, const uint8_t* ninputs,
                                                   const BnVK* vk, const uint32_t* comb, BJ1* accp) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  const int j = blockIdx.y;
  if (i >= n) return;
  int cnt = ninputs ? ninputs[i] : 9;
  cnt = cnt < vk->ic_len - 1 ? cnt : vk->ic_len - 1;
  BJ1 r = bj1_inf();
  if (j < cnt) r = bn_comb_mul(r, comb, j + 1, inputs + (size_t)9 * 32 * i + 32 * j, 32);
  accp[9 * (size_t)i + j] = r;
}

// lane per proof: the statuses in the reference's order (a failed decode, then a non-canonical
// input), acc = ic0 + the nine comb products, acc + a and acc + a + c
__global__ void __launch_bounds__(64) k_pghr_prep(int n, const uint8_t* inputs, const uint8_t* ninputs,
                                                   const BnVK* vk, const uint8_t* okb, const BJ1* accp,
                                                   PghrDec* dec, uint8_t* status) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool ok = true;  // b's verdict (okb[8 i + 2]) joins in k_pghr_g2status: its decode runs concurrently
  for (int w = 0; w < 8; w++) ok = ok && (w == 2 || okb[8 * (size_t)i + w]);
  if (!ok) {
    status[i] = ZG_STATUS_DECODE_INVALID;
    return;
  }
  // acc = ic0 + sum x_j ic_{j+1} over min(count, ic_len - 1) inputs (the reference's zip)
  int cnt = ninputs ? ninputs[i] : 9;
  cnt = cnt < vk->ic_len - 1 ? cnt : vk->ic_len - 1;
  const uint8_t* xin = inputs + (size_t)9 * 32 * i;
  BJ1 acc = bj1_from(vk->ic[0]);
  for (int j = 0; j < cnt; j++) {
    Bq x;
    for (int l = 0; l < 8; l++)
      x.l[l] = (uint32_t)xin[32 * j + 4 * l] | ((uint32_t)xin[32 * j + 4 * l + 1] << 8) |
               ((uint32_t)xin[32 * j + 4 * l + 2] << 16) | ((uint32_t)xin[32 * j + 4 * l + 3] << 24);
    uint64_t br = 0;  // x < r (bn::Fr)
    for (int l = 0; l < 8; l++) {
      const uint64_t d = (uint64_t)x.l[l] - BN_R[l] - br;
      br = (d >> 63) & 1u;
    }
    if (!br) {
      status[i] = ZG_STATUS_INPUT_NONCANONICAL;
      return;
    }
    acc = bj1_add(acc, accp[9 * (size_t)i + j]);
  }
  PghrDec& o = dec[i];
  const BA1 a = o.pt[0], c = o.pt[3];
  const BA1 acca = bj1_to_aff(acc);
  const BA1 aa = ba1_add(acca, a);  // acc + a
  o.pt[7] = aa;
  o.pt[8] = ba1_add(aa, c);  // acc + a + c
  status[i] = ZG_STATUS_OK;
}

// after k_pghr_decode_g2 (its own stream, concurrent with the G1 decodes, prep and rho): a proof
// whose b failed to decode is DECODE_INVALID -- which precedes the input check, so it overrides
// prep's INPUT_NONCANONICAL as well as OK (the reference's order)
__global__ void __launch_bounds__(64) k_pghr_g2status(int n, const uint8_t* okb, uint8_t* status) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && !okb[8 * (size_t)i + 2]) status[i] = ZG_STATUS_DECODE_INVALID;
}

// the ten products rho_j Q of a proof, one per wave of a 640-lane block (64 proofs): wave w computes
// PGHR_RHO_MUL[w] = (point, rho index), affine, -> mul[10 i + w]. A weight is rho = a + b lambda mod r
// for its 16 random bytes a (LE 0..7), b (8..15) -- 2^128 distinct values (zg_bn254.h bj1_mul_glv) --
// so each product is a 64-bit joint double-and-add over q and phi(q).
#define ZG_PGHR_RHO_BYTES 80  // rho2, rho3, rho4, rho5, rho1: (a, b) 16 LE bytes each
#define ZG_PGHR_NMUL 10
__device__ __constant__ const int8_t PGHR_RHO_MUL[ZG_PGHR_NMUL][2] = {
    {2, 0},  // rho2 b'
    {4, 1},  // rho3 c'
    {3, 3},  // rho5 c
    {3, 1},  // rho3 c
    {5, 2},  // rho4 k
    {8, 2},  // rho4 (acc + a + c)
    {6, 3},  // rho5 h
    {7, 3},  // rho5 (acc + a)
    {0, 4},  // rho1 a
    {1, 4},  // rho1 a'
};
__global__ void __launch_bounds__(64 * ZG_PGHR_NMUL) k_pghr_rho(int n, const PghrDec* dec, const uint8_t* rho,
                                                                const uint8_t* status, BA1* mul) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;  // wave-uniform
  if (i >= n || status[i] != ZG_STATUS_OK) return;
  const int pj = PGHR_RHO_MUL[w][0], rj = PGHR_RHO_MUL[w][1];
  const uint8_t* r = rho + (size_t)ZG_PGHR_RHO_BYTES * i + 16 * rj;
  uint32_t rw[4];
  for (int l = 0; l < 4; l++)
    rw[l] = (uint32_t)r[4 * l] | ((uint32_t)r[4 * l + 1] << 8) | ((uint32_t)r[4 * l + 2] << 16) |
            ((uint32_t)r[4 * l + 3] << 24);
  const BA1 q = dec[i].pt[pj];
  mul[ZG_PGHR_NMUL * (size_t)i + w] = q.inf ? q : bj1_to_aff(bj1_mul_glv(q, rw));
}

// lane per proof: the seven G1 operands of the folded check from the products
//   P1' = -(rho1 a' + rho2 b' + rho3 c' + rho5 c)     P5 = -rho4 (acc + a + c)     P6 = -rho5 h
//   (and P0 = rho1 a: with rho1 random too, one proof's check and the batch's share its operands)
//   P7  = rho2 vk.b - rho4 gammaBeta1 + rho5 (acc + a)          (vk.b, gammaBeta1: comb tables)
__global__ void __launch_bounds__(64) k_pghr_combine(int n, const PghrDec* dec, const BA1* mul, const uint8_t* rho,
                                                      const uint32_t* comb, const uint8_t* status, PghrPts* pts) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || status[i] != ZG_STATUS_OK) return;
  const PghrDec& d = dec[i];
  const BA1* m = mul + ZG_PGHR_NMUL * (size_t)i;
  const uint8_t* r = rho + (size_t)ZG_PGHR_RHO_BYTES * i;
  PghrPts& o = pts[i];
  o.p[0] = m[8];  // rho1 a
  BJ1 s = bj1_from(m[9]);  // rho1 a'
  s = bj1_add_aff(s, m[0]);
  s = bj1_add_aff(s, m[1]);
  s = bj1_add_aff(s, m[2]);
  o.p[1] = ba1_neg(bj1_to_aff(s));
  o.p[2] = m[3];
  o.p[3] = m[4];
  o.p[4] = d.pt[8].inf ? d.pt[8] : ba1_neg(m[5]);
  o.p[5] = ba1_neg(m[6]);
  // rho G = a G + b phi(G) for the comb tables' fixed G: the halves' byte windows, phi on the b half
  BJ1 t = bn_comb_mul(bn_comb_mul(bj1_inf(), comb, ZG_BN_MAX_IC, r, 8), comb, ZG_BN_MAX_IC, r + 8, 8, true);
  const BA1 g4 = bj1_to_aff(
      bn_comb_mul(bn_comb_mul(bj1_inf(), comb, ZG_BN_MAX_IC + 1, r + 32, 8), comb, ZG_BN_MAX_IC + 1, r + 40, 8, true));
  t = bj1_add_aff(t, ba1_neg(g4));
  if (!d.pt[7].inf) t = bj1_add_aff(t, m[7]);
  o.p[6] = bj1_to_aff(t);
  o.qb = d.qb;
}

// ---- the batch path's G1 operands without the nine per-proof products that only feed sums.
// Of the ten weighted products of a proof, nine enter the batch check only through the six key pairs'
// operand sums S_j = sum_i P_ij (the per-proof path's P_i0..P_i5), so k_pghr_straus forms those sums directly: lane
// (family f, group g) carries the B proofs g, g + G, .. (G = ceil(n / B)) and computes
// sum_k [a_k + b_k lambda] q_k as ONE joint double-and-add -- 64 doublings shared by its B proofs,
// each adding q, phi(q) or q + phi(q) by its two bits (Straus' interleaving over the GLV halves)
// instead of 64 doublings per product. Only the b pair's operand P_i7 (one product per proof,
// k_pghr_p7) stays per proof; a failing batch's per-proof path forms every P_i (k_pghr_rho, combine).
// family: (point, weight, sum, negated): the PGHR_RHO_MUL rows but {7, 3} (P7's)
#define ZG_PGHR_NFAM 9
__device__ __constant__ const int8_t PGHR_FAM[ZG_PGHR_NFAM][4] = {
    {2, 0, 1, 1},  // rho2 b'           -> -S1
    {4, 1, 1, 1},  // rho3 c'           -> -S1
    {3, 3, 1, 1},  // rho5 c            -> -S1
    {1, 4, 1, 1},  // rho1 a'           -> -S1
    {3, 1, 2, 0},  // rho3 c            ->  S2
    {5, 2, 3, 0},  // rho4 k            ->  S3
    {8, 2, 4, 1},  // rho4 (acc + a + c) -> -S4
    {6, 3, 5, 1},  // rho5 h            -> -S5
    {0, 4, 0, 0},  // rho1 a            ->  S0
};
ZG_INL void pghr_rho_words(const uint8_t* r, uint32_t* rw) {
  for (int l = 0; l < 4; l++)
    rw[l] = (uint32_t)r[4 * l] | ((uint32_t)r[4 * l + 1] << 8) | ((uint32_t)r[4 * l + 2] << 16) |
            ((uint32_t)r[4 * l + 3] << 24);
}
// grid (ceil(G / 64), families) -> part[f G + g] (Jacobian; infinity where no proof of the lane is OK)
template <int B>
__global__ void __launch_bounds__(64) k_pghr_straus(int n, const PghrDec* dec, const uint8_t* rho,
                                                     const uint8_t* status, BJ1* part) {
  const int g = blockIdx.x * 64 + threadIdx.x, f = blockIdx.y, G = (n + B - 1) / B;
  if (g >= G) return;
  const int pj = PGHR_FAM[f][0], rj = PGHR_FAM[f][1];
  BA1 q[B], s[B];
  uint32_t rw[B][4];
#pragma unroll
  for (int k = 0; k < B; k++) {
    const int i = g + k * G;
    q[k] = {bq_zero(), bq_zero(), true};
    if (i < n && status[i] == ZG_STATUS_OK) q[k] = dec[i].pt[pj];
    pghr_rho_words(rho + (size_t)ZG_PGHR_RHO_BYTES * (q[k].inf ? 0 : i) + 16 * rj, rw[k]);
    s[k] = q[k].inf ? q[k] : ba1_add(q[k], ba1_phi(q[k]));  // != O: phi(q) = -q would need lambda = -1
  }
  BJ1 acc = bj1_inf();
  for (int b = 63; b >= 0; b--) {
    acc = bj1_dbl(acc);
#pragma unroll
    for (int k = 0; k < B; k++) {
      if (q[k].inf) continue;
      const uint32_t ba = (rw[k][b >> 5] >> (b & 31)) & 1u, bb = (rw[k][2 + (b >> 5)] >> (b & 31)) & 1u;
      if (ba | bb) acc = bj1_add_aff(acc, ba & bb ? s[k] : ba ? q[k] : ba1_phi(q[k]));
    }
  }
  part[(size_t)f * G + g] = acc;
}
// sum j's entries are the G partials of each of its families; block (j, c) adds entries
// [c CH, (c + 1) CH) of that list (64 lanes strided, then an LDS tree), negated for the negated sums
// -> part1[c * 6 + j] (infinity past the list): k_pghr_bsum_final's input layout
#define ZG_PGHR_SSUM_CH 1024
__global__ void __launch_bounds__(64) k_pghr_ssum(int G, const BJ1* part, BJ1* part1) {
  __shared__ BJ1 sh[64];
  const int j = blockIdx.x, c = blockIdx.y, t = threadIdx.x;
  int fam[4], nf = 0;
  bool neg = false;
  for (int f = 0; f < ZG_PGHR_NFAM; f++)
    if (PGHR_FAM[f][2] == j) {
      fam[nf++] = f;
      neg = PGHR_FAM[f][3];
    }
  const long long len = (long long)nf * G, e0 = (long long)c * ZG_PGHR_SSUM_CH;
  BJ1 acc = bj1_inf();
  for (long long e = e0 + t; e < e0 + ZG_PGHR_SSUM_CH && e < len; e += 64)
    acc = bj1_add(acc, part[(size_t)fam[e / G] * G + (size_t)(e % G)]);
  sh[t] = acc;
  __syncthreads();
  for (int d = 32; d >= 1; d >>= 1) {
    if (t < d) sh[t] = bj1_add(sh[t], sh[t + d]);
    __syncthreads();
  }
  if (t == 0) {
    BJ1 r = sh[0];
    if (neg) r.Y = bq_neg(r.Y);
    part1[(size_t)c * ZG_BN_FIXED_Q + j] = r;
  }
}
// lane per proof: P_i7 = rho2 vk.b - rho4 gammaBeta1 + rho5 (acc + a) (k_pghr_combine's, with the
// one variable-base product here) and b -> pts[i].p[6], pts[i].qb
__global__ void __launch_bounds__(64) k_pghr_p7(int n, const PghrDec* dec, const uint8_t* rho, const uint32_t* comb,
                                                 const uint8_t* status, PghrPts* pts) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || status[i] != ZG_STATUS_OK) return;
  const PghrDec& d = dec[i];
  const uint8_t* r = rho + (size_t)ZG_PGHR_RHO_BYTES * i;
  uint32_t rw[4];
  pghr_rho_words(r + 16 * 3, rw);  // rho5
  BJ1 t = bn_comb_mul(bn_comb_mul(bj1_inf(), comb, ZG_BN_MAX_IC, r, 8), comb, ZG_BN_MAX_IC, r + 8, 8, true);
  const BA1 g4 = bj1_to_aff(
      bn_comb_mul(bn_comb_mul(bj1_inf(), comb, ZG_BN_MAX_IC + 1, r + 32, 8), comb, ZG_BN_MAX_IC + 1, r + 40, 8, true));
  t = bj1_add_aff(t, ba1_neg(g4));
  if (!d.pt[7].inf) t = bj1_add(t, bj1_mul_glv(d.pt[7], rw));
  pts[i].p[6] = bj1_to_aff(t);
  pts[i].qb = d.qb;
}
// B by size: enough (family, group) lanes for ~2 waves per SIMD, the rest as shared doublings (B = 4
// keeps its 4 x 3 points in scratch)
static int straus_b(size_t n) {
  static const int forced = getenv("ZG_STRAUS_B") ? atoi(getenv("ZG_STRAUS_B")) : 0;
  if (forced == 1 || forced == 2 || forced == 4) return forced;
  return n >= 28672 ? 2 : 1;  // 64k: B = 1 / 2 / 4 28.6 / 28.1 / 30.0 ms (profiles/r03s5_pghr13_bench.txt)
}

// the multi-Miller loop of one proof's 7 pairs, split over two waves of a 128-lane block (the same
// 64 proofs): wave 0 carries pairs 0..3 (fixed G2 points), wave 1 pairs 4, 5 and the proof's own b
// (its doubling / addition steps), each with its own accumulator (one extra Fq12 squaring per step),
// so a small batch fills twice the SIMDs (8,192 proofs: 87 -> 49 ms for the whole check). The
// kernel holds ~460 VGPRs (one wave per SIMD), so from 32,768 proofs -- as many waves as SIMDs --
// one wave per proof carries all seven pairs (halves 1: the split only adds a squaring per step).
// fout[halves i + h] = half h's product; k_fe_easy multiplies the two.
#define ZG_PGHR_SPLIT 4  // pairs [0, SPLIT) on wave 0
#define ZG_PGHR_SPLIT_BELOW 32768  // batches of fewer proofs run the two-wave split
__global__ void __launch_bounds__(128) k_pghr_miller(int n, const PghrPts* pts, const BLine* lines,
                                                      const uint8_t* status, Bq12* fout, int halves) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int h = threadIdx.x >> 6;  // wave-uniform
  if (i >= n || status[i] != ZG_STATUS_OK) return;
  const PghrPts& P = pts[i];
  // halves 1 (64-lane blocks): wave 0 alone carries all seven pairs
  const bool own_b = halves == 1 || h == 1;
  const int j0 = h ? ZG_PGHR_SPLIT : 0, j1 = (h || halves == 1) ? ZG_BN_FIXED_Q : ZG_PGHR_SPLIT;
  BA2 qb;
  BH2 t;
  if (own_b) {
    qb = P.qb;
    t = {qb.x, qb.y, b2_one()};
  }
  Bq12 f = b12_one();
  int li = 0;
  for (int bit = ZG_BN_ATE_BITS - 2; bit >= -2; bit--) {
    // bit >= 0: a doubling step (+ an addition when set); -1, -2: the pi(Q), -pi^2(Q) additions
    const int nsub = bit >= 0 ? (bn_ate_bit(bit) ? 2 : 1) : 1;
    if (bit >= 0) f = b12_sqr(f);
    for (int s = 0; s < nsub; s++, li++) {
      for (int j = j0; j < j1; j++) {
        const BA1 p = P.p[j];
        if (p.inf) continue;
        f = b12_mul_bline(f, lines[(size_t)j * ZG_BN_NLINES + li], p);
      }
      if (!own_b) continue;
      BLine l;
      if (bit >= 0)
        l = s == 0 ? bh2_dbl_step(&t) : bh2_add_step(&t, qb);
      else if (bit == -1)
        l = bh2_add_step(&t, ba2_frob(qb));
      else {
        const BA2 q2 = ba2_frob2(qb);
        l = bh2_add_step(&t, {q2.x, b2_neg(q2.y)});
      }
      if (!P.p[6].inf) f = b12_mul_bline(f, l, P.p[6]);
    }
  }
  fout[(size_t)halves * i + h] = f;
}

// ---- the batch check (one final exponentiation for the whole call). The per-proof check is
//   prod_j e(P_ij, Q_j) = 1 with six fixed Q_j (the key's G2 points) and Q_7 = b_i (the proof's);
// with every weight rho random (rho1 too) the product over proofs of the per-proof checks is
//   prod_{j<6} e(sum_i P_ij, Q_j) * prod_i e(P_i7, b_i)
// -- six Miller loops for the batch, one single-pair loop per proof, ONE final exponentiation -- and
// it equals 1 iff every proof's five equalities hold, but for a probability <= 2^-128 per false
// one (each equality of each proof carries its own independent 128-bit weight). A batch that fails
// re-runs the per-proof path (k_pghr_miller + k_fe_*) for the exact statuses.
// block j of six: sum_i P_ij over the nb chunk partials of k_pghr_ssum (lanes stride, then an LDS
// tree) -> agg->p[j];
// agg->p[6] = infinity (the aggregate has no b pair)
__global__ void __launch_bounds__(64) k_pghr_bsum_final(int nb, const BJ1* part, PghrPts* agg) {
  __shared__ BJ1 sh[64];
  const int j = blockIdx.x, t = threadIdx.x;
  BJ1 acc = bj1_inf();
  for (int b = t; b < nb; b += 64) acc = bj1_add(acc, part[(size_t)b * ZG_BN_FIXED_Q + j]);
  sh[t] = acc;
  __syncthreads();
  for (int d = 32; d >= 1; d >>= 1) {
    if (t < d) sh[t] = bj1_add(sh[t], sh[t + d]);
    __syncthreads();
  }
  if (t == 0) {
    agg->p[j] = bj1_to_aff(sh[0]);
    if (j == 0) {
      agg->p[6] = {bq_zero(), bq_zero(), true};
      agg->qb = {b2_one(), b2_one()};  // unused (p[6] infinite); any value keeps the b steps finite
    }
  }
}
// The batch check's Miller loop, split by loop position (a lone lane carrying the six key pairs took
// 39 ms, as long as the whole per-proof loop at 64k): segment h of the loop's 66 positions (bits
// 63..0 -- a doubling step and an addition when set -- then the pi(Q), -pi^2(Q) additions) runs from
// f = 1 (k_pghr_bseg). The loop's value is the Horner product over the segments
//   (((seg[0])^(2^sq(1)) seg[1])^(2^sq(2)) ...) seg[S-1],  sq(h) = the doublings of segment h
// which k_pghr_fe_coop forms after k_fe_easy's map x -> x^((p^6 - 1)(p^2 + 1)) (a homomorphism) has
// put every seg[h] in the cyclotomic subgroup, where a squaring is Granger-Scott's.
#define ZG_PGHR_FSEG 8
#define ZG_FE_SLOTS 6  // the final exponentiation's per-value HBM workspace (k_fe_easy below)
#define ZG_BN_POS (ZG_BN_ATE_BITS + 1)  // loop positions: q = 0 is bit 63, q = 64, 65 the two additions
ZG_INL int pghr_pos_bit(int q) { return ZG_BN_ATE_BITS - 2 - q; }
ZG_INL int pghr_seg_lo(int h) { return h * ZG_BN_POS / ZG_PGHR_FSEG; }
ZG_INL int pghr_seg_sq(int h) {  // doubling steps (squarings of f) in segment h
  int sq = 0;
  for (int q = pghr_seg_lo(h); q < pghr_seg_lo(h + 1); q++) sq += pghr_pos_bit(q) >= 0;
  return sq;
}
#ifndef ZG_BSEG_WPE
#define ZG_BSEG_WPE 1  // waves per SIMD the register budget allows (2 spills ~460 B/lane)
#endif
// grid (1 + blocks of 64 lanes, S), segment h = blockIdx.y; each lane runs ONE multi-pair loop over
// its segment -- a squaring per doubling step shared by all its pairs, then each pair's line:
//  * block 0, lanes 0..5: key pair j on the batch's operand sums agg (lines from the key's table);
//    the block is dispatched first, so it never waits behind the proofs' blocks (as a one-block
//    kernel on a second stream, k_pghr_fseg, it waited for a free SIMD: 1.4 -> 5.2 ms);
//  * block 1 + b, lane l: group g = 64 b + l carries the proofs g, g + G, .., g + (K - 1) G
//    (G = ceil(n / K): a wave's line loads stay contiguous), lines from k_pghr_blines.
// Each block multiplies its 64 values -> part[h gridDim.x + block] (1 where nothing takes part).
// The Horner product over segments is multiplicative,
//   prod_i Horner(s_i0, .., s_i7) = Horner(prod_i s_i0, .., prod_i s_i7),
// so one product tree per segment joins every pair of the batch before the shared Horner squarings
// and final exponentiation.
__global__ void __launch_bounds__(64, ZG_BSEG_WPE) k_pghr_bseg(int n, int K, const PghrPts* pts, const uint8_t* status,
                                                               const BLine* bl, const PghrPts* agg,
                                                               const BLine* klines, Bq12* part) {
  __shared__ Bq12 sh[64];
  const bool key = blockIdx.x == 0;  // block-uniform
  const int g = ((int)blockIdx.x - 1) * 64 + threadIdx.x, h = blockIdx.y, G = (n + K - 1) / K;
  const int np = key ? 1 : K;  // a key lane carries one pair (lane j < 6: pair j)
  uint32_t live = 0;            // pair k of the lane takes part
  for (int k = 0; k < np; k++) {
    if (key) {
      if (threadIdx.x < ZG_BN_FIXED_Q && !agg->p[threadIdx.x].inf) live = 1;
    } else {
      const int i = g + k * G;
      if (g < G && i < n && status[i] == ZG_STATUS_OK && !pts[i].p[6].inf) live |= 1u << k;
    }
  }
  Bq12 f = b12_one();
  if (live) {
    const int q0 = pghr_seg_lo(h), q1 = pghr_seg_lo(h + 1);
    int li = 0;
    for (int q = 0; q < q0; q++) {
      const int bit = pghr_pos_bit(q);
      li += bit >= 0 && bn_ate_bit(bit) ? 2 : 1;
    }
    for (int q = q0; q < q1; q++) {
      const int bit = pghr_pos_bit(q);
      if (bit >= 0 && q > q0) f = b12_sqr(f);  // the segment's first squaring is of 1 (counted in sq(h))
      const int nsub = bit >= 0 && bn_ate_bit(bit) ? 2 : 1;
      for (int s = 0; s < nsub; s++, li++)
        for (int k = 0; k < np; k++) {
          if (!((live >> k) & 1u)) continue;
          // one call site for both kinds of lane (two inlined copies of the sparse product cost
          // the kernel its instruction cache)
          const size_t i = (size_t)g + (size_t)k * G;
          const BLine* l = key ? klines + (size_t)threadIdx.x * ZG_BN_NLINES + li : bl + (size_t)li * n + i;
          const BA1* p = key ? &agg->p[threadIdx.x] : &pts[i].p[6];
          f = b12_mul_bline(f, *l, *p);
        }
    }
  }
  sh[threadIdx.x] = f;
  __syncthreads();
  for (int d = 32; d >= 1; d >>= 1) {
    if ((int)threadIdx.x < d) sh[threadIdx.x] = b12_mul(sh[threadIdx.x], sh[threadIdx.x + d]);
    __syncthreads();
  }
  if (threadIdx.x == 0) part[(size_t)h * gridDim.x + blockIdx.x] = sh[0];
}
// the per-segment tree roots b[h stride] -> seg[h], seg[S] = 1 (k_fe_easy / k_pghr_fe_coop keep
// their S + 1 inputs)
__global__ void __launch_bounds__(64) k_pghr_segcopy(Bq12* seg, const Bq12* b, size_t stride) {
  const int h = threadIdx.x;
  if (h < ZG_PGHR_FSEG) seg[h] = b[stride * h];
  if (h == ZG_PGHR_FSEG) seg[h] = b12_one();
}
// one level of the product tree over the block products: dst[k] = src[2k] * src[2k + 1] (an odd
// last one moves up); blockIdx.y selects one of several independent trees (stride apart)
__global__ void __launch_bounds__(64) k_bn_tree(const Bq12* src, Bq12* dst, int m, size_t stride) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (m + 1) / 2) return;
  src += stride * blockIdx.y;
  dst += stride * blockIdx.y;
  dst[k] = 2 * k + 1 < m ? b12_mul(src[2 * k], src[2 * k + 1]) : src[2 * k];
}

// The proofs' own pairs e(P_i7, b_i) of the batch check go by segment too (one lane carrying a
// proof's whole single-pair loop left 64k proofs at one wave per SIMD, 11.6 ms): k_pghr_blines walks
// each b_i's doubling / addition chain (lane per proof, G2 only) and stores its 102 lines
// proof-minor (bl[li n + i], a wave's stores contiguous) for k_pghr_bseg. It needs only the decoded
// b, so it follows k_pghr_decode_g2 on the side stream, concurrent with the G1 chain (decode, combs,
// prep, rho); a proof that fails elsewhere leaves its lines unread.
__global__ void __launch_bounds__(64) k_pghr_blines(int n, const PghrDec* dec, const uint8_t* okb, BLine* bl) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n || !okb[8 * (size_t)i + 2]) return;
  const BA2 qb = dec[i].qb;
  BH2 t = {qb.x, qb.y, b2_one()};
  int li = 0;
  for (int bit = ZG_BN_ATE_BITS - 2; bit >= 0; bit--) {
    bl[(size_t)(li++) * n + i] = bh2_dbl_step(&t);
    if (bn_ate_bit(bit)) bl[(size_t)(li++) * n + i] = bh2_add_step(&t, qb);
  }
  bl[(size_t)(li++) * n + i] = bh2_add_step(&t, ba2_frob(qb));
  const BA2 q2 = ba2_frob2(qb);
  bl[(size_t)li * n + i] = bh2_add_step(&t, {q2.x, b2_neg(q2.y)});
}

// the final exponentiation of zg_bn254.h bn_final_exp, split so that no kernel holds more than
// a few Fq12 values at once (a lane-per-proof Fq12 is 96 VGPRs): the chain's intermediates live in
// a per-proof HBM workspace w[0..5] = t, b, d, e, g, (spare)
// halves 2: f holds two partial Miller products per proof (k_pghr_miller), multiplied here
__global__ void __launch_bounds__(64) k_fe_easy(int n, const Bq12* f, const uint8_t* status, Bq12* w, int halves) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || status[i] != ZG_STATUS_OK) return;
  const Bq12 x = halves == 2 ? b12_mul(f[2 * (size_t)i], f[2 * (size_t)i + 1]) : f[i];
  const Bq12 t = b12_mul(b12_conj(x), b12_inv(x));
  w[(size_t)ZG_FE_SLOTS * i + 0] = b12_mul(b12_frob(t, 2), t);
}
// stage 1: a = t^-u, b = a^2, d = b^3 ; stage 2: e = d^-u ; stage 3: g = (e^2)^-u
template <int STAGE>
__global__ void __launch_bounds__(64) k_fe_exp(int n, const uint8_t* status, Bq12* w) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || status[i] != ZG_STATUS_OK) return;
  Bq12* s = w + (size_t)ZG_FE_SLOTS * i;
  if (STAGE == 1) {
    const Bq12 b = b12_csqr(b12_exp_by_neg_u(s[0]));  // cyclotomic from here on: Granger-Scott squarings
    s[1] = b;
    s[2] = b12_mul(b12_csqr(b), b);
  } else if (STAGE == 2) {
    const Bq12 e = b12_exp_by_neg_u(s[2]);
    s[3] = e;
    s[5] = b12_csqr(e);  // stage 3's input (its own kernel holding csqr + the chain spilled ~390 VGPRs)
  } else {
    s[4] = b12_exp_by_neg_u(s[5]);
  }
}
// k = g^-1 e d^-1, l = k b, n = t k e ; result = (t^-1 l)^(p^3) k^(p^2) l^p n == 1 ?
__global__ void __launch_bounds__(64) k_fe_last(int n, uint8_t* status, Bq12* w) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || status[i] != ZG_STATUS_OK) return;
  Bq12* s = w + (size_t)ZG_FE_SLOTS * i;
  const Bq12 k = b12_mul(b12_mul(b12_conj(s[4]), s[3]), b12_conj(s[2]));
  s[5] = k;
  const Bq12 l = b12_mul(k, s[1]);
  s[4] = l;  // g is dead
  Bq12 r = b12_mul(s[0], b12_mul(k, s[3]));           // n
  r = b12_mul(b12_frob(l, 1), r);                      // p
  r = b12_mul(b12_frob(s[5], 2), r);                   // r
  r = b12_mul(b12_frob(b12_mul(b12_conj(s[0]), s[4]), 3), r);
  status[i] = b12_is_one(r) ? ZG_STATUS_OK : ZG_STATUS_VERIFY_FAILED;
}

// ---- the batch check's one final exponentiation on one wave. As a lane-serial chain (k_fe_exp on
// one lane) its three exponentiations by -u took 12 ms; here an Fq12 lives in LDS as its six Fq2
// coefficients by power of w (z[e], e = a + 2b for the tower's c_a.c_b: z[0] = c0.c0, z[2] = c0.c1,
// z[4] = c0.c2, z[1] = c1.c0, z[3] = c1.c1, z[5] = c1.c2) and each operation spreads its Fq
// products over the wave's lanes, then six lanes form the coefficients:
//   mul   the 36 Fq2 products z_i z'_j (Karatsuba, 3 Fq products each: 108 on 64 lanes, two rounds);
//         out[e] = the sum over i + j = e (mod 6), those with i + j >= 6 times xi (w^6 = v^3 = xi)
//   csqr  Granger-Scott (b12_csqr): the pairs (z[p], z[p + 3]) give A B and (A + B)(xi B + A), 6 Fq2
//         products = 18 Fq products, one round
//   conj, frob, copy  lane e on z[e]
// A product then costs about two Fq products of latency and a cyclotomic squaring one, against 54 and
// 18 on one lane. The chain is bn_final_exp's (zg_bn254.h; oracle.bn254.final_exponentiation_fc).
struct BcF12 {
  Bq2 z[6];
};
#define ZG_BC_SLOTS 8
struct BcWS {
  BcF12 s[ZG_BC_SLOTS];
  Bq m[108];
};
ZG_INL int bc_tower(int e) { return (e & 1) * 3 + (e >> 1); }  // index of z[e] among Bq12's six Bq2
__device__ void bc_load(BcWS* ws, int dst, const Bq12* x) {
  const int e = threadIdx.x;
  if (e < 6) ws->s[dst].z[e] = reinterpret_cast<const Bq2*>(x)[bc_tower(e)];
  __syncthreads();
}
__device__ void bc_mul(BcWS* ws, int dst, int a, int b) {
  for (int t = threadIdx.x; t < 108; t += 64) {
    const int k = t / 3, m = t - 3 * k, i = k / 6, j = k - 6 * i;
    const Bq2 x = ws->s[a].z[i], y = ws->s[b].z[j];
    const Bq u = m == 0 ? x.c0 : m == 1 ? x.c1 : bq_add(x.c0, x.c1);
    const Bq v = m == 0 ? y.c0 : m == 1 ? y.c1 : bq_add(y.c0, y.c1);
    ws->m[t] = bq_mul(u, v);
  }
  __syncthreads();
  const int e = threadIdx.x;
  if (e < 6) {
    Bq2 lo = b2_zero(), hi = b2_zero();
    for (int i = 0; i < 6; i++) {
      const int j = (e - i + 6) % 6, k = 6 * i + j;
      const Bq m0 = ws->m[3 * k], m1 = ws->m[3 * k + 1], m2 = ws->m[3 * k + 2];
      const Bq2 q = {bq_sub(m0, m1), bq_sub(bq_sub(m2, m0), m1)};
      if (i + j >= 6)
        hi = b2_add(hi, q);
      else
        lo = b2_add(lo, q);
    }
    ws->s[dst].z[e] = b2_add(lo, b2_mul_xi(hi));
  }
  __syncthreads();
}
__device__ void bc_csqr(BcWS* ws, int dst, int a) {
  const int t = threadIdx.x;
  if (t < 18) {
    const int q = t / 3, m = t - 3 * q, pr = q >> 1;
    const Bq2 A = ws->s[a].z[pr], B = ws->s[a].z[pr + 3];
    const Bq2 x = (q & 1) ? b2_add(A, B) : A, y = (q & 1) ? b2_add(b2_mul_xi(B), A) : B;
    const Bq u = m == 0 ? x.c0 : m == 1 ? x.c1 : bq_add(x.c0, x.c1);
    const Bq v = m == 0 ? y.c0 : m == 1 ? y.c1 : bq_add(y.c0, y.c1);
    ws->m[t] = bq_mul(u, v);
  }
  __syncthreads();
  const int e = t;
  if (e < 6) {
    // pair of z[e]: (z0, z3) -> 0, (z2, z5) -> 1, (z4, z1) -> 2
    const int pr = (e & 1) ? ((e + 3) % 6) / 2 : e / 2;
    auto prod = [&](int q) {
      const Bq m0 = ws->m[3 * q], m1 = ws->m[3 * q + 1], m2 = ws->m[3 * q + 2];
      return Bq2{bq_sub(m0, m1), bq_sub(bq_sub(m2, m0), m1)};
    };
    const Bq2 ab = prod(2 * pr), z = ws->s[a].z[e];
    Bq2 r;
    if ((e & 1) == 0) {  // 3 t0 - 2 z, t0 = (A + B)(xi B + A) - A B - xi A B
      const Bq2 t0 = b2_sub(b2_sub(prod(2 * pr + 1), ab), b2_mul_xi(ab));
      const Bq2 d = b2_sub(t0, z);
      r = b2_add(b2_add(d, d), t0);
    } else {  // 3 t1 + 2 z, t1 = 2 A B (times xi for z[1])
      Bq2 t1 = b2_add(ab, ab);
      if (e == 1) t1 = b2_mul_xi(t1);
      const Bq2 d = b2_add(t1, z);
      r = b2_add(b2_add(d, d), t1);
    }
    ws->s[dst].z[e] = r;
  }
  __syncthreads();
}
__device__ void bc_copy(BcWS* ws, int dst, int a, bool conj) {
  const int e = threadIdx.x;
  if (e < 6) {
    const Bq2 x = ws->s[a].z[e];
    ws->s[dst].z[e] = conj && (e & 1) ? b2_neg(x) : x;
  }
  __syncthreads();
}
__device__ void bc_frob(BcWS* ws, int dst, int a, int k) {
  const int e = threadIdx.x;
  if (e < 6) {
    Bq2 x = ws->s[a].z[e];
    if (k & 1) x = b2_conj(x);
    if (e) {
      const uint32_t* const g[3][5] = {{BQ_FROB1_1, BQ_FROB1_2, BQ_FROB1_3, BQ_FROB1_4, BQ_FROB1_5},
                                       {BQ_FROB2_1, BQ_FROB2_2, BQ_FROB2_3, BQ_FROB2_4, BQ_FROB2_5},
                                       {BQ_FROB3_1, BQ_FROB3_2, BQ_FROB3_3, BQ_FROB3_4, BQ_FROB3_5}};
      x = b2_mul(x, b2_c(g[k - 1][e - 1]));
    }
    ws->s[dst].z[e] = x;
  }
  __syncthreads();
}
// dst = src^-u (src cyclotomic); tmp != src, dst
__device__ void bc_exp_by_neg_u(BcWS* ws, int dst, int src, int tmp) {
  bc_copy(ws, tmp, src, false);
  for (int i = 61; i >= 0; i--) {
    bc_csqr(ws, tmp, tmp);
    if ((BN_U >> i) & 1ull) bc_mul(ws, tmp, tmp, src);
  }
  bc_copy(ws, dst, tmp, true);
}
// w: slot 0 of lanes 0..S of k_fe_easy's workspace (the segments' values and the b pairs' product,
// each mapped into the cyclotomic subgroup) -> the Horner product (k_pghr_bseg's note), its hard part,
// status[0] = OK iff the result is 1
__global__ void __launch_bounds__(64) k_pghr_fe_coop(const Bq12* w, uint8_t* status) {
  __shared__ BcWS ws;
  enum { T, B, D, E, G, X, Y, Z };
  bc_load(&ws, T, w);
  for (int h = 1; h <= ZG_PGHR_FSEG; h++) {
    const int sq = h < ZG_PGHR_FSEG ? pghr_seg_sq(h) : 0;
    for (int k = 0; k < sq; k++) bc_csqr(&ws, T, T);
    bc_load(&ws, X, w + (size_t)ZG_FE_SLOTS * h);
    bc_mul(&ws, T, T, X);
  }
  bc_exp_by_neg_u(&ws, X, T, Y);  // a = t^-u
  bc_csqr(&ws, B, X);             // b = a^2
  bc_csqr(&ws, X, B);             // c = b^2
  bc_mul(&ws, D, X, B);           // d = c b
  bc_exp_by_neg_u(&ws, E, D, Y);  // e = d^-u
  bc_csqr(&ws, X, E);
  bc_exp_by_neg_u(&ws, G, X, Y);  // g = (e^2)^-u
  bc_copy(&ws, X, G, true);
  bc_mul(&ws, X, X, E);
  bc_copy(&ws, Y, D, true);
  bc_mul(&ws, G, X, Y);           // k = g^-1 e d^-1 (in G)
  bc_mul(&ws, X, G, B);           // l = k b
  bc_mul(&ws, Y, G, E);
  bc_mul(&ws, Y, T, Y);           // n = t k e
  bc_frob(&ws, Z, X, 1);
  bc_mul(&ws, Z, Z, Y);           // l^p n
  bc_frob(&ws, B, G, 2);
  bc_mul(&ws, Z, B, Z);           // k^(p^2) l^p n
  bc_copy(&ws, Y, T, true);
  bc_mul(&ws, Y, Y, X);
  bc_frob(&ws, Y, Y, 3);          // (t^-1 l)^(p^3)
  bc_mul(&ws, Y, Y, Z);
  if (threadIdx.x == 0) {
    bool one = b2_eq(ws.s[Y].z[0], b2_one());
    for (int e = 1; e < 6; e++) one = one && b2_is_zero(ws.s[Y].z[e]);
    status[0] = one ? ZG_STATUS_OK : ZG_STATUS_VERIFY_FAILED;
  }
}

// zg_bn254_pairing (tests): the Miller loop of e(P, Q) -> f; the final exponentiation then runs
// through the k_fe_* kernels above and k_bn_gt writes GT as 12 canonical LE Fq in the order
// w^0.c0, w^0.c1, w^1.c0, ..., w^5.c1 (oracle.bn254.gt_ints)
__global__ void __launch_bounds__(64) k_bn_miller1(int n, const uint32_t* g1, const uint32_t* g2, Bq12* fout) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* a = g1 + 16 * (size_t)i;
  const uint32_t* q = g2 + 32 * (size_t)i;
  const BA1 p = {bq_to_mont(bq_c(a)), bq_to_mont(bq_c(a + 8)), false};
  const BA2 Q = {{bq_to_mont(bq_c(q)), bq_to_mont(bq_c(q + 8))}, {bq_to_mont(bq_c(q + 16)), bq_to_mont(bq_c(q + 24))}};
  fout[i] = bn_miller_single(p, Q);
}
// the full exponent's last stage (k_fe_last without the comparison)
__global__ void __launch_bounds__(64) k_bn_gt(int n, Bq12* w, uint32_t* gt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Bq12* s = w + (size_t)ZG_FE_SLOTS * i;
  const Bq12 k = b12_mul(b12_mul(b12_conj(s[4]), s[3]), b12_conj(s[2]));
  s[5] = k;
  const Bq12 l = b12_mul(k, s[1]);
  s[4] = l;
  Bq12 r = b12_mul(s[0], b12_mul(k, s[3]));
  r = b12_mul(b12_frob(l, 1), r);
  r = b12_mul(b12_frob(s[5], 2), r);
  r = b12_mul(b12_frob(b12_mul(b12_conj(s[0]), s[4]), 3), r);
  const Bq2 cs[6] = {r.c0.c0, r.c1.c0, r.c0.c1, r.c1.c1, r.c0.c2, r.c1.c2};  // w^0 .. w^5
  uint32_t* o = gt + 96 * (size_t)i;
  for (int k2 = 0; k2 < 6; k2++) {
    const Bq x0 = bq_from_mont(cs[k2].c0), x1 = bq_from_mont(cs[k2].c1);
    for (int l2 = 0; l2 < 8; l2++) {
      o[16 * k2 + l2] = x0.l[l2];
      o[16 * k2 + 8 + l2] = x1.l[l2];
    }
  }
}

// ------------------------------------------------------------------ host side
// One prepared PGHR13 key: the key, its line table and comb tables. Built into fresh buffers
// and published in the device's cache only once complete and valid; never modified or freed
// while the device lives, so a context verifying with it needs no lock (a key loaded on one
// context does not change the key of any other context).
struct BnKey {
  std::vector<uint32_t> raw;  // the parsed key words (the cache key)
  int refs = 0;               // contexts pointing at this entry (BnDev::mu); freed at 0
  BnVK* vk = nullptr;
  BLine* lines = nullptr;
  uint32_t* comb = nullptr;
};

struct BnDev {
  std::mutex mu;                // the cache
  std::vector<BnKey*> keys;     // every distinct key loaded on this device
};

static void bn_key_free(BnKey* k) {
  if (!k) return;
  if (k->vk) hipFree(k->vk);
  if (k->lines) hipFree(k->lines);
  if (k->comb) hipFree(k->comb);
  delete k;
}

BnDev* bn_dev_new() { return new BnDev(); }
// a context stops pointing at k (it loaded another key, or it is destroyed): the entry and its HBM
// (VK, line table, comb tables) go once no context uses it, so rotating keys does not grow the cache
void bn_key_release(BnDev* d, const BnKey* k) {
  if (!d || !k) return;
  std::lock_guard<std::mutex> g(d->mu);
  for (size_t i = 0; i < d->keys.size(); i++)
    if (d->keys[i] == k) {
      if (--d->keys[i]->refs == 0) {
        bn_key_free(d->keys[i]);
        d->keys.erase(d->keys.begin() + i);
      }
      return;
    }
}
void bn_dev_free(BnDev* d) {
  if (!d) return;
  for (BnKey* k : d->keys) bn_key_free(k);
  delete d;
}

#define BCHK(expr)                                            \
  do {                                                        \
    hipError_t e_ = (expr);                                   \
    if (e_ != hipSuccess) {                                   \
      *err = std::string(#expr ": ") + hipGetErrorString(e_); \
      return ZG_E_HIP;                                        \
    }                                                         \
  } while (0)

static unsigned bn_blocks(long long n) { return (unsigned)((n + 63) / 64); }
// k_pghr_bseg's proofs per lane (ZG_BSEG_K overrides): ceil(n / K) >= 8,192 lanes x 8 segments
// (1,024 waves of the one-wave-per-SIMD kernel), the rest as shared squarings: 64k proofs K = 8
// (kernels 39.0 / 36.0 / 34.6 / 32.9 ms for K = 1 / 2 / 4 / 8, profiles/r03v_pghr13_bench.txt)
static int bseg_k(size_t n) {
  static const int forced = getenv("ZG_BSEG_K") ? atoi(getenv("ZG_BSEG_K")) : 0;
  if (forced > 0) return forced < 32 ? forced : 32;
  int k = 1;
  while (k < 8 && n / (size_t)(2 * k) >= 8192) k *= 2;
  return k;
}

// hex strings of the key's JSON members in document order (crypto/src/json/pghr13.rs layout)
static bool json_hex_list(const std::string& js, const char* key, std::vector<std::string>* out) {
  const std::string k = std::string("\"") + key + "\"";
  size_t pos = js.find(k);
  if (pos == std::string::npos) return false;
  pos = js.find('[', pos);
  if (pos == std::string::npos) return false;
  int depth = 0;
  for (size_t i = pos; i < js.size(); i++) {
    const char ch = js[i];
    if (ch == '[') depth++;
    if (ch == ']' && --depth == 0) return true;
    if (ch == '"') {
      const size_t e = js.find('"', i + 1);
      if (e == std::string::npos) return false;
      std::string s = js.substr(i + 1, e - i - 1);
      if (s.rfind("0x", 0) == 0) s = s.substr(2);
      out->push_back(s);
      i = e;
    }
  }
  return false;
}

// a big-endian hex Fq (Fq::from_slice: at most 32 bytes, < p) -> 8 LE words
static bool hex_fq(const std::string& h, uint32_t* w) {
  if (h.size() > 64 || h.empty()) return false;
  uint8_t b[32] = {0};
  const std::string s = std::string(64 - h.size(), '0') + h;
  for (int i = 0; i < 32; i++) {
    unsigned v;
    if (sscanf(s.c_str() + 2 * i, "%2x", &v) != 1) return false;
    b[i] = (uint8_t)v;
  }
  for (int l = 0; l < 8; l++) {
    const uint8_t* q = b + 28 - 4 * l;
    w[l] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
  for (int l = 7; l >= 0; l--)
    if (w[l] != BQ_P[l]) return w[l] < BQ_P[l];
  return false;
}

int bn_load_vk_json(BnDev* d, hipStream_t st, const char* json, size_t len, const BnKey** out, std::string* err) {
  const std::string js(json, len);
  std::vector<uint32_t> raw;
  auto put = [&](const std::string& h) {
    uint32_t w[8];
    if (!hex_fq(h, w)) return false;
    raw.insert(raw.end(), w, w + 8);
    return true;
  };
  // G2 [x_a, x_b, y_a, y_b] -> x = (x_b, x_a), y = (y_b, y_a)
  for (const char* k : {"alphaA", "alphaC", "gamma", "gammaBeta2", "zeta"}) {
    std::vector<std::string> v;
    if (!json_hex_list(js, k, &v) || v.size() != 4) {
      *err = std::string("PGHR13 key: bad member ") + k;
      return ZG_E_VK;
    }
    if (!put(v[1]) || !put(v[0]) || !put(v[3]) || !put(v[2])) {
      *err = std::string("PGHR13 key: field element of ") + k;
      return ZG_E_VK;
    }
  }
  for (const char* k : {"alphaB", "gammaBeta1"}) {
    std::vector<std::string> v;
    if (!json_hex_list(js, k, &v) || v.size() != 2 || !put(v[0]) || !put(v[1])) {
      *err = std::string("PGHR13 key: bad member ") + k;
      return ZG_E_VK;
    }
  }
  std::vector<std::string> ic;
  if (!json_hex_list(js, "ic", &ic) || ic.size() % 2 || ic.size() < 2 || ic.size() / 2 > ZG_BN_MAX_IC) {
    *err = "PGHR13 key: bad ic";
    return ZG_E_VK;
  }
  for (const auto& h : ic)
    if (!put(h)) {
      *err = "PGHR13 key: ic field element";
      return ZG_E_VK;
    }
  const int ic_len = (int)ic.size() / 2;
  std::lock_guard<std::mutex> g(d->mu);  // one build per distinct key, never a half-built entry visible
  for (BnKey* k : d->keys)
    if (k->raw == raw) {
      k->refs++;
      *out = k;
      return ZG_OK;
    }
  BnKey* k = new BnKey();
  k->raw = raw;
  uint32_t* draw = nullptr;
  int verr = 0;
  hipError_t e = hipMalloc(&k->vk, sizeof(BnVK));
  if (e == hipSuccess) e = hipMalloc(&k->lines, sizeof(BLine) * ZG_BN_FIXED_Q * ZG_BN_NLINES);
  if (e == hipSuccess) e = hipMalloc(&k->comb, (size_t)ZG_BN_COMB_BASES * ZG_BN_COMB_W * ZG_BN_COMB_D * 64);
  if (e == hipSuccess) e = hipMalloc(&draw, raw.size() * 4);
  if (e == hipSuccess) e = hipMemcpyAsync(draw, raw.data(), raw.size() * 4, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_bn_vk, dim3(1), dim3(64), 0, st, draw, ic_len, k->vk);
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_bn_lines, dim3(1), dim3(64), 0, st, k->vk, k->lines);
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_bn_comb, dim3(bn_blocks(ZG_BN_COMB_BASES * ZG_BN_COMB_W * ZG_BN_COMB_D)), dim3(64), 0, st,
                       k->vk, k->comb);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(&verr, &k->vk->err, sizeof(int), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (draw) hipFree(draw);
  if (e != hipSuccess) {
    bn_key_free(k);
    *err = std::string("PGHR13 key upload: ") + hipGetErrorString(e);
    return ZG_E_HIP;
  }
  if (verr) {
    bn_key_free(k);
    *err = "PGHR13 key: a point is not on its curve or not of order r (AffineG*::new)";
    return ZG_E_VK;
  }
  k->refs = 1;
  d->keys.push_back(k);
  *out = k;
  return ZG_OK;
}

int bn_pghr13_verify(const BnKey* d, hipStream_t st, hipStream_t side, size_t n, const uint8_t* proofs,
                     const uint8_t* inputs, const uint8_t* ninputs, const uint8_t* rho, uint8_t* status,
                     float* kernel_ms, bool* batch_failed, void** arena, size_t* arena_cap, std::string* err) {
  if (batch_failed) *batch_failed = false;
  if (!n) return ZG_OK;
  // the call's device buffers, carved from the context's grow-only arena (a 64k call needs
  // ~1.5 GB; allocating and freeing that per call cost more wall time than most kernels)
  const unsigned nb = bn_blocks(n);
  struct Part {
    void** p;
    size_t b;
  };
  uint8_t *dp, *din, *dni = nullptr, *drho, *dst, *dokb, *dbst;
  PghrPts *dpts, *dagg;
  PghrDec* ddec;
  BA1* dmul;
  BJ1 *daccp, *dpart, *dstr;
  BLine* dbl;
  Bq12 *df, *dw, *dbseg, *dbtmp, *dseg, *dbw;
  const Part parts[] = {
      {(void**)&dp, 296 * n},
      {(void**)&din, 9 * 32 * n},
      {(void**)&drho, ZG_PGHR_RHO_BYTES * n},
      {(void**)&dst, n},
      {(void**)&dni, ninputs ? n : 0},
      {(void**)&dpts, sizeof(PghrPts) * n},
      {(void**)&ddec, sizeof(PghrDec) * n},
      {(void**)&dmul, sizeof(BA1) * ZG_PGHR_NMUL * n},
      {(void**)&daccp, sizeof(BJ1) * 9 * n},
      {(void**)&dokb, 8 * n},
      {(void**)&df, sizeof(Bq12) * 2 * n},
      {(void**)&dw, sizeof(Bq12) * ZG_FE_SLOTS * n},
      {(void**)&dbl, sizeof(BLine) * ZG_BN_NLINES * n},
      {(void**)&dpart, sizeof(BJ1) * ZG_BN_FIXED_Q * (nb + 4 * n / ZG_PGHR_SSUM_CH + 1)},
      {(void**)&dstr, sizeof(BJ1) * ZG_PGHR_NFAM * n},
      {(void**)&dagg, sizeof(PghrPts)},
      {(void**)&dbseg, sizeof(Bq12) * ZG_PGHR_FSEG * (nb + 1)},
      {(void**)&dbtmp, sizeof(Bq12) * ZG_PGHR_FSEG * (nb + 1)},
      {(void**)&dseg, sizeof(Bq12) * (ZG_PGHR_FSEG + 1)},
      {(void**)&dbw, sizeof(Bq12) * ZG_FE_SLOTS * (ZG_PGHR_FSEG + 1)},
      {(void**)&dbst, ZG_PGHR_FSEG + 1},
  };
  size_t need = 0;
  for (const Part& q : parts) need += (q.b + 255) & ~(size_t)255;
  if (*arena_cap < need) {
    BCHK(hipStreamSynchronize(st));
    if (*arena) hipFree(*arena);
    *arena = nullptr;
    *arena_cap = 0;
    BCHK(hipMalloc(arena, need));
    *arena_cap = need;
  }
  char* bump = (char*)*arena;
  for (const Part& q : parts) {
    *q.p = q.b ? bump : nullptr;
    bump += (q.b + 255) & ~(size_t)255;
  }
  struct Events {
    hipEvent_t e[8] = {};
    ~Events() {
      for (hipEvent_t x : e)
        if (x) hipEventDestroy(x);
    }
  } ev;
  hipEvent_t &e0 = ev.e[0], &e1 = ev.e[1], &g2fork = ev.e[4], &g2join = ev.e[5], &g2dec = ev.e[6], &stready = ev.e[7];
  for (hipEvent_t* x : {&g2fork, &g2join, &g2dec, &stready}) BCHK(hipEventCreateWithFlags(x, hipEventDisableTiming));
  BCHK(hipMemcpyAsync(dp, proofs, 296 * n, hipMemcpyHostToDevice, st));
  BCHK(hipMemcpyAsync(din, inputs, 9 * 32 * n, hipMemcpyHostToDevice, st));
  BCHK(hipMemcpyAsync(drho, rho, ZG_PGHR_RHO_BYTES * n, hipMemcpyHostToDevice, st));
  if (ninputs) BCHK(hipMemcpyAsync(dni, ninputs, n, hipMemcpyHostToDevice, st));
  if (kernel_ms) {
    BCHK(hipEventCreate(&e0));
    BCHK(hipEventCreate(&e1));
    BCHK(hipEventRecord(e0, st));
  }
  // b's decode (Fq2 sqrt + G2 membership) and its lines (lane per proof at ~280 registers: one
  // wave per SIMD) on the side stream, sharing the SIMDs with the G1 decodes, combs, prep and rho
  // from the fork on, every return (an error included) first drains the side stream: its kernels
  // use this call's arena, which the next call on this context reuses
  struct SideJoin {
    hipStream_t s;
    ~SideJoin() { hipStreamSynchronize(s); }
  } side_join{side};
  BCHK(hipEventRecord(g2fork, st));
  BCHK(hipStreamWaitEvent(side, g2fork, 0));
  hipLaunchKernelGGL(k_pghr_decode_g2, dim3(nb), dim3(64), 0, side, (int)n, dp, ddec, dokb);
  BCHK(hipGetLastError());
  BCHK(hipEventRecord(g2dec, side));
  hipLaunchKernelGGL(k_pghr_blines, dim3(nb), dim3(64), 0, side, (int)n, ddec, dokb, dbl);
  BCHK(hipGetLastError());
  // one-wave blocks: a multi-wave block must find all its waves' registers on one CU, and beside the
  // side stream's ~280-register G2 waves it waited for them to finish (the 576-lane combs: 1.4 ->
  // 10.5 ms, profiles/r03s3_pghr_timeline.txt)
  hipLaunchKernelGGL(k_pghr_decode_g1, dim3(nb, 7), dim3(64), 0, st, (int)n, dp, ddec, dokb);
  BCHK(hipGetLastError());
  hipLaunchKernelGGL(k_pghr_accp, dim3(nb, 9), dim3(64), 0, st, (int)n, din, dni, d->vk, d->comb, daccp);
  BCHK(hipGetLastError());
  hipLaunchKernelGGL(k_pghr_prep, dim3(nb), dim3(64), 0, st, (int)n, din, dni, d->vk, dokb, daccp, ddec, dst);
  BCHK(hipGetLastError());
  BCHK(hipStreamWaitEvent(st, g2dec, 0));  // the final statuses (b's decode verdict joins)
  hipLaunchKernelGGL(k_pghr_g2status, dim3(nb), dim3(64), 0, st, (int)n, dokb, dst);
  // the b pairs' operands P_i7 (one GLV product + combs per proof): on the side stream after the b
  // lines from 32k proofs, where the main stream's Straus sums are the longer chain; below, the side
  // stream's G2 chain (128 waves of decodes and lines at 8k) is, and P_i7 follows the sums on main
  const bool p7_side = n >= 32768;
  if (p7_side) {
    BCHK(hipEventRecord(stready, st));
    BCHK(hipStreamWaitEvent(side, stready, 0));
    hipLaunchKernelGGL(k_pghr_p7, dim3(nb), dim3(64), 0, side, (int)n, ddec, drho, d->comb, dst, dpts);
    BCHK(hipGetLastError());
  }
  BCHK(hipEventRecord(g2join, side));
  // the six key pairs' operand sums (Straus over the GLV halves, B proofs per lane), concurrent with
  // the side stream's b lines and P_i7
  const int B = straus_b(n);
  const long long G = ((long long)n + B - 1) / B;
  const dim3 sg((unsigned)((G + 63) / 64), ZG_PGHR_NFAM);
  if (B == 4)
    hipLaunchKernelGGL(k_pghr_straus<4>, sg, dim3(64), 0, st, (int)n, ddec, drho, dst, dstr);
  else if (B == 2)
    hipLaunchKernelGGL(k_pghr_straus<2>, sg, dim3(64), 0, st, (int)n, ddec, drho, dst, dstr);
  else
    hipLaunchKernelGGL(k_pghr_straus<1>, sg, dim3(64), 0, st, (int)n, ddec, drho, dst, dstr);
  BCHK(hipGetLastError());
  const unsigned nch = (unsigned)((4 * G + ZG_PGHR_SSUM_CH - 1) / ZG_PGHR_SSUM_CH);
  hipLaunchKernelGGL(k_pghr_ssum, dim3(ZG_BN_FIXED_Q, nch), dim3(64), 0, st, (int)G, dstr, dpart);
  hipLaunchKernelGGL(k_pghr_bsum_final, dim3(ZG_BN_FIXED_Q), dim3(64), 0, st, (int)nch, dpart, dagg);
  BCHK(hipGetLastError());
  if (!p7_side) {
    hipLaunchKernelGGL(k_pghr_p7, dim3(nb), dim3(64), 0, st, (int)n, ddec, drho, d->comb, dst, dpts);
    BCHK(hipGetLastError());
  }
  // the batch check: every pair of the batch by loop segment (k_pghr_bseg: the key pairs on the sums
  // in block 0, the b pairs from the side stream's lines) and one product tree per segment ->
  // dseg[0..S); the easy part of the S values, their Horner product and ONE hard part
  BCHK(hipMemsetAsync(dbst, ZG_STATUS_OK, ZG_PGHR_FSEG + 1, st));
  BCHK(hipStreamWaitEvent(st, g2join, 0));
  const int K = bseg_k(n);
  const unsigned gb = 1 + bn_blocks(((long long)n + K - 1) / K);  // + the key pairs' block
  hipLaunchKernelGGL(k_pghr_bseg, dim3(gb, ZG_PGHR_FSEG), dim3(64), 0, st, (int)n, K, dpts, dst, dbl, dagg, d->lines,
                     dbseg);
  BCHK(hipGetLastError());
  const size_t stride = gb;  // tree h over dbseg[h gb ..), dbtmp[h gb ..)
  Bq12 *src = dbseg, *dstb = dbtmp;
  for (int m = (int)gb; m > 1; m = (m + 1) / 2) {
    hipLaunchKernelGGL(k_bn_tree, dim3(bn_blocks((m + 1) / 2), ZG_PGHR_FSEG), dim3(64), 0, st, src, dstb, m, stride);
    std::swap(src, dstb);
  }
  BCHK(hipGetLastError());
  hipLaunchKernelGGL(k_pghr_segcopy, dim3(1), dim3(64), 0, st, dseg, src, stride);
  hipLaunchKernelGGL(k_fe_easy, dim3(1), dim3(64), 0, st, ZG_PGHR_FSEG + 1, dseg, dbst, dbw, 1);
  hipLaunchKernelGGL(k_pghr_fe_coop, dim3(1), dim3(64), 0, st, dbw, dbst);
  BCHK(hipGetLastError());
  uint8_t bok = 0;
  BCHK(hipMemcpyAsync(&bok, dbst, 1, hipMemcpyDeviceToHost, st));
  BCHK(hipStreamSynchronize(st));
  if (batch_failed) *batch_failed = bok != ZG_STATUS_OK;
  if (bok != ZG_STATUS_OK) {  // some proof fails: the per-proof path for the exact statuses
    hipLaunchKernelGGL(k_pghr_rho, dim3(nb), dim3(64 * ZG_PGHR_NMUL), 0, st, (int)n, ddec, drho, dst, dmul);
    hipLaunchKernelGGL(k_pghr_combine, dim3(nb), dim3(64), 0, st, (int)n, ddec, dmul, drho, d->comb, dst, dpts);
    BCHK(hipGetLastError());
    const int halves = n < ZG_PGHR_SPLIT_BELOW ? 2 : 1;
    hipLaunchKernelGGL(k_pghr_miller, dim3(nb), dim3(64 * halves), 0, st, (int)n, dpts, d->lines, dst, df, halves);
    BCHK(hipGetLastError());
    hipLaunchKernelGGL(k_fe_easy, dim3(nb), dim3(64), 0, st, (int)n, df, dst, dw, halves);
    BCHK(hipGetLastError());
    hipLaunchKernelGGL(k_fe_exp<1>, dim3(nb), dim3(64), 0, st, (int)n, dst, dw);
    BCHK(hipGetLastError());
    hipLaunchKernelGGL(k_fe_exp<2>, dim3(nb), dim3(64), 0, st, (int)n, dst, dw);
    BCHK(hipGetLastError());
    hipLaunchKernelGGL(k_fe_exp<3>, dim3(nb), dim3(64), 0, st, (int)n, dst, dw);
    BCHK(hipGetLastError());
    hipLaunchKernelGGL(k_fe_last, dim3(nb), dim3(64), 0, st, (int)n, dst, dw);
    BCHK(hipGetLastError());
  }
  if (kernel_ms) BCHK(hipEventRecord(e1, st));
  BCHK(hipMemcpyAsync(status, dst, n, hipMemcpyDeviceToHost, st));
  BCHK(hipStreamSynchronize(st));
  if (kernel_ms) BCHK(hipEventElapsedTime(kernel_ms, e0, e1));
  return ZG_OK;
}

int bn_pairing(hipStream_t st, size_t n, const uint8_t* g1, const uint8_t* g2, uint8_t* gt, std::string* err) {
  if (!n) return ZG_OK;
  uint32_t *a = nullptr, *b = nullptr, *o = nullptr;
  Bq12 *f = nullptr, *w = nullptr;
  uint8_t* ok = nullptr;
  hipError_t e = hipMalloc(&a, 64 * n);
  if (e == hipSuccess) e = hipMalloc(&b, 128 * n);
  if (e == hipSuccess) e = hipMalloc(&o, 384 * n);
  if (e == hipSuccess) e = hipMalloc(&f, sizeof(Bq12) * n);
  if (e == hipSuccess) e = hipMalloc(&w, sizeof(Bq12) * ZG_FE_SLOTS * n);
  if (e == hipSuccess) e = hipMalloc(&ok, n);
  if (e == hipSuccess) e = hipMemsetAsync(ok, ZG_STATUS_OK, n, st);
  if (e == hipSuccess) e = hipMemcpyAsync(a, g1, 64 * n, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(b, g2, 128 * n, hipMemcpyHostToDevice, st);
  const unsigned nb = bn_blocks(n);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_bn_miller1, dim3(nb), dim3(64), 0, st, (int)n, a, b, f);
    hipLaunchKernelGGL(k_fe_easy, dim3(nb), dim3(64), 0, st, (int)n, f, ok, w, 1);
    hipLaunchKernelGGL(k_fe_exp<1>, dim3(nb), dim3(64), 0, st, (int)n, ok, w);
    hipLaunchKernelGGL(k_fe_exp<2>, dim3(nb), dim3(64), 0, st, (int)n, ok, w);
    hipLaunchKernelGGL(k_fe_exp<3>, dim3(nb), dim3(64), 0, st, (int)n, ok, w);
    hipLaunchKernelGGL(k_bn_gt, dim3(nb), dim3(64), 0, st, (int)n, w, o);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(gt, o, 384 * n, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  for (void* q : {(void*)a, (void*)b, (void*)o, (void*)f, (void*)w, (void*)ok})
    if (q) hipFree(q);
  if (e != hipSuccess) {
    *err = std::string("zg_bn254_pairing: ") + hipGetErrorString(e);
    return ZG_E_HIP;
  }
  return ZG_OK;
}

}  // namespace zg
