// zg_coop.h -- lane-cooperative Fq12 engine: one wave (64 lanes) evaluates one chain of
// Fq12 operations (the final exponentiation, the product of a node's Miller values), with
// every Fq product of an operation on its own lane.
//
// A single-lane Fq12 product is 54 dependent-in-program-order Fq multiplications; the
// final exponentiation is ~15,600 of them in sequence, which on one lane is pure latency
// (97 ms in round 1). Here an operation runs as levels of independent lane tasks (tables
// from gen_coop.py): up to 54 Fq products on separate lanes, then the Karatsuba recombination
// as levels of short linear forms (Fq2 products, Fq6 products, outputs). Linear forms are
// evaluated branch-free with lazy reduction (LazyAcc): the lanes of a wave evaluate
// different forms without diverging. Operands and the form tables live in LDS.
#pragma once
#include "zg_coop_tables.h"
#include "zg_pairing.h"

namespace zg {

#define ZG_COOP_SLOTS 8
// LDS copy of a form: up to 8 terms packed from t[0], a zero term ends the list (a real term
// has a nonzero coefficient); 16 B so that one ds_read_b128 fetches the whole form.
struct alignas(16) CoopFormL {
  int16_t t[ZG_COOP_MAXT];
};
struct alignas(16) CoopWS {
  Fq slot[ZG_COOP_SLOTS][12];       // Fq12 registers, coefficient order of f12_coeffs
  Fq v[24 + ZG_COOP_MAXATOMS];      // op workspace: inputs a (0..11), b (12..23), then atoms
  CoopFormL forms[ZG_COOP_NFORMS];  // LDS copy of COOP_FORMS (per-lane table reads at LDS latency)
};
static_assert(sizeof(Fq) == 48 && offsetof(CoopWS, v) % 16 == 0 && offsetof(CoopWS, forms) % 16 == 0, "LDS layout");
// The workspace always lives in LDS; kernels hand it around as a generic pointer, so the hot
// paths re-qualify it once (LDS instructions instead of flat ones with null checks).
#define ZG_LDS __attribute__((address_space(3)))
typedef ZG_LDS CoopWS LdsWS;
ZG_INL LdsWS* lds_ws(CoopWS* ws) { return (LdsWS*)ws; }
ZG_INL void lds_get(const ZG_LDS Fq* p, u32x4& a, u32x4& b, u32x4& c) {
  const ZG_LDS u32x4* q = (const ZG_LDS u32x4*)p;
  a = q[0];
  b = q[1];
  c = q[2];
}
ZG_INL Fq lds_fq(const ZG_LDS Fq* p) {
  u32x4 a, b, c;
  lds_get(p, a, b, c);
  return {{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w}};
}
ZG_INL void lds_put(ZG_LDS Fq* p, const Fq& x) {
  ZG_LDS u32x4* q = (ZG_LDS u32x4*)p;
  q[0] = u32x4{x.l[0], x.l[1], x.l[2], x.l[3]};
  q[1] = u32x4{x.l[4], x.l[5], x.l[6], x.l[7]};
  q[2] = u32x4{x.l[8], x.l[9], x.l[10], x.l[11]};
}

// Lazy linear forms  sum_t c_t x_t  (|c_t| < 128, <= 8 terms, x_t any 384-bit value):
// one 64-bit accumulator per limb, no carry chain per term. A negative term adds
// |c| * ~x  (= |c| (2^384 - 1 - x)), i.e. -|c| x + |c| - |c| 2^384; the per-lane count B of
// such |c| is corrected once at the end by adding B + B (p - 2^384 mod p).
struct LazyAcc {
  uint64_t l[12];
  uint32_t b;
};
ZG_INL void lazy_zero(LazyAcc& a) {
#pragma unroll
  for (int i = 0; i < 12; i++) a.l[i] = 0;
  a.b = 0;
}
ZG_INL void lazy_term(LazyAcc& a, const Fq& x, int c) {
  const uint32_t m = (uint32_t)(c < 0 ? -c : c);
  const uint32_t neg = c < 0 ? 0xffffffffu : 0u;
#pragma unroll
  for (int i = 0; i < 12; i++) a.l[i] += (uint64_t)(x.l[i] ^ neg) * m;  // v_xor + v_mad_u64_u32
  a.b += m & neg;
}
// value mod p, < 2.2 p (a valid Montgomery-product operand); canon = true: < p
ZG_INL Fq lazy_finish(const LazyAcc& a, bool canon) {
  uint32_t w[13];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {  // carry-propagate (each l[i] < 2^42)
    const uint64_t s = a.l[i] + c;
    w[i] = (uint32_t)s;
    c = s >> 32;
  }
  w[12] = (uint32_t)c;
  uint64_t t = (uint64_t)w[0] + a.b;  // + B + B (p - 2^384 mod p)
  c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint64_t s = (uint64_t)a.b * FQ_NEG_R[i] + (i == 0 ? t : (uint64_t)w[i]) + c;
    w[i] = (uint32_t)s;
    c = s >> 32;
  }
  w[12] += (uint32_t)c;  // W < 2^395 < 2^14 p
  // q = floor(float(W >> 352) * (1 - 2^-20) 2^352 / p): W/p - 1.2 < q <= W/p
  const float top = (float)w[12] * 4294967296.0f + (float)w[11];
  const uint32_t q = (uint32_t)(top * FQ_QSCALE);
  Fq r;
  uint32_t borrow = 0, carry = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint64_t qp = (uint64_t)q * FQ_P[i] + carry;
    carry = (uint32_t)(qp >> 32);
    const uint64_t d = (uint64_t)w[i] - (uint32_t)qp - borrow;
    r.l[i] = (uint32_t)d;
    borrow = (uint32_t)(d >> 63);
  }
  if (canon) r = fp_reduce_once<FqM>(fp_reduce_once<FqM>(r));
  return r;
}

ZG_INL void lazy_term4(LazyAcc& a, const u32x4& x0, const u32x4& x1, const u32x4& x2, int c) {
  const Fq x = {{x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w, x2.x, x2.y, x2.z, x2.w}};
  lazy_term(a, x, c);
}

// One linear form: the descriptor in one LDS read, then its terms two at a time with both
// operands' loads in flight together (a zero coefficient adds nothing).
ZG_INL Fq coop_form(const LdsWS* ws, int fi, bool canon) {
  const u32x4 d = *(const ZG_LDS u32x4*)&ws->forms[fi];
  const uint32_t w[4] = {d.x, d.y, d.z, d.w};
  LazyAcc acc;
  lazy_zero(acc);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int t0 = (int)(int16_t)(w[q] & 0xffffu), t1 = (int)(int16_t)(w[q] >> 16);
    if (t0 == 0) break;
    u32x4 a0, a1, a2, b0, b1, b2;
    lds_get(&ws->v[t0 & 0xff], a0, a1, a2);
    lds_get(&ws->v[t1 & 0xff], b0, b1, b2);
    lazy_term4(acc, a0, a1, a2, t0 >> 8);
    lazy_term4(acc, b0, b1, b2, t1 >> 8);
  }
  return lazy_finish(acc, canon);
}

// copy the form tables into the block's LDS (once per kernel, before any coop op)
__device__ void coop_init(CoopWS* ws_g) {
  LdsWS* ws = lds_ws(ws_g);
  for (int i = threadIdx.x; i < ZG_COOP_NFORMS * ZG_COOP_MAXT; i += blockDim.x) {
    const CoopForm& f = COOP_FORMS[i / ZG_COOP_MAXT];
    const int q = i % ZG_COOP_MAXT;
    ws->forms[i / ZG_COOP_MAXT].t[q] = q < f.n ? f.t[q] : (int16_t)0;
  }
  __syncthreads();
}

// slot[dst] = op(slot[a], slot[b]) for op = ZG_COOP_{MUL,SQR,CSQR,M014}; dst may alias a / b.
// Level 0: one Fq product per lane; later levels: one linear form per lane; the last level
// writes the 12 output coefficients.
__device__ void coop_run(CoopWS* ws_g, int opid, int dst, int a, int b) {
  LdsWS* ws = lds_ws(ws_g);
  const int lane = threadIdx.x & 63;
  if (lane < 24) lds_put(&ws->v[lane], lds_fq(&ws->slot[lane < 12 ? a : b][lane < 12 ? lane : lane - 12]));
  __syncthreads();
  const CoopOp& op = COOP_OPS[opid];
  const int nlev = op.nlev;
  int base = 24;
  for (int l = 0; l < nlev; l++) {
    const int cnt = op.cnt[l], off = op.off[l];
    if (lane < cnt) {
      if (l == 0) {
        const Fq x = coop_form(ws, off + 2 * lane, false), y = coop_form(ws, off + 2 * lane + 1, false);
        lds_put(&ws->v[base + lane], fq_mul(x, y));
      } else {
        const Fq x = coop_form(ws, off + lane, l == nlev - 1);
        lds_put(l == nlev - 1 ? &ws->slot[dst][lane] : &ws->v[base + lane], x);
      }
    }
    base += cnt;
    __syncthreads();
  }
}

// 384-bit a + b and a + p - b without reduction (a, b < p: results < 2p, valid fq_mul operands)
ZG_INL Fq raw_add(const Fq& a, const Fq& b) {
  Fq r;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    c += (uint64_t)a.l[i] + b.l[i];
    r.l[i] = (uint32_t)c;
    c >>= 32;
  }
  return r;
}
ZG_INL Fq raw_sub_p(const Fq& a, const Fq& b) {
  Fq r;
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    c += (int64_t)a.l[i] + FQ_P[i] - b.l[i];
    r.l[i] = (uint32_t)c;
    c >>= 32;
  }
  return r;
}

// Granger-Scott squaring (cyclotomic subgroup only) in ONE product level: lane k < 18 squares
// a coefficient of an Fp4 pair with its operands formed in code (gen_coop.py
// check_csqr1_products pins the mapping), then 12 lanes evaluate the output forms of ZG_COOP_CSQR1
// (products and inputs, <= 4 terms). Same value as coop_csqr; about half its latency.
__device__ void coop_csqr1(CoopWS* ws_g, int dst, int a) {
  LdsWS* ws = lds_ws(ws_g);
  const int lane = threadIdx.x & 63;
  if (lane < 12) lds_put(&ws->v[lane], lds_fq(&ws->slot[a][lane]));
  __syncthreads();
  if (lane < 18) {
    const int p = lane / 6, w = (lane % 6) >> 1, h = lane & 1;
    const int ja = p == 0 ? 0 : p == 1 ? 3 : 1, jb = p == 0 ? 4 : p == 1 ? 2 : 5;
    const int j = w == 1 ? jb : ja;
    Fq x0 = lds_fq(&ws->v[2 * j]), x1 = lds_fq(&ws->v[2 * j + 1]);
    if (w == 2) {
      x0 = fq_add(x0, lds_fq(&ws->v[2 * jb]));
      x1 = fq_add(x1, lds_fq(&ws->v[2 * jb + 1]));
    }
    Fq l = x0, r = x1;
    if (h) {
      l = raw_add(x0, x1);
      r = raw_sub_p(x0, x1);
    }
    lds_put(&ws->v[24 + lane], fq_mul(l, r));
  }
  __syncthreads();
  const CoopOp& op = COOP_OPS[ZG_COOP_CSQR1];
  if (lane < 12) lds_put(&ws->slot[dst][lane], coop_form(ws, op.off[1] + lane, true));
  __syncthreads();
}

__device__ __forceinline__ void coop_mul(CoopWS* ws, int dst, int a, int b) { coop_run(ws, ZG_COOP_MUL, dst, a, b); }
__device__ __forceinline__ void coop_sqr(CoopWS* ws, int dst, int a) { coop_run(ws, ZG_COOP_SQR, dst, a, a); }
// squaring in the cyclotomic subgroup (Granger-Scott); only valid after the easy part
__device__ __forceinline__ void coop_csqr(CoopWS* ws, int dst, int a) { coop_run(ws, ZG_COOP_CSQR, dst, a, a); }
// slot[dst] = slot[a] * line, the line in slot[b] as written by coop_line (mul_by_014)
__device__ __forceinline__ void coop_mul014(CoopWS* ws, int dst, int a, int b) {
  coop_run(ws, ZG_COOP_M014, dst, a, b);
}

__device__ __forceinline__ void coop_copy(CoopWS* ws, int dst, int a) {
  const int lane = threadIdx.x & 63;
  if (lane < 12) ws->slot[dst][lane] = ws->slot[a][lane];
  __syncthreads();
}
__device__ __forceinline__ void coop_conj(CoopWS* ws, int dst, int a) {
  const int lane = threadIdx.x & 63;
  if (lane < 12) ws->slot[dst][lane] = lane < 6 ? ws->slot[a][lane] : fq_neg(ws->slot[a][lane]);
  __syncthreads();
}
__device__ __forceinline__ void coop_set_one(CoopWS* ws, int dst) {
  const int lane = threadIdx.x & 63;
  if (lane < 12) ws->slot[dst][lane] = lane == 0 ? fq_one() : fp_zero<FqM>();
  __syncthreads();
}

ZG_INL Fq2 coop_get2(const CoopWS* ws, int s, int j) { return {ws->slot[s][2 * j], ws->slot[s][2 * j + 1]}; }

// Frobenius x -> x^(p^k): lane j < 6 maps Fq2 coefficient j
__device__ void coop_frob(CoopWS* ws, int dst, int a, int k) {
  const int lane = threadIdx.x & 63;
  Fq2 v;
  if (lane < 6) {
    v = coop_get2(ws, a, lane);
    if (k & 1) v = f2_conj(v);
    const uint32_t(*c6)[12] = nullptr;
    const int pos = lane % 3;  // v power within the Fq6 half
    if (pos == 1) c6 = k == 1 ? FROB6_C1_1 : k == 2 ? FROB6_C1_2 : FROB6_C1_3;
    if (pos == 2) c6 = k == 1 ? FROB6_C2_1 : k == 2 ? FROB6_C2_2 : FROB6_C2_3;
    if (c6) v = f2_mul(v, f2_const(c6));
    if (lane >= 3) v = f2_mul(v, f2_const(k == 1 ? FROB12_C1_1 : k == 2 ? FROB12_C1_2 : FROB12_C1_3));
  }
  __syncthreads();
  if (lane < 6) {
    ws->slot[dst][2 * lane] = v.c0;
    ws->slot[dst][2 * lane + 1] = v.c1;
  }
  __syncthreads();
}

// slot[dst] = slot[a]^-1 through the norm to Fq6 (round 6: the tower arithmetic off lane 0 -- on one lane
// it was four Fq6 and twelve Fq2 products in sequence, ~0.35 ms of the final exponentiation's ~1.7):
//   g = f conj(f) = f0^2 - v f1^2 in Fq6 (coop_mul), then the Fq6 inverse of g on lanes 0..5 (its six,
//   then three, then three Fq2 products in parallel), the Fq2 norm's Fq inverse on lane 0 (zg_bingcd.h),
//   and f^-1 = conj(f) g^-1 (coop_mul). Uses slot tmp (!= dst, a) and the op workspace v.
__device__ void coop_inv(CoopWS* ws, int dst, int a, int tmp) {
  const int lane = threadIdx.x & 63;
  coop_conj(ws, tmp, a);
  coop_mul(ws, dst, a, tmp);  // g: coefficients 0..5 = (t0, t1, t2), 6..11 = 0
  Fq2* x = reinterpret_cast<Fq2*>(&ws->v[24]);  // exchange: x[0..5] products, x[6..8] c, x[9..11] q, x[12] nin
  if (lane < 6) {  // t0^2, t1 t2, t2^2, t0 t1, t1^2, t0 t2
    const int i = lane == 0 || lane == 3 || lane == 5 ? 0 : lane == 1 || lane == 4 ? 1 : 2;
    const int j = lane == 0 ? 0 : lane == 1 || lane == 2 ? 2 : lane == 3 || lane == 4 ? 1 : 2;
    x[lane] = f2_mul(coop_get2(ws, dst, i), coop_get2(ws, dst, j));
  }
  __syncthreads();
  if (lane < 3) {  // c0 = t0^2 - xi t1 t2, c1 = xi t2^2 - t0 t1, c2 = t1^2 - t0 t2
    const Fq2 u = x[2 * lane], w = x[2 * lane + 1];
    x[6 + lane] = lane == 0 ? f2_sub(u, f2_mul_nr(w)) : lane == 1 ? f2_sub(f2_mul_nr(u), w) : f2_sub(u, w);
  }
  __syncthreads();
  if (lane < 3)  // q = t0 c0, t2 c1, t1 c2
    x[9 + lane] = f2_mul(coop_get2(ws, dst, lane == 0 ? 0 : lane == 1 ? 2 : 1), x[6 + lane]);
  __syncthreads();
  if (lane == 0) {  // n = q0 + xi (q1 + q2); n^-1 = conj(n) / (n0^2 + n1^2)
    const Fq2 n = f2_add(x[9], f2_mul_nr(f2_add(x[10], x[11])));
    const Fq ni = fq_inv(fq_add(fq_sqr(n.c0), fq_sqr(n.c1)));
    x[12] = {fq_mul(n.c0, ni), fq_neg(fq_mul(n.c1, ni))};
  }
  __syncthreads();
  Fq2 gi;
  if (lane < 3) gi = f2_mul(x[6 + lane], x[12]);
  __syncthreads();
  if (lane < 6) {  // g^-1 = (c0, c1, c2) n^-1 as an Fq12 with a zero w part
    ws->slot[dst][2 * lane] = lane < 3 ? gi.c0 : fp_zero<FqM>();
    ws->slot[dst][2 * lane + 1] = lane < 3 ? gi.c1 : fp_zero<FqM>();
  }
  __syncthreads();
  coop_mul(ws, dst, tmp, dst);
}

// slot[dst] = conj(slot[a]^x)  (exp_by_x of the pairing chain; a cyclotomic)
__device__ void coop_exp_by_x(CoopWS* ws, int dst, int a, uint64_t x, int tmp) {
  coop_copy(ws, tmp, a);
  int top = 63;
  while (!((x >> top) & 1ull)) top--;
  for (int i = top - 1; i >= 0; i--) {
    coop_csqr1(ws, tmp, tmp);
    if ((x >> i) & 1ull) coop_mul(ws, tmp, tmp, a);
  }
  coop_conj(ws, dst, tmp);
}

// pairing 0.14.2 Bls12::final_exponentiation of slot[in] -> slot[out]. Uses slots 0..7.
// Slot map: 0 in/f, 1 r, 2 y0, 3 y1, 4 y2, 5 y3, 6 tmp, 7 f2
__device__ void coop_final_exp(CoopWS* ws, int in, int out) {
  enum { F = 0, Rr = 1, Y0 = 2, Y1 = 3, Y2 = 4, Y3 = 5, T = 6, F2 = 7 };
  if (in != F) coop_copy(ws, F, in);
  coop_conj(ws, Rr, F);         // f1 = conj(f)
  coop_inv(ws, F2, F, T);       // f2 = f^-1
  coop_mul(ws, Rr, Rr, F2);     // r = f1 * f2
  coop_copy(ws, F2, Rr);        // f2 = r
  coop_frob(ws, Rr, Rr, 2);
  coop_mul(ws, Rr, Rr, F2);     // r = frob2(r) * f2
  const uint64_t x = BLS_X;
  coop_csqr1(ws, Y0, Rr);                // y0 = r^2
  coop_exp_by_x(ws, Y1, Y0, x, T);       // y1 = y0^x
  coop_exp_by_x(ws, Y2, Y1, x >> 1, T);  // y2 = y1^(x/2)
  coop_conj(ws, Y3, Rr);                 // y3 = conj(r)
  coop_mul(ws, Y1, Y1, Y3);
  coop_conj(ws, Y1, Y1);
  coop_mul(ws, Y1, Y1, Y2);
  coop_exp_by_x(ws, Y2, Y1, x, T);
  coop_exp_by_x(ws, Y3, Y2, x, T);
  coop_conj(ws, Y1, Y1);
  coop_mul(ws, Y3, Y3, Y1);
  coop_conj(ws, Y1, Y1);
  coop_frob(ws, Y1, Y1, 3);
  coop_frob(ws, Y2, Y2, 2);
  coop_mul(ws, Y1, Y1, Y2);
  coop_exp_by_x(ws, Y2, Y3, x, T);
  coop_mul(ws, Y2, Y2, Y0);
  coop_mul(ws, Y2, Y2, Rr);
  coop_mul(ws, Y1, Y1, Y2);
  coop_frob(ws, Y2, Y3, 1);
  coop_mul(ws, out, Y1, Y2);
}

// load / store an Fq12 between a slot and global memory (tower structs)
__device__ void coop_load(CoopWS* ws, int dst, const Fq12& g) {
  const int lane = threadIdx.x & 63;
  if (lane < 12) {
    const Fq* c = reinterpret_cast<const Fq*>(&g);
    ws->slot[dst][lane] = c[lane];
  }
  __syncthreads();
}
__device__ void coop_store(const CoopWS* ws, int s, Fq12& g) {
  const int lane = threadIdx.x & 63;
  if (lane < 12) {
    Fq* c = reinterpret_cast<Fq*>(&g);
    c[lane] = ws->slot[s][lane];
  }
  __syncthreads();
}
__device__ bool coop_is_one(const CoopWS* ws, int s) {
  __shared__ int flag;
  const int lane = threadIdx.x & 63;
  if (lane == 0) flag = 1;
  __syncthreads();
  if (lane < 12) {
    Fq want = lane == 0 ? fq_one() : fp_zero<FqM>();
    if (!fq_eq(ws->slot[s][lane], want)) atomicAnd(&flag, 0);
  }
  __syncthreads();
  return flag != 0;
}

}  // namespace zg
