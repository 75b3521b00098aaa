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
struct CoopWS {
  Fq slot[ZG_COOP_SLOTS][12];       // Fq12 registers, coefficient order of f12_coeffs
  Fq v[24 + ZG_COOP_MAXATOMS];      // op workspace: inputs a (0..11), b (12..23), then atoms
  CoopForm forms[ZG_COOP_NFORMS];   // LDS copy of COOP_FORMS (per-lane table reads at LDS latency)
};

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

__device__ __forceinline__ Fq coop_form(const CoopWS* ws, int fi, bool canon) {
  const CoopForm& f = ws->forms[fi];
  LazyAcc acc;
  lazy_zero(acc);
  const int n = f.n;
  for (int q = 0; q < n; q++) {
    const int v = f.t[q];
    lazy_term(acc, ws->v[v & 0xff], v >> 8);
  }
  return lazy_finish(acc, canon);
}

// copy the form tables into the block's LDS (once per kernel, before any coop op)
__device__ void coop_init(CoopWS* ws) {
  const uint16_t* src = reinterpret_cast<const uint16_t*>(COOP_FORMS);
  uint16_t* dst = reinterpret_cast<uint16_t*>(ws->forms);
  constexpr int nw = (int)(sizeof(CoopForm) * ZG_COOP_NFORMS / 2);
  for (int i = threadIdx.x; i < nw; i += blockDim.x) dst[i] = src[i];
  __syncthreads();
}

// slot[dst] = op(slot[a], slot[b]) for op = ZG_COOP_{MUL,SQR,CSQR,M014}; dst may alias a / b.
// Level 0: one Fq product per lane; later levels: one linear form per lane; the last level
// writes the 12 output coefficients.
__device__ void coop_run(CoopWS* ws, int opid, int dst, int a, int b) {
  const int lane = threadIdx.x & 63;
  if (lane < 12) {
    ws->v[lane] = ws->slot[a][lane];
    ws->v[12 + lane] = ws->slot[b][lane];
  }
  __syncthreads();
  const CoopOp& op = COOP_OPS[opid];
  const int nlev = op.nlev;
  int base = 24;
  for (int l = 0; l < nlev; l++) {
    const int cnt = op.cnt[l], off = op.off[l];
    if (lane < cnt) {
      if (l == 0) {
        const Fq x = coop_form(ws, off + 2 * lane, false), y = coop_form(ws, off + 2 * lane + 1, false);
        ws->v[base + lane] = fq_mul(x, y);
      } else {
        const Fq x = coop_form(ws, off + lane, l == nlev - 1);
        if (l == nlev - 1)
          ws->slot[dst][lane] = x;
        else
          ws->v[base + lane] = x;
      }
    }
    base += cnt;
    __syncthreads();
  }
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

// slot[dst] = slot[a]^-1 (one lane: the tower inversion is a few Fq2 products + one Fq inverse)
__device__ void coop_inv(CoopWS* ws, int dst, int a) {
  const int lane = threadIdx.x & 63;
  if (lane == 0) {
    Fq12 f;
    Fq2* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
    for (int j = 0; j < 6; j++) *c[j] = coop_get2(ws, a, j);
    Fq6 t = f6_sub(f6_mul(f.c0, f.c0), f6_mul_nr(f6_mul(f.c1, f.c1)));
    Fq2 c0 = f2_sub(f2_sqr(t.c0), f2_mul_nr(f2_mul(t.c1, t.c2)));
    Fq2 c1 = f2_sub(f2_mul_nr(f2_sqr(t.c2)), f2_mul(t.c0, t.c1));
    Fq2 c2 = f2_sub(f2_sqr(t.c1), f2_mul(t.c0, t.c2));
    Fq2 n = f2_add(f2_mul(t.c0, c0), f2_mul_nr(f2_add(f2_mul(t.c2, c1), f2_mul(t.c1, c2))));
    Fq ni = fq_inv_vartime(fq_add(fq_sqr(n.c0), fq_sqr(n.c1)));
    Fq2 nin = {fq_mul(n.c0, ni), fq_neg(fq_mul(n.c1, ni))};
    Fq6 ti = {f2_mul(c0, nin), f2_mul(c1, nin), f2_mul(c2, nin)};
    Fq12 r = {f6_mul(f.c0, ti), f6_neg(f6_mul(f.c1, ti))};
    Fq2* o[6] = {&r.c0.c0, &r.c0.c1, &r.c0.c2, &r.c1.c0, &r.c1.c1, &r.c1.c2};
    for (int j = 0; j < 6; j++) {
      ws->slot[dst][2 * j] = o[j]->c0;
      ws->slot[dst][2 * j + 1] = o[j]->c1;
    }
  }
  __syncthreads();
}

// slot[dst] = conj(slot[a]^x)  (exp_by_x of the pairing chain; a cyclotomic)
__device__ void coop_exp_by_x(CoopWS* ws, int dst, int a, uint64_t x, int tmp) {
  coop_copy(ws, tmp, a);
  int top = 63;
  while (!((x >> top) & 1ull)) top--;
  for (int i = top - 1; i >= 0; i--) {
    coop_csqr(ws, tmp, tmp);
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
  coop_inv(ws, F2, F);          // f2 = f^-1
  coop_mul(ws, Rr, Rr, F2);     // r = f1 * f2
  coop_copy(ws, F2, Rr);        // f2 = r
  coop_frob(ws, Rr, Rr, 2);
  coop_mul(ws, Rr, Rr, F2);     // r = frob2(r) * f2
  const uint64_t x = BLS_X;
  coop_csqr(ws, Y0, Rr);                 // y0 = r^2
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
