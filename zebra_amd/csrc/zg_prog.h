// zg_prog.h -- staged-program engine: lane = proof, wave = product.
//
// A program from zg_prog_tables.h is a sequence of stages of independent Fq2 products over
// "atoms" (program inputs and earlier products), plus output linear forms. A block runs
// one program for 64 proofs (one per lane): in each stage, wave w computes product
// lo + w (+ NW, ...) for all 64 proofs. Every lane of a wave executes the same product, so
// control flow and the term tables are wave-uniform (scalar loads, scalar branches on the
// coefficients). Atoms live in global memory (L2-resident) in a coalesced layout
//   atom a of the block's 64 proofs = 6 rows of 64 x 16 B  (Fq2 = 2 x 12 limbs = 6 x uint4)
// so per-lane state is one product at a time (small VGPR count, high occupancy), and the
// product-level parallelism of a stage (4-13 products) becomes wave-level parallelism.
// The atom space of a block (<= 24 atoms x 6 KB) is a static LDS array: one block per CU.
#pragma once
#include "zg_prog_tables.h"
#include "zg_tower.h"

namespace zg {

#define ZG_ATOM_ROWS 6  // uint4 rows per Fq2

struct AtomSpace {
  uint4* base;  // block's region: [atom][row][64]
  __device__ __forceinline__ Fq2 get(int atom) const {
    const int lane = threadIdx.x & 63;
    const uint4* p = base + (size_t)atom * ZG_ATOM_ROWS * 64 + lane;
    uint4 r[ZG_ATOM_ROWS];
#pragma unroll
    for (int q = 0; q < ZG_ATOM_ROWS; q++) r[q] = p[q * 64];
    Fq2 v;
#pragma unroll
    for (int q = 0; q < 3; q++) {
      v.c0.l[4 * q + 0] = r[q].x;
      v.c0.l[4 * q + 1] = r[q].y;
      v.c0.l[4 * q + 2] = r[q].z;
      v.c0.l[4 * q + 3] = r[q].w;
      v.c1.l[4 * q + 0] = r[3 + q].x;
      v.c1.l[4 * q + 1] = r[3 + q].y;
      v.c1.l[4 * q + 2] = r[3 + q].z;
      v.c1.l[4 * q + 3] = r[3 + q].w;
    }
    return v;
  }
  __device__ __forceinline__ void put(int atom, const Fq2& v) const {
    const int lane = threadIdx.x & 63;
    uint4* p = base + (size_t)atom * ZG_ATOM_ROWS * 64 + lane;
#pragma unroll
    for (int q = 0; q < 3; q++) {
      p[q * 64] = make_uint4(v.c0.l[4 * q], v.c0.l[4 * q + 1], v.c0.l[4 * q + 2], v.c0.l[4 * q + 3]);
      p[(3 + q) * 64] = make_uint4(v.c1.l[4 * q], v.c1.l[4 * q + 1], v.c1.l[4 * q + 2], v.c1.l[4 * q + 3]);
    }
  }
};

// c * x for a small integer c (binary method)
ZG_INL Fq fq_mul_small(const Fq& x, int c) {
  int m = c < 0 ? -c : c;
  Fq r = fp_zero<FqM>(), pw = x;
  while (m) {
    if (m & 1) r = fq_add(r, pw);
    m >>= 1;
    if (m) pw = fq_dbl(pw);
  }
  return c < 0 ? fq_neg(r) : r;
}

// acc + (c0 + c1 u) * x   (c0, c1 wave-uniform: the branches are scalar)
ZG_INL Fq2 f2_gauss_madd(const Fq2& acc, const Fq2& x, int c0, int c1) {
  if (c1 == 0) {
    if (c0 == 1) return f2_add(acc, x);
    if (c0 == -1) return f2_sub(acc, x);
    return f2_add(acc, {fq_mul_small(x.c0, c0), fq_mul_small(x.c1, c0)});
  }
  if (c0 == 1 && c1 == 1) return f2_add(acc, f2_mul_nr(x));  // xi
  if (c0 == -1 && c1 == -1) return f2_sub(acc, f2_mul_nr(x));
  Fq r0 = fq_sub(fq_mul_small(x.c0, c0), fq_mul_small(x.c1, c1));
  Fq r1 = fq_add(fq_mul_small(x.c0, c1), fq_mul_small(x.c1, c0));
  return f2_add(acc, {r0, r1});
}

__device__ __forceinline__ int wave_uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ Fq2 prog_form(const AtomSpace& at, int form) {
  form = wave_uniform(form);
  const int off = PROG_FORMS[form][0], n = PROG_FORMS[form][1];
  Fq2 acc = f2_zero();
  for (int q = 0; q < n; q++) {
    const PTerm t = PROG_TERMS[off + q];
    acc = f2_gauss_madd(acc, at.get(t.atom), t.c0, t.c1);
  }
  return acc;
}

// all stages of program pid; nw = waves in the block
__device__ __forceinline__ void prog_run_stages(int pid, const AtomSpace& at, int nw) {
  const ProgDesc& d = PROG_DESC[pid];
  const int wave = wave_uniform(threadIdx.x >> 6);
  for (int s = 0; s < d.nstage; s++) {
    const int lo = d.stage[s][0], hi = d.stage[s][1];
    for (int k = lo + wave; k < hi; k += nw) at.put(d.nin + k, f2_mul(prog_form(at, d.L + k), prog_form(at, d.R + k)));
    __syncthreads();
  }
}

// outputs j = wave (+ nw ...) of program pid, evaluated into v[] (slots per wave)
__device__ __forceinline__ Fq2 prog_out(int pid, const AtomSpace& at, int j) {
  return prog_form(at, PROG_DESC[pid].O + j);
}

}  // namespace zg
