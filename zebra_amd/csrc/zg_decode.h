// zg_decode.h -- the decode kernels (SURVEY.md 8(a) rows a3/a4/a8 inputs), compiled in their own
// translation unit (zg_decode.hip) so that the register budget of the launch bounds reaches
// every function they call: at two waves per SIMD two independent point streams share each
// SIMD (one wave alone issues a VALU instruction every 4 cycles, two every 2).
#pragma once
#include "zg_batch.h"

namespace zg {

// ZG_DECODE_FQD (default 1): the subgroup checks and GLV products in lazy digits (zg_fqd.h);
// 0: the word form (zg_curve.h / zg_groth16.h)
#ifndef ZG_DECODE_FQD
#define ZG_DECODE_FQD 1
#endif
#if ZG_DECODE_FQD
#define ZG_DEC_SUBGROUP g1_in_subgroup_d
// GLV r_i A_i one column per step (64 doublings + 64 mixed additions of +-P or +-(P + sigma P),
// operands selected from registers). g1_glv_mul_w2 (two columns per step from an eight-entry
// per-lane table: 32 additions fewer) is 2.5% faster on the decode kernel but gathers its table
// entries from the private segment with a different index per lane -- 2.1 GB of HBM traffic per
// 64k launch against 0.18 GB (profiles/r04p_*, r04o_*)
#ifndef ZG_DEC_GLV
#define ZG_DEC_GLV g1_glv_mul_d
#endif
#else
#define ZG_DEC_SUBGROUP g1_in_subgroup
#define ZG_DEC_GLV g1_glv_mul
#endif

// K1 + K2 + K3 as three launches.
//
// k_decode_sqrt: one wave per (64 proofs, G1 point), blocks alternating A / C of the same 64
// proofs: flags, x < p, Fq sqrt and the sign choice of G1Compressed::into_affine. The affine
// point goes to ptAC (inf = the point did not decode).
//
// k_decode_points: one wave per (64 proofs, job), the jobs of a decoded point being independent
// of each other. Two grid layouts (G = npad / 64 groups of 64 proofs):
//   K4 (cglv = 0: shards from ZG_K4_MIN padded proofs, or any batch with others in flight):
//     blocks [0, G) the GLV products [r_i] A_i (to affine -> ptA); [G, 3G) alternate the G1
//     subgroup checks of A and C (sigma(P) = -[x^2] P -> okbits); [3G, 4G) decompress B (Fq2
//     sqrt; its G2 subgroup check rides on k_batch_lines). C needs no per-proof scalar product:
//     sum r_i C_i is K4's Pippenger MSM (zg_msm.h) on the side stream.
//   GLV C sums (cglv = 1: a lone batch below ZG_K4_MIN): blocks [0, G) [r_i] A_i as above,
//     [G, 2G) the GLV products [r_i] C_i into the C-sum tree leaves ctree[npad + i] (the proof's
//     key; infinity for the other keys), which the side stream sums up the tree (k_tree_c); the
//     subgroup checks move to [2G, 4G) and B to [4G, 5G).
// The heavy waves are dispatched first, two per SIMD (ZG_DECODE_WPE), and the B waves fill the
// tail. The scalar products run before the statuses are known (a point that did not decode
// skips its own; the rest are masked by k_decode_finish).
#if defined(ZG_TU_DECODE_SQRT)  // zg_decode_sqrt.hip: every callee inlined, no call frames
#ifndef ZG_DECODE_SQRT_WPE
#define ZG_DECODE_SQRT_WPE ZG_DECODE_WPE
#endif
__global__ void __launch_bounds__(64, ZG_DECODE_SQRT_WPE) k_decode_sqrt(BatchBufs b) {
  const int role = blockIdx.x & 1;  // 0 A, 1 C (wave-uniform)
  const int i = (blockIdx.x >> 1) * 64 + (threadIdx.x & 63);
  // the pipeline's first kernel clears the batch flags (B subgroup failures, fused-wait failure):
  // no fill launch in front of the batch
  if (blockIdx.x == 0 && threadIdx.x < 2) b.bfail[threadIdx.x] = 0;
  if (i >= b.npad) return;
  G1A p;
  p.inf = true;
  if (i < b.n && g1_decompress(b.proofs + (size_t)i * 192 + (role == 0 ? 0 : 144), &p, false) != DEC_OK)
    p.inf = true;
  b.ptAC[(size_t)role * b.npad + i] = p;
}
#else

// JOB < 0: every job in one launch (grid 4G, the product's only launch); JOB = 0 / 1 / 2: that job
// alone (grid G / 2G / G: round 4's per-job profiles, profiles/r04b_kernel_stats_decode_split.csv,
// compiled only by tooling)
// cglv (small shards, ZG_K4_MIN): the GLV products r_i C_i run here too, as blocks [G, 2G) beside
// those of A, and go to the C-sum tree leaves (ctree[npad + i], the proof's key; the other keys'
// entries the point at infinity) -- the side stream then sums them by the tree levels instead of
// K4's Pippenger buckets. k_decode_finish masks the leaves of proofs that are not pending.
template <int JOB>
__global__ void __launch_bounds__(64, ZG_DECODE_WPE) k_decode_points(BatchBufs b, int cglv) {
  const int G = (b.npad + 63) / 64, nglv = cglv ? 2 * G : G;
  const int blk = JOB < 0 ? (int)blockIdx.x : JOB == 0 ? (int)blockIdx.x : JOB == 1 ? nglv + (int)blockIdx.x
                                                                                     : nglv + 2 * G + (int)blockIdx.x;
  // 0 GLV (A, or C from block G on), 1 subgroup, 2 B (wave-uniform)
  const int job = JOB >= 0 ? JOB : blk < nglv ? 0 : blk < nglv + 2 * G ? 1 : 2;
  const int role = job == 0 ? (blk < G ? 0 : 1) : job == 2 ? 2 : ((blk - nglv) & 1);  // 0 A, 1 C, 2 B
  const int grp = job == 0 ? (blk < G ? blk : blk - G) : job == 2 ? blk - nglv - 2 * G : (blk - nglv) >> 1;
  const int i = grp * 64 + (threadIdx.x & 63);
  if (i >= b.npad) return;
  if (job == 2) {
    G2A q;
    q.inf = true;
    bool ok = false;
    if (i < b.n) ok = g2_decompress(b.proofs + (size_t)i * 192 + 48, &q, false) == DEC_OK;
    b.ptB[i] = q;
    b.okbits[3 * i + 2] = ok;
    return;
  }
  const G1A p = b.ptAC[(size_t)role * b.npad + i];
  const bool ok = !p.inf;
  if (job == 1) {
    b.okbits[3 * i + role] = ok && ZG_DEC_SUBGROUP(p);
    return;
  }
  uint64_t ra = 0, rb = 0;
  if (ok) batch_scalar_ab(b.r + (size_t)i * 16, &ra, &rb);
  if (role == 1) {  // r_i C_i -> the C-sum tree leaf of the proof's key
    const int kind = i < b.n ? b.kinds[i] : 0;
    const G1J o = ok ? ZG_DEC_GLV(p, ra, rb) : jac_infinity<Fq>();
    for (int k = 0; k < ZG_NKINDS; k++) b.ctree[((size_t)b.npad + i) * ZG_NKINDS + k] = k == kind ? o : jac_infinity<Fq>();
    return;
  }
  G1A o;
  o.inf = true;
  if (ok) o = jac_to_aff(ZG_DEC_GLV(p, ra, rb));
  b.ptA[i] = o;
}

// k_decode_finish: lane = proof. bellman's precedence (sapling.rs:157-167): input canonicity,
// Proof::read, input count; statuses; masks the point results of proofs that are not pending;
// the Fr leaves r_i, r_i x_ij of its kind, the other kinds' leaves zero.
__global__ void __launch_bounds__(64) k_decode_finish(BatchBufs b) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  if (i >= b.npad) return;
  const bool live = i < b.n;
  const int leaf = b.npad + i;
  const int kind = live ? b.kinds[i] : 0;
  uint8_t st = ST_PENDING;
  int k = 0, kk = 0;
  // the inputs are read where they are used (canonicity here, the Fr leaves below): no per-lane
  // array of them, so no private segment
  const uint8_t* in = b.inputs + (size_t)i * 288;
  if (live) {
    k = b.ninputs ? b.ninputs[i] : KIND_NINPUTS[kind];
    kk = k < ZG_MAX_INPUTS ? k : ZG_MAX_INPUTS;
    const bool ok = b.okbits[3 * i] && b.okbits[3 * i + 1] && b.okbits[3 * i + 2];
    bool canon = true;
#pragma unroll
    for (int j = 0; j < ZG_MAX_INPUTS; j++)
      if (j < kk) canon = canon && fp_lt_modulus<FrM>(fr_limbs_from_le(in + 32 * j));
    if (!canon)
      st = ST_INPUT_NONCANONICAL;
    else if (!ok)
      st = ST_DECODE_INVALID;
    else if (k + 1 != b.vks[kind].ic_len)
      st = ST_MALFORMED_VK;
    b.status[i] = st;
  }
  const bool pend = live && st == ST_PENDING;
  if (!pend) b.ptA[i].inf = true;
  // the C-sum leaves (small shards: r_i C_i from k_decode_points; bisection rewrites them anyway)
  if (!pend)
    for (int kd = 0; kd < ZG_NKINDS; kd++) b.ctree[(size_t)leaf * ZG_NKINDS + kd] = jac_infinity<Fq>();
  // B still owes its subgroup check (k_batch_lines) if Proof::read got that far
  b.ptB[i].inf = !(live && (st == ST_PENDING || st == ST_MALFORMED_VK));
  for (int kd = 0; kd < ZG_NKINDS; kd++) {
    Fr* s = b.stree + (leaf * ZG_NKINDS + kd) * ZG_MAX_IC;
    for (int m = 0; m < ZG_MAX_IC; m++) s[m] = fp_zero<FrM>();
  }
  if (pend) {
    uint64_t ra, rb;
    batch_scalar_ab(b.r + (size_t)i * 16, &ra, &rb);
    const Fr rf = batch_scalar_fr(ra, rb);
    Fr* s = b.stree + (leaf * ZG_NKINDS + kind) * ZG_MAX_IC;
    s[0] = rf;
#pragma unroll
    for (int j = 0; j < ZG_MAX_INPUTS; j++)
      if (j < kk) s[1 + j] = fr_mul(rf, fr_to_mont(fr_limbs_from_le(in + 32 * j)));
  }
}

#endif  // ZG_TU_DECODE_SQRT

}  // namespace zg
