// zg_decode.h -- the decode kernels (SURVEY.md 8(a) rows a3/a4/a8 inputs), compiled in their own
// translation unit (zg_decode.hip) so that the register budget of the launch bounds reaches
// every function they call: at two waves per SIMD two independent point streams share each
// SIMD (one wave alone issues a VALU instruction every 4 cycles, two every 2).
#pragma once
#include "zg_batch.h"

namespace zg {

// K1 + K2 + K3 as two launches.
//
// k_decode_points: one wave per (64 proofs, point). Blocks [0, 2G) alternate A / C of the same
// 64 proofs: Fq sqrt, G1 subgroup check and the GLV product [r_i] P (A: to affine -> ptA,
// C: Jacobian -> the proof's ctree leaf of its kind); blocks [2G, 3G) decompress B (Fq2 sqrt;
// its G2 subgroup check rides on k_batch_lines). The heavy G1 waves are dispatched first, two
// per SIMD (ZG_DECODE_WPE), and the shorter B waves fill the tail. The scalar products run
// before the statuses are known (a failed decode skips its own; the rest are masked below).
// A 64k batch is 3072 waves: 3x the waves of one lane-per-proof kernel, at twice its issue rate
// per SIMD.
__global__ void __launch_bounds__(64, ZG_DECODE_WPE) k_decode_points(BatchBufs b) {
  const int G = (b.npad + 63) / 64;
  const int blk = blockIdx.x;
  const int role = blk < 2 * G ? (blk & 1) : 2;  // 0 A, 1 C, 2 B (wave-uniform)
  const int grp = blk < 2 * G ? (blk >> 1) : blk - 2 * G;
  const int lane = threadIdx.x & 63;
  const int i = grp * 64 + lane;
  const bool inb = i < b.npad, live = i < b.n;
  const int leaf = b.npad + i;
  bool ok = false;
  if (role == 2) {
    G2A q;
    q.inf = true;
    if (live) ok = g2_decompress(b.proofs + (size_t)i * 192 + 48, &q, false) == DEC_OK;
    if (inb) b.ptB[i] = q;
  } else {
    G1A p;
    p.inf = true;
    if (live) ok = g1_decompress(b.proofs + (size_t)i * 192 + (role == 0 ? 0 : 144), &p) == DEC_OK;
    uint64_t ra = 0, rb = 0;
    if (ok) batch_scalar_ab(b.r + (size_t)i * 16, &ra, &rb);
    if (role == 0) {
      G1A o;
      o.inf = true;
      if (ok) o = jac_to_aff(g1_glv_mul(p, ra, rb));
      if (inb) b.ptA[i] = o;
    } else if (ok) {
      b.ctree[leaf * ZG_NKINDS + b.kinds[i]] = g1_glv_mul(p, ra, rb);
    }
  }
  if (inb) b.okbits[3 * i + role] = ok;
}

// k_decode_finish: lane = proof. bellman's precedence (sapling.rs:157-167): input canonicity,
// Proof::read, input count; statuses; masks the point results of proofs that are not pending;
// the Fr leaves r_i, r_i x_ij of its kind, the other kinds' leaves zero / infinity.
__global__ void __launch_bounds__(64) k_decode_finish(BatchBufs b) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  if (i >= b.npad) return;
  const bool live = i < b.n;
  const int leaf = b.npad + i;
  const int kind = live ? b.kinds[i] : 0;
  uint8_t st = ST_PENDING;
  Fr x[ZG_MAX_INPUTS];
  int k = 0, kk = 0;
  if (live) {
    k = b.ninputs ? b.ninputs[i] : KIND_NINPUTS[kind];
    kk = k < ZG_MAX_INPUTS ? k : ZG_MAX_INPUTS;
    const bool ok = b.okbits[3 * i] && b.okbits[3 * i + 1] && b.okbits[3 * i + 2];
    if (!inputs_canonical(b.inputs + (size_t)i * 288, kk, x))
      st = ST_INPUT_NONCANONICAL;
    else if (!ok)
      st = ST_DECODE_INVALID;
    else if (k + 1 != b.vks[kind].ic_len)
      st = ST_MALFORMED_VK;
    b.status[i] = st;
  }
  const bool pend = live && st == ST_PENDING;
  if (!pend) b.ptA[i].inf = true;
  // B still owes its subgroup check (k_batch_lines) if Proof::read got that far
  b.ptB[i].inf = !(live && (st == ST_PENDING || st == ST_MALFORMED_VK));
  for (int kd = 0; kd < ZG_NKINDS; kd++) {
    if (kd != kind || !pend) b.ctree[leaf * ZG_NKINDS + kd] = jac_infinity<Fq>();
    Fr* s = b.stree + (leaf * ZG_NKINDS + kd) * ZG_MAX_IC;
    for (int m = 0; m < ZG_MAX_IC; m++) s[m] = fp_zero<FrM>();
  }
  if (pend) {
    uint64_t ra, rb;
    batch_scalar_ab(b.r + (size_t)i * 16, &ra, &rb);
    const Fr rf = batch_scalar_fr(ra, rb);
    Fr* s = b.stree + (leaf * ZG_NKINDS + kind) * ZG_MAX_IC;
    s[0] = rf;
    for (int j = 0; j < kk; j++) s[1 + j] = fr_mul(rf, fr_to_mont(x[j]));
  }
}

}  // namespace zg
