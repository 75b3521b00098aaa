// zg_decode.h -- the per-proof decode kernel (SURVEY.md 8(a) rows a3/a4/a8 inputs), compiled in
// its own translation unit (zg_decode.hip) so that the register budget of its launch bounds
// reaches every function it calls: at two waves per SIMD two independent proof streams
// share each SIMD (one wave alone issues a VALU instruction every 4 cycles, two every 2).
#pragma once
#include "zg_batch.h"

namespace zg {

// K1 + K2 + K3: decode/subgroup-check A, B, C; public-input canonicity and count; r_i A_i;
// r_i C_i and the Fr scalars r_i, r_i x_ij as tree leaves. Lane = proof; a block = 64 proofs.
// Three independent chains per proof:
//   A: Fq sqrt, G1 subgroup check, [r_i] A_i by GLV columns, to affine
//   B: Fq2 sqrt (its G2 subgroup check rides on k_batch_lines); public inputs, status, Fr
//      scalar leaves
//   C: Fq sqrt, G1 subgroup check, [r_i] C_i by GLV columns
// W = 1: one wave runs all three (a 64k batch already puts one wave on every SIMD);
// W = 3: one wave per chain, for small batches / shards (3x the waves, ~1/3 the latency).
template <int W>
__global__ void __launch_bounds__(64 * W, ZG_DECODE_WPE) k_batch_decode(BatchBufs b) {
  __shared__ uint8_t ok_sh[3][64];
  __shared__ uint8_t st_sh[64];
  const int lane = threadIdx.x & 63, wave = W == 1 ? 0 : wave_uniform(threadIdx.x >> 6);
  const bool runA = W == 1 || wave == 0, runB = W == 1 || wave == 1, runC = W == 1 || wave == 2;
  const int i = blockIdx.x * 64 + lane;
  const bool inb = i < b.npad, live = i < b.n;
  const int leaf = b.npad + i;
  const int kind = live ? b.kinds[i] : 0;
  G1A pa, pc;
  G2A q;
  pa.inf = pc.inf = q.inf = true;
  bool oka = false, okb = false, okc = false;
  uint8_t st_in = ST_PENDING;
  Fr x[ZG_MAX_INPUTS];
  int k = 0, kk = 0;
  if (runB) {
    if (inb)
      for (int kd = 0; kd < ZG_NKINDS; kd++)
        for (int m = 0; m < ZG_MAX_IC; m++) b.stree[(leaf * ZG_NKINDS + kd) * ZG_MAX_IC + m] = fp_zero<FrM>();
    if (live) {
      k = b.ninputs ? b.ninputs[i] : KIND_NINPUTS[kind];
      kk = k < ZG_MAX_INPUTS ? k : ZG_MAX_INPUTS;
      if (!inputs_canonical(b.inputs + (size_t)i * 288, kk, x)) st_in = ST_INPUT_NONCANONICAL;
      // the G2 subgroup check of B is fused into k_batch_lines: the R-chain ends at [x] B
      okb = g2_decompress(b.proofs + (size_t)i * 192 + 48, &q, false) == DEC_OK;
    }
  }
  if (runA) {
    if (inb)
      for (int kd = 0; kd < ZG_NKINDS; kd++) b.ctree[leaf * ZG_NKINDS + kd] = jac_infinity<Fq>();
    if (live) oka = g1_decompress(b.proofs + (size_t)i * 192, &pa) == DEC_OK;
  }
  if (runC && live) okc = g1_decompress(b.proofs + (size_t)i * 192 + 144, &pc) == DEC_OK;
  if (W > 1) {
    ok_sh[wave][lane] = wave == 0 ? oka : wave == 1 ? okb : okc;
    __syncthreads();
    oka = ok_sh[0][lane];
    okb = ok_sh[1][lane];
    okc = ok_sh[2][lane];
  }
  // bellman's precedence (sapling.rs:157-167): input canonicity, Proof::read, input count
  uint8_t st = ST_PENDING;
  if (runB) {
    if (st_in != ST_PENDING)
      st = st_in;
    else if (!(oka && okb && okc))
      st = ST_DECODE_INVALID;
    else if (live && k + 1 != b.vks[kind].ic_len)
      st = ST_MALFORMED_VK;
    if (live) b.status[i] = st;
  }
  if (W > 1) {
    if (wave == 1) st_sh[lane] = st;
    __syncthreads();
    st = st_sh[lane];
  }
  const bool pend = live && st == ST_PENDING;
  uint64_t ra = 0, rb = 0;
  if (pend) batch_scalar_ab(b.r + (size_t)i * 16, &ra, &rb);
  if (runA) {
    G1A o;
    o.inf = true;
    if (pend) o = jac_to_aff(g1_glv_mul(pa, ra, rb));
    if (inb) b.ptA[i] = o;
  }
  if (runC && pend) b.ctree[leaf * ZG_NKINDS + kind] = g1_glv_mul(pc, ra, rb);
  if (runB && inb) {  // B still owes its subgroup check (k_batch_lines) if Proof::read got that far
    G2A qq = q;
    qq.inf = !(live && (st == ST_PENDING || st == ST_MALFORMED_VK));
    b.ptB[i] = qq;
  }
  if (runB && pend) {
    const Fr rf = batch_scalar_fr(ra, rb);
    Fr* s = b.stree + (leaf * ZG_NKINDS + kind) * ZG_MAX_IC;
    s[0] = rf;
    for (int j = 0; j < kk; j++) s[1 + j] = fr_mul(rf, fr_to_mont(x[j]));
  }
}

}  // namespace zg
