// zg_lines.hip -- the R-chain as straight-line code, lane = proof (its own translation unit, so
// the launch bounds' register budget reaches every inlined product; cf. zg_decode.hip).
//
// Per proof: G2Prepared(B_i) of pairing 0.14.2 -- 63 doubling steps and 5 addition steps of
// [x] B in homogeneous projective coordinates (zg_pairing.h line_double / line_add, the same
// formulas) -- with the `ell` scaling by r_i A_i folded in: step n writes the triple
// (c2, c1 px, c0 py) = (A, B, C) to lines[n][proof] for the f-chain. The last point is [x] B,
// so the G2 subgroup check of B (psi(B) = [u] B) closes the kernel. Same values as the staged
// program k_batch_lines (zg_kernels.h: lane = proof, wave = product, LDS atoms, a barrier per
// round): here every lane runs its proof's products back to back in registers, no LDS, no
// barriers, two waves per SIMD -- the issue pattern of the decode kernels.
#include <hip/hip_runtime.h>

#include "../../include/zg.h"
#include "zg_lines.h"

namespace zg {

template <int WPE>
__global__ void __launch_bounds__(64, WPE) k_batch_lines_lane(BatchBufs b, Fq2* lines) {
  const int proof = blockIdx.x * 64 + (threadIdx.x & 63);
  if (proof >= b.npad) return;
  const bool act = proof < b.n && b.status[proof] == ST_PENDING && !b.ptA[proof].inf;
  const bool chk = proof < b.n && !b.ptB[proof].inf;  // B owes its subgroup check
  // B and r_i A_i stay in HBM (re-read per step, L1 / L2 hits): registers hold only the running
  // point and one step's temporaries
  const G2A* pq = &b.ptB[chk ? proof : 0];
  const G1A* pa = &b.ptA[act ? proof : 0];
  __shared__ uint4 lds_pt[3 * ZG_ATOM_ROWS * 64];  // X, Y, Z of the block's 64 proofs (18 KB)
  AtomSpace st{lds_pt};
  if (chk) {
    st.put(0, pq->x);
    st.put(1, pq->y);
  } else {
    st.put(0, f2_one());
    st.put(1, f2_one());
  }
  st.put(2, f2_one());
  int n = 0;
  for (int i = ZG_XH_TOP; i >= -1; i--) {
    ls_double(st, pa, lines + ((size_t)(n++) * b.npad + proof) * 3, act);
    if (i >= 0 && ((ZG_XH >> i) & 1ull)) ls_add(st, pq, pa, lines + ((size_t)(n++) * b.npad + proof) * 3, act && chk);
  }
  const G2J r = {st.get(0), st.get(1), st.get(2)};
  // r = [x] B (Jacobian). B in G2  <=>  psi(B) = [u] B = -[x] B  <=>  X = psi_x Z^2, Y = -psi_y Z^3,
  // Z != 0 (the step formulas are exact unless they degenerate, which only a B outside G2 can
  // make happen, and then Z = 0)
  if (chk) {
    const G2A s = g2_psi(*pq);
    const Fq2 z2 = ls_sqr(r.z), z3 = ls_mul(z2, r.z);
    const bool in_g2 = !f2_is_zero(r.z) && f2_eq(r.x, ls_mul(s.x, z2)) && f2_eq(r.y, f2_neg(ls_mul(s.y, z3)));
    if (!in_g2) {
      atomicAdd(b.bfail, 1);
      b.status[proof] = ST_DECODE_INVALID;
      const int leaf = b.npad + proof, kind = b.kinds[proof];
      for (int m = 0; m < ZG_MAX_IC; m++) b.stree[(leaf * ZG_NKINDS + kind) * ZG_MAX_IC + m] = fp_zero<FrM>();
      b.ctree[(size_t)leaf * ZG_NKINDS + kind] = jac_infinity<Fq>();  // small shards' C-sum leaf
    }
  }
}

// wpe: waves per SIMD the register budget is sized for (2: 256 VGPRs, 1: 512)
hipError_t launch_lines_lane(unsigned groups, hipStream_t st, const BatchBufs& b, Fq2* lines, int wpe) {
  if (wpe == 1)
    hipLaunchKernelGGL(k_batch_lines_lane<1>, dim3(groups), dim3(64), 0, st, b, lines);
  else
    hipLaunchKernelGGL(k_batch_lines_lane<2>, dim3(groups), dim3(64), 0, st, b, lines);
  return hipGetLastError();
}

}  // namespace zg
