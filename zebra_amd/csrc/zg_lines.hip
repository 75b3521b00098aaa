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

// ---- The affine R-chain (ZG_LINES_AFFINE, round 6): G2Prepared(B_i) in affine
// coordinates, every step's denominator inverted by Montgomery's trick over the K proofs of a lane
// (lane-local: K - 1 products forward, 2 (K - 1) back, ONE Fq inversion per lane and step) -- XL
// additionally chains the 64 lanes' products across the wave (prefix / suffix scans through lane
// shuffles, one inversion of the wave's product, as VERDICT r05 asked); on SIMT hardware a wave
// executes an inversion once whether one lane or all 64 need it, so XL costs the scans and saves
// nothing (measured). Denominators are batched as Fq norms (1 / d = conj(d) / N(d)).
// Output: the lines normalised to a unit v w coefficient, a + b v + v w, as lines[n][2][npad] (a, b)
// -- two Fq2 per proof and step instead of the projective three -- consumed by k_line_prod's AQ4
// program (21 products per four lines against Q4I's 27). (1/py, px/py) of each proof sit after the
// lines (aux) and are batch-inverted the same way at the start. A proof without a line (inactive,
// padding) gets (0, 0): the line v w = w^3, whose square is in Fq2, so the final exponentiation
// maps it to 1 (oracle/bls12_381.py AFFINE_IDLE_LINE). A denominator that vanishes -- only a B
// outside G2 can make one (its chain would reach O or +-B) -- is replaced by 1 so that the lane's
// other proofs keep exact inverses, and that B fails its subgroup check. The last point is [x] B,
// so the check psi(B) = -[x] B closes the kernel as in the projective chains.
template <int K, bool XL>
__global__ void __launch_bounds__(64, 1) k_batch_lines_aff(BatchBufs b, Fq2* lines) {
  const int lane = threadIdx.x & 63;
  __shared__ uint4 lds_pt[2 * K * ZG_ATOM_ROWS * 64];  // x_k, y_k of the lane's K proofs (Fq2 slots)
  __shared__ uint4 lds_fq[2 * K * 3 * 64];              // per k: the exclusive prefix of the norms, the norm
  const AtomSpace st{lds_pt};
  auto fq_put = [&](int s, const Fq& v) {
    uint4* p = lds_fq + (size_t)s * 3 * 64 + lane;
#pragma unroll
    for (int q = 0; q < 3; q++) p[q * 64] = make_uint4(v.l[4 * q], v.l[4 * q + 1], v.l[4 * q + 2], v.l[4 * q + 3]);
  };
  auto fq_get = [&](int s) {
    const uint4* p = lds_fq + (size_t)s * 3 * 64 + lane;
    Fq v;
#pragma unroll
    for (int q = 0; q < 3; q++) {
      const uint4 r = p[q * 64];
      v.l[4 * q] = r.x;
      v.l[4 * q + 1] = r.y;
      v.l[4 * q + 2] = r.z;
      v.l[4 * q + 3] = r.w;
    }
    return v;
  };
  // the inverse of this lane's product `run` (XL: through the wave's product)
  auto lane_inverse = [&](const Fq& run) {
    if constexpr (!XL) {
      return fq_inv(run);
    } else {
      auto shfl = [&](const Fq& v, int src) {
        Fq r;
#pragma unroll
        for (int i = 0; i < 12; i++) r.l[i] = (uint32_t)__shfl((int)v.l[i], src, 64);
        return r;
      };
      const Fq one = fq_one();
      Fq pin = run, sin = run;  // inclusive prefix / suffix products over the lanes
      for (int s = 1; s < 64; s <<= 1) {
        const Fq up = shfl(pin, lane >= s ? lane - s : lane), dn = shfl(sin, lane + s < 64 ? lane + s : lane);
        pin = ls_fqmul(pin, lane >= s ? up : one);
        sin = ls_fqmul(sin, lane + s < 64 ? dn : one);
      }
      const Fq tinv = fq_inv(shfl(pin, 63));  // the wave's product: ONE inversion per wave
      const Fq pex = shfl(pin, lane > 0 ? lane - 1 : 0), sex = shfl(sin, lane < 63 ? lane + 1 : 63);
      return ls_fqmul(ls_fqmul(tinv, lane > 0 ? pex : one), lane < 63 ? sex : one);
    }
  };
  Fq2* aux = lines + (size_t)2 * ZG_NCOEFF * b.npad;  // (1/py, px/py) per proof
  const G2A gen = g2_generator();
  uint32_t chk = 0, bad = 0;  // bit k: B owes its subgroup check; a denominator of proof k vanished
  auto proof_of = [&](int k) { return (int)((blockIdx.x * K + k) * 64 + lane); };
  // setup: the points, and (1/py, px/py) by the same trick
  {
    Fq run = fq_one();
    for (int k = 0; k < K; k++) {
      const int pr = proof_of(k);
      const bool c = pr < b.n && !b.ptB[pr].inf;
      chk |= c ? 1u << k : 0u;
      const G2A q = c ? b.ptB[pr] : gen;
      st.put(2 * k, q.x);
      st.put(2 * k + 1, q.y);
      const bool a = pr < b.npad && (pr < b.n && b.status[pr] == ST_PENDING && !b.ptA[pr].inf);
      const Fq py = a ? b.ptA[pr].y : fq_one();
      fq_put(2 * k, run);
      run = ls_fqmul(run, py);
    }
    Fq inv = lane_inverse(run);
    for (int k = K - 1; k >= 0; k--) {
      const int pr = proof_of(k);
      const bool a = pr < b.npad && (pr < b.n && b.status[pr] == ST_PENDING && !b.ptA[pr].inf);
      const Fq py = a ? b.ptA[pr].y : fq_one();
      const Fq ipy = ls_fqmul(inv, fq_get(2 * k));
      inv = ls_fqmul(inv, py);
      if (pr < b.npad) aux[pr] = a ? Fq2{ipy, ls_fqmul(b.ptA[pr].x, ipy)} : f2_zero();
    }
  }
  int n = 0;
  for (int i = ZG_XH_TOP; i >= -1; i--) {
    for (int pass = 0; pass < 2; pass++) {
      if (pass == 1 && (i < 0 || !((ZG_XH >> i) & 1ull))) break;
      const bool dbl = pass == 0;
      Fq run = fq_one();
      for (int k = 0; k < K; k++) {
        const int pr = proof_of(k);
        const G2A* q = (chk >> k) & 1u ? &b.ptB[pr] : &gen;
        const Fq2 d = dbl ? f2_dbl(st.get(2 * k + 1)) : f2_sub(q->x, st.get(2 * k));
        Fq nn = ls_norm(d);
        if (fq_is_zero(nn)) {
          bad |= 1u << k;
          nn = fq_one();
        }
        fq_put(2 * k, run);
        fq_put(2 * k + 1, nn);
        run = ls_fqmul(run, nn);
      }
      Fq inv = lane_inverse(run);
      for (int k = K - 1; k >= 0; k--) {
        const int pr = proof_of(k);
        const G2A* q = (chk >> k) & 1u ? &b.ptB[pr] : &gen;
        const Fq ninv = ls_fqmul(inv, fq_get(2 * k));
        inv = ls_fqmul(inv, fq_get(2 * k + 1));
        Fq2 x = st.get(2 * k), y = st.get(2 * k + 1), la, lb;
        const Fq2 ab = pr < b.npad ? aux[pr] : f2_zero();
        ls_aff_step(x, y, q, dbl, ninv, ab, &la, &lb);
        if (pr < b.npad) {
          lines[((size_t)n * 2) * b.npad + pr] = la;
          lines[((size_t)n * 2 + 1) * b.npad + pr] = lb;
        }
        st.put(2 * k, x);
        st.put(2 * k + 1, y);
      }
      n++;
    }
  }
  // (x, y) = [x] B. B in G2  <=>  psi(B) = [u] B = -[x] B
  for (int k = 0; k < K; k++) {
    if (!((chk >> k) & 1u)) continue;
    const int pr = proof_of(k);
    const G2A s = g2_psi(b.ptB[pr]);
    const bool in_g2 = !((bad >> k) & 1u) && f2_eq(st.get(2 * k), s.x) && f2_eq(st.get(2 * k + 1), f2_neg(s.y));
    if (!in_g2) {
      atomicAdd(b.bfail, 1);
      b.status[pr] = ST_DECODE_INVALID;
      const int leaf = b.npad + pr, kind = b.kinds[pr];
      for (int m = 0; m < ZG_MAX_IC; m++) b.stree[(leaf * ZG_NKINDS + kind) * ZG_MAX_IC + m] = fp_zero<FrM>();
      b.ctree[(size_t)leaf * ZG_NKINDS + kind] = jac_infinity<Fq>();
    }
  }
}

// the affine R-chain over npad proofs, K proofs per lane (lane l of block g: proofs (g K + k) 64 + l),
// xl: the cross-lane variant
hipError_t launch_lines_aff(hipStream_t st, const BatchBufs& b, Fq2* lines, int k, int xl) {
  const unsigned blocks = (unsigned)((b.npad + 64 * k - 1) / (64 * k));
  if (k == 2 && !xl) hipLaunchKernelGGL((k_batch_lines_aff<2, false>), dim3(blocks), dim3(64), 0, st, b, lines);
  else if (k == 4 && !xl) hipLaunchKernelGGL((k_batch_lines_aff<4, false>), dim3(blocks), dim3(64), 0, st, b, lines);
  else if (k == 8 && !xl) hipLaunchKernelGGL((k_batch_lines_aff<8, false>), dim3(blocks), dim3(64), 0, st, b, lines);
  else if (k == 4 && xl) hipLaunchKernelGGL((k_batch_lines_aff<4, true>), dim3(blocks), dim3(64), 0, st, b, lines);
  else return hipErrorInvalidValue;
  return hipGetLastError();
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
