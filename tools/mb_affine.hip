// Microbenchmark (tooling): is an AFFINE G2 R-chain with a batched Fq2 inversion cheaper than the
// product's projective R-chain (zg_lines.h ls_double, pairing 0.14.2's doubling_step)?
//
// Every lane runs `iters` dependent steps on its own G2 point (64k lanes, two waves per SIMD, as
// k_batch_lines_lane in flight). Kernels:
//   PROJ   ls_double: 8 Fq2 squarings + 3 Fq2 products + 2 Fq2 x Fq (the scaled line coefficients)
//   AFF<K> K points per lane (K proofs), one step each: d_k = 2 y_k, Montgomery's trick over the K
//          denominators (K - 1 products forward, 2 (K - 1) back) and ONE Fq2 inversion (norm, Fq
//          binary-GCD inverse zg_bingcd.h, 2 Fq products); then per point lambda = 3 x^2 / (2 y),
//          x' = lambda^2 - 2x, y' = lambda (x - x') - y and the two line coefficients an affine line
//          normalised to a unit coefficient needs: lambda px/py and (lambda x - y) / py (Fq2 x Fq)
//   INV    the Fq2 inversion alone; MUL / SQR the Fq2 product / squaring alone (29-bit digits)
// Checks: after the run, the projective point of PROJ converted to affine equals AFF<1>'s point
// (same start, same number of doublings) on every lane -- the affine formulas are the same group law.
// Prints ns per lane-step (throughput at full occupancy) of each kernel; the cost model in DESIGN.md
// §4c uses these numbers. (PROJ and AFF<K> hold their points in registers here and spill; the product's
// lane R-chain keeps its point in LDS with 0 B of scratch, so the model is built from MUL / SQR / MULFQ /
// INV, which do not spill, and checked against the product kernel's own measured step time.)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../zebra_amd/csrc/zg_lines.h"

using namespace zg;

#define CK(e)                                                         \
  do {                                                                \
    hipError_t r = (e);                                               \
    if (r != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(r), __LINE__); \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

struct Pt {
  Fq2 x, y;
};

enum { PROJ = 0, MUL = 1, SQR = 2, INV = 3, MULFQ = 4, AFF1 = 11, AFF2 = 12, AFF4 = 14 };

__device__ __forceinline__ Fq2 xr(const Fq2& a, const Fq2& b) {
  Fq2 r;
  for (int i = 0; i < 12; i++) {
    r.c0.l[i] = a.c0.l[i] ^ b.c0.l[i];
    r.c1.l[i] = a.c1.l[i] ^ b.c1.l[i];
  }
  return r;
}

// one affine doubling step for K points with a batched inversion; acc collects the line coefficients
template <int K>
__device__ __forceinline__ void aff_step(Pt* p, const Fq& pxpy, const Fq& ipy, Fq2& acc) {
  Fq2 pre[K];
  pre[0] = f2_dbl(p[0].y);
#pragma unroll
  for (int k = 1; k < K; k++) pre[k] = ls_mul(pre[k - 1], f2_dbl(p[k].y));
  Fq2 inv = f2_inv(pre[K - 1]);
#pragma unroll
  for (int k = K - 1; k >= 0; k--) {
    Fq2 ik = inv;
    if (k > 0) {
      ik = ls_mul(inv, pre[k - 1]);
      inv = ls_mul(inv, f2_dbl(p[k].y));
    }
    const Fq2 x2 = ls_sqr(p[k].x);
    const Fq2 lam = ls_mul(f2_add(f2_dbl(x2), x2), ik);
    const Fq2 nx = f2_sub(ls_sqr(lam), f2_dbl(p[k].x));
    const Fq2 t = ls_mul(lam, p[k].x);
    const Fq2 ny = f2_sub(f2_sub(t, ls_mul(lam, nx)), p[k].y);
    acc = xr(acc, ls_mulfq(lam, pxpy));
    acc = xr(acc, ls_mulfq(f2_sub(t, p[k].y), ipy));
    p[k] = {nx, ny};
  }
}

template <int MODE>
__global__ void __launch_bounds__(64, 2) k_run(const Pt* in, const Fq* px, Fq2* out, Pt* pout, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const Fq s = px[i];
  Fq2 acc = f2_zero();
  if (MODE == PROJ) {
    LinesHost st;
    st.put(0, in[i].x);
    st.put(1, in[i].y);
    st.put(2, f2_one());
    G1A pa = {s, s, false};
    for (int it = 0; it < iters; it++) {
      Fq2 d[3];
      ls_double(st, &pa, d, true);
      acc = xr(acc, xr(d[0], xr(d[1], d[2])));
    }
    // to affine for the check: x = X / Z^2, y = Y / Z^3
    const Fq2 zi = f2_inv(st.get(2)), zi2 = ls_sqr(zi);
    pout[i] = {ls_mul(st.get(0), zi2), ls_mul(st.get(1), ls_mul(zi2, zi))};
  } else if (MODE == MUL || MODE == SQR || MODE == INV || MODE == MULFQ) {
    Fq2 a = in[i].x, b = in[i].y;
    for (int it = 0; it < iters; it++)
      a = MODE == MUL ? ls_mul(a, b) : MODE == SQR ? ls_sqr(a) : MODE == MULFQ ? ls_mulfq(a, s) : f2_add(f2_inv(a), b);
    acc = a;
  } else {
    constexpr int K = MODE > 10 ? MODE - 10 : 1;
    Pt p[K];
#pragma unroll
    for (int k = 0; k < K; k++) p[k] = in[(i * K + k) % (gridDim.x * blockDim.x)];
    for (int it = 0; it < iters; it++) aff_step<K>(p, s, s, acc);
    pout[i] = p[0];
  }
  out[i] = acc;
}

template <int MODE>
static float run(int blocks, const Pt* in, const Fq* px, Fq2* out, Pt* pout, int iters) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms = 0;
  for (int rep = 0; rep < 2; rep++) {
    CK(hipEventRecord(e0));
    k_run<MODE><<<blocks, 64>>>(in, px, out, pout, iters);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
  }
  return ms;
}

int main(int argc, char** argv) {
  const int lanes = argc > 1 ? atoi(argv[1]) : 65536, iters = argc > 2 ? atoi(argv[2]) : 16;
  const int blocks = lanes / 64;
  // every lane starts at the G2 generator (the timing does not depend on the point; the check
  // compares the two formulas' doubling chains)
  Pt* h = (Pt*)malloc(sizeof(Pt) * lanes);
  Fq* hp = (Fq*)malloc(sizeof(Fq) * lanes);
  // the G2 generator (x = x0 + x1 u, y = y0 + y1 u), big-endian canonical
  static const char* G2HEX[4] = {
      "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8",
      "13e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e",
      "0ce5d527727d6e118cc9cdc6da2e351aadfd9baa8cbdd3a76d429a695160d12c923ac9cc3baca289e193548608b82801",
      "0606c4a02ea734cc32acd2b02bc28b99cb3e287e85a763af267492ab572e99ab3f370d275cec1da1aaa9075ff05f79be"};
  Fq gc[4];
  for (int c = 0; c < 4; c++) {
    uint8_t be[48];
    for (int k = 0; k < 48; k++) sscanf(G2HEX[c] + 2 * k, "%2hhx", &be[k]);
    gc[c] = fq_to_mont(fq_limbs_from_be(be));
  }
  for (int i = 0; i < lanes; i++) {
    h[i] = {{gc[0], gc[1]}, {gc[2], gc[3]}};
    hp[i] = fq_one();
  }
  Pt *din, *dp0, *dp1;
  Fq* dpx;
  Fq2* dout;
  CK(hipMalloc(&din, sizeof(Pt) * lanes));
  CK(hipMalloc(&dp0, sizeof(Pt) * lanes));
  CK(hipMalloc(&dp1, sizeof(Pt) * lanes));
  CK(hipMalloc(&dpx, sizeof(Fq) * lanes));
  CK(hipMalloc(&dout, sizeof(Fq2) * lanes));
  CK(hipMemcpy(din, h, sizeof(Pt) * lanes, hipMemcpyHostToDevice));
  CK(hipMemcpy(dpx, hp, sizeof(Fq) * lanes, hipMemcpyHostToDevice));
  // check: PROJ and AFF<1> reach the same affine point after `iters` doublings of G2
  k_run<PROJ><<<blocks, 64>>>(din, dpx, dout, dp0, iters);
  k_run<AFF1><<<blocks, 64>>>(din, dpx, dout, dp1, iters);
  CK(hipDeviceSynchronize());
  Pt* a = (Pt*)malloc(sizeof(Pt) * lanes);
  Pt* b = (Pt*)malloc(sizeof(Pt) * lanes);
  CK(hipMemcpy(a, dp0, sizeof(Pt) * lanes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b, dp1, sizeof(Pt) * lanes, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < lanes; i++)
    bad += !(f2_eq(a[i].x, b[i].x) && f2_eq(a[i].y, b[i].y));
  printf("affine vs projective doubling chains (%d steps): %d of %d lanes differ\n", iters, bad, lanes);
  const double steps = (double)lanes * iters;
  struct {
    const char* name;
    float ms;
    double per;  // lane-steps per launch per lane-iteration
  } r[] = {{"PROJ  ls_double (8 S + 3 M + 2 Fq2xFq)", run<PROJ>(blocks, din, dpx, dout, dp0, iters), 1},
           {"MUL   Fq2 product", run<MUL>(blocks, din, dpx, dout, dp0, iters), 1},
           {"SQR   Fq2 squaring", run<SQR>(blocks, din, dpx, dout, dp0, iters), 1},
           {"INV   Fq2 inversion (binary GCD)", run<INV>(blocks, din, dpx, dout, dp0, iters), 1},
           {"MULFQ Fq2 x Fq", run<MULFQ>(blocks, din, dpx, dout, dp0, iters), 1},
           {"AFF1  affine step, 1 proof/lane", run<AFF1>(blocks, din, dpx, dout, dp0, iters), 1},
           {"AFF2  affine step, 2 proofs/lane", run<AFF2>(blocks, din, dpx, dout, dp0, iters), 2},
           {"AFF4  affine step, 4 proofs/lane", run<AFF4>(blocks, din, dpx, dout, dp0, iters), 4}};
  const double mul_ns = r[1].ms * 1e6 / steps;
  for (auto& x : r) {
    const double ns = x.ms * 1e6 / (steps * x.per);
    printf("%-42s %8.3f ms  %7.3f ns per proof-step  = %5.2f Fq2 products\n", x.name, x.ms, ns, ns / mul_ns);
  }
  return bad != 0;
}
