// Microbenchmark (tooling): Fq / Fq2 Montgomery products on gfx950, 32-bit-word FIPS
// (zg_fips.h, v_mad_u64_u32 + v_addc_co_u32 per MAC) against the 29-bit-digit forms
// (zg_fq29.h, one carry-free v_mad_u64_u32 per digit product). Checks that both agree.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../zebra_amd/csrc/zg_prog.h"
#include "../zebra_amd/csrc/zg_fq29.h"

using namespace zg;

template <int MODE>
__global__ void __launch_bounds__(256) k_mul(const Fq* in, Fq* out, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  Fq x = in[i], y = in[i + 1], z = in[i + 2], w = in[i + 3];
  for (int k = 0; k < iters; k++) {
    if (MODE == 0) {
      fq_mul_fips(x.l, x.l, y.l);
    } else if (MODE == 1) {
      fq29_mul(x.l, x.l, y.l);
    } else if (MODE == 2) {
      Fq2 a = f2_mul_lazy({x, z}, {y, w});
      x = a.c0;
      z = a.c1;
    } else if (MODE == 3) {
      Fq2 a;
      f2_mul29(a.c0.l, a.c1.l, x.l, z.l, y.l, w.l);
      x = a.c0;
      z = a.c1;
    }
  }
  for (int q = 0; q < 12; q++) x.l[q] ^= z.l[q] * 3;
  out[i] = x;
}

#define CK(e)                                                         \
  do {                                                                \
    hipError_t r = (e);                                               \
    if (r != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(r), __LINE__); \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

template <int MODE>
static float run(int blocks, const Fq* din, Fq* dout, int iters) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms = 0;
  for (int rep = 0; rep < 2; rep++) {
    CK(hipEventRecord(e0));
    k_mul<MODE><<<blocks, 256>>>(din, dout, iters);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
  }
  return ms;
}

int main() {
  const int maxthreads = 256 * 256 * 8 + 4;
  Fq* h = (Fq*)malloc(sizeof(Fq) * maxthreads);
  srand(1);
  for (int i = 0; i < maxthreads; i++) {
    for (int w = 0; w < 12; w++) h[i].l[w] = (uint32_t)rand() * 2654435761u + w;
    h[i].l[11] &= 0x0fffffff;  // < p
  }
  Fq *din, *d0, *d1;
  CK(hipMalloc(&din, sizeof(Fq) * maxthreads));
  CK(hipMalloc(&d0, sizeof(Fq) * maxthreads));
  CK(hipMalloc(&d1, sizeof(Fq) * maxthreads));
  CK(hipMemcpy(din, h, sizeof(Fq) * maxthreads, hipMemcpyHostToDevice));
  const int n = 64 * 256;
  Fq* a = (Fq*)malloc(sizeof(Fq) * n);
  Fq* b = (Fq*)malloc(sizeof(Fq) * n);
  for (int pair = 0; pair < 2; pair++) {
    if (pair == 0) {
      k_mul<0><<<64, 256>>>(din, d0, 9);
      k_mul<1><<<64, 256>>>(din, d1, 9);
    } else {
      k_mul<2><<<64, 256>>>(din, d0, 9);
      k_mul<3><<<64, 256>>>(din, d1, 9);
    }
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(a, d0, sizeof(Fq) * n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b, d1, sizeof(Fq) * n, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < n; i++)
      for (int w = 0; w < 12; w++) bad += a[i].l[w] != b[i].l[w];
    printf("%s: 32-bit FIPS vs 29-bit digits mismatches: %d\n", pair ? "Fq2" : "Fq", bad);
  }
  const int iters = 256;
  const char* names[4] = {"Fq  FIPS32", "Fq  29-bit", "Fq2 lazy32", "Fq2 29-bit"};
  for (int wps = 1; wps <= 4; wps *= 2) {
    const int blocks = 256 * wps;
    float ms[4] = {run<0>(blocks, din, d0, iters), run<1>(blocks, din, d0, iters), run<2>(blocks, din, d0, iters),
                   run<3>(blocks, din, d0, iters)};
    for (int m = 0; m < 4; m++) {
      const double prods = (double)blocks * 256 * iters * (m >= 2 ? 3 : 1);  // Fq-mul-eq (Fq2 = 3)
      printf("%s waves/SIMD=%d  %.3f ms  %.2f G Fq-mul-eq/s  %.2f T alg-MAC/s\n", names[m], wps, ms[m],
             prods / (ms[m] * 1e-3) / 1e9, prods * 288 / (ms[m] * 1e-3) / 1e12);
    }
  }
  return 0;
}
