// Microbenchmark (tooling): Fq multiplication throughput/latency on gfx950.
//   C  : zg_field.h fp_mul_inl (no-carry CIOS in C; the compiler's lowering)
//   ASM: zg_fq_asm.h fq_mul_fips (v_mad_u64_u32 carry-out product scanning)
// Prints Fq-mul/s and cycles per Fq-mul per SIMD for several occupancies, and checks
// that both agree on random inputs.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../zebra_amd/csrc/zg_field.h"
#include "../zebra_amd/csrc/zg_fq_asm.h"

using namespace zg;

template <int MODE>
__global__ void __launch_bounds__(256) k_mul(const Fq* in, Fq* out, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  Fq x = in[i], y = in[i + 1], z = in[i + 2];
  for (int k = 0; k < iters; k++) {
    if (MODE == 0)
      x = fp_mul_inl<FqM>(x, y);
    else if (MODE == 1)
      fq_mul_fips(x.l, x.l, y.l);
    else {  // two independent chains per lane (ILP 2), each counts as one mul per iteration
      fq_mul_fips(x.l, x.l, y.l);
      fq_mul_fips(z.l, z.l, y.l);
    }
  }
  if (MODE == 2)
    for (int w = 0; w < 12; w++) x.l[w] ^= z.l[w];
  out[i] = x;
}

#define CK(e)                                                     \
  do {                                                            \
    hipError_t r = (e);                                           \
    if (r != hipSuccess) {                                        \
      printf("HIP error %s at %d\n", hipGetErrorString(r), __LINE__); \
      exit(1);                                                    \
    }                                                             \
  } while (0)

int main() {
  const int maxthreads = 256 * 256 * 8 + 2;
  Fq* h = (Fq*)malloc(sizeof(Fq) * maxthreads);
  srand(1);
  for (int i = 0; i < maxthreads; i++) {
    for (int w = 0; w < 12; w++) h[i].l[w] = (uint32_t)rand() * 2654435761u + w;
    h[i].l[11] &= 0x0fffffff;  // < p
  }
  Fq *din, *dout, *dout2;
  CK(hipMalloc(&din, sizeof(Fq) * maxthreads));
  CK(hipMalloc(&dout, sizeof(Fq) * maxthreads));
  CK(hipMalloc(&dout2, sizeof(Fq) * maxthreads));
  CK(hipMemcpy(din, h, sizeof(Fq) * maxthreads, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // correctness
  k_mul<0><<<64, 256>>>(din, dout, 7);
  k_mul<1><<<64, 256>>>(din, dout2, 7);
  CK(hipDeviceSynchronize());
  Fq* a = (Fq*)malloc(sizeof(Fq) * 64 * 256);
  Fq* b = (Fq*)malloc(sizeof(Fq) * 64 * 256);
  CK(hipMemcpy(a, dout, sizeof(Fq) * 64 * 256, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b, dout2, sizeof(Fq) * 64 * 256, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < 64 * 256; i++)
    for (int w = 0; w < 12; w++) bad += a[i].l[w] != b[i].l[w];
  printf("asm vs C mismatches: %d\n", bad);
  const int iters = 512;
  int waves_per_simd[] = {1, 2, 4, 8};
  for (int mode = 0; mode < 3; mode++) {
    for (int wi = 0; wi < 4; wi++) {
      int wps = waves_per_simd[wi];
      int blocks = 256 * wps;  // 256 threads = 4 waves = 1 per SIMD per block
      for (int rep = 0; rep < 2; rep++) {
        CK(hipEventRecord(e0));
        if (mode == 0)
          k_mul<0><<<blocks, 256>>>(din, dout, iters);
        else if (mode == 1)
          k_mul<1><<<blocks, 256>>>(din, dout, iters);
        else
          k_mul<2><<<blocks, 256>>>(din, dout, iters);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        double muls = (double)blocks * 256 * iters * (mode == 2 ? 2 : 1);
        double rate = muls / (ms * 1e-3);
        // cycles per Fq-mul per SIMD assuming 2.4 GHz: SIMDs = 1024, each wave = 64 muls in parallel
        double cyc = (ms * 1e-3) * 2.4e9 / ((double)iters * wps);
        if (rep == 1)
          printf("%s waves/SIMD=%d  %.3f ms  %.2f G Fq-mul/s  ~%.0f cycles per wave-Fq-mul (latency view)\n",
                 mode == 2 ? "ASM-ILP2" : mode ? "ASM" : "C  ", wps, ms, rate / 1e9, cyc);
      }
    }
  }
  return 0;
}
