// Microbenchmark (tooling): latency of the lane-cooperative Fq12 engine (zg_coop.h) on ONE
// wave -- the final exponentiation's regime. Prints cycles (clock64) per op.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../zebra_amd/csrc/zg_kernels.h"

using namespace zg;

__global__ void __launch_bounds__(64) k_bench(const Fq12* in, Fq12* out, long long* cyc, int iters) {
  __shared__ CoopWS ws;
  coop_init(&ws);
  coop_load(&ws, 0, in[0]);
  coop_load(&ws, 1, in[1]);
  long long t0 = clock64();
  for (int i = 0; i < iters; i++) coop_csqr(&ws, 0, 0);
  long long t1 = clock64();
  for (int i = 0; i < iters; i++) coop_mul(&ws, 0, 0, 1);
  long long t2 = clock64();
  for (int i = 0; i < iters; i++) coop_sqr(&ws, 0, 0);
  long long t3 = clock64();
  for (int i = 0; i < iters; i++) coop_mul014(&ws, 0, 0, 1);
  long long t4 = clock64();
  Fq a = ws.slot[0][threadIdx.x % 12];
  for (int i = 0; i < iters; i++) a = fq_mul(a, a);
  long long t5 = clock64();
  ws.slot[2][threadIdx.x % 12] = a;
  __syncthreads();
  for (int i = 0; i < iters; i++) coop_copy(&ws, 3, 2);
  long long t6 = clock64();
  coop_load(&ws, 4, in[0]);
  coop_csqr(&ws, 5, 4);
  coop_csqr1(&ws, 6, 4);
  int diff = 0;
  for (int k = 0; k < 12; k++) diff |= !fq_eq(ws.slot[5][k], ws.slot[6][k]);
  long long t7 = clock64();
  for (int i = 0; i < iters; i++) coop_csqr1(&ws, 4, 4);
  long long t8 = clock64();
  coop_store(&ws, 0, out[0]);
  coop_store(&ws, 2, out[1]);
  if (threadIdx.x == 0) {
    cyc[0] = t1 - t0;
    cyc[1] = t2 - t1;
    cyc[2] = t3 - t2;
    cyc[3] = t4 - t3;
    cyc[4] = t5 - t4;
    cyc[5] = t6 - t5;
    cyc[6] = t8 - t7;
    cyc[7] = diff;
  }
}

__global__ void __launch_bounds__(64) k_fe(const Fq12* in, Fq12* out, long long* cyc) {
  __shared__ CoopWS ws;
  coop_init(&ws);
  coop_load(&ws, 0, in[0]);
  long long t0 = clock64();
  coop_final_exp(&ws, 0, 0);
  long long t1 = clock64();
  coop_store(&ws, 0, out[0]);
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// the final exponentiation's single-lane pieces: the Fq12 inversion (coop_inv, lane 0) and a Frobenius
__global__ void __launch_bounds__(64) k_inv(const Fq12* in, Fq12* out, long long* cyc) {
  __shared__ CoopWS ws;
  coop_init(&ws);
  coop_load(&ws, 0, in[0]);
  long long t0 = clock64();
  coop_inv(&ws, 1, 0, 5);
  long long t1 = clock64();
  coop_frob(&ws, 2, 1, 2);
  long long t2 = clock64();
  coop_exp_by_x(&ws, 3, 2, BLS_X, 4);
  long long t3 = clock64();
  coop_store(&ws, 3, out[0]);
  if (threadIdx.x == 0) {
    cyc[0] = t1 - t0;
    cyc[1] = t2 - t1;
    cyc[2] = t3 - t2;
  }
}

int main() {
  Fq12 h[2];
  uint32_t* w = (uint32_t*)h;
  for (size_t i = 0; i < sizeof(h) / 4; i++)
    w[i] = (uint32_t)(i * 2654435761u) & ((i % 12) == 11 ? 0x0fffffffu : ~0u);
  Fq12 *din, *dout;
  long long* dc;
  hipMalloc(&din, sizeof(h));
  hipMalloc(&dout, sizeof(h));
  hipMalloc(&dc, 64);
  hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
  const int iters = 64;
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_bench, dim3(1), dim3(64), 0, 0, din, dout, dc, iters);
    hipDeviceSynchronize();
  }
  long long c[8];
  const char* names[] = {"csqr", "mul", "sqr", "mul014", "fq_mul (1 lane chain)", "copy"};
  hipMemcpy(c, dc, 64, hipMemcpyDeviceToHost);
  for (int i = 0; i < 6; i++) printf("%-22s %8.0f cycles/op\n", names[i], (double)c[i] / iters);
  printf("%-22s %8.0f cycles/op  (equals coop_csqr: %s)\n", "csqr1", (double)c[6] / iters, c[7] ? "NO" : "yes");
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k_fe, dim3(1), dim3(64), 0, 0, din, dout, dc);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_fe, dim3(1), dim3(64), 0, 0, din, dout, dc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  hipMemcpy(c, dc, 8, hipMemcpyDeviceToHost);
  Fq12 o[2];
  hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
  unsigned long long hsh = 0xcbf29ce484222325ull;
  for (size_t i = 0; i < sizeof(Fq12) / 4; i++) hsh = (hsh ^ ((const uint32_t*)o)[i]) * 0x100000001b3ull;
  printf("final_exp: %lld cycles, %.3f ms, output hash %016llx\n", c[0], ms, hsh);
  hipLaunchKernelGGL(k_inv, dim3(1), dim3(64), 0, 0, din, dout, dc);
  hipDeviceSynchronize();
  hipMemcpy(c, dc, 24, hipMemcpyDeviceToHost);
  printf("coop_inv %lld cycles, coop_frob %lld cycles, coop_exp_by_x %lld cycles\n", c[0], c[1], c[2]);
  return 0;
}
