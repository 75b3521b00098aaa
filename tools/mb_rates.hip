// Microbenchmark (tooling): issue rate of the integer VALU instructions the Fq products use on
// gfx950 (v_mad_u64_u32, v_mul_lo_u32, v_lshrrev_b64, v_lshl_add_u64, v_add_u32), 8 independent
// chains per lane, 4 waves per SIMD. Prints wave-instructions per clock per SIMD (1.0 = full rate
// for a wave64 on SIMD16 would be 0.25/clk; printed normalised so full rate = 1).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int OP>
__global__ void __launch_bounds__(256) k_rate(uint64_t* out, int iters, uint32_t s) {
  uint64_t a[8];
  uint32_t b[8];
  for (int j = 0; j < 8; j++) {
    a[j] = threadIdx.x * 7 + j + s;
    b[j] = threadIdx.x * 13 + j * 5 + s;
  }
  for (int k = 0; k < iters; k++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (OP == 0) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]) : "vcc");
      if (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(b[j]) : "v"(b[(j + 3) & 7]));
      if (OP == 2) asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(a[j]));
      if (OP == 3) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a[j]) : "v"(a[(j + 1) & 7]));
      if (OP == 4) asm volatile("v_add_u32 %0, %0, %1" : "+v"(b[j]) : "v"(b[(j + 3) & 7]));
      if (OP == 5) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(b[j]) : "v"(b[(j + 3) & 7]));
    }
  }
  uint64_t r = 0;
  for (int j = 0; j < 8; j++) r += a[j] + b[j];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
  uint64_t* d;
  hipMalloc(&d, 8 * 256 * 1024 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* nm[6] = {"v_mad_u64_u32", "v_mul_lo_u32", "v_lshrrev_b64", "v_lshl_add_u64", "v_add_u32", "v_alignbit_b32"};
  const int iters = 4096, blocks = 256 * 4;
  for (int op = 0; op < 6; op++) {
    float ms = 0;
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0);
      switch (op) {
        case 0: k_rate<0><<<blocks, 256>>>(d, iters, 1); break;
        case 1: k_rate<1><<<blocks, 256>>>(d, iters, 1); break;
        case 2: k_rate<2><<<blocks, 256>>>(d, iters, 1); break;
        case 3: k_rate<3><<<blocks, 256>>>(d, iters, 1); break;
        case 4: k_rate<4><<<blocks, 256>>>(d, iters, 1); break;
        case 5: k_rate<5><<<blocks, 256>>>(d, iters, 1); break;
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
    }
    const double winstr = (double)blocks * 4 * iters * 8;  // wave-instructions
    const double per_simd_clk = winstr / 1024 / (ms * 1e-3 * 2.4e9);
    printf("%-16s %.3f ms  %.3f wave-instr/clk/SIMD at 2.4 GHz (x4 = %.2f of full rate)\n", nm[op], ms, per_simd_clk,
           per_simd_clk * 4);
  }
  return 0;
}
