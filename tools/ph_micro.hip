// Microbenchmark (measurement only, not part of the library): lone-wave latency of the pieces
// of one Pedersen Merkle hash on gfx950 -- Fr products (out-of-line / inlined), a niels
// addition, a full addition, the binary-GCD and Fermat inversions, and the whole 8-lane hash.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/ph_micro.hip -o tools/ph_micro
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../zebra_amd/csrc/zg_merkle.h"

using namespace zg;

template <int OP>
__global__ void __launch_bounds__(64) k_micro(uint32_t* io, int reps, const uint32_t* table) {
  Fr a, b;
  for (int i = 0; i < 8; i++) {
    a.l[i] = io[i] + threadIdx.x;
    b.l[i] = io[8 + i];
  }
  a.l[7] &= 0x0fffffffu;
  b.l[7] &= 0x0fffffffu;
  JExt p = jx_from_aff(a, b);
  for (int r = 0; r < reps; r++) {
    if (OP == 0) a = fr_mul(a, b);
    if (OP == 1) a = ph_mul(a, b);
    if (OP == 2) p = jx_add_niels(p, a, b, a);
    if (OP == 3) p = ph_add(p, p);
    if (OP == 4) a = fr_inv_vt(a);
    if (OP == 5) a = prep_fr_inv(a);
    if (OP == 6) {
      uint32_t o[8];
      ph_merkle<ZG_PH_LANES_WIDE>(a.l, b.l, r & 31, table, threadIdx.x % ZG_PH_LANES_WIDE, o);
      for (int i = 0; i < 8; i++) a.l[i] ^= o[i];
    }
  }
  uint32_t x = 0;
  for (int i = 0; i < 8; i++) x ^= a.l[i] ^ p.X.l[i] ^ p.T.l[i];
  if (x == 0x12345678u) io[threadIdx.x] = x;
}


int main() {
  uint32_t* io;
  uint32_t* table;
  hipMalloc(&io, 4096);
  hipMalloc(&table, ZG_PH_TABLE_BYTES);
  hipMemset(io, 7, 4096);
  hipMemset(table, 3, ZG_PH_TABLE_BYTES);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"fr_mul (call)", "fr_mul (inline)", "niels add", "full add", "inv binary-gcd",
                         "inv fermat", "ph_merkle (group)"};
  const int reps[] = {1000, 1000, 200, 200, 20, 5, 5};
  for (int op = 0; op < 7; op++) {
    for (int pass = 0; pass < 2; pass++) {
      hipEventRecord(e0);
      switch (op) {
        case 0: hipLaunchKernelGGL(k_micro<0>, 1, 64, 0, 0, io, reps[op], table); break;
        case 1: hipLaunchKernelGGL(k_micro<1>, 1, 64, 0, 0, io, reps[op], table); break;
        case 2: hipLaunchKernelGGL(k_micro<2>, 1, 64, 0, 0, io, reps[op], table); break;
        case 3: hipLaunchKernelGGL(k_micro<3>, 1, 64, 0, 0, io, reps[op], table); break;
        case 4: hipLaunchKernelGGL(k_micro<4>, 1, 64, 0, 0, io, reps[op], table); break;
        case 5: hipLaunchKernelGGL(k_micro<5>, 1, 64, 0, 0, io, reps[op], table); break;
        case 6: hipLaunchKernelGGL(k_micro<6>, 1, 64, 0, 0, io, reps[op], table); break;
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (pass) printf("%-20s %9.2f us per op (lone wave)\n", names[op], 1e3 * ms / reps[op]);
    }
  }
  return 0;
}
