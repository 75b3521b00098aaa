// Tooling: device check of the 29-bit-digit Fr (BLS12-381 scalar field) and BN254 Fq products
// against the 32-bit-word FIPS forms on random canonical inputs.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../zebra_amd/csrc/zg_bn254.h"
#include "mb_fr29_variants.h"
using namespace zg;

__global__ void k_out(const uint32_t* in, int n, uint32_t* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t a[8], b[8], r1[8], r2[8];
  for (int k = 0; k < 8; k++) {
    a[k] = in[(size_t)i * 16 + k];
    b[k] = in[(size_t)i * 16 + 8 + k];
  }
  fr_mul_fips(r1, a, b);
  fr29_mul(r2, a, b);
  uint32_t v1[8], v2[8], v3[8];
  fr29_v1(v1, a, b);
  fr29_v2(v2, a, b);
  fr29_v3(v3, a, b);
  for (int k = 0; k < 8; k++) {
    out[(size_t)i * 16 + k] = r1[k];
    out[(size_t)i * 16 + 8 + k] = r2[k];
    out[(size_t)(1024 + i) * 16 + k] = v1[k];
    out[(size_t)(1024 + i) * 16 + 8 + k] = v2[k];
    out[(size_t)(2048 + i) * 16 + k] = v3[k];
  }
}

__global__ void k_cmp(const uint32_t* in, int n, int* bad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t a[8], b[8], r1[8], r2[8], s1[8], s2[8];
  for (int k = 0; k < 8; k++) {
    a[k] = in[(size_t)i * 16 + k];
    b[k] = in[(size_t)i * 16 + 8 + k];
  }
  fr_mul_fips(r1, a, b);
  fr29_mul(r2, a, b);
  bq_mul_fips(s1, a, b);
  bq29_mul(s2, a, b);
  int d = 0, e = 0;
  for (int k = 0; k < 8; k++) {
    d |= r1[k] != r2[k];
    e |= s1[k] != s2[k];
  }
  if (d) atomicAdd(bad, 1);
  if (e) atomicAdd(bad + 1, 1);
  if (d && atomicAdd(bad + 2, 1) == 0) {
    printf("Fr mismatch a=");
    for (int k = 7; k >= 0; k--) printf("%08x", a[k]);
    printf(" b=");
    for (int k = 7; k >= 0; k--) printf("%08x", b[k]);
    printf("\n fips=");
    for (int k = 7; k >= 0; k--) printf("%08x", r1[k]);
    printf("\n 29  =");
    for (int k = 7; k >= 0; k--) printf("%08x", r2[k]);
    printf("\n");
  }
}

int main() {
  const int n = 1 << 20;
  uint32_t* h = (uint32_t*)malloc((size_t)n * 64);
  srand(7);
  for (int i = 0; i < n * 16; i++) h[i] = (uint32_t)rand() * 2654435761u ^ (uint32_t)rand();
  for (int i = 0; i < n; i++) {  // < min(r, p_bn): top word < 0x30000000
    h[(size_t)i * 16 + 7] &= 0x2fffffff;
    h[(size_t)i * 16 + 15] &= 0x2fffffff;
  }
  uint32_t* d;
  int* bad;
  hipMalloc(&d, (size_t)n * 64);
  hipMalloc(&bad, 16);
  hipMemset(bad, 0, 16);
  hipMemcpy(d, h, (size_t)n * 64, hipMemcpyHostToDevice);
  k_cmp<<<n / 256, 256>>>(d, n, bad);
  int hb[4];
  hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost);
  printf("Fr mismatches %d / %d, BN254 Fq mismatches %d / %d\n", hb[0], n, hb[1], n);
  // which side is wrong: device outputs against the host's CIOS and the host's fr29_mul
  uint32_t* o;
  hipMalloc(&o, (size_t)3072 * 64);
  k_out<<<4, 256>>>(d, 1024, o);
  uint32_t* ho = (uint32_t*)malloc(3072 * 64);
  hipMemcpy(ho, o, 3072 * 64, hipMemcpyDeviceToHost);
  int bf = 0, b29 = 0, bh = 0, bv1 = 0, bv2 = 0, bv3 = 0;
  for (int i = 0; i < 1024; i++) {
    Fr a, b;
    for (int k = 0; k < 8; k++) {
      a.l[k] = h[(size_t)i * 16 + k];
      b.l[k] = h[(size_t)i * 16 + 8 + k];
    }
    Fr c = fp_mul_inl<FrM>(a, b), e;
    fr29_mul(e.l, a.l, b.l);
    for (int k = 0; k < 8; k++) {
      bf += ho[(size_t)i * 16 + k] != c.l[k];
      b29 += ho[(size_t)i * 16 + 8 + k] != c.l[k];
      bh += e.l[k] != c.l[k];
      bv1 += ho[(size_t)(1024 + i) * 16 + k] != c.l[k];
      bv2 += ho[(size_t)(1024 + i) * 16 + 8 + k] != c.l[k];
    }
    uint32_t tr[8];
    fr29_v3(tr, a.l, b.l);
    for (int k = 0; k < 8; k++) bv3 += ho[(size_t)(2048 + i) * 16 + k] != tr[k];
  }
  printf("vs host CIOS: device fips %d, device fr29 %d, host fr29 %d word mismatches\n", bf, b29, bh);
  printf("device variants: alignbit->shift %d, canon->C %d, raw t vs host raw t %d\n", bv1, bv2, bv3);
  return hb[0] || hb[1];
}
