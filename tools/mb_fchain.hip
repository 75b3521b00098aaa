// Microbenchmark (tooling): the f-chain kernel k_batch_fchain4 alone on synthetic line triples,
// with optional per-round s_memtime traces of the first blocks (-DZG_FC_TRACE). Prints the launch
// time, a hash of the quad nodes it writes (variants of the kernel must print the same hash), and
// with the trace, where a quad-step's clocks go (operand forms, read barrier, product, LDS store,
// end-of-round barrier, output forms, line loads).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/mb_fchain.hip -o tools/mb_fchain
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#ifndef ZG_MB_SPLIT
#define ZG_MB_SPLIT true  // the product kernel's default (zg_kernels.h fchain4_body)
#endif
#ifdef ZG_FC_TRACE
#define TRB 4               // traced blocks
#define TRS 80              // events per step
#define TRMAX (68 * TRS)
__device__ unsigned long long g_tr[TRB * 8 * TRMAX];
__device__ int g_trstep[TRB];
#define ZG_TR_PUT(idx)                                                                                     \
  do {                                                                                                     \
    if (blockIdx.x < TRB && (threadIdx.x & 63) == 0)                                                       \
      g_tr[((size_t)blockIdx.x * 8 + (threadIdx.x >> 6)) * TRMAX + (idx)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define ZG_TRACE_S(n, ev)                                     \
  do {                                                        \
    if (blockIdx.x < TRB && (ev) == 0) zg_tr_step = (n);      \
    ZG_TR_PUT((n) * TRS + (ev));                              \
  } while (0)
#define ZG_TRACE_R(r, ev) ZG_TR_PUT(zg_tr_step * TRS + 6 + (r) * 6 + (ev))
static __device__ int zg_tr_step_dummy;
#define zg_tr_step (*zg_tr_step_ptr())
__device__ __forceinline__ int* zg_tr_step_ptr() {
  __shared__ int s;
  return &s;
}
#endif

#include "../include/zg.h"
#define ZG_TU_PROG
#define ZG_TU_PROG_FCHAIN4
#include "../zebra_amd/csrc/zg_kernels.h"

using namespace zg;

#define CK(e)                                                                    \
  do {                                                                           \
    hipError_t r_ = (e);                                                         \
    if (r_ != hipSuccess) {                                                      \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(r_), __FILE__, __LINE__); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__device__ __forceinline__ uint32_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return (uint32_t)x;
}
// random values below p (top word < 2^28 < p's top word), 24 words per Fq2
__global__ void k_fill(uint32_t* w, size_t nwords) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nwords; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t v = mix(i * 0x9e3779b97f4a7c15ull + 12345);
    if (i % 12 == 11) v &= 0x0fffffffu;
    w[i] = v;
  }
}
__global__ void k_init(uint8_t* status, G1A* ptA, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    status[i] = ST_PENDING;
    ptA[i].inf = false;
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 65536;
  const int reps = argc > 2 ? atoi(argv[2]) : 3;
  const int npad = n;
  uint8_t* status;
  G1A* ptA;
  Fq12* ftree;
  Fq2* lines;
  CK(hipMalloc(&status, n));
  CK(hipMalloc(&ptA, sizeof(G1A) * npad));
  CK(hipMalloc(&ftree, sizeof(Fq12) * 2 * npad));
  const size_t nl = (size_t)ZG_NCOEFF * npad * 3;
  CK(hipMalloc(&lines, sizeof(Fq2) * nl));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint32_t*)lines, nl * 24);
  hipLaunchKernelGGL(k_init, dim3((n + 255) / 256), dim3(256), 0, 0, status, ptA, n);
  CK(hipMemset(ftree, 0, sizeof(Fq12) * 2 * npad));
  int* bfail;
  CK(hipMalloc(&bfail, 8));
  CK(hipMemset(bfail, 0, 8));
  BatchBufs b{};
  b.bfail = bfail;
  b.status = status;
  b.ptA = ptA;
  b.ftree = ftree;
  b.n = n;
  b.npad = npad;
  const unsigned blocks = (unsigned)((npad / 4 + 63) / 64);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f, sum = 0;
  for (int r = 0; r <= reps; r++) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_batch_fchain4<ZG_MB_SPLIT>, dim3(blocks), dim3(64 * ZG_FC_NW), 0, 0, b, (const Fq2*)lines);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r > 0) {
      sum += ms;
      if (ms < best) best = ms;
    }
  }
  CK(hipGetLastError());
  std::vector<uint32_t> h((size_t)npad / 4 * 144);
  CK(hipMemcpy(h.data(), ftree + npad / 4, h.size() * 4, hipMemcpyDeviceToHost));
  uint64_t hash = 0xcbf29ce484222325ull;
  for (uint32_t w : h) hash = (hash ^ w) * 0x100000001b3ull;
  int hf[2];
  CK(hipMemcpy(hf, bfail, 8, hipMemcpyDeviceToHost));
  if (hf[1]) printf("bfail[1] = %d\n", hf[1]);
  const double macs = 5192.0 * 288.0 * n;
  printf("fchain4 n=%d blocks=%u: best %.3f ms, mean %.3f ms, %.2f T alg-MAC/s, nodes hash %016llx\n", n, blocks, best,
         sum / reps, macs / (best * 1e-3) / 1e12, (unsigned long long)hash);
#ifdef ZG_FC_TRACE
  std::vector<unsigned long long> tr((size_t)TRB * 8 * TRMAX);
  CK(hipMemcpyFromSymbol(tr.data(), HIP_SYMBOL(g_tr), tr.size() * 8));
  // per-step event offsets relative to the step start (ev 0 of wave 0), averaged over the traced
  // blocks, the waves and the steps with a squaring (q4sq)
  const int nr = PROG_INFO[ZG_PROG_Q4SQ].nrounds;
  double acc[TRS] = {0}, cnt[TRS] = {0}, stepclk = 0;
  int nsteps = 0;
  for (int blk = 0; blk < TRB; blk++)
    for (int s = 1; s < ZG_NCOEFF - 1; s++) {
      const unsigned long long t0 = tr[((size_t)blk * 8 + 0) * TRMAX + s * TRS + 0];
      const unsigned long long tn = tr[((size_t)blk * 8 + 0) * TRMAX + (s + 1) * TRS + 0];
      if (!t0 || !tn) continue;
      // q4sq steps only: skip steps whose round count differs (their last round event is absent)
      if (!tr[((size_t)blk * 8 + 0) * TRMAX + s * TRS + 6 + (nr - 1) * 6 + 4]) continue;
      stepclk += (double)(tn - t0);
      nsteps++;
      for (int w = 0; w < 8; w++)
        for (int e = 0; e < TRS; e++) {
          const unsigned long long t = tr[((size_t)blk * 8 + w) * TRMAX + s * TRS + e];
          if (t) {
            acc[e] += (double)(long long)(t - t0);
            cnt[e]++;
          }
        }
    }
  printf("trace: %d q4sq steps, %.0f clocks per step (s_memtime)\n", nsteps, stepclk / nsteps);
  auto at = [&](int e) { return cnt[e] ? acc[e] / cnt[e] : -1.0; };
  double prev = at(0);
  printf("  round   opforms  rdbarrier   product   ldsput  endbarrier   (mean clocks, all waves)\n");
  double tot[5] = {0};
  for (int r = 0; r < nr; r++) {
    double t[5];
    for (int e = 0; e < 5; e++) t[e] = at(6 + r * 6 + e);
    const double nxt = r + 1 < nr ? at(6 + (r + 1) * 6) : at(1);
    double d[5] = {t[1] - t[0], t[2] - t[1], t[3] - t[2], t[4] - t[3], nxt - t[4]};
    printf("  %5d %9.0f %10.0f %9.0f %8.0f %11.0f\n", r, d[0], d[1], d[2], d[3], d[4]);
    for (int e = 0; e < 5; e++) tot[e] += d[e];
    prev = nxt;
  }
  printf("  total %9.0f %10.0f %9.0f %8.0f %11.0f\n", tot[0], tot[1], tot[2], tot[3], tot[4]);
  printf("  output forms %.0f, barrier %.0f, put + line loads %.0f, barrier %.0f\n", at(2) - at(1), at(3) - at(2),
         at(4) - at(3), at(5) - at(4));
  (void)prev;
  // the product's clocks by wave (idle waves have ev3 == ev2)
  for (int w = 0; w < 8; w++) {
    double pr = 0, c = 0;
    for (int blk = 0; blk < TRB; blk++)
      for (int s = 1; s < ZG_NCOEFF - 1; s++)
        for (int r = 0; r < nr; r++) {
          const size_t base = ((size_t)blk * 8 + w) * TRMAX + s * TRS + 6 + r * 6;
          if (tr[base + 3] && tr[base + 2]) {
            pr += (double)(tr[base + 3] - tr[base + 2]);
            c++;
          }
        }
    printf("  wave %d: mean product+idle %.0f clocks per round\n", w, pr / c);
  }
#endif
  return 0;
}
