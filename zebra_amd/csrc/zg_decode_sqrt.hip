// zg_decode_sqrt.hip -- translation unit of k_decode_sqrt (zg_decode.h) alone, built with
// ZG_INLINE_ALL: flags, x < p, x^3 + 4 and the Fq square root (fq_pow_pm3_4_p's w = 4 chain with
// its table in registers) inline into the kernel, so it has no call frames and no private segment.
#define ZG_INLINE_ALL 1
#define ZG_TU_DECODE_SQRT 1
#include <hip/hip_runtime.h>

#include "../../include/zg.h"
#ifndef ZG_DECODE_WPE
#define ZG_DECODE_WPE 2
#endif
#ifndef ZG_DECODE_SQRT_WPE
#define ZG_DECODE_SQRT_WPE 2  // w = 4: 242 VGPRs, two waves per SIMD (w = 3 fits three at 151, 2.7% slower)
#endif
#include "zg_decode.h"

namespace zg {

// one wave per (64 proofs, G1 point): blocks alternate A / C
hipError_t launch_decode_sqrt(unsigned groups, hipStream_t st, const BatchBufs& b) {
  hipLaunchKernelGGL(k_decode_sqrt, dim3(2 * groups), dim3(64), 0, st, b);
  return hipGetLastError();
}

}  // namespace zg
