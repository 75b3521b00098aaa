// zg_decode.hip -- translation unit of the decode kernel (zg_decode.h). Kept apart from
// zg.hip so that the functions it calls are reachable from this kernel only and inherit its
// waves-per-SIMD register budget (a callee shared with other kernels is compiled for the
// loosest budget of its callers).
#include <hip/hip_runtime.h>
#include <stdlib.h>

#define ZG_TU_DECODE 1  // ZG_DEC_INL wrappers inline here (zg_field.h)
#define ZG_SQRT_W 3      // B's inlined square roots: the w = 3 chain's 56-register table fits beside
                         // f2_sqrt's state (w = 4 spilled 40 VGPRs here; k_decode_sqrt keeps w = 4)
#include "../../include/zg.h"
#ifndef ZG_DECODE_WPE
#define ZG_DECODE_WPE 2
#endif
#include "zg_decode.h"

namespace zg {

hipError_t launch_decode_sqrt(unsigned groups, hipStream_t st, const BatchBufs& b);  // zg_decode_sqrt.hip

// G1 square roots, then the point jobs (GLV r_i A_i, subgroup checks, B), then per-proof statuses and Fr leaves
hipError_t launch_batch_decode(unsigned groups, hipStream_t st, const BatchBufs& b, int cglv) {
  const hipError_t e = launch_decode_sqrt(groups, st, b);
  if (e != hipSuccess) return e;
  const unsigned nglv = cglv ? 2 * groups : groups;
  hipLaunchKernelGGL(k_decode_points<-1>, dim3(nglv + 3 * groups), dim3(64), 0, st, b, cglv);
  hipLaunchKernelGGL(k_decode_finish, dim3(groups), dim3(64), 0, st, b);
  return hipGetLastError();
}

}  // namespace zg
