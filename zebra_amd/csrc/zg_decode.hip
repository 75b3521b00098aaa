// zg_decode.hip -- translation unit of the decode kernel (zg_decode.h). Kept apart from
// zg.hip so that the functions it calls are reachable from this kernel only and inherit its
// waves-per-SIMD register budget (a callee shared with other kernels is compiled for the
// loosest budget of its callers).
#include <hip/hip_runtime.h>

#include "../../include/zg.h"
#define ZG_DECODE_WPE 2
#include "zg_decode.h"

namespace zg {

// W = 1: one wave per 64 proofs runs the A, B and C chains; W = 3: one wave per chain.
hipError_t launch_batch_decode(int w, unsigned groups, hipStream_t st, const BatchBufs& b) {
  if (w == 1)
    hipLaunchKernelGGL(k_batch_decode<1>, dim3(groups), dim3(64), 0, st, b);
  else
    hipLaunchKernelGGL(k_batch_decode<3>, dim3(groups), dim3(192), 0, st, b);
  return hipGetLastError();
}

}  // namespace zg
