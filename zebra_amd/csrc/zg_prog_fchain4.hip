// zg_prog_fchain4.hip -- translation unit of staged-program kernels of zg_kernels.h (ZG_TU_PROG_FCHAIN4): compiled apart from
// zg.hip so that the build runs the big generated kernels in parallel; zg.hip launches them through
// the wrapper below.
#include <hip/hip_runtime.h>

#include "../../include/zg.h"
#define ZG_TU_PROG
#define ZG_TU_PROG_FCHAIN4
#include "zg_kernels.h"

namespace zg {

// split: the four lines' product first, then into f (Q4IK + GMSQ / GM; zg_kernels.h fchain4_body)
hipError_t launch_prog_fchain4(unsigned blocks, hipStream_t st, const BatchBufs& b, const Fq2* lines, int split) {
  if (split)
    hipLaunchKernelGGL(k_batch_fchain4<true>, dim3(blocks), dim3(64 * ZG_FC_NW), 0, st, b, lines);
  else
    hipLaunchKernelGGL(k_batch_fchain4<false>, dim3(blocks), dim3(64 * ZG_FC_NW), 0, st, b, lines);
  return hipGetLastError();
}
// group line products of steps [n0, n1), then the groups' chains over them: m = npad / gsize groups
// (gsize a power of two >= 4); fstate carries each chain's f between parts
// split: Q4IK + GM per four lines (else Q4); affine: the lines are the affine R-chain's (a, b) pairs (AQ4 + GM)
hipError_t launch_prog_lineprod(hipStream_t st, const BatchBufs& b, const Fq2* lines, Fq2* lprod, int gsize, int n0,
                                int n1, int split, int affine) {
  const size_t m = (size_t)b.npad / gsize;
  const dim3 grid((unsigned)((n1 - n0) * ((m + 63) / 64)));
  if (affine)
    hipLaunchKernelGGL((k_line_prod<true, true>), grid, dim3(64 * ZG_FC_NW), 0, st, b, lines, lprod, gsize, n0);
  else if (split)
    hipLaunchKernelGGL((k_line_prod<true, false>), grid, dim3(64 * ZG_FC_NW), 0, st, b, lines, lprod, gsize, n0);
  else
    hipLaunchKernelGGL((k_line_prod<false, false>), grid, dim3(64 * ZG_FC_NW), 0, st, b, lines, lprod, gsize, n0);
  return hipGetLastError();
}
hipError_t launch_prog_fchaing(hipStream_t st, const BatchBufs& b, const Fq2* lprod, Fq2* fstate, int m, int n0,
                               int n1) {
  hipLaunchKernelGGL(k_batch_fchaing, dim3((unsigned)((m + 63) / 64)), dim3(64 * ZG_FC_NW), 0, st, b, lprod, fstate, m,
                     n0, n1);
  return hipGetLastError();
}

}  // namespace zg
