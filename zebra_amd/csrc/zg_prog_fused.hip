// zg_prog_fused.hip -- translation unit of staged-program kernels of zg_kernels.h (ZG_TU_PROG_FUSED): compiled apart from
// zg.hip so that the build runs the big generated kernels in parallel; zg.hip launches them through
// the wrapper below.
#include <hip/hip_runtime.h>

#include "../../include/zg.h"
#define ZG_TU_PROG
#define ZG_TU_PROG_FUSED
#include "zg_kernels.h"

namespace zg {

// per: proofs per f-chain lane (1: MSQ / M programs, leaves; 2: pair nodes)
hipError_t launch_prog_lines_fchain(unsigned blocks, hipStream_t st, const BatchBufs& b, Fq2* lines, int* prog,
                                    int* fail, int per) {
  if (per == 1)
    hipLaunchKernelGGL(k_lines_fchain<1>, dim3(blocks), dim3(64 * ZG_FC_NW), 0, st, b, lines, prog, fail);
  else
    hipLaunchKernelGGL(k_lines_fchain<2>, dim3(blocks), dim3(64 * ZG_FC_NW), 0, st, b, lines, prog, fail);
  return hipGetLastError();
}

}  // namespace zg
