// zg_prog_fused.hip -- translation unit of staged-program kernels of zg_kernels.h (ZG_TU_PROG_FUSED): compiled apart from
// zg.hip so that the build runs the big generated kernels in parallel; zg.hip launches them through
// the wrapper below.
#include <hip/hip_runtime.h>

#include "../../include/zg.h"
#define ZG_TU_PROG
#define ZG_TU_PROG_FUSED
#include "zg_kernels.h"

namespace zg {

hipError_t launch_prog_lines_fchain(unsigned blocks, hipStream_t st, const BatchBufs& b, Fq2* lines, int* prog,
                                    int* fail) {
  hipLaunchKernelGGL(k_lines_fchain, dim3(blocks), dim3(64 * ZG_FC_NW), 0, st, b, lines, prog, fail);
  return hipGetLastError();
}

}  // namespace zg
