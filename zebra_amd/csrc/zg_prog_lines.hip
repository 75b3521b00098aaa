// zg_prog_lines.hip -- translation unit of staged-program kernels of zg_kernels.h (ZG_TU_PROG_LINES): compiled apart from
// zg.hip so that the build runs the big generated kernels in parallel; zg.hip launches them through
// the wrapper below.
#include <hip/hip_runtime.h>

#include "../../include/zg.h"
#define ZG_TU_PROG
#define ZG_TU_PROG_LINES
#include "zg_kernels.h"

namespace zg {

hipError_t launch_prog_lines(unsigned groups, hipStream_t st, const BatchBufs& b, Fq2* lines) {
  hipLaunchKernelGGL(k_batch_lines, dim3(groups), dim3(64 * ZG_LINES_NW), 0, st, b, lines);
  return hipGetLastError();
}
hipError_t launch_prog_leaf_fchain(unsigned blocks, hipStream_t st, const BatchBufs& b, const Fq2* lines,
                                   const int* nodes, int m) {
  hipLaunchKernelGGL(k_leaf_fchain, dim3(blocks), dim3(64 * ZG_FC_NW), 0, st, b, lines, nodes, m);
  return hipGetLastError();
}

}  // namespace zg
