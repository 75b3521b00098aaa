// zg_prog_fchain.hip -- translation unit of staged-program kernels of zg_kernels.h (ZG_TU_PROG_FCHAIN): compiled apart from
// zg.hip so that the build runs the big generated kernels in parallel; zg.hip launches them through
// the wrapper below.
#include <hip/hip_runtime.h>

#include "../../include/zg.h"
#define ZG_TU_PROG
#define ZG_TU_PROG_FCHAIN
#include "zg_kernels.h"

namespace zg {

hipError_t launch_prog_fchain(unsigned blocks, hipStream_t st, const BatchBufs& b, const Fq2* lines,
                              const int* gate) {
  hipLaunchKernelGGL(k_batch_fchain, dim3(blocks), dim3(64 * ZG_FC_NW), 0, st, b, lines, gate);
  return hipGetLastError();
}
// one proof per lane (the leaves): the gated re-run of the fused single-proof launch
hipError_t launch_prog_fchain1(unsigned blocks, hipStream_t st, const BatchBufs& b, const Fq2* lines,
                               const int* gate) {
  hipLaunchKernelGGL(k_batch_fchain1, dim3(blocks), dim3(64 * ZG_FC_NW), 0, st, b, lines, gate);
  return hipGetLastError();
}

}  // namespace zg
