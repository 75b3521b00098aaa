// zg_msm.hip -- translation unit of K4, the Pippenger MSM for sum r_i C_i per key and the root
// Fr sums (zg_msm.h), plus the bisection-only per-proof C leaves.
#include <hip/hip_runtime.h>

#include "../../include/zg.h"
#include "zg_msm.h"

namespace zg {

// the batch root's C sums (ctree node 1) and Fr sums (stree node 1) from the decoded batch;
// gate: null = always, else only if *gate != 0 (the recompute after a deferred B failure)
hipError_t launch_msm_root(hipStream_t st, const BatchBufs& b, const MsmBufs& m, const int* gate) {
  const unsigned pts = (unsigned)((2 * (size_t)b.npad + 63) / 64);
  hipError_t e = hipMemsetAsync(m.count, 0, sizeof(int) * ZG_MSM_NCOUNT, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_msm_count, dim3(pts), dim3(64), 0, st, b, m, gate);
  hipLaunchKernelGGL(k_msm_scan, dim3(1), dim3(ZG_MSM_SCAN_T), 0, st, m, gate);
  hipLaunchKernelGGL(k_msm_scatter, dim3(pts), dim3(64), 0, st, b, m, gate);
  hipLaunchKernelGGL(k_msm_bucket, dim3((ZG_MSM_NCOUNT * ZG_MSM_PARTS + 63) / 64), dim3(64), 0, st, b, m, gate);
  hipLaunchKernelGGL(k_msm_window, dim3(ZG_MSM_GROUPS), dim3(ZG_MSM_WT), 0, st, m, gate);
  hipLaunchKernelGGL(k_msm_final, dim3(1), dim3(64), 0, st, b, m, gate);
  const int nchunks = (b.npad + ZG_FR_CHUNK - 1) / ZG_FR_CHUNK;
  hipLaunchKernelGGL(k_fr_root, dim3(ZG_NKINDS * ZG_MAX_IC, nchunks), dim3(256), 0, st, b, m, gate);
  hipLaunchKernelGGL(k_fr_final, dim3(1), dim3(64), 0, st, b, m, nchunks, gate);
  return hipGetLastError();
}

hipError_t launch_c_leaves(hipStream_t st, const BatchBufs& b) {
  hipLaunchKernelGGL(k_c_leaves, dim3((b.npad + 63) / 64), dim3(64), 0, st, b);
  return hipGetLastError();
}

}  // namespace zg
