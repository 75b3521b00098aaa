// Library debug entry: the field products every kernel builds on, evaluated on the device one
// per lane, so a test can compare them with exact integer arithmetic on the host.
//
// Why it exists: the gfx950 lowering of a 64-bit multiply-add whose two 32-bit operands the
// compiler knows to fit 24 bits gave wrong results for the 256-bit products (Fr, BN254 Fq) while
// the same C is exact on the host; the generated code hides those ranges behind zg_opaque
// (zg_fq29_gen.h). tests/test_gpu_field.py runs this entry on random and edge operands so a
// compiler or flag change that brings the miscompile back is caught directly, not only through
// whichever protocol fixture happens to hit a bad operand.
#include <hip/hip_runtime.h>
#include <string.h>

#include "../../include/zg.h"
#include "zg_field.h"

namespace zg {

// field: 0 Fq product (fq29_mul), 1 Fq square (fq29_sqr, b unused), 2 Fq2 product (f2_mul29,
// a lazy < 2p per coefficient), 3 Fr product (fr29_mul), 4 BN254 Fq product (bq29_mul).
__global__ void k_debug_field(int field, int n, const uint32_t* a, const uint32_t* b, uint32_t* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int w = field == 2 ? 24 : field <= 1 ? 12 : 8;
  uint32_t x[24], y[24], r[24];
  for (int k = 0; k < w; k++) {
    x[k] = a[(size_t)i * w + k];
    y[k] = b[(size_t)i * w + k];
  }
  switch (field) {
    case 0: fq29_mul(r, x, y); break;
    case 1: fq29_sqr(r, x); break;
    case 2: f2_mul29(r, r + 12, x, x + 12, y, y + 12); break;
    case 3: fr29_mul(r, x, y); break;
    default: bq29_mul(r, x, y); break;
  }
  for (int k = 0; k < w; k++) out[(size_t)i * w + k] = r[k];
}

}  // namespace zg

extern "C" int zg_debug_field_mul(int device, int field, size_t n, const uint8_t* a, const uint8_t* b,
                                  uint8_t* out) {
  if (field < 0 || field > 4 || (n && (!a || !b || !out)) || n > (1u << 24)) return ZG_E_INVAL;
  if (!n) return ZG_OK;
  const size_t bytes = n * (field == 2 ? 96 : field <= 1 ? 48 : 32);
  if (hipSetDevice(device) != hipSuccess) return ZG_E_HIP;
  uint32_t *da = nullptr, *db = nullptr, *dout = nullptr;
  hipError_t e = hipMalloc(&da, bytes);
  if (e == hipSuccess) e = hipMalloc(&db, bytes);
  if (e == hipSuccess) e = hipMalloc(&dout, bytes);
  if (e == hipSuccess) e = hipMemcpy(da, a, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(db, b, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(zg::k_debug_field, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, 0, field, (int)n, da, db,
                       dout);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost);
  for (void* p : {(void*)da, (void*)db, (void*)dout})
    if (p) hipFree(p);
  return e == hipSuccess ? ZG_OK : ZG_E_HIP;
}
