// zg_jubjub.hip -- the Sapling signature kernels (zg_jubjub.h): lane per signature / point /
// transaction. Their own translation unit: they share nothing with the Groth16 batch kernels.
#include <hip/hip_runtime.h>

#include "../../include/zg.h"
#include "zg_jubjub.h"

namespace zg {

// comb tables: lane per (generator, window w, digit d) -> d * 2^(8 w) * G (affine, Montgomery)
__global__ void __launch_bounds__(64) k_jj_comb(uint32_t* table) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ZG_JJ_COMB_POINTS) return;
  const int d = t % ZG_JJ_COMB_D + 1, w = (t / ZG_JJ_COMB_D) % ZG_JJ_COMB_W, gen = t / (ZG_JJ_COMB_D * ZG_JJ_COMB_W);
  const Fr gx = jj_const(gen == 0 ? JUBJUB_G_SPEND_AUTH_X : gen == 1 ? JUBJUB_G_BINDING_X : JUBJUB_G_VALUE_X);
  const Fr gy = jj_const(gen == 0 ? JUBJUB_G_SPEND_AUTH_Y : gen == 1 ? JUBJUB_G_BINDING_Y : JUBJUB_G_VALUE_Y);
  uint32_t k[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  k[w >> 2] = (uint32_t)d << (8 * (w & 3));
  Fr x, y;
  jx_to_aff(jx_mul(jx_from_aff(gx, gy), k, 256), &x, &y);
  uint32_t* e = table + (size_t)t * ZG_JJ_COMB_WORDS;
  for (int l = 0; l < 8; l++) {
    e[l] = x.l[l];
    e[8 + l] = y.l[l];
  }
}

// redjubjub::PublicKey::read(vk) + verify(msg, sig, generator) -> ok (1 valid, 0 invalid)
__global__ void __launch_bounds__(64) k_redjubjub(const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                                                  const uint8_t* gen, int n, const uint32_t* comb, uint8_t* ok) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* s = sig + (size_t)64 * i;
  const uint8_t* mg = msg + (size_t)64 * i;
  // c = H*(Rbar || M): BLAKE2b-512("Zcash_RedJubjubH") of 96 bytes, one block
  uint64_t m[16], h[8];
  for (int w = 0; w < 16; w++) {
    uint64_t v = 0;
    if (w < 12)
      for (int b = 7; b >= 0; b--) v = (v << 8) | (w < 4 ? s[8 * w + b] : mg[8 * (w - 4) + b]);
    m[w] = v;
  }
  blake2b512_block(m, 96, "Zcash_RedJubjubH", h);
  const Fs c = fs_from_512(h);
  Fr vx, vy, rx, ry;
  bool valid = jj_read(vk + (size_t)32 * i, &vx, &vy) && jj_read(s, &rx, &ry);
  Fs sc;
  for (int l = 0; l < 8; l++)
    sc.l[l] = (uint32_t)s[32 + 4 * l] | ((uint32_t)s[33 + 4 * l] << 8) | ((uint32_t)s[34 + 4 * l] << 16) |
              ((uint32_t)s[35 + 4 * l] << 24);
  valid = valid && fp_lt_modulus<FsM>(sc);  // S < order(G)
  if (valid) {
    const int g = gen[i] == ZG_GEN_BINDING ? 1 : 0;
    JExt p = jx_mul(jx_from_aff(vx, vy), c.l, 252);  // r_J < 2^252
    p = jx_add_aff(p, rx, ry);
    p = jx_add(p, jx_neg(jj_fixed_mul(comb, g, sc.l)));
    p = jx_dbl(jx_dbl(jx_dbl(p)));  // the cofactor h_G = 8
    valid = jx_is_zero(p);
  }
  ok[i] = valid ? 1 : 0;
}

// edwards::Point::read + is_small_order: status 0 ok, 1 invalid, 2 small order; xy canonical LE
__global__ void __launch_bounds__(64) k_jj_decode(const uint8_t* pts, int n, uint8_t* status, uint8_t* xy) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fr x, y;
  uint8_t st = 1;
  if (jj_read(pts + (size_t)32 * i, &x, &y)) st = jj_small_order(x, y) ? 2 : 0;
  status[i] = st;
  if (xy) {
    uint8_t* o = xy + (size_t)64 * i;
    const Fr xc = st == 1 ? fp_zero<FrM>() : fr_from_mont(x), yc = st == 1 ? fp_zero<FrM>() : fr_from_mont(y);
    for (int l = 0; l < 8; l++)
      for (int k = 0; k < 4; k++) {
        o[4 * l + k] = (uint8_t)(xc.l[l] >> (8 * k));
        o[32 + 4 * l + k] = (uint8_t)(yc.l[l] >> (8 * k));
      }
  }
}

// binding verification key per transaction (sapling.rs:82-94,216-226,247-269):
// bvk = sum cv(spends) - sum cv(outputs) - [valueBalance] G_v; status 0 ok, 1 a cv does not
// decode, 2 valueBalance == i64::MIN (InvalidBalanceValue)
__global__ void __launch_bounds__(64) k_sapling_bvk(int ntx, const uint32_t* off, const uint32_t* nspends,
                                                    const uint8_t* cvs, const int64_t* vb, const uint32_t* comb,
                                                    uint8_t* bvk, uint8_t* status) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntx) return;
  JExt acc = jx_zero();
  uint8_t st = 0;
  for (uint32_t j = off[t]; j < off[t + 1] && !st; j++) {
    Fr x, y;
    if (!jj_read(cvs + (size_t)32 * j, &x, &y)) {
      st = 1;
      break;
    }
    if (j - off[t] >= nspends[t]) x = fp_neg<FrM>(x);  // outputs enter negated
    acc = jx_add_aff(acc, x, y);
  }
  const int64_t v = vb[t];
  if (!st && v == INT64_MIN) st = 2;
  if (!st) {
    const uint64_t a = v < 0 ? (uint64_t)(-v) : (uint64_t)v;
    uint32_t k[8] = {(uint32_t)a, (uint32_t)(a >> 32), 0, 0, 0, 0, 0, 0};
    JExt vbp = jj_fixed_mul(comb, 2, k);  // [|v|] G_v
    acc = jx_add(acc, v < 0 ? vbp : jx_neg(vbp));
  }
  status[t] = st;
  uint8_t* o = bvk + (size_t)32 * t;
  if (st) {
    for (int b = 0; b < 32; b++) o[b] = 0;
    return;
  }
  Fr x, y;
  jx_to_aff(acc, &x, &y);
  jj_write(x, y, o);
}

// Sapling public-input preparation for a window (zg_prep_batch): lane per description, kinds
// ZG_PREP_KIND_SPEND / _OUTPUT (the JoinSplits are prepared on the host meanwhile and skipped here).
// The same checks in the same order as prep_spend / prep_output (zg_prep.h; accept_spend
// sapling.rs:101-155, accept_output :171-200): the first failing one is the code; every check is
// evaluated (no early exit) so a wave's lanes stay together. Rows: 7 / 5 x 32 B LE Fr, zero padded.
__global__ void __launch_bounds__(64) k_prep_sapling(const uint8_t* kinds, const uint8_t* fields, int n,
                                                     uint8_t* inputs, uint8_t* codes) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int kind = kinds[i];
  if (kind != ZG_PREP_KIND_SPEND && kind != ZG_PREP_KIND_OUTPUT) return;
  const bool spend = kind == ZG_PREP_KIND_SPEND;
  const uint8_t* f = fields + (size_t)ZG_PREP_FIELD_BYTES * i;
  uint8_t* out = inputs + (size_t)288 * i;
  // points: cv (both), then rk (spend, field 3) or epk (output, field 2); the field value: anchor / cmu
  Fr cx, cy, px, py;
  const int c = jj_read(f, &cx, &cy) ? (jj_small_order(cx, cy) ? 2 : 0) : 1;
  const int q = jj_read(f + (spend ? 96 : 64), &px, &py) ? (jj_small_order(px, py) ? 2 : 0) : 1;
  Fr v;
  const bool vin = prep_fr_from_repr(f + 32, &v);
  int code = PREP_OK;
  if (c == 1) code = PREP_VALUE_COMMITMENT_INVALID;
  else if (c == 2) code = PREP_VALUE_COMMITMENT_SMALL_ORDER;
  else if (!vin) code = spend ? PREP_ANCHOR : PREP_NOTE_COMMITMENT;
  else if (q == 1) code = spend ? PREP_RANDOMIZED_KEY_INVALID : PREP_EPHEMERAL_KEY_INVALID;
  else if (q == 2) code = spend ? PREP_RANDOMIZED_KEY_SMALL_ORDER : PREP_EPHEMERAL_KEY_SMALL_ORDER;
  codes[i] = (uint8_t)code;
  for (int b = 0; b < 288; b++) out[b] = 0;
  if (code != PREP_OK) return;
  // spend: rk.x rk.y cv.x cv.y anchor nf0 nf1; output: cv.x cv.y epk.x epk.y cmu
  prep_put(out, spend ? 2 : 0, cx);
  prep_put(out, spend ? 3 : 1, cy);
  prep_put(out, spend ? 0 : 2, px);
  prep_put(out, spend ? 1 : 3, py);
  prep_fr_to_le(v, out + 32 * 4);
  if (spend) prep_multipack_nf(f + 64, out + 32 * 5, out + 32 * 6);
}

hipError_t launch_prep_sapling(hipStream_t st, const uint8_t* kinds, const uint8_t* fields, int n, uint8_t* inputs,
                               uint8_t* codes) {
  hipLaunchKernelGGL(k_prep_sapling, dim3((n + 63) / 64), dim3(64), 0, st, kinds, fields, n, inputs, codes);
  return hipGetLastError();
}

hipError_t launch_jj_comb(hipStream_t st, uint32_t* table) {
  hipLaunchKernelGGL(k_jj_comb, dim3((ZG_JJ_COMB_POINTS + 63) / 64), dim3(64), 0, st, table);
  return hipGetLastError();
}
hipError_t launch_redjubjub(hipStream_t st, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                            const uint8_t* gen, int n, const uint32_t* comb, uint8_t* ok) {
  hipLaunchKernelGGL(k_redjubjub, dim3((n + 63) / 64), dim3(64), 0, st, vk, sig, msg, gen, n, comb, ok);
  return hipGetLastError();
}
hipError_t launch_jj_decode(hipStream_t st, const uint8_t* pts, int n, uint8_t* status, uint8_t* xy) {
  hipLaunchKernelGGL(k_jj_decode, dim3((n + 63) / 64), dim3(64), 0, st, pts, n, status, xy);
  return hipGetLastError();
}
hipError_t launch_sapling_bvk(hipStream_t st, int ntx, const uint32_t* off, const uint32_t* nspends,
                              const uint8_t* cvs, const int64_t* vb, const uint32_t* comb, uint8_t* bvk,
                              uint8_t* status) {
  hipLaunchKernelGGL(k_sapling_bvk, dim3((ntx + 63) / 64), dim3(64), 0, st, ntx, off, nspends, cvs, vb, comb, bvk,
                     status);
  return hipGetLastError();
}

}  // namespace zg
