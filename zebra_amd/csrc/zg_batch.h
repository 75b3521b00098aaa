// zg_batch.h -- declarations shared by the batch kernels (zg_kernels.h) and the decode kernel
// (zg_decode.h, its own translation unit): the batch buffer table and per-kind constants.
#pragma once
#include "zg_coop.h"
#include "zg_groth16.h"
#include "zg_prog.h"

namespace zg {

#define ZG_MSM_SLOTS (ZG_MAX_IC + 1)  // ic terms + the alpha term
#define ZG_NPAIRS 3                   // per kind: (acc,-gamma) (C,-delta) (-S alpha, beta)
// VK-side pairs per checked node: 9 = 3 per key; 5 when the loaded keys share alpha, beta and
// gamma (the three Zcash keys do): FE is bilinear, so the keys' gamma pairs merge
// into ONE pair (sum_k acc_k, -gamma) and their beta pairs into ONE (-(sum_k S_k0) alpha, beta),
// next to one (C_k, -delta_k) pair per key. Pair slot p of a node: merged 0 = gamma, 1..3 =
// delta of key p - 1, 4 = beta; otherwise 3 * key + {0 gamma, 1 delta, 2 beta}.
#define ZG_NODE_PAIRS (ZG_NKINDS * ZG_NPAIRS)
#define ZG_NODE_PAIRS_MERGED (ZG_NKINDS + 2)

__device__ __constant__ const int KIND_NINPUTS[ZG_NKINDS] = {7, 5, 9};

struct BatchBufs {
  const DevVK* vks;
  const uint8_t* proofs;   // n x 192
  const uint8_t* kinds;    // n
  const uint8_t* inputs;   // n x 288
  const uint8_t* ninputs;  // n or null
  const uint8_t* r;        // n x 16
  uint8_t* status;         // n
  G1A* ptA;                // npad: r_i A_i (affine)
  G2A* ptB;                // npad: B_i
  G1A* ptAC;               // 2 npad: A_i then C_i as decompressed (k_decode_sqrt -> k_decode_points)
  Fq12* ftree;             // 2 npad
  G1J* ctree;              // 2 npad x 3 kinds
  Fr* stree;               // 2 npad x 3 kinds x ZG_MAX_IC (Montgomery)
  int* bfail;              // count of B_i failing the (deferred) G2 subgroup check
  uint8_t* okbits;         // npad x {A, C, B}: the point decoded (k_decode_points -> k_decode_finish)
  int n, npad;
  int merged;              // the loaded keys share alpha, beta, gamma: 5 VK-side pairs per node
};

}  // namespace zg
