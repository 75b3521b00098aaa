// zg_msm.h -- K4: Pippenger multi-scalar multiplication for the batch's sum_{i in k} r_i C_i
// per verifying key k (SURVEY.md 2.3 K4, 8(d) "Pippenger"), and the root Fr scalar sums.
//
// bellman's verify_proof pairs every proof's C with -delta (verification/src/sapling.rs:162,
// 207, sprout.rs:73-77); the batch folds them into ONE pairing per key with the point
// sum_i r_i C_i. r_i = k0 + k1 lambda (zg_groth16.h), so the sum is an MSM over the 2N points
// {C_i, sigma(C_i)} with scalars {k0_i (65 bits), k1_i (64 bits)}, sigma(x, y) = (beta x, y).
//
// Signed-digit buckets, c = 11 bits per window, 6 windows (66 bits), 1024 buckets per
// (key, window): digit d in [-1023, 1024] puts +-P into bucket |d| - 1.
//   k_msm_count    lane per (proof, point): bucket sizes (atomic counters)
//   k_msm_scan     one block: exclusive scan of the 18,432 counters -> bucket offsets
//   k_msm_scatter  lane per (proof, point): 4-byte entries (proof, sigma?, sign) into buckets
//   k_msm_bucket   ZG_MSM_PARTS lanes per bucket: each sums a contiguous quarter of its
//                  entries with mixed Jacobian + affine additions (the bucket phase: entries
//                  and affine C_i streamed from HBM / L2, partial sums written once)
//   k_msm_window   a 512-lane block per (key, window): sum_b (b + 1) S_b as local running
//                  sums + an LDS suffix scan + an LDS tree reduction (wavefront/LDS-level, no
//                  atomics on points)
//   k_msm_final    per key: sum_w 2^(11 w) W_w (Horner) -> the C-sum root node ctree[1]
//   k_fr_root / k_fr_final  the root Fr sums S_k0 = sum r_i, S_kj = sum r_i x_ij per key
// The random batch scalars are secret and uniform, so bucket sizes are Poisson whatever the
// proofs: ~2N/1024 entries per bucket and key. Per-proof r_i C_i (GLV) and the full C / Fr
// trees exist only for bisection (k_c_leaves, then the k_tree_cs levels).
#pragma once
#include "zg_batch.h"
// (the kernels are in zg_msm.hip; this header is shared with zg.hip for the buffer table)

namespace zg {

#define ZG_MSM_C 11
#define ZG_MSM_W 6
#define ZG_MSM_NB 1024
#define ZG_MSM_PARTS 4
#define ZG_MSM_GROUPS (ZG_NKINDS * ZG_MSM_W)
#define ZG_MSM_NCOUNT (ZG_MSM_GROUPS * ZG_MSM_NB)
#define ZG_MSM_WT 512       // lanes of the window-reduction block (2 buckets each)
#define ZG_MSM_SCAN_T 1024  // lanes of the scan block (18 counters each)
#define ZG_FR_CHUNK 4096    // proofs per k_fr_root block

struct MsmBufs {
  int* count;          // ZG_MSM_NCOUNT
  int* start;          // ZG_MSM_NCOUNT + 1
  int* cursor;         // ZG_MSM_NCOUNT
  uint32_t* entries;   // 2 x cap x ZG_MSM_W: (proof << 2) | (sigma << 1) | negate
  G1J* bsum;           // ZG_MSM_NCOUNT x ZG_MSM_PARTS
  G1J* wsum;           // ZG_MSM_GROUPS
  Fr* frpart;          // (cap / ZG_FR_CHUNK + 1) x 3 kinds x ZG_MAX_IC
};

}  // namespace zg
