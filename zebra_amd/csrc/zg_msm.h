// zg_msm.h -- K4: Pippenger multi-scalar multiplication for the batch's sum_{i in k} r_i C_i
// per verifying key k (SURVEY.md 2.3 K4, 8(d) "Pippenger"), and the root Fr scalar sums.
//
// bellman's verify_proof pairs every proof's C with -delta (verification/src/sapling.rs:162,
// 207, sprout.rs:73-77); the batch folds them into ONE pairing per key with the point
// sum_i r_i C_i. r_i = k0 + k1 lambda (zg_groth16.h), so the sum is an MSM over the 2N points
// {C_i, sigma(C_i)} with scalars {k0_i (65 bits), k1_i (64 bits)}, sigma(x, y) = (beta x, y).
//
// Signed-digit buckets: W windows whose widths sum to exactly 66 bits (the 65-bit k0 plus the
// signed-digit carry): the first K windows are c bits wide, the rest c - 1 (K = 66 - (c - 1) W),
// 2^(c-1) bucket slots per (key, window); digit d in [-(2^(cw-1) - 1), 2^(cw-1)] puts +-P into
// bucket |d| - 1. The shape follows the shard (msm_shape): c = 11 x 6 from 32k padded proofs,
// [10 x 3, 9 x 4] from 8k, [9 x 2, 8 x 6] below, so a small shard does not pay for 18,432
// buckets. (Round 3 first used c = 10 x 7 and 9 x 8 windows: their top window held only the 6
// or 3 bits left above bit 60 / 63, so every point of a key landed in 32 or 4 buckets and one
// lane summed hundreds of entries -- 40 ms bucket phases at 4,096 proofs.)
//   k_msm_count    lane per (proof, point): bucket sizes (atomic counters); lane (i, 0) also
//                  converts C_i once to lazy 29-bit digits (x, beta x, y: zg_fqd.h), so the bucket
//                  phase gathers ready operands instead of converting every entry
//   k_msm_scan     one block: exclusive scan of the counters -> bucket offsets
//   k_msm_scatter  lane per (proof, point): 4-byte entries (proof, sigma?, sign) into buckets
//   k_msm_bucket   the bucket phase and the first reduction level in one pass. A wave holds a
//                  segment of 64/P consecutive buckets of one (key, window), P lanes per bucket.
//                  The wave first stages its segment's sorted entries in LDS (one coalesced copy),
//                  then each lane sums its share of a bucket's entries with lazy-digit mixed
//                  Jacobian + affine additions (the entry's digit operands gathered from HBM / L2
//                  one entry ahead), the P parts merge in LDS, and the wave forms the segment's
//                  T = sum_j (j + 1) S_j and U = sum_j S_j by an LDS suffix scan and an LDS tree
//                  (wavefront-level reductions, no atomics on points). A (key, window) group with
//                  no entries (a key absent from the batch) exits at once.
//   k_msm_group    a wave per (key, window): sum_s (T_s + 64/P s U_s) over the group's segments
//                  (suffix scan of U, doublings by 64/P, tree) -> the window sum, already scaled by
//                  2^shift(w) (the windows' doubling chains run in parallel, one per group)
//   k_msm_final    per key: sum_w of the scaled window sums -> the C-sum root node ctree[1]
//   k_fr_root / k_fr_final  the root Fr sums S_k0 = sum r_i, S_kj = sum r_i x_ij per key
// P (parts) follows the batch's situation: a lone batch is latency-bound (P = 4 from 8k proofs,
// 2 below: short lane chains), batches in flight are issue-bound (P = 1 below 32k proofs, 2 from
// 32k: no merge levels, a quarter of the waves, and the wave's entries still fit its LDS stage).
// The random batch scalars are secret and uniform, so bucket sizes are Poisson whatever the
// proofs: ~2N/2^(c-1) entries per bucket and key. Per-proof r_i C_i (GLV) and the full C / Fr
// trees exist only for bisection (k_c_leaves, then the k_tree_cs levels).
#pragma once
#include "zg_batch.h"
#include "zg_fqd.h"
// (the kernels are in zg_msm.hip; this header is shared with zg.hip for the buffer table)

namespace zg {

#define ZG_MSM_WMAX 8                              // windows at c = 9
#define ZG_MSM_NCOUNT_MAX (ZG_NKINDS * 6 * 1024)   // the most buckets over the shapes (c = 11)
#define ZG_MSM_GROUPS_MAX (ZG_NKINDS * ZG_MSM_WMAX)
#define ZG_MSM_SEG_MAX 64                          // segments (waves) per (key, window)
#define ZG_MSM_BT 256                              // threads per k_msm_bucket block (4 waves)
#define ZG_MSM_STAGE 4096                          // entries a bucket wave stages in LDS (16 KB; more: read
                                                   // from HBM in place)
#define ZG_MSM_CD 48                               // u32 per proof of the digit operands: x, beta x, y (16 each)
#define ZG_MSM_SCAN_T 1024                         // lanes of the scan block
#define ZG_FR_CHUNK 64                             // proofs per k_fr_root block (1,024 blocks at 64k;
                                                   // r03: 4,096 gave 16 blocks and a 5.3 ms launch)

// the window shape of a batch of npad (padded) proofs: c bits, w windows, nb = 2^(c-1) buckets
// per (key, window), parts = lanes per bucket in the bucket phase (small shards: more parts, so a
// lane's chain of dependent additions -- its share of the bucket, then the wave's LDS levels -- is
// shorter; the bucket phase is latency-bound there)
#define ZG_MSM_BITS 66
struct MsmShape {
  int c, w, nb, parts;
  ZG_HD int wide() const { return ZG_MSM_BITS - (c - 1) * w; }            // windows of c bits
  ZG_HD int width(int q) const { return q < wide() ? c : c - 1; }         // bits of window q
  ZG_HD int shift(int q) const { return q * (c - 1) + (q < wide() ? q : wide()); }
  ZG_HD int groups() const { return ZG_NKINDS * w; }
  ZG_HD int ncount() const { return groups() * nb; }
  ZG_HD int bs() const { return 64 / parts; }            // buckets per wave (segment)
  ZG_HD int nseg() const { return nb / bs(); }           // segments per group
};
ZG_HD inline MsmShape msm_shape(size_t npad, bool alone = true) {
  MsmShape s = npad >= 32768 ? MsmShape{11, 6, 1024, 4} : npad >= 8192 ? MsmShape{10, 7, 512, 4} : MsmShape{9, 8, 256, 2};
  if (!alone) s.parts = npad >= 32768 ? 2 : 1;
  return s;
}

// window w of the 66-bit scalar lo + 2^64 hi (S.width(w) bits from bit S.shift(w)), as a signed
// digit with carry
ZG_INL int msm_digit(uint64_t lo, uint32_t hi, const MsmShape& S, int w, int* carry) {
  const int sh = S.shift(w), c = S.width(w);  // sh <= 66 - (c - 1) < 64 for every shape
  uint64_t v = lo >> sh;
  if (sh + c > 64) v |= (uint64_t)hi << (64 - sh);
  int t = (int)(v & ((1u << c) - 1)) + *carry;
  if (t > (1 << (c - 1))) {
    *carry = 1;
    return t - (1 << c);
  }
  *carry = 0;
  return t;
}

struct MsmBufs {
  int* count;          // ZG_MSM_NCOUNT_MAX
  int* start;          // ZG_MSM_NCOUNT_MAX + 1
  int* cursor;         // ZG_MSM_NCOUNT_MAX
  uint32_t* entries;   // 2 x cap x ZG_MSM_WMAX: (proof << 2) | (sigma << 1) | negate
  uint32_t* cd;        // cap x ZG_MSM_CD: C_i as lazy digits (x, beta x, y; zg_fqd.h FqD, 16-word rows)
  G1D* seg;            // ZG_MSM_GROUPS_MAX x ZG_MSM_SEG_MAX x 2: (T, U) per segment
  G1D* wsum;           // ZG_MSM_GROUPS_MAX
  Fr* frpart;          // (cap / ZG_FR_CHUNK + 1) x 3 kinds x ZG_MAX_IC
  MsmShape s;          // this batch's shape (set by launch_msm_root)
};

}  // namespace zg
