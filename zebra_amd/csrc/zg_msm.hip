// zg_msm.hip -- translation unit of K4, the Pippenger MSM for sum r_i C_i per key and the root
// Fr sums (zg_msm.h), plus the bisection-only per-proof C leaves.
#include <hip/hip_runtime.h>

#include "../../include/zg.h"
#include "zg_msm.h"

namespace zg {

// window w (11 bits) of the 66-bit scalar lo + 2^64 hi, as a signed digit with carry
ZG_INL int msm_digit(uint64_t lo, uint32_t hi, int w, int* carry) {
  const int sh = ZG_MSM_C * w;
  uint64_t v = sh < 64 ? lo >> sh : 0;
  if (sh + ZG_MSM_C > 64) v |= (uint64_t)hi << (64 - sh);
  int t = (int)(v & ((1u << ZG_MSM_C) - 1)) + *carry;
  if (t > (1 << (ZG_MSM_C - 1))) {
    *carry = 1;
    return t - (1 << ZG_MSM_C);
  }
  *carry = 0;
  return t;
}

// the scalar of point j of proof i: j = 0 -> k0 = 2a + 1 (65 bits), j = 1 -> k1 = b
ZG_INL void msm_scalar(const BatchBufs& b, int i, int j, uint64_t* lo, uint32_t* hi) {
  uint64_t ra, rb;
  batch_scalar_ab(b.r + (size_t)i * 16, &ra, &rb);
  *lo = j ? rb : (ra << 1) | 1u;
  *hi = j ? 0u : (uint32_t)(ra >> 63);
}

ZG_INL bool msm_live(const BatchBufs& b, int i) { return i < b.n && b.status[i] == ST_PENDING; }

__global__ void __launch_bounds__(64) k_msm_count(BatchBufs b, MsmBufs m, const int* gate) {
  if (gate && *gate == 0) return;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = t >> 1, j = t & 1;
  if (i >= b.npad || !msm_live(b, i)) return;
  const int kind = b.kinds[i];
  uint64_t lo;
  uint32_t hi;
  msm_scalar(b, i, j, &lo, &hi);
  int carry = 0;
  for (int w = 0; w < ZG_MSM_W; w++) {
    const int d = msm_digit(lo, hi, w, &carry);
    if (d) atomicAdd(&m.count[(kind * ZG_MSM_W + w) * ZG_MSM_NB + (d < 0 ? -d : d) - 1], 1);
  }
}

__global__ void __launch_bounds__(ZG_MSM_SCAN_T) k_msm_scan(MsmBufs m, const int* gate) {
  if (gate && *gate == 0) return;
  constexpr int PER = ZG_MSM_NCOUNT / ZG_MSM_SCAN_T;
  static_assert(PER * ZG_MSM_SCAN_T == ZG_MSM_NCOUNT, "scan tiling");
  __shared__ int sh[ZG_MSM_SCAN_T];
  const int t = threadIdx.x;
  int c[PER], s = 0;
#pragma unroll
  for (int q = 0; q < PER; q++) {
    c[q] = m.count[t * PER + q];
    s += c[q];
  }
  sh[t] = s;
  __syncthreads();
  for (int d = 1; d < ZG_MSM_SCAN_T; d <<= 1) {  // inclusive Hillis-Steele
    const int v = t >= d ? sh[t - d] : 0;
    __syncthreads();
    sh[t] += v;
    __syncthreads();
  }
  int off = sh[t] - s;
#pragma unroll
  for (int q = 0; q < PER; q++) {
    m.start[t * PER + q] = off;
    m.cursor[t * PER + q] = off;
    off += c[q];
  }
  if (t == ZG_MSM_SCAN_T - 1) m.start[ZG_MSM_NCOUNT] = off;
}

__global__ void __launch_bounds__(64) k_msm_scatter(BatchBufs b, MsmBufs m, const int* gate) {
  if (gate && *gate == 0) return;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = t >> 1, j = t & 1;
  if (i >= b.npad || !msm_live(b, i)) return;
  const int kind = b.kinds[i];
  uint64_t lo;
  uint32_t hi;
  msm_scalar(b, i, j, &lo, &hi);
  int carry = 0;
  for (int w = 0; w < ZG_MSM_W; w++) {
    const int d = msm_digit(lo, hi, w, &carry);
    if (!d) continue;
    const int pos = atomicAdd(&m.cursor[(kind * ZG_MSM_W + w) * ZG_MSM_NB + (d < 0 ? -d : d) - 1], 1);
    m.entries[pos] = ((uint32_t)i << 2) | ((uint32_t)j << 1) | (d < 0 ? 1u : 0u);
  }
}

__global__ void __launch_bounds__(64) k_msm_bucket(BatchBufs b, MsmBufs m, const int* gate) {
  if (gate && *gate == 0) return;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ZG_MSM_NCOUNT * ZG_MSM_PARTS) return;
  const int bucket = t / ZG_MSM_PARTS, part = t % ZG_MSM_PARTS;
  const int lo = m.start[bucket], len = m.start[bucket + 1] - lo;
  const int beg = lo + len * part / ZG_MSM_PARTS, end = lo + len * (part + 1) / ZG_MSM_PARTS;
  const Fq beta = fq_const(G1_BETA);
  G1J acc = jac_infinity<Fq>();
  for (int e = beg; e < end; e++) {
    const uint32_t ent = m.entries[e];
    // (an entry past what k_msm_scatter wrote can only be stale when k_batch_lines flipped a
    // status between count and scatter -- then bfail > 0 and the gated recompute redoes it;
    // it must still stay inside the buffers)
    if ((ent >> 2) >= (uint32_t)b.npad) continue;
    const G1A c = b.ptAC[(size_t)b.npad + (ent >> 2)];
    const Fq x = (ent & 2u) ? fq_mul(c.x, beta) : c.x;
    const Fq y = (ent & 1u) ? fq_neg(c.y) : c.y;
    acc = jac_add_aff_inl(acc, G1A{x, y, false});
  }
  m.bsum[t] = acc;
}

// sum_{b < 1024} (b + 1) S_b of one (key, window). Lane t holds buckets 2t, 2t + 1:
// a_t = S_2t + 2 S_2t+1, R_t = S_2t + S_2t+1; sum = sum_t a_t + 2 sum_{t >= 1} H_t with the
// suffix sums H_t = sum_{t' >= t} R_t' (an LDS scan), then an LDS tree reduction.
__global__ void __launch_bounds__(ZG_MSM_WT) k_msm_window(MsmBufs m, const int* gate) {
  if (gate && *gate == 0) return;
  static_assert(2 * ZG_MSM_WT == ZG_MSM_NB, "two buckets per lane");
  __shared__ G1J sh[ZG_MSM_WT];
  const int g = blockIdx.x, t = threadIdx.x;
  const G1J* bs = m.bsum + ((size_t)g * ZG_MSM_NB + 2 * t) * ZG_MSM_PARTS;
  G1J s0 = bs[0], s1 = bs[ZG_MSM_PARTS];
  for (int p = 1; p < ZG_MSM_PARTS; p++) {
    s0 = jac_add_full(s0, bs[p]);
    s1 = jac_add_full(s1, bs[ZG_MSM_PARTS + p]);
  }
  const G1J R = jac_add_full(s0, s1);
  const G1J a = jac_add_full(R, s1);
  sh[t] = R;
  __syncthreads();
  for (int d = 1; d < ZG_MSM_WT; d <<= 1) {  // inclusive suffix scan
    G1J v = sh[t];
    if (t + d < ZG_MSM_WT) v = jac_add_full(v, sh[t + d]);
    __syncthreads();
    sh[t] = v;
    __syncthreads();
  }
  G1J v = a;
  if (t >= 1) v = jac_add_full(v, jac_dbl_inl(sh[t]));
  __syncthreads();
  sh[t] = v;
  __syncthreads();
  for (int s = ZG_MSM_WT / 2; s >= 1; s >>= 1) {
    if (t < s) sh[t] = jac_add_full(sh[t], sh[t + s]);
    __syncthreads();
  }
  if (t == 0) m.wsum[g] = sh[0];
}

// per key: sum_w 2^(11 w) W_w -> the root node of the C-sum tree (node 1)
__global__ void __launch_bounds__(64) k_msm_final(BatchBufs b, MsmBufs m, const int* gate) {
  if (gate && *gate == 0) return;
  const int kind = threadIdx.x;
  if (kind >= ZG_NKINDS) return;
  G1J acc = m.wsum[kind * ZG_MSM_W + ZG_MSM_W - 1];
  for (int w = ZG_MSM_W - 2; w >= 0; w--) {
    for (int q = 0; q < ZG_MSM_C; q++) acc = jac_dbl_inl(acc);
    acc = jac_add_full(acc, m.wsum[kind * ZG_MSM_W + w]);
  }
  b.ctree[1 * ZG_NKINDS + kind] = acc;
}

// root Fr sums from the stree leaves (decode_finish: r_i, r_i x_ij in the proof's kind, zero
// elsewhere): block `chunk` sums ZG_FR_CHUNK leaves for all 30 (kind, slot) sums at once --
// lanes t = 30 g + ks read a leaf's 30 consecutive Fr (960 contiguous bytes per 30 lanes), so
// every leaf byte is fetched once
#define ZG_FR_G 8
__global__ void __launch_bounds__(ZG_NKINDS * ZG_MAX_IC * ZG_FR_G) k_fr_root(BatchBufs b, MsmBufs m, const int* gate) {
  if (gate && *gate == 0) return;
  constexpr int KS = ZG_NKINDS * ZG_MAX_IC;
  __shared__ Fr sh[KS * ZG_FR_G];
  const int chunk = blockIdx.x, t = threadIdx.x, ks = t % KS, g = t / KS;
  Fr acc = fp_zero<FrM>();
  const int lo = chunk * ZG_FR_CHUNK, hi = min(lo + ZG_FR_CHUNK, b.npad);
  for (int i = lo + g; i < hi; i += ZG_FR_G) acc = fr_add(acc, b.stree[(size_t)(b.npad + i) * KS + ks]);
  sh[t] = acc;
  __syncthreads();
  for (int s = ZG_FR_G / 2; s >= 1; s >>= 1) {
    if (g < s) sh[t] = fr_add(sh[t], sh[t + s * KS]);
    __syncthreads();
  }
  if (g == 0) m.frpart[(size_t)chunk * KS + ks] = sh[t];
}

__global__ void __launch_bounds__(64) k_fr_final(BatchBufs b, MsmBufs m, int nchunks, const int* gate) {
  if (gate && *gate == 0) return;
  const int ks = threadIdx.x;
  if (ks >= ZG_NKINDS * ZG_MAX_IC) return;
  Fr acc = fp_zero<FrM>();
  for (int c = 0; c < nchunks; c++) acc = fr_add(acc, m.frpart[(size_t)c * ZG_NKINDS * ZG_MAX_IC + ks]);
  b.stree[(size_t)1 * ZG_NKINDS * ZG_MAX_IC + ks] = acc;
}

// bisection only: the per-proof leaves r_i C_i (GLV) of the C-sum trees, infinity for the other
// keys and for proofs that are not pending
__global__ void __launch_bounds__(64, 2) k_c_leaves(BatchBufs b) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= b.npad) return;
  const size_t leaf = (size_t)b.npad + i;
  const bool live = msm_live(b, i);
  const int kind = live ? b.kinds[i] : -1;
  for (int k = 0; k < ZG_NKINDS; k++)
    if (k != kind) b.ctree[leaf * ZG_NKINDS + k] = jac_infinity<Fq>();
  if (live) {
    uint64_t ra, rb;
    batch_scalar_ab(b.r + (size_t)i * 16, &ra, &rb);
    b.ctree[leaf * ZG_NKINDS + kind] = g1_glv_mul(b.ptAC[leaf], ra, rb);
  }
}


// the batch root's C sums (ctree node 1) and Fr sums (stree node 1) from the decoded batch;
// gate: null = always, else only if *gate != 0 (the recompute after a deferred B failure)
hipError_t launch_msm_root(hipStream_t st, const BatchBufs& b, const MsmBufs& m, const int* gate, hipEvent_t bucket0,
                           hipEvent_t bucket1) {
  const unsigned pts = (unsigned)((2 * (size_t)b.npad + 63) / 64);
  hipError_t e = hipMemsetAsync(m.count, 0, sizeof(int) * ZG_MSM_NCOUNT, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_msm_count, dim3(pts), dim3(64), 0, st, b, m, gate);
  hipLaunchKernelGGL(k_msm_scan, dim3(1), dim3(ZG_MSM_SCAN_T), 0, st, m, gate);
  hipLaunchKernelGGL(k_msm_scatter, dim3(pts), dim3(64), 0, st, b, m, gate);
  if (bucket0 && (e = hipEventRecord(bucket0, st)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_msm_bucket, dim3((ZG_MSM_NCOUNT * ZG_MSM_PARTS + 63) / 64), dim3(64), 0, st, b, m, gate);
  if (bucket1 && (e = hipEventRecord(bucket1, st)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_msm_window, dim3(ZG_MSM_GROUPS), dim3(ZG_MSM_WT), 0, st, m, gate);
  hipLaunchKernelGGL(k_msm_final, dim3(1), dim3(64), 0, st, b, m, gate);
  const int nchunks = (b.npad + ZG_FR_CHUNK - 1) / ZG_FR_CHUNK;
  hipLaunchKernelGGL(k_fr_root, dim3(nchunks), dim3(ZG_NKINDS * ZG_MAX_IC * ZG_FR_G), 0, st, b, m, gate);
  hipLaunchKernelGGL(k_fr_final, dim3(1), dim3(64), 0, st, b, m, nchunks, gate);
  return hipGetLastError();
}

hipError_t launch_c_leaves(hipStream_t st, const BatchBufs& b) {
  hipLaunchKernelGGL(k_c_leaves, dim3((b.npad + 63) / 64), dim3(64), 0, st, b);
  return hipGetLastError();
}

}  // namespace zg
