// zg_msm.hip -- translation unit of K4, the Pippenger MSM for sum r_i C_i per key and the root
// Fr sums (zg_msm.h), plus the bisection-only per-proof C leaves.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "../../include/zg.h"
#include "zg_msm.h"

namespace zg {

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
  const MsmShape S = m.s;
  const int kind = b.kinds[i];
  uint64_t lo;
  uint32_t hi;
  msm_scalar(b, i, j, &lo, &hi);
  int carry = 0;
  for (int w = 0; w < S.w; w++) {
    const int d = msm_digit(lo, hi, S, w, &carry);
    if (d) atomicAdd(&m.count[(kind * S.w + w) * S.nb + (d < 0 ? -d : d) - 1], 1);
  }
}

__global__ void __launch_bounds__(ZG_MSM_SCAN_T) k_msm_scan(MsmBufs m, const int* gate) {
  if (gate && *gate == 0) return;
  constexpr int PER = ZG_MSM_NCOUNT_MAX / ZG_MSM_SCAN_T;
  static_assert(PER * ZG_MSM_SCAN_T == ZG_MSM_NCOUNT_MAX, "scan tiling");
  __shared__ int sh[ZG_MSM_SCAN_T];
  const int t = threadIdx.x, nc = m.s.ncount();
  int c[PER], s = 0;
#pragma unroll
  for (int q = 0; q < PER; q++) {
    c[q] = t * PER + q < nc ? m.count[t * PER + q] : 0;
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
    if (t * PER + q < nc) {
      m.start[t * PER + q] = off;
      m.cursor[t * PER + q] = off;
    }
    off += c[q];
  }
  if (t == ZG_MSM_SCAN_T - 1) m.start[nc] = off;
}

__global__ void __launch_bounds__(64) k_msm_scatter(BatchBufs b, MsmBufs m, const int* gate) {
  if (gate && *gate == 0) return;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = t >> 1, j = t & 1;
  if (i >= b.npad || !msm_live(b, i)) return;
  const MsmShape S = m.s;
  const int kind = b.kinds[i];
  uint64_t lo;
  uint32_t hi;
  msm_scalar(b, i, j, &lo, &hi);
  int carry = 0;
  for (int w = 0; w < S.w; w++) {
    const int d = msm_digit(lo, hi, S, w, &carry);
    if (!d) continue;
    const int pos = atomicAdd(&m.cursor[(kind * S.w + w) * S.nb + (d < 0 ? -d : d) - 1], 1);
    m.entries[pos] = ((uint32_t)i << 2) | ((uint32_t)j << 1) | (d < 0 ? 1u : 0u);
  }
}

// The bucket phase with the first reduction level (see zg_msm.h). Wave gw of the grid holds
// buckets [gw BS, (gw + 1) BS) (BS = 64 / P, inside one (key, window) group), lane = (bucket j,
// part); the segment's outputs are T = sum_j (j + 1) S_j and U = sum_j S_j.
__global__ void __launch_bounds__(ZG_MSM_BT) k_msm_bucket(BatchBufs b, MsmBufs m, const int* gate) {
  if (gate && *gate == 0) return;
  __shared__ G1J sh[ZG_MSM_BT];
  const MsmShape S = m.s;
  const int lane = threadIdx.x & 63, w0 = threadIdx.x & ~63;
  const int gw = blockIdx.x * (ZG_MSM_BT / 64) + (threadIdx.x >> 6);
  const int P = S.parts, BS = S.bs();
  const bool live = gw * BS < S.ncount();  // whole waves are live or not
  const int j = lane / P, part = lane % P;
  G1J acc = jac_infinity<Fq>();
  if (live) {
    const int bucket = gw * BS + j;
    const int lo = m.start[bucket], len = m.start[bucket + 1] - lo;
    const int beg = lo + len * part / P, end = lo + len * (part + 1) / P;
    const Fq beta = fq_const(G1_BETA);
    // (an entry past what k_msm_scatter wrote can only be stale when k_batch_lines flipped a
    // status between count and scatter -- then bfail > 0 and the gated recompute redoes it; it
    // must still stay inside the buffers). The next entry's point is gathered while the current
    // one is added (software pipelining: its L2 / HBM latency hides behind the addition).
    auto gather = [&](int e, uint32_t* ent, G1A* c) {
      *ent = m.entries[e];
      const uint32_t pi = *ent >> 2;
      *c = b.ptAC[(size_t)b.npad + (pi < (uint32_t)b.npad ? pi : 0)];
    };
    uint32_t ent_n = 0;
    G1A c_n;
    if (beg < end) gather(beg, &ent_n, &c_n);
    for (int e = beg; e < end; e++) {
      const uint32_t ent = ent_n;
      const G1A c = c_n;
      if (e + 1 < end) gather(e + 1, &ent_n, &c_n);
      if ((ent >> 2) >= (uint32_t)b.npad) continue;
      const Fq x = (ent & 2u) ? fq_mul(c.x, beta) : c.x;
      const Fq y = (ent & 1u) ? fq_neg(c.y) : c.y;
      acc = jac_add_aff_inl(acc, G1A{x, y, false});
    }
  }
  // merge the P parts of each bucket: S_j lands in lane j P
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int d = 1; d < P; d <<= 1) {
    G1J v = sh[threadIdx.x];
    if (part % (2 * d) == 0) v = jac_add_full(v, sh[threadIdx.x + d]);
    __syncthreads();
    sh[threadIdx.x] = v;
    __syncthreads();
  }
  // compact: lane j < BS holds S_j
  G1J v = lane < BS ? sh[w0 + lane * P] : jac_infinity<Fq>();
  __syncthreads();
  sh[threadIdx.x] = v;
  __syncthreads();
  // suffix sums H_j = sum_{j' >= j} S_j' (inclusive Hillis-Steele, BS lanes)
  for (int d = 1; d < BS; d <<= 1) {
    G1J u = sh[threadIdx.x];
    if (lane + d < BS) u = jac_add_full(u, sh[threadIdx.x + d]);
    __syncthreads();
    sh[threadIdx.x] = u;
    __syncthreads();
  }
  const G1J U = sh[w0];  // H_0
  // T = sum_j H_j: tree over the BS suffix sums
  for (int d = BS / 2; d >= 1; d >>= 1) {
    G1J u = sh[threadIdx.x];
    if (lane < d) u = jac_add_full(u, sh[threadIdx.x + d]);
    __syncthreads();
    sh[threadIdx.x] = u;
    __syncthreads();
  }
  if (live && lane == 0) {
    const int g = gw / S.nseg(), s = gw % S.nseg();
    m.seg[((size_t)g * ZG_MSM_SEG_MAX + s) * 2 + 0] = sh[w0];
    m.seg[((size_t)g * ZG_MSM_SEG_MAX + s) * 2 + 1] = U;
  }
}

// one wave per (key, window) group: sum_b (b + 1) S_b = sum_s (T_s + BS s U_s), with
// sum_s s U_s = sum_{s >= 1} H_s, H_s = sum_{s' >= s} U_s' (lane s = segment s)
__global__ void __launch_bounds__(64) k_msm_group(MsmBufs m, const int* gate) {
  if (gate && *gate == 0) return;
  __shared__ G1J sh[64];
  const MsmShape S = m.s;
  const int g = blockIdx.x, s = threadIdx.x, ns = S.nseg();
  const G1J* sg = m.seg + (size_t)g * ZG_MSM_SEG_MAX * 2;
  const G1J T = s < ns ? sg[2 * s] : jac_infinity<Fq>();
  sh[s] = s < ns ? sg[2 * s + 1] : jac_infinity<Fq>();
  __syncthreads();
  for (int d = 1; d < ns; d <<= 1) {
    G1J u = sh[s];
    if (s + d < ns) u = jac_add_full(u, sh[s + d]);
    __syncthreads();
    sh[s] = u;
    __syncthreads();
  }
  G1J x = T;
  if (s >= 1 && s < ns) {
    G1J h = sh[s];
    for (int q = S.bs(); q > 1; q >>= 1) h = jac_dbl_inl(h);  // BS = 2^k
    x = jac_add_full(x, h);
  }
  // (the doubling chains run in lazy digits, zg_fqd.h: no split / repack / canonicalisation per
  // product -- the window's 2^shift(w) chain is this kernel's critical path)
  __syncthreads();
  sh[s] = x;
  __syncthreads();
  int top = 1;
  while (top < ns) top <<= 1;
  for (int d = top / 2; d >= 1; d >>= 1) {  // the lanes past ns hold infinity
    G1J u = sh[s];
    if (s < d) u = jac_add_full(u, sh[s + d]);
    __syncthreads();
    sh[s] = u;
    __syncthreads();
  }
  if (s == 0) {  // 2^shift(w) W_w: this window's part of sum_w 2^shift(w) W_w
    const G1J x = sh[0];
    const int w = g % S.w;
    G1D q = {fqd_from(x.x), fqd_from(x.y), fqd_from(x.z)};  // < 2p each: g1d_dbl's invariant holds
    for (int k = 0; k < S.shift(w); k++) q = g1d_dbl(q);   // infinity (Z = 0) stays infinity
    m.wsum[g] = g1d_to_jac(q);
  }
}

// per key: sum_w of the scaled window sums (k_msm_group) -> the root node of the C-sum tree (node 1)
__global__ void __launch_bounds__(64) k_msm_final(BatchBufs b, MsmBufs m, const int* gate) {
  if (gate && *gate == 0) return;
  const int kind = threadIdx.x;
  if (kind >= ZG_NKINDS) return;
  const MsmShape S = m.s;
  G1J acc = m.wsum[kind * S.w];
  for (int w = 1; w < S.w; w++) acc = jac_add_full(acc, m.wsum[kind * S.w + w]);
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
#pragma unroll 4
  for (int i = lo + g; i < hi; i += ZG_FR_G) acc = fr_add(acc, b.stree[(size_t)(b.npad + i) * KS + ks]);
  sh[t] = acc;
  __syncthreads();
  for (int s = ZG_FR_G / 2; s >= 1; s >>= 1) {
    if (g < s) sh[t] = fr_add(sh[t], sh[t + s * KS]);
    __syncthreads();
  }
  if (g == 0) m.frpart[(size_t)chunk * KS + ks] = sh[t];
}

// the chunk partials -> stree node 1: lanes t = 30 g + ks stride over the chunks, then an LDS tree
__global__ void __launch_bounds__(ZG_NKINDS * ZG_MAX_IC * ZG_FR_G) k_fr_final(BatchBufs b, MsmBufs m, int nchunks,
                                                                            const int* gate) {
  if (gate && *gate == 0) return;
  constexpr int KS = ZG_NKINDS * ZG_MAX_IC;
  __shared__ Fr sh[KS * ZG_FR_G];
  const int t = threadIdx.x, ks = t % KS, g = t / KS;
  Fr acc = fp_zero<FrM>();
  for (int c = g; c < nchunks; c += ZG_FR_G) acc = fr_add(acc, m.frpart[(size_t)c * KS + ks]);
  sh[t] = acc;
  __syncthreads();
  for (int s = ZG_FR_G / 2; s >= 1; s >>= 1) {
    if (g < s) sh[t] = fr_add(sh[t], sh[t + s * KS]);
    __syncthreads();
  }
  if (g == 0) b.stree[(size_t)1 * KS + ks] = sh[t];
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
    b.ctree[leaf * ZG_NKINDS + kind] = g1_glv_mul_d(b.ptAC[leaf], ra, rb);
  }
}


// the batch root's C sums (ctree node 1) and Fr sums (stree node 1) from the decoded batch;
// gate: null = always, else only if *gate != 0 (the recompute after a deferred B failure)
// k4 = 0 (small shards): only the root Fr sums; the C sums are the tree levels of the GLV leaves
hipError_t launch_msm_root(hipStream_t st, const BatchBufs& b, MsmBufs m, const int* gate, hipEvent_t bucket0,
                           hipEvent_t bucket1, int k4) {
  m.s = msm_shape(b.npad);
  // ZG_MSM_PARTS (tooling): lanes per bucket in the bucket phase, 1 / 2 / 4 / 8, kept only while a
  // (key, window) group still fits one k_msm_group wave (nb / (64 / parts) <= ZG_MSM_SEG_MAX)
  static const int parts_env = getenv("ZG_MSM_PARTS") ? atoi(getenv("ZG_MSM_PARTS")) : 0;
  if ((parts_env == 1 || parts_env == 2 || parts_env == 4 || parts_env == 8) &&
      m.s.nb / (64 / parts_env) <= ZG_MSM_SEG_MAX)
    m.s.parts = parts_env;
  if (!k4) {
    hipError_t e;  // the bucket-phase events still bracket something (an empty phase): callers time them
    if (bucket0 && (e = hipEventRecord(bucket0, st)) != hipSuccess) return e;
    if (bucket1 && (e = hipEventRecord(bucket1, st)) != hipSuccess) return e;
    const int nchunks = (b.npad + ZG_FR_CHUNK - 1) / ZG_FR_CHUNK;
    hipLaunchKernelGGL(k_fr_root, dim3(nchunks), dim3(ZG_NKINDS * ZG_MAX_IC * ZG_FR_G), 0, st, b, m, gate);
    hipLaunchKernelGGL(k_fr_final, dim3(1), dim3(ZG_NKINDS * ZG_MAX_IC * ZG_FR_G), 0, st, b, m, nchunks, gate);
    return hipGetLastError();
  }
  const unsigned pts = (unsigned)((2 * (size_t)b.npad + 63) / 64);
  hipError_t e = hipMemsetAsync(m.count, 0, sizeof(int) * m.s.ncount(), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_msm_count, dim3(pts), dim3(64), 0, st, b, m, gate);
  hipLaunchKernelGGL(k_msm_scan, dim3(1), dim3(ZG_MSM_SCAN_T), 0, st, m, gate);
  hipLaunchKernelGGL(k_msm_scatter, dim3(pts), dim3(64), 0, st, b, m, gate);
  if (bucket0 && (e = hipEventRecord(bucket0, st)) != hipSuccess) return e;
  const int waves = m.s.ncount() / m.s.bs();
  hipLaunchKernelGGL(k_msm_bucket, dim3((waves + ZG_MSM_BT / 64 - 1) / (ZG_MSM_BT / 64)), dim3(ZG_MSM_BT), 0, st, b,
                     m, gate);
  if (bucket1 && (e = hipEventRecord(bucket1, st)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_msm_group, dim3(m.s.groups()), dim3(64), 0, st, m, gate);
  hipLaunchKernelGGL(k_msm_final, dim3(1), dim3(64), 0, st, b, m, gate);
  const int nchunks = (b.npad + ZG_FR_CHUNK - 1) / ZG_FR_CHUNK;
  hipLaunchKernelGGL(k_fr_root, dim3(nchunks), dim3(ZG_NKINDS * ZG_MAX_IC * ZG_FR_G), 0, st, b, m, gate);
  hipLaunchKernelGGL(k_fr_final, dim3(1), dim3(ZG_NKINDS * ZG_MAX_IC * ZG_FR_G), 0, st, b, m, nchunks, gate);
  return hipGetLastError();
}

hipError_t launch_c_leaves(hipStream_t st, const BatchBufs& b) {
  hipLaunchKernelGGL(k_c_leaves, dim3((b.npad + 63) / 64), dim3(64), 0, st, b);
  return hipGetLastError();
}

}  // namespace zg
