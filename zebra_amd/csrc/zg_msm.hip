// zg_msm.hip -- translation unit of K4, the Pippenger MSM for sum r_i C_i per key and the root
// Fr sums (zg_msm.h), plus the bisection-only per-proof C leaves.
#include <hip/hip_runtime.h>
#include <stdlib.h>

// (the lazy-digit products stay out of line, zg_fqd.h ZG_FQD_CALL = 1: inlined, k_msm_bucket drops
// its 8-B call frame and runs 0.89 -> 0.82 ms isolated at 64k, but k_msm_group's 39 k inlined
// instructions take its window-doubling chain -- K4's critical path -- from ~0.9 to 1.3 ms;
// profiles/r05l_kernel_stats_iso_k4_inline.csv)

#include "../../include/zg.h"
#include "zg_msm.h"

#ifndef ZG_K4_DBL_WAVE
#define ZG_K4_DBL_WAVE 1  // k_msm_group's window doublings on three lanes (g1d_dbl_wave, round 6)
#endif

namespace zg {

// the scalar of point j of proof i: j = 0 -> k0 = 2a + 1 (65 bits), j = 1 -> k1 = b
ZG_INL void msm_scalar(const BatchBufs& b, int i, int j, uint64_t* lo, uint32_t* hi) {
  uint64_t ra, rb;
  batch_scalar_ab(b.r + (size_t)i * 16, &ra, &rb);
  *lo = j ? rb : (ra << 1) | 1u;
  *hi = j ? 0u : (uint32_t)(ra >> 63);
}

ZG_INL bool msm_live(const BatchBufs& b, int i) { return i < b.n && b.status[i] == ST_PENDING; }

// lane (proof i, point j): the bucket sizes; lanes (i, 0) and (i, 1) also write C_i's digit
// operands once for the bucket phase: (x, y) and beta x respectively (zg_fqd.h FqD, < 2p each)
__global__ void __launch_bounds__(64) k_msm_count(BatchBufs b, MsmBufs m, const int* gate) {
  if (gate && *gate == 0) return;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = t >> 1, j = t & 1;
  if (i >= b.npad || !msm_live(b, i)) return;
  {
    const G1A c = b.ptAC[(size_t)b.npad + i];
    uint32_t* row = m.cd + (size_t)i * ZG_MSM_CD;
    const FqD u = j ? fqd_from(fq_mul(c.x, fq_const(G1_BETA))) : fqd_from(c.x);
#pragma unroll
    for (int q = 0; q < 14; q++) row[16 * j + q] = u.d[q];
    if (!j) {
      const FqD y = fqd_from(c.y);
#pragma unroll
      for (int q = 0; q < 14; q++) row[32 + q] = y.d[q];
    }
  }
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

// 14 digits of an FqD operand row (16 words, 4 x uint4; the last two words are padding)
ZG_INL FqD msm_ld_digits(const uint32_t* row) {
  const uint4* v = (const uint4*)row;
  const uint4 a = v[0], c = v[1], d = v[2], e = v[3];
  return FqD{{a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w, e.x, e.y}};
}

// whether (key, window) group g holds any entry (a key absent from the batch: none)
ZG_INL bool msm_group_live(const MsmBufs& m, int g) { return m.start[(g + 1) * m.s.nb] > m.start[g * m.s.nb]; }

// The bucket phase with the first reduction level (see zg_msm.h). Wave gw of the grid holds
// segment gw: buckets [gw BS, (gw + 1) BS) (BS = 64 / P, inside one (key, window) group), lane =
// (bucket j, part); the segment's outputs are T = sum_j (j + 1) S_j and U = sum_j S_j. LDS: the
// waves' staged entries, then (the same bytes) the block's lane points for the reductions.
__global__ void __launch_bounds__(ZG_MSM_BT) k_msm_bucket(BatchBufs b, MsmBufs m, const int* gate) {
  if (gate && *gate == 0) return;
  constexpr int NW = ZG_MSM_BT / 64;
  constexpr int WORDS = NW * ZG_MSM_STAGE > ZG_MSM_BT * (int)(sizeof(G1D) / 4) ? NW * ZG_MSM_STAGE
                                                                               : ZG_MSM_BT * (int)(sizeof(G1D) / 4);
  __shared__ uint32_t lds[WORDS];
  G1D* sh = (G1D*)lds;
  const MsmShape S = m.s;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, w0 = threadIdx.x & ~63;
  const int gw = blockIdx.x * NW + wv;
  const int P = S.parts, BS = S.bs();
  // whole waves are live or not: past the grid's buckets, or a group without entries
  const bool live = gw * BS < S.ncount() && msm_group_live(m, gw / S.nseg());
  const int j = lane / P, part = lane % P;
  // stage the segment's sorted entries in LDS (coalesced); a segment past the stage reads in place
  const int slo = live ? m.start[gw * BS] : 0, shi = live ? m.start[(gw + 1) * BS] : 0;
  const bool staged = shi - slo <= ZG_MSM_STAGE;
  uint32_t* st = lds + wv * ZG_MSM_STAGE;
  if (live && staged)
    for (int e = lane; e < shi - slo; e += 64) st[e] = m.entries[slo + e];
  __syncthreads();
  G1D acc = g1d_infinity();
  if (live) {
    const int bucket = gw * BS + j;
    const int lo = m.start[bucket], len = m.start[bucket + 1] - lo;
    const int beg = lo + len * part / P, end = lo + len * (part + 1) / P;
    // (an entry past what k_msm_scatter wrote can only be stale when the R-chain flipped a
    // status between count and scatter -- then bfail > 0 and settle_batch (zg.hip) recomputes the
    // root sums on the host's request; it must still stay inside the buffers). The next entry's operands are gathered while the
    // current one is added: their L2 / HBM latency hides behind the addition.
    auto entry = [&](int e) { return staged ? st[e - slo] : m.entries[e]; };
    auto gather = [&](uint32_t ent, FqD* x, FqD* y) {
      const uint32_t pi = ent >> 2;
      const uint32_t* row = m.cd + (size_t)(pi < (uint32_t)b.npad ? pi : 0) * ZG_MSM_CD;
      *x = msm_ld_digits(row + ((ent & 2u) ? 16 : 0));
      *y = msm_ld_digits(row + 32);
    };
    uint32_t ent_n = 0;
    FqD x_n, y_n;
    if (beg < end) {
      ent_n = entry(beg);
      gather(ent_n, &x_n, &y_n);
    }
    for (int e = beg; e < end; e++) {
      const uint32_t ent = ent_n;
      const FqD x = x_n, y = y_n;
      if (e + 1 < end) {
        ent_n = entry(e + 1);
        gather(ent_n, &x_n, &y_n);
      }
      if ((ent >> 2) >= (uint32_t)b.npad) continue;
      acc = g1d_add_aff(acc, x, (ent & 1u) ? fqd_neg2(y) : y);  // x < 2p, y < 3p
    }
  }
  __syncthreads();  // the stage is read: its bytes become the lane points
  // merge the P parts of each bucket: S_j lands in lane j P
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int d = 1; d < P; d <<= 1) {
    G1D v = sh[threadIdx.x];
    if (part % (2 * d) == 0) v = g1d_add_full(v, sh[threadIdx.x + d]);
    __syncthreads();
    sh[threadIdx.x] = v;
    __syncthreads();
  }
  // compact: lane j < BS holds S_j
  if (P > 1) {
    G1D v = lane < BS ? sh[w0 + lane * P] : g1d_infinity();
    __syncthreads();
    sh[threadIdx.x] = v;
    __syncthreads();
  }
  // suffix sums H_j = sum_{j' >= j} S_j' (inclusive Hillis-Steele, BS lanes)
  for (int d = 1; d < BS; d <<= 1) {
    G1D u = sh[threadIdx.x];
    if (lane + d < BS) u = g1d_add_full(u, sh[threadIdx.x + d]);
    __syncthreads();
    sh[threadIdx.x] = u;
    __syncthreads();
  }
  // U = H_0, written at once (held across the tree it would live in the private segment)
  const bool out = gw * BS < S.ncount() && lane == 0;  // (a group without entries writes infinity)
  G1D* seg = m.seg + ((size_t)(gw / S.nseg()) * ZG_MSM_SEG_MAX + gw % S.nseg()) * 2;
  if (out) seg[1] = sh[w0];
  // T = sum_j H_j: tree over the BS suffix sums
  for (int d = BS / 2; d >= 1; d >>= 1) {
    G1D u = sh[threadIdx.x];
    if (lane < d) u = g1d_add_full(u, sh[threadIdx.x + d]);
    __syncthreads();
    sh[threadIdx.x] = u;
    __syncthreads();
  }
  if (out) seg[0] = sh[w0];
}

// one wave per (key, window) group: sum_b (b + 1) S_b = sum_s (T_s + BS s U_s), with
// sum_s s U_s = sum_{s >= 1} H_s, H_s = sum_{s' >= s} U_s' (lane s = segment s). Lazy digits
// throughout (zg_fqd.h): the window's 2^shift(w) doubling chain is this kernel's critical path.
__global__ void __launch_bounds__(64) k_msm_group(MsmBufs m, const int* gate) {
  if (gate && *gate == 0) return;
  __shared__ G1D sh[64];
  const MsmShape S = m.s;
  const int g = blockIdx.x, s = threadIdx.x, ns = S.nseg();
  if (!msm_group_live(m, g)) {  // a key absent from the batch (wave-uniform)
    if (s == 0) m.wsum[g] = g1d_infinity();
    return;
  }
  const G1D* sg = m.seg + (size_t)g * ZG_MSM_SEG_MAX * 2;
  const G1D T = s < ns ? sg[2 * s] : g1d_infinity();
  sh[s] = s < ns ? sg[2 * s + 1] : g1d_infinity();
  __syncthreads();
  for (int d = 1; d < ns; d <<= 1) {
    G1D u = sh[s];
    if (s + d < ns) u = g1d_add_full(u, sh[s + d]);
    __syncthreads();
    sh[s] = u;
    __syncthreads();
  }
  G1D x = T;
  if (s >= 1 && s < ns) {
    G1D h = sh[s];
    for (int q = S.bs(); q > 1; q >>= 1) h = g1d_dbl(h);  // BS = 2^k
    x = g1d_add_full(x, h);
  }
  __syncthreads();
  sh[s] = x;
  __syncthreads();
  int top = 1;
  while (top < ns) top <<= 1;
  for (int d = top / 2; d >= 1; d >>= 1) {  // the lanes past ns hold infinity
    G1D u = sh[s];
    if (s < d) u = g1d_add_full(u, sh[s + d]);
    __syncthreads();
    sh[s] = u;
    __syncthreads();
  }
  // 2^shift(w) W_w: this window's part of sum_w 2^shift(w) W_w, the kernel's critical path (the top
  // window: 55 doublings at 64k). ZG_K4_DBL_WAVE (default): each doubling's seven products as three
  // levels over lanes 0..2 (g1d_dbl_wave, same digits); 0: the doublings on lane 0 alone.
  // Infinity (Z = 0) stays infinity.
  const int w = g % S.w;
#if ZG_K4_DBL_WAVE
  __shared__ FqD xch[3];
  G1D q = sh[0];
  for (int k = 0; k < S.shift(w); k++) q = g1d_dbl_wave(q, xch);
  if (s == 0) m.wsum[g] = q;
#else
  if (s == 0) {
    G1D q = sh[0];
    for (int k = 0; k < S.shift(w); k++) q = g1d_dbl(q);
    m.wsum[g] = q;
  }
#endif
}

// per key: sum_w of the scaled window sums (k_msm_group) -> the root node of the C-sum tree (node 1)
__global__ void __launch_bounds__(64) k_msm_final(BatchBufs b, MsmBufs m, const int* gate) {
  if (gate && *gate == 0) return;
  const int kind = threadIdx.x;
  if (kind >= ZG_NKINDS) return;
  const MsmShape S = m.s;
  G1D acc = m.wsum[kind * S.w];
  for (int w = 1; w < S.w; w++) acc = g1d_add_full(acc, m.wsum[kind * S.w + w]);
  b.ctree[1 * ZG_NKINDS + kind] = g1d_to_jac(acc);
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
// alone: no other batch on the device (the bucket phase's lanes per bucket: zg_msm.h)
hipError_t launch_msm_root(hipStream_t st, const BatchBufs& b, MsmBufs m, const int* gate, hipEvent_t bucket0,
                           hipEvent_t bucket1, int k4, bool alone) {
  m.s = msm_shape(b.npad, alone);
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
