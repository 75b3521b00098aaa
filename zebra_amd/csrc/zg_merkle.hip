// zg_merkle.hip -- note-commitment trees on the GPU: the kernels of
// zg_merkle.h and the host side of zg_merkle_combine / zg_tree_empty_roots / zg_tree_roots.
//
// zg_tree_roots is the window form of the reference's per-block tree work: starting from a
// TreeState (storage/src/tree_state.rs:193-264, in its serialized form :284-309) it appends a
// run of commitments and returns the root after each requested prefix -- one per block for
// db/src/block_chain_db.rs:254-304 and accept_block.rs:290-320 (BlockSaplingRoot), one per
// JoinSplit for tree_cache.rs:57-71 -- plus the final state. Sequentially that is one append
// (amortised ~1 hash) per leaf and HEIGHT hashes per root, all dependent. Here:
//
//   * the nodes of every level that the window completes are built level by level (level l+1
//     from level l: n / 2^(l+1) + 1 independent hashes), the input state's frontier standing
//     in for the nodes left of the window;
//   * each requested root is the usual right-edge walk -- at level l the running node is
//     combined with its completed left sibling, or with the empty root of the level -- and
//     the walks of all roots advance together with the level build, in the same launch.
//
// HEIGHT launches in all (one per level, each ~ one hash deep), n + HEIGHT x roots hashes.
// Roots equal the reference's for every prefix (TreeState::root pads with H::empty()[level],
// which is the padded full tree: tests/test_merkle.py).
#include <hip/hip_runtime.h>

#include <string.h>

#include <algorithm>
#include <array>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/zg.h"
#include "zg_merkle.h"

namespace zg {

#define ZG_TREE_EMPTY_LEVELS 64  // H::empty()[0..63] (MerkleTree(depth) needs depth < 63)

// (enc0 + 16 enc1) 2^(8 w) G_g as a niels point; lane per entry
__global__ void __launch_bounds__(64) k_ph_table(uint32_t* table) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ZG_PH_POINTS) return;
  const int code = t % ZG_PH_CODES, w = (t / ZG_PH_CODES) % ZG_PH_WIN, g = t / (ZG_PH_CODES * ZG_PH_WIN);
  const int e = ph_enc(code & 7) + (w < ZG_PH_WIN - 1 ? 16 * ph_enc((uint32_t)code >> 3) : 0);
  const uint32_t* gx = g == 0 ? PEDERSEN_G0_X : g == 1 ? PEDERSEN_G1_X : PEDERSEN_G2_X;
  const uint32_t* gy = g == 0 ? PEDERSEN_G0_Y : g == 1 ? PEDERSEN_G1_Y : PEDERSEN_G2_Y;
  uint32_t k[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t m = (uint64_t)(e < 0 ? -e : e) << (8 * (w & 3));
  k[w >> 2] = (uint32_t)m;
  if ((w >> 2) < 7) k[(w >> 2) + 1] = (uint32_t)(m >> 32);
  Fr x, y;
  jx_to_aff(jx_mul(jx_from_aff(jj_const(gx), jj_const(gy)), k, 256), &x, &y);
  if (e < 0) x = fp_neg<FrM>(x);
  const Fr ypx = fr_add(y, x), ymx = fp_sub<FrM>(y, x), kk = fr_mul(fr_mul(x, y), jj_const(JUBJUB_D2));
  uint32_t* o = table + (size_t)t * ZG_PH_WORDS;
  for (int l = 0; l < 8; l++) {
    o[l] = ypx.l[l];
    o[8 + l] = ymx.l[l];
    o[16 + l] = kk.l[l];
  }
}

template <int KIND, int LANES>
__global__ void __launch_bounds__(64) k_merkle_combine(int n, const uint32_t* l, const uint32_t* r,
                                                       const uint8_t* depth, const uint32_t* table, uint32_t* out) {
  const long long t = blockIdx.x * 64ll + threadIdx.x;
  const int i = (int)(t / LANES), sub = (int)(t % LANES);
  if (i >= n) return;
  tree_combine<KIND, LANES>(l + 8 * (size_t)i, r + 8 * (size_t)i, depth ? depth[i] : 0, table, sub, out + 8 * (size_t)i);
}

// H::empty() one level at a time: e[l + 1] = combine(e[l], e[l], l) (a one-time, per device
// table; e[0], the uncommitted leaf, is written by the host)
template <int KIND, int LANES>
__global__ void __launch_bounds__(64) k_tree_empty_step(uint32_t* e, int l, const uint32_t* table) {
  if (blockIdx.x || threadIdx.x >= LANES) return;
  tree_combine<KIND, LANES>(e + 8 * l, e + 8 * l, l, table, threadIdx.x, e + 8 * (l + 1));
}

// one level: items [0, nm) advance a root walk (pos = leaf index of the root's last leaf),
// items [nm, nm + cnt_next) build the next level's nodes base_next + j
template <int KIND, int LANES>
__global__ void __launch_bounds__(64) k_tree_level(TreeLevel L, int level, int nm, const unsigned long long* pos,
                                                   uint32_t* cur, uint32_t* wnext, long long base_next,
                                                   long long cnt_next, const uint32_t* table) {
  const long long t = (blockIdx.x * 64ll + threadIdx.x) / LANES;
  const int sub = (int)(threadIdx.x % LANES);
  const uint32_t *a, *b;
  uint32_t* o;
  if (t < nm) {
    const long long p = (long long)(pos[t] >> level);
    const uint32_t* c = level == 0 ? tree_node(L, p) : cur + 8 * t;
    if (p & 1) {
      a = tree_node(L, p - 1);
      b = c;
    } else {
      a = c;
      b = L.empty;
    }
    o = cur + 8 * t;
  } else if (t - nm < cnt_next) {
    const long long i = base_next + (t - nm);
    a = tree_node(L, 2 * i);
    b = tree_node(L, 2 * i + 1);
    o = wnext + 8 * (t - nm);
  } else {
    return;
  }
  tree_combine<KIND, LANES>(a, b, level, table, sub, o);
}

__global__ void k_gather32(int n, const uint32_t* const* src, uint32_t* out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 8 * n) return;
  out[t] = src[t >> 3][t & 7];
}

// ------------------------------------------------------------------ host side
struct MerkleDev {
  std::mutex mu;
  uint32_t* ph = nullptr;                                    // Pedersen table (first Sapling use)
  uint32_t* empty[2] = {nullptr, nullptr};                   // device H::empty() per kind
  uint8_t empty_h[2][ZG_TREE_EMPTY_LEVELS][32] = {};         // host copy
};

MerkleDev* merkle_dev_new() { return new MerkleDev(); }
void merkle_dev_free(MerkleDev* m) {
  if (!m) return;
  if (m->ph) hipFree(m->ph);
  for (auto* e : m->empty)
    if (e) hipFree(e);
  delete m;
}

struct Scratch {
  std::vector<void*> p;
  ~Scratch() {
    for (void* q : p) hipFree(q);
  }
  template <class T>
  hipError_t alloc(T** x, size_t bytes) {
    hipError_t e = hipMalloc((void**)x, bytes ? bytes : 1);
    if (e == hipSuccess) p.push_back(*x);
    return e;
  }
};

#define MCHK(expr)                                                         \
  do {                                                                     \
    hipError_t e_ = (expr);                                                \
    if (e_ != hipSuccess) {                                                \
      *err = std::string(#expr ": ") + hipGetErrorString(e_);              \
      return ZG_E_HIP;                                                     \
    }                                                                      \
  } while (0)

static unsigned blocks64(long long n) { return (unsigned)((n + 63) / 64); }

// the Pedersen table and the kind's empty roots, built once per device
static int merkle_ready(MerkleDev* m, hipStream_t st, int kind, std::string* err) {
  std::lock_guard<std::mutex> g(m->mu);
  if (kind == ZG_TREE_SAPLING && !m->ph) {
    uint32_t* t = nullptr;
    MCHK(hipMalloc(&t, ZG_PH_TABLE_BYTES));
    hipLaunchKernelGGL(k_ph_table, dim3(blocks64(ZG_PH_POINTS)), dim3(64), 0, st, t);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
      hipFree(t);
      *err = std::string("Pedersen table: ") + hipGetErrorString(e);
      return ZG_E_HIP;
    }
    m->ph = t;
  }
  if (!m->empty[kind]) {
    uint32_t* e = nullptr;
    MCHK(hipMalloc(&e, ZG_TREE_EMPTY_LEVELS * 32));
    uint8_t e0[32] = {0};
    e0[0] = kind == ZG_TREE_SAPLING ? 1 : 0;  // pedersen_uncommitted() = Fr one; Sprout: zero
    hipError_t he = hipMemcpyAsync(e, e0, 32, hipMemcpyHostToDevice, st);
    for (int l = 0; he == hipSuccess && l + 1 < ZG_TREE_EMPTY_LEVELS; l++) {
      if (kind == ZG_TREE_SAPLING)
        hipLaunchKernelGGL((k_tree_empty_step<ZG_TREE_SAPLING, ZG_PH_LANES_WIDE>), dim3(1), dim3(64), 0, st, e, l, (const uint32_t*)m->ph);
      else
        hipLaunchKernelGGL((k_tree_empty_step<ZG_TREE_SPROUT, 1>), dim3(1), dim3(64), 0, st, e, l, (const uint32_t*)m->ph);
      he = hipGetLastError();
    }
    if (he == hipSuccess) he = hipMemcpyAsync(m->empty_h[kind], e, ZG_TREE_EMPTY_LEVELS * 32, hipMemcpyDeviceToHost, st);
    if (he == hipSuccess) he = hipStreamSynchronize(st);
    if (he != hipSuccess) {
      hipFree(e);
      *err = std::string("empty roots: ") + hipGetErrorString(he);
      return ZG_E_HIP;
    }
    m->empty[kind] = e;
  }
  return ZG_OK;
}

int merkle_combine(MerkleDev* m, hipStream_t st, int kind, size_t n, const uint8_t* l, const uint8_t* r,
                   const uint8_t* depth, uint8_t* out, std::string* err) {
  int rc = merkle_ready(m, st, kind, err);
  if (rc || !n) return rc;
  Scratch s;
  uint32_t *dl, *dr, *dout;
  uint8_t* dd = nullptr;
  MCHK(s.alloc(&dl, 32 * n));
  MCHK(s.alloc(&dr, 32 * n));
  MCHK(s.alloc(&dout, 32 * n));
  MCHK(hipMemcpyAsync(dl, l, 32 * n, hipMemcpyHostToDevice, st));
  MCHK(hipMemcpyAsync(dr, r, 32 * n, hipMemcpyHostToDevice, st));
  if (depth) {
    MCHK(s.alloc(&dd, n));
    MCHK(hipMemcpyAsync(dd, depth, n, hipMemcpyHostToDevice, st));
  }
  if (kind == ZG_TREE_SAPLING)
    hipLaunchKernelGGL((k_merkle_combine<ZG_TREE_SAPLING, ZG_PH_LANES_NARROW>), dim3(blocks64(n * ZG_PH_LANES_NARROW)),
                       dim3(64), 0, st, (int)n, dl, dr, dd, (const uint32_t*)m->ph, dout);
  else
    hipLaunchKernelGGL((k_merkle_combine<ZG_TREE_SPROUT, 1>), dim3(blocks64(n)), dim3(64), 0, st, (int)n, dl, dr, dd,
                       (const uint32_t*)m->ph, dout);
  MCHK(hipGetLastError());
  MCHK(hipMemcpyAsync(out, dout, 32 * n, hipMemcpyDeviceToHost, st));
  MCHK(hipStreamSynchronize(st));
  return ZG_OK;
}

int merkle_empty_roots(MerkleDev* m, hipStream_t st, int kind, size_t levels, uint8_t* out, std::string* err) {
  if (levels > ZG_TREE_EMPTY_LEVELS) return ZG_E_INVAL;
  int rc = merkle_ready(m, st, kind, err);
  if (rc) return rc;
  memcpy(out, m->empty_h[kind], 32 * levels);
  return ZG_OK;
}

// the reference's TreeState in its serialized form (tree_state.rs:284-309): Option<H256> is a
// bool byte then the hash; parents a CompactSize-prefixed list of HEIGHT - 1 options
struct HostTree {
  bool has[2] = {false, false};
  uint8_t lr[2][32];
  std::vector<int> phas;
  std::vector<std::array<uint8_t, 32>> par;
};

static bool parse_state(const uint8_t* b, size_t len, int height, HostTree* t) {
  size_t pos = 0;
  auto opt = [&](bool* has, uint8_t* h) -> bool {
    if (pos >= len || b[pos] > 1) return false;
    *has = b[pos++] == 1;
    if (*has) {
      if (pos + 32 > len) return false;
      memcpy(h, b + pos, 32);
      pos += 32;
    }
    return true;
  };
  if (!opt(&t->has[0], t->lr[0]) || !opt(&t->has[1], t->lr[1])) return false;
  if (pos >= len || b[pos] >= 0xfd) return false;
  const size_t np = b[pos++];
  if ((int)np != height - 1) return false;
  t->phas.assign(np, 0);
  t->par.assign(np, {});
  for (size_t i = 0; i < np; i++) {
    bool h;
    if (!opt(&h, t->par[i].data())) return false;
    t->phas[i] = h;
  }
  return pos == len;
}

static size_t write_state(const HostTree& t, uint8_t* out) {
  size_t pos = 0;
  auto opt = [&](bool has, const uint8_t* h) {
    out[pos++] = has ? 1 : 0;
    if (has) {
      memcpy(out + pos, h, 32);
      pos += 32;
    }
  };
  opt(t.has[0], t.lr[0]);
  opt(t.has[1], t.lr[1]);
  out[pos++] = (uint8_t)t.par.size();
  for (size_t i = 0; i < t.par.size(); i++) opt(t.phas[i], t.par[i].data());
  return pos;
}

size_t merkle_state_max_bytes(int height) { return 2 * 33 + 1 + (size_t)(height > 0 ? height - 1 : 0) * 33; }

// Sapling levels with at most ZG_PH_WIDE_ITEMS hashes (one 32-lane group per SIMD, about) run
// wide groups: their time is one hash's latency. Bigger levels run 8-lane groups.
#define ZG_PH_WIDE_ITEMS 512
template <int KIND, int LANES>
static void launch_level(hipStream_t st, const TreeLevel& L, int level, int nm, const unsigned long long* pos,
                         uint32_t* cur, uint32_t* wnext, long long base_next, long long cnt_next,
                         const uint32_t* table) {
  hipLaunchKernelGGL((k_tree_level<KIND, LANES>), dim3(blocks64((nm + cnt_next) * LANES)), dim3(64), 0, st, L,
                     level, nm, pos, cur, wnext, base_next, cnt_next, table);
}

int merkle_tree_roots(MerkleDev* m, hipStream_t st, int kind, int height, const uint8_t* state, size_t state_len,
                      size_t n, const void* leaves, int leaves_on_device, size_t nmarks, const uint64_t* marks,
                      uint8_t* roots, uint8_t* state_out, size_t* state_out_len, float* kernel_ms,
                      void** arena, size_t* arena_cap, std::string* err) {
  if (height < 1 || height > 62 || (kind != ZG_TREE_SPROUT && kind != ZG_TREE_SAPLING)) return ZG_E_INVAL;
  HostTree t;
  t.phas.assign(height - 1, 0);
  t.par.assign(height - 1, {});
  if (state && state_len && !parse_state(state, state_len, height, &t)) {
    *err = "tree state does not parse (TreeState serialization of this height)";
    return ZG_E_INVAL;
  }
  // the frontier must be one that appends produce: left before right before any parent
  bool any_parent = false;
  for (int p : t.phas) any_parent |= p != 0;
  if ((!t.has[0] && (t.has[1] || any_parent))) {
    *err = "tree state is not an append frontier (right or a parent set without left)";
    return ZG_E_INVAL;
  }
  for (size_t k = 0; k < nmarks; k++)
    if (marks[k] > n) {
      *err = "a mark exceeds the number of leaves";
      return ZG_E_INVAL;
    }
  if (state_out && (!state_out_len || *state_out_len < merkle_state_max_bytes(height))) {
    *err = "state_out smaller than zg_tree_state_max_bytes(height)";
    return ZG_E_INVAL;
  }
  int rc = merkle_ready(m, st, kind, err);
  if (rc) return rc;
  // s0: leaves in the input state ((s0 - 1) >> 1 pairs in the parents counter + 1 or 2)
  unsigned long long c = 0;
  for (int i = 0; i < height - 1; i++)
    if (t.phas[i]) c |= 1ull << i;
  const unsigned long long s0 = t.has[0] ? 2 * c + (t.has[1] ? 2 : 1) : 0;
  const unsigned long long capacity = 1ull << height;
  const unsigned long long n_eff = std::min<unsigned long long>(n, capacity - s0);
  const unsigned long long s1 = s0 + n_eff;

  // level extents (W_l holds nodes base .. base + cnt - 1 of level l)
  std::vector<long long> lbase(height, 0), lcnt(height, 0);
  lbase[0] = (long long)s0;
  lcnt[0] = (long long)n_eff;
  for (int l = 1; l < height; l++) {
    lbase[l] = s0 ? (long long)((s0 - 1) >> l) : 0;
    const long long last = s1 ? (long long)((s1 - 1) >> l) : -1;
    lcnt[l] = std::max(0ll, last - lbase[l] + 1);
  }
  // root walks: marks with at least one leaf and within capacity
  std::vector<unsigned long long> pos;
  std::vector<size_t> which;
  bool full = false;
  for (size_t k = 0; k < nmarks; k++) {
    if (marks[k] > n_eff) {
      full = true;
      continue;
    }
    const unsigned long long sz = s0 + marks[k];
    if (sz) {
      pos.push_back(sz - 1);
      which.push_back(k);
    }
  }
  const int nm = (int)pos.size();
  // one device allocation per context, reused across calls (grow-only, zg_destroy frees it)
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  size_t need = al(32 * (2 + (size_t)height)) + (leaves_on_device ? 0 : al(32 * n_eff)) +
                al(sizeof(unsigned long long) * (nm + 1)) + al(32 * (size_t)(nm + 1)) +
                2 * al(32 * (size_t)(height + 1));
  for (int l = 1; l < height; l++) need += al(32 * (size_t)lcnt[l]);
  if (*arena_cap < need) {
    if (*arena) hipFree(*arena);
    *arena = nullptr;
    *arena_cap = 0;
    MCHK(hipMalloc(arena, need));
    *arena_cap = need;
  }
  char* bump = (char*)*arena;
  auto take = [&](size_t b) {
    char* p = bump;
    bump += al(b);
    return (void*)p;
  };
  // frontier slots: [0] leaf s0 - 1, [1] leaf s0 - 2, [2 + i] parents[i] (level i + 1)
  std::vector<uint8_t> fh(32 * (2 + height), 0);
  if (s0) {
    const bool even = (s0 & 1) == 0;
    memcpy(&fh[0], even ? t.lr[1] : t.lr[0], 32);
    if (even) memcpy(&fh[32], t.lr[0], 32);
  }
  for (int i = 0; i < height - 1; i++)
    if (t.phas[i]) memcpy(&fh[32 * (2 + i)], t.par[i].data(), 32);
  uint32_t* dfront = (uint32_t*)take(fh.size());
  MCHK(hipMemcpyAsync(dfront, fh.data(), fh.size(), hipMemcpyHostToDevice, st));
  const uint32_t* dleaves = (const uint32_t*)leaves;
  if (!leaves_on_device) {
    uint32_t* dl = (uint32_t*)take(32 * n_eff);
    if (n_eff) MCHK(hipMemcpyAsync(dl, leaves, 32 * n_eff, hipMemcpyHostToDevice, st));
    dleaves = dl;
  }
  const uint32_t* E = m->empty[kind];
  // level descriptors
  std::vector<TreeLevel> L(height);
  L[0] = {dleaves, lbase[0], lcnt[0], dfront, dfront + 8, E};
  std::vector<uint32_t*> wbuf(height, nullptr);
  for (int l = 1; l < height; l++) {
    wbuf[l] = (uint32_t*)take(32 * (size_t)lcnt[l]);
    L[l] = {wbuf[l], lbase[l], lcnt[l], dfront + 8 * (2 + (l - 1)), nullptr, E + 8 * l};
  }
  unsigned long long* dpos = (unsigned long long*)take(sizeof(unsigned long long) * (nm + 1));
  uint32_t* dcur = (uint32_t*)take(32 * (size_t)(nm + 1));
  if (nm) MCHK(hipMemcpyAsync(dpos, pos.data(), sizeof(unsigned long long) * nm, hipMemcpyHostToDevice, st));
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (kernel_ms) {
    MCHK(hipEventCreate(&e0));
    MCHK(hipEventCreate(&e1));
    MCHK(hipEventRecord(e0, st));
  }
  for (int l = 0; l < height; l++) {
    const bool top = l + 1 == height;
    const long long cnt_next = top ? 0 : L[l + 1].cnt;
    if (!nm && !cnt_next) continue;
    uint32_t* wn = top ? nullptr : wbuf[l + 1];
    const long long bn = top ? 0 : L[l + 1].base;
    if (kind == ZG_TREE_SPROUT)
      launch_level<ZG_TREE_SPROUT, 1>(st, L[l], l, nm, dpos, dcur, wn, bn, cnt_next, m->ph);
    else if (nm + cnt_next <= ZG_PH_WIDE_ITEMS)
      launch_level<ZG_TREE_SAPLING, ZG_PH_LANES_WIDE>(st, L[l], l, nm, dpos, dcur, wn, bn, cnt_next, m->ph);
    else
      launch_level<ZG_TREE_SAPLING, ZG_PH_LANES_NARROW>(st, L[l], l, nm, dpos, dcur, wn, bn, cnt_next, m->ph);
    MCHK(hipGetLastError());
  }
  if (kernel_ms) MCHK(hipEventRecord(e1, st));
  std::vector<uint8_t> cur(32 * (size_t)nm);
  if (nm) MCHK(hipMemcpyAsync(cur.data(), dcur, cur.size(), hipMemcpyDeviceToHost, st));
  // the final frontier: left / right = leaves s1 - 1, s1 - 2 by parity; parents[i] = the
  // completed level-(i+1) node left of the last leaf's ancestor when that ancestor is odd
  HostTree fin;
  fin.phas.assign(height - 1, 0);
  fin.par.assign(height - 1, {});
  std::vector<const uint32_t*> src;
  std::vector<int> slot;  // 0 left, 1 right, 2 + i parents[i]
  if (s1) {
    if (s1 & 1) {
      src.push_back(tree_node(L[0], (long long)s1 - 1));
      slot.push_back(0);
    } else {
      src.push_back(tree_node(L[0], (long long)s1 - 2));
      slot.push_back(0);
      src.push_back(tree_node(L[0], (long long)s1 - 1));
      slot.push_back(1);
    }
    for (int i = 0; i + 1 < height; i++) {
      const long long P = (long long)((s1 - 1) >> (i + 1));
      if (P & 1) {
        src.push_back(tree_node(L[i + 1], P - 1));
        slot.push_back(2 + i);
      }
    }
  }
  std::vector<uint8_t> fr(32 * src.size());
  if (!src.empty() && state_out && !full) {
    const uint32_t** dsrc = (const uint32_t**)take(sizeof(void*) * src.size());
    uint32_t* dout = (uint32_t*)take(fr.size());
    MCHK(hipMemcpyAsync(dsrc, src.data(), sizeof(void*) * src.size(), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_gather32, dim3(blocks64(8 * (long long)src.size())), dim3(64), 0, st, (int)src.size(),
                       (const uint32_t* const*)dsrc, dout);
    MCHK(hipGetLastError());
    MCHK(hipMemcpyAsync(fr.data(), dout, fr.size(), hipMemcpyDeviceToHost, st));
  }
  MCHK(hipStreamSynchronize(st));
  if (kernel_ms) {
    MCHK(hipEventElapsedTime(kernel_ms, e0, e1));
    hipEventDestroy(e0);
    hipEventDestroy(e1);
  }
  if (roots) {
    for (size_t k = 0; k < nmarks; k++) {
      if (marks[k] > n_eff)
        memset(roots + 32 * k, 0, 32);
      else if (!(s0 + marks[k]))
        memcpy(roots + 32 * k, m->empty_h[kind][height], 32);
    }
    for (int j = 0; j < nm; j++) memcpy(roots + 32 * which[j], &cur[32 * (size_t)j], 32);
  }
  if (full) {
    *err = "Appending to full tree";
    return ZG_E_TREE_FULL;
  }
  if (state_out) {
    for (size_t j = 0; j < slot.size(); j++) {
      if (slot[j] < 2) {
        fin.has[slot[j]] = true;
        memcpy(fin.lr[slot[j]], &fr[32 * j], 32);
      } else {
        fin.phas[slot[j] - 2] = 1;
        memcpy(fin.par[slot[j] - 2].data(), &fr[32 * j], 32);
      }
    }
    *state_out_len = write_state(fin, state_out);
  }
  return ZG_OK;
}

}  // namespace zg
