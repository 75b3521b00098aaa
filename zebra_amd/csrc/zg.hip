// zg.hip -- host side of the MI355X batch Groth16 verifier: the C ABI of include/zg.h.
// One translation unit: the kernels (zg_kernels.h) are launched from here on the
// context's private HIP stream. Everything that touches curve or field arithmetic runs
// on the GPU; the host parses bytes, drives launches and the bisection, and moves data.
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include <sys/random.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/zg.h"
#include "zg_blake2b.h"
#include "zg_chacha.h"
#include "zg_kernels.h"
#include "zg_msm.h"
#include "zg_prep.h"
#include "zg_vk_embed.h"  // generated from zebra_amd/res/*.json by zebra_amd/build.py

using namespace zg;

#define ZG_BLOCK 64
#define ZG_NODE_CHUNK 4096
#define ZG_LP_PARTS_MAX 8
#define ZG_EV_SETTLE (15 + ZG_LP_PARTS_MAX)  // settle_batch's recompute (no timing)
#define ZG_NEV (16 + ZG_LP_PARTS_MAX)  // [13]: zg_gt_check; [14..] line-product parts, [14 + max] chains done,
                                       // [15 + max] settle_batch (no timing)
// the pinned host block of a context: the root's 576-B Miller partial, the pipeline flags
// (bfail, fused-wait failure), the K4 entry count, then the n statuses
#define ZG_PIN_FLAGS 576
#define ZG_PIN_ENTRIES 584
#define ZG_PIN_STATUS 640
#define ZG_NTIMINGS 9
#define ZG_NSTATS 13
#define ZG_TREE_COOP_BELOW 4096  // product-tree levels with fewer nodes run one wave per node
#define ZG_LINE_PROD_MIN 32768   // shards from this many padded proofs run the f-chain as group line products
#define ZG_QUAD_MIN 8192         // shards from this many (padded) proofs run the f-chain four proofs per lane (r02z: -4% at 16k, -1% at 8k)
#define ZG_K4_MIN 16384          // lone batches from this many (padded) proofs sum r_i C_i by K4's Pippenger
                                 // buckets; smaller lone batches by the GLV products in decode + the C tree
                                 // levels (run_pipeline: batches in flight always use K4)
#define ZG_LINES_LANE_MIN 32768  // straight-line R-chain from here (r03: 64k 14.93 -> 14.47 ms per batch in
                                 // flight; 16k 4.90 -> 5.14 and 8k 3.21 -> 3.63 favour the staged program)
#define ZG_DEFAULT_PAIRS 8       // stream pairs per device (ZG_STREAM_PAIRS overrides, 1..16)
#define ZG_HI_PAIRS 4            // high-priority stream pairs per device (zg_set_priority round-robin)

namespace zg {  // zg_merkle.hip
struct MerkleDev;
MerkleDev* merkle_dev_new();
void merkle_dev_free(MerkleDev* m);
int merkle_combine(MerkleDev* m, hipStream_t st, int kind, size_t n, const uint8_t* l, const uint8_t* r,
                   const uint8_t* depth, uint8_t* out, std::string* err);
int merkle_empty_roots(MerkleDev* m, hipStream_t st, int kind, size_t levels, uint8_t* out, std::string* err);
size_t merkle_state_max_bytes(int height);
int merkle_tree_roots(MerkleDev* m, hipStream_t st, int kind, int height, const uint8_t* state, size_t state_len,
                      size_t n, const void* leaves, int leaves_on_device, size_t nmarks, const uint64_t* marks,
                      uint8_t* roots, uint8_t* state_out, size_t* state_out_len, float* kernel_ms,
                      void** arena, size_t* arena_cap, std::string* err);
// zg_pghr13.hip
struct BnDev;
struct BnKey;
BnDev* bn_dev_new();
void bn_dev_free(BnDev* d);
int bn_load_vk_json(BnDev* d, hipStream_t st, const char* json, size_t len, const BnKey** out, std::string* err);
void bn_key_release(BnDev* d, const BnKey* k);
int bn_pghr13_verify(const BnKey* k, hipStream_t st, hipStream_t side, size_t n, const uint8_t* proofs,
                     const uint8_t* inputs, const uint8_t* ninputs, const uint8_t* rho, uint8_t* status,
                     float* kernel_ms, bool* batch_failed, void** arena, size_t* arena_cap, std::string* err);
int bn_pairing(hipStream_t st, size_t n, const uint8_t* g1, const uint8_t* g2, uint8_t* gt, std::string* err);
}  // namespace zg

// Per-device state shared by every context (batch slot) on that GPU: a FIXED pool of stream
// pairs, created once, and the prepared verifying keys. A context only owns buffers, so a
// process can hold any number of slots without creating another HIP stream / hardware queue.
// Why: each hardware queue that dispatches a kernel with a private (scratch) segment keeps a
// scratch allocation sized for the whole device; the process's scratch pool is bounded, and
// with a stream pair per context the 7th in-flight context on one GPU pushed it over
// (HSA_STATUS_ERROR_OUT_OF_RESOURCES from the queue). With the pool, the
// number of queues -- hence of scratch reservations -- no longer grows with the slots.
struct zg_dev {
  int device = 0;
  int ncu = 0;
  int refs = 0;
  std::mutex mu;  // the pool cursor and the VK cache
  int npairs = 0;
  hipStream_t main[16] = {}, side[16] = {};
  // high-priority pairs (lazy, zg_set_priority): a few, so that concurrent checker contexts (one per
  // verdict thread) do not serialise their final exponentiations on one stream
  hipStream_t hi_main[ZG_HI_PAIRS] = {}, hi_side[ZG_HI_PAIRS] = {};
  int hi_next = 0;
  int next = 0;
  struct VKEntry {
    RawVK raw;
    DevVK* d = nullptr;
    uint32_t* comb = nullptr;  // the key's comb tables (ZG_COMB_POINTS x 96 B, k_vk_comb)
    int err = 0;
  };
  std::vector<VKEntry*> vks;  // prepare_verifying_key once per distinct key per device
  uint32_t* jj_comb = nullptr;  // Jubjub generators' comb tables (zg_jubjub.h), built on first use
  zg::MerkleDev* merkle = nullptr;  // Pedersen table + empty roots (zg_merkle.hip), first use
  zg::BnDev* bn = nullptr;          // PGHR13 key, line and comb tables (zg_pghr13.hip), first use
  std::atomic<int> inflight{0};     // contexts on this device with a batch begun and not finished
};

static std::mutex g_devs_mu;
static zg_dev* g_devs[64] = {};
static thread_local std::string g_create_err;

struct zg_ctx {
  int device = 0;
  zg_dev* dev = nullptr;
  hipStream_t stream = nullptr;  // from the device pool (not owned)
  hipStream_t side = nullptr;    // VK-side root work, concurrent with the Miller kernels
  int pair = 0;
  std::mutex mu;
  std::string err;
  uint32_t cap = 0;  // power of two >= max_batch
  int seeded = 0;
  uint64_t seed = 0;
  int vk_loaded[ZG_NKINDS] = {0, 0, 0};
  int vk_iclen[ZG_NKINDS] = {0, 0, 0};
  RawVK vk_raw[ZG_NKINDS];  // host copies of the loaded keys (shared alpha / beta / gamma test)
  int merged = 0;           // loaded keys share alpha, beta, gamma: merged VK-side pairs (zg_batch.h)
  DevVK* d_vk = nullptr;  // this slot's 3 kinds (copied from the device cache)
  int* d_int = nullptr;   // scratch ints: [8] bfail, [9] fused-wait failure
  // batch
  uint8_t *d_proofs = nullptr, *d_kinds = nullptr, *d_inputs = nullptr, *d_ninputs = nullptr, *d_r = nullptr,
          *d_status = nullptr, *d_bytes = nullptr, *d_okbits = nullptr;
  G1A* d_ptA = nullptr;
  G1A* d_ptAC = nullptr;
  int* d_prog = nullptr;  // cap / 64: per lines block, steps published (fused R-chain + f-chain)
  int ncu = 0;            // compute units of the device
  int fuse = -1;          // ZG_LINES_FCHAIN: -1 auto (both grids resident at once), 0 never, 1 always
  int fuse_off = 0;       // a fused launch ever timed out waiting: split launches from then on
  int serial_side = 0;    // ZG_SERIAL_SIDE=1: the side-stream work runs on the main stream after the
                          // product tree (measurement: the Miller kernels alone on the device)
  G2A* d_ptB = nullptr;
  Fq12* d_ftree = nullptr;
  Fq2* d_lines = nullptr;  // cap x 68 x 3: per-proof line triples (R-chain -> f-chain)
  Fq2* d_lprod = nullptr;  // cap / 4 x 68 x 6: per-group line products (k_line_prod)
  Fq2* d_fstate = nullptr; // cap / 4 x 6: each group chain's f between its parts (k_batch_fchaing)
  G1J* d_ctree = nullptr;
  Fr* d_stree = nullptr;
  MsmBufs msm = {};       // K4: Pippenger sum r_i C_i per key + root Fr sums (zg_msm.h)
  int trees_built = 0;    // the full C / Fr trees exist for this batch (bisection only)
  int c_tree_pending = 0; // the C tree is still being built on the side stream (ev[12])
  // node checks
  int* d_nodes = nullptr;
  G1J* d_msm = nullptr;
  Fq12* d_pairf = nullptr;
  int* d_ok = nullptr;
  Fq12* d_out = nullptr;
  // state of the split API
  int state = 0;
  size_t n = 0, npad = 0;
  const uint8_t* cur_ninputs = nullptr;  // device pointer or null
  // this batch's inputs on the device: the context's own buffers (host-buffer calls copy into
  // them), or the caller's HBM-resident buffers (zg_batch_begin_device: read in place, no copy)
  const uint8_t *cur_proofs = nullptr, *cur_kinds = nullptr, *cur_inputs = nullptr;
  int root_pairs_ready = 0;  // the pipeline already ran the root's MSM + VK pairs on `side`
  int settled = 0;           // settle_batch ran for this batch
  int alone_last = 0;        // the last batch ran with no other batch in flight (K4 shape)
  int eager = 0;             // the pipeline's last steps copied the root partial, flags and statuses to h_pin (ev[4])
  uint8_t* h_pin = nullptr;  // pinned host memory: ZG_PIN_* layout
  uint8_t* h_gt = nullptr;   // pinned staging of zg_gt_check (partials in, verdict out; grow-only)
  size_t h_gt_cap = 0;
  int fused_last = 0;        // the last batch used the fused R-chain + f-chain launch
  int lines_lane = -1;      // ZG_LINES_LANE: -1 auto (the straight-line R-chain from ZG_LINES_LANE_MIN padded
                            // proofs, sized for 1 wave per SIMD when the batch is alone on the device, else
                            // 2; the staged program below), 1 / 2 always straight-line sized for 2 / 1
                            // waves per SIMD, 0 always the staged program (zg_kernels.h)
  int quads = -1;            // ZG_FCHAIN_QUADS: -1 auto (npad >= ZG_QUAD_MIN), 0 never, 1 always (npad >= 4)
  int line_group = -1;       // ZG_LINE_GROUP: proofs per group (k_line_prod): -1 auto (32 from ZG_LINE_PROD_MIN
                             // padded proofs, else the quad chain), 0 never, a power of two >= 4 always
  int lineprod_last = 0;     // the last batch's f-chain ran on group line products (no tree below the groups)
  int lines_affine = 0;      // ZG_LINES_AFFINE: K (2, 4, 8) -- the group line products run on affine lines from
                             // k_batch_lines_aff, K proofs per lane (round 6); 0 projective
  int lines_affine_xl = 0;   // ZG_LINES_AFFINE_XL=1: its cross-lane variant (one inversion per wave; K = 4)
  int affine_last = 0;       // the last batch's lines are affine (bisection re-forms projective ones)
  int quad_split = 1;        // ZG_QUAD_SPLIT: 1 a step's four lines multiply first, then into f (Q4IK + GM / GMSQ,
                             // round 6), 0 the fused Q4 / Q4SQ programs (same values)
  int lp_parts = 0;          // ZG_LINE_PROD_PARTS: step parts overlapping line products and chains: 1..8 equal
                             // parts, 0 (default) wave-aligned parts (lineprod_parts)
  int pairs_late = 0;        // ZG_PAIRS_LATE=1: with group line products, the root's VK MSM + pairs go on the side
                             // stream AFTER the group chains instead of before them (round 6, r06f: 8k with line
                             // products 2.88 -> 2.77 ms per batch, still behind the quad chain's 2.61; 16k 4.19 ->
                             // 4.30, 64k 12.33 -> 12.46: not the default)
  long k4_min = ZG_K4_MIN;   // ZG_K4_MIN overrides: K4 Pippenger from this many padded proofs, else decode GLV + C tree
  int k4_last = 1;           // the last batch summed r_i C_i with K4 (0: the C tree is built, bisection reuses it)
  int quads_last = 0;        // the last batch's f-chain ran four proofs per lane (no pair-level nodes)
  int singles = -1;          // ZG_FCHAIN_SINGLE: -1 auto (a fused launch runs one proof per f-chain lane), 0 never
  int singles_last = 0;      // the last batch's f-chain wrote the per-proof leaves (bisection reuses them)
  size_t coop_below = ZG_TREE_COOP_BELOW;  // ZG_TREE_COOP_BELOW overrides (product-tree wave-per-node levels)
  hipEvent_t ev[ZG_NEV] = {};
  float timings[ZG_NTIMINGS] = {};
  // [0] batches, [1] fused launches, [2] fused-wait failures, [3] B subgroup failures
  // (bfail, deferred recomputes), [4] bisections, [5] nodes checked by bisection,
  // [6] K4 bucket entries of the last batch (points with a non-zero digit, summed over windows)
  uint64_t stats[ZG_NSTATS] = {};
  uint64_t calls = 0;
  int debug_each = 0;         // ZG_DEBUG_EACH=1: every batch's statuses re-checked per proof
  uint8_t* d_dbg = nullptr;   // the per-proof statuses of that re-check
  const zg::BnKey* bn_key = nullptr;  // this slot's PGHR13 key (an immutable, reference-counted entry of the device cache)
  uint8_t* prep_arena = nullptr;  // zg_prep_batch device buffers (grow-only)
  size_t prep_arena_cap = 0;
  void* tree_arena = nullptr;  // zg_tree_roots scratch (grow-only, zg_merkle.hip)
  size_t tree_arena_cap = 0;
  void* bn_arena = nullptr;  // zg_pghr13_verify scratch (grow-only, zg_pghr13.hip)
  size_t bn_arena_cap = 0;
};

static int fail(zg_ctx* c, int code, const std::string& msg) {
  c->err = msg;
  return code;
}
#define HIPCHK(expr)                                                                              \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess) return fail(ctx, ZG_E_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

// Wait for an event by polling (hipEventQuery + a short sleep) instead of hipEventSynchronize /
// hipStreamSynchronize: the host loop of batches in flight calls into the runtime from two threads
// (batch launches / harvests on the main one, the verdicts' final exponentiations on a worker), and
// a blocking synchronize on one thread held up the other's calls until the GPU work it waited for
// had finished (8k shards: every relaunch came ~1 ms after the verdict's final exponentiation).
static hipError_t wait_event(hipEvent_t e) {
  for (;;) {
    const hipError_t r = hipEventQuery(e);
    if (r != hipErrorNotReady) return r;
    std::this_thread::sleep_for(std::chrono::microseconds(10));
  }
}

static unsigned nblocks(size_t n) { return (unsigned)((n + ZG_BLOCK - 1) / ZG_BLOCK); }

extern "C" const char* zg_last_error(zg_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_err.c_str(); }

template <class T>
static hipError_t dalloc(T** p, size_t count) {
  return hipMalloc((void**)p, sizeof(T) * (count ? count : 1));
}

static void dev_release(zg_dev* d) {
  std::lock_guard<std::mutex> g(g_devs_mu);
  if (--d->refs > 0) return;
  hipSetDevice(d->device);
  for (int i = 0; i < d->npairs; i++) {
    if (d->main[i]) hipStreamDestroy(d->main[i]);
    if (d->side[i]) hipStreamDestroy(d->side[i]);
  }
  for (int k = 0; k < ZG_HI_PAIRS; k++) {
    if (d->hi_main[k]) hipStreamDestroy(d->hi_main[k]);
    if (d->hi_side[k]) hipStreamDestroy(d->hi_side[k]);
  }
  for (auto* e : d->vks) {
    if (e->d) hipFree(e->d);
    if (e->comb) hipFree(e->comb);
    delete e;
  }
  if (d->jj_comb) hipFree(d->jj_comb);
  merkle_dev_free(d->merkle);
  bn_dev_free(d->bn);
  g_devs[d->device] = nullptr;
  delete d;
}

// the device's state, created on first use (streams created here, never per context)
static zg_dev* dev_acquire(int device, std::string* err) {
  std::lock_guard<std::mutex> g(g_devs_mu);
  if (device < 0 || device >= 64) {
    *err = "bad device ordinal";
    return nullptr;
  }
  zg_dev* d = g_devs[device];
  if (!d) {
    d = new zg_dev();
    d->device = device;
    int np = ZG_DEFAULT_PAIRS;
    if (const char* e = getenv("ZG_STREAM_PAIRS")) np = atoi(e);
    np = np < 1 ? 1 : np > 16 ? 16 : np;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&d->ncu, hipDeviceAttributeMultiprocessorCount, device);
    for (int i = 0; e == hipSuccess && i < np; i++) {
      e = hipStreamCreateWithFlags(&d->main[i], hipStreamNonBlocking);
      if (e == hipSuccess) e = hipStreamCreateWithFlags(&d->side[i], hipStreamNonBlocking);
      if (e == hipSuccess) d->npairs = i + 1;
    }
    if (e != hipSuccess) {
      *err = std::string("device init: ") + hipGetErrorString(e);
      d->refs = 1;
      g_devs[device] = d;
      g_devs_mu.unlock();
      dev_release(d);
      g_devs_mu.lock();
      return nullptr;
    }
    g_devs[device] = d;
  }
  d->refs++;
  return d;
}

extern "C" zg_ctx* zg_create(const zg_config* cfg) {
  zg_config def = {0, 65536, 0, 0};
  if (!cfg) cfg = &def;
  g_create_err.clear();
  zg_dev* dev = dev_acquire(cfg->device, &g_create_err);
  if (!dev) return nullptr;
  zg_ctx* ctx = new zg_ctx();
  ctx->dev = dev;
  ctx->device = cfg->device;
  uint32_t mb = cfg->max_batch ? cfg->max_batch : 65536;
  uint32_t cap = 2;
  while (cap < mb) cap <<= 1;
  ctx->cap = cap;
  ctx->seeded = cfg->seeded;
  ctx->seed = cfg->seed;
  ctx->ncu = dev->ncu;
  {
    std::lock_guard<std::mutex> g(dev->mu);
    ctx->pair = dev->next++ % dev->npairs;
  }
  ctx->stream = dev->main[ctx->pair];
  ctx->side = dev->side[ctx->pair];
  if (const char* e = getenv("ZG_LINES_FCHAIN")) ctx->fuse = atoi(e);
  if (const char* e = getenv("ZG_SERIAL_SIDE")) ctx->serial_side = atoi(e);
  if (const char* e = getenv("ZG_FCHAIN_QUADS")) ctx->quads = atoi(e);
  if (const char* e = getenv("ZG_LINE_GROUP")) ctx->line_group = atoi(e);
  if (const char* e = getenv("ZG_QUAD_SPLIT")) ctx->quad_split = atoi(e) ? 1 : 0;
  if (const char* e = getenv("ZG_LINES_AFFINE")) {
    const int k = atoi(e);
    ctx->lines_affine = k == 2 || k == 4 || k == 8 ? k : 0;
  }
  if (const char* e = getenv("ZG_LINES_AFFINE_XL")) ctx->lines_affine_xl = atoi(e) ? 1 : 0;
  if (ctx->lines_affine_xl) ctx->lines_affine = 4;
  if (const char* e = getenv("ZG_LINE_PROD_PARTS")) ctx->lp_parts = std::max(1, std::min(ZG_LP_PARTS_MAX, atoi(e)));
  if (const char* e = getenv("ZG_PAIRS_LATE")) ctx->pairs_late = atoi(e) ? 1 : 0;
  if (ctx->line_group != -1 && (ctx->line_group < 4 || (ctx->line_group & (ctx->line_group - 1)))) ctx->line_group = 0;
  if (const char* e = getenv("ZG_K4_MIN")) ctx->k4_min = atol(e);
  if (const char* e = getenv("ZG_FCHAIN_SINGLE")) ctx->singles = atoi(e);
  if (const char* e = getenv("ZG_LINES_LANE")) ctx->lines_lane = atoi(e);
  if (const char* e = getenv("ZG_TREE_COOP_BELOW")) ctx->coop_below = (size_t)atol(e);
  if (const char* e = getenv("ZG_DEBUG_EACH")) ctx->debug_each = atoi(e);
  hipError_t e = hipSetDevice(ctx->device);
  auto A = [&](hipError_t r) {
    if (e == hipSuccess) e = r;
  };
  A(dalloc(&ctx->d_vk, ZG_NKINDS));
  A(dalloc(&ctx->d_int, 16));
  A(dalloc(&ctx->d_proofs, (size_t)cap * 192));
  A(dalloc(&ctx->d_kinds, cap));
  A(dalloc(&ctx->d_inputs, (size_t)cap * 288));
  A(dalloc(&ctx->d_ninputs, cap));
  A(dalloc(&ctx->d_r, ((size_t)cap + 3) / 4 * 64));  // whole ChaCha20 blocks
  A(dalloc(&ctx->d_status, cap));
  A(dalloc(&ctx->d_okbits, (size_t)cap * 3));
  A(dalloc(&ctx->d_bytes, (size_t)576 * ZG_NODE_CHUNK));
  A(dalloc(&ctx->d_ptA, cap));
  A(dalloc(&ctx->d_ptAC, 2 * (size_t)cap));
  A(dalloc(&ctx->d_prog, (size_t)cap / 64 + 1));
  A(dalloc(&ctx->d_ptB, cap));
  A(dalloc(&ctx->d_ftree, 2 * (size_t)cap));
  A(dalloc(&ctx->d_lines, (size_t)cap * ZG_NCOEFF * 3));
  // group line products: sized for the smallest group that can run on this context (an explicit
  // ZG_LINE_GROUP, else the automatic 32 from ZG_LINE_PROD_MIN padded proofs; none below that)
  const uint32_t lp_gmin = ctx->line_group > 0 ? (uint32_t)ctx->line_group
                                                : ctx->line_group < 0 && cap >= ZG_LINE_PROD_MIN ? 32u : 0u;
  if (lp_gmin) A(dalloc(&ctx->d_lprod, ((size_t)cap / lp_gmin + 1) * ZG_NCOEFF * 6));
  if (lp_gmin) A(dalloc(&ctx->d_fstate, ((size_t)cap / lp_gmin + 1) * 6));
  A(dalloc(&ctx->d_ctree, 2 * (size_t)cap * ZG_NKINDS));
  A(dalloc(&ctx->d_stree, 2 * (size_t)cap * ZG_NKINDS * ZG_MAX_IC));
  A(dalloc(&ctx->msm.count, ZG_MSM_NCOUNT_MAX));
  A(dalloc(&ctx->msm.start, ZG_MSM_NCOUNT_MAX + 1));
  A(dalloc(&ctx->msm.cursor, ZG_MSM_NCOUNT_MAX));
  A(dalloc(&ctx->msm.entries, 2 * (size_t)cap * ZG_MSM_WMAX));
  A(dalloc(&ctx->msm.cd, (size_t)cap * ZG_MSM_CD));
  A(dalloc(&ctx->msm.seg, (size_t)ZG_MSM_GROUPS_MAX * ZG_MSM_SEG_MAX * 2));
  A(dalloc(&ctx->msm.wsum, ZG_MSM_GROUPS_MAX));
  A(dalloc(&ctx->msm.frpart, ((size_t)cap / ZG_FR_CHUNK + 1) * ZG_NKINDS * ZG_MAX_IC));
  A(dalloc(&ctx->d_nodes, ZG_NODE_CHUNK));
  A(dalloc(&ctx->d_msm, (size_t)ZG_NODE_CHUNK * ZG_NKINDS * ZG_MSM_SLOTS * ZG_SHIFTS));
  A(dalloc(&ctx->d_pairf, (size_t)ZG_NODE_CHUNK * ZG_NODE_PAIRS));
  A(dalloc(&ctx->d_ok, ZG_NODE_CHUNK));
  A(dalloc(&ctx->d_out, ZG_NODE_CHUNK));
  if (ctx->debug_each) A(dalloc(&ctx->d_dbg, cap));
  A(hipHostMalloc((void**)&ctx->h_pin, ZG_PIN_STATUS + (size_t)cap, hipHostMallocDefault));
  for (int i = 0; i < ZG_NEV; i++)
    A(i < 14 ? hipEventCreate(&ctx->ev[i]) : hipEventCreateWithFlags(&ctx->ev[i], hipEventDisableTiming));
  // surface a broken device / stream now rather than inside a later batch
  A(hipMemsetAsync(ctx->d_vk, 0, sizeof(DevVK) * ZG_NKINDS, ctx->stream));
  A(hipMemsetAsync(ctx->d_int, 0, sizeof(int) * 16, ctx->side));
  A(hipMemsetAsync(ctx->msm.entries, 0, sizeof(uint32_t) * 2 * (size_t)cap * ZG_MSM_WMAX, ctx->side));
  A(hipStreamSynchronize(ctx->stream));
  A(hipStreamSynchronize(ctx->side));
  if (e != hipSuccess) {
    g_create_err = std::string(e == hipErrorOutOfMemory ? "out of device memory: " : "HIP error: ") +
                   hipGetErrorString(e);
    zg_destroy(ctx);
    return nullptr;
  }
  return ctx;
}

static void set_state(zg_ctx* ctx, int st);

extern "C" void zg_destroy(zg_ctx* ctx) {
  if (!ctx) return;
  hipSetDevice(ctx->device);
  // the pool's streams outlive the slot: drain this slot's work before its buffers go
  if (ctx->stream) hipStreamSynchronize(ctx->stream);
  if (ctx->side) hipStreamSynchronize(ctx->side);
  if (ctx->bn_key && ctx->dev) zg::bn_key_release(ctx->dev->bn, ctx->bn_key);
  void* ptrs[] = {ctx->d_vk, ctx->d_int, ctx->d_proofs, ctx->d_kinds, ctx->d_inputs, ctx->d_ninputs,
                  ctx->d_r, ctx->d_status, ctx->d_bytes, ctx->d_ptA, ctx->d_ptB, ctx->d_ftree, ctx->d_ctree,
                  ctx->d_stree, ctx->d_nodes, ctx->d_msm, ctx->d_pairf, ctx->d_ok, ctx->d_out, ctx->d_lines, ctx->d_lprod, ctx->d_fstate,
                  ctx->d_okbits, ctx->d_ptAC, ctx->d_prog, ctx->msm.count, ctx->msm.start, ctx->msm.cursor,
                  ctx->msm.entries, ctx->msm.cd, ctx->msm.seg, ctx->msm.wsum, ctx->msm.frpart, ctx->tree_arena,
                  ctx->bn_arena, ctx->d_dbg, ctx->prep_arena};
  for (void* p : ptrs)
    if (p) hipFree(p);
  if (ctx->h_pin) hipHostFree(ctx->h_pin);
  if (ctx->h_gt) hipHostFree(ctx->h_gt);
  for (int i = 0; i < ZG_NEV; i++)
    if (ctx->ev[i]) hipEventDestroy(ctx->ev[i]);
  set_state(ctx, 0);
  zg_dev* d = ctx->dev;
  delete ctx;
  if (d) dev_release(d);
}

// ------------------------------------------------------------------ verifying keys
// the loaded keys share alpha_g1, beta_g2 and gamma_g2 (byte-identical): their gamma pairs and
// their beta pairs merge (zg_batch.h ZG_NODE_PAIRS_MERGED)
static void update_merged(zg_ctx* ctx) {
  int first = -1, same = 1;
  for (int k = 0; k < ZG_NKINDS; k++) {
    if (!ctx->vk_loaded[k]) continue;
    if (first < 0) {
      first = k;
      continue;
    }
    const RawVK &a = ctx->vk_raw[first], &c = ctx->vk_raw[k];
    same = same && !memcmp(a.alpha_g1, c.alpha_g1, 96) && !memcmp(a.beta_g2, c.beta_g2, 192) &&
           !memcmp(a.gamma_g2, c.gamma_g2, 192);
  }
  ctx->merged = same;
}

// prepare_verifying_key runs once per distinct key per device (k_vk_prepare, one thread,
// ~140 ms); every further slot that loads the same key gets a device-to-device copy.
static int vk_upload(zg_ctx* ctx, int kind, const RawVK& raw) {
  if (kind < 0 || kind >= ZG_NKINDS) return fail(ctx, ZG_E_INVAL, "bad kind");
  if (raw.n_ic > ZG_MAX_IC) return fail(ctx, ZG_E_INVAL, "ic longer than 10");
  if (ctx->state) return fail(ctx, ZG_E_STATE, "verifying key load with a batch in flight");
  HIPCHK(hipSetDevice(ctx->device));
  zg_dev* dev = ctx->dev;
  zg_dev::VKEntry* ent = nullptr;
  {
    std::lock_guard<std::mutex> g(dev->mu);
    for (auto* e : dev->vks)
      if (memcmp(&e->raw, &raw, sizeof(RawVK)) == 0) ent = e;
    if (!ent) {
      ent = new zg_dev::VKEntry();
      ent->raw = raw;
      RawVK* d_raw = nullptr;
      hipError_t e = hipMalloc(&ent->d, sizeof(DevVK));
      if (e == hipSuccess) e = hipMalloc(&ent->comb, sizeof(uint32_t) * ZG_COMB_WORDS * (size_t)ZG_COMB_POINTS);
      if (e == hipSuccess) e = hipMalloc(&d_raw, sizeof(RawVK));
      if (e == hipSuccess) e = hipMemcpyAsync(d_raw, &raw, sizeof(RawVK), hipMemcpyHostToDevice, ctx->stream);
      if (e == hipSuccess) e = hipMemsetAsync(ent->d, 0, sizeof(DevVK), ctx->stream);
      if (e == hipSuccess) {
        hipLaunchKernelGGL(k_vk_prepare, dim3(1), dim3(1), 0, ctx->stream, d_raw, ent->d, ctx->d_int,
                           (const uint32_t*)ent->comb);
        e = hipGetLastError();
      }
      if (e == hipSuccess) {
        hipLaunchKernelGGL(k_vk_comb, dim3((ZG_COMB_POINTS + 63) / 64), dim3(64), 0, ctx->stream,
                           (const DevVK*)ent->d, ent->comb);
        e = hipGetLastError();
      }
      if (e == hipSuccess) e = hipMemcpyAsync(&ent->err, ctx->d_int, sizeof(int), hipMemcpyDeviceToHost, ctx->stream);
      if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
      if (d_raw) hipFree(d_raw);
      if (e != hipSuccess) {
        if (ent->d) hipFree(ent->d);
        if (ent->comb) hipFree(ent->comb);
        delete ent;
        return fail(ctx, ZG_E_HIP, std::string("prepare_verifying_key: ") + hipGetErrorString(e));
      }
      dev->vks.push_back(ent);
    }
  }
  if (ent->err) {
    HIPCHK(hipMemsetAsync(ctx->d_vk + kind, 0, sizeof(DevVK), ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->vk_loaded[kind] = 0;
    update_merged(ctx);
    return fail(ctx, ZG_E_VK, "Invalid curve point in verifying key (field " + std::to_string(ent->err) + ")");
  }
  HIPCHK(hipMemcpyAsync(ctx->d_vk + kind, ent->d, sizeof(DevVK), hipMemcpyDeviceToDevice, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  ctx->vk_loaded[kind] = 1;
  ctx->vk_iclen[kind] = raw.n_ic;
  ctx->vk_raw[kind] = raw;
  update_merged(ctx);
  return ZG_OK;
}

extern "C" int zg_vk_load_uncompressed(zg_ctx* ctx, int kind, const uint8_t alpha_g1[96], const uint8_t beta_g1[96],
                                       const uint8_t beta_g2[192], const uint8_t gamma_g2[192],
                                       const uint8_t delta_g1[96], const uint8_t delta_g2[192], size_t n_ic,
                                       const uint8_t* ic) {
  if (!ctx) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  RawVK raw;
  memset(&raw, 0, sizeof(raw));
  memcpy(raw.alpha_g1, alpha_g1, 96);
  memcpy(raw.beta_g1, beta_g1, 96);
  memcpy(raw.beta_g2, beta_g2, 192);
  memcpy(raw.gamma_g2, gamma_g2, 192);
  memcpy(raw.delta_g1, delta_g1, 96);
  memcpy(raw.delta_g2, delta_g2, 192);
  if (n_ic > ZG_MAX_IC) return fail(ctx, ZG_E_INVAL, "ic longer than 10");
  raw.n_ic = (int)n_ic;
  if (n_ic) memcpy(raw.ic, ic, 96 * n_ic);
  return vk_upload(ctx, kind, raw);
}

// crypto/src/json/groth16.rs:33-102: serde fields -> hex (optional 0x) of exact length
static bool json_str_after(const std::string& s, size_t pos, size_t* b, size_t* e) {
  size_t q = s.find('"', pos);
  if (q == std::string::npos) return false;
  size_t r = s.find('"', q + 1);
  if (r == std::string::npos) return false;
  *b = q + 1;
  *e = r;
  return true;
}
static bool hex_decode(const std::string& s, size_t b, size_t e, uint8_t* out, size_t want) {
  if (e - b >= 2 && s[b] == '0' && s[b + 1] == 'x') b += 2;
  if (e - b != 2 * want) return false;
  auto nib = [](char c) -> int {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  };
  for (size_t i = 0; i < want; i++) {
    int h = nib(s[b + 2 * i]), l = nib(s[b + 2 * i + 1]);
    if (h < 0 || l < 0) return false;
    out[i] = (uint8_t)(h * 16 + l);
  }
  return true;
}
static bool json_field(const std::string& s, const char* key, uint8_t* out, size_t want) {
  std::string k = std::string("\"") + key + "\"";
  size_t p = s.find(k);
  if (p == std::string::npos) return false;
  p = s.find(':', p + k.size());
  if (p == std::string::npos) return false;
  size_t b, e;
  return json_str_after(s, p, &b, &e) && hex_decode(s, b, e, out, want);
}

extern "C" int zg_vk_load_json(zg_ctx* ctx, int kind, const char* json, size_t len) {
  if (!ctx || !json) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  std::string s(json, len);
  RawVK raw;
  memset(&raw, 0, sizeof(raw));
  if (!json_field(s, "alphaG1", raw.alpha_g1, 96) || !json_field(s, "betaG1", raw.beta_g1, 96) ||
      !json_field(s, "betaG2", raw.beta_g2, 192) || !json_field(s, "gammaG2", raw.gamma_g2, 192) ||
      !json_field(s, "deltaG1", raw.delta_g1, 96) || !json_field(s, "deltaG2", raw.delta_g2, 192))
    return fail(ctx, ZG_E_VK, "Expected hex string of the right length");
  size_t p = s.find("\"ic\"");
  if (p == std::string::npos) return fail(ctx, ZG_E_VK, "missing ic");
  p = s.find('[', p);
  size_t end = s.find(']', p);
  if (p == std::string::npos || end == std::string::npos) return fail(ctx, ZG_E_VK, "bad ic");
  int n = 0;
  size_t b, e;
  while (json_str_after(s, p, &b, &e) && e < end) {
    if (n >= ZG_MAX_IC) return fail(ctx, ZG_E_VK, "ic longer than 10");
    if (!hex_decode(s, b, e, raw.ic[n], 96)) return fail(ctx, ZG_E_VK, "Expected hex string of length 96");
    n++;
    p = e + 1;
  }
  raw.n_ic = n;
  return vk_upload(ctx, kind, raw);
}

extern "C" int zg_vk_load_builtin(zg_ctx* ctx, int kind) {
  if (!ctx || kind < 0 || kind >= ZG_NKINDS) return ZG_E_INVAL;
  const char* j = ZG_VK_JSON[kind];
  return zg_vk_load_json(ctx, kind, j, strlen(j));
}

static int f12_download(zg_ctx* ctx, const Fq12* d, int count, uint8_t* out) {
  hipLaunchKernelGGL(k_f12_to_bytes, dim3(nblocks(count)), dim3(ZG_BLOCK), 0, ctx->stream, d, count, ctx->d_bytes);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, ctx->d_bytes, (size_t)576 * count, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return ZG_OK;
}

extern "C" int zg_vk_alpha_beta(zg_ctx* ctx, int kind, uint8_t gt[576]) {
  if (!ctx || kind < 0 || kind >= ZG_NKINDS) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (!ctx->vk_loaded[kind]) return fail(ctx, ZG_E_NOVK, "verifying key not loaded");
  HIPCHK(hipSetDevice(ctx->device));
  return f12_download(ctx, &ctx->d_vk[kind].alpha_beta, 1, gt);
}

// ------------------------------------------------------------------ single proof (parity path)
extern "C" int zg_verify_one_gt(zg_ctx* ctx, int kind, const uint8_t proof[192], const uint8_t* inputs,
                                size_t n_inputs, uint8_t* status, uint8_t gt[576]) {
  if (!ctx || kind < 0 || kind >= ZG_NKINDS || !proof || !status || n_inputs > 255) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (!ctx->vk_loaded[kind]) return fail(ctx, ZG_E_NOVK, "verifying key not loaded");
  HIPCHK(hipSetDevice(ctx->device));
  uint8_t in[288];
  memset(in, 0, sizeof(in));
  size_t kk = n_inputs < ZG_MAX_INPUTS ? n_inputs : ZG_MAX_INPUTS;
  if (kk) memcpy(in, inputs, 32 * kk);
  uint8_t k8 = (uint8_t)n_inputs, kind8 = (uint8_t)kind;
  HIPCHK(hipMemcpyAsync(ctx->d_proofs, proof, 192, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipMemcpyAsync(ctx->d_inputs, in, 288, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipMemcpyAsync(ctx->d_kinds, &kind8, 1, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipMemcpyAsync(ctx->d_ninputs, &k8, 1, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(k_verify_single, dim3(1), dim3(ZG_BLOCK), 0, ctx->stream, ctx->d_vk, 1, ctx->d_proofs,
                     ctx->d_kinds, ctx->d_inputs, ctx->d_ninputs, ctx->d_status, ctx->d_bytes);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(status, ctx->d_status, 1, hipMemcpyDeviceToHost, ctx->stream));
  if (gt) HIPCHK(hipMemcpyAsync(gt, ctx->d_bytes, 576, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return ZG_OK;
}

extern "C" int zg_verify_each(zg_ctx* ctx, size_t n, const uint8_t* proofs, const uint8_t* kinds,
                              const uint8_t* inputs, const uint8_t* n_inputs, uint8_t* status, uint8_t* gts) {
  if (!ctx || (n && (!proofs || !kinds || !inputs || !status))) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (n > ctx->cap) return fail(ctx, ZG_E_NOMEM, "batch larger than max_batch");
  HIPCHK(hipSetDevice(ctx->device));
  for (size_t i = 0; i < n; i++)
    if (kinds[i] >= ZG_NKINDS || !ctx->vk_loaded[kinds[i]]) return fail(ctx, ZG_E_NOVK, "verifying key not loaded");
  if (!n) return ZG_OK;
  uint8_t* d_gts = nullptr;
  if (gts) HIPCHK(hipMalloc(&d_gts, 576 * n));
  HIPCHK(hipMemcpyAsync(ctx->d_proofs, proofs, 192 * n, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipMemcpyAsync(ctx->d_kinds, kinds, n, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipMemcpyAsync(ctx->d_inputs, inputs, 288 * n, hipMemcpyHostToDevice, ctx->stream));
  if (n_inputs) HIPCHK(hipMemcpyAsync(ctx->d_ninputs, n_inputs, n, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(k_verify_single, dim3(nblocks(n)), dim3(ZG_BLOCK), 0, ctx->stream, ctx->d_vk, (int)n,
                     ctx->d_proofs, ctx->d_kinds, ctx->d_inputs, n_inputs ? ctx->d_ninputs : nullptr, ctx->d_status,
                     d_gts);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(status, ctx->d_status, n, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess && gts) e = hipMemcpyAsync(gts, d_gts, 576 * n, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (d_gts) hipFree(d_gts);
  if (e != hipSuccess) return fail(ctx, ZG_E_HIP, std::string("zg_verify_each: ") + hipGetErrorString(e));
  return ZG_OK;
}

// ------------------------------------------------------------------ batch
static void gen_scalars(zg_ctx* ctx, size_t n, std::vector<uint8_t>& r) {
  r.resize(n * 16);
  if (ctx->seeded) {
    for (size_t i = 0; i < n; i++) {
      Blake2b h(16);
      h.update("zg-batch-r", 10);
      uint8_t le[8];
      for (int b = 0; b < 8; b++) le[b] = (uint8_t)(ctx->seed >> (8 * b));
      h.update(le, 8);
      for (int b = 0; b < 8; b++) le[b] = (uint8_t)((uint64_t)i >> (8 * b));
      h.update(le, 8);
      h.final(&r[16 * i]);
    }
  }
  // any 16 bytes are a valid batch scalar: r_i = (2a + 1) + b lambda != 0 (zg_groth16.h)
}

static bool os_random(void* buf, size_t len) {
  uint8_t* p = (uint8_t*)buf;
  size_t off = 0;
  while (off < len) {
    ssize_t got = getrandom(p + off, len - off, 0);
    if (got < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    off += (size_t)got;
  }
  return true;
}

// r_i of the current batch into d_r. Seeded contexts (tests) derive them on the host
// (BLAKE2b(seed, i), see gen_scalars); otherwise one fresh 256-bit OS-random ChaCha20 key per
// batch is expanded on the device: 4 proofs per 64-byte block, no host round trip.
static int stage_scalars(zg_ctx* ctx, size_t n) {
  if (!n) return ZG_OK;
  if (ctx->seeded) {
    std::vector<uint8_t> rr;
    gen_scalars(ctx, n, rr);
    HIPCHK(hipMemcpyAsync(ctx->d_r, rr.data(), n * 16, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return ZG_OK;
  }
  ChachaKey k;
  if (!os_random(k.key, sizeof(k.key))) return fail(ctx, ZG_E_INVAL, "getrandom failed");
  k.nonce[0] = k.nonce[1] = k.nonce[2] = 0;  // the key is single-use
  const size_t nb = (n + 3) / 4;
  hipLaunchKernelGGL(k_chacha20, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, ctx->stream, k, 0u, nb,
                     (uint4*)ctx->d_r);
  HIPCHK(hipGetLastError());
  return ZG_OK;
}

static BatchBufs batch_bufs(zg_ctx* ctx) {
  BatchBufs b;
  b.vks = ctx->d_vk;
  b.proofs = ctx->cur_proofs;
  b.kinds = ctx->cur_kinds;
  b.inputs = ctx->cur_inputs;
  b.ninputs = ctx->cur_ninputs;
  b.r = ctx->d_r;
  b.status = ctx->d_status;
  b.ptA = ctx->d_ptA;
  b.ptB = ctx->d_ptB;
  b.ptAC = ctx->d_ptAC;
  b.ftree = ctx->d_ftree;
  b.ctree = ctx->d_ctree;
  b.stree = ctx->d_stree;
  b.bfail = ctx->d_int + 8;
  b.okbits = ctx->d_okbits;
  b.merged = ctx->merged;
  b.n = (int)ctx->n;
  b.npad = (int)ctx->npad;
  return b;
}

static int launch_node_msm_pairs(zg_ctx* ctx, const BatchBufs& b, const NodeBufs& nb, hipStream_t st,
                                 const int* gate = nullptr) {
  hipLaunchKernelGGL(k_node_msm, dim3(nblocks((size_t)nb.m * ZG_NKINDS * ZG_MSM_SLOTS * ZG_SHIFTS)), dim3(ZG_BLOCK),
                     0, st, b, nb, gate);
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(k_node_pairs, dim3(nb.m * (b.merged ? ZG_NODE_PAIRS_MERGED : ZG_NODE_PAIRS)), dim3(64), 0, st,
                     b, nb, gate);
  HIPCHK(hipGetLastError());
  return ZG_OK;
}

namespace zg {
hipError_t launch_batch_decode(unsigned groups, hipStream_t st, const BatchBufs& b, int cglv);  // zg_decode.hip
hipError_t launch_msm_root(hipStream_t st, const BatchBufs& b, MsmBufs m, const int* gate, hipEvent_t bucket0,
                           hipEvent_t bucket1, int k4, bool alone);                                       // zg_msm.hip
hipError_t launch_c_leaves(hipStream_t st, const BatchBufs& b);                                // zg_msm.hip
hipError_t launch_lines_lane(unsigned groups, hipStream_t st, const BatchBufs& b, Fq2* lines, int wpe);  // zg_lines.hip
// the staged-program kernels of zg_kernels.h, one translation unit each (zg_prog_*.hip)
hipError_t launch_prog_lines(unsigned groups, hipStream_t st, const BatchBufs& b, Fq2* lines);
hipError_t launch_prog_leaf_fchain(unsigned blocks, hipStream_t st, const BatchBufs& b, const Fq2* lines,
                                   const int* nodes, int m);
hipError_t launch_prog_fchain(unsigned blocks, hipStream_t st, const BatchBufs& b, const Fq2* lines, const int* gate);
hipError_t launch_prog_fchain4(unsigned blocks, hipStream_t st, const BatchBufs& b, const Fq2* lines, int split);
hipError_t launch_prog_lineprod(hipStream_t st, const BatchBufs& b, const Fq2* lines, Fq2* lprod, int gsize, int n0,
                                int n1, int split, int affine);
hipError_t launch_lines_aff(hipStream_t st, const BatchBufs& b, Fq2* lines, int k, int xl);  // zg_lines.hip
hipError_t launch_prog_fchaing(hipStream_t st, const BatchBufs& b, const Fq2* lprod, Fq2* fstate, int m, int n0,
                               int n1);
hipError_t launch_prog_lines_fchain(unsigned blocks, hipStream_t st, const BatchBufs& b, Fq2* lines, int* prog,
                                    int* fail, int per);
hipError_t launch_prog_fchain1(unsigned blocks, hipStream_t st, const BatchBufs& b, const Fq2* lines, const int* gate);
hipError_t launch_jj_comb(hipStream_t st, uint32_t* table);                                    // zg_jubjub.hip
hipError_t launch_redjubjub(hipStream_t st, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                            const uint8_t* gen, int n, const uint32_t* comb, uint8_t* ok);
hipError_t launch_jj_decode(hipStream_t st, const uint8_t* pts, int n, uint8_t* status, uint8_t* xy);
hipError_t launch_prep_sapling(hipStream_t st, const uint8_t* kinds, const uint8_t* fields, int n, uint8_t* inputs,
                               uint8_t* codes);
hipError_t launch_sapling_bvk(hipStream_t st, int ntx, const uint32_t* off, const uint32_t* nspends,
                              const uint8_t* cvs, const int64_t* vb, const uint32_t* comb, uint8_t* bvk,
                              uint8_t* status);
}

// The pipeline on device-resident inputs already in ctx buffers.
//   main stream: decode -> R-chain (lines + G2 subgroup checks) -> f-chain -> Fq12 product tree
//   side stream: (after decode) K4 Pippenger sum r_i C_i per key + root Fr sums (zg_msm.h)
//                -> root VK-side MSM -> root VK Miller loops
// The side stream only needs the decode results, so its few-thread work overlaps the lines
// and f-chain kernels instead of extending the critical path. A B_i that fails its G2
// subgroup check in k_batch_lines (invalid proofs only) counts in bfail, and the side-stream
// results are then recomputed on the main stream (gated kernels: no-ops when bfail == 0).
// the C-sum tree levels above the leaves (small shards: the GLV leaves k_decode_points wrote), root
// ctree[1]; gate as for the recompute kernels (null: always)
static hipError_t launch_c_tree(zg_ctx* ctx, const BatchBufs& b, hipStream_t st, const int* gate) {
  for (size_t lo = ctx->npad / 2; lo >= 1; lo /= 2)
    hipLaunchKernelGGL(k_tree_c, dim3(nblocks(lo * ZG_NKINDS)), dim3(ZG_BLOCK), 0, st, b, (int)lo, gate);
  return hipGetLastError();
}
// the Fq12 product-tree levels above `top` nodes (ftree[top .. 2 top) written), root ftree[1]
static hipError_t launch_f_tree(zg_ctx* ctx, const BatchBufs& b, size_t top) {
  for (size_t lo = top / 2; lo >= 1; lo /= 2) {
    if (lo >= ctx->coop_below)
      hipLaunchKernelGGL(k_tree_f, dim3(nblocks(lo)), dim3(ZG_BLOCK), 0, ctx->stream, b, (int)lo);
    else
      hipLaunchKernelGGL(k_tree_f_coop, dim3((unsigned)lo), dim3(64), 0, ctx->stream, b, (int)lo);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
// The step parts of the group line products (k_line_prod over steps [n0, n1) while the side stream
// runs the chains of the part before). A launch holds (n1 - n0) x ceil(m / 64) blocks of one CU each
// (153.6 KB of LDS), so a part whose block count is not a multiple of the CU count ends in a partial
// wave of blocks: 64k with four equal parts of 17 steps was 544 blocks = 2.125 block waves in 3.
// wave-aligned (req = 0): parts of two full block waves, the remainder last -- a short last part whose
// chain (the exposed tail) is short too. From the second part on, the previous part's chains hold
// ceil(m / 64) CUs of their own (same block shape), so a wave there has ncu - that many CUs: 64k, 2,048
// groups, 32 blocks a step: steps [0, 16), then 14-step parts, [58, 68) last. req >= 1: req equal parts.
static int lineprod_parts(int req, int m, int ncu, int* bounds) {
  int parts = req;
  if (req <= 0) {
    const int bps = (m + 63) / 64;
    const int first = 2 * std::max(1, ncu / bps), spw = std::max(1, (ncu - bps) / bps);
    int len = 2 * spw;
    while (1 + (ZG_NCOEFF - std::min(first, ZG_NCOEFF) + len - 1) / len > ZG_LP_PARTS_MAX) len += spw;
    parts = 0;
    for (int n = 0; n < ZG_NCOEFF; n += parts == 1 ? first : len) bounds[parts++] = n;
    bounds[parts] = ZG_NCOEFF;
    return parts;
  }
  for (int k = 0; k <= parts; k++) bounds[k] = ZG_NCOEFF * k / parts;
  return parts;
}

static int run_pipeline(zg_ctx* ctx) {
  BatchBufs b = batch_bufs(ctx);
  ctx->eager = 0;
  // the flags (bfail, fused-wait failure) are cleared by the first kernel (k_decode_sqrt); the root's node
  // list is implicit (NodeBufs::nodes null)
  ctx->settled = 0;
  HIPCHK(hipEventRecord(ctx->ev[0], ctx->stream));
  const unsigned dgroups = (unsigned)((ctx->npad + 63) / 64);
  // a lone small batch is latency-bound: the GLV products ride on decode and the tree replaces K4's
  // chains of lone-lane additions (config 2 7.18 -> 6.24 ms with the single-proof f-chain, config 4
  // 25.3 -> 20.7 ms: bisection reuses the tree). With other batches in flight the device is
  // issue-bound and K4's few, mostly waiting waves cost less than the GLV products' work (8k shards,
  // 6 in flight: 2.74 ms per batch with K4, 2.96 with the GLV path; profiles/r04h_env8k.txt)
  const bool alone = ctx->dev->inflight.load(std::memory_order_relaxed) == 0;
  const int k4 = (long)ctx->npad >= ctx->k4_min || !alone ? 1 : 0;
  ctx->k4_last = k4;
  HIPCHK(launch_batch_decode(dgroups, ctx->stream, b, !k4));
  HIPCHK(hipEventRecord(ctx->ev[1], ctx->stream));
  ctx->trees_built = 0;
  ctx->c_tree_pending = 0;
  NodeBufs nb = {nullptr, ctx->d_msm, ctx->d_pairf, ctx->d_ok, ctx->d_out, 1};
  ctx->alone_last = alone;
  // side stream: K4 + the root's VK-side work (or, serial_side, on the main stream after the tree)
  auto side_k4 = [&](hipStream_t st) -> int {
    HIPCHK(hipEventRecord(ctx->ev[5], st));
    HIPCHK(launch_msm_root(st, b, ctx->msm, nullptr, ctx->ev[8], ctx->ev[9], k4, alone));
    if (!k4) HIPCHK(launch_c_tree(ctx, b, st, nullptr));
    HIPCHK(hipEventRecord(ctx->ev[10], st));
    return ZG_OK;
  };
  auto side_pairs = [&](hipStream_t st) -> int {
    int r = launch_node_msm_pairs(ctx, b, nb, st);
    if (r) return r;
    HIPCHK(hipEventRecord(ctx->ev[6], st));
    return ZG_OK;
  };
  int rc;
  // main stream: the R-chain (lines; also the G2 subgroup checks of the B_i), then the f-chain
  // two proofs per lane: the f-chain writes the tree level of proof pairs (npad/2 nodes)
  const unsigned groups = (unsigned)((ctx->npad + 63) / 64);
  const unsigned pgroups = (unsigned)((ctx->npad / 2 + 63) / 64);
  // auto: fuse only a lone batch whose two grids are resident at once. With other batches in
  // flight on the device the split launches overlap them better (8k shards, 6 in flight: 3.79
  // vs 4.20 ms/batch, profiles/r02i_sweep8k.txt), and a fused grid would share the CUs anyway.
  // A fused (lone, small) batch is latency-bound: one proof per f-chain lane, 4 rounds per step
  // instead of the pair step's 6 (config 2: the fused launch 2.95 ms with pairs, r03v). That shape
  // launches 2 groups blocks (pairs: groups + pgroups), and every block must be resident at once.
  const bool want_singles = ctx->singles != 0;
  const unsigned fused_blocks = want_singles ? 2 * groups : groups + pgroups;
  const bool fused = ctx->fuse == 1 ||
                     (ctx->fuse < 0 && !ctx->fuse_off && fused_blocks <= (unsigned)ctx->ncu &&
                      ctx->dev->inflight.load(std::memory_order_relaxed) == 0);
  ctx->fused_last = fused;
  const bool singles = fused && want_singles;
  ctx->singles_last = singles;
  // four proofs per lane on large shards (one block per CU from 64k proofs on): 64 Fq2 products
  // per four proofs and step instead of 76 (k_batch_fchain4)
  const bool quads = !fused && ctx->npad >= 4 && (ctx->quads == 1 || (ctx->quads < 0 && ctx->npad >= ZG_QUAD_MIN));
  ctx->quads_last = quads;
  // group line products (k_line_prod + k_batch_fchaing) instead of the quad chain: auto from
  // ZG_LINE_PROD_MIN, 32 proofs a group (in flight, ms per batch, quad chain -> line products with the
  // chains in four parts, groups of 16 / 32 / 64 / 128: 64k 13.67 -> 12.84 / 12.69 / 12.72 / 13.05, 32k
  // 7.33 -> 7.01 (64: 7.09), 16k 4.15 -> 4.20, 8k 2.63 -> 2.89 with one part;
  // profiles/r05p_lineprod_ab.txt, r05v_lineprod_sweep.txt)
  int gsize = ctx->line_group < 0 ? (ctx->npad >= ZG_LINE_PROD_MIN ? 32 : 0) : ctx->line_group;
  if ((size_t)gsize > ctx->npad || !ctx->d_lprod) gsize = 0;  // (d_lprod: zg_create sized it for this gsize)
  const bool lineprod = quads && gsize;
  ctx->lineprod_last = lineprod;
  // affine R-chain (ZG_LINES_AFFINE = K proofs per lane): only for the group line products, whose AQ4
  // program reads its (a, b) lines; bisection re-forms projective lines for the chains below the groups
  const bool affine = lineprod && ctx->lines_affine;
  ctx->affine_last = affine;
  // the group chains run on the side stream in parts (below): with pairs_late the root's VK MSM + pairs
  // follow the last chain part there instead of preceding the first (8k with line products, r05aa: the
  // first chain waited 2.8 ms behind k_node_pairs although its part was formed)
  const bool late = lineprod && ctx->lp_parts != 1 && ctx->pairs_late && !ctx->serial_side;
  if (!ctx->serial_side) {
    HIPCHK(hipStreamWaitEvent(ctx->side, ctx->ev[1], 0));
    if ((rc = side_k4(ctx->side))) return rc;
    if (!late && (rc = side_pairs(ctx->side))) return rc;
  }
  if (fused) {  // one launch, f-chain blocks consuming each published lines step (k_lines_fchain)
    HIPCHK(hipEventRecord(ctx->ev[7], ctx->stream));
    HIPCHK(hipMemsetAsync(ctx->d_prog, 0, groups * sizeof(int), ctx->stream));
    if (singles) {
      HIPCHK(launch_prog_lines_fchain(2 * groups, ctx->stream, b, ctx->d_lines, ctx->d_prog, b.bfail + 1, 1));
      // no-op unless bfail / wait failure
      HIPCHK(launch_prog_fchain1(groups, ctx->stream, b, (const Fq2*)ctx->d_lines, (const int*)b.bfail));
    } else {
      HIPCHK(launch_prog_lines_fchain(groups + pgroups, ctx->stream, b, ctx->d_lines, ctx->d_prog, b.bfail + 1, 2));
      // no-op unless bfail / wait failure
      HIPCHK(launch_prog_fchain(pgroups, ctx->stream, b, (const Fq2*)ctx->d_lines, (const int*)b.bfail));
    }
  } else {
    const bool lane = ctx->lines_lane > 0 || (ctx->lines_lane < 0 && ctx->npad >= ZG_LINES_LANE_MIN);
    if (affine) {  // affine lines for the group line products (zg_lines.hip k_batch_lines_aff)
      HIPCHK(launch_lines_aff(ctx->stream, b, ctx->d_lines, ctx->lines_affine, ctx->lines_affine_xl));
    } else if (lane) {  // lane = proof, straight-line products (zg_lines.hip)
      // register budget: auto sizes for one wave per SIMD (512 VGPRs: 64k alone 3.70 -> 3.38 ms) when no
      // other batch is on the device, else two (in flight the SIMDs' second slot serves the other
      // batches' kernels: 4 in flight 14.93 vs 14.47 ms per batch; profiles/r03c_bench_lines_lane*.json)
      const bool alone = ctx->dev->inflight.load(std::memory_order_relaxed) == 0;
      const int wpe = ctx->lines_lane == 2 ? 1 : ctx->lines_lane == 1 ? 2 : alone ? 1 : 2;
      HIPCHK(launch_lines_lane(groups, ctx->stream, b, ctx->d_lines, wpe));
    } else {                // staged program, lane = proof, wave = product (zg_kernels.h)
      HIPCHK(launch_prog_lines(groups, ctx->stream, b, ctx->d_lines));
    }
    HIPCHK(hipEventRecord(ctx->ev[7], ctx->stream));
    const unsigned qgroups = (unsigned)((ctx->npad / 4 + 63) / 64);
    if (lineprod) {  // group line products, one chain per group (k_line_prod, k_batch_fchaing)
      // in parts of the 68 steps: the side stream (its K4 / VK work long done by then) runs the
      // chains over part k while the main stream forms part k + 1, so the chains' latency hides
      // behind the line products except for the last part
      const int m = (int)(ctx->npad / gsize);
      int bounds[ZG_LP_PARTS_MAX + 1];
      const int parts = lineprod_parts(ctx->lp_parts, m, ctx->ncu, bounds);
      if (parts <= 1) {
        HIPCHK(launch_prog_lineprod(ctx->stream, b, (const Fq2*)ctx->d_lines, ctx->d_lprod, gsize, 0, ZG_NCOEFF,
                                          ctx->quad_split, affine));
        HIPCHK(launch_prog_fchaing(ctx->stream, b, (const Fq2*)ctx->d_lprod, ctx->d_fstate, m, 0, ZG_NCOEFF));
      } else {
        for (int k = 0; k < parts; k++) {
          const int n0 = bounds[k], n1 = bounds[k + 1];
          HIPCHK(launch_prog_lineprod(ctx->stream, b, (const Fq2*)ctx->d_lines, ctx->d_lprod, gsize, n0, n1,
                                            ctx->quad_split, affine));
          HIPCHK(hipEventRecord(ctx->ev[14 + k], ctx->stream));
          HIPCHK(hipStreamWaitEvent(ctx->side, ctx->ev[14 + k], 0));
          HIPCHK(launch_prog_fchaing(ctx->side, b, (const Fq2*)ctx->d_lprod, ctx->d_fstate, m, n0, n1));
        }
        HIPCHK(hipEventRecord(ctx->ev[14 + ZG_LP_PARTS_MAX], ctx->side));
        HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev[14 + ZG_LP_PARTS_MAX], 0));
        if (late && (rc = side_pairs(ctx->side))) return rc;  // beside the product tree on the main stream
      }
    } else if (quads) {
      HIPCHK(launch_prog_fchain4(qgroups, ctx->stream, b, (const Fq2*)ctx->d_lines, ctx->quad_split));
    } else {
      HIPCHK(launch_prog_fchain(pgroups, ctx->stream, b, (const Fq2*)ctx->d_lines, (const int*)nullptr));
    }
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ctx->ev[2], ctx->stream));
  HIPCHK(launch_f_tree(ctx, b, lineprod ? ctx->npad / gsize : ctx->npad / (singles ? 1 : quads ? 4 : 2)));
  HIPCHK(hipEventRecord(ctx->ev[3], ctx->stream));
  if (ctx->serial_side) {
    if ((rc = side_k4(ctx->stream)) || (rc = side_pairs(ctx->stream))) return rc;
  } else {
    HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev[6], 0));  // side-stream K4 + root pairs complete
  }
  // a B_i that failed its subgroup check in the R-chain (invalid proofs only) was still in the side
  // stream's root sums: settle_batch recomputes them when the flags say so
  ctx->root_pairs_ready = 1;
  // the root's Miller partial, the pipeline flags and the statuses go to pinned host memory as the
  // last steps (ev[4]), so zg_batch_partial / zg_batch_finish find them ready: computed only when
  // the host asked, the partial serialised the host loop of batches in flight behind a wave that
  // waited for a whole free SIMD
  hipLaunchKernelGGL(k_node_partial, dim3(1), dim3(64), 0, ctx->stream, b, nb);
  hipLaunchKernelGGL(k_f12_to_bytes, dim3(1), dim3(ZG_BLOCK), 0, ctx->stream, ctx->d_out, 1, ctx->d_bytes);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(ctx->h_pin, ctx->d_bytes, 576, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipMemcpyAsync(ctx->h_pin + ZG_PIN_FLAGS, ctx->d_int + 8, 2 * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipMemcpyAsync(ctx->h_pin + ZG_PIN_ENTRIES, ctx->msm.start + msm_shape(ctx->npad).ncount(), sizeof(int),
                        hipMemcpyDeviceToHost, ctx->stream));
  if (ctx->n)
    HIPCHK(hipMemcpyAsync(ctx->h_pin + ZG_PIN_STATUS, ctx->d_status, ctx->n, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipEventRecord(ctx->ev[4], ctx->stream));
  ctx->eager = 1;
  return ZG_OK;
}

static int check_kinds(zg_ctx* ctx, size_t n, const uint8_t* kinds) {
  for (size_t i = 0; i < n; i++) {
    if (kinds[i] >= ZG_NKINDS) return fail(ctx, ZG_E_INVAL, "bad kind at " + std::to_string(i));
    if (!ctx->vk_loaded[kinds[i]]) return fail(ctx, ZG_E_NOVK, "verifying key not loaded for proof " + std::to_string(i));
  }
  return ZG_OK;
}

// ctx->state 0 <-> 1 transitions keep the device's in-flight count (the auto fusion policy)
static void set_state(zg_ctx* ctx, int st) {
  if (ctx->state == st) return;
  if (ctx->dev) ctx->dev->inflight.fetch_add(st ? 1 : -1, std::memory_order_relaxed);
  ctx->state = st;
}

static int begin_common(zg_ctx* ctx, size_t n) {
  if (ctx->state != 0) return fail(ctx, ZG_E_STATE, "zg_batch_begin with a batch in flight (finish it first)");
  if (n > ctx->cap) return fail(ctx, ZG_E_NOMEM, "batch larger than max_batch");
  ctx->root_pairs_ready = 0;
  ctx->n = n;
  size_t npad = 2;  // at least one proof pair (the f-chain's unit)
  while (npad < n) npad <<= 1;
  ctx->npad = npad;
  ctx->calls++;
  return ZG_OK;
}

// the *_locked helpers assume ctx->mu is held: zg_verify_batch holds it from begin to finish,
// so no other thread can begin a batch on the same context in between
static int batch_begin_locked(zg_ctx* ctx, size_t n, const uint8_t* proofs, const uint8_t* kinds,
                              const uint8_t* inputs, const uint8_t* n_inputs, const uint8_t* r) {
  HIPCHK(hipSetDevice(ctx->device));
  int rc = begin_common(ctx, n);
  if (rc) return rc;
  if ((rc = check_kinds(ctx, n, kinds))) return rc;
  if (n) {
    HIPCHK(hipMemcpyAsync(ctx->d_proofs, proofs, n * 192, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(ctx->d_kinds, kinds, n, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(ctx->d_inputs, inputs, n * 288, hipMemcpyHostToDevice, ctx->stream));
    if (r)
      HIPCHK(hipMemcpyAsync(ctx->d_r, r, n * 16, hipMemcpyHostToDevice, ctx->stream));
    else if ((rc = stage_scalars(ctx, n)))
      return rc;
    if (n_inputs) HIPCHK(hipMemcpyAsync(ctx->d_ninputs, n_inputs, n, hipMemcpyHostToDevice, ctx->stream));
  }
  ctx->cur_ninputs = n_inputs ? ctx->d_ninputs : nullptr;
  ctx->cur_proofs = ctx->d_proofs;
  ctx->cur_kinds = ctx->d_kinds;
  ctx->cur_inputs = ctx->d_inputs;
  if ((rc = run_pipeline(ctx))) return rc;
  set_state(ctx, 1);
  return ZG_OK;
}

extern "C" int zg_batch_begin(zg_ctx* ctx, size_t n, const uint8_t* proofs, const uint8_t* kinds,
                              const uint8_t* inputs, const uint8_t* n_inputs, const uint8_t* r) {
  if (!ctx || (n && (!proofs || !kinds || !inputs))) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  return batch_begin_locked(ctx, n, proofs, kinds, inputs, n_inputs, r);
}

extern "C" int zg_batch_begin_device(zg_ctx* ctx, size_t n, const void* d_proofs, const void* d_kinds,
                                     const void* d_inputs, const void* d_n_inputs, const void* d_r) {
  if (!ctx || (n && (!d_proofs || !d_kinds || !d_inputs))) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  int rc = begin_common(ctx, n);
  if (rc) return rc;
  for (int k = 0; k < ZG_NKINDS; k++)
    if (!ctx->vk_loaded[k]) {
      // device-resident kinds are not inspected on the host: require every VK loaded
      return fail(ctx, ZG_E_NOVK, "device batches need all three verifying keys loaded");
    }
  // the inputs are read in place (the caller keeps them unchanged until zg_batch_finish): a
  // shard already resident in HBM is not copied again
  if (n) {
    if (d_r) {
      HIPCHK(hipMemcpyAsync(ctx->d_r, d_r, n * 16, hipMemcpyDeviceToDevice, ctx->stream));
    } else if ((rc = stage_scalars(ctx, n))) {
      return rc;
    }
  }
  ctx->cur_ninputs = (const uint8_t*)d_n_inputs;
  ctx->cur_proofs = (const uint8_t*)d_proofs;
  ctx->cur_kinds = (const uint8_t*)d_kinds;
  ctx->cur_inputs = (const uint8_t*)d_inputs;
  if ((rc = run_pipeline(ctx))) return rc;
  set_state(ctx, 1);
  return ZG_OK;
}

// check a list of tree nodes; mode per k_node_final. ok / out are host arrays (may be null).
// The per-proof Miller leaves (leaf f-chain from the stored line triples) run on the side stream
// while the main stream runs the nodes' VK-side MSM and Miller loops; the final exponentiations
// wait for both.
static int check_nodes(zg_ctx* ctx, const std::vector<int>& nodes, int mode, std::vector<int>* ok, uint8_t* out_bytes) {
  BatchBufs b = batch_bufs(ctx);
  if (ok) ok->assign(nodes.size(), 0);
  // the root's VK-side MSM + pairs were computed by the pipeline on the side stream
  const bool reuse_root = ctx->root_pairs_ready && nodes.size() == 1 && nodes[0] == 1;
  for (size_t off = 0; off < nodes.size(); off += ZG_NODE_CHUNK) {
    int m = (int)std::min((size_t)ZG_NODE_CHUNK, nodes.size() - off);
    // the pipeline's root pairs: its node list is implicit (null: the root)
    NodeBufs nb = {reuse_root ? nullptr : ctx->d_nodes, ctx->d_msm, ctx->d_pairf, ctx->d_ok, ctx->d_out, m};
    if (!reuse_root) {
      ctx->root_pairs_ready = 0;  // d_msm / d_pairf are about to be overwritten
      HIPCHK(hipMemcpyAsync(ctx->d_nodes, nodes.data() + off, sizeof(int) * m, hipMemcpyHostToDevice, ctx->stream));
      bool leaves = false;
      for (int q = 0; q < m; q++) leaves = leaves || nodes[off + q] >= (int)ctx->npad;
      if (leaves && !ctx->singles_last) {  // per-proof Miller leaves on demand (unless the f-chain wrote them)
        HIPCHK(hipEventRecord(ctx->ev[10], ctx->stream));
        HIPCHK(hipStreamWaitEvent(ctx->side, ctx->ev[10], 0));
        HIPCHK(launch_prog_leaf_fchain(nblocks(m), ctx->side, b, (const Fq2*)ctx->d_lines, (const int*)ctx->d_nodes, m));
        HIPCHK(hipEventRecord(ctx->ev[11], ctx->side));
      }
      hipLaunchKernelGGL(k_node_msm, dim3(nblocks((size_t)nb.m * ZG_NKINDS * ZG_MSM_SLOTS * ZG_SHIFTS)),
                         dim3(ZG_BLOCK), 0, ctx->stream, b, nb, (const int*)nullptr);
      HIPCHK(hipGetLastError());
      if (ctx->c_tree_pending) {  // the C tree (side stream) feeds the delta pairs
        HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev[12], 0));
        ctx->c_tree_pending = 0;
      }
      hipLaunchKernelGGL(k_node_pairs, dim3(nb.m * (b.merged ? ZG_NODE_PAIRS_MERGED : ZG_NODE_PAIRS)), dim3(64), 0,
                         ctx->stream, b, nb,
                         (const int*)nullptr);
      HIPCHK(hipGetLastError());
      if (leaves && !ctx->singles_last) HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev[11], 0));
    }
    hipLaunchKernelGGL(k_node_final, dim3(m), dim3(64), 0, ctx->stream, b, nb, mode);
    HIPCHK(hipGetLastError());
    if (ok) HIPCHK(hipMemcpyAsync(ok->data() + off, ctx->d_ok, sizeof(int) * m, hipMemcpyDeviceToHost, ctx->stream));
    if (out_bytes) {
      int rc = f12_download(ctx, ctx->d_out, m, out_bytes + (size_t)576 * off);
      if (rc) return rc;
    }
  }
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return ZG_OK;
}

// after the batch's device work: timings and the pipeline's flags (B subgroup failures, whose root
// sums settle_batch recomputed; a fused launch whose consumers timed out waiting, which turns
// the fused shape off for this context). The timings are the pipeline's own (ev[0..10]): the
// settle recompute waits on an event of its own and is not in them.
static int collect_batch_stats(zg_ctx* ctx) {
  int flags[2] = {0, 0}, entries = 0;
  HIPCHK(wait_event(ctx->ev[4]));  // the pipeline's last step (run_pipeline)
  memcpy(flags, ctx->h_pin + ZG_PIN_FLAGS, sizeof(flags));
  memcpy(&entries, ctx->h_pin + ZG_PIN_ENTRIES, sizeof(int));
  ctx->stats[0]++;
  if (ctx->fused_last) ctx->stats[1]++;
  if (ctx->quads_last) ctx->stats[7]++;
  if (ctx->lineprod_last) ctx->stats[11]++;
  if (ctx->affine_last) ctx->stats[12]++;
  if (flags[1]) {
    ctx->stats[2]++;
    ctx->fuse_off = 1;
  }
  if (flags[0]) ctx->stats[3]++;
  ctx->stats[6] = ctx->k4_last ? (uint64_t)entries : 0;
  if (!ctx->k4_last) ctx->stats[10]++;
  hipEventElapsedTime(&ctx->timings[0], ctx->ev[0], ctx->ev[1]);  // decode
  hipEventElapsedTime(&ctx->timings[1], ctx->ev[1], ctx->ev[7]);  // lines (R-chain)
  hipEventElapsedTime(&ctx->timings[2], ctx->ev[7], ctx->ev[2]);  // f-chain
  hipEventElapsedTime(&ctx->timings[3], ctx->ev[2], ctx->ev[3]);  // Fq12 product tree
  hipEventElapsedTime(&ctx->timings[4], ctx->ev[3], ctx->ev[4]);  // root partial: waits for the side stream
                                                                  // (serial_side: runs it)
  hipEventElapsedTime(&ctx->timings[5], ctx->ev[5], ctx->ev[6]);  // side stream: trees + VK-side root work
  hipEventElapsedTime(&ctx->timings[6], ctx->ev[0], ctx->ev[4]);  // whole device pipeline
  hipEventElapsedTime(&ctx->timings[7], ctx->ev[5], ctx->ev[10]);  // K4 (Pippenger + root Fr sums)
  hipEventElapsedTime(&ctx->timings[8], ctx->ev[8], ctx->ev[9]);   // K4 bucket phase (k_msm_bucket)
  return ZG_OK;
}

// After the pipeline's last step: if a B_i failed its G2 subgroup check in the R-chain (flags[0],
// invalid proofs only), the side stream's root work -- K4 / the C tree, the root's VK-side MSM and
// pairs -- ran with that proof still in; recompute it without (its leaves were cleared by the R-chain
// kernel), then the root partial. A valid batch pays nothing here: round 4 queued this recompute as
// ~12 gated no-op launches at the end of every batch's main stream.
static int settle_batch(zg_ctx* ctx) {
  HIPCHK(wait_event(ctx->ev[4]));
  if (ctx->settled) return ZG_OK;
  ctx->settled = 1;
  int flags[2] = {0, 0};
  memcpy(flags, ctx->h_pin + ZG_PIN_FLAGS, sizeof(flags));
  if (!flags[0]) return ZG_OK;
  BatchBufs b = batch_bufs(ctx);
  NodeBufs nb = {nullptr, ctx->d_msm, ctx->d_pairf, ctx->d_ok, ctx->d_out, 1};
  HIPCHK(launch_msm_root(ctx->stream, b, ctx->msm, nullptr, nullptr, nullptr, ctx->k4_last, ctx->alone_last));
  if (!ctx->k4_last) HIPCHK(launch_c_tree(ctx, b, ctx->stream, nullptr));
  int rc = launch_node_msm_pairs(ctx, b, nb, ctx->stream);
  if (rc) return rc;
  hipLaunchKernelGGL(k_node_partial, dim3(1), dim3(64), 0, ctx->stream, b, nb);
  hipLaunchKernelGGL(k_f12_to_bytes, dim3(1), dim3(ZG_BLOCK), 0, ctx->stream, ctx->d_out, 1, ctx->d_bytes);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(ctx->h_pin, ctx->d_bytes, 576, hipMemcpyDeviceToHost, ctx->stream));
  // its own event: ev[4] stays the pipeline's end (collect_batch_stats' timings)
  HIPCHK(hipEventRecord(ctx->ev[ZG_EV_SETTLE], ctx->stream));
  HIPCHK(wait_event(ctx->ev[ZG_EV_SETTLE]));
  return ZG_OK;
}

extern "C" int zg_batch_partial(zg_ctx* ctx, uint8_t partial[576]) {
  if (!ctx || !partial) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (ctx->state != 1) return fail(ctx, ZG_E_STATE, "zg_batch_partial before zg_batch_begin");
  HIPCHK(hipSetDevice(ctx->device));
  if (!ctx->eager) return fail(ctx, ZG_E_STATE, "zg_batch_partial: no pipeline result");
  int rc = settle_batch(ctx);
  if (rc) return rc;
  memcpy(partial, ctx->h_pin, 576);
  return collect_batch_stats(ctx);
}

extern "C" int zg_batch_ready(zg_ctx* ctx) {
  if (!ctx) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (ctx->state != 1 || !ctx->eager) return fail(ctx, ZG_E_STATE, "zg_batch_ready before zg_batch_begin");
  HIPCHK(hipSetDevice(ctx->device));
  const hipError_t e = hipEventQuery(ctx->ev[4]);
  if (e == hipErrorNotReady) return 0;
  HIPCHK(e);
  return 1;
}

extern "C" int zg_gt_check_many(zg_ctx* ctx, size_t nsets, const size_t* counts, const uint8_t* partials,
                                int* ok) {
  if (!ctx || !counts || !partials || !ok || nsets == 0 || nsets > ZG_GT_SETS_MAX) return ZG_E_INVAL;
  GtSets sets;
  size_t count = 0;
  sets.off[0] = 0;
  for (size_t b = 0; b < nsets; b++) {
    if (counts[b] == 0 || counts[b] > ZG_NODE_CHUNK) return ZG_E_INVAL;
    count += counts[b];
    if (count > ZG_NODE_CHUNK) return ZG_E_INVAL;
    sets.off[b + 1] = (int)count;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  // pinned staging (asynchronous copies), then a polling wait (wait_event)
  const size_t need = 576 * count + sizeof(int) * ZG_GT_SETS_MAX;
  if (ctx->h_gt_cap < need) {
    if (ctx->h_gt) HIPCHK(hipHostFree(ctx->h_gt));
    ctx->h_gt = nullptr;
    ctx->h_gt_cap = 0;
    HIPCHK(hipHostMalloc((void**)&ctx->h_gt, need, hipHostMallocDefault));
    ctx->h_gt_cap = need;
  }
  memcpy(ctx->h_gt, partials, 576 * count);
  HIPCHK(hipMemcpyAsync(ctx->d_bytes, ctx->h_gt, 576 * count, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(k_f12_from_bytes, dim3(nblocks(count)), dim3(ZG_BLOCK), 0, ctx->stream, ctx->d_bytes, (int)count,
                     ctx->d_pairf);
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(k_partials_check, dim3((unsigned)nsets), dim3(64), 0, ctx->stream, ctx->d_pairf, sets, ctx->d_ok,
                     ctx->d_out);
  HIPCHK(hipGetLastError());
  int* hok = (int*)(ctx->h_gt + 576 * count);
  HIPCHK(hipMemcpyAsync(hok, ctx->d_ok, sizeof(int) * nsets, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipEventRecord(ctx->ev[13], ctx->stream));
  HIPCHK(wait_event(ctx->ev[13]));
  for (size_t b = 0; b < nsets; b++) ok[b] = hok[b];
  return ZG_OK;
}

extern "C" int zg_gt_check(zg_ctx* ctx, size_t count, const uint8_t* partials, int* ok) {
  if (!ctx || !partials || !ok || count == 0 || count > ZG_NODE_CHUNK) return ZG_E_INVAL;
  return zg_gt_check_many(ctx, 1, &count, partials, ok);
}

// Moves the context to the device's high-priority stream pair (created once per device) or
// back to its pool pair. No stream is created or destroyed per context.
extern "C" int zg_set_priority(zg_ctx* ctx, int high) {
  if (!ctx) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (ctx->state != 0) return fail(ctx, ZG_E_STATE, "zg_set_priority with a batch in flight");
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->side));
  zg_dev* d = ctx->dev;
  if (high) {
    std::lock_guard<std::mutex> gd(d->mu);
    const int k = d->hi_next++ % ZG_HI_PAIRS;
    if (!d->hi_main[k]) {
      int lo = 0, hi = 0;
      HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));  // numerically lower = higher priority
      HIPCHK(hipStreamCreateWithPriority(&d->hi_main[k], hipStreamNonBlocking, hi));
      HIPCHK(hipStreamCreateWithPriority(&d->hi_side[k], hipStreamNonBlocking, hi));
    }
    ctx->stream = d->hi_main[k];
    ctx->side = d->hi_side[k];
  } else {
    ctx->stream = d->main[ctx->pair];
    ctx->side = d->side[ctx->pair];
  }
  return ZG_OK;
}

// Bisection over the product trees: a failing node's children are re-checked exactly;
// a failing leaf is a proof whose own check fails (r_i != 0 makes it bellman's check).
// bisection needs every node's C and Fr sums: the per-proof r_i C_i (GLV) leaves and the full
// trees, built only now (a valid batch never needs them: K4 forms the root directly). The Fr
// tree (cheap; all the node MSM needs) is built on the main stream, the C leaves and tree on
// the side stream, joined before the first delta pairs (ev[12]).
static int build_trees(zg_ctx* ctx) {
  if (ctx->trees_built) return ZG_OK;
  BatchBufs b = batch_bufs(ctx);
  // group line products: the tree exists from the groups up only; the quad f-chain on the lines
  // (still in HBM) and the levels above write every node (those from the groups up again, with
  // the same values)
  if (ctx->lineprod_last) {
    // affine lines: the chains below the groups read projective triples -- re-form them (the lane
    // R-chain; its G2 checks repeat the affine chain's verdicts, every B already settled)
    if (ctx->affine_last) HIPCHK(launch_lines_lane((unsigned)((ctx->npad + 63) / 64), ctx->stream, b, ctx->d_lines, 2));
    HIPCHK(launch_prog_fchain4((unsigned)((ctx->npad / 4 + 63) / 64), ctx->stream, b, (const Fq2*)ctx->d_lines,
                               ctx->quad_split));
    HIPCHK(launch_f_tree(ctx, b, ctx->npad / 4));
  }
  HIPCHK(hipEventRecord(ctx->ev[10], ctx->stream));
  HIPCHK(hipStreamWaitEvent(ctx->side, ctx->ev[10], 0));
  // small shards (k4_last = 0): the pipeline already built the whole C tree from the GLV leaves
  if (ctx->k4_last) HIPCHK(launch_c_leaves(ctx->side, b));
  for (size_t lo = ctx->npad / 2; lo >= 1; lo /= 2) {
    if (ctx->k4_last) {
      hipLaunchKernelGGL(k_tree_c, dim3(nblocks(lo * ZG_NKINDS)), dim3(ZG_BLOCK), 0, ctx->side, b, (int)lo,
                         (const int*)nullptr);
      HIPCHK(hipGetLastError());
    }
    hipLaunchKernelGGL(k_tree_s, dim3(nblocks(lo)), dim3(ZG_BLOCK), 0, ctx->stream, b, (int)lo);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipEventRecord(ctx->ev[12], ctx->side));
  ctx->c_tree_pending = 1;
  ctx->trees_built = 1;
  return ZG_OK;
}

// Each round checks, in one launch group, the descendants of every failing node k levels down,
// k as large as keeps the round within ZG_BISECT_BUDGET nodes (at least one level): a round
// costs about the same for 16 or 512 nodes (single-wave Miller loops and final
// exponentiations, latency-bound), so few failing nodes descend many levels at once. E.g.
// 4,096 proofs with 27 failing: 512 nodes of 8, then 216 leaves.
#define ZG_BISECT_BUDGET 512
static size_t bisect_budget() {  // ZG_BISECT_BUDGET=<nodes> overrides (tuning)
  static const long v = getenv("ZG_BISECT_BUDGET") ? atol(getenv("ZG_BISECT_BUDGET")) : 0;
  return v >= 16 ? (size_t)v : (size_t)ZG_BISECT_BUDGET;
}
static int bisect(zg_ctx* ctx, std::vector<uint8_t>& st, bool root_failed) {
  const int npad = (int)ctx->npad, n = (int)ctx->n;
  int depth_leaf = 0;
  while ((1 << depth_leaf) < npad) depth_leaf++;
  ctx->stats[4]++;
  int rc0 = build_trees(ctx);
  if (rc0) return rc0;
  std::vector<int> fails;  // failing nodes of the last round, all at the same depth
  if (root_failed) {
    fails.push_back(1);
  } else {
    std::vector<int> ok;
    ctx->stats[5] += 1;
    int rc = check_nodes(ctx, std::vector<int>{1}, 0, &ok, nullptr);
    if (rc) return rc;
    if (!ok[0]) fails.push_back(1);
  }
  int d = 0;  // depth of the failing nodes
  while (!fails.empty() && d < depth_leaf) {
    int k = 1;
    const size_t budget = bisect_budget();
    while (k < depth_leaf - d && fails.size() * (size_t)(2 << k) <= budget) k++;
    // four proofs per lane wrote no pair-level nodes: go from the quad level (or above) straight
    // to the leaves, or stop one level higher
    if (ctx->quads_last && d + k == depth_leaf - 1) {
      if (k > 1 && fails.size() * (size_t)(2 << (k + 1)) > budget)
        k--;
      else
        k++;
    }
    std::vector<int> level;
    for (int node : fails)  // descendants that start at or beyond n hold only padding: skipped
      for (int c = node << k; c < (node + 1) << k; c++)
        if (((long long)c << (depth_leaf - d - k)) - npad < n) level.push_back(c);
    std::vector<int> ok;
    ctx->stats[5] += level.size();
    int rc = check_nodes(ctx, level, 0, &ok, nullptr);
    if (rc) return rc;
    fails.clear();
    for (size_t q = 0; q < level.size(); q++)
      if (!ok[q]) fails.push_back(level[q]);
    d += k;
  }
  for (int node : fails) {  // failing leaves: proofs whose own check fails
    const int i = node - npad;
    if (i >= 0 && i < n && st[i] == ST_PENDING) st[i] = ST_VERIFY_FAILED;
  }
  return ZG_OK;
}

static int batch_finish_locked(zg_ctx* ctx, int batch_ok, uint8_t* status, bool root_failed = false) {
  if (ctx->state != 1) return fail(ctx, ZG_E_STATE, "zg_batch_finish before zg_batch_begin");
  HIPCHK(hipSetDevice(ctx->device));
  std::vector<uint8_t> st(ctx->n);
  if (ctx->eager) {
    int rc = settle_batch(ctx);
    if (rc) return rc;
  }
  if (ctx->eager && batch_ok) {  // the pipeline's own status copy (run_pipeline, ev[4])
    if (ctx->n) memcpy(st.data(), ctx->h_pin + ZG_PIN_STATUS, ctx->n);
  } else {
    if (ctx->n) HIPCHK(hipMemcpyAsync(st.data(), ctx->d_status, ctx->n, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
  }
  if (!batch_ok) {
    int rc = bisect(ctx, st, root_failed);
    if (rc) {
      set_state(ctx, 0);  // the batch is abandoned; the context stays usable
      return rc;
    }
  }
  for (size_t i = 0; i < ctx->n; i++) status[i] = st[i] == ST_PENDING ? ST_OK : st[i];
  if (ctx->debug_each && ctx->n) {
    // debug cross-check: bellman's per-proof verify_proof (k_verify_single, one pairing check per
    // proof, no batch scalars) on the batch's own device inputs must give the same statuses
    const size_t n = ctx->n;
    hipLaunchKernelGGL(k_verify_single, dim3(nblocks(n)), dim3(ZG_BLOCK), 0, ctx->stream, ctx->d_vk, (int)n,
                       ctx->cur_proofs, ctx->cur_kinds, ctx->cur_inputs, ctx->cur_ninputs, ctx->d_dbg, nullptr);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(st.data(), ctx->d_dbg, n, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    for (size_t i = 0; i < n; i++)
      if (st[i] != status[i]) {
        set_state(ctx, 0);
        return fail(ctx, ZG_E_DEBUG, "ZG_DEBUG_EACH: proof " + std::to_string(i) + ": batch status " +
                                         std::to_string(status[i]) + ", per-proof verify_proof status " +
                                         std::to_string(st[i]));
      }
  }
  set_state(ctx, 0);
  return ZG_OK;
}

extern "C" int zg_batch_finish(zg_ctx* ctx, int batch_ok, uint8_t* status) {
  if (!ctx || (!status && ctx->n)) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  return batch_finish_locked(ctx, batch_ok, status);
}

extern "C" int zg_verify_batch(zg_ctx* ctx, size_t n, const uint8_t* proofs, const uint8_t* kinds,
                               const uint8_t* inputs, const uint8_t* n_inputs, const uint8_t* r, uint8_t* status,
                               uint8_t* gt_out) {
  if (!ctx || !status || (n && (!proofs || !kinds || !inputs))) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = batch_begin_locked(ctx, n, proofs, kinds, inputs, n_inputs, r);
  if (rc) return rc;
  if ((rc = settle_batch(ctx))) {
    set_state(ctx, 0);
    return rc;
  }
  std::vector<int> root = {1}, okv;
  if (gt_out) rc = check_nodes(ctx, root, 2, nullptr, gt_out);
  if (!rc) rc = check_nodes(ctx, root, 0, &okv, nullptr);
  if (!rc) rc = collect_batch_stats(ctx);
  if (rc) {
    set_state(ctx, 0);
    return rc;
  }
  return batch_finish_locked(ctx, okv[0], status, /*root_failed=*/okv[0] == 0);
}

extern "C" int zg_last_timings(zg_ctx* ctx, float* ms7) { return zg_last_phase_ms(ctx, ms7, 7); }

extern "C" int zg_last_phase_ms(zg_ctx* ctx, float* ms, size_t n) {
  if (!ctx || (n && !ms)) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  for (size_t i = 0; i < n; i++) ms[i] = i < ZG_NTIMINGS ? ctx->timings[i] : 0.0f;
  return ZG_OK;
}

extern "C" int zg_stats(zg_ctx* ctx, uint64_t* out, size_t n) {
  if (!ctx || (n && !out)) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  for (size_t i = 0; i < n; i++) out[i] = i < ZG_NSTATS ? ctx->stats[i] : 0;
  return ZG_OK;
}

// ------------------------------------------------------------------ Sapling signatures (zg_jubjub.h)
#define ZG_JJ_COMB_BYTES (sizeof(uint32_t) * 16 * (size_t)(3 * 32 * 255))
static int jj_comb(zg_ctx* ctx, const uint32_t** out) {
  zg_dev* d = ctx->dev;
  std::lock_guard<std::mutex> g(d->mu);
  if (!d->jj_comb) {
    uint32_t* t = nullptr;
    HIPCHK(hipMalloc(&t, ZG_JJ_COMB_BYTES));
    hipError_t e = launch_jj_comb(ctx->stream, t);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
      hipFree(t);
      return fail(ctx, ZG_E_HIP, std::string("Jubjub comb tables: ") + hipGetErrorString(e));
    }
    d->jj_comb = t;
  }
  *out = d->jj_comb;
  return ZG_OK;
}

// device buffers of one call, freed on every path
struct DevScratch {
  std::vector<void*> p;
  ~DevScratch() {
    for (void* q : p) hipFree(q);
  }
  template <class T>
  hipError_t alloc(T** x, size_t bytes) {
    hipError_t e = hipMalloc((void**)x, bytes ? bytes : 1);
    if (e == hipSuccess) p.push_back(*x);
    return e;
  }
};

extern "C" int zg_redjubjub_verify(zg_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                                   const uint8_t* gen, uint8_t* ok) {
  if (!ctx || (n && (!vk || !sig || !msg || !gen || !ok)) || n > (1u << 30)) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (!n) return ZG_OK;
  HIPCHK(hipSetDevice(ctx->device));
  const uint32_t* comb = nullptr;
  int rc = jj_comb(ctx, &comb);
  if (rc) return rc;
  DevScratch s;
  uint8_t *dvk, *dsig, *dmsg, *dgen, *dok;
  HIPCHK(s.alloc(&dvk, 32 * n));
  HIPCHK(s.alloc(&dsig, 64 * n));
  HIPCHK(s.alloc(&dmsg, 64 * n));
  HIPCHK(s.alloc(&dgen, n));
  HIPCHK(s.alloc(&dok, n));
  HIPCHK(hipMemcpyAsync(dvk, vk, 32 * n, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipMemcpyAsync(dsig, sig, 64 * n, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipMemcpyAsync(dmsg, msg, 64 * n, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipMemcpyAsync(dgen, gen, n, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(launch_redjubjub(ctx->stream, dvk, dsig, dmsg, dgen, (int)n, comb, dok));
  HIPCHK(hipMemcpyAsync(ok, dok, n, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return ZG_OK;
}

extern "C" int zg_sapling_bvk(zg_ctx* ctx, size_t ntx, const uint32_t* n_spends, const uint32_t* n_outputs,
                              const uint8_t* cvs, const int64_t* value_balance, uint8_t* bvk, uint8_t* status) {
  if (!ctx || (ntx && (!n_spends || !n_outputs || !value_balance || !bvk || !status)) || ntx > (1u << 30))
    return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (!ntx) return ZG_OK;
  std::vector<uint32_t> off(ntx + 1, 0);
  for (size_t t = 0; t < ntx; t++) {
    const uint64_t next = (uint64_t)off[t] + n_spends[t] + n_outputs[t];
    if (next > (1u << 30)) return fail(ctx, ZG_E_INVAL, "too many value commitments");
    off[t + 1] = (uint32_t)next;
  }
  if (off[ntx] && !cvs) return ZG_E_INVAL;
  HIPCHK(hipSetDevice(ctx->device));
  const uint32_t* comb = nullptr;
  int rc = jj_comb(ctx, &comb);
  if (rc) return rc;
  DevScratch s;
  uint32_t *doff, *dns;
  uint8_t *dcv, *dbvk, *dst;
  int64_t* dvb;
  HIPCHK(s.alloc(&doff, sizeof(uint32_t) * (ntx + 1)));
  HIPCHK(s.alloc(&dns, sizeof(uint32_t) * ntx));
  HIPCHK(s.alloc(&dcv, (size_t)32 * off[ntx]));
  HIPCHK(s.alloc(&dvb, sizeof(int64_t) * ntx));
  HIPCHK(s.alloc(&dbvk, 32 * ntx));
  HIPCHK(s.alloc(&dst, ntx));
  HIPCHK(hipMemcpyAsync(doff, off.data(), sizeof(uint32_t) * (ntx + 1), hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipMemcpyAsync(dns, n_spends, sizeof(uint32_t) * ntx, hipMemcpyHostToDevice, ctx->stream));
  if (off[ntx]) HIPCHK(hipMemcpyAsync(dcv, cvs, (size_t)32 * off[ntx], hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipMemcpyAsync(dvb, value_balance, sizeof(int64_t) * ntx, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(launch_sapling_bvk(ctx->stream, (int)ntx, doff, dns, dcv, dvb, comb, dbvk, dst));
  HIPCHK(hipMemcpyAsync(bvk, dbvk, 32 * ntx, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipMemcpyAsync(status, dst, ntx, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return ZG_OK;
}

extern "C" int zg_jubjub_decode(zg_ctx* ctx, size_t n, const uint8_t* points, uint8_t* status, uint8_t* xy) {
  if (!ctx || (n && (!points || !status)) || n > (1u << 30)) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (!n) return ZG_OK;
  HIPCHK(hipSetDevice(ctx->device));
  DevScratch s;
  uint8_t *dp, *dst, *dxy = nullptr;
  HIPCHK(s.alloc(&dp, 32 * n));
  HIPCHK(s.alloc(&dst, n));
  if (xy) HIPCHK(s.alloc(&dxy, 64 * n));
  HIPCHK(hipMemcpyAsync(dp, points, 32 * n, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(launch_jj_decode(ctx->stream, dp, (int)n, dst, dxy));
  HIPCHK(hipMemcpyAsync(status, dst, n, hipMemcpyDeviceToHost, ctx->stream));
  if (xy) HIPCHK(hipMemcpyAsync(xy, dxy, 64 * n, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return ZG_OK;
}

// ------------------------------------------------------------------ host input preparation
// (zg_prep.h). CPU only: no context, no GPU.
extern "C" int zg_prep_spend(const uint8_t cv[32], const uint8_t anchor[32], const uint8_t nullifier[32],
                             const uint8_t rk[32], uint8_t inputs[7 * 32]) {
  if (!cv || !anchor || !nullifier || !rk || !inputs) return ZG_E_INVAL;
  return prep_spend(cv, anchor, nullifier, rk, inputs);
}

extern "C" int zg_prep_output(const uint8_t cv[32], const uint8_t cmu[32], const uint8_t epk[32],
                              uint8_t inputs[5 * 32]) {
  if (!cv || !cmu || !epk || !inputs) return ZG_E_INVAL;
  return prep_output(cv, cmu, epk, inputs);
}

// A window's preparation in one call: the Sapling descriptions on the GPU (k_prep_sapling, zg_jubjub.hip),
// the JoinSplits on host threads while it runs (BLAKE2b is host code; ~17 us each), then their rows
// over the kernel's. Per description the same results as the single functions above (tests/
// test_gpu_prep_batch.py): a window of 9,609 descriptions took ~380 ms through per-description host
// calls from a Python thread pool (its per-task overhead under the GIL, not the C, was the bound).
extern "C" int zg_prep_batch(zg_ctx* ctx, size_t n, const uint8_t* kinds, const uint8_t* fields, uint8_t* inputs,
                             uint8_t* codes) {
  if (!ctx || (n && (!kinds || !fields || !inputs || !codes)) || n > (1u << 26)) return ZG_E_INVAL;
  std::vector<size_t> js;
  size_t nsap = 0;
  for (size_t i = 0; i < n; i++) {
    if (kinds[i] > ZG_PREP_KIND_JOINSPLIT_BN) return ZG_E_INVAL;
    if (kinds[i] <= ZG_PREP_KIND_OUTPUT)
      nsap++;
    else
      js.push_back(i);
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  if (!n) return ZG_OK;
  HIPCHK(hipSetDevice(ctx->device));
  if (nsap) {  // one grow-only device buffer: kinds | fields | rows | codes
    const size_t need = n * (2 + ZG_PREP_FIELD_BYTES + 288) + 64;
    if (ctx->prep_arena_cap < need) {
      if (ctx->prep_arena) HIPCHK(hipFree(ctx->prep_arena));
      ctx->prep_arena = nullptr;
      ctx->prep_arena_cap = 0;
      HIPCHK(hipMalloc((void**)&ctx->prep_arena, need));
      ctx->prep_arena_cap = need;
    }
    uint8_t* const dk = ctx->prep_arena;
    uint8_t* const df = dk + n;
    uint8_t* const din = df + (size_t)ZG_PREP_FIELD_BYTES * n;
    uint8_t* const dc = din + (size_t)288 * n;
    HIPCHK(hipMemcpyAsync(dk, kinds, n, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(df, fields, (size_t)ZG_PREP_FIELD_BYTES * n, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(launch_prep_sapling(ctx->stream, dk, df, (int)n, din, dc));
    HIPCHK(hipMemcpyAsync(inputs, din, (size_t)288 * n, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpyAsync(codes, dc, n, hipMemcpyDeviceToHost, ctx->stream));
  }
  // the JoinSplits meanwhile, into their own rows (written over the copied-back buffer after the sync)
  std::vector<uint8_t> jrows(js.size() * 288, 0);
  auto work = [&](size_t lo, size_t hi) {
    for (size_t k = lo; k < hi; k++) {
      const uint8_t* f = fields + (size_t)ZG_PREP_FIELD_BYTES * js[k];
      uint64_t vo = 0, vn = 0;
      for (int b = 7; b >= 0; b--) {
        vo = (vo << 8) | f[288 + b];
        vn = (vn << 8) | f[296 + b];
      }
      prep_joinsplit_bits(f, f + 32, f + 64, f + 96, f + 128, f + 160, f + 192, f + 224, vo, vn, f + 256,
                          kinds[js[k]] == ZG_PREP_KIND_JOINSPLIT ? 254 : 253, &jrows[288 * k]);
    }
  };
  const size_t nt = std::min<size_t>({16, std::max(1u, std::thread::hardware_concurrency()), js.size() / 64 + 1});
  std::vector<std::thread> th;
  for (size_t t = 1; t < nt; t++) th.emplace_back(work, js.size() * t / nt, js.size() * (t + 1) / nt);
  work(0, js.size() / nt);
  for (auto& t : th) t.join();
  if (nsap) {
    HIPCHK(hipEventRecord(ctx->ev[13], ctx->stream));
    HIPCHK(wait_event(ctx->ev[13]));
  }
  for (size_t k = 0; k < js.size(); k++) {
    memcpy(inputs + (size_t)288 * js[k], &jrows[288 * k], 288);
    codes[js[k]] = ZG_PREP_OK;
  }
  return ZG_OK;
}

extern "C" int zg_hsig(const uint8_t random_seed[32], const uint8_t nf0[32], const uint8_t nf1[32],
                       const uint8_t pubkey[32], uint8_t out[32]) {
  if (!random_seed || !nf0 || !nf1 || !pubkey || !out) return ZG_E_INVAL;
  prep_hsig(random_seed, nf0, nf1, pubkey, out);
  return ZG_OK;
}

extern "C" int zg_prep_joinsplit(const uint8_t anchor[32], const uint8_t random_seed[32],
                                 const uint8_t nullifiers[64], const uint8_t macs[64],
                                 const uint8_t commitments[64], uint64_t vpub_old, uint64_t vpub_new,
                                 const uint8_t pubkey[32], uint8_t inputs[9 * 32]) {
  if (!anchor || !random_seed || !nullifiers || !macs || !commitments || !pubkey || !inputs) return ZG_E_INVAL;
  prep_joinsplit(anchor, random_seed, nullifiers, nullifiers + 32, macs, macs + 32, commitments, commitments + 32,
                 vpub_old, vpub_new, pubkey, inputs);
  return ZG_OK;
}

extern "C" int zg_prep_joinsplit_bn(const uint8_t anchor[32], const uint8_t random_seed[32],
                                    const uint8_t nullifiers[64], const uint8_t macs[64],
                                    const uint8_t commitments[64], uint64_t vpub_old, uint64_t vpub_new,
                                    const uint8_t pubkey[32], uint8_t inputs[9 * 32]) {
  if (!anchor || !random_seed || !nullifiers || !macs || !commitments || !pubkey || !inputs) return ZG_E_INVAL;
  prep_joinsplit_bits(anchor, random_seed, nullifiers, nullifiers + 32, macs, macs + 32, commitments,
                      commitments + 32, vpub_old, vpub_new, pubkey, 253, inputs);
  return ZG_OK;
}

// ------------------------------------------------------------------ synthetic workload
static void reduce_mod_r(uint8_t* le32) {
  // value < 2^256 < 3r: subtract r while >= r
  for (int rep = 0; rep < 3; rep++) {
    uint32_t v[8];
    for (int w = 0; w < 8; w++)
      v[w] = (uint32_t)le32[4 * w] | ((uint32_t)le32[4 * w + 1] << 8) | ((uint32_t)le32[4 * w + 2] << 16) |
             ((uint32_t)le32[4 * w + 3] << 24);
    uint32_t d[8], borrow = 0;
    for (int w = 0; w < 8; w++) {
      uint64_t t = (uint64_t)v[w] - FR_R[w] - borrow;
      d[w] = (uint32_t)t;
      borrow = (uint32_t)(t >> 63);
    }
    if (borrow) return;
    for (int w = 0; w < 8; w++)
      for (int b = 0; b < 4; b++) le32[4 * w + b] = (uint8_t)(d[w] >> (8 * b));
  }
}

extern "C" int zg_synth_rerandomize(zg_ctx* ctx, size_t n_src, const uint8_t* src_proofs, const uint8_t* src_kinds,
                                    size_t n, const uint32_t* src_index, uint64_t seed, uint8_t* out_proofs) {
  if (!ctx || !src_proofs || !src_kinds || !src_index || !out_proofs || n_src == 0) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  for (size_t i = 0; i < n_src; i++)
    if (src_kinds[i] >= ZG_NKINDS || !ctx->vk_loaded[src_kinds[i]]) return fail(ctx, ZG_E_NOVK, "source kind VK");
  for (size_t i = 0; i < n; i++)
    if (src_index[i] >= n_src) return fail(ctx, ZG_E_INVAL, "src_index out of range");
  std::vector<uint32_t> ts(16 * n);
  for (size_t i = 0; i < n; i++) {
    Blake2b h(64);
    h.update("zg-rerand", 9);
    uint8_t le[8];
    for (int b = 0; b < 8; b++) le[b] = (uint8_t)(seed >> (8 * b));
    h.update(le, 8);
    for (int b = 0; b < 8; b++) le[b] = (uint8_t)((uint64_t)i >> (8 * b));
    h.update(le, 8);
    uint8_t dg[64];
    h.final(dg);
    for (int half = 0; half < 2; half++) {
      uint8_t* x = dg + 32 * half;
      reduce_mod_r(x);
      uint8_t acc = 0;
      for (int b = 0; b < 32; b++) acc |= x[b];
      if (!acc) x[0] = 1;
      for (int w = 0; w < 8; w++)
        ts[16 * i + 8 * half + w] = (uint32_t)x[4 * w] | ((uint32_t)x[4 * w + 1] << 8) |
                                    ((uint32_t)x[4 * w + 2] << 16) | ((uint32_t)x[4 * w + 3] << 24);
    }
  }
  uint8_t *d_src, *d_sk, *d_out;
  uint32_t *d_idx, *d_ts;
  HIPCHK(hipMalloc(&d_src, 192 * n_src));
  HIPCHK(hipMalloc(&d_sk, n_src));
  HIPCHK(hipMalloc(&d_out, 192 * (n ? n : 1)));
  HIPCHK(hipMalloc(&d_idx, 4 * (n ? n : 1)));
  HIPCHK(hipMalloc(&d_ts, 64 * (n ? n : 1)));
  int rc = ZG_OK;
  if (hipMemcpy(d_src, src_proofs, 192 * n_src, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(d_sk, src_kinds, n_src, hipMemcpyHostToDevice) != hipSuccess ||
      (n && hipMemcpy(d_idx, src_index, 4 * n, hipMemcpyHostToDevice) != hipSuccess) ||
      (n && hipMemcpy(d_ts, ts.data(), 64 * n, hipMemcpyHostToDevice) != hipSuccess)) {
    rc = fail(ctx, ZG_E_HIP, "copy");
  } else if (n) {
    hipLaunchKernelGGL(k_rerandomize, dim3(nblocks(n)), dim3(ZG_BLOCK), 0, ctx->stream, ctx->d_vk, d_src, d_sk, d_idx,
                       d_ts, (int)n, d_out);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(ctx->stream) != hipSuccess ||
        hipMemcpy(out_proofs, d_out, 192 * n, hipMemcpyDeviceToHost) != hipSuccess)
      rc = fail(ctx, ZG_E_HIP, "rerandomize kernel");
  }
  hipFree(d_src);
  hipFree(d_sk);
  hipFree(d_out);
  hipFree(d_idx);
  hipFree(d_ts);
  return rc;
}

extern "C" int zg_bench_mad_rate(zg_ctx* ctx, double* macs_per_s) { return zg_bench_mad_rate_clock(ctx, macs_per_s, nullptr); }

extern "C" int zg_bench_mad_rate_clock(zg_ctx* ctx, double* macs_per_s, double* clock_hz) {
  if (!ctx || !macs_per_s) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  const int blocks = 256 * 16, threads = 256, iters = 2048;
  uint64_t* d_st = nullptr;
  HIPCHK(hipMalloc(&d_st, sizeof(uint64_t) * 2 * blocks));
  hipLaunchKernelGGL(k_mad_rate, dim3(blocks), dim3(threads), 0, ctx->stream, (uint64_t*)ctx->d_int, 16, 1u,
                     (uint64_t*)nullptr);
  hipError_t e = hipStreamSynchronize(ctx->stream);
  if (e == hipSuccess) e = hipEventRecord(ctx->ev[0], ctx->stream);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_mad_rate, dim3(blocks), dim3(threads), 0, ctx->stream, (uint64_t*)ctx->d_int, iters, 1u,
                       d_st);
    e = hipEventRecord(ctx->ev[1], ctx->stream);
  }
  if (e == hipSuccess) e = hipEventSynchronize(ctx->ev[1]);
  float ms = 0;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[1]);
  std::vector<uint64_t> st(2 * blocks);
  if (e == hipSuccess) e = hipMemcpy(st.data(), d_st, sizeof(uint64_t) * 2 * blocks, hipMemcpyDeviceToHost);
  hipFree(d_st);
  if (e != hipSuccess) return fail(ctx, ZG_E_HIP, std::string("mad rate probe: ") + hipGetErrorString(e));
  *macs_per_s = (double)blocks * threads * iters * 64.0 / (ms * 1e-3);
  if (clock_hz) {  // median over blocks of shader ticks / (constant ticks / 100 MHz)
    std::vector<double> hz;
    for (int i = 0; i < blocks; i++)
      if (st[2 * i + 1]) hz.push_back((double)st[2 * i] / ((double)st[2 * i + 1] / 100e6));
    std::sort(hz.begin(), hz.end());
    *clock_hz = hz.empty() ? 0.0 : hz[hz.size() / 2];
  }
  return ZG_OK;
}

// ChaCha20 blocks on the device (the batch-scalar CSPRNG), for known-answer tests
extern "C" int zg_chacha20_blocks(zg_ctx* ctx, const uint8_t key[32], const uint8_t nonce[12], uint32_t counter,
                                  size_t nblocks, uint8_t* out) {
  if (!ctx || !key || !nonce || (nblocks && !out)) return ZG_E_INVAL;
  if (!nblocks) return ZG_OK;
  std::lock_guard<std::mutex> g(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  ChachaKey k;
  memcpy(k.key, key, 32);
  memcpy(k.nonce, nonce, 12);
  uint4* d = nullptr;
  HIPCHK(hipMalloc(&d, 64 * nblocks));
  hipLaunchKernelGGL(k_chacha20, dim3((unsigned)((nblocks + 255) / 256)), dim3(256), 0, ctx->stream, k, counter,
                     nblocks, d);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(out, d, 64 * nblocks, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  hipFree(d);
  if (e != hipSuccess) return fail(ctx, ZG_E_HIP, std::string("zg_chacha20_blocks: ") + hipGetErrorString(e));
  return ZG_OK;
}

// ------------------------------------------------------------------ note-commitment trees (zg_merkle.hip)
static zg::MerkleDev* merkle_dev(zg_ctx* ctx) {
  zg_dev* d = ctx->dev;
  std::lock_guard<std::mutex> g(d->mu);
  if (!d->merkle) d->merkle = merkle_dev_new();
  return d->merkle;
}

extern "C" int zg_merkle_combine(zg_ctx* ctx, int kind, size_t n, const uint8_t* left, const uint8_t* right,
                                 const uint8_t* depth, uint8_t* out) {
  if (!ctx || (kind != ZG_TREE_SPROUT && kind != ZG_TREE_SAPLING) || (n && (!left || !right || !out)) ||
      n > (1u << 30))
    return ZG_E_INVAL;
  if (kind == ZG_TREE_SAPLING && depth)
    for (size_t i = 0; i < n; i++)
      if (depth[i] >= 63) return fail(ctx, ZG_E_INVAL, "MerkleTree depth must be < 63");
  std::lock_guard<std::mutex> g(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  return merkle_combine(merkle_dev(ctx), ctx->stream, kind, n, left, right, depth, out, &ctx->err);
}

extern "C" int zg_tree_empty_roots(zg_ctx* ctx, int kind, size_t levels, uint8_t* out) {
  if (!ctx || (kind != ZG_TREE_SPROUT && kind != ZG_TREE_SAPLING) || levels > 64 || (levels && !out))
    return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  return merkle_empty_roots(merkle_dev(ctx), ctx->stream, kind, levels, out, &ctx->err);
}

extern "C" size_t zg_tree_state_max_bytes(int height) { return merkle_state_max_bytes(height); }

static int tree_roots(zg_ctx* ctx, int kind, int height, const uint8_t* state, size_t state_len, size_t n,
                      const void* leaves, int on_device, size_t n_marks, const uint64_t* marks, uint8_t* roots,
                      uint8_t* state_out, size_t* state_out_len, float* kernel_ms) {
  if (!ctx || (kind != ZG_TREE_SPROUT && kind != ZG_TREE_SAPLING) || height < 1 || height > 62 ||
      (n && !leaves) || (n_marks && (!marks || !roots)) || (state_len && !state) || n > (1ull << 40) ||
      n_marks > (1u << 30))
    return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  return merkle_tree_roots(merkle_dev(ctx), ctx->stream, kind, height, state, state_len, n, leaves, on_device,
                           n_marks, marks, roots, state_out, state_out_len, kernel_ms, &ctx->tree_arena,
                           &ctx->tree_arena_cap, &ctx->err);
}

extern "C" int zg_tree_roots(zg_ctx* ctx, int kind, int height, const uint8_t* state, size_t state_len,
                             size_t n_leaves, const uint8_t* leaves, size_t n_marks, const uint64_t* marks,
                             uint8_t* roots, uint8_t* state_out, size_t* state_out_len) {
  return tree_roots(ctx, kind, height, state, state_len, n_leaves, leaves, 0, n_marks, marks, roots, state_out,
                    state_out_len, nullptr);
}

extern "C" int zg_tree_roots_device(zg_ctx* ctx, int kind, int height, const uint8_t* state, size_t state_len,
                                    size_t n_leaves, const void* d_leaves, size_t n_marks, const uint64_t* marks,
                                    uint8_t* roots, uint8_t* state_out, size_t* state_out_len, float* kernel_ms) {
  return tree_roots(ctx, kind, height, state, state_len, n_leaves, d_leaves, 1, n_marks, marks, roots, state_out,
                    state_out_len, kernel_ms);
}

// ------------------------------------------------------------------ PGHR13 Sprout proofs (zg_pghr13.hip)
static zg::BnDev* bn_dev(zg_ctx* ctx) {
  zg_dev* d = ctx->dev;
  std::lock_guard<std::mutex> g(d->mu);
  if (!d->bn) d->bn = bn_dev_new();
  return d->bn;
}

// a key is parsed, prepared into fresh buffers and published in the device cache, then this
// context points at it (other contexts keep theirs); a failed load leaves the context's key as it was
static int pghr13_load_locked(zg_ctx* ctx, const char* json, size_t len) {
  HIPCHK(hipSetDevice(ctx->device));
  const zg::BnKey* k = nullptr;
  zg::BnDev* d = bn_dev(ctx);
  const int rc = bn_load_vk_json(d, ctx->stream, json, len, &k, &ctx->err);
  if (rc == ZG_OK) {
    if (ctx->bn_key) bn_key_release(d, ctx->bn_key);  // the old key goes once no context uses it
    ctx->bn_key = k;
  }
  return rc;
}

extern "C" int zg_pghr13_vk_load_json(zg_ctx* ctx, const char* json, size_t len) {
  if (!ctx || !json) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  return pghr13_load_locked(ctx, json, len);
}

extern "C" int zg_pghr13_vk_load_builtin(zg_ctx* ctx) {
  return zg_pghr13_vk_load_json(ctx, ZG_PGHR13_VK_JSON, strlen(ZG_PGHR13_VK_JSON));
}

#define ZG_PGHR_CHUNK ((size_t)65536)
extern "C" int zg_pghr13_verify(zg_ctx* ctx, size_t n, const uint8_t* proofs, const uint8_t* inputs,
                                const uint8_t* n_inputs, uint8_t* status, float* kernel_ms) {
  if (!ctx || (n && (!proofs || !inputs || !status)) || n > (1u << 24)) return ZG_E_INVAL;
  if (n_inputs)
    for (size_t i = 0; i < n; i++)
      if (n_inputs[i] > 9) return fail(ctx, ZG_E_INVAL, "at most 9 PGHR13 inputs per proof");
  std::lock_guard<std::mutex> g(ctx->mu);
  if (!ctx->bn_key) {  // first use: the builtin key (res/sprout-verifying-key.json)
    int rc = pghr13_load_locked(ctx, ZG_PGHR13_VK_JSON, strlen(ZG_PGHR13_VK_JSON));
    if (rc) return rc;
  }
  HIPCHK(hipSetDevice(ctx->device));
  if (!n) return ZG_OK;
  // the equality weights rho_2..rho_5 and rho_1 (16 bytes each, zg_pghr13.hip ZG_PGHR_RHO_BYTES):
  // seeded contexts (tests) derive them, others take them from the OS
  std::vector<uint8_t> rho(80 * n);
  if (ctx->seeded) {
    for (size_t i = 0; i < n; i++) {
      uint8_t le[8], h1[64];
      Blake2b h(64);
      h.update("zg-pghr13-rho", 13);
      for (int b = 0; b < 8; b++) le[b] = (uint8_t)(ctx->seed >> (8 * b));
      h.update(le, 8);
      for (int b = 0; b < 8; b++) le[b] = (uint8_t)((uint64_t)i >> (8 * b));
      h.update(le, 8);
      h.final(&rho[80 * i]);
      Blake2b g(64);
      g.update("zg-pghr13-rho1", 14);
      for (int b = 0; b < 8; b++) le[b] = (uint8_t)(ctx->seed >> (8 * b));
      g.update(le, 8);
      for (int b = 0; b < 8; b++) le[b] = (uint8_t)((uint64_t)i >> (8 * b));
      g.update(le, 8);
      g.final(h1);
      memcpy(&rho[80 * i + 64], h1, 16);
    }
  } else if (!os_random(rho.data(), rho.size())) {
    return fail(ctx, ZG_E_INVAL, "getrandom failed");
  }
  // one batch check per chunk of at most ZG_PGHR_CHUNK proofs: the call's arena (~27 KB per proof,
  // mostly the b lines) stays bounded at the chunk size however large the caller's window is
  if (kernel_ms) *kernel_ms = 0;
  bool any_failed = false;
  for (size_t o = 0; o < n; o += ZG_PGHR_CHUNK) {
    const size_t m = n - o < ZG_PGHR_CHUNK ? n - o : ZG_PGHR_CHUNK;
    bool batch_failed = false;
    float ms = 0;
    const int rc = bn_pghr13_verify(ctx->bn_key, ctx->stream, ctx->side, m, proofs + 296 * o, inputs + 9 * 32 * o,
                                    n_inputs ? n_inputs + o : nullptr, rho.data() + 80 * o, status + o,
                                    kernel_ms ? &ms : nullptr, &batch_failed, &ctx->bn_arena, &ctx->bn_arena_cap,
                                    &ctx->err);
    if (rc != ZG_OK) return rc;
    if (kernel_ms) *kernel_ms += ms;
    any_failed = any_failed || batch_failed;
  }
  if (n) {  // once per call, however many chunks it took (include/zg.h zg_stats [8], [9])
    ctx->stats[8]++;
    if (any_failed) ctx->stats[9]++;
  }
  return ZG_OK;
}

extern "C" int zg_bn254_pairing(zg_ctx* ctx, size_t n, const uint8_t* g1, const uint8_t* g2, uint8_t* gt) {
  if (!ctx || (n && (!g1 || !g2 || !gt)) || n > (1u << 20)) return ZG_E_INVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  return bn_pairing(ctx->stream, n, g1, g2, gt, &ctx->err);
}
