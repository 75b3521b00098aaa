/* zg.h -- C ABI of the MI355X batch Groth16 verifier (BLS12-381) for Zebra's
 * `verification` crate. Plain pointers and sizes; caller-owned buffers only; no
 * allocation crosses the ABI.
 *
 * Reference interfaces replaced (defuse/zebra @ 2025-01-12, bellman 0.1.0, pairing 0.14.2):
 *   zg_vk_load_builtin / zg_vk_load_json   <- crypto::load_sapling_spend_verifying_key,
 *        load_sapling_output_verifying_key, load_joinsplit_groth16_verifying_key
 *        (crypto/src/json/groth16.rs:11-28) + bellman::groth16::prepare_verifying_key
 *        (called at crypto/src/json/groth16.rs:14,21,27); statics network/src/consensus.rs:4-11
 *   zg_vk_load_uncompressed               <- bellman::groth16::VerifyingKey { .. } +
 *        prepare_verifying_key (as built in verification/src/sapling.rs:345-358)
 *   zg_verify_one_gt                       <- bellman::groth16::Proof::<Bls12>::read +
 *        verify_proof for ONE proof (verification/src/sapling.rs:158-167,203-212,
 *        verification/src/sprout.rs:69-80, crypto/src/groth16.rs:52-56)
 *   zg_verify_batch                        <- the per-description loops that call the two
 *        above (sapling.rs:85-94, accept_transaction.rs:575-596) fanned out by rayon
 *        (verification/src/accept_chain.rs:76-81): one call verifies a whole block /
 *        import window with per-proof statuses in the reference's error classes.
 *   zg_batch_* / zg_gt_check               <- (no reference analogue) the 8-GPU split: each
 *        rank produces one 576-byte Miller partial, gathered over RCCL, one final exp.
 *
 * Threading: calls on different contexts are independent; one call at a time per
 * context (internal mutex; zg_verify_batch holds it from begin to finish). A context is a
 * BATCH SLOT: it owns device buffers only. The HIP streams (a fixed pool of stream pairs per
 * device, ZG_STREAM_PAIRS, default 8) and the prepared verifying keys (prepare_verifying_key
 * once per distinct key per device) belong to a per-device state shared by all contexts of the
 * process, so any number of slots can be created without new hardware queues. Slots keep
 * several batches in flight on one GPU (zg_batch_begin returns once the batch is queued);
 * slot i uses pair i mod ZG_STREAM_PAIRS. HIP maps streams onto GPU_MAX_HW_QUEUES hardware
 * queues (HIP default 4): the library is correct at any value; for batches in flight to
 * overlap, set GPU_MAX_HW_QUEUES >= 2 x (pairs in use) + 2 before the HIP runtime starts.
 * ZG_LINES_FCHAIN (environment, read by zg_create): unset = pick the R-chain/f-chain launch
 * shape by size, 0 = two launches, 1 = one fused launch.
 */
#ifndef ZG_H
#define ZG_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* proof kinds == verifying keys */
#define ZG_KIND_SPEND 0  /* res/sapling-spend-verifying-key.json, 7 public inputs */
#define ZG_KIND_OUTPUT 1 /* res/sapling-output-verifying-key.json, 5 public inputs */
#define ZG_KIND_SPROUT 2 /* res/sprout-groth16-key.json, 9 public inputs */

/* per-proof status (reference error class in brackets) */
#define ZG_STATUS_OK 0             /* verify_proof == Ok(true) */
#define ZG_STATUS_DECODE_INVALID 1 /* Proof::read -> io::Error(InvalidData): ProofError::Invalid /
                                      sprout ErrorKind::InvalidEncoding */
#define ZG_STATUS_MALFORMED_VK 2   /* SynthesisError::MalformedVerifyingKey: ProofError::Synthesis /
                                      InvalidGrothProof */
#define ZG_STATUS_VERIFY_FAILED 3  /* verify_proof == Ok(false): ProofError::Failed /
                                      InvalidGrothProof */
#define ZG_STATUS_INPUT_NONCANONICAL 4 /* a public input >= r (unreachable from the reference,
                                          whose Fr are always reduced) */

/* return codes */
#define ZG_OK 0
#define ZG_E_INVAL (-1)   /* bad argument */
#define ZG_E_HIP (-2)     /* HIP runtime / device error */
#define ZG_E_NOVK (-3)    /* a proof refers to a kind whose VK is not loaded */
#define ZG_E_VK (-4)      /* VK JSON/points failed to decode (crypto/src/json/groth16.rs:88-99) */
#define ZG_E_NOMEM (-5)   /* batch larger than max_batch / allocation failure */
#define ZG_E_STATE (-6)   /* batch API called out of order */
#define ZG_E_TREE_FULL (-7) /* TreeState::append: "Appending to full tree" (tree_state.rs:238) */
#define ZG_E_DEBUG (-8)   /* ZG_DEBUG_EACH=1 (environment, read by zg_create): a batch's statuses differ
                             from the per-proof verify_proof re-check of the same inputs */

#define ZG_PROOF_BYTES 192
#define ZG_FR_BYTES 32
#define ZG_MAX_INPUTS 9
#define ZG_INPUT_STRIDE (ZG_MAX_INPUTS * ZG_FR_BYTES) /* 288 B per proof, unused slots ignored */
#define ZG_GT_BYTES 576 /* Fq12: 12 x 48-byte big-endian canonical coefficients, tower order */
#define ZG_R_BYTES 16   /* batch scalar r_i: two little-endian u64 (a, b) meaning
                           r_i = (2a + 1) + b * lambda mod r, lambda = -x^2 mod r (the G1
                           endomorphism's eigenvalue): 2^128 distinct non-zero scalars */

typedef struct zg_config {
  int device;         /* HIP device ordinal (one process per GPU) */
  uint32_t max_batch; /* capacity of one batch (proofs); 0 -> 65536 */
  int seeded;         /* 1: batch scalars r_i from BLAKE2b(seed, i) (tests); 0: OS-random
                         ChaCha20 key per batch, expanded on the GPU (zg_chacha20_blocks) */
  uint64_t seed;
} zg_config;

typedef struct zg_ctx zg_ctx;

/* NULL on failure (no device, out of device memory, HIP error); zg_last_error(NULL) then
 * describes it (per calling thread). */
zg_ctx* zg_create(const zg_config* cfg);
void zg_destroy(zg_ctx* ctx);
const char* zg_last_error(zg_ctx* ctx);
/* library build tag (architecture + version), static string */
const char* zg_version(void);

/* ---- verifying keys (prepared once per process, resident in HBM) */
int zg_vk_load_builtin(zg_ctx* ctx, int kind);
int zg_vk_load_json(zg_ctx* ctx, int kind, const char* json, size_t len);
int zg_vk_load_uncompressed(zg_ctx* ctx, int kind, const uint8_t alpha_g1[96], const uint8_t beta_g1[96],
                            const uint8_t beta_g2[192], const uint8_t gamma_g2[192],
                            const uint8_t delta_g1[96], const uint8_t delta_g2[192], size_t n_ic,
                            const uint8_t* ic /* n_ic x 96 */);
/* the prepared alpha_g1_beta_g2 (GT) of a loaded VK */
int zg_vk_alpha_beta(zg_ctx* ctx, int kind, uint8_t gt[ZG_GT_BYTES]);

/* ---- one proof, bellman-exact: status and, for OK / VERIFY_FAILED, the final-exponentiated
 * left-hand side  FE(ML(A,B) * ML(acc,-gamma) * ML(C,-delta))  (== alpha_g1_beta_g2 iff OK) */
int zg_verify_one_gt(zg_ctx* ctx, int kind, const uint8_t proof[ZG_PROOF_BYTES], const uint8_t* inputs,
                     size_t n_inputs, uint8_t* status, uint8_t gt[ZG_GT_BYTES]);

/* ---- n proofs, each verified on its own exactly like bellman verify_proof (no batch
 * randomness): one GPU thread per proof. Same layouts as zg_verify_batch; gts optional
 * (n x 576, written for OK / VERIFY_FAILED). */
int zg_verify_each(zg_ctx* ctx, size_t n, const uint8_t* proofs, const uint8_t* kinds, const uint8_t* inputs,
                   const uint8_t* n_inputs, uint8_t* status, uint8_t* gts);

/* ---- a batch of n proofs (host buffers).
 *   proofs   n x 192 B (A || B || C compressed)
 *   kinds    n x ZG_KIND_*
 *   inputs   n x ZG_INPUT_STRIDE (canonical little-endian Fr; slots past k ignored)
 *   n_inputs optional n x count (NULL: 7 / 5 / 9 by kind); count + 1 != |ic| -> MALFORMED_VK
 *   r        optional n x 16 B batch scalars (NULL: generated per zg_config)
 *   status   out, n bytes (ZG_STATUS_*), exact per proof (bisection on failure)
 *   gt_out   optional out: prod_i LHS_i^{r_i} over proofs that decoded with a well-formed VK
 */
int zg_verify_batch(zg_ctx* ctx, size_t n, const uint8_t* proofs, const uint8_t* kinds, const uint8_t* inputs,
                    const uint8_t* n_inputs, const uint8_t* r, uint8_t* status, uint8_t* gt_out);

/* ---- split form for multi-GPU (one process per GPU):
 *   zg_batch_begin[_device]  decode + batch algebra + Miller loops + product trees
 *   zg_batch_partial         this rank's Miller partial F_g (576 B, not final-exponentiated)
 *   zg_gt_check              product of `count` partials, ONE final exponentiation, == 1 ?
 *   zg_batch_finish          statuses; when batch_ok == 0 bisects this rank's shard
 * The *_device variant takes device pointers (HBM-resident inputs; same layouts) and reads them in
 * place, without a copy: they must stay allocated and unchanged until zg_batch_finish returns
 * (bisection re-reads them). */
int zg_batch_begin(zg_ctx* ctx, size_t n, const uint8_t* proofs, const uint8_t* kinds, const uint8_t* inputs,
                   const uint8_t* n_inputs, const uint8_t* r);
int zg_batch_begin_device(zg_ctx* ctx, size_t n, const void* d_proofs, const void* d_kinds,
                          const void* d_inputs, const void* d_n_inputs, const void* d_r);
int zg_batch_partial(zg_ctx* ctx, uint8_t partial[ZG_GT_BYTES]);
/* zg_batch_ready: 1 when the batch begun on ctx has finished its pipeline (zg_batch_partial and a
 * true-verdict zg_batch_finish then return without waiting -- unless a B_i failed its G2 subgroup
 * check: the root sums then still hold that proof and zg_batch_partial first recomputes them and
 * the partial, synchronously), 0 while it runs, < 0 on error. It never blocks: a host loop keeping
 * several batches in flight harvests whichever finishes first (batches in flight finish out of
 * order). */
int zg_batch_ready(zg_ctx* ctx);
int zg_gt_check(zg_ctx* ctx, size_t count, const uint8_t* partials, int* ok);
/* zg_gt_check_many (round 6): the verdicts of `nsets` (1..16) batches in one launch, one final
 * exponentiation per set, side by side on the device: set b is the next counts[b] partials of
 * `partials` (576 B each, sum(counts) <= 4096); ok[b] = its verdict. A verdict thread that finds
 * several batches' gathered partials waiting checks them together in the time of one. */
int zg_gt_check_many(zg_ctx* ctx, size_t nsets, const size_t* counts, const uint8_t* partials, int* ok);
int zg_batch_finish(zg_ctx* ctx, int batch_ok, uint8_t* status);
/* zg_set_priority: recreate the context's two streams at the device's highest (high != 0) or
 * default priority; only between batches. A context that only runs zg_gt_check (the verdict of
 * batches kept in flight on other contexts) gets its final exponentiation dispatched ahead of
 * their waiting workgroups. */
int zg_set_priority(zg_ctx* ctx, int high);

/* ---- host-side public-input preparation (CPU; no context, no GPU). The reference does this
 * in Rust before calling bellman; these restate it so a caller can go from description bytes
 * to the `inputs` rows of zg_verify_batch. Returns ZG_PREP_* (>= 0) or ZG_E_INVAL.
 *   zg_prep_spend      <- accept_spend      verification/src/sapling.rs:101-155 (7 x 32 B out:
 *                         rk.x rk.y cv.x cv.y anchor nf0 nf1; the spend_auth_sig check stays
 *                         with the caller, between the rk check and the proof)
 *   zg_prep_output     <- accept_output     verification/src/sapling.rs:171-200 (5 x 32 B out:
 *                         cv.x cv.y epk.x epk.y cmu)
 *   zg_prep_joinsplit  <- sprout::verify    verification/src/sprout.rs:34-58,86-153 (9 x 32 B,
 *                         Input::into_bls_frs: the Groth16 branch, 254-bit chunks)
 *   zg_prep_joinsplit_bn <- the same Input, into_bn_frs (sprout.rs:119-133: 253-bit chunks, 9 x
 *                         32-byte LE BN254 Fr): the inputs of zg_pghr13_verify for a PHGR JoinSplit
 *   zg_hsig            <- compute_hsig      verification/src/sprout.rs:16-32 */
#define ZG_PREP_OK 0
#define ZG_PREP_VALUE_COMMITMENT_INVALID 1     /* ValueCommitment(Invalid) */
#define ZG_PREP_VALUE_COMMITMENT_SMALL_ORDER 2 /* ValueCommitment(SmallOrder) */
#define ZG_PREP_ANCHOR 3                       /* SpendError::Anchor */
#define ZG_PREP_RANDOMIZED_KEY_INVALID 4       /* SpendError::RandomizedKey(Invalid) */
#define ZG_PREP_RANDOMIZED_KEY_SMALL_ORDER 5   /* SpendError::RandomizedKey(SmallOrder) */
#define ZG_PREP_NOTE_COMMITMENT 6              /* OutputError::NoteCommitment */
#define ZG_PREP_EPHEMERAL_KEY_INVALID 7        /* OutputError::EphemeralKey(Invalid) */
#define ZG_PREP_EPHEMERAL_KEY_SMALL_ORDER 8    /* OutputError::EphemeralKey(SmallOrder) */
int zg_prep_spend(const uint8_t cv[32], const uint8_t anchor[32], const uint8_t nullifier[32], const uint8_t rk[32],
                  uint8_t inputs[7 * 32]);
int zg_prep_output(const uint8_t cv[32], const uint8_t cmu[32], const uint8_t epk[32], uint8_t inputs[5 * 32]);
int zg_prep_joinsplit(const uint8_t anchor[32], const uint8_t random_seed[32], const uint8_t nullifiers[64],
                      const uint8_t macs[64], const uint8_t commitments[64], uint64_t vpub_old, uint64_t vpub_new,
                      const uint8_t pubkey[32], uint8_t inputs[9 * 32]);
int zg_prep_joinsplit_bn(const uint8_t anchor[32], const uint8_t random_seed[32], const uint8_t nullifiers[64],
                         const uint8_t macs[64], const uint8_t commitments[64], uint64_t vpub_old, uint64_t vpub_new,
                         const uint8_t pubkey[32], uint8_t inputs[9 * 32]);
int zg_hsig(const uint8_t random_seed[32], const uint8_t nf0[32], const uint8_t nf1[32], const uint8_t pubkey[32],
            uint8_t out[32]);

/* ---- the same preparation for a whole import window in ONE call (round 6): the Sapling
 * descriptions on the GPU (one lane each: both Jubjub decodes and small-order checks, the field
 * checks, multipacking -- the per-description work of zg_prep_spend / zg_prep_output), the
 * JoinSplits on host threads meanwhile (BLAKE2b hSig and bit packing, as zg_prep_joinsplit[_bn]).
 * The caller side of accept_chain.rs:76-81 (rayon over a block's transactions) feeds it a block or
 * window at once. kinds[i] ZG_PREP_KIND_*; fields n x ZG_PREP_FIELD_BYTES per kind:
 *   SPEND        cv | anchor | nullifier | rk                                     (4 x 32 B)
 *   OUTPUT       cv | cmu | epk                                                   (3 x 32 B)
 *   JOINSPLIT[_BN] anchor | random_seed | nf0 | nf1 | mac0 | mac1 | cm0 | cm1 | pubkey (9 x 32 B)
 *                | vpub_old | vpub_new                                          (2 x 8 B LE)
 * -> inputs n x 288 B (the rows of zg_verify_batch / zg_pghr13_verify: 7 / 5 / 9 x 32 B, zero
 * padded), codes n x ZG_PREP_* (the single-description functions' return values, same order of
 * checks). Returns ZG_OK or an error code. */
#define ZG_PREP_KIND_SPEND 0
#define ZG_PREP_KIND_OUTPUT 1
#define ZG_PREP_KIND_JOINSPLIT 2
#define ZG_PREP_KIND_JOINSPLIT_BN 3
#define ZG_PREP_FIELD_BYTES 304
int zg_prep_batch(zg_ctx* ctx, size_t n, const uint8_t* kinds, const uint8_t* fields, uint8_t* inputs,
                  uint8_t* codes);

/* ---- Sapling signatures and Jubjub points on the GPU: the checks that sit
 * next to the Groth16 proofs in accept_sapling, batched. Any n; device memory per call.
 *   zg_redjubjub_verify <- redjubjub::PublicKey::read + verify (sapling-crypto @21084bde), called at
 *        verification/src/sapling.rs:124-137 (spend_auth_sig: vk = rk, msg = rk || sighash,
 *        ZG_GEN_SPEND_AUTH) and :228-238 (binding_sig: vk = bvk, msg = bvk || sighash,
 *        ZG_GEN_BINDING). vk n x 32, sig n x 64 (Rbar || Sbar), msg n x 64, gen n -> ok n (1 / 0)
 *   zg_sapling_bvk      <- the binding verification key of each transaction (sapling.rs:82-94,
 *        216-226, 247-269): sum cv(spends) - sum cv(outputs) - [valueBalance] G_v. cvs: per tx its
 *        n_spends spend cvs then n_outputs output cvs (32 B each), transactions back to back;
 *        -> bvk ntx x 32 (edwards::Point::write) and status ntx: 0 ok, 1 a cv does not decode,
 *        2 valueBalance == INT64_MIN (InvalidBalanceValue)
 *   zg_jubjub_decode    <- edwards::Point::read + is_small_order (sapling.rs:280-292): status n
 *        (0 ok, 1 invalid, 2 small order), xy optional n x 64 (x || y canonical LE Fr) */
#define ZG_GEN_SPEND_AUTH 0 /* FixedGenerators::SpendingKeyGenerator */
#define ZG_GEN_BINDING 1    /* FixedGenerators::ValueCommitmentRandomness */
int zg_redjubjub_verify(zg_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                        const uint8_t* gen, uint8_t* ok);
int zg_sapling_bvk(zg_ctx* ctx, size_t ntx, const uint32_t* n_spends, const uint32_t* n_outputs, const uint8_t* cvs,
                   const int64_t* value_balance, uint8_t* bvk, uint8_t* status);
int zg_jubjub_decode(zg_ctx* ctx, size_t n, const uint8_t* points, uint8_t* status, uint8_t* xy);

/* ---- note-commitment trees on the GPU. Hashes are H256 byte strings
 * (32 B, storage order). kind ZG_TREE_SPROUT: SproutTreeHash, combine = sha256_compress
 * (crypto/src/lib.rs:188-198); ZG_TREE_SAPLING: SaplingTreeHash, combine = pedersen_hash(left,
 * right, depth) (crypto/src/lib.rs:250-275, Personalization::MerkleTree(depth), depth < 63).
 *   zg_merkle_combine   <- TreeHash::combine (storage/src/tree_state.rs:175-177,188-190) on n
 *        pairs: out[i] = combine(left[i], right[i], depth[i]) (depth NULL = all 0)
 *   zg_tree_empty_roots <- H::empty() (tree_state.rs:5-138): levels (<= 64) entries, empty[0] =
 *        the uncommitted leaf, empty[l + 1] = combine(empty[l], empty[l], l); computed on the
 *        device on first use
 *   zg_tree_roots       <- TreeState<D, H> (tree_state.rs:193-264) over a run of appends: from
 *        `state` (the reference's serialized TreeState of this height, tree_state.rs:284-309;
 *        NULL / state_len 0 = TreeState::new()) append the n_leaves leaves (n x 32 B) and write
 *        roots[k] = root() after the first marks[k] of them (any order, each <= n_leaves):
 *        one per block for the Sapling / Sprout block roots (db/src/block_chain_db.rs:254-304,
 *        verification/src/accept_block.rs:290-320), one per JoinSplit for tree_cache.rs:57-71.
 *        state_out (optional; capacity *state_out_len >= zg_tree_state_max_bytes(height)) gets
 *        the serialized state after all n_leaves, *state_out_len its length. If the leaves
 *        overflow the 2^height capacity: ZG_E_TREE_FULL, roots of the marks that fit are still
 *        written (zeros for the others), state_out untouched. A state the appends could not
 *        have produced (right or a parent without left, a parents list of another length) is
 *        ZG_E_INVAL. Height 1..62 (29 Sprout H29, 32 Sapling H32).
 *   zg_tree_roots_device: the same with the leaves already in device memory; kernel_ms
 *        (optional) = device time of the level kernels (HIP events on the context stream) */
#define ZG_TREE_SPROUT 0
#define ZG_TREE_SAPLING 1
int zg_merkle_combine(zg_ctx* ctx, int kind, size_t n, const uint8_t* left, const uint8_t* right,
                      const uint8_t* depth, uint8_t* out);
int zg_tree_empty_roots(zg_ctx* ctx, int kind, size_t levels, uint8_t* out);
size_t zg_tree_state_max_bytes(int height);
int zg_tree_roots(zg_ctx* ctx, int kind, int height, const uint8_t* state, size_t state_len, size_t n_leaves,
                  const uint8_t* leaves, size_t n_marks, const uint64_t* marks, uint8_t* roots, uint8_t* state_out,
                  size_t* state_out_len);
int zg_tree_roots_device(zg_ctx* ctx, int kind, int height, const uint8_t* state, size_t state_len,
                         size_t n_leaves, const void* d_leaves, size_t n_marks, const uint64_t* marks,
                         uint8_t* roots, uint8_t* state_out, size_t* state_out_len, float* kernel_ms);

/* ---- PGHR13 Sprout proofs on BN254: pre-Sapling JoinSplits (the `bn` crate).
 *   zg_pghr13_vk_load_builtin / _json <- crypto/src/json/pghr13.rs decode of
 *        res/sprout-verifying-key.json (embedded unchanged); points through AffineG1/G2::new
 *        (ZG_E_VK when one is off its curve or, in G2, not of order r). The key is the calling
 *        context's own: prepared once per distinct key per device into fresh buffers and
 *        published complete (other contexts keep their keys; a failed load leaves the
 *        context's key unchanged). zg_pghr13_verify loads the builtin key on first use.
 *   zg_pghr13_verify <- Proof::from_raw + pghr13::verify (crypto/src/pghr13.rs:69-105), called at
 *        verification/src/sprout.rs:61-67: proofs n x 296 bytes (the JoinSplit's PHGR proof),
 *        inputs n x 9 x 32 bytes (BN254 Fr, little-endian: Input::into_bn_frs, 253-bit chunks),
 *        n_inputs optional (count per proof, <= 9; NULL = 9; fewer inputs contribute fewer
 *        ic terms, as the reference's zip). status n: ZG_STATUS_OK, ZG_STATUS_DECODE_INVALID
 *        (-> ErrorKind::InvalidEncoding), ZG_STATUS_VERIFY_FAILED (-> InvalidPGHRProof),
 *        ZG_STATUS_INPUT_NONCANONICAL (an input >= r: not constructible as bn::Fr). The five
 *        pairing equalities of a proof are checked as one product with OS-random 128-bit weights
 *        (false accept ~2^-128). One batch check per chunk of at most 65,536 proofs (the
 *        call's device scratch stays bounded however large n is). kernel_ms optional: device
 *        time of the kernels, summed over the chunks. A key is freed from the device cache once
 *        no context points at it (a context that loads another key, or is destroyed).
 *   zg_bn254_pairing (tests): e(P, Q) to the power 2u(6u^2 + 3u + 1) (the device's final
 *        exponentiation, see zg_bn254.h): P n x 64 (x, y), Q n x 128 (x.c0, x.c1, y.c0, y.c1),
 *        canonical little-endian Fq; GT n x 384 (12 Fq, coefficients of w^0..w^5 as c0, c1). */
int zg_pghr13_vk_load_builtin(zg_ctx* ctx);
int zg_pghr13_vk_load_json(zg_ctx* ctx, const char* json, size_t len);
int zg_pghr13_verify(zg_ctx* ctx, size_t n, const uint8_t* proofs, const uint8_t* inputs, const uint8_t* n_inputs,
                     uint8_t* status, float* kernel_ms);
int zg_bn254_pairing(zg_ctx* ctx, size_t n, const uint8_t* g1, const uint8_t* g2, uint8_t* gt);

/* ---- synthetic workload (bench/tests): Groth16 re-randomization of real proofs,
 * out[i] = rerandomize(src[src_index[i]]) with (t, s) = BLAKE2b-512("zg-rerand"||seed||i)
 * (A,B,C) -> (t^-1 A, t B + t s delta, C + s A); valid iff the source is. */
int zg_synth_rerandomize(zg_ctx* ctx, size_t n_src, const uint8_t* src_proofs, const uint8_t* src_kinds,
                         size_t n, const uint32_t* src_index, uint64_t seed, uint8_t* out_proofs);

/* ---- measurement helpers */
/* time (ms, HIP events on the context streams) of the most recent zg_batch_begin* +
 * zg_batch_partial: [0] decode (main stream), [1] R-chain / line coefficients (+ G2 subgroup
 * checks), [2] f-chain (per-proof Miller values), [3] Fq12 product tree, [4] root partial
 * (waiting for the side stream, gated recompute, root product), [5] side stream (K4 Pippenger
 * sum r_i C_i + root Fr sums + VK-side MSM + VK Miller loops, overlapping [1]-[3]; with
 * ZG_SERIAL_SIDE=1 in the environment at zg_create it runs on the main stream after [3]),
 * [6] whole device pipeline */
int zg_last_timings(zg_ctx* ctx, float* ms7);
/* the same, n values: [0]-[6] as above, [7] K4 (the Pippenger MSM + root Fr sums, part of [5]),
 * [8] K4's bucket phase (k_msm_bucket alone). Writes min(n, 9) values, zero beyond. */
int zg_last_phase_ms(zg_ctx* ctx, float* ms, size_t n);
/* cumulative counters of this context: [0] batches, [1] fused R-chain + f-chain launches,
 * [2] fused launches whose consumers timed out waiting (the f-chain was recomputed by the
 * split kernel; the context uses split launches from then on), [3] batches with a B that
 * failed its G2 subgroup check (the VK-side root work recomputed at harvest, settle_batch), [4] bisections,
 * [5] tree nodes checked by bisection, [6] K4 bucket entries of the last batch (points with a
 * non-zero window digit, summed over the windows), [7] f-chain launches with four proofs per lane
 * (k_batch_fchain4; shards of 8,192 or more padded proofs -- ZG_QUAD_MIN -- or as ZG_FCHAIN_QUADS
 * forces), [8] zg_pghr13_verify calls with proofs (once per call, however many 65,536-proof chunks it
 * took), [9] those in which a chunk's batch check failed (that chunk then ran the per-proof check
 * for the exact statuses), [10] batches whose sums r_i C_i came
 * from the GLV products in decode and the C-sum tree (shards below 16,384 padded proofs -- ZG_K4_MIN
 * -- instead of K4's Pippenger buckets; [6] is 0 for them), [11] of the four-proofs-per-lane batches
 * ([7]) those whose f-chain ran as group line products + one chain per group (k_line_prod,
 * k_batch_fchaing; ZG_LINE_GROUP proofs a group), [12] of those the batches whose lines came from the affine
 * R-chain (k_batch_lines_aff, ZG_LINES_AFFINE). Writes min(n, 13) values, zero beyond. */
int zg_stats(zg_ctx* ctx, uint64_t* out, size_t n);
/* the batch-scalar CSPRNG (contexts with seeded = 0): per batch a fresh 256-bit key from
 * getrandom(2), expanded on the device by ChaCha20 (RFC 8439), nonce 0, block j -> r_{4j..4j+3}.
 * This entry runs the same device block function for known-answer tests: out = nblocks x 64 B
 * of the keystream for (key, nonce) from block `counter` on. */
int zg_chacha20_blocks(zg_ctx* ctx, const uint8_t key[32], const uint8_t nonce[12], uint32_t counter,
                       size_t nblocks, uint8_t* out);
/* microbenchmark: v_mad_u64_u32 chains; returns achieved 32x32->64 MACs per second */
int zg_bench_mad_rate(zg_ctx* ctx, double* macs_per_s);
/* the same probe, plus the shader clock it ran at (median over workgroups of s_memtime ticks
 * per 100 MHz s_memrealtime tick, stamped around the loop); clock_hz may be NULL */
int zg_bench_mad_rate_clock(zg_ctx* ctx, double* macs_per_s, double* clock_hz);
/* debug: the 29-bit-digit Montgomery products every kernel uses, one per lane on `device`, for
 * exact host comparison (tests/test_gpu_field.py; guards the zg_opaque workaround of DESIGN.md
 * section 4). field 0: Fq a b 2^-384 mod p (48-B LE operands), 1: Fq a^2 2^-384 (b unused, a < 2p),
 * 2: Fq2 (96 B = c0 || c1; a lazy < 2p per coefficient, b canonical), 3: BLS12-381 Fr a b 2^-256 mod r
 * (32 B), 4: BN254 Fq a b 2^-256 mod q (32 B). out has the operands' size. */
int zg_debug_field_mul(int device, int field, size_t n, const uint8_t* a, const uint8_t* b, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif
