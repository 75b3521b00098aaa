//! verification/src/gpu/ffi.rs -- the `extern "C"` declarations of include/zg.h, one for one.
//! tests/test_rust_binding.py checks every signature here against the C header (no cargo in
//! the build image, so the binding is verified textually, not compiled there).
#![allow(dead_code)]
use std::os::raw::{c_char, c_int, c_void};

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct ZgConfig {
    /// HIP device ordinal (one process per GPU)
    pub device: c_int,
    /// capacity of one batch (proofs); 0 -> 65536
    pub max_batch: u32,
    /// 1: batch scalars from BLAKE2b(seed, i) (tests); 0: OS-random ChaCha20 key per batch
    pub seeded: c_int,
    pub seed: u64,
}

/// opaque batch slot (include/zg.h `zg_ctx`)
#[repr(C)]
pub struct ZgCtx {
    _private: [u8; 0],
}

pub const ZG_KIND_SPEND: u8 = 0;
pub const ZG_KIND_OUTPUT: u8 = 1;
pub const ZG_KIND_SPROUT: u8 = 2;

pub const ZG_STATUS_OK: u8 = 0;
pub const ZG_STATUS_DECODE_INVALID: u8 = 1;
pub const ZG_STATUS_MALFORMED_VK: u8 = 2;
pub const ZG_STATUS_VERIFY_FAILED: u8 = 3;
pub const ZG_STATUS_INPUT_NONCANONICAL: u8 = 4;

pub const ZG_OK: c_int = 0;
pub const ZG_E_INVAL: c_int = -1;
pub const ZG_E_HIP: c_int = -2;
pub const ZG_E_NOVK: c_int = -3;
pub const ZG_E_VK: c_int = -4;
pub const ZG_E_NOMEM: c_int = -5;
pub const ZG_E_STATE: c_int = -6;
pub const ZG_E_TREE_FULL: c_int = -7;
pub const ZG_E_DEBUG: c_int = -8;

pub const ZG_PREP_KIND_SPEND: u8 = 0;
pub const ZG_PREP_KIND_OUTPUT: u8 = 1;
pub const ZG_PREP_KIND_JOINSPLIT: u8 = 2;
pub const ZG_PREP_KIND_JOINSPLIT_BN: u8 = 3;
pub const ZG_PREP_FIELD_BYTES: usize = 304;

pub const ZG_PROOF_BYTES: usize = 192;
pub const ZG_FR_BYTES: usize = 32;
pub const ZG_MAX_INPUTS: usize = 9;
pub const ZG_INPUT_STRIDE: usize = ZG_MAX_INPUTS * ZG_FR_BYTES;
pub const ZG_GT_BYTES: usize = 576;
pub const ZG_R_BYTES: usize = 16;

pub const ZG_GEN_SPEND_AUTH: u8 = 0;
pub const ZG_GEN_BINDING: u8 = 1;
pub const ZG_TREE_SPROUT: c_int = 0;
pub const ZG_TREE_SAPLING: c_int = 1;

pub const ZG_PREP_OK: c_int = 0;
pub const ZG_PREP_VALUE_COMMITMENT_INVALID: c_int = 1;
pub const ZG_PREP_VALUE_COMMITMENT_SMALL_ORDER: c_int = 2;
pub const ZG_PREP_ANCHOR: c_int = 3;
pub const ZG_PREP_RANDOMIZED_KEY_INVALID: c_int = 4;
pub const ZG_PREP_RANDOMIZED_KEY_SMALL_ORDER: c_int = 5;
pub const ZG_PREP_NOTE_COMMITMENT: c_int = 6;
pub const ZG_PREP_EPHEMERAL_KEY_INVALID: c_int = 7;
pub const ZG_PREP_EPHEMERAL_KEY_SMALL_ORDER: c_int = 8;

#[link(name = "zg")]
extern "C" {
    pub fn zg_create(cfg: *const ZgConfig) -> *mut ZgCtx;
    pub fn zg_destroy(ctx: *mut ZgCtx);
    pub fn zg_last_error(ctx: *mut ZgCtx) -> *const c_char;
    pub fn zg_version() -> *const c_char;

    pub fn zg_vk_load_builtin(ctx: *mut ZgCtx, kind: c_int) -> c_int;
    pub fn zg_vk_load_json(ctx: *mut ZgCtx, kind: c_int, json: *const c_char, len: usize) -> c_int;
    pub fn zg_vk_load_uncompressed(ctx: *mut ZgCtx, kind: c_int, alpha_g1: *const u8, beta_g1: *const u8,
                                   beta_g2: *const u8, gamma_g2: *const u8, delta_g1: *const u8,
                                   delta_g2: *const u8, n_ic: usize, ic: *const u8) -> c_int;
    pub fn zg_vk_alpha_beta(ctx: *mut ZgCtx, kind: c_int, gt: *mut u8) -> c_int;

    pub fn zg_verify_one_gt(ctx: *mut ZgCtx, kind: c_int, proof: *const u8, inputs: *const u8, n_inputs: usize,
                            status: *mut u8, gt: *mut u8) -> c_int;
    pub fn zg_verify_each(ctx: *mut ZgCtx, n: usize, proofs: *const u8, kinds: *const u8, inputs: *const u8,
                          n_inputs: *const u8, status: *mut u8, gts: *mut u8) -> c_int;
    pub fn zg_verify_batch(ctx: *mut ZgCtx, n: usize, proofs: *const u8, kinds: *const u8, inputs: *const u8,
                           n_inputs: *const u8, r: *const u8, status: *mut u8, gt_out: *mut u8) -> c_int;

    pub fn zg_batch_begin(ctx: *mut ZgCtx, n: usize, proofs: *const u8, kinds: *const u8, inputs: *const u8,
                          n_inputs: *const u8, r: *const u8) -> c_int;
    pub fn zg_batch_begin_device(ctx: *mut ZgCtx, n: usize, d_proofs: *const c_void, d_kinds: *const c_void,
                                 d_inputs: *const c_void, d_n_inputs: *const c_void, d_r: *const c_void) -> c_int;
    pub fn zg_batch_partial(ctx: *mut ZgCtx, partial: *mut u8) -> c_int;
    pub fn zg_batch_ready(ctx: *mut ZgCtx) -> c_int;
    pub fn zg_gt_check(ctx: *mut ZgCtx, count: usize, partials: *const u8, ok: *mut c_int) -> c_int;
    pub fn zg_gt_check_many(ctx: *mut ZgCtx, nsets: usize, counts: *const usize, partials: *const u8,
                            ok: *mut c_int) -> c_int;
    pub fn zg_batch_finish(ctx: *mut ZgCtx, batch_ok: c_int, status: *mut u8) -> c_int;
    pub fn zg_set_priority(ctx: *mut ZgCtx, high: c_int) -> c_int;

    pub fn zg_prep_spend(cv: *const u8, anchor: *const u8, nullifier: *const u8, rk: *const u8,
                         inputs: *mut u8) -> c_int;
    pub fn zg_prep_output(cv: *const u8, cmu: *const u8, epk: *const u8, inputs: *mut u8) -> c_int;
    pub fn zg_prep_joinsplit(anchor: *const u8, random_seed: *const u8, nullifiers: *const u8, macs: *const u8,
                             commitments: *const u8, vpub_old: u64, vpub_new: u64, pubkey: *const u8,
                             inputs: *mut u8) -> c_int;
    pub fn zg_prep_joinsplit_bn(anchor: *const u8, random_seed: *const u8, nullifiers: *const u8, macs: *const u8,
                                commitments: *const u8, vpub_old: u64, vpub_new: u64, pubkey: *const u8,
                                inputs: *mut u8) -> c_int;
    pub fn zg_hsig(random_seed: *const u8, nf0: *const u8, nf1: *const u8, pubkey: *const u8, out: *mut u8) -> c_int;
    pub fn zg_prep_batch(ctx: *mut ZgCtx, n: usize, kinds: *const u8, fields: *const u8, inputs: *mut u8,
                         codes: *mut u8) -> c_int;

    pub fn zg_redjubjub_verify(ctx: *mut ZgCtx, n: usize, vk: *const u8, sig: *const u8, msg: *const u8,
                               gen: *const u8, ok: *mut u8) -> c_int;
    pub fn zg_sapling_bvk(ctx: *mut ZgCtx, ntx: usize, n_spends: *const u32, n_outputs: *const u32, cvs: *const u8,
                          value_balance: *const i64, bvk: *mut u8, status: *mut u8) -> c_int;
    pub fn zg_jubjub_decode(ctx: *mut ZgCtx, n: usize, points: *const u8, status: *mut u8, xy: *mut u8) -> c_int;

    pub fn zg_pghr13_vk_load_builtin(ctx: *mut ZgCtx) -> c_int;
    pub fn zg_pghr13_vk_load_json(ctx: *mut ZgCtx, json: *const c_char, len: usize) -> c_int;
    pub fn zg_pghr13_verify(ctx: *mut ZgCtx, n: usize, proofs: *const u8, inputs: *const u8, n_inputs: *const u8,
                            status: *mut u8, kernel_ms: *mut f32) -> c_int;
    pub fn zg_bn254_pairing(ctx: *mut ZgCtx, n: usize, g1: *const u8, g2: *const u8, gt: *mut u8) -> c_int;

    pub fn zg_merkle_combine(ctx: *mut ZgCtx, kind: c_int, n: usize, left: *const u8, right: *const u8,
                             depth: *const u8, out: *mut u8) -> c_int;
    pub fn zg_tree_empty_roots(ctx: *mut ZgCtx, kind: c_int, levels: usize, out: *mut u8) -> c_int;
    pub fn zg_tree_state_max_bytes(height: c_int) -> usize;
    pub fn zg_tree_roots(ctx: *mut ZgCtx, kind: c_int, height: c_int, state: *const u8, state_len: usize,
                         n_leaves: usize, leaves: *const u8, n_marks: usize, marks: *const u64, roots: *mut u8,
                         state_out: *mut u8, state_out_len: *mut usize) -> c_int;
    pub fn zg_tree_roots_device(ctx: *mut ZgCtx, kind: c_int, height: c_int, state: *const u8, state_len: usize,
                                n_leaves: usize, d_leaves: *const c_void, n_marks: usize, marks: *const u64,
                                roots: *mut u8, state_out: *mut u8, state_out_len: *mut usize,
                                kernel_ms: *mut f32) -> c_int;

    pub fn zg_synth_rerandomize(ctx: *mut ZgCtx, n_src: usize, src_proofs: *const u8, src_kinds: *const u8,
                                n: usize, src_index: *const u32, seed: u64, out_proofs: *mut u8) -> c_int;
    pub fn zg_last_timings(ctx: *mut ZgCtx, ms7: *mut f32) -> c_int;
    pub fn zg_last_phase_ms(ctx: *mut ZgCtx, ms: *mut f32, n: usize) -> c_int;
    pub fn zg_stats(ctx: *mut ZgCtx, out: *mut u64, n: usize) -> c_int;
    pub fn zg_chacha20_blocks(ctx: *mut ZgCtx, key: *const u8, nonce: *const u8, counter: u32, nblocks: usize,
                              out: *mut u8) -> c_int;
    pub fn zg_bench_mad_rate(ctx: *mut ZgCtx, macs_per_s: *mut f64) -> c_int;
    pub fn zg_bench_mad_rate_clock(ctx: *mut ZgCtx, macs_per_s: *mut f64, clock_hz: *mut f64) -> c_int;
    pub fn zg_debug_field_mul(device: c_int, field: c_int, n: usize, a: *const u8, b: *const u8, out: *mut u8)
                              -> c_int;
}
