//! verification/src/gpu/mod.rs -- the MI355X batch Groth16 verifier behind Zebra's proof checks.
//!
//! A thin safe layer over the C ABI of include/zg.h (libzg.so, HIP for gfx950, built by
//! build.rs). It replaces, for a whole block or import window, the per-description
//! `Proof::<Bls12>::read` + `bellman::groth16::verify_proof` calls of
//! verification/src/sapling.rs:157-167,202-212 and verification/src/sprout.rs:69-80; the
//! queueing and re-injection in reference order is `collect` (a transcription of
//! zebra_amd/collector.py, which tests/test_collector.py checks against the reference's real
//! transactions).
pub mod collect;
pub mod cpu;
pub mod ffi;
pub mod writer;

use std::ffi::CStr;
use std::os::raw::c_int;
use std::sync::Mutex;

pub use ffi::{ZG_KIND_OUTPUT, ZG_KIND_SPEND, ZG_KIND_SPROUT};
pub use ffi::{ZG_STATUS_DECODE_INVALID, ZG_STATUS_MALFORMED_VK, ZG_STATUS_OK, ZG_STATUS_VERIFY_FAILED};

/// A C-ABI error: the ZG_E_* code and zg_last_error's text.
#[derive(Debug, Clone)]
pub struct GpuError {
    pub code: i32,
    pub message: String,
}

/// One queued Groth16 check: the 192 proof bytes, the kind (= verifying key) and its public
/// inputs as canonical little-endian Fr (`FrRepr::write_le`), 7 / 5 / 9 of them.
#[derive(Clone)]
pub struct Item {
    pub proof: [u8; 192],
    pub kind: u8,
    pub inputs: Vec<[u8; 32]>,
}

/// One batch slot on one GPU (device buffers only; the streams and the prepared verifying keys
/// are shared per device inside libzg). Several slots keep several windows in flight.
pub struct GpuVerifier {
    ctx: *mut ffi::ZgCtx,
    max_batch: usize,
    lock: Mutex<()>,
}
unsafe impl Send for GpuVerifier {}
unsafe impl Sync for GpuVerifier {}

fn last_error(ctx: *mut ffi::ZgCtx) -> String {
    unsafe { CStr::from_ptr(ffi::zg_last_error(ctx)) }.to_string_lossy().into_owned()
}

fn check(ctx: *mut ffi::ZgCtx, rc: c_int) -> Result<(), GpuError> {
    if rc == ffi::ZG_OK {
        Ok(())
    } else {
        Err(GpuError { code: rc, message: last_error(ctx) })
    }
}

/// the flat layouts of zg_verify_batch: n x 192 proof bytes, n kinds, n x 288 input bytes, n counts
fn pack(items: &[Item]) -> (Vec<u8>, Vec<u8>, Vec<u8>, Vec<u8>) {
    let n = items.len();
    let mut proofs = Vec::with_capacity(ffi::ZG_PROOF_BYTES * n);
    let mut kinds = Vec::with_capacity(n);
    let mut inputs = vec![0u8; ffi::ZG_INPUT_STRIDE * n];
    let mut counts = Vec::with_capacity(n);
    for (i, it) in items.iter().enumerate() {
        proofs.extend_from_slice(&it.proof);
        kinds.push(it.kind);
        counts.push(it.inputs.len().min(255) as u8);
        for (j, x) in it.inputs.iter().enumerate().take(ffi::ZG_MAX_INPUTS) {
            let o = ffi::ZG_INPUT_STRIDE * i + ffi::ZG_FR_BYTES * j;
            inputs[o..o + ffi::ZG_FR_BYTES].copy_from_slice(x);
        }
    }
    (proofs, kinds, inputs, counts)
}

impl GpuVerifier {
    /// A slot on `device` for batches of up to `max_batch` proofs, with the three unchanged
    /// verifying keys of res/*.json (embedded at build time) prepared on the GPU.
    pub fn new(device: i32, max_batch: u32) -> Result<Self, GpuError> {
        // seeded = 0: every batch draws a fresh 256-bit getrandom(2) key, expanded on the GPU
        // by ChaCha20 into the 128-bit batch scalars
        let cfg = ffi::ZgConfig { device, max_batch, seeded: 0, seed: 0 };
        let ctx = unsafe { ffi::zg_create(&cfg) };
        if ctx.is_null() {
            return Err(GpuError { code: ffi::ZG_E_HIP, message: last_error(std::ptr::null_mut()) });
        }
        let v = GpuVerifier { ctx, max_batch: if max_batch == 0 { 65536 } else { max_batch as usize }, lock: Mutex::new(()) };
        for k in [ZG_KIND_SPEND, ZG_KIND_OUTPUT, ZG_KIND_SPROUT] {
            check(ctx, unsafe { ffi::zg_vk_load_builtin(ctx, k as c_int) })?;
        }
        Ok(v)
    }

    pub fn max_batch(&self) -> usize {
        self.max_batch
    }

    /// Every item's status (ZG_STATUS_*), exact per proof: a failing batch is bisected on the
    /// GPU. Windows larger than max_batch go as consecutive batches.
    pub fn verify(&self, items: &[Item]) -> Result<Vec<u8>, GpuError> {
        let _g = self.lock.lock().unwrap();
        let mut out = Vec::with_capacity(items.len());
        for chunk in items.chunks(self.max_batch.max(1)) {
            let (proofs, kinds, inputs, counts) = pack(chunk);
            let mut status = vec![0u8; chunk.len()];
            check(self.ctx, unsafe {
                ffi::zg_verify_batch(self.ctx, chunk.len(), proofs.as_ptr(), kinds.as_ptr(), inputs.as_ptr(),
                                     counts.as_ptr(), std::ptr::null(), status.as_mut_ptr(), std::ptr::null_mut())
            })?;
            out.extend_from_slice(&status);
        }
        Ok(out)
    }

    /// Multi-GPU split (one process per GPU): queue this rank's shard and return its 576-byte
    /// Miller partial. Gather the partials of all ranks (RCCL all-gather), then `verdict` and
    /// `finish` on every rank.
    pub fn begin_partial(&self, items: &[Item]) -> Result<[u8; 576], GpuError> {
        let (proofs, kinds, inputs, counts) = pack(items);
        check(self.ctx, unsafe {
            ffi::zg_batch_begin(self.ctx, items.len(), proofs.as_ptr(), kinds.as_ptr(), inputs.as_ptr(),
                                counts.as_ptr(), std::ptr::null())
        })?;
        let mut part = [0u8; 576];
        check(self.ctx, unsafe { ffi::zg_batch_partial(self.ctx, part.as_mut_ptr()) })?;
        Ok(part)
    }

    /// ONE final exponentiation of the product of all ranks' partials: the batch verdict.
    pub fn verdict(&self, partials: &[[u8; 576]]) -> Result<bool, GpuError> {
        let flat: Vec<u8> = partials.iter().flat_map(|p| p.iter().copied()).collect();
        let mut ok: c_int = 0;
        check(self.ctx, unsafe { ffi::zg_gt_check(self.ctx, partials.len(), flat.as_ptr(), &mut ok) })?;
        Ok(ok != 0)
    }

    /// Per-proof statuses of this rank's shard; a false verdict bisects the shard.
    pub fn finish(&self, n: usize, batch_ok: bool) -> Result<Vec<u8>, GpuError> {
        let mut status = vec![0u8; n];
        check(self.ctx, unsafe { ffi::zg_batch_finish(self.ctx, batch_ok as c_int, status.as_mut_ptr()) })?;
        Ok(status)
    }
}

impl GpuVerifier {
    /// RedJubjub PublicKey::read(vk) + verify(msg, sig, generator) for every item, on the GPU
    /// (spend_auth_sig: vk = rk, msg = rk || sighash, ZG_GEN_SPEND_AUTH; binding_sig: vk = bvk,
    /// msg = bvk || sighash, ZG_GEN_BINDING).
    pub fn redjubjub_verify(&self, items: &[([u8; 32], [u8; 64], [u8; 64], u8)]) -> Result<Vec<bool>, GpuError> {
        let _g = self.lock.lock().unwrap();
        let n = items.len();
        let mut vk = Vec::with_capacity(32 * n);
        let mut sig = Vec::with_capacity(64 * n);
        let mut msg = Vec::with_capacity(64 * n);
        let mut gen = Vec::with_capacity(n);
        for (v, s, m, g) in items {
            vk.extend_from_slice(v);
            sig.extend_from_slice(s);
            msg.extend_from_slice(m);
            gen.push(*g);
        }
        let mut ok = vec![0u8; n];
        check(self.ctx, unsafe {
            ffi::zg_redjubjub_verify(self.ctx, n, vk.as_ptr(), sig.as_ptr(), msg.as_ptr(), gen.as_ptr(), ok.as_mut_ptr())
        })?;
        Ok(ok.into_iter().map(|b| b == 1).collect())
    }

    /// PHGR JoinSplit proofs (sprout.rs:61-67): per item the 296-byte proof and its
    /// into_bn_frs inputs (`prep_joinsplit_bn`) -> ZG_STATUS_* (DECODE_INVALID = InvalidEncoding,
    /// VERIFY_FAILED = InvalidPGHRProof). The builtin res/sprout-verifying-key.json is loaded on
    /// first use.
    pub fn pghr13_verify(&self, items: &[([u8; 296], Vec<[u8; 32]>)]) -> Result<Vec<u8>, GpuError> {
        let _g = self.lock.lock().unwrap();
        let n = items.len();
        let mut proofs = Vec::with_capacity(296 * n);
        let mut inputs = vec![0u8; ffi::ZG_INPUT_STRIDE * n];
        let mut counts = Vec::with_capacity(n);
        for (i, (p, x)) in items.iter().enumerate() {
            proofs.extend_from_slice(p);
            counts.push(x.len().min(ffi::ZG_MAX_INPUTS) as u8);
            for (j, v) in x.iter().enumerate().take(ffi::ZG_MAX_INPUTS) {
                let o = ffi::ZG_INPUT_STRIDE * i + ffi::ZG_FR_BYTES * j;
                inputs[o..o + ffi::ZG_FR_BYTES].copy_from_slice(v);
            }
        }
        let mut status = vec![0u8; n];
        check(self.ctx, unsafe {
            ffi::zg_pghr13_verify(self.ctx, n, proofs.as_ptr(), inputs.as_ptr(), counts.as_ptr(), status.as_mut_ptr(),
                                  std::ptr::null_mut())
        })?;
        Ok(status)
    }

    /// zg_prep_batch: a window's public-input preparation in one call (kinds ZG_PREP_KIND_*, fields
    /// n x ZG_PREP_FIELD_BYTES; the Sapling descriptions on the GPU, the JoinSplits on host threads)
    /// -> (inputs n x 288 bytes, codes ZG_PREP_*)
    pub fn prep_batch(&self, kinds: &[u8], fields: &[u8]) -> Result<(Vec<u8>, Vec<u8>), GpuError> {
        let n = kinds.len();
        assert_eq!(fields.len(), n * ffi::ZG_PREP_FIELD_BYTES, "fields must be n x ZG_PREP_FIELD_BYTES");
        let _g = self.lock.lock().unwrap();
        let mut inputs = vec![0u8; ffi::ZG_INPUT_STRIDE * n];
        let mut codes = vec![0u8; n];
        check(self.ctx, unsafe {
            ffi::zg_prep_batch(self.ctx, n, kinds.as_ptr(), fields.as_ptr(), inputs.as_mut_ptr(), codes.as_mut_ptr())
        })?;
        Ok((inputs, codes))
    }

    /// binding verification keys: per tx (spend cvs, output cvs, valueBalance) -> (status, bvk)
    pub fn sapling_bvk(&self, txs: &[(Vec<[u8; 32]>, Vec<[u8; 32]>, i64)]) -> Result<Vec<(u8, [u8; 32])>, GpuError> {
        let _g = self.lock.lock().unwrap();
        let n = txs.len();
        let ns: Vec<u32> = txs.iter().map(|t| t.0.len() as u32).collect();
        let no: Vec<u32> = txs.iter().map(|t| t.1.len() as u32).collect();
        let vb: Vec<i64> = txs.iter().map(|t| t.2).collect();
        let mut cvs = Vec::new();
        for t in txs {
            for c in t.0.iter().chain(t.1.iter()) {
                cvs.extend_from_slice(c);
            }
        }
        let mut bvk = vec![0u8; 32 * n];
        let mut st = vec![0u8; n];
        check(self.ctx, unsafe {
            ffi::zg_sapling_bvk(self.ctx, n, ns.as_ptr(), no.as_ptr(), cvs.as_ptr(), vb.as_ptr(), bvk.as_mut_ptr(),
                                st.as_mut_ptr())
        })?;
        Ok((0..n).map(|i| (st[i], bvk[32 * i..32 * i + 32].try_into().unwrap())).collect())
    }

    /// Note-commitment tree roots over an import window (storage::TreeState, serialized as the
    /// reference stores it): from `state` (empty = TreeState::new()) append `leaves` and return the
    /// root after each `marks[k]` of them (one per block for BlockSaplingRoot / the Sprout block
    /// root, one per JoinSplit for TreeCache::continue_root) and the serialized final state.
    /// kind: ffi::ZG_TREE_SPROUT (H29) or ffi::ZG_TREE_SAPLING (H32). Err(ZG_E_TREE_FULL) when the
    /// leaves overflow the tree ("Appending to full tree").
    pub fn tree_roots(&self, kind: c_int, height: c_int, state: &[u8], leaves: &[[u8; 32]], marks: &[u64])
                      -> Result<(Vec<[u8; 32]>, Vec<u8>), GpuError> {
        let _g = self.lock.lock().unwrap();
        let flat: Vec<u8> = leaves.iter().flat_map(|h| h.iter().copied()).collect();
        let mut roots = vec![0u8; 32 * marks.len()];
        let mut out_len = unsafe { ffi::zg_tree_state_max_bytes(height) };
        let mut out = vec![0u8; out_len];
        check(self.ctx, unsafe {
            ffi::zg_tree_roots(self.ctx, kind, height, state.as_ptr(), state.len(), leaves.len(), flat.as_ptr(),
                               marks.len(), marks.as_ptr(), roots.as_mut_ptr(), out.as_mut_ptr(), &mut out_len)
        })?;
        out.truncate(out_len);
        Ok((roots.chunks(32).map(|c| c.try_into().unwrap()).collect(), out))
    }
}

impl Drop for GpuVerifier {
    fn drop(&mut self) {
        unsafe { ffi::zg_destroy(self.ctx) }
    }
}

/// The Groth16 public-input preparation of the reference, restated in libzg (CPU only):
/// accept_spend (sapling.rs:101-155) -> 7 Fr, or the ZG_PREP_* error class.
pub fn prep_spend(cv: &[u8; 32], anchor: &[u8; 32], nullifier: &[u8; 32], rk: &[u8; 32]) -> Result<Vec<[u8; 32]>, i32> {
    let mut out = [0u8; 7 * 32];
    let rc = unsafe { ffi::zg_prep_spend(cv.as_ptr(), anchor.as_ptr(), nullifier.as_ptr(), rk.as_ptr(), out.as_mut_ptr()) };
    if rc != 0 {
        return Err(rc);
    }
    Ok(out.chunks(32).map(|c| c.try_into().unwrap()).collect())
}

/// accept_output (sapling.rs:171-200) -> 5 Fr
pub fn prep_output(cv: &[u8; 32], cmu: &[u8; 32], epk: &[u8; 32]) -> Result<Vec<[u8; 32]>, i32> {
    let mut out = [0u8; 5 * 32];
    let rc = unsafe { ffi::zg_prep_output(cv.as_ptr(), cmu.as_ptr(), epk.as_ptr(), out.as_mut_ptr()) };
    if rc != 0 {
        return Err(rc);
    }
    Ok(out.chunks(32).map(|c| c.try_into().unwrap()).collect())
}

/// sprout::verify's input (sprout.rs:34-58,86-153) -> 9 BLS12-381 Fr (into_bls_frs, the
/// Groth16 branch); `bn = true`: the same bits as 9 BN254 Fr (into_bn_frs, the PHGR branch)
#[allow(clippy::too_many_arguments)]
fn prep_joinsplit_any(bn: bool, anchor: &[u8; 32], random_seed: &[u8; 32], nullifiers: &[[u8; 32]; 2],
                      macs: &[[u8; 32]; 2], commitments: &[[u8; 32]; 2], vpub_old: u64, vpub_new: u64,
                      pubkey: &[u8; 32]) -> Vec<[u8; 32]> {
    let cat = |x: &[[u8; 32]; 2]| -> [u8; 64] {
        let mut o = [0u8; 64];
        o[..32].copy_from_slice(&x[0]);
        o[32..].copy_from_slice(&x[1]);
        o
    };
    let (nf, mc, cm) = (cat(nullifiers), cat(macs), cat(commitments));
    let mut out = [0u8; 9 * 32];
    unsafe {
        if bn {
            ffi::zg_prep_joinsplit_bn(anchor.as_ptr(), random_seed.as_ptr(), nf.as_ptr(), mc.as_ptr(), cm.as_ptr(),
                                      vpub_old, vpub_new, pubkey.as_ptr(), out.as_mut_ptr());
        } else {
            ffi::zg_prep_joinsplit(anchor.as_ptr(), random_seed.as_ptr(), nf.as_ptr(), mc.as_ptr(), cm.as_ptr(),
                                   vpub_old, vpub_new, pubkey.as_ptr(), out.as_mut_ptr());
        }
    }
    out.chunks(32).map(|c| c.try_into().unwrap()).collect()
}

#[allow(clippy::too_many_arguments)]
pub fn prep_joinsplit(anchor: &[u8; 32], random_seed: &[u8; 32], nullifiers: &[[u8; 32]; 2], macs: &[[u8; 32]; 2],
                      commitments: &[[u8; 32]; 2], vpub_old: u64, vpub_new: u64, pubkey: &[u8; 32]) -> Vec<[u8; 32]> {
    prep_joinsplit_any(false, anchor, random_seed, nullifiers, macs, commitments, vpub_old, vpub_new, pubkey)
}

#[allow(clippy::too_many_arguments)]
pub fn prep_joinsplit_bn(anchor: &[u8; 32], random_seed: &[u8; 32], nullifiers: &[[u8; 32]; 2], macs: &[[u8; 32]; 2],
                         commitments: &[[u8; 32]; 2], vpub_old: u64, vpub_new: u64, pubkey: &[u8; 32]) -> Vec<[u8; 32]> {
    prep_joinsplit_any(true, anchor, random_seed, nullifiers, macs, commitments, vpub_old, vpub_new, pubkey)
}
