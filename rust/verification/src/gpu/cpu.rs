//! verification/src/gpu/cpu.rs -- the GPU-error degradation path ("a fallback
//! handles no-GPU / error cases").
//!
//! When a GPU call fails mid-window (`GpuError`: a HIP error, a lost device, ZG_E_DEBUG from the
//! ZG_DEBUG_EACH cross-check), `collect::verify_block_or_cpu` re-runs the WHOLE window through
//! this backend: the reference's own per-proof calls, exactly as the CPU path makes them today,
//! fanned out with rayon like `ChainAcceptor::check_transactions` (accept_chain.rs:76-81):
//!
//!   Groth16   Proof::<Bls12>::read + bellman::groth16::verify_proof
//!             (verification/src/sapling.rs:157-167,202-212, sprout.rs:69-80)
//!   PGHR13    Pghr13Proof::from_raw + crypto::pghr13_verify (sprout.rs:61-67)
//!   RedJubjub redjubjub::PublicKey::read + verify (sapling.rs:119-137, 216-244), the binding
//!             verification key as accept_sapling / accept_sapling_final accumulate it
//!
//! Nothing here is the test oracle: these are the reference crates' functions. The statuses use
//! the same ZG_STATUS_* codes as the GPU, so the re-injection of `collect` is shared.
use rayon::prelude::*;

use crypto::bellman::groth16::{verify_proof, Proof};
use crypto::curve::bn;
use crypto::pairing::bls12_381::{Bls12, Fr, FrRepr};
use crypto::pairing::{PrimeField, PrimeFieldRepr};
use crypto::sapling_crypto::jubjub::{edwards, fs::FsRepr, FixedGenerators, JubjubParams, Unknown};
use crypto::sapling_crypto::redjubjub::{self, Signature};
use crypto::{pghr13_verify, Groth16VerifyingKey, Pghr13Proof, Pghr13VerifyingKey, JUBJUB};

use super::ffi::{ZG_GEN_BINDING, ZG_STATUS_INPUT_NONCANONICAL};
use super::{GpuError, Item, ZG_KIND_OUTPUT, ZG_KIND_SPEND, ZG_STATUS_DECODE_INVALID, ZG_STATUS_MALFORMED_VK,
            ZG_STATUS_OK, ZG_STATUS_VERIFY_FAILED};

type Point = edwards::Point<Bls12, Unknown>;

/// The verifying keys the CPU path already holds (ConsensusParams: the three Groth16 keys of
/// res/*.json and the PGHR13 Sprout key).
pub struct CpuBackend<'a> {
    pub spend_vk: &'a Groth16VerifyingKey,
    pub output_vk: &'a Groth16VerifyingKey,
    pub sprout_groth16_vk: &'a Groth16VerifyingKey,
    pub sprout_pghr13_vk: &'a Pghr13VerifyingKey,
}

fn read_fr(x: &[u8; 32]) -> Option<Fr> {
    let mut repr = FrRepr::default();
    repr.read_le(&x[..]).ok()?;
    Fr::from_repr(repr).ok()
}

fn read_point(x: &[u8; 32]) -> Option<Point> {
    let p = Point::read(&x[..], &JUBJUB).ok()?;
    if p.double(&JUBJUB).double(&JUBJUB).double(&JUBJUB) == edwards::Point::zero() {
        return None;
    }
    Some(p)
}

impl<'a> CpuBackend<'a> {
    fn key(&self, kind: u8) -> &Groth16VerifyingKey {
        match kind {
            ZG_KIND_SPEND => self.spend_vk,
            ZG_KIND_OUTPUT => self.output_vk,
            _ => self.sprout_groth16_vk,
        }
    }

    /// one Groth16 check, the reference's way: Proof::read -> DECODE_INVALID, verify_proof's
    /// Err -> MALFORMED_VK, Ok(false) -> VERIFY_FAILED
    pub fn groth16_status(&self, it: &Item) -> u8 {
        let mut inputs = Vec::with_capacity(it.inputs.len());
        for x in &it.inputs {
            match read_fr(x) {
                Some(f) => inputs.push(f),
                None => return ZG_STATUS_INPUT_NONCANONICAL,
            }
        }
        let proof = match Proof::<Bls12>::read(&it.proof[..]) {
            Ok(p) => p,
            Err(_) => return ZG_STATUS_DECODE_INVALID,
        };
        match verify_proof(&self.key(it.kind).0, &proof, &inputs[..]) {
            Ok(true) => ZG_STATUS_OK,
            Ok(false) => ZG_STATUS_VERIFY_FAILED,
            Err(_) => ZG_STATUS_MALFORMED_VK,
        }
    }

    /// one PHGR check (sprout.rs:61-67): from_raw -> DECODE_INVALID (InvalidEncoding),
    /// pghr13_verify false -> VERIFY_FAILED (InvalidPGHRProof); inputs are into_bn_frs' 32-byte
    /// LE values (bn::Fr::from_slice reads big-endian)
    pub fn pghr13_status(&self, proof: &[u8; 296], inputs: &[[u8; 32]]) -> u8 {
        let p = match Pghr13Proof::from_raw(proof) {
            Ok(p) => p,
            Err(_) => return ZG_STATUS_DECODE_INVALID,
        };
        let mut frs = Vec::with_capacity(inputs.len());
        for x in inputs {
            let mut be = *x;
            be.reverse();
            match bn::Fr::from_slice(&be) {
                Ok(f) => frs.push(f),
                Err(_) => return ZG_STATUS_INPUT_NONCANONICAL,
            }
        }
        if pghr13_verify(self.sprout_pghr13_vk, &frs, &p) {
            ZG_STATUS_OK
        } else {
            ZG_STATUS_VERIFY_FAILED
        }
    }
}

impl<'a> super::collect::Backend for CpuBackend<'a> {
    fn verify(&self, items: &[Item]) -> Result<Vec<u8>, GpuError> {
        Ok(items.par_iter().map(|it| self.groth16_status(it)).collect())
    }

    fn pghr13_verify(&self, items: &[([u8; 296], Vec<[u8; 32]>)]) -> Result<Vec<u8>, GpuError> {
        Ok(items.par_iter().map(|(p, x)| self.pghr13_status(p, x)).collect())
    }

    /// RedJubjub PublicKey::read + verify for every (vk, sig, msg, generator)
    fn redjubjub_verify(&self, items: &[([u8; 32], [u8; 64], [u8; 64], u8)]) -> Result<Vec<bool>, GpuError> {
        Ok(items
            .par_iter()
            .map(|(vk, sig, msg, gen)| {
                let key = match redjubjub::PublicKey::<Bls12>::read(&vk[..], &JUBJUB) {
                    Ok(k) => k,
                    Err(_) => return false,
                };
                let sig = match Signature::read(&sig[..]) {
                    Ok(s) => s,
                    Err(_) => return false,
                };
                let g = if *gen == ZG_GEN_BINDING {
                    FixedGenerators::ValueCommitmentRandomness
                } else {
                    FixedGenerators::SpendingKeyGenerator
                };
                key.verify(&msg[..], &sig, g, &JUBJUB)
            })
            .collect())
    }

    /// the binding verification key as accept_sapling / accept_sapling_final form it:
    /// sum of spend cvs - sum of output cvs - valueBalance * G_v; status 1 when a cv does not
    /// decode or is of small order (its description fails first), 2 for InvalidBalanceValue
    fn sapling_bvk(&self, txs: &[(Vec<[u8; 32]>, Vec<[u8; 32]>, i64)]) -> Result<Vec<(u8, [u8; 32])>, GpuError> {
        Ok(txs
            .par_iter()
            .map(|(spends, outputs, vb)| {
                let mut total = edwards::Point::zero();
                for cv in spends {
                    match read_point(cv) {
                        Some(p) => total = total.add(&p, &JUBJUB),
                        None => return (1u8, [0u8; 32]),
                    }
                }
                for cv in outputs {
                    match read_point(cv) {
                        Some(p) => total = total.add(&p.negate(), &JUBJUB),
                        None => return (1u8, [0u8; 32]),
                    }
                }
                let abs = match vb.checked_abs() {
                    Some(a) => a as u64,
                    None => return (2u8, [0u8; 32]),
                };
                let mut bal: Point = JUBJUB
                    .generator(FixedGenerators::ValueCommitmentValue)
                    .mul(FsRepr::from(abs), &JUBJUB)
                    .into();
                if vb.is_negative() {
                    bal = bal.negate();
                }
                let bvk = total.add(&bal.negate(), &JUBJUB);
                let mut out = [0u8; 32];
                bvk.write(&mut out[..]).expect("bvk is 32 bytes");
                (0u8, out)
            })
            .collect())
    }
}
