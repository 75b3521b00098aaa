//! verification/src/gpu/writer.rs -- import-window batching of `BlocksWriter::append_block`
//!, a transcription of zebra_amd/blocks_writer.py
//! (`DeferredBlocksWriter`, which tests/test_blocks_writer.py checks against the reference's
//! sequential writer on the reference's own writer scenarios and randomized streams).
//!
//! The reference imports one block at a time (sync/src/blocks_writer.rs:63-90): a known block is
//! skipped; a block with an unknown parent goes to the orphan pool (more than
//! MAX_ORPHANED_BLOCKS -> TooManyOrphanBlocks); otherwise the block and its orphan descendants
//! are verified in order and inserted, and the first error ends the call. Here each block's
//! non-proof checks run when it is appended (against the chain as it will be once the window's
//! earlier blocks are accepted), its transactions join a window, and the window's proofs and
//! Sapling signatures are verified by ONE `collect::verify_block` call when it holds
//! `window_proofs` proofs, when a block's own checks fail, or on `flush`. Blocks are inserted
//! only after their window verified, in append order, up to the first failing block, whose
//! error is returned; the window's later blocks are dropped.
//!
//! Contract (as in the Python original): identical storage and first error for a caller that
//! stops at the first error -- the reference's only caller, zebra/commands/import.rs:20-28,
//! returns on any Err.
use std::collections::{HashMap, HashSet, VecDeque};

use super::collect::{verify_block, Backend, Tx, TxError};
use super::GpuError;

/// sync/src/blocks_writer.rs:20
pub const MAX_ORPHANED_BLOCKS: usize = 1024;

/// sync::Error, plus the backend failure of the window's verification
#[derive(Debug)]
pub enum WriterError {
    TooManyOrphanBlocks,
    /// the first failing block's error: its own checks, or (tx index, collector error)
    Verification(String),
    Database(String),
    /// the window could not be verified (GPU error): nothing of the window was inserted and the
    /// window is still held by the writer; the caller re-runs it on another backend
    /// (`DeferredBlocksWriter::flush_with`, e.g. the CPU backend of cpu.rs) or aborts the import
    Backend(GpuError),
}

/// What the writer needs of an indexed block.
pub trait ImportBlock {
    fn hash(&self) -> [u8; 32];
    fn parent(&self) -> [u8; 32];
    /// ChainVerifier::check's header / block / context-free transaction checks and the
    /// BlockAcceptor / HeaderAcceptor checks (chain_verifier.rs:32-132) against the chain in
    /// which `known` blocks exist; Err(text) fails the block before its transactions.
    fn precheck(&self, known: &dyn Fn(&[u8; 32]) -> bool) -> Result<(), String>;
    /// the collector view of the transactions (the caller's non-proof outcomes filled in)
    fn txs(&self) -> &[Tx];
}

/// storage::Store as the writer uses it
pub trait BlockStore<B> {
    fn contains(&self, hash: &[u8; 32]) -> bool;
    fn insert(&mut self, block: B) -> Result<(), String>;
}

fn n_proofs(txs: &[Tx]) -> usize {
    txs.iter().map(|t| t.joinsplits.len() + t.spends.len() + t.outputs.len()).sum()
}

/// OrphanBlocksPool (sync/src/utils/orphan_blocks_pool.rs): by parent hash, insertion ordered
struct OrphanPool<B> {
    by_parent: HashMap<[u8; 32], Vec<B>>,
    len: usize,
}

impl<B: ImportBlock> OrphanPool<B> {
    fn insert(&mut self, b: B) {
        self.by_parent.entry(b.parent()).or_default().push(b);
        self.len += 1;
    }

    /// every descendant of `h`, parents before children
    fn remove_for_parent(&mut self, h: [u8; 32]) -> Vec<B> {
        let mut out = Vec::new();
        let mut queue = VecDeque::from(vec![h]);
        while let Some(p) = queue.pop_front() {
            if let Some(kids) = self.by_parent.remove(&p) {
                for b in kids {
                    self.len -= 1;
                    queue.push_back(b.hash());
                    out.push(b);
                }
            }
        }
        out
    }
}

pub struct DeferredBlocksWriter<'a, S: BlockStore<B>, B: ImportBlock, V: Backend> {
    storage: S,
    backend: &'a V,
    orphans: OrphanPool<B>,
    window: Vec<B>,
    pending: HashSet<[u8; 32]>,
    window_proofs: usize,
}

impl<'a, S: BlockStore<B>, B: ImportBlock, V: Backend> DeferredBlocksWriter<'a, S, B, V> {
    /// window_proofs: proofs per window (65,536 fills one GPU batch at the headline size)
    pub fn new(storage: S, backend: &'a V, window_proofs: usize) -> Self {
        DeferredBlocksWriter {
            storage,
            backend,
            orphans: OrphanPool { by_parent: HashMap::new(), len: 0 },
            window: Vec::new(),
            pending: HashSet::new(),
            window_proofs: window_proofs.max(1),
        }
    }

    pub fn storage(&self) -> &S {
        &self.storage
    }

    fn known(&self, h: &[u8; 32]) -> bool {
        self.pending.contains(h) || self.storage.contains(h)
    }

    /// BlocksWriter::append_block with the proofs deferred to the window's one batch
    pub fn append_block(&mut self, block: B) -> Result<(), WriterError> {
        if self.known(&block.hash()) {
            return Ok(());
        }
        if !self.known(&block.parent()) {
            self.orphans.insert(block);
            if self.orphans.len > MAX_ORPHANED_BLOCKS {
                self.flush()?; // blocks appended before keep their verdicts first
                return Err(WriterError::TooManyOrphanBlocks);
            }
            return Ok(());
        }
        let h = block.hash();
        let mut queue = vec![block];
        queue.extend(self.orphans.remove_for_parent(h));
        for b in queue {
            let pre = {
                let known = |x: &[u8; 32]| self.pending.contains(x) || self.storage.contains(x);
                b.precheck(&known)
            };
            if let Err(e) = pre {
                // an earlier block of the window may hold the first error: verify those first
                self.flush()?;
                return Err(WriterError::Verification(e));
            }
            self.pending.insert(b.hash());
            self.window.push(b);
            if self.window.iter().map(|x| n_proofs(x.txs())).sum::<usize>() >= self.window_proofs {
                self.flush()?;
            }
        }
        Ok(())
    }

    /// verify the window, insert its blocks up to the first failing one, return its error
    pub fn flush(&mut self) -> Result<(), WriterError> {
        let backend = self.backend;
        self.flush_on(backend)
    }

    /// after `WriterError::Backend`: verify the window the writer still holds on another backend
    /// (the CPU backend of cpu.rs), with the same insertion and first-error contract as `flush`
    pub fn flush_with<W: Backend>(&mut self, other: &W) -> Result<(), WriterError> {
        self.flush_on(other)
    }

    fn flush_on<W: Backend>(&mut self, backend: &W) -> Result<(), WriterError> {
        if self.window.is_empty() {
            return Ok(());
        }
        // the window's transactions, flattened in block order (one verify_block call)
        let mut owner = Vec::new();
        let mut flat: Vec<&Tx> = Vec::new();
        for (bi, b) in self.window.iter().enumerate() {
            for (ti, t) in b.txs().iter().enumerate() {
                flat.push(t);
                owner.push((bi, ti));
            }
        }
        // verify BEFORE the window is taken: on a backend failure the window and the pending
        // set stay as they were, so `flush_with` (or a later flush) can still verify them
        let res: Option<(usize, TxError)> = if flat.is_empty() {
            None
        } else {
            let txs: Vec<Tx> = flat.into_iter().map(clone_tx).collect();
            verify_block(backend, &txs).map_err(WriterError::Backend)?
        };
        let blocks = std::mem::take(&mut self.window);
        self.pending.clear();
        let (fail_block, err) = match res {
            None => (blocks.len(), None),
            Some((idx, e)) => {
                let (bi, ti) = owner[idx];
                (bi, Some(format!("transaction {}: {:?}", ti, e)))
            }
        };
        for b in blocks.into_iter().take(fail_block) {
            self.storage.insert(b).map_err(WriterError::Database)?;
        }
        match err {
            Some(e) => Err(WriterError::Verification(e)),
            None => Ok(()),
        }
    }
}

fn clone_tx(t: &Tx) -> Tx {
    t.clone()
}

#[cfg(test)]
mod tests {
    //! The Python mirror's test_backend_failure_keeps_the_window (tests/test_blocks_writer.py):
    //! a backend that fails twice leaves the window held and the storage untouched; flush_with on
    //! another backend then gives the sequential writer's storage and first error.
    use super::super::collect::JoinSplit;
    use super::super::ffi::{ZG_STATUS_OK, ZG_STATUS_VERIFY_FAILED};
    use super::super::Item;
    use super::*;
    use std::cell::Cell;

    #[derive(Clone)]
    struct TBlock {
        h: [u8; 32],
        p: [u8; 32],
        txs: Vec<Tx>,
    }
    impl ImportBlock for TBlock {
        fn hash(&self) -> [u8; 32] {
            self.h
        }
        fn parent(&self) -> [u8; 32] {
            self.p
        }
        fn precheck(&self, _known: &dyn Fn(&[u8; 32]) -> bool) -> Result<(), String> {
            Ok(())
        }
        fn txs(&self) -> &[Tx] {
            &self.txs
        }
    }

    #[derive(Default)]
    struct TStore {
        order: Vec<[u8; 32]>,
        set: HashSet<[u8; 32]>,
    }
    impl BlockStore<TBlock> for TStore {
        fn contains(&self, h: &[u8; 32]) -> bool {
            self.set.contains(h)
        }
        fn insert(&mut self, b: TBlock) -> Result<(), String> {
            self.set.insert(b.h);
            self.order.push(b.h);
            Ok(())
        }
    }

    /// statuses from the proof's first byte (0xEE: VERIFY_FAILED); the first `fails` calls fail
    struct Flaky {
        fails: Cell<u32>,
    }
    impl Backend for Flaky {
        fn verify(&self, items: &[Item]) -> Result<Vec<u8>, GpuError> {
            if self.fails.get() > 0 {
                self.fails.set(self.fails.get() - 1);
                return Err(GpuError { code: -1, message: "device lost".to_string() });
            }
            Ok(items.iter().map(|it| if it.proof[0] == 0xEE { ZG_STATUS_VERIFY_FAILED } else { ZG_STATUS_OK }).collect())
        }
        fn pghr13_verify(&self, items: &[([u8; 296], Vec<[u8; 32]>)]) -> Result<Vec<u8>, GpuError> {
            Ok(vec![ZG_STATUS_OK; items.len()])
        }
        fn redjubjub_verify(&self, items: &[([u8; 32], [u8; 64], [u8; 64], u8)]) -> Result<Vec<bool>, GpuError> {
            Ok(vec![true; items.len()])
        }
        fn sapling_bvk(&self, txs: &[(Vec<[u8; 32]>, Vec<[u8; 32]>, i64)]) -> Result<Vec<(u8, [u8; 32])>, GpuError> {
            Ok(vec![(0, [0u8; 32]); txs.len()])
        }
    }

    /// block i + 1 on parent i: one transaction with one Groth16 JoinSplit
    fn block(i: u8, bad: bool) -> TBlock {
        let mut proof = [0u8; 192];
        proof[0] = if bad { 0xEE } else { 0x01 };
        let js = JoinSplit {
            anchor: [i; 32],
            random_seed: [1; 32],
            nullifiers: [[2; 32], [3; 32]],
            macs: [[4; 32], [5; 32]],
            commitments: [[6; 32], [7; 32]],
            vpub_old: 0,
            vpub_new: 0,
            groth_proof: Some(proof),
            pghr_proof: None,
            pghr_ok: None,
            tree_error: None,
        };
        let tx = Tx { js_pubkey: Some([9; 32]), js_sig_ok: true, joinsplits: vec![js], ..Default::default() };
        TBlock { h: [i + 1; 32], p: [i; 32], txs: vec![tx] }
    }

    #[test]
    fn backend_failure_keeps_the_window() {
        // genesis [0; 32] stored; blocks 1..=6 with block 4's proof failing
        let blocks: Vec<TBlock> = (0u8..6).map(|i| block(i, i == 3)).collect();
        let mut st = TStore::default();
        st.set.insert([0u8; 32]);
        let gpu = Flaky { fails: Cell::new(2) };
        let cpu = Flaky { fails: Cell::new(0) };
        let mut w = DeferredBlocksWriter::new(st, &gpu, 1 << 20);
        for b in blocks.iter().cloned() {
            w.append_block(b).unwrap();
        }
        for _ in 0..2 {
            match w.flush() {
                Err(WriterError::Backend(e)) => assert_eq!(e.message, "device lost"),
                other => panic!("expected a backend failure, got {:?}", other.err()),
            }
            assert!(w.storage().order.is_empty());
            assert_eq!(w.window.len(), 6);
            assert!(blocks.iter().all(|b| w.known(&b.h)));
        }
        // the sequential writer's outcome: blocks 1..=3 inserted, block 4's JoinSplit reported
        match w.flush_with(&cpu) {
            Err(WriterError::Verification(e)) => {
                assert_eq!(e, format!("transaction 0: {:?}", TxError::InvalidJoinSplit(0)))
            }
            other => panic!("expected block 4's verification error, got {:?}", other.err()),
        }
        let want: Vec<[u8; 32]> = (1u8..4).map(|i| [i; 32]).collect();
        assert_eq!(w.storage().order, want);
        assert!(w.window.is_empty());
    }
}
