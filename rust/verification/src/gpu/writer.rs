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
        // set stay as they were, so `retry_on` (or a later flush) can still verify them
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
