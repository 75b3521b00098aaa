"""Import-window batching of block acceptance.

The reference imports blocks one at a time (sync/src/blocks_writer.rs:63-90): a block already
in storage is skipped; a block whose parent is unknown goes to the orphan pool (at most
MAX_ORPHANED_BLOCKS = 1024, else TooManyOrphanBlocks); otherwise the block and every orphan
descendant are verified in order and inserted, and the first verification error ends the call.
A real block carries few Groth16 proofs, so a GPU batch per block would be tiny.

DeferredBlocksWriter keeps exactly that observable behaviour -- the same blocks end up in
storage, in the same order, and the same first error is reported -- while the Groth16 proofs and
Sapling signatures of many consecutive blocks are verified together: each block's other checks
run when it is appended (against a pending view of the chain that already includes the blocks
appended before it), its proof-carrying transactions join a window, and the window is verified
with ONE zebra_amd.collector.verify_block call when it holds `window_proofs` proofs, when a
block's own checks fail (the blocks before it may hold an earlier error), or on flush(). Blocks
are inserted into storage only once their window has verified, in chain order, up to the first
failing block; that block's error is raised and the window's later blocks are dropped, just as
the sequential writer would never have inserted them.

Error precedence inside a block is the collector's (accept_transaction.rs:68-84,
accept_chain.rs:76-81: the lowest failing transaction wins); across blocks the lowest block wins.

Contract: the equivalence holds for a caller that stops at the first error, as the reference's
only caller does (zebra/commands/import.rs:20-28 returns on any Err from append_block). The
error of a block surfaces when its window is verified -- at that block's append_block or at a
later append_block / flush -- and the window's blocks after the failing one are dropped,
including blocks on a sibling fork that the sequential writer would have inserted had the caller
kept appending after the error. Forks inside a window are otherwise handled like the sequential
writer (tests/test_blocks_writer.py: sibling forks with and without failures).
"""
from collections import OrderedDict

from . import collector

MAX_ORPHANED_BLOCKS = 1024


class WriterError(Exception):
    """sync::Error: kind is "TooManyOrphanBlocks" | "Verification" | "Database"."""

    def __init__(self, kind, detail=None):
        super().__init__("%s%s" % (kind, "" if detail is None else ": %r" % (detail,)))
        self.kind = kind
        self.detail = detail

    def __eq__(self, other):
        return isinstance(other, WriterError) and (self.kind, self.detail) == (other.kind, other.detail)

    def __hash__(self):
        return hash((self.kind, repr(self.detail)))


class Block:
    """an indexed block: its hash, its parent's hash and the collector view of its transactions.
    precheck(writer) -> None | error: the block's checks that precede every transaction
    acceptor (chain_verifier.rs:32-132: ChainVerifier::check -- header, block and the
    context-free transaction checks -- then BlockAcceptor / HeaderAcceptor), run against the chain
    as it will be once every block appended before this one is accepted. The transaction-level
    outcomes that are not proofs (scripts, tree roots, nullifiers, ...) are set on the collector
    Tx objects by the same caller."""

    def __init__(self, hash, parent, txs, precheck=None):
        self.hash, self.parent, self.txs, self.precheck = hash, parent, txs, precheck

    def n_proofs(self):
        return sum(len(t.joinsplits) + len(t.spends) + len(t.outputs) for t in self.txs)


class _OrphanPool:
    """OrphanBlocksPool (sync/src/utils/orphan_blocks_pool.rs): orphans by parent hash, insertion
    ordered; remove_blocks_for_parent returns every descendant, parents before children."""

    def __init__(self):
        self.by_parent = OrderedDict()

    def __len__(self):
        return sum(len(v) for v in self.by_parent.values())

    def insert(self, block):
        self.by_parent.setdefault(block.parent, OrderedDict())[block.hash] = block

    def remove_for_parent(self, h):
        out, queue = [], [h]
        while queue:
            p = queue.pop(0)
            kids = self.by_parent.pop(p, None)
            if kids:
                for b in kids.values():
                    out.append(b)
                    queue.append(b.hash)
        return out


class SequentialBlocksWriter:
    """BlocksWriter::append_block as the reference runs it: every block verified on its own as
    it is appended (check(block) -> None | error), then inserted."""

    def __init__(self, storage, check):
        self.storage, self.check, self.orphans = storage, check, _OrphanPool()

    def append_block(self, block):
        if self.storage.contains(block.hash):
            return
        if not self.storage.contains(block.parent):
            self.orphans.insert(block)
            if len(self.orphans) > MAX_ORPHANED_BLOCKS:
                raise WriterError("TooManyOrphanBlocks")
            return
        for b in [block] + self.orphans.remove_for_parent(block.hash):
            err = self.check(b)
            if err is not None:
                raise WriterError("Verification", err)
            self.storage.insert(b)

    def flush(self):
        return None


class DeferredBlocksWriter:
    """The same behaviour with the proofs of a window verified in one batch.

    verify_window(txs) -> None | (tx_index, error): the collector over the window's flattened
    transactions (default: collector.verify_block with `ctx`, i.e. one GPU batch)."""

    def __init__(self, storage, ctx=None, verify_window=None, window_proofs=65536):
        self.storage = storage
        self.orphans = _OrphanPool()
        self.window = []          # pending blocks in chain order (prechecked, not inserted)
        self.pending = set()      # their hashes: children may build on them
        self.window_proofs = window_proofs
        if verify_window is None:
            def verify_window(txs):
                return collector.verify_block(txs, ctx=ctx)
        self.verify_window = verify_window

    def _known(self, h):
        return h in self.pending or self.storage.contains(h)

    def append_block(self, block):
        if self._known(block.hash):
            return
        if not self._known(block.parent):
            self.orphans.insert(block)
            if len(self.orphans) > MAX_ORPHANED_BLOCKS:
                self.flush()               # blocks appended before keep their verdicts first
                raise WriterError("TooManyOrphanBlocks")
            return
        for b in [block] + self.orphans.remove_for_parent(block.hash):
            pre = b.precheck(self) if b.precheck else None
            if pre is not None:
                # the block fails before its transactions are accepted; an earlier block of the
                # window may hold the first error: verify (and accept) those first
                self.flush()
                raise WriterError("Verification", pre)
            self.window.append(b)
            self.pending.add(b.hash)
            if sum(x.n_proofs() for x in self.window) >= self.window_proofs:
                self.flush()

    def flush(self):
        """verify the window, insert its blocks up to the first failing one, raise its error"""
        if not self.window:
            return
        blocks = self.window
        flat, owner = [], []
        for bi, b in enumerate(blocks):
            for ti, t in enumerate(b.txs):
                flat.append(t)
                owner.append((bi, ti))
        # verify BEFORE the window is taken: a backend failure (GPU error) raises with the window
        # and the pending set unchanged, so the caller can retry or re-run it on another backend
        res = self.verify_window(flat) if flat else None
        self.window, self.pending = [], set()
        fail_block = len(blocks)
        err = None
        if res is not None:
            idx, e = res
            fail_block, ti = owner[idx]
            err = (ti, e)
        for b in blocks[:fail_block]:
            self.storage.insert(b)
        if err is not None:
            raise WriterError("Verification", err)


class MemoryStorage:
    """storage::Store stand-in (db::BlockChainDatabase::init_test_chain on MemoryDatabase)"""

    def __init__(self, genesis_hash):
        self.blocks = [genesis_hash]
        self.set = {genesis_hash}

    def contains(self, h):
        return h in self.set

    def insert(self, block):
        assert block.parent in self.set, "inserted before its parent"
        self.blocks.append(block.hash)
        self.set.add(block.hash)
