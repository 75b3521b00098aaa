"""Import-window batching (zebra_amd/blocks_writer.py): the deferred writer,
which verifies the proofs of many blocks in one batch, is observably identical to the reference's
one-block-at-a-time BlocksWriter::append_block (sync/src/blocks_writer.rs:63-90) -- same blocks in
storage in the same order, same first error -- including the reference's own test scenarios
(:174-238: append, TooManyOrphanBlocks at MAX_ORPHANED_BLOCKS + 1, out-of-order parent) and
randomized block streams with failing proofs, failing signatures, failing block checks and
orphans. CPU tier: the C++ bellman restatement verifies the proofs; GPU tier: the product."""
import random

import pytest

from tests.test_collector import SRC_TX, fields, make_tx


@pytest.fixture(scope="module")
def cpu_verify():
    from tests import cpulib
    L = cpulib.load()

    def verify(proofs, kinds, inputs, n_inputs):
        return cpulib.verify(L, proofs, kinds, inputs, n_inputs, threads=8)[0]
    return verify


def chain(n, seed, F, bad_proof=(), bad_pre=(), orphan_swaps=0):
    """n blocks b1..bn on genesis "g"; each block 1-3 of the reference's real transactions.
    bad_proof: block indices with one corrupted proof; bad_pre: blocks failing their own checks"""
    from zebra_amd.blocks_writer import Block
    rng = random.Random(seed)
    names = list(SRC_TX.values())
    blocks, parent = [], "g"
    for i in range(n):
        txs = [make_tx(rng.choice(names), F) for _ in range(rng.randint(1, 3))]
        if i in bad_proof:
            t = rng.randrange(len(txs))
            tx = txs[t]
            if tx.joinsplits:
                p = tx.joinsplits[0].zkproof
                tx.joinsplits[0].zkproof = p[144:] + p[48:144] + p[:48]
            elif tx.spends:
                tx.spends[0].nullifier = bytes(32)
            else:
                c = bytearray(tx.outputs[0].zkproof)
                c[10] ^= 1
                tx.outputs[0].zkproof = bytes(c)
        pre = (lambda w, i=i: "BadMerkleRoot@%d" % i) if i in bad_pre else None
        h = "b%d" % (i + 1)
        blocks.append(Block(h, parent, txs, pre))
        parent = h
    order = list(range(n))
    for _ in range(orphan_swaps):   # deliver some blocks before their parents
        a = rng.randrange(n - 1)
        order[a], order[a + 1] = order[a + 1], order[a]
    return [blocks[k] for k in order]


def run(writer_cls, blocks, **kw):
    from zebra_amd.blocks_writer import MemoryStorage, WriterError
    st = MemoryStorage("g")
    w = writer_cls(st, **kw)
    err = None
    try:
        for b in blocks:
            w.append_block(b)
        w.flush()
    except WriterError as e:
        err = e
    return st.blocks, err


def seq_kw(cpu_verify):
    from zebra_amd.collector import verify_block

    def check(b):
        pre = b.precheck(None) if b.precheck else None
        return pre if pre is not None else verify_block(b.txs, verify=cpu_verify)
    return {"check": check}


def deferred_kw(cpu_verify, window):
    from zebra_amd.collector import verify_block
    return {"verify_window": lambda txs: verify_block(txs, verify=cpu_verify), "window_proofs": window}


def test_reference_scenarios(cpu_verify):
    from zebra_amd.blocks_writer import (MAX_ORPHANED_BLOCKS, Block, DeferredBlocksWriter, SequentialBlocksWriter,
                                         WriterError)
    F = fields()
    # blocks_writer_appends_blocks / append_to_existing_db
    blocks = chain(1, 1, F)
    for cls, kw in ((SequentialBlocksWriter, seq_kw(cpu_verify)), (DeferredBlocksWriter, deferred_kw(cpu_verify, 64))):
        assert run(cls, blocks, **kw) == (["g", "b1"], None)
    # blocks_writer_verification_error: MAX + 2 blocks delivered without b1 -> TooManyOrphanBlocks
    orphans = [Block("o%d" % i, "o%d" % (i - 1), []) for i in range(2, MAX_ORPHANED_BLOCKS + 3)]
    for cls, kw in ((SequentialBlocksWriter, seq_kw(cpu_verify)), (DeferredBlocksWriter, deferred_kw(cpu_verify, 64))):
        blocks_, err = run(cls, orphans, **kw)
        assert blocks_ == ["g"] and err == WriterError("TooManyOrphanBlocks")
    # blocks_writer_out_of_order_block: a block failing its own checks is not inserted
    bad = chain(3, 2, F, bad_pre={1})
    a = run(SequentialBlocksWriter, bad, **seq_kw(cpu_verify))
    b = run(DeferredBlocksWriter, bad, **deferred_kw(cpu_verify, 64))
    assert a == b and a[0] == ["g", "b1"] and a[1].kind == "Verification"


@pytest.mark.parametrize("seed", range(6))
def test_deferred_equals_sequential(cpu_verify, seed):
    from zebra_amd.blocks_writer import DeferredBlocksWriter, SequentialBlocksWriter
    F = fields()
    rng = random.Random(100 + seed)
    n = 24
    bad_proof = set(rng.sample(range(n), rng.randint(0, 2)))
    bad_pre = set(rng.sample(range(n), rng.randint(0, 1)))
    blocks = chain(n, seed, F, bad_proof, bad_pre, orphan_swaps=rng.randint(0, 4))
    want = run(SequentialBlocksWriter, blocks, **seq_kw(cpu_verify))
    for window in (1, 7, 10 ** 6):
        got = run(DeferredBlocksWriter, blocks, **deferred_kw(cpu_verify, window))
        assert got == want, (seed, window, bad_proof, bad_pre)


@pytest.mark.gpu
def test_deferred_writer_on_gpu():
    """a 40-block stream through the deferred writer with the product collector (one GPU batch per
    window): the same outcome as the sequential writer on the same verifier"""
    from zebra_amd import Context
    from zebra_amd.blocks_writer import DeferredBlocksWriter, SequentialBlocksWriter
    from zebra_amd.collector import verify_block
    F = fields()
    blocks = chain(40, 9, F, bad_proof={27}, orphan_swaps=3)
    ctx = Context(device=0, max_batch=4096)
    try:
        def check(b):
            return verify_block(b.txs, ctx=ctx)
        want = run(SequentialBlocksWriter, blocks, check=check)
        got = run(DeferredBlocksWriter, blocks, ctx=ctx, window_proofs=64)
        assert got == want and got[1] is not None and got[0][-1] == "b27"
    finally:
        ctx.close()


def fork_stream(n, seed, F, bad_proof=(), bad_pre=()):
    """a main chain b1..bn plus sibling fork blocks f<i> (parent b<i>) and a fork child f<i>c,
    delivered a few blocks after their parent; failures on main or fork blocks"""
    from zebra_amd.blocks_writer import Block
    rng = random.Random(seed)
    names = list(SRC_TX.values())
    main = chain(n, seed, F, bad_proof=bad_proof, bad_pre=bad_pre)
    out = list(main)
    for i in sorted(rng.sample(range(1, n - 2), 3)):
        txs = [make_tx(rng.choice(names), F) for _ in range(rng.randint(1, 2))]
        if ("f%d" % i) in bad_proof:
            txs[0].outputs.append(make_tx(["O1"], F).outputs[0])
            c = bytearray(txs[0].outputs[-1].zkproof)
            c[10] ^= 1
            txs[0].outputs[-1].zkproof = bytes(c)
        fb = Block("f%d" % i, "b%d" % i, txs)
        fc = Block("f%dc" % i, "f%d" % i, [make_tx(rng.choice(names), F)])
        at = out.index(main[min(n - 1, i + 1)]) + 1
        out[at:at] = [fb, fc]
    return out


@pytest.mark.parametrize("seed", range(4))
def test_deferred_equals_sequential_with_forks(cpu_verify, seed):
    """sibling forks in the stream: identical storage order and first error, with
    the failure on the main chain, on a fork block, or nowhere"""
    from zebra_amd.blocks_writer import DeferredBlocksWriter, SequentialBlocksWriter
    F = fields()
    rng = random.Random(300 + seed)
    n = 16
    bad = {0: (), 1: {rng.randrange(n)}, 2: set(), 3: {rng.randrange(n)}}[seed]
    stream = fork_stream(n, seed, F, bad_proof=bad)
    if seed == 2:   # a failing fork block
        stream = fork_stream(n, seed, F, bad_proof={"f%d" % int(b.hash[1:]) for b in stream
                                                   if b.hash.startswith("f") and not b.hash.endswith("c")})
    want = run(SequentialBlocksWriter, stream, **seq_kw(cpu_verify))
    assert any(h.startswith("f") for h in want[0]) or want[1] is not None
    for window in (1, 5, 10 ** 6):
        assert run(DeferredBlocksWriter, stream, **deferred_kw(cpu_verify, window)) == want, (seed, window)


def test_backend_failure_keeps_the_window(cpu_verify):
    """a window whose verification raises (a GPU error) is neither dropped nor
    inserted; the writer still holds it, so a retried flush (here: the backend recovers after
    two failures) ends with exactly the sequential writer's storage and first error"""
    from zebra_amd.blocks_writer import DeferredBlocksWriter, MemoryStorage, SequentialBlocksWriter
    from zebra_amd.collector import verify_block
    F = fields()
    blocks = chain(12, 5, F, bad_proof={9}, orphan_swaps=2)
    want = run(SequentialBlocksWriter, blocks, **seq_kw(cpu_verify))
    fails = {"left": 2}

    class GpuError(RuntimeError):
        pass

    def flaky(txs):
        if fails["left"]:
            fails["left"] -= 1
            raise GpuError("device lost")
        return verify_block(txs, verify=cpu_verify)
    st = MemoryStorage("g")
    w = DeferredBlocksWriter(st, verify_window=flaky, window_proofs=10 ** 6)
    for b in blocks:
        w.append_block(b)
    held = list(w.window)
    for _ in range(2):
        with pytest.raises(GpuError):
            w.flush()
        assert w.window == held and st.blocks == ["g"]
        assert all(w._known(b.hash) for b in held)
    err = None
    try:
        w.flush()
    except Exception as e:  # WriterError
        err = e
    assert (st.blocks, err) == want
