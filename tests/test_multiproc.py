"""CPU tier: the N>1 protocol of zebra_amd.dist (all-gather of 576-byte Miller partials,
ONE final exponentiation on rank 0, verdict broadcast) with world_size 2 over gloo.
Partials are formed by the oracle (oracle.groth16.batch_partial, the same product the GPU
forms per shard); the check is the oracle's final exponentiation of their product."""
import os
import socket

import pytest

from tests.conftest import ROOT, load_golden

VK_FILES = {0: "sapling-spend-verifying-key.json", 1: "sapling-output-verifying-key.json",
            2: "sprout-groth16-key.json"}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _items(entries):
    from oracle import groth16 as G
    out = []
    for e in entries:
        out.append((e["kind"], bytes.fromhex(e["proof"]),
                    [int.from_bytes(bytes.fromhex(x), "little") for x in e["inputs"]],
                    G.batch_r(bytes.fromhex(e["r"]))))
    return out


def _worker(rank, world, port, shards, want, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from oracle import bls12_381 as B, groth16 as G
    from zebra_amd.dist import combine_partials, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pvks = {k: G.prepare_verifying_key(G.load_vk_json(open(os.path.join(ROOT, "zebra_amd", "res", f)).read()))
                for k, f in VK_FILES.items()}
        lo, hi = shard_range(len(shards), world, rank)
        assert (lo, hi) == (rank, rank + 1)
        part = B.f12_to_bytes(G.batch_partial(pvks, shards[rank]))

        def check(parts):
            f = B.F12_ONE
            for p in parts:
                f = B.f12_mul(f, B.f12_from_bytes(p))
            return B.final_exponentiation(f) == B.F12_ONE

        ok = combine_partials(part, check, world, rank, "cpu")
        # a rank whose own partial fails its own check holds the failing shard
        own = check([part])
        q.put((rank, ok, own))
        assert ok == want
    finally:
        dist.destroy_process_group()


def _run(shards, want):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, shards, want, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    res = sorted(q.get(timeout=5) for _ in range(2))
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return res


@pytest.fixture(scope="module")
def batch():
    return load_golden("batch64.json")["items"]


def test_two_ranks_all_valid(batch):
    good = [e for e in batch if e["status"] == 0]
    res = _run([_items(good[0:2]), _items(good[2:4])], True)
    assert [r[1] for r in res] == [True, True]
    assert [r[2] for r in res] == [True, True]


def test_two_ranks_one_bad_shard(batch):
    good = [e for e in batch if e["status"] == 0]
    bad = [e for e in batch if e["status"] == 3]
    res = _run([_items(good[0:2]), _items([bad[0], good[2]])], False)
    assert [r[1] for r in res] == [False, False]       # verdict broadcast to both ranks
    assert [r[2] for r in res] == [True, False]        # rank 1's own partial localises the failure


class _FakeCtx:
    """stands in for a zg context: batch b's partial is a deterministic 576-byte string"""

    def __init__(self, rank, log):
        self.rank, self.log, self.batch, self.busy = rank, log, None, False

    def launch(self, b):
        assert not self.busy, "context relaunched while its batch is in flight"
        self.busy, self.batch = True, b
        self.log.append(("launch", b))

    def partial(self):
        import hashlib
        return (hashlib.sha256(b"%d/%d" % (self.batch, self.rank)).digest() * 18)[:576]


def _pipeline_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from zebra_amd.dist import combine_partials, run_pipelined
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        log = []
        ctxs = [_FakeCtx(rank, log) for _ in range(3)]
        nxt = [0]

        def launch(c):
            c.launch(nxt[0])
            nxt[0] += 1

        def complete(c):
            # the verdict of batch b: rank 0 sees every rank's partial of that same batch
            def check(parts):
                return all(p == _FakeCtx(r, None).__class__.partial(_Probe(c.batch, r)) for r, p in enumerate(parts))
            ok = combine_partials(c.partial(), check, world, rank, "cpu")
            c.busy = False
            log.append(("done", c.batch))
            return c.batch, ok

        res = run_pipelined(ctxs, 7, launch, complete)
        q.put((rank, res, log))
    finally:
        dist.destroy_process_group()


class _Probe:
    def __init__(self, batch, rank):
        self.batch, self.rank = batch, rank


def test_pipelined_batches_world2():
    """bench.py's batches in flight: 7 batches, 3 contexts per rank, gloo world 2 -- every batch's
    gather pairs the two ranks' partials of that same batch, in order, and no context is
    relaunched while busy"""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipeline_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    got = sorted(q.get(timeout=5) for _ in range(2))
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for rank, res, log in got:
        assert res == [(b, True) for b in range(7)]
        assert log[:3] == [("launch", 0), ("launch", 1), ("launch", 2)]
        assert [e for e in log if e[0] == "done"] == [("done", b) for b in range(7)]


def _deferred_worker(rank, world, port, q, coalesce=False):
    import sys
    import threading
    import time
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from zebra_amd.dist import combine_partials, gather_partials, run_pipelined_deferred
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        log, bad = [], 4   # batch 4's partial on rank 1 is corrupted: that batch's verdict is false
        ctxs = [_FakeCtx(rank, log) for _ in range(3)]
        nxt = [0]

        def launch(c):
            c.launch(nxt[0])
            nxt[0] += 1

        def harvest(c):
            part = c.partial() if not (c.batch == bad and rank == 1) else bytes(576)
            c.busy = False
            log.append(("harvest", c.batch))
            return (c.batch, part), ["provisional", c.batch]

        def verdict(item):
            b, part = item
            assert threading.current_thread() is not threading.main_thread()
            log.append(("verdict", b))

            def check(parts):
                return all(p == _FakeCtx.partial(_Probe(b, r)) for r, p in enumerate(parts))
            return combine_partials(part, check, world, rank, "cpu")

        def redo(s):
            log.append(("redo", s))
            return ["bisected", s]

        def gather(item):   # the ordered stage: the all-gather of batch b's partials
            b, part = item
            log.append(("verdict", b))
            return b, gather_partials(part, world, rank, "cpu")

        def verdict_many(sets):   # the coalescing checker: several batches' gathered sets per call
            log.append(("check", [b for b, _ in sets]))
            time.sleep(0.01)
            return [all(p == _FakeCtx.partial(_Probe(b, r)) for r, p in enumerate(parts)) for b, parts in sets]

        if coalesce:
            res = run_pipelined_deferred(ctxs, 7, launch, harvest, None, redo, gather=gather,
                                         verdict_many=verdict_many)
        else:
            res = run_pipelined_deferred(ctxs, 7, launch, harvest, verdict, redo)
        q.put((rank, res, log))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("coalesce", [False, True], ids=["one-verdict-thread", "gather-then-coalesced-checks"])
def test_deferred_verdicts_world2(coalesce):
    """bench.py's default schedule: a context is relaunched right after its partial and statuses
    are read, the verdicts (the all-gather + check) run on one worker thread in batch order on
    both ranks, and a batch with a false verdict gets redo()'s statuses on every rank.
    coalesce (bench.py under torch.distributed, round 6): the all-gathers stay in batch order on the
    ordered thread, the checks of the batches gathered meanwhile are taken together, every batch once"""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_deferred_worker, args=(r, 2, port, q, coalesce)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    got = sorted(q.get(timeout=5) for _ in range(2))
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for rank, res, log in got:
        assert res == [(b != 4, ["provisional" if b != 4 else "bisected", b]) for b in range(7)]
        assert [e for e in log if e[0] == "verdict"] == [("verdict", b) for b in range(7)]
        assert [e for e in log if e[0] == "harvest"] == [("harvest", b) for b in range(7)]
        assert [e for e in log if e[0] == "redo"] == [("redo", 4)]
        if coalesce:
            checked = [b for e in log if e[0] == "check" for b in e[1]]
            assert checked == list(range(7))
        # the 4th launch (batch 3) reuses the first context right after batch 0's harvest,
        # without waiting for batch 0's verdict (the worker thread logs verdicts concurrently)
        main = [e for e in log if e[0] not in ("verdict", "check")]
        assert main.index(("launch", 3)) == main.index(("harvest", 0)) + 1


def _multi_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from zebra_amd.dist import combine_partials
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = [bytes([16 * rank + j]) * 576 for j in range(3)]
        seen = []
        ok = combine_partials(mine, lambda parts: seen.extend(parts) or True, world, rank, "cpu")
        q.put((rank, ok, [p[0] for p in seen]))
    finally:
        dist.destroy_process_group()


def test_two_ranks_several_shards_each():
    """a rank holding k shards sends its k partials in the same single all-gather; every rank
    sees all world x k of them, rank-major (the order of the contiguous shards)"""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_multi_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    res = sorted(q.get(timeout=5) for _ in range(2))
    assert all(p.exitcode == 0 for p in procs)
    for _, ok, order in res:
        assert ok and order == [0, 1, 2, 16, 17, 18]
