"""CPU tier: the host schedule of batches in flight (zebra_amd.dist.run_pipelined_deferred) with
contexts that finish OUT of launch order, as batches sharing a device do. The loop must harvest
whichever batch is ready first, relaunch its context at once, still run the verdicts (the
per-batch collectives) strictly in batch order, and return results in batch order with false
verdicts re-verified by redo."""
import random

import pytest

from zebra_amd.dist import run_pipelined_deferred


class FakeCtx:
    def __init__(self, name, clock):
        self.name, self.clock, self.batch, self.done_at = name, clock, None, None


def test_first_ready_harvest_keeps_batch_order():
    rng = random.Random(5)
    clock = [0]
    ctxs = [FakeCtx(i, clock) for i in range(4)]
    k, bad = 23, {3, 11, 17}
    launched, harvested, verdicts = [], [], []

    def launch(c):
        c.batch = len(launched)
        launched.append(c.batch)
        c.done_at = clock[0] + rng.randint(1, 12)   # finishes after a random number of polls

    def ready(c):
        clock[0] += 1
        return clock[0] >= c.done_at

    def harvest(c):
        harvested.append(c.batch)
        return ("part", c.batch), ["sts", c.batch]

    def verdict(part):
        verdicts.append(part[1])
        return part[1] not in bad

    res = run_pipelined_deferred(ctxs, k, launch, harvest, verdict, lambda s: ["redo", s], ready=ready)
    assert launched == list(range(k))
    assert sorted(harvested) == list(range(k))
    assert harvested != sorted(harvested)          # out-of-order completion was exercised
    assert verdicts == list(range(k))              # collectives in batch order
    for s, (ok, sts) in enumerate(res):
        assert ok == (s not in bad)
        assert sts == (["redo", s] if s in bad else ["sts", s])


def test_without_ready_harvests_oldest_first():
    ctxs = [FakeCtx(i, None) for i in range(3)]
    order = []
    seq = iter(range(100))

    def launch(c):
        c.batch = next(seq)

    def harvest(c):
        order.append(c.batch)
        return ("p", c.batch), c.batch

    res = run_pipelined_deferred(ctxs, 9, launch, harvest, lambda p: True, lambda s: None)
    assert order == list(range(9))
    assert [sts for _, sts in res] == list(range(9))


def test_gather_stage_ordered_checks_overlap():
    """gather / checks (round 6): the exchange runs in batch order on one thread, the final
    exponentiations on a pool -- two of them are in progress at once, results still in batch
    order, false verdicts still re-verified."""
    import threading
    import time
    ctxs = [FakeCtx(i, None) for i in range(3)]
    seq = iter(range(100))
    gathered, active, peak = [], [0], [0]
    lock = threading.Lock()

    def launch(c):
        c.batch = next(seq)

    def harvest(c):
        return ("p", c.batch), c.batch

    def gather(part):
        gathered.append(part[1])
        return [part, part]              # as if two ranks' partials

    def verdict(parts):
        assert len(parts) == 2
        with lock:
            active[0] += 1
            peak[0] = max(peak[0], active[0])
        time.sleep(0.02)
        with lock:
            active[0] -= 1
        return parts[0][1] != 4

    res = run_pipelined_deferred(ctxs, 10, launch, harvest, verdict, lambda s: ("redo", s),
                                 gather=gather, checks=2)
    assert gathered == list(range(10))
    assert peak[0] == 2
    assert [ok for ok, _ in res] == [s != 4 for s in range(10)]
    assert res[4][1] == ("redo", 4) and res[5][1] == 5


def test_coalescing_checker_batches_waiting_sets():
    """verdict_many (round 6): one checker thread takes every gathered set waiting for it and checks
    them in one call -- sets coalesce while a check is running, results stay in batch order, a
    false verdict is still re-verified, every set is checked exactly once."""
    import time
    ctxs = [FakeCtx(i, None) for i in range(4)]
    seq = iter(range(100))
    calls = []

    def launch(c):
        c.batch = next(seq)

    def harvest(c):
        return ("p", c.batch), c.batch

    def gather(part):
        return [part]

    def verdict_many(sets):
        calls.append([p[0][1] for p in sets])
        time.sleep(0.02)                 # a final exponentiation: later batches pile up meanwhile
        return [p[0][1] != 7 for p in sets]

    def verdict(_parts):
        raise AssertionError("the pool is not used with verdict_many")

    res = run_pipelined_deferred(ctxs, 12, launch, harvest, verdict, lambda s: ("redo", s),
                                 gather=gather, verdict_many=verdict_many, max_sets=3)
    assert sorted(b for c in calls for b in c) == list(range(12))
    assert all(c == sorted(c) for c in calls)
    assert max(len(c) for c in calls) > 1 and max(len(c) for c in calls) <= 3
    assert [ok for ok, _ in res] == [s != 7 for s in range(12)]
    assert res[7][1] == ("redo", 7) and res[8][1] == 8


def test_coalescing_checker_failure_reaches_every_batch():
    ctxs = [FakeCtx(i, None) for i in range(2)]
    seq = iter(range(100))

    def launch(c):
        c.batch = next(seq)

    def verdict_many(sets):
        raise RuntimeError("device lost")

    with pytest.raises(RuntimeError, match="device lost"):
        run_pipelined_deferred(ctxs, 4, launch, lambda c: (("p", c.batch), c.batch), None, lambda s: s,
                               gather=lambda p: [p], verdict_many=verdict_many)
