"""GPU tier: bench.py's default schedule (zebra_amd.dist.run_pipelined_deferred) on real contexts.
Batch contexts are relaunched as soon as their partial and provisional statuses are read; the
verdicts run off the loop: an ordered gather stage, then each final exponentiation on one of the
high-priority checker contexts (zg_set_priority). A batch
whose verdict is false (config 4's 41 corrupted proofs among 4,096) is re-run with bisection and
must come back with the exact reject set; the valid batches around it are unaffected."""
import pytest

from tests.conftest import load_golden
from tests.test_gpu_parity import corrupted_4096

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("poll,checks,many", [(False, 1, False), (True, 1, False), (True, 2, False),
                                              (True, 1, True)],
                         ids=["in-order", "first-ready", "first-ready-2-checkers", "first-ready-coalesced"])
def test_deferred_verdicts_exact_statuses(poll, checks, many):
    """checks = 2: bench.py's pooled verdicts (round 6) -- the ordered gather stage, then the final
    exponentiations on two checker contexts with their own high-priority stream pairs; many: the
    coalescing checker (bench.py --coalesce on), waiting batches' verdicts in one zg_gt_check_many"""
    import queue
    from zebra_amd import Context, pack_inputs
    from zebra_amd.dist import run_pipelined_deferred
    n = 4096
    cs = [Context(device=0, max_batch=n, seed=13) for _ in range(2)]
    checkers = [Context(device=0, max_batch=64) for _ in range(checks)]
    free = queue.SimpleQueue()
    for chk in checkers:
        chk.set_priority(True)
        free.put(chk)
    try:
        real = load_golden("real_proofs.json")["proofs"]
        src_proofs = b"".join(bytes.fromhex(e["proof"]) for e in real)
        src_kinds = bytes(e["kind"] for e in real)
        batches = []
        for b in range(5):
            if b == 2:
                proofs, kinds, inputs, want = corrupted_4096(cs[0])
            else:
                idx = [(i + b) % len(real) for i in range(n)]
                proofs = cs[0].synth_rerandomize(src_proofs, src_kinds, idx, 40 + b)
                kinds = bytes(src_kinds[j] for j in idx)
                inputs = pack_inputs([[bytes.fromhex(x) for x in real[j]["inputs"]] for j in idx])
                want = [0] * n
            batches.append((proofs, kinds, inputs, want))
        nxt = [0]

        def launch(c):
            c.batch_begin(*batches[nxt[0]][:3])
            nxt[0] += 1

        def harvest(c):
            part = c.batch_partial()
            return part, c.batch_finish(True, n)

        def verdict(parts):
            chk = free.get()
            try:
                return chk.gt_check(parts)
            finally:
                free.put(chk)

        def redo(s):
            c = cs[0]
            c.batch_begin(*batches[s][:3])
            ok = c.gt_check([c.batch_partial()])
            return c.batch_finish(ok, n)

        res = run_pipelined_deferred(cs, 5, launch, harvest, verdict, redo,
                                     ready=(lambda c: c.batch_ready()) if poll else None,
                                     gather=lambda part: [part], checks=checks,
                                     verdict_many=checkers[0].gt_check_many if many else None)
        assert [ok for ok, _ in res] == [True, True, False, True, True]
        for b, (_, sts) in enumerate(res):
            assert sts == batches[b][3], b
    finally:
        for c in cs + checkers:
            c.close()
