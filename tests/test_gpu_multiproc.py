"""GPU tier: the multi-GPU protocol with REAL HIP partials exchanged between processes.

Two ranks (gloo process group, world size 2, both on device 0 of the one-GPU box) each run
the product's split API on their contiguous shard -- zg_batch_begin, zg_batch_partial, the
all-gather of the 576-byte partials (zebra_amd.dist.combine_partials), ONE final
exponentiation of their product (zg_gt_check) on every rank, zg_batch_finish -- first on an
all-valid batch, then with corrupted proofs in rank 1's shard: both ranks must see the same
false verdict, rank 1's own partial must fail its own check, and the per-rank statuses after
bisection must be exactly the oracle's (C++ restatement of bellman's verify_proof)."""
import os
import socket

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu

SHARD = 512


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from tests.test_gpu_configs import _sources, config3_indices, corrupt, oracle_statuses
    from tests import cpulib
    from zebra_amd import Context, pack_inputs
    from zebra_amd.dist import combine_partials, shard_range
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {"rank": rank}
    try:
        n = SHARD * world
        _, src_proofs, src_kinds, rows = _sources()
        idx = config3_indices(n)
        c = Context(device=0, max_batch=SHARD)
        try:
            proofs = c.synth_rerandomize(src_proofs, src_kinds, idx, 9)   # same bytes on every rank
            kinds = bytes(src_kinds[j] for j in idx)
            inputs = pack_inputs([rows[["S1", "S2", "O1", "O2", "O3"][j]] for j in idx])
            lo, hi = shard_range(n, world, rank)
            seen = {}

            def run(pr, xs, tag):
                c.batch_begin(pr[192 * lo:192 * hi], kinds[lo:hi], xs[288 * lo:288 * hi])
                part = c.batch_partial()

                def check(parts):
                    seen[tag] = parts
                    return c.gt_check(parts)
                ok = combine_partials(part, check, world, rank, "cpu")
                own = c.gt_check([part])
                assert seen[tag][rank] == part
                sts = c.batch_finish(own, hi - lo)
                return ok, own, sts

            out["clean"] = run(proofs, inputs, "clean")
            # corruptions only inside rank 1's shard: indices from corrupt() shifted there
            bp, bx, bad = corrupt(proofs[192 * SHARD:], kinds[SHARD:], inputs[288 * SHARD:], 4, 5)
            bp, bx = proofs[:192 * SHARD] + bp, inputs[:288 * SHARD] + bx
            bad = [SHARD + i for i in bad]
            out["bad"] = run(bp, bx, "bad")
            want = oracle_statuses(cpulib.load(), bp, kinds, bx, bad)
            out["want"] = {i - lo: s for i, s in want.items() if lo <= i < hi}
        finally:
            c.close()
    except Exception as e:   # reported to the parent
        out["error"] = repr(e)
    finally:
        q.put(out)
        dist.destroy_process_group()


def test_two_ranks_real_partials():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in range(2)), key=lambda d: d["rank"])
    for p in procs:
        p.join(60)
    assert [r.get("error") for r in res] == [None, None], res
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for r in res:
        ok, own, sts = r["clean"]
        assert ok and own and sts == [0] * SHARD
        ok, own, sts = r["bad"]
        assert not ok                          # one verdict for the whole batch, on both ranks
        got = {i: s for i, s in enumerate(sts) if s != 0}
        assert got == r["want"]
        assert own == (not any(s == 3 for s in r["want"].values()))
    assert res[0]["want"] == {} and res[1]["want"]
