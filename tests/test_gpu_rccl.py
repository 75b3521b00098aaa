"""GPU tier: the RCCL leg of config 3 ("65,536 mixed Sapling spend/output proofs sharded across
8 x MI355X with RCCL Fq12 gather") on the one-GPU box.

A fresh spawned child (never an exec of a process that touched the GPU) initialises a
world-size-1 process group with backend "nccl" -- RCCL on ROCm -- and runs the product's split
API on two contiguous 4,096-proof shards of config 3: zg_batch_begin on two contexts (both
batches in flight), zg_batch_partial, ONE RCCL all-gather of both 576-byte Miller partials
(zebra_amd.dist.combine_partials with k = 2 partials per rank), ONE final exponentiation of
their product (zg_gt_check), zg_batch_finish. First clean, then with corruptions inside shard 1:
the gathered verdict is false, shard 0's own partial passes, shard 1's fails, and bisection
gives exactly the oracle's reject set (C++ restatement of bellman's verify_proof).

The gather replaces the rayon fan-out of /root/reference/verification/src/accept_chain.rs:76-81
(every transaction's proofs checked on some core, the lowest failing index reported).

The second test runs bench.py itself with --dist at world size 1 in a child process, so the
headline pipeline's collective path (batches in flight, deferred verdicts on the checker
context, RCCL gather on a high-priority stream) runs on the box too."""
import json
import os
import socket
import subprocess
import sys

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu

SHARD = 4096


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, q):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    out = {}
    try:
        import torch
        import torch.distributed as dist
        from tests.test_gpu_configs import _sources, config3_indices, corrupt, oracle_statuses, SRCS
        from tests import cpulib
        from zebra_amd import Context, pack_inputs
        from zebra_amd.dist import combine_partials
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        out["backend"] = dist.get_backend()
        n = 2 * SHARD
        _, src_proofs, src_kinds, rows = _sources()
        idx = config3_indices(n)
        ctxs = [Context(device=0, max_batch=SHARD) for _ in range(2)]
        try:
            proofs = ctxs[0].synth_rerandomize(src_proofs, src_kinds, idx, 2)
            kinds = bytes(src_kinds[j] for j in idx)
            inputs = pack_inputs([rows[SRCS[j]] for j in idx])
            seen = {}

            def run(pr, xs, tag):
                for g, c in enumerate(ctxs):   # both shards in flight before either partial is read
                    lo = g * SHARD
                    c.batch_begin(pr[192 * lo:192 * (lo + SHARD)], kinds[lo:lo + SHARD],
                                  xs[288 * lo:288 * (lo + SHARD)])
                parts = [c.batch_partial() for c in ctxs]

                def check(gathered):
                    seen[tag] = gathered
                    return ctxs[0].gt_check(gathered)
                ok = combine_partials(parts, check, 1, 0, dev)
                assert seen[tag] == parts, "RCCL gather changed the partials"
                owns = [c.gt_check([p]) for c, p in zip(ctxs, parts)]
                sts = []
                for c, own in zip(ctxs, owns):
                    sts += c.batch_finish(own, SHARD)
                return ok, owns, sts

            out["clean"] = run(proofs, inputs, "clean")
            bp, bx, bad = corrupt(proofs[192 * SHARD:], kinds[SHARD:], inputs[288 * SHARD:], 6, 7)
            bp, bx = proofs[:192 * SHARD] + bp, inputs[:288 * SHARD] + bx
            bad = [SHARD + i for i in bad]
            out["bad"] = run(bp, bx, "bad")
            out["want"] = oracle_statuses(cpulib.load(), bp, kinds, bx, bad)
        finally:
            for c in ctxs:
                c.close()
        dist.destroy_process_group()
    except Exception as e:   # reported to the parent
        import traceback
        out["error"] = repr(e) + "\n" + traceback.format_exc()
    finally:
        q.put(out)


def test_rccl_world1_two_shards():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=300)
    p.join(60)
    assert res.get("error") is None, res.get("error")
    assert p.exitcode == 0
    assert res["backend"] == "nccl"
    ok, owns, sts = res["clean"]
    assert ok and owns == [True, True] and sts == [0] * (2 * SHARD)
    ok, owns, sts = res["bad"]
    want = res["want"]
    assert not ok                                       # the gathered product fails
    assert owns[0]                                      # shard 0 is clean
    assert owns[1] == (not any(s == 3 for s in want.values()))
    got = {i: s for i, s in enumerate(sts) if s != 0}
    assert got == want and all(i >= SHARD for i in got)


def test_bench_dist_world1():
    """bench.py --dist at world size 1: the headline pipeline with every verdict through an RCCL
    all-gather (a fresh child process; the test process itself never initialises RCCL)"""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dist", "--proofs", "8192",
                        "--steps", "6", "--warmup", "2", "--no-cpu", "--no-configs", "--no-iso"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["config"]["collective"].startswith("RCCL all-gather")
    assert line["config"]["parallelism"] == "dp1"
    assert line["value"] > 0 and line["steps"] == 6
