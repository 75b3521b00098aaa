"""GPU tier: the two ways the batch forms its per-key sums sum_i r_i C_i.

Shards from ZG_K4_MIN (16,384) padded proofs use K4's Pippenger buckets (zg_msm.hip); smaller
shards -- the 8-GPU rank size, config 2, bisection-heavy config 4 -- take the GLV products
r_i C_i in decode (the job that already forms r_i A_i) and sum them up the C-sum tree
(k_tree_c), which bisection then reuses. The two must be the same group element per key, so
the 576-byte Miller partial (which pairs its affine form with -delta_k) is byte-identical, and
the reject set is the oracle's either way. ZG_K4_MIN is read when a context is created, so each
path gets its own context.

Reference: the C term of verify_proof (verification/src/sapling.rs:162, sprout.rs:73-77), one
pairing per proof in bellman; here one per key and batch."""
import os
import random

import pytest

from tests.conftest import load_golden
from tests.test_gpu_configs import SRCS, _sources, config3_indices, corrupt, oracle_statuses

pytestmark = pytest.mark.gpu


def _ctx(k4_min, n):
    from zebra_amd import Context
    old = os.environ.get("ZG_K4_MIN")
    os.environ["ZG_K4_MIN"] = str(k4_min)
    try:
        return Context(device=0, max_batch=n)
    finally:
        if old is None:
            del os.environ["ZG_K4_MIN"]
        else:
            os.environ["ZG_K4_MIN"] = old


@pytest.fixture(scope="module")
def work4k():
    from zebra_amd import Context, pack_inputs
    _, src_proofs, src_kinds, rows = _sources()
    idx = config3_indices(4096)
    c = Context(device=0, max_batch=64)
    try:
        proofs = c.synth_rerandomize(src_proofs, src_kinds, idx, 7)
    finally:
        c.close()
    kinds = bytes(src_kinds[j] for j in idx)
    inputs = pack_inputs([rows[SRCS[j]] for j in idx])
    return proofs, kinds, inputs


@pytest.mark.parametrize("n", [1024, 4096])
def test_glv_tree_and_k4_give_the_same_partial(work4k, n):
    """clean batch, seeded batch scalars: the GLV + tree path and K4 give byte-identical Miller
    partials and both accept"""
    proofs, kinds, inputs = work4k
    proofs, kinds, inputs = proofs[:192 * n], kinds[:n], inputs[:288 * n]
    r = random.Random(n).randbytes(16 * n)
    parts = {}
    for k4_min, path in ((1 << 30, "glv"), (1, "k4")):
        c = _ctx(k4_min, n)
        try:
            c.batch_begin(proofs, kinds, inputs, r=r)
            parts[path] = c.batch_partial()
            assert c.gt_check([parts[path]])
            assert c.batch_finish(True, n) == [0] * n
            st = c.stats()
            assert st["glv_csum_batches"] == (1 if path == "glv" else 0)
            assert (st["k4_entries"] > 0) == (path == "k4")
        finally:
            c.close()
    assert parts["glv"] == parts["k4"]


def test_glv_tree_exact_reject_set_with_deferred_b(work4k):
    """4,096 proofs with 24 corruptions rotating through every class (non-subgroup B: the deferred
    G2 check and gated C-tree recompute; non-subgroup C: masked GLV leaf; A <-> C swaps, input
    tweaks, flags, infinity): the GLV + tree path gives the oracle's exact statuses, through
    bisection that reuses the C tree the pipeline built; K4 agrees"""
    from tests import cpulib
    proofs, kinds, inputs = work4k
    bp, bx, bad = corrupt(proofs, kinds, inputs, 24, 11)
    cpu = cpulib.load()
    want = oracle_statuses(cpu, bp, kinds, bx, bad)
    got = {}
    for k4_min, path in ((1 << 30, "glv"), (1, "k4")):
        c = _ctx(k4_min, 4096)
        try:
            sts, _ = c.verify_batch(bp, kinds, bx)
            st = c.stats()
        finally:
            c.close()
        got[path] = {i: s for i, s in enumerate(sts) if s != 0}
        assert st["bisections"] == 1 and st["b_subgroup_recomputes"] >= 1
    assert got["glv"] == want
    assert got["k4"] == want


def _ctx_env(env, n):
    from zebra_amd import Context
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return Context(device=0, max_batch=n)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("env", [{"ZG_SERIAL_SIDE": 1}, {"ZG_TREE_COOP_BELOW": 1}, {"ZG_TREE_COOP_BELOW": 1 << 30},
                                 {"ZG_FCHAIN_SINGLE": 0}, {"ZG_LINES_FCHAIN": 0, "ZG_FCHAIN_QUADS": 1},
                                 {"ZG_LINES_FCHAIN": 0, "ZG_FCHAIN_QUADS": 1, "ZG_LINE_GROUP": 0},
                                 {"ZG_LINES_FCHAIN": 0, "ZG_FCHAIN_QUADS": 1, "ZG_LINE_GROUP": 4},
                                 {"ZG_LINES_FCHAIN": 0, "ZG_FCHAIN_QUADS": 1, "ZG_LINE_GROUP": 2048},
                                 {"ZG_LINES_FCHAIN": 0, "ZG_FCHAIN_QUADS": 1, "ZG_LINE_GROUP": 32},
                                 {"ZG_LINES_FCHAIN": 0, "ZG_FCHAIN_QUADS": 1, "ZG_LINE_GROUP": 32, "ZG_LINE_PROD_PARTS": 1},
                                 {"ZG_LINES_FCHAIN": 0, "ZG_FCHAIN_QUADS": 1, "ZG_LINE_GROUP": 32, "ZG_LINE_PROD_PARTS": 3},
                                 {"ZG_LINES_FCHAIN": 0, "ZG_FCHAIN_QUADS": 1, "ZG_LINE_GROUP": 32, "ZG_SERIAL_SIDE": 1},
                                 {"ZG_LINES_FCHAIN": 0, "ZG_FCHAIN_QUADS": 1, "ZG_LINE_GROUP": 4, "ZG_PAIRS_LATE": 1},
                                 {"ZG_LINES_FCHAIN": 0, "ZG_LINES_LANE": 1}, {"ZG_K4_MIN": 1}],
                         ids=lambda e: ",".join("%s=%s" % kv for kv in e.items()))
def test_context_knobs_give_the_same_partial(work4k, env):
    """every per-context schedule switch (zg.hip zg_create: side work serialised on the main stream,
    product-tree levels lane-per-node or wave-per-node, the fused launch with proof pairs instead of
    single proofs, split quads as group line products + per-group chains (4, 32 or all 2,048
    proofs a group; their chains in 1, 3 or 4 step parts overlapping the line products) or as the quad
    chain, the straight-line R-chain, K4 on a lone small batch) computes the
    same batch: byte-identical 576-B Miller partial to the default schedule's for seeded scalars"""
    n = 2048
    proofs, kinds, inputs = work4k
    proofs, kinds, inputs = proofs[:192 * n], kinds[:n], inputs[:288 * n]
    r = random.Random(77).randbytes(16 * n)
    parts = []
    for e in ({}, env):
        c = _ctx_env(e, n)
        try:
            c.batch_begin(proofs, kinds, inputs, r=r)
            parts.append(c.batch_partial())
            assert c.gt_check([parts[-1]])
            assert c.batch_finish(True, n) == [0] * n
        finally:
            c.close()
    assert parts[0] == parts[1]
