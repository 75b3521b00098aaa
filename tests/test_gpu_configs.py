"""GPU tier: BASELINE.json configs 2 and 3 at full size, with exact expected statuses.

  config 2  1,024 Sapling spend proofs (S[i mod 2] re-randomized, seed 1), one batch
  config 3  65,536 mixed proofs (even i -> S[(i/2) mod 2], odd i -> O[(i/2) mod 3], seed 2):
            all-accept; 20 corruptions spread over the index range -> exact reject set; and the
            8-GPU protocol on one GPU: 8 contiguous 8,192-proof shards on 8 contexts (all eight
            batches in flight at once), their 576-byte Miller partials through ONE zg_gt_check

Expected statuses come from the oracle: the corrupted proofs are re-verified one by one by
the C++ restatement of bellman's verify_proof (oracle/cpu, checker only), and the accumulated
GT of config 2's first 64 proofs is recomputed from the oracle's per-proof left-hand sides.
Reference semantics: verification/src/sapling.rs:157-167 (per-proof classes),
verification/src/accept_chain.rs:76-81 (lowest failing index of a block)."""
import random

import pytest

from tests.conftest import load_golden

pytestmark = pytest.mark.gpu

SRCS = ["S1", "S2", "O1", "O2", "O3"]


def _sources():
    real = {e["name"]: e for e in load_golden("real_proofs.json")["proofs"]}
    src_proofs = b"".join(bytes.fromhex(real[s]["proof"]) for s in SRCS)
    src_kinds = bytes(real[s]["kind"] for s in SRCS)
    rows = {s: [bytes.fromhex(x) for x in real[s]["inputs"]] for s in SRCS}
    return real, src_proofs, src_kinds, rows


def config3_indices(n):
    return [(i // 2) % 2 if i % 2 == 0 else 2 + (i // 2) % 3 for i in range(n)]


@pytest.fixture(scope="module")
def cpu():
    from tests import cpulib
    return cpulib.load()


@pytest.fixture(scope="module")
def workload3():
    """config 3's 65,536 proofs (GPU re-randomization, seed 2) and their inputs"""
    from zebra_amd import Context, pack_inputs
    _, src_proofs, src_kinds, rows = _sources()
    idx = config3_indices(65536)
    c = Context(device=0, max_batch=64)
    try:
        proofs = c.synth_rerandomize(src_proofs, src_kinds, idx, 2)
    finally:
        c.close()
    kinds = bytes(src_kinds[j] for j in idx)
    row_bytes = [pack_inputs([rows[SRCS[j]]]) for j in range(len(SRCS))]
    inputs = b"".join(row_bytes[j] for j in idx)
    return proofs, kinds, inputs, idx


def corrupt(proofs, kinds, inputs, count, seed):
    """`count` corruptions spread over the index range, rotating through the classes of
    SURVEY.md 8(d) config 4 -> (proofs, inputs, corrupted indices)"""
    pts = load_golden("points.json")
    n = len(kinds)
    proofs, inputs = bytearray(proofs), bytearray(inputs)
    rng = random.Random(seed)
    stride = n // count
    bad = sorted(q * stride + rng.randrange(stride) for q in range(count))
    for q, i in enumerate(bad):
        cls = q % 6
        if cls == 0:      # public-input tweak (a nullifier / cmu byte) -> VERIFY_FAILED
            inputs[288 * i + 32 * (4 if kinds[i] == 0 else 3)] ^= 1
        elif cls == 1:    # A <-> C swap -> VERIFY_FAILED
            p = proofs[192 * i:192 * i + 192]
            proofs[192 * i:192 * i + 192] = p[144:] + p[48:144] + p[:48]
        elif cls == 2:    # compression flag cleared -> DECODE_INVALID
            proofs[192 * i] &= 0x7F
        elif cls == 3:    # non-subgroup G2 B -> DECODE_INVALID (deferred G2 check, gated recompute)
            proofs[192 * i + 48:192 * i + 144] = bytes.fromhex(pts["g2_not_in_subgroup"])
        elif cls == 4:    # non-subgroup G1 C -> DECODE_INVALID
            proofs[192 * i + 144:192 * i + 192] = bytes.fromhex(pts["g1_not_in_subgroup"])
        else:             # infinity-encoded A -> DECODE_INVALID
            proofs[192 * i:192 * i + 48] = bytes([0xC0]) + bytes(47)
    return bytes(proofs), bytes(inputs), bad


def oracle_statuses(cpu, proofs, kinds, inputs, idx):
    from tests import cpulib
    sub_p = b"".join(proofs[192 * i:192 * i + 192] for i in idx)
    sub_k = bytes(kinds[i] for i in idx)
    sub_x = b"".join(inputs[288 * i:288 * i + 288] for i in idx)
    sts, _ = cpulib.verify(cpu, sub_p, sub_k, sub_x, threads=8)
    return dict(zip(idx, sts))


def test_config2_1024_spends():
    """1,024 spends in ONE zg_verify_batch: all accept (OS-random batch scalars)"""
    from zebra_amd import Context, pack_inputs
    _, src_proofs, src_kinds, rows = _sources()
    idx = [i % 2 for i in range(1024)]
    c = Context(device=0, max_batch=1024)
    try:
        proofs = c.synth_rerandomize(src_proofs, src_kinds, idx, 1)
        kinds = bytes(src_kinds[j] for j in idx)
        assert set(kinds) == {0}
        inputs = pack_inputs([rows[SRCS[j]] for j in idx])
        sts, _ = c.verify_batch(proofs, kinds, inputs)
        assert sts == [0] * 1024
        assert c.stats()["bisections"] == 0
    finally:
        c.close()


def test_config2_gt_out_matches_oracle(cpu):
    """seeded run: the accumulated GT of config 2's first 64 proofs equals the oracle's
    prod_i LHS_i^{r_i}, LHS_i = bellman's final-exponentiated left-hand side"""
    from oracle import bls12_381 as B, groth16 as G
    from tests import cpulib
    from zebra_amd import Context, pack_inputs
    _, src_proofs, src_kinds, rows = _sources()
    idx = [i % 2 for i in range(64)]
    c = Context(device=0, max_batch=1024)
    try:
        proofs = c.synth_rerandomize(src_proofs, src_kinds, idx, 1)
        kinds = bytes(src_kinds[j] for j in idx)
        inputs = pack_inputs([rows[SRCS[j]] for j in idx])
        r = random.Random(1).randbytes(16 * 64)
        sts, gt = c.verify_batch(proofs, kinds, inputs, r=r, want_gt=True)
    finally:
        c.close()
    assert sts == [0] * 64
    osts, lhs = cpulib.verify(cpu, proofs, kinds, inputs, threads=8, want_gt=True)
    assert osts == [0] * 64
    want = G.batch_gt([B.f12_from_bytes(x) for x in lhs], [G.batch_r(r[16 * i:16 * i + 16]) for i in range(64)])
    assert gt == B.f12_to_bytes(want)


def test_config3_all_accept(workload3):
    from zebra_amd import Context
    proofs, kinds, inputs, _ = workload3
    c = Context(device=0, max_batch=65536)
    try:
        sts, _ = c.verify_batch(proofs, kinds, inputs)
        assert sts == [0] * 65536
        assert c.stats()["bisections"] == 0
    finally:
        c.close()


def test_config3_exact_reject_set(workload3, cpu):
    """20 corruptions spread over 65,536 proofs: the batch fails, bisection isolates exactly
    the oracle's reject set with the oracle's classes; everything else accepts"""
    from zebra_amd import Context
    proofs, kinds, inputs, _ = workload3
    bp, bx, bad = corrupt(proofs, kinds, inputs, 20, 2)
    want = oracle_statuses(cpu, bp, kinds, bx, bad)
    assert all(v in (1, 3) for v in want.values()), want
    c = Context(device=0, max_batch=65536)
    try:
        sts, _ = c.verify_batch(bp, kinds, bx)
        st = c.stats()
    finally:
        c.close()
    got = {i: s for i, s in enumerate(sts) if s != 0}
    assert got == want
    # the 64k shard ran the four-proofs-per-lane f-chain, and bisection descended through its
    # quad-level tree (no pair-level nodes) to the exact reject set
    assert st["quad_fchain_launches"] >= 1 and st["bisections"] == 1


def _shards_run(ctxs, proofs, kinds, inputs, shard):
    """8 contiguous shards, all in flight at once (one context each), then their partials"""
    for g, c in enumerate(ctxs):
        lo = g * shard
        c.batch_begin(proofs[192 * lo:192 * (lo + shard)], kinds[lo:lo + shard], inputs[288 * lo:288 * (lo + shard)])
    return [c.batch_partial() for c in ctxs]


def test_config3_eight_shards_one_gpu(workload3, cpu):
    """the 8-GPU protocol on one GPU: 8 x 8,192-proof shards on 8 contexts with all 8 batches in
    flight together, ONE final exponentiation over the 8 partials; then the same with the
    corrupted copy: the combined verdict fails, each shard's own partial localises it, and
    per-shard bisection gives the exact reject set"""
    from zebra_amd import Context
    proofs, kinds, inputs, _ = workload3
    shard = 8192
    ctxs = [Context(device=0, max_batch=shard) for _ in range(8)]
    try:
        parts = _shards_run(ctxs, proofs, kinds, inputs, shard)
        assert ctxs[0].gt_check(parts)
        for c in ctxs:
            assert c.batch_finish(True, shard) == [0] * shard
        bp, bx, bad = corrupt(proofs, kinds, inputs, 20, 2)
        want = oracle_statuses(cpu, bp, kinds, bx, bad)
        parts = _shards_run(ctxs, bp, kinds, bx, shard)
        assert not ctxs[0].gt_check(parts)
        got = {}
        for g, c in enumerate(ctxs):
            own = c.gt_check([parts[g]])
            sts = c.batch_finish(own, shard)
            has_bad_in_shard = any(g * shard <= i < (g + 1) * shard and want[i] == 3 for i in want)
            assert own == (not has_bad_in_shard), g
            got.update({g * shard + i: s for i, s in enumerate(sts) if s != 0})
        assert got == want
        assert sum(c.stats()["batches"] for c in ctxs) == 16
    finally:
        for c in ctxs:
            c.close()


def test_config3_gt_split_invariance(workload3, cpu):
    """size-independent GT parity at the full 65,536: with the same explicit batch scalars, the
    accumulated GT of the whole batch (four proofs per f-chain lane, K4 at c = 11) equals the
    product of the GTs of its 8 x 8,192 shards (c = 10) and of its 16 x 4,096 shards (two proofs
    per lane, c = 9); and for 64 random indices of the same workload the device GT equals the
    oracle's prod LHS_i^{r_i} (C++ restatement of bellman's per-proof left-hand sides)"""
    from oracle import bls12_381 as B, groth16 as G
    from tests import cpulib
    from zebra_amd import Context
    proofs, kinds, inputs, _ = workload3
    n = 65536
    r = random.Random(11).randbytes(16 * n)
    big = Context(device=0, max_batch=n)
    try:
        sts, gt_full = big.verify_batch(proofs, kinds, inputs, r=r, want_gt=True)
        assert sts == [0] * n and big.stats()["quad_fchain_launches"] >= 1
    finally:
        big.close()
    for shard in (8192, 4096):
        c = Context(device=0, max_batch=shard)
        try:
            acc = B.F12_ONE
            for lo in range(0, n, shard):
                hi = lo + shard
                s, g = c.verify_batch(proofs[192 * lo:192 * hi], kinds[lo:hi], inputs[288 * lo:288 * hi],
                                      r=r[16 * lo:16 * hi], want_gt=True)
                assert s == [0] * shard
                acc = B.f12_mul(acc, B.f12_from_bytes(g))
        finally:
            c.close()
        assert B.f12_to_bytes(acc) == gt_full, shard
    idx = sorted(random.Random(12).sample(range(n), 64))
    sp = b"".join(proofs[192 * i:192 * i + 192] for i in idx)
    sk = bytes(kinds[i] for i in idx)
    sx = b"".join(inputs[288 * i:288 * i + 288] for i in idx)
    sr = b"".join(r[16 * i:16 * i + 16] for i in idx)
    c = Context(device=0, max_batch=64)
    try:
        s, g = c.verify_batch(sp, sk, sx, r=sr, want_gt=True)
    finally:
        c.close()
    osts, lhs = cpulib.verify(cpu, sp, sk, sx, threads=8, want_gt=True)
    assert s == osts == [0] * 64
    want = G.batch_gt([B.f12_from_bytes(x) for x in lhs], [G.batch_r(sr[16 * q:16 * q + 16]) for q in range(64)])
    assert g == B.f12_to_bytes(want)


def test_config3_many_non_subgroup_b(workload3, cpu):
    """5% of the 65,536 proofs carry a B on the twist but outside G2: the deferred G2 check in the
    R-chain turns each DECODE_INVALID (Proof::read) while K4 and the VK-side root work already ran
    on the side stream -- the gated recompute must give exactly the reference's statuses"""
    from zebra_amd import Context
    proofs, kinds, inputs, _ = workload3
    pts = load_golden("points.json")
    bad_b = bytes.fromhex(pts["g2_not_in_subgroup"])
    pr = bytearray(proofs)
    bad = list(range(7, 65536, 20))
    for i in bad:
        pr[192 * i + 48:192 * i + 144] = bad_b
    pr = bytes(pr)
    want = oracle_statuses(cpu, pr, kinds, inputs, bad[::400])
    assert set(want.values()) == {1}
    c = Context(device=0, max_batch=65536)
    try:
        sts, _ = c.verify_batch(pr, kinds, inputs)
        st = c.stats()
    finally:
        c.close()
    assert {i: s for i, s in enumerate(sts) if s} == {i: 1 for i in bad}
    assert st["b_subgroup_recomputes"] >= 1 and st["bisections"] == 0
