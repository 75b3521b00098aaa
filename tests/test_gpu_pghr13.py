"""GPU parity of PGHR13 on BN254 against the oracle: the device pairing's
GT bytes equal oracle.bn254's (Miller loop + the same final-exponentiation chain), every case of
tests/golden/pghr13.json (the reference's vectors, mainnet block 522, mutants) gets the oracle's
status, a mixed batch of 1,024, and the verifying-key checks."""
import json
import os
import random

import pytest

from oracle import bn254 as B
from tests.conftest import ROOT, load_golden

GOLDEN = load_golden("pghr13.json")


@pytest.fixture(scope="module")
def ctx():
    from zebra_amd import Context
    c = Context(device=0, max_batch=64, load_builtin=False, seed=7)
    yield c
    c.close()


def _inputs(case):
    return [bytes.fromhex(x) for x in case["inputs"]]


@pytest.mark.gpu
def test_gpu_bn254_pairing_bytes(ctx):
    rnd = random.Random(2)
    ps = [B.G1_GEN, B.ec_mul(B._F1, B.G1_GEN, rnd.randrange(1, B.R))]
    qs = [B.G2_GEN, B.ec_mul(B._F2, B.G2_GEN, rnd.randrange(1, B.R))]
    got = ctx.bn254_pairing(ps, qs)
    for p, q, g in zip(ps, qs, got):
        assert g == B.gt_ints(B.final_exponentiation_fc(B.miller_loop([(p, q)])))
    # bilinearity on the device alone
    e1, e6 = ctx.bn254_pairing([B.G1_GEN, B.ec_mul(B._F1, B.G1_GEN, 6)], [B.ec_mul(B._F2, B.G2_GEN, 7), B.ec_mul(B._F2, B.G2_GEN, 7)])
    assert e1 != e6


@pytest.mark.gpu
def test_gpu_pghr13_fixtures(ctx):
    cases = GOLDEN["cases"]
    got = ctx.pghr13_verify([bytes.fromhex(c["proof"]) for c in cases], [_inputs(c) for c in cases])
    assert got == [c["status"] for c in cases], [(c["name"], g, c["status"]) for c, g in zip(cases, got)
                                                  if g != c["status"]]


@pytest.mark.gpu
def test_gpu_pghr13_mixed_batch(ctx):
    """1,024 proofs cycling through every fixture case (valid mainnet proofs and mutants)"""
    cases = GOLDEN["cases"]
    rnd = random.Random(4)
    pick = [rnd.randrange(len(cases)) for _ in range(1024)]
    got = ctx.pghr13_verify([bytes.fromhex(cases[k]["proof"]) for k in pick], [_inputs(cases[k]) for k in pick])
    assert got == [cases[k]["status"] for k in pick]


@pytest.mark.gpu
def test_gpu_pghr13_inputs(ctx):
    from zebra_amd import zg
    c = next(c for c in GOLDEN["cases"] if c["name"] == "smoky_pghr")
    ins = _inputs(c)
    big = list(ins)
    big[2] = B.R.to_bytes(32, "little")
    got = ctx.pghr13_verify([bytes.fromhex(c["proof"])] * 3, [ins, big, ins[:8]])
    assert got == [zg.STATUS_OK, zg.STATUS_INPUT_NONCANONICAL, zg.STATUS_VERIFY_FAILED]


@pytest.mark.gpu
def test_gpu_pghr13_vk_checks(ctx):
    from zebra_amd import zg
    d = json.load(open(os.path.join(ROOT, "zebra_amd", "res", "sprout-verifying-key.json")))
    bad = dict(d)
    bad["alphaB"] = [d["alphaB"][0], d["alphaB"][0]]      # off the curve
    with pytest.raises(zg.ZgError) as ei:
        ctx.pghr13_vk_load_json(json.dumps(bad))
    assert ei.value.code == -4
    # a twist point outside the order-r subgroup (AffineG2::new's order check)
    x0 = 1
    while True:
        xx = (x0, 1)
        y = B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(xx), xx), B.B2))
        if y is not None and B.ec_mul(B._F2, (xx, y), B.R) is not None:
            break
        x0 += 1
    bad = dict(d)
    bad["zeta"] = ["0x%064x" % xx[1], "0x%064x" % xx[0], "0x%064x" % y[1], "0x%064x" % y[0]]
    with pytest.raises(zg.ZgError) as ei:
        ctx.pghr13_vk_load_json(json.dumps(bad))
    assert ei.value.code == -4
    ctx.pghr13_vk_load_json(json.dumps(d))
    c = GOLDEN["cases"][0]
    assert ctx.pghr13_verify([bytes.fromhex(c["proof"])], [_inputs(c)]) == [c["status"]]


@pytest.mark.gpu
def test_gpu_pghr13_keys_per_context():
    """keys belong to the context that loaded them: two fresh contexts verifying
    concurrently on first use both get the builtin key; a different valid key loaded on one
    context changes only that context's verdicts; a failed load leaves its key unchanged"""
    import threading
    from zebra_amd import Context, zg
    valid = [c for c in GOLDEN["cases"] if c["status"] == 0]
    proofs = [bytes.fromhex(c["proof"]) for c in valid] * 8
    inputs = [_inputs(c) for c in valid] * 8
    a, b = Context(device=0, max_batch=64, load_builtin=False), Context(device=0, max_batch=64, load_builtin=False)
    try:
        res = {}
        ts = [threading.Thread(target=lambda k=k, c=c: res.__setitem__(k, c.pghr13_verify(proofs, inputs)))
              for k, c in (("a", a), ("b", b))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert res == {"a": [0] * len(proofs), "b": [0] * len(proofs)}
        d = json.load(open(os.path.join(ROOT, "zebra_amd", "res", "sprout-verifying-key.json")))
        other = dict(d)
        other["ic"] = d["ic"][2:4] + d["ic"][0:2] + d["ic"][4:]   # ic[0] <-> ic[1]: a valid, different key
        a.pghr13_vk_load_json(json.dumps(other))
        assert a.pghr13_verify(proofs, inputs) == [zg.STATUS_VERIFY_FAILED] * len(proofs)
        assert b.pghr13_verify(proofs, inputs) == [0] * len(proofs)
        bad = dict(d)
        bad["alphaB"] = [d["alphaB"][0], d["alphaB"][0]]
        with pytest.raises(zg.ZgError):
            a.pghr13_vk_load_json(json.dumps(bad))
        assert a.pghr13_verify(proofs[:2], inputs[:2]) == [zg.STATUS_VERIFY_FAILED] * 2   # still `other`
        a.pghr13_vk_load_builtin()
        assert a.pghr13_verify(proofs, inputs) == [0] * len(proofs)
    finally:
        a.close()
        b.close()


@pytest.mark.gpu
def test_gpu_pghr13_batch_check_paths(ctx):
    """the one-check-per-call path (zg_pghr13.hip: the key pairs on the batch's sums, one single-pair
    loop per proof split by segments, one final exponentiation): 2,061 valid proofs (33 blocks, the
last one partial: odd product trees), also through the packed buffers, then the same with decode-invalid
    and non-canonical cases mixed in (excluded from the batch, which still passes), then with one
    VERIFY_FAILED proof (the batch fails and the per-proof path gives the exact statuses)"""
    from zebra_amd import zg
    cases = GOLDEN["cases"]
    valid = [c for c in cases if c["status"] == zg.STATUS_OK]
    skipped = [c for c in cases if c["status"] not in (zg.STATUS_OK, zg.STATUS_VERIFY_FAILED)]
    failing = [c for c in cases if c["status"] == zg.STATUS_VERIFY_FAILED]
    assert valid and skipped and failing
    rnd = random.Random(9)
    base = [valid[rnd.randrange(len(valid))] for _ in range(2061)]
    for extra, fails in (([], 0), (skipped, 0), (skipped + failing[:1], 1)):
        batch = list(base)
        for c in extra:
            batch[rnd.randrange(len(batch))] = c
        st0 = ctx.stats()
        got = ctx.pghr13_verify([bytes.fromhex(c["proof"]) for c in batch], [_inputs(c) for c in batch])
        assert got == [c["status"] for c in batch]
        st1 = ctx.stats()
        assert st1["pghr13_calls"] == st0["pghr13_calls"] + 1
        # the batch check alone decides an all-valid call (a wrong batch check would only show here:
        # the per-proof path would still give the right statuses)
        assert st1["pghr13_batch_failures"] - st0["pghr13_batch_failures"] == fails
        if not extra:  # the ABI's packed buffers give the same
            ins = [_inputs(c) for c in batch]
            packed = ctx.pghr13_verify(b"".join(bytes.fromhex(c["proof"]) for c in batch),
                                       b"".join(b"".join(r) + bytes(32 * (9 - len(r))) for r in ins),
                                       bytes(len(r) for r in ins))
            assert packed == got


@pytest.mark.gpu
def test_gpu_pghr13_batch_check_large(ctx):
    """the large-call shapes of the batch path (40,000 proofs: Straus sums two proofs per lane, four
    proofs per segment lane, P_i7 on the side stream -- zg_pghr13.hip straus_b / bseg_k / p7_side):
    all valid (decided by the batch check alone), then with failing and decode-invalid cases mixed
    in (the per-proof path's exact statuses)"""
    from zebra_amd import zg
    cases = GOLDEN["cases"]
    valid = [c for c in cases if c["status"] == zg.STATUS_OK]
    other = [c for c in cases if c["status"] != zg.STATUS_OK]
    rnd = random.Random(41)
    n = 40000
    batch = [valid[rnd.randrange(len(valid))] for _ in range(n)]

    def run(b):
        ins = [_inputs(c) for c in b]
        st0 = ctx.stats()
        got = ctx.pghr13_verify(b"".join(bytes.fromhex(c["proof"]) for c in b),
                                b"".join(b"".join(r) + bytes(32 * (9 - len(r))) for r in ins),
                                bytes(len(r) for r in ins))
        return got, ctx.stats()["pghr13_batch_failures"] - st0["pghr13_batch_failures"]

    got, fails = run(batch)
    assert got == [0] * n and fails == 0
    for c in other:
        batch[rnd.randrange(n)] = c
    got, fails = run(batch)
    assert got == [c["status"] for c in batch]
    assert fails == (1 if any(c["status"] == zg.STATUS_VERIFY_FAILED for c in other) else 0)
