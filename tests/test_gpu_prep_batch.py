"""GPU tier: zg_prep_batch (round 6) -- a window's public-input preparation in one call, the Sapling
descriptions' Jubjub decodes on the GPU (k_prep_sapling) and the JoinSplits on host threads -- gives
per description exactly the rows and error codes of the single-description host functions
(zg_prep_spend / zg_prep_output / zg_prep_joinsplit[_bn]), which tests/test_input_prep.py pins to the
reference's real transactions, its accept_spend_fails / accept_output_fails error classes
(verification/src/sapling.rs:365-510) and the oracle's restatement. Cases: the real descriptions, the
reference error classes, random byte flips of every field, and a mixed window of 3,000 descriptions."""
import random

import pytest

from tests.conftest import load_golden

pytestmark = pytest.mark.gpu


def h(x):
    return bytes.fromhex(x)


@pytest.fixture(scope="module")
def ctx():
    from zebra_amd import Context
    c = Context(device=0, max_batch=64)
    yield c
    c.close()


def _host(Z, kind, args):
    """the single-description host function: (code, 288-byte row)"""
    fn = {Z.PREP_KIND_SPEND: Z.prep_spend, Z.PREP_KIND_OUTPUT: Z.prep_output,
          Z.PREP_KIND_JOINSPLIT: Z.prep_joinsplit, Z.PREP_KIND_JOINSPLIT_BN: Z.prep_joinsplit_bn}[kind]
    try:
        return 0, Z.pack_inputs([fn(*args)])
    except Z.PrepError as e:
        return e.code, None


def _check(ctx, jobs):
    from zebra_amd import zg as Z
    rows, codes = ctx.prep_batch(bytes(k for k, _ in jobs), b"".join(Z.prep_fields(k, *a) for k, a in jobs))
    for i, (k, a) in enumerate(jobs):
        code, row = _host(Z, k, a)
        assert codes[i] == code, (i, k)
        if code == 0:
            assert rows[288 * i:288 * i + 288] == row, (i, k)
    return codes


def _golden_jobs():
    from zebra_amd import zg as Z
    tf = load_golden("input_prep.json")["tx_fields"]
    jobs = []
    for s in tf["spends"]:
        jobs.append((Z.PREP_KIND_SPEND, (h(s["cv"]), h(s["anchor"]), h(s["nullifier"]), h(s["rk"]))))
    for o in tf["outputs"]:
        jobs.append((Z.PREP_KIND_OUTPUT, (h(o["cv"]), h(o["cmu"]), h(o["epk"]))))
    for j in tf["joinsplits"]:
        a = (h(j["anchor"]), h(j["random_seed"]), [h(x) for x in j["nullifiers"]], [h(x) for x in j["macs"]],
             [h(x) for x in j["commitments"]], j["vpub_old"], j["vpub_new"], h(j["pubkey"]))
        jobs.append((Z.PREP_KIND_JOINSPLIT, a))
        jobs.append((Z.PREP_KIND_JOINSPLIT_BN, a))
    return jobs


def test_real_descriptions(ctx):
    jobs = _golden_jobs()
    codes = _check(ctx, jobs)
    assert not any(codes)


def test_reference_error_classes(ctx):
    from zebra_amd import zg as Z
    jobs = []
    for e in load_golden("input_prep.json")["prep_errors"]:
        f = e["fields"]
        if e["kind"] == "spend":
            jobs.append((Z.PREP_KIND_SPEND, (h(f["cv"]), h(f["anchor"]), h(f["nullifier"]), h(f["rk"]))))
        else:
            jobs.append((Z.PREP_KIND_OUTPUT, (h(f["cv"]), h(f["cmu"]), h(f["epk"]))))
    codes = _check(ctx, jobs)
    assert all(codes)


def test_random_flips_and_a_mixed_window(ctx):
    """every field of every kind flipped at random (invalid points, small order, non-canonical
    anchors / cmu), interleaved with valid descriptions and JoinSplits: 3,000 descriptions"""
    base = _golden_jobs()
    rng = random.Random(6)
    jobs = []
    for _ in range(3000):
        k, a = base[rng.randrange(len(base))]
        a = list(a)
        if rng.random() < 0.6:
            idx = rng.randrange(len(a))
            if isinstance(a[idx], bytes) and len(a[idx]) == 32:
                b = bytearray(a[idx])
                if rng.random() < 0.2:
                    b[31] |= 0x7f   # y >= r (not in field) for points, >= r for anchor / cmu
                else:
                    b[rng.randrange(32)] ^= 1 << rng.randrange(8)
                a[idx] = bytes(b)
        jobs.append((k, tuple(a)))
    codes = _check(ctx, jobs)
    assert 0 < sum(1 for c in codes if c) < len(codes)


def test_collector_window_gpu_prep_matches_host_prep(ctx):
    """collector.verify_block's queue with the GPU preparation (ctx) gives the host path's items"""
    from zebra_amd import collector
    from tools import bench_config5 as b5

    class Src:
        def synth_rerandomize(self, src, kinds, idx, seed):
            return b"".join(src[192 * i:192 * i + 192] for i in idx)
    blocks = b5.build_blocks(Src(), 3, 120, 9)
    txs = [tx for t, _ in blocks for tx in t]
    assert len(collector._jobs(txs)) >= collector._GPU_PREP_MIN
    assert collector._queue(txs, ctx) == collector._queue(txs, None)
