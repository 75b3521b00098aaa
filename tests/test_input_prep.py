"""CPU tier: the product's host-side public-input preparation (zebra_amd/csrc/zg_prep.h via the
C ABI zg_prep_*) against the golden fixtures: the public inputs of
the reference's real spends / outputs / JoinSplits, the reference's accept_spend_fails /
accept_output_fails error classes (verification/src/sapling.rs:365-510) and the hSig known
answers (verification/src/sprout.rs:198-278). Also cross-checked against the oracle's
restatement (oracle/zcash.py) on mutated descriptions. No GPU: host code only."""
import random

import pytest

from tests.conftest import load_golden


@pytest.fixture(scope="module")
def Z():
    from zebra_amd import zg
    zg.lib()
    return zg


def h(x):
    return bytes.fromhex(x)


def test_real_spend_output_joinsplit_inputs(Z):
    tf = load_golden("input_prep.json")["tx_fields"]
    for s in tf["spends"]:
        got = Z.prep_spend(h(s["cv"]), h(s["anchor"]), h(s["nullifier"]), h(s["rk"]))
        assert [g.hex() for g in got] == s["inputs"], s["name"]
    for o in tf["outputs"]:
        got = Z.prep_output(h(o["cv"]), h(o["cmu"]), h(o["epk"]))
        assert [g.hex() for g in got] == o["inputs"], o["name"]
    for j in tf["joinsplits"]:
        got = Z.prep_joinsplit(h(j["anchor"]), h(j["random_seed"]), [h(x) for x in j["nullifiers"]],
                               [h(x) for x in j["macs"]], [h(x) for x in j["commitments"]], j["vpub_old"],
                               j["vpub_new"], h(j["pubkey"]))
        assert [g.hex() for g in got] == j["inputs"], j["name"]


def test_reference_error_classes(Z):
    for e in load_golden("input_prep.json")["prep_errors"]:
        f = e["fields"]
        with pytest.raises(Z.PrepError) as ex:
            if e["kind"] == "spend":
                Z.prep_spend(h(f["cv"]), h(f["anchor"]), h(f["nullifier"]), h(f["rk"]))
            else:
                Z.prep_output(h(f["cv"]), h(f["cmu"]), h(f["epk"]))
        assert ex.value.name == e["error"], (e["name"], e["pinned_by"])


def test_hsig_known_answers(Z):
    for v in load_golden("input_prep.json")["hsig"]:
        got = Z.hsig(h(v["random_seed"]), h(v["nullifiers"][0]), h(v["nullifiers"][1]), h(v["pubkey"]))
        assert got.hex() == v["hsig"]


def test_mutated_points_match_oracle(Z):
    """random byte flips of real cv / rk / epk / cmu / anchor: same accept / error class and
    inputs as the oracle's restatement (sapling-crypto Point::read semantics)."""
    from oracle import zcash as ZO
    tf = load_golden("input_prep.json")["tx_fields"]
    rng = random.Random(21)
    for it in range(60):
        s = dict(tf["spends"][it % len(tf["spends"])])
        field = rng.choice(["cv", "rk", "anchor"])
        b = bytearray(h(s[field]))
        b[rng.randrange(32)] ^= 1 << rng.randrange(8)
        s[field] = b.hex()
        args = [h(s["cv"]), h(s["anchor"]), h(s["nullifier"]), h(s["rk"])]
        try:
            want = [x.to_bytes(32, "little") for x in ZO.spend_inputs(*args)]
        except ZO.InputError as e:
            want = e.where
        try:
            got = Z.prep_spend(*args)
        except Z.PrepError as e:
            got = e.name
        assert got == want, (field, it)
    for it in range(40):
        o = dict(tf["outputs"][it % len(tf["outputs"])])
        field = rng.choice(["cv", "epk", "cmu"])
        b = bytearray(h(o[field]))
        b[rng.randrange(32)] ^= 1 << rng.randrange(8)
        o[field] = b.hex()
        args = [h(o["cv"]), h(o["cmu"]), h(o["epk"])]
        try:
            want = [x.to_bytes(32, "little") for x in ZO.output_inputs(*args)]
        except ZO.InputError as e:
            want = e.where
        try:
            got = Z.prep_output(*args)
        except Z.PrepError as e:
            got = e.name
        assert got == want, (field, it)
