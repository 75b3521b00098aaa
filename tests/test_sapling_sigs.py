"""Sapling signature checks: RedJubjub spend_auth_sig / binding_sig, the
binding verification key and Jubjub point decoding, on the GPU against the oracle
(oracle/sapling_sig.py), which is pinned here by the reference's own data.

CPU tier: the oracle's ZIP-143/243 signature hash against the official vectors the reference
holds (script/data/sighash_tests.json, sample in tests/golden/sapling_sigs.json), and its
RedJubjub verdicts on the reference's real transactions (sapling.rs:303-305 accept_sapling_works;
block 419221, test-data/src/lib.rs:117-131) and on the pinned failure classes (zero signature
-> BadSpendAuthSig, sapling.rs:414-419; total = 0 -> BadBindingSignature, :525-529).
GPU tier: zg_redjubjub_verify / zg_sapling_bvk / zg_jubjub_decode give the oracle's answers."""
import random

import pytest

from tests.conftest import load_golden


def fx():
    return load_golden("sapling_sigs.json")


def test_oracle_sighash_matches_reference_vectors():
    from oracle import sapling_sig as S
    vecs = fx()["sighash_vectors"]
    assert len(vecs) >= 40 and {v["branch_id"] for v in vecs} >= {0x5BA81B19, 0x76B809BB}
    for v in vecs:
        t = S.parse_tx_raw(bytes.fromhex(v["tx"]))
        got = S.sighash(t, v["input_index"], bytes.fromhex(v["script"]), 0, v["hashtype"], v["branch_id"])
        assert got.hex() == v["sighash"]


def test_oracle_signature_verdicts():
    from oracle import sapling_sig as S
    for s in fx()["sigs"]:
        got = S.redjubjub_verify(bytes.fromhex(s["vk"]), bytes.fromhex(s["sig"]), bytes.fromhex(s["msg"]), s["gen"])
        assert got == s["ok"], s["name"]
    names = {s["name"]: s["ok"] for s in fx()["sigs"]}
    assert names["bd4fe81c:spend_auth"] and names["bd4fe81c:binding"]       # accept_sapling_works
    assert not names["zero_sig"] and not names["bd4fe81c:binding_total_zero"]
    for t in fx()["txs"]:
        bvk = S.binding_verification_key([bytes.fromhex(c) for c in t["spend_cvs"]],
                                         [bytes.fromhex(c) for c in t["output_cvs"]], t["value_balance"])
        assert S.encode(bvk).hex() == t["bvk"]


def _ctx():
    from zebra_amd import Context
    return Context(device=0, max_batch=64, load_builtin=False)


@pytest.mark.gpu
def test_gpu_redjubjub_fixtures():
    c = _ctx()
    try:
        sigs = fx()["sigs"] + fx()["signed_batch"]
        got = c.redjubjub_verify([bytes.fromhex(s["vk"]) for s in sigs], [bytes.fromhex(s["sig"]) for s in sigs],
                                 [bytes.fromhex(s["msg"]) for s in sigs], [s["gen"] for s in sigs])
        assert got == [s["ok"] for s in sigs], [s.get("name") for s, g in zip(sigs, got) if g != s["ok"]]
    finally:
        c.close()


@pytest.mark.gpu
def test_gpu_redjubjub_batch_4096_exact():
    """4,096 signatures (the oracle-signed batch and the real ones, repeated), 1 % corrupted in
    rotating ways: the GPU's per-signature verdicts equal the oracle's"""
    from oracle import sapling_sig as S
    base = [s for s in fx()["sigs"] if s["ok"]] + fx()["signed_batch"]
    rng = random.Random(11)
    items, want = [], []
    for i in range(4096):
        s = base[i % len(base)]
        vk, sig, msg, gen = bytearray.fromhex(s["vk"]), bytearray.fromhex(s["sig"]), bytearray.fromhex(s["msg"]), s["gen"]
        if rng.random() < 0.01:
            k = rng.randrange(5)
            if k == 0:
                msg[rng.randrange(64)] ^= 1 << rng.randrange(8)
            elif k == 1:
                sig[32 + rng.randrange(31)] ^= 1 << rng.randrange(8)
            elif k == 2:
                sig[rng.randrange(32)] ^= 1 << rng.randrange(8)
            elif k == 3:
                vk[rng.randrange(32)] ^= 1 << rng.randrange(8)
            else:
                gen ^= 1
            want.append(S.redjubjub_verify(bytes(vk), bytes(sig), bytes(msg), gen))
        else:
            want.append(True)
        items.append((bytes(vk), bytes(sig), bytes(msg), gen))
    c = _ctx()
    try:
        got = c.redjubjub_verify(*[list(x) for x in zip(*items)])
    finally:
        c.close()
    assert got == want
    assert 20 < want.count(False) < 60


@pytest.mark.gpu
def test_gpu_binding_verification_keys():
    from oracle import sapling_sig as S
    txs = fx()["txs"]
    rows = [([bytes.fromhex(x) for x in t["spend_cvs"]], [bytes.fromhex(x) for x in t["output_cvs"]], t["value_balance"])
            for t in txs]
    cv = rows[0][0][0]
    rows += [([cv], [], -(1 << 63)), ([cv[16:] + cv[:16]], [], 5), ([], [], 0), ([cv], [cv], -123456789),
             ([], [rows[0][1][0]], (1 << 63) - 1)]
    c = _ctx()
    try:
        got = c.sapling_bvk(rows)
    finally:
        c.close()
    for i, (st, bvk) in enumerate(got):
        sp, op, vb = rows[i]
        if i < len(txs):
            assert st == 0 and bvk.hex() == txs[i]["bvk"]
            continue
        try:
            want = S.binding_verification_key(sp, op, vb)
        except S.PointError:
            assert st == 1, i
            continue
        if want is None:
            assert st == 2, i
        else:
            assert st == 0 and bvk == S.encode(want), i


@pytest.mark.gpu
def test_gpu_jubjub_decode_vs_oracle():
    from oracle import zcash as Z
    tf = load_golden("input_prep.json")["tx_fields"]
    pts = [bytes.fromhex(e[k]) for k in ("cv", "rk", "epk") for grp in ("spends", "outputs") for e in tf[grp] if k in e]
    rng = random.Random(5)
    pts += [bytes(32), b"\xff" * 32, (1).to_bytes(32, "little"), (Z.R - 1).to_bytes(32, "little"),
            ((Z.R - 1) | (1 << 255)).to_bytes(32, "little"), (1 | (1 << 255)).to_bytes(32, "little")]
    pts += [p[16:] + p[:16] for p in pts[:6]] + [rng.randbytes(32) for _ in range(200)]
    c = _ctx()
    try:
        got = c.jubjub_decode(pts)
    finally:
        c.close()
    for p, (st, x, y) in zip(pts, got):
        try:
            q = Z.jubjub_read(p)
            want = 2 if Z.is_small_order(q) else 0
        except Z.PointError:
            want, q = 1, None
        assert st == want, p.hex()
        if want != 1:
            assert (x, y) == q
