"""The block-level collector (zebra_amd/collector.py) keeps the
reference's error precedence while verifying a whole block in one batch.

CPU tier: the collector's ordering logic on the reference's real transactions, with the
oracle's C++ bellman restatement as the per-proof verifier (checker only).
GPU tier: config 5 -- a replayed block stream mixing Sprout-Groth16 and
Sapling proofs 1 : 4 (Groth16 re-randomization, seed 4) through the product path: all accept,
and a single corrupted JoinSplit surfaces as InvalidJoinSplit(idx) on the right tx."""
import random

import pytest

from tests.conftest import load_golden

SRC_TX = {"bd4fe81c": ["S1", "O1"], "smoky": ["J1"], "991edf59": ["S2", "O3"], "56afac11": ["O2"],
          "53cf8971": ["J2"], "a2a2fe38": ["J3"], "70abe357": ["J4"]}


def h(x):
    return bytes.fromhex(x)


def fields():
    tf = load_golden("input_prep.json")["tx_fields"]
    out = {}
    for kind in ("spends", "outputs", "joinsplits"):
        for e in tf[kind]:
            out[e["name"]] = e
    return out


def make_tx(names, F, proof_of=None):
    """a transaction carrying the named real descriptions (proof bytes optionally replaced)"""
    from zebra_amd.collector import JoinSplit, Output, Spend, Tx
    tx = Tx()
    for nm in names:
        e = F[nm]
        pb = proof_of(nm) if proof_of else h(e["zkproof"])
        if nm[0] == "J":
            tx.js_pubkey = h(e["pubkey"])
            tx.joinsplits.append(JoinSplit(h(e["anchor"]), h(e["random_seed"]), [h(x) for x in e["nullifiers"]],
                                           [h(x) for x in e["macs"]], [h(x) for x in e["commitments"]],
                                           e["vpub_old"], e["vpub_new"], pb))
        elif nm[0] == "S":
            tx.spends.append(Spend(h(e["cv"]), h(e["anchor"]), h(e["nullifier"]), h(e["rk"]), pb))
        else:
            tx.outputs.append(Output(h(e["cv"]), h(e["cmu"]), h(e["epk"]), pb))
    return tx


@pytest.fixture(scope="module")
def cpu_verify():
    from tests import cpulib
    L = cpulib.load()

    def verify(proofs, kinds, inputs, n_inputs):
        return cpulib.verify(L, proofs, kinds, inputs, n_inputs, threads=8)[0]
    return verify


def test_real_block_accepts(cpu_verify):
    from zebra_amd.collector import verify_block
    F = fields()
    txs = [make_tx(v, F) for v in SRC_TX.values()]
    assert verify_block(txs, verify=cpu_verify) is None


def test_error_precedence(cpu_verify):
    """lowest failing tx wins; inside a tx: JoinSplit sig -> JS proofs (index) with tree roots in
    between -> JS nullifiers -> Sapling (any spend/output/binding failure) -> Sapling nullifiers"""
    from zebra_amd.collector import verify_block
    F = fields()
    bad = bytearray(h(F["J1"]["zkproof"]))
    bad[100] ^= 1   # corrupts B -> decode failure or verify failure: either way InvalidJoinSplit

    def txs():
        # a tx's JoinSplits share its pubkey: tx 1 carries J1 twice
        return [make_tx(["S1", "O1"], F), make_tx(["J1", "J1"], F), make_tx(["S2", "O3"], F)]
    t = txs()
    t[1].joinsplits[1].zkproof = bytes(bad)
    assert verify_block(t, verify=cpu_verify) == (1, ("InvalidJoinSplit", 1))
    t = txs()
    t[2].spends[0].cv = bytes(32)                    # small-order cv -> prep error -> InvalidSapling
    assert verify_block(t, verify=cpu_verify) == (2, "InvalidSapling")
    t[1].joinsplits[0].tree_error = "UnknownAnchor"  # lower tx index wins
    assert verify_block(t, verify=cpu_verify) == (1, "UnknownAnchor")
    t[1].joinsplits[0].zkproof = bytes(bad)          # JS 0 proof precedes its own tree root
    assert verify_block(t, verify=cpu_verify) == (1, ("InvalidJoinSplit", 0))
    t[1].js_sig_ok = False                           # ed25519 sig precedes the proofs
    assert verify_block(t, verify=cpu_verify) == (1, "JoinSplitSignature")
    t[0].pre_error = "Eval"                          # an earlier tx's transparent failure wins
    assert verify_block(t, verify=cpu_verify) == (0, "Eval")
    t = txs()
    t[0].spends[0].sig_ok = False
    t[0].sapling_nullifier_error = "SaplingNullifiers"
    assert verify_block(t, verify=cpu_verify) == (0, "InvalidSapling")
    t = txs()
    t[0].sapling_nullifier_error = "SaplingNullifiers"
    assert verify_block(t, verify=cpu_verify) == (0, "SaplingNullifiers")
    t = txs()
    t[1].js_nullifier_error = "JoinSplitNullifiers"
    t[1].joinsplits[0].zkproof = bytes(bad)
    assert verify_block(t, verify=cpu_verify) == (1, ("InvalidJoinSplit", 0))


def test_window_larger_than_max_batch(cpu_verify):
    """an import window with more proofs than one batch holds is verified as
    consecutive batches (verify.max_batch = 3 here) with the statuses joined in order: same
    outcome, same error position as one batch"""
    from zebra_amd.collector import verify_block
    F = fields()
    calls = []

    def small(proofs, kinds, inputs, n_inputs):
        assert len(kinds) <= 3
        calls.append(len(kinds))
        return cpu_verify(proofs, kinds, inputs, n_inputs)
    small.max_batch = 3
    txs = [make_tx(v, F) for v in SRC_TX.values()]
    assert verify_block(txs, verify=small) is None
    assert sum(calls) == 9 and max(calls) == 3 and len(calls) == 3
    bad = bytearray(h(F["O2"]["zkproof"]))
    bad[150] ^= 1
    txs[3].outputs[0].zkproof = bytes(bad)
    calls.clear()
    assert verify_block(txs, verify=small) == (3, "InvalidSapling")
    assert verify_block(txs, verify=cpu_verify) == (3, "InvalidSapling")


@pytest.mark.gpu
def test_config5_replay_block_stream():
    """config 5: blocks of re-randomized real transactions, Sprout-Groth16 : Sapling = 1 : 4 by
    proof count, one zg_verify_batch per block; a corrupted JS surfaces on its tx and index."""
    from zebra_amd import Context
    from zebra_amd.collector import verify_block
    F = fields()
    real = {e["name"]: e for e in load_golden("real_proofs.json")["proofs"]}
    names = ["S1", "S2", "O1", "O2", "O3", "J1", "J2", "J3", "J4"]
    ctx = Context(device=0, max_batch=4096)
    try:
        src = b"".join(h(real[n]["proof"]) for n in names)
        kinds = bytes(real[n]["kind"] for n in names)
        rng = random.Random(4)
        sap = [v for v in SRC_TX.values() if v[0][0] != "J"]
        spr = [v for v in SRC_TX.values() if v[0][0] == "J"]
        blocks = []
        for b in range(6):
            txs_names = []
            nsap = nspr = 0
            while nsap + nspr < 400:
                if nspr * 4 < nsap:
                    pick = rng.choice(spr)
                    nspr += len(pick)
                else:
                    pick = rng.choice(sap)
                    nsap += len(pick)
                txs_names.append(pick)
            blocks.append(txs_names)
        for bi, txs_names in enumerate(blocks):
            flat = [n for t in txs_names for n in t]
            rr = ctx.synth_rerandomize(src, kinds, [names.index(n) for n in flat], 4000 + bi)
            it = iter(range(len(flat)))
            proofs = {}
            txs = []
            for t in txs_names:
                cur = {}
                for n in t:
                    k = next(it)
                    cur[n] = rr[192 * k:192 * k + 192]
                txs.append(make_tx(t, F, proof_of=lambda n, cur=cur: cur[n]))
                proofs[len(txs) - 1] = cur
            assert verify_block(txs, ctx=ctx) is None, bi
            if bi == 2:   # one corrupted JoinSplit proof (A <-> C swapped) in a late tx
                js_tx = [i for i, t in enumerate(txs_names) if t[0][0] == "J"]
                ti = js_tx[len(js_tx) // 2]
                pb = txs[ti].joinsplits[0].zkproof
                txs[ti].joinsplits[0].zkproof = pb[144:] + pb[48:144] + pb[:48]
                assert verify_block(txs, ctx=ctx) == (ti, ("InvalidJoinSplit", 0))
    finally:
        ctx.close()


def signed_txs():
    """the reference's real Sapling transactions with their sighash, signatures and valueBalance
    (tests/golden/sapling_sigs.json): bd4fe81c (S1, O1), 991edf59 (S2, O3), 56afac11 (O2)"""
    F = fields()
    sg = load_golden("sapling_sigs.json")
    sigs = {s["name"]: s for s in sg["sigs"]}
    out = []
    for t in sg["txs"]:
        tx = make_tx(SRC_TX[t["name"]], F)
        tx.sighash = h(t["sighash"])
        tx.value_balance = t["value_balance"]
        tx.binding_sig = h(t["binding_sig"])
        for s in tx.spends:
            s.spend_auth_sig = h(sigs[t["name"] + ":spend_auth"]["sig"])
        out.append(tx)
    return out


def oracle_sig_fns():
    from oracle import sapling_sig as S

    def verify_sigs(vks, sigs, msgs, gens):
        return [S.redjubjub_verify(v, s, m, g) for v, s, m, g in zip(vks, sigs, msgs, gens)]

    def bvk(rows):
        out = []
        for sp, op, vb in rows:
            try:
                p = S.binding_verification_key(sp, op, vb)
            except S.PointError:
                out.append((1, bytes(32)))
                continue
            out.append((2, bytes(32)) if p is None else (0, S.encode(p)))
        return out
    return verify_sigs, bvk


def _sig_cases(run):
    txs = signed_txs()
    assert run(txs) is None
    txs = signed_txs()
    assert [len(t.spends) for t in txs] == [1, 0, 1]
    txs[2].spends[0].spend_auth_sig = bytes(64)            # BadSpendAuthSig -> InvalidSapling
    assert run(txs) == (2, "InvalidSapling")
    txs = signed_txs()
    bs = bytearray(txs[1].binding_sig)
    bs[40] ^= 1
    txs[1].binding_sig = bytes(bs)                          # BadBindingSignature
    assert run(txs) == (1, "InvalidSapling")
    txs[0].spends[0].sig_ok = False                         # unchanged: the GPU verdict is used
    assert run(txs) == (1, "InvalidSapling")
    txs = signed_txs()
    txs[0].value_balance = -(1 << 63)                       # InvalidBalanceValue
    assert run(txs) == (0, "InvalidSapling")
    txs = signed_txs()
    txs[0].value_balance += 1                               # a different bvk: binding fails
    assert run(txs) == (0, "InvalidSapling")
    txs = signed_txs()
    txs[0].sighash = None                                   # no sighash: the caller's verdicts
    txs[0].binding_ok = False
    assert run(txs) == (0, "InvalidSapling")


def test_signatures_in_reference_order_cpu(cpu_verify):
    """the window's RedJubjub checks (oracle verifier here) feed the same precedence"""
    from zebra_amd.collector import verify_block
    vs, bvk = oracle_sig_fns()
    _sig_cases(lambda txs: verify_block(txs, verify=cpu_verify, verify_sigs=vs, sapling_bvk=bvk))


@pytest.mark.gpu
def test_signatures_in_reference_order_gpu():
    """the same with every signature and binding key of the window on the GPU"""
    from zebra_amd import Context
    from zebra_amd.collector import verify_block
    ctx = Context(device=0, max_batch=64)
    try:
        _sig_cases(lambda txs: verify_block(txs, ctx=ctx))
    finally:
        ctx.close()


# ---- PHGR (PGHR13) JoinSplits in the window: mainnet block 522 (tests/golden/pghr13.json)
def pghr_txs():
    """block 522's five transactions with PHGR JoinSplits (one carries two), as the collector's
    Tx view; the BN inputs are derived by the collector (zg_prep_joinsplit_bn)"""
    from zebra_amd.collector import JoinSplit, Tx
    out = []
    for t in load_golden("pghr13.json")["joinsplit_txs"]:
        tx = Tx(js_pubkey=h(t["js_pubkey"]))
        for d in t["joinsplits"]:
            tx.joinsplits.append(JoinSplit(h(d["anchor"]), h(d["random_seed"]), [h(x) for x in d["nullifiers"]],
                                           [h(x) for x in d["macs"]], [h(x) for x in d["commitments"]],
                                           d["vpub_old"], d["vpub_new"], h(d["zkproof"]), groth=False))
        out.append(tx)
    return out


def test_prep_joinsplit_bn_matches_block_522():
    """zg_prep_joinsplit_bn (into_bn_frs, 253-bit chunks) reproduces the inputs of the block-522
    PHGR cases; the BLS packing of the same bits differs (254-bit chunks)"""
    from zebra_amd import zg
    cases = {c["name"]: c for c in load_golden("pghr13.json")["cases"]}
    n = 0
    for t in load_golden("pghr13.json")["joinsplit_txs"]:
        for d in t["joinsplits"]:
            args = (h(d["anchor"]), h(d["random_seed"]), [h(x) for x in d["nullifiers"]], [h(x) for x in d["macs"]],
                    [h(x) for x in d["commitments"]], d["vpub_old"], d["vpub_new"], h(t["js_pubkey"]))
            got = zg.prep_joinsplit_bn(*args)
            assert [g.hex() for g in got] == cases[d["case"]]["inputs"], d["case"]
            assert zg.prep_joinsplit(*args) != got
            n += 1
    assert n == 6


def _corrupt_sign(proof):
    b = bytearray(proof)
    b[0] ^= 1                   # a's y-parity flag: decodes, fails verification (InvalidPGHRProof)
    return bytes(b)


def _corrupt_prefix(proof):
    b = bytearray(proof)
    b[66] = 2                   # b's G2 prefix: from_raw fails (InvalidEncoding)
    return bytes(b)


def _pghr_cases(run, groth_txs):
    """PHGR descriptions in reference precedence, mixed with Groth16 transactions"""
    txs = groth_txs() + pghr_txs()
    base = len(txs) - 5
    assert run(txs) is None
    txs = groth_txs() + pghr_txs()
    js = txs[base + 4].joinsplits                    # the transaction with two PHGR JoinSplits
    js[1].zkproof = _corrupt_sign(js[1].zkproof)
    assert run(txs) == (base + 4, ("InvalidJoinSplit", 1))
    js[0].tree_error = "UnknownAnchor"               # description 0 passes its proof, then its root fails
    assert run(txs) == (base + 4, "UnknownAnchor")
    js[0].zkproof = _corrupt_prefix(js[0].zkproof)   # now description 0's proof fails first
    assert run(txs) == (base + 4, ("InvalidJoinSplit", 0))
    txs[base + 1].joinsplits[0].zkproof = _corrupt_prefix(txs[base + 1].joinsplits[0].zkproof)
    assert run(txs) == (base + 1, ("InvalidJoinSplit", 0))   # the lowest failing transaction wins
    s = txs[1].spends[0] if txs[1].spends else None
    if s is not None:
        s.nullifier = bytes(32)                      # an earlier Groth16 failure wins over both
        assert run(txs) == (1, "InvalidSapling")
    txs = groth_txs() + pghr_txs()
    txs[base + 2].joinsplits[0].pghr_ok = False      # a verdict the caller already holds
    assert run(txs) == (base + 2, ("InvalidJoinSplit", 0))


def _groth_txs():
    F = fields()
    return [make_tx(SRC_TX[k], F) for k in ("smoky", "bd4fe81c", "991edf59")]


def test_pghr_joinsplits_in_reference_order_cpu(cpu_verify):
    """the collector's PHGR queue and precedence with the oracle's PGHR13 verifier (checker only;
    known fixture statements answered from their pinned statuses, mutants verified by the oracle)"""
    from oracle import pghr13 as PG
    from zebra_amd.collector import verify_block
    known = {(c["proof"], tuple(c["inputs"])): c["status"] for c in load_golden("pghr13.json")["cases"]}
    vk = []

    def verify_pghr(proofs, inputs):
        out = []
        for p, x in zip(proofs, inputs):
            k = (bytes(p).hex(), tuple(bytes(v).hex() for v in x))
            if k not in known:
                if not vk:
                    import os
                    from tests.conftest import ROOT
                    vk.append(PG.load_vk_json(open(os.path.join(ROOT, "zebra_amd", "res",
                                                                "sprout-verifying-key.json")).read()))
                known[k] = PG.verify_raw(vk[0], bytes(p), [int.from_bytes(bytes(v), "little") for v in x])
            out.append(known[k])
        return out
    _pghr_cases(lambda txs: verify_block(txs, verify=cpu_verify, verify_pghr=verify_pghr), _groth_txs)


@pytest.mark.gpu
def test_pghr_joinsplits_block_522_gpu():
    """block 522's six PHGR JoinSplits mixed with Groth16 transactions through verify_block on the
    product: one zg_verify_batch + one zg_pghr13_verify per window; corrupted PHGR proofs surface
    as InvalidJoinSplit(index) on the right transaction (accept_transaction.rs:575-592)"""
    from zebra_amd import Context
    from zebra_amd.collector import verify_block
    ctx = Context(device=0, max_batch=64)
    try:
        _pghr_cases(lambda txs: verify_block(txs, ctx=ctx), _groth_txs)
    finally:
        ctx.close()
