"""GPU tier: the affine R-chain (ZG_LINES_AFFINE; zebra_amd/csrc/zg_lines.hip k_batch_lines_aff) feeding
the group line products (k_line_prod's AQ4 program) -- the Miller loop "over affine G2 line
coefficients" of BASELINE.json's north_star, built as a selectable product path.

Lines normalised to a unit v w coefficient differ from pairing's projective lines by factors in
Fq2 * Fq, which the final exponentiation kills, so the 576-B partial is a different element with the
same GT image. Checked: the partial equals the oracle's affine restatement byte for byte
(oracle/groth16.py batch_partial(affine_slots=...), lines from oracle/bls12_381.py affine_lines);
partials of the affine and projective paths have the same final exponentiation (the product of one
and the other's inverse passes zg_gt_check); a corrupted batch -- non-subgroup B among them, whose
vanishing denominators must not poison the lane's other proofs -- gets the exact reject set, through
bisection's re-formed projective lines.

Reference: prepare(B) and miller_loop inside verify_proof, verification/src/sapling.rs:161,206,
verification/src/sprout.rs:73-77."""
import os
import random

import pytest

from tests.conftest import load_golden
from tests.test_gpu_csum import _ctx_env, work4k  # noqa: F401 (fixture)
from tests.test_gpu_parity import corrupted_4096, fx_batch

pytestmark = pytest.mark.gpu

LINE_PROD = {"ZG_LINES_FCHAIN": 0, "ZG_FCHAIN_QUADS": 1}
VARIANTS = [{"ZG_LINES_AFFINE": 2}, {"ZG_LINES_AFFINE": 4}, {"ZG_LINES_AFFINE": 8}, {"ZG_LINES_AFFINE_XL": 1}]


def _ids(e):
    return ",".join("%s=%s" % kv for kv in e.items())


def _pvks():
    from oracle import groth16 as G
    from tests.conftest import ROOT
    files = {0: "sapling-spend-verifying-key.json", 1: "sapling-output-verifying-key.json",
             2: "sprout-groth16-key.json"}
    return {k: G.prepare_verifying_key(G.load_vk_json(open(os.path.join(ROOT, "zebra_amd", "res", f)).read()))
            for k, f in files.items()}


@pytest.mark.parametrize("env", VARIANTS, ids=_ids)
def test_affine_partial_bitexact_vs_oracle(env):
    """golden batch items (incl. a padding slot: 6 proofs, 8 slots), groups of 4: the partial equals the
    oracle's affine batch partial (v w for every slot without a live proof)"""
    from oracle import bls12_381 as B, groth16 as G
    items = load_golden("batch64.json")["items"][:6]
    proofs, kinds, inputs, nin = fx_batch(items)
    r = b"".join(bytes.fromhex(e["r"]) for e in items)
    c = _ctx_env(dict(LINE_PROD, ZG_LINE_GROUP=4, **env), 8)
    try:
        c.batch_begin(proofs, kinds, inputs, nin, r=r)
        part = c.batch_partial()
        c.batch_finish(True, len(items))
        st = c.stats()
    finally:
        c.close()
    assert st["affine_line_batches"] == 1 and st["line_product_batches"] == 1
    want = G.batch_partial(_pvks(), [(e["kind"], bytes.fromhex(e["proof"]),
                                      [int.from_bytes(bytes.fromhex(x), "little") for x in e["inputs"]],
                                      G.batch_r(bytes.fromhex(e["r"]))) for e in items], affine_slots=8)
    assert part == B.f12_to_bytes(want)


@pytest.mark.parametrize("env", VARIANTS, ids=_ids)
def test_affine_and_projective_partials_have_the_same_gt(work4k, env):
    """2,048 proofs, groups of 32, seeded scalars: both paths accept, and FE(affine) = FE(projective)
    (zg_gt_check of the affine partial times the projective partial's inverse)"""
    from oracle import bls12_381 as B
    n = 2048
    proofs, kinds, inputs = work4k
    proofs, kinds, inputs = proofs[:192 * n], kinds[:n], inputs[:288 * n]
    r = random.Random(78).randbytes(16 * n)
    parts = []
    for e in (dict(LINE_PROD, ZG_LINE_GROUP=32), dict(LINE_PROD, ZG_LINE_GROUP=32, **env)):
        c = _ctx_env(e, n)
        try:
            c.batch_begin(proofs, kinds, inputs, r=r)
            parts.append(c.batch_partial())
            assert c.gt_check([parts[-1]])
            assert c.batch_finish(True, n) == [0] * n
            assert c.stats()["affine_line_batches"] == (1 if "ZG_LINES_AFFINE" in str(e) else 0)
        finally:
            c.close()
    assert parts[0] != parts[1]  # different elements ...
    inv = B.f12_to_bytes(B.f12_inv(B.f12_from_bytes(parts[0])))
    from zebra_amd import Context
    c = Context(device=0, max_batch=64)
    try:
        assert c.gt_check([parts[1], inv])  # ... with the same GT image
    finally:
        c.close()


@pytest.mark.parametrize("env", [{"ZG_LINES_AFFINE": 4}, {"ZG_LINES_AFFINE_XL": 1}], ids=_ids)
def test_affine_corrupted_4096_exact_reject_set(env):
    """config 4's 41-in-4,096 batch (non-subgroup B and A, swapped points, tweaked inputs, bad
    encodings) on the affine path with groups of 32: exact statuses; bisection re-forms projective
    lines for the levels below the groups"""
    from zebra_amd import Context
    base = Context(device=0, max_batch=64)
    try:
        proofs, kinds, inputs, want = corrupted_4096(base)
    finally:
        base.close()
    c = _ctx_env(dict(LINE_PROD, ZG_LINE_GROUP=32, **env), 4096)
    try:
        sts, _ = c.verify_batch(proofs, kinds, inputs)
        st = c.stats()
    finally:
        c.close()
    assert sts == want
    assert st["affine_line_batches"] == 1 and st["bisections"] == 1 and st["b_subgroup_recomputes"] == 1
