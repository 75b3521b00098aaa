"""GPU tier (MI355X): the HIP path through the C ABI against the golden fixtures (oracle
outputs on the reference's own proofs) and size-independent properties at larger sizes.
Bar: bit-exact statuses and GT bytes."""
import pytest

from tests.conftest import load_golden

pytestmark = pytest.mark.gpu

KN = {0: "spend", 1: "output", 2: "sprout"}


@pytest.fixture(scope="module")
def ctx():
    from zebra_amd import Context
    c = Context(device=0, max_batch=8192, seed=7)
    yield c
    c.close()


def fx_batch(items):
    from zebra_amd import pack_inputs
    proofs = b"".join(bytes.fromhex(e["proof"]) for e in items)
    kinds = bytes(e["kind"] for e in items)
    inputs = pack_inputs([[bytes.fromhex(x) for x in e["inputs"]] for e in items])
    nin = bytes(len(e["inputs"]) for e in items)
    return proofs, kinds, inputs, nin


def test_library_is_gfx950_hip():
    """the loaded library is the gfx950 build of exactly the sources in this tree (zg_version
    carries their hash, zebra_amd/build.py source_hash)"""
    from zebra_amd import build, zg
    v = zg.lib().zg_version().decode()
    assert "gfx950" in v
    assert v.endswith(" src " + build.source_hash()), (v, build.source_hash())


def test_mad_rate_probe(ctx):
    rate = ctx.bench_mad_rate()
    assert rate > 1e12, rate


def test_alpha_beta(ctx):
    vk = load_golden("vk.json")
    for k, name in KN.items():
        assert ctx.alpha_beta(k).hex() == vk[name]["alpha_g1_beta_g2"]


def test_verify_one_gt_real(ctx):
    for e in load_golden("real_proofs.json")["proofs"]:
        st, gt = ctx.verify_one_gt(e["kind"], bytes.fromhex(e["proof"]), [bytes.fromhex(x) for x in e["inputs"]])
        assert st == 0, e["name"]
        assert gt.hex() == e["lhs_gt"], e["name"]


def test_verify_each_real_and_mutants(ctx):
    items = load_golden("real_proofs.json")["proofs"] + [
        m for m in load_golden("mutants.json")["mutants"] if m["vk"] == "builtin"]
    proofs, kinds, inputs, nin = fx_batch(items)
    sts, gts = ctx.verify_each(proofs, kinds, inputs, nin)
    for e, st, gt in zip(items, sts, gts):
        assert st == e["status"], e.get("name")
        if e.get("lhs_gt"):
            assert gt.hex() == e["lhs_gt"], e.get("name")


def test_bad_vk_malformed(ctx):
    """verification/src/sapling.rs:428-432: an empty-ic VK -> Proof(Synthesis)."""
    from zebra_amd import Context
    c = Context(device=0, max_batch=64, load_builtin=False)
    g1 = bytes([0x40]) + bytes(95)
    g2 = bytes([0x40]) + bytes(191)
    c.vk_load_uncompressed(0, g1, g1, g2, g2, g1, g2, [])
    e = load_golden("real_proofs.json")["proofs"][0]
    st, _ = c.verify_one_gt(0, bytes.fromhex(e["proof"]), [bytes.fromhex(x) for x in e["inputs"]])
    assert st == 2
    c.close()


def test_rerandomize_matches_oracle(ctx):
    b = load_golden("batch64.json")
    real = {e["name"]: e for e in load_golden("real_proofs.json")["proofs"]}
    srcs = ["S1", "S2", "O1", "O2", "O3", "J1", "J2", "J3", "J4"]
    src_proofs = b"".join(bytes.fromhex(real[s]["proof"]) for s in srcs)
    src_kinds = bytes(real[s]["kind"] for s in srcs)
    out = ctx.synth_rerandomize(src_proofs, src_kinds, [i % 9 for i in range(64)], b["seed"])
    for i, it in enumerate(b["items"]):
        if it["corruption"] in (None, "input0_plus1"):
            assert out[192 * i:192 * (i + 1)].hex() == it["proof"], i


def test_batch64_statuses_and_gt(ctx):
    b = load_golden("batch64.json")
    items = b["items"]
    proofs, kinds, inputs, nin = fx_batch(items)
    r = b"".join(bytes.fromhex(e["r"]) for e in items)
    sts, gt = ctx.verify_batch(proofs, kinds, inputs, nin, r=r, want_gt=True)
    assert sts == [e["status"] for e in items]
    assert gt.hex() == b["gt_out"]


def test_batch_all_valid_real(ctx):
    items = load_golden("real_proofs.json")["proofs"]
    proofs, kinds, inputs, nin = fx_batch(items)
    sts, _ = ctx.verify_batch(proofs, kinds, inputs, nin)
    assert sts == [0] * len(items)


def test_split_partials(ctx):
    """two shards -> two 576-byte partials -> one final exponentiation (the RCCL path's math)."""
    b = load_golden("batch64.json")
    good = [e for e in b["items"] if e["status"] == 0]
    parts = []
    for shard in (good[:20], good[20:]):
        proofs, kinds, inputs, nin = fx_batch(shard)
        ctx.batch_begin(proofs, kinds, inputs, nin)
        parts.append(ctx.batch_partial())
        assert ctx.batch_finish(True, len(shard)) == [0] * len(shard)
    assert ctx.gt_check(parts)
    bad = [e for e in b["items"] if e["status"] == 3]
    proofs, kinds, inputs, nin = fx_batch(bad + good[:5])
    ctx.batch_begin(proofs, kinds, inputs, nin)
    p2 = ctx.batch_partial()
    assert not ctx.gt_check([parts[0], p2])
    assert ctx.batch_finish(False, len(bad) + 5) == [3] * len(bad) + [0] * 5
    # zg_gt_check_many (round 6): several batches' verdicts in one launch, each its own set -- the
    # same verdicts as one zg_gt_check per set, a false set among true ones, 16 sets at the limit
    sets = [parts, [parts[0], p2], parts[::-1], [parts[0], p2, parts[1]]]
    assert ctx.gt_check_many(sets) == [ctx.gt_check(p) for p in sets] == [True, False, True, False]
    assert ctx.gt_check_many(sets * 4) == [True, False, True, False] * 4
    assert ctx.gt_check_many([parts]) == [True]
    with pytest.raises(ValueError):
        ctx.gt_check_many(sets * 5)
    with pytest.raises(ValueError):
        ctx.gt_check_many([parts, []])


def test_batch_4096_one_percent_corrupted(ctx):
    """config 4 shape: 4,096 re-randomized proofs, 41 corrupted -> exact reject set."""
    proofs, kinds, inputs, want = corrupted_4096(ctx)
    sts, _ = ctx.verify_batch(proofs, kinds, inputs)
    assert sts == want


@pytest.mark.parametrize("group", [None, "32", "4096"])
def test_batch_4096_corrupted_quad_fchain(ctx, monkeypatch, group):
    """the same 41-in-4,096 batch with the four-proofs-per-lane f-chain forced (ZG_FCHAIN_QUADS=1,
    split launches): the quad tree level has no pair nodes below it, and bisection must still
    reach the exact reject set. group: ZG_LINE_GROUP -- default (below 32,768 proofs the quad chain),
    32 (group line products of 32 proofs: no tree below the groups until bisection runs the quad
    chain), 4096 (one group: the chain writes the root)"""
    from zebra_amd import Context
    proofs, kinds, inputs, want = corrupted_4096(ctx)
    monkeypatch.setenv("ZG_FCHAIN_QUADS", "1")
    monkeypatch.setenv("ZG_LINES_FCHAIN", "0")
    if group is not None:
        monkeypatch.setenv("ZG_LINE_GROUP", group)
    q = Context(device=0, max_batch=4096)
    try:
        sts, _ = q.verify_batch(proofs, kinds, inputs)
        st = q.stats()
    finally:
        q.close()
    assert sts == want
    assert st["quad_fchain_launches"] >= 1 and st["fused_launches"] == 0 and st["bisections"] == 1
    assert st["line_product_batches"] == (0 if group is None else st["quad_fchain_launches"])


def corrupted_4096(ctx):
    import random
    from zebra_amd import pack_inputs
    real = load_golden("real_proofs.json")["proofs"]
    pts = load_golden("points.json")
    n = 4096
    src_proofs = b"".join(bytes.fromhex(e["proof"]) for e in real)
    src_kinds = bytes(e["kind"] for e in real)
    idx = [i % len(real) for i in range(n)]
    proofs = bytearray(ctx.synth_rerandomize(src_proofs, src_kinds, idx, 3))
    rows = [[bytes.fromhex(x) for x in real[j]["inputs"]] for j in idx]
    rng = random.Random(3)
    bad = sorted(rng.sample(range(n), 41))
    want = [0] * n
    for q, i in enumerate(bad):
        kind = q % 5
        if kind == 0:     # public-input tweak -> VERIFY_FAILED
            x = bytearray(rows[i][0])
            x[0] ^= 1
            rows[i] = [bytes(x)] + rows[i][1:]
            want[i] = 3
        elif kind == 1:   # A <-> C swap -> VERIFY_FAILED
            p = proofs[192 * i:192 * i + 192]
            proofs[192 * i:192 * i + 192] = p[144:] + p[48:144] + p[:48]
            want[i] = 3
        elif kind == 2:   # compression flag cleared -> DECODE_INVALID
            proofs[192 * i] &= 0x7F
            want[i] = 1
        elif kind == 3:   # non-subgroup G2 B -> DECODE_INVALID
            proofs[192 * i + 48:192 * i + 144] = bytes.fromhex(pts["g2_not_in_subgroup"])
            want[i] = 1
        else:             # non-subgroup G1 A -> DECODE_INVALID
            proofs[192 * i:192 * i + 48] = bytes.fromhex(pts["g1_not_in_subgroup"])
            want[i] = 1
    return bytes(proofs), bytes(src_kinds[j] for j in idx), pack_inputs(rows), want


def test_partial_bitexact_vs_oracle(ctx):
    """the 576-byte Miller partial a rank contributes equals the oracle's batch_partial."""
    import os
    from oracle import bls12_381 as B, groth16 as G
    from tests.conftest import ROOT
    files = {0: "sapling-spend-verifying-key.json", 1: "sapling-output-verifying-key.json",
             2: "sprout-groth16-key.json"}
    pvks = {k: G.prepare_verifying_key(G.load_vk_json(open(os.path.join(ROOT, "zebra_amd", "res", f)).read()))
            for k, f in files.items()}
    items = load_golden("batch64.json")["items"][:6]
    proofs, kinds, inputs, nin = fx_batch(items)
    r = b"".join(bytes.fromhex(e["r"]) for e in items)
    ctx.batch_begin(proofs, kinds, inputs, nin, r=r)
    part = ctx.batch_partial()
    ctx.batch_finish(True, len(items))
    want = G.batch_partial(pvks, [(e["kind"], bytes.fromhex(e["proof"]),
                                   [int.from_bytes(bytes.fromhex(x), "little") for x in e["inputs"]],
                                   G.batch_r(bytes.fromhex(e["r"]))) for e in items])
    assert part == B.f12_to_bytes(want)


def test_batch_state_errors(ctx):
    """a second zg_batch_begin while a batch is in flight is ZG_E_STATE (the first
    batch is not silently discarded); finishing it then works; finish without begin is
    ZG_E_STATE too"""
    from zebra_amd.zg import ZgError
    items = load_golden("real_proofs.json")["proofs"]
    proofs, kinds, inputs, nin = fx_batch(items)
    ctx.batch_begin(proofs, kinds, inputs, nin)
    with pytest.raises(ZgError) as e:
        ctx.batch_begin(proofs, kinds, inputs, nin)
    assert e.value.code == -6
    part = ctx.batch_partial()
    assert ctx.gt_check([part])
    assert ctx.batch_finish(True, len(items)) == [0] * len(items)
    with pytest.raises(ZgError) as e:
        ctx.batch_finish(True, len(items))
    assert e.value.code == -6


def test_many_slots_in_flight():
    """20 contexts (batch slots) on one GPU, all with a batch in flight at once: the slots share
    the device's fixed stream pool and its prepared VKs (no stream or queue per slot), and
    every batch verifies"""
    from zebra_amd import Context, pack_inputs
    real = load_golden("real_proofs.json")["proofs"]
    src_proofs = b"".join(bytes.fromhex(e["proof"]) for e in real)
    src_kinds = bytes(e["kind"] for e in real)
    n = 256
    cs = [Context(device=0, max_batch=n) for _ in range(20)]
    try:
        idx = [i % len(real) for i in range(n)]
        proofs = cs[0].synth_rerandomize(src_proofs, src_kinds, idx, 31)
        kinds = bytes(src_kinds[j] for j in idx)
        inputs = pack_inputs([[bytes.fromhex(x) for x in real[j]["inputs"]] for j in idx])
        for c in cs:
            c.batch_begin(proofs, kinds, inputs)
        parts = [c.batch_partial() for c in cs]
        for c, p in zip(cs, parts):
            assert c.gt_check([p])
            assert c.batch_finish(True, n) == [0] * n
        assert len(set(parts)) == 20   # independent OS-random batch scalars per batch
    finally:
        for c in cs:
            c.close()


def test_debug_each_cross_check():
    """ZG_DEBUG_EACH=1 (debug mode): every batch's statuses are re-checked on the
    device by the per-proof verify_proof kernel; a clean and a corrupted batch pass the check
    (no ZG_E_DEBUG) and keep the oracle's reject set"""
    import os
    from tests import cpulib
    from tests.test_gpu_configs import SRCS, _sources, config3_indices, corrupt, oracle_statuses
    from zebra_amd import Context, pack_inputs
    _, src_proofs, src_kinds, rows = _sources()
    n = 512
    idx = config3_indices(n)
    os.environ["ZG_DEBUG_EACH"] = "1"
    try:
        c = Context(device=0, max_batch=n)
    finally:
        del os.environ["ZG_DEBUG_EACH"]
    try:
        proofs = c.synth_rerandomize(src_proofs, src_kinds, idx, 5)
        kinds = bytes(src_kinds[j] for j in idx)
        inputs = pack_inputs([rows[SRCS[j]] for j in idx])
        assert c.verify_batch(proofs, kinds, inputs)[0] == [0] * n
        bp, bx, bad = corrupt(proofs, kinds, inputs, 12, 3)
        want = oracle_statuses(cpulib.load(), bp, kinds, bx, bad)
        sts, _ = c.verify_batch(bp, kinds, bx)
        assert {i: s for i, s in enumerate(sts) if s} == want
    finally:
        c.close()
