"""PGHR13 on BN254: the oracle (oracle/bn254.py, oracle/pghr13.py) against
the reference's own vectors (tests/golden/pghr13.json: crypto/src/pghr13.rs proof_decode /
verification tests, sprout.rs smoky_pghr, the PHGR JoinSplits of mainnet block 522), plus the
pairing's bilinearity."""
import os

import pytest

from oracle import bn254 as B, pghr13 as PG
from tests.conftest import ROOT, load_golden

GOLDEN = load_golden("pghr13.json")


@pytest.fixture(scope="module")
def vk():
    return PG.load_vk_json(open(os.path.join(ROOT, "zebra_amd", "res", "sprout-verifying-key.json")).read())


def test_pairing_is_bilinear_and_non_degenerate():
    e = B.pairing(B.G1_GEN, B.G2_GEN)
    assert e != B.F12_ONE and B.f12_pow(e, B.R) == B.F12_ONE
    assert B.pairing(B.ec_mul(B._F1, B.G1_GEN, 6), B.ec_mul(B._F2, B.G2_GEN, 7)) == B.f12_pow(e, 42)


def test_proof_decode_matches_reference():
    """pghr13.rs proof_decode: the 8 decoded points of the sample proof (both compressed forms,
    the G2 Fq2 blob layout and y_gt sign rule); and encoding round trips"""
    pr = PG.proof_from_raw(bytes.fromhex(GOLDEN["sample_proof"]))
    want = GOLDEN["sample_points"]
    for k, v in want.items():
        got = pr[k]
        if k == "b":
            assert [list(got[0]), list(got[1])] == v
        else:
            assert list(got) == v
    assert PG.proof_to_raw(pr).hex() == GOLDEN["sample_proof"]


def test_vk_points_checked(vk):
    assert len(vk["ic"]) == 10
    for k in ("a", "c", "z", "gamma", "gamma_beta_2"):
        assert B.ec_mul(B._F2, vk[k], B.R) is None


@pytest.mark.parametrize("name", ["verification", "smoky_pghr", "mut_b_sign", "mut_b_not_in_subgroup", "mut_input3"])
def test_oracle_verdicts(vk, name):
    c = next(c for c in GOLDEN["cases"] if c["name"] == name)
    inputs = [int.from_bytes(bytes.fromhex(x), "little") for x in c["inputs"]]
    assert PG.verify_raw(vk, bytes.fromhex(c["proof"]), inputs) == c["status"]


def test_fixture_shape():
    st = {c["name"]: c["status"] for c in GOLDEN["cases"]}
    real = [n for n in st if n.startswith(("verification", "smoky", "h522"))]
    assert len(real) == 9 and all(st[n] == PG.OK for n in real)
    assert {st[n] for n in st if n.startswith("mut_")} == {PG.INVALID_ENCODING, PG.INVALID_PROOF}


# ---- the product's BN254 code (zg_bn254.h) on the CPU (tests/native host harness)
def _host():
    from tests import hostlib
    return hostlib.lib(), hostlib.buf


def test_host_bn254_decoders_match_oracle():
    """every point of every fixture proof through the device decoders compiled for the host:
    same accept / reject and the same coordinates as the oracle (bn crate codecs)"""
    L, buf = _host()
    out = buf(128)
    for c in GOLDEN["cases"]:
        raw = bytes.fromhex(c["proof"])
        for off, ln in ((0, 33), (33, 33), (66, 65), (131, 33), (164, 33), (197, 33), (230, 33), (263, 33)):
            enc = raw[off:off + ln]
            try:
                want = B.g1_from_compressed(enc) if ln == 33 else B.g2_from_compressed(enc)
            except B.DecodeError:
                want = None
            ok = (L.zgt_bn_g1_decode if ln == 33 else L.zgt_bn_g2_decode)(enc, out)
            assert bool(ok) == (want is not None), (c["name"], off)
            if ok and ln == 33:
                assert (int.from_bytes(out.raw[:32], "little"), int.from_bytes(out.raw[32:64], "little")) == want
            elif ok:
                v = [int.from_bytes(out.raw[32 * k:32 * k + 32], "little") for k in range(4)]
                assert ((v[0], v[1]), (v[2], v[3])) == want


def test_host_bn254_pairing_matches_oracle():
    import random
    L, buf = _host()
    rnd = random.Random(3)
    p = B.ec_mul(B._F1, B.G1_GEN, rnd.randrange(1, B.R))
    q = B.ec_mul(B._F2, B.G2_GEN, rnd.randrange(1, B.R))
    g1 = p[0].to_bytes(32, "little") + p[1].to_bytes(32, "little")
    g2 = b"".join(v.to_bytes(32, "little") for v in (q[0][0], q[0][1], q[1][0], q[1][1]))
    out = buf(384)
    L.zgt_bn_pairing(g1, g2, out)
    got = [int.from_bytes(out.raw[32 * k:32 * k + 32], "little") for k in range(12)]
    assert got == B.gt_ints(B.final_exponentiation_fc(B.miller_loop([(p, q)])))


def test_host_g2_membership_psi_equals_order_check():
    """the product's G2 membership test [u + 1] Q + psi([u] Q) + psi^2([u] Q) == psi^3([2u] Q)
    (zg_bn254.h ba2_in_subgroup: a 63-bit scalar) decides exactly like AffineG2::new's [r] Q == O
    (ba2_in_subgroup_r, the oracle): G2 points, random twist points, points of the cofactor subgroup
    ([r] of a twist point) and a point of each prime order dividing the cofactor"""
    import ctypes
    import random
    from oracle import bn254 as BN
    from tests import hostlib
    L = hostlib.lib()
    F = BN._F2
    rng = random.Random(23)
    b32 = lambda v: v.to_bytes(32, "little")
    pts = [(BN.ec_mul(F, BN.G2_GEN, rng.randrange(1, BN.R)), True) for _ in range(3)]
    while len(pts) < 9:
        x = (rng.randrange(BN.P), rng.randrange(BN.P))
        y = BN.f2_sqrt(F.add(F.mul(F.mul(x, x), x), F.b))
        if y is None:
            continue
        pts.append(((x, y), False))
        if len(pts) % 3 == 0:
            c = BN.ec_mul(F, (x, y), BN.R)   # order divides the cofactor 2p - r
            if c is not None:
                pts.append((c, False))
    # a point of each prime order l | h' = 2p - r (the twist's cofactor is squarefree: every Sylow
    # subgroup is cyclic, so one point per l pins the product's 63-bit test, zg_bn254.h
    # ba2_in_subgroup, to reject the whole l-part)
    h = 2 * BN.P - BN.R
    primes = [10069, 5864401, 1875725156269, h // (10069 * 5864401 * 1875725156269)]
    assert h == primes[0] * primes[1] * primes[2] * primes[3] and len(set(primes)) == 4
    q = next(p for p, want in pts if not want and BN.ec_mul(F, p, BN.R) is not None)
    for l in primes:
        c = BN.ec_mul(F, q, BN.R * (h // l))
        assert c is not None and BN.ec_mul(F, c, l) is None
        pts.append((c, False))
    for (x, y), want in pts:
        res = (ctypes.c_int * 2)()
        assert L.zgt_bn_g2_membership(b32(x[0]), b32(x[1]), b32(y[0]), b32(y[1]), res) == 1
        assert res[0] == res[1] == int(want)


def test_host_g1_glv_weights():
    """the batch check's weights rho = a + b lambda (zg_pghr13.hip k_pghr_rho, zg_bn254.h bj1_mul_glv):
    the joint 64-bit double-and-add over q and phi(q) equals [a + b lambda mod r] q, and phi(q) =
    (beta x, y) is [lambda] q, on random G1 points and edge halves (0, all-ones)"""
    import ctypes
    import random
    from oracle import bn254 as BN
    from tests import hostlib
    L = hostlib.lib()
    lam = 0xb3c4d79d41a917585bfc41088d8daaa78b17ea66b99c90dd
    rng = random.Random(31)
    b32 = lambda v: v.to_bytes(32, "little")
    halves = [(0, 1), (1, 0), (2**64 - 1, 2**64 - 1), (0, 2**64 - 1)] + \
             [(rng.getrandbits(64), rng.getrandbits(64)) for _ in range(6)]
    for a, b in halves:
        q = BN.ec_mul(BN._F1, BN.G1_GEN, rng.randrange(1, BN.R))
        res = (ctypes.c_int * 2)()
        k = a.to_bytes(8, "little") + b.to_bytes(8, "little")
        assert L.zgt_bn_glv_check(b32(q[0]), b32(q[1]), k, b32((a + b * lam) % BN.R), res) == 1
        assert list(res) == [1, 1], (a, b)
