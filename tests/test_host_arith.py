"""CPU tier: the product's device arithmetic (zebra_amd/csrc/*.h, compiled for the host by
tests/native) against the oracle (oracle/bls12_381.py)."""
import random

import pytest

from oracle import bls12_381 as B
from tests import hostlib

P = B.P


@pytest.fixture(scope="module")
def L():
    return hostlib.lib()


def fq_b(x):
    return x.to_bytes(48, "big")


def rnd_f12(rng):
    return B.f12_from_coeffs([rng.randrange(P) for _ in range(12)])


def test_fq_ops(L):
    rng = random.Random(1)
    out = hostlib.buf(48)
    for _ in range(200):
        a, b = rng.randrange(P), rng.randrange(P)
        for fn, want in ((L.zgt_fq_mul, a * b % P), (L.zgt_fq_add, (a + b) % P), (L.zgt_fq_sub, (a - b) % P)):
            fn(fq_b(a), fq_b(b), out)
            assert int.from_bytes(out.raw, "big") == want
    for a in (1, 2, P - 1, rng.randrange(P)):
        L.zgt_fq_inv(fq_b(a), out)
        assert int.from_bytes(out.raw, "big") * a % P == 1
        ok = L.zgt_fq_sqrt(fq_b(a), out)
        assert bool(ok) == (B.fq_sqrt(a) is not None)
        if ok:
            assert pow(int.from_bytes(out.raw, "big"), 2, P) == a


def test_binary_gcd_inverse(L):
    """zg_bingcd.h (Pornin's binary GCD, variable time) against pow(y, -1, p): Fr and Fq, random
    and edge residues (0 -> 0, 1, p - 1, powers of two, values with long runs of equal bits)"""
    rng = random.Random(4)
    R = B.R
    out = hostlib.buf(48)
    edge_r = [0, 1, 2, R - 1, R - 2, 1 << 254, (1 << 255) % R, (1 << 200) - 1, R >> 1, 3]
    for y in edge_r + [rng.randrange(R) for _ in range(3000)]:
        L.zgt_fr_inv_vt(y.to_bytes(32, "little"), out)
        assert int.from_bytes(out.raw[:32], "little") == (pow(y, -1, R) if y else 0), hex(y)
    for y in edge_r[:4] + [rng.randrange(1, R) for _ in range(300)]:
        L.zgt_fr_inv_vt_mont(y.to_bytes(32, "little"), out)
        assert int.from_bytes(out.raw[:32], "little") == (pow(y, -1, R) if y else 0), hex(y)
    edge_q = [0, 1, 2, P - 1, P - 2, 1 << 380, (1 << 381) % P, (1 << 300) - 1, P >> 1]
    for y in edge_q + [rng.randrange(P) for _ in range(1500)]:
        L.zgt_fq_inv_vt(fq_b(y), out)
        assert int.from_bytes(out.raw, "big") == (pow(y, -1, P) if y else 0), hex(y)


def test_fr_mul(L):
    rng = random.Random(2)
    out = hostlib.buf(32)
    for _ in range(100):
        a, b = rng.randrange(B.R), rng.randrange(B.R)
        L.zgt_fr_mul(a.to_bytes(32, "little"), b.to_bytes(32, "little"), out)
        assert int.from_bytes(out.raw, "little") == a * b % B.R


def test_f12_ops(L):
    rng = random.Random(3)
    out = hostlib.buf(576)
    for _ in range(5):
        a, b = rnd_f12(rng), rnd_f12(rng)
        L.zgt_f12_mul(B.f12_to_bytes(a), B.f12_to_bytes(b), out)
        assert out.raw == B.f12_to_bytes(B.f12_mul(a, b))
        L.zgt_f12_sqr(B.f12_to_bytes(a), out)
        assert out.raw == B.f12_to_bytes(B.f12_sqr(a))
        L.zgt_f12_inv(B.f12_to_bytes(a), out)
        assert out.raw == B.f12_to_bytes(B.f12_inv(a))
        for k in (1, 2, 3):
            L.zgt_f12_frob(B.f12_to_bytes(a), k, out)
            assert out.raw == B.f12_to_bytes(B.f12_frob(a, k))


def test_f2_sqrt(L):
    rng = random.Random(4)
    out = hostlib.buf(96)
    cases = [(rng.randrange(P), rng.randrange(P)) for _ in range(40)]
    # a in Fq (both branches: a0 a square / -a0 a square), zero, pure imaginary, squares of x + 0u / 0 + xu
    cases += [(rng.randrange(P), 0) for _ in range(6)] + [(0, 0), (0, rng.randrange(P)), (P - 1, 0), (1, 0)]
    for _ in range(4):
        x = rng.randrange(P)
        cases += [B.f2_sqr((x, 0)), B.f2_sqr((0, x)), B.f2_sqr((x, rng.randrange(P)))]
    for a in cases:
        ok = L.zgt_f2_sqrt(fq_b(a[0]) + fq_b(a[1]), out)
        want = B.f2_sqrt(a)
        assert bool(ok) == (want is not None)
        if ok:
            s = (int.from_bytes(out.raw[:48], "big"), int.from_bytes(out.raw[48:], "big"))
            assert B.f2_sqr(s) == a


def test_final_exp_and_miller(L):
    rng = random.Random(5)
    out = hostlib.buf(576)
    f = rnd_f12(rng)
    L.zgt_final_exp(B.f12_to_bytes(f), out)
    assert out.raw == B.f12_to_bytes(B.final_exponentiation(f))
    p = B.ec_mul(B.FQ, B.G1_GEN, 12345)
    q = B.ec_mul(B.FQ2, B.G2_GEN, 678)
    L.zgt_miller(fq_b(p[0]) + fq_b(p[1]), b"".join(fq_b(v) for v in (q[0][0], q[0][1], q[1][0], q[1][1])), out)
    assert out.raw == B.f12_to_bytes(B.miller_loop([(p, B.g2_prepare(q))]))


def test_subgroup_checks(L):
    rng = random.Random(6)
    out = hostlib.buf(192)
    # in-subgroup points
    for k in (1, 7, rng.randrange(B.R)):
        p = B.ec_mul(B.FQ, B.G1_GEN, k)
        assert L.zgt_g1_in_subgroup(fq_b(p[0]) + fq_b(p[1])) == 1
        q = B.ec_mul(B.FQ2, B.G2_GEN, k)
        assert L.zgt_g2_in_subgroup(b"".join(fq_b(v) for v in (q[0][0], q[0][1], q[1][0], q[1][1]))) == 1
    # random on-curve points: compare with the oracle's naive [r]P check
    n1 = n2 = 0
    while n1 < 6:
        x = rng.randrange(P)
        y = B.fq_sqrt((x ** 3 + 4) % P)
        if y is None:
            continue
        n1 += 1
        assert L.zgt_g1_in_subgroup(fq_b(x) + fq_b(y)) == int(B.g1_in_subgroup((x, y)))
    while n2 < 3:
        x = (rng.randrange(P), rng.randrange(P))
        y = B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(x), x), B.B2))
        if y is None:
            continue
        n2 += 1
        assert L.zgt_g2_in_subgroup(b"".join(fq_b(v) for v in (x[0], x[1], y[0], y[1]))) == int(
            B.g2_in_subgroup((x, y)))


def test_lazy_linear_forms(L):
    """zg_coop.h LazyAcc: any 384-bit terms, |c| < 128, <= 8 terms -> value mod p, < 2.2p
    (canon: < p); the extremes of the bounds included."""
    import ctypes
    rng = random.Random(8)
    out = (ctypes.c_uint32 * 12)()
    top = (1 << 384) - 1
    for it in range(400):
        n = rng.randrange(1, 9)
        if it % 4 == 0:
            xs = [top] * n
            cs = [rng.choice((-127, 127)) for _ in range(n)]
        else:
            xs = [rng.choice((rng.randrange(P), rng.randrange(1 << 384), rng.randrange(3 * P))) % (1 << 384)
                  for _ in range(n)]
            cs = [rng.randrange(-127, 128) for _ in range(n)]
        xa = (ctypes.c_uint32 * (12 * n))(*[(x >> (32 * i)) & 0xFFFFFFFF for x in xs for i in range(12)])
        ca = (ctypes.c_int * n)(*cs)
        want = sum(c * x for c, x in zip(cs, xs)) % P
        for canon in (0, 1):
            L.zgt_lazy_form(xa, ca, n, canon, out)
            got = sum(int(out[i]) << (32 * i) for i in range(12))
            assert got % P == want
            assert got < (P if canon else (22 * P) // 10)


def test_batch_scalar_glv(L):
    """zg_groth16.h: r_i = (2a+1) + b lambda from 16 bytes, and [r_i] P by the sign-aligned GLV
    columns, against the oracle's plain scalar multiplication."""
    from oracle import groth16 as G
    rng = random.Random(9)
    out = hostlib.buf(96)
    fr = hostlib.buf(32)
    assert (G.LAMBDA * G.LAMBDA + G.LAMBDA + 1) % B.R == 0
    cases = [bytes(16), b"\xff" * 16, b"\xff" * 8 + bytes(8), bytes(8) + b"\xff" * 8]
    cases += [bytes(rng.getrandbits(8) for _ in range(16)) for _ in range(8)]
    for k, r16 in enumerate(cases):
        r = G.batch_r(r16)
        L.zgt_batch_scalar(r16, fr)
        assert int.from_bytes(fr.raw, "little") == r
        p = B.ec_mul(B.FQ, B.G1_GEN, 1 + 7919 * k)
        L.zgt_g1_glv_mul(fq_b(p[0]) + fq_b(p[1]), r16, out)
        q = B.ec_mul(B.FQ, p, r)
        assert (int.from_bytes(out.raw[:48], "big"), int.from_bytes(out.raw[48:], "big")) == q


@pytest.mark.parametrize("field", [0, 1, 2, 3, 4])
def test_field_products_host_edges(L, field):
    """the operand sets of tests/test_gpu_field.py through the same generated products on the
    host (zgt_field_mul == zg_debug_field_mul's switch): pins the expected values the GPU test
    asserts, and the generated C itself on its edge operands"""
    import ctypes
    from tests import test_gpu_field as TF
    fn = L.zgt_field_mul
    fn.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
    if field == 2:
        pairs = TF.fq2_cases()[:1500]
        for x, y in pairs:
            out = ctypes.create_string_buffer(96)
            fn(2, TF.fq2_enc(x), TF.fq2_enc(y), out)
            assert (int.from_bytes(out.raw[:48], "little"), int.from_bytes(out.raw[48:], "little")) == \
                TF.fq2_expected(x, y)
        return
    w = TF.FIELDS[field][2]
    pairs = TF.cases(field)[:3000]
    got = []
    for x, y in pairs:
        out = ctypes.create_string_buffer(w)
        fn(field, x.to_bytes(w, "little"), y.to_bytes(w, "little"), out)
        got.append(out.raw)
    assert not TF.mismatches(field, pairs, got)


def test_lines_lane_equals_g2_prepared(L):
    """the straight-line R-chain steps of zg_lines.h (k_batch_lines_lane) give exactly the scaled
    G2Prepared lines of pairing's doubling_step / addition_step (zg_pairing.h g2_prepare + ell's
    px / py scaling), all 68 triples, for random B in G2 and P in G1"""
    import ctypes
    rng = random.Random(31)
    for _ in range(3):
        q = B.ec_mul(B.FQ2, B.G2_GEN, rng.randrange(1, B.R))
        p = B.ec_mul(B.FQ, B.G1_GEN, rng.randrange(1, B.R))
        qb = b"".join(fq_b(v) for v in (q[0][0], q[0][1], q[1][0], q[1][1]))
        pb = fq_b(p[0]) + fq_b(p[1])
        a, r = ctypes.create_string_buffer(68 * 3 * 96), ctypes.create_string_buffer(68 * 3 * 96)
        L.zgt_lines_lane(qb, pb, a, r)
        assert a.raw == r.raw


def test_affine_lines_equal_oracle(L):
    """the affine R-chain step of zg_lines.h (k_batch_lines_aff, ZG_LINES_AFFINE) gives the oracle's
    unit-normalised lines (oracle/bls12_381.py affine_lines) for all 68 steps, and ends at [x] B; the
    oracle's lines are pairing's projective lines up to Fq2 * Fq factors (same GT image,
    test_affine_miller_value_has_the_pairing_gt)"""
    import ctypes
    rng = random.Random(32)
    for _ in range(3):
        q = B.ec_mul(B.FQ2, B.G2_GEN, rng.randrange(1, B.R))
        p = B.ec_mul(B.FQ, B.G1_GEN, rng.randrange(1, B.R))
        qb = b"".join(fq_b(v) for v in (q[0][0], q[0][1], q[1][0], q[1][1]))
        pb = fq_b(p[0]) + fq_b(p[1])
        out, last = ctypes.create_string_buffer(68 * 2 * 96), ctypes.create_string_buffer(192)
        L.zgt_lines_affine(qb, pb, out, last)
        want = b"".join(fq_b(c) for ab in B.affine_lines(q, p) for f in ab for c in f)
        assert out.raw == want
        xq = B.ec_mul(B.FQ2, q, B.BLS_X)
        assert last.raw == b"".join(fq_b(v) for v in (xq[0][0], xq[0][1], xq[1][0], xq[1][1]))


def test_affine_miller_value_has_the_pairing_gt():
    """the Miller chain over unit-normalised affine lines has the projective miller_loop's final
    exponentiation (the normalisations are Fq2 * Fq factors), and the idle line v w maps to 1"""
    rng = random.Random(33)
    q = B.ec_mul(B.FQ2, B.G2_GEN, rng.randrange(1, B.R))
    p = B.ec_mul(B.FQ, B.G1_GEN, rng.randrange(1, B.R))
    fa = B.miller_chain_affine([B.affine_lines(q, p)])
    fp = B.miller_loop([(p, B.g2_prepare(q))])
    assert fa != fp and B.final_exponentiation(fa) == B.final_exponentiation(fp)
    assert B.final_exponentiation(B.miller_chain_affine([[B.AFFINE_IDLE_LINE] * 68])) == B.F12_ONE


def test_msm_windows_cover_the_scalar_evenly():
    """K4's signed-digit windows (zg_msm.h msm_shape / msm_digit, k_msm_count / k_msm_scatter):
    for every shard shape the digits reconstruct the 65-bit k0 and the 64-bit k1 exactly with a
    zero final carry, every bucket index is inside the shape, the widths sum to 66 bits, and no
    window is narrower than c - 1 bits -- a 3-bit top window (round 3's first c = 9 shape) put
    every point of a key into 4 buckets and made the bucket phase 40x slower"""
    import ctypes
    L = hostlib.lib()
    L.zgt_msm_digits.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64] + [ctypes.c_void_p] * 4
    rng = random.Random(5)
    for npad in (2, 1024, 4096, 8192, 16384, 32768, 65536, 1 << 20):
        d, sh, wd, shape = (ctypes.c_int * 8)(), (ctypes.c_int * 8)(), (ctypes.c_int * 8)(), (ctypes.c_int * 4)()
        edge = [(1 << 65) - 1, (1 << 65) - 3, 1, (1 << 64) + 1, (1 << 64) - 1, 1 << 63]
        for k in edge + [rng.getrandbits(65) | 1 for _ in range(300)] + [rng.getrandbits(64) for _ in range(300)]:
            nw = L.zgt_msm_digits(k & ((1 << 64) - 1), k >> 64, npad, d, sh, wd, shape)
            c, w, nb = shape[0], shape[1], shape[2]
            assert nw == w
            assert sum(wd[:w]) == 66 and min(wd[:w]) >= c - 1 and max(wd[:w]) == c and nb == 1 << (c - 1)
            assert all(sh[q] == sum(wd[:q]) for q in range(w))
            assert sum(d[q] << sh[q] for q in range(w)) == k
            assert all(-(1 << (wd[q] - 1)) < d[q] <= 1 << (wd[q] - 1) for q in range(w))
            assert all(abs(d[q]) <= nb for q in range(w))


def _g1_points(rng, n):
    """random G1 points, random curve points outside G1, and the order-3 points (0, +-2)"""
    pts = [B.ec_mul(B.FQ, B.G1_GEN, rng.randrange(1, B.R)) for _ in range(n)]
    out = []
    while len(out) < n:
        x = rng.randrange(P)
        rhs = (x * x * x + 4) % P
        y = pow(rhs, (P + 1) // 4, P)
        if y * y % P == rhs:
            out.append((x, y))
    return [(p, True) for p in pts] + [(p, False) for p in out] + [((0, 2), False), ((0, P - 2), False)]


def test_g1_digit_arith_equals_word_form():
    """the decode kernels' lazy-digit G1 arithmetic (zg_fqd.h: g1_in_subgroup_d, g1_glv_mul_d and the
    two-column g1_glv_mul_w2)
    against the word form (zg_curve.h / zg_groth16.h) and the oracle: subgroup verdicts on G1
    points, curve points outside G1 and the order-3 points (0, +-2) (exceptional additions in the
    chain), and r A for random and extreme GLV scalars"""
    import ctypes
    L = hostlib.lib()
    L.zgt_g1_check_glv.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64,
                                   ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p]
    rng = random.Random(7)
    lam = None
    for (x, y), ing1 in _g1_points(rng, 6):
        for a, b in [(rng.getrandbits(64), rng.getrandbits(64)), (0, 0), ((1 << 64) - 1, (1 << 64) - 1),
                     ((1 << 64) - 1, 0), (0, (1 << 64) - 1)]:
            res = (ctypes.c_int * 3)()
            ow, od = ctypes.create_string_buffer(96), ctypes.create_string_buffer(96)
            L.zgt_g1_check_glv(fq_b(x), fq_b(y), a, b, res, ow, od)
            assert res[0] == res[1] == int(ing1)
            assert ow.raw == od.raw
            assert res[2] == 1 or not ing1   # the two-column GLV (decode's) agrees on G1 points
            if ing1 and a == 0 and b == 0:   # k = 1: r A = A
                assert ow.raw == fq_b(x) + fq_b(y)


def test_g1_digit_point_sums_equal_word_form():
    """K4's lazy-digit sums (zg_fqd.h g1d_add_full: merges, scans, trees; g1d_add_aff with the
    bucket phase's negated y < 3p) against the word form on random Jacobian scalings: generic sums,
    P + P (doubling), P + (-P) (infinity), infinity on either side, points outside G1"""
    import ctypes
    L = hostlib.lib()
    L.zgt_g1d_add.argtypes = [ctypes.c_char_p] * 6 + [ctypes.c_char_p] * 4
    rng = random.Random(11)
    pts = [p for p, _ in _g1_points(rng, 4)]
    z = lambda: fq_b(rng.randrange(1, P))
    zero = fq_b(0)
    cases = []
    for a in pts:
        for b in pts:
            cases.append((a, z(), b, z()))
        cases.append((a, z(), a, z()))                      # doubling
        cases.append((a, z(), (a[0], P - a[1]), z()))      # infinity
        cases.append((a, zero, a, z()))                     # inf + q
        cases.append((a, z(), a, zero))                     # p + inf
    for (x1, y1), z1, (x2, y2), z2 in cases:
        ow, od, mw, md = (ctypes.create_string_buffer(96) for _ in range(4))
        L.zgt_g1d_add(fq_b(x1), fq_b(y1), z1, fq_b(x2), fq_b(y2), z2, ow, od, mw, md)
        assert ow.raw == od.raw
        assert mw.raw == md.raw
