"""CPU tier: the generated staged programs (zebra_amd/csrc/gen_prog.py -> zg_prog_tables.h),
run on the generator's LDS-slot model with its round schedule, and the cooperative tables
(gen_coop.py) compute exactly the oracle's operations: pairing's doubling/addition line steps
with the ell scaling, the f-chain step (mul_by_014 then square), Fq12 mul/square, cyclotomic
square."""
import os
import random
import sys

from oracle import bls12_381 as B
from tests.conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "zebra_amd", "csrc"))
import gen_coop  # noqa: E402
import gen_prog  # noqa: E402

P = B.P


def rnd2(rng):
    return (rng.randrange(P), rng.randrange(P))


def progs():
    return {name: (prog, outs, sch) for name, prog, outs, nw, sch in gen_prog.build_all()}


def run(name, inputs):
    """the scheduled program on the LDS slot model (reads of a round before its writes)"""
    prog, outs, sch = progs()[name]
    got = gen_prog.simulate(prog, outs, sch, inputs)
    assert got == gen_prog.reference(prog, outs, inputs)
    return got


def test_prog_schedule_structure():
    for name, prog, outs, nw, sch in gen_prog.build_all():
        assert all(len(r) <= nw for r in sch["rounds"])
        # LDS: one f-chain block per CU; two R-chain blocks per CU (13 slots x 6 KB each)
        assert sch["nslots"] * 6 * 1024 <= 160 * 1024, name
        if name in ("dbl", "add"):
            assert sch["nslots"] <= 13 and nw == 4 and sch["rb"] == 1, name
            # B and C (outputs 4, 5) leave through their products' waves: no slot
            assert sorted(sch["sinks"].values()) == [4, 5], name
        elif name in ("q4sq", "q4", "gm", "gmsq", "q4i", "q4ik", "aq4"):
            # four proofs per lane: 18 inputs fit 25 slots only with the same-round reuse (and the
            # group chain's general products run in the same LDS budget, k_batch_fchaing; aq4: the
            # affine line products of k_line_prod, round 6)
            assert sch["nslots"] <= 25 and sch["rb"] == 1, name
        else:
            # no read barrier: a slot is never written in the round that reads its previous content
            assert sch["rb"] == 0, name


def test_line_programs_match_pairing_steps():
    rng = random.Random(11)
    q = B.ec_mul(B.FQ2, B.G2_GEN, 99991)
    px, py = rng.randrange(P), rng.randrange(P)
    r = (q[0], q[1], B.F2_ONE)
    for step in range(3):
        r = (B.f2_mul(r[0], rnd2(rng)), r[1], B.f2_mul(r[2], rnd2(rng)))  # arbitrary Jacobian-ish state
        nr_, c = B._doubling_step(r)
        out = run("dbl", [r[0], r[1], r[2], (px, py)])
        assert out[:3] == list(nr_)
        assert out[3] == c[2] and out[4] == B.f2_scale(c[1], px) and out[5] == B.f2_scale(c[0], py)
        na, ca = B._addition_step(r, q)
        out = run("add", [r[0], r[1], r[2], (px, py), q[0], q[1]])
        assert out[:3] == list(na)
        assert out[3] == ca[2] and out[4] == B.f2_scale(ca[1], px) and out[5] == B.f2_scale(ca[0], py)


def f12_pairs(f):
    return [c for h in f for c in h]


def test_fchain_programs():
    rng = random.Random(12)
    for _ in range(3):
        f = B.f12_from_coeffs([rng.randrange(P) for _ in range(12)])
        A, Bc, C = rnd2(rng), rnd2(rng), rnd2(rng)
        line = ((A, Bc, B.F2_ZERO), (B.F2_ZERO, C, B.F2_ZERO))
        fl = B.f12_mul(f, line)
        assert run("m", f12_pairs(f) + [A, Bc, C]) == f12_pairs(fl)
        assert run("msq", f12_pairs(f) + [A, Bc, C]) == f12_pairs(B.f12_sqr(fl))
        # four proofs per lane: f * l0 * l1 * l2 * l3 (then squared)
        ls = [(rnd2(rng), rnd2(rng), rnd2(rng)) for _ in range(4)]
        f4 = f
        for (a_, b_, c_) in ls:
            f4 = B.f12_mul(f4, ((a_, b_, B.F2_ZERO), (B.F2_ZERO, c_, B.F2_ZERO)))
        flat = [x for l in ls for x in l]
        assert run("q4", f12_pairs(f) + flat) == f12_pairs(f4)
        # a group's first four lines from scratch (k_line_prod): (l0 l1)(l2 l3), f unused
        assert run("q4i", f12_pairs(f) + flat) == f12_pairs(B.f12_mul(B.f12_mul(B.f12_mul(
            ((ls[0][0], ls[0][1], B.F2_ZERO), (B.F2_ZERO, ls[0][2], B.F2_ZERO)),
            ((ls[1][0], ls[1][1], B.F2_ZERO), (B.F2_ZERO, ls[1][2], B.F2_ZERO))),
            ((ls[2][0], ls[2][1], B.F2_ZERO), (B.F2_ZERO, ls[2][2], B.F2_ZERO))),
            ((ls[3][0], ls[3][1], B.F2_ZERO), (B.F2_ZERO, ls[3][2], B.F2_ZERO))))
        assert run("q4sq", f12_pairs(f) + flat) == f12_pairs(B.f12_sqr(f4))
        # the same four-line product with f kept in its slots (the split quad step, round 6): the
        # kernel then multiplies it into f with GM / GMSQ, which gives Q4 / Q4SQ's values
        prog, outs, sch = progs()["q4ik"]
        assert all(sch["slot"][("in", i)] == i for i in range(6)) and set(prog.keep) == set(range(6))
        quad = run("q4ik", f12_pairs(f) + flat)
        assert quad == run("q4i", f12_pairs(f) + flat)
        assert run("gm", f12_pairs(f) + quad) == f12_pairs(f4)
        assert run("gmsq", f12_pairs(f) + quad) == f12_pairs(B.f12_sqr(f4))
        # the group chain (k_batch_fchaing): f * L and (f * L)^2 for a general Fq12 L (the product
        # of a group's lines at one step, k_line_prod)
        g = B.f12_from_coeffs([rng.randrange(P) for _ in range(12)])
        assert run("gm", f12_pairs(f) + f12_pairs(g)) == f12_pairs(B.f12_mul(f, g))
        assert run("gmsq", f12_pairs(f) + f12_pairs(g)) == f12_pairs(B.f12_sqr(B.f12_mul(f, g)))



def test_coop_tables():
    ops = {o["name"]: o for o in [gen_coop.build("mul", gen_coop.f12_mul), gen_coop.build("sqr", gen_coop.f12_sqr),
                                  gen_coop.build("csqr", gen_coop.f12_cyc_sqr),
                                  gen_coop.build("m014", gen_coop.f12_mul_014)]}
    rng = random.Random(13)
    a = B.f12_from_coeffs([rng.randrange(P) for _ in range(12)])
    b = B.f12_from_coeffs([rng.randrange(P) for _ in range(12)])
    assert gen_coop.evaluate(ops["mul"], B.f12_coeffs(a), B.f12_coeffs(b)) == B.f12_coeffs(B.f12_mul(a, b))
    assert gen_coop.evaluate(ops["sqr"], B.f12_coeffs(a), None) == B.f12_coeffs(B.f12_sqr(a))
    cb = B.f12_coeffs(b)
    sparse = [cb[0], cb[1], cb[2], cb[3], 0, 0, 0, 0, cb[8], cb[9], 0, 0]
    assert gen_coop.evaluate(ops["m014"], B.f12_coeffs(a), cb) == B.f12_coeffs(
        B.f12_mul(a, B.f12_from_coeffs(sparse)))
    c = B.f12_mul(B.f12_conj(a), B.f12_inv(a))
    c = B.f12_mul(B.f12_frob(c, 2), c)
    assert gen_coop.evaluate(ops["csqr"], B.f12_coeffs(c), None) == B.f12_coeffs(B.f12_sqr(c))


def test_lazy_operand_forms():
    """the emitted lazy operand forms (plain 12-word sums with K p offsets, never reduced) and
    the products' ZG_KIND codes, interpreted on extreme (0, p - 1) and random atoms: every carry
    chain stays within [0, 2^384), operands equal the forms mod p, outputs are canonical, and the
    raw product bounds fit the conditional subtractions / quotient estimate the code selects"""
    if not gen_prog.LAZY:
        return
    gen_prog.check_lazy(gen_prog.build_all(), trials=12)
