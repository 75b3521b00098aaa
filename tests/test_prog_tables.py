"""CPU tier: the generated staged programs (zebra_amd/csrc/gen_prog.py -> zg_prog_tables.h)
and cooperative tables (gen_coop.py) compute exactly the oracle's operations:
pairing's doubling/addition line steps with the ell scaling, mul_by_014, Fq12 square/mul,
cyclotomic square."""
import os
import random
import sys

from oracle import bls12_381 as B
from tests.conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "zebra_amd", "csrc"))
import gen_coop  # noqa: E402
import gen_prog  # noqa: E402

P = B.P


def gmul(c, x):
    return ((c[0] * x[0] - c[1] * x[1]) % P, (c[1] * x[0] + c[0] * x[1]) % P)


def run(prog, inputs):
    atoms = list(inputs)

    def ev(form):
        acc = (0, 0)
        for a, c0, c1 in form:
            acc = B.f2_add(acc, gmul((c0, c1), atoms[a]))
        return acc
    for lo, hi in prog["stages"]:
        vals = [B.f2_mul(ev(prog["prods"][k][0]), ev(prog["prods"][k][1])) for k in range(lo, hi)]
        atoms.extend(vals)
    return [ev(o) for o in prog["outs"]]


def rnd2(rng):
    return (rng.randrange(P), rng.randrange(P))


def test_prog_structure():
    for pr in gen_prog.build_all():
        assert len(pr["stages"]) <= 8
        # products of a stage only reference atoms of earlier stages
        for s, (lo, hi) in enumerate(pr["stages"]):
            limit = pr["nin"] + lo
            for k in range(lo, hi):
                for form in pr["prods"][k][:2]:
                    assert all(a < limit for a, _, _ in form)


def test_line_programs_match_pairing_steps():
    progs = {p["name"]: p for p in gen_prog.build_all()}
    rng = random.Random(11)
    q = B.ec_mul(B.FQ2, B.G2_GEN, 99991)
    px, py = rng.randrange(P), rng.randrange(P)
    r = (q[0], q[1], B.F2_ONE)
    for step in range(3):
        r = (B.f2_mul(r[0], rnd2(rng)), r[1], B.f2_mul(r[2], rnd2(rng)))  # arbitrary Jacobian-ish state
        nr_, c = B._doubling_step(r)
        out = run(progs["dbl"], [r[0], r[1], r[2], q[0], q[1], (px, 0), (py, 0)])
        assert out[:3] == list(nr_)
        assert out[3] == c[2] and out[4] == B.f2_scale(c[1], px) and out[5] == B.f2_scale(c[0], py)
        na, ca = B._addition_step(r, q)
        out = run(progs["add"], [r[0], r[1], r[2], q[0], q[1], (px, 0), (py, 0)])
        assert out[:3] == list(na)
        assert out[3] == ca[2] and out[4] == B.f2_scale(ca[1], px) and out[5] == B.f2_scale(ca[0], py)


def f12_pairs(f):
    return [c for h in f for c in h]


def test_fq12_programs():
    progs = {p["name"]: p for p in gen_prog.build_all()}
    rng = random.Random(12)
    for _ in range(3):
        f = B.f12_from_coeffs([rng.randrange(P) for _ in range(12)])
        g = B.f12_from_coeffs([rng.randrange(P) for _ in range(12)])
        A, Bc, C = rnd2(rng), rnd2(rng), rnd2(rng)
        line = ((A, Bc, B.F2_ZERO), (B.F2_ZERO, C, B.F2_ZERO))
        assert run(progs["m014"], f12_pairs(f) + [A, Bc, C]) == f12_pairs(B.f12_mul(f, line))
        assert run(progs["sqr"], f12_pairs(f)) == f12_pairs(B.f12_sqr(f))
        assert run(progs["mul"], f12_pairs(f) + f12_pairs(g)) == f12_pairs(B.f12_mul(f, g))


def test_coop_tables():
    ops = {o["name"]: o for o in [gen_coop.build("mul", gen_coop.f12_mul, True),
                                  gen_coop.build("csqr", gen_coop.f12_cyc_sqr, False)]}
    rng = random.Random(13)
    a = B.f12_from_coeffs([rng.randrange(P) for _ in range(12)])
    b = B.f12_from_coeffs([rng.randrange(P) for _ in range(12)])
    assert gen_coop.evaluate(ops["mul"], B.f12_coeffs(a), B.f12_coeffs(b)) == B.f12_coeffs(B.f12_mul(a, b))
    c = B.f12_mul(B.f12_conj(a), B.f12_inv(a))
    c = B.f12_mul(B.f12_frob(c, 2), c)
    assert gen_coop.evaluate(ops["csqr"], B.f12_coeffs(c), None) == B.f12_coeffs(B.f12_sqr(c))
