#!/usr/bin/env python3
"""Generate zg_prog_tables.h: Fq2-granularity staged programs for the multi-instance
cooperative engine (zg_prog.h).

A program is a straight-line formula over Fq2 values (pairing 0.14.2's line doubling /
addition steps with the `ell` scaling, the sparse line product mul_by_014, Fq12 squaring)
run symbolically: every Fq2 multiplication becomes a *product* whose operands are linear
forms, with Gaussian-integer coefficients (c0 + c1 u), over earlier atoms (program inputs or
earlier products). Products are scheduled ASAP into stages; within a stage they are
independent, so the engine runs them on separate lanes (several program instances -- proofs
-- packed per wave). Outputs are linear forms over atoms. Build tooling.

    python zebra_amd/csrc/gen_prog.py > zebra_amd/csrc/zg_prog_tables.h
"""
import sys


class G(dict):
    """linear form: atom -> Gaussian integer coefficient (c0, c1) meaning c0 + c1 u"""

    def __add__(self, o):
        r = G(self)
        for k, (a, b) in o.items():
            c0, c1 = r.get(k, (0, 0))
            c0, c1 = c0 + a, c1 + b
            if c0 == 0 and c1 == 0:
                r.pop(k, None)
            else:
                r[k] = (c0, c1)
        return r

    def __neg__(self):
        return G({k: (-a, -b) for k, (a, b) in self.items()})

    def __sub__(self, o):
        return self + (-o)

    def gmul(self, c):  # multiply by Gaussian integer c = (c0, c1)
        r = G()
        for k, (a, b) in self.items():
            v = (a * c[0] - b * c[1], a * c[1] + b * c[0])
            if v != (0, 0):
                r[k] = v
        return r

    def dbl(self):
        return self + self

    def nr(self):  # multiply by xi = 1 + u
        return self.gmul((1, 1))


class Prog:
    def __init__(self, name, inputs):
        self.name = name
        self.inputs = list(inputs)
        self.prods = []  # (L, R, stage)
        self.stage_of = {("in", i): 0 for i in range(len(inputs))}

    def inp(self, i):
        return G({("in", i): (1, 0)})

    def mul(self, x, y):
        st = 1 + max([self.stage_of[k] for k in list(x) + list(y)] or [0])
        k = ("p", len(self.prods))
        self.prods.append((x, y, st))
        self.stage_of[k] = st
        return G({k: (1, 0)})

    def sqr(self, x):
        return self.mul(x, x)

    def finish(self, outputs):
        # renumber products grouped by stage (stable), atoms: inputs 0.., products nin..
        order = sorted(range(len(self.prods)), key=lambda i: (self.prods[i][2], i))
        newidx = {("p", old): len(self.inputs) + new for new, old in enumerate(order)}
        aidx = {("in", i): i for i in range(len(self.inputs))}
        aidx.update(newidx)

        def conv(f):
            return [(aidx[k], c0, c1) for k, (c0, c1) in sorted(f.items(), key=lambda kv: aidx[kv[0]])]
        prods = [(conv(self.prods[o][0]), conv(self.prods[o][1]), self.prods[o][2]) for o in order]
        nst = max(p[2] for p in prods)
        bounds = []
        for s in range(1, nst + 1):
            idx = [i for i, p in enumerate(prods) if p[2] == s]
            bounds.append((idx[0], idx[-1] + 1))
        return {"name": self.name, "nin": len(self.inputs), "prods": prods, "stages": bounds,
                "outs": [conv(f) for f in outputs]}


# ---------------------------------------------------------------- programs
def prog_dbl():
    """pairing doubling_step + ell scaling. in: X Y Z QX QY PX PY (PX = (px, 0); Q unused, the
    layout is shared with `add`). out: X' Y' Z' A B C, the line f * (A + B v + C v w) with
    A = c2, B = c1 px, C = c0 py"""
    p = Prog("dbl", ["X", "Y", "Z", "QX", "QY", "PX", "PY"])
    X, Y, Z, PX, PY = p.inp(0), p.inp(1), p.inp(2), p.inp(5), p.inp(6)
    tmp0 = p.sqr(X)
    tmp1 = p.sqr(Y)
    tmp2 = p.sqr(tmp1)
    tmp3 = (p.sqr(tmp1 + X) - tmp0 - tmp2).dbl()
    tmp4 = tmp0.dbl() + tmp0
    tmp6 = X + tmp4
    tmp5 = p.sqr(tmp4)
    zsq = p.sqr(Z)
    nx = tmp5 - tmp3 - tmp3
    nz = p.sqr(Z + Y) - tmp1 - zsq
    ny = p.mul(tmp3 - nx, tmp4) - tmp2.dbl().dbl().dbl()
    tmp3b = -(p.mul(tmp4, zsq).dbl())
    tmp6 = p.sqr(tmp6) - tmp0 - tmp5 - tmp1.dbl().dbl()
    tmp0b = p.mul(nz, zsq).dbl()
    # coeffs (c0, c1, c2) = (tmp0b, tmp3b, tmp6)
    A = tmp6
    B = p.mul(tmp3b, PX)
    C = p.mul(tmp0b, PY)
    return p.finish([nx, ny, nz, A, B, C])


def prog_add():
    """pairing addition_step + ell scaling. in: X Y Z QX QY PX PY."""
    p = Prog("add", ["X", "Y", "Z", "QX", "QY", "PX", "PY"])
    X, Y, Z, QX, QY, PX, PY = (p.inp(i) for i in range(7))
    zsq = p.sqr(Z)
    ysq = p.sqr(QY)
    t0 = p.mul(zsq, QX)
    t1 = p.mul(p.sqr(QY + Z) - ysq - zsq, zsq)
    t2 = t0 - X
    t3 = p.sqr(t2)
    t4 = t3.dbl().dbl()
    t5 = p.mul(t4, t2)
    t6 = t1 - Y - Y
    t9 = p.mul(t6, QX)
    t7 = p.mul(t4, X)
    nx = p.sqr(t6) - t5 - t7 - t7
    nz = p.sqr(Z + t2) - zsq - t3
    t10 = QY + nz
    t8 = p.mul(t7 - nx, t6)
    t0b = p.mul(Y, t5).dbl()
    ny = t8 - t0b
    t10 = p.sqr(t10) - ysq - p.sqr(nz)
    t9 = t9.dbl() - t10
    t10b = nz.dbl()
    t1b = (-t6).dbl()
    # coeffs (c0, c1, c2) = (t10b, t1b, t9)
    A = t9
    B = p.mul(t1b, PX)
    C = p.mul(t10b, PY)
    return p.finish([nx, ny, nz, A, B, C])


def f6_mul_by_01(p, a, b0, b1):
    t0 = p.mul(a[0], b0)
    t1 = p.mul(a[1], b1)
    c0 = p.mul(a[1] + a[2], b1).nr() + t0 - t1.nr()
    c1 = p.mul(a[0] + a[1], b0 + b1) - t0 - t1
    c2 = p.mul(a[0] + a[2], b0) - t0 + t1
    return (c0, c1, c2)


def f6_mul_by_1(p, a, b1):
    return (p.mul(a[2], b1).nr(), p.mul(a[0], b1), p.mul(a[1], b1))


def prog_m014():
    """f * (A + B v + C v w). in: f0..f5 (c0.c0 c0.c1 c0.c2 c1.c0 c1.c1 c1.c2), A, B, C."""
    p = Prog("m014", ["F0", "F1", "F2", "F3", "F4", "F5", "A", "B", "C"])
    f = [p.inp(i) for i in range(6)]
    A, B, C = p.inp(6), p.inp(7), p.inp(8)
    F0, F1 = f[0:3], f[3:6]
    aa = f6_mul_by_01(p, F0, A, B)
    bb = f6_mul_by_1(p, F1, C)
    s = f6_mul_by_01(p, [x + y for x, y in zip(F0, F1)], A, B + C)
    c0 = [aa[0] + bb[2].nr(), aa[1] + bb[0], aa[2] + bb[1]]
    c1 = [s[i] - aa[i] - bb[i] for i in range(3)]
    return p.finish(c0 + c1)


def f6_mul(p, a, b):
    t0, t1, t2 = p.mul(a[0], b[0]), p.mul(a[1], b[1]), p.mul(a[2], b[2])
    c0 = (p.mul(a[1] + a[2], b[1] + b[2]) - t1 - t2).nr() + t0
    c1 = p.mul(a[0] + a[1], b[0] + b[1]) - t0 - t1 + t2.nr()
    c2 = p.mul(a[0] + a[2], b[0] + b[2]) - t0 - t2 + t1
    return [c0, c1, c2]


def f6_nr(a):
    return [a[2].nr(), a[0], a[1]]


def prog_sqr():
    """complex squaring of an Fq12: 2 Fq6 products = 12 Fq2 products."""
    p = Prog("sqr", ["F0", "F1", "F2", "F3", "F4", "F5"])
    f = [p.inp(i) for i in range(6)]
    a0, a1 = f[0:3], f[3:6]
    ab = f6_mul(p, a0, a1)
    t = f6_mul(p, [x + y for x, y in zip(a0, a1)], [x + y for x, y in zip(a0, f6_nr(a1))])
    c0 = [t[i] - ab[i] - f6_nr(ab)[i] for i in range(3)]
    c1 = [ab[i].dbl() for i in range(3)]
    return p.finish(c0 + c1)


def prog_mul():
    p = Prog("mul", ["A0", "A1", "A2", "A3", "A4", "A5", "B0", "B1", "B2", "B3", "B4", "B5"])
    a = [p.inp(i) for i in range(6)]
    b = [p.inp(6 + i) for i in range(6)]
    t0 = f6_mul(p, a[0:3], b[0:3])
    t1 = f6_mul(p, a[3:6], b[3:6])
    t2 = f6_mul(p, [x + y for x, y in zip(a[0:3], a[3:6])], [x + y for x, y in zip(b[0:3], b[3:6])])
    c0 = [t0[i] + f6_nr(t1)[i] for i in range(3)]
    c1 = [t2[i] - t0[i] - t1[i] for i in range(3)]
    return p.finish(c0 + c1)


PROGS = [prog_dbl, prog_add, prog_m014, prog_sqr, prog_mul]


def emit(progs):
    out = ["// GENERATED by zebra_amd/csrc/gen_prog.py -- do not edit.", "#pragma once", "#include <stdint.h>",
           "namespace zg {", "struct PTerm { uint8_t atom; int8_t c0, c1; };  // coefficient c0 + c1 u"]
    terms = []     # flat term pool
    forms = []     # (offset, count)

    def add_form(f):
        off = len(terms)
        terms.extend(f)
        forms.append((off, len(f)))
        return len(forms) - 1
    specs = []
    for pr in progs:
        pl = [add_form(l) for l, _, _ in pr["prods"]]
        prr = [add_form(r) for _, r, _ in pr["prods"]]
        po = [add_form(o) for o in pr["outs"]]
        specs.append((pr, pl, prr, po))
    out.append("__device__ __constant__ const PTerm PROG_TERMS[%d] = {%s};" % (
        len(terms), ", ".join("{%d, %d, %d}" % t for t in terms)))
    out.append("__device__ __constant__ const uint16_t PROG_FORMS[%d][2] = {%s};" % (
        len(forms), ", ".join("{%d, %d}" % f for f in forms)))
    out.append("struct ProgDesc { uint8_t nin, nprod, nstage, nout; uint8_t stage[8][2]; uint16_t L, R, O; };")
    out.append("// L/R: first form index of product operands; O: first form index of outputs")
    descs = []
    for pr, pl, prr, po in specs:
        st = pr["stages"] + [(0, 0)] * (8 - len(pr["stages"]))
        assert len(pr["stages"]) <= 8
        descs.append("{%d, %d, %d, %d, {%s}, %d, %d, %d}" % (
            pr["nin"], len(pr["prods"]), len(pr["stages"]), len(pr["outs"]),
            ", ".join("{%d, %d}" % s for s in st), pl[0], prr[0], po[0]))
        out.append("#define ZG_PROG_%s %d   // %d products in %d stages, atoms %d" % (
            pr["name"].upper(), len(descs) - 1, len(pr["prods"]), len(pr["stages"]),
            pr["nin"] + len(pr["prods"])))
    out.append("__device__ __constant__ const ProgDesc PROG_DESC[%d] = {%s};" % (len(descs), ", ".join(descs)))
    maxatoms = max(pr["nin"] + len(pr["prods"]) for pr in progs)
    out.append("#define ZG_PROG_MAXATOMS %d" % maxatoms)
    out.append("}  // namespace zg")
    return out


def build_all():
    return [f() for f in PROGS]


if __name__ == "__main__":
    progs = build_all()
    for pr in progs:
        sys.stderr.write("%s: %d products, stages %s, max |coef| %d\n" % (
            pr["name"], len(pr["prods"]), [b - a for a, b in pr["stages"]],
            max(max(abs(c0), abs(c1)) for f in [x for p_ in pr["prods"] for x in p_[:2]] + pr["outs"]
                for _, c0, c1 in f)))
    sys.stdout.write("\n".join(emit(progs)) + "\n")
