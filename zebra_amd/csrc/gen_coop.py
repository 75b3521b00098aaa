#!/usr/bin/env python3
"""Generate zg_coop_tables.h: Fq12 operations decomposed into levels of independent lane
tasks for the lane-cooperative engine (zg_coop.h). Build tooling; self-checking.

An operation reads two Fq12 inputs a, b (24 Fq values, indices 0..23) and computes atoms
(indices 24..) in levels:
  level 0   products   P_k = L_k * R_k, L_k / R_k small-integer linear forms of the inputs;
  level l   sums       S   = small-integer linear form of inputs and atoms of lower levels;
  last      outputs    the 12 Fq coefficients of the result (a linear form like a sum).
Every task of a level runs on its own lane; levels are separated by a barrier. The tower
formulas (Karatsuba Fq2/Fq6/Fq12 multiplication, complex squaring, Granger-Scott cyclotomic
squaring, pairing's mul_by_014) are run on symbolic forms; each Fq2 / Fq6 product result is
materialised as its own level of atoms so that no form has more than a handful of terms
(the engine evaluates a term in ~60 VALU instructions, branch-free).

    python zebra_amd/csrc/gen_coop.py > zebra_amd/csrc/zg_coop_tables.h
"""
import random
import sys

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
NIN = 24


class Lin(dict):
    def __add__(self, o):
        r = Lin(self)
        for k, v in o.items():
            r[k] = r.get(k, 0) + v
            if r[k] == 0:
                del r[k]
        return r

    def __neg__(self):
        return Lin({k: -v for k, v in self.items()})

    def __sub__(self, o):
        return self + (-o)


class Op:
    def __init__(self, name, flat=False):
        self.name = name
        self.flat = flat  # flat: no intermediate sums, outputs are forms of products and inputs
        self.atoms = []  # (kind, level, forms): kind 'p' (L, R) or 's' (form,)

    def level_of(self, f):
        lv = -1
        for k in f:
            if k >= NIN:
                lv = max(lv, self.atoms[k - NIN][1])
        return lv

    def mul(self, x, y):
        assert self.level_of(x) < 0 and self.level_of(y) < 0, "products read inputs only"
        self.atoms.append(("p", 0, (x, y)))
        return Lin({NIN + len(self.atoms) - 1: 1})

    def mat(self, f):
        """materialise a form as a sum atom (one lane task)"""
        if self.flat or len(f) == 1 and list(f.values())[0] == 1:
            return f
        self.atoms.append(("s", 1 + max(0, self.level_of(f)), (f,)))
        return Lin({NIN + len(self.atoms) - 1: 1})


# ---------------------------------------------------------------- tower on tuples of Lin
def f2_add(a, b):
    return (a[0] + b[0], a[1] + b[1])


def f2_sub(a, b):
    return (a[0] - b[0], a[1] - b[1])


def f2_nr(a):
    return (a[0] - a[1], a[0] + a[1])


def f2_mat(op, a):
    return (op.mat(a[0]), op.mat(a[1]))


def f2_mul(op, a, b):
    t0 = op.mul(a[0], b[0])
    t1 = op.mul(a[1], b[1])
    t2 = op.mul(a[0] + a[1], b[0] + b[1])
    return f2_mat(op, (t0 - t1, t2 - t0 - t1))


def f2_sqr(op, a):
    t = op.mul(a[0], a[1])
    return f2_mat(op, (op.mul(a[0] + a[1], a[0] - a[1]), t + t))


def f6_add(a, b):
    return tuple(f2_add(x, y) for x, y in zip(a, b))


def f6_sub(a, b):
    return tuple(f2_sub(x, y) for x, y in zip(a, b))


def f6_nr(a):
    return (f2_nr(a[2]), a[0], a[1])


def f6_mat(op, a):
    return tuple(f2_mat(op, x) for x in a)


def f6_mul(op, a, b):
    t0, t1, t2 = f2_mul(op, a[0], b[0]), f2_mul(op, a[1], b[1]), f2_mul(op, a[2], b[2])
    c0 = f2_add(f2_nr(f2_sub(f2_sub(f2_mul(op, f2_add(a[1], a[2]), f2_add(b[1], b[2])), t1), t2)), t0)
    c1 = f2_add(f2_sub(f2_sub(f2_mul(op, f2_add(a[0], a[1]), f2_add(b[0], b[1])), t0), t1), f2_nr(t2))
    c2 = f2_add(f2_sub(f2_sub(f2_mul(op, f2_add(a[0], a[2]), f2_add(b[0], b[2])), t0), t2), t1)
    return f6_mat(op, (c0, c1, c2))


def f12_mul(op, a, b):
    t0, t1 = f6_mul(op, a[0], b[0]), f6_mul(op, a[1], b[1])
    c1 = f6_sub(f6_sub(f6_mul(op, f6_add(a[0], a[1]), f6_add(b[0], b[1])), t0), t1)
    return (f6_add(t0, f6_nr(t1)), c1)


def f12_sqr(op, a, _b):
    """complex squaring (pairing Fq12::square): 2 Fq6 products"""
    a0, a1 = a
    ab = f6_mul(op, a0, a1)
    t = f6_mul(op, f6_add(a0, a1), f6_add(a0, f6_nr(a1)))
    c0 = f6_sub(f6_sub(t, ab), f6_nr(ab))
    return (c0, f6_add(ab, ab))


def fp4_square(op, a, b):
    t0 = f2_sqr(op, a)
    t1 = f2_sqr(op, b)
    c0 = f2_add(f2_nr(t1), t0)
    t2 = f2_sqr(op, f2_add(a, b))
    return c0, f2_sub(f2_sub(t2, t0), t1)


def f12_cyc_sqr(op, f, _b):
    """Granger-Scott squaring, valid in the cyclotomic subgroup."""
    z0, z4, z3 = f[0]
    z2, z1, z5 = f[1]
    t0, t1 = fp4_square(op, z0, z1)
    z0 = f2_add(f2_add(f2_sub(t0, z0), f2_sub(t0, z0)), t0)
    z1 = f2_add(f2_add(f2_add(t1, z1), f2_add(t1, z1)), t1)
    t0, t1 = fp4_square(op, z2, z3)
    t2, t3 = fp4_square(op, z4, z5)
    z4 = f2_add(f2_add(f2_sub(t0, z4), f2_sub(t0, z4)), t0)
    z5 = f2_add(f2_add(f2_add(t1, z5), f2_add(t1, z5)), t1)
    t0 = f2_nr(t3)
    z2 = f2_add(f2_add(f2_add(t0, z2), f2_add(t0, z2)), t0)
    z3 = f2_add(f2_add(f2_sub(t2, z3), f2_sub(t2, z3)), t2)
    return ((z0, z4, z3), (z2, z1, z5))


def f6_mul_by_01(op, a, b0, b1):
    t0 = f2_mul(op, a[0], b0)
    t1 = f2_mul(op, a[1], b1)
    c0 = f2_add(f2_sub(f2_nr(f2_mul(op, f2_add(a[1], a[2]), b1)), f2_nr(t1)), t0)
    c1 = f2_sub(f2_sub(f2_mul(op, f2_add(a[0], a[1]), f2_add(b0, b1)), t0), t1)
    c2 = f2_add(f2_sub(f2_mul(op, f2_add(a[0], a[2]), b0), t0), t1)
    return f6_mat(op, (c0, c1, c2))


def f6_mul_by_1(op, a, b1):
    return (f2_nr(f2_mul(op, a[2], b1)), f2_mul(op, a[0], b1), f2_mul(op, a[1], b1))


def f12_mul_014(op, a, b):
    """pairing Fq12::mul_by_014: a * (c0 + c1 v + c4 v w); the sparse operand is b with
    c0 = b.c0.c0, c1 = b.c0.c1, c4 = b.c1.c1 (the other coefficients of b are ignored)"""
    c0, c1, c4 = b[0][0], b[0][1], b[1][1]
    aa = f6_mul_by_01(op, a[0], c0, c1)
    bb = f6_mul_by_1(op, a[1], c4)
    o = f2_add(c1, c4)
    s = f6_mul_by_01(op, f6_add(a[1], a[0]), c0, o)
    r1 = f6_sub(f6_sub(s, aa), bb)
    r0 = f6_add(f6_nr(bb), aa)
    return (r0, r1)


def sym(base):
    c = [Lin({base + i: 1}) for i in range(12)]
    return (((c[0], c[1]), (c[2], c[3]), (c[4], c[5])), ((c[6], c[7]), (c[8], c[9]), (c[10], c[11])))


def flat(x):
    return [v for h in x for c in h for v in c]


def build(name, fn, flat_forms=False):
    op = Op(name, flat_forms)
    out = flat(fn(op, sym(0), sym(12)))
    # levels: products 0, sums by dependency, outputs last
    nlev = 1 + max([a[1] for a in op.atoms] + [0])
    levels = [[] for _ in range(nlev)]
    for i, a in enumerate(op.atoms):
        levels[a[1]].append(i)
    # renumber atoms level-major
    order = [i for lv in levels for i in lv]
    new = {NIN + old: NIN + k for k, old in enumerate(order)}

    def ren(f):
        return {(new[k] if k >= NIN else k): c for k, c in f.items()}
    lev_forms = []
    for lv in levels:
        forms = []
        for i in lv:
            kind, _, fs = op.atoms[i]
            forms.append([ren(f) for f in fs])
        lev_forms.append(forms)
    outs = [ren(f) for f in out]
    return {"name": name, "levels": lev_forms, "outs": outs, "natoms": len(order)}


def evaluate(op, a, b):
    env = {i: a[i] for i in range(12)}
    env.update({12 + i: (b[i] if b else 0) for i in range(12)})
    k = NIN
    for li, forms in enumerate(op["levels"]):
        for fs in forms:
            vals = [sum(c * env[x] for x, c in f.items()) % P for f in fs]
            env[k] = vals[0] * vals[1] % P if li == 0 else vals[0]
            k += 1
    return [sum(c * env[x] for x, c in f.items()) % P for f in op["outs"]]


# reference tower (plain ints) for the self-check
def rf2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def rf2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def rf2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def rf2_nr(a):
    return ((a[0] - a[1]) % P, (a[0] + a[1]) % P)


def rf6_mul(a, b):
    r = [(0, 0)] * 5
    for i in range(3):
        for j in range(3):
            r[i + j] = rf2_add(r[i + j], rf2_mul(a[i], b[j]))
    return (rf2_add(r[0], rf2_nr(r[3])), rf2_add(r[1], rf2_nr(r[4])), r[2])


def rf12_mul(a, b):
    t0, t1 = rf6_mul(a[0], b[0]), rf6_mul(a[1], b[1])
    s = rf6_mul(tuple(rf2_add(x, y) for x, y in zip(a[0], a[1])), tuple(rf2_add(x, y) for x, y in zip(b[0], b[1])))
    v_t1 = (rf2_nr(t1[2]), t1[0], t1[1])
    return (tuple(rf2_add(x, y) for x, y in zip(t0, v_t1)),
            tuple(rf2_sub(rf2_sub(x, y), z) for x, y, z in zip(s, t0, t1)))


def unflat(v):
    c = [(v[2 * i], v[2 * i + 1]) for i in range(6)]
    return ((c[0], c[1], c[2]), (c[3], c[4], c[5]))


def check(ops):
    rng = random.Random(7)
    for op in ops:
        for _ in range(3):
            a = [rng.randrange(P) for _ in range(12)]
            b = [rng.randrange(P) for _ in range(12)]
            got = evaluate(op, a, b)
            if op["name"] == "mul":
                want = flat(rf12_mul(unflat(a), unflat(b)))
            elif op["name"] == "sqr":
                want = flat(rf12_mul(unflat(a), unflat(a)))
            elif op["name"] == "m014":
                bs = [b[0], b[1], b[2], b[3], 0, 0, 0, 0, b[8], b[9], 0, 0]
                want = flat(rf12_mul(unflat(a), unflat(bs)))
            elif op["name"] == "csqr1":
                want = evaluate([o for o in ops if o["name"] == "csqr"][0], a, b)  # same map, one level
            else:
                continue  # csqr: valid only on cyclotomic elements (checked on the device path)
            assert got == want, op["name"]


def emit(ops):
    lines = ["// GENERATED by zebra_amd/csrc/gen_coop.py -- do not edit.", "#pragma once", "#include <stdint.h>",
             "namespace zg {"]
    maxt = 0
    forms = []

    def add(f):
        nonlocal maxt
        t = sorted(f.items())
        assert all(-128 < c < 128 for _, c in t) and sum(abs(c) for _, c in t) < 256
        maxt = max(maxt, len(t))
        forms.append(t)
        return len(forms) - 1
    descs = []
    maxlev = max(len(o["levels"]) + 1 for o in ops)
    maxatoms = max(o["natoms"] for o in ops)
    for o in ops:
        cnt, off = [], []
        for li, lv in enumerate(o["levels"]):
            off.append(len(forms))
            cnt.append(len(lv))
            for fs in lv:
                for f in fs:
                    add(f)
        off.append(len(forms))
        cnt.append(12)
        for f in o["outs"]:
            add(f)
        assert max(cnt) <= 64
        descs.append((o["name"], len(cnt), cnt, off))
    lines.append("#define ZG_COOP_NFORMS %d" % len(forms))
    lines.append("#define ZG_COOP_MAXT %d    // terms per form" % maxt)
    lines.append("#define ZG_COOP_MAXLEV %d  // levels per op (products, sums..., outputs)" % maxlev)
    lines.append("#define ZG_COOP_MAXATOMS %d" % maxatoms)
    lines.append("// term = (coefficient << 8) | index ; index: a_i = i, b_i = 12 + i, atom k = 24 + k")
    lines.append("struct CoopForm { int16_t n; int16_t t[ZG_COOP_MAXT]; };")
    lines.append("struct CoopOp { int nlev; int cnt[ZG_COOP_MAXLEV]; int off[ZG_COOP_MAXLEV]; };")
    body = []
    for t in forms:
        ts = ["(int16_t)(%d * 256 + %d)" % (c, k) for k, c in t] + ["0"] * (maxt - len(t))
        body.append("{%d, {%s}}" % (len(t), ", ".join(ts)))
    lines.append("__device__ __constant__ const CoopForm COOP_FORMS[%d] = {%s};" % (len(forms), ", ".join(body)))
    for i, (name, n, cnt, off) in enumerate(descs):
        lines.append("#define ZG_COOP_%s %d  // levels %s" % (name.upper(), i, cnt))
    lines.append("__device__ __constant__ const CoopOp COOP_OPS[%d] = {%s};" % (len(descs), ", ".join(
        "{%d, {%s}, {%s}}" % (n, ", ".join(map(str, cnt + [0] * (maxlev - n))),
                             ", ".join(map(str, off + [0] * (maxlev - n)))) for _, n, cnt, off in descs)))
    lines.append("}  // namespace zg")
    return lines


def check_csqr1_products(op):
    """coop_csqr1 computes the product operands in code, not from these forms: product
    k = 6 p + 2 w + h squares x = z_a (w 0), z_b (w 1) or z_a + z_b (w 2) of the Fp4 pair p,
    with operands (x0, x1) for h = 0 and (x0 + x1, x0 - x1) for h = 1; the pairs' Fq2
    coefficient indices are (0, 4), (3, 2), (1, 5)."""
    pairs = [(0, 4), (3, 2), (1, 5)]
    (prods,) = op["levels"]
    assert len(prods) == 18
    for k, (L, R) in enumerate(prods):
        p, w, h = k // 6, (k % 6) // 2, k % 2
        ja, jb = pairs[p]
        sel = [ja] if w == 0 else [jb] if w == 1 else [ja, jb]
        x0 = Lin({2 * j: 1 for j in sel})
        x1 = Lin({2 * j + 1: 1 for j in sel})
        want = (x0, x1) if h == 0 else (x0 + x1, x0 - x1)
        assert (dict(L), dict(R)) == (dict(want[0]), dict(want[1])), k


def main():
    ops = [build("mul", f12_mul), build("sqr", f12_sqr), build("csqr", f12_cyc_sqr), build("m014", f12_mul_014),
           build("csqr1", f12_cyc_sqr, flat_forms=True)]
    check(ops)
    check_csqr1_products(ops[-1])
    sys.stdout.write("\n".join(emit(ops)) + "\n")
    for o in ops:
        sys.stderr.write("%s: levels %s, max terms %d\n" % (
            o["name"], [len(lv) for lv in o["levels"]] + [12],
            max(len(f) for lv in o["levels"] for fs in lv for f in fs)))


if __name__ == "__main__":
    main()
