#!/usr/bin/env python3
"""Generate zg_prog_tables.h: the staged programs of the per-proof Miller loop (zg_prog.h),
as round schedules, LDS slot maps and generated straight-line operand/output code.

A program is a straight-line formula over Fq2 values -- pairing 0.14.2's line doubling /
addition steps with the `ell` scaling by (px, py), and the f-chain step "sparse line
product then squaring" -- run symbolically: every Fq2 multiplication becomes a *product*
whose operands are linear forms (Gaussian-integer coefficients c0 + c1 u) over earlier atoms
(program inputs or products). The engine runs one program for 64 proofs at once (lane =
proof) on NW waves (wave = product): the generator list-schedules the products into rounds
of at most NW independent products, allocates LDS slots with reuse (a slot is rewritten
only in a round after its last read), and emits each product's operand evaluation and each
output's form as generated C++ (a switch on a global product / output id, so the kernel has
exactly one inlined Fq2-product site). Build tooling; self-checking.

    python zebra_amd/csrc/gen_prog.py > zebra_amd/csrc/zg_prog_tables.h
"""
import json
import os
import random
import sys

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB

# product kinds (zg_prog.h f2_mul_kind)
K_MUL, K_SQR, K_MULC0, K_MULC1 = 0, 1, 2, 3


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

    def gmul(self, c):
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
    def __init__(self, name, inputs, keep=(), glob=None):
        self.name = name
        self.inputs = list(inputs)
        self.keep = set(keep)  # inputs whose slots must survive the program
        self.glob = dict(glob or {})  # input -> index of a per-lane global-memory operand (no LDS slot)
        self.prods = []        # (L, R, kind)
        self.sink_from = None  # outputs >= this index may be stored by their product's wave

    def inp(self, i):
        return G({("in", i): (1, 0)})

    def _p(self, x, y, kind):
        self.prods.append((x, y, kind))
        return G({("p", len(self.prods) - 1): (1, 0)})

    def mul(self, x, y):
        return self._p(x, y, K_MUL)

    def sqr(self, x):
        return self._p(x, x, K_SQR)

    def mul_c0(self, x, y):  # x * y.c0 (y an input atom holding an Fq in c0)
        return self._p(x, y, K_MULC0)

    def mul_c1(self, x, y):  # x * y.c1
        return self._p(x, y, K_MULC1)


# ---------------------------------------------------------------- programs
def prog_dbl():
    """pairing doubling_step + ell scaling. in: X Y Z PQ (PQ = (px, py)). out: X' Y' Z' and
    the scaled line A + B v + C v w with A = c2, B = c1 px, C = c0 py"""
    p = Prog("dbl", ["X", "Y", "Z", "PQ"], keep=[3])
    p.sink_from = 3
    X, Y, Z, PQ = (p.inp(i) for i in range(4))
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
    B = p.mul_c0(tmp3b, PQ)
    C = p.mul_c1(tmp0b, PQ)
    return p, [nx, ny, nz, A, B, C]


def prog_add():
    """pairing addition_step + ell scaling. in: X Y Z PQ QX QY."""
    # QX, QY (the proof's B) are read from HBM where an operand needs them: two LDS slots fewer
    p = Prog("add", ["X", "Y", "Z", "PQ", "QX", "QY"], keep=[3], glob={4: 0, 5: 1})
    p.sink_from = 3
    X, Y, Z, PQ, QX, QY = (p.inp(i) for i in range(6))
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
    B = p.mul_c0(t1b, PQ)
    C = p.mul_c1(t10b, PQ)
    return p, [nx, ny, nz, A, B, C]


def f6_mul_by_01(p, a, b0, b1):
    t0 = p.mul(a[0], b0)
    t1 = p.mul(a[1], b1)
    c0 = p.mul(a[1] + a[2], b1).nr() + t0 - t1.nr()
    c1 = p.mul(a[0] + a[1], b0 + b1) - t0 - t1
    c2 = p.mul(a[0] + a[2], b0) - t0 + t1
    return [c0, c1, c2]


def f6_mul_by_1(p, a, b1):
    return [p.mul(a[2], b1).nr(), p.mul(a[0], b1), p.mul(a[1], b1)]


def m014(p, f, A, B, C):
    """f * (A + B v + C v w)   (pairing mul_by_014(c0 = A, c1 = B, c4 = C))"""
    F0, F1 = f[0:3], f[3:6]
    aa = f6_mul_by_01(p, F0, A, B)
    bb = f6_mul_by_1(p, F1, C)
    s = f6_mul_by_01(p, [x + y for x, y in zip(F0, F1)], A, B + C)
    c0 = [aa[0] + bb[2].nr(), aa[1] + bb[0], aa[2] + bb[1]]
    c1 = [s[i] - aa[i] - bb[i] for i in range(3)]
    return c0 + c1


def f6_mul(p, a, b):
    t0, t1, t2 = p.mul(a[0], b[0]), p.mul(a[1], b[1]), p.mul(a[2], b[2])
    c0 = (p.mul(a[1] + a[2], b[1] + b[2]) - t1 - t2).nr() + t0
    c1 = p.mul(a[0] + a[1], b[0] + b[1]) - t0 - t1 + t2.nr()
    c2 = p.mul(a[0] + a[2], b[0] + b[2]) - t0 - t2 + t1
    return [c0, c1, c2]


def f6_nr(a):
    return [a[2].nr(), a[0], a[1]]


def f12_sqr(p, f):
    """pairing Fq12::square (complex squaring: 2 Fq6 products)"""
    a0, a1 = f[0:3], f[3:6]
    ab = f6_mul(p, a0, a1)
    t = f6_mul(p, [x + y for x, y in zip(a0, a1)], [x + y for x, y in zip(a0, f6_nr(a1))])
    c0 = [t[i] - ab[i] - f6_nr(ab)[i] for i in range(3)]
    c1 = [ab[i].dbl() for i in range(3)]
    return c0 + c1


def prog_msq():
    """f-chain step: f = (f * line)^2. in: F0..F5 A B C."""
    p = Prog("msq", ["F0", "F1", "F2", "F3", "F4", "F5", "A", "B", "C"])
    ins = [p.inp(i) for i in range(9)]
    return p, f12_sqr(p, m014(p, ins[0:6], ins[6], ins[7], ins[8]))


def prog_m():
    """f-chain step without the squaring: f = f * line. in: F0..F5 A B C."""
    p = Prog("m", ["F0", "F1", "F2", "F3", "F4", "F5", "A", "B", "C"])
    ins = [p.inp(i) for i in range(9)]
    return p, m014(p, ins[0:6], ins[6], ins[7], ins[8])


def prog_mmsq():
    """two-proof f-chain step: f = (f * line_0 * line_1)^2, the squaring shared by the pair of
    proofs of one lane (their Miller values multiply into one product-tree node).
    in: F0..F5 A B C (proof 2j) A2 B2 C2 (proof 2j+1)."""
    p = Prog("mmsq", ["F0", "F1", "F2", "F3", "F4", "F5", "A", "B", "C", "A2", "B2", "C2"])
    ins = [p.inp(i) for i in range(12)]
    f1 = m014(p, ins[0:6], ins[6], ins[7], ins[8])
    return p, f12_sqr(p, m014(p, f1, ins[9], ins[10], ins[11]))


def prog_mm():
    """two-proof f-chain step without the squaring: f = f * line_0 * line_1."""
    p = Prog("mm", ["F0", "F1", "F2", "F3", "F4", "F5", "A", "B", "C", "A2", "B2", "C2"])
    ins = [p.inp(i) for i in range(12)]
    f1 = m014(p, ins[0:6], ins[6], ins[7], ins[8])
    return p, m014(p, f1, ins[9], ins[10], ins[11])


def prog_q4sq():
    """four-proof f-chain step: f = (f * l_0 * l_1 * l_2 * l_3)^2, the squaring shared by the
    four proofs of one lane (64 products instead of 2 x 38 for two pairs).
    in: F0..F5, then A B C of proofs 4j .. 4j+3."""
    p = Prog("q4sq", ["F%d" % i for i in range(6)] + ["%s%d" % (c, j) for j in range(4) for c in "ABC"])
    ins = [p.inp(i) for i in range(18)]
    f = ins[0:6]
    for j in range(4):
        f = m014(p, f, ins[6 + 3 * j], ins[7 + 3 * j], ins[8 + 3 * j])
    return p, f12_sqr(p, f)


def prog_q4():
    """four-proof f-chain step without the squaring."""
    p = Prog("q4", ["F%d" % i for i in range(6)] + ["%s%d" % (c, j) for j in range(4) for c in "ABC"])
    ins = [p.inp(i) for i in range(18)]
    f = ins[0:6]
    for j in range(4):
        f = m014(p, f, ins[6 + 3 * j], ins[7 + 3 * j], ins[8 + 3 * j])
    return p, f


def f12_mul(p, a, b):
    """pairing Fq12::mul (Karatsuba over Fq6): 18 products"""
    aa = f6_mul(p, a[0:3], b[0:3])
    bb = f6_mul(p, a[3:6], b[3:6])
    s = f6_mul(p, [x + y for x, y in zip(a[0:3], a[3:6])], [x + y for x, y in zip(b[0:3], b[3:6])])
    return [aa[i] + f6_nr(bb)[i] for i in range(3)] + [s[i] - aa[i] - bb[i] for i in range(3)]


GEN_IN = ["F%d" % i for i in range(6)] + ["L%d" % i for i in range(6)]


def prog_gm():
    """f-chain step on a group's line product L_n (k_line_prod: the product over the group's proofs
    of their step-n lines, a general Fq12) without the squaring: f = f * L. in: F0..F5 L0..L5."""
    p = Prog("gm", GEN_IN)
    ins = [p.inp(i) for i in range(12)]
    return p, f12_mul(p, ins[0:6], ins[6:12])


def prog_gmsq():
    """the group f-chain step: f = (f * L)^2 (30 products for a whole group of proofs)."""
    p = Prog("gmsq", GEN_IN)
    ins = [p.inp(i) for i in range(12)]
    return p, f12_sqr(p, f12_mul(p, ins[0:6], ins[6:12]))


def line_pair(p, l, l2):
    """the product of two sparse lines (A + B v) + (C v) w as (E0 + E1 v + E2 v^2) + (E4 v + E5 v^2) w
    (w^2 = v, v^3 = xi): 6 products"""
    A, B, C = l
    A2, B2, C2 = l2
    aa, bb, cc = p.mul(A, A2), p.mul(B, B2), p.mul(C, C2)
    return [aa + cc.nr(), p.mul(A + B, A2 + B2) - aa - bb, bb, p.mul(A + C, A2 + C2) - aa - cc,
            p.mul(B + C, B2 + C2) - bb - cc]


def pair_pair(p, P, P2):
    """the product of two line pairs (c1[0] = 0 in both): 15 products, a general Fq12"""
    E0, E1, E2, E4, E5 = P
    F0, F1, F2, F4, F5 = P2
    aa = f6_mul(p, [E0, E1, E2], [F0, F1, F2])
    xx, yy = p.mul(E4, F4), p.mul(E5, F5)
    bb = [(p.mul(E4 + E5, F4 + F5) - xx - yy).nr(), yy.nr(), xx]  # (x v + y v^2)(x' v + y' v^2)
    s = f6_mul(p, [E0, E1 + E4, E2 + E5], [F0, F1 + F4, F2 + F5])
    return [aa[i] + f6_nr(bb)[i] for i in range(3)] + [s[i] - aa[i] - bb[i] for i in range(3)]


def prog_q4i():
    """a group's first four lines (k_line_prod): l_0 l_1 l_2 l_3 from scratch as (l_0 l_1)(l_2 l_3),
    27 products (Q4 on f = 1: 52). in: F0..F5 (unused), then A B C of the four proofs."""
    p = Prog("q4i", ["F%d" % i for i in range(6)] + ["%s%d" % (c, j) for j in range(4) for c in "ABC"])
    ins = [p.inp(i) for i in range(18)]
    ls = [ins[6 + 3 * j: 9 + 3 * j] for j in range(4)]
    return p, pair_pair(p, line_pair(p, ls[0], ls[1]), line_pair(p, ls[2], ls[3]))


def prog_q4ik():
    """the same four-line product with the accumulator f kept in slots 0..5 (k_line_prod's later
    quads, the quad chain): the kernel stores the quad to slots 6..11 and multiplies it into f with
    GM / GMSQ -- 27 + 18 products per four lines instead of Q4's 52 (27 + 30 instead of Q4SQ's 64)"""
    p = Prog("q4ik", ["F%d" % i for i in range(6)] + ["%s%d" % (c, j) for j in range(4) for c in "ABC"],
             keep=range(6))
    ins = [p.inp(i) for i in range(18)]
    ls = [ins[6 + 3 * j: 9 + 3 * j] for j in range(4)]
    return p, pair_pair(p, line_pair(p, ls[0], ls[1]), line_pair(p, ls[2], ls[3]))


def aline_pair(p, l, l2, one):
    """the product of two affine lines normalised to a unit vw coefficient, (a + b v + v w)(a' + b' v + v w)
    = (a a' + xi + (a b' + a' b) v + b b' v^2) + ((a + a') v + (b + b') v^2) w (w^2 = v, v^3 = xi): 3
    products, in line_pair's layout (E0, E1, E2, E4, E5); `one` is an atom holding 1 (the xi term)"""
    a, b = l
    a2, b2 = l2
    aa, bb = p.mul(a, a2), p.mul(b, b2)
    return [aa + one.nr(), p.mul(a + b, a2 + b2) - aa - bb, bb, a + a2, b + b2]


def prog_aq4():
    """four affine lines (k_line_prod over the affine R-chain's lines, ZG_LINES_AFFINE): (l0 l1)(l2 l3)
    with unit-normalised lines l = a + b v + v w, 3 + 3 + 15 = 21 products (Q4I: 27). in: F0..F5 (kept:
    the group's accumulator), a0 b0 .. a3 b3, ONE (kept: the constant 1)."""
    p = Prog("aq4", ["F%d" % i for i in range(6)] + ["%s%d" % (c, j) for j in range(4) for c in "ab"] + ["ONE"],
             keep=list(range(6)) + [14])
    ins = [p.inp(i) for i in range(15)]
    ls = [ins[6 + 2 * j: 8 + 2 * j] for j in range(4)]
    one = ins[14]
    return p, pair_pair(p, aline_pair(p, ls[0], ls[1], one), aline_pair(p, ls[2], ls[3], one))


# ---------------------------------------------------------------- scheduling + slots
# Cost model (clocks of one SIMD, gfx950, measured with tools/mb_fq29 and tools/mb_rates): an
# Fq2 product in 29-bit digits is ~8,600 (x*y, 1,171 v_mad_u64_u32) or ~6,500 (square, x*Fq);
# operand formation ~4.4 per instruction of its mod-p add / sub chains (37 per Fq op).
PROD_CLK = {K_MUL: 8600, K_SQR: 6500, K_MULC0: 6500, K_MULC1: 6500}


def _form_instr(f, lazy):
    terms = list(f.values())
    if len(terms) == 1 and terms[0] == (1, 0):
        return 0
    if lazy and len(terms) == 2 and all(t == (1, 0) for t in terms):
        return 24
    n = 0
    for c0, c1 in terms:
        if (c0, c1) in ((1, 0), (-1, 0)):
            pass
        elif (c0, c1) in ((1, 1), (-1, -1)) or c1 == 0 and abs(c0) == 2:
            n += 74
        elif (c0, c1) in ((0, 1), (0, -1)):
            n += 25
        else:
            n += 74 * 3
    return n + 74 * (len(terms) - 1)


def _lazy_cost(lines, code):
    n = 0
    for ln in lines:
        if ln.startswith(("f2a_lzadd", "f2p_")):
            n += 24
        elif "f2_kp" in ln:
            n += 24
        elif "f2_reduce_q" in ln:
            n += 110
    red = int(code.split(",")[2].strip(" )"))
    return n + {1: 0, 2: 50, 0: 60}[red]


def prod_costs(prog):
    out = []
    if LAZY:
        slot = {}  # costs do not depend on the slot map
        for k in {k for L, R, _ in prog.prods for k in list(L) + list(R)}:
            slot[k] = ("g", 0) if k[0] == "in" and k[1] in prog.glob else 0
        for L, R, kind in prog.prods:
            lines, code = lazy_product(L, R, kind, slot)
            out.append(PROD_CLK[kind] + 4.4 * _lazy_cost(lines, code))
        return out
    for L, R, kind in prog.prods:
        c = _form_instr(L, True) + (0 if kind == K_SQR else _form_instr(R, False))
        out.append(PROD_CLK[kind] + 4.4 * c)
    return out


def balance_rounds(sch, costs, nw, share=2):
    """order each round's products over the waves so that the two waves of a SIMD (w, w + nw/2)
    carry a heavy and a light product; returns the modelled time (sum over rounds of the
    busiest SIMD's load). share 1 (the R-chain: one wave per SIMD): a round costs its heaviest
    product."""
    if share == 1:
        total = 0
        for r, pick in enumerate(sch["rounds"]):
            srt = sorted([i for i in pick if i is not None], key=lambda i: -costs[i])
            total += costs[srt[0]] if srt else 0
            sch["rounds"][r] = srt + [None] * (nw - len(srt))
        return total
    half = nw // 2
    total = 0
    for r, pick in enumerate(sch["rounds"]):
        srt = sorted(pick, key=lambda i: -costs[i])
        srt += [None] * (nw - len(srt))
        order = [None] * nw
        for sidx in range(half):  # heaviest with lightest
            order[sidx], order[sidx + half] = srt[sidx], srt[nw - 1 - sidx]
        c = lambda i: 0 if i is None else costs[i]
        total += max(c(order[k]) + c(order[k + half]) for k in range(half))
        sch["rounds"][r] = order  # None: an idle wave
    return total


def schedule(prog, outs, nw, search=0, max_slots=None, shift=1, partial=False, cost=False, share=2):
    """list-schedule products into rounds of <= nw; allocate LDS slots with reuse.
    search > 0: also try that many seeded random tie-breaks among ready products and keep the
    schedule with the fewest rounds whose slots fit max_slots (then the fewest slots).
    shift 0: a slot may be rewritten in the round of its last read (the engine then puts a
    barrier between a round's operand reads and its writes: ProgInfo.rb). partial: the random
    candidates may also take fewer than nw ready products in a round (shorter live ranges)."""
    best = _schedule(prog, outs, nw, None, 0, shift)
    if cost:
        costs = prod_costs(prog)
        best["time"] = balance_rounds(best, costs, nw, share)
    if search:
        rng = random.Random(20260101)
        for t in range(search):
            slacks = [0.5, 1.5, 3, 6, 12] if partial else [0.5, 1.5, 3, 6]
            cand = _schedule(prog, outs, nw, rng, rng.choice(slacks), shift, partial)
            fits = max_slots is None or cand["nslots"] <= max_slots
            bfits = max_slots is None or best["nslots"] <= max_slots
            if cost:  # modelled time (SIMD-balanced rounds) instead of the round count
                cand["time"] = balance_rounds(cand, costs, nw, share)
                key = (not fits, cand["time"], cand["nslots"])
                bkey = (not bfits, best["time"], best["nslots"])
            else:
                key = (not fits, len(cand["rounds"]), cand["nslots"])
                bkey = (not bfits, len(best["rounds"]), best["nslots"])
            if key < bkey:
                best = cand
    return best


def _schedule(prog, outs, nw, rng, slack, shift=1, partial=False, fixed=None):
    n = len(prog.prods)
    deps = []
    for L, R, _ in prog.prods:
        deps.append(sorted({k[1] for k in list(L) + list(R) if k[0] == "p"}))
    succ = [[] for _ in range(n)]
    for i, d in enumerate(deps):
        for j in d:
            succ[j].append(i)
    height = [0] * n
    for i in reversed(range(n)):
        height[i] = 1 + max([height[j] for j in succ[i]] or [0])
    # sinks: products whose only use is to be output j >= sink_from as they stand (a line
    # coefficient that goes to HBM): the wave stores them there and they take no LDS slot
    sinks = {}
    if prog.sink_from is not None:
        used = {k[1] for L, R, _ in prog.prods for k in list(L) + list(R) if k[0] == "p"}
        for j, f in enumerate(outs):
            if j >= prog.sink_from and len(f) == 1:
                (k, c), = f.items()
                if k[0] == "p" and c == (1, 0) and k[1] not in used and k[1] not in sinks:
                    sinks[k[1]] = j
    rnd = [None] * n
    rounds = []
    done = set()
    if fixed is not None:  # a cached round assignment (zg_prog_sched.json)
        for r, pick in enumerate(fixed):
            for i in pick:
                assert all(j in done for j in deps[i]), "cached schedule violates a dependency"
                rnd[i] = r
            rounds.append(list(pick))
            done.update(pick)
        assert len(done) == n
    while len(done) < n:
        ready = [i for i in range(n) if rnd[i] is None and all(j in done for j in deps[i])]
        ready.sort(key=lambda i: (-height[i] + (rng.random() * slack if rng else 0), i))
        take = nw
        if partial and rng is not None and rng.random() < 0.3:
            take = rng.randrange(1, nw + 1)
        pick = ready[:take]
        for i in pick:
            rnd[i] = len(rounds)
        rounds.append(pick)
        done.update(pick)
    nr = len(rounds)
    # last read round of every atom (output forms are read in round nr)
    last = {}
    for i, (L, R, _) in enumerate(prog.prods):
        for k in list(L) + list(R):
            last[k] = max(last.get(k, -1), rnd[i])
    for j, f in enumerate(outs):
        for k in f:
            if not (k[0] == "p" and sinks.get(k[1]) == j):
                last[k] = max(last.get(k, -1), nr)
    nin = len(prog.inputs)
    lds_in = [i for i in range(nin) if i not in prog.glob]
    assert lds_in == list(range(len(lds_in))), "global-memory inputs come last"
    slot = {("in", i): i for i in lds_in}
    slot.update({("in", i): ("g", j) for i, j in prog.glob.items()})
    free_at = {}  # slot -> first round it may be rewritten
    for i in lds_in:
        if i not in prog.keep:
            free_at[i] = last.get(("in", i), -1) + shift
    nslots = len(lds_in)
    for r, pick in enumerate(rounds):
        for i in pick:
            if i in sinks:
                slot[("p", i)] = ("sink", sinks[i])
                continue
            cand = sorted(s for s, fr in free_at.items() if fr <= r)
            if cand:
                s = cand[0]
            else:
                s = nslots
                nslots += 1
            slot[("p", i)] = s
            free_at[s] = last.get(("p", i), nr) + shift
    # outputs are written to input slots 0.. after the output round: they must not clobber a
    # kept input
    assert all(j not in prog.keep for j in range(len(outs)) if j < nin) or prog.name in ("dbl", "add", "q4ik", "aq4")
    return {"rounds": rounds, "slot": slot, "nslots": nslots, "rnd": rnd, "rb": int(shift == 0), "sinks": sinks}


def simulate(prog, outs, sch, vals):
    """run the schedule on an LDS model with the slot map; returns output values"""
    lds = {}
    for i, v in enumerate(vals):
        lds[sch["slot"][("in", i)]] = v

    def ev(f):
        r0 = r1 = 0
        for k, (c0, c1) in f.items():
            x0, x1 = lds[sch["slot"][k]]
            r0 += c0 * x0 - c1 * x1
            r1 += c0 * x1 + c1 * x0
        return (r0 % P, r1 % P)
    for pick in sch["rounds"]:
        res = []
        for i in pick:
            if i is None:
                continue
            L, R, kind = prog.prods[i]
            x, y = ev(L), ev(R)
            if kind == K_MULC0:
                y = (y[0], 0)
            elif kind == K_MULC1:
                y = (y[1], 0)
            res.append((i, ((x[0] * y[0] - x[1] * y[1]) % P, (x[0] * y[1] + x[1] * y[0]) % P)))
        for i, v in res:  # all reads of a round precede its writes (rb: enforced by a barrier)
            lds[sch["slot"][("p", i)]] = v
    return [lds[("sink", j)] if j in sch["sinks"].values() else ev(f) for j, f in enumerate(outs)]


def reference(prog, outs, vals):
    env = {("in", i): v for i, v in enumerate(vals)}

    def ev(f):
        r0 = r1 = 0
        for k, (c0, c1) in f.items():
            x0, x1 = env[k]
            r0 += c0 * x0 - c1 * x1
            r1 += c0 * x1 + c1 * x0
        return (r0 % P, r1 % P)
    for i, (L, R, kind) in enumerate(prog.prods):
        x, y = ev(L), ev(R)
        if kind == K_MULC0:
            y = (y[0], 0)
        elif kind == K_MULC1:
            y = (y[1], 0)
        env[("p", i)] = ((x[0] * y[0] - x[1] * y[1]) % P, (x[0] * y[1] + x[1] * y[0]) % P)
    return [ev(f) for f in outs]


# ---------------------------------------------------------------- code generation
def scaled(s, c0, c1):
    """(C++ expression, sign) of (c0 + c1 u) * atom-in-slot-s"""
    x = "at.q(%d)" % s[1] if isinstance(s, tuple) else "at.get(%d)" % s
    if (c0, c1) in ((1, 0), (-1, 0)):
        return x, c0
    if (c0, c1) in ((1, 1), (-1, -1)):
        return "f2_mul_nr(%s)" % x, c0
    if (c0, c1) in ((0, 1), (0, -1)):
        return "f2_mul_u(%s)" % x, c1
    if c1 == 0:
        return "f2_smul<%d>(%s)" % (abs(c0), x), 1 if c0 > 0 else -1
    return "f2_gmul<%d, %d>(%s)" % (c0, c1, x), 1


def form_code(f, slot, lazy):
    """C++ expression for a form. lazy: the value feeds a product as its lazy operand, so a
    plain sum / difference of two canonical atoms may skip the reduction (< 2p)."""
    order = lambda kv: (1, slot[kv[0]][1]) if isinstance(slot[kv[0]], tuple) else (0, slot[kv[0]])
    terms = [scaled(slot[k], c0, c1) for k, (c0, c1) in sorted(f.items(), key=order)]
    terms.sort(key=lambda t: -t[1])  # a positive term first
    if lazy and len(terms) == 2 and all(t[0].startswith(("at.get", "at.q")) for t in terms) and terms[0][1] > 0:
        return "f2_lz_%s(%s, %s)" % ("add" if terms[1][1] > 0 else "sub", terms[0][0], terms[1][0])
    e, sg = terms[0]
    acc = e if sg > 0 else "f2_neg(%s)" % e
    for e, sg in terms[1:]:
        acc = "f2_%s(%s, %s)" % ("add" if sg > 0 else "sub", acc, e)
    return acc


# ---------------------------------------------------------------- lazy operand forms
# An operand coefficient is evaluated as a plain 12-word integer: the K p offset that covers its
# negative terms, plus / minus atom coefficients one unit at a time (f2a_lzadd / f2p_* dual carry
# chains over both coefficients), never reduced. Its bound B (value <= B p) is the number of units
# (<= 9 so that it stays below 2^384); a longer form is reduced mid-way (fq_reduce_q). The product
# gets ZG_KIND(kind, k, red) from the bounds: red conditional subtractions (or 0: fq_reduce_q)
# bring its raw result t < S / 2^384 + p, S <= M p^2, back below p.
LAZY = True
SEG_FIRST, SEG_NEXT = 9, 8
KMAX = 12


def lazy_form(f, slot, var, canon):
    """C++ lines assigning Fq2 `var` from form f; returns (lines, bound B). Atoms are read from
    LDS right before their first use (short live ranges). A coefficient c with |c| >= 2 becomes ONE
    accumulation of a temporary |c| * atom built by doublings (6 a: 3 dual ops + 1, not 6)."""
    items = sorted(f.items(), key=lambda kv: (1, slot[kv[0]][1]) if isinstance(slot[kv[0]], tuple) else (0, slot[kv[0]]))
    ref = lambda k: "at.q(%d)" % slot[k][1] if isinstance(slot[k], tuple) else "at.get(%d)" % slot[k]
    if len(items) == 1 and items[0][1] == (1, 0):
        return ["%s = %s;" % (var, ref(items[0][0]))], 1
    ops = []  # (atom index, weight, (sign, comp-0 part), (sign, comp-1 part))
    sg = lambda v: 1 if v > 0 else -1
    for jj, (k, (c0, c1)) in enumerate(items):
        if c0:
            ops.append((jj, abs(c0), (sg(c0), ".c0"), (sg(c0), ".c1")))
        if c1:
            ops.append((jj, abs(c1), (-sg(c1), ".c1"), (sg(c1), ".c0")))
    lines, loaded, temps = [], set(), set()
    u = lambda jj: "%s_u%d" % (var, jj)

    def load(jj):
        if jj not in loaded:
            loaded.add(jj)
            lines.append("const Fq2 %s = %s;" % (u(jj), ref(items[jj][0])))

    def scaled(jj, w):  # the name of w * atom jj (w <= 9: < 9p < 2^384)
        load(jj)
        if w == 1:
            return u(jj)
        t = "%s_w%d_%d" % (var, jj, w)
        if t not in temps:
            temps.add(t)
            bits = bin(w)[3:]
            lines.append("Fq2 %s = %s;" % (t, u(jj)))
            for bit in bits:
                lines.append("f2a_lzadd(%s.c0.l, %s.c0.l, %s.c0.l, %s.c1.l, %s.c1.l, %s.c1.l);" % ((t,) * 6))
                if bit == "1":
                    lines.append("f2a_lzadd(%s.c0.l, %s.c0.l, %s.c0.l, %s.c1.l, %s.c1.l, %s.c1.l);" % (
                        t, t, u(jj), t, t, u(jj)))
        return t
    # segments of at most SEG_FIRST (then SEG_NEXT) units; an op is split across a boundary
    segs, cur, room, cap = [], [], SEG_FIRST, SEG_FIRST
    for (jj, w, a, b) in ops:
        if cur and w > room and w <= SEG_NEXT:  # start a new segment rather than split the op
            segs.append(cur)
            cur, room = [], SEG_NEXT
        while w:
            take = min(w, room)
            cur.append((jj, take, a, b))
            w -= take
            room -= take
            if room == 0:
                segs.append(cur)
                cur, room = [], SEG_NEXT
    if cur:
        segs.append(cur)
    B = 0
    for si, seg in enumerate(segs):
        k0 = sum(w for (jj, w, a, b) in seg if a[0] < 0)
        k1 = sum(w for (jj, w, a, b) in seg if b[0] < 0)
        units = sum(w for (jj, w, a, b) in seg)
        seg = list(seg)
        if si == 0:
            if k0 == 0 and k1 == 0:
                jj, w, a, b = seg.pop(0)
                t = scaled(jj, w)
                lines.append("%s.c0 = %s%s; %s.c1 = %s%s;" % (var, t, a[1], var, t, b[1]))
            else:
                lines.append("%s = f2_kp<%d, %d>();" % (var, k0, k1))
            B = units
        else:
            lines.append("%s = f2_reduce_q(%s);" % (var, var))
            if k0 or k1:
                lines.append("{ const Fq2 o = f2_kp<%d, %d>(); f2a_lzadd(%s.c0.l, %s.c0.l, o.c0.l, %s.c1.l, %s.c1.l, o.c1.l); }"
                             % (k0, k1, var, var, var, var))
            B = 1 + units
        for (jj, w, a, b) in seg:
            t = scaled(jj, w)
            fn = {(1, 1): "f2a_lzadd", (1, -1): "f2p_as", (-1, 1): "f2p_sa", (-1, -1): "f2p_ss"}[(a[0], b[0])]
            lines.append("%s(%s.c0.l, %s.c0.l, %s%s.l, %s.c1.l, %s.c1.l, %s%s.l);" % (
                fn, var, var, t, a[1], var, var, t, b[1]))
    assert B <= 9
    if canon:
        lines.append("%s = f2_reduce_q(%s);" % (var, var) if B >= 2 else
                     "fq29_canon(%s.c0.l, %s.c0.l); fq29_canon(%s.c1.l, %s.c1.l);" % (var, var, var, var))
        B = 1
    return lines, B


def fits(M):
    """the raw product t < M p^2 / 2^384 + p stays below 2^384 (12 words, fq_reduce_q)"""
    return M * P * P + P * 2 ** 384 < 2 ** 768


def red_of(M):
    """conditional subtractions that bring t < M p^2 / 2^384 + p below p (0: quotient estimate)"""
    r = -(-M * P // 2 ** 384)
    return r if r <= 2 else 0


HOIST = int(os.environ.get("ZG_GEN_HOIST", "0"))  # issue the first HOIST LDS / HBM atom loads of a product's operands before its first carry chain


def hoist_loads(lines):
    """move the atom loads (`const Fq2 v = at.get(s);` / `at.q(j)`) to the front, in order: the carry
    chains are asm volatile, which the compiler does not move loads across, so a load emitted right
    before its first use exposes one LDS round trip per atom; hoisted, they are all in flight at once"""
    if not HOIST:
        return lines
    ld = [ln for ln in lines if ln.startswith("const Fq2 ") and (" = at.get(" in ln or " = at.q(" in ln)]
    ld = ld[:HOIST]  # the first HOIST atoms (24 VGPRs each, live next to the forms' accumulators)
    return ld + [ln for ln in lines if ln not in ld]


HOIST_GLOBAL = int(os.environ.get("ZG_GEN_HOIST_GLOBAL", "1"))  # hoist over both operands (else per operand)


def hoist_op(lines):
    return lines if HOIST_GLOBAL else hoist_loads(lines)


def lazy_product(L, R, kind, slot):
    """(lines, encoded kind expression) for one product"""
    lines, code = _lazy_product(L, R, kind, slot)
    return (hoist_loads(lines) if HOIST_GLOBAL else lines), code


def _lazy_product(L, R, kind, slot):
    if kind == K_SQR:
        lx, bx = lazy_form(L, slot, "x", False)
        M = 4 * bx * bx
        if bx > 4 or not fits(M):  # x0 + k p - x1 <= 2 B p must stay below 2^384
            lx.append("x = f2_reduce_q(x);")
            bx, M = 1, 4
        assert fits(M) and 2 * bx * P < 2 ** 384
        return hoist_op(lx), "ZG_KIND(1, %d, %d)" % (bx, red_of(M))
    if kind in (K_MULC0, K_MULC1):
        assert len(R) == 1 and list(R.values())[0] == (1, 0), "the Fq factor is an input atom"
        lx, bx = lazy_form(L, slot, "x", False)
        ly, _ = lazy_form(R, slot, "y", False)
        assert fits(bx)
        return hoist_op(lx) + hoist_op(ly), "ZG_KIND(%d, 0, %d)" % (kind, red_of(bx))
    best = None
    for A, Bf in ((L, R), (R, L)):
        lx, bx = lazy_form(A, slot, "x", False)
        ly, by = lazy_form(Bf, slot, "y", False)
        M = bx * (2 * by + 1)
        cost = (len(lx) + len(ly), M)
        cand = (not fits(M), red_of(M) == 0, cost, lx, bx, ly, by)
        if best is None or cand[:3] < best[:3]:
            best = cand
    _, _, _, lx, bx, ly, by = best
    M = bx * (2 * by + 1)
    while not fits(M):  # too large for 12 words: reduce the larger operand
        if bx >= by:
            lx.append("x = f2_reduce_q(x);")
            bx = 1
        else:
            ly.append("y = f2_reduce_q(y);")
            by = 1
        M = bx * (2 * by + 1)
    assert by + 1 <= KMAX and fits(M) and bx <= 9 and by <= 9
    return hoist_op(lx) + hoist_op(ly), "ZG_KIND(0, %d, %d)" % (by + 1, red_of(M))


def _run_lines(lines, atoms, env):
    """interpret the emitted lazy-form lines on integers (exact, with the carry-chain
    preconditions of every step asserted); atoms: slot -> (c0, c1), global q(j) -> ('g', j)"""
    import re
    for ln in lines:
        for st in [x.strip() for x in ln.replace("{ ", "").replace(" }", "").split(";") if x.strip()]:
            m = re.match(r"const Fq2 (\w+) = at\.(get|q)\((\d+)\)$", st)
            if m:
                env[m.group(1)] = atoms[int(m.group(3)) if m.group(2) == "get" else ("g", int(m.group(3)))]
                continue
            m = re.match(r"(\w+) = at\.(get|q)\((\d+)\)$", st)
            if m:
                env[m.group(1)] = atoms[int(m.group(3)) if m.group(2) == "get" else ("g", int(m.group(3)))]
                continue
            m = re.match(r"Fq2 (\w+) = (\w+)$", st)
            if m:
                env[m.group(1)] = env[m.group(2)]
                continue
            m = re.match(r"(const Fq2 )?(\w+) = f2_kp<(\d+), (\d+)>\(\)$", st)
            if m:
                env[m.group(2)] = (int(m.group(3)) * P, int(m.group(4)) * P)
                continue
            m = re.match(r"(\w+) = f2_reduce_q\((\w+)\)$", st)
            if m:
                v = env[m.group(2)]
                assert all(0 <= c < 2 ** 384 for c in v)
                env[m.group(1)] = (v[0] % P, v[1] % P)
                continue
            m = re.match(r"(\w+)\.c0 = (\w+)\.(c[01]); (\w+)\.c1 = (\w+)\.(c[01])$", st + "")
            if m:
                pass
            m = re.match(r"(\w+)\.c([01]) = (\w+)\.c([01])$", st)
            if m:
                v = list(env.get(m.group(1), (0, 0)))
                v[int(m.group(2))] = env[m.group(3)][int(m.group(4))]
                env[m.group(1)] = tuple(v)
                continue
            m = re.match(r"(f2a_lzadd|f2p_as|f2p_sa|f2p_ss)\((\w+)\.c0\.l, \w+\.c0\.l, (\w+)\.(c[01])\.l, "
                         r"\w+\.c1\.l, \w+\.c1\.l, (\w+)\.(c[01])\.l\)$", st)
            if m:
                fn, v = m.group(1), list(env[m.group(2)])
                a0 = env[m.group(3)][int(m.group(4)[1])]
                a1 = env[m.group(5)][int(m.group(6)[1])]
                sgn = {"f2a_lzadd": (1, 1), "f2p_as": (1, -1), "f2p_sa": (-1, 1), "f2p_ss": (-1, -1)}[fn]
                for c, (sg_, aa) in enumerate(zip(sgn, (a0, a1))):
                    v[c] = v[c] + sg_ * aa
                    assert 0 <= v[c] < 2 ** 384, (st, v[c])
                env[m.group(2)] = tuple(v)
                continue
            m = re.match(r"fq29_canon\((\w+)\.c([01])\.l, \w+\.c[01]\.l\)$", st)
            if m:
                v = list(env[m.group(1)])
                c = int(m.group(2))
                assert v[c] < 2 * P
                v[c] = v[c] - P if v[c] >= P else v[c]
                env[m.group(1)] = tuple(v)
                continue
            raise AssertionError("unparsed: " + st)
    return env


def check_lazy(specs, trials=40):
    """the emitted lazy forms and product codes, interpreted on extreme and random atoms: every
    carry-chain precondition holds, operands are the forms' values mod p, and each product's raw
    result bound matches its ZG_KIND red"""
    import re
    rng = random.Random(21)
    for name, prog, outs, nw, sch in specs:
        slot = sch["slot"]
        atoms_needed = set(v for v in slot.values() if not (isinstance(v, tuple) and v[0] == "sink"))
        for t in range(trials):
            pick = [lambda: 0, lambda: P - 1, lambda: rng.randrange(P)][t % 3] if t < 6 else (lambda: rng.choice([0, P - 1, rng.randrange(P)]))
            atoms = {a: (pick(), pick()) for a in atoms_needed}
            val = lambda f: tuple(sum(((c0 * atoms[slot[k]][0] - c1 * atoms[slot[k]][1]) if comp == 0 else
                                       (c0 * atoms[slot[k]][1] + c1 * atoms[slot[k]][0])) for k, (c0, c1) in f.items()) % P
                                  for comp in (0, 1))
            for i, (L, R, kind) in enumerate(prog.prods):
                lines, code = lazy_product(L, R, kind, slot)
                env = _run_lines(lines, atoms, {})
                kd, k, red = map(int, re.match(r"ZG_KIND\((\d+), (\d+), (\d+)\)", code).groups())
                x = env["x"]
                assert all(0 <= c < 2 ** 384 for c in x)
                if kd == 1:
                    assert (x[0] % P, x[1] % P) == val(L)
                    d = x[0] + k * P
                    assert d < 2 ** 384
                    d -= x[1]
                    assert d >= 0
                    S = [(x[0] + x[1]) * d, x[0] * 2 * x[1]]
                else:
                    y = env["y"]
                    assert all(0 <= c < 2 ** 384 for c in y)
                    assert {(x[0] % P, x[1] % P), (y[0] % P, y[1] % P)} <= {val(L), val(R)} or kd != 0
                    if kd == 0:
                        assert y[1] <= (k - 1) * P
                        S = [x[0] * y[0] + x[1] * (k * P - y[1]), x[0] * y[1] + x[1] * y[0]]
                    else:
                        S = [x[0] * y[0], x[1] * y[0]] if kd == 2 else [x[0] * y[1], x[1] * y[1]]
                for Sc in S:
                    assert Sc >= 0
                    tmax = Sc // 2 ** 384 + P  # t < S / 2^384 + p
                    assert tmax <= (2 ** 384 if red == 0 else (red + 1) * P), (name, i, red)
            for j, f in enumerate(outs):
                if j in sch.get("sinks", {}).values():
                    continue
                lines, _ = lazy_form(f, slot, "v", True)
                env = _run_lines(lines, atoms, {})
                assert env["v"] == val(f) and all(c < P for c in env["v"]), (name, j)


def emit(specs):
    out = ["// GENERATED by zebra_amd/csrc/gen_prog.py -- do not edit.", "#pragma once",
           "// included by zg_prog.h (needs AtomSpace and the Fq2 helpers)", "namespace zg {"]
    prod_cases, out_cases = [], []
    infos, sched = [], []
    gk, go = 0, 0
    for pidx, (name, prog, outs, nw, sch) in enumerate(specs):
        nin = len(prog.inputs)
        use = "if constexpr (M & (1u << %d))" % pidx  # the kernel's program mask (prog_run<RB, M>)
        # products
        for i, (L, R, kind) in enumerate(prog.prods):
            s = sch["slot"]
            if LAZY:
                d = s[("p", i)]
                dst = SINK_BASE + d[1] if isinstance(d, tuple) else d
                lines, code = lazy_product(L, R, kind, s)
                prod_cases.append("  case %d: %s {  // %s p%d round %d%s\n    %s\n    dst = %d; return %s;\n  } break;" % (
                    gk + i, use, name, i, sch["rnd"][i], " -> HBM output %d" % d[1] if isinstance(d, tuple) else "",
                    "\n    ".join(lines), dst, code))
                continue
            if kind == K_SQR:
                x, y = form_code(L, s, False), "x"
            elif kind in (K_MULC0, K_MULC1):
                x, y = form_code(L, s, True), form_code(R, s, False)
            else:
                # at most one lazy operand: the one that is a plain two-term sum
                lx = form_code(L, s, True)
                if lx.startswith("f2_lz_"):
                    x, y = lx, form_code(R, s, False)
                else:
                    x, y = form_code(R, s, True), form_code(L, s, False)
            d = s[("p", i)]
            dst = SINK_BASE + d[1] if isinstance(d, tuple) else d
            prod_cases.append("  case %d: %s { x = %s; y = %s; dst = %d; return %d; } break;  // %s p%d round %d%s" % (
                gk + i, use, x, y, dst, kind, name, i, sch["rnd"][i], " -> HBM output %d" % d[1] if isinstance(d, tuple) else ""))
        for j, f in enumerate(outs):
            if j in sch.get("sinks", {}).values():
                out_cases.append("  case %d: return f2_zero();  // %s out %d: stored by its product" % (go + j, name, j))
            elif LAZY:
                lines, _ = lazy_form(f, sch["slot"], "v", True)
                lines = hoist_loads(lines)
                out_cases.append("  case %d: %s {  // %s out %d\n    Fq2 v;\n    %s\n    return v;\n  } break;" % (
                    go + j, use, name, j, "\n    ".join(lines)))
            else:
                out_cases.append("  case %d: %s { return %s; } break;  // %s out %d" % (
                    go + j, use, form_code(f, sch["slot"], False), name, j))
        off = len(sched)
        for pick in sch["rounds"]:
            sched.extend([-1 if i is None else i for i in pick] + [-1] * (nw - len(pick)))
        infos.append((name, nin, len(prog.prods), len(outs), len(sch["rounds"]), nw, off, gk, go, sch["nslots"],
                      sch["rb"]))
        gk += len(prog.prods)
        go += len(outs)
    out.append("#define ZG_PROG_LAZY %d  // operands as lazy forms, products return ZG_KIND codes" % int(LAZY))
    out.append("struct ProgInfo { int nin, nprod, nout, nrounds, nw, sched, gk, go, nslots, rb; };")
    for k, (name, nin, npr, nout, nr, nw, off, g1, g2, ns, rb) in enumerate(infos):
        out.append("#define ZG_PROG_%s %d  // %d products in %d rounds of %d waves, %d LDS slots%s" % (
            name.upper(), k, npr, nr, nw, ns, ", read barrier" if rb else ""))
    out.append("__device__ __constant__ const ProgInfo PROG_INFO[%d] = {%s};" % (len(infos), ", ".join(
        "{%d, %d, %d, %d, %d, %d, %d, %d, %d, %d}" % i[1:] for i in infos)))
    out.append("__device__ __constant__ const int8_t PROG_SCHED[%d] = {%s};" % (len(sched), ", ".join(
        map(str, sched))))
    lsinks = [sorted(sch.get("sinks", {}).values()) for name, prog, outs, nw, sch in specs if name in ("dbl", "add")]
    assert all(x == lsinks[0] for x in lsinks), lsinks
    out.append("#define ZG_SINK_BASE %d  // dst >= this: the product is output (dst - base), stored to HBM" % SINK_BASE)
    out.append("#define ZG_LINES_SINK_MASK 0x%x  // lines outputs stored by their products" %
               sum(1 << j for j in lsinks[0]))
    for name, nslots in (("LINES", max(i[9] for i in infos if i[0] in ("dbl", "add"))),
                         ("FCHAIN", max(i[9] for i in infos if i[0] in ("msq", "m", "mmsq", "mm", "q4sq", "q4", "gm", "gmsq", "q4i", "q4ik", "aq4")))):
        out.append("#define ZG_%s_SLOTS %d" % (name, nslots))
    out.append("// program mask of a kernel: ZG_PMASK(A) | ZG_PMASK(B) ... (bit k: program ZG_PROG_* = k)")
    out.append("#define ZG_PMASK(P) (1u << ZG_PROG_##P)")
    out.append("// operands of global product gk; returns the product kind (f2_mul_kind). M: the programs the")
    out.append("// calling kernel runs -- only their cases are compiled in, so the register allocation of one")
    out.append("// kernel does not carry the operand forms of every other program")
    out.append("template <uint32_t M>")
    out.append("__device__ __forceinline__ int prog_operands(int gk, const AtomSpace& at, Fq2& x, Fq2& y, int& dst) {")
    out.append("  switch (gk) {")
    out.extend(prod_cases)
    out.append("  default: break;")
    out.append("  }")
    out.append("  x = y = f2_zero();")
    out.append("  dst = 0;")
    out.append("  return 0;")
    out.append("}")
    out.append("template <uint32_t M>")
    out.append("__device__ __forceinline__ Fq2 prog_output(int go, const AtomSpace& at) {")
    out.append("  switch (go) {")
    out.extend(out_cases)
    out.append("  default: break;")
    out.append("  }")
    out.append("  return f2_zero();")
    out.append("}")
    out.append("}  // namespace zg")
    return out


SINK_BASE = 64
NW_LINES = 4   # one wave per SIMD; 13 slots (78 KB) so that two blocks share a CU
NW_FCHAIN = 8
LINES_MAX_SLOTS = 13


SCHED_CACHE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "zg_prog_sched.json")
SEARCH = {"mmsq": 3000, "mm": 3000, "q4sq": 3000, "q4": 3000, "gm": 3000, "gmsq": 3000, "q4i": 3000, "q4ik": 3000,
          "aq4": 3000,
          "dbl": 6000, "add": 6000}


def build_all(search=None):
    """search None: the round assignments cached in zg_prog_sched.json where present (checked:
    dependencies, slot budget); search N: a fresh seeded search of N candidates per program"""
    cache = {}
    if search is None and os.path.exists(SCHED_CACHE):
        cache = json.load(open(SCHED_CACHE))
    specs = []
    for fn, nw in ((prog_dbl, NW_LINES), (prog_add, NW_LINES), (prog_msq, NW_FCHAIN), (prog_m, NW_FCHAIN),
                   (prog_mmsq, NW_FCHAIN), (prog_mm, NW_FCHAIN), (prog_q4sq, NW_FCHAIN), (prog_q4, NW_FCHAIN),
                   (prog_gm, NW_FCHAIN), (prog_gmsq, NW_FCHAIN), (prog_q4i, NW_FCHAIN), (prog_q4ik, NW_FCHAIN),
                   (prog_aq4, NW_FCHAIN)):
        prog, outs = fn()
        # the two-proof programs must fit the one-proof f-chain's LDS (25 slots x 6 KB)
        shift, partial, cost, slots = {prog_mmsq: (1, False, True, 25), prog_mm: (1, False, True, 25),
                                       prog_q4sq: (0, True, True, 25), prog_q4: (0, True, True, 25),
                                       prog_gm: (0, True, True, 25), prog_gmsq: (0, True, True, 25),
                                       prog_q4i: (0, True, True, 25), prog_q4ik: (0, True, True, 25),
                                       prog_aq4: (0, True, True, 25),
                                       prog_dbl: (0, True, True, LINES_MAX_SLOTS),
                                       prog_add: (0, True, True, LINES_MAX_SLOTS)}.get(fn, (1, False, False, None))
        share = 1 if fn in (prog_dbl, prog_add) else 2
        if prog.name in cache:
            sch = _schedule(prog, outs, nw, None, 0, shift, partial,
                            fixed=[[i for i in r if i is not None] for r in cache[prog.name]])
            if cost:
                sch["time"] = balance_rounds(sch, prod_costs(prog), nw, share)
        elif slots is not None:
            n = search if search is not None else SEARCH[prog.name]
            sch = schedule(prog, outs, nw, n, slots, shift=shift, partial=partial, cost=cost, share=share)
        else:
            sch = schedule(prog, outs, nw)
        if slots is not None:
            assert sch["nslots"] <= slots, (prog.name, sch["nslots"])
        specs.append((prog.name, prog, outs, nw, sch))
    return specs


def selfcheck(specs):
    rng = random.Random(11)
    for name, prog, outs, nw, sch in specs:
        for _ in range(3):
            vals = [(rng.randrange(P), rng.randrange(P)) for _ in prog.inputs]
            if name in ("dbl", "add"):
                vals[3] = (rng.randrange(P), rng.randrange(P))
            assert simulate(prog, outs, sch, vals) == reference(prog, outs, vals), name


if __name__ == "__main__":
    search = int(sys.argv[sys.argv.index("--search") + 1]) if "--search" in sys.argv else None
    specs = build_all(search)
    if search is not None:  # record the round assignments (waves in order, None = idle)
        json.dump({name: sch["rounds"] for name, prog, outs, nw, sch in specs if name in SEARCH},
                  open(SCHED_CACHE, "w"), indent=0)
    selfcheck(specs)
    if LAZY:
        check_lazy(specs)
    for name, prog, outs, nw, sch in specs:
        sys.stderr.write("%s: %d products, rounds %s (nw %d), %d slots\n" % (
            name, len(prog.prods), [sum(i is not None for i in r) for r in sch["rounds"]], nw, sch["nslots"]))
    sys.stdout.write("\n".join(emit(specs)) + "\n")
