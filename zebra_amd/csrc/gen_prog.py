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


def prod_costs(prog):
    out = []
    for L, R, kind in prog.prods:
        c = _form_instr(L, True) + (0 if kind == K_SQR else _form_instr(R, False))
        out.append(PROD_CLK[kind] + 4.4 * c)
    return out


def balance_rounds(sch, costs, nw):
    """order each round's products over the waves so that the two waves of a SIMD (w, w + nw/2)
    carry a heavy and a light product; returns the modelled time (sum over rounds of the
    busiest SIMD's load)"""
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


def schedule(prog, outs, nw, search=0, max_slots=None, shift=1, partial=False, cost=False):
    """list-schedule products into rounds of <= nw; allocate LDS slots with reuse.
    search > 0: also try that many seeded random tie-breaks among ready products and keep the
    schedule with the fewest rounds whose slots fit max_slots (then the fewest slots).
    shift 0: a slot may be rewritten in the round of its last read (the engine then puts a
    barrier between a round's operand reads and its writes: ProgInfo.rb). partial: the random
    candidates may also take fewer than nw ready products in a round (shorter live ranges)."""
    best = _schedule(prog, outs, nw, None, 0, shift)
    if cost:
        costs = prod_costs(prog)
        best["time"] = balance_rounds(best, costs, nw)
    if search:
        rng = random.Random(20260101)
        for t in range(search):
            slacks = [0.5, 1.5, 3, 6, 12] if partial else [0.5, 1.5, 3, 6]
            cand = _schedule(prog, outs, nw, rng, rng.choice(slacks), shift, partial)
            fits = max_slots is None or cand["nslots"] <= max_slots
            bfits = max_slots is None or best["nslots"] <= max_slots
            if cost:  # modelled time (SIMD-balanced rounds) instead of the round count
                cand["time"] = balance_rounds(cand, costs, nw)
                key = (not fits, cand["time"], cand["nslots"])
                bkey = (not bfits, best["time"], best["nslots"])
            else:
                key = (not fits, len(cand["rounds"]), cand["nslots"])
                bkey = (not bfits, len(best["rounds"]), best["nslots"])
            if key < bkey:
                best = cand
    return best


def _schedule(prog, outs, nw, rng, slack, shift=1, partial=False):
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
    assert all(j not in prog.keep for j in range(len(outs)) if j < nin) or prog.name in ("dbl", "add")
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


def emit(specs):
    out = ["// GENERATED by zebra_amd/csrc/gen_prog.py -- do not edit.", "#pragma once",
           "// included by zg_prog.h (needs AtomSpace and the Fq2 helpers)", "namespace zg {"]
    prod_cases, out_cases = [], []
    infos, sched = [], []
    gk, go = 0, 0
    for name, prog, outs, nw, sch in specs:
        nin = len(prog.inputs)
        # products
        for i, (L, R, kind) in enumerate(prog.prods):
            s = sch["slot"]
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
            prod_cases.append("  case %d: x = %s; y = %s; dst = %d; return %d;  // %s p%d round %d%s" % (
                gk + i, x, y, dst, kind, name, i, sch["rnd"][i], " -> HBM output %d" % d[1] if isinstance(d, tuple) else ""))
        for j, f in enumerate(outs):
            if j in sch.get("sinks", {}).values():
                out_cases.append("  case %d: return f2_zero();  // %s out %d: stored by its product" % (go + j, name, j))
            else:
                out_cases.append("  case %d: return %s;  // %s out %d" % (go + j, form_code(f, sch["slot"], False),
                                                                        name, j))
        off = len(sched)
        for pick in sch["rounds"]:
            sched.extend([-1 if i is None else i for i in pick] + [-1] * (nw - len(pick)))
        infos.append((name, nin, len(prog.prods), len(outs), len(sch["rounds"]), nw, off, gk, go, sch["nslots"],
                      sch["rb"]))
        gk += len(prog.prods)
        go += len(outs)
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
                         ("FCHAIN", max(i[9] for i in infos if i[0] in ("msq", "m", "mmsq", "mm")))):
        out.append("#define ZG_%s_SLOTS %d" % (name, nslots))
    out.append("// operands of global product gk; returns the product kind (f2_mul_kind)")
    out.append("__device__ __forceinline__ int prog_operands(int gk, const AtomSpace& at, Fq2& x, Fq2& y, int& dst) {")
    out.append("  switch (gk) {")
    out.extend(prod_cases)
    out.append("  default: x = y = f2_zero(); dst = 0; return 0;")
    out.append("  }")
    out.append("}")
    out.append("__device__ __forceinline__ Fq2 prog_output(int go, const AtomSpace& at) {")
    out.append("  switch (go) {")
    out.extend(out_cases)
    out.append("  default: return f2_zero();")
    out.append("  }")
    out.append("}")
    out.append("}  // namespace zg")
    return out


SINK_BASE = 64
NW_LINES = 4   # one wave per SIMD; 13 slots (78 KB) so that two blocks share a CU
NW_FCHAIN = 8
LINES_MAX_SLOTS = 13


def build_all():
    specs = []
    for fn, nw in ((prog_dbl, NW_LINES), (prog_add, NW_LINES), (prog_msq, NW_FCHAIN), (prog_m, NW_FCHAIN),
                   (prog_mmsq, NW_FCHAIN), (prog_mm, NW_FCHAIN)):
        prog, outs = fn()
        # the two-proof programs must fit the one-proof f-chain's LDS (25 slots x 6 KB)
        if fn in (prog_mmsq, prog_mm):
            sch = schedule(prog, outs, nw, 3000, 25, cost=True)
        elif fn in (prog_dbl, prog_add):
            sch = schedule(prog, outs, nw, 6000, LINES_MAX_SLOTS, shift=0, partial=True)
            assert sch["nslots"] <= LINES_MAX_SLOTS, (prog.name, sch["nslots"])
        else:
            sch = schedule(prog, outs, nw)
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
    specs = build_all()
    selfcheck(specs)
    for name, prog, outs, nw, sch in specs:
        sys.stderr.write("%s: %d products, rounds %s (nw %d), %d slots\n" % (
            name, len(prog.prods), [sum(i is not None for i in r) for r in sch["rounds"]], nw, sch["nslots"]))
    sys.stdout.write("\n".join(emit(specs)) + "\n")
