#!/usr/bin/env python3
"""Generate zg_fq29_gen.h: straight-line Fq Montgomery products in 29-bit digits. Build tooling.

Storage stays 12 x 32-bit words in Montgomery form R = 2^384. A product splits its operands
into 14 digits of 29 bits (v_alignbit + v_and), so every digit product is < 2^58 and a whole
column -- up to 56 a*b, a'*b' and m*p terms -- fits one 64-bit accumulator: ONE carry-free
v_mad_u64_u32 per digit product, against v_mad_u64_u32 + v_addc_co_u32 per 32x32 product in
the word form (gen_fips.py). The reduction is finely integrated (FIPS) and mixed-radix: 13
digits of 29 bits and a last one of 7 bits divide by exactly 2^384 (377 + 7); the 7-bit tail
is absorbed by the bit offsets of the final repacking into 32-bit words.

The code is plain C (no inline asm): the same text runs on the CPU in tests/native, and on
gfx950 the compiler maps `acc += (uint64_t)x * y` to v_mad_u64_u32. Everything is unrolled
here, with constant digit indices, so no array ever needs indexed register access.

    python zebra_amd/csrc/gen_fq29.py > zebra_amd/csrc/zg_fq29_gen.h
"""
import sys

P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
D = 14          # digits
W = 29          # digit bits
MASK = (1 << W) - 1
P29 = [(P >> (W * i)) & MASK for i in range(D)]
PINV = (-pow(P, -1, 1 << W)) % (1 << W)
# 2p with borrowed digits: digits 0..12 >= 2^29 - 1, so (2p - y) digit-wise is >= 0 for y < p
_q = [((2 * P) >> (W * i)) & MASK for i in range(D)]
P2B = [_q[i] + ((1 << W) if i < D - 1 else 0) - (1 if i > 0 else 0) for i in range(D)]
assert sum(b << (W * i) for i, b in enumerate(P2B)) == 2 * P and all(b >= MASK for b in P2B[:D - 1])
assert P2B[D - 1] >= (P >> (W * (D - 1)))


KP_MAX = 12


def borrowed(k):
    """k p as 14 digits with digits 0..12 raised by 2^29 (borrowed from the next digit)"""
    q = [((k * P) >> (W * i)) & MASK for i in range(D)]
    if k == 0:
        return q
    b = [q[i] + ((1 << W) if i < D - 1 else 0) - (1 if i > 0 else 0) for i in range(D)]
    assert sum(x << (W * i) for i, x in enumerate(b)) == k * P and all(x >= MASK for x in b[:D - 1])
    # dominance: any y < (k - 1) p has top digit <= ((k - 1) p - 1) >> 377 <= b[13]
    if k >= 2:
        assert ((k - 1) * P) >> (W * (D - 1)) <= b[D - 1], k
    return b


def split(dst, src):
    out = []
    for L in range(D):
        b = W * L
        w, o = b >> 5, b & 31
        if o + W <= 32:
            e = "%s[%d]" % (src, w) if o == 0 else "(%s[%d] >> %d)" % (src, w, o)
            if o + W < 32:
                e = "%s & FQ29_MASK" % e
        elif w + 1 < 12:
            e = "zg_alignbit(%s[%d], %s[%d], %d) & FQ29_MASK" % (src, w + 1, src, w, o)
        else:
            e = "%s[%d] >> %d" % (src, w, o)
            out.append("  %s[%d] = %s;" % (dst, L, e))
            out.append("  zg_opaque(%s[%d]);  // narrow top digit: see gen_mont29" % (dst, L))
            continue
        out.append("  %s[%d] = %s;" % (dst, L, e))
    return out


def terms(a, b, k, step=1):
    """digit products of column k of a * b (a, b digit arrays)"""
    return [(a, i, b, k - i) for i in range(D) if 0 <= k - i < D]


def sq_terms(a, a2, k):
    """column k of a^2 with a2 = 2a digit-wise: sum_{i<j} a2_i a_j + a_{k/2}^2"""
    t = [(a2, i, a, k - i) for i in range(D) if i < k - i < D]
    if k % 2 == 0 and k // 2 < D:
        t.append((a, k // 2, a, k // 2))
    return t


def redc(chains, canon=True):
    """chains: list of (out_name, acc_name, column_terms(k) -> list of (x, i, y, j)).
    Emits the interleaved FIPS reduction of every chain; results as 12 words in out_name."""
    out = []
    for (r, a, _) in chains:
        out.append("  uint32_t %s_m[14], %s_u[14];" % (a, a))
        out.append("  uint64_t %s = 0;" % a)
    for k in range(2 * D - 1):
        cols = [(r, a, f(k)) for (r, a, f) in chains]
        n = max(len(t) for _, _, t in cols)
        for q in range(n):  # interleave the chains term by term
            for (r, a, t) in cols:
                if q < len(t):
                    x, i, y, j = t[q]
                    out.append("  %s += (uint64_t)%s[%d] * %s[%d];" % (a, x, i, y, j))
        for j in range(D):
            if j < k and k - j < D:
                for (r, a, _) in cols:
                    out.append("  %s += (uint64_t)%s_m[%d] * 0x%08xu;" % (a, a, j, P29[k - j]))
        for (r, a, _) in cols:
            if k < D - 1:
                out.append("  %s_m[%d] = ((uint32_t)%s * 0x%08xu) & FQ29_MASK;" % (a, k, a, PINV))
            elif k == D - 1:
                out.append("  %s_m[%d] = ((uint32_t)%s * 0x%08xu) & 127u;" % (a, k, a, PINV))
                out.append("  zg_opaque(%s_m[%d]);" % (a, k))
        for (r, a, _) in cols:
            if k <= D - 1:
                out.append("  %s += (uint64_t)%s_m[%d] * 0x%08xu;" % (a, a, k, P29[0]))
            if k >= D - 1:
                out.append("  %s_u[%d] = (uint32_t)%s & FQ29_MASK;" % (a, k - (D - 1), a))
            out.append("  %s >>= 29;" % a)
    # u = (S + m p) / 2^377, low 7 bits zero: r = u >> 7 as words
    for (r, a, _) in chains:
        for w in range(12):
            b = 7 + 32 * w
            L, o = b // W, b % W
            parts = ["(%s_u[%d] >> %d)" % (a, L, o) if o else "%s_u[%d]" % (a, L),
                     "(%s_u[%d] << %d)" % (a, L + 1, W - o)]
            if o + 32 > 2 * W:
                parts.append("(%s_u[%d] << %d)" % (a, L + 2, 2 * W - o))
            tgt = "%s_t[%d]" % (a, w) if canon else "%s[%d]" % (r, w)
            if w == 0 and canon:
                out.append("  uint32_t %s_t[12];" % a)
            out.append("  %s = %s;" % (tgt, " | ".join(parts)))
        if canon:
            out.append("  fq29_canon(%s, %s_t);" % (r, a))
    return out


def redc_full(chains):
    """full-radix FIPS reduction by 2^406 (14 digits of 29 bits): results as 14 normalized digits
    in out_name (digit-resident chains: no split / repack between products)"""
    out = []
    for (r, a, _) in chains:
        out.append("  uint32_t %s_m[14];" % a)
        out.append("  uint64_t %s = 0;" % a)
    for k in range(2 * D - 1):
        cols = [(r, a, f(k)) for (r, a, f) in chains]
        n = max(len(t) for _, _, t in cols)
        for q in range(n):
            for (r, a, t) in cols:
                if q < len(t):
                    x, i, y, j = t[q]
                    out.append("  %s += (uint64_t)%s[%d] * %s[%d];" % (a, x, i, y, j))
        for j in range(D):
            if j < k and k - j < D:
                for (r, a, _) in cols:
                    out.append("  %s += (uint64_t)%s_m[%d] * 0x%08xu;" % (a, a, j, P29[k - j]))
        for (r, a, _) in cols:
            if k < D:
                out.append("  %s_m[%d] = ((uint32_t)%s * 0x%08xu) & FQ29_MASK;" % (a, k, a, PINV))
                out.append("  %s += (uint64_t)%s_m[%d] * 0x%08xu;" % (a, a, k, P29[0]))
            else:
                out.append("  %s[%d] = (uint32_t)%s & FQ29_MASK;" % (r, k - D, a))
            out.append("  %s >>= 29;" % a)
    for (r, a, _) in chains:
        out.append("  %s[13] = (uint32_t)%s;" % (r, a))
    return out


def gen_mont29(name, M, NW, mname, doc_bound):
    """generic r = a b 2^(-32 NW) mod M in 29-bit digits (M < 2^(32 NW - 1)): NW words -> D digits,
    mixed-radix FIPS reduction (D - 1 digits of 29 bits and one of 32 NW - 29 (D - 1)), repack, one
    conditional subtraction. Column bound: D a*b + D m*M terms < 2^58."""
    Dm = -(-32 * NW // W)
    last = 32 * NW - W * (Dm - 1)
    Md = [(M >> (W * i)) & MASK for i in range(Dm)]
    pinv = (-pow(M, -1, 1 << W)) % (1 << W)
    assert 2 * Dm * (1 << 58) < 1 << 64
    out = ["  uint32_t A[%d], B[%d], m[%d], u[%d], t[%d];" % (Dm, Dm, Dm, Dm + 1, NW), "  uint64_t acc = 0;"]
    for L in range(Dm):  # split
        b_ = W * L
        w, o_ = b_ >> 5, b_ & 31
        for (X, src) in (("A", "a"), ("B", "b")):
            if o_ + W <= 32:
                e = "%s[%d]" % (src, w) if o_ == 0 else "(%s[%d] >> %d)" % (src, w, o_)
                if o_ + W < 32:
                    e += " & FQ29_MASK"
            elif w + 1 < NW:
                e = "zg_alignbit(%s[%d], %s[%d], %d) & FQ29_MASK" % (src, w + 1, src, w, o_)
            else:
                e = "%s[%d] >> %d" % (src, w, o_)
            out.append("  %s[%d] = %s;" % (X, L, e))
    # the top digits are narrower than 29 bits; hide their known range from the compiler, whose
    # gfx950 lowering of 64-bit multiply-adds of two operands known to fit 24 bits gave wrong
    # results here (found by tools/mb_fr29.hip: the same C is exact on the host)
    out.append("  zg_opaque(A[%d]); zg_opaque(B[%d]);" % (Dm - 1, Dm - 1))
    for k in range(2 * Dm - 1):
        for i in range(Dm):
            if 0 <= k - i < Dm:
                out.append("  acc += (uint64_t)A[%d] * B[%d];" % (i, k - i))
        for j in range(Dm):
            if j < k and k - j < Dm:
                out.append("  acc += (uint64_t)m[%d] * 0x%08xu;" % (j, Md[k - j]))
        if k < Dm - 1:
            out.append("  m[%d] = ((uint32_t)acc * 0x%08xu) & FQ29_MASK;" % (k, pinv))
        elif k == Dm - 1:
            out.append("  m[%d] = ((uint32_t)acc * 0x%08xu) & 0x%08xu;" % (k, pinv, (1 << last) - 1))
            out.append("  zg_opaque(m[%d]);" % k)
        if k <= Dm - 1:
            out.append("  acc += (uint64_t)m[%d] * 0x%08xu;" % (k, Md[0]))
        if k >= Dm - 1:
            out.append("  u[%d] = (uint32_t)acc & FQ29_MASK;" % (k - (Dm - 1)))
        out.append("  acc >>= 29;")
    out.append("  u[%d] = (uint32_t)acc;  // u = t 2^%d < 2M 2^%d needs a digit more" % (Dm, last, last))
    for w in range(NW):  # r = u >> last as words
        b_ = last + 32 * w
        L, o_ = b_ // W, b_ % W
        parts = ["(u[%d] >> %d)" % (L, o_) if o_ else "u[%d]" % L]
        if L + 1 <= Dm:
            parts.append("(u[%d] << %d)" % (L + 1, W - o_))
        if o_ + 32 > 2 * W and L + 2 <= Dm:
            parts.append("(u[%d] << %d)" % (L + 2, 2 * W - o_))
        out.append("  t[%d] = %s;" % (w, " | ".join(parts)))
    out += ["#if defined(__HIP_DEVICE_COMPILE__)",
            "  uint32_t pm[%d];" % NW,
            "#pragma unroll",
            "  for (int i = 0; i < %d; i++) pm[i] = %s[i];" % (NW, mname),
            "  mp_reduce_once<%d>(r, t, pm);" % NW,
            "#else",
            "  uint32_t d[%d];" % NW, "  uint64_t bo = 0;",
            "  for (int i = 0; i < %d; i++) {" % NW,
            "    const uint64_t x = (uint64_t)t[i] - %s[i] - bo;" % mname,
            "    d[i] = (uint32_t)x;", "    bo = (x >> 63) & 1;", "  }",
            "  for (int i = 0; i < %d; i++) r[i] = bo ? t[i] : d[i];" % NW,
            "#endif"]
    return fn(name, "uint32_t* r, const uint32_t* a, const uint32_t* b", out,
              ["r = a b 2^-%d mod %s in 29-bit digits (%d digits, mixed radix: %d x 29 + %d): %s" % (
                  32 * NW, mname, Dm, Dm - 1, last, doc_bound)])


def fn(name, args, body, doc):
    return ["// " + d for d in doc] + ["ZG_INL void %s(%s) {" % (name, args)] + body + ["}", ""]


def main():
    o = ["// GENERATED by zebra_amd/csrc/gen_fq29.py -- do not edit.", "#pragma once", "namespace zg {", ""]
    o.append("static constexpr uint32_t FQ29_MASK = 0x%08xu;" % MASK)
    o.append("static constexpr uint32_t FQ_2P_B29[14] = {%s};  // 2p, digits 0..12 >= 2^29 - 1" %
             ", ".join("0x%08xu" % x for x in P2B))
    o.append("")
    o += ["ZG_INL uint32_t zg_alignbit(uint32_t hi, uint32_t lo, int s) {",
          "#if defined(__HIP_DEVICE_COMPILE__)",
          "  return __builtin_amdgcn_alignbit(hi, lo, s);",
          "#else",
          "  return (uint32_t)((((uint64_t)hi << 32) | lo) >> s);",
          "#endif",
          "}", ""]
    o += ["// an optimisation barrier: the compiler forgets what it knows about x's range (no instruction)",
          "ZG_INL void zg_opaque(uint32_t& x) {",
          "#if defined(__HIP_DEVICE_COMPILE__)",
          '  asm volatile("" : "+v"(x));',
          "#else",
          "  (void)x;",
          "#endif",
          "}", ""]
    o += ["// r = t >= p ? t - p : t  (t < 2p)",
          "ZG_INL void fq29_canon(uint32_t* r, const uint32_t* t) {",
          "#if defined(__HIP_DEVICE_COMPILE__)",
          "  uint32_t pm[12];",
          "#pragma unroll",
          "  for (int i = 0; i < 12; i++) pm[i] = FQ_P[i];",
          "  mp_reduce_once<12>(r, t, pm);",
          "#else",
          "  uint32_t d[12];",
          "  uint64_t bo = 0;",
          "  for (int i = 0; i < 12; i++) {",
          "    const uint64_t x = (uint64_t)t[i] - FQ_P[i] - bo;",
          "    d[i] = (uint32_t)x;",
          "    bo = (x >> 63) & 1;",
          "  }",
          "  for (int i = 0; i < 12; i++) r[i] = bo ? t[i] : d[i];",
          "#endif",
          "}", ""]

    # Fq product
    body = ["  uint32_t A[14], B[14];"] + split("A", "a") + split("B", "b")
    body += redc([("r", "acc", lambda k: terms("A", "B", k))])
    o += fn("fq29_mul", "uint32_t* r, const uint32_t* a, const uint32_t* b", body,
            ["r = a b 2^-384 mod p; a b < 2^384 p (e.g. a < 4p, b < 2p) -> r < p.",
             "Column bound: 14 a*b + 14 m*p terms < 2^58 each."])
    # Fq square
    body = ["  uint32_t A[14], A2[14];"] + split("A", "a") + ["  A2[%d] = A[%d] << 1;" % (i, i) for i in range(D)]
    body += redc([("r", "acc", lambda k: sq_terms("A", "A2", k))])
    o += fn("fq29_sqr", "uint32_t* r, const uint32_t* a", body,
            ["r = a^2 2^-384 mod p for a < 2p (a^2 < 2^384 p) -> r < p: 105 digit products, the",
             "off-diagonal ones once with a doubled operand (< 2^59: 7 + 14 terms per column, fine)."])
    # Fq2 product, schoolbook
    body = ["  uint32_t X0[14], X1[14], Y0[14], Y1[14], N1[14];"] + split("X0", "x0") + split("X1", "x1") + \
        split("Y0", "y0") + split("Y1", "y1") + ["  N1[%d] = 0x%08xu - Y1[%d];" % (i, P2B[i], i) for i in range(D)]
    body += redc([("c0", "a0", lambda k: terms("X0", "Y0", k) + terms("X1", "N1", k)),
                  ("c1", "a1", lambda k: terms("X0", "Y1", k) + terms("X1", "Y0", k))])
    o += fn("f2_mul29", "uint32_t* c0, uint32_t* c1, const uint32_t* x0, const uint32_t* x1, const uint32_t* y0, "
            "const uint32_t* y1", body,
            ["Fq2 product, schoolbook in 29-bit digits with two reductions:",
             "  c0 = REDC(x0 y0 + x1 (2p - y1)),  c1 = REDC(x0 y1 + x1 y0)",
             "x lazy (< 2p per coefficient), y canonical: c0's sum < 2p p + 2p 2p = 6p^2 < 2^384 p, so both",
             "results are < p after the conditional subtraction (the contract of f2_mul_kind). Column bound",
             "for c0: 14 terms < 2^58, 14 terms < 2^59 (2p - y1 digits < 2^30), 14 m*p terms: < 2^64."])
    # Fq2 times an Fq
    body = ["  uint32_t X0[14], X1[14], S[14];"] + split("X0", "x0") + split("X1", "x1") + split("S", "s")
    body += redc([("c0", "a0", lambda k: terms("X0", "S", k)), ("c1", "a1", lambda k: terms("X1", "S", k))])
    o += fn("f2_mul_fq29", "uint32_t* c0, uint32_t* c1, const uint32_t* x0, const uint32_t* x1, const uint32_t* s",
            body, ["(x0 s, x1 s) for x lazy (< 2p), s canonical -> canonical"])
    # Fq2 square
    body = ["  uint32_t X0[14], X1[14], D[14], S[14], T[14];"] + split("X0", "x0") + split("X1", "x1") + \
        split("D", "dif") + ["  S[%d] = X0[%d] + X1[%d];\n  T[%d] = X1[%d] << 1;" % (i, i, i, i, i) for i in range(D)]
    body += redc([("c0", "a0", lambda k: terms("S", "D", k)), ("c1", "a1", lambda k: terms("X0", "T", k))])
    o += fn("f2_sqr29", "uint32_t* c0, uint32_t* c1, const uint32_t* x0, const uint32_t* x1, const uint32_t* dif",
            body, ["x^2 for canonical x given dif = x0 - x1 mod p: c0 = (x0 + x1) dif, c1 = x0 (2 x1). The sum and",
                   "the doubled digits are formed digit-wise (< 2^30). Column bound: 14 terms < 2^59 + 14 m*p."])
    # ---- digit-resident products (Montgomery R' = 2^406, 14 normalized digits in and out): chains
    # of products (exponentiations) skip the split / repack / canonicalisation of every product
    RP = 2 ** (D * W)
    kin = (2 ** (2 * D * W - 384)) % P    # a R -> a R' : REDC'(a R * kin)
    kout = (2 ** 384) % P                  # a R' -> a R : REDC'(a R' * kout)
    o.append("static constexpr uint32_t FQ29D_KIN[14] = {%s};  // 2^428 mod p: R -> R' = 2^406" %
             ", ".join("0x%08xu" % ((kin >> (W * i)) & MASK) for i in range(D)))
    o.append("static constexpr uint32_t FQ29D_KOUT[14] = {%s};  // 2^384 mod p: R' -> R" %
             ", ".join("0x%08xu" % ((kout >> (W * i)) & MASK) for i in range(D)))
    o.append("")
    body = redc_full([("r", "acc", lambda k: terms("a", "b", k))])
    o += fn("fq29d_mul", "uint32_t* r, const uint32_t* a, const uint32_t* b", body,
            ["r = a b 2^-406 mod p in digits: a, b < 2p (normalized digits) -> r < 2p (normalized).",
             "r may alias neither a nor b."])
    body = ["  uint32_t A2[14];"] + ["  A2[%d] = a[%d] << 1;" % (i, i) for i in range(D)]
    body += redc_full([("r", "acc", lambda k: sq_terms("a", "A2", k))])
    o += fn("fq29d_sqr", "uint32_t* r, const uint32_t* a", body,
            ["r = a^2 2^-406 mod p in digits (a < 2p) -> r < 2p; r may not alias a."])
    body = ["  uint32_t A[14];"] + split("A", "a")
    body += redc_full([("r", "acc", lambda k: terms("A", "FQ29D_KIN", k))])
    o += fn("fq29d_from_mont", "uint32_t* r, const uint32_t* a",
            body, ["12-word a R (any a < 2^384) -> 14-digit a R' (< 2p)"])
    body = ["  uint32_t u[14], t[12];"] + redc_full([("u", "acc", lambda k: terms("a", "FQ29D_KOUT", k))])
    for w in range(12):
        b_ = 32 * w
        L, o_ = b_ // W, b_ % W
        parts = ["(u[%d] >> %d)" % (L, o_) if o_ else "u[%d]" % L, "(u[%d] << %d)" % (L + 1, W - o_)]
        if o_ + 32 > 2 * W:
            parts.append("(u[%d] << %d)" % (L + 2, 2 * W - o_))
        body.append("  t[%d] = %s;" % (w, " | ".join(parts)))
    body.append("  fq29_canon(r, t);")
    o += fn("fq29d_to_mont", "uint32_t* r, const uint32_t* a", body,
            ["14-digit a R' (< 2p) -> canonical 12-word a R"])

    # ---- the 256-bit moduli: BLS12-381 Fr (Jubjub base field) and BN254 Fq (PGHR13)
    R_BLS = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
    P_BN = 0x30644e72e131a029b85045b68181585d97816a916871ca8d3c208c16d87cfd47
    o += gen_mont29("fr29_mul", R_BLS, 8, "FR_R", "a, b < r -> r' < r")
    o += gen_mont29("bq29_mul", P_BN, 8, "BQ_P", "a, b < p -> r < p")

    # ---- raw-output forms for the staged engine's lazy operands (zg_prog.h f2_mul_kind): the
    # caller bounds the column sum S < M p^2 and finishes the 12-word result t < S / 2^384 + p
    # (fq_finish: conditional subtractions or a quotient estimate)
    o.append("#define ZG_KP_MAX %d" % KP_MAX)
    o.append("// k p (12 words) and k p with borrowed 29-bit digits (digits 0..12 >= 2^29 - 1, top digit")
    o.append("// >= the top digit of any y <= (k - 1) p), k = 0..%d" % KP_MAX)
    o.append("static constexpr uint32_t FQ_KP[%d][12] = {%s};" % (KP_MAX + 1, ", ".join(
        "{%s}" % ", ".join("0x%08xu" % ((k * P >> (32 * i)) & 0xffffffff) for i in range(12)) for k in range(KP_MAX + 1))))
    o.append("static constexpr uint32_t FQ_KP_B29[%d][14] = {%s};" % (KP_MAX + 1, ", ".join(
        "{%s}" % ", ".join("0x%08xu" % x for x in borrowed(k)) for k in range(KP_MAX + 1))))
    o.append("")
    body = ["  uint32_t X0[14], X1[14], Y0[14], Y1[14], N1[14];"] + split("X0", "x0") + split("X1", "x1") + \
        split("Y0", "y0") + split("Y1", "y1") + ["  N1[%d] = off[%d] - Y1[%d];" % (i, i, i) for i in range(D)]
    body += redc([("c0", "a0", lambda k: terms("X0", "Y0", k) + terms("X1", "N1", k)),
                  ("c1", "a1", lambda k: terms("X0", "Y1", k) + terms("X1", "Y0", k))], canon=False)
    o += fn("f2_mul29_raw", "uint32_t* c0, uint32_t* c1, const uint32_t* x0, const uint32_t* x1, const uint32_t* y0, "
            "const uint32_t* y1, const uint32_t* off", body,
            ["f2_mul29 with y1 <= (k - 1) p and off = FQ_KP_B29[k]: c0 = REDC(x0 y0 + x1 (k p - y1)),",
             "c1 = REDC(x0 y1 + x1 y0), unreduced (< S / 2^384 + p). x, y < 2^384 (digits < 2^29)."])
    body = ["  uint32_t X0[14], X1[14], S[14];"] + split("X0", "x0") + split("X1", "x1") + split("S", "s")
    body += redc([("c0", "a0", lambda k: terms("X0", "S", k)), ("c1", "a1", lambda k: terms("X1", "S", k))],
                 canon=False)
    o += fn("f2_mul_fq29_raw", "uint32_t* c0, uint32_t* c1, const uint32_t* x0, const uint32_t* x1, const uint32_t* s",
            body, ["(x0 s, x1 s), unreduced"])
    body = ["  uint32_t X0[14], X1[14], D[14], S[14], T[14];"] + split("X0", "x0") + split("X1", "x1") + \
        split("D", "dif") + ["  S[%d] = X0[%d] + X1[%d];\n  T[%d] = X1[%d] << 1;" % (i, i, i, i, i) for i in range(D)]
    body += redc([("c0", "a0", lambda k: terms("S", "D", k)), ("c1", "a1", lambda k: terms("X0", "T", k))],
                 canon=False)
    o += fn("f2_sqr29_raw", "uint32_t* c0, uint32_t* c1, const uint32_t* x0, const uint32_t* x1, const uint32_t* dif",
            body, ["x^2 with dif = x0 - x1 + k p (any x < 2^384): c0 = (x0 + x1) dif, c1 = x0 (2 x1), unreduced"])
    o.append("}  // namespace zg")
    sys.stdout.write("\n".join(o) + "\n")


if __name__ == "__main__":
    main()
