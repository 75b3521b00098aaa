#!/usr/bin/env python3
"""Generate zg_fips.h: the gfx950 Montgomery product for Fq (12 x 32-bit limbs), Finely
Integrated Product Scanning, as one inline-asm statement per column group. Build tooling.

Every 32x32 product is one v_mad_u64_u32 into the 64-bit {lo, mid} column accumulator; its
carry-out (an SGPR-pair lane mask) feeds one v_addc_co_u32 into the high word. hipcc pads
every inline-asm statement boundary with a wait state, so the round-1 form (one statement per
instruction) paid ~250 s_nop per product. Here a whole column is one statement and the carry
masks alternate between two SGPR pairs so that each v_addc_co_u32 sits one instruction after
the v_mad_u64_u32 whose carry it consumes (the same one-state spacing the round-1 form had
from the boundary pad):  mad_1 mad_2 addc_1 mad_3 addc_2 ... mad_n addc_(n-1) addc_n.

    python zebra_amd/csrc/gen_fips.py > zebra_amd/csrc/zg_fips.h
"""
import sys

N = 12


def column(prods, tag):
    """asm statement accumulating prods = [(x_operand, y_operand)] into (lm, h)."""
    ins = []
    opnames = {}

    def op(expr, cons):
        if expr not in opnames:
            opnames[expr] = "%s%d" % (cons[0] if cons != "s" else "k", len(opnames))
            ins.append((opnames[expr], cons, expr))
        return "%[" + opnames[expr] + "]"
    text = []
    n = len(prods)
    for k, (x, y) in enumerate(prods):
        c = "%[c0]" if k % 2 == 0 else "%[c1]"
        text.append("v_mad_u64_u32 %%[lm], %s, %s, %s, %%[lm]" % (c, op(x, "v"), op(y, "s" if y.startswith(("FQ_P", "FR_R", "BQ_P")) else "v")))
        if k >= 1:
            cp = "%[c0]" if (k - 1) % 2 == 0 else "%[c1]"
            text.append("v_addc_co_u32 %%[h], vcc, 0, %%[h], %s" % cp)
    if n == 1:
        text.append("s_nop 0")
    cl = "%[c0]" if (n - 1) % 2 == 0 else "%[c1]"
    text.append("v_addc_co_u32 %%[h], vcc, 0, %%[h], %s" % cl)
    body = "\\n\\t".join(text)
    inputs = ", ".join('[%s] "%s"(%s)' % (nm, cons, expr) for nm, cons, expr in ins)
    return ('  asm volatile("%s"\n               : [lm] "+v"(lm), [h] "+v"(h), [c0] "=&s"(c0), [c1] "=&s"(c1)\n'
            '               : %s\n               : "vcc");  // %s' % (body, inputs, tag))


# ---------------------------------------------------------------- add / sub carry chains
# An Fq op is a few carry chains over 12 limbs plus per-limb selects. Instructions:
#   (text, reads_carry, writes_carry, chain_id, seq)   operands as %[name]
# The scheduler interleaves the chains of one statement so that no instruction reads a carry
# mask written by the instruction right before it (one wait state, as above), inserting
# s_nop 0 only when nothing else is ready.
def op_add(tag, r, a, b):
    """r = (a + b) mod p: s = a + b ; d = s - p ; r = borrow ? s : d"""
    ins = []
    for i in range(N):
        x = "v_add_co_u32 %%[%ss%d], %%[%sk0], %s, %s" % (tag, i, tag, a(i), b(i)) if i == 0 else \
            "v_addc_co_u32 %%[%ss%d], %%[%sk0], %s, %s, %%[%sk0]" % (tag, i, tag, a(i), b(i), tag)
        ins.append((x, None if i == 0 else tag + "k0", tag + "k0", tag + "A", i, []))
    for i in range(N):
        x = "v_sub_co_u32 %s, %%[%sk1], %%[%ss%d], %%[p%d]" % (r(i), tag, tag, i, i) if i == 0 else \
            "v_subb_co_u32 %s, %%[%sk1], %%[%ss%d], %%[p%d], %%[%sk1]" % (r(i), tag, tag, i, i, tag)
        ins.append((x, None if i == 0 else tag + "k1", tag + "k1", tag + "B", i, []))
    for i in range(N):
        ins.append(("v_cndmask_b32 %s, %s, %%[%ss%d], %%[%sk1]" % (r(i), r(i), tag, i, tag), tag + "k1", None,
                    tag + "C", i, ["B%d" % (N - 1)]))
    return ins, ["%ss%d" % (tag, i) for i in range(N)], [tag + "k0", tag + "k1"]


def op_sub(tag, r, a, b):
    """r = (a - b) mod p: d = a - b ; e = d + p ; r = borrow ? e : d"""
    ins = []
    for i in range(N):
        x = "v_sub_co_u32 %s, %%[%sk0], %s, %s" % (r(i), tag, a(i), b(i)) if i == 0 else \
            "v_subb_co_u32 %s, %%[%sk0], %s, %s, %%[%sk0]" % (r(i), tag, a(i), b(i), tag)
        ins.append((x, None if i == 0 else tag + "k0", tag + "k0", tag + "A", i, []))
    for i in range(N):
        x = "v_add_co_u32 %%[%se%d], %%[%sk1], %s, %%[p%d]" % (tag, i, tag, r(i), i) if i == 0 else \
            "v_addc_co_u32 %%[%se%d], %%[%sk1], %s, %%[p%d], %%[%sk1]" % (tag, i, tag, r(i), i, tag)
        ins.append((x, None if i == 0 else tag + "k1", tag + "k1", tag + "B", i, []))
    for i in range(N):
        ins.append(("v_cndmask_b32 %s, %s, %%[%se%d], %%[%sk0]" % (r(i), r(i), tag, i, tag), tag + "k0", None,
                    tag + "C", i, ["B%d" % i, "A%d" % (N - 1)]))
    return ins, ["%se%d" % (tag, i) for i in range(N)], [tag + "k0", tag + "k1"]


def op_lzadd(tag, r, a, b):
    """r = a + b (no reduction)"""
    ins = []
    for i in range(N):
        x = "v_add_co_u32 %s, %%[%sk0], %s, %s" % (r(i), tag, a(i), b(i)) if i == 0 else \
            "v_addc_co_u32 %s, %%[%sk0], %s, %s, %%[%sk0]" % (r(i), tag, a(i), b(i), tag)
        ins.append((x, None if i == 0 else tag + "k0", tag + "k0", tag + "A", i, []))
    return ins, [], [tag + "k0"]


def op_lzsub(tag, r, a, b):
    """r = a + (p - b) (no reduction)"""
    ins = []
    for i in range(N):
        x = "v_sub_co_u32 %%[%sd%d], %%[%sk0], %%[p%d], %s" % (tag, i, tag, i, b(i)) if i == 0 else \
            "v_subb_co_u32 %%[%sd%d], %%[%sk0], %%[p%d], %s, %%[%sk0]" % (tag, i, tag, i, b(i), tag)
        ins.append((x, None if i == 0 else tag + "k0", tag + "k0", tag + "A", i, []))
    for i in range(N):
        x = "v_add_co_u32 %s, %%[%sk1], %s, %%[%sd%d]" % (r(i), tag, a(i), tag, i) if i == 0 else \
            "v_addc_co_u32 %s, %%[%sk1], %s, %%[%sd%d], %%[%sk1]" % (r(i), tag, a(i), tag, i, tag)
        ins.append((x, None if i == 0 else tag + "k1", tag + "k1", tag + "B", i, []))
    return ins, ["%sd%d" % (tag, i) for i in range(N)], [tag + "k0", tag + "k1"]


def op_psub(tag, r, a, b):
    """r = a - b (no reduction; the caller guarantees a >= b)"""
    ins = []
    for i in range(N):
        x = "v_sub_co_u32 %s, %%[%sk0], %s, %s" % (r(i), tag, a(i), b(i)) if i == 0 else \
            "v_subb_co_u32 %s, %%[%sk0], %s, %s, %%[%sk0]" % (r(i), tag, a(i), b(i), tag)
        ins.append((x, None if i == 0 else tag + "k0", tag + "k0", tag + "A", i, []))
    return ins, [], [tag + "k0"]


OPS = {"add": op_add, "sub": op_sub, "lzadd": op_lzadd, "lzsub": op_lzsub, "psub": op_psub}


def schedule_chains(ops):
    """ops: list of (tag, instruction list). Dependencies: an instruction (chain X, limb i) needs
    (X, i-1) and the listed extra deps ('B5' = this op's chain B limb 5); a carry read must not
    directly follow its carry write."""
    pending = []
    for tag, ins in ops:
        for (txt, rc, wc, chain, i, deps) in ins:
            d = set()
            if i > 0:
                d.add((chain, i - 1))
            for dep in deps:
                d.add((tag + dep[0], int(dep[1:])))
            # chain B of add/sub/lzsub reads chain A's limb i
            if chain.endswith("B"):
                d.add((tag + "A", i))
            pending.append({"txt": txt, "rc": rc, "wc": wc, "id": (chain, i), "deps": d, "tag": tag})
    done, out, last_wc = set(), [], None
    while pending:
        left = {}
        for ins in pending:
            left[ins["tag"]] = left.get(ins["tag"], 0) + 1
        pick, best = None, -1
        for k, ins in enumerate(pending):  # ready, hazard-free, from the op with the most work left
            if ins["deps"] <= done and not (ins["rc"] is not None and ins["rc"] == last_wc):
                if left[ins["tag"]] > best:
                    pick, best = k, left[ins["tag"]]
        if pick is None:
            out.append("s_nop 0")
            last_wc = None
            continue
        ins = pending.pop(pick)
        out.append(ins["txt"])
        done.add(ins["id"])
        last_wc = ins["wc"]
    return out


def fq_ops_fn(name, kinds):
    """a device function computing len(kinds) independent Fq ops in one asm statement.
    Op j: r_j = kinds[j](a_j, b_j)."""
    ops, temps, carries = [], [], []
    for j, kd in enumerate(kinds):
        tag = "o%d" % j
        ins, tmp, car = OPS[kd](tag, lambda i, j=j: "%%[r%d_%d]" % (j, i), lambda i, j=j: "%%[a%d_%d]" % (j, i),
                                lambda i, j=j: "%%[b%d_%d]" % (j, i))
        ops.append((tag, ins))
        temps += tmp
        carries += car
    text = schedule_chains(ops)
    nops = sum(1 for t in text if t == "s_nop 0")
    args = ", ".join("uint32_t* r%d, const uint32_t* a%d, const uint32_t* b%d" % (j, j, j) for j in range(len(kinds)))
    outs = ['[r%d_%d] "=&v"(r%d[%d])' % (j, i, j, i) for j in range(len(kinds)) for i in range(N)]
    outs += ['[%s] "=&v"(tmp[%d])' % (t, k) for k, t in enumerate(temps)]
    outs += ['[%s] "=&s"(car[%d])' % (c, k) for k, c in enumerate(carries)]
    ins = ['[a%d_%d] "v"(a%d[%d])' % (j, i, j, i) for j in range(len(kinds)) for i in range(N)]
    ins += ['[b%d_%d] "v"(b%d[%d])' % (j, i, j, i) for j in range(len(kinds)) for i in range(N)]
    ins += ['[p%d] "v"(FQ_P[%d])' % (i, i) for i in range(N)]
    lines = ["// %s: %s (%d instructions, %d s_nop)" % (name, ", ".join(kinds), len(text) - nops, nops),
             "__device__ __forceinline__ void %s(%s) {" % (name, args),
             "  uint32_t tmp[%d];" % max(1, len(temps)), "  uint64_t car[%d];" % len(carries),
             # not volatile: a pure function of its operands (carries in explicit SGPR outputs, no
             # implicit vcc), so the compiler may issue the LDS loads of a lazy form ahead of it
             '  asm("%s"' % "\\n\\t".join(text),
             "               : " + ", ".join(outs),
             "               : " + ", ".join(ins) + ");", "}"]
    return lines


FQ_FNS = [("fqa_add", ["add"]), ("fqa_sub", ["sub"]), ("fqa_lzadd", ["lzadd"]), ("fqa_lzsub", ["lzsub"]),
          ("f2a_add", ["add", "add"]), ("f2a_sub", ["sub", "sub"]), ("f2a_lzadd", ["lzadd", "lzadd"]),
          ("f2a_lzsub", ["lzsub", "lzsub"]), ("f2a_sub_add", ["sub", "add"]), ("f2a_lzadd_lzsub", ["lzadd", "lzsub"]),
          # plain (unreduced) accumulation steps of the staged engine's lazy operand forms
          ("f2p_as", ["lzadd", "psub"]), ("f2p_sa", ["psub", "lzadd"]), ("f2p_ss", ["psub", "psub"]), ("fqp_sub", ["psub"])]


def gen_mul(name, n, pname, inv, rinv, bound, tbound):
    """the FIPS Montgomery product over n limbs (modulus pname, -p^-1 mod 2^32 = inv)"""
    out = ["// r = a * b * %s mod p ; a * b < 2^%d p (e.g. %s)  ->  r < p" % (rinv, 32 * n, bound),
           "__device__ __forceinline__ void %s(uint32_t* r, const uint32_t* a, const uint32_t* b) {" % name,
           "  uint32_t m[%d], t[%d];" % (n, n), "  uint64_t lm = 0, c0, c1;", "  uint32_t h = 0;"]
    for i in range(n):
        prods = [("a[%d]" % j, "b[%d]" % (i - j)) for j in range(i + 1)]
        prods += [("m[%d]" % j, "%s[%d]" % (pname, i - j)) for j in range(i)]
        out.append(column(prods, "column %d: a b and m p products" % i))
        out.append("  m[%d] = (uint32_t)lm * %s;" % (i, inv))
        out.append(column([("m[%d]" % i, "%s[0]" % pname)], "column %d: m_%d p_0" % (i, i)))
        out.append("  lm = (lm >> 32) | ((uint64_t)h << 32);")
        out.append("  h = 0;")
    for i in range(n, 2 * n - 1):
        prods = [("a[%d]" % j, "b[%d]" % (i - j)) for j in range(i - n + 1, n)]
        prods += [("m[%d]" % j, "%s[%d]" % (pname, i - j)) for j in range(i - n + 1, n)]
        out.append(column(prods, "column %d" % i))
        out.append("  t[%d] = (uint32_t)lm;" % (i - n))
        out.append("  lm = (lm >> 32) | ((uint64_t)h << 32);")
        out.append("  h = 0;")
    out.append("  t[%d] = (uint32_t)lm;  // %s: no further carry" % (n - 1, tbound))
    out.append("  uint32_t pm[%d];" % n)
    out.append("#pragma unroll")
    out.append("  for (int i = 0; i < %d; i++) pm[i] = %s[i];" % (n, pname))
    out.append("  mp_reduce_once<%d>(r, t, pm);" % n)
    out.append("}")
    return out


def main():
    out = ["// GENERATED by zebra_amd/csrc/gen_fips.py -- do not edit.", "#pragma once"]
    out += gen_mul("fq_mul_fips", 12, "FQ_P", "FQ_INV", "2^-384", "a < 4p, b < 2p", "< 2p < 2^382")
    out.append("")
    # Fr (the Jubjub base field): a, b < r < 2^255, so a b < 2^256 r and t < 2r < 2^256
    out += gen_mul("fr_mul_fips", 8, "FR_R", "FR_INV", "2^-256", "a, b < r", "< 2r < 2^256")
    out.append("")
    # BN254 Fq (PGHR13): a, b < p < 2^254
    out += gen_mul("bq_mul_fips", 8, "BQ_P", "BQ_INV", "2^-256", "a, b < p", "< 2p < 2^255")
    out.append("")
    # ---- lazy-reduction building blocks: the 24-limb product and the Montgomery reduction of a
    # 24-limb value, the same column statements split in two (an Fq2 Karatsuba product reduces
    # twice instead of three times: zg_prog.h f2_mul_kind)
    out += ["// t = a * b (24 limbs, no reduction)",
            "__device__ __forceinline__ void fq_mul_wide(uint32_t* t, const uint32_t* a, const uint32_t* b) {",
            "  uint64_t lm = 0, c0, c1;", "  uint32_t h = 0;"]
    for i in range(2 * N - 1):
        prods = [("a[%d]" % j, "b[%d]" % (i - j)) for j in range(max(0, i - N + 1), min(i, N - 1) + 1)]
        out.append(column(prods, "column %d" % i))
        out.append("  t[%d] = (uint32_t)lm;" % i)
        out.append("  lm = (lm >> 32) | ((uint64_t)h << 32);")
        out.append("  h = 0;")
    out.append("  t[%d] = (uint32_t)lm;" % (2 * N - 1))
    out.append("}")
    out.append("")
    out += ["// r = t * 2^-384 mod p for t < 2^384 p (24 limbs)  ->  r < p",
            "__device__ __forceinline__ void fq_redc_wide(uint32_t* r, const uint32_t* t) {",
            "  uint32_t m[12], u[12];", "  uint64_t lm = 0, c0, c1;", "  uint32_t h = 0;"]
    for i in range(N):
        out.append("  lm += t[%d];  // lm < 2^38 here: no overflow" % i)
        prods = [("m[%d]" % j, "FQ_P[%d]" % (i - j)) for j in range(i)]
        if prods:
            out.append(column(prods, "column %d: m p products" % i))
        out.append("  m[%d] = (uint32_t)lm * FQ_INV;" % i)
        out.append(column([("m[%d]" % i, "FQ_P[0]")], "column %d: m_%d p_0" % (i, i)))
        out.append("  lm = (lm >> 32) | ((uint64_t)h << 32);")
        out.append("  h = 0;")
    for i in range(N, 2 * N - 1):
        out.append("  lm += t[%d];" % i)
        prods = [("m[%d]" % j, "FQ_P[%d]" % (i - j)) for j in range(i - N + 1, N)]
        out.append(column(prods, "column %d" % i))
        out.append("  u[%d] = (uint32_t)lm;" % (i - N))
        out.append("  lm = (lm >> 32) | ((uint64_t)h << 32);")
        out.append("  h = 0;")
    out.append("  lm += t[%d];" % (2 * N - 1))
    out.append("  u[11] = (uint32_t)lm;  // < 2p < 2^382: no further carry")
    out.append("  uint32_t pm[12];")
    out.append("#pragma unroll")
    out.append("  for (int i = 0; i < 12; i++) pm[i] = FQ_P[i];")
    out.append("  mp_reduce_once<12>(r, u, pm);")
    out.append("}")
    out.append("")
    out.append("// ---- Fq add / sub carry chains, one asm statement each (interleaved chains, see above)")
    for name, kinds in FQ_FNS:
        out += fq_ops_fn(name, kinds)
    sys.stdout.write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
