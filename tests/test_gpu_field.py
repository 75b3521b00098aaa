"""GPU tier: the device's 29-bit-digit Montgomery products against exact integer arithmetic.

zg_debug_field_mul runs the same generated products every kernel uses (zg_fq29_gen.h: fq29_mul,
fq29_sqr, f2_mul29, fr29_mul, bq29_mul), one per lane. Operands: random canonical values plus
edge values chosen to stress the digit split -- 0, 1, the top of the range (p - 1, and 2p - 1
where the contract allows lazy operands), values whose 29-bit digits are all at their maximum,
and values whose narrow top digit is at its maximum (the operands whose known 24-bit range the
gfx950 lowering mishandled before the zg_opaque barrier; round 2's
tools/mb_fr29.hip isolated it). Every product must equal a b 2^-k mod m exactly."""
import random

import pytest

from oracle import bls12_381 as BLS, bn254 as BN

pytestmark = pytest.mark.gpu

FIELDS = {   # field id -> (modulus, Montgomery bits, operand bytes, lazy bound of a)
    0: (BLS.P, 384, 48, 1),
    1: (BLS.P, 384, 48, 2),
    3: (BLS.R, 256, 32, 1),
    4: (BN.P, 256, 32, 1),
}


def _edges(m, lazy, bits):
    top = m * lazy - 1
    vals = [0, 1, 2, m - 1, m - 2, top, top - 1, m // 2, (m + 1) // 2]
    # all 29-bit digits at their maximum below the bound: 2^(29k) - 1
    k = 29
    while (1 << k) - 1 <= top:
        vals.append((1 << k) - 1)
        k += 29
    # the narrow top digit at its maximum with low digits zero / full
    ndig = (bits + 28) // 29
    hi_shift = 29 * (ndig - 1)
    for low in (0, (1 << hi_shift) - 1):
        for hi in range(top >> hi_shift, max(-1, (top >> hi_shift) - 4), -1):
            v = (hi << hi_shift) | low
            if v <= top:
                vals.append(v)
    # powers of two and their neighbours inside the range
    for j in range(0, bits):
        for v in ((1 << j) - 1, 1 << j, (1 << j) + 1):
            if 0 <= v <= top:
                vals.append(v)
    return sorted(set(vals))


def cases(field):
    """(a, b) operand pairs for a scalar field id: edges x sampled edges, random, near-top"""
    m, bits, w, lazy = FIELDS[field]
    rnd = random.Random(1000 + field)
    ea = _edges(m, lazy, bits)
    eb = _edges(m, 1, bits)
    pairs = [(x, y) for x in ea for y in eb[::max(1, len(eb) // 40)]]
    pairs += [(rnd.randrange(m * lazy), rnd.randrange(m)) for _ in range(8192)]
    # both operands near the top of their digit ranges at once
    pairs += [(m * lazy - 1 - rnd.randrange(1 << 40), m - 1 - rnd.randrange(1 << 40)) for _ in range(1024)]
    return pairs


def fq2_cases():
    p = BLS.P
    rnd = random.Random(77)
    edge_x = [0, 1, p - 1, p, 2 * p - 1, (1 << 377) - 1]
    edge_y = [0, 1, p - 1, (1 << 377) - 1 if (1 << 377) - 1 < p else p - 3]
    xs = [(a, b) for a in edge_x for b in edge_x] + [(rnd.randrange(2 * p), rnd.randrange(2 * p)) for _ in range(2048)]
    ys = [(a, b) for a in edge_y for b in edge_y] + [(rnd.randrange(p), rnd.randrange(p)) for _ in range(2048)]
    return [(xs[i % len(xs)], ys[(7 * i) % len(ys)]) for i in range(max(len(xs), len(ys)))]


def fq2_expected(x, y):
    p = BLS.P
    rinv = pow(1 << 384, -1, p)
    return (((x[0] * y[0] - x[1] * y[1]) * rinv) % p, ((x[0] * y[1] + x[1] * y[0]) * rinv) % p)


def mismatches(field, pairs, got):
    m, bits, w, _ = FIELDS[field]
    rinv = pow(1 << bits, -1, m)
    bad = []
    for (x, y), g in zip(pairs, got):
        want = (x * (x if field == 1 else y) * rinv) % m
        if int.from_bytes(g, "little") != want:
            bad.append((hex(x), hex(y)))
    return bad


def fq2_enc(c):
    return c[0].to_bytes(48, "little") + c[1].to_bytes(48, "little")


@pytest.mark.parametrize("field", sorted(FIELDS))
def test_device_products_exact(field):
    from zebra_amd import zg
    w = FIELDS[field][2]
    pairs = cases(field)
    got = zg.debug_field_mul(field, [x.to_bytes(w, "little") for x, _ in pairs],
                             [y.to_bytes(w, "little") for _, y in pairs])
    bad = mismatches(field, pairs, got)
    assert not bad, (len(bad), bad[:4])


def test_device_fq2_products_exact():
    """f2_mul29: c0 = x0 y0 - x1 y1, c1 = x0 y1 + x1 y0 (times 2^-384), x lazy < 2p, y canonical"""
    from zebra_amd import zg
    pairs = fq2_cases()
    got = zg.debug_field_mul(2, [fq2_enc(x) for x, _ in pairs], [fq2_enc(y) for _, y in pairs])
    for (x, y), g in zip(pairs, got):
        assert (int.from_bytes(g[:48], "little"), int.from_bytes(g[48:], "little")) == fq2_expected(x, y), (x, y)
