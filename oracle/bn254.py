"""ORACLE (test infrastructure only) -- CPU restatement of the BN254 ("alt_bn128") curve as the
reference's PGHR13 path uses it. Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may use it, as the checker.

The curve code lives in the third-party crate `bn` (crypto/Cargo.toml:12, git paritytech/bn, not
vendored in /root/reference); this module restates what the reference's PGHR13 verifier observes
of it (crypto/src/pghr13.rs:1-105, crypto/src/json/pghr13.rs):
  * Fq / Fr: p, r below; Fq::from_slice / Fr: 32 big-endian bytes, rejected when >= modulus
  * Fq2 = Fq[u]/(u^2 + 1); Fq2::from_slice: 64 big-endian bytes read as ONE 512-bit integer
    U = c1 p + c0 (divrem by p, c1 must be < p) -- the zcash `Fq2` blob layout
  * G1: y^2 = x^3 + 3; G2 (D-type twist): y^2 = x^3 + 3 / (9 + u)
  * AffineG1::new: on-curve check; AffineG2::new: on-curve and r Q = O (bn's check_order)
  * G1::from_compressed (33 bytes): prefix 2 -> even y, 3 -> odd y (of the canonical integer)
  * G2::from_compressed (65 bytes): prefix 10 / 11, x = Fq2::from_slice(bytes[1..65]); with the
    512-bit order above, 10 takes the smaller of {y, -y}, 11 the greater (zcash's y_gt flag)
  * pairing: an optimal ate pairing (loop 6u + 2, u = 4965661367192848881, then the two
    Frobenius-twisted steps) and the final exponentiation (p^12 - 1) / r. The reference only
    compares pairing products for equality, which any non-degenerate bilinear pairing decides
    identically, so GT bytes are not part of the contract.

Pinned by crypto/src/pghr13.rs's proof_decode test (the decoded coordinates of a real proof's 8
points, both compressed encodings), its verification / verification2 tests and sprout.rs's
smoky_pghr (valid proofs under res/sprout-verifying-key.json), and the PHGR JoinSplits of mainnet
block 522 (test-data/src/lib.rs:97-98): tests/golden/pghr13.json, tests/test_pghr13.py.
Pure Python, small cases only (~0.1 s per pairing).
"""
P = 21888242871839275222246405745257275088696311157297823662689037894645226208583
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
U = 4965661367192848881
ATE_LOOP = 6 * U + 2


class DecodeError(ValueError):
    pass


# ----------------------------------------------------------------------------- Fq, Fq2
def fq_inv(a):
    return pow(a, P - 2, P)


def fq_sqrt(a):
    """p = 3 mod 4: a^((p+1)/4), None for a non-residue"""
    a %= P
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a else None


F2_ZERO, F2_ONE = (0, 0), (1, 0)
XI = (9, 1)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2_sqr(a):
    return f2_mul(a, a)


def f2_scale(a, s):
    return (a[0] * s % P, a[1] * s % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    t = fq_inv((a[0] * a[0] + a[1] * a[1]) % P)
    return (a[0] * t % P, (-a[1]) * t % P)


def f2_pow(a, e):
    r = F2_ONE
    for bit in bin(e)[2:]:
        r = f2_sqr(r)
        if bit == "1":
            r = f2_mul(r, a)
    return r


def f2_sqrt(a):
    """a square root in Fq2 (p = 3 mod 4, eprint 2012/685 algorithm 9) or None; the decoder
    fixes the sign"""
    if a == F2_ZERO:
        return F2_ZERO
    a1 = f2_pow(a, (P - 3) // 4)
    alpha = f2_mul(f2_sqr(a1), a)
    a0 = f2_mul(f2_conj(alpha), alpha)
    if a0 == (P - 1, 0):
        return None
    x0 = f2_mul(a1, a)
    if alpha == (P - 1, 0):
        r = f2_mul(x0, (0, 1))
    else:
        r = f2_mul(f2_pow(f2_add(alpha, F2_ONE), (P - 1) // 2), x0)
    return r if f2_sqr(r) == a else None


def f2_to_u512(a):
    """bn's Fq2 order / serialization: c1 p + c0"""
    return a[1] * P + a[0]


# ----------------------------------------------------------------------------- Fq12 = Fq2[w]/(w^6 - xi)
F12_ONE = [F2_ONE] + [F2_ZERO] * 5


def f12_mul(a, b):
    t = [F2_ZERO] * 11
    for i in range(6):
        if a[i] == F2_ZERO:
            continue
        for j in range(6):
            if b[j] != F2_ZERO:
                t[i + j] = f2_add(t[i + j], f2_mul(a[i], b[j]))
    return [f2_add(t[k], f2_mul(t[k + 6], XI)) if k + 6 < 11 else t[k] for k in range(6)]


def f12_sqr(a):
    return f12_mul(a, a)


def f12_pow(a, e):
    r = F12_ONE
    for bit in bin(e)[2:]:
        r = f12_sqr(r)
        if bit == "1":
            r = f12_mul(r, a)
    return r


def f12_frob(a, k=1):
    """a^(p^k): conj^k of each coefficient times gamma_k,i = xi^(i (p^k - 1) / 6)"""
    out = []
    for i, c in enumerate(a):
        if k % 2:
            c = f2_conj(c)
        out.append(f2_mul(c, f2_pow(XI, i * (P ** k - 1) // 6)))
    return out


def f12_conj(a):
    """a^(p^6): w -> -w"""
    return [c if i % 2 == 0 else f2_neg(c) for i, c in enumerate(a)]


def f12_inv(a):
    """a^-1 = conj(a) / (a conj(a)); a conj(a) lies in Fq6 = Fq2[v], v = w^2, v^3 = xi"""
    ca = f12_conj(a)
    n = f12_mul(a, ca)
    c0, c1, c2 = n[0], n[2], n[4]
    t0 = f2_sub(f2_sqr(c0), f2_mul(XI, f2_mul(c1, c2)))
    t1 = f2_sub(f2_mul(XI, f2_sqr(c2)), f2_mul(c0, c1))
    t2 = f2_sub(f2_sqr(c1), f2_mul(c0, c2))
    det = f2_add(f2_mul(c0, t0), f2_mul(XI, f2_add(f2_mul(c2, t1), f2_mul(c1, t2))))
    di = f2_inv(det)
    inv6 = [f2_mul(t0, di), F2_ZERO, f2_mul(t1, di), F2_ZERO, f2_mul(t2, di), F2_ZERO]
    return f12_mul(ca, inv6)


def final_exponentiation(f):
    """f^((p^12 - 1) / r): easy part (p^6 - 1)(p^2 + 1) by Frobenius, hard part by exponentiation"""
    t = f12_mul(f12_conj(f), f12_inv(f))      # f^(p^6 - 1)
    t = f12_mul(f12_frob(t, 2), t)            # ^(p^2 + 1)
    return f12_pow(t, (P ** 4 - P ** 2 + 1) // R)


# ----------------------------------------------------------------------------- curves
B1 = 3
B2 = f2_mul((3, 0), f2_inv(XI))

G1_GEN = (1, 2)
G2_GEN = ((10857046999023057135944570762232829481370756359578518086990519993285655852781,
           11559732032986387107991004021392285783925812861821192530917403151452391805634),
          (8495653923123431417604973247489272438418190587263600148770280649306958101930,
           4082367875863433681332203403145435568316851327593401208105741076214120093531))


class _F1:
    add = staticmethod(lambda a, b: (a + b) % P)
    sub = staticmethod(lambda a, b: (a - b) % P)
    mul = staticmethod(lambda a, b: a * b % P)
    inv = staticmethod(fq_inv)
    zero, one = 0, 1
    b = B1

    @staticmethod
    def small(k):
        return k % P


class _F2:
    add, sub, mul, inv = staticmethod(f2_add), staticmethod(f2_sub), staticmethod(f2_mul), staticmethod(f2_inv)
    zero, one = F2_ZERO, F2_ONE
    b = B2

    @staticmethod
    def small(k):
        return (k % P, 0)


def on_curve(F, pt):
    x, y = pt
    return F.mul(y, y) == F.add(F.mul(F.mul(x, x), x), F.b)


def ec_add(F, p1, p2):
    """affine, None = infinity"""
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    (x1, y1), (x2, y2) = p1, p2
    if x1 == x2:
        if F.add(y1, y2) == F.zero:
            return None
        lam = F.mul(F.mul(F.small(3), F.mul(x1, x1)), F.inv(F.mul(F.small(2), y1)))
    else:
        lam = F.mul(F.sub(y2, y1), F.inv(F.sub(x2, x1)))
    x3 = F.sub(F.sub(F.mul(lam, lam), x1), x2)
    return (x3, F.sub(F.mul(lam, F.sub(x1, x3)), y1))


def ec_neg(F, p):
    return None if p is None else (p[0], F.sub(F.zero, p[1]))


def ec_mul(F, p, k):
    r = None
    for bit in bin(k)[2:] if k > 0 else "":
        r = ec_add(F, r, r)
        if bit == "1":
            r = ec_add(F, r, p)
    return r


def g1_new(x, y):
    """AffineG1::new"""
    if not on_curve(_F1, (x, y)):
        raise DecodeError("NotMember")
    return (x, y)


def g2_new(x, y):
    """AffineG2::new: on the twist and in the order-r subgroup"""
    if not on_curve(_F2, (x, y)):
        raise DecodeError("NotMember")
    if ec_mul(_F2, (x, y), R) is not None:
        raise DecodeError("NotMember (order)")
    return (x, y)


def fq_from_slice(b):
    v = int.from_bytes(bytes(b), "big")
    if len(b) != 32 or v >= P:
        raise DecodeError("InvalidFieldElement")
    return v


def fq2_from_slice(b):
    u = int.from_bytes(bytes(b), "big")
    c1, c0 = divmod(u, P)
    if len(b) != 64 or c1 >= P:
        raise DecodeError("NotFq2Member")
    return (c0, c1)


def g1_from_compressed(b):
    b = bytes(b)
    if len(b) != 33:
        raise DecodeError("InvalidEncoding")
    sign = b[0]
    x = fq_from_slice(b[1:])
    y = fq_sqrt(x * x * x + B1)
    if y is None:
        raise DecodeError("NotMember")
    if sign == 2:
        y = (-y) % P if y & 1 else y
    elif sign == 3:
        y = y if y & 1 else (-y) % P
    else:
        raise DecodeError("InvalidEncoding")
    return g1_new(x, y)


def g2_from_compressed(b):
    b = bytes(b)
    if len(b) != 65:
        raise DecodeError("InvalidEncoding")
    sign = b[0]
    x = fq2_from_slice(b[1:])
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        raise DecodeError("NotMember")
    yn = f2_neg(y)
    y_gt = f2_to_u512(y) > f2_to_u512(yn)
    if sign == 10:
        y = yn if y_gt else y
    elif sign == 11:
        y = y if y_gt else yn
    else:
        raise DecodeError("InvalidEncoding")
    return g2_new(x, y)


# ----------------------------------------------------------------------------- pairing
def _line(t, slope, p):
    """the line through the twist point t with twist slope `slope`, at p in G1, as an Fq12
    element (untwist (x, y) -> (x w^2, y w^3)): y_P - slope x_P w + (slope x_T - y_T) w^3"""
    xt, yt = t
    xp, yp = p
    return [(yp, 0), f2_neg(f2_scale(slope, xp)), F2_ZERO, f2_sub(f2_mul(slope, xt), yt), F2_ZERO, F2_ZERO]


def _dbl_step(t, p):
    x, y = t
    slope = f2_mul(f2_scale(f2_sqr(x), 3), f2_inv(f2_scale(y, 2)))
    line = _line(t, slope, p)
    x3 = f2_sub(f2_sqr(slope), f2_scale(x, 2))
    return (x3, f2_sub(f2_mul(slope, f2_sub(x, x3)), y)), line


def _add_step(t, q, p):
    (x1, y1), (x2, y2) = t, q
    slope = f2_mul(f2_sub(y2, y1), f2_inv(f2_sub(x2, x1)))
    line = _line(t, slope, p)
    x3 = f2_sub(f2_sub(f2_sqr(slope), x1), x2)
    return (x3, f2_sub(f2_mul(slope, f2_sub(x1, x3)), y1)), line


GAMMA_X1 = f2_pow(XI, (P - 1) // 3)
GAMMA_Y1 = f2_pow(XI, (P - 1) // 2)
GAMMA_X2 = f2_pow(XI, (P * P - 1) // 3)
GAMMA_Y2 = f2_pow(XI, (P * P - 1) // 2)


def twist_frob(q):
    """pi(q) on the twist: (conj(x) xi^((p-1)/3), conj(y) xi^((p-1)/2))"""
    return (f2_mul(f2_conj(q[0]), GAMMA_X1), f2_mul(f2_conj(q[1]), GAMMA_Y1))


def twist_frob2(q):
    return (f2_mul(q[0], GAMMA_X2), f2_mul(q[1], GAMMA_Y2))


def miller_loop(pairs):
    """prod over (p, q) of the optimal ate Miller function f_{6u+2, q}(p) l_{T, pi(q)} l_{T', -pi^2(q)};
    pairs with an infinite point contribute 1"""
    pairs = [(p, q) for p, q in pairs if p is not None and q is not None]
    f = F12_ONE
    ts = [q for _, q in pairs]
    for bit in bin(ATE_LOOP)[3:]:
        f = f12_sqr(f)
        for k, (p, q) in enumerate(pairs):
            ts[k], line = _dbl_step(ts[k], p)
            f = f12_mul(f, line)
            if bit == "1":
                ts[k], line = _add_step(ts[k], q, p)
                f = f12_mul(f, line)
    for k, (p, q) in enumerate(pairs):
        q1 = twist_frob(q)
        q2 = twist_frob2(q)
        ts[k], line = _add_step(ts[k], q1, p)
        f = f12_mul(f, line)
        _, line = _add_step(ts[k], (q2[0], f2_neg(q2[1])), p)
        f = f12_mul(f, line)
    return f


def pairing(p, q):
    return final_exponentiation(miller_loop([(p, q)]))


def pairing_product_is_one(pairs):
    return final_exponentiation(miller_loop(pairs)) == F12_ONE


def g1_to_compressed(pt):
    """the inverse of g1_from_compressed (test fixtures)"""
    x, y = pt
    return bytes([3 if y & 1 else 2]) + x.to_bytes(32, "big")


def g2_to_compressed(pt):
    x, y = pt
    gt = f2_to_u512(y) > f2_to_u512(f2_neg(y))
    return bytes([11 if gt else 10]) + f2_to_u512(x).to_bytes(64, "big")


# ----------------------------------------------------------------------------- the device's final exponentiation
def f12_exp_by_neg_u(f):
    return f12_conj(f12_pow(f, U))


def final_exponentiation_fc(f):
    """the addition chain the GPU runs for the hard part (Fuentes-Castaneda, Knapp and
    Rodriguez-Henriquez; the `bn` crate's final_exponentiation_last_chunk): it raises the
    easy-part output to 2u(6u^2 + 3u + 1) (p^4 - p^2 + 1) / r, a multiple of the hard exponent by a
    factor coprime to r -- the same equality decisions; tests pin the device's GT bytes to this"""
    t = f12_mul(f12_conj(f), f12_inv(f))
    t = f12_mul(f12_frob(t, 2), t)
    a = f12_exp_by_neg_u(t)
    b = f12_sqr(a)
    c = f12_sqr(b)
    d = f12_mul(c, b)
    e = f12_exp_by_neg_u(d)
    f_ = f12_sqr(e)
    g = f12_exp_by_neg_u(f_)
    h = f12_conj(d)
    i = f12_conj(g)
    j = f12_mul(i, e)
    k = f12_mul(j, h)
    l_ = f12_mul(k, b)
    m = f12_mul(k, e)
    n = f12_mul(t, m)
    o = f12_frob(l_, 1)
    p_ = f12_mul(o, n)
    q = f12_frob(k, 2)
    r_ = f12_mul(q, p_)
    s = f12_conj(t)
    t2 = f12_mul(s, l_)
    u_ = f12_frob(t2, 3)
    return f12_mul(u_, r_)


def gt_ints(f):
    """the device's GT layout: w^0.c0, w^0.c1, ..., w^5.c1"""
    return [x for c in f for x in c]
