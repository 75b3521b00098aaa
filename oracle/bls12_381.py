"""ORACLE (test infrastructure only) -- CPU restatement of BLS12-381 as used by the
reference's Groth16 path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as a checker. The product path (``zebra_amd``) never does.

What it restates (the crates are NOT vendored in /root/reference; pinned versions from
``crypto/Cargo.toml:7,13`` and ``Cargo.lock:1072-1078``):
  * pairing 0.14.2  -- Fq/Fr, the Fq2/Fq6/Fq12 tower, G1/G2 affine + Jacobian,
    compressed/uncompressed point codecs (``into_affine``), subgroup checks,
    ``G2Prepared`` line coefficients, ``Bls12::miller_loop`` and
    ``Bls12::final_exponentiation`` (the chain whose exponent is 3*Phi12(p)/r, see
    SURVEY.md section 8 row a11).
Call sites on the reference path: ``verification/src/sapling.rs:115,158,162,184,203,207``,
``verification/src/sprout.rs:73-77,135-153``, ``crypto/src/json/groth16.rs:94``.

Pinning: accept/reject behaviour is pinned by the reference tests listed in
SURVEY.md section 8(c) (tests/golden/*.json, checked by tests/test_oracle_golden.py).
Raw GT bytes, infinity encodings and non-subgroup points are *parity unpinned* by the
reference tests (no test exposes them); they follow the pinned-crate semantics restated here.

Integers only; pure Python; intended for small cases (a pairing takes ~0.1 s).
"""

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
BLS_X = 0xD201000000010000          # |u|; u = -BLS_X (BLS_X_IS_NEGATIVE = true)
U = -BLS_X
FR_CAPACITY = 254

# ----------------------------------------------------------------------------- Fq
def fq_inv(a):
    if a % P == 0:
        raise ZeroDivisionError
    return pow(a, P - 2, P)


def fq_sqrt(a):
    """pairing Fq::sqrt: p = 3 mod 4 -> a^((p+1)/4); None if a is a non-residue."""
    a %= P
    if a == 0:
        return 0
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a else None


# ----------------------------------------------------------------------------- Fq2 = Fq[u]/(u^2+1)
F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2(a, b=0):
    return (a % P, b % P)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    t0 = a[0] * b[0]
    t1 = a[1] * b[1]
    return ((t0 - t1) % P, ((a[0] + a[1]) * (b[0] + b[1]) - t0 - t1) % P)


def f2_sqr(a):
    return (((a[0] + a[1]) * (a[0] - a[1])) % P, (2 * a[0] * a[1]) % P)


def f2_scale(a, s):
    return (a[0] * s % P, a[1] * s % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    n = fq_inv(a[0] * a[0] + a[1] * a[1])
    return (a[0] * n % P, (-a[1] * n) % P)


def f2_mul_nr(a):
    """multiply by the Fq6 non-residue xi = u + 1."""
    return ((a[0] - a[1]) % P, (a[0] + a[1]) % P)


def f2_pow(a, e):
    r = F2_ONE
    for bit in bin(e)[2:]:
        r = f2_sqr(r)
        if bit == '1':
            r = f2_mul(r, a)
    return r


def f2_is_zero(a):
    return a[0] == 0 and a[1] == 0


def f2_sqrt(a):
    """pairing Fq2::sqrt -- Algorithm 9 of eprint 2012/685 (any root is fine: decoders
    choose the sign afterwards)."""
    if f2_is_zero(a):
        return F2_ZERO
    a1 = f2_pow(a, (P - 3) // 4)
    alpha = f2_mul(f2_sqr(a1), a)
    a0 = f2_mul(f2_conj(alpha), alpha)      # alpha^p * alpha
    neg1 = f2(-1)
    if a0 == neg1:
        return None
    a1 = f2_mul(a1, a)
    if alpha == neg1:
        return f2_mul(a1, (0, 1))
    alpha = f2_pow(f2_add(alpha, F2_ONE), (P - 1) // 2)
    return f2_mul(a1, alpha)


def f2_cmp_gt(a, b):
    """Fq2 Ord (pairing 0.14): compare c1 first, then c0."""
    if a[1] != b[1]:
        return a[1] > b[1]
    return a[0] > b[0]


# ----------------------------------------------------------------------------- Fq6 = Fq2[v]/(v^3 - xi)
F6_ZERO = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE = (F2_ONE, F2_ZERO, F2_ZERO)


def f6_add(a, b):
    return (f2_add(a[0], b[0]), f2_add(a[1], b[1]), f2_add(a[2], b[2]))


def f6_sub(a, b):
    return (f2_sub(a[0], b[0]), f2_sub(a[1], b[1]), f2_sub(a[2], b[2]))


def f6_neg(a):
    return (f2_neg(a[0]), f2_neg(a[1]), f2_neg(a[2]))


def f6_mul(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    t0 = f2_mul(a0, b0)
    t1 = f2_mul(a1, b1)
    t2 = f2_mul(a2, b2)
    c0 = f2_add(f2_mul_nr(f2_sub(f2_sub(f2_mul(f2_add(a1, a2), f2_add(b1, b2)), t1), t2)), t0)
    c1 = f2_add(f2_sub(f2_sub(f2_mul(f2_add(a0, a1), f2_add(b0, b1)), t0), t1), f2_mul_nr(t2))
    c2 = f2_add(f2_sub(f2_sub(f2_mul(f2_add(a0, a2), f2_add(b0, b2)), t0), t2), t1)
    return (c0, c1, c2)


def f6_mul_nr(a):
    """multiply by v: (c0, c1, c2) -> (xi*c2, c0, c1)."""
    return (f2_mul_nr(a[2]), a[0], a[1])


def f6_inv(a):
    a0, a1, a2 = a
    c0 = f2_sub(f2_sqr(a0), f2_mul_nr(f2_mul(a1, a2)))
    c1 = f2_sub(f2_mul_nr(f2_sqr(a2)), f2_mul(a0, a1))
    c2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    t = f2_add(f2_mul(a0, c0), f2_mul_nr(f2_add(f2_mul(a2, c1), f2_mul(a1, c2))))
    ti = f2_inv(t)
    return (f2_mul(c0, ti), f2_mul(c1, ti), f2_mul(c2, ti))


# ----------------------------------------------------------------------------- Fq12 = Fq6[w]/(w^2 - v)
F12_ONE = (F6_ONE, F6_ZERO)


def f12_mul(a, b):
    t0 = f6_mul(a[0], b[0])
    t1 = f6_mul(a[1], b[1])
    c1 = f6_sub(f6_sub(f6_mul(f6_add(a[0], a[1]), f6_add(b[0], b[1])), t0), t1)
    c0 = f6_add(t0, f6_mul_nr(t1))
    return (c0, c1)


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    return (a[0], f6_neg(a[1]))


def f12_inv(a):
    t = f6_sub(f6_mul(a[0], a[0]), f6_mul_nr(f6_mul(a[1], a[1])))
    ti = f6_inv(t)
    return (f6_mul(a[0], ti), f6_neg(f6_mul(a[1], ti)))


def f12_pow(a, e):
    r = F12_ONE
    for bit in bin(e)[2:]:
        r = f12_sqr(r)
        if bit == '1':
            r = f12_mul(r, a)
    return r


def f12_is_zero(a):
    return all(f2_is_zero(c) for h in a for c in h)


def f12_from_coeffs(c):
    """12 Fq ints in canonical order -> Fq12."""
    return (((c[0], c[1]), (c[2], c[3]), (c[4], c[5])), ((c[6], c[7]), (c[8], c[9]), (c[10], c[11])))


def f12_coeffs(a):
    return [x for h in a for c in h for x in c]


def f12_to_bytes(a):
    """576-byte canonical GT encoding used by this build (the reference has no Fq12
    serialization): the 12 Fq coefficients in tower order c0.c0.c0, c0.c0.c1, c0.c1.c0, ...,
    c1.c2.c1, each 48-byte big-endian, non-Montgomery."""
    return b''.join(x.to_bytes(48, 'big') for x in f12_coeffs(a))


def f12_from_bytes(b):
    assert len(b) == 576
    return f12_from_coeffs([int.from_bytes(b[48 * i:48 * i + 48], 'big') for i in range(12)])


# Frobenius constants computed from first principles: the Frobenius on Fq12 in this
# tower is  c0 + c1 w  ->  frob(c0) + frob(c1) * gamma_w,k  etc.
def _xi_pow(e):
    return f2_pow((1, 1), e)


FROB6_C1 = [_xi_pow((P ** k - 1) // 3) for k in range(12)]   # for v coefficient
FROB6_C2 = [_xi_pow(2 * (P ** k - 1) // 3) for k in range(12)]
FROB12_C1 = [_xi_pow((P ** k - 1) // 6) for k in range(12)]  # for w coefficient


def _f2_frob(a, k):
    return a if k % 2 == 0 else f2_conj(a)


def f6_frob(a, k):
    return (_f2_frob(a[0], k), f2_mul(_f2_frob(a[1], k), FROB6_C1[k % 12]),
            f2_mul(_f2_frob(a[2], k), FROB6_C2[k % 12]))


def f12_frob(a, k):
    c0 = f6_frob(a[0], k)
    c1 = f6_frob(a[1], k)
    g = FROB12_C1[k % 12]
    return (c0, (f2_mul(c1[0], g), f2_mul(c1[1], g), f2_mul(c1[2], g)))


# ----------------------------------------------------------------------------- curves
# Points are affine tuples (x, y) or None for infinity. Field ops selected by 'F'.
class _Field:
    def __init__(self, add, sub, mul, sqr, neg, inv, zero, one, is_zero, scal):
        self.add, self.sub, self.mul, self.sqr = add, sub, mul, sqr
        self.neg, self.inv, self.zero, self.one, self.is_zero = neg, inv, zero, one, is_zero
        self.scal = scal


FQ = _Field(lambda a, b: (a + b) % P, lambda a, b: (a - b) % P, lambda a, b: a * b % P,
            lambda a: a * a % P, lambda a: (-a) % P, fq_inv, 0, 1, lambda a: a % P == 0,
            lambda a, s: a * s % P)
FQ2 = _Field(f2_add, f2_sub, f2_mul, f2_sqr, f2_neg, f2_inv, F2_ZERO, F2_ONE, f2_is_zero,
             f2_scale)

B1 = 4
B2 = (4, 4)          # 4(u+1)


def on_curve(F, b, pt):
    if pt is None:
        return True
    x, y = pt
    return F.sub(F.sqr(y), F.add(F.mul(F.sqr(x), x), b)) == F.zero


def ec_neg(F, pt):
    return None if pt is None else (pt[0], F.neg(pt[1]))


def ec_add(F, p1, p2):
    """affine addition (complete case analysis)."""
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    x1, y1 = p1
    x2, y2 = p2
    if x1 == x2:
        if y1 == y2 and not F.is_zero(y1):
            lam = F.mul(F.scal(F.sqr(x1), 3), F.inv(F.scal(y1, 2)))
        else:
            return None
    else:
        lam = F.mul(F.sub(y2, y1), F.inv(F.sub(x2, x1)))
    x3 = F.sub(F.sub(F.sqr(lam), x1), x2)
    y3 = F.sub(F.mul(lam, F.sub(x1, x3)), y1)
    return (x3, y3)


# Jacobian (X, Y, Z), Z == zero means infinity. Used for speed in scalar multiplication.
def _jac_dbl(F, p):
    X, Y, Z = p
    if F.is_zero(Z):
        return p
    A = F.sqr(X)
    B = F.sqr(Y)
    C = F.sqr(B)
    D = F.scal(F.sub(F.sub(F.sqr(F.add(X, B)), A), C), 2)
    E = F.scal(A, 3)
    Fv = F.sqr(E)
    X3 = F.sub(Fv, F.scal(D, 2))
    Y3 = F.sub(F.mul(E, F.sub(D, X3)), F.scal(C, 8))
    Z3 = F.scal(F.mul(Y, Z), 2)
    return (X3, Y3, Z3)


def _jac_add(F, p, q):
    X1, Y1, Z1 = p
    X2, Y2, Z2 = q
    if F.is_zero(Z1):
        return q
    if F.is_zero(Z2):
        return p
    Z1Z1 = F.sqr(Z1)
    Z2Z2 = F.sqr(Z2)
    U1 = F.mul(X1, Z2Z2)
    U2 = F.mul(X2, Z1Z1)
    S1 = F.mul(F.mul(Y1, Z2), Z2Z2)
    S2 = F.mul(F.mul(Y2, Z1), Z1Z1)
    if U1 == U2:
        if S1 == S2:
            return _jac_dbl(F, p)
        return (F.one, F.one, F.zero)
    H = F.sub(U2, U1)
    I = F.sqr(F.scal(H, 2))
    J = F.mul(H, I)
    r = F.scal(F.sub(S2, S1), 2)
    V = F.mul(U1, I)
    X3 = F.sub(F.sub(F.sqr(r), J), F.scal(V, 2))
    Y3 = F.sub(F.mul(r, F.sub(V, X3)), F.scal(F.mul(S1, J), 2))
    Z3 = F.mul(F.sub(F.sub(F.sqr(F.add(Z1, Z2)), Z1Z1), Z2Z2), H)
    return (X3, Y3, Z3)


def _to_jac(F, pt):
    return (F.one, F.one, F.zero) if pt is None else (pt[0], pt[1], F.one)


def _from_jac(F, p):
    X, Y, Z = p
    if F.is_zero(Z):
        return None
    zi = F.inv(Z)
    zi2 = F.sqr(zi)
    return (F.mul(X, zi2), F.mul(Y, F.mul(zi2, zi)))


def ec_mul(F, pt, k):
    """k*pt for any non-negative integer k (double-and-add, MSB first)."""
    if pt is None or k == 0:
        return None
    acc = (F.one, F.one, F.zero)
    base = _to_jac(F, pt)
    for bit in bin(k)[2:]:
        acc = _jac_dbl(F, acc)
        if bit == '1':
            acc = _jac_add(F, acc, base)
    return _from_jac(F, acc)


def g1_in_subgroup(pt):
    """pairing 0.14 is_in_correct_subgroup_assuming_on_curve: [r]P == O."""
    return ec_mul(FQ, pt, R) is None


def g2_in_subgroup(pt):
    return ec_mul(FQ2, pt, R) is None


# Generators (standard BLS12-381; used only for self-tests / synthetic keys).
G1_GEN = (0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
          0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1)
G2_GEN = ((0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
           0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E),
          (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
           0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE))


# ----------------------------------------------------------------------------- codecs
class DecodeError(Exception):
    """GroupDecodingError / io::ErrorKind::InvalidData."""


def _be(b):
    return int.from_bytes(b, 'big')


def g1_decompress(data):
    """pairing 0.14 G1Compressed::into_affine (incl. subgroup check). Returns None for
    the point at infinity, raises DecodeError on any failure."""
    assert len(data) == 48
    c = bytearray(data)
    if not c[0] & 0x80:
        raise DecodeError("UnexpectedCompressionMode")
    if c[0] & 0x40:
        c[0] &= 0x3F
        if any(c):
            raise DecodeError("UnexpectedInformation")
        return None
    greatest = bool(c[0] & 0x20)
    c[0] &= 0x1F
    x = _be(c)
    if x >= P:
        raise DecodeError("x coordinate not in field")
    y = fq_sqrt((x * x * x + B1) % P)
    if y is None:
        raise DecodeError("NotOnCurve")
    ny = (-y) % P
    if not ((y < ny) ^ greatest):
        y = ny
    pt = (x, y)
    if not g1_in_subgroup(pt):
        raise DecodeError("NotInSubgroup")
    return pt


def g2_decompress(data):
    """pairing 0.14 G2Compressed::into_affine. x = x.c1 (48 B, carries flags) || x.c0."""
    assert len(data) == 96
    c = bytearray(data)
    if not c[0] & 0x80:
        raise DecodeError("UnexpectedCompressionMode")
    if c[0] & 0x40:
        c[0] &= 0x3F
        if any(c):
            raise DecodeError("UnexpectedInformation")
        return None
    greatest = bool(c[0] & 0x20)
    c[0] &= 0x1F
    x1 = _be(c[:48])
    x0 = _be(c[48:])
    if x1 >= P or x0 >= P:
        raise DecodeError("x coordinate not in field")
    x = (x0, x1)
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        raise DecodeError("NotOnCurve")
    ny = f2_neg(y)
    y_lt = f2_cmp_gt(ny, y)
    if not (y_lt ^ greatest):
        y = ny
    pt = (x, y)
    if not g2_in_subgroup(pt):
        raise DecodeError("NotInSubgroup")
    return pt


def g1_decode_uncompressed(data):
    """pairing 0.14 G1Uncompressed::into_affine (96 B: x || y)."""
    assert len(data) == 96
    c = bytearray(data)
    if c[0] & 0x80:
        raise DecodeError("UnexpectedCompressionMode")
    if c[0] & 0x40:
        c[0] &= 0x3F
        if any(c):
            raise DecodeError("UnexpectedInformation")
        return None
    if c[0] & 0x20:
        raise DecodeError("UnexpectedInformation")
    c[0] &= 0x1F
    x = _be(c[:48])
    y = _be(c[48:])
    if x >= P or y >= P:
        raise DecodeError("coordinate not in field")
    pt = (x, y)
    if not on_curve(FQ, B1, pt):
        raise DecodeError("NotOnCurve")
    if not g1_in_subgroup(pt):
        raise DecodeError("NotInSubgroup")
    return pt


def g2_decode_uncompressed(data):
    """pairing 0.14 G2Uncompressed::into_affine (192 B: x.c1 || x.c0 || y.c1 || y.c0)."""
    assert len(data) == 192
    c = bytearray(data)
    if c[0] & 0x80:
        raise DecodeError("UnexpectedCompressionMode")
    if c[0] & 0x40:
        c[0] &= 0x3F
        if any(c):
            raise DecodeError("UnexpectedInformation")
        return None
    if c[0] & 0x20:
        raise DecodeError("UnexpectedInformation")
    c[0] &= 0x1F
    vals = [_be(c[48 * i:48 * i + 48]) for i in range(4)]
    if any(v >= P for v in vals):
        raise DecodeError("coordinate not in field")
    pt = ((vals[1], vals[0]), (vals[3], vals[2]))
    if not on_curve(FQ2, B2, pt):
        raise DecodeError("NotOnCurve")
    if not g2_in_subgroup(pt):
        raise DecodeError("NotInSubgroup")
    return pt


def g1_compress(pt):
    if pt is None:
        return bytes([0xC0]) + bytes(47)
    x, y = pt
    out = bytearray(x.to_bytes(48, 'big'))
    out[0] |= 0x80
    if y > (-y) % P:
        out[0] |= 0x20
    return bytes(out)


def g2_compress(pt):
    if pt is None:
        return bytes([0xC0]) + bytes(95)
    x, y = pt
    out = bytearray(x[1].to_bytes(48, 'big') + x[0].to_bytes(48, 'big'))
    out[0] |= 0x80
    if f2_cmp_gt(y, f2_neg(y)):
        out[0] |= 0x20
    return bytes(out)


def g1_uncompressed(pt):
    if pt is None:
        return bytes([0x40]) + bytes(95)
    return pt[0].to_bytes(48, 'big') + pt[1].to_bytes(48, 'big')


def g2_uncompressed(pt):
    if pt is None:
        return bytes([0x40]) + bytes(191)
    (x0, x1), (y0, y1) = pt
    return b''.join(v.to_bytes(48, 'big') for v in (x1, x0, y1, y0))


# ----------------------------------------------------------------------------- pairing
_X_BITS = bin(BLS_X >> 1)[3:]   # bits of x>>1 after the leading one (MSB first)


def _doubling_step(r):
    """pairing 0.14 G2Prepared doubling_step (Alg. 26 of eprint 2010/354), Jacobian Fq2."""
    rx, ry, rz = r
    tmp0 = f2_sqr(rx)
    tmp1 = f2_sqr(ry)
    tmp2 = f2_sqr(tmp1)
    tmp3 = f2_sub(f2_sub(f2_sqr(f2_add(tmp1, rx)), tmp0), tmp2)
    tmp3 = f2_add(tmp3, tmp3)
    tmp4 = f2_add(f2_add(tmp0, tmp0), tmp0)
    tmp6 = f2_add(rx, tmp4)
    tmp5 = f2_sqr(tmp4)
    zsquared = f2_sqr(rz)
    nx = f2_sub(f2_sub(tmp5, tmp3), tmp3)
    nz = f2_sub(f2_sub(f2_sqr(f2_add(rz, ry)), tmp1), zsquared)
    ny = f2_mul(f2_sub(tmp3, nx), tmp4)
    tmp2 = f2_scale(tmp2, 8)
    ny = f2_sub(ny, tmp2)
    tmp3 = f2_neg(f2_scale(f2_mul(tmp4, zsquared), 2))
    tmp6 = f2_sub(f2_sub(f2_sqr(tmp6), tmp0), tmp5)
    tmp1 = f2_scale(tmp1, 4)
    tmp6 = f2_sub(tmp6, tmp1)
    tmp0 = f2_scale(f2_mul(nz, zsquared), 2)
    return (nx, ny, nz), (tmp0, tmp3, tmp6)


def _addition_step(r, q):
    """pairing 0.14 G2Prepared addition_step (Alg. 27 of eprint 2010/354)."""
    rx, ry, rz = r
    qx, qy = q
    zsquared = f2_sqr(rz)
    ysquared = f2_sqr(qy)
    t0 = f2_mul(zsquared, qx)
    t1 = f2_mul(f2_sub(f2_sub(f2_sqr(f2_add(qy, rz)), ysquared), zsquared), zsquared)
    t2 = f2_sub(t0, rx)
    t3 = f2_sqr(t2)
    t4 = f2_scale(t3, 4)
    t5 = f2_mul(t4, t2)
    t6 = f2_sub(f2_sub(t1, ry), ry)
    t9 = f2_mul(t6, qx)
    t7 = f2_mul(t4, rx)
    nx = f2_sub(f2_sub(f2_sub(f2_sqr(t6), t5), t7), t7)
    nz = f2_sub(f2_sub(f2_sqr(f2_add(rz, t2)), zsquared), t3)
    t10 = f2_add(qy, nz)
    t8 = f2_mul(f2_sub(t7, nx), t6)
    t0 = f2_scale(f2_mul(ry, t5), 2)
    ny = f2_sub(t8, t0)
    t10 = f2_sub(f2_sub(f2_sqr(t10), ysquared), f2_sqr(nz))
    t9 = f2_sub(f2_scale(t9, 2), t10)
    t10 = f2_scale(nz, 2)
    t6 = f2_neg(t6)
    t1 = f2_scale(t6, 2)
    return (nx, ny, nz), (t10, t1, t9)


def g2_prepare(q):
    """G2Prepared::from_affine -> list of 68 (c0, c1, c2) Fq2 triples, [] for infinity."""
    if q is None:
        return []
    coeffs = []
    r = (q[0], q[1], F2_ONE)
    for bit in _X_BITS:
        r, c = _doubling_step(r)
        coeffs.append(c)
        if bit == '1':
            r, c = _addition_step(r, q)
            coeffs.append(c)
    r, c = _doubling_step(r)
    coeffs.append(c)
    return coeffs


def _mul_by_014(f, c0, c1, c4):
    """Fq12::mul_by_014 == f * ((c0 + c1 v) + (c4 v) w), computed densely."""
    line = ((c0, c1, F2_ZERO), (F2_ZERO, c4, F2_ZERO))
    return f12_mul(f, line)


def _ell(f, coeffs, p):
    c0 = f2_scale(coeffs[0], p[1])
    c1 = f2_scale(coeffs[1], p[0])
    return _mul_by_014(f, coeffs[2], c1, c0)


def miller_loop(pairs):
    """Bls12::miller_loop over [(G1 affine | None, G2Prepared list)]; pairs with an
    infinity point are skipped; f is conjugated at the end (u < 0)."""
    live = [(p, q) for (p, q) in pairs if p is not None and q]
    idx = [0] * len(live)
    f = F12_ONE
    for bit in _X_BITS:
        for j, (p, q) in enumerate(live):
            f = _ell(f, q[idx[j]], p)
            idx[j] += 1
        if bit == '1':
            for j, (p, q) in enumerate(live):
                f = _ell(f, q[idx[j]], p)
                idx[j] += 1
        f = f12_sqr(f)
    for j, (p, q) in enumerate(live):
        f = _ell(f, q[idx[j]], p)
        idx[j] += 1
    return f12_conj(f)


# --- affine G2 lines normalised to a unit vw coefficient (zebra_amd's ZG_LINES_AFFINE path; test
# infrastructure). The line through R with slope lambda, evaluated at p = (px, py), is pairing's
# `ell` operand up to a factor in Fq2 * Fq: (lambda x_R - y_R) + (-lambda px) v + py v w. Divided by py:
#   a + b v + v w,  a = (lambda x_R - y_R) / py,  b = -lambda px / py.
# The final exponentiation kills Fq2 and Fq factors (p^6 - 1 divides its exponent), so a Miller value
# over these lines has the same GT image as miller_loop's; the 576-B partial is a different element.
def affine_lines(q, p):
    """G2Prepared(q)'s 68 steps in affine coordinates with the lines for p normalised: [(a, b)]"""
    px, py = p
    ipy = fq_inv(py)
    pxy = px * ipy % P
    qx, qy = q
    x, y = q
    out = []

    def step(x, y, dbl):
        if dbl:
            lam = f2_mul(f2_scale(f2_sqr(x), 3), f2_inv(f2_scale(y, 2)))
            x3 = f2_sub(f2_sqr(lam), f2_scale(x, 2))
        else:
            lam = f2_mul(f2_sub(qy, y), f2_inv(f2_sub(qx, x)))
            x3 = f2_sub(f2_sub(f2_sqr(lam), x), qx)
        y3 = f2_sub(f2_mul(lam, f2_sub(x, x3)), y)
        out.append((f2_scale(f2_sub(f2_mul(lam, x), y), ipy), f2_neg(f2_scale(lam, pxy))))
        return x3, y3
    for bit in _X_BITS:
        x, y = step(x, y, True)
        if bit == '1':
            x, y = step(x, y, False)
    step(x, y, True)
    return out


def _aline(ab):
    a, b = ab
    return ((a, b, F2_ZERO), (F2_ZERO, F2_ONE, F2_ZERO))


AFFINE_IDLE_LINE = (F2_ZERO, F2_ZERO)   # the line v w (= w^3, FE-trivial) a slot without a proof contributes


def miller_chain_affine(lines_list):
    """the Miller chain over the products of several proofs' normalised lines (one list of 68 (a, b)
    per proof, AFFINE_IDLE_LINE lists for empty slots), conjugated (u < 0): the group chain of
    k_line_prod / k_batch_fchaing on affine lines"""
    f = F12_ONE
    n = 0

    def mul_step(f, n):
        for ls in lines_list:
            f = f12_mul(f, _aline(ls[n]))
        return f
    for bit in _X_BITS:
        f = mul_step(f, n)
        n += 1
        if bit == '1':
            f = mul_step(f, n)
            n += 1
        f = f12_sqr(f)
    f = mul_step(f, n)
    return f12_conj(f)


def _exp_by_x(f, x):
    return f12_conj(f12_pow(f, x))


def final_exponentiation(f):
    """Bls12::final_exponentiation (pairing 0.14.2 chain). Returns None for f == 0."""
    if f12_is_zero(f):
        return None
    f1 = f12_conj(f)
    f2 = f12_inv(f)
    r = f12_mul(f1, f2)
    f2 = r
    r = f12_mul(f12_frob(r, 2), f2)
    x = BLS_X
    y0 = f12_sqr(r)
    y1 = _exp_by_x(y0, x)
    y2 = _exp_by_x(y1, x >> 1)
    y3 = f12_conj(r)
    y1 = f12_mul(y1, y3)
    y1 = f12_conj(y1)
    y1 = f12_mul(y1, y2)
    y2 = _exp_by_x(y1, x)
    y3 = _exp_by_x(y2, x)
    y1 = f12_conj(y1)
    y3 = f12_mul(y3, y1)
    y1 = f12_conj(y1)
    y1 = f12_frob(y1, 3)
    y2 = f12_frob(y2, 2)
    y1 = f12_mul(y1, y2)
    y2 = _exp_by_x(y3, x)
    y2 = f12_mul(y2, y0)
    y2 = f12_mul(y2, r)
    y1 = f12_mul(y1, y2)
    y2 = f12_frob(y3, 1)
    y1 = f12_mul(y1, y2)
    return y1


# The exponent the chain above applies, as an integer.
HARD_EXP_TIMES_3 = (U - 1) ** 2 * (U + P) * (U * U + P * P - 1) + 3
PHI12 = P ** 4 - P ** 2 + 1
assert PHI12 % R == 0 and HARD_EXP_TIMES_3 == 3 * (PHI12 // R)
FINAL_EXP = (P ** 6 - 1) * (P ** 2 + 1) * HARD_EXP_TIMES_3


def pairing(p, q):
    """E::pairing(p, q) = final_exponentiation(miller_loop([(p, prepare(q))]))."""
    return final_exponentiation(miller_loop([(p, g2_prepare(q))]))
