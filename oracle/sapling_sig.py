"""ORACLE (test infrastructure only) -- CPU restatement of the Sapling signature checks that sit
next to the Groth16 proofs in accept_sapling, and of the transaction
signature hash they sign:

  * Jubjub (twisted Edwards a = -1, d = -10240/10241 over Fr), extended coordinates
  * sapling-crypto @21084bde (not vendored; crypto/Cargo.toml:17):
      - group_hash / find_group_hash: BLAKE2s-256(personal, GH_FIRST_BLOCK || tag), Point::read,
        times the cofactor 8  -> SpendingKeyGenerator ("Zcash_G_", tag ""),
        ValueCommitmentValue ("Zcash_cv", "v"), ValueCommitmentRandomness ("Zcash_cv", "r")
      - redjubjub::PublicKey::verify: c = H*(Rbar || M) = BLAKE2b-512("Zcash_RedJubjubH") mod
        r_J; Rbar must decode, Sbar < r_J; [8](-[S] P_G + R + [c] vk) == O
  * verification/src/sapling.rs:75-98,216-269: spend_auth_sig over rk || sighash with the
    spending-key generator; binding_sig over bvk || sighash with the value-commitment
    randomness generator, bvk = sum cv(spends) - sum cv(outputs) - [valueBalance] G_v
  * script/src/sign.rs:249-474: the ZIP-143 / ZIP-243 signature hash of an overwintered
    transaction (hashPrevouts, hashSequence, hashOutputs, hashJoinSplits, hashShieldedSpends,
    hashShieldedOutputs; BLAKE2b-256 personal "ZcashSigHash" || branch id)

Pinned by the reference's own data: the sighash against script/data/sighash_tests.json (the
official Zcash vectors, tests/golden/sighash.json), and the signatures of the reference's real
Sapling transaction bd4fe81c (sapling.rs:303-305, accept_sapling_works: both signatures valid)
and of block 419221's transactions.
"""
import hashlib

from .bls12_381 import R
from .zcash import JUBJUB_D, PointError, jubjub_read

RJ = 0x0e7db4ea6533afa906673b0101343b00a6682093ccc81082d0970e5ed6f72cb7   # Jubjub subgroup order (Fs)
GH_FIRST_BLOCK = b"096b36a5804bfacef1691e173c366a47ff5ba84a44f26ddd7e8d9f79d5b42df0"
SAPLING_BRANCH_ID = 0x76B809BB


# ----------------------------------------------------------------------------- Jubjub
def _inv(a):
    return pow(a, R - 2, R)


# extended twisted Edwards coordinates (X, Y, Z, T), x = X/Z, y = Y/Z, xy = T/Z
ZERO = (0, 1, 1, 0)


def ext(p):
    x, y = p
    return (x, y, 1, x * y % R)


def aff(P):
    X, Y, Z, _ = P
    zi = _inv(Z)
    return (X * zi % R, Y * zi % R)


def add(P, Q):
    """add-2008-hwcd (a = -1, complete)"""
    X1, Y1, Z1, T1 = P
    X2, Y2, Z2, T2 = Q
    A = X1 * X2 % R
    B = Y1 * Y2 % R
    C = JUBJUB_D * T1 % R * T2 % R
    D = Z1 * Z2 % R
    E = ((X1 + Y1) * (X2 + Y2) - A - B) % R
    F = (D - C) % R
    G = (D + C) % R
    H = (B + A) % R          # B - a A, a = -1
    return (E * F % R, G * H % R, F * G % R, E * H % R)


def neg(P):
    X, Y, Z, T = P
    return ((-X) % R, Y, Z, (-T) % R)


def dbl(P):
    return add(P, P)


def mul(P, k):
    acc = ZERO
    for i in range(k.bit_length() - 1, -1, -1):
        acc = dbl(acc)
        if (k >> i) & 1:
            acc = add(acc, P)
    return acc


def is_zero(P):
    X, Y, Z, _ = P
    return X % R == 0 and (Y - Z) % R == 0


def eq(P, Q):
    return (P[0] * Q[2] - Q[0] * P[2]) % R == 0 and (P[1] * Q[2] - Q[1] * P[2]) % R == 0


def encode(P):
    """edwards::Point::write: y LE with x's parity in bit 255"""
    x, y = aff(P)
    return (y | ((x & 1) << 255)).to_bytes(32, "little")


def read(b):
    """edwards::Point::read -> extended point, PointError('Invalid') on failure"""
    return ext(jubjub_read(bytes(b)))


# ----------------------------------------------------------------------------- generators
def group_hash(tag, personal):
    h = hashlib.blake2s(GH_FIRST_BLOCK + bytes(tag), digest_size=32, person=personal).digest()
    try:
        p = read(h)
    except PointError:
        return None
    p = mul(p, 8)
    return None if is_zero(p) else p


def find_group_hash(m, personal):
    tag = bytearray(m) + b"\x00"
    while True:
        gh = group_hash(tag, personal)
        assert tag[-1] != 0xFF
        tag[-1] += 1
        if gh is not None:
            return gh


SPENDING_KEY_GENERATOR = find_group_hash(b"", b"Zcash_G_")
VALUE_COMMITMENT_VALUE = find_group_hash(b"v", b"Zcash_cv")
VALUE_COMMITMENT_RANDOMNESS = find_group_hash(b"r", b"Zcash_cv")
GEN_SPEND_AUTH, GEN_BINDING = 0, 1
GENERATORS = {GEN_SPEND_AUTH: SPENDING_KEY_GENERATOR, GEN_BINDING: VALUE_COMMITMENT_RANDOMNESS}


# ----------------------------------------------------------------------------- RedJubjub
def h_star(a, b):
    d = hashlib.blake2b(bytes(a) + bytes(b), digest_size=64, person=b"Zcash_RedJubjubH").digest()
    return int.from_bytes(d, "little") % RJ


def redjubjub_verify(vk_bytes, sig, msg, gen):
    """redjubjub::PublicKey::read(vk) then PublicKey::verify(msg, sig, generator). A vk that
    does not decode is the caller's RandomizedKey(Invalid) error; here it is just invalid."""
    try:
        vk = read(vk_bytes)
    except PointError:
        return False
    return redjubjub_verify_point(vk, sig, msg, gen)


def redjubjub_verify_point(vk, sig, msg, gen):
    sig = bytes(sig)
    c = h_star(sig[:32], msg)
    try:
        r = read(sig[:32])
    except PointError:
        return False
    s = int.from_bytes(sig[32:], "little")
    if s >= RJ:
        return False
    p = add(add(mul(vk, c), r), neg(mul(GENERATORS[gen], s)))
    return is_zero(mul(p, 8))


def redjubjub_sign(sk, msg, gen, rand):
    """a signature the verifier accepts (test data generation; rand: 80 random bytes)"""
    r = int.from_bytes(hashlib.blake2b(bytes(rand) + bytes(msg), digest_size=64,
                                       person=b"Zcash_RedJubjubH").digest(), "little") % RJ
    rbar = encode(mul(GENERATORS[gen], r))
    c = h_star(rbar, msg)
    s = (r + c * sk) % RJ
    return rbar + s.to_bytes(32, "little")


def public_key(sk, gen):
    return encode(mul(GENERATORS[gen], sk))


# ----------------------------------------------------------------------------- Sapling bundle checks
def value_balance_point(v):
    """compute_value_balance (sapling.rs:247-269): [|v|] G_v, negated for v < 0; None for i64::MIN"""
    if v == -(1 << 63):
        return None
    p = mul(VALUE_COMMITMENT_VALUE, abs(v))
    return neg(p) if v < 0 else p


def binding_verification_key(spend_cvs, output_cvs, value_balance):
    """accept_sapling (sapling.rs:82-94) + accept_sapling_final (:216-226): None if a cv does not
    decode or the value balance is i64::MIN (the caller's errors come first)"""
    total = ZERO
    for cv in spend_cvs:
        total = add(total, read(cv))
    for cv in output_cvs:
        total = add(total, neg(read(cv)))
    vb = value_balance_point(value_balance)
    if vb is None:
        return None
    return add(total, neg(vb))


def spend_auth_ok(rk, sighash, sig):
    """accept_spend's spend_auth_sig check (sapling.rs:119-137): message rk || sighash"""
    return redjubjub_verify(rk, sig, bytes(rk) + bytes(sighash), GEN_SPEND_AUTH)


def binding_sig_ok(spend_cvs, output_cvs, value_balance, sighash, sig):
    bvk = binding_verification_key(spend_cvs, output_cvs, value_balance)
    if bvk is None:
        return False
    return redjubjub_verify_point(bvk, sig, encode(bvk) + bytes(sighash), GEN_BINDING)


# ----------------------------------------------------------------------------- ZIP-143 / ZIP-243 sighash
class _Rd:
    def __init__(self, d):
        self.d, self.o = d, 0

    def take(self, n):
        v = self.d[self.o:self.o + n]
        assert len(v) == n, "unexpected end"
        self.o += n
        return v

    def u32(self):
        return int.from_bytes(self.take(4), "little")

    def compact(self):
        b = self.take(1)[0]
        if b < 0xFD:
            return b
        return int.from_bytes(self.take({0xFD: 2, 0xFE: 4, 0xFF: 8}[b]), "little")


def compact_bytes(n):
    if n < 0xFD:
        return bytes([n])
    if n <= 0xFFFF:
        return b"\xfd" + n.to_bytes(2, "little")
    if n <= 0xFFFFFFFF:
        return b"\xfe" + n.to_bytes(4, "little")
    return b"\xff" + n.to_bytes(8, "little")


def parse_tx_raw(raw):
    """Transaction::deserialize (chain/src/transaction.rs:250-330), keeping the serialized pieces
    the signature hash covers"""
    rd = _Rd(bytes(raw))
    header = rd.u32()
    t = {"overwintered": bool(header & 0x80000000), "version": header & 0x7FFFFFFF, "header": header}
    t["vgid"] = rd.u32() if t["overwintered"] else 0
    t["inputs"] = []
    for _ in range(rd.compact()):
        prev = rd.take(36)
        rd.take(rd.compact())
        t["inputs"].append({"prevout": prev, "sequence": rd.take(4)})
    t["outputs"] = []
    for _ in range(rd.compact()):
        o0 = rd.o
        rd.take(8)
        rd.take(rd.compact())
        t["outputs"].append(rd.d[o0:rd.o])
    t["lock_time"] = rd.take(4)
    t["expiry"] = rd.take(4) if t["overwintered"] and t["version"] >= 3 else b"\x00" * 4
    sap = t["overwintered"] and t["version"] >= 4
    t["spends"], t["soutputs"] = [], []
    if sap:
        t["value_balance"] = rd.take(8)
        for _ in range(rd.compact()):
            t["spends"].append(rd.take(384))
        for _ in range(rd.compact()):
            t["soutputs"].append(rd.take(948))
    t["joinsplits"], t["js_pubkey"] = [], None
    if t["version"] >= 2:
        groth = t["overwintered"] and t["version"] >= 4
        n = rd.compact()
        for _ in range(n):
            t["joinsplits"].append(rd.take(8 + 8 + 32 + 64 + 64 + 32 + 32 + 64 + (192 if groth else 296) + 2 * 601))
        if n:
            t["js_pubkey"] = rd.take(32)
            rd.take(64)
    if sap and (t["spends"] or t["soutputs"]):
        t["binding_sig"] = rd.take(64)
    assert rd.o == len(rd.d), "trailing bytes"
    return t


def _b2b(person, data):
    return hashlib.blake2b(data, digest_size=32, person=person).digest()


def sighash(t, input_index=None, script=b"", amount=0, hashtype=1, branch_id=SAPLING_BRANCH_ID):
    """TransactionInputSigner::signature_hash_post_overwinter (script/src/sign.rs:249-329) of a
    parsed overwintered transaction; returns the 32 hash bytes as the reference's H256 holds them"""
    assert t["overwintered"], "pre-Overwinter (Sprout) signature hash not restated"
    sapling = t["version"] >= 4 and t["vgid"] == 0x892F2085
    acp = (hashtype & 0x80) == 0x80
    base = {2: 2, 3: 3}.get(hashtype & 0x1F, 1)
    zero = b"\x00" * 32
    hp = _b2b(b"ZcashPrevoutHash", b"".join(i["prevout"] for i in t["inputs"])) if not acp else zero
    hs = _b2b(b"ZcashSequencHash", b"".join(i["sequence"] for i in t["inputs"])) \
        if base == 1 and not acp else zero
    if base == 1:
        ho = _b2b(b"ZcashOutputsHash", b"".join(t["outputs"]))
    elif base == 3 and input_index is not None and input_index < len(t["outputs"]):
        ho = _b2b(b"ZcashOutputsHash", t["outputs"][input_index])
    else:
        ho = zero
    hj = _b2b(b"ZcashJSplitsHash", b"".join(t["joinsplits"]) + t["js_pubkey"]) if t["joinsplits"] else zero
    hss = _b2b(b"ZcashSSpendsHash", b"".join(s[:320] for s in t["spends"])) if sapling and t["spends"] else zero
    hso = _b2b(b"ZcashSOutputHash", b"".join(t["soutputs"])) if sapling and t["soutputs"] else zero
    s = (t["header"].to_bytes(4, "little") + t["vgid"].to_bytes(4, "little") + hp + hs + ho + hj)
    if sapling:
        s += hss + hso
    s += t["lock_time"] + t["expiry"]
    if sapling:
        s += t.get("value_balance", b"\x00" * 8)
    s += (hashtype & 0xFFFFFFFF).to_bytes(4, "little")
    if input_index is not None:
        inp = t["inputs"][input_index]
        s += inp["prevout"] + compact_bytes(len(script)) + bytes(script) + amount.to_bytes(8, "little") + inp["sequence"]
    person = b"ZcashSigHash" + branch_id.to_bytes(4, "little")
    return hashlib.blake2b(s, digest_size=32, person=person).digest()


def sapling_checks(raw_tx, branch_id=SAPLING_BRANCH_ID):
    """the signature checks accept_sapling makes on a v4 transaction, with the no-input sighash
    the acceptor computes (accept_transaction.rs:377-387): (spend_auth oks, binding ok | None)"""
    t = parse_tx_raw(raw_tx)
    sh = sighash(t, None, b"", 0, 1, branch_id)
    auth = [spend_auth_ok(s[96:128], sh, s[320:384]) for s in t["spends"]]
    bind = None
    if t["spends"] or t["soutputs"]:
        vb = int.from_bytes(t["value_balance"], "little", signed=True)
        bind = binding_sig_ok([s[0:32] for s in t["spends"]], [o[0:32] for o in t["soutputs"]], vb, sh,
                              t["binding_sig"])
    return auth, bind, sh
