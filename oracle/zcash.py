"""ORACLE (test infrastructure only) -- CPU restatement of the reference's host-side
input preparation for the Groth16 path, and of the wire formats that carry the proofs.

Restates:
  * Jubjub ``edwards::Point::read`` + small-order check  (sapling-crypto @21084bde, not
    vendored; called at verification/src/sapling.rs:108-128,177-189,280-292)
  * ``accept_spend`` public inputs  -- verification/src/sapling.rs:101-155
  * ``accept_output`` public inputs -- verification/src/sapling.rs:171-200
  * multipack (bytes_to_bits_le + compute_multipacking, CAPACITY 254) -- sapling.rs:140-142
  * Sprout hSig + 2176-bit input + into_bls_frs -- verification/src/sprout.rs:16-153
  * v3/v4 transaction + block wire layout -- chain/src/transaction.rs:250-330,
    chain/src/sapling.rs:37-75, chain/src/join_split.rs:169-186
"""
import hashlib

from .bls12_381 import R
from . import groth16 as G

# ----------------------------------------------------------------------------- Jubjub
JUBJUB_D = (-10240 * pow(10241, R - 2, R)) % R       # a = -1 twisted Edwards over Fr


def fr_sqrt(a):
    """Tonelli-Shanks in Fr (r - 1 = 2^32 * t)."""
    a %= R
    if a == 0:
        return 0
    if pow(a, (R - 1) // 2, R) != 1:
        return None
    q, s = R - 1, 0
    while q % 2 == 0:
        q //= 2
        s += 1
    z = 7   # Fr multiplicative generator (7 is a non-residue)
    m, c, t, x = s, pow(z, q, R), pow(a, q, R), pow(a, (q + 1) // 2, R)
    while t != 1:
        i, t2 = 0, t
        while t2 != 1:
            t2 = t2 * t2 % R
            i += 1
        b = pow(c, 1 << (m - i - 1), R)
        m, c, t, x = i, b * b % R, t * b * b % R, x * b % R
    return x


class PointError(Exception):
    def __init__(self, kind):
        super().__init__(kind)
        self.kind = kind            # "Invalid" | "SmallOrder"


def jubjub_read(b):
    """edwards::Point::read: 32 B LE y with the x sign in bit 255; y < r; x from the curve
    equation; x negated when its parity differs from the sign bit (x = 0 stays 0)."""
    v = int.from_bytes(b, "little")
    sign = v >> 255
    y = v & ((1 << 255) - 1)
    if y >= R:
        raise PointError("Invalid")          # "y is not in field"
    y2 = y * y % R
    den = (JUBJUB_D * y2 + 1) % R
    num = (y2 - 1) % R
    x = fr_sqrt(num * pow(den, R - 2, R) % R)
    if x is None:
        raise PointError("Invalid")          # "not on curve"
    if (x & 1) != sign:
        x = (-x) % R
    return (x, y)


def jubjub_add(p, q):
    x1, y1 = p
    x2, y2 = q
    t = JUBJUB_D * x1 * x2 * y1 * y2 % R
    x3 = (x1 * y2 + y1 * x2) * pow((1 + t) % R, R - 2, R) % R
    y3 = (y1 * y2 + x1 * x2) * pow((1 - t) % R, R - 2, R) % R
    return (x3, y3)


def is_small_order(p):
    """sapling.rs:290-292: 8P == identity."""
    q = p
    for _ in range(3):
        q = jubjub_add(q, q)
    return q == (0, 1)


def require_non_small_order_point(b):
    p = jubjub_read(b)
    if is_small_order(p):
        raise PointError("SmallOrder")
    return p


class FieldError(Exception):
    """PrimeFieldDecodingError::NotInField."""


def fr_from_repr_le(b):
    v = int.from_bytes(b, "little")
    if v >= R:
        raise FieldError("NotInField")
    return v


def multipack_le(b, capacity=254):
    v = int.from_bytes(b, "little")
    nbits = 8 * len(b)
    out = []
    for off in range(0, nbits, capacity):
        out.append((v >> off) & ((1 << min(capacity, nbits - off)) - 1))
    return out


class InputError(Exception):
    """host input-prep error carrying the reference's error class name."""
    def __init__(self, where):
        super().__init__(where)
        self.where = where


def spend_inputs(cv, anchor, nf, rk):
    """accept_spend public input, in reference check order (sapling.rs:107-155; the
    RedJubjub spend_auth_sig check between rk and the proof is out of scope)."""
    try:
        cvp = require_non_small_order_point(cv)
    except PointError as e:
        raise InputError("ValueCommitment(%s)" % e.kind)
    try:
        a = fr_from_repr_le(anchor)
    except FieldError:
        raise InputError("Anchor")
    try:
        rkp = jubjub_read(rk)
    except PointError:
        raise InputError("RandomizedKey(Invalid)")
    if is_small_order(rkp):
        raise InputError("RandomizedKey(SmallOrder)")
    nfp = multipack_le(nf)
    assert len(nfp) == 2
    return [rkp[0], rkp[1], cvp[0], cvp[1], a, nfp[0], nfp[1]]


def output_inputs(cv, cmu, epk):
    """accept_output public input (sapling.rs:171-200)."""
    try:
        cvp = require_non_small_order_point(cv)
    except PointError as e:
        raise InputError("ValueCommitment(%s)" % e.kind)
    try:
        cm = fr_from_repr_le(cmu)
    except FieldError:
        raise InputError("NoteCommitment")
    try:
        ep = require_non_small_order_point(epk)
    except PointError as e:
        raise InputError("EphemeralKey(%s)" % e.kind)
    return [cvp[0], cvp[1], ep[0], ep[1], cm]


def compute_hsig(random_seed, nf0, nf1, pubkey):
    """sprout.rs:16-32."""
    h = hashlib.blake2b(digest_size=32, person=b"ZcashComputehSig")
    for part in (random_seed, nf0, nf1, pubkey):
        h.update(part)
    return h.digest()


def sprout_bits(desc, pubkey):
    """sprout.rs:42-58 + Input::push_bytes (MSB-first per byte)."""
    hsig = compute_hsig(desc["random_seed"], desc["nullifiers"][0], desc["nullifiers"][1], pubkey)
    parts = [desc["anchor"], hsig, desc["nullifiers"][0], desc["macs"][0], desc["nullifiers"][1],
             desc["macs"][1], desc["commitments"][0], desc["commitments"][1],
             desc["vpub_old"].to_bytes(8, "little"), desc["vpub_new"].to_bytes(8, "little")]
    bits = []
    for p in parts:
        for byte in p:
            for i in range(7, -1, -1):
                bits.append((byte >> i) & 1)
    assert len(bits) == 2176
    return bits


def bits_to_frs(bits, capacity=254):
    """Input::into_bls_frs (sprout.rs:135-153)."""
    out = []
    for off in range(0, len(bits), capacity):
        chunk = bits[off:off + capacity]
        out.append(sum(b << j for j, b in enumerate(chunk)) % R)
    return out


def sprout_inputs(desc, pubkey):
    return bits_to_frs(sprout_bits(desc, pubkey))


# ----------------------------------------------------------------------------- wire formats
class _Reader:
    def __init__(self, data):
        self.d = data
        self.o = 0

    def take(self, n):
        if self.o + n > len(self.d):
            raise ValueError("unexpected end")
        v = self.d[self.o:self.o + n]
        self.o += n
        return v

    def u32(self):
        return int.from_bytes(self.take(4), "little")

    def u64(self):
        return int.from_bytes(self.take(8), "little")

    def i64(self):
        return int.from_bytes(self.take(8), "little", signed=True)

    def compact(self):
        b = self.take(1)[0]
        if b < 0xFD:
            return b
        return int.from_bytes(self.take({0xFD: 2, 0xFE: 4, 0xFF: 8}[b]), "little")


SAPLING_VERSION_GROUP_ID = 0x892F2085
OVERWINTER_VERSION_GROUP_ID = 0x03C48270


def parse_tx(rd):
    """Transaction::deserialize (chain/src/transaction.rs:250-330)."""
    start = rd.o
    header = rd.u32()
    overwintered = bool(header & 0x80000000)
    version = header & 0x7FFFFFFF
    vgid = rd.u32() if overwintered else 0
    is_ow = overwintered and version == 3 and vgid == OVERWINTER_VERSION_GROUP_ID
    is_sap = overwintered and version == 4 and vgid == SAPLING_VERSION_GROUP_ID
    if overwintered and not (is_ow or is_sap):
        raise ValueError("invalid overwinter version")
    for _ in range(rd.compact()):        # transparent inputs
        rd.take(36)
        rd.take(rd.compact())
        rd.take(4)
    for _ in range(rd.compact()):        # transparent outputs
        rd.take(8)
        rd.take(rd.compact())
    rd.take(4)                            # lock_time
    if is_ow or is_sap:
        rd.take(4)                        # expiry
    tx = {"version": version, "overwintered": overwintered, "spends": [], "outputs": [],
          "joinsplits": [], "js_pubkey": None}
    if is_sap:
        tx["value_balance"] = rd.i64()
        for _ in range(rd.compact()):
            s = rd.take(384)
            tx["spends"].append({"cv": s[0:32], "anchor": s[32:64], "nullifier": s[64:96],
                                 "rk": s[96:128], "zkproof": s[128:320],
                                 "spend_auth_sig": s[320:384]})
        for _ in range(rd.compact()):
            o = rd.take(948)
            tx["outputs"].append({"cv": o[0:32], "cmu": o[32:64], "epk": o[64:96],
                                  "zkproof": o[756:948]})
    if version >= 2:
        use_groth = overwintered and version >= 4
        n = rd.compact()
        for _ in range(n):
            d = {"vpub_old": rd.u64(), "vpub_new": rd.u64(), "anchor": rd.take(32),
                 "nullifiers": [rd.take(32), rd.take(32)],
                 "commitments": [rd.take(32), rd.take(32)],
                 "ephemeral_key": rd.take(32), "random_seed": rd.take(32),
                 "macs": [rd.take(32), rd.take(32)]}
            d["groth"] = use_groth
            d["zkproof"] = rd.take(192 if use_groth else 296)
            rd.take(2 * 601)
            tx["joinsplits"].append(d)
        if n:
            tx["js_pubkey"] = rd.take(32)
            rd.take(64)
    if is_sap and (tx["spends"] or tx["outputs"]):
        tx["binding_sig"] = rd.take(64)
    raw = rd.d[start:rd.o]
    tx["txid"] = hashlib.sha256(hashlib.sha256(raw).digest()).digest()[::-1].hex()
    return tx


def parse_tx_hex(h):
    rd = _Reader(bytes.fromhex(h))
    tx = parse_tx(rd)
    assert rd.o == len(rd.d), "trailing bytes"
    return tx


def parse_block_hex(h):
    """Zcash block: 140-byte header prefix + compact-size solution, then txs."""
    rd = _Reader(bytes.fromhex(h))
    hdr = rd.take(140)
    sol = rd.take(rd.compact())
    header = hdr + bytes([0xFD]) + len(sol).to_bytes(2, "little") + sol if len(sol) >= 0xFD else None
    bhash = hashlib.sha256(hashlib.sha256(header).digest()).digest()[::-1].hex() if header else None
    txs = [parse_tx(rd) for _ in range(rd.compact())]
    assert rd.o == len(rd.d)
    return bhash, txs


def groth_items_of_tx(tx):
    """All Groth16 proof checks a tx carries, as (kind, proof bytes, inputs | InputError)."""
    items = []
    if tx["js_pubkey"] is not None:
        for d in tx["joinsplits"]:
            if d["groth"]:
                items.append((G.SPROUT, d["zkproof"], sprout_inputs(d, tx["js_pubkey"])))
    for s in tx["spends"]:
        items.append((G.SPEND, s["zkproof"], spend_inputs(s["cv"], s["anchor"], s["nullifier"], s["rk"])))
    for o in tx["outputs"]:
        items.append((G.OUTPUT, o["zkproof"], output_inputs(o["cv"], o["cmu"], o["epk"])))
    return items
