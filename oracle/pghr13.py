"""ORACLE (test infrastructure only) -- CPU restatement of the reference's PGHR13 Sprout proof
check, on oracle/bn254.py:

  * crypto/src/json/pghr13.rs: the verifying key JSON (res/sprout-verifying-key.json): G1 as
    [x, y], G2 as [x_a, x_b, y_a, y_b] with x = Fq2::new(x_b, x_a), y = Fq2::new(y_b, y_a)
    (0x-prefixed big-endian hex), every point through AffineG1::new / AffineG2::new
  * crypto/src/pghr13.rs:69-81 Proof::from_raw (296 bytes: a, a', b (G2, 65 B), b', c, c', k, h)
  * crypto/src/pghr13.rs:84-105 verify: acc = ic[0] + sum x_i ic[i+1], then
        e(a, vk.a) = e(a', P2),  e(vk.b, b) = e(b', P2),  e(c, vk.c) = e(c', P2),
        e(k, vk.gamma) = e(acc + a + c, vk.gamma_beta_2) e(vk.gamma_beta_1, b),
        e(acc + a, b) = e(h, vk.z) e(c, P2)            (P2 = G2::one())
  * verification/src/sprout.rs:34-67,119-133 the JoinSplit statement: the same 2176 bits as the
    Groth16 branch, packed into BN254 Fr elements 253 bits at a time (Input::into_bn_frs);
    Proof::from_raw failing -> ErrorKind::InvalidEncoding, verify false -> InvalidPGHRProof
Each equality is decided as one product of pairings (a Miller loop over its pairs, one final
exponentiation) compared with 1, which is the same predicate.
"""
import json

from . import bn254 as B
from .zcash import sprout_bits

OK, INVALID_ENCODING, INVALID_PROOF = 0, 1, 3   # mirrors zg ZG_STATUS_* (DECODE_INVALID / VERIFY_FAILED)
FR_CAPACITY = 253


def _h(s):
    s = s[2:] if s.startswith("0x") else s
    return bytes.fromhex(s)


def load_vk_json(text):
    d = json.loads(text)

    def g1(v):
        return B.g1_new(B.fq_from_slice(_h(v[0])), B.fq_from_slice(_h(v[1])))

    def g2(v):
        xa, xb, ya, yb = (B.fq_from_slice(_h(x)) for x in v)
        return B.g2_new((xb, xa), (yb, ya))

    return {"a": g2(d["alphaA"]), "b": g1(d["alphaB"]), "c": g2(d["alphaC"]), "z": g2(d["zeta"]),
            "gamma": g2(d["gamma"]), "gamma_beta_1": g1(d["gammaBeta1"]), "gamma_beta_2": g2(d["gammaBeta2"]),
            "ic": [g1(v) for v in d["ic"]]}


def proof_from_raw(data):
    """Proof::from_raw -> dict of points; raises bn254.DecodeError"""
    data = bytes(data)
    if len(data) != 296:
        raise B.DecodeError("InvalidRawInput")
    return {"a": B.g1_from_compressed(data[0:33]), "a_prime": B.g1_from_compressed(data[33:66]),
            "b": B.g2_from_compressed(data[66:131]), "b_prime": B.g1_from_compressed(data[131:164]),
            "c": B.g1_from_compressed(data[164:197]), "c_prime": B.g1_from_compressed(data[197:230]),
            "k": B.g1_from_compressed(data[230:263]), "h": B.g1_from_compressed(data[263:296])}


def _eq(lhs, rhs):
    """prod e(lhs) == prod e(rhs)"""
    pairs = list(lhs) + [(B.ec_neg(B._F1, p), q) for p, q in rhs]
    return B.pairing_product_is_one(pairs)


def verify(vk, inputs, proof):
    """crypto/src/pghr13.rs:84-105 (inputs: BN254 Fr integers)"""
    F1 = B._F1
    acc = None
    for x, ic in zip(inputs, vk["ic"][1:]):
        acc = B.ec_add(F1, acc, B.ec_mul(F1, ic, x % B.R))
    acc = B.ec_add(F1, acc, vk["ic"][0])
    p2 = B.G2_GEN
    pr = proof
    aa = B.ec_add(F1, acc, pr["a"])
    return (_eq([(pr["a"], vk["a"])], [(pr["a_prime"], p2)]) and
            _eq([(vk["b"], pr["b"])], [(pr["b_prime"], p2)]) and
            _eq([(pr["c"], vk["c"])], [(pr["c_prime"], p2)]) and
            _eq([(pr["k"], vk["gamma"])],
                [(B.ec_add(F1, aa, pr["c"]), vk["gamma_beta_2"]), (vk["gamma_beta_1"], pr["b"])]) and
            _eq([(aa, pr["b"])], [(pr["h"], vk["z"]), (pr["c"], p2)]))


def bits_to_bn_frs(bits):
    """Input::into_bn_frs (sprout.rs:119-133): 253-bit chunks, bit j weighted 2^j"""
    return [sum(b << j for j, b in enumerate(bits[o:o + FR_CAPACITY])) for o in range(0, len(bits), FR_CAPACITY)]


def joinsplit_inputs(desc, pubkey):
    return bits_to_bn_frs(sprout_bits(desc, pubkey))


def verify_raw(vk, proof_bytes, inputs):
    """-> OK / INVALID_ENCODING / INVALID_PROOF (sprout.rs:61-67)"""
    try:
        pr = proof_from_raw(proof_bytes)
    except B.DecodeError:
        return INVALID_ENCODING
    return OK if verify(vk, inputs, pr) else INVALID_PROOF


def proof_to_raw(pt):
    """Proof::from_raw's inverse (test fixtures)"""
    return (B.g1_to_compressed(pt["a"]) + B.g1_to_compressed(pt["a_prime"]) + B.g2_to_compressed(pt["b"]) +
            B.g1_to_compressed(pt["b_prime"]) + B.g1_to_compressed(pt["c"]) + B.g1_to_compressed(pt["c_prime"]) +
            B.g1_to_compressed(pt["k"]) + B.g1_to_compressed(pt["h"]))
