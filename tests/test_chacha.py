"""The batch-scalar CSPRNG: with seeded = 0 every batch draws a fresh 256-bit key from
getrandom(2) and expands it on the GPU with ChaCha20 (zebra_amd/csrc/zg_chacha.h). The checker
is a plain-Python ChaCha20 written from RFC 8439 section 2.3, pinned by the RFC's own
known-answer block (section 2.3.2)."""
import os
import struct

import pytest


def _rotl(x, n):
    return ((x << n) | (x >> (32 - n))) & 0xFFFFFFFF


def _qr(s, a, b, c, d):
    s[a] = (s[a] + s[b]) & 0xFFFFFFFF
    s[d] = _rotl(s[d] ^ s[a], 16)
    s[c] = (s[c] + s[d]) & 0xFFFFFFFF
    s[b] = _rotl(s[b] ^ s[c], 12)
    s[a] = (s[a] + s[b]) & 0xFFFFFFFF
    s[d] = _rotl(s[d] ^ s[a], 8)
    s[c] = (s[c] + s[d]) & 0xFFFFFFFF
    s[b] = _rotl(s[b] ^ s[c], 7)


def chacha20_block(key, counter, nonce):
    init = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + list(struct.unpack("<8I", key)) + [counter] + \
        list(struct.unpack("<3I", nonce))
    s = list(init)
    for _ in range(10):
        _qr(s, 0, 4, 8, 12)
        _qr(s, 1, 5, 9, 13)
        _qr(s, 2, 6, 10, 14)
        _qr(s, 3, 7, 11, 15)
        _qr(s, 0, 5, 10, 15)
        _qr(s, 1, 6, 11, 12)
        _qr(s, 2, 7, 8, 13)
        _qr(s, 3, 4, 9, 14)
    return struct.pack("<16I", *[(x + y) & 0xFFFFFFFF for x, y in zip(s, init)])


RFC_KEY = bytes(range(32))
RFC_NONCE = bytes.fromhex("000000090000004a00000000")
RFC_BLOCK1 = bytes.fromhex(
    "10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
    "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e")


def test_python_chacha20_matches_rfc8439():
    assert chacha20_block(RFC_KEY, 1, RFC_NONCE) == RFC_BLOCK1


@pytest.mark.gpu
def test_device_chacha20_keystream():
    from zebra_amd import Context
    ctx = Context(device=0, max_batch=64)
    try:
        assert ctx.chacha20_blocks(RFC_KEY, RFC_NONCE, 1, 1) == RFC_BLOCK1
        key, nonce = os.urandom(32), os.urandom(12)
        n = 300   # > one 256-thread launch block, ragged
        got = ctx.chacha20_blocks(key, nonce, 0xFFFFFF00, n)
        want = b"".join(chacha20_block(key, (0xFFFFFF00 + j) & 0xFFFFFFFF, nonce) for j in range(n))
        assert got == want
    finally:
        ctx.close()


@pytest.mark.gpu
def test_unseeded_batches_accept_and_reject():
    """OS-random r_i (device ChaCha20): a valid batch passes, and the exact reject set of a
    corrupted batch does not depend on the scalars drawn"""
    from tests.conftest import load_golden
    from zebra_amd import Context
    from zebra_amd import zg
    real = load_golden("real_proofs.json")["proofs"]
    ctx = Context(device=0, max_batch=256)   # seed=None: OS RNG
    try:
        src = b"".join(bytes.fromhex(p["proof"]) for p in real)
        kinds_src = bytes(p["kind"] for p in real)
        idx = [i % len(real) for i in range(37)]
        proofs = ctx.synth_rerandomize(src, kinds_src, idx, 11)
        kinds = bytes(real[i]["kind"] for i in idx)
        inputs = zg.pack_inputs([[bytes.fromhex(x) for x in real[i]["inputs"]] for i in idx])
        for _ in range(2):
            st = ctx.verify_batch(proofs, kinds, inputs)[0]
            assert list(st) == [zg.STATUS_OK] * 37
        bad = bytearray(proofs)
        bad[192 * 5 + 150] ^= 0x01   # C of proof 5 changes (decodes or not): proof 5 fails
        st = list(ctx.verify_batch(bytes(bad), kinds, inputs)[0])
        assert st[5] != zg.STATUS_OK and st[:5] + st[6:] == [zg.STATUS_OK] * 36
    finally:
        ctx.close()
