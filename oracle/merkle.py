"""ORACLE (test infrastructure only) -- CPU restatement of the note-commitment tree hashing on the
block-accept path. Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use it, as the checker.

Restates:
  * crypto/src/lib.rs:188-198  sha256_compress(left, right): the SHA-256 compression function on
    one 64-byte block (left || right) from the standard IV, no padding, state words big-endian
    (rust-crypto Sha256::result_no_padding)
  * crypto/src/lib.rs:250-275  pedersen_hash(left, right, depth): the 255 low bits of each input
    (LE, FrRepr::read_le + BitIterator reversed + take(Fr::NUM_BITS)) fed, after the 6-bit
    personalization MerkleTree(depth) (depth LE), to sapling-crypto's pedersen_hash, whose
    output's u coordinate is written LE. sapling-crypto @21084bde (crypto/Cargo.toml:17) is not
    vendored; its published algorithm (Zcash protocol spec 5.4.1.7, sapling-crypto
    src/pedersen_hash.rs): bits split into 3-bit chunks (a, b, c), enc = (1 - 2c)(1 + a + 2b),
    chunk i of a segment weighted 2^(4 i), 63 chunks per segment, segment j's sum times the
    generator find_group_hash(LE32(j), "Zcash_PH"); missing trailing bits are 0
  * storage/src/tree_state.rs:167-264  TreeState<D, H>: left / right / parents frontier, append
    (error "Appending to full tree"), root (empty slots padded with H::empty()[level]),
    empty_root = H::empty()[HEIGHT], SproutTreeHash (H29, sha256_compress) and SaplingTreeHash
    (H32, pedersen_hash); tree_state.rs:284-309 the serialized form (Option<H256> as a bool byte
    then the hash, parents as a CompactSize-prefixed list)
  * window_roots: the roots a sequence of appends passes through (db/src/block_chain_db.rs:254-304
    and verification/src/accept_block.rs:290-320 take one per block; verification/src/
    tree_cache.rs:57-71 one per JoinSplit) -- the contract of zg_tree_roots

Pinned by the reference's own vectors (tests/golden/tree_state.json, tests/test_merkle.py):
SPROUT_EMPTY_ROOTS and SAPLING_EMPTY_ROOTS (every level is combine(empty[l], empty[l], l)), the
Sprout single_root / empty_29_root / appended_1_29_root / commitments_full / glass cases and the
Sapling sapling_empty_root / sapling_tree_state_root cases (zcash test_merkletree.cpp vectors).
"""
import struct

from .sapling_sig import RJ, ZERO, add, aff, find_group_hash, mul, neg

# ----------------------------------------------------------------------------- SHA-256 compress
_K = [
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2]
_IV = [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19]
_M32 = 0xFFFFFFFF


def _rotr(x, k):
    return ((x >> k) | (x << (32 - k))) & _M32


def sha256_compress(left, right):
    """crypto/src/lib.rs:188-198"""
    assert len(left) == 32 and len(right) == 32
    w = list(struct.unpack(">16I", bytes(left) + bytes(right)))
    for t in range(16, 64):
        s0 = _rotr(w[t - 15], 7) ^ _rotr(w[t - 15], 18) ^ (w[t - 15] >> 3)
        s1 = _rotr(w[t - 2], 17) ^ _rotr(w[t - 2], 19) ^ (w[t - 2] >> 10)
        w.append((w[t - 16] + s0 + w[t - 7] + s1) & _M32)
    a, b, c, d, e, f, g, h = _IV
    for t in range(64):
        t1 = (h + (_rotr(e, 6) ^ _rotr(e, 11) ^ _rotr(e, 25)) + ((e & f) ^ (~e & g)) + _K[t] + w[t]) & _M32
        t2 = ((_rotr(a, 2) ^ _rotr(a, 13) ^ _rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c))) & _M32
        a, b, c, d, e, f, g, h = (t1 + t2) & _M32, a, b, c, (d + t1) & _M32, e, f, g
    return struct.pack(">8I", *[(x + y) & _M32 for x, y in zip(_IV, (a, b, c, d, e, f, g, h))])


# ----------------------------------------------------------------------------- Pedersen hash
PEDERSEN_CHUNKS_PER_GENERATOR = 63
FR_NUM_BITS = 255
_GENERATORS = []


def pedersen_generator(j):
    """JubjubBls12::new: find_group_hash(LE32(j), "Zcash_PH") (prime order)"""
    while len(_GENERATORS) <= j:
        _GENERATORS.append(find_group_hash(struct.pack("<I", len(_GENERATORS)), b"Zcash_PH"))
    return _GENERATORS[j]


def merkle_personalization_bits(depth):
    """Personalization::MerkleTree(depth).get_bits(): 6 bits, LE"""
    assert 0 <= depth < 63
    return [(depth >> i) & 1 for i in range(6)]


def pedersen_hash_point(bits):
    """sapling-crypto pedersen_hash over an already personalized bit list -> extended point"""
    result = ZERO
    pos, seg = 0, 0
    while pos < len(bits):
        acc, cur = 0, 1
        for _ in range(PEDERSEN_CHUNKS_PER_GENERATOR):
            if pos >= len(bits):
                break
            a = bits[pos]
            b = bits[pos + 1] if pos + 1 < len(bits) else 0
            c = bits[pos + 2] if pos + 2 < len(bits) else 0
            pos += 3
            tmp = cur * (1 + a + 2 * b)
            acc += -tmp if c else tmp
            cur <<= 4
        result = add(result, mul(pedersen_generator(seg), acc % RJ))
        seg += 1
    return result


def _bits_le(b, n):
    v = int.from_bytes(bytes(b), "little")
    return [(v >> i) & 1 for i in range(n)]


def pedersen_hash(left, right, depth):
    """crypto/src/lib.rs:250-275 -> 32 bytes (u coordinate, LE)"""
    assert len(left) == 32 and len(right) == 32
    bits = merkle_personalization_bits(depth) + _bits_le(left, FR_NUM_BITS) + _bits_le(right, FR_NUM_BITS)
    x, _ = aff(pedersen_hash_point(bits))
    return x.to_bytes(32, "little")


# ----------------------------------------------------------------------------- tree state
SPROUT, SAPLING = 0, 1
SPROUT_HEIGHT, SAPLING_HEIGHT = 29, 32
_EMPTY = {SPROUT: [bytes(32)], SAPLING: [(1).to_bytes(32, "little")]}   # pedersen_uncommitted: Fr one


def combine(kind, left, right, depth):
    """SproutTreeHash / SaplingTreeHash::combine (tree_state.rs:175-177,188-190)"""
    return sha256_compress(left, right) if kind == SPROUT else pedersen_hash(left, right, depth)


def empty_roots(kind, upto):
    """H::empty()[0..=upto]: empty[l + 1] = combine(empty[l], empty[l], l)"""
    e = _EMPTY[kind]
    while len(e) <= upto:
        e.append(combine(kind, e[-1], e[-1], len(e) - 1))
    return e[:upto + 1]


class TreeFull(Exception):
    """TreeState::append's Err("Appending to full tree")"""


class TreeState:
    """storage/src/tree_state.rs:193-264 (append / root / empty_root), is_empty as the reference
    keeps it (set by the first append; recomputed from the slots on deserialize)"""

    def __init__(self, kind, height):
        self.kind, self.height = kind, height
        self.left = self.right = None
        self.parents = [None] * (height - 1)
        self.is_empty = True

    def copy(self):
        t = TreeState(self.kind, self.height)
        t.left, t.right, t.parents, t.is_empty = self.left, self.right, list(self.parents), self.is_empty
        return t

    def append(self, h):
        h = bytes(h)
        if self.left is None:
            self.left = h
        elif self.right is None:
            self.right = h
        else:
            former_left, former_right = self.left, self.right
            self.left, self.right = h, None
            combined = combine(self.kind, former_left, former_right, 0)
            for i in range(self.height - 1):
                if self.parents[i] is None:
                    self.parents[i] = combined
                    return
                combined = combine(self.kind, self.parents[i], combined, i + 1)
                self.parents[i] = None
            raise TreeFull("Appending to full tree")
        self.is_empty = False

    def root(self):
        e = empty_roots(self.kind, self.height)
        if self.is_empty:
            return e[self.height]
        left = self.left if self.left is not None else e[0]
        right = self.right if self.right is not None else e[0]
        root = combine(self.kind, left, right, 0)
        for i in range(self.height - 1):
            if self.parents[i] is not None:
                root = combine(self.kind, self.parents[i], root, i + 1)
            else:
                root = combine(self.kind, root, e[i + 1], i + 1)
        return root

    def size(self):
        """the number of leaves appended (the frontier's binary counter: (size - 1) >> 1 pairs
        were pushed into parents, then left, right hold the last one or two leaves)"""
        if self.left is None:
            return 0
        c = sum(1 << i for i, p in enumerate(self.parents) if p is not None)
        return 2 * c + (2 if self.right is not None else 1)

    def serialize(self):
        """tree_state.rs:284-290: Option<H256> left, right, then the parents list"""
        def opt(h):
            return b"\x00" if h is None else b"\x01" + h
        n = len(self.parents)
        assert n < 0xfd
        return opt(self.left) + opt(self.right) + bytes([n]) + b"".join(opt(p) for p in self.parents)

    @classmethod
    def deserialize(cls, kind, height, data):
        """tree_state.rs:292-309 (a parents list of another length is taken as it comes)"""
        data = bytes(data)
        pos = 0

        def opt():
            nonlocal pos
            flag = data[pos]
            pos += 1
            if flag == 0:
                return None
            if flag != 1:
                raise ValueError("bad Option flag")
            h = data[pos:pos + 32]
            if len(h) != 32:
                raise ValueError("short hash")
            pos += 32
            return h

        t = cls(kind, height)
        t.left, t.right = opt(), opt()
        n = data[pos]
        pos += 1
        if n >= 0xfd:
            raise ValueError("unsupported list length")
        t.parents = [opt() for _ in range(n)]
        if pos != len(data):
            raise ValueError("trailing bytes")
        t.is_empty = t.left is None and t.right is None and all(p is None for p in t.parents)
        return t


def window_roots(state, leaves, marks):
    """the roots after marks[k] of `leaves` are appended to `state` (marks in any order), and
    the final state. A mark past the tree's capacity raises TreeFull after the roots before it
    were taken (the reference rejects that block: accept_block.rs:302-304)."""
    t = state.copy()
    roots, done = [None] * len(marks), 0
    for k in sorted(range(len(marks)), key=lambda k: marks[k]):
        while done < marks[k]:
            t.append(leaves[done])
            done += 1
        roots[k] = t.root()
    while done < len(leaves):
        t.append(leaves[done])
        done += 1
    return roots, t
