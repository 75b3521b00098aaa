"""Note-commitment tree hashing: the oracle against the reference's own
vectors (storage/src/tree_state.rs tests, tests/golden/tree_state.json), and its tree-state
logic against a direct full-tree computation."""
import json
import os
import random

import pytest

from oracle import merkle as M

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "tree_state.json")))
KINDS = {"sprout": M.SPROUT, "sapling": M.SAPLING}


def test_sprout_empty_roots():
    """every SPROUT_EMPTY_ROOTS entry is sha256_compress of the one below (tree_state.rs:5-72)"""
    assert [h.hex() for h in M.empty_roots(M.SPROUT, len(GOLDEN["sprout_empty"]) - 1)] == GOLDEN["sprout_empty"]


def test_sapling_empty_roots():
    """every SAPLING_EMPTY_ROOTS entry is the Pedersen MerkleTree(l) hash of the one below
    (tree_state.rs:74-138), up to depth 62, the last MerkleTree personalization"""
    assert [h.hex() for h in M.empty_roots(M.SAPLING, len(GOLDEN["sapling_empty"]) - 1)] == GOLDEN["sapling_empty"]


@pytest.mark.parametrize("case", GOLDEN["cases"], ids=[c["test"] for c in GOLDEN["cases"]])
def test_reference_tree_cases(case):
    t = M.TreeState(KINDS[case["kind"]], case["height"])
    leaves = [bytes.fromhex(h) for h in case["leaves"]]
    roots = []
    for i, leaf in enumerate(leaves):
        if case.get("full_after") == i:
            break
        t.append(leaf)
        roots.append(t.root().hex())
    if "roots" in case:
        assert roots == case["roots"]
    else:
        assert t.root().hex() == case["final_root"]
    if "full_after" in case:
        with pytest.raises(M.TreeFull):
            t.append(leaves[-1])


def test_glass_frontier():
    """tree_state.rs glass(): the frontier slots after 3 and 5 appends"""
    c = [bytes.fromhex(h) for h in GOLDEN["cases"][7]["leaves"]]
    t = M.TreeState(M.SPROUT, 4)
    for h in c[:3]:
        t.append(h)
    assert t.left == c[2] and t.right is None
    assert t.parents[0] == M.sha256_compress(c[0], c[1]) and t.parents[1] is None
    t.append(c[3])
    t.append(c[4])
    assert t.left == c[4] and t.right is None and t.parents[0] is None
    assert t.parents[1] == M.sha256_compress(M.sha256_compress(c[0], c[1]), M.sha256_compress(c[2], c[3]))


def _full_tree_root(kind, height, leaves):
    e = M.empty_roots(kind, height)
    level = list(leaves)
    for lv in range(height):
        if len(level) % 2:
            level.append(e[lv])
        level = [M.combine(kind, level[2 * i], level[2 * i + 1], lv) for i in range(len(level) // 2)]
        if not level:
            level = [e[lv + 1]]
    return level[0]


@pytest.mark.parametrize("kind", [M.SPROUT, M.SAPLING])
def test_frontier_matches_full_tree(kind):
    """TreeState's incremental root equals the padded full binary tree at every size, and the
    serialized form round-trips (tree_state.rs serde / serde_empty)"""
    rnd = random.Random(7 + kind)
    height = 5
    leaves = [bytes(rnd.getrandbits(8) for _ in range(31)) + b"\x00" for _ in range(1 << height)]
    t = M.TreeState(kind, height)
    assert t.root() == M.empty_roots(kind, height)[height]
    for n in range(1, len(leaves) + 1 if kind == M.SPROUT else 12):
        t.append(leaves[n - 1])
        assert t.size() == n
        assert t.root() == _full_tree_root(kind, height, leaves[:n]), n
        u = M.TreeState.deserialize(kind, height, t.serialize())
        assert u.root() == t.root() and u.size() == n
    e = M.TreeState.deserialize(kind, height, M.TreeState(kind, height).serialize())
    assert e.is_empty


def test_window_roots_matches_appends():
    rnd = random.Random(3)
    leaves = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(40)]
    st = M.TreeState(M.SPROUT, 8)
    for h in leaves[:5]:
        st.append(h)
    marks = [0, 3, 3, 17, 35]
    roots, fin = M.window_roots(st, leaves[5:], marks)
    t = st.copy()
    for k, m in enumerate(marks):
        u = st.copy()
        for h in leaves[5:5 + m]:
            u.append(h)
        assert roots[k] == u.root()
    for h in leaves[5:]:
        t.append(h)
    assert fin.root() == t.root() and fin.serialize() == t.serialize()


def test_cpu_port_matches_oracle():
    """oracle/cpu/merkle_cpu.cpp (the bench's cpu_baseline for trees: the reference's algorithm in
    C++) against the Python oracle: combine for both trees, the golden empty roots, a window"""
    from tests import cpulib
    import ctypes
    L = cpulib.load_merkle()
    rnd = random.Random(12)
    out = ctypes.create_string_buffer(32)
    for kind, n in ((M.SPROUT, 50), (M.SAPLING, 12)):
        for _ in range(n):
            a, b, d = bytes(rnd.getrandbits(8) for _ in range(32)), bytes(rnd.getrandbits(8) for _ in range(32)), rnd.randrange(63)
            assert L.mc_combine(kind, a, b, d, out) == 0
            assert out.raw == M.combine(kind, a, b, d)
    for case in GOLDEN["cases"]:
        kind, h = KINDS[case["kind"]], case["height"]
        leaves = [bytes.fromhex(x) for x in case["leaves"]][:case.get("full_after", 99)]
        marks = list(range(1, len(leaves) + 1)) if "roots" in case else [len(leaves)]
        rc, roots = cpulib.merkle_window(L, kind, h, b"", leaves, marks)
        assert rc == 0
        assert [r.hex() for r in roots] == case.get("roots", [case.get("final_root")])
    st = M.TreeState(M.SAPLING, 32)
    for _ in range(5):
        st.append(bytes(rnd.getrandbits(8) for _ in range(32)))
    leaves = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(4)]
    rc, roots = cpulib.merkle_window(L, M.SAPLING, 32, st.serialize(), leaves, [1, 4])
    assert rc == 0 and roots == M.window_roots(st, leaves, [1, 4])[0]
