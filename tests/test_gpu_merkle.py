"""GPU parity of the note-commitment tree hashing against the oracle
(oracle/merkle.py, pinned by storage/src/tree_state.rs's vectors in tests/golden/tree_state.json):
TreeHash::combine bit-exact for both trees, H::empty(), the reference's own tree cases through
zg_tree_roots, random windows over random frontiers against oracle.merkle.window_roots (roots and
the serialized final state), the full-tree error, and at the bench size (Sapling H32, 64k leaves,
1024 roots) the size-independent property that splitting a window anywhere changes nothing."""
import os
import random

import pytest

from oracle import merkle as M
from tests.conftest import load_golden

GOLDEN = load_golden("tree_state.json")
KINDS = {"sprout": M.SPROUT, "sapling": M.SAPLING}


@pytest.fixture(scope="module")
def ctx():
    from zebra_amd import Context
    c = Context(device=0, max_batch=64, load_builtin=False)
    yield c
    c.close()


def _rand32(rnd):
    return bytes(rnd.getrandbits(8) for _ in range(32))


def random_frontier(rnd, kind, height, s0):
    """a TreeState holding s0 leaves with random slot contents (the frontier shape of s0)"""
    t = M.TreeState(kind, height)
    if s0:
        c = (s0 - 1) >> 1
        t.left = _rand32(rnd)
        t.right = _rand32(rnd) if s0 % 2 == 0 else None
        t.parents = [_rand32(rnd) if (c >> i) & 1 else None for i in range(height - 1)]
        t.is_empty = False
        assert t.size() == s0
    return t


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [M.SPROUT, M.SAPLING])
def test_gpu_combine_parity(ctx, kind):
    rnd = random.Random(11 + kind)
    n = 256 if kind == M.SPROUT else 48
    L = [_rand32(rnd) for _ in range(n)] + [bytes(32), b"\xff" * 32, b"\xff" * 32]
    R = [_rand32(rnd) for _ in range(n)] + [bytes(32), b"\xff" * 32, bytes(32)]
    D = [rnd.randrange(63) for _ in range(n)] + [0, 62, 31]
    got = ctx.merkle_combine(kind, L, R, D)
    want = [M.combine(kind, a, b, d) for a, b, d in zip(L, R, D)]
    assert got == want


@pytest.mark.gpu
def test_gpu_empty_roots(ctx):
    assert [h.hex() for h in ctx.tree_empty_roots(M.SPROUT, 64)] == GOLDEN["sprout_empty"][:64]
    assert [h.hex() for h in ctx.tree_empty_roots(M.SAPLING, 63)] == GOLDEN["sapling_empty"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", GOLDEN["cases"], ids=[c["test"] for c in GOLDEN["cases"]])
def test_gpu_reference_tree_cases(ctx, case):
    from zebra_amd import zg
    kind, h = KINDS[case["kind"]], case["height"]
    leaves = [bytes.fromhex(x) for x in case["leaves"]]
    if "roots" in case:
        k = len(case["roots"])
        roots, _ = ctx.tree_roots(kind, h, b"", leaves[:k], list(range(1, k + 1)))
        assert [r.hex() for r in roots] == case["roots"]
    else:
        roots, _ = ctx.tree_roots(kind, h, b"", leaves, [len(leaves)])
        assert roots[0].hex() == case["final_root"]
    if "full_after" in case:
        # the 17th append of a height-4 tree: "Appending to full tree"; the roots before it stand
        with pytest.raises(zg.ZgError) as ei:
            ctx.tree_roots(kind, h, b"", leaves + [leaves[-1]], [16, 17])
        assert ei.value.code == zg.E_TREE_FULL
        assert ei.value.roots[0].hex() == case["roots"][15] and ei.value.roots[1] == bytes(32)


def _check_window(ctx, rnd, kind, height, st, n, nmarks):
    leaves = [_rand32(rnd) for _ in range(n)]
    marks = sorted(rnd.randrange(n + 1) for _ in range(nmarks)) + [0, n]
    rnd.shuffle(marks)
    want, fin = M.window_roots(st, leaves, marks)
    got, state = ctx.tree_roots(kind, height, st.serialize(), leaves, marks)
    assert got == want, (height, st.size(), n, marks)
    assert state == fin.serialize()


@pytest.mark.gpu
def test_gpu_sprout_windows_vs_oracle(ctx):
    rnd = random.Random(5)
    for height in (1, 2, 3, 5, 8):
        for _ in range(6):
            s0 = min(1 << height, rnd.choice([0, 1, 2, 3, rnd.randrange(1 << height), (1 << height) - 1, 1 << height]))
            st = random_frontier(rnd, M.SPROUT, height, s0)
            _check_window(ctx, rnd, M.SPROUT, height, st, rnd.randrange((1 << height) - s0 + 1), 5)
    # the real heights, frontiers deep into the tree
    for s0 in (0, 1, 12345, (1 << 28) + 7, (1 << 29) - 40):
        _check_window(ctx, rnd, M.SPROUT, 29, random_frontier(rnd, M.SPROUT, 29, s0), 37, 6)


@pytest.mark.gpu
def test_gpu_sapling_windows_vs_oracle(ctx):
    rnd = random.Random(6)
    for height, s0, n in ((4, 0, 16), (4, 5, 9), (32, 0, 6), (32, 1, 5), (32, 6, 7), (32, 0xB2D05E00, 9),
                          (32, (1 << 32) - 5, 5)):
        _check_window(ctx, rnd, M.SAPLING, height, random_frontier(rnd, M.SAPLING, height, s0), n, 3)


@pytest.mark.gpu
def test_gpu_window_edges(ctx):
    from zebra_amd import zg
    rnd = random.Random(8)
    # no leaves: the roots of the state itself; an empty tree's root is H::empty()[HEIGHT]
    e = ctx.tree_empty_roots(M.SPROUT, 30)
    roots, state = ctx.tree_roots(M.SPROUT, 29, b"", [], [0, 0])
    assert roots == [e[29], e[29]] and state == M.TreeState(M.SPROUT, 29).serialize()
    st = random_frontier(rnd, M.SPROUT, 29, 1000)
    roots, state = ctx.tree_roots(M.SPROUT, 29, st.serialize(), [], [0])
    assert roots == [st.root()] and state == st.serialize()
    # overflow past 2^H from a deep frontier: TREE_FULL, the marks that fit are computed
    st = random_frontier(rnd, M.SPROUT, 6, 60)
    leaves = [_rand32(rnd) for _ in range(7)]
    with pytest.raises(zg.ZgError) as ei:
        ctx.tree_roots(M.SPROUT, 6, st.serialize(), leaves, [2, 4, 5, 7])
    assert ei.value.code == zg.E_TREE_FULL
    want, _ = M.window_roots(st, leaves[:4], [2, 4])
    assert ei.value.roots[:2] == want and ei.value.roots[2:] == [bytes(32)] * 2
    # states the appends cannot produce / of another height are rejected
    bad = b"\x00\x01" + bytes(32) + bytes([28]) + b"\x00" * 28
    for s in (bad, M.TreeState(M.SPROUT, 28).serialize(), b"\x02"):
        with pytest.raises(zg.ZgError) as ei:
            ctx.tree_roots(M.SPROUT, 29, s, [], [0])
        assert ei.value.code == -1
    with pytest.raises(zg.ZgError):
        ctx.tree_roots(M.SPROUT, 29, b"", [bytes(32)], [2])


@pytest.mark.gpu
@pytest.mark.parametrize("kind,height", [(M.SPROUT, 29), (M.SAPLING, 32)])
def test_gpu_window_split_invariance_full_size(ctx, kind, height):
    """bench size (64k leaves, a root per 64): one window == the same leaves as two windows
    chained through the serialized state, for every root; the state after a split point has the
    oracle's root; and a mark's root is the oracle root of the chained state at that mark"""
    rnd = random.Random(9 + kind)
    n, per = 65536, 64
    s0 = rnd.randrange(1 << (height - 1))
    st = random_frontier(rnd, kind, height, s0)
    leaves = [_rand32(rnd) for _ in range(n)]
    marks = list(range(per, n + 1, per))
    roots, fin = ctx.tree_roots(kind, height, st.serialize(), leaves, marks)
    cut = 23 * per + 17
    r1, mid = ctx.tree_roots(kind, height, st.serialize(), leaves[:cut], [m for m in marks if m <= cut] + [cut])
    r2, fin2 = ctx.tree_roots(kind, height, mid, leaves[cut:], [m - cut for m in marks if m > cut])
    assert r1[:-1] + r2 == roots and fin2 == fin
    t = M.TreeState.deserialize(kind, height, mid)
    assert t.size() == s0 + cut and t.root() == r1[-1]
    _, at = ctx.tree_roots(kind, height, st.serialize(), leaves[:marks[40]], [])
    assert M.TreeState.deserialize(kind, height, at).root() == roots[40]
