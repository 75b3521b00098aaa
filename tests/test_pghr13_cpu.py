"""CPU tier: the C++ restatement of the reference's PGHR13 check (oracle/cpu/pghr13_cpu.cpp, the
f4 CPU baseline) is pinned before it is timed: its pairing equals the Python oracle's (Miller
loop + the Fuentes-Castaneda final exponentiation, GT bytes) on random pairs, it is bilinear,
and every case of tests/golden/pghr13.json -- the reference's proof_decode / verification /
verification2 / smoky_pghr vectors, mainnet block 522's PHGR JoinSplits and the encoding /
subgroup / statement mutants -- gets its pinned status, on 1 and 4 threads."""
import random

import pytest

from oracle import bn254 as B
from tests import cpulib
from tests.conftest import load_golden


@pytest.fixture(scope="module")
def L():
    return cpulib.load_pghr13()


def test_pairing_bytes_match_oracle(L):
    rnd = random.Random(5)
    ps = [B.G1_GEN, B.ec_mul(B._F1, B.G1_GEN, rnd.randrange(1, B.R))]
    qs = [B.G2_GEN, B.ec_mul(B._F2, B.G2_GEN, rnd.randrange(1, B.R))]
    got = cpulib.pg_pairing(L, ps, qs)
    for p, q, g in zip(ps, qs, got):
        assert g == B.gt_ints(B.final_exponentiation_fc(B.miller_loop([(p, q)])))
    # bilinearity: e(6 P, 7 Q) == e(42 P, Q)
    a, b = cpulib.pg_pairing(L, [B.ec_mul(B._F1, B.G1_GEN, 6), B.ec_mul(B._F1, B.G1_GEN, 42)],
                             [B.ec_mul(B._F2, B.G2_GEN, 7), B.G2_GEN])
    assert a == b


@pytest.mark.parametrize("threads", [1, 4])
def test_golden_cases(L, threads):
    cases = load_golden("pghr13.json")["cases"]
    got = cpulib.pg_verify(L, [bytes.fromhex(c["proof"]) for c in cases],
                           [[bytes.fromhex(x) for x in c["inputs"]] for c in cases], threads=threads)
    assert got == [c["status"] for c in cases], [(c["name"], g, c["status"]) for c, g in zip(cases, got)
                                                  if g != c["status"]]
