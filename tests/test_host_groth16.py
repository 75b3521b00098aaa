"""CPU tier: the product's per-proof Groth16 path (zg_groth16.h verify_single, compiled for
the host by tests/native) against the golden fixtures: 9 real proofs accept with the
oracle's GT; every mutant lands in the reference's error class."""
import json
import os

import pytest

from tests import hostlib
from tests.conftest import ROOT, load_golden

VK_FILES = {0: "sapling-spend-verifying-key.json", 1: "sapling-output-verifying-key.json",
            2: "sprout-groth16-key.json"}


def vk_raw(kind):
    d = json.load(open(os.path.join(ROOT, "zebra_amd", "res", VK_FILES[kind])))
    h = lambda s: bytes.fromhex(s[2:] if s.startswith("0x") else s)  # noqa: E731
    fields = b"".join(h(d[k]) for k in ("alphaG1", "betaG1", "betaG2", "gammaG2", "deltaG1", "deltaG2"))
    return fields, [h(x) for x in d["ic"]]


def bad_vk_raw():
    g1 = bytes([0x40]) + bytes(95)
    g2 = bytes([0x40]) + bytes(191)
    return g1 + g1 + g2 + g2 + g1 + g2, []


@pytest.fixture(scope="module")
def L():
    return hostlib.lib()


def prep(L, raw):
    fields, ic = raw
    ab = hostlib.buf(576)
    assert L.zgt_vk_prepare(fields, len(ic), b"".join(ic) or None, ab) == 0
    return ab.raw


def run_items(L, items, vkinfo):
    gt = hostlib.buf(576)
    cur = None
    for e in items:
        vk = e.get("vk", "builtin")
        key = (e["kind"], vk)
        if key != cur:
            ab = prep(L, vk_raw(e["kind"]) if vk == "builtin" else bad_vk_raw())
            if vk == "builtin":
                assert ab.hex() == vkinfo[["spend", "output", "sprout"][e["kind"]]]["alpha_g1_beta_g2"]
            cur = key
        inputs = b"".join(bytes.fromhex(x) for x in e["inputs"])
        st = L.zgt_verify_single(bytes.fromhex(e["proof"]), inputs, len(e["inputs"]), gt)
        assert st == e["status"], e.get("name")
        if e.get("lhs_gt"):
            assert gt.raw.hex() == e["lhs_gt"], e.get("name")


def test_real_proofs(L):
    run_items(L, load_golden("real_proofs.json")["proofs"], load_golden("vk.json"))


def test_mutants(L):
    run_items(L, load_golden("mutants.json")["mutants"], load_golden("vk.json"))
