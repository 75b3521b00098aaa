"""CPU tier: the C++ restatement of bellman's per-proof path (oracle/cpu, the bench's
cpu_baseline) reproduces the golden fixtures -- statuses and GT bytes -- before it is
trusted as a baseline."""
from tests import cpulib
from tests.conftest import load_golden


def pack(items):
    proofs = b"".join(bytes.fromhex(e["proof"]) for e in items)
    kinds = bytes(e["kind"] for e in items)
    inputs = bytearray(288 * len(items))
    for i, e in enumerate(items):
        for j, x in enumerate(e["inputs"]):
            inputs[288 * i + 32 * j:288 * i + 32 * j + 32] = bytes.fromhex(x)
    return proofs, kinds, bytes(inputs), bytes(len(e["inputs"]) for e in items)


def test_cpu_restatement_matches_fixtures():
    L = cpulib.load()
    items = load_golden("real_proofs.json")["proofs"] + [
        m for m in load_golden("mutants.json")["mutants"] if m["vk"] == "builtin"]
    sts, gts = cpulib.verify(L, *pack(items), threads=4, want_gt=True)
    for e, st, gt in zip(items, sts, gts):
        assert st == e["status"], e.get("name")
        if e.get("lhs_gt"):
            assert gt.hex() == e["lhs_gt"], e.get("name")
