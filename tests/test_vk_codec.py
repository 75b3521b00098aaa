"""The reference's verifying-key codec vectors (crypto/src/json/groth16.rs:108-148, extracted as
data into tests/golden/vk_codec.json by gen_golden.py --vk-codec) and the reference-pinned
mutant classes, against the oracle (CPU tier) and through the product's VK loaders
zg_vk_load_json / zg_vk_load_uncompressed (GPU tier: prepare_verifying_key runs on the device).

A valid point must load; too few / too many hex characters and an off-curve point (halves
swapped) must fail with ZG_E_VK (the reference's serde error)."""
import json
import os

import pytest

from tests.conftest import ROOT, load_golden

VK_FILE = os.path.join(ROOT, "zebra_amd", "res", "sapling-spend-verifying-key.json")
FIELD = {"g1": "alphaG1", "g2": "betaG2"}


def vectors():
    return load_golden("vk_codec.json")["vectors"]


def substituted(v):
    d = json.load(open(VK_FILE))
    d[FIELD[v["group"]]] = v["hex"]
    return json.dumps(d)


def test_oracle_agrees_with_reference_vectors():
    from oracle import bls12_381 as B, groth16 as G
    assert len(vectors()) == 8
    for v in vectors():
        try:
            G.load_vk_json(substituted(v))
            ok = True
        except B.DecodeError:
            ok = False
        assert ok == v["ok"], (v["group"], v["case"])


def test_pinned_mutants_in_reference_class():
    """sapling.rs:420-440, 486-509: [0;192] -> Invalid, empty ic -> Synthesis, nullifier zeroed
    and cmu := cv -> Failed (status 1 / 2 / 3)"""
    want = {"zero_proof": 1, "bad_vk_empty_ic": 2, "nullifier_zeroed": 3, "cmu_is_cv": 3}
    seen = set()
    for m in load_golden("mutants.json")["mutants"]:
        if m["pinned_by"]:
            cls = m["name"].split(":", 1)[1]
            assert m["status"] == want[cls], m["name"]
            seen.add(cls)
    assert seen == set(want)


def test_cpu_restatement_vk_decode():
    """oracle/cpu (bellman restatement) loads the valid points and rejects the off-curve ones"""
    import ctypes
    from tests import cpulib
    L = cpulib.load()
    d = json.load(open(VK_FILE))
    h = lambda s: bytes.fromhex(s[2:] if s.startswith("0x") else s)  # noqa: E731
    for v in vectors():
        if v["case"] not in ("valid", "invalid_curve_point"):
            continue
        dd = dict(d)
        dd[FIELD[v["group"]]] = v["hex"]
        fields = b"".join(h(dd[k]) for k in ("alphaG1", "betaG1", "betaG2", "gammaG2", "deltaG1", "deltaG2"))
        ic = [h(x) for x in dd["ic"]]
        ab = ctypes.create_string_buffer(576)
        rc = L.zgcpu_vk_load(0, fields, len(ic), b"".join(ic), ab)
        assert (rc == 0) == v["ok"], (v["group"], v["case"], rc)
    for k in cpulib.VK_FILES:   # restore the builtin keys of the shared library state
        f, ic = cpulib.vk_fields(k)
        assert L.zgcpu_vk_load(k, f, len(ic), b"".join(ic), ctypes.create_string_buffer(576)) == 0


@pytest.mark.gpu
def test_gpu_vk_load_json_vectors():
    from zebra_amd import Context
    from zebra_amd.zg import ZgError
    c = Context(device=0, max_batch=64, load_builtin=False)
    try:
        for v in vectors():
            if v["ok"]:
                c.vk_load_json(0, substituted(v))
            else:
                with pytest.raises(ZgError) as e:
                    c.vk_load_json(0, substituted(v))
                assert e.value.code == -4, (v["group"], v["case"])
        # the unchanged key still loads and prepares to the oracle's alpha_g1_beta_g2
        c.vk_load_json(0, open(VK_FILE).read())
        assert c.alpha_beta(0).hex() == load_golden("vk.json")["spend"]["alpha_g1_beta_g2"]
    finally:
        c.close()


@pytest.mark.gpu
def test_gpu_vk_load_uncompressed_vectors():
    """the same points through the raw-bytes loader (length errors cannot occur there)"""
    from zebra_amd import Context
    from zebra_amd.zg import ZgError
    d = json.load(open(VK_FILE))
    h = lambda s: bytes.fromhex(s[2:] if s.startswith("0x") else s)  # noqa: E731
    c = Context(device=0, max_batch=64, load_builtin=False)
    try:
        for v in vectors():
            if v["case"] not in ("valid", "invalid_curve_point"):
                continue
            dd = dict(d)
            dd[FIELD[v["group"]]] = v["hex"]
            args = [h(dd[k]) for k in ("alphaG1", "betaG1", "betaG2", "gammaG2", "deltaG1", "deltaG2")]
            ic = [h(x) for x in dd["ic"]]
            if v["ok"]:
                c.vk_load_uncompressed(0, *args, ic)
            else:
                with pytest.raises(ZgError) as e:
                    c.vk_load_uncompressed(0, *args, ic)
                assert e.value.code == -4
    finally:
        c.close()
