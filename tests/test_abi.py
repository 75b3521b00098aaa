"""CPU tier: the C-ABI library builds for gfx950, loads, and exports every symbol that
include/zg.h declares (no compute calls: there is no GPU in this tier)."""
import ctypes
import os
import re
import subprocess

from tests.conftest import ROOT


def declared_symbols():
    h = open(os.path.join(ROOT, "include", "zg.h")).read()
    return sorted(set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(zg_\w+)\s*\(", h, flags=re.M)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("zg_create", "zg_destroy", "zg_vk_load_builtin", "zg_vk_load_json", "zg_vk_load_uncompressed",
              "zg_verify_one_gt", "zg_verify_each", "zg_verify_batch", "zg_batch_begin", "zg_batch_begin_device",
              "zg_batch_partial", "zg_gt_check", "zg_batch_finish", "zg_last_error"):
        assert s in syms


def test_library_exports_all_declared_symbols():
    from zebra_amd import build
    lib = build.build()
    L = ctypes.CDLL(lib)
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing
    L.zg_version.restype = ctypes.c_char_p
    assert b"gfx950" in L.zg_version()
    # build provenance: the library reports the hash of the sources it was compiled from
    assert L.zg_version().decode().endswith(" src " + build.source_hash())


def test_code_object_targets_gfx950():
    from zebra_amd import build
    lib = build.build()
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", lib], capture_output=True, text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(lib, "rb").read()
    assert b"gfx950" in blob
