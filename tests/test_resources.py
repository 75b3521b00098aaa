"""Kernel resource guards (CPU tier: hipcc cross-compiles gfx950 here, no GPU needed).

The decode kernels and the lane R-chain were taken off the private segment in round 4 (DESIGN.md §4,
"Decode off scratch", "Lane R-chain without spills"); scratch there was HBM traffic (round 3: 1.08 GB
per 64k batch for decode, 3.98 GB for the in-flight R-chain). These tests compile the units with
-Rpass-analysis=kernel-resource-usage (tools/resource_table.py) into a scratch directory and hold the
line: every decode kernel <= 64 B/lane, both lane R-chain variants 0 B, and the f-chain block within
the CU's LDS and the 256-VGPR budget of two waves per SIMD."""
import concurrent.futures
import os
import shutil
import tempfile

import pytest

from tools import resource_table

pytestmark = pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc not on PATH")

UNITS = ["zg_decode.hip", "zg_decode_sqrt.hip", "zg_lines.hip", "zg_prog_fchain4.hip"]


@pytest.fixture(scope="module")
def kernels():
    with tempfile.TemporaryDirectory() as tmp, concurrent.futures.ThreadPoolExecutor(max_workers=4) as ex:
        rows = [r for rs in ex.map(lambda u: resource_table.unit(u, tmp), UNITS) for r in rs]
    return {r["name"]: r for r in rows if "occ" in r}


def _find(kernels, part):
    got = {n: r for n, r in kernels.items() if part in n}
    assert got, "no kernel matching %r (have %s)" % (part, sorted(kernels))
    return got


def test_decode_kernels_at_most_64_bytes_of_scratch(kernels):
    for part in ("k_decode_sqrt", "k_decode_points", "k_decode_finish"):
        for name, r in _find(kernels, part).items():
            assert r["scratch"] <= 64, (name, r)


def test_lane_r_chain_has_no_scratch(kernels):
    got = _find(kernels, "k_batch_lines_lane")
    assert len(got) == 2  # the one- and two-waves-per-SIMD register budgets
    for name, r in got.items():
        assert r["scratch"] == 0 and r.get("vspill", 0) == 0, (name, r)


def test_fchain4_fits_one_block_per_cu(kernels):
    got = _find(kernels, "k_batch_fchain4")
    assert len(got) == 2  # the split (Q4IK + GMSQ) and fused (Q4SQ) step programs
    for name, r in got.items():
        assert r["lds"] <= 160 * 1024 and r["vgpr"] <= 256 and r["occ"] >= 2, (name, r)
        if "<true>" in name:  # the default (the fused variant is an A/B knob, ZG_QUAD_SPLIT=0)
            assert r["scratch"] <= 32, (name, r)


def test_group_line_product_kernels_fit(kernels):
    """k_line_prod / k_batch_fchaing: one block per CU, two waves per SIMD, at most 40 B/lane of
    scratch (their program masks are chosen for that, zg_prog.h prog_run; the split k_line_prod's
    best mask leaves 9 spilled VGPRs outside the product loop, 40 B)"""
    for part in ("k_line_prod", "k_batch_fchaing"):
        for name, r in _find(kernels, part).items():
            assert r["lds"] <= 160 * 1024 and r["vgpr"] <= 256 and r["occ"] >= 2 and r["scratch"] <= 40, (name, r)

