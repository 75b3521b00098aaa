#!/usr/bin/env python3
"""Kernel resource table of the in-tree library (tooling): compiles every unit of zebra_amd/build.py
SOURCES with -Rpass-analysis=kernel-resource-usage into a scratch directory (the in-tree objects are
not touched) and prints one row per kernel: VGPRs, AGPRs, SGPRs, scratch bytes per lane, VGPR/SGPR
spills, occupancy (waves per SIMD), LDS bytes per block.

    python tools/resource_table.py > profiles/<tag>_resource_usage.txt
"""
import concurrent.futures
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from zebra_amd import build as zb  # noqa: E402

FIELDS = [("VGPRs", "vgpr"), ("AGPRs", "agpr"), ("TotalSGPRs", "sgpr"), ("ScratchSize [bytes/lane]", "scratch"),
          ("VGPRs Spill", "vspill"), ("SGPRs Spill", "sspill"), ("Occupancy [waves/SIMD]", "occ"),
          ("LDS Size [bytes/block]", "lds")]


def unit(src, tmp):
    cmd = ["hipcc"] + zb.FLAGS + ["-Rpass-analysis=kernel-resource-usage", "-I" + os.path.join(ROOT, "include"),
                                   "-c", "-o", os.path.join(tmp, src + ".o"), os.path.join(zb.CSRC, src)]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", line)
        if m:
            cur = {"unit": src, "name": m.group(1)}
            rows.append(cur)
            continue
        for label, key in FIELDS:
            m = re.search(r"remark:\s+%s: (\d+)" % re.escape(label), line)
            if m and cur is not None:
                cur[key] = int(m.group(1))
    return rows


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                             text=True).stdout.splitlines()
        return out if len(out) == len(names) else names
    except OSError:
        return names


def main():
    srcs = [s for s in zb.SOURCES if os.path.exists(os.path.join(zb.CSRC, s))]
    with tempfile.TemporaryDirectory() as tmp, concurrent.futures.ThreadPoolExecutor(max_workers=8) as ex:
        rows = [r for rs in ex.map(lambda s: unit(s, tmp), srcs) for r in rs]
    # kernels only (device functions have no occupancy line)
    rows = [r for r in rows if "occ" in r]
    names = demangle([r["name"] for r in rows])
    print("# kernel resource usage, hipcc %s -Rpass-analysis=kernel-resource-usage (tools/resource_table.py)"
          % " ".join(zb.FLAGS))
    print("%-22s %-60s %5s %5s %5s %8s %6s %6s %4s %7s" % ("unit", "kernel", "vgpr", "agpr", "sgpr", "scratch",
                                                         "vspill", "sspill", "occ", "lds"))
    for r, n in sorted(zip(rows, names), key=lambda t: (t[0]["unit"], t[1])):
        n = re.sub(r"\(.*", "", n)
        print("%-22s %-60s %5d %5d %5d %8d %6d %6d %4d %7d" % (r["unit"], n[:60], r.get("vgpr", 0), r.get("agpr", 0),
                                                             r.get("sgpr", 0), r.get("scratch", 0), r.get("vspill", 0),
                                                             r.get("sspill", 0), r.get("occ", 0), r.get("lds", 0)))


if __name__ == "__main__":
    main()
