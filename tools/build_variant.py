#!/usr/bin/env python3
"""A/B tooling: link zebra_amd/libzg_<name>.so from the in-tree objects, with the listed units
recompiled under extra -D switches (loaded by ZG_LIB_VARIANT=<name>, zebra_amd/zg.py).
Usage: python tools/build_variant.py NAME UNIT.hip[,UNIT.hip] -DFOO=1 [-DBAR=0 ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from zebra_amd import build as zb  # noqa: E402


def main():
    name, units, defs = sys.argv[1], sys.argv[2].split(","), sys.argv[3:]
    zb.build()
    objs = []
    for s in zb.SOURCES:
        o = zb._obj(s)
        if s in units:
            o = os.path.join(zb.OBJ, "%s.%s.o" % (s.replace(".hip", ""), name))
            subprocess.check_call(["hipcc"] + zb.FLAGS + defs + ["-I" + os.path.join(zb.HERE, "..", "include"), "-c",
                                                              "-o", o, os.path.join(zb.CSRC, s)])
        objs.append(o)
    out = os.path.join(zb.HERE, "libzg_%s.so" % name)
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs)
    print(out)


if __name__ == "__main__":
    main()
