#!/usr/bin/env python3
"""Static instruction mix of kernels in a hipcc -S device assembly file (tooling)."""
import re
import sys
s = open(sys.argv[1]).read()
for name in sys.argv[2:]:
    i = s.index(name + "E")
    i = s.index(":", i)
    j = s.index(".Lfunc_end", i)
    body = s[i:j]
    n = len(re.findall(r"^\s+v_", body, re.M))
    print("%-18s VALU %7d  mad %4d  lshl_add_u64 %6d  mov %6d  scratch %4d  ds %5d" % (
        name, n, body.count("v_mad_u64_u32"), body.count("v_lshl_add_u64"), body.count("v_mov_b32"),
        len(re.findall("scratch_", body)), len(re.findall(r"^\s+ds_", body, re.M))))
