#!/usr/bin/env python3
"""Call graph of a kernel in a hipcc -S device assembly file, with each function's scratch
instruction count and private segment size (tooling: where do a kernel's spills come from).
Usage: callgraph.py FILE.s KERNEL_SYMBOL"""
import re
import sys

s = open(sys.argv[1]).read()


def body(name):
    i = s.index("\n" + name + ":")
    j = s.index(".Lfunc_end", i)
    return s[i:j]


seen, todo = set(), [sys.argv[2]]
while todo:
    f = todo.pop()
    if f in seen:
        continue
    seen.add(f)
    try:
        b = body(f)
    except ValueError:
        continue
    calls = set(re.findall(r"(_Z\w+)@rel32@lo", b))
    ncall = len(re.findall(r"s_swappc", b))
    nscr = len(re.findall(r"scratch_", b))
    nv = len(re.findall(r"^\s+v_", b, re.M))
    m = re.search(r"\.set " + re.escape(f) + r"\.private_seg_size, (\d+)", s)
    print("%-64s valu=%6d scratch_ops=%5d seg=%5s callsites=%3d" % (f[:64], nv, nscr, m.group(1) if m else "?", ncall))
    todo += sorted(calls)
