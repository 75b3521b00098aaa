#!/usr/bin/env python3
"""Short per-kernel table (calls, avg ms, total ms) from a rocprofv3 rocpd .db."""
import sqlite3
import sys
db = sqlite3.connect(sys.argv[1])
agg = {}
for name, s, e in db.execute("select name, start, end from kernels"):
    agg.setdefault(name.split("(")[0].replace("zg::", ""), []).append((e - s) / 1e6)
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print("%-26s calls=%4d avg=%9.3f ms total=%9.3f ms" % (k, len(v), sum(v) / len(v), sum(v)))
