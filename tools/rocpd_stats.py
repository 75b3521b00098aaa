#!/usr/bin/env python3
"""Kernel stats (name, calls, total/avg/min/max ns, %) from a rocprofv3 rocpd .db (sqlite),
the same columns as rocprofv3's kernel_stats.csv. Usage: rocpd_stats.py run_results.db [out.csv]"""
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, start, end from kernels").fetchall()
agg = {}
for name, s, e in rows:
    a = agg.setdefault(name, [])
    a.append(e - s)
tot = sum(sum(v) for v in agg.values()) or 1
out = [("Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs")]
for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    out.append((name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / tot, min(v), max(v)))
w = csv.writer(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout)
w.writerows(out)
