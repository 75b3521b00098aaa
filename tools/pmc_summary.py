#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection.csv files: per kernel (short name), the mean of
each counter over its dispatches. Usage: pmc_summary.py DIR [DIR...]"""
import csv
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for d in sys.argv[1:]:
    import glob
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("zg::", "")
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            key = (f, r["Dispatch_Id"])
            if key not in seen:
                seen.add(key)
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, cs in vals.items():
    print("%-22s ms=%.3f" % (k, sum(dur[k]) / len(dur[k])))
    for c, v in sorted(cs.items()):
        print("    %-22s %.4g" % (c, sum(v) / len(v)))
