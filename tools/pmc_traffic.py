#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE in their own
runs, see tools/gpu_pmc.sh), corrected as MI355X_MICROARCH.md's HBM section prescribes:
FETCH_SIZE is in KB and reports 1/2 of the bytes on gfx950 (doubled here); WRITE_SIZE is in KB.
Per kernel (short name, template args kept): mean over the dispatches of the LONGEST-running
configuration, so the 64k-proof bench launches are not averaged with small warm-up batches.
Usage: pmc_traffic.py FETCH_DIR WRITE_DIR > profiles/pmc_traffic.json"""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(d, counter):
    per = defaultdict(dict)   # kernel -> dispatch -> (value, ms)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("zg::", "").replace("void ", "")
            ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            key = (f, r["Dispatch_Id"])
            v, _ = per[k].get(key, (0.0, ms))
            per[k][key] = (v + float(r["Counter_Value"]), ms)
    out = {}
    for k, ds in per.items():
        vals = list(ds.values())
        top = max(ms for _, ms in vals)
        big = [v for v, ms in vals if ms >= 0.5 * top]   # the full-size launches
        out[k] = (sum(big) / len(big), len(big), top)
    return out


fetch = load(sys.argv[1], "FETCH_SIZE")
write = load(sys.argv[2], "WRITE_SIZE")
res = {}
for k in sorted(set(fetch) & set(write)):
    fb = 2 * fetch[k][0] * 1024
    wb = write[k][0] * 1024
    res[k] = {"bytes_per_launch": fb + wb, "read_bytes": fb, "write_bytes": wb,
              "launches": fetch[k][1], "max_ms": round(fetch[k][2], 3)}
# bench.py looks kernels up by base name (template argument dropped): keep the longest variant
base = {}
for k, v in res.items():
    b = k.split("<")[0]
    if b not in base or v["max_ms"] > base[b]["max_ms"]:
        base[b] = dict(v, variant=k)
json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; FETCH_SIZE x2 (gfx950)",
           "kernels": res, **{k: v["bytes_per_launch"] for k, v in base.items()}}, sys.stdout, indent=1)
print()
