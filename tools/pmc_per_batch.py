#!/usr/bin/env python3
"""Per-batch totals of rocprofv3 --pmc counters by kernel: the sum over every dispatch of a counter,
divided by the number of batches the run verified, with each kernel's share of the total. Used to
compare where the VALU instructions of one batch go at two shard sizes (e.g. 8k vs 64k in flight).
Usage: pmc_per_batch.py DIR BATCHES [COUNTER]"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    d, batches = sys.argv[1], float(sys.argv[2])
    want = sys.argv[3] if len(sys.argv) > 3 else "SQ_INSTS_VALU"
    tot = defaultdict(float)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == want:
                tot[r["Kernel_Name"].split("(")[0].replace("zg::", "").replace("void ", "")] += float(r["Counter_Value"])
    skip = ("k_mad_rate", "k_vk_comb", "k_vk_prepare", "k_rerandomize")
    s = sum(v for k, v in tot.items() if not k.startswith(skip))
    print("%s per batch (%g batches; setup kernels excluded): %.4g" % (want, batches, s / batches))
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        if k.startswith(skip):
            continue
        print("  %-26s %12.4g  %5.1f%%" % (k, v / batches, 100 * v / s))


if __name__ == "__main__":
    main()
