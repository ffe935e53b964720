#!/usr/bin/env python3
"""Per-kernel mean of each counter in rocprofv3 --pmc counter_collection.csv files.
    python tools/pmc_kernels.py <counter_collection.csv>... [--match substr]"""
import collections
import csv
import sys

args = sys.argv[1:]
match = ""
if "--match" in args:
    i = args.index("--match")
    match = args[i + 1]
    del args[i:i + 2]
files = args
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in files:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if match and match not in k:
            continue
        acc[k[:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    n = max(len(v) for v in cs.values())
    print("%s (dispatch-counter rows %d)" % (k, n))
    for c, v in sorted(cs.items()):
        print("   %-28s %.4g" % (c, sum(v) / len(v)))
