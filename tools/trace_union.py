#!/usr/bin/env python3
"""Per-kernel busy time from a rocprofv3 kernel trace (csv) when launches of
one kernel overlap (bench.py's free step order): the plain average of
End - Start counts the overlap twice; the union of the launches' intervals
divided by their count is the per-launch device time the HIP events see.
    python tools/trace_union.py x_kernel_trace.csv [substring ...]"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
names = sys.argv[2:] or sorted({r["Kernel_Name"].split("(")[0] for r in rows})
print("kernel,launches,avg_ms,median_ms,union_ms_per_launch,max_overlap")
for n in names:
    k = [r for r in rows if n in r["Kernel_Name"]]
    if not k:
        continue
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in k)
    d = [(e - s) / 1e6 for s, e in iv]
    tot, cur, depth, ends = 0, None, 0, []
    for s, e in iv:
        ends = [x for x in ends if x > s] + [e]
        depth = max(depth, len(ends))
        if cur is None or s > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [s, e]
        else:
            cur[1] = max(cur[1], e)
    tot += cur[1] - cur[0]
    print("%s,%d,%.4f,%.4f,%.4f,%d" % (n.replace(",", ";")[:80], len(iv), sum(d) / len(d), statistics.median(d),
                                       tot / 1e6 / len(iv), depth))
