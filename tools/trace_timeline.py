#!/usr/bin/env python3
"""Timeline of one context's life from a rocprofv3 --hip-trace --kernel-trace
run of tools/first_pass.py: HIP API calls (allocations, copies, syncs, and any
call over 20 us) and kernels between the K-th and (K+1)-th stream creation,
in ms from the first.  Prints the API totals over the whole trace first.
    tools/trace_timeline.py TRACE_DIR [K=1] [MAX_LINES=60]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 1
lim = int(sys.argv[3]) if len(sys.argv) > 3 else 60
api = list(csv.DictReader(open(glob.glob(d + "/**/*hip_api_trace.csv", recursive=True)[0])))
ker = list(csv.DictReader(open(glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0])))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in api:
    agg[r["Function"]][0] += 1
    agg[r["Function"]][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
print("HIP API totals (calls, ms):")
for name, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:12]:
    print("  %-34s %7d %9.3f" % (name, n, t))
sc = sorted(int(r["Start_Timestamp"]) for r in api if r["Function"] == "hipStreamCreateWithFlags")
t0, t1 = sc[k], sc[k + 1] if k + 1 < len(sc) else float("inf")
keep = ("hipMalloc", "hipFree", "hipLaunchKernel", "hipStreamSynchronize", "hipEventSynchronize", "hipMemcpyAsync")
ev = []
for r in api:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if t0 <= s < t1 and (e - s > 20000 or r["Function"] in keep):
        ev.append((s, e, "api " + r["Function"]))
for r in ker:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if t0 <= s < t1:
        ev.append((s, e, "kernel " + r["Kernel_Name"].split("(")[0]))
ev.sort()
print("context %d (start, duration in ms):" % k)
prev = None
for s, e, n in ev[:lim]:
    gap = "" if prev is None or s - prev < 200000 else "   <- %.3f ms with no HIP call" % ((s - prev) / 1e6)
    print("%9.3f %8.3f  %s%s" % ((s - t0) / 1e6, (e - s) / 1e6, n, gap))
    prev = max(prev or 0, e)
