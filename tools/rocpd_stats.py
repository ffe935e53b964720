#!/usr/bin/env python3
"""Per-kernel statistics (launches, average / min / max duration) from a
rocprofv3 SQLite output (rocpd *_results.db), in the kernel_stats.csv shape:
    python tools/rocpd_stats.py path/to/x_results.db > kernel_stats.csv"""
import collections
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
q = ("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
     "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
agg = collections.defaultdict(list)
for name, st, en in db.execute(q):
    agg[name].append(en - st)
tot = sum(sum(v) for v in agg.values())
print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"')
for name, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
    print('"%s",%d,%d,%.1f,%.3f,%d,%d' % (name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / tot, min(v), max(v)))
