#!/usr/bin/env python3
"""Writes profiles/traffic.json's entry for the pair kernel from rocprofv3
--pmc passes (FETCH_SIZE, WRITE_SIZE, TCC_HIT/MISS in separate runs):
  tools/traffic_json.py PMC_DIR KEY SOURCE_NOTE [LDS_DMA_BYTES] [KERNEL_SUBSTRING]
KERNEL_SUBSTRING (e.g. "pair_mfma_kernel<3, 1, false>", the screen) restricts the
average to one kernel instantiation; default: every pair kernel dispatch."""
import collections
import csv
import glob
import json
import os
import sys

pmc, key, source = sys.argv[1], sys.argv[2], sys.argv[3]
ksub = sys.argv[5] if len(sys.argv) > 5 else ""
vals = collections.defaultdict(list)
for f in glob.glob(pmc + "/**/*_counter_collection.csv", recursive=True):
    rows = [r for r in csv.DictReader(open(f))
            if ((ksub in r["Kernel_Name"]) if ksub else ("pair_mfma" in r["Kernel_Name"] or "pair_valu" in r["Kernel_Name"]))]
    # full launches only: a screen's sample run (every 64th entry) is a
    # dispatch of the same kernel a fraction as long
    dur = {r["Dispatch_Id"]: int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows}
    if dur:
        med = sorted(dur.values())[len(dur) // 2]
        for r in rows:
            if dur[r["Dispatch_Id"]] >= med / 2:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in vals.items()}
fetch, write = m.get("FETCH_SIZE", 0.0), m.get("WRITE_SIZE", 0.0)
path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "traffic.json")
data = json.load(open(path)) if os.path.exists(path) else {}
old = data.get(key, {})
entry = {
    "hbm_bytes_per_launch": (2 * fetch + write) * 1024,
    "fetch_size_kb": fetch,
    "write_size_kb": write,
    "dispatches_averaged": len(vals.get("FETCH_SIZE", [])),
    "correction": "FETCH_SIZE x2 (gfx950 reports half the bytes of 16-B/lane streaming reads and LDS-DMA; "
                  "MI355X_MICROARCH.md HBM section); WRITE_SIZE as reported; x1024 (KB)",
    "note": os.environ.get("WLD_TRAFFIC_NOTE") or
            "FETCH_SIZE counts L2->fabric requests, Infinity-Cache (MALL) hits included; the two 41 MB "
            "fragment copies fit the 256 MB MALL",
    "source": source,
}
if ksub:
    entry["kernel"] = ksub
if "TCC_HIT_sum" in m:
    entry["l2_hit_rate"] = m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
lds = int(sys.argv[4]) if len(sys.argv) > 4 and sys.argv[4] else old.get("lds_dma_bytes_per_launch")
if lds:
    entry["lds_dma_bytes_per_launch"] = lds
data[key] = entry
json.dump(data, open(path, "w"), indent=1)
print(json.dumps(entry, indent=1))
