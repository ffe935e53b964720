#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs for the pair kernel: per-dispatch averages,
effective clock (GRBM_GUI_ACTIVE / 8 / duration) and MFMA busy fraction."""
import collections
import csv
import glob
import sys

for f in sorted(glob.glob(sys.argv[1] + "/**/*_counter_collection.csv", recursive=True)):
  by_kernel = collections.defaultdict(lambda: (collections.defaultdict(list), {}))
  for r in csv.DictReader(open(f)):
    if not any(k in r["Kernel_Name"] for k in ("pair_mfma", "pair_valu", "pair_fp6", "pair_i8", "ref_item")):
        continue
    agg, dur = by_kernel[r["Kernel_Name"].split("(")[0]]
    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
  for kname, (agg, dur) in sorted(by_kernel.items()):
        m = {k: sum(v) / len(v) for k, v in agg.items()}
        d = sum(dur.values()) / len(dur)
        out = {"file": f.split("/")[-1], "kernel": kname.replace("void wld::", ""), "dispatches": len(dur), "ms": round(d * 1e3, 3)}
        if "GRBM_GUI_ACTIVE" in m:
            cyc = m["GRBM_GUI_ACTIVE"] / 8
            out["ghz"] = round(cyc / d / 1e9, 3)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                out["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / cyc, 3)
        if "SQ_WAVE_CYCLES" in m:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if k in m:
                    out[k] = round(m[k] / m["SQ_WAVE_CYCLES"], 3)
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_VALU", "SQ_LDS_BANK_CONFLICT", "FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"):
            if k in m:
                out[k] = m[k]
        print(out)
