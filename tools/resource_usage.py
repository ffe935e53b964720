#!/usr/bin/env python3
"""Per-kernel VGPR / spill / occupancy table of one HIP source (gfx950).
    python tools/resource_usage.py weightedld_amd/csrc/pair_mfma.hip"""
import re, subprocess, sys

src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-slp-vectorize",
       "-Iinclude", "-Iweightedld_amd/csrc", "-c", src, "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2)
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    name = re.sub(r"\(.*", "", r["name"])
    print("%-55s VGPR %4s AGPR %4s spill %3s/%3s occ %s LDS %s" % (
        name[:55], r.get("VGPRs", "?"), r.get("AGPRs", "?"), r.get("VGPRs Spill", "?"), r.get("SGPRs Spill", "?"),
        r.get("Occupancy [waves/SIMD]", "?"), r.get("LDS Size [bytes/block]", "?")))
