#!/usr/bin/env python3
"""One line per bench JSON log: ms/step, value, pair phase, screen, candidate launch.
    python tools/bench_summary.py gpurun_out/r03h/*.log"""
import json
import sys

for f in sys.argv[1:]:
    for line in open(f):
        if not line.startswith("{"):
            continue
        j = json.loads(line)
        r = j["roofline"]
        s = r.get("screen") or {}
        print("%-40s ms/step %.4f value %.4g pair %.4f screen %s cand %s ctiles %s cblk %s cfrac %s rows %s" % (
            f.split("/")[-1], j["ms_per_step"], j["value"], r.get("pair_phase_ms", float("nan")),
            "%.4f" % s["screen_ms"] if s else "-", "%.4f" % s["candidate_launch_ms"] if s else "-",
            s.get("candidate_tiles"), s.get("candidate_blocks"),
            None if s.get("candidate_frac") is None else round(s["candidate_frac"], 3), j["config"]["rows_passing"]))
