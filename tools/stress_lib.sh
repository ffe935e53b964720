#!/bin/bash
# tools/stress_lib.sh NAME LIB THR RUNS: ring-vs-site-major bit-exact screen of one build
name=$1; lib=$2; thr=$3; runs=$4
WLD_INITIAL_STAGING_ROWS=100000000 WLD_TOOL_LIB=$lib timeout -k 10 400 python tools/stress_ring.py --thr $thr --runs $runs > gpurun_out/st_${name}_$thr.log 2>&1
rc=$?
python3 - "$name" "$thr" <<'PY'
import json, sys
name, thr = sys.argv[1], sys.argv[2]
for l in open("gpurun_out/st_%s_%s.log" % (name, thr)):
    if l.startswith("{"):
        d = json.loads(l)
        print(name, thr, "ref", d["ref_rows"], "bad per run", [r["bad_rows"] for r in d["ring_runs"]])
PY
exit $rc
